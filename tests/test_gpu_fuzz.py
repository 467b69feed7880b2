"""Randomized package-mode batches over every layout the engine dispatches on, against
the oracle, bit-exact.  Each case draws a shape that steers run_encrypt / run_decrypt
into one kernel family -- K2 / K2c / K2q / K2h (three threshold settings) for encryption; K1d (plain, keyed, ragged),
K1k and K1 for decryption -- plus key lengths, key counts, in-place or not, and
lengths including 0 and non-multiples of 16.  The decrypt input is the encrypt output
of the same case, so each case also checks the round trip.  Seeds are fixed."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"

ENGINES = ["engine", "engine", "hybrid_engine", "hybrid_lane_engine", "hybrid_quad_engine"]
SHAPES = ["uniform", "dense", "dense_partial", "keyed_dense", "keyed_lane", "contiguous", "gapped", "ragged_keys"]


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _case(rng, shape):
    """-> (n, buffer size, layout kwargs (numpy arrays / ints), number of keys)"""
    n = int(rng.integers(1, 2500))
    if shape in ("uniform", "dense", "dense_partial", "keyed_dense", "keyed_lane"):
        if shape == "uniform":
            L = int(rng.integers(0, 3000))
            stride = L + int(rng.integers(0, 40))
        elif shape == "dense":
            L = 16 * int(rng.integers(2, 200))
            stride = L
        elif shape == "dense_partial":
            L = 16 * int(rng.integers(2, 200)) + int(rng.integers(1, 16))
            stride = L
        elif shape == "keyed_dense":
            L = 1024 * int(rng.integers(1, 5))
            stride = L
        else:
            L = 16 * int(rng.integers(2, 150))
            stride = L
        kw = dict(stride=stride, uniform_len=L)
        size = n * stride + 64
        nkeys = 1 if shape in ("uniform", "dense", "dense_partial") else int(rng.integers(2, 300))
        return n, size, kw, nkeys
    lens = rng.integers(0, 4000, n)
    if shape == "contiguous":
        lens = (lens // 16) * 16
        gaps = np.zeros(n, np.int64)
    else:
        gaps = rng.integers(0, 9, n)
    offs = 32 + np.concatenate([[0], np.cumsum(lens[:-1] + gaps[:-1])]).astype(np.int64)
    kw = dict(in_off=offs.astype(np.int64), lens=lens.astype(np.int32))
    size = int(offs[-1] + lens[-1] + 64)
    nkeys = int(rng.integers(2, 50)) if shape == "ragged_keys" else 1
    return n, size, kw, nkeys


@pytest.mark.parametrize("seed", range(64))
def test_fuzz_package_batches(request, oracle, seed):
    import fpnn_amd
    rng = np.random.default_rng(4242 + seed)
    shape = SHAPES[seed % len(SHAPES)]
    engine = request.getfixturevalue(ENGINES[(seed + seed // len(SHAPES)) % len(ENGINES)])
    keylen = int(rng.choice([16, 24, 32]))
    n, size, kw, nkeys = _case(rng, shape)
    keys = rng.integers(0, 256, nkeys * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, nkeys * 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), keylen, ivs.tobytes())
    slots = rng.integers(0, nkeys, n).astype(np.int32) if nkeys > 1 else None
    inplace = bool(rng.integers(0, 2))
    plain = rng.integers(0, 256, size, dtype=np.uint8)

    okw = dict(keys=keys, keylen=keylen, ivs=ivs, threads=8,
               key_slot=slots.astype(np.uint32) if slots is not None else None)
    ekw = {}
    for k, v in kw.items():
        if k in ("stride", "uniform_len"):
            okw[k] = v
            ekw[k] = v
        elif k == "in_off":
            okw[k] = v.astype(np.uint64)
            ekw[k] = _dev(v)
        else:
            okw[k] = v.astype(np.uint32)
            ekw[k] = _dev(v)
    if slots is not None:
        ekw["key_slot"] = _dev(slots)

    exp_c = plain.copy()
    oracle.package_batch(True, plain, exp_c, n, **okw)
    exp_p = exp_c.copy()
    oracle.package_batch(False, exp_c, exp_p, n, **okw)

    src = _dev(plain)
    dst = src if inplace else _dev(plain)
    engine.package_encrypt(src, dst, n, ks, **ekw)
    torch.cuda.synchronize()
    got_c = dst.cpu().numpy()
    assert np.array_equal(got_c, exp_c), (shape, n, keylen, nkeys, inplace, "encrypt")
    src2 = dst if inplace else _dev(exp_c)
    dst2 = src2 if inplace else _dev(exp_c)
    engine.package_decrypt(src2, dst2, n, ks, **ekw)
    torch.cuda.synchronize()
    assert np.array_equal(dst2.cpu().numpy(), exp_p), (shape, n, keylen, nkeys, inplace, "decrypt")
    assert np.array_equal(exp_p, plain)  # segments never overlap: the round trip restores every byte
