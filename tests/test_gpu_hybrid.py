"""K2h (fpnn_amd/csrc/k_hybrid.hip): ragged encrypt batches with lane- and quad-per-chain
sessions, against the oracle, bit-exact.

The wire form -- htole32(len) || ciphertext, PackageEncryptor::encrypt(std::string*),
core/Encryptor.cpp:34-51 -- puts every body 4 bytes off the block grid of its frame; K2h
writes such output as whole 16-byte slots assembled from two cipher blocks (funnel
shift), so these tests place frames at every byte offset mod 16 and check that the gap
bytes between frames are never written.  The sizes keep the oracle to a second or two.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
ENGINES = ["engine", "hybrid_engine", "hybrid_lane_engine", "hybrid_quad_engine"]


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _wire_expected(oracle, plain, dst0, n, in_off, out_off, lens, slots, keys, keylen, ivs):
    """Frames as PackageEncryptor::encrypt(std::string*) writes them at out_off[i]."""
    exp = dst0.copy()
    oracle.package_batch(True, plain, exp, n, in_off=in_off.astype(np.uint64),
                         out_off=(out_off + 4).astype(np.uint64), lens=lens.astype(np.uint32),
                         key_slot=None if slots is None else slots.astype(np.uint32), keys=keys, keylen=keylen,
                         ivs=ivs, threads=8)
    for o, L in zip(out_off, lens):
        exp[o:o + 4] = np.frombuffer(int(L).to_bytes(4, "little"), np.uint8)
    return exp


@pytest.mark.parametrize("eng_kind", ENGINES)
@pytest.mark.parametrize("keylen,nkeys", [(16, 1), (24, 5), (32, 1), (32, 200)])
@pytest.mark.parametrize("grid", [1, 4])
def test_wire_frames_every_offset(request, oracle, eng_kind, keylen, nkeys, grid):
    """Ragged bodies (0..3000 B, incl. sub-block and block-multiple lengths) into wire
    frames packed with 0..17-byte gaps, so frame starts take every offset mod 16
    (grid 1: K2h's quads funnel-shift the blocks into 16-byte slots) or every multiple of 4
    (grid 4: every body on the 4-byte grid, blocks stored as words where they fall)."""
    import fpnn_amd
    engine = request.getfixturevalue(eng_kind)
    rng = np.random.default_rng(7000 + 10 * keylen + nkeys + len(eng_kind) + 100 * grid)
    n = 2500
    lens = rng.integers(0, 3001, n)
    special = np.array([0, 1, 4, 11, 12, 15, 16, 17, 28, 32, 124, 127, 128, 129, 1024, 1025])
    pick = rng.random(n) < 0.3
    lens[pick] = rng.choice(special, pick.sum())
    in_off = np.concatenate([[0], np.cumsum(lens[:-1] + 5)]).astype(np.int64) + 3
    gaps = rng.integers(0, 18, n)
    span = (lens + 4 + gaps + grid - 1) // grid * grid
    out_off = np.concatenate([[0], np.cumsum(span[:-1])]).astype(np.int64) + int(gaps[-1]) // grid * grid
    plain = rng.integers(0, 256, int(in_off[-1] + lens[-1] + 32), dtype=np.uint8)
    dst0 = rng.integers(0, 256, int(out_off[-1] + lens[-1] + 4 + 64), dtype=np.uint8)
    keys = rng.integers(0, 256, nkeys * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, nkeys * 16, dtype=np.uint8)
    slots = rng.integers(0, nkeys, n).astype(np.int32) if nkeys > 1 else None
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), keylen, ivs.tobytes())
    exp = _wire_expected(oracle, plain, dst0, n, in_off, out_off, lens, slots, keys, keylen, ivs)
    dst = _dev(dst0)
    engine.package_encrypt(_dev(plain), dst, n, ks, in_off=_dev(in_off), out_off=_dev(out_off),
                           lens=_dev(lens.astype(np.int32)), key_slot=None if slots is None else _dev(slots),
                           wire_prefix=True)
    got = _host(dst)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"


@pytest.mark.parametrize("eng_kind", ENGINES)
def test_wire_frames_r1_shape(request, oracle, eng_kind):
    """R1's send side at 1/256 size: 4096 frames of htole32(1024) + 1 KiB packed back to
    back (frame i at 1028 i: the body offset mod 16 cycles through 4, 8, 12, 0)."""
    import fpnn_amd
    engine = request.getfixturevalue(eng_kind)
    rng = np.random.default_rng(4242)
    n, L = 4096, 1024
    lens = np.full(n, L, np.int64)
    in_off = np.arange(n, dtype=np.int64) * L
    out_off = np.arange(n, dtype=np.int64) * (L + 4)
    plain = rng.integers(0, 256, n * L, dtype=np.uint8)
    dst0 = np.zeros(n * (L + 4), dtype=np.uint8)
    key, iv = rng.integers(0, 256, 32, dtype=np.uint8), rng.integers(0, 256, 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, key.tobytes(), 32, iv.tobytes())
    exp = _wire_expected(oracle, plain, dst0, n, in_off, out_off, lens, None, key, 32, iv)
    dst = _dev(dst0)
    engine.package_encrypt(_dev(plain), dst, n, ks, in_off=_dev(in_off), out_off=_dev(out_off),
                           lens=_dev(lens.astype(np.int32)), wire_prefix=True)
    assert np.array_equal(_host(dst), exp)


@pytest.mark.parametrize("eng_kind", ENGINES)
@pytest.mark.parametrize("inplace", [False, True])
def test_long_and_short_chains(request, oracle, eng_kind, inplace):
    """A Zipf-like mix: a few chains of up to 64 KiB among many short ones (the C4 shape
    at small size), unaligned starts, one key; both sessions and the hand-over between
    them run in every engine setting."""
    import fpnn_amd
    engine = request.getfixturevalue(eng_kind)
    rng = np.random.default_rng(99 + inplace + 7 * len(eng_kind))
    n = 3000
    lens = (64 * np.minimum(rng.zipf(1.3, n), 1024)).astype(np.int64)
    tails = rng.random(n) < 0.25
    lens[tails] += rng.integers(1, 16, tails.sum())
    offs = np.concatenate([[0], np.cumsum(lens[:-1] + rng.integers(0, 3, n - 1))]).astype(np.int64) + 1
    plain = rng.integers(0, 256, int(offs[-1] + lens[-1] + 16), dtype=np.uint8)
    key, iv = rng.integers(0, 256, 32, dtype=np.uint8), rng.integers(0, 256, 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, key.tobytes(), 32, iv.tobytes())
    exp = plain.copy()
    oracle.package_batch(True, plain, exp, n, in_off=offs.astype(np.uint64), lens=lens.astype(np.uint32),
                         keys=key, keylen=32, ivs=iv, threads=8)
    src = _dev(plain)
    dst = src if inplace else _dev(plain)
    engine.package_encrypt(src, dst, n, ks, in_off=_dev(offs), lens=_dev(lens.astype(np.int32)))
    assert np.array_equal(_host(dst), exp)


@pytest.mark.parametrize("eng_kind", ENGINES)
@pytest.mark.parametrize("keylen", [16, 32])
def test_many_stream_segments(request, oracle, eng_kind, keylen):
    """3000 stream segments at random CFB positions (head and tail partial blocks), per
    stream keys, two successive calls: outputs and the carried (iv, pos) state."""
    import fpnn_amd
    engine = request.getfixturevalue(eng_kind)
    rng = np.random.default_rng(31 * keylen + len(eng_kind))
    S = 3000
    keys = rng.integers(0, 256, S * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, S * 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), keylen, ivs.tobytes())
    iv_h, pos_h = ivs.copy(), rng.integers(0, 16, S).astype(np.uint32)
    iv_d, pos_d = _dev(iv_h), _dev(pos_h.astype(np.int32))
    slots = np.arange(S, dtype=np.uint32)
    for call in range(2):
        lens = rng.integers(0, 2500, S).astype(np.int64)
        lens[rng.random(S) < 0.05] = 0
        offs = np.concatenate([[0], np.cumsum(lens[:-1] + 1)]).astype(np.int64)
        inp = rng.integers(0, 256, int(offs[-1] + lens[-1] + 16), dtype=np.uint8)
        exp = inp.copy()
        oracle.stream_batch(True, inp, exp, S, in_off=offs.astype(np.uint64), out_off=offs.astype(np.uint64),
                            lens=lens.astype(np.uint32), key_slot=slots, keys=keys, keylen=keylen,
                            iv_state=iv_h, pos_state=pos_h, threads=8)
        dst = _dev(inp)
        engine.stream_encrypt(_dev(inp), dst, S, ks, iv_d, pos_d, in_off=_dev(offs), lens=_dev(lens.astype(np.int32)),
                              key_slot=_dev(slots.astype(np.int32)))
        assert np.array_equal(_host(dst), exp), call
        assert np.array_equal(_host(iv_d), iv_h), call
        assert np.array_equal(_host(pos_d).astype(np.uint32), pos_h), call


@pytest.mark.parametrize("path,wire", [("k2c", False), ("k2h", False), ("k2h", True), ("k2h_lanes", False)])
def test_dirty_length_order_block_reported(oracle, path, wire):
    """The length-order block must be zero when a ragged encrypt starts (kernels.hpp).  With
    its bucket counts dirtied on purpose (FPNN_AES_DEBUG_POISON_ORDER: once, before the call)
    the call must stay in bounds -- no HIP fault -- and report FPNN_AES_ERR_DEVICE at the next
    sync; the engine then zeroes the block and the next call is right again."""
    import fpnn_amd
    from fpnn_amd._lib import ERR_DEVICE, FpnnAesError
    from conftest import _env_engine
    env = {"FPNN_AES_DEBUG_POISON_ORDER": "1"}
    if path != "k2c":
        env["FPNN_AES_HYB_FORCE"] = "1"
    if path == "k2h_lanes":
        env.update({"FPNN_AES_HYB_LONG": "1000000000", "FPNN_AES_HYB_QW": "2"})
    eng = _env_engine(env)
    try:
        rng = np.random.default_rng(5150 + len(path) + wire)
        n = 3000
        lens = rng.integers(0, 2000, n)
        in_off = np.concatenate([[0], np.cumsum(lens[:-1] + 3)]).astype(np.int64) + 1
        out_off = np.concatenate([[0], np.cumsum(lens[:-1] + 7)]).astype(np.int64) + 2
        plain = rng.integers(0, 256, int(in_off[-1] + lens[-1] + 32), dtype=np.uint8)
        dst0 = rng.integers(0, 256, int(out_off[-1] + lens[-1] + 64), dtype=np.uint8)
        key, iv = rng.integers(0, 256, 16, dtype=np.uint8), rng.integers(0, 256, 16, dtype=np.uint8)
        ks = fpnn_amd.KeySet(eng, key.tobytes(), 16, iv.tobytes())
        if wire:
            exp = _wire_expected(oracle, plain, dst0, n, in_off, out_off, lens, None, key, 16, iv)
        else:
            exp = dst0.copy()
            oracle.package_batch(True, plain, exp, n, in_off=in_off.astype(np.uint64),
                                 out_off=out_off.astype(np.uint64), lens=lens.astype(np.uint32),
                                 keys=key, keylen=16, ivs=iv, threads=8)
        args = dict(in_off=_dev(in_off), out_off=_dev(out_off), lens=_dev(lens.astype(np.int32)), wire_prefix=wire)
        src = _dev(plain)
        dst = _dev(dst0)
        eng.package_encrypt(src, dst, n, ks, **args)
        torch.cuda.synchronize()  # a wild access would surface here as a HIP error
        with pytest.raises(FpnnAesError) as ei:
            eng.sync()
        assert ei.value.status == ERR_DEVICE and "length order" in str(ei.value)
        dst = _dev(dst0)
        eng.package_encrypt(src, dst, n, ks, **args)
        assert np.array_equal(_host(dst), exp)
        eng.sync()
    finally:
        eng.close()
