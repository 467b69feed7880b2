"""GPU parity: the HIP kernels (through the C-ABI) against the oracle and the
reference's golden fixtures.  Bit-exact everywhere (byte work, no tolerance)."""
import hashlib
import os
import sys

import numpy as np
import pytest
import torch

import workloads as W
from conftest import load_golden

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def to_dev(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.array(a, copy=True)).to(DEV)


def to_host(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy()


def dev_u8(n):
    return torch.zeros(max(1, n), dtype=torch.uint8, device=DEV)


def keyset(engine, keys: np.ndarray, keylen: int, ivs: np.ndarray):
    import fpnn_amd
    return fpnn_amd.KeySet(engine, keys.tobytes(), keylen, ivs.tobytes())


# --------------------------------------------------------------------------------------
# data generator + key schedule


def test_device_fill_matches_generator(engine):
    for n, off, shift in [(1, 0, 0), (7, 3, 1), (1000, 13, 5), (65536 + 11, 8, 0), (4097, 12345, 3)]:
        t = dev_u8(n + 8)
        engine.fill_synthetic(t[shift:shift + n], seed=42, byte_offset=off, nbytes=n)
        torch.cuda.synchronize()
        assert (to_host(t)[shift:shift + n] == W.synth_bytes(n, 42, off)).all()


@pytest.mark.parametrize("keylen", [16, 24, 32])
def test_device_key_expansion(engine, oracle, keylen):
    rng = np.random.default_rng(keylen + 100)
    n = 300
    keys = rng.integers(0, 256, n * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, n * 16, dtype=np.uint8)
    import fpnn_amd
    ks = fpnn_amd.KeySet(engine, to_dev(keys), keylen, to_dev(ivs))
    assert ks.nrounds == keylen // 4 + 6
    for i in (0, 1, 77, n - 1):
        got = ks.schedule(i)
        exp = oracle.setup_encrypt(keys[i * keylen:(i + 1) * keylen].tobytes())
        nw = 4 * (exp.nrounds + 1)
        assert got.nrounds == exp.nrounds and list(got.rk[:nw]) == list(exp.rk[:nw])


# --------------------------------------------------------------------------------------
# golden fixtures (produced by the compiled reference)


def test_golden_kat(engine, golden):
    import fpnn_amd
    g = golden("kat.json")
    for v in g["cfb"]:
        key, iv, pt = (bytes.fromhex(v[k]) for k in ("key", "iv", "in"))
        ctx = fpnn_amd.setup_encrypt(key)
        assert engine.cfb(ctx, True, pt, iv)[0].hex() == v["out"], v["name"]
        assert engine.cfb(ctx, False, bytes.fromhex(v["out"]), iv)[0] == pt
        # same through the device batch API (one packet, package mode)
        ks = fpnn_amd.KeySet(engine, key, len(key), iv)
        src, dst = to_dev(np.frombuffer(pt, np.uint8)), dev_u8(len(pt))
        engine.package_encrypt(src, dst, 1, ks, stride=len(pt), uniform_len=len(pt))
        torch.cuda.synchronize()
        assert to_host(dst).tobytes().hex() == v["out"]
    for v in g["ecb"]:  # one CFB block from IV = plaintext block with zero data = E(block)
        key, pt = bytes.fromhex(v["key"]), bytes.fromhex(v["in"])
        out = engine.cfb(fpnn_amd.setup_encrypt(key), True, bytes(16), pt)[0]
        assert out.hex() == v["out"], v["name"]


def test_golden_cfb_cases_host_path(engine, golden):
    """rijndael_cfb_encrypt semantics incl. (ivec, pos) carry via fpnn_aes_cfb_host."""
    import fpnn_amd
    for c in golden("cfb_cases.json"):
        ctx = fpnn_amd.setup_encrypt(bytes.fromhex(c["key"]))
        out, iv, pos = engine.cfb(ctx, c["encrypt"], bytes.fromhex(c["in"]), bytes.fromhex(c["iv"]), c["pos"])
        assert (out.hex(), iv.hex(), pos) == (c["out"], c["iv_out"], c["pos_out"])


@pytest.mark.parametrize("keylen", [16, 24, 32])
def test_small_call_kernel_vs_oracle(engine, oracle, keylen):
    """K0 (k_small.hip), the single-call kernel behind every fpnn_aes_cfb_host call of up to
    16 KiB (the drop-in Encryptor's per-call path): random lengths around every edge (1,
    15/16/17, one block short of / at / one past the 16 KiB limit, which takes the batch
    kernels), random entry positions, both directions, and chains of calls carrying
    (ivec, pos) as StreamEncryptor does -- byte-exact against the oracle's
    rijndael_cfb_encrypt, output and state."""
    import fpnn_amd
    rng = np.random.default_rng(404 + keylen)
    key = rng.bytes(keylen)
    ctx = fpnn_amd.setup_encrypt(key)
    lens = [1, 2, 15, 16, 17, 31, 32, 33, 1023, 1024, 1025, 4096, 16368, 16383, 16384, 16385, 20000]
    lens += [int(x) for x in rng.integers(1, 16384, 24)]
    for enc in (True, False):
        iv_g, pos_g = rng.bytes(16), 0
        iv_o, pos_o = iv_g, 0
        for n in lens:
            data = rng.bytes(n)
            pos_in = int(rng.integers(0, 16)) if rng.random() < 0.3 else None
            if pos_in is not None:  # a fresh entry state, else carry the chain's
                iv_g = iv_o = rng.bytes(16)
                pos_g = pos_o = pos_in
            out, iv_g, pos_g = engine.cfb(ctx, enc, data, iv_g, pos_g)
            exp, iv_o, pos_o = oracle.cfb(key, enc, data, iv_o, pos_o)
            assert out == exp, (enc, n)
            assert (iv_g, pos_g) == (iv_o, pos_o), (enc, n)


def test_small_call_receiver_pattern(engine, oracle):
    """The call sequence of EncryptedStreamReceiver on one connection
    (core/EncryptedStreamReceiver.cpp:89,124): decrypt the 12-byte header, then the body
    at position 12 mod 16, message after message, state carried -- 400 messages through
    K0, each call against the oracle."""
    import fpnn_amd
    rng = np.random.default_rng(1212)
    for keylen in (16, 32):
        key = rng.bytes(keylen)
        ctx = fpnn_amd.setup_encrypt(key)
        iv_g = iv_o = rng.bytes(16)
        pos_g = pos_o = 0
        for m in range(400):
            for n in (12, int(rng.integers(1, 1500))):
                data = rng.bytes(n)
                out, iv_g, pos_g = engine.cfb(ctx, False, data, iv_g, pos_g)
                exp, iv_o, pos_o = oracle.cfb(key, False, data, iv_o, pos_o)
                assert (out, iv_g, pos_g) == (exp, iv_o, pos_o), (keylen, m, n)


def test_golden_cfb_cases_stream_batch(engine, golden):
    """The same cases as ONE device stream batch: each case is a stream segment with its
    own key, carried (iv, pos) in and out (fpnn_aes_stream_encrypt/decrypt)."""
    cases = golden("cfb_cases.json")
    for keylen in (16, 24, 32):
        for enc in (True, False):
            sel = [c for c in cases if len(c["key"]) == 2 * keylen and c["encrypt"] == enc]
            n = len(sel)
            datas = [bytes.fromhex(c["in"]) for c in sel]
            lens = np.array([len(d) for d in datas], dtype=np.int32)
            offs = np.concatenate([[0], np.cumsum(lens[:-1] + 5)]).astype(np.int64)  # odd gaps: unaligned segments
            buf = np.zeros(int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
            for o, d in zip(offs, datas):
                buf[o:o + len(d)] = np.frombuffer(d, np.uint8)
            keys = np.concatenate([np.frombuffer(bytes.fromhex(c["key"]), np.uint8) for c in sel])
            ivs = np.concatenate([np.frombuffer(bytes.fromhex(c["iv"]), np.uint8) for c in sel])
            ks = keyset(engine, keys, keylen, ivs)
            src, dst = to_dev(buf), dev_u8(len(buf))
            iv_state = to_dev(ivs.copy())
            pos_state = to_dev(np.array([c["pos"] for c in sel], dtype=np.int32))
            fn = engine.stream_encrypt if enc else engine.stream_decrypt
            fn(src, dst, n, ks, iv_state, pos_state, in_off=to_dev(offs), lens=to_dev(lens),
               key_slot=to_dev(np.arange(n, dtype=np.int32)))
            torch.cuda.synchronize()
            out, ivo, poso = to_host(dst), to_host(iv_state), to_host(pos_state)
            for i, c in enumerate(sel):
                assert out[offs[i]:offs[i] + lens[i]].tobytes().hex() == c["out"]
                assert ivo[16 * i:16 * i + 16].tobytes().hex() == c["iv_out"]
                assert int(poso[i]) == c["pos_out"]


@pytest.mark.parametrize("eng_kind", ["engine", "hybrid_engine", "hybrid_lane_engine",
                                      "hybrid_quad_engine"])
def test_golden_package_cases(request, golden, eng_kind):
    engine = request.getfixturevalue(eng_kind)
    import fpnn_amd
    cases = golden("package_cases.json")
    for c in cases:  # per-call drop-in surface
        key, iv, data = (bytes.fromhex(c[k]) for k in ("key", "iv", "in"))
        pe = fpnn_amd.PackageEncryptor(engine, key, iv)
        assert pe.encrypt(data).hex() == c["encrypt"]
        assert pe.decrypt(data).hex() == c["decrypt"]
        assert pe.encrypt_frame(data).hex() == c["frame"]
    # all cases of one key as one device batch, incl. the wire-prefix frame form
    groups = {}
    for c in cases:
        groups.setdefault((c["key"], c["iv"]), []).append(c)
    for (k, v), cs in groups.items():
        key, iv = bytes.fromhex(k), bytes.fromhex(v)
        ks = fpnn_amd.KeySet(engine, key, len(key), iv)
        datas = [bytes.fromhex(c["in"]) for c in cs]
        lens = np.array([len(d) for d in datas], dtype=np.int32)
        offs = np.concatenate([[0], np.cumsum(lens[:-1] + 7)]).astype(np.int64)
        buf = np.zeros(int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
        for o, d in zip(offs, datas):
            buf[o:o + len(d)] = np.frombuffer(d, np.uint8)
        src = to_dev(buf)
        for mode in ("encrypt", "decrypt"):
            dst = dev_u8(len(buf))
            fn = engine.package_encrypt if mode == "encrypt" else engine.package_decrypt
            fn(src, dst, len(cs), ks, in_off=to_dev(offs), lens=to_dev(lens))
            torch.cuda.synchronize()
            out = to_host(dst)
            for i, c in enumerate(cs):
                assert out[offs[i]:offs[i] + lens[i]].tobytes().hex() == c[mode]
        out_offs = (offs + 4 * np.arange(len(cs))).astype(np.int64)
        dst = dev_u8(len(buf) + 4 * len(cs))
        engine.package_encrypt(src, dst, len(cs), ks, in_off=to_dev(offs), out_off=to_dev(out_offs),
                               lens=to_dev(lens), wire_prefix=True)
        torch.cuda.synchronize()
        out = to_host(dst)
        for i, c in enumerate(cs):
            assert out[out_offs[i]:out_offs[i] + lens[i] + 4].tobytes().hex() == c["frame"]


def test_golden_stream_cases(engine, golden):
    import fpnn_amd
    for c in golden("stream_cases.json"):
        key, iv = bytes.fromhex(c["key"]), bytes.fromhex(c["iv"])
        se = fpnn_amd.StreamEncryptor(engine, key, iv)
        # device-state twin: one stream, one call per frame
        ks = fpnn_amd.KeySet(engine, key, len(key), iv)
        iv_state = to_dev(np.frombuffer(iv, np.uint8).copy())
        pos_state = torch.zeros(1, dtype=torch.int32, device=DEV)
        for fr in c["frames"]:
            data = bytes.fromhex(fr["in"])
            got = se.encrypt(data) if c["encrypt"] else se.decrypt(data)
            assert got.hex() == fr["out"]
            if data:
                src, dst = to_dev(np.frombuffer(data, np.uint8)), dev_u8(len(data))
                fn = engine.stream_encrypt if c["encrypt"] else engine.stream_decrypt
                fn(src, dst, 1, ks, iv_state, pos_state, stride=0, uniform_len=len(data))
                torch.cuda.synchronize()
                assert to_host(dst)[:len(data)].tobytes().hex() == fr["out"]
        assert to_host(iv_state).tobytes() == se.state[0] and int(to_host(pos_state)[0]) == se.state[1]


# --------------------------------------------------------------------------------------
# randomized batches against the oracle


def make_ragged(rng, n, max_len, align_gap=True):
    lens = rng.integers(0, max_len + 1, n)
    special = np.array([0, 1, 15, 16, 17, 31, 32, 33, 1024, 1025, 4096])
    pick = rng.random(n) < 0.3
    lens[pick] = rng.choice(special, pick.sum())
    gaps = rng.integers(0, 9, n) if align_gap else np.zeros(n, np.int64)
    offs = np.concatenate([[0], np.cumsum(lens[:-1] + gaps[:-1])]).astype(np.int64) + int(gaps[-1])
    return lens.astype(np.int32), offs


@pytest.mark.parametrize("keylen", [16, 24, 32])
@pytest.mark.parametrize("nkeys", [1, 7])
@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("eng_kind", ["engine", "hybrid_engine", "hybrid_lane_engine",
                                      "hybrid_quad_engine"])
def test_random_package_batch(request, oracle, keylen, nkeys, inplace, eng_kind):
    engine = request.getfixturevalue(eng_kind)
    rng = np.random.default_rng(1000 * keylen + 10 * nkeys + inplace)
    n = 700
    lens, offs = make_ragged(rng, n, 3000)
    total = int(offs[-1] + lens[-1] + 64)
    inp = rng.integers(0, 256, total, dtype=np.uint8)
    keys = rng.integers(0, 256, nkeys * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, nkeys * 16, dtype=np.uint8)
    slots = rng.integers(0, nkeys, n).astype(np.int32)
    ks = keyset(engine, keys, keylen, ivs)
    kw = dict(in_off=to_dev(offs), lens=to_dev(lens), key_slot=to_dev(slots) if nkeys > 1 else None)
    for encrypt in (True, False):
        exp = inp.copy()
        oracle.package_batch(encrypt, inp, exp, n, in_off=offs.astype(np.uint64), lens=lens.astype(np.uint32),
                             key_slot=slots.astype(np.uint32) if nkeys > 1 else None, keys=keys, keylen=keylen,
                             ivs=ivs, threads=8)
        src = to_dev(inp)
        dst = src if inplace else to_dev(inp)  # untouched gap bytes must survive
        fn = engine.package_encrypt if encrypt else engine.package_decrypt
        fn(src, dst, n, ks, **kw)
        torch.cuda.synchronize()
        assert np.array_equal(to_host(dst), exp), f"encrypt={encrypt}"


@pytest.mark.parametrize("keylen,nk", [(16, 1000), (32, 1000), (32, 1)])
def test_many_short_frames_bounded_length_take_lane_chains(engine, oracle, keylen, nk):
    """fpnn_aes_batch.max_len: a ragged per-key package encrypt of >= 1 chain per GPU lane
    whose lengths the caller bounds by <= 2048 bytes runs one lane per chain in grid-stride
    order (K2) instead of the length-ordered hybrid (Q1: 491 vs 343 GiB/s; bounds of <= 175
    bytes take K2s, test_short_frames_whole_frame_passes).  1.1 M frames of
    1-300 bytes (sub-block, block-aligned and ragged tails) from 1000 keyed connections,
    the ciphertext against the oracle (and from one key: R1's send side); the same batch
    without the bound takes K2h and must give the same bytes."""
    import fpnn_amd
    rng = np.random.default_rng(9900 + keylen + nk)
    n = 1_100_000
    lens = rng.integers(1, 301, n).astype(np.int64)
    pick = rng.random(n) < 0.1
    lens[pick] = 16 * rng.integers(1, 19, int(pick.sum()))  # whole blocks
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    keys = rng.integers(0, 256, nk * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, nk * 16, dtype=np.uint8)
    slots = rng.integers(0, nk, n).astype(np.int32)
    ks = keyset(engine, keys, keylen, ivs)
    total = int(offs[-1] + lens[-1])
    inp = rng.integers(0, 256, total, dtype=np.uint8)
    exp = inp.copy()
    oracle.package_batch(True, inp, exp, n, in_off=offs.astype(np.uint64), lens=lens.astype(np.uint32),
                         key_slot=slots.astype(np.uint32), keys=keys, keylen=keylen, ivs=ivs, threads=8)
    src = to_dev(inp)
    kw = dict(in_off=to_dev(offs), lens=to_dev(lens.astype(np.int32)), key_slot=to_dev(slots))
    for bound, kernel in ((300, "cfb_encrypt_chains"), (0, "cfb_encrypt_hybrid")):
        dst = torch.zeros_like(src)
        engine.package_encrypt(src, dst, n, ks, max_len=bound, **kw)
        torch.cuda.synchronize()
        assert engine.last_kernel(fpnn_amd.K_ENCRYPT) == kernel, (bound, engine.last_kernel(fpnn_amd.K_ENCRYPT))
        assert np.array_equal(to_host(dst), exp), bound
    # the wire frames of the same batch (htole32(len) || C, PackageEncryptor::encrypt(std::string*))
    wout = (offs + 4 * np.arange(n)).astype(np.int64)  # frames back to back, 4 bytes longer each
    for bound, kernel in ((300, "cfb_encrypt_chains"), (0, "cfb_encrypt_hybrid")):
        wdst = torch.zeros(total + 4 * n, dtype=torch.uint8, device="cuda")
        engine.package_encrypt(src, wdst, n, ks, wire_prefix=True, max_len=bound, out_off=to_dev(wout), **kw)
        torch.cuda.synchronize()
        assert engine.last_kernel(fpnn_amd.K_ENCRYPT) == kernel
        got = to_host(wdst)
        for i in rng.integers(0, n, 2000):  # a sample of frames against the ciphertext above
            o, ln = int(wout[i]), int(lens[i])
            assert np.array_equal(got[o:o + 4 + ln], np.concatenate(
                [np.frombuffer(ln.to_bytes(4, "little"), np.uint8), exp[int(offs[i]):int(offs[i]) + ln]])), (bound, i)


@pytest.mark.parametrize("keylen,nk", [(16, 1000), (24, 7), (32, 1000), (32, 1)])
@pytest.mark.parametrize("wire", [False, True])
def test_short_frames_whole_frame_passes(engine, oracle, keylen, nk, wire):
    """K2s-DB (k_cfb_frames_db, round 6): ragged package encrypts whose caller bounds every
    length by <= 175 bytes (fpnn_aes_batch.max_len; FPNN's 145-B quests) with at least one
    chain per GPU lane load each frame whole, cipher it in registers and store it whole.
    300 000 frames of 0-175 bytes (FPNN's 145, whole blocks, 1-15-byte tails, empty) at
    unaligned offsets, one key or keyed connections, plain and wire frames
    (htole32(len) || C, core/Encryptor.cpp:34-51) against the oracle -- and a few frames past
    the bound (up to 400 B) still come out right, in several passes."""
    import fpnn_amd
    rng = np.random.default_rng(7700 + keylen + nk + 3 * wire)
    n = 300_000
    lens = rng.integers(0, 176, n).astype(np.int64)
    pick = rng.random(n)
    lens[pick < 0.3] = 145
    lens[(pick >= 0.3) & (pick < 0.4)] = 16 * rng.integers(0, 11, int(((pick >= 0.3) & (pick < 0.4)).sum()))
    over = rng.integers(0, n, 40)
    lens[over] = rng.integers(176, 401, 40)  # (past the caller's bound)
    gaps = rng.integers(0, 3, n)
    offs = np.concatenate([[0], np.cumsum(lens[:-1] + gaps[:-1])]).astype(np.int64) + 1
    keys = rng.integers(0, 256, nk * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, nk * 16, dtype=np.uint8)
    slots = rng.integers(0, nk, n).astype(np.int32)
    ks = keyset(engine, keys, keylen, ivs)
    total = int(offs[-1] + lens[-1] + 16)
    inp = rng.integers(0, 256, total, dtype=np.uint8)
    kw = dict(in_off=to_dev(offs), lens=to_dev(lens.astype(np.int32)))
    if nk > 1:
        kw["key_slot"] = to_dev(slots)
    if not wire:
        exp = inp.copy()
        oracle.package_batch(True, inp, exp, n, in_off=offs.astype(np.uint64), lens=lens.astype(np.uint32),
                             key_slot=slots.astype(np.uint32) if nk > 1 else None, keys=keys, keylen=keylen, ivs=ivs,
                             threads=8)
        dst = to_dev(inp)
        engine.package_encrypt(to_dev(inp), dst, n, ks, max_len=175, **kw)
    else:
        wout = (offs + 4 * np.arange(n) + np.cumsum(rng.integers(0, 2, n))).astype(np.int64)  # (never overlapping)
        dst0 = rng.integers(0, 256, int(wout[-1] + lens[-1] + 4 + 16), dtype=np.uint8)
        from test_gpu_hybrid import _wire_expected
        exp = _wire_expected(oracle, inp, dst0, n, offs, wout, lens, slots if nk > 1 else None, keys, keylen, ivs)
        dst = to_dev(dst0)
        engine.package_encrypt(to_dev(inp), dst, n, ks, wire_prefix=True, max_len=175, out_off=to_dev(wout), **kw)
    torch.cuda.synchronize()
    assert engine.last_kernel(fpnn_amd.K_ENCRYPT) == "cfb_encrypt_frames"
    got = to_host(dst)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"


@pytest.mark.parametrize("keylen,nk", [(16, 1000), (24, 7), (32, 1000), (32, 1)])
@pytest.mark.parametrize("inplace", [False, True])
def test_short_frames_decrypt_whole_frames(engine, oracle, keylen, nk, inplace):
    """D2s (k_cfb_frames_db<..., DEC>, round 6): ragged package decrypts whose caller
    bounds every length by <= 175 bytes, at least one frame per GPU lane: one lane per frame,
    the next frame loaded while this one is deciphered.  300 000 frames of 0-175 bytes
    (FPNN's 145, whole blocks, 1-15-byte tails, empty, under 16 B) at unaligned offsets, a
    few past the bound (block by block), one key or keyed connections, in place and not,
    against the oracle; and the batch without the bound (K1r) gives the same bytes."""
    import fpnn_amd
    rng = np.random.default_rng(9900 + keylen + nk + 5 * inplace)
    n = 300_000
    lens = rng.integers(0, 176, n).astype(np.int64)
    pick = rng.random(n)
    lens[pick < 0.3] = 145
    lens[(pick >= 0.3) & (pick < 0.4)] = 16 * rng.integers(0, 11, int(((pick >= 0.3) & (pick < 0.4)).sum()))
    over = rng.integers(0, n, 40)
    lens[over] = rng.integers(176, 401, 40)  # (past the caller's bound)
    gaps = rng.integers(0, 3, n)
    offs = np.concatenate([[0], np.cumsum(lens[:-1] + gaps[:-1])]).astype(np.int64) + 1
    keys = rng.integers(0, 256, nk * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, nk * 16, dtype=np.uint8)
    slots = rng.integers(0, nk, n).astype(np.int32)
    ks = keyset(engine, keys, keylen, ivs)
    total = int(offs[-1] + lens[-1])  # (the last frame ends the buffer)
    inp = rng.integers(0, 256, total, dtype=np.uint8)
    kw = dict(in_off=to_dev(offs), lens=to_dev(lens.astype(np.int32)))
    if nk > 1:
        kw["key_slot"] = to_dev(slots)
    exp = inp.copy()
    oracle.package_batch(False, inp, exp, n, in_off=offs.astype(np.uint64), lens=lens.astype(np.uint32),
                         key_slot=slots.astype(np.uint32) if nk > 1 else None, keys=keys, keylen=keylen, ivs=ivs,
                         threads=8)
    src = to_dev(inp)
    dst = src if inplace else to_dev(rng.integers(0, 256, total, dtype=np.uint8))
    if not inplace:  # bytes between frames keep the destination's own
        keep = np.ones(total, bool)
        for o, ln in zip(offs, lens):
            keep[o:o + ln] = False
        exp = np.where(keep, to_host(dst), exp)
    engine.package_decrypt(src, dst, n, ks, max_len=175, **kw)
    torch.cuda.synchronize()
    assert engine.last_kernel(fpnn_amd.K_DECRYPT) == "cfb_decrypt_frames"
    got = to_host(dst)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
    if not inplace:
        dst2 = to_dev(to_host(dst))
        engine.package_decrypt(src, dst2, n, ks, **kw)  # no bound: K1r
        torch.cuda.synchronize()
        assert engine.last_kernel(fpnn_amd.K_DECRYPT) != "cfb_decrypt_frames"
        assert torch.equal(dst2, dst)


@pytest.mark.parametrize("keylen", [16, 32])
@pytest.mark.parametrize("eng_kind", ["engine", "hybrid_lane_engine", "hybrid_quad_engine"])
def test_keyset_writes_refresh_first_keystream_block(request, oracle, keylen, eng_kind):
    """Block 0 of a package chain takes its keystream from the key set's per-slot E_k(IV)
    (KBatch::eiv, k_slot_eiv; SURVEY section 0 point 3), which every key-set write must
    refresh: slots set into a reserved table, two slots rewritten with new keys / IVs, and
    the table grown past its capacity.  Frames of FPNN's typical 145 B (whole waves start
    their chains together, so the kernels skip block 0's rounds), sub-block frames (the
    keystream of a lone partial block) and a spread of other lengths, against the oracle
    after each write."""
    import fpnn_amd
    engine = request.getfixturevalue(eng_kind)
    rng = np.random.default_rng(8800 + keylen + len(eng_kind))
    keys = rng.integers(0, 256, (6, keylen), dtype=np.uint8)
    ivs = rng.integers(0, 256, (6, 16), dtype=np.uint8)
    ks = fpnn_amd.KeySet.reserve(engine, 4, keylen)

    def check(nused):
        n = 3000
        lens = np.full(n, 145, np.int64)
        pick = rng.random(n) < 0.25
        lens[pick] = rng.choice(np.array([1, 7, 15, 16, 17, 31, 32, 160, 1024]), pick.sum())
        offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
        slots = rng.integers(0, nused, n).astype(np.int32)
        total = int(offs[-1] + lens[-1] + 16)
        inp = rng.integers(0, 256, total, dtype=np.uint8)
        exp = inp.copy()
        oracle.package_batch(True, inp, exp, n, in_off=offs.astype(np.uint64), lens=lens.astype(np.uint32),
                             key_slot=slots.astype(np.uint32), keys=keys[:nused].reshape(-1).copy(),
                             keylen=keylen, ivs=ivs[:nused].reshape(-1).copy(), threads=8)
        src, dst = to_dev(inp), to_dev(inp)
        engine.package_encrypt(src, dst, n, ks, in_off=to_dev(offs), lens=to_dev(lens.astype(np.int32)),
                               key_slot=to_dev(slots))
        torch.cuda.synchronize()
        assert np.array_equal(to_host(dst), exp), nused

    ks.set(0, keys[:4], ivs[:4])
    check(4)
    keys[1] = rng.integers(0, 256, keylen, dtype=np.uint8)
    ivs[2] = rng.integers(0, 256, 16, dtype=np.uint8)
    ks.set(1, keys[1:3], ivs[1:3])
    check(4)
    ks.set(4, keys[4:6], ivs[4:6])  # past the reserved capacity: the table grows
    check(6)
    ks.close()


@pytest.mark.parametrize("keylen", [16, 32])
@pytest.mark.parametrize("length", [1, 5, 16, 17, 64, 100, 1024, 1040, 4096])
def test_uniform_layout(engine, oracle, keylen, length):
    """Uniform fast path (stride/length, one key), incl. the in-place variant."""
    rng = np.random.default_rng(length * 7 + keylen)
    n = 2500
    stride = length + (length % 3)  # strides that are not multiples of 16
    inp = rng.integers(0, 256, n * stride + 8, dtype=np.uint8)
    key, iv = rng.bytes(keylen), rng.bytes(16)
    import fpnn_amd
    ks = fpnn_amd.KeySet(engine, key, keylen, iv)
    kb, ib = np.frombuffer(key, np.uint8).copy(), np.frombuffer(iv, np.uint8).copy()
    for encrypt in (True, False):
        exp = inp.copy()
        oracle.package_batch(encrypt, inp, exp, n, stride=stride, uniform_len=length, keys=kb, keylen=keylen, ivs=ib,
                             threads=8)
        for inplace in (False, True):
            src = to_dev(inp)
            dst = src if inplace else to_dev(inp)
            fn = engine.package_encrypt if encrypt else engine.package_decrypt
            fn(src, dst, n, ks, stride=stride, uniform_len=length)
            torch.cuda.synchronize()
            assert np.array_equal(to_host(dst), exp), (encrypt, inplace)


@pytest.mark.parametrize("keylen", [16, 32])
@pytest.mark.parametrize("length", [32, 48, 1008, 1024, 1040, 2048, 4096])
@pytest.mark.parametrize("n", [64, 2501])
def test_dense_layout(engine, oracle, keylen, length, n):
    """Dense whole-block batches (stride == length, length % 16 == 0): the K1d decrypt
    path -- chunk-aligned packets (length % 1 KiB == 0) and packet starts inside a
    chunk, partial last chunk (n = 2501), in place and out of place.  The 64 guard
    bytes after the batch must survive."""
    rng = np.random.default_rng(length * 11 + keylen + n)
    inp = rng.integers(0, 256, n * length + 64, dtype=np.uint8)
    key, iv = rng.bytes(keylen), rng.bytes(16)
    import fpnn_amd
    ks = fpnn_amd.KeySet(engine, key, keylen, iv)
    kb, ib = np.frombuffer(key, np.uint8).copy(), np.frombuffer(iv, np.uint8).copy()
    for encrypt in (True, False):
        exp = inp.copy()
        oracle.package_batch(encrypt, inp, exp, n, stride=length, uniform_len=length, keys=kb, keylen=keylen,
                             ivs=ib, threads=8)
        for inplace in (False, True):
            src = to_dev(inp)
            dst = src if inplace else to_dev(inp)
            fn = engine.package_encrypt if encrypt else engine.package_decrypt
            fn(src, dst, n, ks, stride=length, uniform_len=length)
            torch.cuda.synchronize()
            assert np.array_equal(to_host(dst), exp), (encrypt, inplace)


@pytest.mark.parametrize("layout", ["contiguous", "shifted_out", "inplace", "one_gap", "odd_len"])
def test_contiguous_ragged_decrypt(engine, oracle, layout):
    """Ragged package batches whose segments are back to back in whole 16-byte blocks
    (the C4 shape): the decrypt runs K1d with the segment-start mask.  'one_gap' and
    'odd_len' break contiguity and must fall back to K1 with the same results."""
    rng = np.random.default_rng(["contiguous", "shifted_out", "inplace", "one_gap", "odd_len"].index(layout) + 90)
    n = 3001
    lens = (rng.integers(0, 257, n) * 16).astype(np.int64)
    lens[rng.random(n) < 0.05] = 0
    lens[:3] = (16, 1024, 0)
    if layout == "odd_len":
        lens[1500] += 5
    base = 48  # the batch does not start at the buffer start
    offs = base + np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    if layout == "one_gap":
        offs[2000:] += 32
    total = int(offs[-1] + lens[-1] + 64)
    inp = rng.integers(0, 256, total, dtype=np.uint8)
    key, iv = rng.bytes(32), rng.bytes(16)
    import fpnn_amd
    ks = fpnn_amd.KeySet(engine, key, 32, iv)
    kb, ib = np.frombuffer(key, np.uint8).copy(), np.frombuffer(iv, np.uint8).copy()
    out_offs = offs + 96 if layout == "shifted_out" else offs
    exp = np.zeros(total + 96, dtype=np.uint8) if layout == "shifted_out" else inp.copy()
    oracle.package_batch(False, inp, exp, n, in_off=offs.astype(np.uint64), out_off=out_offs.astype(np.uint64),
                         lens=lens.astype(np.uint32), keys=kb, keylen=32, ivs=ib, threads=8)
    src = to_dev(inp)
    if layout == "inplace":
        dst = src
    elif layout == "shifted_out":
        dst = dev_u8(total + 96)
    else:
        dst = to_dev(inp)
    kw = dict(in_off=to_dev(offs), lens=to_dev(lens.astype(np.int32)))
    if layout == "shifted_out":
        kw["out_off"] = to_dev(out_offs)
    engine.package_decrypt(src, dst, n, ks, **kw)
    torch.cuda.synchronize()
    assert np.array_equal(to_host(dst), exp)


@pytest.mark.parametrize("gaps,inplace", [(g, ip) for ip in (False, True)
                                          for g in ("wire4", "random", "reversed", "shifted_out", "odd_len")
                                          if not (ip and g == "shifted_out")])  # a shifted output is out of place
def test_gapped_ragged_decrypt(engine, oracle, gaps, inplace):
    """Ragged whole-block package segments with gaps between them (the receive path:
    bodies behind 4-byte length prefixes), empty segments interleaved, through K1r
    ('reversed': segments in descending memory order; 'odd_len': one partial block)."""
    rng = np.random.default_rng(["wire4", "random", "reversed", "shifted_out", "odd_len"].index(gaps) + 31 * inplace)
    n = 2500
    lens = (rng.integers(0, 200, n) * 16).astype(np.int64)
    lens[rng.random(n) < 0.05] = 0
    lens[:3] = (64, 1024, 0)
    if gaps == "odd_len":
        lens[1200] += 3
    gap = np.full(n, 4, np.int64) if gaps == "wire4" else rng.integers(0, 100, n).astype(np.int64)
    gap[rng.random(n) < 0.1] = 0  # some runs are contiguous
    offs = 20 + np.concatenate([[0], np.cumsum(lens[:-1] + gap[:-1])]).astype(np.int64)
    total = int(offs[-1] + lens[-1] + 64)
    if gaps == "reversed":  # segment 0 last in memory, segment n-1 first
        offs = total - 64 - offs - lens + 20
    inp = rng.integers(0, 256, total, dtype=np.uint8)
    key, iv = rng.bytes(32), rng.bytes(16)
    import fpnn_amd
    ks = fpnn_amd.KeySet(engine, key, 32, iv)
    kb, ib = np.frombuffer(key, np.uint8).copy(), np.frombuffer(iv, np.uint8).copy()
    shift = 80 if gaps == "shifted_out" else 0
    out_offs = offs + shift
    exp = np.zeros(total + shift, dtype=np.uint8) if shift else inp.copy()
    oracle.package_batch(False, inp, exp, n, in_off=offs.astype(np.uint64), out_off=out_offs.astype(np.uint64),
                         lens=lens.astype(np.uint32), keys=kb, keylen=32, ivs=ib, threads=8)
    src = to_dev(inp)
    dst = src if inplace else (dev_u8(total + shift) if shift else to_dev(inp))
    kw = dict(in_off=to_dev(offs), lens=to_dev(lens.astype(np.int32)))
    if shift:
        kw["out_off"] = to_dev(out_offs)
    engine.package_decrypt(src, dst, n, ks, **kw)
    torch.cuda.synchronize()
    assert np.array_equal(to_host(dst), exp)


@pytest.mark.parametrize("length", [32, 48, 1040, 1472, 1024, 2048, 3072, 4096])
@pytest.mark.parametrize("inplace", [False, True])
def test_dense_keyed_layout(engine, oracle, length, inplace):
    """Dense packets with one key slot each.  Whole 1 KiB chunks (the C5 shape): K1d
    with a wave-uniform key per step (U = 4, 2 or 1 chunks); other lengths (the U1
    shape): K1k with per-lane keys and packets starting inside chunks.  Mixed key
    lengths, a partial last chunk (777 packets)."""
    rng = np.random.default_rng(length + inplace)
    n, nkeys = 777, 97
    inp = rng.integers(0, 256, n * length + 64, dtype=np.uint8)
    for keylen in (16, 24, 32):
        keys = rng.integers(0, 256, nkeys * keylen, dtype=np.uint8)
        ivs = rng.integers(0, 256, nkeys * 16, dtype=np.uint8)
        slots = rng.integers(0, nkeys, n).astype(np.int32)
        ks = keyset(engine, keys, keylen, ivs)
        for encrypt in (True, False):
            exp = inp.copy()
            oracle.package_batch(encrypt, inp, exp, n, stride=length, uniform_len=length,
                                 key_slot=slots.astype(np.uint32), keys=keys, keylen=keylen, ivs=ivs, threads=8)
            src = to_dev(inp)
            dst = src if inplace else to_dev(inp)
            fn = engine.package_encrypt if encrypt else engine.package_decrypt
            fn(src, dst, n, ks, stride=length, uniform_len=length, key_slot=to_dev(slots))
            torch.cuda.synchronize()
            assert np.array_equal(to_host(dst), exp), (keylen, encrypt)


@pytest.mark.parametrize("keylen", [16, 32])
@pytest.mark.parametrize("eng_kind", ["engine", "hybrid_engine", "hybrid_lane_engine",
                                      "hybrid_quad_engine"])
def test_random_stream_batches(request, oracle, keylen, eng_kind):
    """Many streams, several successive calls each with random lengths; outputs and the
    carried (iv, pos) state must follow the reference byte loop exactly."""
    engine = request.getfixturevalue(eng_kind)
    rng = np.random.default_rng(500 + keylen)
    S = 333
    keys = rng.integers(0, 256, S * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, S * 16, dtype=np.uint8)
    ks = keyset(engine, keys, keylen, ivs)
    for encrypt in (True, False):
        iv_h = ivs.copy()
        pos_h = rng.integers(0, 16, S).astype(np.uint32)
        iv_d, pos_d = to_dev(iv_h), to_dev(pos_h.astype(np.int32))
        for call in range(6):
            lens = rng.integers(0, 200 if call % 2 else 2000, S).astype(np.int32)
            lens[rng.random(S) < 0.1] = 0
            offs = np.concatenate([[0], np.cumsum(lens[:-1] + 3)]).astype(np.int64)
            inp = rng.integers(0, 256, int(offs[-1] + lens[-1] + 16), dtype=np.uint8)
            exp = inp.copy()
            slots = np.arange(S, dtype=np.uint32)
            oracle.stream_batch(encrypt, inp, exp, S, in_off=offs.astype(np.uint64), out_off=offs.astype(np.uint64),
                                lens=lens.astype(np.uint32), key_slot=slots, keys=keys, keylen=keylen,
                                iv_state=iv_h, pos_state=pos_h, threads=8)
            src, dst = to_dev(inp), to_dev(inp)
            fn = engine.stream_encrypt if encrypt else engine.stream_decrypt
            fn(src, dst, S, ks, iv_d, pos_d, in_off=to_dev(offs), lens=to_dev(lens),
               key_slot=to_dev(slots.astype(np.int32)))
            torch.cuda.synchronize()
            assert np.array_equal(to_host(dst), exp), (encrypt, call)
            assert np.array_equal(to_host(iv_d), iv_h), (encrypt, call)
            assert np.array_equal(to_host(pos_d).astype(np.uint32), pos_h), (encrypt, call)


@pytest.mark.parametrize("length", [1024, 3072, 4096])
@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("arrays", [False, True])
def test_dense_stream_decrypt(engine, oracle, length, inplace, arrays):
    """Dense stream decrypt (the C3 shape: one key slot per stream, stride = length,
    whole 1 KiB chunks).  Calls where every stream sits at CFB position 0 run K1d keyed
    with the streams' carried IVs and write (last ciphertext block, 0) as the new state;
    a call with one stream mid-block falls back to K1.  With `arrays` the batch comes as
    offset arrays (in_off = s * length, checked on the device).  Output and (iv, pos)
    state must follow the reference byte loop (base/rijndael.c:1171-1201) call after call."""
    rng = np.random.default_rng(length + 7 * inplace + 13 * arrays)
    S = 333  # partial last chunk of the batch is irrelevant (whole chunks), odd stream count
    for keylen in (16, 32):
        keys = rng.integers(0, 256, S * keylen, dtype=np.uint8)
        ivs = rng.integers(0, 256, S * 16, dtype=np.uint8)
        ks = keyset(engine, keys, keylen, ivs)
        slots = rng.permutation(S).astype(np.uint32)
        iv_h, pos_h = ivs.copy(), np.zeros(S, dtype=np.uint32)
        iv_d, pos_d = to_dev(iv_h), to_dev(pos_h.astype(np.int32))
        offs = (np.arange(S, dtype=np.uint64) * length)
        lens = np.full(S, length, dtype=np.uint32)
        for call in range(4):
            if call == 2:  # one stream mid-block: the K1 fallback, then back to dense
                pos_h[S // 2] = 7
                pos_d[S // 2] = 7
            inp = rng.integers(0, 256, S * length, dtype=np.uint8)
            exp = inp.copy()
            oracle.stream_batch(False, inp, exp, S, in_off=offs, out_off=offs, lens=lens, key_slot=slots,
                                keys=keys, keylen=keylen, iv_state=iv_h, pos_state=pos_h, threads=8)
            src = to_dev(inp)
            dst = src if inplace else to_dev(inp)
            lay = dict(in_off=to_dev(offs.astype(np.int64))) if arrays else dict(stride=length)
            engine.stream_decrypt(src, dst, S, ks, iv_d, pos_d, uniform_len=length,
                                  key_slot=to_dev(slots.astype(np.int32)), **lay)
            torch.cuda.synchronize()
            assert np.array_equal(to_host(dst), exp), (keylen, call)
            assert np.array_equal(to_host(iv_d), iv_h), (keylen, call)
            assert np.array_equal(to_host(pos_d).astype(np.uint32), pos_h), (keylen, call)
            if call == 2:  # realign that stream for the last (dense) call
                pos_h[S // 2] = 0
                pos_d[S // 2] = 0


@pytest.mark.parametrize("encrypt", [True, False])
def test_long_stream_segments(engine, oracle, encrypt):
    """Few streams, segments of many 64-block chunks: every wave of a segment must see
    the state the call started from, not the one its last-block lane writes back."""
    rng = np.random.default_rng(77 + encrypt)
    S, keylen = 6, 16
    keys = rng.integers(0, 256, S * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, S * 16, dtype=np.uint8)
    ks = keyset(engine, keys, keylen, ivs)
    iv_h, pos_h = ivs.copy(), rng.integers(0, 16, S).astype(np.uint32)
    iv_d, pos_d = to_dev(iv_h), to_dev(pos_h.astype(np.int32))
    for call in range(4):
        lens = rng.integers(100_000, 300_000, S).astype(np.int32)
        offs = np.concatenate([[0], np.cumsum(lens[:-1] + 1)]).astype(np.int64)
        inp = rng.integers(0, 256, int(offs[-1] + lens[-1]), dtype=np.uint8)
        exp = inp.copy()
        slots = np.arange(S, dtype=np.uint32)
        oracle.stream_batch(encrypt, inp, exp, S, in_off=offs.astype(np.uint64), out_off=offs.astype(np.uint64),
                            lens=lens.astype(np.uint32), key_slot=slots, keys=keys, keylen=keylen,
                            iv_state=iv_h, pos_state=pos_h, threads=8)
        for inplace in ((False, True) if call == 3 else (False,)):
            if inplace:  # replay the last call in place from the same starting state
                iv_d, pos_d = to_dev(iv_prev), to_dev(pos_prev.astype(np.int32))
            else:
                iv_prev, pos_prev = to_host(iv_d).copy(), to_host(pos_d).astype(np.uint32).copy()
            src = to_dev(inp)
            dst = src if inplace else to_dev(inp)
            fn = engine.stream_encrypt if encrypt else engine.stream_decrypt
            fn(src, dst, S, ks, iv_d, pos_d, in_off=to_dev(offs), lens=to_dev(lens),
               key_slot=to_dev(slots.astype(np.int32)))
            torch.cuda.synchronize()
            assert np.array_equal(to_host(dst), exp), (call, inplace)
            assert np.array_equal(to_host(iv_d), iv_h) and np.array_equal(to_host(pos_d).astype(np.uint32), pos_h)


def test_empty_and_degenerate(engine):
    import fpnn_amd
    ks = fpnn_amd.KeySet(engine, bytes(32), 32, bytes(16))
    t = dev_u8(64)
    engine.package_encrypt(t, t, 0, ks, stride=16, uniform_len=16)
    engine.package_decrypt(t, t, 0, ks, stride=16, uniform_len=16)
    engine.package_encrypt(t, t, 3, ks, stride=16, uniform_len=0)
    engine.package_decrypt(t, t, 3, ks, stride=16, uniform_len=0)
    torch.cuda.synchronize()
    assert int(t.sum()) == 0
    with pytest.raises(fpnn_amd.FpnnAesError):
        fpnn_amd.KeySet(engine, bytes(20), 20, bytes(16))


# --------------------------------------------------------------------------------------
# full-size configs (BASELINE.json configs[1..4]) against reference digests / oracle


@pytest.mark.slow
def test_c2_full_digest(engine, golden):
    import fpnn_amd
    d = golden("digests.json")["C2"]
    c = W.C2
    P, L = c["packets"], c["length"]
    key, iv = W.single_key(c)
    ks = fpnn_amd.KeySet(engine, key, len(key), iv)
    plain = torch.empty(P * L, dtype=torch.uint8, device=DEV)
    engine.fill_synthetic(plain, c["payload_seed"])
    cipher = torch.empty_like(plain)
    engine.package_encrypt(plain, cipher, P, ks, stride=L, uniform_len=L)
    back = torch.empty_like(plain)
    engine.package_decrypt(cipher, back, P, ks, stride=L, uniform_len=L)
    torch.cuda.synchronize()
    assert hashlib.sha256(to_host(plain)).hexdigest() == d["plain_sha256"]
    assert hashlib.sha256(to_host(cipher)).hexdigest() == d["cipher_sha256"]
    assert torch.equal(back, plain)


@pytest.mark.slow
def test_c5_full_digest(engine, golden):
    d = golden("digests.json")["C5"]
    c = W.C5
    P, L = c["packets"], c["length"]
    keys, ivs = W.many_keys(c)
    ks = keyset(engine, keys, c["keylen"], ivs)
    slots = torch.arange(P, dtype=torch.int32, device=DEV)
    plain = torch.empty(P * L, dtype=torch.uint8, device=DEV)
    engine.fill_synthetic(plain, c["payload_seed"])
    cipher = torch.empty_like(plain)
    engine.package_encrypt(plain, cipher, P, ks, stride=L, uniform_len=L, key_slot=slots)
    back = torch.empty_like(plain)
    engine.package_decrypt(cipher, back, P, ks, stride=L, uniform_len=L, key_slot=slots)
    torch.cuda.synchronize()
    assert hashlib.sha256(to_host(cipher)).hexdigest() == d["cipher_sha256"]
    assert torch.equal(back, plain)


@pytest.mark.slow
def test_c3_full_stream_digest(engine, golden):
    """4096 streams x 4 MiB AES-128, each stream cut into random frames (1 B .. 64 KiB)
    submitted as successive stream-mode calls; whole-stream digests must match the
    reference's, and decryption with a different cut must restore the plaintext."""
    d = golden("digests.json")["C3"]
    c = W.C3
    S, L = c["streams"], c["length"]
    keys, ivs = W.many_keys(c)
    ks = keyset(engine, keys, c["keylen"], ivs)
    plain = torch.empty(S * L, dtype=torch.uint8, device=DEV)
    engine.fill_synthetic(plain, c["payload_seed"])
    cipher = torch.empty_like(plain)
    slots = torch.arange(S, dtype=torch.int32, device=DEV)
    base = torch.arange(S, dtype=torch.int64, device=DEV) * L

    def run(fn, src, dst, split_salt):
        splits = [W.stream_splits(c, s if split_salt == 0 else s + 100000) for s in range(S)]
        nmax = max(len(x) for x in splits)
        lens = np.zeros((nmax, S), dtype=np.int32)
        for s, x in enumerate(splits):
            lens[:len(x), s] = x
        starts = np.cumsum(np.vstack([np.zeros((1, S), np.int64), lens[:-1]]), axis=0)
        iv_state = to_dev(ivs.copy())
        pos_state = torch.zeros(S, dtype=torch.int32, device=DEV)
        for f in range(nmax):
            offs = base + to_dev(starts[f])
            fn(src, dst, S, ks, iv_state, pos_state, in_off=offs, lens=to_dev(lens[f]), key_slot=slots)
        torch.cuda.synchronize()

    run(engine.stream_encrypt, plain, cipher, 0)
    host = to_host(cipher)
    per = [hashlib.sha256(host[s * L:(s + 1) * L]).digest() for s in range(S)]
    assert per[0].hex() == d["first_stream_sha256"]
    assert hashlib.sha256(b"".join(per)).hexdigest() == d["stream_digests_sha256"]
    back = torch.empty_like(plain)
    run(engine.stream_decrypt, cipher, back, 1)
    assert torch.equal(back, plain)


@pytest.mark.slow
def test_c4_zipf_vs_oracle(engine, oracle):
    import fpnn_amd
    c = W.C4
    sizes = W.zipf_sizes(c)
    n = len(sizes)
    offs = np.concatenate([[0], np.cumsum(sizes[:-1].astype(np.int64))]).astype(np.int64)
    total = int(offs[-1] + sizes[-1])
    key, iv = W.single_key(c)
    ks = fpnn_amd.KeySet(engine, key, len(key), iv)
    plain = torch.empty(total, dtype=torch.uint8, device=DEV)
    engine.fill_synthetic(plain, c["payload_seed"])
    cipher = torch.empty_like(plain)
    kw = dict(in_off=to_dev(offs), lens=to_dev(sizes.astype(np.int32)))
    engine.package_encrypt(plain, cipher, n, ks, **kw)
    back = torch.empty_like(plain)
    engine.package_decrypt(cipher, back, n, ks, **kw)
    torch.cuda.synchronize()
    inp = to_host(plain)
    exp = np.empty_like(inp)
    oracle.package_batch(True, inp, exp, n, in_off=offs.astype(np.uint64), lens=sizes.astype(np.uint32),
                         keys=np.frombuffer(key, np.uint8).copy(), keylen=len(key),
                         ivs=np.frombuffer(iv, np.uint8).copy(), threads=min(16, os.cpu_count() or 1))
    got = to_host(cipher)
    assert np.array_equal(got, exp)
    assert torch.equal(back, plain)
    # and against the reference itself: digests.json "shards" C4/w1/r0 is the whole batch
    # encrypted by base/rijndael.c + core/Encryptor.cpp (oracle/_ref, oracle/gen_golden.py)
    gold = load_golden("digests.json")["shards"]["C4/w1/r0"]
    assert hashlib.sha256(got.tobytes()).hexdigest() == gold


# --------------------------------------------------------------------------------------
# the C++ drop-in surface (include/Encryptor.h, include/rijndael.h) used as FPNN uses it


def test_cpp_dropin_matches_reference(golden, tmp_path):
    from test_abi import build_dropin
    exe = build_dropin(tmp_path)
    lines, expect = [], []
    for c in golden("package_cases.json"):
        lines.append(f"P {c['key']} {c['iv']} {c['in'] or '-'}")
        expect.append(f"{c['encrypt'] or '-'} {c['decrypt'] or '-'} {c['frame']}")
    for c in golden("stream_cases.json"):
        frames = [f for f in c["frames"]]
        lines.append(f"S {'E' if c['encrypt'] else 'D'} {c['key']} {c['iv']} " +
                     " ".join(f["in"] or "-" for f in frames))
        expect.append(" ".join(f["out"] or "-" for f in frames))
    demo = golden("package_cases.json")[-1]  # base/test/rijndaelDemo.cpp inputs
    lines.append(f"R {demo['key']} {demo['iv']} {demo['in']}")
    expect.append(f"0 {demo['encrypt']}")
    import subprocess
    res = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr
    got = res.stdout.strip().split("\n")
    assert got == expect


def test_cpp_encryptor_batch_matches_reference(golden, tmp_path, oracle):
    """fpnn::EncryptorBatch (include/EncryptorBatch.h): the golden package/stream cases,
    all queued on one batch across many encryptors and flushed at once, give the
    reference's outputs; plus random many-connection cases checked against the oracle."""
    from test_abi import build_dropin
    exe = build_dropin(tmp_path)
    lines, expect = [], []
    for c in golden("package_cases.json"):
        lines.append(f"BP {c['key']} {c['iv']} {c['in'] or '-'}")
        expect.append(f"{c['encrypt'] or '-'} {c['decrypt'] or '-'} {c['frame']}")
    for c in golden("stream_cases.json"):
        lines.append(f"BS {'E' if c['encrypt'] else 'D'} {c['key']} {c['iv']} " +
                     " ".join(f["in"] or "-" for f in c["frames"]))
        expect.append(" ".join(f["out"] or "-" for f in c["frames"]))
    lines.append("F")
    rng = np.random.default_rng(31337)
    for conn in range(300):  # a second flush: many connections, mixed key lengths
        kl = (16, 24, 32)[conn % 3]
        key, iv = rng.bytes(kl), rng.bytes(16)
        if conn % 2:
            data = rng.bytes(int(rng.integers(0, 3000)))
            lines.append(f"BP {key.hex()} {iv.hex()} {data.hex() or '-'}")
            expect.append(f"{oracle.package(key, iv, True, data).hex() or '-'} "
                          f"{oracle.package(key, iv, False, data).hex() or '-'} {oracle.package_frame(key, iv, data).hex()}")
        else:
            enc = bool(conn % 4)
            frames = [rng.bytes(int(rng.integers(0, 700))) for _ in range(int(rng.integers(1, 6)))]
            outs, st_iv, st_pos = [], iv, 0
            for f in frames:
                o, st_iv, st_pos = oracle.cfb(key, enc, f, st_iv, st_pos)
                outs.append(o.hex() or "-")
            lines.append(f"BS {'E' if enc else 'D'} {key.hex()} {iv.hex()} " + " ".join(f.hex() or "-" for f in frames))
            expect.append(" ".join(outs))
    lines.append("F")
    # StreamEncryptor::encrypt(std::string*) of "" queued FIRST on a stream, then real frames
    # in both forms (the empty op used to mark the encryptor as listed without
    # grouping it, so its (iv, pos) was never staged nor taken back)
    for conn in range(24):
        kl = (16, 32)[conn % 2]
        key, iv = rng.bytes(kl), rng.bytes(16)
        frames = [b""] + [rng.bytes(int(rng.integers(1, 700))) for _ in range(int(rng.integers(1, 5)))]
        if conn % 3 == 0:
            frames.insert(2, b"")
        toks, outs, st_iv, st_pos = [], [], iv, 0
        for j, f in enumerate(frames):
            o, st_iv, st_pos = oracle.cfb(key, True, f, st_iv, st_pos)
            outs.append(o.hex() or "-")
            toks.append(("s" + (f.hex() or "-")) if (j + conn) % 2 == 0 or not f else (f.hex() or "-"))
        lines.append(f"BS E {key.hex()} {iv.hex()} " + " ".join(toks))
        expect.append(" ".join(outs))
    lines.append("F")
    import subprocess
    res = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr
    assert res.stdout.strip().split("\n") == expect


# --------------------------------------------------------------------------------------
# many frames straight from host memory (fpnn_aes_package_host: gather -> pinned ->
# pipelined H2D / kernel / D2H -> scatter)


@pytest.mark.parametrize("wire_prefix", [False, True])
def test_package_host_frames(engine, oracle, wire_prefix):
    import fpnn_amd
    rng = np.random.default_rng(4242 + wire_prefix)
    nkeys, keylen = 5, 32
    keys = rng.integers(0, 256, nkeys * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, nkeys * 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), keylen, ivs.tobytes())
    lens = list(rng.integers(0, 5000, 3000)) + [0, 1, 16, 17, 40 << 20]  # one frame > a pipeline chunk
    frames, srcs = [], []
    for i, L in enumerate(lens):
        src = rng.integers(0, 256, int(L), dtype=np.uint8)
        dst = np.zeros(int(L) + (4 if wire_prefix else 0), dtype=np.uint8)
        frames.append((src, dst, i % nkeys))
        srcs.append(src)
    engine.package_host(True, frames, ks, wire_prefix=wire_prefix)
    for src, dst, slot in frames[:400] + frames[-5:]:
        k = keys[slot * keylen:(slot + 1) * keylen].tobytes()
        v = ivs[slot * 16:(slot + 1) * 16].tobytes()
        exp = oracle.package_frame(k, v, src.tobytes()) if wire_prefix else oracle.package(k, v, True, src.tobytes())
        assert dst.tobytes() == exp
    if not wire_prefix:  # decrypt back, in place
        back = [(d.copy(), None, sl) for _, d, sl in frames]
        engine.package_host(False, [(c, c, sl) for c, _, sl in back], ks)
        for (c, _, _), src in zip(back, srcs):
            assert np.array_equal(c, src)


@pytest.mark.parametrize("keylen", [16, 32])
def test_stream_host_frames(engine, oracle, keylen):
    """fpnn_aes_stream_host: frames of many streams interleaved in one call, each
    stream's frames in order, equal to successive StreamEncryptor calls; one stream
    is longer than a pipeline chunk (split across chunks, state chained)."""
    import fpnn_amd
    rng = np.random.default_rng(777 + keylen)
    ns = 37
    keys = rng.integers(0, 256, ns * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, ns * 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), keylen, ivs.tobytes())
    iv0 = rng.integers(0, 256, (ns, 16), dtype=np.uint8)
    pos0 = rng.integers(0, 16, ns).astype(np.uint32)
    pos0[:3] = 0
    frames = []
    for i in range(2500):
        s = int(rng.integers(0, ns - 1))  # stream ns-1 is untouched: state must stay
        L = int(rng.choice([0, 1, 15, 16, 17, int(rng.integers(0, 3000))]))
        frames.append((rng.integers(0, 256, L, dtype=np.uint8), s))
    big = 3
    frames.insert(100, (rng.integers(0, 256, 21 << 20, dtype=np.uint8), big))
    frames.insert(900, (rng.integers(0, 256, (19 << 20) + 5, dtype=np.uint8), big))
    outs = [np.zeros_like(f) for f, _ in frames]
    iv_s, pos_s = iv0.copy(), pos0.copy()
    engine.stream_host(True, [(f, o, s) for (f, s), o in zip(frames, outs)], ks, iv_s, pos_s)
    # oracle: per stream, successive calls
    st = {s: (iv0[s].tobytes(), int(pos0[s])) for s in range(ns)}
    for (f, s), o in zip(frames, outs):
        k = keys[s * keylen:(s + 1) * keylen].tobytes()
        exp, iv, pos = oracle.cfb(k, True, f.tobytes(), st[s][0], st[s][1])
        st[s] = (iv, pos)
        assert o.tobytes() == exp, s
    for s in range(ns):
        assert iv_s[s].tobytes() == st[s][0] and int(pos_s[s]) == st[s][1], s
    # decrypt in place from the initial state
    iv_d, pos_d = iv0.copy(), pos0.copy()
    bufs = [o.copy() for o in outs]
    engine.stream_host(False, [(b, b, s) for b, (_, s) in zip(bufs, frames)], ks, iv_d, pos_d)
    for b, (f, _) in zip(bufs, frames):
        assert np.array_equal(b, f)
    assert np.array_equal(iv_d, iv_s) and np.array_equal(pos_d, pos_s)


# --------------------------------------------------------------------------------------
# receive side: wire framing on the device (fpnn_aes_package_recv / fpnn_aes_stream_recv)


def _package_wire(rng, oracle, key, iv, nframes, max_len, partial, oversize):
    wire, plain_bodies = b"", []
    for j in range(nframes):
        if oversize and j == 2:
            wire += (max_len + 1 + int(rng.integers(0, 100))).to_bytes(4, "little") + rng.bytes(50)
            return wire, plain_bodies
        body = rng.bytes(int(rng.choice([0, 1, 16, int(rng.integers(0, max_len + 1))])))
        plain_bodies.append(body)
        wire += len(body).to_bytes(4, "little") + oracle.package(key, iv, True, body)
    if partial:
        body = rng.bytes(int(rng.integers(1, 600)))
        full = len(body).to_bytes(4, "little") + oracle.package(key, iv, True, body)
        wire += full[:int(rng.integers(1, len(full)))]
    return wire, plain_bodies


@pytest.mark.parametrize("inplace", [False, True])
def test_package_recv_frames(engine, oracle, inplace, scan_mode):
    import fpnn_amd
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as PO
    rng = np.random.default_rng(2024 + inplace)
    nconn, keylen, max_len, max_frames = 60, 32, 3000, 12
    keys = rng.integers(0, 256, nconn * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, nconn * 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), keylen, ivs.tobytes())
    segs, bodies = [], []
    for c in range(nconn):
        k, v = keys[c * keylen:(c + 1) * keylen].tobytes(), ivs[c * 16:(c + 1) * 16].tobytes()
        w, b = _package_wire(rng, oracle, k, v, int(rng.integers(0, 16)), max_len, partial=c % 3 == 1,
                             oversize=c % 11 == 4)
        segs.append(w)
        bodies.append(b)
    offs = np.cumsum([0] + [len(w) + 7 for w in segs[:-1]]).astype(np.int64)  # ragged, unaligned
    total = int(offs[-1] + len(segs[-1]) + 7)
    host = np.zeros(total, dtype=np.uint8)
    for o, w in zip(offs, segs):
        host[o:o + len(w)] = np.frombuffer(w, np.uint8)
    inp = torch.from_numpy(host).to(DEV)
    out = inp if inplace else torch.full_like(inp, 0xA5)
    lens = torch.tensor([len(w) for w in segs], dtype=torch.int32, device=DEV)
    slots = torch.arange(nconn, dtype=torch.int32, device=DEV)
    foff, flen, scan = engine.package_recv(inp, out, nconn, ks, max_len, max_frames, in_off=torch.from_numpy(offs).to(DEV),
                                           lens=lens, key_slot=slots)
    torch.cuda.synchronize()
    frames, status, consumed = fpnn_amd.Engine.decode_scan(scan)
    foff, flen, res = foff.cpu().numpy(), flen.cpu().numpy(), out.cpu().numpy()
    for c in range(nconn):
        exp_frames, exp_status, exp_consumed = PO.scan_package(segs[c], max_len, max_frames)
        assert (frames[c], status[c], consumed[c]) == (len(exp_frames), exp_status, exp_consumed), c
        for j, (bo, n) in enumerate(exp_frames):
            assert (foff[c * max_frames + j], flen[c * max_frames + j]) == (bo, n)
            got = res[offs[c] + bo: offs[c] + bo + n].tobytes()
            assert got == bodies[c][j], (c, j)
        if not inplace:  # nothing but complete bodies was written
            mask = np.ones(len(segs[c]), bool)
            for bo, n in exp_frames:
                mask[bo:bo + n] = False
            assert (res[offs[c]:offs[c] + len(segs[c])][mask] == 0xA5).all(), c
    assert (status == PO.SCAN_FULL).any() and (status == PO.SCAN_TOO_LARGE).any()


@pytest.mark.parametrize("inplace", [False, True])
def test_package_recv_quests_whole_frames(engine, inplace):
    """fpnn_aes_package_recv with a frame-size cap of 175 B over 16 384 connections x 16
    frame slots: every accepted frame is within the cap, so the decrypt behind the scan takes
    D2s (one lane per frame).  FPNN's 145-B quests (and a spread of shorter ones, empty
    included) as wire frames htole32(len) || C made by the wire encrypt, received and
    deciphered back to the plaintext."""
    import fpnn_amd
    rng = np.random.default_rng(3131 + inplace)
    nconn, per, cap = 16384, 16, 175
    keys = rng.integers(0, 256, nconn * 32, dtype=np.uint8)
    ivs = rng.integers(0, 256, nconn * 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), 32, ivs.tobytes())
    nfr = rng.integers(0, per + 1, nconn)  # frames per connection
    lens = np.where(rng.random((nconn, per)) < 0.6, 145, rng.integers(0, cap + 1, (nconn, per)))
    lens[np.arange(per)[None, :] >= nfr[:, None]] = 0
    flat_len = lens.reshape(-1).astype(np.int64)
    conn = np.repeat(np.arange(nconn), per)
    wire_len = np.where(np.arange(per)[None, :] < nfr[:, None], lens + 4, 0)
    seg_len = wire_len.sum(1)
    seg_off = np.concatenate([[0], np.cumsum(seg_len[:-1] + 3)]).astype(np.int64)
    wout = (seg_off[:, None] + np.concatenate([np.zeros((nconn, 1), np.int64), np.cumsum(wire_len, 1)[:, :-1]], 1))
    plain_off = np.concatenate([[0], np.cumsum(flat_len[:-1])]).astype(np.int64)
    plain = rng.integers(0, 256, int(flat_len.sum()) + 1, dtype=np.uint8)
    live = (np.arange(per)[None, :] < nfr[:, None]).reshape(-1)
    n = int(live.sum())
    wire = torch.zeros(int(seg_off[-1] + seg_len[-1] + 3), dtype=torch.uint8, device=DEV)
    engine.package_encrypt(to_dev(plain), wire, n, ks, wire_prefix=True, max_len=cap,
                           in_off=to_dev(plain_off[live]), out_off=to_dev(wout.reshape(-1)[live]),
                           lens=to_dev(flat_len[live].astype(np.int32)), key_slot=to_dev(conn[live].astype(np.int32)))
    out = wire if inplace else torch.zeros_like(wire)
    foff, flen, scan = engine.package_recv(wire, out, nconn, ks, cap, per, in_off=to_dev(seg_off),
                                           lens=to_dev(seg_len.astype(np.int32)),
                                           key_slot=to_dev(np.arange(nconn, dtype=np.int32)))
    torch.cuda.synchronize()
    assert engine.last_kernel(fpnn_amd.K_DECRYPT) == "cfb_decrypt_frames"
    frames, status, consumed = fpnn_amd.Engine.decode_scan(scan)
    assert (frames == nfr).all() and (consumed == seg_len).all()
    res, fo, fl = to_host(out), to_host(foff), to_host(flen)
    got_idx = (seg_off[:, None] + fo.reshape(nconn, per).astype(np.int64)).reshape(-1)[live]
    assert (fl.reshape(-1)[live] == flat_len[live]).all()
    for i in np.nonzero(live)[0][rng.permutation(int(live.sum()))[:20000]]:
        o, ln, po = int(seg_off[conn[i]] + fo[i]), int(flat_len[i]), int(plain_off[i])
        assert np.array_equal(res[o:o + ln], plain[po:po + ln]), i
    assert len(got_idx) == n


def _fpnn_message(rng, mtype, ss, psize):
    hdr = b"FPNN" + bytes([1, 0x80, mtype, ss]) + psize.to_bytes(4, "little")
    body = {1: psize + ss + 4, 2: psize + 4, 0: psize + ss}[mtype]
    return hdr + rng.bytes(body)


def test_stream_recv_messages(engine, oracle, scan_mode):
    """Two receive calls per stream: the first ends mid-message, its plaintext tail is
    carried in front of the second call's segment; malformed headers stop the scan with
    the reference's verdict."""
    import fpnn_amd
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as PO
    rng = np.random.default_rng(99)
    ns, keylen, max_len, max_frames = 40, 16, 6000, 64
    keys = rng.integers(0, 256, ns * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, ns * 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), keylen, ivs.tobytes())
    plains = []
    for s in range(ns):
        msgs = [_fpnn_message(rng, int(rng.integers(0, 3)), int(rng.integers(0, 30)), int(rng.integers(0, 2000)))
                for _ in range(int(rng.integers(0, 12)))]
        bad = s % 8
        if bad == 1:
            msgs.append(b"FPNX" + bytes(20))
        elif bad == 2:
            msgs.append(b"FPNN" + bytes([1, 0, 7, 0]) + bytes(8))
        elif bad == 3:
            msgs.append(b"FPNN" + bytes([1, 0, 0, 0]) + (0).to_bytes(4, "little"))  # BodyLen 0
        elif bad == 4:
            msgs.append(b"FPNN" + bytes([1, 0, 0, 0]) + (0x80000000).to_bytes(4, "little"))  # negative int
        elif bad == 5:
            msgs.append(_fpnn_message(rng, 2, 0, max_len))  # 12 + BodyLen > max_len
        elif bad == 6:
            msgs.append(b"FPNN" + bytes([1, 0, 2, 0]) + (0xFFFFFFFF).to_bytes(4, "little") + rng.bytes(3))  # wraps
        plains.append(b"".join(msgs))
    iv0 = ivs.reshape(ns, 16)
    ciphers = [oracle.cfb(keys[s * keylen:(s + 1) * keylen].tobytes(), True, plains[s], iv0[s].tobytes(), 0)[0]
               for s in range(ns)]
    cut = [int(rng.integers(0, len(p) + 1)) for p in plains]
    CARRY = max_len + 16
    slot = CARRY + max(len(p) for p in plains) + 32
    in_off = np.arange(ns, dtype=np.int64) * slot + CARRY
    d_iv = torch.from_numpy(iv0.copy()).to(DEV)
    d_pos = torch.zeros(ns, dtype=torch.int32, device=DEV)
    slots = torch.arange(ns, dtype=torch.int32, device=DEV)
    out = torch.zeros(ns * slot, dtype=torch.uint8, device=DEV)
    carry = np.zeros(ns, dtype=np.int32)
    for call in range(2):
        parts = [c[:k] if call == 0 else c[k:] for c, k in zip(ciphers, cut)]
        host = np.zeros(ns * slot, dtype=np.uint8)
        for s, p in enumerate(parts):
            host[in_off[s]:in_off[s] + len(p)] = np.frombuffer(p, np.uint8)
        inp = torch.from_numpy(host).to(DEV)
        foff, flen, scan = engine.stream_recv(inp, out, ns, ks, d_iv, d_pos, max_len, max_frames,
                                              carry=torch.from_numpy(carry).to(DEV),
                                              in_off=torch.from_numpy(in_off).to(DEV),
                                              lens=torch.tensor([len(p) for p in parts], dtype=torch.int32, device=DEV),
                                              key_slot=slots)
        torch.cuda.synchronize()
        frames, status, consumed = fpnn_amd.Engine.decode_scan(scan)
        foff, flen, res = foff.cpu().numpy(), flen.cpu().numpy(), out.cpu().numpy()
        new_carry = np.zeros(ns, dtype=np.int32)
        for s in range(ns):
            start = 0 if call == 0 else cut[s] - int(carry[s])
            region = plains[s][start:cut[s]] if call == 0 else plains[s][start:]
            got_region = res[in_off[s] - carry[s]: in_off[s] - carry[s] + len(region)].tobytes()
            assert got_region == region, (call, s)  # decrypted plaintext incl. the carried tail
            exp_frames, exp_status, exp_consumed = PO.scan_stream(region, max_len, max_frames)
            assert (frames[s], status[s], consumed[s]) == (len(exp_frames), exp_status, exp_consumed), (call, s)
            for j, (o, n) in enumerate(exp_frames):
                assert (foff[s * max_frames + j], flen[s * max_frames + j]) == (o, n)
            if call == 0 and exp_status == PO.SCAN_OK:  # keep the incomplete message's plaintext
                tail = region[exp_consumed:]
                new_carry[s] = len(tail)
                res[in_off[s] - len(tail): in_off[s]] = np.frombuffer(tail, np.uint8)
        if call == 0:
            out = torch.from_numpy(res).to(DEV)
            carry = new_carry  # streams stopped by a bad header carry nothing
    # after both calls the stream state equals the oracle's over the whole stream
    for s in range(ns):
        _, iv_end, pos_end = oracle.cfb(keys[s * keylen:(s + 1) * keylen].tobytes(), True, plains[s],
                                        iv0[s].tobytes(), 0)
        assert d_iv[s].cpu().numpy().tobytes() == iv_end and int(d_pos[s]) == pos_end


def _runs(rng, total, maxlen):
    """Frame lengths in runs of equal length (the wave walk's guess holds inside a run)."""
    out = []
    while len(out) < total:
        out += [int(rng.integers(0, maxlen + 1))] * int(rng.choice([1, 2, 5, 63, 64, 65, 130]))
    return out[:total]


def test_recv_runs_of_equal_frames(engine, oracle, scan_mode):
    """Both receive modes over connections whose frames come in runs of equal length, the
    runs ending in every way the walk can stop: end of data, a partial frame, an oversize
    prefix / bad header after a run, and max_frames reached inside a run."""
    import fpnn_amd
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as PO
    rng = np.random.default_rng(77)
    nconn, keylen, max_len, max_frames = 24, 16, 3000, 200
    keys = rng.integers(0, 256, nconn * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, nconn * 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), keylen, ivs.tobytes())
    kv = [(keys[c * keylen:(c + 1) * keylen].tobytes(), ivs[c * 16:(c + 1) * 16].tobytes()) for c in range(nconn)]

    def layout(segs):
        offs = np.cumsum([0] + [len(w) + 3 for w in segs[:-1]]).astype(np.int64)
        host = np.zeros(int(offs[-1] + len(segs[-1]) + 3), dtype=np.uint8)
        for o, w in zip(offs, segs):
            host[o:o + len(w)] = np.frombuffer(w, np.uint8)
        lens = torch.tensor([len(w) for w in segs], dtype=torch.int32, device=DEV)
        return offs, host, lens

    # package mode
    segs, bodies = [], []
    for c in range(nconn):
        k, v = kv[c]
        nfr = 250 if c % 4 == 3 else int(rng.integers(0, 190))
        bs = [rng.bytes(n) for n in _runs(rng, nfr, 300)]
        wire = b"".join(len(b).to_bytes(4, "little") + oracle.package(k, v, True, b) for b in bs)
        if c % 4 == 1:
            wire += (200).to_bytes(4, "little") + rng.bytes(int(rng.integers(0, 200)))
        elif c % 4 == 2:
            wire += (max_len + 1).to_bytes(4, "little") + rng.bytes(64)
        segs.append(wire)
        bodies.append(bs)
    offs, host, lens = layout(segs)
    inp = torch.from_numpy(host).to(DEV)
    out = torch.zeros_like(inp)
    foff, flen, scan = engine.package_recv(inp, out, nconn, ks, max_len, max_frames,
                                           in_off=torch.from_numpy(offs).to(DEV), lens=lens,
                                           key_slot=torch.arange(nconn, dtype=torch.int32, device=DEV))
    torch.cuda.synchronize()
    frames, status, consumed = fpnn_amd.Engine.decode_scan(scan)
    foff, flen, res = foff.cpu().numpy(), flen.cpu().numpy(), out.cpu().numpy()
    for c in range(nconn):
        ef, es, ec = PO.scan_package(segs[c], max_len, max_frames)
        assert (frames[c], status[c], consumed[c]) == (len(ef), es, ec), c
        assert [tuple(x) for x in zip(foff[c * max_frames:c * max_frames + len(ef)],
                                      flen[c * max_frames:c * max_frames + len(ef)])] == ef, c
        assert (flen[c * max_frames + len(ef):(c + 1) * max_frames] == 0).all(), c
        for j, (bo, n) in enumerate(ef):
            assert res[offs[c] + bo:offs[c] + bo + n].tobytes() == bodies[c][j], (c, j)
    assert set(status.tolist()) == {PO.SCAN_OK, PO.SCAN_TOO_LARGE, PO.SCAN_FULL}

    # stream mode: runs of identical message headers
    plains = []
    for c in range(nconn):
        nmsg = 250 if c % 4 == 3 else int(rng.integers(0, 190))
        msgs, i = [], 0
        while i < nmsg:
            run = min(nmsg - i, int(rng.choice([1, 3, 64, 65, 100])))
            mt, ss, ps = int(rng.integers(0, 3)), int(rng.integers(0, 8)), int(rng.integers(0, 200))
            msgs += [_fpnn_message(rng, mt, ss, ps) for _ in range(run)]
            i += run
        if c % 4 == 1:
            msgs.append(_fpnn_message(rng, 2, 0, 100)[:50])  # partial
        elif c % 4 == 2:
            msgs.append(b"FPNX" + bytes(20))
        plains.append(b"".join(msgs))
    ciphers = [oracle.cfb(kv[c][0], True, plains[c], kv[c][1], 0)[0] for c in range(nconn)]
    offs, host, lens = layout(ciphers)
    inp = torch.from_numpy(host).to(DEV)
    out = torch.zeros_like(inp)
    d_iv = torch.from_numpy(ivs.copy()).to(DEV)
    d_pos = torch.zeros(nconn, dtype=torch.int32, device=DEV)
    foff, flen, scan = engine.stream_recv(inp, out, nconn, ks, d_iv, d_pos, max_len, max_frames,
                                          in_off=torch.from_numpy(offs).to(DEV), lens=lens,
                                          key_slot=torch.arange(nconn, dtype=torch.int32, device=DEV))
    torch.cuda.synchronize()
    frames, status, consumed = fpnn_amd.Engine.decode_scan(scan)
    foff, flen, res = foff.cpu().numpy(), flen.cpu().numpy(), out.cpu().numpy()
    for c in range(nconn):
        assert res[offs[c]:offs[c] + len(plains[c])].tobytes() == plains[c], c
        ef, es, ec = PO.scan_stream(plains[c], max_len, max_frames)
        assert (frames[c], status[c], consumed[c]) == (len(ef), es, ec), c
        assert [tuple(x) for x in zip(foff[c * max_frames:c * max_frames + len(ef)],
                                      flen[c * max_frames:c * max_frames + len(ef)])] == ef, c
    assert set(status.tolist()) == {PO.SCAN_OK, PO.SCAN_BAD_MAGIC, PO.SCAN_FULL}


def test_udp_datagram_batches(engine, oracle):
    """SURVEY.md 8f row 2, UDP v2 shape: MTU-sized datagrams of many connections (whole-
    datagram package encryption, UDPEncryptor::packageEncrypt/Decrypt) and the
    reinforced data stream (UDPEncryptor::dataEncrypt, a StreamEncryptor per
    connection), as one device batch and as host frames."""
    import fpnn_amd
    rng = np.random.default_rng(1472)
    nconn, n = 97, 3000
    for keylen in (16, 32):  # non-reinforced / reinforced key length
        keys = rng.integers(0, 256, nconn * keylen, dtype=np.uint8)
        ivs = rng.integers(0, 256, nconn * 16, dtype=np.uint8)
        ks = fpnn_amd.KeySet(engine, keys.tobytes(), keylen, ivs.tobytes())
        lens = rng.choice([548, 1472, int(rng.integers(1, 1473))], n).astype(np.int32)
        conn = rng.integers(0, nconn, n).astype(np.int32)
        offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.int64))])
        data = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
        exp = np.empty_like(data)
        for i in range(n):
            k = keys[conn[i] * keylen:(conn[i] + 1) * keylen].tobytes()
            v = ivs[conn[i] * 16:(conn[i] + 1) * 16].tobytes()
            exp[offs[i]:offs[i] + lens[i]] = np.frombuffer(
                oracle.package(k, v, True, data[offs[i]:offs[i] + lens[i]].tobytes()), np.uint8)
        d_in = torch.from_numpy(data).to(DEV)
        d_out = torch.empty_like(d_in)
        kw = dict(in_off=torch.from_numpy(offs).to(DEV), lens=torch.from_numpy(lens).to(DEV),
                  key_slot=torch.from_numpy(conn).to(DEV))
        engine.package_encrypt(d_in, d_out, n, ks, **kw)
        torch.cuda.synchronize()
        assert np.array_equal(d_out.cpu().numpy(), exp)
        dst = np.empty_like(data)
        fr = np.zeros(n, dtype=fpnn_amd.engine.HOST_FRAME_DTYPE)
        fr["src"] = data.ctypes.data + offs.astype(np.uint64)
        fr["dst"] = dst.ctypes.data + offs.astype(np.uint64)
        fr["len"] = lens
        fr["key_slot"] = conn
        engine.package_host_array(True, fr, ks)
        assert np.array_equal(dst, exp)
        # reinforced data stream: each connection's datagram payloads in send order
        iv_s = ivs.reshape(nconn, 16).copy()
        pos_s = np.zeros(nconn, dtype=np.uint32)
        engine.stream_host_array(True, fr, ks, iv_s, pos_s)
        st = {c: (ivs[c * 16:(c + 1) * 16].tobytes(), 0) for c in range(nconn)}
        for i in range(n):
            k = keys[conn[i] * keylen:(conn[i] + 1) * keylen].tobytes()
            o, iv2, p2 = oracle.cfb(k, True, data[offs[i]:offs[i] + lens[i]].tobytes(), *st[conn[i]])
            st[conn[i]] = (iv2, p2)
            assert dst[offs[i]:offs[i] + lens[i]].tobytes() == o, i


def test_cpp_encryptor_batch_persistent_table_across_flushes(tmp_path, oracle):
    """EncryptorBatch's persistent device key table: 64 connections that live across 6
    flushes (stream state carried between flushes, package connections re-used), each
    flush touching a random subset plus short-lived connections created and destroyed in
    between (so addresses are reused by new keys), mixed key lengths; every output
    against the oracle."""
    from test_abi import build_dropin
    exe = build_dropin(tmp_path)
    rng = np.random.default_rng(777)
    conns = {}
    lines, expect = [], []
    for c in range(64):
        kl = (16, 24, 32)[c % 3]
        key, iv = rng.bytes(kl), rng.bytes(16)
        stream = c % 2 == 0
        enc = bool(c % 4) if stream else True
        conns[f"c{c}"] = dict(key=key, iv=iv, stream=stream, enc=enc, st_iv=iv, st_pos=0)
        lines.append(f"{'NS' if stream else 'NP'} c{c} {'E' if enc else 'D'} {key.hex()} {iv.hex()}")
    for fl in range(6):
        for name in rng.choice(sorted(conns), 40, replace=False):
            cc = conns[name]
            frames = [rng.bytes(int(rng.integers(0, 900))) for _ in range(int(rng.integers(1, 4)))]
            lines.append(f"NF {name} " + " ".join(f.hex() or "-" for f in frames))
            outs = []
            for f in frames:
                if cc["stream"]:
                    o, cc["st_iv"], cc["st_pos"] = oracle.cfb(cc["key"], cc["enc"], f, cc["st_iv"], cc["st_pos"])
                else:
                    o = oracle.package(cc["key"], cc["iv"], True, f)
                outs.append(o.hex() or "-")
            expect.append(" ".join(outs))
        for t in range(20):  # short-lived connections
            kl = (16, 32)[t % 2]
            key, iv = rng.bytes(kl), rng.bytes(16)
            data = rng.bytes(int(rng.integers(0, 600)))
            lines.append(f"BP {key.hex()} {iv.hex()} {data.hex() or '-'}")
            expect.append(f"{oracle.package(key, iv, True, data).hex() or '-'} "
                          f"{oracle.package(key, iv, False, data).hex() or '-'} {oracle.package_frame(key, iv, data).hex()}")
        lines.append("F")
    import subprocess
    res = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr
    assert res.stdout.strip().split("\n") == expect


def test_host_frames_over_two_engines(engine, oracle):
    """fpnn_aes_package_host_multi / fpnn_aes_stream_host_multi with two engines (the
    multi-GPU host path, here two engines on one GPU): byte-balanced package split and
    whole-stream assignment give exactly the one-engine / oracle results."""
    import fpnn_amd
    rng = np.random.default_rng(4242)
    e2 = fpnn_amd.Engine(0)
    nconn, kl = 97, 32
    keys = rng.bytes(nconn * kl)
    ivs = rng.bytes(nconn * 16)
    ks = [fpnn_amd.KeySet(engine, keys, kl, ivs), fpnn_amd.KeySet(e2, keys, kl, ivs)]
    n = 3000
    lens = rng.integers(0, 5000, n).astype(np.uint32)
    src = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    dst = np.zeros_like(src)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
    fr = np.zeros(n, dtype=fpnn_amd.engine.HOST_FRAME_DTYPE)
    fr["src"] = src.ctypes.data + offs
    fr["dst"] = dst.ctypes.data + offs
    fr["len"] = lens
    fr["key_slot"] = rng.integers(0, nconn, n)
    fpnn_amd.package_host_multi([engine, e2], ks, True, fr)
    for i in range(0, n, 7):
        s = int(fr["key_slot"][i])
        k, v = keys[s * kl:(s + 1) * kl], ivs[s * 16:(s + 1) * 16]
        seg = src[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
        assert dst[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes() == oracle.package(k, v, True, seg), i
    # stream mode: 97 streams, frames interleaved; state carried in the shared arrays
    iv_state = np.frombuffer(ivs, dtype=np.uint8).copy()
    pos_state = rng.integers(0, 16, nconn).astype(np.uint32)
    iv0, pos0 = iv_state.copy(), pos_state.copy()
    dst[:] = 0
    fpnn_amd.stream_host_multi([engine, e2], ks, False, fr, iv_state, pos_state)
    for s in range(nconn):
        idx = np.nonzero(fr["key_slot"] == s)[0]
        data = b"".join(src[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes() for i in idx)
        exp, iv_end, pos_end = oracle.cfb(keys[s * kl:(s + 1) * kl], False, data, iv0[16 * s:16 * s + 16].tobytes(),
                                          int(pos0[s]))
        got = b"".join(dst[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes() for i in idx)
        assert got == exp, s
        assert (iv_state[16 * s:16 * s + 16].tobytes(), int(pos_state[s])) == (iv_end, pos_end), s


@pytest.mark.parametrize("layout", ["same_offsets", "inplace", "shifted_out", "stream"])
@pytest.mark.parametrize("keylen", [16, 32])
def test_quad_line_aligned_steps(hybrid_quad_engine, oracle, layout, keylen):
    """K2h's quad session, line-aligned steps (k_hybrid.hip): a chain whose input and output sit at the
    same 16-B multiple inside a 128-B line takes a short first step to the line boundary.
    Ragged batches with 16-B multiple offsets at every line position and lengths from one
    block to many 8-block steps (some with a partial last block); 'shifted_out' (output
    16 B off the input) keeps the unaligned steps; 'stream' starts at random CFB
    positions, so the aligned step begins after the head bytes."""
    engine = hybrid_quad_engine
    rng = np.random.default_rng(77 + 3 * keylen + ["same_offsets", "inplace", "shifted_out", "stream"].index(layout))
    n = 1200
    lens = (rng.integers(0, 200, n) * 16 + rng.choice([0, 0, 0, 5, 11], n)).astype(np.int64)
    lens[:8] = (16, 32, 112, 128, 144, 1, 0, 4096)
    offs = np.concatenate([[0], np.cumsum(lens[:-1] + 16 + rng.integers(0, 8, n - 1) * 16)]).astype(np.int64)
    offs = (offs + 15) // 16 * 16  # 16-B multiples (a partial last block shifts the next one)
    total = int(offs[-1] + lens[-1] + 256)
    inp = rng.integers(0, 256, total, dtype=np.uint8)
    keys = rng.integers(0, 256, n * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, n * 16, dtype=np.uint8)
    slots = rng.permutation(n).astype(np.int32)
    ks = keyset(engine, keys, keylen, ivs)
    out_offs = offs + 16 if layout == "shifted_out" else offs
    exp = inp.copy()
    if layout == "stream":
        iv_h = rng.integers(0, 256, n * 16, dtype=np.uint8)
        pos_h = rng.integers(0, 16, n).astype(np.uint32)
        iv_d, pos_d = to_dev(iv_h), to_dev(pos_h.astype(np.int32))
        oracle.stream_batch(True, inp, exp, n, in_off=offs.astype(np.uint64), out_off=offs.astype(np.uint64),
                            lens=lens.astype(np.uint32), key_slot=slots.astype(np.uint32), keys=keys, keylen=keylen,
                            iv_state=iv_h, pos_state=pos_h, threads=8)
        src, dst = to_dev(inp), to_dev(inp)
        engine.stream_encrypt(src, dst, n, ks, iv_d, pos_d, in_off=to_dev(offs), lens=to_dev(lens.astype(np.int32)),
                              key_slot=to_dev(slots))
        torch.cuda.synchronize()
        assert np.array_equal(to_host(dst), exp)
        assert np.array_equal(to_host(iv_d), iv_h) and np.array_equal(to_host(pos_d).astype(np.uint32), pos_h)
        return
    oracle.package_batch(True, inp, exp, n, in_off=offs.astype(np.uint64), out_off=out_offs.astype(np.uint64),
                         lens=lens.astype(np.uint32), key_slot=slots.astype(np.uint32), keys=keys, keylen=keylen,
                         ivs=ivs, threads=8)
    src = to_dev(inp)
    dst = src if layout == "inplace" else to_dev(inp)
    engine.package_encrypt(src, dst, n, ks, in_off=to_dev(offs), out_off=to_dev(out_offs),
                           lens=to_dev(lens.astype(np.int32)), key_slot=to_dev(slots))
    torch.cuda.synchronize()
    assert np.array_equal(to_host(dst), exp)
