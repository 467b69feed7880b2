"""GPU parity of the host-mapped frame path (fpnn_aes_host_register + fpnn_aes_package_host):
frames that live in registered host memory are gathered from and scattered to that memory by
the GPU itself (k_move_segments) around the ordinary device cipher.  Results must equal n
PackageEncryptor calls (core/Encryptor.cpp:10-51) -- checked against the oracle -- and bytes
of the arenas outside the frames must stay untouched."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def aligned(nbytes, fill, align=4096):
    raw = np.full(nbytes + align, fill, dtype=np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


def place(rng, lens, gap_max=40):
    """disjoint offsets for the frames in random order, with random gaps"""
    order = rng.permutation(len(lens))
    offs = np.zeros(len(lens), dtype=np.int64)
    at = 0
    for i in order:
        at += int(rng.integers(0, gap_max))
        offs[i] = at
        at += int(lens[i]) + 4
    return offs, at + 64


def frames_array(src_base, src_offs, dst_base, dst_offs, lens, slots):
    import fpnn_amd
    fr = np.zeros(len(lens), dtype=fpnn_amd.engine.HOST_FRAME_DTYPE)
    fr["src"] = np.uint64(src_base) + src_offs.astype(np.uint64)
    fr["dst"] = np.uint64(dst_base) + dst_offs.astype(np.uint64)
    fr["len"] = lens
    fr["key_slot"] = slots
    return fr


@pytest.fixture
def arenas():
    """register numpy arenas for one test, unregister afterwards"""
    import fpnn_amd
    held = []

    def make(nbytes, fill):
        a = aligned(nbytes, fill)
        fpnn_amd.host_register(a)
        held.append(a)
        return a
    yield make
    for a in held:
        fpnn_amd.host_unregister(a)


@pytest.mark.parametrize("keylen", [16, 32])
@pytest.mark.parametrize("wire_prefix", [False, True])
def test_mapped_ragged_frames(engine, oracle, arenas, keylen, wire_prefix):
    import fpnn_amd
    rng = np.random.default_rng(900 + keylen + wire_prefix)
    nkeys = 7
    keys = rng.integers(0, 256, nkeys * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, nkeys * 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), keylen, ivs.tobytes())
    lens = np.concatenate([rng.integers(0, 5000, 3000), [0, 1, 15, 16, 17, 1024, 1025]]).astype(np.uint32)
    slots = rng.integers(0, nkeys, len(lens)).astype(np.uint32)
    soffs, ssize = place(rng, lens)
    doffs, dsize = place(rng, lens)
    src = arenas(ssize, 0)
    src[:] = rng.integers(0, 256, ssize, dtype=np.uint8)
    dst = arenas(dsize, 0xA5)
    fr = frames_array(src.ctypes.data, soffs, dst.ctypes.data, doffs, lens, slots)
    engine.package_host_array(True, fr, ks, wire_prefix=wire_prefix)
    assert engine.last_kernel(fpnn_amd.K_HOST) == "host_mapped"
    pre = 4 if wire_prefix else 0
    exp = np.full(dsize, 0xA5, dtype=np.uint8)
    for i in range(len(lens)):
        s, d, L = int(soffs[i]), int(doffs[i]), int(lens[i])
        if pre:
            exp[d:d + 4] = np.frombuffer(int(L).to_bytes(4, "little"), dtype=np.uint8)
        exp[d + pre:d + pre + L] = src[s:s + L]
    oracle.package_batch(True, exp.copy(), exp, len(lens), in_off=(doffs + pre).astype(np.uint64),
                         lens=lens, key_slot=slots, keys=keys, keylen=keylen, ivs=ivs, threads=8)
    assert np.array_equal(dst, exp)  # frames ciphered, every other byte untouched
    if not wire_prefix:  # decrypt back in place
        fr2 = frames_array(dst.ctypes.data, doffs, dst.ctypes.data, doffs, lens, slots)
        engine.package_host_array(False, fr2, ks)
        assert engine.last_kernel(fpnn_amd.K_HOST) == "host_mapped"
        bad = [i for i in range(len(lens))
               if not np.array_equal(dst[int(doffs[i]):int(doffs[i]) + int(lens[i])],
                                     src[int(soffs[i]):int(soffs[i]) + int(lens[i])])]
        assert not bad, (len(bad), bad[:8])  # every frame, not a sample (the r04n failure)


def _triples(rng, ntri, nkeys):
    """(short slot a, short slot b, long slot a) triples: the 64-block chunk before a long
    frame's interior holds the slots a, b, a, so K1r's last per-slot key pass in it is b's
    while the long frame that continues is a's (the shape of the r04n mismatch)."""
    lens, slots = [], []
    for t in range(ntri):
        a, b = (2 * t) % nkeys, (2 * t + 1) % nkeys
        lens += [int(rng.integers(1, 40)), int(rng.integers(1, 40)), int(rng.integers(4000, 20000))]
        slots += [a, b, a]
    return np.array(lens, np.uint32), np.array(slots, np.uint32)


@pytest.mark.parametrize("keylen", [16, 32])
def test_mapped_perkey_inplace_after_growth(oracle, arenas, keylen):
    """the r04n shape made deterministic.  A fresh engine encrypts
    per-key ragged frames (mapped, out of place), then a larger unrelated ragged decrypt
    grows the engine's scratch (block map, plan, descriptors: the old buffers are released
    behind the stream while the move stream is idle), then the frames are decrypted back IN
    PLACE through the mapped path.  Every byte of every frame must come back, and the
    ciphertext must equal the oracle's."""
    import fpnn_amd
    from test_gpu_parity import to_dev
    import torch
    eng = fpnn_amd.Engine(0)
    try:
        rng = np.random.default_rng(7700 + keylen)
        nkeys = 7
        lens, slots = _triples(rng, 1400, nkeys)  # ~3.5 chunks per wave of the grid: runs are reached
        keys = rng.integers(0, 256, nkeys * keylen, dtype=np.uint8)
        ivs = rng.integers(0, 256, nkeys * 16, dtype=np.uint8)
        ks = fpnn_amd.KeySet(eng, keys.tobytes(), keylen, ivs.tobytes())
        soffs, ssize = place(rng, lens)
        doffs, dsize = place(rng, lens)
        src = arenas(ssize, 0)
        src[:] = rng.integers(0, 256, ssize, dtype=np.uint8)
        dst = arenas(dsize, 0xA5)
        fr = frames_array(src.ctypes.data, soffs, dst.ctypes.data, doffs, lens, slots)
        eng.package_host_array(True, fr, ks)
        assert eng.last_kernel(fpnn_amd.K_HOST) == "host_mapped"
        exp = np.full(dsize, 0xA5, dtype=np.uint8)
        for i in range(len(lens)):
            exp[int(doffs[i]):int(doffs[i]) + int(lens[i])] = src[int(soffs[i]):int(soffs[i]) + int(lens[i])]
        oracle.package_batch(True, exp.copy(), exp, len(lens), in_off=doffs.astype(np.uint64), lens=lens,
                             key_slot=slots, keys=keys, keylen=keylen, ivs=ivs, threads=8)
        assert np.array_equal(dst, exp)
        # scratch growth: a ragged device decrypt with 20x the segments
        n2 = 20 * len(lens)
        l2 = rng.integers(0, 300, n2).astype(np.int32)
        o2 = np.concatenate([[0], np.cumsum(l2[:-1].astype(np.int64))])
        buf = to_dev(rng.integers(0, 256, int(o2[-1] + l2[-1]) + 64, dtype=np.uint8))
        eng.package_decrypt(buf, buf, n2, ks, in_off=to_dev(o2), lens=to_dev(l2),
                            key_slot=to_dev(rng.integers(0, nkeys, n2).astype(np.int32)))
        fr2 = frames_array(dst.ctypes.data, doffs, dst.ctypes.data, doffs, lens, slots)
        eng.package_host_array(False, fr2, ks)  # in place
        assert eng.last_kernel(fpnn_amd.K_HOST) == "host_mapped"
        torch.cuda.synchronize()
        bad = [i for i in range(len(lens))
               if not np.array_equal(dst[int(doffs[i]):int(doffs[i]) + int(lens[i])],
                                     src[int(soffs[i]):int(soffs[i]) + int(lens[i])])]
        assert not bad, (len(bad), bad[:8])
    finally:
        eng.sync()
        eng.close()


@pytest.mark.parametrize("nkeys", [1, 64])
def test_mapped_uniform_frames(engine, oracle, arenas, nkeys):
    """1 KiB frames at shuffled arena positions: the staging is dense and uniform, so the
    cipher takes the K2 / K1d (or per-packet-key) fast paths."""
    import fpnn_amd
    rng = np.random.default_rng(31 + nkeys)
    n, L, keylen = 70000, 1024, 32  # > one 64 MiB chunk
    keys = rng.integers(0, 256, nkeys * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, nkeys * 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), keylen, ivs.tobytes())
    slots = rng.integers(0, nkeys, n).astype(np.uint32)
    perm = rng.permutation(n).astype(np.int64)
    src = arenas(n * L, 0)
    src[:] = rng.integers(0, 256, n * L, dtype=np.uint8)
    dst = arenas(n * L, 0)
    lens = np.full(n, L, dtype=np.uint32)
    fr = frames_array(src.ctypes.data, perm * L, dst.ctypes.data, perm[::-1].copy() * L, lens, slots)
    engine.package_host_array(True, fr, ks)
    assert engine.last_kernel(fpnn_amd.K_HOST) == "host_mapped"
    exp = np.empty(n * L, dtype=np.uint8)
    dpos = perm[::-1]
    for i in range(n):
        exp[dpos[i] * L:(dpos[i] + 1) * L] = src[perm[i] * L:(perm[i] + 1) * L]
    oracle.package_batch(True, exp.copy(), exp, n, in_off=(dpos * L).astype(np.uint64), lens=lens,
                         key_slot=slots if nkeys > 1 else None, keys=keys, keylen=keylen, ivs=ivs, threads=8)
    assert np.array_equal(dst, exp)
    fr2 = frames_array(dst.ctypes.data, dpos * L, src.ctypes.data, perm * L, lens, slots)  # decrypt back
    engine.package_host_array(False, fr2, ks)
    assert engine.last_kernel(fpnn_amd.K_HOST) == "host_mapped"
    exp2 = np.empty_like(exp)
    oracle.package_batch(False, exp.copy(), exp2, n, in_off=(dpos * L).astype(np.uint64), lens=lens,
                         key_slot=slots if nkeys > 1 else None, keys=keys, keylen=keylen, ivs=ivs, threads=8)
    for i in range(0, n, 97):
        assert np.array_equal(src[perm[i] * L:(perm[i] + 1) * L], exp2[dpos[i] * L:(dpos[i] + 1) * L])


def test_partly_mapped_batch(engine, oracle, arenas):
    import fpnn_amd
    rng = np.random.default_rng(5)
    key, iv = rng.integers(0, 256, 32, dtype=np.uint8), rng.integers(0, 256, 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, key.tobytes(), 32, iv.tobytes())
    src = arenas(1 << 20, 0)
    src[:] = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    outside = np.zeros(5000, dtype=np.uint8)  # not registered
    lens = np.array([1000, 333, 4000], dtype=np.uint32)
    fr = frames_array(src.ctypes.data, np.array([0, 5000, 9000]), src.ctypes.data, np.array([100000, 200000, 0]),
                      lens, np.zeros(3, dtype=np.uint32))
    fr["dst"][2] = outside.ctypes.data
    assert fpnn_amd.host_is_mapped(int(fr["src"][0]), 1000)
    assert not fpnn_amd.host_is_mapped(outside.ctypes.data, 4000)
    engine.package_host_array(True, fr, ks)
    assert engine.last_kernel(fpnn_amd.K_HOST) == "host_mapped+staged"  # frames 0-1 mapped, 2 staged
    k, v = key.tobytes(), iv.tobytes()
    assert src[100000:101000].tobytes() == oracle.package(k, v, True, src[0:1000].tobytes())
    assert src[200000:200333].tobytes() == oracle.package(k, v, True, src[5000:5333].tobytes())
    assert outside[:4000].tobytes() == oracle.package(k, v, True, src[9000:13000].tobytes())
    fr2 = fr[::-1].copy()  # the unregistered frame first: all staged
    outside[:] = 0
    engine.package_host_array(True, fr2, ks)
    assert engine.last_kernel(fpnn_amd.K_HOST) == "host_staged"
    assert outside[:4000].tobytes() == oracle.package(k, v, True, src[9000:13000].tobytes())


def test_register_rules(arenas):
    import fpnn_amd
    a = arenas(1 << 16, 0)
    with pytest.raises(fpnn_amd.FpnnAesError):  # overlapping registration
        fpnn_amd.host_register(a[4096:])
    b = aligned(1 << 16, 0)
    with pytest.raises(fpnn_amd.FpnnAesError):  # never registered
        fpnn_amd.host_unregister(b)
    assert fpnn_amd.host_is_mapped(a.ctypes.data, a.nbytes)
    assert not fpnn_amd.host_is_mapped(a.ctypes.data, a.nbytes + 1)


def test_mapped_frames_over_two_engines(engine, oracle, arenas):
    """package_host_multi: each engine's share goes through its own mapped pipeline"""
    import fpnn_amd
    rng = np.random.default_rng(77)
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8), rng.integers(0, 256, 16, dtype=np.uint8)
    e2 = fpnn_amd.Engine(0)
    ks = [fpnn_amd.KeySet(e, key.tobytes(), 16, iv.tobytes()) for e in (engine, e2)]
    lens = rng.integers(1, 3000, 5000).astype(np.uint32)
    soffs, ssize = place(rng, lens)
    src = arenas(ssize, 0)
    src[:] = rng.integers(0, 256, ssize, dtype=np.uint8)
    fr = frames_array(src.ctypes.data, soffs, src.ctypes.data, soffs, lens, np.zeros(len(lens), dtype=np.uint32))
    orig = src.copy()
    fpnn_amd.package_host_multi([engine, e2], ks, True, fr)  # in place
    assert engine.last_kernel(fpnn_amd.K_HOST) == "host_mapped"
    assert e2.last_kernel(fpnn_amd.K_HOST) == "host_mapped"
    exp = orig.copy()
    oracle.package_batch(True, orig, exp, len(lens), in_off=soffs.astype(np.uint64), lens=lens, keys=key, keylen=16,
                         ivs=iv, threads=8)
    assert np.array_equal(src, exp)
    del ks
    e2.close()


@pytest.mark.parametrize("ragged", [False, True])
def test_staged_many_chunks(engine, oracle, ragged):
    """The staged host path over many pipeline chunks (pageable frames, not registered):
    the chunks' kernels share the engine's scratch (length order, block map, plan), so they
    must run in order on the engine stream -- a regression test for chunks whose kernels
    overlapped on their slot streams and read each other's scratch."""
    import fpnn_amd
    rng = np.random.default_rng(11 + ragged)
    n = 200000
    lens = rng.integers(1, 2048, n).astype(np.uint32) if ragged else np.full(n, 1024, dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.int64))])
    total = int(offs[-1] + lens[-1])
    key, iv = rng.integers(0, 256, 32, dtype=np.uint8), rng.integers(0, 256, 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, key.tobytes(), 32, iv.tobytes())
    src = rng.integers(0, 256, total, dtype=np.uint8)
    dst = np.zeros(total, dtype=np.uint8)
    fr = frames_array(src.ctypes.data, offs, dst.ctypes.data, offs, lens, np.zeros(n, dtype=np.uint32))
    exp = src.copy()
    oracle.package_batch(True, src, exp, n, in_off=offs.astype(np.uint64), lens=lens, keys=key, keylen=32, ivs=iv,
                         threads=8)
    for _ in range(2):
        dst[:] = 0
        engine.package_host_array(True, fr, ks)
        assert engine.last_kernel(fpnn_amd.K_HOST) == "host_staged"
        assert np.array_equal(dst, exp)
    fr2 = frames_array(dst.ctypes.data, offs, dst.ctypes.data, offs, lens, np.zeros(n, dtype=np.uint32))
    engine.package_host_array(False, fr2, ks)
    assert np.array_equal(dst, src)


def _stream_expected(oracle, encrypt, keys, keylen, frames, src, dst0, iv_state, pos_state, src_base, dst_base):
    """StreamEncryptor semantics per key slot, frames in array order (core/Encryptor.cpp:53-70)."""
    exp = dst0.copy()
    iv, pos = iv_state.copy(), pos_state.copy()
    for f in frames:
        s, n = int(f["key_slot"]), int(f["len"])
        if not n:
            continue
        so, do = int(f["src"]) - src_base, int(f["dst"]) - dst_base
        key = keys[keylen * s:keylen * (s + 1)].tobytes()
        out, ivo, po = oracle.cfb(key, encrypt, src[so:so + n].tobytes(), iv[16 * s:16 * s + 16].tobytes(), int(pos[s]))
        exp[do:do + n] = np.frombuffer(out, np.uint8)
        iv[16 * s:16 * s + 16] = np.frombuffer(ivo, np.uint8)
        pos[s] = po
    return exp, iv, pos


@pytest.mark.parametrize("keylen", [16, 32])
@pytest.mark.parametrize("shape", ["many_streams", "split_streams"])
def test_mapped_stream_frames(engine, oracle, arenas, keylen, shape):
    """fpnn_aes_stream_host with every frame in registered memory: the GPU gathers and
    scatters the frames itself (host_mapped), the streams' (iv, pos) carried across frames
    and -- split_streams: four 16 MiB streams, more than one pipeline chunk each -- across
    chunks.  Frames of a stream interleave with other streams' in the array and sit at
    random places of the arenas; bytes between frames stay untouched."""
    import fpnn_amd
    rng = np.random.default_rng(4400 + keylen + (shape == "split_streams"))
    if shape == "many_streams":
        S, n = 300, 3000
        lens = rng.integers(0, 5000, n).astype(np.uint32)
        short = rng.random(n) < 0.1
        lens[short] = rng.integers(0, 17, short.sum())
    else:
        S, n = 4, 64
        lens = np.full(n, 1 << 20, dtype=np.uint32)
        lens[::7] -= rng.integers(1, 1000, len(lens[::7])).astype(np.uint32)
    slots = rng.integers(0, S, n).astype(np.uint32)
    src_offs, src_size = place(rng, lens)
    dst_offs, dst_size = place(rng, lens)
    src = arenas(src_size, 0x11)
    src[:] = rng.integers(0, 256, src_size, dtype=np.uint8)
    dst = arenas(dst_size, 0x5A)
    keys = rng.integers(0, 256, S * keylen, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), keylen, bytes(16 * S))
    fr = frames_array(src.ctypes.data, src_offs, dst.ctypes.data, dst_offs, lens, slots)
    for encrypt in (True, False):
        iv0 = rng.integers(0, 256, 16 * S, dtype=np.uint8)
        pos0 = rng.integers(0, 16, S).astype(np.uint32)
        dst[:] = 0x5A
        exp, iv_e, pos_e = _stream_expected(oracle, encrypt, keys, keylen, fr, src, dst.copy(), iv0, pos0,
                                            src.ctypes.data, dst.ctypes.data)
        iv, pos = iv0.copy(), pos0.copy()
        engine.stream_host_array(encrypt, fr, ks, iv, pos)
        assert engine.last_kernel(fpnn_amd.K_HOST) == "host_mapped"
        bad = np.nonzero(dst != exp)[0]
        assert len(bad) == 0, (encrypt, len(bad), bad[:8])
        assert np.array_equal(iv, iv_e) and np.array_equal(pos, pos_e), encrypt


def test_stream_frames_partly_mapped_go_staged(engine, oracle, arenas):
    """One frame outside registered memory: the whole stream call takes the staged path
    (stream frames depend on each other), with the same results."""
    import fpnn_amd
    rng = np.random.default_rng(4500)
    S, n = 20, 200
    lens = rng.integers(1, 3000, n).astype(np.uint32)
    slots = rng.integers(0, S, n).astype(np.uint32)
    src_offs, src_size = place(rng, lens)
    dst_offs, dst_size = place(rng, lens)
    src = arenas(src_size, 0x11)
    src[:] = rng.integers(0, 256, src_size, dtype=np.uint8)
    dst = aligned(dst_size, 0x5A)  # NOT registered
    keys = rng.integers(0, 256, S * 16, dtype=np.uint8)
    ks = fpnn_amd.KeySet(engine, keys.tobytes(), 16, bytes(16 * S))
    fr = frames_array(src.ctypes.data, src_offs, dst.ctypes.data, dst_offs, lens, slots)
    iv0, pos0 = rng.integers(0, 256, 16 * S, dtype=np.uint8), np.zeros(S, dtype=np.uint32)
    exp, iv_e, pos_e = _stream_expected(oracle, True, keys, 16, fr, src, dst.copy(), iv0, pos0, src.ctypes.data,
                                        dst.ctypes.data)
    iv, pos = iv0.copy(), pos0.copy()
    engine.stream_host_array(True, fr, ks, iv, pos)
    assert engine.last_kernel(fpnn_amd.K_HOST) == "host_staged"
    assert np.array_equal(dst, exp) and np.array_equal(iv, iv_e) and np.array_equal(pos, pos_e)
