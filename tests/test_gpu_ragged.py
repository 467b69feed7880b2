"""K1r, the ragged decrypt (fpnn_amd/csrc/k_ragged.hip), against the oracle on the
shapes that stress its per-wave segment window: runs of empty segments and more than 64
segment starts inside one 64-block chunk (the per-lane search fallback), one segment
spanning many waves, tiny totals, out_off == in_off in place -- and the queue-only
contract: ragged calls return before their kernels finish (no host round trip)."""
import numpy as np
import pytest
import torch

from test_gpu_parity import dev_u8, keyset, to_dev, to_host

pytestmark = pytest.mark.gpu


def _package_case(engine, oracle, rng, lens, offs, keylen=32, nkeys=1, inplace=False, out_off_same=False):
    n = len(lens)
    total = int(max(offs + lens)) + 64 if n else 64
    inp = rng.integers(0, 256, total, dtype=np.uint8)
    keys = rng.integers(0, 256, nkeys * keylen, dtype=np.uint8)
    ivs = rng.integers(0, 256, nkeys * 16, dtype=np.uint8)
    slots = rng.integers(0, nkeys, n).astype(np.int32)
    ks = keyset(engine, keys, keylen, ivs)
    kw = dict(in_off=to_dev(offs.astype(np.int64)), lens=to_dev(lens.astype(np.int32)),
              key_slot=to_dev(slots) if nkeys > 1 else None)
    if out_off_same:
        kw["out_off"] = to_dev(offs.astype(np.int64))  # same values, a different array
    exp = inp.copy()
    oracle.package_batch(False, inp, exp, n, in_off=offs.astype(np.uint64), lens=lens.astype(np.uint32),
                         key_slot=slots.astype(np.uint32) if nkeys > 1 else None, keys=keys, keylen=keylen, ivs=ivs,
                         threads=8)
    src = to_dev(inp)
    dst = src if inplace else to_dev(inp)
    engine.package_decrypt(src, dst, n, ks, **kw)
    torch.cuda.synchronize()
    assert np.array_equal(to_host(dst), exp)


@pytest.mark.parametrize("inplace", [False, True])
def test_many_segment_starts_in_one_chunk(engine, oracle, inplace):
    """Runs of 200 empty segments and of 1..3-byte segments: far more than 64 segment
    starts fall inside single chunks, so the window re-anchors and the per-lane search
    fallback runs."""
    rng = np.random.default_rng(31 + inplace)
    parts = []
    for _ in range(40):
        kind = rng.integers(0, 3)
        if kind == 0:
            parts.append(np.zeros(200, np.int64))
        elif kind == 1:
            parts.append(rng.integers(1, 4, 150))
        else:
            parts.append(rng.integers(0, 5000, 20))
    lens = np.concatenate(parts)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64) + 16
    _package_case(engine, oracle, rng, lens, offs, nkeys=5, inplace=inplace)


@pytest.mark.parametrize("keylen", [16, 32])
def test_empty_and_tiny_totals(engine, oracle, keylen):
    rng = np.random.default_rng(keylen)
    for lens in (np.zeros(50, np.int64), np.array([0, 0, 7, 0]), np.array([16] * 3), np.array([1]),
                 np.array([0] * 70 + [33] + [0] * 70)):
        offs = np.concatenate([[0], np.cumsum(lens[:-1] + 5)]).astype(np.int64)
        _package_case(engine, oracle, rng, lens.astype(np.int64), offs, keylen=keylen)


def test_one_segment_over_many_waves(engine, oracle):
    """One 12 MiB + 7 B segment: every wave of the grid holds part of it, so every wave's
    first chunk takes its predecessor block from the plan (also in place)."""
    rng = np.random.default_rng(5)
    lens = np.array([12 * 1024 * 1024 + 7])
    offs = np.array([3])
    for inplace in (False, True):
        _package_case(engine, oracle, rng, lens, offs, inplace=inplace)


def test_inplace_with_out_off_equal_in_off(engine, oracle):
    """src is dst and out_off holds in_off's values in another array: still
    in place, no wave may read a block another wave already decrypted."""
    rng = np.random.default_rng(77)
    lens = rng.integers(0, 40000, 3000)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    _package_case(engine, oracle, rng, lens, offs, inplace=True, out_off_same=True)
    _package_case(engine, oracle, rng, lens, offs, nkeys=3, inplace=True, out_off_same=True)


@pytest.mark.parametrize("keylen", [16, 32])
def test_stream_segments_random_positions(engine, oracle, keylen):
    """Stream decrypt through K1r: 997 streams at random CFB positions with lengths from
    0 to 70 000 B (partial first and last blocks, empties), state written back."""
    rng = np.random.default_rng(400 + keylen)
    n = 997
    lens = rng.integers(0, 70000, n)
    lens[rng.random(n) < 0.1] = 0
    lens[rng.random(n) < 0.1] = rng.integers(1, 20, 1)[0]
    offs = np.concatenate([[0], np.cumsum(lens[:-1] + 3)]).astype(np.int64)
    total = int(offs[-1] + lens[-1] + 64)
    inp = rng.integers(0, 256, total, dtype=np.uint8)
    keys = rng.integers(0, 256, n * keylen, dtype=np.uint8)
    iv_state = rng.integers(0, 256, n * 16, dtype=np.uint8)
    pos_state = rng.integers(0, 16, n).astype(np.uint32)
    slots = np.arange(n, dtype=np.uint32)
    exp = inp.copy()
    iv_exp, pos_exp = iv_state.copy(), pos_state.copy()
    oracle.stream_batch(False, inp, exp, n, in_off=offs.astype(np.uint64), out_off=offs.astype(np.uint64),
                        lens=lens.astype(np.uint32), key_slot=slots, keys=keys, keylen=keylen, iv_state=iv_exp,
                        pos_state=pos_exp, threads=8)
    ks = keyset(engine, keys, keylen, np.zeros(n * 16, np.uint8))
    for inplace in (False, True):
        src = to_dev(inp)
        dst = src if inplace else to_dev(inp)
        ivd, posd = to_dev(iv_state), to_dev(pos_state.astype(np.int32))
        engine.stream_decrypt(src, dst, n, ks, ivd, posd, in_off=to_dev(offs), lens=to_dev(lens.astype(np.int32)),
                              key_slot=to_dev(slots.astype(np.int32)))
        torch.cuda.synchronize()
        assert np.array_equal(to_host(dst), exp)
        assert np.array_equal(to_host(ivd), iv_exp)
        assert np.array_equal(to_host(posd).astype(np.uint32), pos_exp)


@pytest.mark.parametrize("n", [1, 63, 64, 1023, 1024, 1025, 4097, 5000, 16383, 16384, 16385, 262145, 300001])
def test_block_map_round_boundaries(engine, oracle, n):
    """The single-workgroup block map (k_scan_small, up to 16 384 segments) takes segment
    k*1024 + t in thread t and scans per wave, then the wave totals, in groups of four
    rounds: segment counts at and around the 64 / 1024 / 4096 multiples and the
    small/large switch.  Past 16 384 segments the one-pass look-back map runs: 262 145 and
    300 001 segments are 65 and 74 tiles, so the look-back crosses its 64-tile window.
    Stream mode (the (iv, pos) snapshot comes from the same kernel) and package mode out
    of place (per-wave plan inside K1r) and in place (plan launch)."""
    rng = np.random.default_rng(9000 + n)
    lens = rng.integers(0, 300, n)
    lens[rng.random(n) < 0.05] = 0
    offs = np.concatenate([[0], np.cumsum(lens[:-1] + 1)]).astype(np.int64)
    for inplace in (False, True):
        _package_case(engine, oracle, rng, lens.astype(np.int64), offs, keylen=16, inplace=inplace)
    total = int(offs[-1] + lens[-1] + 64)
    inp = rng.integers(0, 256, total, dtype=np.uint8)
    keys = rng.integers(0, 256, 4 * 16, dtype=np.uint8)
    iv_state = rng.integers(0, 256, n * 16, dtype=np.uint8)
    pos_state = rng.integers(0, 16, n).astype(np.uint32)
    slots = rng.integers(0, 4, n).astype(np.uint32)
    exp = inp.copy()
    iv_exp, pos_exp = iv_state.copy(), pos_state.copy()
    oracle.stream_batch(False, inp, exp, n, in_off=offs.astype(np.uint64), out_off=offs.astype(np.uint64),
                        lens=lens.astype(np.uint32), key_slot=slots, keys=keys, keylen=16, iv_state=iv_exp,
                        pos_state=pos_exp, threads=8)
    ks = keyset(engine, keys, 16, np.zeros(4 * 16, np.uint8))
    src, dst = to_dev(inp), to_dev(inp)
    ivd, posd = to_dev(iv_state), to_dev(pos_state.astype(np.int32))
    engine.stream_decrypt(src, dst, n, ks, ivd, posd, in_off=to_dev(offs), lens=to_dev(lens.astype(np.int32)),
                          key_slot=to_dev(slots.astype(np.int32)))
    torch.cuda.synchronize()
    assert np.array_equal(to_host(dst), exp)
    assert np.array_equal(to_host(ivd), iv_exp)
    assert np.array_equal(to_host(posd).astype(np.uint32), pos_exp)


@pytest.mark.parametrize("env", [{"FPNN_AES_K1R_RUNS": "0"}, {"FPNN_AES_K1R_RUNS": "1"}], ids=["runs0", "runs1"])
@pytest.mark.parametrize("inplace", [False, True])
def test_one_kib_segments_on_chunk_boundaries(oracle, env, inplace):
    """One-key AES-256 package batches of 1 KiB segments, each exactly one 64-block chunk
    (R1's receive bodies, at 4-byte-misaligned offsets), broken by other lengths (1 KiB
    +- 1, 2 KiB, 16 B, 0 B, sub-block) so chunk boundaries drift off the segments and
    back, in place and out of place, interior runs on and off.  (A run loop over such
    segments back to back measured slower than K1r's general path -- 904-910 against
    942 GiB/s on R1 -- and was not kept: its per-segment descriptor loads sat on the
    chunk's critical path.)"""
    from conftest import _env_engine
    eng = _env_engine(env)
    try:
        rng = np.random.default_rng(5150 + 2 * inplace + len(str(env)))
        lens = []
        for _ in range(300):
            lens += [1024] * int(rng.integers(1, 40))
            lens.append(int(rng.choice([0, 5, 16, 1023, 1025, 2048, 3000])))
        lens = np.array(lens, np.int64)
        n = len(lens)
        gaps = np.full(n, 4, np.int64)  # the wire prefix between bodies
        offs = (np.concatenate([[0], np.cumsum(lens[:-1] + gaps[:-1])]) + 4).astype(np.int64)
        total = int(offs[-1] + lens[-1]) + 64
        key = rng.integers(0, 256, 32, dtype=np.uint8)
        iv = rng.integers(0, 256, 16, dtype=np.uint8)
        ks = keyset(eng, key, 32, iv)
        inp = rng.integers(0, 256, total, dtype=np.uint8)
        exp = inp.copy()
        oracle.package_batch(False, inp, exp, n, in_off=offs.astype(np.uint64), out_off=offs.astype(np.uint64),
                             lens=lens.astype(np.uint32), keys=key, keylen=32, ivs=iv, threads=8)
        src = to_dev(inp)
        dst = src if inplace else to_dev(inp)
        kw = dict(in_off=to_dev(offs), lens=to_dev(lens.astype(np.int32)))
        for _ in range(2):  # the second call: scratch reused
            if inplace:
                src.copy_(torch.from_numpy(inp).to(src.device))
            eng.package_decrypt(src, dst, n, ks, **kw)
            torch.cuda.synchronize()
            assert np.array_equal(to_host(dst), exp)
    finally:
        eng.close()


def test_large_block_map_repeated_calls(oracle):
    """The one-pass map resets its own tickets and tags its tile status with a per-launch
    epoch: back-to-back calls of different sizes (more tiles, then fewer, then more
    again) must each read only their own launch's status words.  (The three-launch scan
    this test also ran until round 5 was removed with its FPNN_AES_ONEPASS switch.)"""
    from conftest import _env_engine
    eng = _env_engine({})
    try:
        rng = np.random.default_rng(77 + len(str({"FPNN_AES_ONEPASS": "1"})))
        key = rng.integers(0, 256, 32, dtype=np.uint8)
        iv = rng.integers(0, 256, 16, dtype=np.uint8)
        ks = keyset(eng, key, 32, iv)
        for n in (300001, 20000, 140000, 16385, 300001):
            lens = rng.integers(0, 200, n).astype(np.int64)
            offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
            total = int(lens.sum()) + 16
            plain = rng.integers(0, 256, total, dtype=np.uint8)
            ct = plain.copy()
            oracle.package_batch(True, plain, ct, n, in_off=offs.astype(np.uint64), out_off=offs.astype(np.uint64),
                                 lens=lens.astype(np.uint32), keys=key, keylen=32, ivs=iv, threads=8)
            src, dst = to_dev(ct), to_dev(np.zeros_like(ct))
            eng.package_decrypt(src, dst, n, ks, in_off=to_dev(offs), lens=to_dev(lens.astype(np.int32)))
            torch.cuda.synchronize()
            got = to_host(dst)
            assert np.array_equal(got[: total - 16], plain[: total - 16]), n
    finally:
        eng.close()


# ------------------------------------------------------------------------------------
# queue-only: the C-ABI's ragged calls must not wait for the GPU (fpnn_aes.h)


def _big_ragged(rng, total_bytes, mean):
    lens = rng.integers(1, 2 * mean, int(total_bytes // mean))
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    return lens.astype(np.int32), offs


def _returns_before_done(call):
    call()  # warm-up: scratch allocations
    torch.cuda.synchronize()
    call()
    pending = not torch.cuda.current_stream().query()
    torch.cuda.synchronize()
    return pending


def test_ragged_calls_do_not_block(engine):
    import fpnn_amd
    rng = np.random.default_rng(9)
    lens, offs = _big_ragged(rng, 768 << 20, 3000)
    n = len(lens)
    buf = dev_u8(int(offs[-1] + lens[-1]) + 64)
    ks = fpnn_amd.KeySet(engine, rng.bytes(32), 32, rng.bytes(16))
    kw = dict(in_off=to_dev(offs), lens=to_dev(lens))
    assert _returns_before_done(lambda: engine.package_decrypt(buf, buf, n, ks, **kw)), "package_decrypt waited"
    # stream mode, per-stream keys and carried positions
    keys = fpnn_amd.KeySet(engine, rng.bytes(16 * n), 16, rng.bytes(16 * n))
    ivs = to_dev(rng.integers(0, 256, 16 * n, dtype=np.uint8))
    pos = to_dev(rng.integers(0, 16, n).astype(np.int32))
    slots = to_dev(np.arange(n, dtype=np.int32))
    assert _returns_before_done(lambda: engine.stream_decrypt(buf, buf, n, keys, ivs, pos, key_slot=slots, **kw)), \
        "stream_decrypt waited"
    # dense whole-stream layout (the C3 shape: every stream at position 0, s * L)
    S, L = 256, 1 << 20
    dense = dev_u8(S * L)
    zpos = torch.zeros(S, dtype=torch.int32, device=dense.device)
    dkeys = fpnn_amd.KeySet(engine, rng.bytes(16 * S), 16, rng.bytes(16 * S))
    div = to_dev(rng.integers(0, 256, 16 * S, dtype=np.uint8))
    dslots = to_dev(np.arange(S, dtype=np.int32))
    assert _returns_before_done(lambda: engine.stream_decrypt(dense, dense, S, dkeys, div, zpos.zero_(), stride=L,
                                                              uniform_len=L, key_slot=dslots)), "dense stream waited"


def test_recv_calls_do_not_block(engine):
    import fpnn_amd
    rng = np.random.default_rng(10)
    conns, per, body = 8192, 64, 1020
    seg = per * (body + 4)
    wire = np.zeros(conns * seg, np.uint8).reshape(conns, per, body + 4)
    wire[:, :, :4] = np.frombuffer(np.uint32(body).tobytes(), np.uint8)
    buf = to_dev(wire.reshape(-1))
    ks = fpnn_amd.KeySet(engine, rng.bytes(32), 32, rng.bytes(16))
    assert _returns_before_done(lambda: engine.package_recv(buf, buf, conns, ks, 8 << 20,
                                                            per, stride=seg, uniform_len=seg)), "package_recv waited"


@pytest.mark.parametrize("stream", [False, True])
def test_offsets_beyond_2gib(engine, oracle, stream):
    """Segments at byte offsets across and past 2^31 in a 2.3 GB buffer, long enough that
    each wave walks many chunks of one segment (the descriptor cache): 64-bit offsets
    must survive every cross-lane move (a sign-extended low half once faulted on C4)."""
    rng = np.random.default_rng(2031 + stream)
    base = (1 << 31) - (48 << 20)
    n = 1500
    lens = rng.integers(1, 200_000, n)
    offs_rel = np.concatenate([[0], np.cumsum(lens[:-1] + rng.integers(0, 40, n - 1))]).astype(np.int64)
    span = int(offs_rel[-1] + lens[-1]) + 64
    host = rng.integers(0, 256, span, dtype=np.uint8)
    keys = rng.integers(0, 256, n * 16, dtype=np.uint8)
    ivs = rng.integers(0, 256, n * 16, dtype=np.uint8)
    slots = np.arange(n, dtype=np.uint32)
    exp = host.copy()
    if stream:
        pos = rng.integers(0, 16, n).astype(np.uint32)
        iv_exp, pos_exp = ivs.copy(), pos.copy()
        oracle.stream_batch(False, host, exp, n, in_off=offs_rel.astype(np.uint64), out_off=offs_rel.astype(np.uint64),
                            lens=lens.astype(np.uint32), key_slot=slots, keys=keys, keylen=16, iv_state=iv_exp,
                            pos_state=pos_exp, threads=8)
    else:
        oracle.package_batch(False, host, exp, n, in_off=offs_rel.astype(np.uint64), lens=lens.astype(np.uint32),
                             key_slot=slots, keys=keys, keylen=16, ivs=ivs, threads=8)
    big = torch.empty(base + span, dtype=torch.uint8, device="cuda:0")
    big[base:].copy_(torch.from_numpy(host))
    kw = dict(in_off=to_dev(offs_rel + base), lens=to_dev(lens.astype(np.int32)), key_slot=to_dev(slots.astype(np.int32)))
    if stream:
        ks = keyset(engine, keys, 16, np.zeros(n * 16, np.uint8))
        ivd, posd = to_dev(ivs), to_dev(pos.astype(np.int32))
        engine.stream_decrypt(big, big, n, ks, ivd, posd, **kw)
    else:
        ks = keyset(engine, keys, 16, ivs)
        engine.package_decrypt(big, big, n, ks, **kw)
    torch.cuda.synchronize()
    assert np.array_equal(big[base:].cpu().numpy(), exp)
    if stream:
        assert np.array_equal(to_host(ivd), iv_exp) and np.array_equal(to_host(posd).astype(np.uint32), pos_exp)
    del big
    torch.cuda.empty_cache()


@pytest.mark.parametrize("env", [{"FPNN_AES_K1R_RUNS": "0"}, {"FPNN_AES_K1R_RUNS": "1"}], ids=["runs0", "runs1"])
@pytest.mark.parametrize("stream,keylen,inplace,nkeys",
                         [(st, kl, ip, 8) for st in (False, True) for kl in (16, 32) for ip in (False, True)] +
                         # one key, AES-256 package: the kernel the runs are built into (C4, R1)
                         [(False, 32, False, 1), (False, 32, True, 1)])
def test_interior_runs_after_key_switch(oracle, env, stream, keylen, inplace, nkeys):
    """K1r's interior runs (FPNN_AES_K1R_RUNS, k_ragged.hip) on per-key batches whose
    chunks end on another slot's pass: triples (short slot A, short slot B, long slot A),
    so the chunk before a long segment's run holds A, B, A and the general path's last
    key pass is B's.  Lengths off the block grid, gaps between segments, and in stream
    mode random carried (ivec, pos), two calls in a row; with runs off every chunk takes
    the general path.  This is the r04n mismatch: a tree that built the runs
    into the per-key kernels deciphered the long segment's interior with B's round keys;
    tools/probe/k1r_runs_perkey.patch rebuilds that form and fails here.  In place, the
    fresh engine first runs a ragged encrypt, so the decrypt grows the scratch the encrypt
    left (the r04n call order)."""
    from conftest import _env_engine
    eng = _env_engine(env)
    try:
        rng = np.random.default_rng(4100 + 10 * keylen + 2 * stream + len(str(env)) + nkeys)
        # big enough that every wave of the persistent grid (256 CUs x 16 waves) owns several
        # chunks -- a wave with one chunk never reaches a run (round 4's 120 triples never did)
        ntri = 1400
        lens, slots = [], []
        for t in range(ntri):
            a, b = (2 * t) % nkeys, (2 * t + 1) % nkeys
            lens += [int(rng.integers(1, 40)), int(rng.integers(1, 40)), int(rng.integers(4000, 20000))]
            slots += [a, b, a]
        lens = np.array(lens, np.int64)
        slots = np.array(slots, np.int32)
        n = len(lens)
        gaps = rng.integers(0, 20, n)
        offs = (np.concatenate([[0], np.cumsum(lens[:-1] + gaps[:-1])]) + 7).astype(np.int64)
        total = int(offs[-1] + lens[-1]) + 64
        inp = rng.integers(0, 256, total, dtype=np.uint8)
        keys = rng.integers(0, 256, nkeys * keylen, dtype=np.uint8)
        ivs = rng.integers(0, 256, nkeys * 16, dtype=np.uint8)
        ks = keyset(eng, keys, keylen, ivs)
        exp = inp.copy()
        kw = dict(in_off=to_dev(offs), lens=to_dev(lens.astype(np.int32)), key_slot=to_dev(slots))
        dst = to_dev(inp)
        if stream:
            iv0 = rng.integers(0, 256, 16 * n, dtype=np.uint8)
            pos0 = rng.integers(0, 16, n).astype(np.uint32)
            iv_h, pos_h = iv0.copy(), pos0.copy()
            oracle.stream_batch(False, inp, exp, n, in_off=offs.astype(np.uint64), out_off=offs.astype(np.uint64),
                                lens=lens.astype(np.uint32), key_slot=slots.astype(np.uint32), keys=keys,
                                keylen=keylen, iv_state=iv_h, pos_state=pos_h, threads=8)
            iv_d, pos_d = to_dev(iv0), to_dev(pos0.astype(np.int32))
            eng.stream_decrypt(dst if inplace else to_dev(inp), dst, n, ks, iv_d, pos_d, **kw)
            torch.cuda.synchronize()
            assert np.array_equal(to_host(dst), exp)
            # a second call continues every stream from the state the first one left
            inp2 = rng.integers(0, 256, total, dtype=np.uint8)
            exp = inp2.copy()
            oracle.stream_batch(False, inp2, exp, n, in_off=offs.astype(np.uint64), out_off=offs.astype(np.uint64),
                                lens=lens.astype(np.uint32), key_slot=slots.astype(np.uint32), keys=keys,
                                keylen=keylen, iv_state=iv_h, pos_state=pos_h, threads=8)
            dst = to_dev(inp2)
            eng.stream_decrypt(dst if inplace else to_dev(inp2), dst, n, ks, iv_d, pos_d, **kw)
            torch.cuda.synchronize()
            assert np.array_equal(to_host(iv_d), iv_h)
            assert np.array_equal(to_host(pos_d).astype(np.uint32), pos_h)
        else:
            oracle.package_batch(False, inp, exp, n, in_off=offs.astype(np.uint64), lens=lens.astype(np.uint32),
                                 key_slot=slots.astype(np.uint32), keys=keys, keylen=keylen, ivs=ivs, threads=8)
            if inplace:
                scratch = to_dev(inp)  # the encrypt grows the ordering scratch first
                eng.package_encrypt(to_dev(inp), scratch, n, ks, **kw)
                eng.package_decrypt(dst, dst, n, ks, **kw)
            else:
                eng.package_decrypt(to_dev(inp), dst, n, ks, **kw)
            torch.cuda.synchronize()
        assert np.array_equal(to_host(dst), exp)
    finally:
        eng.sync()
        eng.close()
