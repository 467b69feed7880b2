#!/usr/bin/env python3
"""Throughput of every BASELINE.json GPU config (device-resident, HIP-event timed),
for DESIGN.md -- bench.py's single JSON line covers C2 only.

  C2  1M x 1 KiB AES-256 package                    (also: PCIe-inclusive rate)
  C3  4096 streams x 4 MiB AES-128 stream mode      (whole stream per call, and cut into
                                                      random 1 B..64 KiB frames = one call per frame round)
  C4  Zipf 64 B..64 KiB, 4 GiB, AES-256 package
  C5  65536 keys x 4 KiB AES-256, per-key IV
  U1  1M x 1472 B UDP datagrams over 16384 connections, AES-128
  R1  the receive path: 16384 connections x 64 wire frames, fpnn_aes_package_recv (8f row 3)
  S1  stream-mode host frames, 16384 streams x 64 x 1 KiB: staged vs registered (mapped) arenas
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import workloads as W  # noqa: E402


def timed(eng, which, fn, reps, rounds=3, warm_s=0.3):
    """Steady state, as bench.py: warm-up calls for at least warm_s seconds of GPU work (the
    first calls grow scratch buffers, and the chip needs tens of ms of load to reach its
    clock: with two warm-up calls C2 read 866 / 952 GiB/s against bench.py's 1 008 / 1 014 in
    the same session, profiles/r04/timers.json), then `rounds` rounds of `reps` calls issued
    back to back (no host sync between them -- an idle gap lets the clock drop, which
    individually timed calls of a ~1 ms kernel measure instead of the kernel).  Returns the
    medians over rounds of (wall s per call, kernel s per launch of the main kernel `which`
    from HIP events on the engine stream) and the launches per call.  Each round times the
    wall first with the engine's event timing off (its two event records per launch are
    not part of a call), then the same calls again with it on for the kernel time."""
    import statistics
    t0 = time.perf_counter()
    n = 0
    while n < 2 or time.perf_counter() - t0 < warm_s:
        fn()
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    walls, kern, launches = [], [], 0
    for _ in range(max(1, rounds)):
        t0 = time.perf_counter()  # wall: no events in the stream
        for _ in range(max(1, reps)):
            fn()
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) / max(1, reps))
        eng.reset_stats()
        eng.set_timing(True)
        for _ in range(max(1, reps)):
            fn()
        torch.cuda.synchronize()
        eng.set_timing(False)
        n, ms = eng.kernel_stats(which)
        kern.append(ms / max(1, n) / 1e3)
        launches = n // max(1, reps)
    return statistics.median(walls), statistics.median(kern), launches


def gib(nbytes, sec):
    return round(nbytes / sec / 2**30, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5, help="calls per timed round (3 rounds; the median round is reported)")
    ap.add_argument("--configs", default="C2,C3,C4,C5,U1,R1")
    ap.add_argument("--no-host", action="store_true", help="skip the host-memory / PCIe legs (profiling runs)")
    args = ap.parse_args()
    import fpnn_amd
    E, D = fpnn_amd.K_ENCRYPT, fpnn_amd.K_DECRYPT
    eng = fpnn_amd.Engine(0)
    out = {}
    todo = args.configs.split(",")

    if "C2" in todo:
        c = W.C2
        P, L = c["packets"], c["length"]
        key, iv = W.single_key(c)
        ks = fpnn_amd.KeySet(eng, key, len(key), iv)
        a = torch.empty(P * L, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, c["payload_seed"])
        b, r = torch.empty_like(a), torch.empty_like(a)
        we, ke, _ = timed(eng, E, lambda: eng.package_encrypt(a, b, P, ks, stride=L, uniform_len=L), args.reps)
        wd, kd, _ = timed(eng, D, lambda: eng.package_decrypt(b, r, P, ks, stride=L, uniform_len=L), args.reps)
        assert torch.equal(r, a)
        if args.no_host:
            out["C2"] = {"encrypt_kernel_GiBs": gib(P * L, ke), "decrypt_kernel_GiBs": gib(P * L, kd)}
            print(json.dumps({"C2": out["C2"]}), flush=True)
            todo = [t for t in todo if t != "C2"]
    if "C2" in todo:
        # PCIe-inclusive: pinned host -> H2D -> kernel -> D2H, per direction
        h_in = torch.empty(P * L, dtype=torch.uint8, pin_memory=True)
        h_out = torch.empty_like(h_in, pin_memory=True)
        h_in.copy_(a)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            b.copy_(h_in, non_blocking=True)
            eng.package_encrypt(b, r, P, ks, stride=L, uniform_len=L)
            h_out.copy_(r, non_blocking=True)
        torch.cuda.synchronize()
        pe = (time.perf_counter() - t0) / args.reps
        # PCIe-inclusive with overlap: 16 chunks over 3 streams, each chunk
        # H2D -> encrypt -> D2H on its stream, so copies in both directions and the kernel
        # of different chunks run concurrently
        nst, nch = 3, 16
        streams = [torch.cuda.Stream() for _ in range(nst)]
        engs = [fpnn_amd.Engine(0, stream=st) for st in streams]
        kss = [fpnn_amd.KeySet(en, key, len(key), iv) for en in engs]
        per = P // nch

        def overlapped():
            for c in range(nch):
                st, en, kk = streams[c % nst], engs[c % nst], kss[c % nst]
                lo, hi = c * per * L, (c + 1) * per * L
                with torch.cuda.stream(st):
                    b[lo:hi].copy_(h_in[lo:hi], non_blocking=True)
                    en.package_encrypt(b[lo:hi], r[lo:hi], per, kk, stride=L, uniform_len=L)
                    h_out[lo:hi].copy_(r[lo:hi], non_blocking=True)
            torch.cuda.synchronize()

        overlapped()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            overlapped()
        po = (time.perf_counter() - t0) / args.reps
        assert torch.equal(h_out, r.cpu())
        del kss, engs
        t0 = time.perf_counter()
        for _ in range(args.reps):
            b.copy_(h_in, non_blocking=True)
            torch.cuda.synchronize()
        h2d = (time.perf_counter() - t0) / args.reps
        t0 = time.perf_counter()
        for _ in range(args.reps):
            h_out.copy_(r, non_blocking=True)
            torch.cuda.synchronize()
        d2h = (time.perf_counter() - t0) / args.reps
        # host frames (pageable numpy buffers, one frame per packet): the batch path
        # fpnn_aes_package_host = parallel gather -> pinned -> pipelined H2D/kernel/D2H -> scatter
        src_h = a.cpu().numpy()
        dst_h = np.empty_like(src_h)
        fr = np.zeros(P, dtype=fpnn_amd.engine.HOST_FRAME_DTYPE)
        fr["src"] = src_h.ctypes.data + np.arange(P, dtype=np.uint64) * L
        fr["dst"] = dst_h.ctypes.data + np.arange(P, dtype=np.uint64) * L
        fr["len"] = L
        eng.package_host_array(True, fr, ks)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            eng.package_host_array(True, fr, ks)
        hb = (time.perf_counter() - t0) / args.reps
        assert np.array_equal(dst_h, r.cpu().numpy())  # r = encrypt(a) from the PCIe loop
        fr["src"] = fr["dst"]  # decrypt in place
        t0 = time.perf_counter()
        eng.package_host_array(False, fr, ks)
        hbd = time.perf_counter() - t0
        assert np.array_equal(dst_h, src_h)
        # the same frames over two engines (fpnn_aes_package_host_multi; on one GPU this
        # measures the split's overhead -- the multi-GPU host path of SURVEY 8(e))
        fr["src"] = src_h.ctypes.data + np.arange(P, dtype=np.uint64) * L
        e2 = fpnn_amd.Engine(0)
        ks2 = fpnn_amd.KeySet(e2, key, len(key), iv)
        fpnn_amd.package_host_multi([eng, e2], [ks, ks2], True, fr)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fpnn_amd.package_host_multi([eng, e2], [ks, ks2], True, fr)
        hm = (time.perf_counter() - t0) / args.reps
        bad = np.nonzero((dst_h.reshape(P, L) != r.cpu().numpy().reshape(P, L)).any(1))[0]
        assert len(bad) == 0, f"two-engine host frames: {len(bad)} bad frames, first {bad[:8]}, last {bad[-3:]}"
        del ks2, e2
        # the same frames in registered host memory (fpnn_aes_host_register): the GPU gathers
        # them from and scatters them to the host arenas itself over PCIe, frames at shuffled
        # arena positions (socket-buffer shape); the staged path above is the fallback
        perm = np.random.default_rng(1).permutation(P).astype(np.uint64)
        def page_aligned(nbytes):
            raw = np.empty(nbytes + 4096, dtype=np.uint8)
            return raw[(-raw.ctypes.data) % 4096:][:nbytes]
        m_src, m_dst = page_aligned(P * L), page_aligned(P * L)
        fpnn_amd.host_register(m_src)
        fpnn_amd.host_register(m_dst)
        m_src.reshape(P, L)[perm.astype(np.int64)] = src_h.reshape(P, L)
        fm = np.zeros(P, dtype=fpnn_amd.engine.HOST_FRAME_DTYPE)
        fm["src"] = m_src.ctypes.data + perm * L
        fm["dst"] = m_dst.ctypes.data + perm[::-1] * L
        fm["len"] = L
        eng.package_host_array(True, fm, ks)
        assert eng.last_kernel(fpnn_amd.K_HOST) == "host_mapped"
        t0 = time.perf_counter()
        for _ in range(args.reps):
            eng.package_host_array(True, fm, ks)
        hme = (time.perf_counter() - t0) / args.reps
        rows = perm[::-1].astype(np.int64)
        assert np.array_equal(m_dst.reshape(P, L)[rows], dst_h.reshape(P, L)), "mapped host-frame ciphertext"
        fm["src"], fm["dst"] = fm["dst"].copy(), fm["dst"].copy()  # decrypt in place
        t0 = time.perf_counter()
        eng.package_host_array(False, fm, ks)
        hmd = time.perf_counter() - t0
        assert np.array_equal(m_dst.reshape(P, L)[rows], src_h.reshape(P, L))
        fpnn_amd.host_unregister(m_src)
        fpnn_amd.host_unregister(m_dst)
        del m_src, m_dst
        out["C2"] = {"encrypt_kernel_GiBs": gib(P * L, ke), "decrypt_kernel_GiBs": gib(P * L, kd),
                     "host_frames_encrypt_GiBs": gib(P * L, hb), "host_frames_decrypt_GiBs": gib(P * L, hbd),
                     "host_frames_encrypt_2engines_GiBs": gib(P * L, hm),
                     "mapped_host_frames_encrypt_GiBs": gib(P * L, hme),
                     "mapped_host_frames_decrypt_GiBs": gib(P * L, hmd),
                     "encrypt_wall_GiBs": gib(P * L, we), "decrypt_wall_GiBs": gib(P * L, wd),
                     "pcie_inclusive_encrypt_GiBs": gib(P * L, pe),
                     "pcie_inclusive_overlapped_encrypt_GiBs": gib(P * L, po), "h2d_GiBs": gib(P * L, h2d),
                     "d2h_GiBs": gib(P * L, d2h),
                     "note": "PCIe-inclusive = pinned H2D + encrypt + D2H serialized on one stream; "
                             "overlapped = 16 chunks over 3 streams; host frames = 1M pageable 1 KiB frames "
                             "through fpnn_aes_package_host (host gather -> pinned -> DMA -> host scatter); "
                             "mapped host frames = the same frames at shuffled positions of registered host "
                             "arenas, gathered/scattered by the GPU over PCIe"}
        del a, b, r, h_in, h_out
        print(json.dumps({"C2": out["C2"]}), flush=True)

    if "C2R" in todo:
        # C2's packets described as a ragged batch (offset / length arrays): the general
        # decrypt K1r on the exact data K1d decrypts in C2 -- isolates K1r's own cost
        c = W.C2
        P, L = c["packets"], c["length"]
        key, iv = W.single_key(c)
        ks = fpnn_amd.KeySet(eng, key, len(key), iv)
        a = torch.empty(P * L, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, c["payload_seed"])
        b, r = torch.empty_like(a), torch.empty_like(a)
        eng.package_encrypt(a, b, P, ks, stride=L, uniform_len=L)
        kw = dict(in_off=torch.arange(P, dtype=torch.int64, device="cuda") * L,
                  lens=torch.full((P,), L, dtype=torch.int32, device="cuda"))
        wd, kd, _ = timed(eng, D, lambda: eng.package_decrypt(b, r, P, ks, **kw), args.reps)
        assert torch.equal(r, a)
        wu, ku, _ = timed(eng, D, lambda: eng.package_decrypt(b, r, P, ks, stride=L, uniform_len=L), args.reps)
        out["C2R"] = {"ragged_decrypt_kernel_GiBs": gib(P * L, kd), "ragged_decrypt_wall_GiBs": gib(P * L, wd),
                      "dense_decrypt_kernel_GiBs": gib(P * L, ku), "ragged_kernel": eng.last_kernel(D)}
        del a, b, r
        print(json.dumps({"C2R": out["C2R"]}), flush=True)

    if "C5" in todo:
        c = W.C5
        P, L = c["packets"], c["length"]
        keys, ivs = W.many_keys(c)
        ks = fpnn_amd.KeySet(eng, keys.tobytes(), c["keylen"], ivs.tobytes())
        slots = torch.arange(P, dtype=torch.int32, device="cuda")
        a = torch.empty(P * L, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, c["payload_seed"])
        b, r = torch.empty_like(a), torch.empty_like(a)
        kw = dict(stride=L, uniform_len=L, key_slot=slots)
        we, ke, _ = timed(eng, E, lambda: eng.package_encrypt(a, b, P, ks, **kw), args.reps)
        wd, kd, _ = timed(eng, D, lambda: eng.package_decrypt(b, r, P, ks, **kw), args.reps)
        assert torch.equal(r, a)
        t0 = time.perf_counter()
        ks2 = fpnn_amd.KeySet(eng, keys.tobytes(), c["keylen"], ivs.tobytes())
        kexp = time.perf_counter() - t0
        out["C5"] = {"encrypt_kernel_GiBs": gib(P * L, ke), "decrypt_kernel_GiBs": gib(P * L, kd),
                     "encrypt_wall_GiBs": gib(P * L, we), "decrypt_wall_GiBs": gib(P * L, wd),
                     "keyset_create_65536_keys_ms": round(kexp * 1e3, 2)}
        del a, b, r, ks2
        print(json.dumps({"C5": out["C5"]}), flush=True)

    if "U1" in todo:
        c = W.U1
        P, L, NC = c["packets"], c["length"], c["connections"]
        keys, ivs = W.many_keys(c)
        ks = fpnn_amd.KeySet(eng, keys.tobytes(), c["keylen"], ivs.tobytes())
        slots = (torch.arange(P, dtype=torch.int32, device="cuda") % NC).contiguous()
        a = torch.empty(P * L, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, c["payload_seed"])
        b, r = torch.empty_like(a), torch.empty_like(a)
        kw = dict(stride=L, uniform_len=L, key_slot=slots)
        we, ke, _ = timed(eng, E, lambda: eng.package_encrypt(a, b, P, ks, **kw), args.reps)
        wd, kd, _ = timed(eng, D, lambda: eng.package_decrypt(b, r, P, ks, **kw), args.reps)
        assert torch.equal(r, a)
        if args.no_host:
            out["U1"] = {"encrypt_kernel_GiBs": gib(P * L, ke), "decrypt_kernel_GiBs": gib(P * L, kd)}
            print(json.dumps({"U1": out["U1"]}), flush=True)
            todo = [t for t in todo if t != "U1"]
    if "U1" in todo:
        src_h = a.cpu().numpy()
        dst_h = np.empty_like(src_h)
        fr = np.zeros(P, dtype=fpnn_amd.engine.HOST_FRAME_DTYPE)
        fr["src"] = src_h.ctypes.data + np.arange(P, dtype=np.uint64) * L
        fr["dst"] = dst_h.ctypes.data + np.arange(P, dtype=np.uint64) * L
        fr["len"] = L
        fr["key_slot"] = np.arange(P) % NC
        eng.package_host_array(True, fr, ks)
        t0 = time.perf_counter()
        eng.package_host_array(True, fr, ks)
        hb = time.perf_counter() - t0
        assert np.array_equal(dst_h, b.cpu().numpy())
        out["U1"] = {"encrypt_kernel_GiBs": gib(P * L, ke), "decrypt_kernel_GiBs": gib(P * L, kd),
                     "encrypt_wall_GiBs": gib(P * L, we), "decrypt_wall_GiBs": gib(P * L, wd),
                     "host_frames_encrypt_GiBs": gib(P * L, hb),
                     "datagrams_per_s_encrypt_kernel": round(P / ke)}
        del a, b, r
        print(json.dumps({"U1": out["U1"]}), flush=True)

    for qname in [q for q in ("Q1", "Q1g", "Q1s", "Q1h") if q in todo]:
        # FPNN's typical quest frames (145 B: core/test/tcp-test/asyncStressClient.cpp:13-29)
        # from 16 384 connections, each with its own key and IV, as one collector flush would
        # pass them (ragged layout, slot per frame): 9 whole blocks and a 1-byte tail per
        # chain, so block 0 is a tenth of each chain (SURVEY section 0 point 3: E_k(IV))
        # (Q1s: the same as Q1 with FPNN's default 16-byte keys instead of reinforced 32)
        # (Q1h: a quarter of Q1's frames, 2 per GPU lane -- the K2 / K2h cut-over)
        P, L, NC = (2 << 20) >> (2 if qname == "Q1h" else 0), 145, 16384
        kl = 16 if qname == "Q1s" else 32
        keys, ivs = W.many_keys(dict(W.U1, connections=NC, keylen=kl))
        ks = fpnn_amd.KeySet(eng, keys.tobytes(), kl, ivs.tobytes())
        offs = torch.arange(P, dtype=torch.int64, device="cuda") * L
        lens = torch.full((P,), L, dtype=torch.int32, device="cuda")
        # Q1: consecutive frames from different connections (one quest per connection per
        # IO cycle); Q1g: 8 consecutive frames per connection (a window of 8 per cycle)
        idx = torch.arange(P, dtype=torch.int32, device="cuda")
        slots = ((idx // 8) % NC if qname == "Q1g" else idx % NC).contiguous()
        a = torch.empty(P * L, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, 11)
        b, r = torch.empty_like(a), torch.empty_like(a)
        kw = dict(in_off=offs, lens=lens, key_slot=slots)
        # the encrypt passes the frames' length bound, as a collector that built them knows it
        we, ke, _ = timed(eng, E, lambda: eng.package_encrypt(a, b, P, ks, max_len=L, **kw), args.reps)
        # (the receive side knows the bound too: the frames' headers went through the framing)
        wd, kd, _ = timed(eng, D, lambda: eng.package_decrypt(b, r, P, ks, max_len=L, **kw), args.reps)
        assert torch.equal(r, a)
        out[qname] = {"frames": P, "frame_bytes": L, "encrypt_kernel_GiBs": gib(P * L, ke),
                     "decrypt_kernel_GiBs": gib(P * L, kd), "encrypt_wall_GiBs": gib(P * L, we),
                     "decrypt_wall_GiBs": gib(P * L, wd), "frames_per_s_encrypt_wall": round(P / we),
                     "cipher_sha256_16": __import__("hashlib").sha256(b.cpu().numpy()).hexdigest()[:16]}
        del a, b, r
        print(json.dumps({qname: out[qname]}), flush=True)

    if "C4" in todo:
        c = W.C4
        sizes = W.zipf_sizes(c)
        n = len(sizes)
        offs = np.concatenate([[0], np.cumsum(sizes[:-1].astype(np.int64))]).astype(np.int64)
        total = int(offs[-1] + sizes[-1])
        key, iv = W.single_key(c)
        ks = fpnn_amd.KeySet(eng, key, len(key), iv)
        a = torch.empty(total, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, c["payload_seed"])
        b, r = torch.empty_like(a), torch.empty_like(a)
        kw = dict(in_off=torch.from_numpy(offs).cuda(), lens=torch.from_numpy(sizes.astype(np.int32)).cuda())
        we, ke, _ = timed(eng, E, lambda: eng.package_encrypt(a, b, n, ks, **kw), args.reps)
        wd, kd, _ = timed(eng, D, lambda: eng.package_decrypt(b, r, n, ks, **kw), args.reps)
        assert torch.equal(r, a)
        out["C4"] = {"packets": n, "bytes": total, "encrypt_kernel_GiBs": gib(total, ke),
                     "decrypt_kernel_GiBs": gib(total, kd), "encrypt_wall_GiBs": gib(total, we),
                     "decrypt_wall_GiBs": gib(total, wd)}
        del a, b, r
        print(json.dumps({"C4": out["C4"]}), flush=True)

    if "C3" in todo:
        c = W.C3
        S, L = c["streams"], c["length"]
        keys, ivs = W.many_keys(c)
        ks = fpnn_amd.KeySet(eng, keys.tobytes(), c["keylen"], ivs.tobytes())
        a = torch.empty(S * L, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, c["payload_seed"])
        b, r = torch.empty_like(a), torch.empty_like(a)
        slots = torch.arange(S, dtype=torch.int32, device="cuda")
        iv0 = torch.from_numpy(ivs.copy()).cuda()
        st_iv, st_pos = iv0.clone(), torch.zeros(S, dtype=torch.int32, device="cuda")

        def whole(fn, src, dst):
            st_iv.copy_(iv0)
            st_pos.zero_()
            fn(src, dst, S, ks, st_iv, st_pos, stride=L, uniform_len=L, key_slot=slots,
               in_off=torch.arange(S, dtype=torch.int64, device="cuda") * L)

        we, ke, _ = timed(eng, E, lambda: whole(eng.stream_encrypt, a, b), args.reps)
        wd, kd, _ = timed(eng, D, lambda: whole(eng.stream_decrypt, b, r), args.reps)
        assert torch.equal(r, a)
        # framed: one call per frame round (every stream's next frame)
        splits = [W.stream_splits(c, s) for s in range(S)]
        nmax = max(len(x) for x in splits)
        lens = np.zeros((nmax, S), dtype=np.int32)
        for s_, x in enumerate(splits):
            lens[:len(x), s_] = x
        starts = np.cumsum(np.vstack([np.zeros((1, S), np.int64), lens[:-1]]), axis=0) + \
            np.arange(S, dtype=np.int64)[None, :] * L
        d_lens = [torch.from_numpy(lens[f]).cuda() for f in range(nmax)]
        d_offs = [torch.from_numpy(starts[f]).cuda() for f in range(nmax)]

        def framed(fn, src, dst):
            st_iv.copy_(iv0)
            st_pos.zero_()
            for f in range(nmax):
                fn(src, dst, S, ks, st_iv, st_pos, in_off=d_offs[f], lens=d_lens[f], key_slot=slots)

        wfe, kfe, nfe = timed(eng, E, lambda: framed(eng.stream_encrypt, a, b), args.reps)
        wfd, kfd, nfd = timed(eng, D, lambda: framed(eng.stream_decrypt, b, r), args.reps)
        assert torch.equal(r, a)
        if args.no_host:
            out["C3"] = {"whole_stream_encrypt_kernel_GiBs": gib(S * L, ke),
                         "whole_stream_decrypt_kernel_GiBs": gib(S * L, kd),
                         "framed_calls": nmax, "framed_encrypt_wall_GiBs": gib(S * L, wfe),
                         "framed_decrypt_wall_GiBs": gib(S * L, wfd),
                         "framed_decrypt_kernel_GiBs": gib(S * L, kfd * nfd)}
            print(json.dumps({"C3": out["C3"]}), flush=True)
            todo = [t for t in todo if t != "C3"]
    if "C3" in todo:
        # host frames, one stream_host call for the framed streams of a 1 GiB subset
        HS = 256
        src_h = a[:HS * L].cpu().numpy()
        dst_h = np.empty_like(src_h)
        fl = [(s_, int(starts[f, s_]), int(lens[f, s_])) for f in range(nmax) for s_ in range(HS) if lens[f, s_]]
        fr = np.zeros(len(fl), dtype=fpnn_amd.engine.HOST_FRAME_DTYPE)
        fr["src"] = src_h.ctypes.data + np.array([o for _, o, _ in fl], dtype=np.uint64)
        fr["dst"] = dst_h.ctypes.data + np.array([o for _, o, _ in fl], dtype=np.uint64)
        fr["len"] = [x for _, _, x in fl]
        fr["key_slot"] = [s_ for s_, _, _ in fl]
        h_iv = np.ascontiguousarray(np.resize(ivs, (S, 16)))
        h_pos = np.zeros(S, dtype=np.uint32)
        eng.stream_host_array(True, fr, ks, h_iv.copy(), h_pos.copy())  # warm: staging allocation
        t0 = time.perf_counter()
        eng.stream_host_array(True, fr, ks, h_iv, h_pos)
        hse = time.perf_counter() - t0
        assert np.array_equal(dst_h, b[:HS * L].cpu().numpy())
        h_iv = np.ascontiguousarray(np.resize(ivs, (S, 16)))
        h_pos[:] = 0
        fr["src"] = fr["dst"]
        t0 = time.perf_counter()
        eng.stream_host_array(False, fr, ks, h_iv, h_pos)  # in place
        hsd = time.perf_counter() - t0
        assert np.array_equal(dst_h, src_h)
        out["C3"] = {"whole_stream_encrypt_kernel_GiBs": gib(S * L, ke),
                     "whole_stream_decrypt_kernel_GiBs": gib(S * L, kd),
                     "framed_calls": nmax, "framed_encrypt_wall_GiBs": gib(S * L, wfe),
                     "framed_decrypt_wall_GiBs": gib(S * L, wfd),
                     "framed_decrypt_kernel_GiBs": gib(S * L, kfd * nfd),
                     "host_frames_streams": HS, "host_frames": len(fl),
                     "host_frames_encrypt_GiBs": gib(HS * L, hse), "host_frames_decrypt_GiBs": gib(HS * L, hsd),
                     "note": "encrypt = 4096 serial CFB chains (one lane each, latency bound); "
                             "decrypt parallel per block"}
        print(json.dumps({"C3": out["C3"]}), flush=True)
    if "R1" in todo:
        # The receive path: 16384 connection buffers, each holding 64
        # package-mode wire frames (htole32(len) + 1 KiB ciphertext, the form
        # PackageEncryptor::encrypt(std::string*) sends) = 1 GiB of bodies; one
        # fpnn_aes_package_recv call finds the frames on the device and decrypts them.
        NC, F, L = 16384, 64, 1024
        key, iv = W.single_key(W.C2)
        ks = fpnn_amd.KeySet(eng, key, len(key), iv)
        P = NC * F
        a = torch.empty(P * L, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, 7)
        wire = torch.empty(P * (L + 4), dtype=torch.uint8, device="cuda")
        in_off = torch.arange(P, dtype=torch.int64, device="cuda") * L
        out_off = torch.arange(P, dtype=torch.int64, device="cuda") * (L + 4)
        lens = torch.full((P,), L, dtype=torch.int32, device="cuda")
        def wire_encrypt():  # the send side: bodies -> htole32(len) || ciphertext (K2q)
            eng.package_encrypt(a, wire, P, ks, in_off=in_off, out_off=out_off, lens=lens, wire_prefix=True,
                                max_len=L)  # (the sender knows its frames' length bound)

        we, ke, _ = timed(eng, E, wire_encrypt, args.reps)
        conn_off = torch.arange(NC, dtype=torch.int64, device="cuda") * (F * (L + 4))
        conn_len = torch.full((NC,), F * (L + 4), dtype=torch.int32, device="cuda")
        plain = torch.empty_like(wire)

        def recv():
            return eng.package_recv(wire, plain, NC, ks, 8 << 20, F, in_off=conn_off, lens=conn_len)

        wr, kr, _ = timed(eng, D, recv, args.reps)
        foff, flen, scan = recv()
        torch.cuda.synchronize()
        body = plain.view(P, L + 4)[:, 4:]
        assert torch.equal(body.reshape(-1), a), "R1 receive-path plaintext differs"
        out["R1"] = {"frames": P, "body_bytes": P * L, "recv_wall_GiBs": gib(P * L, wr),
                     "wire_encrypt_kernel_GiBs": gib(P * L, ke), "wire_encrypt_wall_GiBs": gib(P * L, we),
                     "decrypt_kernel_GiBs": gib(P * L, kr),
                     "note": "fpnn_aes_package_recv over 16384 connections x 64 wire frames (4-byte LE length + 1 KiB): "
                             "device frame scan + decrypt of the bodies at their frame offsets (wall includes the scan, "
                             "the block-map scan and the plan; no host sync)"}
        del a, wire, plain
        print(json.dumps({"R1": out["R1"]}), flush=True)

    if "S1" in todo:
        # Stream-mode host frames (StreamEncryptor per connection, core/Encryptor.cpp:53-70):
        # 16384 streams x 64 frames of 1 KiB = 1 GiB, the array in arrival order (frame j of
        # every stream before frame j + 1 of any), frames at shuffled places of host arenas.
        # Staged (pageable, host gather/scatter) vs mapped (arenas registered, the GPU moves).
        NS, F, L = 16384, 64, 1024
        P = NS * F
        rng = np.random.default_rng(5)
        keys = rng.integers(0, 256, NS * 16, dtype=np.uint8)
        ks = fpnn_amd.KeySet(eng, keys.tobytes(), 16, bytes(16 * NS))
        def page_aligned(nbytes):
            raw = np.empty(nbytes + 4096, dtype=np.uint8)
            return raw[(-raw.ctypes.data) % 4096:][:nbytes]
        src, dst = page_aligned(P * L), page_aligned(P * L)
        src[:] = rng.integers(0, 256, P * L, dtype=np.uint8)
        perm = rng.permutation(P).astype(np.uint64)
        fr = np.zeros(P, dtype=fpnn_amd.engine.HOST_FRAME_DTYPE)
        fr["src"] = src.ctypes.data + perm * L
        fr["dst"] = dst.ctypes.data + perm[::-1] * L
        fr["len"] = L
        fr["key_slot"] = np.arange(P) % NS
        res = {}
        for mode in ("staged", "mapped"):
            if mode == "mapped":
                fpnn_amd.host_register(src)
                fpnn_amd.host_register(dst)
            for enc in (True, False):
                times = []
                for _ in range(1 + args.reps):
                    iv, pos = np.zeros(16 * NS, np.uint8), np.zeros(NS, np.uint32)
                    t0 = time.perf_counter()
                    eng.stream_host_array(enc, fr, ks, iv, pos)
                    times.append(time.perf_counter() - t0)
                import statistics
                res[f"{mode}_{'encrypt' if enc else 'decrypt'}_GiBs"] = gib(P * L, statistics.median(times[1:]))
                res[f"{mode}_path"] = eng.last_kernel(fpnn_amd.K_HOST)
                if enc:
                    got_enc = dst.copy() if mode == "staged" else None
                    if mode == "mapped":
                        assert np.array_equal(dst, ref_enc), "mapped stream host frames differ from staged"
                    else:
                        ref_enc = got_enc
            if mode == "mapped":
                fpnn_amd.host_unregister(src)
                fpnn_amd.host_unregister(dst)
        out["S1"] = dict(res, frames=P, streams=NS, frame_bytes=L,
                         note="stream host frames: 16384 streams x 64 x 1 KiB in arrival order at shuffled arena "
                              "places; staged = host gather/scatter + pinned DMA, mapped = arenas registered, the "
                              "GPU gathers/scatters over PCIe; mapped encrypt output checked equal to the staged one")
        del src, dst
        print(json.dumps({"S1": out["S1"]}), flush=True)
    if "SB" in todo:
        # Small receive batches (one IO cycle of a server): 256 package frames of 64 .. 2047
        # bytes (AES-256, one key) per call, 2 000 calls back to back -- the shape where a
        # call's fixed launches (block map + K1r) cost more than its decrypt.
        key, iv = W.single_key(W.C2)
        ks = fpnn_amd.KeySet(eng, key, len(key), iv)
        rng = np.random.default_rng(2024)
        P = 256
        blen = rng.integers(64, 2048, P).astype(np.int64)
        offs = np.concatenate([[0], np.cumsum(blen[:-1])]).astype(np.int64)
        total = int(blen.sum())
        a = torch.empty(total, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, 11)
        ct, back = torch.empty_like(a), torch.empty_like(a)
        kw = dict(in_off=torch.from_numpy(offs).cuda(), lens=torch.from_numpy(blen.astype(np.int32)).cuda())
        eng.package_encrypt(a, ct, P, ks, **kw)
        wd, kd, launches = timed(eng, D, lambda: eng.package_decrypt(ct, back, P, ks, **kw), 2000, rounds=3)
        torch.cuda.synchronize()
        assert torch.equal(back, a), "SB round trip"
        out["SB"] = {"frames_per_call": P, "bytes_per_call": total, "us_per_call_wall": round(wd * 1e6, 2),
                     "us_per_call_kernel": round(kd * 1e6, 2), "launches_per_call": launches,
                     "note": "small package receive batches (256 ragged frames, 64..2047 B, AES-256), "
                             "back to back: one-workgroup block map + K1r per call (launches_per_call counts K1r)"}
        del a, ct, back
        print(json.dumps({"SB": out["SB"]}), flush=True)
    if "R1R" in todo:
        # R1 with realistic body lengths: CFB does not pad, so FPNN package bodies have any
        # length -- here uniform 1 .. 2047 bytes (mean ~1 KiB), 64 frames per connection
        NC, F = 16384, 64
        key, iv = W.single_key(W.C2)
        ks = fpnn_amd.KeySet(eng, key, len(key), iv)
        P = NC * F
        rng = np.random.default_rng(1717)
        blen = rng.integers(1, 2048, P).astype(np.int64)
        in_off = np.concatenate([[0], np.cumsum(blen[:-1])]).astype(np.int64)
        out_off = in_off + 4 * np.arange(P, dtype=np.int64)
        total = int(blen.sum())
        a = torch.empty(total, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, 8)
        wire = torch.empty(total + 4 * P, dtype=torch.uint8, device="cuda")
        eng.package_encrypt(a, wire, P, ks, in_off=torch.from_numpy(in_off).cuda(),
                            out_off=torch.from_numpy(out_off).cuda(),
                            lens=torch.from_numpy(blen.astype(np.int32)).cuda(), wire_prefix=True)
        per_conn = (blen + 4).reshape(NC, F).sum(axis=1)
        conn_off = torch.from_numpy(np.concatenate([[0], np.cumsum(per_conn[:-1])]).astype(np.int64)).cuda()
        conn_len = torch.from_numpy(per_conn.astype(np.int32)).cuda()
        plain = torch.empty_like(wire)

        def recv():
            return eng.package_recv(wire, plain, NC, ks, 8 << 20, F, in_off=conn_off, lens=conn_len)

        wr, kr, _ = timed(eng, D, recv, args.reps)
        recv()
        torch.cuda.synchronize()
        body_mask = torch.ones(total + 4 * P, dtype=torch.bool, device="cuda")
        pre = torch.from_numpy(out_off).cuda()
        for k in range(4):
            body_mask[pre + k] = False
        assert torch.equal(plain[body_mask], a), "R1R receive-path plaintext differs"
        out["R1R"] = {"frames": P, "body_bytes": total, "recv_wall_GiBs": gib(total, wr),
                      "decrypt_kernel_GiBs": gib(total, kr),
                      "note": "R1 with body lengths uniform in 1..2047 B (not 16-aligned): frame scan + K1r"}
        del a, wire, plain, body_mask
        print(json.dumps({"R1R": out["R1R"]}), flush=True)

    if "R2" in todo:
        # The stream-mode receive path: 4096 streams (C3's connections, AES-128), each call's
        # segment = 256 KiB of ciphertext holding 256 FPNN answers of 1 KiB (12-byte header
        # + seq + 1008-byte payload); fpnn_aes_stream_recv decrypts it (state carried) and
        # splits it into messages with the reference's BodyLen checks.
        NS, M, L = 4096, 256, 1024
        keys, ivs = W.many_keys(W.C3)
        ks = fpnn_amd.KeySet(eng, keys.tobytes(), 16, np.zeros(NS * 16, np.uint8).tobytes())
        plain = torch.empty(NS * M * L, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(plain, 9)
        msg = plain.view(NS * M, L)
        hdr = torch.tensor(list(b"FPNN") + [1, 0x80, 2, 0] + list((L - 16).to_bytes(4, "little")), dtype=torch.uint8,
                           device="cuda")
        msg[:, :12] = hdr
        wire = torch.empty_like(plain)
        iv0 = torch.from_numpy(ivs.copy()).cuda()
        pos0 = torch.zeros(NS, dtype=torch.int32, device="cuda")
        iv_e, pos_e = iv0.clone(), pos0.clone()
        eng.stream_encrypt(plain, wire, NS, ks, iv_e, pos_e, stride=M * L, uniform_len=M * L)
        out_buf = torch.empty_like(wire)
        seg_len = torch.full((NS,), M * L, dtype=torch.int32, device="cuda")
        seg_off = torch.arange(NS, dtype=torch.int64, device="cuda") * (M * L)
        state = {}

        def recv():
            state["iv"], state["pos"] = iv0.clone(), pos0.clone()
            return eng.stream_recv(wire, out_buf, NS, ks, state["iv"], state["pos"], 8 << 20, M, in_off=seg_off,
                                   lens=seg_len)

        wr, kr, _ = timed(eng, D, recv, args.reps)
        foff, flen, scan = recv()
        torch.cuda.synchronize()
        frames, status, consumed = fpnn_amd.Engine.decode_scan(scan)
        assert (frames == M).all() and (status == 0).all() and (consumed == M * L).all(), "R2 framing"
        assert torch.equal(out_buf, plain), "R2 plaintext differs"
        assert torch.equal(state["iv"], iv_e) and torch.equal(state["pos"], pos_e), "R2 stream state"
        out["R2"] = {"streams": NS, "messages": NS * M, "bytes": NS * M * L, "recv_wall_GiBs": gib(NS * M * L, wr),
                     "decrypt_kernel_GiBs": gib(NS * M * L, kr),
                     "note": "fpnn_aes_stream_recv over 4096 AES-128 streams x 256 KiB (256 FPNN messages of 1 KiB "
                             "each): decrypt with carried state + device message scan; no host sync"}
        del plain, wire, out_buf
        print(json.dumps({"R2": out["R2"]}), flush=True)

    print(json.dumps({"configs": out, "timing": f"median of 3 rounds of {args.reps} back-to-back calls after 2 warm-up calls "
                                                  "(steady state, as bench.py); kernel = HIP events around the main "
                                                  "kernel on the engine stream, per launch"}))


if __name__ == "__main__":
    main()
