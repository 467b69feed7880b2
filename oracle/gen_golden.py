#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the REFERENCE itself -- test infrastructure.

Runs oracle/_ref/libfpnn_ref.so, i.e. the reference's own base/rijndael.c and
core/Encryptor.cpp compiled by `make -C oracle ref` from /root/reference (this
container only).  Writes data only -- inputs and the reference's outputs:

  kat.json          FIPS-197 C.1/C.3, SP 800-38A F.3.13/F.3.17 (inputs + reference outputs)
  cfb_cases.json    random rijndael_cfb_encrypt calls (16/24/32-byte keys, pos carry)
  package_cases.json PackageEncryptor encrypt / decrypt / encrypt(std::string*) frames
  stream_cases.json StreamEncryptor call sequences (state carried across frames)
  modes_cases.json  the rest of rijndael.h: setup_decrypt, ECB decrypt, CBC, OFB
  framing_cases.json wire streams through the reference's EncryptedPackageReceiver /
                    EncryptedStreamReceiver (oracle/_ref/framing_ref): frames, plaintexts, verdicts
  ecdh_cases.json   ECCKeyExchange / ECCKeysMaker (core/KeyExchange.cpp + micro-ecc) on the
                    four curves (oracle/_ref/ecdh_ref): public keys, derived keys and IVs
  digests.json      SHA-256 digests of full-size synthetic config batches (C2, C3, C5) and
                    per-rank shard digests of the bench workloads (C2 r0-7, C4/C5 at world 1/2/4/8)

Usage: python oracle/gen_golden.py [--skip-large]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from pyoracle import Oracle, StreamOracle, synth_bytes  # noqa: E402
sys.path.insert(0, os.path.dirname(HERE))
import workloads as configs  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(HERE), "tests", "golden")


def hx(b: bytes) -> str:
    return b.hex()


def gen_kat(ref: Oracle):
    k128 = bytes(range(16))
    k256 = bytes(range(32))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    sp_pt = bytes.fromhex("6bc1bee22e409f96e93d7e117393172aae2d8a571e03ac9c9eb76fac45af8e51"
                          "30c81c46a35ce411e5fbc1191a0a52eff69f2445df4f9b17ad2b417be66c3710")
    k_sp128 = bytes.fromhex("2b7e151628aed2a6abf7158809cf4f3c")
    k_sp256 = bytes.fromhex("603deb1015ca71be2b73aef0857d77811f352c073b6108d72d9810a30914dff4")
    iv = bytes(range(16))
    out = {
        "ecb": [
            {"name": "FIPS-197 C.1 AES-128", "key": hx(k128), "in": hx(pt), "out": hx(ref.encrypt_block(k128, pt))},
            {"name": "FIPS-197 C.3 AES-256", "key": hx(k256), "in": hx(pt), "out": hx(ref.encrypt_block(k256, pt))},
        ],
        "cfb": [
            {"name": "SP800-38A F.3.13 CFB128-AES128", "key": hx(k_sp128), "iv": hx(iv), "in": hx(sp_pt),
             "out": hx(ref.cfb(k_sp128, True, sp_pt, iv)[0])},
            {"name": "SP800-38A F.3.17 CFB128-AES256", "key": hx(k_sp256), "iv": hx(iv), "in": hx(sp_pt),
             "out": hx(ref.cfb(k_sp256, True, sp_pt, iv)[0])},
        ],
        "source": "outputs produced by oracle/_ref (reference base/rijndael.c)",
    }
    return out


def gen_cfb_cases(ref: Oracle, n=240):
    rng = np.random.default_rng(20261015)
    cases = []
    for i in range(n):
        kl = (16, 24, 32)[i % 3]
        key = rng.bytes(kl)
        iv = rng.bytes(16)
        pos = int(rng.integers(0, 16)) if i % 4 else 0
        length = int(rng.choice([0, 1, 2, 15, 16, 17, 31, 32, 33, 47, 48, 63, 64, 65, 100, 255, 256, 257, 1000]))
        data = rng.bytes(length)
        enc = bool(i & 1)
        out, iv2, pos2 = ref.cfb(key, enc, data, iv, pos)
        cases.append({"key": hx(key), "iv": hx(iv), "pos": pos, "encrypt": enc, "in": hx(data), "out": hx(out),
                      "iv_out": hx(iv2), "pos_out": pos2})
    return cases


def gen_package_cases(ref: Oracle):
    rng = np.random.default_rng(7)
    cases = []
    lens = [0, 1, 3, 15, 16, 17, 31, 32, 33, 64, 100, 145, 1023, 1024, 1025, 1500, 4096]
    for kl in (16, 32):
        key = rng.bytes(kl)
        iv = rng.bytes(16)
        for L in lens:
            data = rng.bytes(L)
            cases.append({"key": hx(key), "iv": hx(iv), "in": hx(data),
                          "encrypt": hx(ref.package(key, iv, True, data)),
                          "decrypt": hx(ref.package(key, iv, False, data)),
                          "frame": hx(ref.package_frame(key, iv, data))})
    # the reference's own demo inputs (base/test/rijndaelDemo.cpp:13-31, round trip only there)
    key = b"aaaaaaaaaaaaaaaa"
    data = b"dasdsa as dsadasd sadsad eesewfsfsf sdfdssfsdfsdf wrwerfw fea fsfdfdsf ewrsfds"
    cases.append({"key": hx(key), "iv": hx(key), "in": hx(data), "encrypt": hx(ref.package(key, key, True, data)),
                  "decrypt": hx(ref.package(key, key, False, data)), "frame": hx(ref.package_frame(key, key, data))})
    return cases


def gen_modes_cases(ref: Oracle, n=150):
    """The rest of rijndael.h: setup_decrypt schedules, single-block decrypt (FIPS-197
    C.1/C.3 inverse + random), CBC encrypt/decrypt (partial last blocks) and OFB (random
    pos carry) -- base/rijndael.c:805-850, 961-1169, run by oracle/_ref."""
    rng = np.random.default_rng(20261016)
    out = {"setup_decrypt": [], "ecb_decrypt": [], "cbc": [], "ofb": []}
    for i in range(24):
        kl = (16, 24, 32)[i % 3]
        key = rng.bytes(kl)
        ctx = ref.setup_decrypt(key)
        out["setup_decrypt"].append({"key": hx(key), "nrounds": ctx.nrounds,
                                     "rk": [int(x) for x in ctx.rk[:4 * (ctx.nrounds + 1)]]})
    fips = [(bytes(range(16)), "69c4e0d86a7b0430d8cdb78070b4c55a"), (bytes(range(32)), "8ea2b7ca516745bfeafc49904b496089")]
    for key, ct in fips:
        out["ecb_decrypt"].append({"key": hx(key), "in": ct, "out": hx(ref.decrypt_block(key, bytes.fromhex(ct)))})
    for i in range(30):
        key = rng.bytes((16, 24, 32)[i % 3])
        blk = rng.bytes(16)
        out["ecb_decrypt"].append({"key": hx(key), "in": hx(blk), "out": hx(ref.decrypt_block(key, blk))})
    lens = [0, 1, 15, 16, 17, 31, 32, 33, 48, 100, 255, 256, 1000]
    for i in range(n):
        key = rng.bytes((16, 24, 32)[i % 3])
        iv = rng.bytes(16)
        L = lens[i % len(lens)]
        data = rng.bytes((L + 15) // 16 * 16)
        enc = bool(i & 1)
        res, iv2 = ref.cbc(key, enc, data[:L] if enc else data, iv, L)
        # decrypt: the reference reads whole 16-byte blocks of ciphertext, writes len bytes
        out["cbc"].append({"key": hx(key), "iv": hx(iv), "encrypt": enc, "len": L,
                           "in": hx(data[:L] if enc else data), "out": hx(res), "iv_out": hx(iv2)})
        pos = int(rng.integers(0, 16)) if i % 3 else 0
        o, iv3, pos3 = ref.ofb(key, data[:L], iv, pos)
        out["ofb"].append({"key": hx(key), "iv": hx(iv), "pos": pos, "in": hx(data[:L]), "out": hx(o),
                           "iv_out": hx(iv3), "pos_out": pos3})
    return out


def gen_stream_cases(ref: Oracle):
    rng = np.random.default_rng(11)
    cases = []
    for kl in (16, 32):
        for enc in (True, False):
            key = rng.bytes(kl)
            iv = rng.bytes(16)
            h = ref._snew(ref_buf(key), kl, ref_buf(iv))
            frames = []
            for _ in range(12):
                L = int(rng.choice([0, 1, 5, 11, 12, 16, 29, 64, 100, 333]))
                data = rng.bytes(L)
                outb = (np.zeros(max(1, L), dtype=np.uint8))
                ref._scrypt(h, int(enc), ref_buf(data), outb.ctypes.data_as(ref_u8p()), L)
                frames.append({"in": hx(data), "out": hx(outb.tobytes()[:L])})
            ref._sfree(h)
            cases.append({"key": hx(key), "iv": hx(iv), "encrypt": enc, "frames": frames})
    return cases


FRAMING_REF = os.path.join(HERE, "_ref", "framing_ref")
MAX_DEFAULT = 8 * 1024 * 1024  # FPNN_DEFAULT_MAX_PACKAGE_LEN, core/Config.h:14


def fp_message(rng, mtype: int, ss: int, payload: int, magic=b"FPNN", psize=None) -> bytes:
    """An FPNN TCP message (proto/FPMessage.h:56-63 header; FPQuest/FPAnswer::raw() body
    order): header, seq (two-way quest / answer), method (quest, ss bytes), payload."""
    ps = payload if psize is None else psize
    hdr = magic + bytes([1, 0x80, mtype, ss]) + (ps & 0xFFFFFFFF).to_bytes(4, "little")
    seq = rng.integers(0, 1 << 32).item().to_bytes(4, "little") if mtype in (1, 2) else b""
    method = bytes(rng.choice(list(b"abcdefghijklmnopqrstuvwxyz_"), ss).tolist()) if mtype in (0, 1) else b""
    return hdr + seq + method + rng.bytes(payload)


def _valid_messages(rng, n, max_payload):
    out = []
    for _ in range(n):
        mt = int(rng.integers(0, 3))
        ss = int(rng.integers(1, 40)) if mt != 2 else int(rng.integers(0, 2))
        out.append(fp_message(rng, mt, ss, int(rng.integers(1, max_payload + 1))))
    return out


def run_framing_ref(mode: str, key: bytes, iv: bytes, max_len: int, piece: int, wire: bytes):
    """Feed `wire` to the reference receiver (oracle/framing_ref.cpp) -> (events, end)."""
    import struct
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        cin, cout = os.path.join(d, "case.bin"), os.path.join(d, "out.jsonl")
        with open(cin, "wb") as f:
            f.write(b"FRG1" + struct.pack("<II", 0 if mode == "package" else 1, len(key)) + key + iv
                    + struct.pack("<iIQ", max_len, piece, len(wire)) + wire)
        subprocess.run([FRAMING_REF, cin, cout], check=True, timeout=120, stdout=subprocess.DEVNULL)
        with open(cout) as f:
            lines = [json.loads(x) for x in f]
    assert lines and "end" in lines[-1], lines
    return lines[:-1], lines[-1]


def gen_framing_cases(ref: Oracle):
    """Wire streams run through the reference's own EncryptedPackageReceiver /
    EncryptedStreamReceiver (core/EncryptedPackageReceiver.cpp:60-150,
    core/EncryptedStreamReceiver.cpp:72-163, with proto/FPMessage.cpp:27-44 BodyLen) over a
    socketpair: every complete frame, the plaintext the receiver decoded (FPQuest/FPAnswer
    raw()), and its verdict at the end of the data.  Each wire is fed in three piece sizes
    and must give identical events (arrival chunking does not change framing)."""
    rng = np.random.default_rng(20261017)
    cases = []

    def add(name, mode, kl, max_len, wire_fn, expect):
        key, iv = rng.bytes(kl), rng.bytes(16)
        wire = wire_fn(key, iv)
        runs = [run_framing_ref(mode, key, iv, max_len, p, wire) for p in (1, 7, 65536)]
        for r in runs[1:]:
            assert r[0] == runs[0][0] and r[1]["end"] == runs[0][1]["end"], name
        ev, end = runs[-1]
        cases.append({"name": name, "mode": mode, "key": hx(key), "iv": hx(iv), "max_len": max_len,
                      "wire": hx(wire), "frames": ev, "end": end, "expect": expect})
        print(f"  framing {name}: {len(ev)} frames, end {end}")

    def pkg(msgs, tail=b""):
        def wire(key, iv):
            w = b"".join(len(m).to_bytes(4, "little") + ref.package(key, iv, True, m) for m in msgs)
            return w + (tail(key, iv) if callable(tail) else tail)
        return wire

    def stream(msgs):
        return lambda key, iv: ref.cfb(key, True, b"".join(msgs), iv, 0)[0]

    # ---- package mode: [htole32(n)][n bytes of PackageEncryptor::encrypt] ----
    add("pkg_valid_aes256", "package", 32, MAX_DEFAULT, pkg(_valid_messages(rng, 24, 900)), "ok")
    add("pkg_valid_aes128", "package", 16, MAX_DEFAULT, pkg(_valid_messages(rng, 16, 300)), "ok")
    m = _valid_messages(rng, 6, 400)
    last = _valid_messages(rng, 1, 500)[0]
    add("pkg_partial_body", "package", 32, MAX_DEFAULT,
        pkg(m, lambda key, iv: len(last).to_bytes(4, "little") + ref.package(key, iv, True, last)[:len(last) // 2]),
        "ok")
    add("pkg_partial_prefix", "package", 16, MAX_DEFAULT, pkg(_valid_messages(rng, 5, 200), b"\x10\x02"), "ok")
    add("pkg_only_prefix", "package", 32, MAX_DEFAULT, pkg([], (777).to_bytes(4, "little")), "ok")
    cap_msg = fp_message(rng, 1, 8, 4096 - 12 - 4 - 8)  # exactly max_len bytes
    add("pkg_cap_boundary", "package", 32, 4096,
        pkg(_valid_messages(rng, 3, 300) + [cap_msg], (4097).to_bytes(4, "little") + rng.bytes(64)), "too_large")
    add("pkg_default_cap", "package", 16, MAX_DEFAULT,
        pkg(_valid_messages(rng, 4, 300), (MAX_DEFAULT + 1).to_bytes(4, "little") + rng.bytes(32)), "too_large")
    add("pkg_huge_prefix", "package", 32, MAX_DEFAULT,
        pkg(_valid_messages(rng, 2, 100), b"\xff\xff\xff\xff"), "too_large")
    garbage = [rng.bytes(int(rng.integers(1, 700))) for _ in range(10)]  # bodies that decode to nothing
    add("pkg_undecodable_bodies", "package", 32, MAX_DEFAULT, pkg(garbage), "ok")

    # ---- stream mode: one CFB stream over concatenated FPNN messages ----
    add("stream_valid_aes256", "stream", 32, MAX_DEFAULT, stream(_valid_messages(rng, 24, 900)), "ok")
    add("stream_valid_aes128", "stream", 16, MAX_DEFAULT, stream(_valid_messages(rng, 16, 300)), "ok")
    m = _valid_messages(rng, 6, 400)
    part = _valid_messages(rng, 1, 600)[0]
    add("stream_partial_body", "stream", 32, MAX_DEFAULT, stream(m + [part[:len(part) // 2]]), "ok")
    add("stream_partial_header", "stream", 16, MAX_DEFAULT, stream(_valid_messages(rng, 4, 200) + [part[:7]]), "ok")
    add("stream_bad_magic", "stream", 32, MAX_DEFAULT,
        stream(_valid_messages(rng, 3, 200) + [fp_message(rng, 1, 4, 30, magic=b"FPNX")]), "bad_magic")
    add("stream_http_magic", "stream", 16, MAX_DEFAULT,
        stream(_valid_messages(rng, 2, 200) + [b"POST / HTTP/1.1\r\n\r\n"]), "bad_magic")
    add("stream_bad_mtype", "stream", 32, MAX_DEFAULT,
        stream(_valid_messages(rng, 2, 200) + [b"FPNN" + bytes([1, 0x80, 3, 0]) + bytes(20)]), "bad_mtype")
    add("stream_zero_bodylen", "stream", 16, MAX_DEFAULT,
        stream(_valid_messages(rng, 2, 100) + [b"FPNN" + bytes([1, 0x80, 0, 0]) + bytes(4) + bytes(8)]),
        "bad_length")
    add("stream_wrapping_bodylen", "stream", 32, MAX_DEFAULT,
        stream(_valid_messages(rng, 2, 100) + [fp_message(rng, 2, 0, 3, psize=0xFFFFFFF8)]), "bad_length")
    add("stream_uint32_wrap", "stream", 16, MAX_DEFAULT,  # BodyLen = 0xFFFFFFFF + 4 wraps to 3
        stream(_valid_messages(rng, 2, 100) + [fp_message(rng, 2, 0, 0, psize=0xFFFFFFFF)[:15]]
               + _valid_messages(rng, 2, 100)), "ok")
    add("stream_negative_int", "stream", 16, MAX_DEFAULT,
        stream(_valid_messages(rng, 1, 100) + [fp_message(rng, 0, 0, 3, psize=0x80000000)]), "bad_length")
    cap = fp_message(rng, 2, 0, 4096 - 12 - 4)  # exactly max_len bytes
    add("stream_cap_boundary", "stream", 32, 4096,
        stream(_valid_messages(rng, 3, 300) + [cap, fp_message(rng, 2, 0, 4096 - 12 - 4 + 1)]), "too_large")
    add("stream_default_cap", "stream", 16, MAX_DEFAULT,
        stream(_valid_messages(rng, 2, 300) + [fp_message(rng, 1, 5, 40, psize=MAX_DEFAULT)]), "too_large")
    return {"source": "reference receivers run by oracle/_ref/framing_ref (make -C oracle framing), "
                      "fed over a socketpair in 1-, 7- and 65536-byte pieces", "cases": cases}


ECHO_REF = os.path.join(HERE, "_ref", "io_echo_ref")
PERCALL_REF = os.path.join(HERE, "_ref", "percall_ref")
# (mode, keylen, quests, payload bytes, window): C1 itself first (BASELINE.json configs[0])
C1_ECHO_CASES = [("package", 32, 10000, 1024, 1), ("package", 16, 400, 1, 1), ("package", 32, 400, 15, 4),
                 ("package", 24, 300, 4000, 2), ("stream", 32, 2000, 1024, 8), ("stream", 16, 500, 333, 3),
                 ("stream", 32, 300, 17, 1)]


def gen_c1_cases():
    """Config C1 through the reference's own IO plumbing (oracle/io_echo.cpp built on the
    reference's core/IOBuffer.cpp SendBuffer, EncryptedPackageReceiver /
    EncryptedStreamReceiver and core/Encryptor.cpp + base/rijndael.c: `make -C oracle echo`):
    an encrypted echo over loopback TCP, the wire checksums of both directions per case; and
    C1's per-call shape (oracle/percall.cpp, `make -C oracle percall`): the checksum of 10 000
    PackageEncryptor::encrypt / encrypt(std::string*) outputs of 1 KiB."""
    import subprocess
    cases = []
    for mode, kl, n, plen, win in C1_ECHO_CASES:
        out = subprocess.run([ECHO_REF, "1" if mode == "stream" else "0", str(kl), str(n), str(plen), str(win)],
                             capture_output=True, text=True, check=True, timeout=300).stdout
        d = json.loads(out.strip().splitlines()[-1])
        assert d["answers_ok"], d
        cases.append({k: d[k] for k in ("mode", "keylen", "quests", "payload", "window", "wire_c2s_bytes",
                                        "wire_c2s_fnv", "wire_s2c_bytes", "wire_s2c_fnv")})
        print("  echo", cases[-1])
    pc = json.loads(subprocess.run([PERCALL_REF, "10000", "1024"], capture_output=True, text=True, check=True,
                                   timeout=300).stdout.strip().splitlines()[-1])
    return {"source": "reference SendBuffer + encrypted receivers (oracle/_ref/io_echo_ref) and reference "
                      "PackageEncryptor per call (oracle/_ref/percall_ref)",
            "echo": cases, "percall": {"frames": pc["frames"], "len": pc["len"], "checksum": pc["checksum"]}}


MULTI_REF = os.path.join(HERE, "_ref", "io_multi_ref")
# SURVEY 8f row 1 inside FPNN's IO plumbing (oracle/io_multi.cpp):
# (name, mode, keylen, conns, quests per conn, payload, window, threads).  M1 is the headline
# shape: 1 024 connections x window 8 x 1 KiB AES-256 package frames.
# M6 / M7: the client connections start as TCPClient's do -- the "*key"
# quest in the clear (SendBuffer::encryptAfterFirstPackage, core/IOBuffer.cpp:36-45,
# core/TCPClient.cpp:238-243), every later frame encrypted (io_multi's first_clear).
MULTI_CASES = [("M1", "package", 32, 1024, 32, 1024, 8, 1), ("M2", "package", 16, 1024, 16, 1024, 8, 4),
               ("M3", "package", 24, 300, 12, 3001, 4, 2), ("M4", "stream", 32, 1024, 16, 1024, 8, 1),
               ("M5", "stream", 16, 256, 24, 777, 4, 2),
               ("M6", "package", 32, 512, 8, 1024, 4, 2, True), ("M7", "stream", 16, 512, 8, 1024, 4, 2, True)]


def gen_multi_cases():
    """Many connections through the reference's own SendBuffer / encrypted receivers and
    cipher (`make -C oracle multi`): per case the folded wire digests of both directions.
    The digests do not depend on the thread count or the transport (each connection's byte
    stream is fixed by its key, IV and quests)."""
    import subprocess
    cases = []
    for name, mode, kl, conns, q, plen, win, thr, *fc in MULTI_CASES:
        first_clear = bool(fc and fc[0])
        out = subprocess.run([MULTI_REF, "1" if mode == "stream" else "0", str(kl), str(conns), str(q), str(plen),
                              str(win), str(thr), "1", "1" if first_clear else "0"],
                             capture_output=True, text=True, check=True, timeout=600).stdout
        d = json.loads(out.strip().splitlines()[-1])
        assert d["ok"] and d["answers_ok"], d
        c = {"name": name, "threads": thr}
        if first_clear:
            c["first_clear"] = True
        c.update({k: d[k] for k in ("mode", "keylen", "conns", "quests_per_conn", "payload", "window",
                                    "wire_c2s_bytes", "wire_c2s_fnv", "wire_s2c_bytes", "wire_s2c_fnv")})
        cases.append(c)
        print("  multi", c, "reference echo/s here:", d["echo_per_s"])
    return {"source": "reference SendBuffer + encrypted receivers + core/Encryptor.cpp + base/rijndael.c, "
                      "many connections (oracle/_ref/io_multi_ref, oracle/io_multi.cpp)", "cases": cases}


UDP_REF = os.path.join(HERE, "_ref", "udp_v2_ref")
# (curve, reinforce package, reinforce data, datagrams per session, seed): every curve, both
# key lengths on each channel
UDP_CASES = [("secp256k1", 0, 0, 300, 7001), ("secp256r1", 1, 1, 300, 7002), ("secp224r1", 0, 1, 200, 7003),
             ("secp192r1", 1, 0, 200, 7004)]


def gen_udp_cases():
    """The reference's UDPEncryptor (core/UDP.v2/UDPCommon.v2.cpp, oracle/udp_v2.cpp) on the
    reference cipher and key exchange (`make -C oracle udp`): per case the server's
    createPair sessions with two clients from ecdh_cases.json, datagrams both ways, and the
    ciphertext digests per channel and direction."""
    import subprocess
    with open(os.path.join(GOLDEN, "ecdh_cases.json")) as f:
        curves = {c["curve"]: c for c in json.load(f)["curves"]}
    cases = []
    for curve, rp, rd, n, seed in UDP_CASES:
        c = curves[curve]
        cl = [x for x in c["clients"] if x["ok"]][:2]
        line = " ".join([curve, c["server_private"], c["server_public"], cl[0]["private"], cl[0]["public"],
                         cl[1]["private"], cl[1]["public"], str(rp), str(rd), str(n), str(seed)])
        out = subprocess.run([UDP_REF], input=line + "\n", capture_output=True, text=True, check=True,
                             timeout=600).stdout
        d = json.loads([x for x in out.splitlines() if x.startswith("{")][-1])
        assert d["init_ok"] and d["pair_a"] and d["pair_b"] and d["client_ok"] and d["roundtrip_ok"], d
        secs = d.pop("seconds")
        cases.append({"input": line, "expect": d})
        print("  udp", curve, d, "reference seconds here:", secs)
    return {"source": "core/UDP.v2/UDPCommon.v2.cpp + core/KeyExchange.cpp + micro-ecc + core/Encryptor.cpp + "
                      "base/rijndael.c (oracle/_ref/udp_v2_ref, oracle/udp_v2.cpp)", "cases": cases}


ECDH_REF = os.path.join(HERE, "_ref", "ecdh_ref")


def gen_ecdh_cases():
    """core/KeyExchange.cpp + core/micro-ecc run by oracle/_ref/ecdh_ref: per curve, client
    key pairs (ECCKeysMaker::publicKey with a chosen private key) and the keys both sides
    derive (ECCKeysMaker::calcKey / ECCKeyExchange::calcKey), plus edge inputs: degenerate
    private keys (1 fails in the co-Z ladder), keys >= n, off-curve / zero / non-reduced
    peer points and wrong lengths."""
    import subprocess
    from ecdh_oracle import CURVES
    rng = np.random.default_rng(20261018)
    lines, meta = [], []

    def run(reqs):
        r = subprocess.run([ECDH_REF], input="\n".join(reqs) + "\n", capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
        res = [ln[2:] for ln in r.stdout.splitlines() if ln.startswith("R ")]
        assert len(res) == len(reqs), (len(res), len(reqs))
        return res

    def rand_below(top):
        while True:
            v = int.from_bytes(rng.bytes((top.bit_length() + 7) // 8), "big") >> (8 - top.bit_length() % 8) % 8
            if 0 < v < top:
                return v

    out = {"source": "oracle/_ref/ecdh_ref: the reference's core/KeyExchange.cpp + core/micro-ecc/uECC.c",
           "curves": []}
    for name, c in CURVES.items():
        nb, pb = c.num_bytes, c.private_bytes
        words = (c.num_n_bits + 63) // 64  # uECC_generate_random_int draws whole 64-bit words (x86-64)
        server = rand_below(c.n).to_bytes(pb, "big")
        # the server's public key, as a client of itself would compute it
        lines.append(f"C {name} {int.from_bytes(server, 'big').to_bytes(8 * words, 'little').hex()} - 16")
        meta.append(("server_pub",))
        privs = [rand_below(c.n) for _ in range(10)] + [2, c.n - 1, c.n - 2, (c.n - 1) // 2]
        for j, k in enumerate(privs):
            lines.append(f"C {name} {k.to_bytes(8 * words, 'little').hex()} SERVERPUB {(16, 32)[j % 2]}")
            meta.append(("client", k, (16, 32)[j % 2]))
        ent = {"curve": name, "server_private": server.hex(), "clients": [], "server": []}
        out["curves"].append(ent)
        # resolve the server public key first
        server_pub = run(lines[:1])[0].split()[0]
        ent["server_public"] = server_pub
        req = [ln.replace("SERVERPUB", server_pub) for ln in lines[1:]]
        res = run(req)
        for (_, k, kl), r in zip(meta[1:], res):
            pub, priv, ok, key, iv = r.split()
            ent["clients"].append({"private": priv, "public": pub, "keylen": kl, "ok": int(ok),
                                   "key": "" if key == "-" else key, "iv": "" if iv == "-" else iv})
        lines, meta = [], []
        # server side: every client's public key, then edge inputs
        peers = [(cl["public"], cl["keylen"]) for cl in ent["clients"]]
        p = c.p
        offc = (rng.bytes(2 * nb).hex(), 32)
        nonreduced = (p + 1).to_bytes(nb, "big").hex() + ent["clients"][0]["public"][2 * nb:]  # x = p + 1
        peers += [offc, ("00" * (2 * nb), 16), (nonreduced, 32),
                  (ent["clients"][1]["public"][:-2], 32),              # one byte short
                  (ent["clients"][2]["public"], 24)]                   # unsupported keylen
        for peer, kl in peers:
            lines.append(f"S {name} {server.hex()} {peer} {kl}")
        extra = [((1).to_bytes(pb, "big"), ent["clients"][3]["public"], 32),
                 ((c.n).to_bytes(pb, "big") if c.n < 1 << (8 * pb) else b"\xff" * pb, ent["clients"][4]["public"], 32),
                 (b"\xff" * pb, ent["clients"][5]["public"], 16),
                 (server[:-1], ent["clients"][6]["public"], 32)]        # private key one byte short
        for priv, peer, kl in extra:
            lines.append(f"S {name} {priv.hex() if priv else '-'} {peer} {kl}")
        res = run(lines)
        privs_used = [server.hex()] * len(peers) + [e[0].hex() for e in extra]
        reqs = peers + [(e[1], e[2]) for e in extra]
        for (peer, kl), priv, r in zip(reqs, privs_used, res):
            init_ok, ok, key, iv = r.split()
            ent["server"].append({"private": priv, "peer": peer, "keylen": kl, "init_ok": int(init_ok),
                                  "ok": int(ok), "key": "" if key == "-" else key, "iv": "" if iv == "-" else iv})
        lines, meta = [], []
        print(f"  ecdh {name}: {len(ent['clients'])} clients, {len(ent['server'])} server calls, "
              f"{sum(s['ok'] for s in ent['server'])} ok")
    return out


def ref_buf(b):
    import ctypes as C
    return C.cast(C.c_char_p(b), C.POINTER(C.c_uint8))


def ref_u8p():
    import ctypes as C
    return C.POINTER(C.c_uint8)


def digest_c2(ref: Oracle, threads: int):
    c = configs.C2
    key, iv = configs.single_key(c)
    P, L = c["packets"], c["length"]
    inp = synth_bytes(P * L, c["payload_seed"], threads=threads)
    out = np.empty_like(inp)
    ref.package_batch(True, inp, out, P, stride=L, uniform_len=L, keys=np.frombuffer(key, np.uint8).copy(),
                      keylen=len(key), ivs=np.frombuffer(iv, np.uint8).copy(), threads=threads)
    return {"config": "C2", "plain_sha256": hashlib.sha256(inp).hexdigest(),
            "cipher_sha256": hashlib.sha256(out).hexdigest(),
            "cipher_head_hex": out[:64].tobytes().hex()}


def digest_c5(ref: Oracle, threads: int):
    c = configs.C5
    keys, ivs = configs.many_keys(c)
    P, L = c["packets"], c["length"]
    inp = synth_bytes(P * L, c["payload_seed"], threads=threads)
    out = np.empty_like(inp)
    slots = np.arange(P, dtype=np.uint32)
    ref.package_batch(True, inp, out, P, stride=L, uniform_len=L, key_slot=slots, keys=keys, keylen=c["keylen"],
                      ivs=ivs, threads=threads)
    return {"config": "C5", "plain_sha256": hashlib.sha256(inp).hexdigest(),
            "cipher_sha256": hashlib.sha256(out).hexdigest()}


def digest_c3(ref: Oracle, threads: int):
    """Whole-stream ciphertext of every stream; digest = sha256(concat(sha256(stream_i)))."""
    c = configs.C3
    keys, ivs = configs.many_keys(c)
    S, L = c["streams"], c["length"]
    per = []
    group = 64
    for g0 in range(0, S, group):
        n = min(group, S - g0)
        inp = synth_bytes(n * L, c["payload_seed"], offset=g0 * L, threads=threads)
        out = np.empty_like(inp)
        in_off = (np.arange(n, dtype=np.uint64) * L)
        lens = np.full(n, L, dtype=np.uint32)
        slots = np.arange(g0, g0 + n, dtype=np.uint32)
        iv_state = ivs[16 * g0: 16 * (g0 + n)].copy()
        pos_state = np.zeros(n, dtype=np.uint32)
        ref.stream_batch(True, inp, out, n, in_off=in_off, out_off=in_off, lens=lens, key_slot=slots, keys=keys,
                         keylen=c["keylen"], iv_state=iv_state, pos_state=pos_state, threads=threads)
        for i in range(n):
            per.append(hashlib.sha256(out[i * L:(i + 1) * L]).digest())
    return {"config": "C3", "stream_digests_sha256": hashlib.sha256(b"".join(per)).hexdigest(),
            "first_stream_sha256": per[0].hex()}


def shard_digests(ref: Oracle, threads: int):
    """Per-rank reference digests of the bench's sharded workloads (bench.py setup_*):
    C2 weak scaling -- rank r owns packets [r*P, (r+1)*P) of one global batch, for any
    world size, so one digest per rank index r = 0..7; C4 (Zipf, byte-balanced contiguous
    ranges) and C5 (even packet split) strong scaling -- one digest per (world, rank) for
    world 1, 2, 4, 8.  The shard split is fpnn_amd/sharding.py's shard_range."""
    sys.path.insert(0, os.path.dirname(HERE))
    from fpnn_amd.sharding import shard_range
    out = {}
    c = configs.C2
    key, iv = configs.single_key(c)
    P, L = c["packets"], c["length"]
    kb, ib = np.frombuffer(key, np.uint8).copy(), np.frombuffer(iv, np.uint8).copy()
    for r in range(8):
        inp = synth_bytes(P * L, c["payload_seed"], offset=r * P * L, threads=threads)
        enc = np.empty_like(inp)
        ref.package_batch(True, inp, enc, P, stride=L, uniform_len=L, keys=kb, keylen=len(key), ivs=ib,
                          threads=threads)
        out[f"C2/r{r}"] = hashlib.sha256(enc).hexdigest()
        print("C2 shard", r, out[f"C2/r{r}"], flush=True)
    # C4: the whole 4 GiB batch once, then each shard's byte range
    c = configs.C4
    sizes = configs.zipf_sizes(c).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(sizes[:-1])]).astype(np.uint64)
    total = int(sizes.sum())
    key, iv = configs.single_key(c)
    inp = synth_bytes(total, c["payload_seed"], threads=threads)
    enc = np.empty_like(inp)
    ref.package_batch(True, inp, enc, len(sizes), in_off=offs, lens=sizes.astype(np.uint32),
                      keys=np.frombuffer(key, np.uint8).copy(), keylen=len(key),
                      ivs=np.frombuffer(iv, np.uint8).copy(), threads=threads)
    del inp
    for world in (1, 2, 4, 8):
        for r in range(world):
            a, b = shard_range(len(sizes), world, r, sizes)
            lo = int(offs[a]) if b > a else 0
            hi = int(offs[b - 1] + sizes[b - 1]) if b > a else 0
            out[f"C4/w{world}/r{r}"] = hashlib.sha256(enc[lo:hi]).hexdigest()
    del enc
    # C5: 65 536 keyed packets, split evenly
    c = configs.C5
    keys, ivs = configs.many_keys(c)
    P, L = c["packets"], c["length"]
    inp = synth_bytes(P * L, c["payload_seed"], threads=threads)
    enc = np.empty_like(inp)
    ref.package_batch(True, inp, enc, P, stride=L, uniform_len=L, key_slot=np.arange(P, dtype=np.uint32), keys=keys,
                      keylen=c["keylen"], ivs=ivs, threads=threads)
    for world in (1, 2, 4, 8):
        for r in range(world):
            a, b = shard_range(P, world, r)
            out[f"C5/w{world}/r{r}"] = hashlib.sha256(enc[a * L:b * L]).hexdigest()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-large", action="store_true")
    ap.add_argument("--shards-only", action="store_true",
                    help="only (re)compute the per-rank shard digests into digests.json")
    ap.add_argument("--modes-only", action="store_true", help="only (re)write modes_cases.json")
    ap.add_argument("--framing-only", action="store_true", help="only (re)write framing_cases.json")
    ap.add_argument("--ecdh-only", action="store_true", help="only (re)write ecdh_cases.json")
    ap.add_argument("--c1-only", action="store_true", help="only (re)write c1_cases.json")
    ap.add_argument("--multi-only", action="store_true", help="only (re)write multi_cases.json")
    ap.add_argument("--udp-only", action="store_true", help="only (re)write udp_cases.json")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 4)
    args = ap.parse_args()
    ref = Oracle("reference")
    os.makedirs(GOLDEN, exist_ok=True)

    def dump(name, obj):
        with open(os.path.join(GOLDEN, name), "w") as f:
            json.dump(obj, f, indent=1)
        print("wrote", name)

    if args.modes_only:
        dump("modes_cases.json", gen_modes_cases(ref))
        return
    if args.framing_only:
        dump("framing_cases.json", gen_framing_cases(ref))
        return
    if args.ecdh_only:
        dump("ecdh_cases.json", gen_ecdh_cases())
        return
    if args.c1_only:
        dump("c1_cases.json", gen_c1_cases())
        return
    if args.multi_only:
        dump("multi_cases.json", gen_multi_cases())
        return
    if args.udp_only:
        dump("udp_cases.json", gen_udp_cases())
        return
    if args.shards_only:
        with open(os.path.join(GOLDEN, "digests.json")) as f:
            d = json.load(f)
        d["shards"] = shard_digests(ref, args.threads)
        dump("digests.json", d)
        return
    dump("kat.json", gen_kat(ref))
    dump("cfb_cases.json", gen_cfb_cases(ref))
    dump("package_cases.json", gen_package_cases(ref))
    dump("stream_cases.json", gen_stream_cases(ref))
    dump("modes_cases.json", gen_modes_cases(ref))
    dump("framing_cases.json", gen_framing_cases(ref))
    dump("ecdh_cases.json", gen_ecdh_cases())
    dump("c1_cases.json", gen_c1_cases())
    dump("multi_cases.json", gen_multi_cases())
    dump("udp_cases.json", gen_udp_cases())
    if not args.skip_large:
        d = {"generator": "oracle/gen_golden.py with oracle/_ref (reference base/rijndael.c + core/Encryptor.cpp)",
             "configs": configs.describe()}
        d["C2"] = digest_c2(ref, args.threads)
        print("C2", d["C2"])
        d["C5"] = digest_c5(ref, args.threads)
        print("C5", d["C5"])
        d["C3"] = digest_c3(ref, args.threads)
        print("C3", d["C3"])
        d["shards"] = shard_digests(ref, args.threads)
        dump("digests.json", d)


if __name__ == "__main__":
    main()
