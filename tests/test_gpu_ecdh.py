"""ECDH key derivation on the GPU (include/fpnn_ecdh.h, k_ecdh.hip) against the reference:
tests/golden/ecdh_cases.json holds the outputs of core/KeyExchange.cpp + core/micro-ecc
run here (oracle/_ref/ecdh_ref); oracle/ecdh_oracle.py (pinned by the same fixtures) checks
random inputs.  Full-size property: 65 536 connections (config C5's key table) derived on
both sides agree byte for byte."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ecdh_oracle as E  # noqa: E402


def _dev(b: bytes) -> torch.Tensor:
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(DEV)


def _golden(golden):
    return golden("ecdh_cases.json")["curves"]


def test_server_batch_matches_reference(engine, golden):
    """fpnn_ecdh_calc_keys: one server private key, the fixture's peers as one batch per
    (private key, keylen) -- every peer whose lengths the reference accepts."""
    for cv in _golden(golden):
        c = E.CURVES[cv["curve"]]
        groups = {}
        for s in cv["server"]:
            if len(s["private"]) // 2 == c.private_bytes and len(s["peer"]) // 2 == 2 * c.num_bytes \
                    and s["keylen"] in (16, 32):
                groups.setdefault((s["private"], s["keylen"]), []).append(s)
        assert groups
        for (priv, kl), cases in groups.items():
            peers = _dev(b"".join(bytes.fromhex(s["peer"]) for s in cases))
            keys, ivs, ok = engine.ecdh_calc_keys(cv["curve"], bytes.fromhex(priv), peers, kl)
            torch.cuda.synchronize()
            keys, ivs, ok = keys.cpu().numpy(), ivs.cpu().numpy(), ok.cpu().numpy()
            for i, s in enumerate(cases):
                assert ok[i] == s["ok"], (cv["curve"], s)
                if s["ok"]:
                    assert (keys[i].tobytes().hex(), ivs[i].tobytes().hex()) == (s["key"], s["iv"]), (cv["curve"], s)


def test_client_side_matches_reference(engine, golden):
    """fpnn_ecdh_public_keys (ECCKeysMaker::publicKey's key pair) and
    fpnn_ecdh_calc_keys_client (ECCKeysMaker::calcKey) for the fixture's clients."""
    for cv in _golden(golden):
        cl = cv["clients"]
        privs = _dev(b"".join(bytes.fromhex(x["private"]) for x in cl))
        pub, ok = engine.ecdh_public_keys(cv["curve"], privs)
        torch.cuda.synchronize()
        pub, ok = pub.cpu().numpy(), ok.cpu().numpy()
        for i, x in enumerate(cl):
            assert ok[i] == 1 and pub[i].tobytes().hex() == x["public"], cv["curve"]
        for kl in (16, 32):
            keys, ivs, ok = engine.ecdh_calc_keys_client(cv["curve"], privs, bytes.fromhex(cv["server_public"]), kl)
            torch.cuda.synchronize()
            keys, ivs, ok = keys.cpu().numpy(), ivs.cpu().numpy(), ok.cpu().numpy()
            for i, x in enumerate(cl):
                if x["keylen"] == kl:
                    assert (int(ok[i]), keys[i].tobytes().hex(), ivs[i].tobytes().hex()) == (x["ok"], x["key"], x["iv"])


def test_single_call_matches_reference_incl_length_checks(engine, golden):
    """fpnn_ecdh_calc_key_host = ECCKeyExchange::init + calcKey, every fixture case,
    including the wrong-length private keys / peers and the unsupported keylen."""
    for cv in _golden(golden):
        for s in cv["server"]:
            ok, key, iv = engine.ecdh_calc_key_host(cv["curve"], bytes.fromhex(s["private"]),
                                                    bytes.fromhex(s["peer"]), s["keylen"])
            assert (int(ok), key.hex(), iv.hex()) == (s["ok"], s["key"], s["iv"]), (cv["curve"], s)
    assert engine.ecdh_calc_key_host("secp999k1", bytes(32), bytes(64), 16)[0] is False


@pytest.mark.parametrize("curve", sorted(E.CURVES))
def test_random_peers_vs_oracle(engine, curve):
    """Random private keys (incl. the degenerate 1, n-1, n-2 and keys >= n), random on-curve
    peers and random off-curve peers, against the oracle restatement."""
    c = E.CURVES[curve]
    rng = np.random.default_rng(len(curve) * 7 + c.num_bytes)
    n = 96
    privs = [int.from_bytes(rng.bytes(c.private_bytes), "big") % c.n for _ in range(n)]
    privs[:4] = [1, c.n - 1, c.n - 2, 2]
    pb = b"".join(k.to_bytes(c.private_bytes, "big") for k in privs)
    pub, ok = engine.ecdh_public_keys(curve, _dev(pb))
    torch.cuda.synchronize()
    pub, ok = pub.cpu().numpy(), ok.cpu().numpy()
    for i, k in enumerate(privs):
        eok, epub = E.public_key(c, k.to_bytes(c.private_bytes, "big"))
        assert (bool(ok[i]), pub[i].tobytes()) == (eok, epub) or (not eok and not ok[i]), (curve, i)
    peers = [pub[i].tobytes() for i in range(n)]
    peers[5] = rng.bytes(2 * c.num_bytes)  # off the curve
    peers[6] = bytes(2 * c.num_bytes)
    for server in (int.from_bytes(rng.bytes(c.private_bytes), "big").to_bytes(c.private_bytes, "big"),
                   b"\xff" * c.private_bytes):
        for kl in (16, 32):
            keys, ivs, okk = engine.ecdh_calc_keys(curve, server, _dev(b"".join(peers)), kl)
            torch.cuda.synchronize()
            keys, ivs, okk = keys.cpu().numpy(), ivs.cpu().numpy(), okk.cpu().numpy()
            for i, p in enumerate(peers):
                eok, ek, ei = E.calc_key(curve, server, p, kl)
                assert bool(okk[i]) == eok, (curve, i)
                if eok:
                    assert keys[i].tobytes() == ek and ivs[i].tobytes() == ei, (curve, i, kl)


def test_c5_key_table_both_sides_agree(engine, oracle):
    """Config C5's 65 536 connections: client key pairs, the server's derivation and each
    client's derivation agree byte for byte (size-independent property), a sample matches
    the oracle, and the derived key set encrypts packages exactly as the reference would
    with those keys."""
    curve, n, kl = "secp256k1", 65536, 32
    c = E.CURVES[curve]
    rng = np.random.default_rng(65536)
    privs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).to(DEV)
    privs[:, 0] &= 0x7F  # below n
    pub, pok = engine.ecdh_public_keys(curve, privs)
    server = bytes(rng.integers(1, 255, 32, dtype=np.uint8))
    server_pub, sok = engine.ecdh_public_keys(curve, _dev(server))
    ks, ok = engine.ecdh_keyset(curve, server, pub, kl)
    skeys, sivs, sok2 = engine.ecdh_calc_keys(curve, server, pub, kl)
    ckeys, civs, cok = engine.ecdh_calc_keys_client(curve, privs, server_pub.cpu().numpy().tobytes(), kl)
    torch.cuda.synchronize()
    assert bool(pok.all()) and bool(ok.all()) and bool(sok2.all()) and bool(cok.all())
    assert torch.equal(skeys, ckeys) and torch.equal(sivs, civs)
    sk, si, pp = skeys.cpu().numpy(), sivs.cpu().numpy(), pub.cpu().numpy()
    for i in rng.choice(n, 24, replace=False):
        eok, ek, ei = E.calc_key(curve, server, pp[i].tobytes(), kl)
        assert eok and sk[i].tobytes() == ek and si[i].tobytes() == ei
    # the key set from fpnn_ecdh_keyset encrypts like PackageEncryptor(key_i, iv_i)
    m, L = 512, 100
    slots = rng.choice(n, m, replace=False).astype(np.int32)
    data = rng.integers(0, 256, m * L, dtype=np.uint8)
    buf = torch.from_numpy(data.copy()).to(DEV)
    engine.package_encrypt(buf, buf, m, ks, stride=L, uniform_len=L, key_slot=torch.from_numpy(slots).to(DEV))
    torch.cuda.synchronize()
    out = buf.cpu().numpy()
    for j in range(0, m, 37):
        s = slots[j]
        exp = oracle.package(sk[s].tobytes(), si[s].tobytes(), True, data[j * L:(j + 1) * L].tobytes())
        assert out[j * L:(j + 1) * L].tobytes() == exp
    assert E.public_key(c, server)[1] == server_pub.cpu().numpy().tobytes()


def test_cpp_keyexchange_dropin(tmp_path, golden):
    """tests/cpp/keyexchange.cpp: the reference-shaped fpnn::ECCKeyExchange / ECCKeysMaker
    (include/KeyExchange.h) linked to libfpnn_aes.so alone -- golden server cases through
    init + calcKey, and a client/server round trip through ECCKeysMaker::publicKey."""
    import fpnn_amd
    exe = os.path.join(str(tmp_path), "keyexchange")
    libdir = os.path.dirname(fpnn_amd.LIB_PATH)
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "keyexchange.cpp"), "-o", exe, "-L", libdir, "-lfpnn_aes",
                    f"-Wl,-rpath,{libdir}"], check=True, capture_output=True, text=True)
    lines = []
    for cv in _golden(golden):
        for s in cv["server"]:
            lines.append(f"S {cv['curve']} {s['private'] or '-'} {s['peer'] or '-'} {s['keylen']}")
        lines.append(f"R {cv['curve']} - - 32")
    r = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = r.stdout.splitlines()
    k = 0
    for cv in _golden(golden):
        for s in cv["server"]:
            init_ok, ok, key, iv = out[k].split()
            k += 1
            assert (int(ok), key.replace("-", ""), iv.replace("-", "")) == (s["ok"], s["key"], s["iv"]), s
        assert out[k] == "roundtrip 1", (cv["curve"], out[k])
        k += 1
