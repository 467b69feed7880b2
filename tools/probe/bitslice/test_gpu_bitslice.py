"""The bitsliced co-kernel (K1b, fpnn_amd/csrc/bs_kernels.hip) against the oracle.

The engine routes a share FPNN_AES_BITSLICE_FRAC of a uniform package-decrypt batch
to K1b on a side stream (the rest to the T-table K1); 1.0 sends everything to K1b.
These cases also pin the v_bitop3 truth-table convention the generated S-box
circuit assumes (tools/gen_bitslice.py)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def engine_with_frac(frac):
    import fpnn_amd
    old = os.environ.get("FPNN_AES_BITSLICE_FRAC")
    os.environ["FPNN_AES_BITSLICE_FRAC"] = str(frac)
    try:
        return fpnn_amd.Engine(0)
    finally:
        if old is None:
            del os.environ["FPNN_AES_BITSLICE_FRAC"]
        else:
            os.environ["FPNN_AES_BITSLICE_FRAC"] = old


@pytest.mark.parametrize("keylen", [16, 24, 32])
@pytest.mark.parametrize("frac", [1.0, 0.37])
@pytest.mark.parametrize("length,stride", [(512, 512), (1024, 1024), (2048, 2064), (4096, 4096)])
def test_bitsliced_decrypt_matches_oracle(oracle, keylen, frac, length, stride):
    import fpnn_amd
    rng = np.random.default_rng(keylen * 1000 + length + int(frac * 100))
    n = 3001
    inp = rng.integers(0, 256, n * stride, dtype=np.uint8)
    key, iv = rng.bytes(keylen), rng.bytes(16)
    eng = engine_with_frac(frac)
    ks = fpnn_amd.KeySet(eng, key, keylen, iv)
    exp = inp.copy()
    oracle.package_batch(False, inp, exp, n, stride=stride, uniform_len=length,
                         keys=np.frombuffer(key, np.uint8).copy(), keylen=keylen,
                         ivs=np.frombuffer(iv, np.uint8).copy(), threads=8)
    src = torch.from_numpy(inp).to(DEV)
    dst = src.clone()
    eng.package_decrypt(src, dst, n, ks, stride=stride, uniform_len=length)
    torch.cuda.synchronize()
    assert np.array_equal(dst.cpu().numpy(), exp)
    eng.close()


def test_bitsliced_c2_roundtrip_and_digest(golden):
    """C2 at full size with half the decrypt batch on K1b."""
    import hashlib
    import fpnn_amd
    import workloads as W
    c = W.C2
    P, L = c["packets"], c["length"]
    key, iv = W.single_key(c)
    eng = engine_with_frac(0.5)
    ks = fpnn_amd.KeySet(eng, key, len(key), iv)
    plain = torch.empty(P * L, dtype=torch.uint8, device=DEV)
    eng.fill_synthetic(plain, c["payload_seed"])
    cipher = torch.empty_like(plain)
    eng.package_encrypt(plain, cipher, P, ks, stride=L, uniform_len=L)
    back = torch.empty_like(plain)
    eng.package_decrypt(cipher, back, P, ks, stride=L, uniform_len=L)
    torch.cuda.synchronize()
    assert hashlib.sha256(cipher.cpu().numpy()).hexdigest() == golden("digests.json")["C2"]["cipher_sha256"]
    assert torch.equal(back, plain)
    eng.close()
