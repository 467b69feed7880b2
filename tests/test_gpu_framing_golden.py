"""Device receive framing (fpnn_aes_package_recv / fpnn_aes_stream_recv) against the
reference's own receivers: tests/golden/framing_cases.json holds wire streams run through
core/EncryptedPackageReceiver.cpp / core/EncryptedStreamReceiver.cpp (built from the
reference sources by `make -C oracle framing`, see oracle/framing_ref.cpp).  Every case is
one connection's segment; the cases of one (mode, max_len, key length) go in one batch."""
import itertools

import numpy as np
import pytest
import torch

from framing_golden import expected, load_cases

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
MAX_FRAMES = 64


def _groups(mode):
    cases = [c for c in load_cases() if c["mode"] == mode]
    key = lambda c: (c["max_len"], len(c["key"]) // 2)  # noqa: E731
    return [(k, list(g)) for k, g in itertools.groupby(sorted(cases, key=key), key=key)]


def _layout(cases, lead):
    """Segments at ragged, unaligned offsets with `lead` free bytes in front of each."""
    wires = [bytes.fromhex(c["wire"]) for c in cases]
    offs, at = [], 0
    for w in wires:
        at += lead
        offs.append(at)
        at += len(w) + 5
    host = np.zeros(at + 16, dtype=np.uint8)
    for o, w in zip(offs, wires):
        host[o:o + len(w)] = np.frombuffer(w, np.uint8)
    return wires, np.array(offs, dtype=np.int64), host


@pytest.mark.parametrize("inplace", [False, True])
def test_package_recv_matches_reference_receiver(engine, inplace, scan_mode):
    import fpnn_amd
    for (max_len, keylen), cases in _groups("package"):
        n = len(cases)
        keys = b"".join(bytes.fromhex(c["key"]) for c in cases)
        ivs = b"".join(bytes.fromhex(c["iv"]) for c in cases)
        ks = fpnn_amd.KeySet(engine, keys, keylen, ivs)
        wires, offs, host = _layout(cases, 3)
        inp = torch.from_numpy(host).to(DEV)
        out = inp if inplace else torch.zeros_like(inp)
        foff, flen, scan = engine.package_recv(
            inp, out, n, ks, max_len, MAX_FRAMES, in_off=torch.from_numpy(offs).to(DEV),
            lens=torch.tensor([len(w) for w in wires], dtype=torch.int32, device=DEV),
            key_slot=torch.arange(n, dtype=torch.int32, device=DEV))
        torch.cuda.synchronize()
        frames, status, consumed = fpnn_amd.Engine.decode_scan(scan)
        foff, flen, res = foff.cpu().numpy(), flen.cpu().numpy(), out.cpu().numpy()
        for i, c in enumerate(cases):
            ef, es, ec, raws = expected(c)
            assert (frames[i], status[i], consumed[i]) == (len(ef), es, ec), c["name"]
            for j, ((o, ln), raw) in enumerate(zip(ef, raws)):
                assert (foff[i * MAX_FRAMES + j], flen[i * MAX_FRAMES + j]) == (o, ln), (c["name"], j)
                if raw is not None:  # the plaintext the reference receiver decoded
                    assert res[offs[i] + o:offs[i] + o + ln].tobytes() == raw, (c["name"], j)


def test_stream_recv_matches_reference_receiver(engine, oracle, scan_mode):
    import fpnn_amd
    for (max_len, keylen), cases in _groups("stream"):
        n = len(cases)
        keys = b"".join(bytes.fromhex(c["key"]) for c in cases)
        ks = fpnn_amd.KeySet(engine, keys, keylen, bytes(16 * n))
        iv0 = np.frombuffer(b"".join(bytes.fromhex(c["iv"]) for c in cases), np.uint8).copy()
        wires, offs, host = _layout(cases, 0)
        inp = torch.from_numpy(host).to(DEV)
        out = torch.zeros_like(inp)
        d_iv = torch.from_numpy(iv0).to(DEV)
        d_pos = torch.zeros(n, dtype=torch.int32, device=DEV)
        foff, flen, scan = engine.stream_recv(
            inp, out, n, ks, d_iv, d_pos, max_len, MAX_FRAMES, in_off=torch.from_numpy(offs).to(DEV),
            lens=torch.tensor([len(w) for w in wires], dtype=torch.int32, device=DEV),
            key_slot=torch.arange(n, dtype=torch.int32, device=DEV))
        torch.cuda.synchronize()
        frames, status, consumed = fpnn_amd.Engine.decode_scan(scan)
        foff, flen, res = foff.cpu().numpy(), flen.cpu().numpy(), out.cpu().numpy()
        ivs, poss = d_iv.cpu().numpy().reshape(n, 16), d_pos.cpu().numpy()
        for i, c in enumerate(cases):
            ef, es, ec, raws = expected(c)
            assert (frames[i], status[i], consumed[i]) == (len(ef), es, ec), c["name"]
            for j, ((o, ln), raw) in enumerate(zip(ef, raws)):
                assert (foff[i * MAX_FRAMES + j], flen[i * MAX_FRAMES + j]) == (o, ln), (c["name"], j)
                if raw is not None:
                    assert res[offs[i] + o:offs[i] + o + ln].tobytes() == raw, (c["name"], j)
            # the stream state advanced over every received byte
            _, iv_end, pos_end = oracle.cfb(bytes.fromhex(c["key"]), False, wires[i], bytes.fromhex(c["iv"]), 0)
            assert (ivs[i].tobytes(), int(poss[i])) == (iv_end, pos_end), c["name"]
