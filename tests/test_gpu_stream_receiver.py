"""fpnn::StreamReceiverBatch (include/StreamReceiverBatch.h) driven from C++ the way an
IO loop would drive EncryptedStreamReceiver (core/EncryptedStreamReceiver.cpp:72-163):
tests/cpp/stream_recv.cpp feeds every connection's wire bytes in pieces (one piece per
connection per cycle) and flushes once per cycle.

  * the reference receivers' own fixtures (tests/golden/framing_cases.json, made by
    running core/EncryptedStreamReceiver.cpp over a socketpair, oracle/framing_ref.cpp):
    the messages fetch() decoded, the verdict, and for good streams the final
    StreamEncryptor state;
  * 200 synthetic connections of valid FPNN messages, encrypted by the oracle's CFB
    stream, against the messages themselves.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from framing_golden import expected, load_cases

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def stream_recv_exe(tmp_path_factory):
    import fpnn_amd
    exe = str(tmp_path_factory.mktemp("srx") / "stream_recv")
    libdir = os.path.dirname(fpnn_amd.LIB_PATH)
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "stream_recv.cpp"), "-o", exe, "-L", libdir, "-lfpnn_aes",
                    f"-Wl,-rpath,{libdir}"], check=True, capture_output=True, text=True)
    return exe


def _run(exe, conns, piece):
    """conns: [(max_len, key, iv, wire)] -> [(status, pending, iv, pos, fed, [messages])]"""
    lines = [f"{m} {k.hex()} {v.hex()} {w.hex() or '-'}" for m, k, v, w in conns]
    res = subprocess.run([exe, str(piece)], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         timeout=600)
    assert res.returncode == 0, res.stderr[-2000:]
    out = []
    for ln in res.stdout.strip().split("\n"):
        f = ln.split()
        out.append((int(f[0]), int(f[1]), bytes.fromhex(f[2]), int(f[3]), int(f[4]), [bytes.fromhex(x) for x in f[5:]]))
    return out


@pytest.mark.parametrize("piece", [1, 7, 65536])
def test_stream_receiver_batch_matches_reference_receiver(stream_recv_exe, oracle, piece):
    cases = [c for c in load_cases() if c["mode"] == "stream"]
    conns = [(c["max_len"], bytes.fromhex(c["key"]), bytes.fromhex(c["iv"]), bytes.fromhex(c["wire"])) for c in cases]
    got = _run(stream_recv_exe, conns, piece)
    for c, (m, key, iv, wire), (status, pending, iv_end, pos_end, fed, msgs) in zip(cases, conns, got):
        frames, es, consumed, raws = expected(c)
        assert status == es, c["name"]
        assert [len(x) for x in msgs] == [ln for _, ln in frames], c["name"]
        for j, raw in enumerate(raws):
            if raw is not None:  # the plaintext the reference receiver handed to its decoder
                assert msgs[j] == raw, (c["name"], j)
        if es == 0:  # a good stream: every byte read, the rest an incomplete message
            assert fed == len(wire) and pending == len(wire) - consumed, c["name"]
            _, iv_ref, pos_ref = oracle.cfb(key, False, wire, iv, 0)
            assert (iv_end, pos_end) == (iv_ref, pos_ref), c["name"]


def test_stream_receiver_batch_many_connections(stream_recv_exe, oracle):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from gen_golden import _valid_messages
    rng = np.random.default_rng(8088)
    conns, want = [], []
    for i in range(200):
        keylen = (16, 24, 32)[i % 3]
        key, iv = rng.bytes(keylen), rng.bytes(16)
        msgs = _valid_messages(rng, int(rng.integers(0, 12)), int(rng.integers(1, 3000)))
        extra = _valid_messages(rng, 1, 500)[0]
        tail = extra[: int(rng.integers(0, min(40, len(extra))))]  # an incomplete message (never all of it)
        plain = b"".join(msgs) + tail
        wire, _, _ = oracle.cfb(key, True, plain, iv, 0)
        conns.append((8 << 20, key, iv, wire))
        want.append((msgs, len(tail)))
    got = _run(stream_recv_exe, conns, 997)
    for i, ((msgs, tail), (status, pending, iv_end, pos_end, fed, got_msgs)) in enumerate(zip(want, got)):
        assert status == 0 and got_msgs == msgs and pending == tail, i
        _, iv_ref, pos_ref = oracle.cfb(conns[i][1], False, conns[i][3], conns[i][2], 0)
        assert (iv_end, pos_end) == (iv_ref, pos_ref), i
