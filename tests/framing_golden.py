"""Expected scan results of the reference-generated framing fixtures
(tests/golden/framing_cases.json, made by oracle/gen_golden.py with oracle/_ref/framing_ref,
i.e. the reference's own EncryptedPackageReceiver / EncryptedStreamReceiver).

The receivers report every complete frame with its length (Receiver::_total) and the
plaintext they decoded, then a verdict at the end of the data: "incomplete" (the rest is a
partial frame kept for the next read), "closed" (recvPackage returned false: the frame is
above Config::_max_recv_package_length, or the stream header is not an FPNN message /
has length <= 0) or "exception" (FPMessage::BodyLen threw on an unknown mtype).  These map
onto the fpnn_aes_frame_scan of the batch receive calls."""
import json
import os

SCAN_OK, SCAN_FULL, SCAN_TOO_LARGE, SCAN_BAD_MAGIC, SCAN_BAD_MTYPE, SCAN_BAD_LENGTH = range(6)
_EXPECT = {"ok": SCAN_OK, "too_large": SCAN_TOO_LARGE, "bad_magic": SCAN_BAD_MAGIC, "bad_mtype": SCAN_BAD_MTYPE,
           "bad_length": SCAN_BAD_LENGTH}
_VERDICT = {"ok": "incomplete", "too_large": "closed", "bad_magic": "closed", "bad_length": "closed",
            "bad_mtype": "exception"}

HERE = os.path.dirname(os.path.abspath(__file__))


def load_cases():
    with open(os.path.join(HERE, "golden", "framing_cases.json")) as f:
        return json.load(f)["cases"]


def expected(case):
    """-> ([(offset, length)], status, consumed, [raw plaintext or None]) for one case.
    Package mode: offset of the body (after its 4-byte prefix) within the wire;
    stream mode: offset of the message within the plaintext stream."""
    assert case["end"]["end"] == _VERDICT[case["expect"]], case["name"]  # generator intent == reference verdict
    pre = 4 if case["mode"] == "package" else 0
    frames, raws, at = [], [], 0
    for ev in case["frames"]:
        frames.append((at + pre, ev["total"]))
        raws.append(bytes.fromhex(ev["raw"]) if ev["fetch"] else None)
        at += pre + ev["total"]
    return frames, _EXPECT[case["expect"]], at, raws


def run_receiver(exe, case, piece):
    """Feed one fixture's wire to a receiver driver built from oracle/framing_ref.cpp
    (oracle/_ref/framing_ref: the reference's receivers on the reference Encryptor;
    oracle/_ref/framing_dropin: the same receivers compiled unchanged against
    include/Encryptor.h on libfpnn_aes.so) -> (frame events, end event)."""
    import struct
    import subprocess
    import tempfile
    key, iv, wire = bytes.fromhex(case["key"]), bytes.fromhex(case["iv"]), bytes.fromhex(case["wire"])
    with tempfile.TemporaryDirectory() as d:
        cin, cout = os.path.join(d, "case.bin"), os.path.join(d, "out.jsonl")
        with open(cin, "wb") as f:
            f.write(b"FRG1" + struct.pack("<II", 0 if case["mode"] == "package" else 1, len(key)) + key + iv
                    + struct.pack("<iIQ", case["max_len"], piece, len(wire)) + wire)
        r = subprocess.run([exe, cin, cout], timeout=120, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                           env=dict(os.environ, LIBC_FATAL_STDERR_="1"))
        assert r.returncode == 0, f"{os.path.basename(exe)} exited {r.returncode}: {r.stderr[-2000:]}"
        with open(cout) as f:
            lines = [json.loads(x) for x in f]
    assert lines and "end" in lines[-1], lines
    return lines[:-1], lines[-1]
