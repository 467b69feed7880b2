"""The north-star drop-in, exercised with the reference's OWN callers (VERDICT r03 items
1 and 2; BASELINE.json configs[0] = C1).

oracle/Makefile `dropin` compiles the reference's EncryptedPackageReceiver /
EncryptedStreamReceiver (core/EncryptedPackageReceiver.cpp, core/EncryptedStreamReceiver.cpp),
SendBuffer (core/IOBuffer.cpp:36-45,257-278) and their dependency closure UNCHANGED,
against include/Encryptor.h + include/rijndael.h through a header overlay (the copy-over
recipe of INTEGRATION.md section 1), and links libfpnn_aes.so in place of
core/Encryptor.cpp + base/rijndael.c:
  oracle/_ref/framing_dropin   the receivers fed the framing fixtures over a socketpair
  oracle/_ref/io_echo_dropin   C1: an encrypted echo over loopback TCP, SendBuffer ->
                               receiver -> answer -> SendBuffer -> receiver
Their outputs must equal what the same sources produced on the reference's own Encryptor
(tests/golden/framing_cases.json, tests/golden/c1_cases.json, made by oracle/gen_golden.py).
C1's per-call shape: oracle/percall.cpp (10 000 x 1 KiB PackageEncryptor calls) compiled
against include/ must reproduce the reference build's checksum.
"""
import json
import os
import subprocess

import pytest

from framing_golden import load_cases, run_receiver

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")


def _exe(name):
    p = os.path.join(REF, name)
    if not os.access(p, os.X_OK):
        from conftest import missing_reference_build
        missing_reference_build(f"oracle/_ref/{name}")  # fails on a GPU machine, skips elsewhere
    return p


def _c1():
    with open(os.path.join(ROOT, "tests", "golden", "c1_cases.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", load_cases(), ids=lambda c: c["name"])
def test_reference_receivers_on_dropin_reproduce_framing_fixtures(case):
    """All 22 framing fixtures: the reference receivers running on libfpnn_aes.so report
    the same frames, decoded plaintexts and verdict as on the reference Encryptor, for
    1-, 7- and 65536-byte arrival pieces."""
    exe = _exe("framing_dropin")
    for piece in (1, 7, 65536):
        ev, end = run_receiver(exe, case, piece)
        assert (len(ev), end["end"]) == (len(case["frames"]), case["end"]["end"]), (case["name"], piece, end)
        assert ev == case["frames"], (case["name"], piece)


@pytest.mark.parametrize("idx", range(len(_c1()["echo"])))
def test_c1_echo_reference_io_plumbing_on_dropin(idx):
    """C1 through the reference's SendBuffer + encrypted receivers on the drop-in: every
    answer equals its quest, and each direction's wire bytes equal the reference build's."""
    exe = _exe("io_echo_dropin")
    g = _c1()["echo"][idx]
    out = subprocess.run([exe, "1" if g["mode"] == "stream" else "0", str(g["keylen"]), str(g["quests"]),
                          str(g["payload"]), str(g["window"])], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, (out.returncode, out.stderr[-2000:])
    d = json.loads(out.stdout.strip().splitlines()[-1])
    print(json.dumps(d))
    assert d["answers_ok"] and d["served"] == g["quests"]
    for k in ("wire_c2s_bytes", "wire_c2s_fnv", "wire_s2c_bytes", "wire_s2c_fnv"):
        assert d[k] == g[k], (k, d[k], g[k])


def test_c1_percall_unchanged_package_encryptor(tmp_path):
    """C1's per-call shape: 10 000 x 1 KiB AES-256 frames through the unchanged
    PackageEncryptor::encrypt / decrypt / encrypt(std::string*) one call at a time
    (core/Encryptor.cpp:22-51) -- the checksum of every output byte equals the reference
    build's (oracle/_ref/percall_ref)."""
    import fpnn_amd
    exe = os.path.join(str(tmp_path), "percall_gpu")
    libdir = os.path.dirname(fpnn_amd.LIB_PATH)
    subprocess.run(["g++", "-std=c++11", "-O2", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "oracle", "percall.cpp"), "-o", exe, "-L", libdir, "-lfpnn_aes",
                    f"-Wl,-rpath,{libdir}"], check=True)
    g = _c1()["percall"]
    out = subprocess.run([exe, str(g["frames"]), str(g["len"])], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    print(json.dumps(d))
    assert d["checksum"] == g["checksum"]
    assert d["batched_matches"] is True
