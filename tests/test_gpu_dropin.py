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


def _multi():
    with open(os.path.join(ROOT, "tests", "golden", "multi_cases.json")) as f:
        return json.load(f)["cases"]


def _run_multi(exe, c, threads=None, timeout=600, env=None):
    out = subprocess.run([exe, "1" if c["mode"] == "stream" else "0", str(c["keylen"]), str(c["conns"]),
                          str(c["quests_per_conn"]), str(c["payload"]), str(c["window"]),
                          str(threads or c["threads"]), "1", "1" if c.get("first_clear") else "0"],
                         capture_output=True, text=True, timeout=timeout, env=env)
    assert out.returncode == 0, (out.returncode, out.stderr[-3000:])
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("case", _multi(), ids=lambda c: c["name"])
def test_collector_in_reference_io_plumbing(case):
    """SURVEY 8f row 1 inside FPNN's own IO plumbing: many connections
    through the reference's SendBuffer and EncryptedPackageReceiver with INTEGRATION.md 2a
    applied by oracle/collect_patch.py -- SendBuffer::encryptData and
    EncryptedPackageReceiver::fetch queue into the IO thread's fpnn::EncryptorBatch, one
    flush per loop cycle and direction (stream mode receives through StreamReceiverBatch).
    Each direction's wire bytes equal the unpatched reference build's, and every answer
    equals its quest.  The reference build is timed on the same box beside it."""
    exe = _exe("io_multi_batched")
    d = _run_multi(exe, case)
    ref = _run_multi(_exe("io_multi_ref"), case)
    print(json.dumps({"case": case["name"], "batched": d, "reference": ref}))
    assert d["build"] == "batched" and d["ok"] and d["answers_ok"] and d["flushes"] > 0, d
    for k in ("wire_c2s_bytes", "wire_c2s_fnv", "wire_s2c_bytes", "wire_s2c_fnv"):
        assert d[k] == case[k], (k, d[k], case[k])
        assert ref[k] == case[k], (k, ref[k], case[k])


@pytest.mark.parametrize("shape", ["M3", "M6", "M7"])
def test_percall_dropin_in_reference_io_plumbing(shape):
    """The same plumbing UNCHANGED on libfpnn_aes.so (one GPU call per frame, the drop-in
    of INTEGRATION.md section 1) on a small many-connection case: identical wire bytes.
    M6 / M7: the clients' first frame ("*key") in the clear, SendBuffer::encryptData's skip
    (core/IOBuffer.cpp:36-45) -- package and stream."""
    case = dict(next(c for c in _multi() if c["name"] == shape))  # fewer quests: per-call is slow by design
    d = _run_multi(_exe("io_multi_dropin"), dict(case, quests_per_conn=2, conns=64))
    ref = _run_multi(_exe("io_multi_ref"), dict(case, quests_per_conn=2, conns=64))
    print(json.dumps({"dropin": d, "reference": ref}))
    assert d["build"] == "dropin" and d["ok"] and d["answers_ok"], d
    for k in ("wire_c2s_bytes", "wire_c2s_fnv", "wire_s2c_bytes", "wire_s2c_fnv"):
        assert d[k] == ref[k], (k, d[k], ref[k])


@pytest.mark.parametrize("policy", ["abort", "throw"])
@pytest.mark.parametrize("build,fail_at", [("io_multi_dropin", 400), ("io_multi_batched", 20)])
def test_device_error_in_reference_io_plumbing(build, fail_at, policy):
    """a device error inside FPNN's own IO code.  The reference
    Encryptor cannot fail, so an exception escaping EncryptedPackageReceiver::fetch or
    SendBuffer::realSend would leave the connection with its receive / send token held and
    the IO pool would swallow it (core/ServerIOWorker.cpp:153-182,
    base/ParamTemplateThreadPool.h:372-375): a wedged connection, nothing logged.  The
    drop-in's contract (fpnn_amd/csrc/fail_policy.hpp): with the
    default FPNN_AES_ON_ERROR=abort the process prints the error and aborts; with =throw
    fpnn::EncryptorError propagates (here it leaves the IO thread: std::terminate).  Either
    way the run ends non-zero within its time limit and names the error -- it never hangs.
    The error is injected at the fail_at-th host data call (FPNN_AES_DEBUG_FAIL_CALL), on
    the per-call drop-in and on the batched collector, package and stream mode."""
    for mode in ("package", "stream"):
        case = dict(_multi()[2] if mode == "package" else _multi()[4], quests_per_conn=2, conns=64)
        exe = _exe(build)
        env = dict(os.environ, FPNN_AES_DEBUG_FAIL_CALL=str(fail_at), FPNN_AES_ON_ERROR=policy)
        try:
            out = subprocess.run([exe, "1" if mode == "stream" else "0", str(case["keylen"]), str(case["conns"]),
                                  str(case["quests_per_conn"]), str(case["payload"]), str(case["window"]), "2"],
                                 capture_output=True, text=True, timeout=120, env=env)
        except subprocess.TimeoutExpired:
            pytest.fail(f"{build} {mode}: hung after the injected device error ({policy})")
        print(build, mode, policy, out.returncode, out.stderr[-600:])
        assert out.returncode != 0, (build, mode, policy, out.stdout[-500:])
        assert "injected device error" in out.stderr, out.stderr[-2000:]
        if policy == "abort":
            assert out.returncode == -6 and "FPNN_AES_ON_ERROR=abort" in out.stderr, (out.returncode, out.stderr[-2000:])
        else:
            assert "EncryptorError" in out.stderr, out.stderr[-2000:]


def test_device_error_in_reference_echo_throw_policy():
    """C1's single-threaded echo through the reference SendBuffer / receivers on the drop-in
    (oracle/io_echo.cpp) with FPNN_AES_ON_ERROR=throw: the caller that catches
    fpnn::EncryptorError (io_echo's main, exit 9) gets it; with the default it aborts."""
    exe = _exe("io_echo_dropin")
    for policy, code in (("throw", 9), ("abort", -6)):
        env = dict(os.environ, FPNN_AES_DEBUG_FAIL_CALL="50", FPNN_AES_ON_ERROR=policy)
        out = subprocess.run([exe, "0", "32", "100", "1024", "1"], capture_output=True, text=True, timeout=120, env=env)
        assert out.returncode == code and "injected device error" in out.stderr, (policy, out.returncode,
                                                                                  out.stderr[-2000:])


def _udp():
    with open(os.path.join(ROOT, "tests", "golden", "udp_cases.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", _udp(), ids=lambda c: c["input"].split()[0])
def test_reference_udp_encryptor_on_dropin(case):
    """SURVEY 8f rows 2 + 4 with the reference's own UDP caller:
    core/UDP.v2/UDPCommon.v2.cpp compiled unchanged against include/Encryptor.h +
    include/KeyExchange.h (oracle/_ref/udp_v2_dropin).  The server's
    UDPEncryptor::createPair (both forms: package only, package + reinforced data) runs the
    ECDH on the GPU; clients configure theirs from ECCKeyExchange::calcKey; datagrams go
    both ways through packageEncrypt/packageDecrypt and data segments through
    dataEncrypt/dataDecrypt.  Every ciphertext digest equals the reference build's
    (tests/golden/udp_cases.json, oracle/_ref/udp_v2_ref), every decrypt returns its
    plaintext, and a malformed public key gets an empty pair on both."""
    out = subprocess.run([_exe("udp_v2_dropin")], input=case["input"] + "\n", capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, (out.returncode, out.stderr[-3000:])
    d = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    print(json.dumps(d))
    d.pop("seconds")
    assert d == case["expect"]


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
