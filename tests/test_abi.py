"""The C-ABI library: loads, exports every symbol include/*.h declares, host-side
logic matches the oracle (CPU only; no compute calls that need a GPU)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = ["fpnn_aes.h", "rijndael.h", "fpnn_ecdh.h"]


def declared_functions():
    names = set()
    for h in HEADERS:
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(", src, flags=re.M):
            name = m.group(1)
            if name not in ("if", "while", "for", "sizeof"):
                names.add(name)
    return names


def test_library_exports_every_declared_symbol():
    import fpnn_amd
    names = declared_functions()
    assert "fpnn_aes_package_encrypt" in names and "rijndael_cfb_encrypt" in names
    out = subprocess.run(["nm", "-D", "--defined-only", fpnn_amd.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = sorted(n for n in names if n not in exported)
    assert not missing, missing
    for n in names:  # and ctypes can bind each of them
        getattr(fpnn_amd.lib, n)


def test_signature_table_covers_header():
    from fpnn_amd._lib import SIGNATURES
    assert declared_functions() <= set(SIGNATURES)


def test_cpp_encryptor_symbols_exported():
    import fpnn_amd
    out = subprocess.run(["nm", "-DC", "--defined-only", fpnn_amd.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    for sym in ("fpnn::PackageEncryptor::encrypt(unsigned char*, unsigned char*, int)",
                "fpnn::PackageEncryptor::decrypt(unsigned char*, unsigned char*, int)",
                "fpnn::PackageEncryptor::encrypt(std::__cxx11::basic_string",
                "fpnn::StreamEncryptor::encrypt(unsigned char*, unsigned char*, int)",
                "fpnn::StreamEncryptor::decrypt(unsigned char*, unsigned char*, int)",
                "fpnn::EncryptorBatch::flush()",
                "fpnn::EncryptorBatch::encrypt(fpnn::Encryptor*, std::__cxx11::basic_string",
                "fpnn::EncryptorBatch::encrypt(fpnn::Encryptor*, unsigned char*, unsigned char*, int)",
                "fpnn::EncryptorBatch::decrypt(fpnn::Encryptor*, unsigned char*, unsigned char*, int)",
                "fpnn::encryptor_retire(unsigned long)",
                "fpnn::StreamReceiverBatch::open(fpnn::StreamEncryptor*)",
                "fpnn::StreamReceiverBatch::received(int, unsigned char const*, unsigned long)",
                "fpnn::StreamReceiverBatch::flush()",
                "fpnn::StreamReceiverBatch::messages[abi:cxx11](int) const",
                "fpnn::StreamReceiverBatch::status(int) const"):
        assert sym in out, sym


def test_kernels_built_for_gfx950():
    import fpnn_amd
    gpu = os.path.join(os.path.dirname(fpnn_amd.LIB_PATH), "libfpnn_aes_gpu.so")
    data = open(gpu, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # offload bundle id of the embedded code object


@pytest.mark.slow
def test_ragged_decrypt_kernels_do_not_spill_vgprs():
    """Every K1r instantiation keeps its registers out of scratch: a scratch reload inside
    the chunk loop waits on vmcnt(0), which drains the prefetch pipeline (a fused-map
    variant that spilled 3 VGPRs ran framed C3 at 407 instead of 955 GiB/s).
    The compiler's resource remarks for k_ragged.hip (tools/kres.sh), gfx950."""
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc in this environment")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run(["bash", os.path.join(root, "tools", "kres.sh"), "k_ragged.hip"], capture_output=True,
                         text=True, timeout=600)
    lines = [ln for ln in out.stdout.splitlines() if "k_cfb_decrypt_ragged<" in ln]
    assert len(lines) >= 12, out.stdout[-2000:] + out.stderr[-2000:]
    spills = [ln for ln in lines if not re.search(r"vgpr_spill=0\b", ln)]
    assert not spills, spills


def test_front_library_has_no_hip_dependency():
    """libfpnn_aes.so (what FPNN links) loads the HIP runtime only on first use, through
    libfpnn_aes_gpu.so: linked at start-up, the runtime's ~30 KiB of static TLS made
    pthread_create refuse FPNN's 16 KiB-stack clock thread (base/msec.c:72-74) and the
    reference's receivers aborted on their first message (tests/test_gpu_dropin.py).  So:
    no HIP library among its dependencies, and a thread with a 16 KiB stack starts in a
    process that has it loaded and initialised."""
    import fpnn_amd
    deps = subprocess.run(["readelf", "-d", fpnn_amd.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "NEEDED" in deps and not any(x in deps for x in ("amdhip", "hsa-runtime", "rocprof")), deps
    tls = subprocess.run(["readelf", "-lW", fpnn_amd.LIB_PATH], capture_output=True, text=True, check=True).stdout
    for line in tls.splitlines():
        if line.split()[:1] == ["TLS"]:
            assert int(line.split()[5], 16) <= 256, line


def test_small_stack_thread_after_first_call(tmp_path):
    """A C program linked with libfpnn_aes.so makes a library call (which loads the GPU
    library and the HIP runtime) and then starts a thread with a 16 KiB stack, as FPNN's
    base/msec.c does; pthread_create must succeed (no GPU needed: the call may fail).  The
    calls leave errno unchanged (FPNN's receivers test errno after a short read with a
    decrypt call in between, core/EncryptedStreamReceiver.cpp:31-55)."""
    import fpnn_amd
    src = tmp_path / "stack.c"
    src.write_text(r"""
#include <pthread.h>
#include <stdio.h>
#include "fpnn_aes.h"
static void *run(void *a) { return a; }
#include <errno.h>
int main(void) {
    int n = 0;
    errno = EAGAIN;  /* every call leaves errno as it found it (front.cpp) */
    fpnn_aes_device_count(&n);
    fpnn_aes_engine *e = 0;
    fpnn_aes_engine_create(0, FPNN_AES_OWN_STREAM, &e);
    if (errno != EAGAIN) { printf("errno %d\n", errno); return 7; }
    pthread_attr_t attr; pthread_t t;
    pthread_attr_init(&attr);
    pthread_attr_setstacksize(&attr, 16 * 1024);
    int rc = pthread_create(&t, &attr, run, 0);
    if (rc == 0) pthread_join(t, 0);
    printf("%d\n", rc);
    return rc;
}
""")
    exe = str(tmp_path / "stack")
    libdir = os.path.dirname(fpnn_amd.LIB_PATH)
    subprocess.run(["gcc", "-O2", "-I", os.path.join(ROOT, "include"), str(src), "-o", exe, "-L", libdir, "-lfpnn_aes",
                    f"-Wl,-rpath,{libdir}", "-pthread"], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "0", (out.stdout, out.stderr[-500:])


def test_version_string():
    import fpnn_amd
    assert "gfx950" in fpnn_amd.version()


@pytest.mark.parametrize("keylen", [16, 24, 32])
def test_setup_encrypt_matches_oracle(oracle, keylen):
    import fpnn_amd
    rng = np.random.default_rng(keylen)
    for _ in range(50):
        key = rng.bytes(keylen)
        ours = fpnn_amd.setup_encrypt(key)
        theirs = oracle.setup_encrypt(key)
        nw = 4 * (theirs.nrounds + 1)
        assert ours.nrounds == theirs.nrounds
        assert list(ours.rk[:nw]) == list(theirs.rk[:nw])


def test_setup_encrypt_matches_reference(ref_oracle):
    import fpnn_amd
    rng = np.random.default_rng(5)
    for kl in (16, 24, 32):
        key = rng.bytes(kl)
        a, b = fpnn_amd.setup_encrypt(key), ref_oracle.setup_encrypt(key)
        nw = 4 * (b.nrounds + 1)
        assert a.nrounds == b.nrounds and list(a.rk[:nw]) == list(b.rk[:nw])


def test_rijndael_setup_encrypt_mirror():
    import fpnn_amd
    from fpnn_amd._lib import Schedule
    ctx = Schedule()
    key = bytes(range(16))
    assert fpnn_amd.lib.rijndael_setup_encrypt(C.byref(ctx), C.cast(C.c_char_p(key), C.POINTER(C.c_uint8)), 16)
    # FIPS-197 C.1 round-10 key 13111d7f e3944a17 f307a78b 4d2b30c5
    assert ctx.nrounds == 10 and ctx.rk[40] == 0x13111d7f and ctx.rk[43] == 0x4d2b30c5
    bad = Schedule()
    assert not fpnn_amd.lib.rijndael_setup_encrypt(C.byref(bad), C.cast(C.c_char_p(key), C.POINTER(C.c_uint8)), 20)
    assert bad.nrounds == 0


def test_bad_key_length_reported():
    import fpnn_amd
    with pytest.raises(fpnn_amd.FpnnAesError) as ei:
        fpnn_amd.setup_encrypt(b"x" * 20)
    assert ei.value.status == fpnn_amd.ERR_KEYLEN


def test_no_device_fails_loudly():
    """Without a GPU the C-ABI reports NODEV (never a silent CPU path)."""
    import torch
    import fpnn_amd
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = C.c_void_p()
    rc = fpnn_amd.lib.fpnn_aes_engine_create(0, None, C.byref(h))
    assert rc == fpnn_amd.ERR_NODEV and not h.value
    n = C.c_int(-1)
    fpnn_amd.lib.fpnn_aes_device_count(C.byref(n))
    assert n.value == 0


def test_null_arguments_rejected():
    import fpnn_amd
    assert fpnn_amd.lib.fpnn_aes_package_encrypt(None, None) == fpnn_amd.ERR_ARG
    assert fpnn_amd.lib.fpnn_aes_package_decrypt(None, None) == fpnn_amd.ERR_ARG
    assert fpnn_amd.lib.fpnn_aes_stream_encrypt(None, None, None, None) == fpnn_amd.ERR_ARG
    assert fpnn_amd.lib.fpnn_aes_engine_create(0, None, None) == fpnn_amd.ERR_ARG
    assert fpnn_amd.lib.fpnn_aes_keyset_create(None, 1, 16, None, None, 1, None) == fpnn_amd.ERR_ARG
    assert fpnn_amd.lib.fpnn_aes_strerror(fpnn_amd.ERR_KEYLEN).startswith(b"key length")


def build_dropin(outdir) -> str:
    """Compile tests/cpp/dropin.cpp against include/Encryptor.h and link libfpnn_aes.so."""
    import fpnn_amd
    exe = os.path.join(str(outdir), "dropin")
    libdir = os.path.dirname(fpnn_amd.LIB_PATH)
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "dropin.cpp"), "-o", exe, "-L", libdir, "-lfpnn_aes",
                    f"-Wl,-rpath,{libdir}"], check=True, capture_output=True, text=True)
    return exe


def test_cpp_stream_receiver_compiles_against_headers(tmp_path):
    """tests/cpp/stream_recv.cpp, the EncryptedStreamReceiver-shaped loop over
    include/StreamReceiverBatch.h, builds with -std=c++11 -Wall -Werror and links."""
    import fpnn_amd
    exe = os.path.join(str(tmp_path), "stream_recv")
    libdir = os.path.dirname(fpnn_amd.LIB_PATH)
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "stream_recv.cpp"), "-o", exe, "-L", libdir, "-lfpnn_aes",
                    f"-Wl,-rpath,{libdir}"], check=True, capture_output=True, text=True)
    assert os.access(exe, os.X_OK)


def test_cpp_dropin_compiles_against_headers(tmp_path):
    """include/Encryptor.h is source-compatible with the way FPNN uses core/Encryptor.h
    (-std=c++11 -Wall -Werror, as the reference's def.mk builds it)."""
    assert os.access(build_dropin(tmp_path), os.X_OK)


def test_setup_decrypt_matches_reference(oracle, golden):
    """rijndael_setup_decrypt (host): the reversed, InvMixColumns'd rk[] of the reference
    (golden modes_cases.json, generated by oracle/_ref) and of the oracle restatement."""
    import fpnn_amd
    for c in golden("modes_cases.json")["setup_decrypt"]:
        key = bytes.fromhex(c["key"])
        ours = fpnn_amd.setup_decrypt(key)
        assert ours.nrounds == c["nrounds"] and list(ours.rk[:len(c["rk"])]) == c["rk"]
        mirror = fpnn_amd.Schedule()
        assert fpnn_amd.lib.rijndael_setup_decrypt(C.byref(mirror), C.cast(C.c_char_p(key), C.POINTER(C.c_uint8)),
                                                   len(key))
        assert list(mirror.rk[:len(c["rk"])]) == c["rk"]
        theirs = oracle.setup_decrypt(key)
        assert list(theirs.rk[:len(c["rk"])]) == c["rk"]


RIJNDAEL_API = ("rijndael_setup_encrypt", "rijndael_setup_decrypt", "rijndael_encrypt", "rijndael_decrypt",
                "rijndael_cbc_encrypt", "rijndael_cbc_decrypt", "rijndael_cfb_encrypt", "rijndael_ofb_encrypt")


def build_rijndael_link(outdir) -> str:
    import fpnn_amd
    exe = os.path.join(str(outdir), "rijndael_link")
    libdir = os.path.dirname(fpnn_amd.LIB_PATH)
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "rijndael_link.cpp"), "-o", exe, "-L", libdir, "-lfpnn_aes",
                    f"-Wl,-rpath,{libdir}"], check=True, capture_output=True, text=True)
    return exe


def test_rijndael_surface_links_without_reference_object(tmp_path):
    """Every function base/rijndael.h:22-60 declares is exported by libfpnn_aes.so, and a
    program calling all of them links with no rijndael.o: each rijndael_* symbol is left
    undefined in the executable and resolved from the shared library."""
    import fpnn_amd
    assert set(RIJNDAEL_API) <= declared_functions()
    exe = build_rijndael_link(tmp_path)
    undef = subprocess.run(["nm", "-u", exe], capture_output=True, text=True, check=True).stdout.split()
    defined_in_exe = subprocess.run(["nm", "--defined-only", exe], capture_output=True, text=True,
                                    check=True).stdout.split()
    lib_syms = subprocess.run(["nm", "-D", "--defined-only", fpnn_amd.LIB_PATH], capture_output=True, text=True,
                              check=True).stdout.split()
    for name in RIJNDAEL_API:
        assert name in undef, f"{name} not imported"
        assert name not in defined_in_exe, f"{name} defined in the program itself"
        assert name in lib_syms, f"{name} not exported by libfpnn_aes.so"


def _plan(env, k, ndev):
    """fpnn_aes_thread_engine_device / _max_thread_engines in a child process with `env`
    (the library reads the environment on each call; a child keeps this one clean)."""
    code = ("import sys; sys.path.insert(0, %r); import fpnn_amd; "
            "print([fpnn_amd.lib.fpnn_aes_thread_engine_device(i, %d) for i in range(%d)], "
            "fpnn_amd.lib.fpnn_aes_max_thread_engines(%d))" % (ROOT, ndev, k, ndev))
    e = {kk: v for kk, v in os.environ.items() if not kk.startswith("FPNN_AES_")}
    e.update(env)
    out = subprocess.run(["python", "-c", code], env=e, capture_output=True, text=True, check=True).stdout
    devs, cap = out.strip().rsplit(" ", 1)
    return eval(devs), int(cap)


def test_thread_engine_device_plan():
    """The C++ classes' engine pool (thread_engine.hpp): engine k on device k % ndev, or
    cyclically over FPNN_AES_DEVICES, or all on FPNN_AES_DEVICE; -1 without devices; at
    most 16 engines per device before threads share."""
    assert _plan({}, 10, 8) == ([0, 1, 2, 3, 4, 5, 6, 7, 0, 1], 128)
    assert _plan({}, 3, 1) == ([0, 0, 0], 16)
    assert _plan({}, 2, 0) == ([-1, -1], 1)
    assert _plan({"FPNN_AES_DEVICES": "3,5,9"}, 5, 8) == ([3, 5, 3, 5, 3], 32)  # 9 is not a device
    assert _plan({"FPNN_AES_DEVICE": "2"}, 3, 4) == ([2, 2, 2], 16)
    assert _plan({"FPNN_AES_DEVICE": "7"}, 2, 4) == ([-1, -1], 1)
    assert _plan({"FPNN_AES_MAX_ENGINES": "3"}, 4, 8)[1] == 3


def test_cpp_threads_program_compiles(tmp_path):
    """tests/cpp/threads.cpp (the engine-pool test of tests/test_gpu_threads.py) builds
    against the headers with -Wall -Werror."""
    import fpnn_amd
    exe = os.path.join(str(tmp_path), "threads")
    libdir = os.path.dirname(fpnn_amd.LIB_PATH)
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-pthread", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "threads.cpp"), "-o", exe, "-L", libdir, "-lfpnn_aes",
                    f"-Wl,-rpath,{libdir}"], check=True, capture_output=True, text=True)
    assert os.access(exe, os.X_OK)
