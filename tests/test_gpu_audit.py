"""The address audit and the guard-page harness (the r05x illegal
memory access in test_wire_frames_every_offset[1-16-1-hybrid_lane_engine]).

* `libfpnn_aes_gpu_audit.so` (`make -C fpnn_amd/csrc audit`, -DFPNN_AES_BOUNDS, audit.hpp)
  checks every global access of K2h, K2's ragged path and the length-order kernels against
  its buffer's extent and the current segment's own bytes; the first violation comes back
  as FPNN_AES_ERR_DEVICE naming the kernel, source line, buffer, workgroup and address.
* `tests/cpp/guard_pages.cpp` runs the wire-frame / ragged / stream / short-quest encrypt
  shapes over arrays that each end (or start) at an unmapped page, so one byte past any
  array faults deterministically.

The parity reference is the oracle (oracle/aes_oracle.c, the restatement of
base/rijndael.c:1171-1201 and core/Encryptor.cpp:22-51 pinned by tests/test_oracle.py).
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AUDIT_LIB = os.path.join(ROOT, "fpnn_amd", "libfpnn_aes_gpu_audit.so")


def test_audit_library_is_built():
    """build() builds the audit variant of the GPU library beside the product one (it
    travels to the GPU box like the product library); its kernels carry the checks."""
    assert os.path.exists(AUDIT_LIB), "make -C fpnn_amd/csrc audit"
    blob = open(AUDIT_LIB, "rb").read()
    assert b"address audit" in blob
    assert b"address audit" not in open(os.path.join(ROOT, "fpnn_amd", "libfpnn_aes_gpu.so"), "rb").read()


def build_guard_pages(outdir) -> str:
    """tests/cpp/guard_pages.cpp + the oracle's C restatement, against the C-ABI front and
    the HIP runtime (for the virtual-memory calls)."""
    import fpnn_amd
    exe = os.path.join(str(outdir), "guard_pages")
    libdir = os.path.dirname(fpnn_amd.LIB_PATH)
    obj = os.path.join(str(outdir), "aes_oracle.o")
    subprocess.run(["gcc", "-O2", "-fPIC", "-c", os.path.join(ROOT, "oracle", "aes_oracle.c"), "-o", obj],
                   check=True, capture_output=True, text=True)
    subprocess.run(["g++", "-std=c++14", "-O2", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    os.path.join(ROOT, "tests", "cpp", "guard_pages.cpp"), obj, "-o", exe, "-L", libdir, "-lfpnn_aes",
                    f"-Wl,-rpath,{libdir}", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-pthread"],
                   check=True, capture_output=True, text=True)
    return exe


def test_guard_pages_harness_compiles(tmp_path):
    assert os.access(build_guard_pages(tmp_path), os.X_OK)


def _run(exe, lib=None, args=(), extra_env=None, timeout=240):
    env = dict(os.environ)
    env.pop("FPNN_AES_GPU_LIB", None)
    if lib:
        env["FPNN_AES_GPU_LIB"] = lib
    env.update(extra_env or {})
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.gpu
def test_guard_pages_product_library(tmp_path):
    """Every shape on every engine setting, each array abutting an unmapped page at its end
    and then at its start: no fault, and outputs equal to the oracle's."""
    res = _run(build_guard_pages(tmp_path))
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-2000:]
    assert "0 of" in res.stdout


@pytest.mark.gpu
def test_guard_pages_audit_library(tmp_path):
    """The same runs through the audit build: no access outside its extent or its segment."""
    res = _run(build_guard_pages(tmp_path), AUDIT_LIB)
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-2000:]
    assert "0 of" in res.stdout and "address audit" not in res.stderr


@pytest.mark.gpu
def test_audit_reports_a_short_extent(tmp_path):
    """The audit's own check: with the registered `out` extent made 3 bytes short, the last
    frame's final bytes fall outside it, and the call must come back as FPNN_AES_ERR_DEVICE
    naming the output buffer (and the bytes must not be written)."""
    res = _run(build_guard_pages(tmp_path), AUDIT_LIB, args=("wire_g1_aes128",),
               extra_env={"FPNN_AES_AUDIT_SHRINK_OUT": "3"})
    assert res.returncode == 1, res.stdout[-2000:] + res.stderr[-2000:]
    fails = [ln for ln in res.stdout.splitlines() if " FAIL " in ln]
    assert fails and all("address audit" in ln and "(out" in ln for ln in fails), res.stdout[-3000:]
