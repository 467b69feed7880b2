"""The engine pool behind the C++ classes (fpnn_amd/csrc/thread_engine.hpp; VERDICT r03
item 5): tests/cpp/threads.cpp runs Encryptors from several threads with fewer
pool engines than threads (FPNN_AES_MAX_ENGINES=2: threads share engines), and an
EncryptorBatch + StreamReceiverBatch first flushed on a thread that is then joined, flushed
again and destroyed on the main thread.  Every thread's ciphertext checksums equal the
oracle's (per call, batched and stream mode); the multi-GPU placement itself is covered on
CPU by tests/test_abi.py::test_thread_engine_device_plan (unmeasured on an 8-GPU node)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M64 = (1 << 64) - 1


def bytes_of(seed, n):
    x = (seed * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & M64
    out = bytearray(n)
    for i in range(n):
        x ^= (x << 13) & M64
        x ^= x >> 7
        x ^= (x << 17) & M64
        out[i] = x & 0xFF
    return bytes(out)


def fnv(h, data):
    for b in data:
        h = ((h ^ b) * 0x100000001B3) & M64
    return h


@pytest.mark.parametrize("max_engines", ["2", "16"])
def test_threads_share_pool_engines(tmp_path, oracle, max_engines):
    import fpnn_amd
    exe = str(tmp_path / "threads")
    libdir = os.path.dirname(fpnn_amd.LIB_PATH)
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-pthread", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "threads.cpp"), "-o", exe, "-L", libdir, "-lfpnn_aes",
                    f"-Wl,-rpath,{libdir}"], check=True, capture_output=True, text=True)
    nthreads, frames = 6, 40
    env = dict(os.environ, FPNN_AES_MAX_ENGINES=max_engines)
    out = subprocess.run([exe, str(nthreads), str(frames)], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = {}
    for line in out.stdout.split("\n"):
        f = line.split()
        if f:
            got[(f[0], f[1] if f[0] != "migrate" else "")] = f[2] if f[0] != "migrate" else (f[1], f[2])
    # migration case: 8 frames, AES-256, key bytes_of(77), iv bytes_of(78)
    key, iv = bytes_of(77, 32), bytes_of(78, 16)
    h = 0xCBF29CE484222325
    for i in range(8):
        h = fnv(h, oracle.package(key, iv, True, bytes_of(500 + i, 100 + 37 * i)))
    assert got[("migrate", "")] == (f"{h:016x}", "1")
    for t in range(nthreads):
        keylen = (16, 24, 32)[t % 3]
        key, iv = bytes_of(1000 + t, 32)[:keylen], bytes_of(2000 + t, 16)
        hp, hs = 0xCBF29CE484222325, 0xCBF29CE484222325
        siv, spos = iv, 0
        for i in range(frames):
            p = bytes_of((t << 32) | i, 1 + (t * 131 + i * 977) % 3000)
            hp = fnv(hp, oracle.package(key, iv, True, p))
            c, siv, spos = oracle.cfb(key, True, p, siv, spos)
            hs = fnv(hs, c)
        assert got[("percall", str(t))] == f"{hp:016x}", t
        assert got[("batch", str(t))] == f"{hp:016x}", t
        assert got[("stream", str(t))] == f"{hs:016x}", t
        assert got[("roundtrip", str(t))] == "1", t
