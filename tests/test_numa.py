"""NUMA placement of an engine's host side (fpnn_amd/csrc/numa_place.cpp).

CPU: the placement logic against sysfs trees the test writes (FPNN_AES_SYSFS), through a
small driver compiled with the module (tests/cpp/numa_place_test.cpp).  GPU: the engine
reports its GPU's node, its pinned arenas' pages are on that node, and the host-frame copy
threads run on that node's CPUs.
"""
import ctypes
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BDF = "0000:c1:00.0"


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("numa") / "numa_place_test")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", os.path.join(ROOT, "tests/cpp/numa_place_test.cpp"),
                    os.path.join(ROOT, "fpnn_amd/csrc/numa_place.cpp"), "-o", exe, "-pthread"], check=True)
    return exe


def fake_sysfs(root, dev_node, cpulists):
    d = root / "bus/pci/devices" / BDF
    d.mkdir(parents=True)
    (d / "numa_node").write_text(f"{dev_node}\n")
    for n, cl in cpulists.items():
        nd = root / f"devices/system/node/node{n}"
        nd.mkdir(parents=True)
        (nd / "cpulist").write_text(cl + "\n")
    return str(root)


def run(driver, sysfs, *bdfs, numa=None):
    env = dict(os.environ, FPNN_AES_SYSFS=sysfs)
    env.pop("FPNN_AES_NUMA", None)
    if numa is not None:
        env["FPNN_AES_NUMA"] = numa
    out = subprocess.run([driver, *bdfs], env=env, check=True, capture_output=True, text=True).stdout
    return json.loads(out)


def cpus_of(cpulist):
    s = set()
    for part in cpulist.split(","):
        a, _, b = part.partition("-")
        s.update(range(int(a), int(b or a) + 1))
    return s


def test_device_node_and_cpus(driver, tmp_path):
    mine = os.sched_getaffinity(0)
    cl = "0-3,6"
    r = run(driver, fake_sysfs(tmp_path, 1, {0: "4-5,7", 1: cl}), BDF.upper(), "0000:00:01.0")
    assert r["nodes"] == {BDF.upper(): 1, "0000:00:01.0": -1}  # case-insensitive; unknown device: -1
    want = sorted(cpus_of(cl) & mine)
    p = r["placement"]
    assert (p["node"], p["device_node"], p["cpus"], p["ncpus"]) == (1, 1, want, len(want))
    assert r["pin_rc"] == 0 and r["affinity_after"] == want


def test_no_affinity_reported_as_none(driver, tmp_path):
    r = run(driver, fake_sysfs(tmp_path, -1, {0: "0-7"}), BDF)
    p = r["placement"]
    assert (p["node"], p["device_node"], p["ncpus"]) == (-1, -1, 0)
    assert "no placement" in p["why"]
    assert r["affinity_after"] == sorted(os.sched_getaffinity(0))  # nothing pinned


def test_node_outside_this_process_cpus(driver, tmp_path):
    # the node's CPUs are all outside our affinity (a container's CPU share on the other
    # socket): memory still goes to the GPU's node, threads stay unpinned
    r = run(driver, fake_sysfs(tmp_path, 1, {1: "4000-4003"}), BDF)
    p = r["placement"]
    assert (p["node"], p["ncpus"], p["cpus"]) == (1, 0, [])
    assert "unpinned" in p["why"]
    assert r["affinity_after"] == sorted(os.sched_getaffinity(0))


@pytest.mark.parametrize("numa,node", [("off", -1), ("0", 0), ("bogus", -1)])
def test_policy_switch(driver, tmp_path, numa, node):
    r = run(driver, fake_sysfs(tmp_path, 1, {0: "0-1", 1: "2-3"}), BDF, numa=numa)
    p = r["placement"]
    assert p["node"] == node and p["device_node"] == 1
    if numa == "0":
        assert p["cpus"] == sorted({0, 1} & os.sched_getaffinity(0))


def test_prefer_scope_places_and_restores(driver, tmp_path):
    r = run(driver, fake_sysfs(tmp_path, 0, {0: "0"}), BDF)
    pr = r["prefer"]
    assert pr["active"] and pr["mode_in"] == 1  # MPOL_PREFERRED inside the scope
    assert pr["mode_after"] == 0                # MPOL_DEFAULT restored
    assert pr["page_node"] == 0                 # (node 0 exists on every host)


# ---- on the GPU box ------------------------------------------------------------------------

SYS_move_pages = 279  # x86_64


def page_node(addr):
    libc = ctypes.CDLL(None, use_errno=True)
    pages = (ctypes.c_void_p * 1)(addr)
    status = (ctypes.c_int * 1)(-99)
    assert libc.syscall(SYS_move_pages, 0, ctypes.c_ulong(1), pages, None, status, 0) == 0
    return status[0]


@pytest.mark.gpu
def test_engine_places_arenas_and_threads():
    import numpy as np
    import torch
    import fpnn_amd
    from fpnn_amd._lib import lib
    eng = fpnn_amd.Engine(0)
    info = eng.numa()
    print(info)
    assert info["node"] == info["device_node"], info  # FPNN_AES_NUMA=auto
    if info["node"] < 0:
        pytest.skip(f"the GPU reports no NUMA node: {info['why']}")
    p = ctypes.c_void_p()
    assert lib.fpnn_aes_pinned_alloc(eng.handle, 1 << 22, ctypes.byref(p)) == 0
    try:
        ctypes.memset(p.value, 1, 1 << 22)
        n = page_node(p.value + (1 << 21))
        # (a runtime that maps pinned memory as device pages leaves them unqueryable: -errno)
        print(f"pinned arena page on node {n}")
        assert n == info["node"] or n < 0
    finally:
        lib.fpnn_aes_pinned_free(eng.handle, p)
    # a host-frame call starts the copy pool; its threads run on the node's CPUs we may use
    before = set(os.listdir("/proc/self/task"))
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 256, (4, 16), dtype=np.uint8)
    ivs = rng.integers(0, 256, (4, 16), dtype=np.uint8)
    ks = fpnn_amd.KeySet(eng, keys.tobytes(), 16, ivs.tobytes())
    srcs = [rng.integers(0, 256, 64 << 10, dtype=np.uint8) for _ in range(64)]  # 4 MiB: several copy parts
    eng.package_host(True, [(x, x, i % 4) for i, x in enumerate(srcs)], ks)
    if info["ncpus"] == 0:
        pytest.skip(f"none of the node's CPUs is ours: {info['why']}")
    node_cpus = cpus_of(open(f"/sys/devices/system/node/node{info['node']}/cpulist").read().strip())
    want = node_cpus & os.sched_getaffinity(0)
    assert len(want) == info["ncpus"]
    seen = []
    for t in set(os.listdir("/proc/self/task")) - before:
        try:
            seen.append(os.sched_getaffinity(int(t)))
        except OSError:
            continue
    pinned = [c for c in seen if c == want]
    print(f"{len(pinned)} of {len(seen)} new threads on node {info['node']}'s {len(want)} CPUs")
    assert pinned, seen
    torch.cuda.synchronize()
