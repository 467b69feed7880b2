#!/usr/bin/env python3
"""Count s_waitcnt vmcnt(N) values and memory ops in one kernel of a source file's gfx950
assembly (a check that a software-pipelined kernel keeps its prefetches in flight).
Usage: tools/waitcnt_report.py k_ragged.hip <kernel-symbol-substring>"""
import re
import subprocess
import sys
from collections import Counter

src, sub = sys.argv[1], sys.argv[2]
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                f"fpnn_amd/csrc/{src}", "-o", "/tmp/wr.s"], check=True, capture_output=True)
s = open("/tmp/wr.s").read()
names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", s, re.M) if sub in m.group(1)]
for name in names:
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    lines = [l.strip() for l in s[i:j].split("\n")]
    w = Counter(re.search(r"vmcnt\((\d+)\)", l).group(1) for l in lines if l.startswith("s_waitcnt") and "vmcnt" in l)
    ops = Counter(l.split()[0] for l in lines if l.startswith(("global_load", "global_store", "s_load")))
    print(name[:90])
    print("  vmcnt waits:", dict(sorted(w.items(), key=lambda kv: int(kv[0]))))
    print("  mem ops:", dict(ops))
