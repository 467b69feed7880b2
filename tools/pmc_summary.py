#!/usr/bin/env python3
"""Summarize rocprofv3 runs (kernel trace + separate PMC passes) into one JSON.

HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reads exactly half of the bytes of a wide coalesced streaming
read, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  The doubling is
calibrated on wide streaming reads only; when the fifth pass (TCC_EA0_RDREQ by request size:
32, 64 and 128 B, gfx950 events 43-45) is present its byte count is reported as
hbm_read_bytes_by_size and used for hbm_bytes_per_launch -- it needs no calibration.  Each pass was
its own rocprofv3 run, so counters are averaged per kernel over that pass's
dispatches.  Effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration.

Usage: python tools/pmc_summary.py gpurun_out/prof/<tag> [-o profiles/pmc_summary.json]
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"fpnn_aes::(?:\(anonymous namespace\)::)?(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")).replace(" ", "") if m else name


def base(name: str) -> str:
    return re.sub(r"^k_", "", short(name).split("<")[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("-o", "--out")
    args = ap.parse_args()

    durations = defaultdict(list)
    for f in glob.glob(os.path.join(args.prof_dir, "trace", "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            durations[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    counters = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in sorted(glob.glob(os.path.join(args.prof_dir, "pmc*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            counters[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = {kk: r[kk] for kk in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count", "SGPR_Count")}
    out = {"source": os.path.abspath(args.prof_dir), "kernels": {}}
    for k, cs in counters.items():
        avg = {c: statistics.mean(v) for c, v in cs.items()}
        d = {"counters_avg_per_dispatch": {c: round(v, 1) for c, v in sorted(avg.items())}, "resources": meta.get(k)}
        dur = durations.get(k)
        if dur:
            d["trace_avg_ns"] = round(statistics.mean(dur), 1)
            d["trace_dispatches"] = len(dur)
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            rd = 2.0 * avg["FETCH_SIZE"] * 1024
            wr = avg["WRITE_SIZE"] * 1024
            d["hbm_read_bytes_corrected"] = rd
            d["hbm_write_bytes"] = wr
            sized = ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")
            if all(c in avg for c in sized):
                n32, n64, n128 = (avg[c] for c in sized)
                rd = 32 * n32 + 64 * n64 + 128 * n128
                d["hbm_read_bytes_by_size"] = rd
                d["hbm_read_requests"] = {"32B": n32, "64B": n64, "128B": n128,
                                          "all": avg.get("TCC_EA0_RDREQ_sum")}
            d["hbm_bytes_per_launch"] = rd + wr
            if dur:
                d["hbm_GBs"] = round((rd + wr) / statistics.mean(dur), 1)
        if "GRBM_GUI_ACTIVE" in avg and dur:
            d["effective_clock_GHz"] = round(avg["GRBM_GUI_ACTIVE"] / 8 / statistics.mean(dur), 3)
        if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"]:
            d["lds_bank_conflict_frac"] = round(avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"], 5)
        if "SQ_LDS_IDX_ACTIVE" in avg and "GRBM_GUI_ACTIVE" in avg and avg["GRBM_GUI_ACTIVE"]:
            # LDS array busy: per-CU LDS-active cycles over the kernel's GPU-active cycles
            # (SQ_ counters sum over the 256 CUs, GRBM_GUI_ACTIVE over the 8 XCDs)
            d["lds_array_busy_frac"] = round((avg["SQ_LDS_IDX_ACTIVE"] / 256) / (avg["GRBM_GUI_ACTIVE"] / 8), 4)
        if "SQ_INSTS_VALU" in avg and avg.get("SQ_INSTS_LDS"):
            d["valu_per_lds_inst"] = round(avg["SQ_INSTS_VALU"] / avg["SQ_INSTS_LDS"], 3)
        if "SQ_WAVE_CYCLES" in avg:
            wc = avg["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if c in avg and wc:
                    d[c.lower() + "_frac_of_wave_cycles"] = round(avg[c] / wc, 4)
        out["kernels"][k] = d
        out.setdefault(base(k), {"hbm_bytes_per_launch": d.get("hbm_bytes_per_launch"), "variant": k})
    text = json.dumps(out, indent=1)
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
