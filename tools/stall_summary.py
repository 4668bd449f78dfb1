#!/usr/bin/env python3
"""Pass-1 issue / stall summary from tools/gpu_r05_stall.sh's four --pmc runs
(OUT dir with d1250_a, d1250_c, d10k_a, d10k_c): the last pair_kernel dispatch
of each run (the timed launch of `bench.py --steps 1 --warmup 0`), its counters
summed over dimensions, per op and as fractions of the waves' cycles.
Usage: stall_summary.py OUT_DIR OUT_JSON"""
import csv
import glob
import json
import os
import sys


def last_pair(d):
    rows = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0])))
    rows = [r for r in rows if "pair_kernel" in r["Kernel_Name"]]
    last = max(int(r["Dispatch_Id"]) for r in rows)
    out = {}
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    res = {"what": "pass-1 (pair_kernel) issue / stall counters, last dispatch of `bench.py --steps 1 --warmup 0` "
                   "(tools/gpu_r05_stall.sh, two --pmc passes per size; tools/stall_summary.py); raw counter sums",
           "sizes": {}}
    for size, ops, tag in (("1250", 1250 * 10000, "d1250"), ("10000", 10000 * 10000, "d10k")):
        raw = last_pair(os.path.join(src, tag + "_a"))
        raw.update(last_pair(os.path.join(src, tag + "_c")))
        per_op = {k: round(raw[k] / ops, 2) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS",
                                                     "SQ_INSTS_SMEM", "SQ_INSTS_VMEM", "SQ_ACTIVE_INST_ANY",
                                                     "SQ_WAVE_CYCLES") if k in raw}
        wc = raw["SQ_WAVE_CYCLES"]
        issue, wait = raw["SQ_ACTIVE_INST_ANY"] / wc, raw["SQ_WAIT_ANY"] / wc
        res["sizes"][size] = {"ops": float(ops), "raw": raw, "per_op": per_op, "fraction_of_wave_cycles": {
            "issuing (SQ_ACTIVE_INST_ANY)": round(issue, 3),
            "waiting on s_waitcnt (SQ_WAIT_ANY)": round(wait, 3),
            "waiting for an issue slot with a ready instruction (SQ_WAIT_INST_ANY)": round(raw["SQ_WAIT_INST_ANY"] / wc, 3),
            "rest (dependency latency, hazards, branch resolution)": round(1 - issue - wait, 3)}}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps({s: v["fraction_of_wave_cycles"] for s, v in res["sizes"].items()}))


if __name__ == "__main__":
    main()
