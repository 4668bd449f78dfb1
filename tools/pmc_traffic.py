#!/usr/bin/env python3
"""HBM traffic per replay launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON [--workload config3] [--sum-last-run]

Both passes run `bench.py --steps 1 --warmup 0 --no-cpu-baseline`, so the
replay kernels are dispatched twice (the accounting run with counters on, then
the timed run without): the LAST dispatch of each kernel is the timed one.
With --sum-last-run (a launch that dispatches kernels many times: the chunked
pass's round phases, config 5) every path kernel dispatched after the last
begin_batch_kernel (the timed launch's first kernel) is summed instead; run
bench.py without its side legs so the timed launch is the last one.
The counters are in KiB.  Corrections per MI355X_MICROARCH.md (HBM/rocprofv3):
FETCH_SIZE counts half the bytes of wide coalesced reads on gfx950, so it is
doubled; WRITE_SIZE is taken as is.  The op records are read by scalar loads
(32 B per op) and the segment planes by dword loads: access widths the guide
lists as uncalibrated, so the raw counter values are kept beside the corrected
sum.  The result is keyed by the sha256 of the libmte.so that was profiled;
bench.py reports it only while that library is the one it runs.
"""
import csv
import hashlib
import json
import os
import sys

PATH_KERNELS = ("begin_batch_kernel", "props_kernel", "round_sync_kernel", "pair_kernel", "big_kernel", "stream_kernel",
                "chunk_kernel", "tree_kernel", "rsmall_kernel", "rnd_plan_kernel", "rnd_count_kernel", "rnd_scan_kernel",
                "rnd_move_kernel", "rnd_cols_kernel", "rnd_resolve_kernel", "rnd_bucket_kernel", "rnd_apply_kernel",
                "rnd_gmove_kernel", "rnd_live_kernel", "rnd_gscan_kernel", "rnd_post_kernel", "rnd_room_kernel")


def last_run_sum(d, counter):
    """Every path kernel dispatched after the last begin_batch_kernel, summed per kernel."""
    rows = [r for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv")))
            if r["Counter_Name"] == counter]
    starts = [int(r["Dispatch_Id"]) for r in rows if "begin_batch_kernel" in r["Kernel_Name"]]
    first = max(starts) if starts else -1
    out = {}
    for r in rows:
        name = r["Kernel_Name"]
        short = next((k for k in PATH_KERNELS if k in name), None)
        if short is None or int(r["Dispatch_Id"]) < first:
            continue
        out[short] = out.get(short, 0.0) + float(r["Counter_Value"])
    return out


def last_dispatch(d, counter):
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    out = {}
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        short = next((k for k in PATH_KERNELS if k in name), None)
        if short is None:
            continue
        disp = int(r["Dispatch_Id"])
        if short not in out or disp > out[short][0]:
            out[short] = (disp, float(r["Counter_Value"]))
    return {k: v[1] for k, v in out.items()}


def main():
    fetch_dir, write_dir, out_json = sys.argv[1:4]
    workload = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else "config3"
    pick = last_run_sum if "--sum-last-run" in sys.argv else last_dispatch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "fluidframework_amd", "_lib", "libmte.so")
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    f = pick(fetch_dir, "FETCH_SIZE")
    w = pick(write_dir, "WRITE_SIZE")
    kern = {}
    for k in sorted(set(f) | set(w)):
        fb = f.get(k, 0.0) * 1024.0
        wb = w.get(k, 0.0) * 1024.0
        kern[k] = {"fetch_size_kib_raw": f.get(k), "write_size_kib_raw": w.get(k),
                   "read_bytes_corrected": 2.0 * fb, "write_bytes": wb, "hbm_bytes": 2.0 * fb + wb}
    total = sum(v["hbm_bytes"] for v in kern.values())
    res = {"workload": workload, "libmte_sha256": sha, "per_launch_kernels": kern,
           "traffic_bytes_per_launch": total,
           "correction": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), MI355X_MICROARCH.md HBM/rocprofv3",
           "passes": [fetch_dir, write_dir]}
    os.makedirs(os.path.dirname(os.path.abspath(out_json)), exist_ok=True)
    with open(out_json, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({"traffic_bytes_per_launch": total, "kernels": {k: v["hbm_bytes"] for k, v in kern.items()}}))


if __name__ == "__main__":
    main()
