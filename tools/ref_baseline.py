"""CPU baseline from the REFERENCE merge-tree itself (VERDICT row N1).

Runs in the build container only (the reference does not travel to the GPU
box): oracle/ts_erase.py downlevels packages/dds/merge-tree/src to Node-12
CommonJS in oracle/_ref/ts (git- and gpurun-ignored); oracle/ref_replay.js
replays documents through the reference Client.applyMsg exactly as the golden
tests do.  A bounded sample of a config's documents (all their ops) is split
over one Node process per core; the rate is the sample's ops over the slowest
process's replay time (Client construction + applyMsg; JSON parsing and the
read-out excluded).  The digests of the sample are checked against the flat
restatement.  Writes profiles/r02/ref_cpu_baseline.json (merged per config).

    python3 tools/ref_baseline.py --config 3 --docs 64 --workers 8
"""
import argparse
import json
import os
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import ref_util  # noqa: E402
from fluidframework_amd import gen  # noqa: E402
from oracle import OracleEngine  # noqa: E402

OUT = os.path.join(ROOT, "profiles", "r02", "ref_cpu_baseline.json")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--docs", type=int, default=64)
    ap.add_argument("--ops", type=int, default=None)
    ap.add_argument("--workers", type=int, default=os.cpu_count() or 1)
    args = ap.parse_args()
    if not ref_util.ref_available():
        sys.exit("the reference sources are not in this container")
    ref_util.build_ref()
    s = gen.generate(args.config, n_docs=args.docs, ops_per_doc=args.ops, round_sync=True)
    docs = ref_util.stream_docs(s, 0, args.docs)
    for d in docs:
        d["segs"] = True
    n_ops = int(s["batch"]["op_offsets"][-1])
    parts = [list(range(w, args.docs, args.workers)) for w in range(args.workers)]

    def run(idx):
        t0 = time.perf_counter()
        out = ref_util.ref_replay([docs[i] for i in idx])
        return idx, out, time.perf_counter() - t0

    t0 = time.perf_counter()
    with ThreadPoolExecutor(args.workers) as ex:
        results = list(ex.map(run, [p for p in parts if p]))
    wall = time.perf_counter() - t0
    per_worker_ms = [sum(r["ms"] for r in out) for _, out, _ in results]
    res = [None] * args.docs
    for idx, out, _ in results:
        for i, r in zip(idx, out):
            res[i] = r
    errors = sum(r["error"] is not None for r in res)
    # digests against the flat restatement on the same sample
    o = OracleEngine(s["n_keys"], threads=8)
    gen.load_stream(o, s)
    o.apply_batch(s["batch"])
    vids = ref_util.value_ids(s)
    equal = all(np.array_equal(np.array(ref_util.content_digest(r["segs"], vids), np.uint64), o.digest()[i])
                for i, r in enumerate(res) if r["error"] is None)
    slowest = max(per_worker_ms) / 1e3
    rec = {"value": n_ops / slowest, "unit": "ops/s", "cores": args.workers, "kind": "reference",
           "sample": f"first {args.docs} docs of config {args.config} (all their ops, {n_ops} ops), "
                     f"{args.workers} Node processes, slowest replay {slowest:.1f} s (wall {wall:.1f} s incl. "
                     "start-up and read-out)",
           "per_core_ops_s": n_ops / (sum(per_worker_ms) / 1e3),
           "errors": errors, "digest_equal_restatement": bool(equal),
           "where": "build container (8 vCPU), Node " + subprocess.run(["node", "--version"], capture_output=True,
                                                                      text=True).stdout.strip(),
           "how": "tools/ref_baseline.py: oracle/ts_erase.py + oracle/ref_replay.js (Client.applyMsg)"}
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    allrec = json.load(open(OUT)) if os.path.exists(OUT) else {}
    allrec[f"config{args.config}"] = rec
    with open(OUT, "w") as fh:
        json.dump(allrec, fh, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
