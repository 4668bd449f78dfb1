#!/usr/bin/env python3
"""Golden vectors from the REFERENCE merge-tree itself (tests/golden/ref_vectors.json.gz).

Runs the reference packages/dds/merge-tree Client — downlevelled by
oracle/ts_erase.py into the git- and gpurun-ignored oracle/_ref/ts and driven by
oracle/ref_replay.js under Node — over seeded generated streams, and records
per document the canonical digest of what it shows (text, markers, properties:
DESIGN.md "Digest") and the error it threw, if any.  The streams are
regenerated from their parameters (fluidframework_amd/gen.py is deterministic),
so the file holds only parameters and expected outputs: data, no reference
source.  Run in the build container (the reference does not exist on the GPU
box); the GPU tests read the committed file.

Usage: python3 tests/golden/make_ref_golden.py
"""
import gzip
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from fluidframework_amd import gen  # noqa: E402
import ref_util  # noqa: E402

OUT = os.path.join(HERE, "ref_vectors.json.gz")

# (name, config, n_docs, ops_per_doc, generator overrides)
SETS = [
    ("legacy_lag8", 3, 200, 2000, dict(length_mode=1, max_lag=8)),
    ("legacy_lag32", 3, 200, 2000, dict(length_mode=1, max_lag=32)),
    ("legacy_lag128", 3, 100, 2000, dict(length_mode=1, max_lag=128)),
    ("mixed_lag64_c2", 2, 300, 1000, dict(length_mode=0, max_lag=64)),
    ("legacy_lag16_c4", 4, 500, 500, dict(length_mode=1, max_lag=16)),
    ("mixed_rounds_c3", 3, 100, 3000, dict(length_mode=0)),
    ("newcalc_lag32", 3, 150, 2000, dict(length_mode=2, max_lag=32)),
    # texts holding '\n': the append-merge refuses a text that ends in one
    ("legacy_lag16_nl", 3, 200, 2000, dict(length_mode=1, max_lag=16, newline_every=3)),
    ("mixed_rounds_nl", 3, 100, 3000, dict(length_mode=0, newline_every=2)),
]


def main():
    """make_ref_golden.py [set names]: (re)generate those sets (default: all),
    keeping the others of the existing file."""
    if not ref_util.ref_available():
        sys.exit("the reference sources are not in this container")
    only = set(sys.argv[1:])
    out = {"generator": "fluidframework_amd/gen.py (mte_gen.cpp), seeded MT19937", "sets": []}
    old = {}
    if only and os.path.exists(OUT):
        with gzip.open(OUT, "rt", encoding="utf-8") as fh:
            old = {r["name"]: r for r in json.load(fh)["sets"]}
    for name, cfg, nd, nops, kw in SETS:
        if only and name not in only and name in old:
            out["sets"].append(old[name])
            continue
        t0 = time.time()
        st = gen.generate(cfg, n_docs=nd, ops_per_doc=nops, **kw)
        res = ref_util.ref_replay(ref_util.stream_docs(st, 0, nd))
        vids = ref_util.value_ids(st)
        docs = []
        for r in res:
            dg = ref_util.content_digest(r["segs"], vids)
            docs.append({"digest": [f"{int(x):016x}" for x in dg], "error": r["error"], "applied": r["applied"]})
        out["sets"].append({"name": name, "config": cfg, "n_docs": nd, "ops_per_doc": nops, "params": kw,
                            "docs": docs})
        print(f"{name}: {nd} docs in {time.time() - t0:.0f} s, errors {sum(d['error'] is not None for d in docs)}",
              flush=True)
    with gzip.open(OUT, "wt", encoding="utf-8") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
