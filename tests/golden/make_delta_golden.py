#!/usr/bin/env python3
"""Golden delta events from the REFERENCE merge-tree itself
(tests/golden/delta_vectors.json.gz).

oracle/ref_replay.js replays seeded generated streams (new length
calculation, lagging refSeqs, properties, markers) through the reference
Client with a mergeTreeDeltaCallback that records, for every insert / remove /
annotate, each delta segment's Client.getPosition and cachedLength — what
SharedString's sequenceDelta listener reads (sequence.ts:203-211, 688-725).
The streams are regenerated from their parameters (fluidframework_amd/gen.py
is deterministic), so the file holds only parameters and the expected events
(flattened [message index, kind, position, length, removed] per range): data, no
reference source.  Run in the build container.

Usage: python3 tests/golden/make_delta_golden.py [--maint]
"""
import gzip
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from fluidframework_amd import gen  # noqa: E402
import ref_util  # noqa: E402

OUT = os.path.join(HERE, "delta_vectors.json.gz")
SETS = [
    ("newcalc_lag16_c3", 3, 60, 800, dict(length_mode=2, max_lag=16)),
    ("newcalc_lag64_c2", 2, 60, 800, dict(length_mode=2, max_lag=64)),
    ("newcalc_rounds_c3", 3, 40, 1200, dict(length_mode=2)),
]


# --maint: the maintenance callbacks of remote-only documents (SPLIT / APPEND /
# UNLINK: an observer acks nothing), new and legacy length calculation ->
# tests/golden/maint_observer_vectors.json.gz
OUT_MAINT = os.path.join(HERE, "maint_observer_vectors.json.gz")
MAINT_SETS = SETS + [("legacy_lag16_c3", 3, 60, 800, dict(length_mode=1, max_lag=16)),
                     ("legacy_rounds_c2", 2, 40, 1200, dict(length_mode=1))]


def main_maint():
    if not ref_util.ref_available():
        sys.exit("the reference sources are not in this container")
    out = {"generator": "fluidframework_amd/gen.py (mte_gen.cpp), seeded MT19937; oracle/ref_replay.js maint",
           "sets": []}
    for name, cfg, nd, nops, kw in MAINT_SETS:
        st = gen.generate(cfg, n_docs=nd, ops_per_doc=nops, **kw)
        docs = ref_util.stream_docs(st, 0, nd)
        for d in docs:
            d["maint"] = True
            d["props"] = False
        res = ref_util.ref_replay(docs)
        out["sets"].append({"name": name, "config": cfg, "n_docs": nd, "ops_per_doc": nops, "params": kw,
                            "docs": [{"error": r["error"], "maint": r["maint"]} for r in res]})
        print(name, sum(len(r["maint"]) for r in res), "callbacks", flush=True)
    with gzip.open(OUT_MAINT, "wt", encoding="utf-8") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print("wrote", OUT_MAINT, os.path.getsize(OUT_MAINT))


def main():
    if not ref_util.ref_available():
        sys.exit("the reference sources are not in this container")
    out = {"generator": "fluidframework_amd/gen.py (mte_gen.cpp), seeded MT19937", "sets": []}
    for name, cfg, nd, nops, kw in SETS:
        st = gen.generate(cfg, n_docs=nd, ops_per_doc=nops, **kw)
        docs = ref_util.stream_docs(st, 0, nd)
        for d in docs:
            d["deltas"] = True
            d["props"] = False
        res = ref_util.ref_replay(docs)
        ev = []
        for r in res:
            flat = [[mi, kind, p, n, rm] for mi, kind, rng in r["deltas"] for p, n, rm in rng]
            ev.append({"error": r["error"], "events": flat})
        out["sets"].append({"name": name, "config": cfg, "n_docs": nd, "ops_per_doc": nops, "params": kw,
                            "docs": ev})
        print(name, sum(len(e["events"]) for e in ev), "events", flush=True)
    with gzip.open(OUT, "wt", encoding="utf-8") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print("wrote", OUT, os.path.getsize(OUT))


if __name__ == "__main__":
    if "--maint" in sys.argv[1:]:
        main_maint()
    else:
        main()
