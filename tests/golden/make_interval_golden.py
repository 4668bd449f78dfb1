#!/usr/bin/env python3
"""Golden interval-collection farm vectors from the REFERENCE itself
(tests/golden/interval_vectors.json.gz).

oracle/ref_interval_farm.js runs conflict farms of reference merge-tree Clients
that also edit a SharedString interval collection -- the reference's own
IntervalCollection (packages/dds/sequence/src/intervalCollection.ts, erased by
oracle/ts_erase.py into the git- and gpurun-ignored oracle/_ref/ts/sequence)
-- with local and remote interval adds, changes of one or both ends, property
changes and deletes among merge-tree inserts, removes and annotates, every
client catching up with the sequenced log at its own pace.  The file holds the
messages, each client's event order and, at checkpoints, each client's text
and intervals (id, start and end positions, properties).  Build container only.

With --ext it writes tests/golden/interval_ext_vectors.json.gz: farms that also
record, per client and checkpoint, the collection's events, its iteration
order, serializeInternal() and seeded queries (findOverlappingIntervals,
previousInterval / nextInterval, the start / end position iterators).

With --reconnect it writes tests/golden/interval_reconnect_vectors.json.gz: ext
farms whose sending clients go offline and reconnect, re-sending their pending
merge-tree ops (regeneratePendingOp) and interval ops (rebaseLocalInterval) in
order.

Usage: python3 tests/golden/make_interval_golden.py [--ext | --reconnect]
"""
import gzip
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import ref_util  # noqa: E402

OUT = os.path.join(HERE, "interval_vectors.json.gz")
OUT_EXT = os.path.join(HERE, "interval_ext_vectors.json.gz")
OUT_REC = os.path.join(HERE, "interval_reconnect_vectors.json.gz")
FARM_JS = os.path.join(ROOT, "oracle", "ref_interval_farm.js")
# (seed, clients incl. the observer, steps, initial text, checkpoints, text bound, interval-op chance)
SETS = [(9000 + i, 2 + i % 5, 300 + 100 * (i % 4), ["", "hello world", "abc\ndef"][i % 3], 5, [64, 200][i % 2],
         [0.2, 0.35, 0.5][i % 3]) for i in range(30)]


# ext: (seed, clients, steps, initial text, checkpoints, text bound, interval-op chance)
EXT_SETS = [(9500 + i, 2 + i % 4, 200 + 100 * (i % 3), ["hello world", "", "abc\ndef"][i % 3], 4, [64, 200][i % 2],
             [0.3, 0.45][i % 2]) for i in range(12)]


# reconnect: (seed, clients, steps, initial text, checkpoints, text bound, interval-op chance, reconnect chance)
RECONNECT_SETS = [(9700 + i, 3 + i % 3, 300 + 100 * (i % 3), ["hello world", "abc\ndef", ""][i % 3], 4, [64, 200][i % 2],
                   [0.3, 0.45][i % 2], [0.04, 0.1][(i // 2) % 2]) for i in range(64)]


def main():
    if not ref_util.ref_available():
        sys.exit("the reference sources are not in this container")
    out = ref_util.build_ref()
    ext = "--ext" in sys.argv[1:]
    rec = "--reconnect" in sys.argv[1:]
    res = {"sets": [], "generator": "oracle/ref_interval_farm.js (reference Client + IntervalCollection)"}
    failed = []
    sets = RECONNECT_SETS if rec else [x + (0,) for x in (EXT_SETS if ext else SETS)]
    for sd, c, n, t, k, m, iv, rc in sets:
        one = {"seed": sd, "clients": c, "steps": n, "initialText": t, "nCheckpoints": k, "maxText": m,
               "intervals": iv}
        if ext or rec:
            one["ext"] = True
        if rec:
            one["reconnect"] = rc
            one["allowDiverge"] = True
        q = subprocess.run(["node", FARM_JS, out], input=json.dumps({"sets": [one]}), capture_output=True,
                           text=True, timeout=600)
        if q.returncode == 0:
            res["sets"] += json.loads(q.stdout)["sets"]
        else:
            failed.append((sd, q.stderr.strip().splitlines()[-1:]))
    res["seeds_the_reference_failed"] = failed
    path = OUT_REC if rec else (OUT_EXT if ext else OUT)
    with gzip.open(path, "wt", encoding="utf-8") as fh:
        json.dump(res, fh, separators=(",", ":"))
    n_iv = sum(1 for s in res["sets"] for e in s["log"] if e[4] == "iv")
    n_k = sum(1 for s in res["sets"] for ev in s["events"] for e in ev if e[0] == "K")
    div = [s["seed"] for s in res["sets"] if s.get("diverged")]
    if rec:
        lv = [(s["seed"], s["leafViews"]["differ"], s["leafViews"]["calls"]) for s in res["sets"]]
        print("leaf-rule views (seed, differ, calls):", lv)
    print(f"wrote {path}: {len(res['sets'])} farms, {n_iv} interval ops ({n_k} rebased), diverged {div}, "
          f"failed {failed}")


if __name__ == "__main__":
    main()
