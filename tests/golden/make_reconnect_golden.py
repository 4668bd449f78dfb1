#!/usr/bin/env python3
"""Golden reconnect-farm vectors from the REFERENCE merge-tree itself
(tests/golden/reconnect_vectors.json.gz).

oracle/ref_farm.js with `reconnect` > 0: sending clients go offline now and
then, keep editing (their ops stay pending, unsent), and on reconnecting catch
up with the sequenced log and re-send every held op through the reference's
Client.regeneratePendingOp (client.ts:972-1002), as
test/client.reconnectFarm.spec.ts:25-59 does.  The file holds the sequenced
messages (the regenerated ops among them), each client's order of events and
every client's text and per-position properties at checkpoints — data only, no
reference source.  Run in the build container (the reference does not exist on
the GPU box).

Usage: python3 tests/golden/make_reconnect_golden.py
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

OUT = os.path.join(HERE, "reconnect_vectors.json.gz")
FARM_JS = os.path.join(ROOT, "oracle", "ref_farm.js")

# (seed, clients incl. the observer, steps, initial text, checkpoints, text bound, reconnect chance)
SETS = [(4000 + i, 2 + i % 7, 300 + 100 * (i % 8), ["", "hello world", "x" * 40, "abc\ndef"][i % 4], 5,
         [64, 200, 400][i % 3], [0.05, 0.1, 0.15][i % 3]) for i in range(40)]
# (offline stretches stay short enough for the 32 pending annotate groups a
# document tracks, MTE_ANNOTATE_SLOTS)


def main():
    if not ref_util.ref_available():
        sys.exit("the reference sources are not in this container")
    out = ref_util.build_ref()
    res = {"sets": [], "generator": "oracle/ref_farm.js reconnect mode (reference Client, mulberry32 seeds)"}
    failed = []
    for sd, c, n, t, k, m, rc in SETS:
        one = {"sets": [{"seed": sd, "clients": c, "steps": n, "initialText": t, "nCheckpoints": k, "maxText": m,
                         "reconnect": rc, "allowDiverge": True}]}
        q = subprocess.run(["node", FARM_JS, out], input=json.dumps(one), capture_output=True, text=True, timeout=600)
        if q.returncode == 0:
            res["sets"] += json.loads(q.stdout)["sets"]
        else:
            failed.append(sd)
    # seeds the reference could not run; on the ones marked "diverged" its own
    # clients end up with different documents (each client's states are kept:
    # the engine must reproduce every client, divergence included)
    res["seeds_the_reference_failed"] = failed
    res["seeds_the_reference_diverged"] = [s["seed"] for s in res["sets"] if s.get("diverged")]
    with gzip.open(OUT, "wt", encoding="utf-8") as fh:
        json.dump(res, fh, separators=(",", ":"))
    n_msgs = sum(len(s["log"]) for s in res["sets"])
    n_regen = sum(1 for s in res["sets"] for ev in s["events"] for e in ev if e[0] == "G")
    print(f"wrote {OUT}: {len(res['sets'])} farms, {n_msgs} sequenced messages, {n_regen} regenerated; "
          f"reference failed on {failed}, diverged on {res['seeds_the_reference_diverged']}")


if __name__ == "__main__":
    main()
