#!/usr/bin/env python3
"""Golden farm vectors from the REFERENCE merge-tree itself
(tests/golden/farm_vectors.json.gz).

oracle/ref_farm.js runs conflict farms of reference Clients (type-erased into
the git- and gpurun-ignored oracle/_ref/ts by oracle/ts_erase.py) with local
ops, acks and clients that catch up with the sequenced log at their own pace,
and records the sequenced messages, each client's order of events (its local
ops and the messages it applied) and every client's text and per-position
properties at checkpoints.  The file holds only that data — messages, event
orders and expected read-outs — no reference source.  Run in the build
container (the reference does not exist on the GPU box).

With --legacy it writes tests/golden/legacy_farm_vectors.json.gz: farms whose
clients keep the default (legacy) length calculation, with lagging clients,
rollbacks of removes, reconnects and local references among the sets.

With --refs it writes tests/golden/localref_vectors.json.gz instead: farms in
which every client (the observer included) also creates local references at
positions of its own view and removes some (Client.createLocalReferencePosition
/ removeLocalReferencePosition, SlideOnRemove or Simple), each checkpoint
holding every reference's localReferencePositionToPosition.

With --relpos it writes tests/golden/relpos_farm_vectors.json.gz: farms in
which local ops also address id'd markers through relative positions
(Client.annotateMarker, and removes / inserts whose relativePos1 / relativePos2
name a marker), in both length calculations, with lagging clients, rollbacks
and reconnects among the sets.

With --stay it writes tests/golden/localref_stay_vectors.json.gz: farms as
--refs in which a third to three fifths of the references made are
StayOnRemove -- they stay on their removed segment (localReference.ts:434,
469) until the lazy zamboni unlinks it, then read detached.

With --combine it writes tests/golden/combine_farm_vectors.json.gz: farms whose
annotates carry combiningOp incr (with and without defaultValue / minValue,
string values among the numbers) or consensus on id'd markers
(annotateMarkerNotifyConsensus), in both length calculations; the observer's
state is what a document of sequenced ops alone must equal.

With --maint it writes tests/golden/maint_farm_vectors.json.gz: farms that also
record every client's mergeTreeMaintenanceCallback (SPLIT / APPEND / UNLINK /
ACKNOWLEDGED): per event the callbacks it raised, each segment's position once
the event is applied and its length at the callback.

With --many it writes tests/golden/many_clients_vectors.json.gz: farms of 34
to 64 clients, so that more than 31 of them send inside one collab window
(short ids past the 32-bit removers mask of the flat passes), in both length
calculations, with rollbacks and references among them.

Usage: python3 tests/golden/make_farm_golden.py [--refs | --stay | --transient | --combine | --legacy | --relpos | --maint
                                                 | --many]
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

OUT = os.path.join(HERE, "farm_vectors.json.gz")
OUT_REFS = os.path.join(HERE, "localref_vectors.json.gz")
OUT_STAY = os.path.join(HERE, "localref_stay_vectors.json.gz")
OUT_COMBINE = os.path.join(HERE, "combine_farm_vectors.json.gz")
OUT_LEGACY = os.path.join(HERE, "legacy_farm_vectors.json.gz")
OUT_RELPOS = os.path.join(HERE, "relpos_farm_vectors.json.gz")
OUT_MAINT = os.path.join(HERE, "maint_farm_vectors.json.gz")
FARM_JS = os.path.join(ROOT, "oracle", "ref_farm.js")

# (seed, clients incl. the observer, steps, initial text, checkpoints, text bound)
SETS = [(1000 + i, 2 + i % 7, 300 + 150 * (i % 8), ["", "hello world", "x" * 40, "abc\ndef"][i % 4], 4,
         [64, 200, 400][i % 3], 0.0) for i in range(40)]
# with rollbacks: a local remove is rolled back instead of sent (Client.rollback)
SETS += [(2000 + i, 2 + i % 7, 400 + 100 * (i % 5), ["", "hello world"][i % 2], 4, [64, 200][i % 2], 0.15)
         for i in range(16)]
# removes and inserts rolled back: the reference's own farm stops on some seeds
# ("MergeTree insert failed" in another client after a rolled-back insert);
# those seeds are left out and counted in the file
ROLLBACK_INSERT_SETS = [(3000 + i, 2 + i % 5, 400, ["", "hello world"][i % 2], 4, 200, 0.15) for i in range(24)]
# annotates rolled back too (previousProps, mergeTree.ts:2036-2072), beside
# removes.  Inserts stay out of these sets: after a rolled-back insert the
# reference's block partial lengths can still count the segment (seed 4016 with
# inserts: a later remote insert lands one unit early in one client), which is
# the reference's own defect, not a rule to restate
ROLLBACK_ANNOTATE_SETS = [(4000 + i, 2 + i % 6, 400 + 100 * (i % 3), ["", "hello world", "abc\ndef"][i % 3], 4,
                           [64, 200][i % 2], 0.25, [1, 2]) for i in range(24)]


# local references: (seed, clients, steps, initial text, checkpoints, text bound,
# rollback chance, rollback types or None, reference-op chance)
REF_SETS = [(7000 + i, 2 + i % 6, 300 + 100 * (i % 5), ["", "hello world", "abc\ndef"][i % 3], 5, [64, 200, 400][i % 3],
             [0.0, 0.2][i % 2], [1, 2] if i % 4 == 3 else None, [0.1, 0.25][(i % 2) if i < 20 else 1 - i % 2])
            for i in range(40)]

# StayOnRemove references among them (--stay): (seed, clients, steps, initial
# text, checkpoints, text bound, rollback, rollback types, refs, stay)
STAY_SETS = [(7500 + i, 2 + i % 6, 400 + 100 * (i % 5), ["", "hello world", "abc\ndef"][i % 3], 6, [64, 200, 400][i % 3],
              [0.0, 0.2][i % 2], [1, 2] if i % 4 == 3 else None, [0.15, 0.3][i % 2], [0.35, 0.6][(i // 2) % 2])
             for i in range(32)]

# Transient references among them (--transient): as STAY_SETS, the last field
# the chance that a reference made is Transient
OUT_TRANSIENT = os.path.join(HERE, "localref_transient_vectors.json.gz")
TRANSIENT_SETS = [(7800 + i, 2 + i % 6, 400 + 100 * (i % 5), ["", "hello world", "abc\ndef"][i % 3], 6,
                   [64, 200, 400][i % 3], [0.0, 0.2][i % 2], [1, 2] if i % 4 == 3 else None, [0.15, 0.3][i % 2],
                   [0.35, 0.6][(i // 2) % 2]) for i in range(24)]

# combining ops (--combine): (seed, clients, steps, initial text, checkpoints,
# text bound, extra parameters)
COMBINE_SETS = ([(7700 + i, 3 + i % 5, 400 + 100 * (i % 4), ["", "hello world", "abc\ndef"][i % 3], 5,
                  [64, 200][i % 2], {"combine": [0.3, 0.6][i % 2], "allowDiverge": True}) for i in range(20)] +
                [(7750 + i, 3 + i % 4, 500, "hello world", 5, 200, {"combine": 0.4, "legacy": True, "allowDiverge": True})
                 for i in range(6)])


# legacy length calculation: (seed, clients, steps, initial text, checkpoints,
# text bound, extra parameters)
LEGACY_SETS = ([(8000 + i, 2 + i % 7, 300 + 150 * (i % 6), ["", "hello world", "abc\ndef"][i % 3], 4,
                 [64, 200, 400][i % 3], {}) for i in range(16)] +
               [(8100 + i, 3 + i % 4, 400, ["hello world", ""][i % 2], 4, 200, {"rollback": 0.15})
                for i in range(8)] +
               [(8200 + i, 3 + i % 4, 400, "hello world", 5, 200, {"reconnect": 0.1, "allowDiverge": True})
                for i in range(10)] +
               [(8300 + i, 2 + i % 5, 300 + 100 * (i % 3), ["", "hello world"][i % 2], 5, 200, {"refs": 0.2})
                for i in range(8)])


# relative positions: (seed, clients, steps, initial text, checkpoints, text
# bound, extra parameters); the legacy sets may diverge (as LEGACY_SETS)
RELPOS_SETS = ([(9000 + i, 2 + i % 6, 300 + 100 * (i % 4), ["", "hello world", "abc\ndef"][i % 3], 4,
                 [64, 200][i % 2], {"relpos": [0.2, 0.35][i % 2]}) for i in range(16)] +
               [(9100 + i, 3 + i % 4, 400, "hello world", 4, 200,
                 {"relpos": 0.3, "rollback": 0.15, "rollbackTypes": [1, 2]}) for i in range(8)] +
               [(9200 + i, 3 + i % 4, 400, "hello world", 5, 200, {"relpos": 0.3, "reconnect": 0.1, "allowDiverge": True})
                for i in range(8)] +
               [(9300 + i, 2 + i % 6, 300 + 100 * (i % 4), ["", "hello world"][i % 2], 4, 200,
                 {"relpos": 0.3, "legacy": True, "allowDiverge": True}) for i in range(12)])


# maintenance callbacks (--maint): (seed, clients, steps, initial text,
# checkpoints, text bound, extra parameters): plain farms (lagging clients:
# splits, acks, the lazy zamboni's appends and unlinks), rollbacks, references,
# the legacy length calculation, long farms (more zamboni work) and reconnects
MAINT_SETS = ([(10000 + i, 2 + i % 6, 300 + 150 * (i % 4), ["", "hello world", "abc\ndef"][i % 3], 4,
                [64, 200][i % 2], {}) for i in range(12)] +
              [(10100 + i, 3 + i % 4, 400, "hello world", 4, 200, {"rollback": 0.15, "rollbackTypes": [1, 2]})
               for i in range(6)] +
              [(10200 + i, 3 + i % 4, 400, ["hello world", ""][i % 2], 4, 200, {"refs": 0.2}) for i in range(4)] +
              [(10300 + i, 3 + i % 4, 400, "hello world", 4, 200, {"legacy": True, "allowDiverge": True})
               for i in range(6)] +
              [(10400 + i, 4, 1500, "the quick brown fox", 6, 120, {}) for i in range(4)] +
              [(10500 + i, 3 + i % 4, 400, "hello world", 4, 200, {"reconnect": 0.1, "allowDiverge": True})
               for i in range(6)])


# many clients (--many): (seed, clients, steps, initial text, checkpoints, text
# bound, extra parameters)
OUT_MANY = os.path.join(HERE, "many_clients_vectors.json.gz")
MANY_SETS = ([(11000 + i, [34, 40, 48, 56][i % 4], 700 + 100 * (i % 3), ["", "hello world", "abc\ndef"][i % 3], 4,
               [64, 200][i % 2], {}) for i in range(8)] +
             [(11100 + i, [40, 56][i % 2], 800, "hello world", 4, 200, {"rollback": 0.15, "rollbackTypes": [1, 2]})
              for i in range(4)] +
             [(11200 + i, [36, 50][i % 2], 700, "hello world", 4, 200, {"refs": 0.2}) for i in range(4)] +
             [(11300 + i, [34, 48][i % 2], 700, "hello world", 4, 200, {"legacy": True, "allowDiverge": True})
              for i in range(4)])


def window_senders(log):
    """The most short ids a document needs at once: the senders whose last op is
    past the collab window's minSeq, plus the document's own client (slot 0) --
    DocClients recycles a slot only once minSeq passed every seq its client used."""
    last, msn, most = {}, 0, 0
    for cid, seq, _ref, m, _t, _c in log:
        last[cid] = seq
        most = max(most, sum(1 for v in last.values() if v > msn) + 1)
        msn = max(msn, m)
    return most


def main_many(out):
    res = {"sets": [], "generator": "oracle/ref_farm.js, 34-64 clients (reference Client, mulberry32 seeds)"}
    failed = []
    for sd, c, n, t, k, m, extra in MANY_SETS:
        one = dict({"seed": sd, "clients": c, "steps": n, "initialText": t, "nCheckpoints": k, "maxText": m,
                    "rollback": 0.0}, **extra)
        q = subprocess.run(["node", "--max-old-space-size=8192", FARM_JS, out], input=json.dumps({"sets": [one]}),
                           capture_output=True, text=True, timeout=1200)
        if q.returncode == 0:
            res["sets"] += json.loads(q.stdout)["sets"]
        else:
            failed.append(sd)
    res["seeds_the_reference_failed"] = failed
    with gzip.open(OUT_MANY, "wt", encoding="utf-8") as fh:
        json.dump(res, fh, separators=(",", ":"))
    most = [window_senders(s["log"]) for s in res["sets"]]
    print(f"wrote {OUT_MANY}: {len(res['sets'])} farms, short ids needed at once {most}, reference failed on {failed}")


def main_maint(out):
    res = {"sets": [], "generator": "oracle/ref_farm.js with maint (reference Client, mulberry32 seeds)"}
    failed = []
    for sd, c, n, t, k, m, extra in MAINT_SETS:
        one = dict({"seed": sd, "clients": c, "steps": n, "initialText": t, "nCheckpoints": k, "maxText": m,
                    "rollback": 0.0, "maint": True}, **extra)
        q = subprocess.run(["node", FARM_JS, out], input=json.dumps({"sets": [one]}), capture_output=True, text=True,
                           timeout=600)
        if q.returncode == 0:
            res["sets"] += json.loads(q.stdout)["sets"]
        else:
            failed.append(sd)
    res["seeds_the_reference_failed"] = failed
    with gzip.open(OUT_MAINT, "wt", encoding="utf-8") as fh:
        json.dump(res, fh, separators=(",", ":"))
    kinds = {}
    for s in res["sets"]:
        for cl in s["maint"]:
            for e in cl:
                kinds[e[1]] = kinds.get(e[1], 0) + 1
    print(f"wrote {OUT_MAINT}: {len(res['sets'])} farms, callbacks by type {kinds}, reference failed on {failed}")


def main_relpos(out):
    res = {"sets": [], "generator": "oracle/ref_farm.js with relpos (reference Client, mulberry32 seeds)"}
    failed = []
    for sd, c, n, t, k, m, extra in RELPOS_SETS:
        one = dict({"seed": sd, "clients": c, "steps": n, "initialText": t, "nCheckpoints": k, "maxText": m},
                   **extra)
        q = subprocess.run(["node", FARM_JS, out], input=json.dumps({"sets": [one]}), capture_output=True, text=True,
                           timeout=600)
        if q.returncode == 0:
            res["sets"] += json.loads(q.stdout)["sets"]
        else:
            failed.append(sd)
    res["seeds_the_reference_failed"] = failed
    with gzip.open(OUT_RELPOS, "wt", encoding="utf-8") as fh:
        json.dump(res, fh, separators=(",", ":"))
    n_rel = sum(1 for s in res["sets"] for e in s["log"] if "relativePos1" in e[5])
    print(f"wrote {OUT_RELPOS}: {len(res['sets'])} farms, {n_rel} relative-position ops, reference failed on {failed}")


def main_legacy(out):
    res = {"sets": [], "generator": "oracle/ref_farm.js, legacy length calculation (reference Client, mulberry32 seeds)"}
    failed = []
    for sd, c, n, t, k, m, extra in LEGACY_SETS:
        # the reference's legacy-calc clients do not always converge (a reason the
        # new calculation exists): each client of ours must equal its reference
        # client, whatever the others hold
        one = dict({"seed": sd, "clients": c, "steps": n, "initialText": t, "nCheckpoints": k, "maxText": m,
                    "legacy": True, "allowDiverge": True}, **extra)
        q = subprocess.run(["node", FARM_JS, out], input=json.dumps({"sets": [one]}), capture_output=True, text=True,
                           timeout=600)
        if q.returncode == 0:
            res["sets"] += json.loads(q.stdout)["sets"]
        else:
            failed.append(sd)
    res["seeds_the_reference_failed"] = failed
    with gzip.open(OUT_LEGACY, "wt", encoding="utf-8") as fh:
        json.dump(res, fh, separators=(",", ":"))
    print(f"{len(res['sets'])} legacy sets, reference failed on {failed}")


def main_combine(out):
    res = {"sets": [], "generator": "oracle/ref_farm.js with combine (reference Client, mulberry32 seeds)"}
    failed = []
    for sd, c, n, t, k, m, extra in COMBINE_SETS:
        one = {"seed": sd, "clients": c, "steps": n, "initialText": t, "nCheckpoints": k, "maxText": m,
               "rollback": 0.0, **extra}
        q = subprocess.run(["node", FARM_JS, out], input=json.dumps({"sets": [one]}), capture_output=True, text=True,
                           timeout=600)
        if q.returncode == 0:
            res["sets"] += json.loads(q.stdout)["sets"]
        else:
            failed.append(sd)
    res["seeds_the_reference_failed"] = failed
    with gzip.open(OUT_COMBINE, "wt", encoding="utf-8") as fh:
        json.dump(res, fh, separators=(",", ":"))
    n_comb = sum(1 for s in res["sets"] for e in s["log"]
                 if e[4] == "op" and isinstance(e[5], dict) and e[5].get("combiningOp"))
    print(f"wrote {OUT_COMBINE}: {len(res['sets'])} farms, {n_comb} combining ops, reference failed on {failed}")


def main_refs(out, stay=False, transient=False):
    res = {"sets": [], "generator": "oracle/ref_farm.js with refs (reference Client, mulberry32 seeds)"}
    failed = []
    for row in (TRANSIENT_SETS if transient else STAY_SETS if stay else REF_SETS):
        sd, c, n, t, k, m, rb, types, refs = row[:9]
        one = {"seed": sd, "clients": c, "steps": n, "initialText": t, "nCheckpoints": k, "maxText": m,
               "rollback": rb, "refs": refs}
        if stay:
            one["stay"] = row[9]
        if transient:
            one["transient"] = row[9]
        if types:
            one["rollbackTypes"] = types
        q = subprocess.run(["node", FARM_JS, out], input=json.dumps({"sets": [one]}), capture_output=True, text=True,
                           timeout=600)
        if q.returncode == 0:
            res["sets"] += json.loads(q.stdout)["sets"]
        else:
            failed.append(sd)
    res["seeds_the_reference_failed"] = failed
    dst = OUT_TRANSIENT if transient else OUT_STAY if stay else OUT_REFS
    with gzip.open(dst, "wt", encoding="utf-8") as fh:
        json.dump(res, fh, separators=(",", ":"))
    n_refs = sum(1 for s in res["sets"] for ev in s["events"] for e in ev if e[0] == "F")
    print(f"wrote {dst}: {len(res['sets'])} farms, {n_refs} local references, reference failed on {failed}")


def main():
    if not ref_util.ref_available():
        sys.exit("the reference sources are not in this container")
    out = ref_util.build_ref()
    if "--refs" in sys.argv[1:]:
        return main_refs(out)
    if "--combine" in sys.argv[1:]:
        return main_combine(out)
    if "--stay" in sys.argv[1:]:
        return main_refs(out, stay=True)
    if "--transient" in sys.argv[1:]:
        return main_refs(out, transient=True)
    if "--legacy" in sys.argv[1:]:
        return main_legacy(out)
    if "--relpos" in sys.argv[1:]:
        return main_relpos(out)
    if "--maint" in sys.argv[1:]:
        return main_maint(out)
    if "--many" in sys.argv[1:]:
        return main_many(out)
    inp = {"sets": [{"seed": s, "clients": c, "steps": n, "initialText": t, "nCheckpoints": k, "maxText": m,
                     "rollback": rb} for s, c, n, t, k, m, rb in SETS]}
    p = subprocess.run(["node", "--max-old-space-size=8192", FARM_JS, out], input=json.dumps(inp),
                       capture_output=True, text=True, timeout=3600)
    if p.returncode != 0:
        sys.exit(p.stderr[-4000:])
    res = json.loads(p.stdout)
    res["generator"] = "oracle/ref_farm.js (reference Client, mulberry32 seeds)"
    failed = []
    for sd, c, n, t, k, m, rb in ROLLBACK_INSERT_SETS:
        one = {"sets": [{"seed": sd, "clients": c, "steps": n, "initialText": t, "nCheckpoints": k, "maxText": m,
                         "rollback": rb, "rollbackInserts": True}]}
        q = subprocess.run(["node", FARM_JS, out], input=json.dumps(one), capture_output=True, text=True, timeout=600)
        if q.returncode == 0:
            res["sets"] += json.loads(q.stdout)["sets"]
        else:
            failed.append(sd)
    res["rollback_insert_seeds_the_reference_failed"] = failed
    failed = []
    for sd, c, n, t, k, m, rb, types in ROLLBACK_ANNOTATE_SETS:
        one = {"sets": [{"seed": sd, "clients": c, "steps": n, "initialText": t, "nCheckpoints": k, "maxText": m,
                         "rollback": rb, "rollbackTypes": types}]}
        q = subprocess.run(["node", FARM_JS, out], input=json.dumps(one), capture_output=True, text=True, timeout=600)
        if q.returncode == 0:
            res["sets"] += json.loads(q.stdout)["sets"]
        else:
            failed.append(sd)
    res["rollback_annotate_seeds_the_reference_failed"] = failed
    with gzip.open(OUT, "wt", encoding="utf-8") as fh:
        json.dump(res, fh, separators=(",", ":"))
    n_msgs = sum(len(s["log"]) for s in res["sets"])
    print(f"wrote {OUT}: {len(res['sets'])} farms, {n_msgs} sequenced messages")


if __name__ == "__main__":
    main()
