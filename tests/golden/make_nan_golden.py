#!/usr/bin/env python3
"""NaN never append-merges (matchProperties compares with !==,
properties.ts:66-100): golden vectors from the REFERENCE merge-tree itself.

Generates seeded observer streams whose annotates mix plain sets with
combiningOp incr (an incr on a number or an absent value leaves NaN,
properties.ts:24-40), followed by no-op messages that advance minSeq so the
reference's lazy zamboni scours every block (mergeTree.ts:800-838, append-merge
at :712).  Each stream is replayed by oracle/ref_replay.js (the type-erased
reference, build container only) and the fixture keeps the messages and what
the reference holds after it: the visible segments in order with their
properties (the segmentation the append-merge leaves), the text and the
per-position properties.  Data only -- no reference source is written.

Output: tests/golden/nan_merge_vectors.json.gz
Usage:  python3 tests/golden/make_nan_golden.py   (needs oracle/_ref, made by oracle/ts_erase.py)
"""
import gzip
import json
import os
import random
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "nan_merge_vectors.json.gz")


def stream(seed, n_ops=160, lag=6, tail=64):
    """One observer stream: clients B..E, each with a refSeq that never
    decreases (inserts lag up to `lag` seqs behind, range ops come from a
    caught-up client), msn = the lowest refSeq; positions drawn from the
    observer's own length model."""
    rnd = random.Random(seed)
    names = ["B", "C", "D", "E"]
    cref = {c: 0 for c in names}  # each client's refSeq: the last seq it processed (never decreases)
    msgs, length, seq = [], 0, 0
    for _ in range(n_ops):
        seq += 1
        c = rnd.choice(names)
        want = rnd.randint(max(0, seq - 1 - lag), seq - 1) if rnd.random() < 0.3 else seq - 1
        cref[c] = max(cref[c], want)
        ref = cref[c]
        msn = min(cref.values())
        r = rnd.random()
        if length < 4 or r < 0.45:
            # only the sender's view matters for the position; keep it within the
            # length the observer saw before the lagging window (no "insert failed")
            pos = rnd.randint(0, max(0, length - lag * 3)) if ref < seq - 1 else rnd.randint(0, length)
            pos = min(pos, length)
            t = c.lower() * rnd.randint(1, 3)
            msgs.append([c, seq, ref, msn, "op", {"type": 0, "pos1": pos, "seg": t}])
            length += len(t)
        elif r < 0.55:
            a = rnd.randint(0, length - 2)
            b = min(length, a + rnd.randint(1, 2))
            cref[c] = seq - 1  # a range op from a caught-up client
            msgs.append([c, seq, seq - 1, min(cref.values()), "op", {"type": 1, "pos1": a, "pos2": b}])
            length -= b - a
        else:
            a = rnd.randint(0, length - 1)
            b = min(length, a + rnd.randint(1, 8))
            key = rnd.choice(["n", "m"])
            if rnd.random() < 0.5:
                op = {"type": 2, "pos1": a, "pos2": b, "props": {key: 1}, "combiningOp": {"name": "incr"}}
            else:
                op = {"type": 2, "pos1": a, "pos2": b, "props": {key: rnd.choice([1, 2, "x"])}}
            cref[c] = seq - 1
            msgs.append([c, seq, seq - 1, min(cref.values()), "op", op])
    # minSeq catches up: every block's scour runs (<= 2 per message, mergeTree.ts:800-838)
    for _ in range(tail):
        seq += 1
        msgs.append(["B", seq, seq - 1, seq - 1, "noop", None])
    return msgs


def main():
    ref = os.path.join(ROOT, "oracle", "_ref", "ts")
    if not os.path.isdir(ref):
        raise SystemExit("oracle/_ref/ts missing: run oracle/ts_erase.py first (build container only)")
    docs = [{"initialText": "", "newCalc": True, "msgs": stream(7000 + i), "segs": True} for i in range(24)]
    r = subprocess.run(["node", os.path.join(ROOT, "oracle", "ref_replay.js"), ref],
                       input=json.dumps({"docs": docs}), capture_output=True, text=True, check=True)
    out = json.loads(r.stdout)["docs"]
    kept = []
    for d, o in zip(docs, out):
        if o["error"]:
            continue  # the stream model drew a position the reference refused
        kept.append({"msgs": d["msgs"], "text": o["text"], "props": o["props"], "segs": o["segs"]})
    with gzip.open(OUT, "wt", encoding="utf-8") as fh:
        json.dump({"docs": kept, "note": "reference merge-tree (oracle/ref_replay.js), new length calc, "
                   "observer 'A'; segs = visible segments after the zamboni, props JSON (NaN as null)"}, fh)
    nan_segs = sum(1 for d in kept for s in d["segs"] if s[1] and None in s[1].values())
    print(f"{len(kept)} docs, {sum(len(d['segs']) for d in kept)} segments, {nan_segs} holding NaN -> {OUT}")


if __name__ == "__main__":
    main()
