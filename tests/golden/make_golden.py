#!/usr/bin/env python3
"""Derive compact golden fixtures from the reference's replay results.

Source: /root/reference/packages/dds/merge-tree/src/test/results/*.json
(30 files, each a ReplayGroup[] = 64 rounds of {msgs, initialText, resultText,
seq}; written by test/mergeTreeOperationRunner.ts:140-144 and replayed by
test/client.replay.spec.ts:16-60).

Only data is kept: per message (clientId, sequenceNumber,
referenceSequenceNumber, minimumSequenceNumber, type, contents), and per round
the expected initialText / resultText.  Per-message boilerplate (timestamp,
term, traces, origin, clientSequenceNumber) is dropped.  Output:
tests/golden/replay_fixtures.json.gz.  This script runs only where
/root/reference exists; the GPU box uses the committed output.
"""
import glob
import gzip
import json
import os
import sys

SRC = "/root/reference/packages/dds/merge-tree/src/test/results"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "replay_fixtures.json.gz")


def main() -> int:
    files = sorted(glob.glob(os.path.join(SRC, "*.json")))
    if not files:
        print("reference fixtures not found", file=sys.stderr)
        return 1
    out = []
    for f in files:
        groups = json.load(open(f))
        rounds = []
        for g in groups:
            msgs = [[m["clientId"], m["sequenceNumber"], m["referenceSequenceNumber"],
                     m["minimumSequenceNumber"], m["type"], m["contents"]] for m in g["msgs"]]
            rounds.append({"initialText": g["initialText"], "resultText": g["resultText"],
                           "seq": g["seq"], "msgs": msgs})
        out.append({"name": os.path.basename(f), "rounds": rounds})
    with gzip.open(OUT, "wt", encoding="utf-8") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print(f"wrote {OUT}: {len(out)} files, "
          f"{sum(len(r['msgs']) for d in out for r in d['rounds'])} msgs")
    return 0


if __name__ == "__main__":
    sys.exit(main())
