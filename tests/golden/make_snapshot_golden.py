"""Digests of the reference's SharedString summary fixtures.

Reads packages/dds/sequence/src/test/snapshots/{legacy,legacyWithCatchUp,v1,
v1Intervals}/*.json (summary trees createSnapshotFiles.ts wrote from the strings
generateSharedStrings.ts:47-147 builds) and records, per merge-tree "content"
blob, the SHA-256 of its chunk as canonical JSON (sorted keys, compact) plus the
chunk's counters and metadata (no segment text).  The tests rebuild those
strings, emit them through the engine's summary writers and compare digests.
Interval blobs (outside "content") are out of scope.  Runs in the build
container only; tests read tests/golden/snapshot_digests.json."""
import glob
import hashlib
import json
import os
import sys

SRC = "/root/reference/packages/dds/sequence/src/test/snapshots"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "snapshot_digests.json")


def chunk_digest(chunk):
    return hashlib.sha256(json.dumps(chunk, sort_keys=True, separators=(",", ":"),
                                     ensure_ascii=False).encode("utf-8")).hexdigest()


def content_blobs(tree):
    for e in tree["entries"]:
        if e["type"] == "Tree" and e["path"] == "content":
            return {b["path"]: json.loads(b["value"]["contents"]) for b in e["value"]["entries"]
                    if b["type"] == "Blob"}
    raise ValueError("no content tree")


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else SRC
    out = {}
    for f in sorted(glob.glob(os.path.join(src, "*", "*.json"))):
        name = os.path.relpath(f, src)[:-len(".json")]
        with open(f, encoding="utf-8") as fh:
            blobs = content_blobs(json.load(fh))
        out[name] = {bid: {"sha256": chunk_digest(c),
                           "meta": {k: v for k, v in c.items() if k not in ("segments", "segmentTexts")}}
                     for bid, c in blobs.items()}
    with open(OUT, "w", encoding="utf-8") as fh:
        json.dump({"source": "packages/dds/sequence/src/test/snapshots", "fixtures": out}, fh, indent=1,
                  sort_keys=True)
    print(f"{len(out)} fixtures -> {OUT}")


if __name__ == "__main__":
    main()
