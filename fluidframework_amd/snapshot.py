"""Summary bodies over the engine's segments.

write_body() is the summary writer: SnapshotV1.extractSegment
(packages/dds/merge-tree/src/snapshotV1.ts:189-265) over the segments a
document holds (mte_read_segments), for an observer (no unacked segments):
  - a segment removed at or below minSeq is elided;
  - a segment inserted at or below minSeq and not removed loses its merge info
    and is coalesced with the previous such segment when TextSegment.canAppend
    (textSegment.ts:72-77) and matchProperties (properties.ts:66) allow;
  - any other segment keeps seq / client (if seq > minSeq) and removedSeq /
    removedClientIds (IJSONSegmentWithMergeInfo, snapshotChunks.ts:48-78).
load_bodies() turns bodies back into mte_seg records for mte_load_segments
(SnapshotLoader.loadBody, snapshotLoader.ts:85-125).

Blob layouts over those bodies:
  - V1 (newMergeTreeSnapshotFormat: true): write_v1() is SnapshotV1.emit
    (snapshotV1.ts:76-165): MergeTreeChunkV1 "header" + "body_N" chunks of
    ~chunkSize units; summary_body() reads V1 and legacy chunks back
    (toLatestVersion, snapshotChunks.ts:142-186; loadHeader / loadBody with
    the 0x061-0x064 asserts, snapshotLoader.ts:126-220);
  - legacy (the default): write_legacy() / legacy_body(), below.
to_json() / from_json() convert between the interned form and the JSON the
reference writes (pinned against packages/dds/sequence/src/test/snapshots,
tests/test_snapshot_fixtures.py).

Bodies are in the engine's interned form: "client" / removed ids are short
client ids, property keys are key indices and values interned value ids (the
host's Interner maps both ways); text is UTF-16 code units (a list of ints).
removedClientIds lists the removers in ascending short id after the first
remover when the caller supplies it (seq -> client of the removing op); only
the set is observable in remote replay.
"""
import json

import numpy as np

from .abi import DOC_INIT_DTYPE, MTE_VALUE_UNEQUAL, NOT_REMOVED, PROP_DTYPE, PROPSET_DTYPE, SEG_DTYPE
from .packing import units_to_str, utf16_units

TEXT_SEGMENT_GRANULARITY = 256  # textSegment.ts (TextSegmentGranularity)
NEWLINE = 0x0A


def _can_append(prev, seg):
    # TextSegment.canAppend (textSegment.ts:72-77); markers never append
    return (prev["kind"] == 0 and seg["kind"] == 0 and (not prev["text"] or prev["text"][-1] != NEWLINE)
            and (len(prev["text"]) <= TEXT_SEGMENT_GRANULARITY or len(seg["text"]) <= TEXT_SEGMENT_GRANULARITY))


def _match(prev, cur):
    # matchProperties (properties.ts:66-100) on interned ids: NaN never matches
    return prev["props"] == cur["props"] and not any(v & MTE_VALUE_UNEQUAL for v in cur["props"])


def _json(seg):
    props = {k: v for k, v in enumerate(seg["props"]) if v}
    if seg["kind"] == 0:
        return {"text": list(seg["text"]), "props": props} if props else list(seg["text"])
    return {"marker": {"refType": seg["kind"] - 1}, "props": props} if props else \
        {"marker": {"refType": seg["kind"] - 1}}


def write_body(engine, doc, min_seq, first_remover=None):
    """-> list of IJSONSegmentWithMergeInfo-shaped dicts (interned form)."""
    segs, props, text = engine.read_segments(doc)
    out = []
    prev = None
    for i in range(len(segs)):
        s = segs[i]
        removed = int(s["removed_seq"]) != NOT_REMOVED
        if removed and int(s["removed_seq"]) <= min_seq:
            continue  # (b) removed at or below the MSN
        cur = {"kind": int(s["kind"]), "props": tuple(int(x) for x in props[i]),
               "text": text[int(s["text_off"]): int(s["text_off"]) + int(s["len"])].tolist()
               if int(s["kind"]) == 0 else None}
        if int(s["seq"]) <= min_seq and not removed:
            if prev is None:
                prev = cur
            elif _can_append(prev, cur) and _match(prev, cur):
                prev = {"kind": 0, "props": prev["props"], "text": prev["text"] + cur["text"]}
            else:
                out.append({"json": _json(prev)})
                prev = cur
            continue
        if prev is not None:
            out.append({"json": _json(prev)})
            prev = None
        raw = {"json": _json(cur)}
        if int(s["seq"]) > min_seq:
            raw["seq"] = int(s["seq"])
            raw["client"] = int(s["client"])
        if removed:
            raw["removedSeq"] = int(s["removed_seq"])
            ids = [c for c in range(32) if (int(s["removers"]) >> c) & 1]
            first = first_remover(raw["removedSeq"]) if first_remover else None
            if first in ids:
                ids.remove(first)
                ids.insert(0, first)
            raw["removedClient"] = ids[0]
            raw["removedClientIds"] = ids
        out.append(raw)
    if prev is not None:
        out.append({"json": _json(prev)})
    return out


def load_bodies(bodies, windows, flags, n_keys):
    """bodies[d] + windows[d] = (min_seq, cur_seq) + flags[d] -> the arguments
    of mte_load_docs + mte_load_segments: (inits, text, propsets, props,
    seg_offsets, segs)."""
    nd = len(bodies)
    inits = np.zeros(nd, DOC_INIT_DTYPE)
    inits["propset"] = 0xFFFFFFFF
    units, psets, pents, rows, offs = [], [], [], [], [0]
    for d, body in enumerate(bodies):
        inits[d]["flags"] = flags[d]
        inits[d]["min_seq"], inits[d]["cur_seq"] = windows[d]
        for sp in body:
            j = sp["json"]
            p = {}
            if isinstance(j, list):
                t, kind = j, 0
            elif "text" in j:
                t, kind, p = j["text"], 0, j.get("props", {})
            else:
                t, kind, p = None, 1 + j["marker"]["refType"], j.get("props", {})
            ps = 0xFFFFFFFF
            items = [(k, v) for k, v in p.items() if k < n_keys and v]
            if items:
                ps = len(psets)
                psets.append((len(pents), len(items)))
                pents.extend(items)
            off = len(units)
            if t is not None:
                units.extend(t)
            removed = "removedSeq" in sp
            mask = 0
            for c in sp.get("removedClientIds", [sp["removedClient"]] if "removedClient" in sp else []):
                mask |= 1 << c
            rows.append((off if t is not None else 0, len(t) if t is not None else 1, sp.get("seq", 0),
                         sp["removedSeq"] if removed else NOT_REMOVED, mask if removed else 0,
                         sp.get("client", -1), kind, ps))
        offs.append(len(rows))
    return (inits, np.array(units, np.uint16), np.array(psets, PROPSET_DTYPE), np.array(pents, PROP_DTYPE),
            np.array(offs, np.uint64), np.array(rows, SEG_DTYPE) if rows else np.zeros(0, SEG_DTYPE))


# --- V1 format (newMergeTreeSnapshotFormat: true) ----------------------------------------------

CHUNK_SIZE_V1 = 10000  # SnapshotV1.chunkSize, snapshotV1.ts:43


def _has_merge_info(spec):
    # hasMergeInfo, snapshotChunks.ts:80-82
    return isinstance(spec, dict) and "json" in spec


def _v1_chunk(specs, lengths, approx_length, start):
    # SnapshotV1.getSeqLengthSegs (snapshotV1.ts:76-110); no attribution
    n = length = 0
    while length < approx_length and start + n < len(specs):
        length += lengths[start + n]
        n += 1
    return {"version": "1", "segmentCount": n, "length": length, "segments": specs[start:start + n],
            "startIndex": start}


def write_v1(engine, doc, min_seq, cur_seq, chunk_size=CHUNK_SIZE_V1, first_remover=None):
    """SnapshotV1.extractSync + emit (snapshotV1.ts:117-165, 185-268) -> {blob name: chunk}:
    "header" carries headerMetadata {minSequenceNumber, sequenceNumber, orderedChunkMetadata,
    totalLength, totalSegmentCount}; "body_0", "body_1", ... the rest, ~chunk_size units each.
    Segments below the MSN are plain specs, the others IJSONSegmentWithMergeInfo."""
    body = write_body(engine, doc, min_seq, first_remover)
    specs = [sp if len(sp) > 1 else sp["json"] for sp in body]
    lengths = [_seg_length(sp["json"]) for sp in body]
    md = {"minSequenceNumber": min_seq, "sequenceNumber": cur_seq, "orderedChunkMetadata": [],
          "totalLength": 0, "totalSegmentCount": 0}
    chunks = []
    while True:  # do { ... } while (totalSegmentCount < segments.length)
        c = _v1_chunk(specs, lengths, chunk_size, md["totalSegmentCount"])
        chunks.append(c)
        md["totalSegmentCount"] += c["segmentCount"]
        md["totalLength"] += c["length"]
        if md["totalSegmentCount"] >= len(specs):
            break
    head = chunks.pop(0)
    md["orderedChunkMetadata"] = [{"id": "header"}] + [{"id": f"body_{i}"} for i in range(len(chunks))]
    head["headerMetadata"] = md
    blobs = {"header": head}
    blobs.update({f"body_{i}": c for i, c in enumerate(chunks)})
    return blobs


def to_latest(path, chunk):
    """toLatestVersion (snapshotChunks.ts:142-186): a legacy chunk read as MergeTreeChunkV1."""
    v = chunk.get("version")
    if v == "1":
        return chunk
    if v is not None:
        raise SnapshotLoadError(f"Unsupported chunk path: {path} version: {v}")
    md = None
    if path == "header":
        md = chunk.get("headerMetadata")
        if md is None:  # buildHeaderMetadataForLegacyChunk
            ids = [{"id": "header"}] + ([{"id": "body"}] if chunk["chunkLengthChars"] < chunk["totalLengthChars"]
                                        else [])
            md = {"orderedChunkMetadata": ids, "minSequenceNumber": chunk.get("chunkMinSequenceNumber"),
                  "sequenceNumber": chunk["chunkSequenceNumber"], "totalLength": chunk["totalLengthChars"],
                  "totalSegmentCount": chunk["totalSegmentCount"]}
    return {"version": "1", "length": chunk["chunkLengthChars"], "segmentCount": chunk["chunkSegmentCount"],
            "headerMetadata": md, "segments": chunk["segmentTexts"], "startIndex": chunk["chunkStartSegmentIndex"]}


def summary_window(blobs):
    """loadHeader (snapshotLoader.ts:126-166): (minSeq, currentSeq) of either format."""
    md = to_latest("header", blobs["header"])["headerMetadata"]
    if md is None:
        raise SnapshotLoadError("header metadata not available")
    ms = md.get("minSequenceNumber")
    return (md["sequenceNumber"] if ms is None else ms, md["sequenceNumber"])


def summary_body(blobs):
    """loadHeader + loadBody (snapshotLoader.ts:126-220) over either format -> (body,
    n_header): the segments in order as load_bodies takes them (plain specs become
    {"json": spec}: NonCollabClient at UniversalSequenceNumber) and how many came from
    the header chunk (the reference reloads those as a tree, reloadFromSegments, and
    appends the rest with insertSegments)."""
    h = to_latest("header", blobs["header"])
    md = h["headerMetadata"]
    if md is None:
        raise SnapshotLoadError("header metadata not available")
    wrap = lambda specs: [sp if _has_merge_info(sp) else {"json": sp} for sp in specs]  # noqa: E731
    body = wrap(h["segments"])
    if h["length"] > md["totalLength"]:
        raise SnapshotLoadError("0x061: Mismatch in totalLength")
    if h["segmentCount"] > md["totalSegmentCount"]:
        raise SnapshotLoadError("0x062: Mismatch in totalSegmentCount")
    n_header = len(body)
    if h["segmentCount"] == md["totalSegmentCount"]:
        return body, n_header
    length = h["length"]
    for meta in md["orderedChunkMetadata"][1:]:
        c = to_latest(meta["id"], blobs[meta["id"]])
        length += c["length"]
        body.extend(wrap(c["segments"]))
    if length != md["totalLength"]:
        raise SnapshotLoadError("0x063: Mismatch in totalLength")
    if len(body) != md["totalSegmentCount"]:
        raise SnapshotLoadError("0x064: Mismatch in totalSegmentCount")
    return body, n_header


def to_json(spec, interner, client_name=str):
    """Interned spec (plain or with merge info) -> the JSON the reference writes."""
    if _has_merge_info(spec):
        out = {"json": to_json(spec["json"], interner)}
        for k in ("client", "removedClient"):
            if k in spec:
                out[k] = client_name(spec[k])
        if "seq" in spec:
            out["seq"] = spec["seq"]
        if "removedSeq" in spec:
            out["removedSeq"] = spec["removedSeq"]
        if "removedClientIds" in spec:
            out["removedClientIds"] = [client_name(c) for c in spec["removedClientIds"]]
        return out
    if isinstance(spec, list):
        return units_to_str(spec)
    props = {interner.key_names[k]: json.loads(interner.json_of(v)) for k, v in spec.get("props", {}).items()}
    base = {"text": units_to_str(spec["text"])} if "text" in spec else {"marker": spec["marker"]}
    if props:
        base["props"] = props
    return base


def from_json(spec, interner, client_id=int):
    """Reference JSON spec -> interned form (text as UTF-16 units, props by key index)."""
    if _has_merge_info(spec):
        out = dict(spec)
        out["json"] = from_json(spec["json"], interner)
        for k in ("client", "removedClient"):
            if k in spec:
                out[k] = client_id(spec[k])
        if "removedClientIds" in spec:
            out["removedClientIds"] = [client_id(c) for c in spec["removedClientIds"]]
        return out
    if isinstance(spec, str):
        return utf16_units(spec).tolist()
    props = dict(interner.kv(k, v) for k, v in (spec.get("props") or {}).items() if v is not None)
    base = {"text": utf16_units(spec["text"]).tolist()} if "text" in spec else {"marker": dict(spec["marker"])}
    if props:
        base["props"] = props
    return base


# --- legacy format (the default when newMergeTreeSnapshotFormat !== true) ---------------------

SIZE_OF_FIRST_CHUNK = 10000  # SnapshotLegacy.sizeOfFirstChunk, snapshotlegacy.ts:52


class SnapshotLoadError(ValueError):
    """The loader's asserts (snapshotLoader.ts:170-211, 0x061-0x064) and the catch-up
    window check (sequence.ts:592-606)."""


def _seg_length(spec):
    return len(spec) if isinstance(spec, list) else len(spec["text"]) if "text" in spec else 1


def extract_legacy(engine, doc, min_seq):
    """SnapshotLegacy.extractSync (snapshotlegacy.ts:153-211): the document as it reads at
    minSeq for NonCollabClient — segments inserted at or below minSeq and not removed at or
    below it, coalesced by canAppend + matchProperties, with no merge info.  Properties are
    the segments' current ones (the reference keeps no per-seq property history either; the
    catch-up ops re-apply every later annotate in order, so the loaded replay converges)."""
    segs, props, text = engine.read_segments(doc)
    out = []
    prev = None
    for i in range(len(segs)):
        s = segs[i]
        if int(s["seq"]) > min_seq or int(s["removed_seq"]) <= min_seq:
            continue  # NOT_REMOVED is INT32_MAX, above every minSeq
        cur = {"kind": int(s["kind"]), "props": tuple(int(x) for x in props[i]),
               "text": text[int(s["text_off"]): int(s["text_off"]) + int(s["len"])].tolist()
               if int(s["kind"]) == 0 else None}
        if prev is not None and _can_append(prev, cur) and _match(prev, cur):
            prev = {"kind": 0, "props": prev["props"], "text": prev["text"] + cur["text"]}
        else:
            if prev is not None:
                out.append(_json(prev))
            prev = cur
    if prev is not None:
        out.append(_json(prev))
    return out


def _legacy_chunk(specs, approx_length, start, total_length, seq):
    # SnapshotLegacy.getSeqLengthSegs (snapshotlegacy.ts:66-99)
    n = 0
    length = 0
    while length < approx_length and start + n < len(specs):
        length += _seg_length(specs[start + n])
        n += 1
    return {"chunkStartSegmentIndex": start, "chunkSegmentCount": n,
            "chunkLengthChars": length, "totalLengthChars": total_length,
            "totalSegmentCount": len(specs), "chunkSequenceNumber": seq,
            "segmentTexts": specs[start:start + n]}


def write_legacy(engine, doc, min_seq, catchup=None, chunk_size=SIZE_OF_FIRST_CHUNK):
    """SnapshotLegacy.emit (snapshotlegacy.ts:105-151) -> {blob name: chunk}.  "header"
    holds the first ~chunk_size units with headerMetadata (buildHeaderMetadataForLegacyChunk,
    snapshotChunks.ts:168-186; minSequenceNumber is absent, so the loader takes
    sequenceNumber = minSeq for both ends of the window), "body" the rest when any, and
    "catchupOps" the caller's messages above minSeq when given."""
    specs = extract_legacy(engine, doc, min_seq)
    total = sum(_seg_length(s) for s in specs)
    c1 = _legacy_chunk(specs, chunk_size, 0, total, min_seq)
    ids = [{"id": "header"}] + ([{"id": "body"}] if c1["chunkLengthChars"] < total else [])
    c1["headerMetadata"] = {"orderedChunkMetadata": ids, "sequenceNumber": min_seq,
                            "totalLength": total, "totalSegmentCount": len(specs)}
    blobs = {"header": c1}
    if c1["chunkSegmentCount"] < len(specs):
        blobs["body"] = _legacy_chunk(specs, total, c1["chunkSegmentCount"], total, min_seq)
    assert sum(c["chunkLengthChars"] for c in blobs.values()) == total  # 0x05d
    assert sum(c["chunkSegmentCount"] for c in blobs.values()) == len(specs)  # 0x05e
    if catchup is not None and len(catchup) > 0:
        blobs["catchupOps"] = catchup
    return blobs


def legacy_window(blobs):
    """SnapshotLoader.loadHeader (snapshotLoader.ts:130-166): (minSeq, currentSeq)."""
    md = blobs["header"]["headerMetadata"]
    return (md.get("minSequenceNumber", md["sequenceNumber"]), md["sequenceNumber"])


def legacy_body(blobs):
    """Header + body chunks -> the body list load_bodies takes (plain specs: seq 0, no
    client), after the loader's consistency asserts (snapshotLoader.ts:168-211)."""
    h = blobs["header"]
    md = h["headerMetadata"]
    if h["chunkLengthChars"] > md["totalLength"]:
        raise SnapshotLoadError("0x061: Mismatch in totalLength")
    if h["chunkSegmentCount"] > md["totalSegmentCount"]:
        raise SnapshotLoadError("0x062: Mismatch in totalSegmentCount")
    specs = list(h["segmentTexts"])
    if h["chunkSegmentCount"] < md["totalSegmentCount"]:
        length = h["chunkLengthChars"]
        for meta in md["orderedChunkMetadata"][1:]:
            c = blobs[meta["id"]]
            length += c["chunkLengthChars"]
            specs.extend(c["segmentTexts"])
        if length != md["totalLength"]:
            raise SnapshotLoadError("0x063: Mismatch in totalLength")
        if len(specs) != md["totalSegmentCount"]:
            raise SnapshotLoadError("0x064: Mismatch in totalSegmentCount")
    return [{"json": s} for s in specs]


def check_catchup(ops, window):
    """SharedSegmentSequence.loadCore's catch-up check (sequence.ts:590-607) over op
    records: every catch-up message lies above the loaded window."""
    min_seq, cur_seq = window
    bad = (ops["min_seq"] < min_seq) | (ops["ref_seq"] < min_seq) | (ops["seq"] <= max(min_seq, cur_seq))
    if bad.any():
        o = ops[int(np.argmax(bad))]
        raise SnapshotLoadError("Invalid catchup operations in snapshot: seq %d minSeq %d refSeq %d, "
                                "window (%d, %d)" % (o["seq"], o["min_seq"], o["ref_seq"], min_seq, cur_seq))
