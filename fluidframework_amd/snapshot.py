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

Bodies are in the engine's interned form: "client" / removed ids are short
client ids, property keys are key indices and values interned value ids (the
host's Interner maps both ways); text is UTF-16 code units (a list of ints).
removedClientIds lists the removers in ascending short id after the first
remover when the caller supplies it (seq -> client of the removing op); only
the set is observable in remote replay.
"""
import numpy as np

from .abi import DOC_INIT_DTYPE, NOT_REMOVED, PROP_DTYPE, PROPSET_DTYPE, SEG_DTYPE

TEXT_SEGMENT_GRANULARITY = 256  # textSegment.ts (TextSegmentGranularity)
NEWLINE = 0x0A


def _can_append(prev, seg):
    # TextSegment.canAppend (textSegment.ts:72-77); markers never append
    return (prev["kind"] == 0 and seg["kind"] == 0 and (not prev["text"] or prev["text"][-1] != NEWLINE)
            and (len(prev["text"]) <= TEXT_SEGMENT_GRANULARITY or len(seg["text"]) <= TEXT_SEGMENT_GRANULARITY))


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
            elif _can_append(prev, cur) and prev["props"] == cur["props"]:
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
