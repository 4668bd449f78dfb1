"""Generated streams (fluidframework_amd/gen.py) as the ISequencedDocumentMessages
the reference would receive: the input of the Node host bench
(fluidframework_amd/node/bench_e2e.js) and of the reference replay harness
(tests/ref_util.py, oracle/ref_replay.js).  Sender short id c becomes the
long id "c<c>"; the observer is "A"."""
import json

import numpy as np

from . import gen
from .abi import F_MARKER, NO_PROPS, OP_ANNOTATE, OP_INSERT, OP_NOOP, OP_REMOVE
from .packing import units_to_str


def _props_json(batch, psi):
    ps = batch["propsets"][psi]
    out = {}
    for k in range(int(ps["first"]), int(ps["first"]) + int(ps["count"])):
        key = int(batch["props"][k]["key"])
        vid = int(batch["props"][k]["value"])
        out[gen.KEY_NAMES[key]] = None if vid == 0 else json.loads(gen.value_json(vid))
    return out


def stream_doc_msgs(stream, d):
    """Doc d of a generated stream as the messages the reference would receive
    (sender short id c -> long id "c<c>"; the observer is "A")."""
    b = stream["batch"]
    o = b["op_offsets"].astype(np.int64)
    text = b["text"]
    msgs = []
    for op in b["ops"][o[d]:o[d + 1]]:
        t = int(op["type"])
        flags = int(op["flags"])
        if t == OP_INSERT:
            if flags & F_MARKER:
                seg = {"marker": {"refType": int(op["pos2"])}}
                if int(op["b"]) != NO_PROPS:
                    seg["props"] = _props_json(b, int(op["b"]))
            else:
                s = units_to_str(text[int(op["a"]):int(op["a"]) + int(op["pos2"])])
                seg = s if int(op["b"]) == NO_PROPS else {"text": s, "props": _props_json(b, int(op["b"]))}
            contents = {"type": 0, "pos1": int(op["pos1"]), "seg": seg}
        elif t == OP_REMOVE:
            contents = {"type": 1, "pos1": int(op["pos1"]), "pos2": int(op["pos2"])}
        elif t == OP_ANNOTATE:
            contents = {"type": 2, "pos1": int(op["pos1"]), "pos2": int(op["pos2"]),
                        "props": _props_json(b, int(op["a"]))}
            if flags & 4:
                contents["combiningOp"] = {"name": "rewrite"}
        else:
            assert t == OP_NOOP
            contents = None
        msgs.append([f"c{int(op['client'])}", int(op["seq"]), int(op["ref_seq"]), int(op["min_seq"]),
                     "op" if contents is not None else "noop", contents])
    return msgs


def stream_docs(stream, d0, d1, segs=True):
    """docs [d0, d1) as {initialText, newCalc, roundSync, props, segs, msgs}."""
    init = stream["init_text"]
    docs = []
    for d in range(d0, d1):
        it = stream["inits"][d]
        docs.append({"initialText": units_to_str(init[int(it["text_off"]):int(it["text_off"]) + int(it["text_len"])]),
                     "newCalc": bool(int(it["flags"]) & 1), "roundSync": bool(int(it["flags"]) & 2),
                     "props": False, "segs": segs,
                     "msgs": stream_doc_msgs(stream, d)})
    return docs
