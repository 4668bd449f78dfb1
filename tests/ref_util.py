"""Bridges between generated streams, the reference merge-tree run under Node
(oracle/ref_replay.js over oracle/_ref/ts, built by oracle/ts_erase.py) and the
canonical digest (DESIGN.md "Digest").  TEST INFRASTRUCTURE.

The reference sources exist only in the build container: ref_available() is
False on the GPU box, where the committed golden vectors (tests/golden/) stand
in for the reference."""
import json
import os
import shutil
import subprocess

import numpy as np

from fluidframework_amd import gen
from fluidframework_amd.abi import F_MARKER, NO_PROPS, OP_ANNOTATE, OP_INSERT, OP_NOOP, OP_REMOVE
from fluidframework_amd.packing import units_to_str

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SRC = "/root/reference/packages/dds/merge-tree/src"
REF_OUT = os.path.join(ROOT, "oracle", "_ref", "ts")
REPLAY_JS = os.path.join(ROOT, "oracle", "ref_replay.js")


def ref_available():
    return os.path.isdir(REF_SRC) and shutil.which("node") is not None


def build_ref():
    """Type-erase the reference into oracle/_ref/ts (again when the eraser or the
    stubs changed since)."""
    stamp = os.path.join(REF_OUT, "client.js")
    newest = max(os.path.getmtime(os.path.join(ROOT, "oracle", f)) for f in ("ts_erase.py", "ref_stubs.js"))
    if not os.path.exists(stamp) or os.path.getmtime(stamp) < newest:
        subprocess.check_call(["python3", os.path.join(ROOT, "oracle", "ts_erase.py"), "--out", REF_OUT],
                              stdout=subprocess.DEVNULL)
    return REF_OUT


def ref_replay(docs, timeout=3600):
    build_ref()
    p = subprocess.run(["node", "--max-old-space-size=8192", REPLAY_JS, REF_OUT], input=json.dumps({"docs": docs}),
                       capture_output=True, text=True, timeout=timeout)
    if p.returncode != 0:
        raise RuntimeError(p.stderr[-4000:])
    return json.loads(p.stdout)["docs"]


# ---- generated streams -> ISequencedDocumentMessage (fluidframework_amd/messages.py)
from fluidframework_amd.messages import stream_doc_msgs, stream_docs  # noqa: E402,F401


# ---- canonical digest of reference output ------------------------------------
M61 = (1 << 61) - 1
M64 = (1 << 64) - 1
B1 = 0x1d8e4e27c47d124f % M61
B2 = 0x0a0761d6478bd642 % M61


def _mix64(z):
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M64
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M64
    return z ^ (z >> 31)


def value_ids(stream):
    """canonical JSON -> interned value id, for every value the stream uses"""
    b = stream["batch"]
    ids = {}
    for v in np.unique(b["props"]["value"]):
        v = int(v)
        if v:
            ids[json.dumps(json.loads(gen.value_json(v)), sort_keys=True, separators=(",", ":"))] = v
    return ids


def content_digest(segs, vids, key_names=gen.KEY_NAMES):
    """the digest of DESIGN.md over reference segments [[text | {marker}, props], ...]"""
    n = h1 = h2 = sm = 0
    for content, props in segs:
        ph = 0
        for k, name in enumerate(key_names):
            if props and name in props and props[name] is not None:
                vid = vids[json.dumps(props[name], sort_keys=True, separators=(",", ":"))]
                ph += _mix64(((k + 1) << 32) | vid)
        ph &= M64
        if isinstance(content, str):
            recs = list(np.frombuffer(content.encode("utf-16-le"), dtype="<u2"))
        else:
            recs = [(1 << 32) | int(content["marker"])]
        for rec in recs:
            x = _mix64((int(rec) * 0x9E3779B97F4A7C15 + ph) & M64) % M61
            h1 = (h1 * B1 + x) % M61
            h2 = (h2 * B2 + x) % M61
            sm = (sm + x) & M64
            n += 1
    return np.array([n, h1, h2, sm], dtype=np.uint64)
