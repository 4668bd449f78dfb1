"""Seeded synthetic op streams for the BASELINE.json configs.

Wraps libmtegen.so (csrc/mte_gen.cpp).  These are engine *inputs*; parity is
always engine-vs-oracle on the same stream.
"""
import ctypes as C
import os

import numpy as np

from . import _native
from .abi import DOC_INIT_DTYPE, DOC_ROUND_SYNC, NOT_REMOVED, OP_DTYPE, PROP_DTYPE, PROPSET_DTYPE, SEG_DTYPE, MergeTreeError  # noqa: F401

MIX_INSERT, MIX_REMOVE, MIX_ANNOTATE = 1, 2, 4
N_KEYS = 4  # client, bold, color, markerId
KEY_NAMES = ["client", "bold", "color", "markerId"]


class GenConfig(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in (
        "config_id", "n_docs", "ops_per_doc", "doc_base", "clients", "min_length", "round_ops",
        "mix", "marker_every", "length_mode", "init_len", "n_threads", "init_segs", "max_range",
        "max_lag", "newline_every")] + [("doc_ids", C.c_void_p)]


class GenSizes(C.Structure):
    _fields_ = [("n_ops", C.c_uint64), ("text_units", C.c_uint64), ("init_units", C.c_uint64),
                ("n_propsets", C.c_uint32), ("n_props", C.c_uint32)]


# BASELINE.json configs (index = config id).  Config 1 is the reference's own
# CPU farm (replay fixtures).  Config 5 preloads 2^20 one-unit segments per doc
# (mte_load_segments) and runs 4 rounds of 65,536 concurrent ops (deep collab
# window, zamboni at each round) through the chunked big-document pass.
PRESETS = {
    2: dict(n_docs=1000, ops_per_doc=1000, clients=8, min_length=16, round_ops=32,
            mix=MIX_INSERT | MIX_REMOVE, marker_every=0, length_mode=0),
    3: dict(n_docs=10000, ops_per_doc=10000, clients=8, min_length=16, round_ops=64,
            mix=MIX_INSERT | MIX_REMOVE | MIX_ANNOTATE, marker_every=16, length_mode=0),
    4: dict(n_docs=100000, ops_per_doc=500, clients=8, min_length=8, round_ops=8,
            mix=MIX_INSERT | MIX_REMOVE | MIX_ANNOTATE, marker_every=16, length_mode=0),
    # config 5 runs the new length calculation: legacy documents take the
    # reference's B+tree placement on the tree passes, which the
    # chunked pass and its round phases do not restate
    5: dict(n_docs=64, ops_per_doc=262144, clients=8, min_length=16, round_ops=65536,
            mix=MIX_INSERT | MIX_REMOVE | MIX_ANNOTATE, marker_every=16, length_mode=2,
            init_segs=1 << 20, max_range=16),
}


def seg_capacity(config_id, params=None):
    """ctx seg_capacity for a config (0 = the library default)."""
    p = params or PRESETS.get(config_id, {})
    n0 = p.get("init_segs", 0)
    if not n0:
        return 0
    # the preload plus up to 3 segments per op (2 splits + 1 insert), rounded
    # up to a power of two
    need = n0 + 3 * p.get("ops_per_doc", 1) + 1024
    return max(8192, 1 << (need - 1).bit_length())


def default_threads():
    n = os.cpu_count() or 1
    return max(1, min(n, 16))


def generate(config_id=2, n_docs=None, ops_per_doc=None, doc_base=0, n_threads=None, doc_ids=None, **over):
    """-> dict(inits, init_text, batch={op_offsets, ops, text, propsets, props}).

    Documents are the global documents doc_base .. doc_base + n_docs - 1, or
    the global indices `doc_ids` (a rank's shard, fluidframework_amd/dist.py)."""
    p = dict(PRESETS.get(config_id, PRESETS[2]))
    ids = None
    if doc_ids is not None:
        ids = np.ascontiguousarray(doc_ids, dtype=np.uint32)
        n_docs = len(ids)
    if n_docs is not None:
        p["n_docs"] = n_docs
    if ops_per_doc is not None:
        p["ops_per_doc"] = ops_per_doc
    p.update(over)
    lib = _native.load_gen()
    cfg = GenConfig(config_id, p["n_docs"], p["ops_per_doc"], doc_base, p["clients"],
                    p["min_length"], p["round_ops"], p["mix"], p["marker_every"],
                    p["length_mode"], p.get("init_len", 0), n_threads or default_threads(),
                    p.get("init_segs", 0), p.get("max_range", 0), p.get("max_lag", 0),
                    p.get("newline_every", 0), ids.ctypes.data if ids is not None and len(ids) else None)
    h = C.c_void_p()
    rc = lib.mteg_generate(C.byref(cfg), C.byref(h))
    if rc:
        raise MergeTreeError(rc, "mteg_generate")
    try:
        sz = GenSizes()
        lib.mteg_get_sizes(h, C.byref(sz))
        nd = p["n_docs"]
        inits = np.zeros(nd, DOC_INIT_DTYPE)
        init_text = np.zeros(max(sz.init_units, 1), np.uint16)
        offs = np.zeros(nd + 1, np.uint64)
        ops = np.zeros(sz.n_ops, OP_DTYPE)
        text = np.zeros(max(sz.text_units, 1), np.uint16)
        ps = np.zeros(sz.n_propsets, PROPSET_DTYPE)
        pe = np.zeros(sz.n_props, PROP_DTYPE)
        rc = lib.mteg_fill(h, inits.ctypes.data, init_text.ctypes.data, offs.ctypes.data,
                           ops.ctypes.data, text.ctypes.data, ps.ctypes.data, pe.ctypes.data)
        if rc:
            raise MergeTreeError(rc, "mteg_fill")
    finally:
        lib.mteg_free(h)
    if p.get("round_sync"):
        # the stream is round-synchronous (max_lag 0): declare it, so legacy
        # documents may replay on the flat passes (MTE_DOC_ROUND_SYNC)
        if p.get("max_lag", 0):
            raise ValueError("round_sync needs max_lag == 0")
        inits["flags"] |= DOC_ROUND_SYNC
    segs = None
    if p.get("init_segs", 0):
        segs = preload_segments(inits, p["init_segs"])
    return {"inits": inits, "init_text": init_text[: sz.init_units], "n_keys": N_KEYS, "segs": segs,
            "batch": {"op_offsets": offs, "ops": ops, "text": text[: sz.text_units],
                      "propsets": ps, "props": pe}, "params": p}


def split_ops(stream, k, parts):
    """Batch k of `parts`: every document's ops [k/parts, (k+1)/parts) of its
    count, cut at message ends (MTE_F_MSG_END) so windows stay whole."""
    return cut_ops(stream, k / parts, (k + 1) / parts)


def cut_ops(stream, f0, f1):
    """Every document's ops [f0, f1) of its count (fractions), cut at message
    ends (MTE_F_MSG_END) so windows stay whole; the batch keeps all the text."""
    b = stream["batch"]
    o = b["op_offsets"].astype(np.int64)
    ops = b["ops"]
    sel, offs = [], [0]
    for d in range(len(o) - 1):
        n = o[d + 1] - o[d]
        ends = np.flatnonzero(ops["flags"][o[d]:o[d + 1]] & 2) + 1  # cut points after MSG_END records
        def cut(x):
            if x <= 0:
                return 0
            if x >= n:
                return int(n)
            i = np.searchsorted(ends, x)
            return int(ends[i]) if i < len(ends) else int(n)
        a, e = cut(int(round(n * f0))), cut(int(round(n * f1)))
        sel.append(np.arange(o[d] + a, o[d] + e))
        offs.append(offs[-1] + (e - a))
    idx = np.concatenate(sel) if sel else np.zeros(0, np.int64)
    return dict(b, ops=ops[idx], op_offsets=np.array(offs, np.uint64))


def preload_segments(inits, n_per_doc):
    """-> (seg_offsets, segs): every doc's load text as one-unit seq-0 segments
    (a summary body of n_per_doc segments, loaded with mte_load_segments)."""
    nd = len(inits)
    offs = np.arange(nd + 1, dtype=np.uint64) * np.uint64(n_per_doc)
    segs = np.zeros(nd * n_per_doc, SEG_DTYPE)
    base = np.repeat(inits["text_off"].astype(np.uint64), n_per_doc)
    segs["text_off"] = (base + np.tile(np.arange(n_per_doc, dtype=np.uint64), nd)).astype(np.uint32)
    segs["len"] = 1
    segs["removed_seq"] = NOT_REMOVED
    segs["client"] = -1
    segs["propset"] = 0xFFFFFFFF
    return offs, segs


def load_stream(engine, stream):
    """load_docs (+ load_segments for a preloaded body) of a generated stream."""
    engine.load_docs(stream["inits"], stream["init_text"])
    if stream.get("segs") is not None:
        engine.load_segments(*stream["segs"])


def prefix_ops(stream, d1, k):
    """Sub-stream of docs [0, d1) with the first k ops of each (bounded
    parity / CPU-baseline samples of long-document workloads)."""
    sub = slice_docs(stream, 0, d1)
    b = sub["batch"]
    o = b["op_offsets"].astype(np.int64)
    cnt = np.minimum(o[1:] - o[:-1], k)
    ops = np.concatenate([b["ops"][o[i]:o[i] + cnt[i]] for i in range(d1)]) if d1 else b["ops"][:0]
    offs = np.zeros(d1 + 1, np.uint64)
    offs[1:] = np.cumsum(cnt)
    sub["batch"] = dict(b, ops=ops, op_offsets=offs)
    return sub


def value_json(value_id):
    lib = _native.load_gen()
    buf = C.create_string_buffer(64)
    n = lib.mteg_value_json(value_id, buf, 64)
    return None if n < 0 else buf.value.decode()


def slice_docs(stream, d0, d1):
    """Sub-stream of docs [d0, d1) (same text/propset tables)."""
    b = stream["batch"]
    o = b["op_offsets"]
    lo, hi = int(o[d0]), int(o[d1])
    segs = stream.get("segs")
    if segs is not None:
        so, sg = segs
        segs = (so[d0:d1 + 1] - so[d0], sg[int(so[d0]):int(so[d1])])
    return {"inits": stream["inits"][d0:d1], "init_text": stream["init_text"], "segs": segs,
            "n_keys": stream["n_keys"],
            "batch": {"op_offsets": o[d0:d1 + 1] - o[d0], "ops": b["ops"][lo:hi],
                      "text": b["text"], "propsets": b["propsets"], "props": b["props"]},
            "params": stream["params"]}
