"""Seeded synthetic op streams for the BASELINE.json configs.

Wraps libmtegen.so (csrc/mte_gen.cpp).  These are engine *inputs*; parity is
always engine-vs-oracle on the same stream.
"""
import ctypes as C
import os

import numpy as np

from . import _native
from .abi import DOC_INIT_DTYPE, OP_DTYPE, PROP_DTYPE, PROPSET_DTYPE, MergeTreeError

MIX_INSERT, MIX_REMOVE, MIX_ANNOTATE = 1, 2, 4
N_KEYS = 4  # client, bold, color, markerId
KEY_NAMES = ["client", "bold", "color", "markerId"]


class GenConfig(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in (
        "config_id", "n_docs", "ops_per_doc", "doc_base", "clients", "min_length", "round_ops",
        "mix", "marker_every", "length_mode", "init_len", "n_threads")]


class GenSizes(C.Structure):
    _fields_ = [("n_ops", C.c_uint64), ("text_units", C.c_uint64), ("init_units", C.c_uint64),
                ("n_propsets", C.c_uint32), ("n_props", C.c_uint32)]


# BASELINE.json configs (index = config id).  Config 1 is the reference's own
# CPU farm (replay fixtures); 5 needs the chunked path (not built yet).
PRESETS = {
    2: dict(n_docs=1000, ops_per_doc=1000, clients=8, min_length=16, round_ops=32,
            mix=MIX_INSERT | MIX_REMOVE, marker_every=0, length_mode=0),
    3: dict(n_docs=10000, ops_per_doc=10000, clients=8, min_length=16, round_ops=64,
            mix=MIX_INSERT | MIX_REMOVE | MIX_ANNOTATE, marker_every=16, length_mode=0),
    4: dict(n_docs=100000, ops_per_doc=500, clients=8, min_length=8, round_ops=8,
            mix=MIX_INSERT | MIX_REMOVE | MIX_ANNOTATE, marker_every=16, length_mode=0),
}


def default_threads():
    n = os.cpu_count() or 1
    return max(1, min(n, 16))


def generate(config_id=2, n_docs=None, ops_per_doc=None, doc_base=0, n_threads=None, **over):
    """-> dict(inits, init_text, batch={op_offsets, ops, text, propsets, props})."""
    p = dict(PRESETS.get(config_id, PRESETS[2]))
    if n_docs is not None:
        p["n_docs"] = n_docs
    if ops_per_doc is not None:
        p["ops_per_doc"] = ops_per_doc
    p.update(over)
    lib = _native.load_gen()
    cfg = GenConfig(config_id, p["n_docs"], p["ops_per_doc"], doc_base, p["clients"],
                    p["min_length"], p["round_ops"], p["mix"], p["marker_every"],
                    p["length_mode"], p.get("init_len", 0), n_threads or default_threads())
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
    return {"inits": inits, "init_text": init_text[: sz.init_units], "n_keys": N_KEYS,
            "batch": {"op_offsets": offs, "ops": ops, "text": text[: sz.text_units],
                      "propsets": ps, "props": pe}, "params": p}


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
    return {"inits": stream["inits"][d0:d1], "init_text": stream["init_text"],
            "n_keys": stream["n_keys"],
            "batch": {"op_offsets": o[d0:d1 + 1] - o[d0], "ops": b["ops"][lo:hi],
                      "text": b["text"], "propsets": b["propsets"], "props": b["props"]},
            "params": stream["params"]}
