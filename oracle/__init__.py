"""Python binding of the CPU restatement (oracle/oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker / the timed CPU baseline,
never as the product path.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from fluidframework_amd.abi import DOC_INIT_DTYPE, PROP_DTYPE, PROPSET_DTYPE, SEG_DTYPE, ptr
from fluidframework_amd.engine import EngineBase, _arr, make_batch_struct

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
    for name, args in {
        "orc_create": [u32, vp], "orc_destroy": [vp],
        "orc_load_docs": [vp, u32, vp, vp, u64, vp, u32, vp, u32],
        "orc_load_segments": [vp, vp, vp, u64],
        "orc_read_segments": [vp, u32, vp],
        "orc_apply_batch": [vp, vp, C.c_int], "orc_read_doc": [vp, u32, vp],
        "orc_digest": [vp, vp, u32], "orc_doc_status": [vp, vp, u32],
        "orc_stats_get": [vp, vp], "orc_doc_nsegs": [vp, u32, vp],
    }.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = C.c_int
    _lib = lib
    return lib


class OracleEngine(EngineBase):
    """Same surface as fluidframework_amd.engine.DeviceEngine, on the CPU."""

    def __init__(self, n_keys=0, threads=1):
        self.lib = load()
        self.n_keys = n_keys
        self.threads = threads
        h = C.c_void_p()
        self._check(self.lib.orc_create(n_keys, C.byref(h)), "orc_create")
        self.ctx = h

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.orc_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_docs(self, inits, text=None, propsets=None, props=None):
        inits = _arr(inits, DOC_INIT_DTYPE)
        text = _arr(text, np.uint16)
        ps = _arr(propsets, PROPSET_DTYPE)
        pe = _arr(props, PROP_DTYPE)
        self.n_docs = len(inits)
        self._check(self.lib.orc_load_docs(self.ctx, len(inits), ptr(inits), ptr(text), len(text),
                                           ptr(ps), len(ps), ptr(pe), len(pe)), "load_docs")

    def _read_segments(self, doc, lp):
        return self.lib.orc_read_segments(self.ctx, doc, lp)

    def load_segments(self, seg_offsets, segs):
        offs = _arr(seg_offsets, np.uint64)
        segs = _arr(segs, SEG_DTYPE)
        self._check(self.lib.orc_load_segments(self.ctx, ptr(offs), ptr(segs), len(segs)), "load_segments")

    def apply_batch(self, batch):
        b, keep = make_batch_struct(self.n_docs, batch)
        self._check(self.lib.orc_apply_batch(self.ctx, C.byref(b), self.threads), "apply_batch")
        del keep
        return 0

    def nsegs(self, doc):
        n = C.c_uint32()
        self._check(self.lib.orc_doc_nsegs(self.ctx, doc, C.byref(n)), "nsegs")
        return n.value

    def _read_doc(self, doc, vptr):
        return self.lib.orc_read_doc(self.ctx, doc, vptr)

    def _digest(self, p, n):
        return self.lib.orc_digest(self.ctx, p, n)

    def _doc_status(self, p, n):
        return self.lib.orc_doc_status(self.ctx, p, n)

    def _stats(self, sp):
        return self.lib.orc_stats_get(self.ctx, sp)
