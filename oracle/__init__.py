"""Python binding of the CPU restatements (oracle/oracle.c flat, oracle/tree.c
tree-exact).

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
    for pre in ("orc", "ort"):
        for name, args in {
            "create": [u32, vp], "destroy": [vp],
            "load_docs": [vp, u32, vp, vp, u64, vp, u32, vp, u32],
            "load_segments": [vp, vp, vp, u64],
            "read_segments": [vp, u32, vp],
            "apply_batch": [vp, vp, C.c_int], "read_doc": [vp, u32, vp],
            "digest": [vp, vp, u32], "doc_status": [vp, vp, u32],
            "stats_get": [vp, vp], "doc_nsegs": [vp, u32, vp],
        }.items():
            f = getattr(lib, f"{pre}_{name}")
            f.argtypes = args
            f.restype = C.c_int
    for name, args in {
        "oti_create": [u32, vp], "oti_destroy": [vp],
        "oti_load_docs": [vp, u32, vp, vp, u64, vp, u32, vp, u32],
        "oti_load_segments": [vp, vp, vp, u64], "oti_apply_batch": [vp, vp, C.c_int],
        "oti_read_doc": [vp, u32, vp], "oti_digest": [vp, vp, u32], "oti_doc_status": [vp, vp, u32],
        "oti_doc_nsegs": [vp, u32, vp],
    }.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = C.c_int
    for pre in ("ort", "oti"):
        f = getattr(lib, f"{pre}_doc_shape")
        f.argtypes = [vp, u32, C.c_char_p, u32]
        f.restype = C.c_int
    _lib = lib
    return lib


class _Fn:
    """lib.<prefix>_<name> lookups for one restatement."""

    def __init__(self, lib, pre):
        self.lib, self.pre = lib, pre

    def __getattr__(self, name):
        return getattr(self.lib, f"{self.pre}_{name}")


class OracleEngine(EngineBase):
    """Same surface as fluidframework_amd.engine.DeviceEngine, on the CPU.

    tree=False: the flat restatement (oracle.c).  tree=True: the tree-exact one
    (tree.c), which keeps the reference's B+tree, its lazy zamboni and therefore
    its insert placement next to tombstones in legacy length-calc documents.
    tree="items": the same tree on a flat item array (titems.c), the spec of
    the GPU tree pass."""

    def __init__(self, n_keys=0, threads=1, tree=False):
        self.lib = load()
        self.f = _Fn(self.lib, "oti" if tree == "items" else ("ort" if tree else "orc"))
        self.tree = tree
        self.n_keys = n_keys
        self.threads = threads
        h = C.c_void_p()
        self._check(self.f.create(n_keys, C.byref(h)), "create")
        self.ctx = h

    def close(self):
        if getattr(self, "ctx", None):
            self.f.destroy(self.ctx)
            self.ctx = None

    def shape(self, doc):
        """(tree shape string, LRU heap size) of one document (tree=True only)."""
        buf = C.create_string_buffer(1 << 16)
        hn = self.f.doc_shape(self.ctx, doc, buf, len(buf))
        return buf.value.decode(), hn

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
        self._check(self.f.load_docs(self.ctx, len(inits), ptr(inits), ptr(text), len(text),
                                           ptr(ps), len(ps), ptr(pe), len(pe)), "load_docs")

    def _read_segments(self, doc, lp):
        return self.f.read_segments(self.ctx, doc, lp)

    def load_segments(self, seg_offsets, segs):
        offs = _arr(seg_offsets, np.uint64)
        segs = _arr(segs, SEG_DTYPE)
        self._check(self.f.load_segments(self.ctx, ptr(offs), ptr(segs), len(segs)), "load_segments")

    def apply_batch(self, batch):
        b, keep = make_batch_struct(self.n_docs, batch)
        self._check(self.f.apply_batch(self.ctx, C.byref(b), self.threads), "apply_batch")
        del keep
        return 0

    def nsegs(self, doc):
        n = C.c_uint32()
        self._check(self.f.doc_nsegs(self.ctx, doc, C.byref(n)), "nsegs")
        return n.value

    def _read_doc(self, doc, vptr):
        return self.f.read_doc(self.ctx, doc, vptr)

    def _digest(self, p, n):
        return self.f.digest(self.ctx, p, n)

    def _doc_status(self, p, n):
        return self.f.doc_status(self.ctx, p, n)

    def _stats(self, sp):
        if self.tree == "items":
            return 0
        return self.f.stats_get(self.ctx, sp)
