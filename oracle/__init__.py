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

from fluidframework_amd.abi import DOC_INIT_DTYPE, DOC_LOCAL_CLIENT, PROP_DTYPE, PROPSET_DTYPE, SEG_DTYPE, ptr  # noqa: F401
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
        "oti_doc_nsegs": [vp, u32, vp], "oti_stats_get": [vp, vp], "oti_read_segments": [vp, u32, vp], "oti_set_limit": [vp, u32],
        "oti_read_deltas": [vp, u32, vp, u64, vp], "oti_read_refs": [vp, u32, vp, u32], "oti_read_refs_transient": [vp, u32, vp, u32], "oti_read_ref_order": [vp, u32, vp, u32],
        "och_create": [u32, vp], "och_destroy": [vp], "och_load_docs": [vp, u32, vp, vp, u64, vp, u32, vp, u32],
        "och_load_segments": [vp, vp, vp, u64], "och_apply_batch": [vp, vp, C.c_int], "och_read_doc": [vp, u32, vp],
        "och_digest": [vp, vp, u32], "och_doc_status": [vp, vp, u32], "och_doc_nsegs": [vp, u32, vp],
        "och_stats_get": [vp, vp], "och_read_segments": [vp, u32, vp],
    }.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = C.c_int
    lib.orc_read_deltas.argtypes = [vp, u32, vp, u64, vp]
    lib.orc_read_deltas.restype = C.c_int
    lib.orc_read_refs.argtypes = [vp, u32, vp, u32]
    lib.orc_read_refs.restype = C.c_int
    lib.orc_read_refs_transient.argtypes = [vp, u32, vp, u32]
    lib.orc_read_refs_transient.restype = C.c_int
    lib.orc_read_ref_order.argtypes = [vp, u32, vp, u32]
    lib.orc_read_ref_order.restype = C.c_int
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
    the GPU tree pass.  tree="chunked": the flat restatement with a chunk index
    (chunked.c), for config 5's documents of millions of segments."""

    def __init__(self, n_keys=0, threads=1, tree=False):
        self.lib = load()
        self.f = _Fn(self.lib, {"items": "oti", "chunked": "och"}.get(tree, "ort" if tree else "orc"))
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

    def _read_deltas(self, doc, p, cap, np_):
        f = self.lib.oti_read_deltas if self.tree == "items" else self.lib.orc_read_deltas
        return f(self.ctx, doc, p, cap, np_)

    def set_event_capacity(self, per_op):
        """The restatement's event buffers grow as needed (mte_set_event_capacity's bound is the engine's)."""

    def set_ref_capacity(self, per_doc):
        """The restatement's reference slots grow as needed; the capacity is
        kept for the packers (EngineBase.doc_clients)."""
        self.ref_capacity = int(per_doc)

    def _read_refs(self, doc, p, n, transient=False):
        pre = "oti" if self.tree == "items" else "orc"
        return getattr(self.lib, f"{pre}_read_refs{'_transient' if transient else ''}")(self.ctx, doc, p, n)

    def read_ref_order(self, doc, n):
        f = self.lib.oti_read_ref_order if self.tree == "items" else self.lib.orc_read_ref_order
        out = np.zeros(max(n, 1), np.int64)
        self._check(f(self.ctx, doc, ptr(out), n), "read_ref_order")
        return out[:n]

    def _digest(self, p, n):
        return self.f.digest(self.ctx, p, n)

    def _doc_status(self, p, n):
        return self.f.doc_status(self.ctx, p, n)

    def _stats(self, sp):
        return self.f.stats_get(self.ctx, sp)


def select_docs(batch, idx):
    """The sub-batch of documents idx (same text / property tables)."""
    o = np.asarray(batch["op_offsets"], dtype=np.uint64).astype(np.int64)
    ops = np.asarray(batch["ops"])
    parts = [ops[o[i]:o[i + 1]] for i in idx]
    cnt = np.array([len(p) for p in parts], dtype=np.uint64)
    offs = np.zeros(len(idx) + 1, np.uint64)
    if len(idx):
        np.cumsum(cnt, out=offs[1:])
    sub = dict(batch)
    sub["ops"] = np.concatenate(parts) if parts else ops[:0]
    sub["op_offsets"] = offs
    return sub


class SpecOracle:
    """The engine's specification, document by document: the flat restatement
    (oracle.c) for new length-calc documents and round-synchronous legacy ones
    (MTE_DOC_ROUND_SYNC, checked per batch) and the tree (titems.c, equal to
    tree.c and to the reference) for the other legacy ones — what libmte.so
    computes, statistics and segment read-outs included."""

    def __init__(self, n_keys=0, threads=1, cap=0):
        self.n_keys = n_keys
        self.flat = OracleEngine(n_keys, threads)
        self.tree = OracleEngine(n_keys, threads, tree="items")
        # the tree pass holds a document in registers up to 1,020 items, then
        # in HBM (mte_htree.h) up to the ctx capacity, 4 slots kept free for
        # one op's new items
        cap = cap or 1024
        self.tree.lib.oti_set_limit(self.tree.ctx, max(cap, 64))
        self.n_docs = 0

    def load_docs(self, inits, text=None, propsets=None, props=None):
        inits = _arr(inits, DOC_INIT_DTYPE)
        # flat: MTE_DOC_NEW_LENGTH_CALC | MTE_DOC_ROUND_SYNC without a local client;
        # the tree: legacy documents and every document with a local client
        flat = ((inits["flags"] & 3) != 0) & ((inits["flags"] & DOC_LOCAL_CLIENT) == 0)
        self.sub = [np.where(flat)[0], np.where(~flat)[0]]  # flat, tree
        self.where = np.zeros((len(inits), 2), np.int64)
        for e, idx in enumerate(self.sub):
            self.where[idx, 0] = e
            self.where[idx, 1] = np.arange(len(idx))
        self.flat.load_docs(inits[self.sub[0]], text, propsets, props)
        self.tree.load_docs(inits[self.sub[1]], text, propsets, props)
        self.n_docs = len(inits)

    def _engines(self):
        return (self.flat, self.tree)

    def load_segments(self, seg_offsets, segs):
        offs = np.asarray(seg_offsets, dtype=np.uint64).astype(np.int64)
        segs = _arr(segs, SEG_DTYPE)
        for eng, idx in zip(self._engines(), self.sub):
            if not len(idx):
                continue
            parts = [segs[offs[i]:offs[i + 1]] for i in idx]
            so = np.zeros(len(idx) + 1, np.uint64)
            if len(idx):
                np.cumsum([len(p) for p in parts], out=so[1:])
            eng.load_segments(so, np.concatenate(parts) if parts else segs[:0])

    def apply_batch(self, batch):
        for eng, idx in zip(self._engines(), self.sub):
            if len(idx):
                eng.apply_batch(select_docs(batch, idx))
        return 0

    def _gather(self, fn, shape, dtype):
        out = np.zeros((self.n_docs,) + shape, dtype)
        for e, idx in zip(self._engines(), self.sub):
            if len(idx):
                out[idx] = fn(e)
        return out

    def statuses(self):
        return self._gather(lambda e: e.statuses(), (), np.int32)

    def digest(self):
        return self._gather(lambda e: e.digest(), (4,), np.uint64)

    def read_doc(self, doc):
        e, i = self.where[doc]
        return self._engines()[e].read_doc(int(i))

    def read_segments(self, doc):
        e, i = self.where[doc]
        return self._engines()[e].read_segments(int(i))

    def nsegs(self, doc):
        e, i = self.where[doc]
        return self._engines()[e].nsegs(int(i))

    def read_refs(self, doc, n, transient=False):
        e, i = self.where[doc]
        return self._engines()[e].read_refs(int(i), n, transient)

    def read_ref_order(self, doc, n):
        e, i = self.where[doc]
        return self._engines()[e].read_ref_order(int(i), n)

    def read_deltas(self, doc):
        e, i = self.where[doc]
        return self._engines()[e].read_deltas(int(i))

    def set_event_capacity(self, per_op):
        """The restatements' event buffers grow as needed."""

    def set_ref_capacity(self, per_doc):
        """The restatements' reference slots grow as needed."""
        self.ref_capacity = int(per_doc)

    def stats(self):
        zero = {"ops_applied": 0, "segs_scanned": 0, "segs_written": 0, "prop_writes": 0, "units_inserted": 0,
                "max_segs": 0, "kernel_ms": 0.0, "algo_bytes": 0.0, "chunk_scanned": 0,
                "round_bytes": 0.0}
        a = self.flat.stats() if len(self.sub[0]) else zero
        b = self.tree.stats() if len(self.sub[1]) else zero
        out = {k: a[k] + b[k] for k in a if k not in ("max_segs", "kernel_ms")}
        out["max_segs"] = max(a["max_segs"], b["max_segs"])
        out["kernel_ms"] = 0.0
        return out
