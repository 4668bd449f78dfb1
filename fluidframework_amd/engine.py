"""Python binding of libmte.so (the HIP engine) through its C-ABI.

`DeviceEngine` is a thin ctypes layer over include/mte.h: documents are loaded
once, batches of op records are uploaded to HBM and replayed by the gfx950
kernels.  There is no CPU fallback: if libmte.so (or a HIP device) is missing
this module raises.
"""
import ctypes as C

import numpy as np

from . import _native
from .abi import (DELTA_DTYPE, DOC_INIT_DTYPE, EXPORTED_SYMBOLS, OP_DTYPE, PROP_DTYPE, PROPSET_DTYPE, SEG_DTYPE,
                  MergeTreeError, MteBatch, MteConfig, MteDocView, MteSegList, MteStats, ptr)
from .packing import units_to_str


def _arr(a, dtype):
    if a is None:
        return np.zeros(0, dtype)
    return np.ascontiguousarray(a, dtype=dtype)


def make_batch_struct(n_docs, batch):
    """-> (MteBatch, keepalive list)."""
    offs = _arr(batch["op_offsets"], np.uint64)
    ops = _arr(batch["ops"], OP_DTYPE)
    text = _arr(batch.get("text"), np.uint16)
    ps = _arr(batch.get("propsets"), PROPSET_DTYPE)
    pe = _arr(batch.get("props"), PROP_DTYPE)
    if len(offs) != n_docs + 1:
        raise ValueError("op_offsets must have n_docs+1 entries")
    b = MteBatch(n_docs, ptr(offs), ptr(ops), len(ops), ptr(text), len(text),
                 ptr(ps), len(ps), ptr(pe), len(pe))
    return b, [offs, ops, text, ps, pe]


class EngineBase:
    """Operations shared by the device engine and the CPU oracle binding."""

    n_keys = 0
    n_docs = 0
    ref_capacity = 1024  # mte_set_ref_capacity's default (include/mte.h)

    def doc_clients(self, observer_id, min_seq=0, local=False):
        """A document's client map (packing.DocClients) that knows this
        engine's per-document reference capacity (set_ref_capacity), as the Node
        host's BatchClient copies engine.refCapacity."""
        from .packing import DocClients
        return DocClients(observer_id, min_seq, local, ref_cap=self.ref_capacity)

    def _check(self, rc, what=""):
        if rc != 0:
            raise MergeTreeError(rc, f"{what}: {self._last_error()}")

    def _last_error(self):
        return ""

    def read_doc(self, doc):
        """-> dict(status, cur_seq, min_seq, length, text, segs=[(len, kind, props)])."""
        v = MteDocView()
        self._check(self._read_doc(doc, C.byref(v)), "read_doc")
        text = np.zeros(max(v.n_text, 1), np.uint16)
        nseg = max(v.n_segs, 1)
        seg_len = np.zeros(nseg, np.uint32)
        seg_kind = np.zeros(nseg, np.uint32)
        seg_props = np.zeros(nseg * max(self.n_keys, 1), np.uint32)
        v.text, v.text_cap = ptr(text), len(text)
        v.seg_len, v.seg_kind, v.seg_props, v.seg_cap = ptr(seg_len), ptr(seg_kind), ptr(seg_props), nseg
        self._check(self._read_doc(doc, C.byref(v)), "read_doc")
        props = seg_props[: v.n_segs * self.n_keys].reshape(v.n_segs, self.n_keys) if self.n_keys else \
            np.zeros((v.n_segs, 0), np.uint32)
        segs = [(int(seg_len[i]), int(seg_kind[i]), tuple(int(x) for x in props[i]))
                for i in range(v.n_segs)]
        return {"status": v.status, "cur_seq": v.cur_seq, "min_seq": v.min_seq,
                "length": v.length, "text": units_to_str(text[: v.n_text]), "segs": segs}

    def read_deltas(self, doc):
        """Delta events of the last batch of an MTE_DOC_EVENTS doc -> DELTA_DTYPE[n]
        (op = record index in the doc's batch, kind, pos in the doc's own view, len)."""
        n = C.c_uint64()
        self._check(self._read_deltas(doc, None, 0, C.byref(n)), "read_deltas")
        out = np.zeros(max(n.value, 1), DELTA_DTYPE)
        self._check(self._read_deltas(doc, ptr(out), n.value, C.byref(n)), "read_deltas")
        return out[: n.value]

    def read_refs(self, doc, n, transient=False):
        """Positions of local reference slots [0, n) of an MTE_DOC_REFS doc in its
        own view (localReferencePositionToPosition; -1 = detached / unused);
        transient: as Transient references (mte_read_refs_transient)."""
        out = np.zeros(max(n, 1), np.int32)
        self._check(self._read_refs(doc, ptr(out), n, transient), "read_refs")
        return out[:n]

    def read_ref_order(self, doc, n):
        """Document order of local reference slots [0, n) (mte_read_ref_order:
        the index of the held text unit each sits on; -1 = detached / unused)."""
        out = np.zeros(max(n, 1), np.int64)
        self._check(self.lib.mte_read_ref_order(self.ctx, doc, ptr(out), n), "read_ref_order")
        return out[:n]

    def read_segments(self, doc):
        """-> (segs SEG_DTYPE[n] with text_off into text, props uint32[n, n_keys], text uint16[])."""
        v = MteSegList()
        self._check(self._read_segments(doc, C.byref(v)), "read_segments")
        segs = np.zeros(max(v.n_segs, 1), SEG_DTYPE)
        props = np.zeros(max(v.n_segs, 1) * max(self.n_keys, 1), np.uint32)
        text = np.zeros(max(v.n_text, 1), np.uint16)
        v.segs, v.props, v.seg_cap = ptr(segs), ptr(props), len(segs)
        v.text, v.text_cap = ptr(text), len(text)
        self._check(self._read_segments(doc, C.byref(v)), "read_segments")
        n = v.n_segs
        return segs[:n], props[: n * self.n_keys].reshape(n, self.n_keys), text[: v.n_text]

    def digest(self):
        out = np.zeros(self.n_docs * 4, np.uint64)
        self._check(self._digest(ptr(out), self.n_docs), "digest")
        return out.reshape(self.n_docs, 4)

    def statuses(self):
        out = np.zeros(self.n_docs, np.int32)
        self._check(self._doc_status(ptr(out), self.n_docs), "doc_status")
        return out

    def stats(self):
        s = MteStats()
        self._check(self._stats(C.byref(s)), "stats")
        return s.as_dict()


class DeviceEngine(EngineBase):
    """One mte_ctx on one HIP device (one per process / GPU)."""

    def __init__(self, n_keys=0, device=0, seg_capacity=0):
        self.lib = _native.load_mte()
        self.n_keys = n_keys
        ctx = C.c_void_p()
        cfg = MteConfig(device, n_keys, seg_capacity, 0)
        rc = self.lib.mte_create(C.byref(cfg), C.byref(ctx))
        if rc != 0:
            raise MergeTreeError(rc, "mte_create: " + self.lib.mte_strerror(rc).decode())
        self.ctx = ctx
        self._keep = []

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.mte_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _last_error(self):
        return self.lib.mte_last_error(self.ctx).decode()

    def load_docs(self, inits, text=None, propsets=None, props=None):
        inits = _arr(inits, DOC_INIT_DTYPE)
        text = _arr(text, np.uint16)
        ps = _arr(propsets, PROPSET_DTYPE)
        pe = _arr(props, PROP_DTYPE)
        self.n_docs = len(inits)
        self._check(self.lib.mte_load_docs(self.ctx, len(inits), ptr(inits), ptr(text), len(text),
                                           ptr(ps), len(ps), ptr(pe), len(pe)), "load_docs")

    def load_segments(self, seg_offsets, segs):
        """Replace docs' loaded content with segment lists (mte_load_segments)."""
        offs = _arr(seg_offsets, np.uint64)
        segs = _arr(segs, SEG_DTYPE)
        self._check(self.lib.mte_load_segments(self.ctx, ptr(offs), ptr(segs), len(segs)), "load_segments")

    def submit(self, batch):
        b, keep = make_batch_struct(self.n_docs, batch)
        self._check(self.lib.mte_submit(self.ctx, C.byref(b)), "submit")
        self._keep = keep  # inputs are copied by mte_submit; kept only for debugging

    def run(self):
        self._check(self.lib.mte_run(self.ctx), "run")

    def sync(self):
        """Raises on a HIP error.  Per-doc replay errors are left in statuses()."""
        rc = self.lib.mte_sync(self.ctx)
        if rc not in (0,) and rc > -4:
            self._check(rc, "sync")
        return rc

    def apply_batch(self, batch):
        self.submit(batch)
        self.run()
        return self.sync()

    def reset(self):
        self._check(self.lib.mte_reset(self.ctx), "reset")

    def set_stats(self, enable):
        """Statistics accounting on (default) / off (mte_set_stats)."""
        self._check(self.lib.mte_set_stats(self.ctx, 1 if enable else 0), "set_stats")

    # ---- node level over RCCL (mte_comm_*, include/mte.h) ----
    def comm_init(self, world, rank, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._check(self.lib.mte_comm_init(self.ctx, world, rank, buf), "comm_init")

    def comm_share(self, other):
        self._check(self.lib.mte_comm_share(self.ctx, other.ctx), "comm_share")

    def comm_barrier(self):
        self._check(self.lib.mte_comm_barrier(self.ctx), "comm_barrier")

    def comm_allreduce(self, value: float, op="sum") -> float:
        v = C.c_double(value)
        self._check(self.lib.mte_comm_allreduce_f64(self.ctx, C.byref(v), 0 if op == "sum" else 1),
                    "comm_allreduce")
        return v.value

    def comm_world(self):
        """(world, rank) of this context's communicator (mte_comm_world)."""
        w, r = C.c_int32(), C.c_int32()
        self._check(self.lib.mte_comm_world(self.ctx, C.byref(w), C.byref(r)), "comm_world")
        return w.value, r.value

    def comm_gather_digests(self, docs_per_rank):
        """Every rank's digests in rank order, sized from the context's own world."""
        world, _ = self.comm_world()
        out = np.zeros(world * docs_per_rank * 4, np.uint64)
        self._check(self.lib.mte_comm_gather_digests(self.ctx, ptr(out), out.size, docs_per_rank),
                    "comm_gather_digests")
        return out.reshape(world, docs_per_rank, 4)

    def comm_destroy(self):
        self._check(self.lib.mte_comm_destroy(self.ctx), "comm_destroy")

    def digest_device(self, device_ptr):
        self._check(self.lib.mte_digest_device(self.ctx, C.c_void_p(device_ptr), self.n_docs),
                    "digest_device")

    def _read_doc(self, doc, vptr):
        return self.lib.mte_read_doc(self.ctx, doc, vptr)

    def _read_deltas(self, doc, p, cap, np_):
        return self.lib.mte_read_deltas(self.ctx, doc, p, cap, np_)

    def set_event_capacity(self, per_op):
        self._check(self.lib.mte_set_event_capacity(self.ctx, per_op), "set_event_capacity")

    def set_ref_capacity(self, per_doc):
        self._check(self.lib.mte_set_ref_capacity(self.ctx, per_doc), "set_ref_capacity")
        self.ref_capacity = int(per_doc)

    def _read_refs(self, doc, p, n, transient=False):
        f = self.lib.mte_read_refs_transient if transient else self.lib.mte_read_refs
        return f(self.ctx, doc, p, n)

    def _digest(self, p, n):
        return self.lib.mte_digest(self.ctx, p, n)

    def _read_segments(self, doc, lp):
        return self.lib.mte_read_segments(self.ctx, doc, lp)

    def _doc_status(self, p, n):
        return self.lib.mte_doc_status(self.ctx, p, n)

    def _stats(self, sp):
        return self.lib.mte_stats_get(self.ctx, sp)


def exported_symbols():
    return list(EXPORTED_SYMBOLS)
