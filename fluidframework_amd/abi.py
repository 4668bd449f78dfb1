"""ctypes / numpy mirror of include/mte.h (the C-ABI of libmte.so).

Plain layout definitions only; no behaviour.  Field order and sizes must match
include/mte.h exactly (checked by tests/test_abi.py).
"""
import ctypes as C

import numpy as np

MTE_ABI_VERSION = 1
MTE_MAX_KEYS = 8
MTE_MAX_CLIENTS = 32
MTE_MAX_CLIENTS_TREE = 64  # local-client and MTE_DOC_TREE documents (include/mte.h)

MTE_OK = 0
MTE_E_INVALID_ARG = -1
MTE_E_NO_DEVICE = -2
MTE_E_HIP = -3
MTE_E_CAPACITY = -4
MTE_E_SEQ_ORDER = -5
MTE_E_MSN_ORDER = -6
MTE_E_MSN_GT_SEQ = -7
MTE_E_INSERT_FAILED = -8
MTE_E_UNSUPPORTED = -9
MTE_E_STATE = -10
MTE_E_OOM = -11
MTE_E_CLIENT_RANGE = -12

ERROR_NAMES = {
    MTE_E_INVALID_ARG: "invalid argument",
    MTE_E_NO_DEVICE: "no HIP device",
    MTE_E_HIP: "HIP runtime error",
    MTE_E_CAPACITY: "segment capacity exceeded",
    MTE_E_SEQ_ORDER: "0x030: Incoming remote op sequence# <= local collabWindow's currentSequence#",
    MTE_E_MSN_ORDER: "0x031: Incoming remote op minSequence# < local collabWindow's minSequence#",
    MTE_E_MSN_GT_SEQ: "0x039: Incoming op sequence# < minSequence#",
    MTE_E_INSERT_FAILED: "MergeTree insert failed",
    MTE_E_UNSUPPORTED: "unsupported op shape",
    MTE_E_STATE: "call out of order",
    MTE_E_OOM: "out of memory",
    MTE_E_CLIENT_RANGE: "too many clients in one document",
}

OP_INSERT, OP_REMOVE, OP_ANNOTATE, OP_NOOP, OP_ACK, OP_ROLLBACK = 0, 1, 2, 3, 4, 5
OP_REGEN = 6          # Client.regeneratePendingOp (a local record; include/mte.h)
OP_RBKEY = 7          # an annotate rollback's previous-value candidates (include/mte.h)
OP_REF = 8            # create / remove a local reference (a local record; include/mte.h)
OP_RELPOS = 9         # relative positions of the record that follows (include/mte.h)
RP_POS1, RP_BEFORE1, RP_POS2, RP_BEFORE2 = 0x100, 0x200, 0x400, 0x800
REF_SLIDE_ON_REMOVE, REF_STAY_ON_REMOVE, REF_TRANSIENT = 0x40, 0x80, 0x100  # ReferenceType (ops.ts)
DELTA_REGEN = 0x10    # kind flag of its output records
DELTA_REBASE = 0x20   # MTE_OP_REF b = 4 / 5: the answer's kind
DELTA_SLIDE = 0x40    # a reference slid off a removed segment (MTE_DOC_SLIDE_EVENTS)
DELTA_REFPOS = 0x80   # every reference as the record that slid one left the document
DELTA_MAINT = 0x100   # | MTE_MAINT_*: a maintenance callback's segment (MTE_DOC_MAINT_EVENTS)
ANNOTATE_SLOTS = 32   # pending local annotate groups tracked per document
F_MARKER, F_MSG_END, F_REWRITE, F_LOCAL = 0x1, 0x2, 0x4, 0x8
F_COMBINE = 0x10         # annotate combiningOp incr / consensus (value maps, include/mte.h)
F_REGENERATED = 0x20     # an ack of a regenerated message (include/mte.h)
COMBINE_PAIR = 0x80000000
MTE_VALUE_UNEQUAL = 0x40000000  # a value id that matches no other (NaN), include/mte.h
LOCAL_SEQ_BASE = 0x40000000
NO_PROPS = 0xFFFFFFFF
DOC_NEW_LENGTH_CALC = 0x1
DOC_ROUND_SYNC = 0x2
DOC_LOCAL_CLIENT = 0x4

# 32-byte mte_op record.
OP_DTYPE = np.dtype([
    ("seq", "<i4"), ("ref_seq", "<i4"), ("min_seq", "<i4"),
    ("type", "u1"), ("client", "u1"), ("flags", "<u2"),
    ("pos1", "<i4"), ("pos2", "<i4"), ("a", "<u4"), ("b", "<u4"),
])
assert OP_DTYPE.itemsize == 32

PROP_DTYPE = np.dtype([("key", "<u4"), ("value", "<u4")])
PROPSET_DTYPE = np.dtype([("first", "<u4"), ("count", "<u4")])
DOC_INIT_DTYPE = np.dtype([
    ("text_off", "<u4"), ("text_len", "<u4"), ("flags", "<u4"), ("propset", "<u4"),
    ("min_seq", "<i4"), ("cur_seq", "<i4"),
])
assert DOC_INIT_DTYPE.itemsize == 24

# mte_seg: a segment with merge info (mte_load_segments, snapshot body).
NOT_REMOVED = 0x7FFFFFFF
SEG_DTYPE = np.dtype([
    ("text_off", "<u4"), ("len", "<u4"), ("seq", "<i4"), ("removed_seq", "<i4"),
    ("removers", "<u4"), ("client", "<i4"), ("kind", "<u4"), ("propset", "<u4")])
assert SEG_DTYPE.itemsize == 32


class MteConfig(C.Structure):
    _fields_ = [("device", C.c_int32), ("n_keys", C.c_uint32),
                ("seg_capacity", C.c_uint32), ("flags", C.c_uint32)]


class MteBatch(C.Structure):
    _fields_ = [("n_docs", C.c_uint32), ("op_offsets", C.c_void_p), ("ops", C.c_void_p),
                ("n_ops", C.c_uint64), ("text", C.c_void_p), ("text_units", C.c_uint64),
                ("propsets", C.c_void_p), ("n_propsets", C.c_uint32),
                ("props", C.c_void_p), ("n_props", C.c_uint32)]


class MteStats(C.Structure):
    _fields_ = [("ops_applied", C.c_uint64), ("segs_scanned", C.c_uint64),
                ("segs_written", C.c_uint64), ("prop_writes", C.c_uint64),
                ("units_inserted", C.c_uint64), ("max_segs", C.c_uint64),
                ("kernel_ms", C.c_double), ("algo_bytes", C.c_double),
                ("chunk_scanned", C.c_uint64), ("round_bytes", C.c_double)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class MteSegList(C.Structure):
    _fields_ = [("segs", C.c_void_p), ("props", C.c_void_p), ("seg_cap", C.c_uint64), ("n_segs", C.c_uint64),
                ("text", C.c_void_p), ("text_cap", C.c_uint64), ("n_text", C.c_uint64)]


class MteDocView(C.Structure):
    _fields_ = [("status", C.c_int32), ("cur_seq", C.c_int32), ("min_seq", C.c_int32),
                ("length", C.c_uint32),
                ("text", C.c_void_p), ("text_cap", C.c_uint32), ("n_text", C.c_uint32),
                ("seg_len", C.c_void_p), ("seg_kind", C.c_void_p), ("seg_props", C.c_void_p),
                ("seg_cap", C.c_uint32), ("n_segs", C.c_uint32)]


# Every symbol include/mte.h declares (tests check libmte.so exports them all).
EXPORTED_SYMBOLS = [
    "mte_abi_version", "mte_strerror", "mte_build_info", "mte_create", "mte_destroy", "mte_last_error",
    "mte_load_docs", "mte_load_segments", "mte_submit", "mte_run", "mte_sync", "mte_reset", "mte_digest",
    "mte_digest_device", "mte_read_doc", "mte_read_segments", "mte_doc_status", "mte_stats_get", "mte_set_stats",
    "mte_comm_unique_id", "mte_comm_init", "mte_comm_share", "mte_comm_barrier", "mte_comm_allreduce_f64",
    "mte_comm_gather_digests", "mte_comm_world", "mte_comm_destroy", "mte_read_deltas", "mte_set_event_capacity",
    "mte_set_ref_capacity", "mte_read_refs", "mte_read_refs_transient", "mte_read_ref_order",
]

DOC_EVENTS = 0x8
DOC_REFS = 0x10
DOC_SLIDE_EVENTS = 0x20
DOC_MAINT_EVENTS = 0x40
DOC_TREE = 0x80  # a new-calc document without a local client on the HBM tree pass (segment-exact events)
DELTA_DTYPE = np.dtype([("op", "<u4"), ("kind", "<u4"), ("pos", "<i4"), ("len", "<i4"), ("removed", "<u4")])


def ptr(a):
    """Address of a numpy array's data (None for empty / None)."""
    if a is None or a.size == 0:
        return None
    return a.ctypes.data


class MergeTreeError(RuntimeError):
    """A replay error, carrying the engine status code (and, where one exists,
    the hex assert code of the reference)."""

    def __init__(self, code, detail=""):
        self.code = code
        msg = ERROR_NAMES.get(code, f"error {code}")
        super().__init__(f"{msg} ({code}){': ' + detail if detail else ''}")
