"""Locate and load the in-tree native libraries (built by __graft_entry__.build()
or `make -C fluidframework_amd/csrc`).  Missing libraries raise: there is no
fallback path."""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "_lib")
# MTE_LIB_DIR: another in-tree build of libmte.so (the profiling build of
# tools/tree_prof.py --prof); the product default is _lib/
MTE_DIR = os.environ.get("MTE_LIB_DIR") or LIB_DIR
_cache = {}


def lib_path(name):
    return os.path.join(MTE_DIR if name == "libmte.so" else LIB_DIR, name)


def _load(name):
    if name in _cache:
        return _cache[name]
    p = lib_path(name)
    if not os.path.exists(p):
        raise ImportError(f"{p} is not built; run `python -c 'import __graft_entry__ as g; g.build()'`"
                          f" or `make -C {os.path.join(_HERE, 'csrc')}`")
    lib = C.CDLL(p)
    _cache[name] = lib
    return lib


def load_mte():
    lib = _load("libmte.so")
    if getattr(lib, "_mte_typed", False):
        return lib
    vp, u32, i32, u64 = C.c_void_p, C.c_uint32, C.c_int32, C.c_uint64
    sig = {
        "mte_abi_version": ([], C.c_int),
        "mte_strerror": ([C.c_int], C.c_char_p),
        "mte_build_info": ([], C.c_char_p),
        "mte_create": ([vp, vp], C.c_int),
        "mte_destroy": ([vp], C.c_int),
        "mte_last_error": ([vp], C.c_char_p),
        "mte_load_docs": ([vp, u32, vp, vp, u64, vp, u32, vp, u32], C.c_int),
        "mte_load_segments": ([vp, vp, vp, u64], C.c_int),
        "mte_submit": ([vp, vp], C.c_int),
        "mte_run": ([vp], C.c_int),
        "mte_sync": ([vp], C.c_int),
        "mte_reset": ([vp], C.c_int),
        "mte_digest": ([vp, vp, u32], C.c_int),
        "mte_digest_device": ([vp, vp, u32], C.c_int),
        "mte_read_doc": ([vp, u32, vp], C.c_int),
        "mte_read_deltas": ([vp, u32, vp, u64, vp], C.c_int),
        "mte_set_event_capacity": ([vp, u32], C.c_int),
        "mte_set_ref_capacity": ([vp, u32], C.c_int),
        "mte_read_refs": ([vp, u32, vp, u32], C.c_int),
        "mte_read_refs_transient": ([vp, u32, vp, u32], C.c_int),
        "mte_read_ref_order": ([vp, u32, vp, u32], C.c_int),
        "mte_read_segments": ([vp, u32, vp], C.c_int),
        "mte_doc_status": ([vp, vp, u32], C.c_int),
        "mte_stats_get": ([vp, vp], C.c_int),
        "mte_set_stats": ([vp, C.c_int], C.c_int),
        "mte_comm_unique_id": ([vp], C.c_int),
        "mte_comm_init": ([vp, C.c_int, C.c_int, vp], C.c_int),
        "mte_comm_share": ([vp, vp], C.c_int),
        "mte_comm_barrier": ([vp], C.c_int),
        "mte_comm_allreduce_f64": ([vp, vp, C.c_int], C.c_int),
        "mte_comm_gather_digests": ([vp, vp, C.c_uint64, u32], C.c_int),
        "mte_comm_world": ([vp, vp, vp], C.c_int),
        "mte_comm_destroy": ([vp], C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    del i32
    lib._mte_typed = True
    return lib


def load_gen():
    lib = _load("libmtegen.so")
    if getattr(lib, "_gen_typed", False):
        return lib
    vp = C.c_void_p
    for name, args in {
        "mteg_generate": [vp, vp], "mteg_get_sizes": [vp, vp],
        "mteg_fill": [vp, vp, vp, vp, vp, vp, vp, vp], "mteg_free": [vp],
        "mteg_value_json": [C.c_uint32, C.c_char_p, C.c_uint32],
    }.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = C.c_int
    lib._gen_typed = True
    return lib
