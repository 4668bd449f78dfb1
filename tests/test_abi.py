"""The C-ABI library loads and exports exactly what include/mte.h declares, and
the ctypes/numpy mirrors match the C layouts.  No compute call needs a GPU."""
import ctypes as C
import os
import re
import subprocess


import pytest

from fluidframework_amd import _native, abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mte.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(mte_\w+)\s*\(", src, re.M)))


def test_header_declares_exported_symbol_list():
    assert declared_functions() == sorted(abi.EXPORTED_SYMBOLS)


def test_libmte_exports_every_declared_symbol():
    path = _native.lib_path("libmte.so")
    assert os.path.exists(path), "libmte.so not built (run __graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    missing = [s for s in declared_functions() if s not in exported]
    assert missing == []


def test_libmte_loads_and_reports_version():
    lib = _native.load_mte()
    assert lib.mte_abi_version() == abi.MTE_ABI_VERSION
    assert lib.mte_strerror(abi.MTE_E_INSERT_FAILED).decode() == "MergeTree insert failed"


def test_create_rejects_bad_config_without_device():
    lib = _native.load_mte()
    ctx = C.c_void_p()
    cfg = abi.MteConfig(0, abi.MTE_MAX_KEYS + 1, 0, 0)
    assert lib.mte_create(C.byref(cfg), C.byref(ctx)) == abi.MTE_E_INVALID_ARG


LAYOUT_PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "mte.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(mte_op), sizeof(mte_prop), sizeof(mte_propset),
         sizeof(mte_config), sizeof(mte_doc_init), sizeof(mte_batch), sizeof(mte_stats), sizeof(mte_doc_view));
  printf("%zu %zu %zu %zu %zu %zu\n", offsetof(mte_op, type), offsetof(mte_op, client), offsetof(mte_op, flags),
         offsetof(mte_op, pos1), offsetof(mte_op, a), offsetof(mte_op, b));
  printf("%zu %zu %zu\n", offsetof(mte_batch, n_ops), offsetof(mte_batch, n_props), offsetof(mte_doc_view, n_segs));
  return 0;
}
"""


def test_struct_layouts_match_c(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(LAYOUT_PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    lines = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    sizes = [int(x) for x in lines[0].split()]
    assert sizes == [abi.OP_DTYPE.itemsize, abi.PROP_DTYPE.itemsize, abi.PROPSET_DTYPE.itemsize,
                     C.sizeof(abi.MteConfig), abi.DOC_INIT_DTYPE.itemsize, C.sizeof(abi.MteBatch),
                     C.sizeof(abi.MteStats), C.sizeof(abi.MteDocView)]
    offs = [int(x) for x in lines[1].split()]
    f = abi.OP_DTYPE.fields
    assert offs == [f["type"][1], f["client"][1], f["flags"][1], f["pos1"][1], f["a"][1], f["b"][1]]
    offs2 = [int(x) for x in lines[2].split()]
    assert offs2 == [abi.MteBatch.n_ops.offset, abi.MteBatch.n_props.offset, abi.MteDocView.n_segs.offset]


def test_no_cpu_fallback_in_product_path():
    """The product package never imports the oracle."""
    pkg = os.path.join(ROOT, "fluidframework_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".cpp", ".hip", ".h", ".js", ".cc")):
                text = open(os.path.join(dirpath, fn), encoding="utf-8").read()
                assert "import oracle" not in text and "from oracle" not in text, fn
                assert "liboracle" not in text and "oracle.h" not in text, fn


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a HIP device may be present")
def test_create_without_device_fails_loudly():
    lib = _native.load_mte()
    ctx = C.c_void_p()
    cfg = abi.MteConfig(0, 4, 0, 0)
    assert lib.mte_create(C.byref(cfg), C.byref(ctx)) == abi.MTE_E_NO_DEVICE
    from fluidframework_amd.engine import DeviceEngine
    with pytest.raises(abi.MergeTreeError):
        DeviceEngine(4)

