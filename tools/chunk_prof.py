#!/usr/bin/env python3
"""Phase clocks of the chunked big-document pass (config 5), from a
diagnostic build with -DMTE_CH_PROF=1 (mte_chunk.h writes per-document phase
cycle totals into the stats slots):
  python3 tools/chunk_prof.py build_var/chP/libmte.so [n_docs] [ops_per_doc]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fluidframework_amd import _native  # noqa: E402

LIB = os.path.abspath(sys.argv[1])
_orig = _native.lib_path
_native.lib_path = lambda name: LIB if name == "libmte.so" else _orig(name)

from fluidframework_amd import gen  # noqa: E402
from fluidframework_amd.engine import DeviceEngine  # noqa: E402

nd = int(sys.argv[2]) if len(sys.argv) > 2 else 64
nops = int(sys.argv[3]) if len(sys.argv) > 3 else None
st = gen.generate(5, n_docs=nd, ops_per_doc=nops)
cap = gen.seg_capacity(5, st["params"])
e = DeviceEngine(st["n_keys"], seg_capacity=cap)
gen.load_stream(e, st)
e.submit(st["batch"])
e.set_stats(True)
for _ in range(2):
    e.reset()
    e.run()
    e.sync()
s = e.stats()
o = s["ops_applied"]
# slot -> mte_stats field: 0 ops, 1 find, 2 load, 3 step, 4 store, 5 pass (max), 6 rebuild, 7 relayout
find, load, step, store = s["segs_scanned"], s["segs_written"], s["prop_writes"], s["units_inserted"]
reloc = s["chunk_scanned"]
canon = find + reloc + (32.0 * o + 20.0 * load + 4.0 * step + 2.0 * store - s["algo_bytes"]) / 20.0
out = {"docs": nd, "ops": o, "kernel_ms": s["kernel_ms"], "pass_cycles_max_doc": s["max_segs"],
       "cycles_per_op": {"find": find / o, "load": load / o, "step": step / o, "store": store / o,
                         "rebuild": canon / o, "relayout": reloc / o},
       "pass_cycles_per_op": s["max_segs"] / (o / nd)}
print(json.dumps(out))
