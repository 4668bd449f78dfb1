"""Time the tree pass alone on legacy-calc documents (config-3 shape).

--prof loads the profiling build (make -C fluidframework_amd/csrc prof) and
reports the tree pass's phase clocks per op (mte_tree.h MTE_TREE_PROF)."""
import argparse
import json
import os
import sys
import time

if "--prof" in sys.argv:
    os.environ["MTE_LIB_DIR"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                             "fluidframework_amd", "_lib", "prof")

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from fluidframework_amd import gen  # noqa: E402
from fluidframework_amd.engine import DeviceEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=2000)
ap.add_argument("--ops", type=int, default=10000)
ap.add_argument("--mode", type=int, default=1)
ap.add_argument("--lag", type=int, default=0)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--stats", action="store_true")
ap.add_argument("--prof", action="store_true")
args = ap.parse_args()
kw = dict(length_mode=args.mode)
if args.lag:
    kw["max_lag"] = args.lag
t0 = time.time()
s = gen.generate(3, n_docs=args.docs, ops_per_doc=args.ops, **kw)
e = DeviceEngine(s["n_keys"])
gen.load_stream(e, s)
e.submit(s["batch"])
e.set_stats(args.stats or args.prof)
ms = []
for r in range(args.reps):
    e.reset()
    e.run()
    e.sync()
    ms.append(e.stats()["kernel_ms"])
st = e.stats()
ops = int(s["batch"]["op_offsets"][-1])
if args.prof:
    n = int(s["batch"]["op_offsets"][-1])
    st["phase_us_per_op"] = {k: st[f] / n / 100.0 for k, f in (("lengths+boundary", "segs_scanned"),
                             ("insert/marks+lru", "segs_written"), ("zamboni", "prop_writes"),
                             ("op total", "units_inserted"))}
print(json.dumps({"docs": args.docs, "ops": ops, "kernel_ms": ms, "gops": ops / min(ms) / 1e6, "stats": st,
                  "gen_s": time.time() - t0}))
