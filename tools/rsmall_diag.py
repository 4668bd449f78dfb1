"""Round phases for small batches (mte_rsmall.h): where each document stopped.
Run with MTE_WAVE_CLOCK set (diagnostics): the kernel leaves its run counts
in the statistics slots."""
import json
import sys

sys.path.insert(0, ".")
from fluidframework_amd import gen  # noqa: E402
from fluidframework_amd.engine import DeviceEngine  # noqa: E402

s = gen.generate(3, n_docs=int(sys.argv[1]) if len(sys.argv) > 1 else 1250, ops_per_doc=10000, round_sync=True)
d = DeviceEngine(s["n_keys"])
d.set_stats(False)
gen.load_stream(d, s)
d.apply_batch(s["batch"])
st = d.stats()
r = int(st["prop_writes"])
print(json.dumps({"ops_by_rsmall": int(st["ops_applied"]), "parallel_runs": int(st["segs_scanned"]),
                  "op_after_op_runs": int(st["segs_written"]), "stop_not_a_run": r & 0xFFFFF,
                  "stop_fallback_too_big": (r >> 20) & 0xFFFFF, "stop_grew": r >> 40,
                  "ops_total": int(s["batch"]["op_offsets"][-1])}))
