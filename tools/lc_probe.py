import sys, json, time
sys.path.insert(0, ".")
import numpy as np
import bench
for n in (614, 2456, 10438):
    r = bench.local_client_leg(n, 0, 3, 16)
    print(json.dumps({"docs": r["docs"], "ops": r["ops"], "kernel_ms": r["kernel_ms"], "ops_per_s": r["ops_per_s"], "eq": r["digest_equal_restatement"]}), flush=True)
