"""The bench's local-client side line alone, under several MTE_HTREE_LDS
budgets (bytes of LDS a document of the HBM tree pass may hold; 0 = HBM only).
--prof: the profiling build (make -C fluidframework_amd/csrc prof) and the HBM
tree pass's phase clocks (mte_htree.h MTE_HTREE_PROF), summed over documents:
wave-microseconds per record in each phase.
Usage: python tools/local_leg.py [--prof] [budget ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PROF = "--prof" in sys.argv
if PROF:
    os.environ["MTE_LIB_DIR"] = os.path.join(ROOT, "fluidframework_amd", "_lib", "prof")
PHASES = ["insert", "range", "ack", "zamboni", "rollback_regen", "refs_relpos", "record", "records"]


def main():
    import bench
    budgets = [int(x) for x in sys.argv[1:] if x != "--prof"] or [0, 24576]
    for b in budgets:
        os.environ["MTE_HTREE_LDS"] = str(b)
        pf = os.path.join(ROOT, "gpurun_out", f"htree_prof_{b}.txt")
        if PROF:
            os.makedirs(os.path.dirname(pf), exist_ok=True)
            if os.path.exists(pf):
                os.remove(pf)
            os.environ["MTE_HTREE_PROF"] = pf
        r = bench.local_client_leg(10000, 0, 3, bench.host_threads())
        out = {"htree_lds": b, **{k: r[k] for k in ("ms_per_step", "kernel_ms", "first_run_kernel_ms", "ops_per_s",
                                                    "digest_equal_restatement")}}
        if PROF and os.path.exists(pf):
            rows = [list(map(int, ln.split())) for ln in open(pf) if ln.strip()]
            last = [r_ for r_ in rows if r_[7] > 0][-1]  # one timed run
            n = max(1, last[7])
            out["us_per_record"] = {PHASES[q]: last[q] / 100.0 / n for q in range(7)}
            out["records"] = n
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
