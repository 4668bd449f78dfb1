#!/usr/bin/env python3
"""Benchmark: sequenced merge-tree ops merged per second (BASELINE.json).

One step = replay of one batch (every doc x every op of the workload) from the
documents' initial state: mte_reset + mte_run (device-resident inputs: ops,
text and property tables are uploaded to HBM before the timed region).

N GPUs: one process per GPU (torch.distributed.run), documents sharded with no
data-path collective ("weak": every rank replays its own 10k-doc shard; doc
seeds are global doc indices).  After the timed region the per-doc digests are
all-gathered over RCCL for verification (the only collective).

Rank 0 prints one JSON line.  At N=1 it also times the CPU restatement
(oracle/, kind "port") on a bounded sample of the same workload and checks the
sampled docs' digests against the GPU's.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "sequenced ops merged/sec (node) at 10k docs×10k ops; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md "Chip-level parameters"
# PMC-measured HBM bytes of one replay launch (tools/pmc_traffic.py over two
# rocprofv3 --pmc passes); reported only for the libmte.so it was measured on
TRAFFIC_JSON = os.path.join(ROOT, "profiles", "r01", "pmc_traffic_config{cfg}.json")

WORKLOADS = {
    3: "config3: 10k docs x 10k ops/doc, insert/remove/annotate 1:1:1, 1/16 markers, 8 clients, R=64, "
       "legacy/new length calc 50/50",
    2: "config2: 1k docs x 1k ops/doc, insert/remove 1:1, 8 clients, R=32",
    4: "config4: 100k docs x 500 ops/doc, insert/remove/annotate, R=8",
    5: "config5: 64 docs x 2^20 preloaded one-unit segments (mte_load_segments), 262,144 ops/doc in 4 rounds "
       "of 65,536 concurrent ops (deep collab window, zamboni per round), insert/remove/annotate 1:1:1, "
       "ranges <= 16 units, 1/16 markers, 8 clients",
}


def host_threads():
    n = os.environ.get("OMP_NUM_THREADS")
    if n and n.isdigit():
        return max(1, int(n))
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except Exception:
        return max(1, min(16, os.cpu_count() or 1))


def pmc_traffic(config, n_docs, ops_per_doc):
    """(bytes per launch, source) from the committed PMC summary, or (None, why)."""
    import hashlib
    path = TRAFFIC_JSON.format(cfg=config)
    if not os.path.exists(path):
        return None, "no PMC summary for this config"
    preset_ok = (n_docs, ops_per_doc) == (None, None)
    if not preset_ok:
        return None, "non-default workload size"
    rec = json.load(open(path))
    lib = os.path.join(ROOT, "fluidframework_amd", "_lib", "libmte.so")
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    if rec.get("libmte_sha256") != sha:
        return None, "PMC summary was taken on a different libmte.so build"
    return rec["traffic_bytes_per_launch"], os.path.relpath(path, ROOT) + " (" + rec["correction"] + ")"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--docs", type=int, default=None, help="docs per GPU (default: the config's)")
    ap.add_argument("--ops", type=int, default=None, help="ops per doc (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stats", action="store_true",
                    help="keep the per-op counters on in the timed runs (default: off)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")

    from fluidframework_amd import dist as fdist
    from fluidframework_amd import gen
    from fluidframework_amd.engine import DeviceEngine

    preset = gen.PRESETS[args.config]
    n_docs = args.docs or preset["n_docs"]
    ops_per_doc = args.ops or preset["ops_per_doc"]
    threads = max(1, host_threads() // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", world))))

    t0 = time.time()
    stream = gen.generate(args.config, n_docs=n_docs, ops_per_doc=ops_per_doc,
                          doc_base=fdist.shard_doc_base(rank, n_docs), n_threads=threads)
    gen_s = time.time() - t0
    n_ops_rank = int(stream["batch"]["op_offsets"][-1])

    cap = gen.seg_capacity(args.config, stream["params"])
    eng = DeviceEngine(stream["n_keys"], device=local_rank, seg_capacity=cap)
    gen.load_stream(eng, stream)
    eng.submit(stream["batch"])

    def step():
        eng.reset()
        eng.run()

    # one accounting run (mte_stats: ops, segments scanned / written, property
    # writes, units -> the algorithmic bytes of SURVEY.md 8(d)); the timed runs
    # then go without the per-op counters (opt-in like the reference's measureOps)
    step()
    eng.sync()
    if (eng.statuses() != 0).any():
        raise SystemExit(f"rank {rank}: replay errors {np.unique(eng.statuses())}")
    stats = eng.stats()
    stats_digest = eng.digest()
    eng.set_stats(args.stats)
    for _ in range(args.warmup):
        step()
    eng.sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    eng.sync()
    kernel_ms = []
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
        # the library brackets its replay kernels with HIP events on its own
        # stream; read them after the step (waits only for that step)
        eng.sync()
        kernel_ms.append(eng.stats()["kernel_ms"])
    eng.sync()
    t_elapsed = time.perf_counter() - t_start
    barrier()

    elapsed = t_elapsed
    total_ops = n_ops_rank * world
    digest = eng.digest()
    if (eng.statuses() != 0).any() or not np.array_equal(digest, stats_digest):
        raise SystemExit(f"rank {rank}: timed runs disagree with the accounting run")
    fold = fdist.digest_fold(digest)
    if dist is not None:
        dev = f"cuda:{local_rank}"
        elapsed = fdist.max_over_ranks(dist, t_elapsed, device=dev)
        total_ops = fdist.sum_over_ranks(dist, n_ops_rank, device=dev)
        # the verification collective: every rank's per-doc digests over RCCL
        fold = fdist.digest_fold(fdist.gather_digests(dist, engine=eng, device=dev))

    ms_per_step = elapsed * 1000.0 / args.steps
    value = total_ops / (elapsed / args.steps)
    avg_kernel_ms = float(np.mean(kernel_ms)) if kernel_ms else None
    algo_bytes = stats["algo_bytes"]
    achieved_gbs = algo_bytes / (avg_kernel_ms * 1e-3) / 1e9 if avg_kernel_ms else None

    traffic, traffic_src = pmc_traffic(args.config, args.docs, args.ops)

    # end-to-end: host op records -> HBM (mte_submit, PCIe),
    # replay, per-doc digests back to the host; one untimed-by-the-contract pass
    eng.sync()
    t0 = time.perf_counter()
    eng.submit(stream["batch"])
    step()
    e2e_digest = eng.digest()
    e2e_s = time.perf_counter() - t0
    if not np.array_equal(e2e_digest, digest):
        raise SystemExit(f"rank {rank}: end-to-end pass disagrees with the timed runs")

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    cpu = None
    parity = None
    if world == 1 and not args.no_cpu_baseline:
        if stream.get("segs") is not None:
            cpu, parity = cpu_baseline_prefix(stream, cap, args.cpu_seconds, threads)
        else:
            cpu, parity = cpu_baseline(stream, digest, args.cpu_seconds)

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded MT19937 conflict-farm streams, fluidframework_amd/gen.py)",
        "config": {
            "workload": WORKLOADS.get(args.config, f"config{args.config}"),
            "docs_per_gpu": n_docs,
            "ops_per_doc": ops_per_doc,
            "ops_per_gpu": n_ops_rank,
            "parallelism": f"doc-sharded x{world} (no data-path collective)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (achieved_gbs / HBM_PEAK_GBS) if achieved_gbs else None,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "traffic_frac_of_algo": (traffic / algo_bytes) if traffic else None,
            "kernel": ("pair_kernel + big_kernel + " + ("chunk_kernel" if cap >= 8192 else "stream_kernel") +
                       " (replay passes 1-3), HIP events on the engine stream"),
            "algo_bytes_note": ("S_live of chunk-pass ops replaced by the chunk slots + summary entries they "
                                "scanned (SURVEY.md 8(d))" if cap >= 8192 else "SURVEY.md 8(d) B_op"),
            "counters_in_timed_runs": bool(args.stats),
            "kernel_ms": avg_kernel_ms,
            "algo_bytes_per_launch": algo_bytes,
            "algo_bytes_per_op": algo_bytes / max(1, stats["ops_applied"]),
        },
        "end_to_end": {"ops_per_s": n_ops_rank / e2e_s, "ms": e2e_s * 1e3,
                       "includes": "mte_submit (host->HBM op upload) + reset + replay + digest read-back, rank 0"},
        "cpu_baseline": cpu,
        "digest_fold": f"{fold:016x}",
        "parity_sample": parity,
        "gen_s": round(gen_s, 2),
    }
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(stream, gpu_digest, target_s):
    """Time the CPU restatement (oracle/, kind 'port') on a bounded doc sample."""
    from fluidframework_amd import gen
    from oracle import OracleEngine

    threads = host_threads()
    n_docs = len(stream["inits"])
    # calibrate on a small slice, then size the sample for ~target_s
    cal = max(threads, min(n_docs, 64))
    sub = gen.slice_docs(stream, 0, cal)
    o = OracleEngine(stream["n_keys"], threads=threads)
    o.load_docs(sub["inits"], sub["init_text"])
    t0 = time.perf_counter()
    o.apply_batch(sub["batch"])
    t_cal = time.perf_counter() - t0
    per_doc = t_cal / cal
    m = int(min(n_docs, max(cal, target_s / max(per_doc, 1e-9))))
    sub = gen.slice_docs(stream, 0, m)
    o = OracleEngine(stream["n_keys"], threads=threads)
    o.load_docs(sub["inits"], sub["init_text"])
    t0 = time.perf_counter()
    o.apply_batch(sub["batch"])
    dt = time.perf_counter() - t0
    ops = int(sub["batch"]["op_offsets"][-1])
    parity = bool(np.array_equal(o.digest(), gpu_digest[:m]) and (o.statuses() == 0).all())
    return ({"value": ops / dt, "unit": "ops/s", "cores": threads, "kind": "port",
             "sample": f"first {m} of {n_docs} docs (all their ops, {ops} ops), {dt:.1f} s, "
                       f"oracle/oracle.c flat restatement, {threads} pthreads"},
            {"docs": m, "digest_equal": parity})


def cpu_baseline_prefix(stream, cap, target_s, threads):
    """Long documents (config 5): the flat restatement costs O(S) per op, so the
    sample is the first k ops of `threads` docs (k sized for ~target_s); its
    digests are checked against a GPU replay of the same prefix."""
    from fluidframework_amd import gen
    from fluidframework_amd.engine import DeviceEngine
    from oracle import OracleEngine

    n_docs = len(stream["inits"])
    m = min(n_docs, threads)
    k = 64
    while True:
        sub = gen.prefix_ops(stream, m, k)
        o = OracleEngine(stream["n_keys"], threads=threads)
        gen.load_stream(o, sub)
        t0 = time.perf_counter()
        o.apply_batch(sub["batch"])
        dt = time.perf_counter() - t0
        if dt >= target_s / 4 or k >= int(np.diff(stream["batch"]["op_offsets"].astype(np.int64)).min()):
            break
        k = int(k * min(16.0, max(2.0, target_s / max(dt, 1e-3))))
    ops = int(sub["batch"]["op_offsets"][-1])
    d = DeviceEngine(stream["n_keys"], seg_capacity=cap)
    gen.load_stream(d, sub)
    d.apply_batch(sub["batch"])
    parity = bool(np.array_equal(o.digest(), d.digest()) and (o.statuses() == 0).all()
                  and (d.statuses() == 0).all())
    return ({"value": ops / dt, "unit": "ops/s", "cores": threads, "kind": "port",
             "sample": f"first {k} ops of the first {m} of {n_docs} docs ({ops} ops at ~2^20 segments/doc), "
                       f"{dt:.1f} s, oracle/oracle.c flat restatement, {threads} pthreads"},
            {"docs": m, "ops_per_doc": k, "digest_equal": parity, "checked_against": "GPU replay of the same prefix"})


if __name__ == "__main__":
    main()
