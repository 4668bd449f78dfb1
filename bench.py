#!/usr/bin/env python3
"""Benchmark: sequenced merge-tree ops merged per second (BASELINE.json).

One step = replay of one batch (every doc x every op of the workload) from the
documents' initial state: mte_reset + mte_run (device-resident inputs: ops,
text and property tables are uploaded to HBM before the timed region).

N GPUs: one process per GPU -- launched by torch.distributed.run, which only
sets RANK / WORLD_SIZE (nothing here imports torch), or, run directly with
--gpus N, by bench.py itself (fluidframework_amd/launch.py) -- documents
sharded with no data-path collective.  Default "strong": the config's documents (BASELINE: 10k
per node) assigned to ranks by expected work, longest first onto the least
loaded rank (fluidframework_amd/dist.py, the Node host's shardByWork rule; doc
seeds are global doc indices); at N > 1 a "weak" side line replays the
config's document count on every rank.  After the timed region the per-doc
digests are all-gathered over RCCL (libmte.so mte_comm_*, the only
collective) and put back in global order for verification.  If RCCL cannot
start, the job exits non-zero.

Legacy length-calc documents of the round-model workloads are declared
round-synchronous (MTE_DOC_ROUND_SYNC: flat passes, declaration checked per
batch); the "tree_placement" side line replays the same job with them on the
tree pass (the reference's B+tree placement) and must give the same digests.

Rank 0 prints one JSON line.  At N=1 it also times the CPU restatement
(oracle/, kind "port") on a bounded sample of the same workload and checks the
sampled docs' digests against the GPU's; the reference merge-tree's own CPU
rate (measured in the build container, tools/ref_baseline.py) is attached.
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
TRAFFIC_JSON = os.path.join(ROOT, "profiles", "r06", "final", "pmc_traffic_config{cfg}.json")

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
    from fluidframework_amd import _native
    sha = hashlib.sha256(open(_native.lib_path("libmte.so"), "rb").read()).hexdigest()
    if rec.get("libmte_sha256") != sha:
        return None, "PMC summary was taken on a different libmte.so build"
    return rec["traffic_bytes_per_launch"], os.path.relpath(path, ROOT) + " (" + rec["correction"] + ")"


def library_build():
    """Which libmte.so ran: its sha256 and file time (a rebuild on the box shows as a
    new time and, if the sources changed, a new hash)."""
    import hashlib
    from fluidframework_amd import _native
    p = _native.lib_path("libmte.so")
    st = os.stat(p)
    # the library reports the digest of the sources it was compiled from
    # (mte_build_info, include/mte.h); the same digest of the sources beside it
    csrc = os.path.join(ROOT, "fluidframework_amd", "csrc")
    names = sorted(f for f in os.listdir(csrc) if f.startswith("mte_") and f.endswith((".h", ".hip")))
    h = hashlib.sha256()
    for f in names + [os.path.join("..", "..", "include", "mte.h")]:
        h.update(open(os.path.join(csrc, f), "rb").read())
    info = _native.load_mte().mte_build_info().decode()
    src = info.split()[0].split("=", 1)[1]
    return {"libmte_sha256": hashlib.sha256(open(p, "rb").read()).hexdigest(),
            "libmte_mtime_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(st.st_mtime)),
            "libmte_path": os.path.relpath(p, ROOT),
            "build_info": info, "sources_sha16": h.hexdigest()[:16],
            "built_from_these_sources": src == h.hexdigest()[:16]}


REF_BASELINE_JSON = os.path.join(ROOT, "profiles", "r02", "ref_cpu_baseline.json")


def reference_cpu_baseline(config):
    """The reference merge-tree itself timed on CPU (tools/ref_baseline.py, run in
    the build container: the reference does not travel to the GPU box), or None."""
    if not os.path.exists(REF_BASELINE_JSON):
        return None
    rec = json.load(open(REF_BASELINE_JSON)).get(f"config{config}")
    return rec


class NodeComm:
    """Barrier, scalar reductions and the digest gather of an N-GPU job: RCCL
    through libmte.so's mte_comm_* on a context of its own (fluidframework_amd/
    comm.py bootstraps the unique id).  No fallback: a job whose communicator
    cannot start exits non-zero."""

    def __init__(self, rank, world, local_rank):
        from fluidframework_amd import comm as fcomm
        from fluidframework_amd.engine import DeviceEngine
        self.rank, self.world = rank, world
        try:
            self.eng = DeviceEngine(0, device=local_rank)
            fcomm.join(self.eng, rank, world)
        except Exception as e:  # pragma: no cover - hardware dependent
            raise SystemExit(f"rank {rank}: RCCL communicator (mte_comm_init) failed: {e}")
        self.kind = "rccl via libmte.so mte_comm_* (no torch)"

    def barrier(self):
        self.eng.comm_barrier()

    def max(self, v):
        return self.eng.comm_allreduce(float(v), "max")

    def sum(self, v):
        return self.eng.comm_allreduce(float(v), "sum")

    def gather_digests(self, eng, docs_per_rank):
        """Every rank's digests, rank-major (world, docs_per_rank, 4)."""
        eng.comm_share(self.eng)
        g = eng.comm_gather_digests(docs_per_rank)
        eng.comm_destroy()  # drops eng's reference; the communicator stays with self.eng
        return g

    def close(self):
        self.eng.comm_destroy()


def run_engine(stream, cap, device, steps, warmup, stats_on, barrier=lambda: None):
    """Load + submit a stream, one accounting run (mte_stats), warmup, then
    `steps` timed steps (reset + run) bracketed by barrier + sync.  Returns a
    dict with the engine, elapsed seconds, kernel ms per step, stats, digest."""
    from fluidframework_amd import gen
    from fluidframework_amd.engine import DeviceEngine

    eng = DeviceEngine(stream["n_keys"], device=device, seg_capacity=cap)
    if stream.get("event_capacity"):
        eng.set_event_capacity(stream["event_capacity"])
    gen.load_stream(eng, stream)
    eng.submit(stream["batch"])

    def step():
        eng.reset()
        eng.run()

    # the first run of a fresh context, counters off: pass 1's issue priority
    # has no schedule estimate from an earlier run yet (MTE_FAIR_PRIO 4)
    eng.set_stats(False)
    step()
    eng.sync()
    first_ms = eng.stats()["kernel_ms"]
    # one accounting run (mte_stats: ops, segments scanned / written, property
    # writes, units -> the algorithmic bytes of SURVEY.md 8(d)); the timed runs
    # then go without the per-op counters (opt-in like the reference's measureOps)
    eng.set_stats(True)
    step()
    eng.sync()
    if (eng.statuses() != 0).any():
        raise SystemExit(f"replay errors {np.unique(eng.statuses())}")
    stats = eng.stats()
    stats_digest = eng.digest()
    eng.set_stats(stats_on)
    for _ in range(warmup):
        step()
    eng.sync()
    barrier()
    eng.sync()
    kernel_ms = []
    t_start = time.perf_counter()
    round_bytes = []
    for _ in range(steps):
        step()
        # the library brackets its replay kernels with HIP events on its own
        # stream; read them after the step (waits only for that step)
        eng.sync()
        st = eng.stats()
        kernel_ms.append(st["kernel_ms"])
        round_bytes.append(st.get("round_bytes", 0.0))
    eng.sync()
    t_elapsed = time.perf_counter() - t_start
    barrier()
    digest = eng.digest()
    if (eng.statuses() != 0).any() or not np.array_equal(digest, stats_digest):
        raise SystemExit("timed runs disagree with the accounting run")
    return {"eng": eng, "elapsed": t_elapsed, "kernel_ms": kernel_ms, "stats": stats, "digest": digest,
            "first_ms": first_ms, "round_bytes": float(np.mean(round_bytes)) if round_bytes else 0.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--docs", type=int, default=None, help="docs in the whole job (default: the config's)")
    ap.add_argument("--ops", type=int, default=None, help="ops per doc (default: the config's)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="strong: the config's documents split over the ranks (BASELINE: 10k docs per node); "
                         "weak: every rank replays that many documents")
    ap.add_argument("--placement", choices=["round_sync", "tree"], default="round_sync",
                    help="legacy-calc documents: declared round-synchronous (MTE_DOC_ROUND_SYNC, flat passes, "
                         "checked per batch) or on the tree pass")
    ap.add_argument("--no-tree-leg", action="store_true", help="skip the tree-placement side measurement")
    ap.add_argument("--no-weak-leg", action="store_true", help="skip the weak-scaling side measurement (N > 1)")
    ap.add_argument("--no-node-leg", action="store_true", help="skip the Node host end-to-end measurement")
    ap.add_argument("--no-local-leg", action="store_true",
                    help="skip the local-client side measurement (reference farms: local ops, acks, rollback, "
                         "reconnect, delta events)")
    ap.add_argument("--local-docs", type=int, default=10000, help="documents in the local-client side measurement")
    ap.add_argument("--node-docs", type=int, default=100, help="documents in the Node host sample")
    ap.add_argument("--node-sharded-docs", type=int, default=1000,
                    help="documents in the Node host sample with parallel packing (ShardedHost)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stats", action="store_true",
                    help="keep the per-op counters on in the timed runs (default: off)")
    args = ap.parse_args()

    # run directly with --gpus N > 1: start the N ranks here (one process per
    # GPU, the rank variables torch.distributed.run would set), before this
    # process touches a GPU; the children run this same main()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        from fluidframework_amd import launch
        raise SystemExit(launch.run_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE {world} != --gpus {args.gpus}")

    from fluidframework_amd import dist as fdist
    from fluidframework_amd import gen
    from fluidframework_amd.engine import DeviceEngine

    # node level: RCCL through libmte.so (mte_comm_*), one communicator per
    # process on a context of its own
    node = None
    if world > 1:
        node = NodeComm(rank, world, local_rank)

    preset = gen.PRESETS[args.config]
    docs_job = args.docs or preset["n_docs"]
    ops_per_doc = args.ops or preset["ops_per_doc"]
    threads = max(1, host_threads() // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", world))))

    # strong scaling: the job's documents onto ranks by expected work (every
    # document of a preset has the same op count and expected live segments,
    # so LPT deals them out round-robin); weak: rank r replays global documents
    # [r * docs_job, (r + 1) * docs_job)
    rank_of = fdist.shard_by_work(np.full(docs_job, float(ops_per_doc)), world)

    def shard(scaling):
        """Global indices of this rank's documents."""
        if scaling == "weak":
            return np.arange(rank * docs_job, (rank + 1) * docs_job, dtype=np.uint32)
        return fdist.rank_docs(rank_of, rank)

    def make_stream(scaling, placement):
        kw = {"round_sync": True} if placement == "round_sync" and not preset.get("max_lag") else {}
        return gen.generate(args.config, ops_per_doc=ops_per_doc, doc_ids=shard(scaling), n_threads=threads, **kw)

    def barrier():
        if node is not None:
            node.barrier()

    t0 = time.time()
    stream = make_stream(args.scaling, args.placement)
    gen_s = time.time() - t0
    n_ops_rank = int(stream["batch"]["op_offsets"][-1])
    cap = gen.seg_capacity(args.config, stream["params"])
    r = run_engine(stream, cap, local_rank, args.steps, args.warmup, args.stats, barrier)
    eng, stats, digest = r["eng"], r["stats"], r["digest"]
    elapsed = r["elapsed"]
    first_ms = r["first_ms"]
    total_ops = n_ops_rank * world
    fold = fdist.digest_fold(digest)
    if node is not None:
        elapsed = node.max(r["elapsed"])
        total_ops = int(node.sum(n_ops_rank))
        # the verification collective: every rank's per-doc digests over RCCL,
        # back in global document order
        if args.scaling == "weak":
            fold = fdist.digest_fold(node.gather_digests(eng, docs_job))
        else:
            g = node.gather_digests(eng, fdist.docs_per_rank(rank_of, world))
            fold = fdist.digest_fold(fdist.unshard_digests(g, rank_of, world))

    ms_per_step = elapsed * 1000.0 / args.steps
    value = total_ops / (elapsed / args.steps)
    avg_kernel_ms = float(np.mean(r["kernel_ms"])) if r["kernel_ms"] else None
    algo_bytes = stats["algo_bytes"]
    # the chunked pass's timed runs take the round phases, whose own bytes the
    # library counts in every run (mte_stats.round_bytes); the statistics run
    # replays op after op, so its algo_bytes describe that pass, not the timed one
    round_bytes = r.get("round_bytes", 0.0)
    timed_bytes = round_bytes if cap >= 8192 and round_bytes > 0 else algo_bytes
    achieved_gbs = timed_bytes / (avg_kernel_ms * 1e-3) / 1e9 if avg_kernel_ms else None

    traffic, traffic_src = pmc_traffic(args.config, args.docs, args.ops)

    # end-to-end: host op records -> HBM (mte_submit, PCIe),
    # replay, per-doc digests back to the host; one untimed-by-the-contract pass
    eng.sync()
    t0 = time.perf_counter()
    eng.submit(stream["batch"])
    eng.reset()
    eng.run()
    e2e_digest = eng.digest()
    e2e_s = time.perf_counter() - t0
    if not np.array_equal(e2e_digest, digest):
        raise SystemExit(f"rank {rank}: end-to-end pass disagrees with the timed runs")
    del eng, r

    # side measurement: the same job with every legacy-calc document on the
    # tree pass (no round-synchronous declaration), digest-checked
    tree_leg = None
    if args.placement == "round_sync" and not args.no_tree_leg and world == 1:
        ts = make_stream(args.scaling, "tree")
        rt = run_engine(ts, cap, local_rank, max(1, args.steps // 2), 1, False)
        if not np.array_equal(rt["digest"], digest):
            raise SystemExit("tree placement disagrees with the round-synchronous replay")
        tms = rt["elapsed"] * 1000.0 / max(1, args.steps // 2)
        tree_leg = {"ms_per_step": tms, "ops_per_s": n_ops_rank / (tms * 1e-3),
                    "kernel_ms": float(np.mean(rt["kernel_ms"])), "first_run_kernel_ms": rt["first_ms"],
                    "digest_equal": True,
                    "note": "legacy-calc documents on the tree pass (reference B+tree placement, mte_tree.h)"}
        del rt, ts

    # side measurement: documents with a local client (the 8(f) rows: local ops
    # + acks, rollback, reconnect, delta events) on the HBM-streamed pass
    local_leg = None
    if not args.no_local_leg and world == 1:
        local_leg = local_client_leg(args.local_docs, local_rank, max(1, args.steps // 2), threads)

    # side measurement at N > 1: weak scaling (every rank the config's docs)
    weak_leg = None
    if world > 1 and args.scaling == "strong" and not args.no_weak_leg:
        ws = make_stream("weak", args.placement)
        rw = run_engine(ws, cap, local_rank, args.steps, 1, False, barrier)
        w_el = node.max(rw["elapsed"])
        w_ops = int(node.sum(int(ws["batch"]["op_offsets"][-1])))
        weak_leg = {"value": w_ops / (w_el / args.steps), "ms_per_step": w_el * 1000.0 / args.steps,
                    "docs_per_gpu": int(len(ws["inits"])), "scaling": "weak"}
        del rw, ws

    if rank != 0:
        if node is not None:
            node.close()
        return

    node_e2e = None
    if world == 1 and not args.no_node_leg and stream.get("segs") is None:
        node_e2e = node_end_to_end(stream, digest, args.node_docs)
        node_e2e["sharded"] = node_sharded(stream, args.node_sharded_docs, host_threads())

    cpu = None
    parity = None
    if world == 1 and not args.no_cpu_baseline:
        if stream.get("segs") is not None:
            cpu, parity = cpu_baseline(stream, digest, args.cpu_seconds, tree="chunked")
        else:
            cpu, parity = cpu_baseline(stream, digest, args.cpu_seconds)
    ref_cpu = reference_cpu_baseline(args.config)

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded MT19937 conflict-farm streams, fluidframework_amd/gen.py)",
        "config": {
            "workload": WORKLOADS.get(args.config, f"config{args.config}"),
            "docs_total": docs_job if args.scaling == "strong" else docs_job * world,
            "docs_per_gpu": int(len(stream["inits"])),
            "ops_per_doc": ops_per_doc,
            "ops_per_gpu": n_ops_rank,
            "placement": ("legacy-calc docs declared round-synchronous (MTE_DOC_ROUND_SYNC): flat passes, "
                          "declaration checked per batch" if args.placement == "round_sync" else
                          "legacy-calc docs on the tree pass (reference B+tree placement)"),
            "parallelism": f"doc-sharded x{world} by expected work (LPT), no data-path collective",
            "collective": node.kind if node is not None else None,
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
            "kernel": ("tree + pair + big + " + ("chunk" if cap >= 8192 else "stream") +
                       " replay passes, HIP events on the engine stream"),
            "algo_bytes_note": ("the round phases' own bytes, counted by the library in the timed runs "
                                "(mte_stats.round_bytes: records, planes re-laid out / applied / gathered, sub-op "
                                "lists); algo_bytes_op_after_op = SURVEY.md 8(d) with S_live replaced by the chunk "
                                "slots + summary entries the op-after-op chunk pass scans"
                                if cap >= 8192 and round_bytes > 0 else "SURVEY.md 8(d) B_op"),
            "counters_in_timed_runs": bool(args.stats),
            "kernel_ms": avg_kernel_ms,
            "first_run_kernel_ms": first_ms,
            "algo_bytes_per_launch": timed_bytes,
            "algo_bytes_per_op": timed_bytes / max(1, stats["ops_applied"]),
            "algo_bytes_op_after_op": algo_bytes if timed_bytes != algo_bytes else None,
        },
        "end_to_end": {"ops_per_s": n_ops_rank / e2e_s, "ms": e2e_s * 1e3,
                       "includes": "mte_submit (host->HBM op upload) + reset + replay + digest read-back, rank 0"},
        "end_to_end_node": node_e2e,
        "tree_placement": tree_leg,
        "local_client": local_leg,
        "weak_scaling": weak_leg,
        "cpu_baseline": cpu,
        "cpu_baseline_reference": ref_cpu,
        "digest_fold": f"{fold:016x}",
        "parity_sample": parity,
        "gen_s": round(gen_s, 2),
        "build": library_build(),
    }
    # a line measured on a library built from other sources (a stale or a
    # diagnostics build) is marked, never passed off as the product's
    out["valid"] = bool(out["build"]["built_from_these_sources"])
    if not out["valid"]:
        out["invalid_reason"] = "libmte.so was not built from the sources beside it (mte_build_info)"
    print(json.dumps(out), flush=True)
    if node is not None:
        node.close()


LOCAL_KEYS = 4  # the farms' property keys: client, bold, color, markerId


def local_client_stream(n_docs):
    """Documents whose own client sends, at bench scale: every client of the
    farms the reference itself ran (tests/golden/farm_vectors.json.gz: local ops,
    acks, lagging remote ops, rollbacks; reconnect_vectors.json.gz: ops held
    offline and regeneratePendingOp) as one MTE_DOC_LOCAL_CLIENT | MTE_DOC_EVENTS
    document with all its events in one batch, the set of documents repeated
    to n_docs (copies share the property tables; text offsets shift).  Returns
    (stream, base stream of the distinct documents, copies)."""
    import gzip

    from fluidframework_amd.abi import DOC_EVENTS, DOC_LOCAL_CLIENT, DOC_NEW_LENGTH_CALC, F_MARKER, OP_INSERT
    from fluidframework_amd.packing import BatchBuilder, DocClients, Interner
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fixtures_util import as_msg, doc_inits

    sets = []
    for name in ("farm_vectors.json.gz", "reconnect_vectors.json.gz"):
        with gzip.open(os.path.join(ROOT, "tests", "golden", name), "rt", encoding="utf-8") as fh:
            sets += json.load(fh)["sets"]
    layout = [(si, ci) for si, st in enumerate(sets) for ci in range(len(st["names"]))]
    inits, text = doc_inits([sets[si]["initialText"] for si, _ in layout],
                            flags=DOC_NEW_LENGTH_CALC | DOC_LOCAL_CLIENT | DOC_EVENTS)
    it = Interner(LOCAL_KEYS)
    bb = BatchBuilder(len(layout), it)
    for d, (si, ci) in enumerate(layout):
        st, cl = sets[si], DocClients(sets[si]["names"][ci], local=True)
        for kind, li in st["events"][ci]:
            if kind == "R":
                bb.add_local(d, cl, li)
                bb.add_rollback(d, cl)
            elif kind == "H":
                bb.add_local(d, cl, li)
            elif kind == "G":
                bb.add_regen(d, cl)
            elif kind == "L":
                bb.add_local(d, cl, as_msg(st["log"][li])["contents"])
            else:
                bb.add_message(d, cl, as_msg(st["log"][li]))
    base_batch = bb.build()
    base = {"n_keys": LOCAL_KEYS, "inits": inits, "init_text": text, "batch": base_batch, "event_capacity": 64}
    nb = len(layout)
    copies = max(1, (n_docs + nb - 1) // nb)
    ops, offs = base_batch["ops"], base_batch["op_offsets"].astype(np.int64)
    tu, iu = len(base_batch["text"]), len(text)
    shifted = []
    txt_rec = (ops["type"] == OP_INSERT) & ((ops["flags"] & F_MARKER) == 0)
    for c in range(copies):
        o = ops.copy()
        o["a"][txt_rec] += np.uint32(c * tu)
        shifted.append(o)
    all_ops = np.concatenate(shifted)
    cnt = offs[1:] - offs[:-1]
    # document order: copy-major, each copy's documents in base order
    all_offs = np.zeros(nb * copies + 1, np.uint64)
    all_offs[1:] = np.cumsum(np.tile(cnt, copies))
    # each copy's records are contiguous in all_ops in base-doc order: the same order
    all_inits = np.concatenate([inits] * copies)
    for c in range(copies):
        all_inits["text_off"][c * nb:(c + 1) * nb] += np.uint32(c * iu)
    batch = dict(base_batch, ops=all_ops, op_offsets=all_offs, text=np.tile(base_batch["text"], copies))
    stream = {"n_keys": LOCAL_KEYS, "inits": all_inits, "init_text": np.tile(text, copies), "batch": batch,
              "event_capacity": 64}
    return stream, base, copies


def local_client_leg(n_docs, device, steps, threads):
    """The local-client side line: replay rate of local_client_stream on the
    GPU (HIP-event kernel time, algorithmic bytes as the headline's), every
    copy's digest equal to the tree restatement's (oracle/titems.c, the HBM
    tree pass's specification) for its base document, and the restatement's
    own rate on the base documents (kind "port")."""
    from oracle import OracleEngine
    t0 = time.time()
    stream, base, copies = local_client_stream(n_docs)
    build_s = time.time() - t0
    r = run_engine(stream, 0, device, steps, 1, False)
    nb = len(base["inits"])
    n_ops = int(stream["batch"]["op_offsets"][-1])
    o = OracleEngine(LOCAL_KEYS, threads=threads, tree="items")
    o.lib.oti_set_limit(o.ctx, 1 << 20)
    o.set_event_capacity(base["event_capacity"])
    o.load_docs(base["inits"], base["init_text"])
    tc = time.perf_counter()
    o.apply_batch(base["batch"])
    cpu_s = time.perf_counter() - tc
    od = o.digest()
    equal = bool((o.statuses() == 0).all() and all(np.array_equal(r["digest"][c * nb:(c + 1) * nb], od)
                                                   for c in range(copies)))
    kms = float(np.mean(r["kernel_ms"]))
    gbs = r["stats"]["algo_bytes"] / (kms * 1e-3) / 1e9
    ms = r["elapsed"] * 1000.0 / steps
    base_ops = int(base["batch"]["op_offsets"][-1])
    return {"docs": int(len(stream["inits"])), "distinct_docs": nb, "ops": n_ops, "ms_per_step": ms,
            "ops_per_s": n_ops / (ms * 1e-3), "kernel_ms": kms, "first_run_kernel_ms": r["first_ms"],
            "achieved_gbs": gbs, "frac": gbs / HBM_PEAK_GBS, "digest_equal_restatement": equal,
            "cpu_port": {"ops_per_s": base_ops / cpu_s, "cores": threads, "ops": base_ops},
            "build_s": round(build_s, 1),
            "note": ("every client of the 76 farm + 35 reconnect farm sets the reference ran (local ops, acks, "
                     "rollbacks, regeneratePendingOp, lagging remote ops), MTE_DOC_LOCAL_CLIENT | MTE_DOC_EVENTS, "
                     "repeated to the doc count; HBM tree pass (mte_htree.h)")}


def node_end_to_end(stream, gpu_digest, n_docs):
    """The Node host path on a bounded sample (fluidframework_amd/node/bench_e2e.js):
    message objects -> BatchClient.applyMsg (JS packing) -> flush (mte_submit +
    mte_run + mte_sync over N-API) -> digests, checked against the GPU run."""
    import shutil
    import subprocess

    from fluidframework_amd import gen, messages
    node = shutil.which("node")
    if node is None:
        return {"skipped": "node not installed"}
    m = min(n_docs, len(stream["inits"]))
    docs = messages.stream_docs(stream, 0, m, segs=False)
    t0 = time.perf_counter()
    r = subprocess.run([node, "--max-old-space-size=8192", os.path.join(ROOT, "fluidframework_amd", "node",
                                                                         "bench_e2e.js")],
                       input=json.dumps({"docs": docs, "reps": 3}), capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": r.stderr[-2000:]}
    j = json.loads(r.stdout.strip().splitlines()[-1])
    # the Node host interns property values in its own order, so digests are
    # not comparable across hosts: the texts are checked against the
    # restatement's instead
    from oracle import OracleEngine
    sub = gen.slice_docs(stream, 0, m)
    o = OracleEngine(stream["n_keys"], threads=4)
    gen.load_stream(o, sub)
    o.apply_batch(sub["batch"])
    want = [o.read_doc(d)["text"] for d in range(m)]
    b = j["best"]
    return {"ops_per_s": j["ops_per_s"], "ms": b["pack_ms"] + b["flush_ms"], "pack_ms": b["pack_ms"],
            "flush_ms": b["flush_ms"], "docs": m, "ops": j["ops"], "errors": b["errors"],
            "texts_equal_restatement": want == j["texts"],
            "pipelined": j["pipelined"],
            "includes": "BatchClient.applyMsg (JS packing) + flush (N-API mte_submit upload + mte_run + mte_sync); "
                        "message objects built before the clock; 'pipelined': the messages in 4 slices, each "
                        "flushed as packed (packing + upload of slice i+1 overlap the replay of slice i)",
            "wall_s": round(time.perf_counter() - t0, 1)}


def write_stream_dir(stream, d, n_docs):
    """Docs [0, n_docs) of a generated stream as the files stream_source.js reads
    (fluidframework_amd/node/stream_source.js)."""
    from fluidframework_amd import gen
    from fluidframework_amd.packing import units_to_str
    os.makedirs(d, exist_ok=True)
    b = stream["batch"]
    o = np.asarray(b["op_offsets"], np.uint64)[: n_docs + 1]
    o.tofile(os.path.join(d, "offsets.u64"))
    np.asarray(b["ops"])[: int(o[-1])].tofile(os.path.join(d, "ops.bin"))
    np.asarray(b["text"], np.uint16).tofile(os.path.join(d, "text.u16"))
    np.asarray(b["propsets"]).tofile(os.path.join(d, "propsets.u32"))
    np.asarray(b["props"]).tofile(os.path.join(d, "props.u32"))
    vids = sorted(set(int(x) for x in np.asarray(b["props"])["value"]) - {0})
    with open(os.path.join(d, "tables.json"), "w") as fh:
        json.dump({"keys": gen.KEY_NAMES, "values": {str(v): gen.value_json(v) for v in vids}}, fh)
    init = stream["init_text"]
    inits = []
    for k in range(n_docs):
        it = stream["inits"][k]
        inits.append({"text": units_to_str(init[int(it["text_off"]):int(it["text_off"]) + int(it["text_len"])]),
                      "newCalc": bool(int(it["flags"]) & 1), "roundSync": bool(int(it["flags"]) & 2),
                      "nMsgs": int(o[k + 1] - o[k])})
    with open(os.path.join(d, "inits.json"), "w") as fh:
        json.dump(inits, fh)


def node_sharded(stream, n_docs, workers):
    """The Node host with parallel packing (fluidframework_amd/node/bench_shards.js):
    ShardedHost workers, one per host thread, pack their document shards'
    messages into one shared batch; submit + replay in 4 slices, packing slice
    i + 1 while slice i replays.  Texts of a sample checked against the
    restatement."""
    import shutil
    import subprocess
    import tempfile

    from fluidframework_amd import gen
    node = shutil.which("node")
    if node is None:
        return {"skipped": "node not installed"}
    m = min(n_docs, len(stream["inits"]))
    d = tempfile.mkdtemp(prefix="mte_stream_")
    t0 = time.perf_counter()
    try:
        write_stream_dir(stream, d, m)
        r = subprocess.run([node, "--max-old-space-size=16384", os.path.join(ROOT, "fluidframework_amd", "node",
                                                                          "bench_shards.js"), d, str(workers), "4"],
                           capture_output=True, text=True, timeout=900)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    if r.returncode != 0:
        return {"error": r.stderr[-2000:]}
    j = json.loads(r.stdout.strip().splitlines()[-1])
    from oracle import OracleEngine
    k = len(j.get("texts", []))
    sub = gen.slice_docs(stream, 0, k)
    o = OracleEngine(stream["n_keys"], threads=4)
    gen.load_stream(o, sub)
    o.apply_batch(sub["batch"])
    want = [o.read_doc(x)["text"] for x in range(k)]
    return {"ops_per_s": j["ops_per_s"], "ms": j["ms"], "docs": m, "ops": j["ops"], "workers": j["workers"],
            "parts": j["parts"], "errors": j.get("errors"), "timing_ms": j.get("timing"),
            "texts_equal_restatement": want == j.get("texts"), "texts_checked": k,
            "includes": "ShardedHost: worker threads pack their document shards (JS) into one shared batch, the host "
                        "merges the interned property ids and submits (N-API mte_submit upload + mte_run), 4 slices "
                        "pipelined, final mte_sync; message objects built in the workers before the clock",
            "wall_s": round(time.perf_counter() - t0, 1)}


def cpu_baseline(stream, gpu_digest, target_s, tree=False):
    """Time the CPU restatement (oracle/, kind 'port') on a bounded doc sample:
    the flat restatement (oracle.c), or for documents of millions of segments
    (config 5) the same rules with a chunk index (tree="chunked", chunked.c),
    whose per-op cost is O(chunks + chunk), not O(S)."""
    from fluidframework_amd import gen
    from oracle import OracleEngine

    threads = host_threads()
    n_docs = len(stream["inits"])
    src = "oracle/chunked.c flat restatement with a chunk index" if tree == "chunked" else \
        "oracle/oracle.c flat restatement"
    # calibrate on a small slice, then size the sample for ~target_s
    cal = max(min(threads, n_docs), min(n_docs, 64 if not tree else threads))
    sub = gen.slice_docs(stream, 0, cal)
    o = OracleEngine(stream["n_keys"], threads=threads, tree=tree)
    gen.load_stream(o, sub)
    t0 = time.perf_counter()
    o.apply_batch(sub["batch"])
    t_cal = time.perf_counter() - t0
    per_doc = t_cal / cal
    m = int(min(n_docs, max(cal, target_s / max(per_doc, 1e-9))))
    if m != cal:
        del o
        sub = gen.slice_docs(stream, 0, m)
        o = OracleEngine(stream["n_keys"], threads=threads, tree=tree)
        gen.load_stream(o, sub)
        t0 = time.perf_counter()
        o.apply_batch(sub["batch"])
        dt = time.perf_counter() - t0
    else:
        dt = t_cal
    ops = int(sub["batch"]["op_offsets"][-1])
    parity = bool(np.array_equal(o.digest(), gpu_digest[:m]) and (o.statuses() == 0).all())
    return ({"value": ops / dt, "unit": "ops/s", "cores": threads, "kind": "port",
             "sample": f"first {m} of {n_docs} docs (all their ops, {ops} ops), {dt:.1f} s, {src}, "
                       f"{threads} pthreads"},
            {"docs": m, "digest_equal": parity, "checked_against": "the timed GPU runs' digests"})


if __name__ == "__main__":
    main()
