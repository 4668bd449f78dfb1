#!/usr/bin/env python3
"""Kernel microbenchmarks (GPU): per-op latency and throughput of the replay
kernel under controlled streams.  Prints one line per experiment."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fluidframework_amd import gen  # noqa: E402
from fluidframework_amd.abi import OP_NOOP  # noqa: E402
from fluidframework_amd.engine import DeviceEngine  # noqa: E402


def run(name, stream, reps=3):
    d = DeviceEngine(stream["n_keys"])
    d.load_docs(stream["inits"], stream["init_text"])
    d.submit(stream["batch"])
    ms = []
    for _ in range(reps):
        d.reset()
        d.run()
        d.sync()
        ms.append(d.stats()["kernel_ms"])
    st = d.stats()
    n_ops = int(stream["batch"]["op_offsets"][-1])
    n_docs = len(stream["inits"])
    best = min(ms)
    print(f"{name:34s} docs={n_docs:6d} ops={n_ops:10d} kernel_ms={best:9.3f} "
          f"Mops/s={n_ops / best / 1e3:9.1f} us/op/doc={best * 1e3 / (n_ops / n_docs):8.3f} "
          f"avgS={st['segs_scanned'] / max(1, st['ops_applied']):6.1f} status={set(d.statuses().tolist())}",
          flush=True)


def main():
    which = sys.argv[1:] or ["all"]
    base3 = gen.generate(3, n_docs=10000, ops_per_doc=2000)
    if "all" in which or "scale" in which:
        for nd in (256, 4096, 10000):
            run(f"cfg3 docs={nd}", gen.slice_docs(base3, 0, nd))
    if "all" in which or "noop" in which:
        s = gen.slice_docs(base3, 0, 10000)
        s["batch"] = dict(s["batch"])
        ops = s["batch"]["ops"].copy()
        ops["type"] = OP_NOOP
        s["batch"]["ops"] = ops
        run("cfg3 all NOOP", s)
    if "all" in which or "lat" in which:
        # one wave per CU (512 docs = 256 pairs): per-op latency by op mix
        for name, kw in (("full", {}),
                         ("ins+rem", {"mix": gen.MIX_INSERT | gen.MIX_REMOVE, "marker_every": 0}),
                         ("ins+ann", {"mix": gen.MIX_INSERT | gen.MIX_ANNOTATE, "marker_every": 0})):
            s = gen.generate(3, n_docs=512, ops_per_doc=2000, **kw)
            run(f"lat512 {name}", s)
            if name == "full":
                s["batch"] = dict(s["batch"])
                ops = s["batch"]["ops"].copy()
                ops["type"] = OP_NOOP
                s["batch"]["ops"] = ops
                run("lat512 NOOP", s)
    if "all" in which or "types" in which:
        s2 = gen.generate(2, n_docs=10000, ops_per_doc=2000)
        run("cfg2 (ins/rem, K=0)", s2)
        s4 = gen.generate(3, n_docs=10000, ops_per_doc=2000, mix=gen.MIX_INSERT | gen.MIX_REMOVE, marker_every=0)
        s4["n_keys"] = 0
        run("cfg3-shape ins/rem K=0", s4)


if __name__ == "__main__":
    main()
