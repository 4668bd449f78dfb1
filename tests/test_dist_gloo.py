"""The N > 1 path of bench.py on CPU: 2 ranks over gloo shard the documents
(weak scaling, global doc seeds), replay their shards independently and
all-gather the per-doc digests.  The gathered digests must equal a single
process replaying all documents.  The CPU restatement (oracle) stands in for
the device engine here (test infrastructure only): what is under test is the
sharding and the collective, not the replay."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

DOCS_PER_RANK = 24
OPS = 300


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    import torch.distributed as dist

    from fluidframework_amd import dist as fdist
    from fluidframework_amd import gen
    from oracle import OracleEngine

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = gen.generate(3, n_docs=DOCS_PER_RANK, ops_per_doc=OPS,
                     doc_base=fdist.shard_doc_base(rank, DOCS_PER_RANK), n_threads=2)
    o = OracleEngine(s["n_keys"], threads=2)
    o.load_docs(s["inits"], s["init_text"])
    o.apply_batch(s["batch"])
    allg = fdist.gather_digests(dist, local_digest=o.digest())
    n_total = fdist.sum_over_ranks(dist, int(s["batch"]["op_offsets"][-1]))
    t = fdist.max_over_ranks(dist, float(rank + 1))
    if rank == 0:
        np.save(out, allg)
        with open(out + ".meta", "w") as fh:
            fh.write(f"{n_total} {t}")
    dist.destroy_process_group()


def test_two_rank_gloo_shard_and_digest_gather(tmp_path):
    out = str(tmp_path / "g.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    allg = np.load(out)
    n_total, t = open(out + ".meta").read().split()
    from fluidframework_amd import gen
    from oracle import OracleEngine

    s = gen.generate(3, n_docs=2 * DOCS_PER_RANK, ops_per_doc=OPS, doc_base=0, n_threads=2)
    o = OracleEngine(s["n_keys"], threads=2)
    o.load_docs(s["inits"], s["init_text"])
    o.apply_batch(s["batch"])
    np.testing.assert_array_equal(allg, o.digest())
    assert int(n_total) == int(s["batch"]["op_offsets"][-1])
    assert float(t) == 2.0
