"""The N > 1 path of bench.py on CPU, without torch: 2 processes take their
shards from the product's work-balanced assignment (fluidframework_amd/dist.py
shard_by_work, the Node host's shardByWork rule), generate and replay their
documents, and gather the per-doc digests in the layout
mte_comm_gather_digests produces (rank-major, each rank padded with zero rows
to docs_per_rank).  The collective is a file-backed stand-in (no RCCL on CPU,
and RCCL cannot put two ranks on one GPU); the replay is the device engine on
a GPU box (the -m gpu variant) and the CPU restatement elsewhere.  The
gathered digests, put back in global order by dist.unshard_digests, must equal
one process replaying every document."""
import multiprocessing as mp
import os
import time

import numpy as np
import pytest

from fluidframework_amd import dist as fdist
from fluidframework_amd import gen

N_DOCS = 37  # not a multiple of the world: ragged shards, padded rows
OPS = 300


def _work():
    # unequal expected work (ops x live segments) so LPT is not round-robin
    return np.array([OPS * (1 + (7 * d) % 5) for d in range(N_DOCS)], np.float64)


class FileComm:
    """Stand-in for mte_comm_{barrier, allreduce_f64, gather_digests} over files."""

    def __init__(self, root, rank, world):
        self.root, self.rank, self.world = root, rank, world
        self.k = 0

    def _exchange(self, payload: np.ndarray):
        self.k += 1
        tmp = os.path.join(self.root, f"{self.k}.{self.rank}.tmp")
        np.save(tmp, payload)
        os.replace(tmp + ".npy", os.path.join(self.root, f"{self.k}.{self.rank}.npy"))
        parts = []
        for r in range(self.world):
            path = os.path.join(self.root, f"{self.k}.{r}.npy")
            t0 = time.time()
            while not os.path.exists(path):
                if time.time() - t0 > 60:
                    raise TimeoutError(path)
                time.sleep(0.01)
            parts.append(np.load(path))
        return parts

    def barrier(self):
        self._exchange(np.zeros(1))

    def allreduce(self, v, op):
        parts = self._exchange(np.array([float(v)]))
        return float(sum(p[0] for p in parts) if op == "sum" else max(p[0] for p in parts))

    def gather_digests(self, digest, docs_per_rank):
        mine = np.zeros((docs_per_rank, 4), np.uint64)
        mine[:len(digest)] = digest
        return np.stack(self._exchange(mine))  # (world, docs_per_rank, 4), rank order


def _engine(use_gpu, n_keys):
    if use_gpu:
        from fluidframework_amd.engine import DeviceEngine
        return DeviceEngine(n_keys)
    from oracle import OracleEngine
    return OracleEngine(n_keys, threads=2)


def _rank(rank, world, root, use_gpu):
    comm = FileComm(root, rank, world)
    rank_of = fdist.shard_by_work(_work(), world)
    ids = fdist.rank_docs(rank_of, rank)
    s = gen.generate(3, ops_per_doc=OPS, doc_ids=ids, n_threads=2, round_sync=True)
    e = _engine(use_gpu, s["n_keys"])
    gen.load_stream(e, s)
    e.apply_batch(s["batch"])
    assert (e.statuses() == 0).all()
    comm.barrier()
    g = comm.gather_digests(e.digest(), fdist.docs_per_rank(rank_of, world))
    total = comm.allreduce(int(s["batch"]["op_offsets"][-1]), "sum")
    t = comm.allreduce(rank + 1.0, "max")
    if rank == 0:
        np.save(os.path.join(root, "gathered.npy"), g)
        with open(os.path.join(root, "meta"), "w") as fh:
            fh.write(f"{total} {t}")


def _run(tmp_path, use_gpu):
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_rank, args=(r, 2, str(tmp_path), use_gpu)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0
    g = np.load(tmp_path / "gathered.npy")
    total, t = open(tmp_path / "meta").read().split()
    rank_of = fdist.shard_by_work(_work(), 2)
    per = fdist.docs_per_rank(rank_of, 2)
    assert g.shape == (2, per, 4)
    for r in range(2):  # padding rows past a rank's shard stay zero
        assert (g[r, len(fdist.rank_docs(rank_of, r)):] == 0).all()
    s = gen.generate(3, n_docs=N_DOCS, ops_per_doc=OPS, doc_base=0, n_threads=2, round_sync=True)
    from oracle import OracleEngine
    o = OracleEngine(s["n_keys"], threads=2)
    gen.load_stream(o, s)
    o.apply_batch(s["batch"])
    np.testing.assert_array_equal(fdist.unshard_digests(g, rank_of, 2), o.digest())
    assert int(float(total)) == int(s["batch"]["op_offsets"][-1])
    assert float(t) == 2.0


def test_lpt_shard_by_work():
    # longest first onto the least loaded rank; equal work deals round-robin
    assert fdist.shard_by_work([5, 1, 4, 2, 3], 2).tolist() == [0, 0, 1, 0, 1]
    assert fdist.shard_by_work(np.ones(10), 4).tolist() == [0, 1, 2, 3, 0, 1, 2, 3, 0, 1]
    for world in (1, 2, 3, 8):
        r = fdist.shard_by_work(_work(), world)
        assert sorted(np.concatenate([fdist.rank_docs(r, k) for k in range(world)]).tolist()) == list(range(N_DOCS))
        loads = np.bincount(r, weights=_work(), minlength=world)
        assert loads.max() - loads.min() <= _work().max()  # the LPT bound


def test_generated_shard_equals_the_same_docs_of_the_whole_job():
    ids = np.array([3, 17, 4, 30], np.uint32)
    part = gen.generate(3, ops_per_doc=OPS, doc_ids=ids, n_threads=2)
    whole = gen.generate(3, n_docs=N_DOCS, ops_per_doc=OPS, n_threads=2)
    for k, d in enumerate(ids):
        a = gen.slice_docs(part, k, k + 1)["batch"]["ops"]
        b = gen.slice_docs(whole, int(d), int(d) + 1)["batch"]["ops"]
        np.testing.assert_array_equal(a[["seq", "ref_seq", "type", "pos1", "pos2"]],
                                      b[["seq", "ref_seq", "type", "pos1", "pos2"]])


def test_two_ranks_shard_replay_and_gather(tmp_path):
    _run(tmp_path, use_gpu=False)


@pytest.mark.gpu
def test_gpu_two_ranks_shard_replay_and_gather(tmp_path):
    _run(tmp_path, use_gpu=True)
