"""One rank of tests/test_dist_shard.py's N > 1 job, started by the product's
launcher (fluidframework_amd/launch.py run_ranks, as bench.py --gpus N starts
its ranks): RANK / WORLD_SIZE from the environment, its shard of the
work-balanced assignment generated and replayed, digests gathered through a
file-backed stand-in for mte_comm_gather_digests.
usage: python tests/dist_rank.py <exchange dir> <0 | 1: the device engine>"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))) + "/tests")

from fluidframework_amd import dist as fdist  # noqa: E402
from fluidframework_amd import gen  # noqa: E402

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



if __name__ == "__main__":
    _rank(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), sys.argv[1], sys.argv[2] == "1")
    if os.environ["RANK"] == "0":
        print(f"rank 0 of {os.environ['WORLD_SIZE']} done, rendezvous {os.environ['MASTER_ADDR']}:"
              f"{os.environ['MASTER_PORT']}")
