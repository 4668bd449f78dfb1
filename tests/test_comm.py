"""Node level over RCCL through the C-ABI (mte_comm_*, include/mte.h).

CPU: the unique-id bootstrap between processes (fluidframework_amd/comm.py)
and the sharding of bench.py.  GPU: a one-rank communicator on the box's GPU —
barrier, reductions and the digest gather equal the engine's own digests
(more ranks need more GPUs: the driver's scaling bench runs them)."""
import multiprocessing as mp
import os

import numpy as np
import pytest

from fluidframework_amd import comm as fcomm
from fluidframework_amd import gen


def _peer(q, env):
    os.environ.update(env)
    import importlib

    import fluidframework_amd.comm as c
    importlib.reload(c)
    q.put(c.exchange_id(1, timeout=30))


def test_unique_id_exchange_between_processes(tmp_path, monkeypatch):
    env = {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29999", "TORCHELASTIC_RUN_ID": f"t{os.getpid()}",
           "WORLD_SIZE": "2", "TMPDIR": str(tmp_path)}
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    import tempfile
    monkeypatch.setattr(tempfile, "tempdir", str(tmp_path))
    # the RCCL id itself needs a GPU (ncclGetUniqueId); the exchange does not
    monkeypatch.setattr(fcomm, "unique_id", lambda: os.urandom(128))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_peer, args=(q, env))
    p.start()
    uid = fcomm.exchange_id(0)
    got = q.get(timeout=60)
    p.join(timeout=60)
    assert len(uid) == 128 and got == uid


def test_strong_shards_cover_the_job():
    # bench.py's strong scaling: 10k docs over N ranks by expected work (LPT)
    from fluidframework_amd import dist as fdist
    for world in (1, 2, 3, 4, 8):
        rank_of = fdist.shard_by_work(np.full(10000, 10000.0), world)
        sizes = [len(fdist.rank_docs(rank_of, r)) for r in range(world)]
        assert sum(sizes) == 10000 and max(sizes) - min(sizes) <= 1
        assert fdist.docs_per_rank(rank_of, world) == max(sizes)


@pytest.mark.gpu
def test_gpu_one_rank_communicator():
    from fluidframework_amd.engine import DeviceEngine
    node = DeviceEngine(0)
    os.environ.setdefault("MASTER_PORT", "29501")
    fcomm.join(node, 0, 1)
    assert node.comm_allreduce(2.5, "sum") == 2.5
    assert node.comm_allreduce(-1.0, "max") == -1.0
    s = gen.generate(3, n_docs=50, ops_per_doc=400, round_sync=True)
    e = DeviceEngine(s["n_keys"])
    gen.load_stream(e, s)
    e.apply_batch(s["batch"])
    e.comm_share(node)
    g = e.comm_gather_digests(64)
    np.testing.assert_array_equal(g[0, :50], e.digest())
    assert (g[0, 50:] == 0).all()
    e.comm_destroy()
    node.comm_destroy()
