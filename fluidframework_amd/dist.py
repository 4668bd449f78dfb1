"""Multi-GPU sharding of documents.

Documents are independent: rank r of a world of N replays its own shard of
`docs_per_rank` documents whose seeds are the global doc indices
[r * docs_per_rank, (r + 1) * docs_per_rank) — weak scaling, no collective on
the data path.  The only collective is the verification gather of the per-doc
32-byte digests (RCCL `all_gather` over xGMI under the "nccl" backend, gloo on
CPU in the tests).
"""
import numpy as np


def shard_doc_base(rank: int, docs_per_rank: int) -> int:
    """Global index of the first document of `rank`'s shard."""
    return rank * docs_per_rank


def gather_digests(dist, local_digest=None, engine=None, device=None):
    """All-gather every rank's (n_docs, 4) uint64 digests -> (world * n_docs, 4).

    Under a device backend pass `engine` and `device`: the digest kernel writes
    straight into a device tensor (mte_digest_device) that RCCL gathers.  On
    CPU (gloo) pass `local_digest` (numpy)."""
    import torch

    world = dist.get_world_size()
    if engine is not None:
        n = engine.n_docs
        mine = torch.empty((n, 4), dtype=torch.int64, device=device)
        engine.digest_device(mine.data_ptr())
        engine.sync()
    else:
        mine = torch.from_numpy(np.ascontiguousarray(local_digest).view(np.int64).copy())
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    return torch.cat(parts).cpu().numpy().view(np.uint64)


def digest_fold(d) -> int:
    """A single 64-bit checksum of checksums for logging (xor of h1 ^ h2)."""
    d = np.asarray(d, dtype=np.uint64).reshape(-1, 4)
    return int(np.bitwise_xor.reduce(d[:, 1] ^ d[:, 2])) if len(d) else 0


def max_over_ranks(dist, value: float, device=None) -> float:
    import torch

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, value: int, device=None) -> int:
    import torch

    t = torch.tensor([value], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
