"""Multi-GPU sharding of documents.  No torch.

Documents are independent, so a node job assigns each document to one rank
(one process per GPU) and no collective touches the replay.  The assignment
is by expected work: documents longest first onto the least
loaded rank (LPT), the same rule as the Node host's
MergeTreeEngine.shardByWork (node/index.js).  The only collective is the
verification all-gather of the per-doc digests (libmte.so mte_comm_gather_
digests over RCCL): rank-major, every rank's rows padded with zero rows to
`docs_per_rank`.  `unshard_digests` turns that layout back into global
document order.
"""
import numpy as np


def shard_by_work(work, world: int) -> np.ndarray:
    """Rank of every document: longest first onto the least loaded rank
    (ties: the lower document index first, the lower rank first)."""
    work = np.asarray(work, dtype=np.float64)
    order = sorted(range(len(work)), key=lambda d: (-work[d], d))
    load = np.zeros(world, np.float64)
    rank_of = np.zeros(len(work), np.int32)
    for d in order:
        r = int(np.argmin(load))  # argmin returns the first (lowest) rank on ties
        rank_of[d] = r
        load[r] += work[d]
    return rank_of


def rank_docs(rank_of, rank: int) -> np.ndarray:
    """Global indices of `rank`'s documents, ascending (its local order)."""
    return np.flatnonzero(np.asarray(rank_of) == rank).astype(np.uint32)


def docs_per_rank(rank_of, world: int) -> int:
    """Rows per rank of the gathered digest layout (the largest shard)."""
    return int(np.bincount(np.asarray(rank_of), minlength=world).max()) if len(rank_of) else 0


def unshard_digests(gathered, rank_of, world: int) -> np.ndarray:
    """(world, docs_per_rank, 4) or (world * docs_per_rank, 4) gathered digests
    (rank-major, zero-padded rows) -> (n_docs, 4) in global document order."""
    rank_of = np.asarray(rank_of)
    g = np.asarray(gathered, dtype=np.uint64).reshape(world, -1, 4)
    out = np.zeros((len(rank_of), 4), np.uint64)
    for r in range(world):
        ids = rank_docs(rank_of, r)
        out[ids] = g[r, :len(ids)]
    return out


def digest_fold(d) -> int:
    """A single 64-bit checksum of checksums for logging (xor of h1 ^ h2)."""
    d = np.asarray(d, dtype=np.uint64).reshape(-1, 4)
    return int(np.bitwise_xor.reduce(d[:, 1] ^ d[:, 2])) if len(d) else 0
