"""Node-level bootstrap for the RCCL entry points of libmte.so (mte_comm_*).

One process per GPU, launched by any launcher that sets RANK / WORLD_SIZE /
LOCAL_RANK (torch.distributed.run does; nothing here imports torch).  Rank 0
draws the RCCL unique id (mte_comm_unique_id) and hands it to the other ranks
through a file next to the job (one node: the driver's scaling bench), named by
the launcher's rendezvous address, port and run id; every rank then joins with
mte_comm_init.  After that the job's barrier, timing reductions and the digest
gather all go over RCCL."""
import os
import tempfile
import time

from ._native import load_mte

_T_IMPORT = time.time()  # an id file older than the job's start is a leftover


def _id_path():
    key = "_".join(os.environ.get(k, "x") for k in ("MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
                                                     "WORLD_SIZE"))
    key = "".join(ch if ch.isalnum() else "_" for ch in key)
    return os.path.join(tempfile.gettempdir(), f"mte_comm_{key}.id")


def unique_id() -> bytes:
    import ctypes as C
    buf = (C.c_uint8 * 128)()
    rc = load_mte().mte_comm_unique_id(buf)
    if rc:
        raise RuntimeError(f"mte_comm_unique_id: {rc}")
    return bytes(buf)


def exchange_id(rank: int, timeout: float = 120.0) -> bytes:
    """Rank 0 publishes a fresh id (atomic rename); the others wait for it."""
    path = _id_path()
    if rank == 0:
        uid = unique_id()
        tmp = path + f".{os.getpid()}"
        with open(tmp, "wb") as fh:
            fh.write(uid)
        os.replace(tmp, path)
        return uid
    t0 = time.time()
    while True:
        try:
            if os.path.getmtime(path) >= _T_IMPORT - 20.0:
                with open(path, "rb") as fh:
                    uid = fh.read()
                if len(uid) == 128:
                    return uid
        except FileNotFoundError:
            pass
        if time.time() - t0 > timeout:
            raise TimeoutError(f"no RCCL id at {path}")
        time.sleep(0.05)


def join(engine, rank: int, world: int):
    """Initialise engine's communicator; rank 0 removes the id file after all joined.
    RCCL prints a version banner on stdout at init: it goes to stderr, so the
    job's stdout stays its own (bench.py prints one JSON line there)."""
    uid = exchange_id(rank)
    import sys
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        engine.comm_init(world, rank, uid)
        engine.comm_barrier()
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    if rank == 0:
        try:
            os.remove(_id_path())
        except FileNotFoundError:
            pass
