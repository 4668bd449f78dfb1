"""One process per GPU without an external launcher (no torch).

`bench.py --gpus N` run directly (no RANK / WORLD_SIZE in its environment)
starts its own N ranks here, before anything in the parent touches a GPU: each
child gets RANK = LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE = N and a
MASTER_ADDR / MASTER_PORT rendezvous on 127.0.0.1 -- what
torch.distributed.run sets, so the ranks run the same code either way and
bootstrap RCCL through libmte.so (comm.py).  The parent forwards rank 0's
stdout (the bench's one JSON line) and exits with the first failing rank's
status, stopping the others."""
import os
import socket
import subprocess
import sys
import time


def visible_devices() -> int:
    """HIP devices a child process can open (hipGetDeviceCount in a throw-away
    process, so this one never initialises the GPU); 0 without a HIP runtime."""
    probe = ("import ctypes\n"
             "try:\n"
             "    h = ctypes.CDLL('libamdhip64.so')\n"
             "except OSError:\n"
             "    print(0); raise SystemExit\n"
             "n = ctypes.c_int(0)\n"
             "print(n.value if h.hipGetDeviceCount(ctypes.byref(n)) == 0 else 0)\n")
    try:
        r = subprocess.run([sys.executable, "-c", probe], capture_output=True, text=True, timeout=120)
        return int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else 0
    except (subprocess.SubprocessError, ValueError, IndexError):
        return 0


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(base, rank, world, port):
    env = dict(base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port), "TORCHELASTIC_RUN_ID": f"mte{os.getpid()}"})
    return env


def run_ranks(world, cmd, need_devices=True, timeout=None, out=None):
    """Run `cmd` as ranks 0..world-1 and wait for all of them.  Rank 0's stdout
    goes to `out` (default: this process's stdout); every rank's stderr is
    inherited.  Returns 0, or the exit status of the first rank that failed
    (the others are then terminated).  need_devices: refuse (status 2) when
    fewer than `world` GPUs are visible."""
    if world < 1:
        print(f"launch: world {world} < 1", file=sys.stderr)
        return 2
    if need_devices:
        have = visible_devices()
        if have < world:
            print(f"launch: {world} ranks need {world} GPUs, {have} visible", file=sys.stderr)
            return 2
    port = free_port()
    procs = []
    for r in range(world):
        procs.append(subprocess.Popen(cmd, env=rank_env(os.environ, r, world, port),
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    t0 = time.time()
    rc = 0
    stdout0 = b""
    live = set(range(world))
    try:
        while live:
            for r in sorted(live):
                p = procs[r]
                if r == 0:
                    try:
                        chunk, _ = p.communicate(timeout=0.2)
                        stdout0 += chunk or b""
                    except subprocess.TimeoutExpired:
                        continue
                elif p.poll() is None:
                    continue
                live.discard(r)
                if p.returncode != 0 and rc == 0:
                    rc = p.returncode if p.returncode > 0 else 128 - p.returncode
                    print(f"launch: rank {r} exited with status {p.returncode}", file=sys.stderr)
            if rc != 0:
                break
            if timeout is not None and time.time() - t0 > timeout:
                print(f"launch: ranks still running after {timeout} s", file=sys.stderr)
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    text = stdout0.decode(errors="replace")
    if out is None:
        sys.stdout.write(text)
        sys.stdout.flush()
    else:
        out.append(text)
    return rc
