"""Single-node rank launcher for ``bench.py --gpus N``.

The driver may start the bench either under ``torch.distributed.run`` (RANK /
LOCAL_RANK / WORLD_SIZE already set) or as a plain ``python bench.py --gpus N``.
In the second case the parent process must not touch the GPU at all: it starts
N child processes of the same script with the rendezvous environment set (one
rank per GPU, LOCAL_RANK = RANK on one node, MASTER_ADDR 127.0.0.1), relays
rank 0's stdout (the bench's one JSON line), and exits non-zero when any rank
fails.  When a rank fails, the others would block in their next collective, so
the launcher terminates them (its own child processes only, by handle).

Children are started with ``subprocess`` -- never by replacing the parent
process (an exec from a process that initialised the GPU is forbidden on the
target pool, and the parent here never initialises it in the first place).
"""
import os
import socket
import subprocess
import sys
import threading
import time

RANK_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def needs_spawn(n_ranks, environ=None):
    """True when ``--gpus n_ranks`` asks for several ranks and no launcher has
    set up this process as one of them."""
    env = os.environ if environ is None else environ
    return n_ranks > 1 and "WORLD_SIZE" not in env


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank, world, port, base=None):
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def launch_ranks(n_ranks, cmd, poll_s=0.2, out=None):
    """Run ``cmd`` (argv list) as ranks 0..n_ranks-1 and wait for all of them.

    Rank 0's stdout is copied to ``out`` (default sys.stdout); every rank's
    stderr goes to the parent's stderr.  Returns 0 when every rank exits 0,
    otherwise the first non-zero exit status seen (a rank killed by a signal
    reports 128 + signal)."""
    out = sys.stdout if out is None else out
    port = free_port()
    procs = []
    for r in range(n_ranks):
        procs.append(subprocess.Popen(cmd, env=rank_env(r, n_ranks, port),
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      stderr=None, text=True))
    # drain rank 0's stdout while the ranks run (a full pipe would block it)
    chunks = []
    reader = threading.Thread(target=lambda: chunks.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    rc_first = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad and rc_first == 0:
                rc_first = bad[0] if bad[0] > 0 else 128 - bad[0]
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
            if all(c is not None for c in codes):
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    reader.join(timeout=30)
    text = "".join(chunks)
    if text:
        out.write(text)
        out.flush()
    return rc_first
