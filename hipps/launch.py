"""Single-node launcher: ``python -m hipps.launch -n 8 train.py [args...]``.

Replaces the reference's ``mpirun -n 2 py.test -s`` (Makefile:3).  Starts one process per GPU
with RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR=127.0.0.1 / MASTER_PORT set (the env contract
``hipps.parallel.dist.init_from_env`` and ``torch.distributed.run`` share), keeps
HSA_ENABLE_IPC_MODE_LEGACY=0 (dmabuf IPC, required by the HIP-IPC mailboxes and RCCL), tags each
rank's output, and tears the whole job down if any rank fails (no orphaned ranks blocking the
others in a collective).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import threading
import time


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pump(stream, prefix, out):
    for line in iter(stream.readline, b""):
        out.write(prefix + line.decode(errors="replace"))
        out.flush()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("-n", "--nproc", type=int, default=1)
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--module", "-m", action="store_true", help="run the target as a module (python -m)")
    ap.add_argument("--no-tag", action="store_true", help="do not prefix output lines with the rank")
    ap.add_argument("target")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    port = a.port or _free_port()
    procs = []
    base = dict(os.environ)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(a.nproc),
                HSA_ENABLE_IPC_MODE_LEGACY="0")
    for r in range(a.nproc):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(a.nproc))
        cmd = [sys.executable] + (["-m", a.target] if a.module else [a.target]) + a.args
        p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True)
        procs.append(p)
        threading.Thread(target=_pump, args=(p.stdout, "" if a.no_tag else f"[rank{r}] ", sys.stdout),
                         daemon=True).start()
    rc = 0
    try:
        alive = set(range(a.nproc))
        while alive:
            for r in list(alive):
                c = procs[r].poll()
                if c is None:
                    continue
                alive.discard(r)
                if c != 0 and rc == 0:
                    rc = c
                    print(f"[hipps.launch] rank {r} exited with {c}; stopping the job", file=sys.stderr)
                    for q in procs:
                        if q.poll() is None:
                            os.killpg(q.pid, signal.SIGTERM)
            time.sleep(0.05)
    except KeyboardInterrupt:
        for q in procs:
            if q.poll() is None:
                os.killpg(q.pid, signal.SIGTERM)
        rc = 130
    for q in procs:
        try:
            q.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(q.pid, signal.SIGKILL)
    return rc


if __name__ == "__main__":
    sys.exit(main())
