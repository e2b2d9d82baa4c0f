"""Communication watchdog for the synchronous engines.

The reference assumes "communication is reliable" (README.md:7) and relies on MPI's
errors-are-fatal default, so one dead rank leaves every other rank blocked in ``Wait()`` forever.
hipps bounds every exchange twice:

  * the engines run their collectives on a process group created with ``cfg.comm_timeout_s``
    (RCCL: the torch NCCL watchdog aborts the communicator -- ``ncclCommAbort`` -- and raises;
    gloo: the collective raises) so a lost peer turns into an exception, not a hang;
  * a host-side watchdog thread covers what the process group cannot see (a host wait on a
    device result, a peer that hangs mid-protocol): if one exchange stays armed longer than
    ``1.5 * comm_timeout_s + 5`` s it prints which exchange and step stalled and exits the
    process with status 3 (``os._exit`` -- never a re-exec), so the launcher tears the job down.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Optional


class CommWatchdog:
    EXIT_CODE = 3

    def __init__(self, timeout_s: float, rank: int = 0, on_abort=None):
        self.limit = 1.5 * float(timeout_s) + 5.0
        self.rank = rank
        self.on_abort = on_abort  # e.g. ncclCommAbort of hipps' own communicator
        self._armed: Optional[tuple] = None  # (what, t0)
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="hipps-watchdog", daemon=True)
        self._thread.start()

    def arm(self, what: str):
        with self._lock:
            self._armed = (what, time.monotonic())

    def disarm(self):
        with self._lock:
            self._armed = None

    def close(self):
        self._stop.set()

    def _run(self):
        while not self._stop.wait(min(1.0, self.limit / 10)):
            with self._lock:
                a = self._armed
            if a is not None and time.monotonic() - a[1] > self.limit:
                sys.stderr.write(f"[hipps] rank {self.rank}: exchange '{a[0]}' stalled for {self.limit:.0f}s "
                                 f"(comm_timeout_s); a peer is dead or hung -- aborting with status "
                                 f"{self.EXIT_CODE}\n")
                sys.stderr.flush()
                if self.on_abort is not None:
                    try:
                        self.on_abort()
                    except Exception:
                        pass
                os._exit(self.EXIT_CODE)


class armed:
    """``with armed(wd, 'allgather step 7'):`` -- no-op when ``wd`` is None."""

    def __init__(self, wd: Optional[CommWatchdog], what: str):
        self.wd, self.what = wd, what

    def __enter__(self):
        if self.wd is not None:
            self.wd.arm(self.what)
        return self

    def __exit__(self, *exc):
        if self.wd is not None:
            self.wd.disarm()
        return False
