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
    process with status 3 (``os._exit`` -- never a re-exec), so the launcher tears the job down;
  * enqueue-only exchanges (hipps' own RCCL communicator returns as soon as the collectives are
    queued, so ``step()`` never blocks on them) hand the watchdog a HIP event recorded after their
    last collective: the thread polls ``ncclCommGetAsyncError`` and the event until the event
    completes, and aborts the communicator and exits if it has not after the same limit.
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
        self._events: list = []  # [(event, what, t0, poll)] device completions still pending
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

    def watch(self, event, what: str, poll=None):
        """Track an enqueued exchange until ``event`` (recorded after its last collective) has
        completed; ``poll()`` raises on an asynchronous communicator error."""
        with self._lock:
            self._events.append((event, what, time.monotonic(), poll))

    def pending(self) -> int:
        with self._lock:
            return len(self._events)

    def close(self, join_s: float = 5.0):
        """Stop the thread and wait for it (bounded), then forget pending events: the caller may
        destroy the communicator next, and a poll racing that destroy would read the destroyed
        comm's error state as a failure and exit with the abort status."""
        self._stop.set()
        if self._thread.is_alive() and self._thread is not threading.current_thread():
            self._thread.join(timeout=join_s)
        with self._lock:
            self._events = []
            self._armed = None

    def _fail(self, what: str, why: str):
        sys.stderr.write(f"[hipps] rank {self.rank}: exchange '{what}' {why}; a peer is dead or hung -- aborting "
                         f"with status {self.EXIT_CODE}\n")
        sys.stderr.flush()
        if self.on_abort is not None:
            try:
                self.on_abort()
            except Exception:
                pass
        os._exit(self.EXIT_CODE)

    def _check_events(self):
        with self._lock:
            evs = list(self._events)
        done = []
        now = time.monotonic()
        for item in evs:
            if self._stop.is_set():  # close() in progress: the communicator may be going away
                return
            ev, what, t0, poll = item
            if ev.query():  # completed: nothing left to poll the communicator for
                done.append(item)
                continue
            if poll is not None:
                try:
                    poll()
                except Exception as e:  # ncclCommGetAsyncError reported a failure
                    if self._stop.is_set():
                        return
                    self._fail(what, f"failed asynchronously ({e})")
            if now - t0 > self.limit:
                self._fail(what, f"did not complete on the device within {self.limit:.0f}s (comm_timeout_s)")
        if done:
            with self._lock:
                self._events = [e for e in self._events if e not in done]

    def _run(self):
        while not self._stop.wait(min(1.0, self.limit / 10)):
            with self._lock:
                a = self._armed
            if a is not None and time.monotonic() - a[1] > self.limit:
                self._fail(a[0], f"stalled for {self.limit:.0f}s (comm_timeout_s)")
            self._check_events()


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
