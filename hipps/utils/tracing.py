"""Per-phase step tracing.

The reference times phases with host ``time.time()`` deltas that include implicit syncs
(/root/reference/ps.py:116, 128-148, 160-191) and returns them in the step dict.  hipps keeps
those host keys and, with ``PSConfig.trace`` (``HIPPS_TRACE=1``), adds DEVICE times:

* each phase (``encode`` per bucket on the comm stream, ``comm``, ``update``) is bracketed by a
  pair of timing HIP events recorded on the stream that runs it, and named with a roctx range
  (``hipps._C.roctx_push/pop``) so ``rocprofv3 --marker-trace`` shows it beside its kernels;
* :meth:`StepTracer.collect` never blocks: it harvests event pairs whose end event has
  completed (``hipEventQuery``), so step *t* usually reports the phases of step *t-1* and the
  async pipeline is not serialized by the tracer.  ``flush()`` drains everything (e.g. at close).

On CPU the same API records host ``perf_counter`` deltas.
"""
from __future__ import annotations

import threading
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List, Optional, Tuple

import torch


def _roctx():
    try:
        from hipps.ops._native import available, native

        if available():
            return native()
    except Exception:  # pragma: no cover - tracing must never break training
        pass
    return None


class StepTracer:
    def __init__(self, enabled: bool, cuda: bool):
        self.enabled = bool(enabled)
        self.cuda = cuda
        self._rt = _roctx() if self.enabled else None
        self._pending: List[Tuple[str, object, object]] = []
        self._host: Dict[str, float] = defaultdict(float)
        self._lock = threading.Lock()
        self.totals: Dict[str, float] = defaultdict(float)  # all harvested ms, for summaries
        self.counts: Dict[str, int] = defaultdict(int)

    def mark(self, name: str):
        if self.enabled and self._rt is not None:
            self._rt.roctx_mark(name)

    @contextmanager
    def phase(self, name: str, stream: Optional["torch.cuda.Stream"] = None):
        if not self.enabled:
            yield
            return
        if self._rt is not None:
            self._rt.roctx_push(name)
        if self.cuda:
            s = stream if stream is not None else torch.cuda.current_stream()
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
        else:
            t0 = time.perf_counter()
        try:
            yield
        finally:
            if self.cuda:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(s)
                with self._lock:
                    self._pending.append((name, e0, e1))
            else:
                with self._lock:
                    self._host[name] += (time.perf_counter() - t0) * 1e3
            if self._rt is not None:
                self._rt.roctx_pop()

    def _harvest(self, block: bool) -> Dict[str, float]:
        out: Dict[str, float] = defaultdict(float)
        with self._lock:
            keep = []
            for name, e0, e1 in self._pending:
                if block:
                    e1.synchronize()
                elif not e1.query():
                    keep.append((name, e0, e1))
                    continue
                out[name] += e0.elapsed_time(e1)
            self._pending = keep
            for k, v in self._host.items():
                out[k] += v
            self._host.clear()
        for k, v in out.items():
            self.totals[k] += v
            self.counts[k] += 1
        return {f"{k}_ms": v for k, v in out.items()}

    def collect(self) -> Dict[str, float]:
        """Device ms of the phases that have finished since the last call (non-blocking)."""
        return self._harvest(False) if self.enabled else {}

    def flush(self) -> Dict[str, float]:
        return self._harvest(True) if self.enabled else {}

    def summary(self) -> Dict[str, float]:
        return {f"{k}_ms_total": v for k, v in self.totals.items()}
