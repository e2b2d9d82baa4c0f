"""Per-step metrics (reference: the ``data`` dict returned by ps.py:step, ps.py:116-191).

Reference keys kept: comm_wait, optim_step_time, decode_time, msg_bytes, packaged_bytes,
code_wait, iallgather_prepare_time, isend_time.  Added: grad_bytes_sent/recv, version, step_time,
``staleness`` (async workers: PS updates between the version a worker's newest consumed gradient
was computed on and the update that applied it, read from the control block's LAST_STALE word,
``PSAsyncEngine.step`` in ps_async.py) and ``samples_per_sec`` (every mode, when ``samples_per_step`` is
configured; optim.py ``step``).  ``MetricsWriter`` appends one JSON line per step per rank.
"""
from __future__ import annotations

import json
import os
import time


class MetricsWriter:
    def __init__(self, path: str, rank: int = 0):
        path = path.replace("{rank}", str(rank))
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self.f = open(path, "a", buffering=1)
        self.rank = rank

    def write(self, step: int, data: dict):
        rec = {"t": time.time(), "rank": self.rank, "step": step}
        rec.update({k: (float(v) if isinstance(v, (int, float)) else v) for k, v in data.items()})
        self.f.write(json.dumps(rec) + "\n")

    def close(self):
        if not self.f.closed:
            self.f.close()


def summarize(records):
    """Mean of every numeric key over a list of per-step dicts (rank-0 summary)."""
    out = {}
    for r in records:
        for k, v in r.items():
            if isinstance(v, (int, float)):
                out.setdefault(k, []).append(v)
    return {k: sum(v) / len(v) for k, v in out.items()}
