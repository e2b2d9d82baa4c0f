"""The AsySG-InCon parameter-server protocol, independent of the transport (README.md:56-81).

``PSCore`` is the PS's bookkeeping: which worker message is which bucket of which step, the
staleness rule (ConditionalAccumulator semantics, README.md:33-35), M-gradient accumulation
(README.md:65-73 -- "until it has 32", possibly several from one fast worker), the per-worker
"included" sequence numbers that ``max_delay`` waits on, and the stop rule that does not wait for
dead workers.  It reads and writes only control words (``load``/``store``/``fetch_add`` on a
control block) and calls a backend for the data plane:

    backend.accumulate(i, slot, bi, seq, scale)   decode + add worker i's message into the accumulator
    backend.note_presence(i, slot, vidx)          last bucket of a kept step (missing-grad masks)
    backend.ack(i, seq)                           the slot may be reused (stream-ordered doorbell)
    backend.update(included, gscale)              optimizer step + publish version ``core.ver``
    backend.flush()                               (optional) issue deferred accumulates / acks

PSAsyncEngine drives it with the shared-memory control block and HIP streams; the in-process
fake transport (hipps.parallel.fake) drives it with scripted arrival orders, so protocol edge
cases are tested deterministically instead of through multi-process timing.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence


class PSCore:
    def __init__(self, ctl, F, W: int, nb: int, order: Sequence[int], slots: int, maxslots: int, M: int,
                 staleness: int = -1, staleness_lr: bool = False, gscale: float = 1.0,
                 stats: Optional[Dict[str, int]] = None):
        self.ctl, self.F = ctl, F
        self.W, self.nb, self.order = W, nb, list(order)
        self.SLOTS, self.MAXSLOTS, self.M = slots, maxslots, M
        self.staleness, self.staleness_lr, self.gscale = staleness, staleness_lr, gscale
        self.stats = stats if stats is not None else {}
        for k in ("drops", "staleness_sum", "accumulated"):
            self.stats.setdefault(k, 0)
        self.ver = 0
        self.count = 0
        self.pending: List[tuple] = []  # (worker, last seq of a completed step) since the last update
        self.seen = [0] * W
        self.dropping = [False] * W
        self.scale = [1.0] * W
        self.backend = None
        self.recent: List[int] = []  # staleness of the newest accumulated steps (look-ahead tau)
        self.RECENT = max(8, 2 * W)

    def pump(self, i: int, upto: Optional[int] = None) -> int:
        """Process every message worker ``i`` has pushed since the last call (or up to message
        ``upto``, for transports that learn about arrival from elsewhere); returns how many."""
        F = self.F
        s_now = self.ctl.load(F.F_PUSH_SEQ, i) if upto is None else upto
        n = 0
        for s in range(self.seen[i] + 1, s_now + 1):
            self._one(i, s)
            n += 1
        self.seen[i] = max(self.seen[i], s_now)
        return n

    def _one(self, i: int, s: int):
        F, be, nb = self.F, self.backend, self.nb
        slot = s % self.SLOTS
        pos = (s - 1) % nb
        bi = self.order[pos]
        vidx = i * self.MAXSLOTS + slot
        if pos == 0:  # a step's first message carries the version its gradient was computed on
            pv = self.ctl.load(F.F_PUSH_VER, vidx)
            stale = self.ver - pv
            self.dropping[i] = 0 <= self.staleness < stale
            self.scale[i] = 1.0 / max(1, stale) if self.staleness_lr else 1.0
            if not self.dropping[i]:
                self.stats["staleness_sum"] += max(0, stale)
                self.recent.append(max(0, stale))
                if len(self.recent) > self.RECENT:
                    del self.recent[0]
            # per-step staleness record the worker reads back into its step() data
            self.ctl.store(F.F_LAST_STALE, i, stale)
            self.ctl.store(F.F_LAST_STALE_SEQ, i, s + nb - 1)
        if not self.dropping[i]:
            be.accumulate(i, slot, bi, s, self.scale[i])
            if pos == nb - 1:
                be.note_presence(i, slot, vidx)
        be.ack(i, s)
        if pos == nb - 1:
            self.pending.append((i, s))  # a dropped step still counts for max_delay
            if self.dropping[i]:
                self.stats["drops"] += 1
                self.ctl.fetch_add(F.F_DROPS, 0, 1)
            else:
                self.stats["accumulated"] += 1
                self.count += 1
                if self.count >= self.M:
                    self.ver += 1
                    if hasattr(be, "flush"):
                        be.flush()
                    be.update(self.pending, self.gscale)
                    self.pending = []
                    self.count = 0

    def mean_staleness(self) -> float:
        """Mean staleness (in updates) of the newest accumulated steps."""
        return sum(self.recent) / len(self.recent) if self.recent else 0.0

    @staticmethod
    def last_included(included) -> Dict[int, int]:
        last: Dict[int, int] = {}
        for i, s in included:
            last[i] = max(last.get(i, 0), s)
        return last

    def should_stop(self, dead: Sequence[int] = ()) -> bool:
        """Stop when every live worker said STOP and all its messages were consumed."""
        F = self.F
        if self.ctl.load(F.F_PS_STOP, 0):
            return True
        dead = set(dead)
        for i in range(self.W):
            if i in dead:
                continue  # failure detection: a silent worker does not hold the PS open
            stop = self.ctl.load(F.F_STOP, i)
            if stop == 0 or self.seen[i] < stop - 1:
                return False
        return True
