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

Bucket granularity (``bucketwise=True``, README.md:64-76: the reference's PS steps and
broadcasts each parameter on its own): every bucket keeps its own accumulation count and version.
Bucket b is updated and published as soon as M messages for b have arrived (the PS update is
pipelined with message arrival), so a worker's next read may mix versions across buckets --
the inconsistent read of README.md:79-81.  The global version ``ver`` is min over buckets.

    backend.note_presence_b(i, slot, vidx, bi)   a kept message (missing-grad mask of bucket bi)
    backend.update_bucket(bi, v, gver, incl, gscale)
                                                 update + publish bucket bi at version v; gver is
                                                 the new global version if it advanced (else
                                                 None); incl = {worker: newest fully included seq}

PSAsyncEngine drives it with the shared-memory control block and HIP streams; the in-process
fake transport (hipps.parallel.fake) drives it with scripted arrival orders, so protocol edge
cases are tested deterministically instead of through multi-process timing.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence


class PSCore:
    def __init__(self, ctl, F, W: int, nb: int, order: Sequence[int], slots: int, maxslots: int, M: int,
                 staleness: int = -1, staleness_lr: bool = False, gscale: float = 1.0,
                 stats: Optional[Dict[str, int]] = None, bucketwise: bool = False):
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
        self.ps_rank = 0
        self.recent: List[int] = []  # staleness of the newest accumulated steps (look-ahead tau)
        self.RECENT = max(8, 2 * W)
        self.bucketwise = bucketwise
        if bucketwise:
            self.count_b = [0] * nb
            self.ver_b = [0] * nb
            self.pending_b: List[List[tuple]] = [[] for _ in range(nb)]  # (worker, step) since b's update
            self.incl_b = [[0] * nb for _ in range(W)]  # [worker][bucket] newest step reflected in b

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
        vidx = i * self.MAXSLOTS + slot
        # the message names its bucket (flag word = ring offset / 256 << 21 | bucket << 1 |
        # presence bit): a worker pushes a step's buckets in completion order, not a fixed order
        bi = (self.ctl.load(F.F_PUSH_FLAG, vidx) >> 1) & ((1 << 20) - 1)
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
        if self.bucketwise:
            self._one_bucket(i, s, slot, pos, bi, vidx)
            return
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

    def _one_bucket(self, i: int, s: int, slot: int, pos: int, bi: int, vidx: int):
        F, be, nb = self.F, self.backend, self.nb
        step = (s - 1) // nb + 1
        kept = not self.dropping[i]
        if kept:
            be.accumulate(i, slot, bi, s, self.scale[i])
            be.note_presence_b(i, slot, vidx, bi)
        be.ack(i, s)
        # a dropped step still counts as included for max_delay once each bucket moves on
        self.pending_b[bi].append((i, step))
        if pos == nb - 1:
            if kept:
                self.stats["accumulated"] += 1
            else:
                self.stats["drops"] += 1
                self.ctl.fetch_add(F.F_DROPS, 0, 1)
        if not kept:
            return
        self.count_b[bi] += 1
        if self.count_b[bi] < self.M:
            return
        self.ver_b[bi] += 1
        self.count_b[bi] = 0
        touched = set()
        for w, st in self.pending_b[bi]:
            if st > self.incl_b[w][bi]:
                self.incl_b[w][bi] = st
            touched.add(w)
        self.pending_b[bi] = []
        incl = {w: min(self.incl_b[w]) * nb for w in touched}
        gver = min(self.ver_b)
        adv = gver > self.ver
        if adv:
            self.ver = gver
        if hasattr(be, "flush"):
            be.flush()
        be.update_bucket(bi, self.ver_b[bi], gver if adv else None, incl, self.gscale)

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
        """Stop when every live worker said STOP and all its messages were consumed.  The PS's own
        rank (0: the co-located worker 0, or the dedicated PS that said STOP in serve()) is never
        skipped as dead, so the PS outlives its own process's long pauses (a barrier, a checkpoint)."""
        F = self.F
        if self.ctl.load(F.F_PS_STOP, 0):
            return True
        dead = set(dead) - {self.ps_rank}
        for i in range(self.W):
            if i in dead:
                continue  # failure detection: a silent worker does not hold the PS open
            stop = self.ctl.load(F.F_STOP, i)
            if stop == 0 or self.seen[i] < stop - 1:
                return False
        return True
