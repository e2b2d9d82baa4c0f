"""In-process fake transport for the async PS protocol (SURVEY.md §4 tier 3).

Runs the real protocol core (hipps.parallel.ps_core.PSCore) against a dict-backed control block
and a Python mailbox, with the test deciding the exact order in which worker messages reach the
PS.  Any-source arrival orders, staleness drops, M-accumulation with fast workers, dead workers
and mailbox flow control become deterministic unit tests instead of multi-process timing.

    fake = FakeAsyncPS(W=3, nb=2, M=3, staleness=1)
    fake.push_step(1, grads=[0.5, 0.25])        # worker 1, computed on its adopted version
    fake.deliver(1)                             # PS consumes whatever worker 1 pushed
    fake.pull(1)                                # worker adopts the newest published version
"""
from __future__ import annotations

from types import SimpleNamespace
from typing import Dict, List, Optional, Sequence

from .ps_core import PSCore

# same field ids as hipps/csrc/runtime/control.cpp
FIELDS = SimpleNamespace(F_PUSH_SEQ=0, F_ACK_SEQ=1, F_PUSH_VER=2, F_APPLIED_VER=3, F_STOP=4, F_HEARTBEAT=5,
                         F_INCL_SEQ=6, F_PUSH_FLAG=7, F_READING=8, F_PULL_REQ=9, F_PUB_VER=10, F_PS_STOP=11,
                         F_ERROR=12, F_DROPS=13, F_UPDATES=14, F_BUF_VER=15, F_SENT_VER=16,
                         F_LAST_STALE=17, F_LAST_STALE_SEQ=18, F_BPUB_VER=19, F_BBUF_VER=20, F_READING_B=21)


class FakeControl:
    """The ControlBlock word API on a dict (no shared memory, no atomics needed: one thread)."""

    def __init__(self):
        self.words: Dict[tuple, int] = {}

    def load(self, field: int, idx: int) -> int:
        return self.words.get((field, idx), 0)

    def store(self, field: int, idx: int, v: int):
        self.words[(field, idx)] = int(v)

    def fetch_add(self, field: int, idx: int, v: int) -> int:
        old = self.load(field, idx)
        self.store(field, idx, old + v)
        return old


class WouldBlock(Exception):
    """A worker tried to reuse a mailbox slot the PS has not consumed (it would wait here)."""


class FakeAsyncPS:
    MAXSLOTS = 64

    def __init__(self, W: int, nb: int = 1, M: Optional[int] = None, staleness: int = -1,
                 staleness_lr: bool = False, slots: int = 4, lr: float = 1.0, average: bool = False,
                 bucketwise: bool = False):
        self.W, self.nb, self.SLOTS = W, nb, slots
        self.M = M if M else W
        self.lr = lr
        self.ctl = FakeControl()
        F = FIELDS
        self.bucketwise = bucketwise
        self.core = PSCore(self.ctl, F, W, nb, list(range(nb))[::-1], slots, self.MAXSLOTS, self.M, staleness,
                           staleness_lr, 1.0 / self.M if average else 1.0, bucketwise=bucketwise)
        self.core.backend = self
        self.mail: Dict[tuple, float] = {}  # (worker, slot) -> gradient value of that bucket
        self.acc = [0.0] * nb
        self.params = [0.0] * nb  # published parameters, one scalar per bucket
        self.history: List[dict] = []  # one record per PS update
        self.accumulated: List[tuple] = []  # (worker, step, bucket, scale) in PS order
        self._cur: List[tuple] = []
        self._cur_b: Dict[int, List[tuple]] = {}
        self.seq = [0] * W
        self.local_ver = [0] * W
        self.steps = [0] * W
        self.ctl.store(F.F_PUB_VER, 0, 0)
        self.local_ver_b = [[0] * nb for _ in range(W)]  # bucketwise: per-bucket adopted versions
        self.pub_b = [[0.0] for _ in range(nb)]  # bucketwise: published value of bucket b per version

    # ---- worker side ------------------------------------------------------------------------
    def push_step(self, i: int, grads: Sequence[float], version: Optional[int] = None, partial: bool = False,
                  order: Optional[Sequence[int]] = None):
        """Worker i pushes one step (nb bucket messages, in ready order or in ``order``) computed on
        ``version`` (default: the version it adopted last)."""
        F = FIELDS
        assert len(grads) == self.nb
        ver = self.local_ver[i] if version is None else version
        for pos in range(self.nb):
            s = self.seq[i] + 1
            if s > self.SLOTS and self.ctl.load(F.F_ACK_SEQ, i) < s - self.SLOTS:
                raise WouldBlock(f"worker {i} message {s}: slot {s % self.SLOTS} not yet consumed")
            slot = s % self.SLOTS
            bi = (order if order is not None else self.core.order)[pos]
            self.mail[(i, slot)] = float(grads[bi])
            vidx = i * self.MAXSLOTS + slot
            self.ctl.store(F.F_PUSH_VER, vidx, ver)
            self.ctl.store(F.F_PUSH_FLAG, vidx, (bi << 1) | (1 if (partial and pos == self.nb - 1) else 0))
            self.ctl.store(F.F_PUSH_SEQ, i, s)
            self.seq[i] = s
        self.steps[i] += 1

    def pull(self, i: int) -> int:
        """AsySG-InCon read: adopt the newest published version (bucketwise: the newest version of
        EACH bucket, which may differ across buckets)."""
        self.local_ver[i] = self.ctl.load(FIELDS.F_PUB_VER, 0)
        if self.bucketwise:
            self.local_ver_b[i] = [self.ctl.load(FIELDS.F_BPUB_VER, b) for b in range(self.nb)]
        return self.local_ver[i]

    def read_params(self, i: int) -> List[float]:
        """The parameters worker i adopted at its last pull (bucketwise: per-bucket versions)."""
        if not self.bucketwise:
            return list(self.history[self.local_ver[i] - 1]["params"]) if self.local_ver[i] else [0.0] * self.nb
        return [self.pub_b[b][v] for b, v in enumerate(self.local_ver_b[i])]

    def deliver_upto(self, i: int, s: int) -> int:
        """PS consumes worker i's messages up to sequence number s (partial arrival)."""
        return self.core.pump(i, upto=s)

    def stop(self, i: int):
        self.ctl.store(FIELDS.F_STOP, i, self.seq[i] + 1)

    def included(self, i: int) -> int:
        return self.ctl.load(FIELDS.F_INCL_SEQ, i)

    # ---- PS side ----------------------------------------------------------------------------
    def deliver(self, i: int) -> int:
        return self.core.pump(i)

    def deliver_order(self, order: Sequence[int]):
        for i in order:
            self.deliver(i)

    def accumulate(self, i, slot, bi, seq, scale):
        self.acc[bi] += scale * self.mail[(i, slot)]
        step = (seq - 1) // self.nb + 1
        self.accumulated.append((i, step, bi, scale))
        if self.bucketwise:
            self._cur_b.setdefault(bi, []).append((i, step))
        else:
            self._cur.append((i, step))

    def note_presence(self, i, slot, vidx):
        pass

    def note_presence_b(self, i, slot, vidx, bi):
        pass

    def update_bucket(self, bi, v, gver, incl, gscale):
        F = FIELDS
        self.params[bi] -= self.lr * gscale * self.acc[bi]
        self.acc[bi] = 0.0
        self.pub_b[bi].append(self.params[bi])
        assert len(self.pub_b[bi]) == v + 1
        self.ctl.store(F.F_BPUB_VER, bi, v)
        if gver is not None:
            self.ctl.store(F.F_PUB_VER, 0, gver)
            self.ctl.fetch_add(F.F_UPDATES, 0, 1)
        for i, s in incl.items():
            self.ctl.store(F.F_INCL_SEQ, i, s)
        contrib = sorted(set(self._cur_b.pop(bi, [])))
        self.history.append({"bucket": bi, "version": v, "global": gver, "params": list(self.params),
                             "contributors": contrib, "included": dict(incl)})

    def flush(self):
        pass

    def ack(self, i, seq):
        self.ctl.store(FIELDS.F_ACK_SEQ, i, seq)

    def update(self, included, gscale):
        F = FIELDS
        for b in range(self.nb):
            self.params[b] -= self.lr * gscale * self.acc[b]
            self.acc[b] = 0.0
        v = self.core.ver
        self.ctl.store(F.F_PUB_VER, 0, v)
        for i, s in self.core.last_included(included).items():
            self.ctl.store(F.F_INCL_SEQ, i, s)
        self.ctl.fetch_add(F.F_UPDATES, 0, 1)
        contrib = sorted({(i, st) for i, st in self._cur})
        self._cur = []
        self.history.append({"version": v, "params": list(self.params), "contributors": contrib,
                             "included": dict(self.core.last_included(included))})

    @property
    def stats(self):
        return dict(self.core.stats, updates=self.ctl.load(FIELDS.F_UPDATES, 0), version=self.core.ver)
