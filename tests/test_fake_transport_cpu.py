"""Deterministic tests of the async PS protocol through the in-process fake transport
(hipps.parallel.fake): the real PSCore, scripted arrival orders (README.md:56-81 semantics)."""
import itertools

import pytest

from hipps.parallel.fake import FakeAsyncPS, WouldBlock


def test_any_source_order_does_not_change_the_update():
    """Every arrival order of 4 workers' gradients gives one update with the same sum (the PS
    receives from ANY_SOURCE, README.md:65-70) -- fp-exact here: the values are dyadic."""
    results = set()
    for order in itertools.permutations(range(4)):
        f = FakeAsyncPS(W=4, nb=2)
        for i in range(4):
            f.push_step(i, [0.5 * (i + 1), 0.25 * (i + 1)])
        f.deliver_order(order)
        assert f.stats["updates"] == 1 and f.stats["staleness_sum"] == 0
        results.add(tuple(f.params))
    assert results == {(-5.0, -2.5)}


def test_m_accumulation_may_take_several_gradients_from_one_worker():
    """M=3 "until it has 32" counts gradients, not workers: a fast worker can fill the round."""
    f = FakeAsyncPS(W=3, M=3, nb=1)
    for _ in range(3):
        f.push_step(0, [1.0])
    f.deliver(0)
    assert f.stats["updates"] == 1
    assert f.history[0]["contributors"] == [(0, 1), (0, 2), (0, 3)]
    f.push_step(1, [1.0])
    f.deliver(1)
    assert f.stats["updates"] == 1 and f.core.count == 1


def test_buckets_stream_and_version_rides_on_the_first_bucket():
    f = FakeAsyncPS(W=2, nb=3, M=2)
    f.push_step(0, [1.0, 2.0, 3.0])
    f.deliver(0)
    assert f.stats["updates"] == 0 and f.acc == [1.0, 2.0, 3.0]  # all buckets accumulated, round open
    f.push_step(1, [1.0, 1.0, 1.0])
    f.deliver(1)
    assert f.history[-1]["params"] == [-2.0, -3.0, -4.0]
    assert [a[2] for a in f.accumulated[:3]] == [2, 1, 0]  # ready order: last layers first


def test_staleness_drop_still_advances_included_seq():
    """ConditionalAccumulator semantics (README.md:33-35): a gradient computed on a version
    older than ``version - staleness`` is dropped, but its step counts as included so a worker
    waiting on max_delay is not stuck."""
    f = FakeAsyncPS(W=2, M=1, nb=1, staleness=1)
    f.push_step(0, [1.0])
    f.deliver(0)
    f.pull(0)
    f.push_step(0, [1.0])
    f.deliver(0)  # version 2
    f.push_step(1, [100.0], version=0)  # two versions behind -> dropped
    f.deliver(1)
    assert f.stats["drops"] == 1 and f.stats["updates"] == 2
    assert f.params == [-2.0]
    f.pull(0)
    f.push_step(0, [1.0])
    f.deliver(0)
    assert f.included(1) == 1  # worker 1's dropped step is reflected as included


def test_staleness_lr_scales_stale_gradients():
    f = FakeAsyncPS(W=2, M=1, nb=1, staleness_lr=True)
    f.push_step(0, [1.0])
    f.deliver(0)
    f.push_step(0, [1.0])
    f.deliver(0)  # version 2, worker 0 computed on 0 -> stale 1 (scale 1)
    f.push_step(1, [8.0], version=0)  # stale 2 -> scale 1/2
    f.deliver(1)
    assert [a[3] for a in f.accumulated] == [1.0, 1.0, 0.5]
    assert f.params == [-1.0 - 1.0 - 4.0]
    assert f.stats["staleness_sum"] == 0 + 1 + 2


def test_mailbox_flow_control_blocks_until_ack():
    f = FakeAsyncPS(W=1, M=1, nb=1, slots=2)
    f.push_step(0, [1.0])
    f.push_step(0, [1.0])
    with pytest.raises(WouldBlock):
        f.push_step(0, [1.0])  # slot of message 1 not consumed yet
    f.deliver(0)
    f.push_step(0, [1.0])
    assert f.deliver(0) == 1


def test_stop_rule_skips_dead_workers():
    f = FakeAsyncPS(W=3, M=1, nb=1)
    for i in range(3):
        f.push_step(i, [1.0])
    f.deliver_order([0, 1, 2])
    f.stop(0)
    f.stop(1)
    assert not f.core.should_stop()
    assert f.core.should_stop(dead=[2])  # a silent worker does not hold the PS open


def test_stop_waits_for_unconsumed_messages():
    f = FakeAsyncPS(W=1, M=1, nb=2)
    f.push_step(0, [1.0, 1.0])
    f.stop(0)
    assert not f.core.should_stop()
    f.deliver(0)
    assert f.core.should_stop()


@pytest.mark.parametrize("seed", range(5))
def test_random_interleavings_apply_every_gradient_exactly_once(seed):
    """Random push/deliver/pull interleavings (3 workers, 2 buckets, M=2): every pushed bucket
    is accumulated exactly once and the published params equal -sum(all gradients) once the PS
    drained everything that completes a round."""
    import random

    rnd = random.Random(seed)
    f = FakeAsyncPS(W=3, nb=2, M=2, slots=8)
    pushed = 0
    for _ in range(60):
        i = rnd.randrange(3)
        act = rnd.random()
        if act < 0.5:
            try:
                f.push_step(i, [1.0, 2.0])
                pushed += 1
            except WouldBlock:
                f.deliver(i)
        elif act < 0.85:
            f.deliver(i)
        else:
            f.pull(i)
    for i in range(3):
        f.deliver(i)
    assert len(f.accumulated) == 2 * pushed
    assert len({(a[0], a[1], a[2]) for a in f.accumulated}) == 2 * pushed  # no duplicates
    rounds = pushed // 2
    assert f.stats["updates"] == rounds
    assert f.params == [-1.0 * 2 * rounds, -2.0 * 2 * rounds]


# ---- bucket granularity (per-bucket PS updates and publication) ----------------------------------

def test_bucketwise_updates_publish_each_bucket_when_complete():
    """README.md:64-76: the PS steps and broadcasts each bucket as soon as M messages for it have
    arrived, so a worker reading in between adopts bucket versions that differ."""
    from hipps.parallel.fake import FakeAsyncPS

    f = FakeAsyncPS(W=2, nb=3, M=2, bucketwise=True)
    order = f.core.order  # messages of a step go in this bucket order
    f.push_step(0, grads=[1.0, 2.0, 4.0])
    f.push_step(1, grads=[1.0, 2.0, 4.0])
    # worker 0's whole step arrives, worker 1's first message only: one bucket has M = 2
    f.deliver(0)
    f.deliver_upto(1, 1)
    first = order[0]
    assert [h["bucket"] for h in f.history] == [first]
    assert f.core.ver_b[first] == 1 and f.core.ver == 0  # global version = min over buckets
    assert f.stats["updates"] == 0
    f.pull(0)
    assert f.local_ver_b[0][first] == 1 and sum(f.local_ver_b[0]) == 1  # a mixed-version read
    p = f.read_params(0)
    g = [1.0, 2.0, 4.0]
    assert p[first] == -2.0 * g[first] and all(p[b] == 0.0 for b in range(3) if b != first)
    f.deliver(1)
    assert f.core.ver_b == [1, 1, 1] and f.core.ver == 1 and f.stats["updates"] == 1
    assert [h["global"] for h in f.history] == [None, None, 1]
    f.pull(0)
    assert f.read_params(0) == [-2.0, -4.0, -8.0]


def test_bucketwise_max_delay_accounting_needs_every_bucket():
    """INCL_SEQ (what max_delay waits on) covers a step only once EVERY bucket holding one of its
    messages has been published."""
    from hipps.parallel.fake import FIELDS, FakeAsyncPS

    f = FakeAsyncPS(W=2, nb=2, M=2, bucketwise=True)
    f.push_step(0, grads=[1.0, 1.0])
    f.push_step(1, grads=[1.0, 1.0])
    f.deliver(0)
    f.deliver_upto(1, 1)  # bucket order[0] complete for step 1, order[1] not yet
    assert f.ctl.load(FIELDS.F_INCL_SEQ, 0) == 0 and f.ctl.load(FIELDS.F_INCL_SEQ, 1) == 0
    f.deliver(1)
    assert f.ctl.load(FIELDS.F_INCL_SEQ, 0) == 2 and f.ctl.load(FIELDS.F_INCL_SEQ, 1) == 2
    # a fast worker runs ahead: its second step is included bucket by bucket
    f.push_step(0, grads=[1.0, 1.0])
    f.push_step(0, grads=[1.0, 1.0])
    f.deliver(0)  # bucket counts reach M = 2 from worker 0 alone (ConditionalAccumulator)
    assert f.ctl.load(FIELDS.F_INCL_SEQ, 0) == 6
    assert f.stats["accumulated"] == 4


def test_bucketwise_staleness_drop_counts_whole_steps():
    from hipps.parallel.fake import FakeAsyncPS

    f = FakeAsyncPS(W=2, nb=2, M=1, staleness=0, bucketwise=True)
    f.push_step(0, grads=[1.0, 1.0])
    f.push_step(1, grads=[1.0, 1.0], version=0)
    f.deliver(0)  # M = 1: both buckets update, global version 1
    f.deliver(1)  # computed on version 0, now stale by 1 > 0: the whole step is dropped
    st = f.stats
    assert st["drops"] == 1 and st["accumulated"] == 1 and st["version"] == 1


@pytest.mark.parametrize("bucketwise", [False, True])
def test_messages_name_their_bucket_any_push_order(bucketwise):
    """A worker pushes a step's buckets in completion order (a bucket with a parameter that got no
    gradient waits for step() without holding back the others): the PS reads each message's bucket
    from its flag word, so per-worker push orders that differ give the same update as ready order."""
    from hipps.parallel.fake import FakeAsyncPS

    def run(orders):
        f = FakeAsyncPS(W=2, nb=3, M=2, bucketwise=bucketwise)
        for i in (0, 1):
            f.push_step(i, grads=[1.0, 2.0, 4.0], order=orders[i])
        f.deliver_order([1, 0])
        return f.params, f.stats

    ready = FakeAsyncPS(W=2, nb=3).core.order
    base_p, base_s = run([ready, ready])
    p, st = run([[1, 0, 2], [2, 1, 0]])
    assert p == base_p == [-2.0, -4.0, -8.0]
    assert st["accumulated"] == base_s["accumulated"] == 2 and st["version"] == base_s["version"] == 1
