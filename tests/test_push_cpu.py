"""The push executor's protocol (substrafl_amd/push.py: push_schedule) checked on the CPU.

Every rank's compiled push runs and waits are replayed symbolically under random interleavings
of the ranks: a run snapshots its input accumulator when it starts and writes its output when it
ends (other ranks' events may fall in between, as kernels overlap), a wait blocks until the
counter it names reaches its value, a signal publishes the step.  An accumulator is a number
that records the call and the blocks applied to it in order (seeded with the call's number,
then acc * (G + 1) + block + 1), so a lost update, a
read of a slot before its data landed or after the next step's data overwrote it, or a block
applied out of order changes the root's result.  The root refills its output before every call
(the GPU test does), so a peer that pushed into it before the root entered the call is caught
too.  No interleaving may deadlock."""

from __future__ import annotations

import random

import numpy as np
import pytest

from substrafl_amd import lockstep
from substrafl_amd.push import push_outgoing, push_schedule, push_tag_waits
from substrafl_amd.sharding import relay_plan, striped_plan


class TagTimeout(AssertionError):
    """A rank is stuck on a landing tag that can never arrive (the executor's wait kernel times out
    and the host raises on the error word instead of computing with what is in the buffer)."""


def _plans(M, G, rounds, relay, rings):
    if relay:
        return [relay_plan(M, G, r, 2048) for r in range(G)]
    return [striped_plan(M, G, r, rings, rounds) for r in range(G)]


def _programs(plans):
    """Per rank: (specs, counter waits, landing tags written, landing-tag waits) -- push.py's."""
    recvs = [[(g, o.peer, o.key, o.buf, o.n) for g, ops in enumerate(p.groups) for o in ops if o.kind == "recv"]
             for p in plans]
    sched = [push_schedule(p, recvs) for p in plans]
    outgoing = [push_outgoing(p, specs) for p, (specs, _w) in zip(plans, sched)]
    return [(specs, waits, outgoing[p.rank], push_tag_waits(p.rank, p.n_steps, outgoing))
            for p, (specs, waits) in zip(plans, sched)]


def _ops(plan, specs, waits, outgoing, tag_waits, base, root_fill):
    """One call of one rank as a list of events, in its stream's order."""
    ops = []
    if root_fill:
        ops.append(("fill",))
    ops.append(("signal", base + 1, []))
    by_step = {}
    for t, q, v in waits:
        by_step.setdefault(t, []).append(("wait", q, base + v))
    for t, q, v, idx in tag_waits:
        by_step.setdefault(t, []).append(("twait", q, base + v, idx))
    tags_of = {}
    for t, c, _e in outgoing:
        tags_of.setdefault(t, []).append((c, plan.rank * plan.n_steps + t))
    for t in range(plan.n_steps):
        ops += by_step.get(t, [])
        for s in (s for s in specs if s.step == t):
            ops += [("start", s), ("end", s)]
        ops.append(("signal", base + t + 2, tags_of.get(t, [])))
    ops += by_step.get(plan.n_steps, [])
    return ops


def _replay(plans, progs, M, calls, seed, delay=False, drop=None):
    """Random interleavings of the ranks' event lists.  ``delay``: a store into a peer's memory is
    in flight on its (producer, consumer) link until a random later ``land`` event, in order per
    link, while the counter a signal publishes is visible at once (it travels over another path) --
    the ordering gap the landing tags close; the signal's tag writes follow the step's data on each
    link.  ``drop = (rank, step, consumer)``: that rank's step-``step`` stores to ``consumer`` and
    their tag never land (a lost piece) in the last call."""
    G = len(plans)
    rng = random.Random(seed)
    root = plans[0].root
    slot_elems = max(max(1, p.slot_elems) for p in plans)
    bufs = [{"slot": np.full((lockstep.SLOTS, slot_elems), -1, np.int64), "out": np.full(M, -1, np.int64)}
            for _ in range(G)]
    tags = [dict() for _ in range(G)]
    progress = [0] * G
    links = {}  # (producer, consumer) -> FIFO of pending writes
    for call in range(calls):
        expect = call + 1  # the call's tag: a value left over from the previous call never matches
        for b in range(G):
            expect = expect * (G + 1) + b + 1
        base = call * (plans[0].n_steps + 1)
        gen = base + 1
        queues = [_ops(plans[r], progs[r][0], progs[r][1], progs[r][2], progs[r][3], base, r == root)
                  for r in range(G)]
        pcs = [0] * G
        pending = [None] * G  # a started run's output, written at its end

        def region(r, loc, n):
            where, slot, off = loc
            return bufs[r]["out"][off: off + n] if where == "out" else bufs[r]["slot"][slot, off: off + n]

        def post(src, dst, write, step):
            if drop is not None and call == calls - 1 and (src, step, dst) == drop:
                return  # lost on the link
            if delay and src != dst:
                links.setdefault((src, dst), []).append(write)
            else:
                write()

        def blocked(r):
            op = queues[r][pcs[r]]
            if op[0] == "wait":
                return progress[op[1]] < op[2]
            if op[0] == "twait":
                return progress[op[1]] < op[2] or tags[r].get(op[3], 0) < gen
            return False

        while any(pcs[r] < len(queues[r]) for r in range(G)):
            ready = [r for r in range(G) if pcs[r] < len(queues[r]) and not blocked(r)]
            inflight = [k for k, v in links.items() if v]
            if not ready and not inflight:
                stuck = [queues[r][pcs[r]] for r in range(G) if pcs[r] < len(queues[r])]
                if any(op[0] == "twait" for op in stuck):
                    raise TagTimeout(f"call {call}: stuck on a landing tag: {stuck}")
                raise AssertionError(f"deadlock (call {call}): {stuck}")
            if inflight and (not ready or rng.random() < 0.5):
                write = links[rng.choice(inflight)].pop(0)
                write()
                continue
            r = rng.choice(ready)
            op = queues[r][pcs[r]]
            pcs[r] += 1
            if op[0] == "fill":
                bufs[r]["out"][:] = -7
            elif op[0] == "signal":
                step = op[1] - base - 2
                for c, idx in op[2]:
                    post(r, c, lambda c=c, idx=idx: tags[c].__setitem__(idx, gen), step)
                progress[r] = op[1]
            elif op[0] == "start":
                s = op[1]
                x = region(r, s.src, s.n).copy() if s.src is not None else np.full(s.n, call + 1, np.int64)
                pending[r] = np.where(x < 0, -99, x * (G + 1) + s.block + 1)  # garbage stays garbage
            elif op[0] == "end":
                s = op[1]
                val = pending[r]

                def write(s=s, val=val):
                    region(s.dst_rank, s.dst, s.n)[:] = val

                post(r, s.dst_rank, write, s.step)
                pending[r] = None
        assert not any(links.values())
        got = bufs[root]["out"][:M]
        bad = int(np.count_nonzero(got != expect))
        assert bad == 0, f"call {call}: {bad} of {M} elements wrong (seed {seed})"


@pytest.mark.parametrize("M,G,rounds,relay,rings", [
    (20000, 2, (1.0,), False, None),
    (30000, 3, (0.5, 0.3, 0.2), False, None),
    (40000, 4, (0.75, 0.25), False, 2),
    (30000, 4, (1.0,), True, None),
    (60000, 6, (0.5, 0.3, 0.2), False, None),   # Latin chains
    (70000, 8, (0.5, 0.3, 0.2), False, None),   # the bench's schedule at 8 GPUs (six Latin chains)
    (50000, 8, (1.0,), False, 4),               # unit rings
])
def test_push_protocol_random_interleavings(M, G, rounds, relay, rings):
    plans = _plans(M, G, rounds, relay, rings)
    progs = _programs(plans)
    for seed in range(12 if G <= 4 else 4):
        _replay(plans, progs, M, calls=2, seed=seed)
        # the stores in flight on their links after the counters (the ordering gap): the tags hold
        _replay(plans, progs, M, calls=2, seed=100 + seed, delay=True)


def test_push_runs_cover_every_output_once():
    """Every element a rank computes at a step goes to exactly one place: the consumer's receive
    location, or (finished) the root's output at its global offset."""
    M, G = 50000, 8
    plans = _plans(M, G, (0.5, 0.3, 0.2), False, None)
    for p, (specs, waits, _o, _tw) in zip(plans, _programs(plans)):
        assert sum(s.n for s in specs) == sum(r.n for runs in p.runs for r in runs)
        for s in specs:
            if s.block == G - 1:  # finished: the root's output (the last block's input sits in "out" too)
                assert s.dst_rank == p.root and s.dst[0] == "out"
            else:
                assert s.dst_rank != p.rank
        assert all(v >= 1 for _t, _q, v in waits)
        assert all(q != p.rank for _t, q, _v in waits)


def test_push_entry_wait_protects_the_refilled_output():
    """Dropping only the waits for the root's entry (step 0 and the finished pieces' pushes) lets a
    peer push into the root's output before the root's refill ran, in some interleaving."""
    M, G = 20000, 2
    plans = _plans(M, G, (1.0,), False, None)
    progs = _programs(plans)
    root = plans[0].root
    stripped = [(specs, [(t, q, v) for t, q, v in waits if not (q == root and p.rank != root and v == max(t, 1)
                                                                  and not _is_producer(p, t, q))], o, tw)
                for p, (specs, waits, o, tw) in zip(plans, progs)]
    failures = 0
    for seed in range(30):
        try:
            _replay(plans, stripped, M, calls=2, seed=seed)
        except AssertionError:
            failures += 1
    assert failures > 0


def _is_producer(plan, t, q) -> bool:
    """Whether q sent this rank an input of step t (a receive of group t - 1 from q)."""
    return t >= 1 and any(o.kind == "recv" and o.peer == q for o in plan.groups[t - 1])


def test_push_waits_catch_a_missing_wait():
    """The replay is sharp: without the step waits a fast rank reads a slot before its data
    landed, or overwrites one (or the root's refilled output) before it was read, and some
    interleaving shows it."""
    M, G = 30000, 3
    plans = _plans(M, G, (0.5, 0.3, 0.2), False, None)
    progs = _programs(plans)
    stripped = []
    for p, (specs, waits, o, _tw) in zip(plans, progs):
        stripped.append((specs, [(t, q, v) for t, q, v in waits if t == p.n_steps], o, []))  # only the root's end waits
    failures = 0
    for seed in range(20):
        try:
            _replay(plans, stripped, M, calls=2, seed=seed)
        except AssertionError:
            failures += 1
    assert failures > 0


@pytest.mark.parametrize("relay", [False, True])
def test_counters_alone_miss_late_data(relay):
    """Without the landing tags, a store still in flight on its link when the producer's counter
    is published is read stale in some interleaving: the gap is real in this model, and the tags
    are what closes it (test_push_protocol_random_interleavings)."""
    M, G = 30000, 4
    plans = _plans(M, G, (0.5, 0.5), relay, None)
    progs = [(specs, waits, o, []) for specs, waits, o, _tw in _programs(plans)]
    failures = 0
    for seed in range(30):
        try:
            _replay(plans, progs, M, calls=2, seed=seed, delay=True)
        except AssertionError:
            failures += 1
    assert failures > 0


@pytest.mark.parametrize("relay", [False, True])
def test_landing_tags_reject_a_dropped_piece(relay):
    """A push that never lands (its data and its tag lost on the link) stops the consumer at that
    tag -- the executor's wait times out and the host raises (PushTransport.execute / errors()) --
    instead of letting it compute with what the buffer held.  Every (rank, step, consumer) push is
    dropped in turn on a small schedule."""
    M, G = 12000, 3
    plans = _plans(M, G, (1.0,), relay, None)
    progs = _programs(plans)
    pushes = [(r, t, c) for r, (_s, _w, o, _tw) in enumerate(progs) for t, c, _e in o]
    assert pushes
    for i, drop in enumerate(pushes):
        with pytest.raises(TagTimeout):
            _replay(plans, progs, M, calls=2, seed=i, delay=True, drop=drop)


def test_tag_waits_point_to_earlier_steps():
    """Every landing-tag wait names another rank's strictly earlier step (the deadlock argument),
    and every tag a rank writes is waited for by its consumer exactly once."""
    M, G = 50000, 8
    plans = _plans(M, G, (0.5, 0.3, 0.2), False, None)
    progs = _programs(plans)
    written = {(r, t, c) for r, (_s, _w, o, _tw) in enumerate(progs) for t, c, _e in o}
    waited = set()
    for p, (_s, _w, _o, tw) in zip(plans, progs):
        for t_wait, q, v, idx in tw:
            t_push = idx - q * p.n_steps
            assert q != p.rank and t_push < t_wait and v == t_push + 2
            waited.add((q, t_push, p.rank))
    assert waited == written


def test_raise_errors_reports_a_timed_out_wait():
    """A wait kernel that gave up leaves its rank's error word set in the shared page: the root's
    check after synchronising (sharding._raise_transport_errors) raises instead of returning the
    numbers computed without the data."""
    from substrafl_amd import _native
    from substrafl_amd.push import PushTransport
    from substrafl_amd.sharding import _raise_transport_errors

    tr = PushTransport.__new__(PushTransport)
    tr.world = 3
    tr._page = np.zeros(3 * tr.world, dtype=np.uint64)
    _raise_transport_errors(tr)  # clean page: nothing to report
    tr._page[tr.world + 2] = 1 + 0  # rank 2 gave up on rank 0's counter
    with pytest.raises(_native.NativeLibraryError, match="counter of rank 0"):
        _raise_transport_errors(tr)
    tr._page[tr.world + 2] = (1 << 32) + 1 + 1  # ... or on rank 1's landing tag
    assert tr.errors() == {2: "landing tag of rank 1"}
    with pytest.raises(_native.NativeLibraryError, match="landing tag of rank 1"):
        tr.raise_errors()
    _raise_transport_errors(object())  # transports without a record of their own: no-op


def test_settle_waits_for_the_group_or_its_failure():
    """a rank whose own part of a push call is done learns from the shared page whether
    the GROUP's call finished (every rank's progress counter at the call's end value) or failed (an
    err word set) before it meets its peers again -- a failed call runs no collective release (a
    dead peer would never meet it) and frees no program buffer."""
    import threading
    import time

    from substrafl_amd import _native
    from substrafl_amd.push import PushTransport

    tr = PushTransport.__new__(PushTransport)
    tr.world, tr.base, tr._timeout_s, tr._programs = 3, 7, 2.0, []
    tr._page = np.zeros(3 * tr.world, dtype=np.uint64)
    tr._page[:3] = 7
    t0 = time.monotonic()
    tr.settle()  # every counter at the call's end value: done at once
    assert time.monotonic() - t0 < 0.5 and not tr.failed()
    tr._page[1] = 5  # rank 1 stopped short; rank 2's wait gives up 0.2 s later

    def give_up():
        time.sleep(0.2)
        tr._page[tr.world + 2] = 1 + 1  # rank 2 gave up on rank 1's counter

    th = threading.Thread(target=give_up)
    th.start()
    t0 = time.monotonic()
    tr.settle()
    th.join()
    assert 0.15 < time.monotonic() - t0 < 1.5
    assert tr.failed()
    with pytest.raises(_native.NativeLibraryError, match="counter of rank 1"):
        tr.raise_errors()
    tr._programs = ["program"]
    tr.device = None
    import torch

    orig = torch.cuda.synchronize
    torch.cuda.synchronize = lambda *a: None
    try:
        tr.release_programs()  # failed: no barrier (tr has no process group at all), nothing freed
    finally:
        torch.cuda.synchronize = orig
    assert tr._programs == [] and "program" in __import__("substrafl_amd.push", fromlist=["_ABANDONED"])._ABANDONED
    # a rank that neither finishes nor reports a failure within the timeout: failed as well
    tr2 = PushTransport.__new__(PushTransport)
    tr2.world, tr2.base, tr2._timeout_s = 2, 3, 0.0
    tr2._page = np.zeros(3 * tr2.world, dtype=np.uint64)
    tr2.settle()  # waits the 5 s margin
    assert tr2.failed()
    with pytest.raises(_native.NativeLibraryError, match="neither finished"):
        tr2.raise_errors()
