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
from substrafl_amd.push import push_schedule
from substrafl_amd.sharding import relay_plan, striped_plan


def _plans(M, G, rounds, relay, rings):
    if relay:
        return [relay_plan(M, G, r, 2048) for r in range(G)]
    return [striped_plan(M, G, r, rings, rounds) for r in range(G)]


def _programs(plans):
    recvs = [[(g, o.peer, o.key, o.buf, o.n) for g, ops in enumerate(p.groups) for o in ops if o.kind == "recv"]
             for p in plans]
    return [push_schedule(p, recvs) for p in plans]


def _ops(plan, specs, waits, base, root_fill):
    """One call of one rank as a list of events, in its stream's order."""
    ops = []
    if root_fill:
        ops.append(("fill",))
    ops.append(("signal", base + 1))
    by_step = {}
    for t, q, v in waits:
        by_step.setdefault(t, []).append(("wait", q, base + v))
    for t in range(plan.n_steps):
        ops += by_step.get(t, [])
        for s in (s for s in specs if s.step == t):
            ops += [("start", s), ("end", s)]
        ops.append(("signal", base + t + 2))
    ops += by_step.get(plan.n_steps, [])
    return ops


def _replay(plans, progs, M, calls, seed):
    G = len(plans)
    rng = random.Random(seed)
    root = plans[0].root
    slot_elems = max(max(1, p.slot_elems) for p in plans)
    bufs = [{"slot": np.full((lockstep.SLOTS, slot_elems), -1, np.int64), "out": np.full(M, -1, np.int64)}
            for _ in range(G)]
    progress = [0] * G
    for call in range(calls):
        expect = call + 1  # the call's tag: a value left over from the previous call never matches
        for b in range(G):
            expect = expect * (G + 1) + b + 1
        base = call * (plans[0].n_steps + 1)
        queues = [_ops(plans[r], *progs[r], base, r == root) for r in range(G)]
        pcs = [0] * G
        pending = [None] * G  # a started run's output, written at its end

        def region(r, loc, n):
            where, slot, off = loc
            return bufs[r]["out"][off: off + n] if where == "out" else bufs[r]["slot"][slot, off: off + n]

        while any(pcs[r] < len(queues[r]) for r in range(G)):
            ready = [r for r in range(G) if pcs[r] < len(queues[r])
                     and not (queues[r][pcs[r]][0] == "wait" and progress[queues[r][pcs[r]][1]] < queues[r][pcs[r]][2])]
            assert ready, f"deadlock (call {call}): {[queues[r][pcs[r]] if pcs[r] < len(queues[r]) else None for r in range(G)]}"
            r = rng.choice(ready)
            op = queues[r][pcs[r]]
            pcs[r] += 1
            if op[0] == "fill":
                bufs[r]["out"][:] = -7
            elif op[0] == "signal":
                progress[r] = op[1]
            elif op[0] == "start":
                s = op[1]
                x = region(r, s.src, s.n).copy() if s.src is not None else np.full(s.n, call + 1, np.int64)
                pending[r] = np.where(x < 0, -99, x * (G + 1) + s.block + 1)  # garbage stays garbage
            elif op[0] == "end":
                s = op[1]
                region(s.dst_rank, s.dst, s.n)[:] = pending[r]
                pending[r] = None
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


def test_push_runs_cover_every_output_once():
    """Every element a rank computes at a step goes to exactly one place: the consumer's receive
    location, or (finished) the root's output at its global offset."""
    M, G = 50000, 8
    plans = _plans(M, G, (0.5, 0.3, 0.2), False, None)
    for p, (specs, waits) in zip(plans, _programs(plans)):
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
                                                                  and not _is_producer(p, t, q))])
                for p, (specs, waits) in zip(plans, progs)]
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
    for p, (specs, waits) in zip(plans, progs):
        stripped.append((specs, [(t, q, v) for t, q, v in waits if t == p.n_steps]))  # only the root's end waits
    failures = 0
    for seed in range(20):
        try:
            _replay(plans, stripped, M, calls=2, seed=seed)
        except AssertionError:
            failures += 1
    assert failures > 0
