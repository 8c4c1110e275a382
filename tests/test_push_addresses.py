"""The push executor's resolved addresses (substrafl_amd/push.py: PushProgram), checked on the CPU
for every rank of a schedule at once -- the arithmetic a real node runs but one GPU cannot show
wrong: a producer computes addresses inside ANOTHER rank's slots, landing buffer, tags and staging
rows from that rank's published sizes.

Every rank's program is built in its own thread over a fake transport (per-rank address spaces
handed out by a fake libfedagg, IPC handles that resolve to them, all_gather over a barrier), then:

* every store of a run (its output range) and every load (its input accumulator) lies inside one
  allocation of the rank it targets -- an out-of-bounds push would write into a peer's memory;
* every input accumulator a run reads at step t was written, exactly, by the runs of step t - 2;
* no two runs of a step write overlapping ranges;
* the root's output [0, M) is written exactly once per accumulator: by its own final runs, or by a
  landing copy whose source the other ranks' final runs wrote;
* the landing tags and the numel == 1 staging rows land inside the consumer's / root's buffers.

Plans: relay and striped (1-3 rounds, unit rings and the G = 8 Latin chains), ragged sizes whose
ranks' slot sizes differ, FedAvg (fp32 accumulators) and Scaffold (two fp64 accumulators)."""

from __future__ import annotations

import threading

import numpy as np
import pytest
import torch

from substrafl_amd.layout import BucketLayout
from substrafl_amd.push import PushProgram
from substrafl_amd.sharding import FedAvgShard, ScaffoldShard, client_blocks, relay_plan, striped_plan

SPACE = 1 << 40  # rank r's fake device allocations live at [(r + 1) * SPACE, (r + 2) * SPACE)


class _FakeLib:
    """The allocations PushProgram makes through libfedagg, recorded per rank."""

    def __init__(self, rank: int, allocs: dict):
        self.rank, self.allocs, self.next = rank, allocs, (rank + 1) * SPACE

    def fedagg_device_alloc_uncached(self, nbytes, pref):
        addr = self.next
        self.next += -(-int(nbytes) // 4096) * 4096 + 4096  # a guard page between allocations
        self.allocs.setdefault(self.rank, []).append((addr, int(nbytes)))
        pref._obj.value = addr
        return 0

    def fedagg_device_free(self, ptr):
        return 0


class _Group:
    def __init__(self, G: int):
        self.G, self.barrier, self.slots = G, threading.Barrier(G, timeout=60), [None] * G


class _FakeTransport:
    """PushTransport's set-up surface: ipc_info / remote / all_gather over a thread group."""

    def __init__(self, group: _Group, rank: int, allocs: dict):
        self.group, self.rank, self.world = group, rank, group.G
        self.lib = _FakeLib(rank, allocs)

    def ipc_info(self, ptr: int):
        return (self.rank, int(ptr)), 0

    def remote(self, info, owner=None) -> int:
        (_owner, base), off = info
        if owner is not None:
            owner._handles.add((_owner, base))
        return base + off

    def all_gather(self, obj) -> list:
        g = self.group
        g.slots[self.rank] = obj
        g.barrier.wait()
        out = list(g.slots)
        g.barrier.wait()
        return out


def _build(G, K, M, relay, rounds, rings, scaffold, kind):
    shapes = [(M - 2,), (1,), (1, 1)]
    layout = BucketLayout(range(len(shapes)), shapes, np.float32)
    ld = layout.ld
    plans = [relay_plan(layout.M, G, r, 2048) if relay else striped_plan(layout.M, G, r, rings, rounds)
             for r in range(G)]
    group, allocs = _Group(G), {}
    progs, errs = [None] * G, []
    tdt = {"f64": torch.float64, "bf16": torch.bfloat16}.get(kind, torch.float32)

    def rank_fn(r):
        try:
            plan, tr = plans[r], _FakeTransport(group, r, allocs)
            blocks = {}
            for b in plan.blocks:
                k0, k1 = client_blocks(K, G)[b]
                rows = torch.zeros((k1 - k0, max(1, plan.block_len[b])), dtype=tdt)
                if scaffold:
                    blocks[b] = ScaffoldShard(kind, rows, rows.clone(), None, np.full(k1 - k0, 1.0 / K), k0, K,
                                              plan.block_len[b], 0.5, np.zeros(0, np.uint64))
                else:
                    blocks[b] = FedAvgShard(kind, rows, np.full(k1 - k0, 1.0 / K, np.float32), k0, K,
                                            plan.block_len[b], np.zeros(0, np.uint64))
            odt = torch.float64 if scaffold else torch.float32
            outs = [torch.zeros(ld, dtype=odt) for _ in range(2 if scaffold else 1)]
            c = torch.zeros(ld, dtype=tdt) if scaffold else None
            prog = PushProgram(tr, plan, blocks, [], outs, kind, scaffold, c=c, lr=0.5)
            ws_bytes = 3 * K * 8
            prog.ws_row = prog.ws_dst(ws_bytes)  # collective
            progs[r] = (prog, outs, c)
        except BaseException as e:  # noqa: BLE001 -- reported by the test
            errs.append((r, repr(e)))
            group.barrier.abort()

    threads = [threading.Thread(target=rank_fn, args=(r,)) for r in range(G)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errs, errs
    return plans, progs, allocs, layout


def _owner(addr: int, nbytes: int, regions) -> int:
    """Index of the region holding [addr, addr + nbytes), else -1."""
    for i, (a, n) in enumerate(regions):
        if a <= addr and addr + nbytes <= a + n:
            return i
    return -1


CASES = [
    # G, K, M, relay, rounds, rings, scaffold, kind
    (2, 3, 9361, False, (1.0,), None, False, "f32"),
    (3, 4, 9361, False, (0.5, 0.3, 0.2), None, False, "f32"),
    (4, 5, 4099, False, (0.5, 0.3, 0.2), None, False, "f32"),  # ragged: slot sizes 512 / 1024
    (4, 5, 4099, False, (0.5, 0.3, 0.2), None, True, "f32"),
    (4, 9, 9361, True, (1.0,), None, False, "f32"),
    (5, 6, 4099, False, (1.0,), None, True, "f64"),  # ragged: 515 / 1024 / 1027
    (8, 9, 4099, False, (1.0,), None, False, "f32"),  # Latin chains, eight different slot sizes
    (8, 9, 70001, False, (0.5, 0.3, 0.2), None, True, "f32"),
    (8, 16, 70001, False, (1.0,), 2, False, "bf16"),
    (8, 9, 30000, True, (1.0,), None, True, "f64"),
]


@pytest.mark.parametrize("G,K,M,relay,rounds,rings,scaffold,kind", CASES)
def test_push_program_addresses(G, K, M, relay, rounds, rings, scaffold, kind):
    plans, progs, allocs, layout = _build(G, K, M, relay, rounds, rings, scaffold, kind)
    nacc, esz = (2, 8) if scaffold else (1, 4)
    root = plans[0].root
    # every rank's memory: its fake allocations, its outputs (real host tensors) and c
    regions = {r: list(allocs.get(r, [])) + [(o.data_ptr(), o.numel() * o.element_size()) for o in progs[r][1]]
               for r in range(G)}

    def rank_of(addr, nbytes):
        hits = [r for r in range(G) if _owner(addr, nbytes, regions[r]) >= 0]
        assert len(hits) == 1, (hex(addr), nbytes, hits)
        return hits[0]

    writes = {}  # step -> list of (lo, hi, writer rank, target rank) byte ranges written
    for r in range(G):
        prog = progs[r][0]
        for i in range(prog.nruns):
            run = prog.runs[i]
            nb = int(run.n) * esz
            dst_rank = rank_of(int(run.acc), nb)  # inside exactly one allocation of one rank
            writes.setdefault(int(run.step), []).append((int(run.acc), int(run.acc) + nb, r, dst_rank))
            if run.acc2:
                assert rank_of(int(run.acc2), nb) == r  # the input accumulator is this rank's own slot
    # no two runs of one step write overlapping bytes
    for t, ws in writes.items():
        ws = sorted(ws)
        for (a0, a1, *_), (b0, b1, *_) in zip(ws, ws[1:]):
            assert a1 <= b0, (t, hex(a0), hex(b0))
    # every input accumulator read at step t was written, exactly, at step t - 2
    for r in range(G):
        prog = progs[r][0]
        for i in range(prog.nruns):
            run = prog.runs[i]
            if not run.acc2:
                continue
            lo, hi = int(run.acc2), int(run.acc2) + int(run.n) * esz
            src = sorted((a, b) for a, b, _q, _d in writes.get(int(run.step) - 2, []) if a < hi and b > lo)
            pos = lo
            for a, b in src:
                assert a <= pos, ("gap in the input accumulator", r, int(run.step), hex(pos), hex(a))
                pos = max(pos, b)
            assert pos >= hi, ("input accumulator not fully written", r, int(run.step))
    # the root's outputs: own final runs + landing copies cover [0, M) once per accumulator
    prog, outs, _c = progs[root]
    for w in range(nacc):
        o0 = outs[w].data_ptr()
        cover = np.zeros(layout.M, np.int32)
        for a, b, _q, d in (x for ws in writes.values() for x in ws):
            if d == root and o0 <= a < o0 + layout.ld * esz:
                cover[(a - o0) // esz: min(layout.M, (b - o0) // esz)] += 1
        for i in range(prog.ncopies):
            cp = prog.copies[i]
            if o0 <= int(cp.dst) < o0 + layout.ld * esz:
                n = int(cp.bytes) // esz
                s0 = (int(cp.dst) - o0) // esz
                cover[s0: min(layout.M, s0 + n)] += 1
                # its source: the root's landing buffer, written there by other ranks' final runs
                land = [x for ws in writes.values() for x in ws if x[3] == root and x[2] != root
                        and x[0] < int(cp.src) + int(cp.bytes) and x[1] > int(cp.src)]
                got = sum(min(b, int(cp.src) + int(cp.bytes)) - max(a, int(cp.src)) for a, b, _q, _d in land)
                want = min(int(cp.bytes), max(0, (layout.M - s0) * esz))
                assert got >= want, ("landing copy reads bytes nobody pushed", w, s0, got, want)
        assert cover.min() == 1 and cover.max() == 1, (w, np.unique(cover, return_counts=True))
    # landing tags and staging rows: inside the consumer's / root's allocations
    for r in range(G):
        prog = progs[r][0]
        for i in range(prog.ntags):
            assert rank_of(int(prog.tags[i].tag), 8) != r
        for i in range(prog.nwaits):
            if prog.waits[i].tag:
                assert rank_of(int(prog.waits[i].tag), 8) == r
        assert rank_of(prog.ws_row, 3 * K * 8) == root
    rows = sorted(progs[r][0].ws_row for r in range(G))
    assert all(b - a >= 3 * K * 8 for a, b in zip(rows, rows[1:]))



def _random_cases(n, seed=20241018):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        G = int(rng.integers(2, 9))
        relay = bool(rng.random() < 0.3)
        rounds = [(1.0,), (0.75, 0.25), (0.5, 0.3, 0.2), (0.4, 0.3, 0.2, 0.1)][int(rng.integers(0, 4))]
        rings = None if rng.random() < 0.7 else int(rng.integers(1, 5))
        scaffold = bool(rng.random() < 0.5)
        kind = ("f32", "f64")[int(rng.integers(0, 2))] if scaffold else ("f32", "bf16")[int(rng.integers(0, 2))]
        out.append((G, G + int(rng.integers(0, 9)), int(rng.integers(1_000, 120_000)), relay, rounds, rings,
                    scaffold, kind))
    return out


@pytest.mark.parametrize("G,K,M,relay,rounds,rings,scaffold,kind", _random_cases(24))
def test_push_program_addresses_random_plans(G, K, M, relay, rounds, rings, scaffold, kind):
    """The same checks over seeded random plans: ranks, clients, sizes, rounds, ring counts."""
    test_push_program_addresses(G, K, M, relay, rounds, rings, scaffold, kind)


@pytest.mark.parametrize("G,K,M,relay,rounds,rings,scaffold,kind", [CASES[1], CASES[3], CASES[7], CASES[9]])
def test_push_program_rebased_to_new_outputs(G, K, M, relay, rounds, rings, scaffold, kind):
    """A call with the same plan and blocks but outputs at new addresses reuses the program on
    EVERY rank (the decision cannot differ between ranks: a miss compiles collectively), and the
    root's launches and landing copies that wrote the old outputs write the new ones at the same
    offsets; nothing else moves."""
    plans, progs, allocs, layout = _build(G, K, M, relay, rounds, rings, scaffold, kind)
    for r in range(G):
        prog, outs, c = progs[r]
        fresh = [torch.zeros_like(o) for o in outs]
        kw = dict(plan=prog.plan, blocks=prog.blocks, accs=[], outs=fresh, kind=kind, scaffold=scaffold, c=c, lr=0.5)
        assert prog.matches(**kw), r
        assert not prog.matches(**dict(kw, outs=[torch.zeros(o.numel() + 1, dtype=o.dtype) for o in outs]))
        span = layout.ld * outs[0].element_size()
        old = [o.data_ptr() for o in outs]

        def expect(addr):
            for o, f in zip(old, fresh):
                if addr and o <= addr < o + span:
                    return addr - o + f.data_ptr()
            return addr

        want_runs = [(expect(prog.runs[i].acc), prog.runs[i].acc2) for i in range(prog.nruns)]
        want_copies = [(expect(prog.copies[i].dst), prog.copies[i].src) for i in range(prog.ncopies)]
        moved = sum(1 for i in range(prog.nruns) if want_runs[i][0] != prog.runs[i].acc)
        moved += sum(1 for i in range(prog.ncopies) if want_copies[i][0] != prog.copies[i].dst)
        assert moved > 0 or r != plans[r].root, (r, moved)  # the root writes its outputs
        prog.rebase_outs(fresh)
        assert [(prog.runs[i].acc, prog.runs[i].acc2) for i in range(prog.nruns)] == want_runs
        assert [(prog.copies[i].dst, prog.copies[i].src) for i in range(prog.ncopies)] == want_copies
        prog.rebase_outs(fresh)  # same addresses: a no-op
        assert [(prog.runs[i].acc, prog.runs[i].acc2) for i in range(prog.nruns)] == want_runs
