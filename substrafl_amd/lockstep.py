"""Lockstep schedules for the bit-exact client-sharded combines (the north-star
mode: "client buckets shard across the node's GPUs with an RCCL exchange over xGMI").

The reference's client sum is sequential per element (fed_avg.py:221-222; scaffold.py:262-263,
293): ``acc = +0.0; acc = fl(acc + fl(x_k * w_k))`` for k in list order.  With the K clients cut
into G contiguous blocks, an element stays bit-exact iff its accumulator visits the blocks 0..G-1
in order.  A :class:`Piece` is a contiguous element range whose accumulator does exactly that:
its block b runs on rank ``ranks[b]`` at step ``t0 + 2 b``.  What a rank computes at step t is
sent in exchange group t + 1 and consumed by the next rank at step t + 2, so a rank's kernel of
step t + 1 overlaps the transfer of what it computed at step t.

Deadlock freedom, whatever the GPU's hardware queues do: every rank issues its exchange groups
0, 1, 2, ... in order, from ONE host thread, on ONE communicator, and every point-to-point op of
group t pairs with an op of group t on its peer (a piece computed on q at step t - 1 is sent by q
in group t and received by r in ITS group t, for use at step t + 1).  Group t on a rank can then
complete once every peer has issued group t, which needs only that their groups < t completed:
by induction every group completes.  (The round-2 striped relay ran one host thread and one
communicator per stripe, whose blocking P2P kernels could be queued in different orders on
different ranks -- NCCL's documented deadlock pattern; this module replaces it.)

Two schedules:

* :func:`relay_pieces` -- the plain relay: every rank holds ONE client block for all elements
  (rank ``(b + 1) % G`` holds block b, the last block on the root), the bucket is cut into
  chunks that are pipelined down the chain.  The root idles while the chain fills: 2 (G - 1)
  steps out of C + 2 (G - 1).
* :func:`striped_pieces` -- the striped relay: the bucket is cut into rounds x 2 chunks x G
  stripes x R rings of pieces; piece (k, j, s, c) places block b on rank ``c[b] + s mod G`` for
  ring (chain) c of :func:`ring_chains`: the unit rings ``c[b] = a (b + 1)`` (a a unit of Z_G, the
  ring's hop length) or, at G = 6 and 8, Latin chains whose hops differ between the chains at
  every step.  At step ``2 G k + 2 p + j`` EVERY rank runs block p of one piece per ring --
  nobody idles, no fill -- and each rank sends on R distinct xGMI links at once (G = 8: six).
  A stripe's final chunks go from the rank that finished them to the root in the next exchange
  groups; the last round's are a tail (``rounds`` weights: a small last round shortens it, at
  the price of more steps).  Each rank holds one client block per stripe --
  K M / G elements, the same bytes as the plain layout.

The schedule is a pure function of (M, K, G, parameters), computed identically on every rank
(:func:`rank_plan`); :func:`run` executes one rank's part through any transport with an
``exchange(ops) -> works`` method (``torch.distributed`` RCCL / gloo, or the loopback of one
process).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

SLOTS = 4  # accumulator buffers per rank: step t uses slot t % 4 (written at t, sent in group t + 1,
# free once group t + 1 is waited at step t + 2; a receive of group t + 3 into it comes after that)
SHARD_ALIGN = 512  # elements: every piece starts on a 2-KiB (fp32) boundary
COL_ALIGN = 64  # elements: columns and slot offsets start 256-B aligned (the kernels' 16-B vector path
# needs every operand 16-B aligned; a ragged last piece must not shift the ones packed after it)


@dataclass(frozen=True)
class Piece:
    """Elements ``[lo, hi)``: block b runs on rank ``ranks[b]`` at step ``t0 + 2 b``."""

    lo: int
    hi: int
    ranks: Tuple[int, ...]
    t0: int


# ======================================================================================
# schedules
# ======================================================================================
def chain_rank(block: int, world: int) -> int:
    """Plain relay: block b on rank (b + 1) % G, so the LAST block sits on the root, rank 0."""
    return (block + 1) % world


def _align_up(n: int, a: int = SHARD_ALIGN) -> int:
    return -(-n // a) * a


def relay_pieces(M: int, G: int, chunk_elems: int) -> List[Piece]:
    """The plain relay: chunk j of ``[0, M)`` starts at step j on rank 1 and ends on the root."""
    step = max(SHARD_ALIGN, _align_up(chunk_elems))
    ranks = tuple(chain_rank(b, G) for b in range(G))
    return [Piece(a, min(M, a + step), ranks, j) for j, a in enumerate(range(0, M, step))]


def ring_units(G: int) -> List[int]:
    """The units of Z_G (ring hop lengths), alternating 1, G-1, 3, G-3, ... (G = 8: 1 7 3 5)."""
    import math

    lo = [a for a in range(1, G) if math.gcd(a, G) == 1] or [1]
    out, i, j = [], 0, len(lo) - 1
    while i <= j:
        out.append(lo[i])
        if j != i:
            out.append(lo[j])
        i, j = i + 1, j - 1
    return out


def ring_multipliers(G: int, rings: Optional[int] = None) -> List[int]:
    """One hop length per ring of the unit family (as many as Z_G has units, at most 4)."""
    u = ring_units(G)
    n = min(len(u), 4) if rings is None else max(1, min(int(rings), len(u)))
    return u[:n]


# Chains beyond the unit rings: G ranks visited in an order whose hop from block b to b + 1
# differs between the chains at EVERY b (the hop rows form a Latin rectangle over 1..G-1 and each
# row is a sequencing of Z_G: its partial sums visit every rank once), so at every step each rank
# sends on -- and receives from -- as many distinct links as there are chains, where the unit
# rings (constant hops 1, G-1, 3, G-3) give Z_G's units only: 4 of the 7 links at G = 8.  Found
# by tools/latin_rings.py (exhaustive over the (G-1)! chains; G = 6: all 5 links, G = 8: 6 of
# the 7, no 7th found; G <= 4 gains nothing over the units).  tools/lockstep_model.py, C3 weak at
# G = 8 with three rounds: 0.92 against 0.86 for the four unit rings at 50 GB/s per link direction,
# 0.84 against 0.78 at 40, equal from 65.
LATIN_HOPS = {
    6: ((1, 1, 1, 1, 1), (2, 5, 3, 5, 2), (3, 2, 2, 3, 4), (4, 3, 4, 4, 5), (5, 4, 5, 2, 3)),
    8: ((1, 1, 1, 1, 1, 1, 1), (2, 7, 2, 2, 7, 3, 7), (3, 6, 3, 6, 4, 7, 2), (4, 5, 4, 5, 5, 4, 3),
        (5, 2, 5, 7, 6, 5, 4), (6, 4, 7, 3, 3, 6, 6)),
}


def ring_chains(G: int, rings: Optional[int] = None) -> List[Tuple[int, ...]]:
    """The chains of the striped schedule: chain c places block b on rank ``c[b] + s mod G`` for
    stripe s.  Default: the Latin family where it has more chains than the unit rings (G = 6, 8),
    else the unit rings (``a (b + 1)``, at most 4).  ``rings=k``: the first k unit rings while
    Z_G has that many units, else the first k Latin chains."""
    units = ring_units(G)
    latin = LATIN_HOPS.get(G, ())
    n_units = min(len(units), 4)
    if rings is None:
        k, use_latin = (len(latin), True) if len(latin) > n_units else (n_units, False)
    else:
        k = max(1, int(rings))
        use_latin = k > len(units) and len(latin) > len(units)
        k = min(k, len(latin) if use_latin else len(units))
    if not use_latin:
        return [tuple((a * (b + 1)) % G for b in range(G)) for a in units[:k]]
    out = []
    for hops in latin[:k]:
        chain = [0]
        for h in hops:
            chain.append((chain[-1] + h) % G)
        out.append(tuple(chain))
    return out


def ring_hops(G: int, rings: Optional[int] = None) -> List[List[int]]:
    """Hop rows of :func:`ring_chains` (reporting: the links each chain uses, step by step)."""
    return [[(c[b + 1] - c[b]) % G for b in range(G - 1)] for c in ring_chains(G, rings)]


# Round split of the striped schedule.  More rounds shorten the last round's gather tail (each
# round's results travel under the next round's kernels) but add steps with shorter runs.  The Python
# executor keeps ONE round: 2 G steps, each long enough (C3 at G = 8: ~0.3 ms of HBM work) that
# issuing it from Python (~30 us per message) stays below its GPU time.  The native executor issues
# a step in microseconds and takes three (tools/lockstep_model.py, C3 weak at G = 8: 0.95 against
# 0.86 for one round at 65 GB/s per link direction, 0.96 against 0.88 at 80).
DEFAULT_ROUNDS = (1.0,)
NATIVE_ROUNDS = (0.5, 0.3, 0.2)


def default_rounds(world: int, native: bool) -> Tuple[float, ...]:
    """NATIVE_ROUNDS for the native executor over >= 2 ranks; one round otherwise (one rank has no
    gather to hide, and its runs are longest in one round)."""
    return NATIVE_ROUNDS if native and world > 1 else DEFAULT_ROUNDS


def striped_pieces(M: int, G: int, rings: Optional[int] = None,
                   rounds: Sequence[float] = DEFAULT_ROUNDS) -> List[Piece]:
    """The striped relay (module docstring).  ``rounds``: relative sizes of the rounds (the last
    round's final chunk is the gather tail, so it is the small one)."""
    chains = ring_chains(G, rings)
    R = len(chains)
    tot = float(sum(rounds)) or 1.0
    pieces: List[Piece] = []
    base = 0
    for k, wk in enumerate(rounds):
        Mk = M - base if k == len(rounds) - 1 else min(M - base, _align_up(int(M * wk / tot)))
        m = _align_up(max(1, -(-Mk // (2 * G * R)))) if Mk > 0 else 0
        for j in range(2):
            for f in range(G):  # the pieces that END on rank f at one step are adjacent in [0, M)
                for ai, chain in enumerate(chains):
                    lo = base + ((j * G + f) * R + ai) * m
                    hi = min(base + Mk, lo + m)
                    if hi > lo:
                        s = (f - chain[G - 1]) % G  # the stripe shift that ends this chain on f
                        ranks = tuple((chain[b] + s) % G for b in range(G))
                        pieces.append(Piece(lo, hi, ranks, 2 * G * k + j))
        base += Mk
    return pieces


# ======================================================================================
# one rank's view of a schedule
# ======================================================================================
@dataclass
class Run:
    """One launch: ``n`` elements of ``block`` starting at column ``col`` of this rank's buffer
    for that block, accumulator at ``acc`` = ("slot", slot, offset) or ("out", 0, global lo) --
    every final run accumulates in the rank's output buffer; ``lo``: global first element (the run
    is globally contiguous when ``final``)."""

    block: int
    col: int
    n: int
    lo: int
    acc: Tuple[str, int, int]
    seed: bool
    final: bool


@dataclass
class Op:
    """A point-to-point message of one exchange group: ``n`` elements at ``buf`` (as Run.acc)."""

    kind: str  # "send" | "recv"
    peer: int
    buf: Tuple[str, int, int]
    n: int
    key: int  # global lo of its first piece (the order of a pair's messages on both sides)


@dataclass
class RankPlan:
    rank: int
    world: int
    root: int
    runs: List[List[Run]]  # per step
    groups: List[List[Op]]  # per exchange group (group t is issued at step t, before step t's launches)
    blocks: Dict[int, List[Tuple[int, int, int]]]  # block -> [(lo, hi, col)] held by this rank
    block_len: Dict[int, int]  # block -> columns of this rank's buffer for it
    slot_elems: int
    n_pieces: int = 0
    stats: Dict[str, int] = field(default_factory=dict)

    @property
    def n_steps(self) -> int:
        return len(self.runs)


def _table(pieces: Sequence[Piece], G: int):
    """(rank, step) -> [(piece index, block)] sorted by lo; slot offsets per (rank, step, piece)."""
    tab: Dict[Tuple[int, int], List[Tuple[int, int]]] = {}
    for i, p in enumerate(pieces):
        if len(p.ranks) != G or sorted(p.ranks) != list(range(G)):
            raise ValueError("a piece's chain must visit every rank once")
        for b, r in enumerate(p.ranks):
            tab.setdefault((r, p.t0 + 2 * b), []).append((i, b))
    for v in tab.values():
        v.sort(key=lambda e: pieces[e[0]].lo)
    return tab


def rank_plan(pieces: Sequence[Piece], G: int, rank: int, root: int = 0, cols: str = "packed",
              gather_spread: int = 0) -> RankPlan:
    """This rank's runs and exchange groups.  ``cols="packed"``: the pieces a rank holds for a
    block lie back to back in its buffer for that block (in step order); ``"global"``: column =
    global element index (one block holding every element, the plain relay).

    A piece's LAST block accumulates straight into the output buffer of the rank running it (the
    root's is the result; another rank's holds its stripes' finished elements until they are
    sent).  A finished piece off the root goes to the root in ``gather_spread`` parts over the
    exchange groups that follow (0: 2 G groups -- a round's worth -- so round k's results travel
    under round k + 1's kernels instead of in one burst; the schedule's last groups take what is
    left)."""
    tab = _table(pieces, G)
    n_steps = 1 + max((p.t0 + 2 * (G - 1) for p in pieces), default=-1)
    spread = int(gather_spread) if gather_spread > 0 else 2 * G

    def is_final(t: int, i: int) -> bool:
        return t == pieces[i].t0 + 2 * (G - 1)

    def acc_loc(r: int, t: int, i: int) -> Tuple[str, int, int]:
        """Where rank r keeps piece i's accumulator at step t."""
        p = pieces[i]
        if is_final(t, i):
            return ("out", 0, p.lo)
        off = 0
        for j, _b in tab[(r, t)]:
            q = pieces[j]
            if j == i:
                return ("slot", t % SLOTS, off)
            if not is_final(t, j):
                off += _align_up(q.hi - q.lo, COL_ALIGN)
        raise AssertionError("piece not at (rank, step)")

    # columns of this rank's block buffers
    blocks: Dict[int, List[Tuple[int, int, int]]] = {}
    col_of: Dict[int, int] = {}
    for t in range(n_steps):
        for i, b in tab.get((rank, t), []):
            p = pieces[i]
            lst = blocks.setdefault(b, [])
            c = p.lo if cols == "global" else (lst[-1][2] + _align_up(lst[-1][1] - lst[-1][0], COL_ALIGN) if lst else 0)
            lst.append((p.lo, p.hi, c))
            col_of[i] = c
    block_len = {b: max(c + hi - lo for lo, hi, c in v) for b, v in blocks.items()}

    # runs: consecutive pieces of one block, contiguous in columns and accumulator, and (final)
    # globally contiguous (Scaffold's `+ c` reads c[lo : lo + n])
    runs: List[List[Run]] = []
    slot_elems = 0
    for t in range(n_steps):
        cur: List[Run] = []
        used = 0
        for i, b in tab.get((rank, t), []):
            p = pieces[i]
            n = p.hi - p.lo
            acc = acc_loc(rank, t, i)
            if acc[0] == "slot":
                used = max(used, acc[2] + n)
            final = b == G - 1
            if cur:
                last = cur[-1]
                if (last.block == b and last.col + last.n == col_of[i] and last.final == final
                        and last.acc[0] == acc[0] and last.acc[2] + last.n == acc[2]
                        and (not final or last.lo + last.n == p.lo)):
                    last.n += n
                    continue
            cur.append(Run(b, col_of[i], n, p.lo, acc, b == 0, final))
        slot_elems = max(slot_elems, used)
        runs.append(cur)

    # messages of every rank pair (computed globally, so both sides merge them identically)
    msgs: Dict[Tuple[int, int, int], List[Tuple[int, Tuple[str, int, int], Tuple[str, int, int], int]]] = {}
    for i, p in enumerate(pieces):
        n = p.hi - p.lo
        for b in range(G):
            q, t = p.ranks[b], p.t0 + 2 * b
            if b < G - 1:
                r = p.ranks[b + 1]
                msgs.setdefault((t + 1, q, r), []).append((p.lo, acc_loc(q, t, i), acc_loc(r, t + 2, i), n))
            elif q != root:  # the finished piece goes to the root's output, in parts over the next groups
                D = max(1, min(spread, n_steps - t))
                part = _align_up(-(-n // D), COL_ALIGN)
                for d, a in enumerate(range(p.lo, p.hi, part)):
                    e = min(p.hi, a + part)
                    msgs.setdefault((t + 1 + d, q, root), []).append((a, ("out", 0, a), ("out", 0, a), e - a))
    groups: List[List[Op]] = [[] for _ in range(n_steps + 1)]
    n_msgs = 0
    for (g, q, r), lst in sorted(msgs.items()):
        if rank not in (q, r):
            continue
        lst.sort(key=lambda e: e[0])
        merged: List[list] = []
        for lo, s, d, n in lst:
            if merged:
                m = merged[-1]
                if (m[1][0] == s[0] and m[1][1] == s[1] and m[1][2] + m[3] == s[2]
                        and m[2][0] == d[0] and m[2][1] == d[1] and m[2][2] + m[3] == d[2]):
                    m[3] += n
                    continue
            merged.append([lo, s, d, n])
        for lo, s, d, n in merged:
            n_msgs += 1
            if q == rank:
                groups[g].append(Op("send", r, s, n, lo))
            if r == rank:
                groups[g].append(Op("recv", q, d, n, lo))
    for grp in groups:
        grp.sort(key=lambda o: (o.peer, o.kind, o.key))
    return RankPlan(rank, G, root, runs, groups, blocks, block_len, slot_elems, len(pieces),
                    {"messages_of_this_rank": n_msgs})


# ======================================================================================
# execution
# ======================================================================================
def run(plan: RankPlan, transport, buffers: Callable[[Tuple[str, int, int], int], list],
        launch: Callable[[Run], None]) -> None:
    """Execute this rank's part: for t = 0, 1, ...: issue exchange group t (its sends read what
    step t - 1 computed, enqueued before it on the caller's stream; its receives fill buffers of
    step t + 1), make the compute stream wait for group t - 1 (the inputs of step t), launch step
    t.  ``buffers(loc, n)``: the tensors of a message (one for FedAvg, two for Scaffold's two
    accumulators); ``launch(run)``: enqueue one run on the current stream.  Every work a group
    returns is waited -- a batched exchange may return one work for the whole group."""
    prev: list = []
    for t in range(plan.n_steps + 1):
        ops = []
        for o in plan.groups[t]:
            for tensor in buffers(o.buf, o.n):
                ops.append((o.kind, tensor, o.peer))
        works = list(transport.exchange(ops)) if ops else []
        for w in prev:
            w.wait()
        if t < plan.n_steps:
            for r in plan.runs[t]:
                launch(r)
        prev = works
    for w in prev:
        w.wait()


def pairwise_segments(plan: RankPlan, pairwise_idx) -> List[Tuple[int, int, int, object]]:
    """The numel == 1 elements this rank holds: ``(block, p0, p1, local_columns)`` -- rows
    ``p0:p1`` of the sorted global list, at those columns of the block's buffer."""
    import numpy as np

    pw = np.asarray(pairwise_idx, np.int64)
    out = []
    if not pw.size:
        return out
    for b, segs in sorted(plan.blocks.items()):
        for lo, hi, col in segs:
            p0, p1 = int(np.searchsorted(pw, lo)), int(np.searchsorted(pw, hi))
            if p1 > p0:
                out.append((b, p0, p1, (pw[p0:p1] - lo + col).astype(np.uint64)))
    return out
