#!/usr/bin/env python3
"""Discrete-event model of the lockstep combines (substrafl_amd/lockstep.py) on G GPUs.

Two uses:

* **Deadlock check** (tests/test_client_shard_cpu.py): every rank's kernels are played in the
  order ``lockstep.run`` issues them -- exchange group t, then the runs of step t -- under
  either stream model:
  ``queues="streams"``: the communicator's kernels on their own queue, the compute kernels on
  another (group t waits for what the compute stream held when it was issued, i.e. step t - 1's
  runs; step t's runs wait for group t - 1);
  ``queues="single"``: EVERY kernel of a rank on ONE in-order hardware queue (the worst case of
  streams sharing GPU_MAX_HW_QUEUES), so a blocked group blocks everything behind it.
  A group completes once each of its messages' peer group has started (the n-th send from q to
  r pairs with the n-th receive of r from q, whatever group either sits in).  The model reports
  a deadlock if some kernel can never start.
* **Timing estimate** (DESIGN.md §6): compute = elements x clients x bytes / HBM rate, a message
  = latency + bytes / link rate (messages to one peer in a group serialised, different peers in
  parallel, the two directions of a link independent), the gather to the root included.  Efficiency = one rank's compute alone / makespan.

    python3 tools/lockstep_model.py --gpus 8 --clients-per-gpu 64 --params 125000000
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path
from typing import Dict, List, Sequence

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from substrafl_amd import lockstep  # noqa: E402


class Deadlock(RuntimeError):
    pass


# chain-kernel rate (TB/s of client reads) against run length at 64 clients, fp32 rows, with the short-bucket
# tiles of shape_for: tools/chunk_probe.py on MI355X (profiles/r03_chunk_probe.log,
# r03f_chunk_probe_short_tiles.log; two sessions averaged where both measured)
RATE_CURVE = ((0.5e6, 5.96), (1.0e6, 6.80), (1.5e6, 6.62), (2.0e6, 7.02), (3.0e6, 6.67), (3.9e6, 6.84),
              (7.8e6, 6.87), (15.6e6, 6.80), (31.2e6, 6.63), (62.5e6, 6.93), (125e6, 6.89))


def rate_tbps(n: float, curve=RATE_CURVE) -> float:
    """Piecewise-linear in log(n); below the first point the rate falls in proportion to n (a
    fixed per-launch cost)."""
    import math

    if n <= curve[0][0]:
        return curve[0][1] * (n / curve[0][0]) ** 0.5
    for (n0, r0), (n1, r1) in zip(curve, curve[1:]):
        if n <= n1:
            f = (math.log(n) - math.log(n0)) / (math.log(n1) - math.log(n0))
            return r0 + f * (r1 - r0)
    return curve[-1][1]


def simulate(plans: Sequence[lockstep.RankPlan], queues: str = "streams", compute_s_per_elem: float = 1.0,
             link_s_per_elem: float = 0.0, latency_s: float = 0.0, run_time=None,
             overlap: float = 1.0) -> Dict[str, float]:
    """Play every rank's kernels; returns {"makespan", "compute_max"} or raises Deadlock.
    ``run_time(n)``: seconds of a step's launch over n elements (default n x compute_s_per_elem).
    ``overlap``: the fraction of exchange group t's own time (latency + its busiest link's bytes)
    that hides under step t's runs on the same rank; the rest is added to those runs (1.0: full
    overlap, the ideal; tools/executor_overlap_probe.py measures it on one GPU)."""
    if run_time is None:
        run_time = lambda n: n * compute_s_per_elem  # noqa: E731
    G = len(plans)
    kernels: List[List[dict]] = []
    for p in plans:
        ks = []
        for t in range(p.n_steps + 1):
            if p.groups[t]:
                ks.append({"kind": "group", "t": t, "ops": p.groups[t]})
            if t < p.n_steps and p.runs[t]:
                ks.append({"kind": "run", "t": t, "n": sum(r.n for r in p.runs[t])})
        kernels.append(ks)
    # pair the n-th send q->r with the n-th receive on r from q (NCCL's per-pair FIFO)
    seq: Dict[tuple, List[tuple]] = {}
    for r, ks in enumerate(kernels):
        for i, k in enumerate(ks):
            if k["kind"] != "group":
                continue
            for o in k["ops"]:
                key = (r, o.peer, "send") if o.kind == "send" else (o.peer, r, "recv")
                seq.setdefault(key, []).append((r, i, o.n))
    partner: Dict[tuple, tuple] = {}
    for (q, r, kind), lst in seq.items():
        if kind != "send":
            continue
        rl = seq.get((q, r, "recv"), [])
        if len(rl) != len(lst):
            raise Deadlock(f"{len(lst)} sends {q}->{r} but {len(rl)} receives")
        for (sq, si, sn), (rr, ri, rn) in zip(lst, rl):
            if sn != rn:
                raise Deadlock(f"message size mismatch {q}->{r}: {sn} vs {rn}")
            partner[(sq, si, "send", len([1 for x in lst if (x[0], x[1]) <= (sq, si)]))] = (rr, ri)
    # per group: the (peer rank, peer kernel index, elements) of each of its messages
    links: Dict[tuple, List[tuple]] = {}
    for (q, r, kind), lst in seq.items():
        if kind != "send":
            continue
        rl = seq[(q, r, "recv")]
        for (sq, si, sn), (rr, ri, _rn) in zip(lst, rl):
            links.setdefault((sq, si), []).append((rr, ri, sn, (r, "out")))
            links.setdefault((rr, ri), []).append((sq, si, sn, (q, "in")))

    start: Dict[tuple, float] = {}
    end: Dict[tuple, float] = {}
    ptr = [0] * G

    def deps(r: int, i: int):
        """Start dependencies of kernel i of rank r (None: not yet known)."""
        k = kernels[r][i]
        d = []
        if queues == "single":
            if i > 0:
                d.append((r, i - 1))
        else:
            same = [j for j in range(i) if (kernels[r][j]["kind"] == "group") == (k["kind"] == "group")]
            if same:
                d.append((r, same[-1]))
            if k["kind"] == "group":  # the compute stream's work issued before it (step t - 1)
                prior = [j for j in range(i) if kernels[r][j]["kind"] == "run"]
                if prior:
                    d.append((r, prior[-1]))
            else:  # step t waits for group t - 1
                prior = [j for j in range(i) if kernels[r][j]["kind"] == "group" and kernels[r][j]["t"] < k["t"]]
                if prior:
                    d.append((r, prior[-1]))
        return d

    progress = True
    while progress:
        progress = False
        for r in range(G):
            for i, k in enumerate(kernels[r]):
                if (r, i) not in start:
                    ds = deps(r, i)
                    if all(x in end for x in ds):
                        start[(r, i)] = max([end[x] for x in ds], default=0.0)
                        progress = True
                if (r, i) in start and (r, i) not in end:
                    if k["kind"] == "run":
                        extra = 0.0
                        if overlap < 1.0:  # the part of the concurrent group t that does not hide
                            gi = [j for j, g in enumerate(kernels[r]) if g["kind"] == "group" and g["t"] == k["t"]]
                            if gi:
                                per: Dict[tuple, int] = {}
                                for _pr, _pi, n, peer in links.get((r, gi[0]), []):
                                    per[peer] = per.get(peer, 0) + n
                                extra = (1.0 - overlap) * (latency_s + max(per.values(), default=0) * link_s_per_elem)
                        end[(r, i)] = start[(r, i)] + run_time(k["n"]) + extra
                        progress = True
                    else:
                        peers = links.get((r, i), [])
                        if all((pr, pi) in start for pr, pi, _n, _p in peers):
                            per_peer: Dict[tuple, int] = {}  # (peer, direction): links are full duplex
                            t0 = start[(r, i)]
                            for pr, pi, n, peer in peers:
                                per_peer[peer] = per_peer.get(peer, 0) + n
                                t0 = max(t0, start[(pr, pi)])
                            xfer = max(per_peer.values(), default=0) * link_s_per_elem
                            end[(r, i)] = t0 + latency_s + xfer
                            progress = True
    missing = [(r, i) for r in range(G) for i in range(len(kernels[r])) if (r, i) not in end]
    if missing:
        raise Deadlock(f"{len(missing)} kernels never complete (first: rank {missing[0][0]}, "
                       f"{kernels[missing[0][0]][missing[0][1]]['kind']} of step "
                       f"{kernels[missing[0][0]][missing[0][1]]['t']})")
    comp = max(sum(run_time(k["n"]) for k in ks if k["kind"] == "run") for ks in kernels)
    return {"makespan": max(end.values(), default=0.0), "compute_max": comp}


def simulate_push(plans: Sequence[lockstep.RankPlan], run_time, link_s_per_elem: float, launch_s: float = 2e-6,
                  order_s: float = 4e-6, streams: int = 4) -> Dict[str, float]:
    """The push executor (substrafl_amd/push.py): no exchange kernels.  Step t of rank r starts
    when its step t - 1 ended and every rank it waits for (push_schedule) ended step t - 2; its
    launches (one per consumer, the xGMI stores inside: a launch lasts at least its bytes over
    the one link it writes to) run round-robin on ``streams`` streams at once, so the step lasts
    the larger of its HBM work and its busiest stream's link time, plus its wait and signal
    kernels (order_s)."""
    from substrafl_amd.push import push_schedule

    G = len(plans)
    recvs = [[(g, o.peer, o.key, o.buf, o.n) for g, ops in enumerate(p.groups) for o in ops if o.kind == "recv"]
             for p in plans]
    progs = [push_schedule(p, recvs) for p in plans]
    S = plans[0].n_steps
    end = [[0.0] * S for _ in range(G)]
    dur = [[0.0] * S for _ in range(G)]
    deps = [[[] for _ in range(S + 1)] for _ in range(G)]
    for r, (specs, waits) in enumerate(progs):
        for t in range(S):
            launches = [s for s in specs if s.step == t]
            lanes = [0.0] * streams  # each stream's links, in series; the HBM work shared by all
            for i, s in enumerate(launches):
                lanes[i % streams] += (s.n * link_s_per_elem if s.dst_rank != r else 0.0) + launch_s
            dur[r][t] = max(sum(run_time(s.n) for s in launches), max(lanes)) if launches else 0.0
        for t, q, _v in waits:
            deps[r][t].append(q)
    for t in range(S):
        for r in range(G):
            start = end[r][t - 1] if t else 0.0
            for q in deps[r][t]:
                if t >= 2:
                    start = max(start, end[q][t - 2])
            end[r][t] = start + dur[r][t] + order_s
    makespan = max(max(end[r][S - 1] for r in range(G)), max(end[q][S - 1] for q in deps[plans[0].root][S]) if S else 0)
    comp = max(sum(run_time(s.n) for s in specs) for specs, _ in progs)
    return {"makespan": makespan, "compute_max": comp}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--clients-per-gpu", type=int, default=64)
    ap.add_argument("--params", type=int, default=125_000_000)
    ap.add_argument("--hbm-GBps", type=float, default=0.0,
                    help="bucket kernel read rate (0: RATE_CURVE, the measured rate against run length)")
    ap.add_argument("--link-GBps", type=float, default=50.0, help="one xGMI link, one direction")
    ap.add_argument("--latency-us", type=float, default=20.0, help="per exchange group")
    ap.add_argument("--chunk", type=int, default=2 << 20, help="relay chunk (elements)")
    ap.add_argument("--rings", type=int, default=0, help="striped chains (0: lockstep.ring_chains' default)")
    ap.add_argument("--overlap", type=float, default=1.0, help="fraction of a group's time hidden under the "
                    "concurrent step's runs (1: ideal; one-GPU probe with RCCL self P2P: ~0.3)")
    ap.add_argument("--push", action="store_true", help="model the push executor (no exchange kernels) instead")
    ap.add_argument("--from-line", default="", help="a bench.py --gpus N JSON line (file): take --gpus and the link "
                    "rate from its client_shard_torch_pg.xgmi_p2p probe (all-peers GB/s per link direction)")
    args = ap.parse_args()
    if args.from_line:
        line = json.loads([ln for ln in Path(args.from_line).read_text().splitlines() if ln.startswith("{")][-1])
        probe = (line.get("client_shard_torch_pg") or {}).get("xgmi_p2p") or {}
        rate = (probe.get("all_peers") or {}).get("GBps_per_link_direction")
        if not rate:
            raise SystemExit(f"{args.from_line}: no xgmi_p2p.all_peers rate in the line")
        args.gpus, args.link_GBps = int(line["n_gpus"]), float(rate)
    G, Kb, M = args.gpus, args.clients_per_gpu, args.params
    if args.hbm_GBps:
        rt = lambda n: n * Kb * 4 / (args.hbm_GBps * 1e9)  # noqa: E731
    else:
        rt = lambda n: n * Kb * 4 / (rate_tbps(n) * 1e12)  # noqa: E731
    link = 4 / (args.link_GBps * 1e9)
    out = {}
    schedules = {"relay": lockstep.relay_pieces(M, G, args.chunk)}
    for rounds in ((1.0,), (0.75, 0.25), (0.5, 0.3, 0.2), (0.4, 0.3, 0.2, 0.1), (0.6, 0.25, 0.15)):
        schedules[f"striped rounds={rounds}"] = lockstep.striped_pieces(M, G, args.rings or None, rounds)
    if args.push:
        for rounds in ((1.0,), (0.75, 0.25), (0.5, 0.3, 0.2)):
            plans = [lockstep.rank_plan(lockstep.striped_pieces(M, G, args.rings or None, rounds), G, r)
                     for r in range(G)]
            res = simulate_push(plans, rt, link)
            t1 = rt(M)
            out[f"push rounds={rounds}"] = {"steps": plans[0].n_steps, "model_ms": round(res["makespan"] * 1e3, 3),
                                            "single_gpu_ms": round(t1 * 1e3, 3),
                                            "weak_efficiency": round(t1 / res["makespan"], 3)}
        schedules = {}
    for name, pieces in schedules.items():
        plans = [lockstep.rank_plan(pieces, G, r, cols="global" if name == "relay" else "packed") for r in range(G)]
        res = simulate(plans, "streams", 0.0, link, args.latency_us * 1e-6, run_time=rt, overlap=args.overlap)
        t1 = rt(M)
        out[name] = {"steps": plans[0].n_steps, "model_ms": round(res["makespan"] * 1e3, 3),
                     "single_gpu_ms": round(t1 * 1e3, 3), "weak_efficiency": round(t1 / res["makespan"], 3)}
    print(json.dumps({"gpus": G, "clients_per_gpu": Kb, "params": M, "hbm_GBps": args.hbm_GBps,
                      "chains": len(lockstep.ring_chains(G, args.rings or None)),
                      "link_GBps": args.link_GBps, "latency_us": args.latency_us, "overlap": args.overlap,
                      "schedules": out}, indent=1))


if __name__ == "__main__":
    main()
