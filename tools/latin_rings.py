#!/usr/bin/env python3
"""Search for the striped schedule's Latin chains (substrafl_amd/lockstep.py, ``LATIN_HOPS``).

A chain visits the G ranks in some order; its hop row is ``h[b] = chain[b + 1] - chain[b] mod G``.
R chains use R distinct links of every rank at every step iff, for every b, the R hops ``h[b]``
are distinct (a Latin rectangle over 1..G-1 whose rows are sequencings of Z_G).  This is a
maximum-clique search over the (G-1)! chains starting at rank 0 (two chains are compatible when no
column repeats a hop), branching on the rows that hold the smallest hop still missing in column 0.

    python3 tools/latin_rings.py 8 --seconds 150
"""

from __future__ import annotations

import argparse
import itertools
import sys
import time


def search(G: int, seconds: float):
    rows = []
    for p in itertools.permutations(range(1, G)):
        chain = (0,) + p
        rows.append(tuple((chain[b + 1] - chain[b]) % G for b in range(G - 1)))
    n = len(rows)
    holder = {}
    for i, r in enumerate(rows):
        for b, h in enumerate(r):
            holder[(b, h)] = holder.get((b, h), 0) | (1 << i)
    full = (1 << n) - 1
    comp = []
    for r in rows:
        bad = 0
        for b, h in enumerate(r):
            bad |= holder[(b, h)]
        comp.append(full & ~bad)
    best = []
    t0 = time.time()

    def dfs(chosen, cand, missing):
        nonlocal best
        if len(chosen) > len(best):
            best = list(chosen)
            if len(best) == G - 1:
                return True
        if time.time() - t0 > seconds or not missing:
            return time.time() - t0 > seconds
        if len(chosen) + bin(cand).count("1") <= len(best):
            return False
        v = min(missing)
        branch = cand & holder[(0, v)]
        while branch:
            low = branch & -branch
            i = low.bit_length() - 1
            branch ^= low
            if dfs(chosen + [i], cand & comp[i], missing - {v}):
                return True
        return False

    dfs([], full, set(range(1, G)))
    # proven maximal when every link is used, or when the search ran to the end
    complete = len(best) == G - 1 or time.time() - t0 <= seconds
    return [rows[i] for i in best], complete


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("G", type=int)
    ap.add_argument("--seconds", type=float, default=60.0)
    a = ap.parse_args()
    hops, complete = search(a.G, a.seconds)
    print(f"G = {a.G}: {len(hops)} chains ({'search complete' if complete else 'time limit reached'})")
    for h in hops:
        print(" ", h)
    return 0


if __name__ == "__main__":
    sys.exit(main())
