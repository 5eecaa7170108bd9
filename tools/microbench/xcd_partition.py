"""Plane blocks fetched per XCD by the direct-staged θ-grad (form 10) at Cora
(n = 2708: 22 row tiles of 128, 253 upper-triangle tiles, one per CU): the
kernel's XCD-grouped order against the best partition of the tiles over the
8 XCDs (at most 32 each) that a local search over tile swaps finds.  Each
(tile row block) plane set is 17 chunks × 2 operands × 12 KB = 408 KB; a
tile (bi, bj) needs blocks bi and bj.  CPU only.
Usage: python tools/microbench/xcd_partition.py"""
import math
import random


def grouped_tile(L, nb, G):
    """csrc/thetagrad.hip grouped_tile: strips of G block columns."""
    s = 0
    while True:
        c1 = min((s + 1) * G, nb)
        if L < c1 * (c1 + 1) // 2:
            break
        s += 1
    c0 = s * G
    g = min(G, nb - c0)
    rem = L - c0 * (c0 + 1) // 2
    if rem < c0 * g:
        return rem // g, c0 + rem % g
    rem -= c0 * g
    i = c0
    while rem >= c0 + g - i:
        rem -= c0 + g - i
        i += 1
    return i, i + rem


def footprint(groups):
    return [len({b for t in g for b in t}) for g in groups]


def main(nb=22, xcds=8, iters=200000, seed=1):
    tiles = [(i, j) for j in range(nb) for i in range(j + 1)]
    per = (len(tiles) + xcds - 1) // xcds
    assign = {}
    for x in range(xcds):
        for q in range(per):
            if x * per + q < len(tiles):
                assign[grouped_tile(x * per + q, nb, 8)] = x

    def cost():
        groups = [[] for _ in range(xcds)]
        for t, x in assign.items():
            groups[x].append(t)
        return sum(footprint(groups)), groups

    cur, groups = cost()
    print("grouped order (G = 8): blocks per XCD", footprint(groups), "total", cur,
          f"= {cur * 408 / 1024:.1f} MB of planes")
    rng = random.Random(seed)
    best, best_groups, T = cur, groups, 2.0
    for _ in range(iters):
        t1, t2 = rng.sample(tiles, 2)
        x1, x2 = assign[t1], assign[t2]
        if x1 == x2:
            continue
        assign[t1], assign[t2] = x2, x1
        c, g = cost()
        if c <= cur or rng.random() < math.exp((cur - c) / T):
            cur = c
            if c < best:
                best, best_groups = c, g
        else:
            assign[t1], assign[t2] = x1, x2
        T = max(0.05, T * 0.99997)
    print("best found: blocks per XCD", footprint(best_groups), "total", best,
          f"= {best * 408 / 1024:.1f} MB of planes")


if __name__ == "__main__":
    main()
