"""Tail study of the headline workload: replay every chain's measured per-iteration work
(gpurun_out/chain_work.npz from scripts/chain_work.py) through a fluid model of the
migrating launch -- 256 tiles of 4 NUTS slots, a chain in a tile hosting k chains advances
at RATE[k] gradients per unit time, chains move between tiles only at iteration boundaries
-- and compare migration policies by their makespan.

RATE is the per-chain gradient rate by occupancy, relative, from the profiling build's tile
occupancy (sweeps share / time share of tiles hosting k chains, divided by k; the k=1 rate
discounts the two-ended producers' discarded sweeps)."""
import sys

import numpy as np

RATE = {1: 0.42, 2: 0.41, 3: 0.374, 4: 0.289}
TILES, SLOTS = 256, 4


def simulate(nl, policy="count", steps=20000, window=50, rate=RATE, verbose=False, ema_alpha=0.0,
             margin=1.0 / 0.9):
    C, I = nl.shape
    cum = np.concatenate([np.zeros((C, 1)), np.cumsum(nl, 1)], 1)   # work at iteration starts
    total = cum[:, -1]
    done_w = np.zeros(C)
    it = np.zeros(C, dtype=np.int64)          # current iteration
    tile = np.arange(C) // SLOTS
    live = np.ones(C, dtype=bool)
    load = np.bincount(tile, minlength=TILES).astype(np.int64)
    T_est = total.mean() / rate[4]
    dt = 1.4 * T_est / steps
    t = 0.0
    occ_time = np.zeros(SLOTS + 1)
    moves = 0
    ema = np.full(C, float(nl[:, 0].mean()))
    for s in range(steps * 3):
        if not live.any():
            break
        k = load[tile]
        r = np.array([0.0] + [rate[j] for j in range(1, SLOTS + 1)])[k]
        done_w = np.where(live, np.minimum(done_w + r * dt, total), done_w)
        occ_time += np.bincount(load, minlength=SLOTS + 1) * dt
        t += dt
        new_it = np.searchsorted(np.arange(1), 0)  # placeholder (keeps numpy import used)
        # iteration index: largest i with cum[c, i] <= done_w
        new_it = (cum <= done_w[:, None]).sum(1) - 1
        crossed = live & (new_it > it)
        if ema_alpha:
            # the chain's moving average of n_leapfrog over the iterations it completed
            for _ in range(int((new_it - it).max()) if crossed.any() else 0):
                adv = live & (new_it > it)
                ema[adv] += ema_alpha * (nl[adv, it[adv]] - ema[adv])
                it = np.where(adv, it + 1, it)
        it = new_it
        fin = live & (done_w >= total)
        if fin.any():
            np.subtract.at(load, tile[fin], 1)
            live &= ~fin
        cand = np.flatnonzero(crossed & live & (it + 2 < I))
        if cand.size == 0:
            continue
        # predicted remaining work: the chain's mean work over its last `window` iterations
        if ema_alpha:
            rem = ema * (I - it)
        else:
            lo = np.maximum(it - window, 0)
            rate_i = (cum[np.arange(C), it] - cum[np.arange(C), lo]) / np.maximum(it - lo, 1)
            rem = rate_i * (I - it)
        if policy in ("heavy", "heavy2", "sorted"):
            cand = cand[np.argsort(-rem[cand])]
        for c in cand:
            L = load[tile[c]]
            free = load < SLOTS
            if not free.any():
                break
            m = np.where(free, load, 99)
            tt = int(np.argmin(m))
            if policy in ("count", "sorted"):
                ok = m[tt] <= L - 2
            elif policy == "heavy":
                # a chain whose remaining work is above the live median may also move to
                # a tile hosting L - 1 (it then runs faster; the donor tile too)
                med = np.median(rem[live])
                ok = m[tt] <= L - 2 or (m[tt] <= L - 1 and rem[c] > 1.2 * med)
            elif policy == "count_heavy":
                # the count rule, but only the heaviest chain (estimated remaining work) of
                # the donor tile moves: the launch's tail is its heaviest chains
                ok = m[tt] <= L - 2 and rem[c] >= margin * rem[live & (tile == tile[c])].max()
            elif policy == "global_heavy":
                # the count rule, for a chain whose remaining work is at least `margin` x the
                # largest of the chains the rule lets move (tiles hosting >= min load + 2)
                ok = m[tt] <= L - 2
                if ok:
                    elig = live & (load[tile] >= m[tt] + 2)
                    ok = rem[c] >= margin * rem[elig].max()
            elif policy == "heavy2":
                # the donor tile's finish estimate against the receiver's
                ok = m[tt] <= L - 2
                if not ok and m[tt] <= L - 1:
                    mates = live & (tile == tile[c])
                    fin_d = rem[mates].max() / rate[L]
                    rec = live & (tile == tt)
                    fin_r_new = max(rem[rec].max() if rec.any() else 0, rem[c]) / rate[m[tt] + 1]
                    ok = fin_r_new < 0.9 * fin_d and rem[c] >= rem[mates].max()
            else:
                raise ValueError(policy)
            if ok:
                load[tile[c]] -= 1
                load[tt] += 1
                tile[c] = tt
                moves += 1
    occ = occ_time / occ_time.sum()
    if verbose:
        print(f"{policy}: makespan {t / T_est:.4f} x ideal, moves {moves}, occupancy "
              + " ".join(f"k={j}:{occ[j]:.3f}" for j in range(SLOTS + 1)))
    return t / T_est, moves, occ


if __name__ == "__main__":
    nl = np.load(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/chain_work.npz")["n_leapfrog"]
    nl = nl.astype(np.float64)
    for pol in ("count", "heavy", "heavy2"):
        simulate(nl, pol, steps=4000, verbose=True)
