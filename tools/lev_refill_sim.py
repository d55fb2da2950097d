"""Host simulation behind k_lev_refill (spk_gamma.hip): scan steps per Levenshtein exact-pass cell and the lane
utilisation of one-cell-per-lane waves vs lane-refill waves.

Cells are drawn like the exact pass's lists: pairs that share a blocking key (cfg5: surname, addresses of
<= 64 units; cfg2: surname / dob, emails whose length / letter-count bounds leave the ratio test undecided).
Steps follow the kernels: common prefix / suffix stripped, the shorter remainder is the text, the scan stops at
the end of the text or when the end cell's diagonal passes the cut (tested every LEVR_STEPS steps).

    python tools/lev_refill_sim.py [cells]
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from splink_amd.synthetic import make_records  # noqa: E402

LEVR_STEPS, LEVR_MIN, HOPS = 2, 16, 3


def steps_of(a, b, t, every):
    """Scan steps of one cell (0 = settled at setup) under a `levenshtein ratio <= t` cut."""
    la, lb = len(a), len(b)
    cut = math.floor(t * (la + lb) / 2) + 1
    mn = min(la, lb)
    pre = 0
    while pre < mn and a[pre] == b[pre]:
        pre += 1
    suf = 0
    while suf < mn - pre and a[la - 1 - suf] == b[lb - 1 - suf]:
        suf += 1
    ra, rb = a[pre:la - suf], b[pre:lb - suf]
    if not ra or not rb:
        return 0
    pat, txt = (ra, rb) if len(ra) >= len(rb) else (rb, ra)
    m, n = len(pat), len(txt)
    if m - n > cut:
        return 0
    col = list(range(m + 1))
    for j in range(n):
        prev, col[0] = col[0], j + 1
        for i in range(1, m + 1):
            cur = min(col[i] + 1, col[i - 1] + 1, prev + (pat[i - 1] != txt[j]))
            prev, col[i] = col[i], cur
        if (j + 1) % every == 0 and col[min(m, j + 1 + m - n)] > cut:
            return j + 1
    return n


def cells_of(cfg, n_cells, rng):
    if cfg == 5:
        df = make_records(200_000, surname_vocab=3000, with_address=True)
        col, t, keys = df.address.to_numpy(), 0.4, ["surname"]
    else:
        df = make_records(300_000, surname_vocab=4500)
        col, t, keys = df.email.to_numpy(), 0.3, ["surname", "dob"]
    out = []
    for key in keys:
        g = df.dropna(subset=[key]).groupby(key).indices
        ks = list(g.keys())
        w = np.array([len(g[k]) * (len(g[k]) - 1) / 2 for k in ks], float)
        w /= w.sum()
        while len(out) < n_cells * (keys.index(key) + 1) // len(keys):
            idx = g[ks[rng.choice(len(ks), p=w)]]
            i, j = rng.choice(idx, 2, replace=False)
            a, b = col[i], col[j]
            if a is None or b is None or a == b or max(len(a), len(b)) > 64:
                continue
            out.append((a, b, t))
    return out


def simt(steps, rng, waves=300):
    """Lane utilisation of one cell per lane: a wave of 64 runs max(steps)."""
    s = np.asarray(steps)
    tot = sum(s[rng.choice(len(s), 64)].max() * 64 for _ in range(waves))
    return s.mean() * 64 * waves / tot


def refill(steps, rng, n=20000):
    """Lane utilisation of the refill kernel's schedule: rounds every LEVR_STEPS steps, a staged cell ready HOPS
    rounds after its lane took the previous one, hand-out when LEVR_MIN lanes are ready or few still scan."""
    q = list(rng.choice(np.asarray(steps), n))
    left = [0] * 64  # steps left of the lane's cell (0 = idle)
    stage = [0] * 64  # rounds since the lane's staged cell was requested (ready at HOPS)
    busy = lane_steps = 0
    while q or any(left):
        ready = [l for l in range(64) if left[l] == 0 and stage[l] >= HOPS]
        act = sum(1 for x in left if x)
        if ready and (len(ready) >= LEVR_MIN or act < LEVR_MIN):
            for l in ready:
                if not q:
                    break
                left[l] = q.pop()
                stage[l] = 0
        for l in range(64):
            stage[l] += 1
        for _ in range(LEVR_STEPS):
            if any(left):
                lane_steps += 64
                for l in range(64):
                    if left[l]:
                        left[l] -= 1
                        busy += 1
    return busy / max(lane_steps, 1)


if __name__ == "__main__":
    n_cells = int(sys.argv[1]) if len(sys.argv) > 1 else 600
    rng = np.random.default_rng(5)
    for cfg in (2, 5):
        cells = cells_of(cfg, n_cells, rng)
        s1 = [steps_of(a, b, t, 1) for a, b, t in cells]
        s2 = [steps_of(a, b, t, LEVR_STEPS) for a, b, t in cells]
        print(f"cfg{cfg}: {len(cells)} cells, mean steps (exit tested every step) {np.mean(s1):.2f}, "
              f"every {LEVR_STEPS} steps {np.mean(s2):.2f}; lane utilisation one-cell-per-lane {simt(s2, rng):.2f}, "
              f"refill {refill(s2, rng):.2f}", flush=True)
