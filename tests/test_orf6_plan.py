"""The C5 six-frame kernel's tile windows, restated on the CPU (test
infrastructure): orf6_plan_tiles (magot_amd/csrc/seqops.hip) and the
interval rows' exception flags (magot_plan_create's run lookup).  Used to
show that a workload reaches a kernel case, e.g. a window whose only flagged
interval is staged by lanes 32-63 (the truncated-ballot bug found by the
full-size C5 check in round 3)."""

import numpy as np

from magot_amd import synth

ORF_TILE, ROW_CAP = 3968, 123
_PLAIN = np.frombuffer(b'ACGTacgt', dtype=np.uint8)


def orf6_windows(w):
    """Per tile: (first row, number of rows staged, row ids that are flagged),
    for the records of ``w.plan_tables()`` (zero-length intervals dropped)."""
    ex, tx = w.plan_tables()
    L = ex['len'].astype(np.int64)
    st = (ex['start_rc'] & np.uint64((1 << 63) - 1)).astype(np.int64)
    gs = w.contig_off[ex['contig'].astype(np.int64)] + st
    exc = ~np.isin(w.genome, _PLAIN)
    cs = np.concatenate([[0], np.cumsum(exc)])
    flag = (cs[gs + L] - cs[gs]) > 0
    keep = L > 0
    out = np.concatenate([[0], np.cumsum(L)])
    starts = np.concatenate([out[:-1][keep], [out[-1]]])
    flag = flag[keep]
    total, n_rows = int(out[-1]), len(starts) - 1
    res = []
    T = 0
    while T < total:
        W0 = (T - 48 if T >= 48 else 0) & ~15
        e = max(int(np.searchsorted(starts, W0, side='right')) - 1, 0)
        T1 = min(T + ORF_TILE, total)
        if e + ROW_CAP < n_rows:
            cap = int(starts[e + ROW_CAP])
            if T1 + 50 > cap:
                T1 = max(T + 1, cap - 50)
        WE = min(T1 + 50, total)
        m = int(np.searchsorted(starts, WE, side='left')) - e
        res.append((e, m, np.nonzero(flag[e:e + m])[0]))
        T = T1
    return res


def upper_lane_workload():
    """Short exons (~55 rows per window) and sparse short N runs: many
    windows whose flagged rows all sit at row index 32-63 or 96-127."""
    rng = np.random.default_rng(2026)
    w = synth.make('small', seed=21, genome_bases=2_000_000, n_tx=2500, iupac_rate=0)
    w.genome[w.genome == ord('N')] = ord('C')
    for p in rng.integers(0, len(w.genome) - 200, size=400):
        w.genome[p:p + int(rng.integers(40, 160))] = ord('N')
    w.ex_len = rng.integers(40, 75, size=w.n_exons).astype(np.int64)
    return w


def upper_only(windows):
    return sum(1 for _, _, f in windows
               if len(f) and all((j & 63) >= 32 for j in f.tolist()))


def test_upper_lane_workload_reaches_the_case():
    wins = orf6_windows(upper_lane_workload())
    assert upper_only(wins) >= 20
    assert max(m for _, m, _ in wins) > 64          # rows staged by both lane halves
    # the kernel stages rows e .. e + m (tile_m, capped at ROW_CAP; the last
    # one the sentinel past the window): the cap never cuts a window here
    assert max(m for _, m, _ in wins) <= ROW_CAP
