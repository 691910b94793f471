"""C2's kernel time with round 5's and round 4's synthetic draw order, in one
process on one box: round 5 draws the record tables before the genome bytes
(synth.py); round 4 drew the genome first, so the same seed gives another
(identically distributed) record set.  Times back-to-back launches of both
plans, alternating, and of both with the class-7 IUPAC bytes (S, W) replaced by
classed ones (R, Y), which moves their intervals off the run-list path.

    python scripts/c2_draw_order.py > profiles/r05/c2_draw_order.json
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def round4_c2(seed):
    """C2 with round 4's draw order (genome, then the records)."""
    from magot_amd import synth
    rng = np.random.default_rng(seed)
    G, T, n_ctg = 100_000_000, 50_000, 16
    L = np.full(n_ctg, G // n_ctg, dtype=np.int64)
    L[-1] += G - L.sum()
    genome = synth._genome(rng, G, iupac_rate=1e-6)
    p = L / L.sum()
    tx_contig = np.sort(rng.choice(n_ctg, size=T, p=p))
    ex_len = rng.integers(150, 1851, size=T)
    room = L[tx_contig] - ex_len
    ex_start = (rng.random(T) * room).astype(np.int64)
    return synth.Workload('C2', genome, L, tx_contig.astype(np.int64), np.ones(T, np.int8),
                          np.ones(T, np.int64), ex_start, ex_len.astype(np.int64), 'nuc')


def main():
    from magot_amd import _lib, engine, synth
    ctx = _lib.Context(0)
    seed = synth.SEED_BASE + 2
    res = {}
    plans = {}
    gens = []
    w5, w4 = synth.make('C2'), round4_c2(seed)
    cases = [('round5_order', w5, w5.genome), ('round4_order', w4, w4.genome)]
    # the same two with the class-7 IUPAC bytes (S, W: no literal class, the
    # run-list path) mapped to classed ones (R, Y)
    for name, w in (('round5_order_no_class7', w5), ('round4_order_no_class7', w4)):
        g = w.genome.copy()
        g[g == ord('S')] = ord('R')
        g[g == ord('W')] = ord('Y')
        cases.append((name, w, g))
    for name, w, genome in cases:
        contigs = [(w.contig_names[i], genome[w.contig_off[i]:w.contig_off[i + 1]])
                   for i in range(len(w.contig_len))]
        dev = engine.DeviceGenome(contigs, ctx=ctx)
        gens.append(dev)
        plans[name] = engine.ExtractionPlan(dev, *w.plan_tables(), engine.OUT_NUC)
        res[name] = {'cds_bases': int(w.cds_bases), 'ms': [],
                     'algorithmic_bytes': plans[name].algorithmic_bytes}
    for p in plans.values():
        p.time_b2b(100)
    for _ in range(5):
        for name, p in plans.items():
            res[name]['ms'].append(p.time_b2b(300))
    for name in res:
        ms = res[name]['ms']
        res[name]['frac_median'] = res[name]['algorithmic_bytes'] / (np.median(ms) * 1e-3) / 8e12
    print(json.dumps(res, indent=1))
    for p in plans.values():
        p.close()
    for g in gens:
        g.close()


if __name__ == '__main__':
    main()
