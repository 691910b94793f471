"""The C4 job's per-GPU shares timed on ONE box, in ONE process (VERDICT r4
item 5): the full C3 job (or, --config C5, the six-frame job) and every
shard of the N = 2, 4 and 8 splits
(bench.py's strong-mode sharding, shard.record_shards) are planned over one
packed genome and timed in alternating rounds, so each projected speed-up
(full job / slowest shard) is a same-box, same-process ratio.

Per plan and round: back-to-back launches (HIP events around K launches on
the library stream, magot_plan_time_b2b).  Also times a one-record plan
(the launch's fixed cost) to account for the N=2 efficiency.

    python scripts/c4_shares.py [--rounds 5] [--launches 200] > profiles/r05/c4_shares.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--launches', type=int, default=200)
    ap.add_argument('--config', default='C3')
    ap.add_argument('--order', default='gff', choices=['gff', 'genome'],
                    help='record order inside each shard: GFF order, or genome order '
                         '(shard.genome_order; the full C3 job then runs as bench.py runs '
                         'it, its records laid out in genome order)')
    a = ap.parse_args()
    from magot_amd import _lib, engine, shard, synth
    t0 = time.perf_counter()
    w = synth.make(a.config)
    ctx = _lib.Context(0)
    dev = engine.DeviceGenome(w.contig_views(), ctx=ctx)
    first = np.zeros(w.n_tx + 1, dtype=np.int64)
    np.cumsum(w.ex_count, out=first[1:])
    tx_bases = np.add.reduceat(w.ex_len, first[:-1])
    c5 = a.config == 'C5'
    outputs = engine.OUT_NUC if c5 else engine.OUT_NUC | engine.OUT_PEP
    keep = []

    def make_plan(tables, flags=0):
        """The timed object: the extraction plan (C3), or its six-frame plan (C5)."""
        p = engine.ExtractionPlan(dev, *tables, outputs | flags)
        if not c5:
            return p
        keep.append(p)
        return engine.Orf6Plan(p)

    full_flags = engine.OUT_GENOME_ORDER if a.order == 'genome' and not c5 else 0
    plans = {'full': make_plan(w.plan_tables(), full_flags)}
    loads = {}
    for n in (2, 4, 8):
        shards, load, _ = shard.record_shards(w.tx_contig, tx_bases, len(w.contig_len), n,
                                              tx_start=w.ex_start[first[:-1]])
        loads[n] = load.tolist()
        for r, sh in enumerate(shards):
            if a.order == 'genome':
                sh = shard.genome_order(sh, w.tx_contig, w.ex_start[first[:-1]])
            plans['%d:%d' % (n, r)] = make_plan(w.plan_tables(tx_subset=sh))
    plans['one_record'] = make_plan(w.plan_tables(tx_subset=np.array([0])))
    sys.stderr.write('planned %d plans in %.1fs\n' % (len(plans), time.perf_counter() - t0))
    for p in plans.values():  # warm every plan once
        p.time_b2b(20)
    times = {k: [] for k in plans}
    for rnd in range(a.rounds):
        for k, p in plans.items():
            times[k].append(p.time_b2b(a.launches))
        sys.stderr.write('round %d: full %.4f ms, 2:0 %.4f, 4:0 %.4f, 8:0 %.4f\n'
                         % (rnd, times['full'][-1], times['2:0'][-1], times['4:0'][-1],
                            times['8:0'][-1]))
    info = ctx.info()
    res = {'config': a.config, 'order': a.order, 'rounds': a.rounds,
           'full_job_layout': 'genome' if full_flags else 'record',
           'launches_per_timing': a.launches,
           'device': info,
           'kernel': 'orf6_kernel' if c5 else 'extract_kernel',
           'plans': {k: {'ms': v,
                         'bytes_out': int(plans[k].total if c5
                                          else plans[k].nuc_bytes + plans[k].pep_bytes),
                         'records': int(plans[k].plan.n_tx if c5 else plans[k].n_tx)}
                     for k, v in times.items()},
           'shard_loads': loads}
    proj = {}
    for n in (2, 4, 8):
        per_round = []
        for i in range(a.rounds):
            slowest = max(times['%d:%d' % (n, r)][i] for r in range(n))
            per_round.append(times['full'][i] / slowest)
        proj[str(n)] = {'speedup_per_round': per_round, 'min': min(per_round),
                        'max': max(per_round), 'mean': sum(per_round) / len(per_round),
                        'efficiency_mean': sum(per_round) / len(per_round) / n}
    res['projected_speedup'] = proj
    res['note'] = ('same box, same process; speed-up = full-job launch time / the slowest '
                   'shard\'s launch time, per alternating round; the collective phases '
                   '(genome broadcast, output gather) are outside the step as in bench.py')
    json.dump(res, sys.stdout, indent=1)
    sys.stdout.write('\n')
    for p in list(plans.values()) + keep:
        p.close()
    dev.close()


if __name__ == '__main__':
    main()
