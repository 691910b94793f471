"""Record-order vs genome-order extraction plans (MAGOT_OUT_GENOME_ORDER) on
one box, in one process: both plans of each configuration are built over one
packed genome and their back-to-back launch times taken in alternating
rounds (HIP events around K launches, magot_plan_time_b2b).  Also times the
delivery each layout pays once per job: magot_plan_copy_outputs into device
memory (a plain D2D copy for record order, the per-record segment copy for
genome order).

    python scripts/plan_order_ab.py [--configs C3,C2] [--rounds 7] > profiles/r05/plan_order.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--configs', default='C3,C2')
    ap.add_argument('--rounds', type=int, default=7)
    ap.add_argument('--plan-only', action='store_true', help='only the plan_create timing')
    ap.add_argument('--launches', type=int, default=200)
    a = ap.parse_args()
    import torch  # the HIP runtime torch loads first
    from magot_amd import _lib, engine, synth
    ctx = _lib.Context(0)
    res = {'rounds': a.rounds, 'launches_per_timing': a.launches, 'device': ctx.info(),
           'configs': {}}
    for cfg in a.configs.split(','):
        t0 = time.perf_counter()
        w = synth.make(cfg)
        dev = engine.DeviceGenome(w.contig_views(), ctx=ctx)
        ex, tx = w.plan_tables()
        outputs = engine.OUT_NUC | (engine.OUT_PEP if w.outputs == 'nuc+pep' else 0)
        sys.stderr.write('%s: generated and packed in %.1fs\n' % (cfg, time.perf_counter() - t0))
        # host cost of magot_plan_create, 3 alternating builds of each layout
        plan_s = {'record': [], 'genome': []}
        for _ in range(3):
            for k, fl in (('record', 0), ('genome', engine.OUT_GENOME_ORDER)):
                t1 = time.perf_counter()
                engine.ExtractionPlan(dev, ex, tx, outputs | fl).close()
                plan_s[k].append(time.perf_counter() - t1)
        sys.stderr.write('%s: plan_create s %s\n' % (cfg, {k: [round(x, 4) for x in v]
                                                          for k, v in plan_s.items()}))
        plans = {'record': engine.ExtractionPlan(dev, ex, tx, outputs),
                 'genome': engine.ExtractionPlan(dev, ex, tx, outputs | engine.OUT_GENOME_ORDER)}
        if a.plan_only:
            res['configs'][cfg] = {'plan_create_s': plan_s}
            for p in plans.values():
                p.close()
            dev.close()
            continue
        for p in plans.values():
            p.time_b2b(20)
        times = {k: [] for k in plans}
        for rnd in range(a.rounds):
            for k, p in plans.items():
                times[k].append(p.time_b2b(a.launches))
            sys.stderr.write('%s round %d: record %.4f ms, genome %.4f ms\n'
                             % (cfg, rnd, times['record'][-1], times['genome'][-1]))
        B, P = plans['record'].nuc_bytes, plans['record'].pep_bytes if outputs & engine.OUT_PEP else 0
        dst = torch.empty(B + P + 64, dtype=torch.uint8, device='cuda')
        torch.cuda.synchronize()
        deliver = {}
        for k, p in plans.items():
            reps = []
            for _ in range(5):
                t1 = time.perf_counter()
                p.copy_outputs(dst.data_ptr(), dst.data_ptr() + ((B + 15) & ~15) if P else None)
                reps.append((time.perf_counter() - t1) * 1e3)
            deliver[k] = reps
        med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
        res['configs'][cfg] = {
            'records': int(w.n_tx), 'nuc_bytes': int(B), 'pep_bytes': int(P),
            'kernel_ms': times, 'median_ms': med,
            'genome_over_record': med['genome'] / med['record'],
            'copy_outputs_ms': deliver, 'plan_create_s': plan_s,
            'algorithmic_bytes': plans['record'].algorithmic_bytes}
        for p in plans.values():
            p.close()
        dev.close()
        del dst
    json.dump(res, sys.stdout, indent=1)
    sys.stdout.write('\n')


if __name__ == '__main__':
    main()
