"""The fixed cost of one extract_kernel launch (what a one-record
plan costs per back-to-back launch, paid once per step at every N).

Times back-to-back launches of a one-record plan and of a one-tile-per-wave
plan on a small genome (magot_plan_time_b2b), and prints a JSON record.  Run it
under `rocprofv3 --kernel-trace` to split that cost into the kernel's own
duration and the gap between dispatches (scripts/launch_cost.py --trace CSV).

    python scripts/launch_cost.py [--launches 400]
    python scripts/launch_cost.py --trace DIR/kt_kernel_trace.csv
"""
import argparse
import csv
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def trace_summary(path):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if 'extract_kernel' in r['Kernel_Name']:
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    rows.sort()
    dur = np.array([(e - s) * 1e-3 for s, e in rows])          # us
    gap = np.array([(rows[i + 1][0] - rows[i][1]) * 1e-3 for i in range(len(rows) - 1)])
    return {'launches': len(rows), 'duration_us_median': float(np.median(dur)),
            'gap_us_median': float(np.median(gap)) if len(gap) else None,
            'period_us_median': float(np.median(np.diff([s for s, _ in rows]) * 1e-3))
            if len(rows) > 1 else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--launches', type=int, default=400)
    ap.add_argument('--trace', default=None)
    a = ap.parse_args()
    if a.trace:
        print(json.dumps(trace_summary(a.trace), indent=1))
        return
    import torch  # before libmagot: torch brings its own HIP runtime (bench.py's order)

    from magot_amd import _lib, engine, synth
    w = synth.make('small', seed=5, genome_bases=2_000_000, n_tx=400)
    ctx = _lib.Context(0)
    dev = engine.DeviceGenome(w.contig_views(), ctx=ctx)
    out = {}
    for name, sub in (('one_record', np.array([0])), ('all_400', None)):
        plan = engine.ExtractionPlan(dev, *w.plan_tables(tx_subset=sub),
                                     engine.OUT_NUC | engine.OUT_PEP)
        plan.time_b2b(50)
        out[name] = {'b2b_ms': [plan.time_b2b(a.launches) for _ in range(3)],
                     'isolated_ms': plan.time(50), 'records': int(plan.n_tx),
                     'bytes_out': int(plan.nuc_bytes + plan.pep_bytes)}
        plan.close()
    dev.close()
    # a minimal kernel for scale: torch's one-element add_, back to back inside
    # one captured graph (no Python between the launches)
    x = torch.zeros(1, device='cuda')
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        for _ in range(10):
            x.add_(1)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(a.launches):
            x.add_(1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    ms = []
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ms.append(e0.elapsed_time(e1) / a.launches)
    out['torch_one_element_add_graph'] = {'b2b_ms': ms}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
