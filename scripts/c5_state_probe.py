"""Is C5's slow state a property of the process or of where its buffers sit?

One process builds the C5 plan once, then creates the six-frame plan
(Orf6Plan: its output streams, rows, tiles and derived planes in one HBM
arena) several times, each after a different-size spacer allocation, and
times 50 back-to-back launches of each (HIP events on the kernel's stream),
twice round.  The memory probe (torch fill / copy bandwidth) runs beside.

    python scripts/c5_state_probe.py [--no-probe] [--rounds N] [--spacers 0,64,...]
        > gpurun_out/c5_state.json

--no-probe skips the memory probe before the first six-frame plan (bench.py
runs its probe after the plan exists).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse

    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument('--no-probe', action='store_true')
    ap.add_argument('--rounds', type=int, default=2)
    ap.add_argument('--spacers', default='0,64,1000,2050,4100,333,0')
    args = ap.parse_args()

    import bench
    from magot_amd import _lib, engine, synth
    w = synth.make('C5')
    ctx = _lib.Context(0)
    dev = engine.DeviceGenome(w.contig_views(), ctx=ctx)
    ex, tx = w.plan_tables()
    plan = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC)
    res = {'probe0': None if args.no_probe else bench.memory_probe(), 'runs': []}
    spacers = [int(x) for x in args.spacers.split(',')]  # MiB
    keep = []
    for rnd in range(args.rounds):
        for mib in spacers:
            pad = torch.empty(max(mib, 1) << 20, dtype=torch.uint8, device='cuda')
            o6 = engine.Orf6Plan(plan)
            o6.execute()
            ctx.sync()
            o6.time_b2b(20)
            ms = [o6.time_b2b(50) for _ in range(3)]
            res['runs'].append({'round': rnd, 'spacer_mib': mib, 'ms': ms, 't': time.time()})
            print(json.dumps(res['runs'][-1]), file=sys.stderr, flush=True)
            o6.close()
            keep.append(pad)  # the next plan lands elsewhere
        keep = []
        torch.cuda.empty_cache()
    res['probe1'] = bench.memory_probe()
    print(json.dumps(res))


if __name__ == '__main__':
    main()
