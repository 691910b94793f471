"""Is C5's slow state a property of the process or of where its buffers sit?

One process builds the C5 plan once, then creates the six-frame plan
(Orf6Plan: its output streams, rows, tiles and derived planes in one HBM
arena) several times, each after a different-size spacer allocation, and
times 50 back-to-back launches of each (HIP events on the kernel's stream),
twice round.  The memory probe (torch fill / copy bandwidth) runs beside.

    python scripts/c5_state_probe.py > gpurun_out/c5_state.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from magot_amd import _lib, engine, synth
    w = synth.make('C5')
    ctx = _lib.Context(0)
    dev = engine.DeviceGenome(w.contig_views(), ctx=ctx)
    ex, tx = w.plan_tables()
    plan = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC)
    res = {'probe0': bench.memory_probe(), 'runs': []}
    spacers = [0, 64, 1000, 2050, 4100, 333, 0]  # MiB
    keep = []
    for rnd in range(2):
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
