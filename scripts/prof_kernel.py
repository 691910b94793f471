"""Profiling driver: build one workload's plan and launch the extraction
kernel --iters times (no verification, no torch).  Used under rocprofv3."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from magot_amd import _lib, engine, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--config', default='C3')
ap.add_argument('--iters', type=int, default=10)
ap.add_argument('--order', default='random')
ap.add_argument('--outputs', default='nuc+pep')
a = ap.parse_args()
w = synth.make(a.config, order=a.order)
dev = engine.DeviceGenome(w.contigs())
ex, tx = w.plan_tables()
outputs = {'nuc+pep': engine.OUT_NUC | engine.OUT_PEP, 'nuc': engine.OUT_NUC,
           'pep': engine.OUT_PEP}[a.outputs]
plan = engine.ExtractionPlan(dev, ex, tx, outputs)
for _ in range(a.iters):
    plan.execute()
plan.sync()
print('plan: B=%d P=%d E=%d T=%d alg_bytes=%d' % (plan.nuc_bytes, plan.pep_bytes, plan.n_exons,
                                                 plan.n_tx, plan.algorithmic_bytes))
