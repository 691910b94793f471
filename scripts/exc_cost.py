"""How much of the C3 launch the exception (slow) path costs: the same
workload timed as generated (N runs ~1 %, IUPAC 1e-6) and with every
non-ACGTacgt byte replaced by 'A' (no interval takes the slow path).
    python scripts/exc_cost.py [config=C3]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from magot_amd import engine, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'C3'
w = synth.make(cfg)
res = {}
for tag in ('as_generated', 'no_exceptions'):
    if tag == 'no_exceptions':
        g = w.genome
        ok = np.isin(g, np.frombuffer(b'ACGTacgt', dtype=np.uint8))
        g[~ok] = ord('A')
    dev = engine.DeviceGenome(w.contigs())
    ex, tx = w.plan_tables()
    plan = engine.ExtractionPlan(dev, ex, tx)
    plan.execute()
    plan.sync()
    res[tag] = [plan.time(20) for _ in range(3)]
    plan.close()
    dev.close()
print(json.dumps(res))
