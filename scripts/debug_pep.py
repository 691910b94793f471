"""Locate peptide mismatches of the extraction kernel against the C oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from magot_amd import engine, synth  # noqa: E402
from oracle import cds_oracle  # noqa: E402

TILE = 12288
for outputs, name in ((engine.OUT_PEP, 'pep-only'), (engine.OUT_NUC | engine.OUT_PEP, 'nuc+pep')):
    w = synth.make('small', seed=1, genome_bases=3_000_000, n_tx=1500, iupac_rate=1e-3)
    dev = engine.DeviceGenome(w.contigs())
    ex, tx = w.plan_tables()
    plan = engine.ExtractionPlan(dev, ex, tx, outputs)
    nuc, noff, pep, poff = plan.run()
    ref, roff, _ = cds_oracle.extract_workload(w, False)
    # untrimmed oracle translation of the oracle nucleotides
    from oracle import magot_oracle as mo
    want = []
    for t in range(w.n_tx):
        s = ref[roff[t]:roff[t + 1]].tobytes().decode('latin-1')
        want.append(''.join(mo.STANDARD_CODE.get(s[i:i + 3].upper(), 'X')
                            for i in range(0, len(s) - 2, 3)))
    want = ''.join(want).encode('latin-1')
    got = pep.tobytes()
    print(name, 'len', len(got), len(want), 'nuc ok', nuc is None or np.array_equal(nuc, ref))
    bad = [i for i in range(min(len(got), len(want))) if got[i] != want[i]]
    print(name, os.environ.get('MAGOT_DEBUG_PATHS'), 'mismatches', len(bad))
    tiles = {}
    for q in bad:
        t = int(np.searchsorted(poff[:-1].astype(np.int64), q, side='right') - 1)
        r = int(noff[t] + 3 * (q - poff[t]))
        tiles[r // TILE] = tiles.get(r // TILE, 0) + 1
    print('  bad tiles', sorted(tiles.items())[:30])
    tn = noff[:-1].astype(np.int64)
    tp = poff[:-1].astype(np.int64)
    for q in bad[:6]:
        t = int(np.searchsorted(tp, q, side='right') - 1)
        while poff[t + 1] <= q:
            t += 1
        r = int(tn[t] + 3 * (q - tp[t]))
        print('  q=%d rec=%d codon_nuc=%d tile=%d off_in_tile=%d got=%r want=%r' % (
            q, t, r, r // TILE, r % TILE, chr(got[q]), chr(want[q])))
    plan.close()
    dev.close()

if os.environ.get('MAGOT_DEBUG_DUMP'):
    w = synth.make('small', seed=1, genome_bases=3_000_000, n_tx=1500, iupac_rate=1e-3)
    dev = engine.DeviceGenome(w.contigs())
    ex, tx = w.plan_tables()
    plan = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC | engine.OUT_PEP)
    nuc, noff, pep, poff = plan.run()
    np.savez(os.path.join(ROOT, 'gpurun_out', 'debug_pep.npz'), nuc=nuc, noff=noff, pep=pep,
             poff=poff)
