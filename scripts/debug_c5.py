"""Diagnostic: the C5 six-frame job against the C oracle, with the details of
every mismatching stream (record, frame, strand, length, contig, exception
bytes, expected vs device residues) written as JSON."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from magot_amd import engine, synth  # noqa: E402
from oracle import cds_oracle, magot_oracle as mo  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'C5'
out_path = sys.argv[2] if len(sys.argv) > 2 else 'gpurun_out/debug_c5.json'
w = synth.make(cfg)
dev = engine.DeviceGenome(w.contigs())
ex, tx = w.plan_tables()
plan = engine.ExtractionPlan(dev, ex, tx, engine.OUT_NUC)
o6 = engine.Orf6Plan(plan)
o6.execute()
out, soff, slen = o6.fetch()
ref, roff, st = cds_oracle.extract_workload(w, False)
bad = []
n, first = cds_oracle.orf6_compare(ref, roff, out, soff, slen, threads=16, bad_list=bad)
first_ex = np.zeros(w.n_tx + 1, dtype=np.int64)
np.cumsum(w.ex_count, out=first_ex[1:])
rows = []
for j in sorted(bad)[:60]:
    r, k = divmod(j, 6)
    f, plus = divmod(k, 2)
    s = ref[roff[r]:roff[r + 1]].tobytes().decode('latin-1')
    want = mo.translate(s, frame=f, strand='+' if plus else '-', trimX=(f != 0))
    got = out[int(soff[j]):int(soff[j] + slen[j])].tobytes().decode('latin-1')
    diff = [i for i in range(min(len(got), len(want or ''))) if got[i] != want[i]]
    exc = sorted(set(c for c in s if c not in 'ACGTacgt'))
    rows.append({'stream': j, 'record': r, 'frame': f, 'strand': '+' if plus else '-',
                 'len': len(s), 'contig': int(w.tx_contig[r]),
                 'exons': [[int(w.ex_start[e]), int(w.ex_len[e])]
                           for e in range(first_ex[r], first_ex[r + 1])][:30],
                 'strand_tx': int(w.tx_strand[r]), 'exception_bytes': exc,
                 'want_len': len(want) if want is not None else None, 'got_len': len(got),
                 'first_diff': diff[:8],
                 'want_at': (want or '')[max(0, (diff or [0])[0] - 5):(diff or [0])[0] + 10],
                 'got_at': got[max(0, (diff or [0])[0] - 5):(diff or [0])[0] + 10],
                 'soff': int(soff[j])})
recs = sorted(set(j // 6 for j in bad))
print(json.dumps({'bad_streams': n, 'bad_records': len(recs), 'records': recs[:200]}))
os.makedirs(os.path.dirname(out_path), exist_ok=True)
with open(out_path, 'w') as fh:
    json.dump({'bad_streams': n, 'records': recs, 'rows': rows}, fh, indent=1)
