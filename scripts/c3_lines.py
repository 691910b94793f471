"""The genome lines extract_kernel must read for a configuration's plan.

Every non-empty interval is read from the forward nibble plane (a '-'
interval without exceptions too: it is reverse-complemented in registers),
one 12-byte window at byte (u >> 3) * 4 per 16-base chunk segment, so an
interval starting at global base g with L bases touches plane bytes
[(g >> 3) * 4, ((g + L - 1) >> 3) * 4 + 12).  This prints, per launch:
  * distinct 128-B lines (and 64-B halves) of that union -- the fills a
    launch needs if every line were fetched once;
  * the per-interval sum -- the fills if no line were ever shared between two
    intervals (every interval fetches its own lines);
  * the descriptor bytes (16 E + 32 T) and the algorithmic genome bytes.
Host only (numpy).  usage: python scripts/c3_lines.py [C3|C2|C5]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

K_ORIGIN = 64


def union_count(lo, hi):
    """Number of integers in the union of the closed ranges [lo, hi]."""
    o = np.argsort(lo, kind='stable')
    lo, hi = lo[o], hi[o]
    run_hi = np.maximum.accumulate(hi)
    # a range starts a new block when it begins after everything before it ended
    new = np.ones(len(lo), dtype=bool)
    new[1:] = lo[1:] > run_hi[:-1]
    starts = np.nonzero(new)[0]
    ends = np.append(starts[1:], len(lo)) - 1
    return int((run_hi[ends] - lo[starts] + 1).sum())


def main(config='C3'):
    from magot_amd import synth
    w = synth.make(config, genome=False)
    first = np.zeros(w.n_tx + 1, dtype=np.int64)
    np.cumsum(w.ex_count, out=first[1:])
    clen = w.contig_len[np.repeat(w.tx_contig, w.ex_count)]
    s0 = np.minimum(w.ex_start, clen)
    L = np.minimum(w.ex_start + w.ex_len, clen) - s0
    keep = L > 0
    cbase = K_ORIGIN + w.contig_off[np.repeat(w.tx_contig, w.ex_count)]
    g = (cbase + s0)[keep]
    L = L[keep]
    b0 = (g >> 3) * 4
    b1 = ((g + L - 1) >> 3) * 4 + 12          # exclusive
    out = {'config': config, 'intervals': int(len(g)), 'records': int(w.n_tx),
           'cds_bases': int(L.sum())}
    for size in (128, 64):
        lo, hi = b0 // size, (b1 - 1) // size
        out['distinct_%d' % size] = union_count(lo, hi) * size
        out['per_interval_sum_%d' % size] = int((hi - lo + 1).sum()) * size
    out['window_bytes_sum'] = int((b1 - b0).sum())
    out['descriptor_bytes'] = 16 * int(len(g)) + 32 * int(w.n_tx)
    out['algorithmic_genome_bytes'] = -(-int(L.sum()) // 4)
    print(json.dumps(out, indent=1))
    return out


if __name__ == '__main__':
    main(*(sys.argv[1:2] or ['C3']))
