"""The code-plane lines orf6_kernel must read for C5.

orf6_kernel stages every interval from the per-plan 2-bit code plane (16
bases per u32, both strands: a '-' interval at its mirror coordinate u =
2 * span - 1 - g), one 8-byte buffer_load_dwordx2 window per 16-base vector,
so an interval over unified bases [u0, u1) touches plane bytes
[(u0 >> 4) * 4, ((u1 - 1) >> 4) * 4 + 8).  Printed per launch:
  * distinct 128-B lines of the union: what the launch must fetch from HBM
    at least once (each line once, if no line left the caches between two
    of its readers);
  * the per-interval sum: the fills if no two intervals ever shared a line;
  * descriptor bytes (16 E + 32 T + 8 T of block offsets).
The fabric reads FETCH_SIZE x 2 counts (profiles/pmc_C5.json) minus this
floor are fills of lines some tile already fetched: under the round-robin
block -> XCD order neighbouring tiles (which share lines: genome-order walk)
sit on different XCDs, each of whose L2s fetches the line itself, from the
Infinity Cache when the first fill left it there.  The exception plane
(windows of flagged intervals only) and the nibble plane of the exact path
are left out (a few MB).  Host only (numpy).
usage: python scripts/c5_lines.py [C5] [--write]   (--write: profiles/r06/c5_lines.json
and the split into profiles/pmc_C5.json)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'scripts'))

from c3_lines import K_ORIGIN, union_count  # noqa: E402


def main(config='C5'):
    from magot_amd import synth
    w = synth.make(config, genome=False)
    span = -(-(K_ORIGIN + int(np.sum(w.contig_len))) // 32) * 32
    clen = w.contig_len[np.repeat(w.tx_contig, w.ex_count)]
    s0 = np.minimum(w.ex_start, clen)
    L = np.minimum(w.ex_start + w.ex_len, clen) - s0
    keep = L > 0
    cbase = K_ORIGIN + w.contig_off[np.repeat(w.tx_contig, w.ex_count)]
    g = (cbase + s0)[keep]
    L = L[keep]
    minus = np.repeat(w.tx_strand < 0, w.ex_count)[keep]
    u0 = np.where(minus, 2 * span - (g + L), g)
    u1 = u0 + L
    b0 = (u0 >> 4) * 4
    b1 = ((u1 - 1) >> 4) * 4 + 8                 # exclusive
    lo, hi = b0 // 128, (b1 - 1) // 128
    out = {'config': config, 'intervals': int(len(g)), 'records': int(w.n_tx),
           'cds_bases': int(L.sum()), 'span': int(span),
           'code_plane_bytes': int(2 * span // 4),
           'distinct_lines_bytes': union_count(lo, hi) * 128,
           'per_interval_lines_bytes': int((hi - lo + 1).sum()) * 128,
           'descriptor_bytes': 16 * int(len(g)) + 40 * int(w.n_tx),
           'algorithmic_genome_bytes': -(-int(L.sum()) // 4)}
    out['hbm_floor_bytes'] = out['distinct_lines_bytes'] + out['descriptor_bytes']
    pmc = os.path.join(ROOT, 'profiles', 'pmc_%s.json' % config)
    if os.path.exists(pmc):
        with open(pmc) as fh:
            reads = json.load(fh)['hbm_read_bytes_per_launch']
        out['fabric_reads_bytes'] = reads
        out['refetch_bytes'] = reads - out['hbm_floor_bytes']
    print(json.dumps(out, indent=1))
    return out


def write(out):
    d = os.path.join(ROOT, 'profiles', 'r06')
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, 'c5_lines.json'), 'w') as fh:
        json.dump(out, fh, indent=1)
        fh.write('\n')
    pmc = os.path.join(ROOT, 'profiles', 'pmc_%s.json' % out['config'])
    with open(pmc) as fh:
        p = json.load(fh)
    p['read_split'] = {
        'hbm_floor_bytes': out['hbm_floor_bytes'],
        'distinct_code_plane_lines_bytes': out['distinct_lines_bytes'],
        'descriptor_bytes': out['descriptor_bytes'],
        'refetch_bytes': out['refetch_bytes'],
        'refetch_fraction': out['refetch_bytes'] / out['fabric_reads_bytes'],
        'source': 'scripts/c5_lines.py (profiles/r06/c5_lines.json)',
        'reading': 'the floor is every distinct 128-B code-plane line the launch touches plus '
                   'its descriptors, each fetched once; the rest are re-fills of lines an '
                   'earlier tile fetched: with one contiguous run of blocks per XCD the '
                   'launch fetches 1.56 GB (the floor), round-robin 2.00 GB, at 1.397 vs '
                   '1.376 ms (profiles/r04z/, DESIGN 4): the re-fills cost no time, so they are '
                   'served on die (Infinity Cache), not by HBM'}
    with open(pmc, 'w') as fh:
        json.dump(p, fh, indent=1)
        fh.write('\n')


if __name__ == '__main__':
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    res = main(*(args[:1] or ['C5']))
    if '--write' in sys.argv:
        write(res)
