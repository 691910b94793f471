"""How much of a workload's CDS a 2-bit genome source could serve (DESIGN §3,
'A 2-bit source for the windows'): the intervals whose bases are all
soft-masked or all upper-case and hold no byte outside ACGTacgt.  CPU only.

    python scripts/mask_uniform.py [--config C3] > profiles/r06/mask_uniform.json
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from magot_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='C3')
    a = ap.parse_args()
    w = synth.make(a.config)
    g = w.genome
    low = (g >= 97) & (g <= 122)
    exc = ~np.isin(g, np.frombuffer(b'ACGTacgt', np.uint8))
    pl = np.concatenate([[0], np.cumsum(low, dtype=np.int64)])
    pe = np.concatenate([[0], np.cumsum(exc, dtype=np.int64)])
    s = w.contig_off[np.repeat(w.tx_contig, w.ex_count)] + w.ex_start
    e = s + w.ex_len
    nl, ne = pl[e] - pl[s], pe[e] - pe[s]
    uni = ((nl == 0) | (nl == w.ex_len)) & (ne == 0)
    print(json.dumps({
        'config': a.config, 'intervals': int(len(s)), 'cds_bases': int(w.ex_len.sum()),
        'genome_soft_masked_fraction': float(low.mean()),
        'intervals_with_exceptions_fraction': float((ne > 0).mean()),
        'mask_uniform_clean_intervals_fraction': float(uni.mean()),
        'mask_uniform_clean_bases_fraction': float(w.ex_len[uni].sum() / w.ex_len.sum())},
        indent=1))


if __name__ == '__main__':
    main()
