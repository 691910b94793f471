"""Write profiles/pmc_<CONFIG>.json (the HBM traffic bench.py quotes as
roofline.traffic) from a directory of rocprofv3 --pmc passes.

    python scripts/pmc_json.py DIR CONFIG KERNEL

FETCH_SIZE and WRITE_SIZE are in KiB per launch; gfx950 tallies each 128-B
read fill as 64 B, so reads are FETCH_SIZE x 2 (MI355X_MICROARCH.md, HBM /
rocprofv3 section); WRITE_SIZE is taken as read.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(d, config, kernel):
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)):
        for r in csv.DictReader(open(f)):
            if kernel in r['Kernel_Name']:
                agg[r['Counter_Name']].append(float(r['Counter_Value']))
    mean = {k: sum(v) / len(v) for k, v in agg.items()}
    fetch = mean['FETCH_SIZE'] * 1024
    write = mean['WRITE_SIZE'] * 1024
    out = {
        'config': config,
        'kernel': kernel,
        'source': os.path.relpath(os.path.abspath(d), ROOT),
        'fetch_size_bytes_raw': fetch,
        'write_size_bytes': write,
        'hbm_read_bytes_per_launch': 2 * fetch,
        'hbm_bytes_per_launch': 2 * fetch + write,
        'tcc_ea_rdreq': mean.get('TCC_EA0_RDREQ'),
        'tcc_ea_wrreq': mean.get('TCC_EA0_WRREQ'),
        'correction': 'FETCH_SIZE x2 (gfx950 128-B fills tallied at 64 B), WRITE_SIZE x1',
        'calibration': 'x2 calibrated for these kernels\' own loads (round 5, '
                       'profiles/r05/fetchcal.json): 12-byte buffer_load_dwordx3 windows '
                       '(extract_kernel) and 8-byte buffer_load_dwordx2 windows (orf6_kernel), '
                       'streaming or one per line anywhere in it, cost one TCC_EA0_RDREQ per '
                       '128-B line and FETCH_SIZE tallies 64 B per request; fabric reads '
                       'include Infinity Cache hits (an upper bound on HBM reads)',
    }
    path = os.path.join(ROOT, 'profiles', 'pmc_%s.json' % config)
    if os.path.exists(path):  # keep an attribution made from the lines (scripts/c5_lines.py)
        with open(path) as fh:
            old = json.load(fh)
        if 'read_split' in old:
            out['read_split'] = old['read_split']
    with open(path, 'w') as fh:
        json.dump(out, fh, indent=1)
        fh.write('\n')
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(*sys.argv[1:4])
