"""Summarise a scripts/fetchcal.hip run (gpu_round.sh stage `fetchcal`):
per calibration kernel, its known unique bytes and 128-B lines, FETCH_SIZE
(KiB -> bytes), TCC_EA0_RDREQ and the kernel-trace duration, and the factors
FETCH_SIZE / unique bytes and bytes per read request.

    python scripts/fetchcal_summary.py gpurun_out/<tag> > profiles/<round>/fetchcal.json
"""
import csv
import glob
import json
import os
import sys


def _counters(path, name):
    out = {}
    for f in glob.glob(os.path.join(path, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] == name and 'cal<' in r['Kernel_Name']:
                mode = int(r['Kernel_Name'].split('cal<')[1].split('>')[0])
                out[mode] = float(r['Counter_Value'])
    return out


def _durations(path):
    out = {}
    for f in glob.glob(os.path.join(path, '**', '*kernel_trace.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if 'cal<' in r['Kernel_Name']:
                mode = int(r['Kernel_Name'].split('cal<')[1].split('>')[0])
                out[mode] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-6
    return out


def main(d):
    rows = [json.loads(x) for x in open(os.path.join(d, 'fetchcal_plain.jsonl')) if x.startswith('{')]
    fetch = _counters(os.path.join(d, 'fetchcal_pmc'), 'FETCH_SIZE')
    rdreq = _counters(os.path.join(d, 'fetchcal_pmc2'), 'TCC_EA0_RDREQ_sum')
    dur = _durations(os.path.join(d, 'fetchcal_kt'))
    out = []
    for r in rows:
        m = r['mode']
        fb = fetch.get(m, 0.0) * 1024
        rec = dict(r, fetch_size_bytes=fb, tcc_ea0_rdreq=rdreq.get(m),
                   kernel_trace_ms=dur.get(m),
                   fetch_over_unique=fb / r['unique_bytes'] if r['unique_bytes'] else None,
                   fetch_over_lines_x128=fb / (128.0 * r['lines_touched']),
                   fetch_bytes_per_rdreq=fb / rdreq[m] if rdreq.get(m) else None)
        out.append(rec)
    res = {'source': d, 'kernels': out,
           'reading': 'one TCC_EA0_RDREQ per 128-B line a 12-byte buffer_load_dwordx3 window '
                      'misses in L2, whatever part of the line it touches (both halves, one '
                      'half, or straddling); FETCH_SIZE tallies 64 B per request, so a 12-B '
                      'window read costs a 128-B line fill and FETCH_SIZE x 2 = line fills x '
                      '128 B -- the guide\'s x2 correction holds for this access width and shape'}
    json.dump(res, sys.stdout, indent=1)
    sys.stdout.write('\n')


if __name__ == '__main__':
    main(sys.argv[1])
