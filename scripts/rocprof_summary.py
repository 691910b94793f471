"""profiles/rocprof_summary.json from rocprofv3 kernel traces: per
configuration, the average duration of its measured kernel, quoted by bench.py
beside its live HIP-event time.

    # the K timed launches only (round 4+): the bench line printed under the
    # profiler names their dispatch indices (roofline.timed_launches)
    python scripts/rocprof_summary.py --timed C3=DIR/kt_kernel_trace.csv,DIR/kt.json ...
    # every launch of the kernel (--stats CSV), as rounds 1-3 quoted
    python scripts/rocprof_summary.py C3=profiles/r03e/kt_kernel_stats.csv ...

With --timed the entry also carries the line's own HIP-event kernel time and
roofline fraction, so the two can be compared launch for launch.
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = {'C2': 'extract_kernel', 'C3': 'extract_kernel', 'C5': 'orf6_kernel'}


def timed_launches(trace_csv, line):
    """Durations (ms) of the bench line's K timed launches, from the kernel
    trace of the same process: the kernel's dispatches in dispatch order,
    [first, first + count)."""
    tl = line['roofline']['timed_launches']
    name, first, count = tl['kernel'], int(tl['first']), int(tl['count'])
    rows = []
    with open(trace_csv) as fh:
        for row in csv.DictReader(fh):
            if name in row['Kernel_Name']:
                rows.append((int(row['Dispatch_Id']), int(row['Start_Timestamp']),
                             int(row['End_Timestamp'])))
    rows.sort()
    sel = rows[first:first + count]
    if len(sel) != count:
        raise SystemExit('%s: %d dispatches of %s, need [%d, %d)' % (trace_csv, len(rows), name,
                                                                     first, first + count))
    dur = [(e - s) * 1e-6 for _, s, e in sel]
    span = (sel[-1][2] - sel[0][1]) * 1e-6  # first start to last end
    return dur, span, len(rows)


def main(argv):
    timed = '--timed' in argv
    argv = [a for a in argv if a != '--timed']
    path = os.path.join(ROOT, 'profiles', 'rocprof_summary.json')
    out = {}
    if os.path.exists(path):
        with open(path) as fh:
            out = json.load(fh)
    for arg in argv:
        cfg, spec = arg.split('=', 1)
        if timed:
            trace_csv, line_json = spec.split(',')
            with open(line_json) as fh:
                line = json.loads([x for x in fh.read().splitlines() if x.startswith('{')][-1])
            dur, span, n_all = timed_launches(trace_csv, line)
            avg = sum(dur) / len(dur)
            r = line['roofline']
            alg = r['algorithmic_bytes_per_launch']
            out[cfg] = {'kernel': KERNEL[cfg], 'avg_ms': avg, 'calls': len(dur),
                        'min_ms': min(dur), 'max_ms': max(dur),
                        'timed_span_ms_per_launch': span / len(dur),
                        'all_calls': n_all,
                        'frac': alg / (avg * 1e-3) / 1e9 / r['peak'],
                        'line_kernel_ms': r['kernel_ms'], 'line_frac': r['frac'],
                        'line_ms_per_step': line['ms_per_step'],
                        'selection': 'the K timed launches (dispatches [%d, %d) of %s)'
                                     % (r['timed_launches']['first'],
                                        r['timed_launches']['first'] + len(dur), KERNEL[cfg]),
                        'source': os.path.relpath(os.path.abspath(trace_csv), ROOT),
                        'line': os.path.relpath(os.path.abspath(line_json), ROOT)}
            continue
        with open(spec) as fh:
            for row in csv.DictReader(fh):
                if KERNEL[cfg] in row['Name']:
                    out[cfg] = {'kernel': KERNEL[cfg], 'avg_ms': float(row['AverageNs']) * 1e-6,
                                'calls': int(row['Calls']),
                                'min_ms': float(row['MinNs']) * 1e-6,
                                'selection': 'every launch in the process (--stats)',
                                'source': os.path.relpath(os.path.abspath(spec), ROOT)}
    with open(path, 'w') as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1:])
