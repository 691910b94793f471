"""profiles/rocprof_summary.json from rocprofv3 --kernel-trace --stats CSVs:
per configuration, the average duration of its measured kernel, quoted by
bench.py beside its live HIP-event time.

    python scripts/rocprof_summary.py C3=profiles/r03e/kt_kernel_stats.csv \
        C5=profiles/r03e/kt_C5_kernel_stats.csv C2=...
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = {'C2': 'extract_kernel', 'C3': 'extract_kernel', 'C5': 'orf6_kernel'}


def main(argv):
    path = os.path.join(ROOT, 'profiles', 'rocprof_summary.json')
    out = {}
    if os.path.exists(path):
        with open(path) as fh:
            out = json.load(fh)
    for arg in argv:
        cfg, csv_path = arg.split('=', 1)
        with open(csv_path) as fh:
            for row in csv.DictReader(fh):
                if KERNEL[cfg] in row['Name']:
                    out[cfg] = {'kernel': KERNEL[cfg], 'avg_ms': float(row['AverageNs']) * 1e-6,
                                'calls': int(row['Calls']),
                                'min_ms': float(row['MinNs']) * 1e-6,
                                'source': os.path.relpath(os.path.abspath(csv_path), ROOT)}
    with open(path, 'w') as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1:])
