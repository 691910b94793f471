"""Average rocprofv3 PMC counters per kernel launch under a directory.

    python scripts/pmc_summary.py DIR [KERNEL_SUBSTRING=extract_kernel]
"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
kernel = sys.argv[2] if len(sys.argv) > 2 else 'extract_kernel'
out = {}
for f in sorted(glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True)):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kernel in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    tag = os.path.relpath(os.path.dirname(f), root)
    out[tag] = {k: sum(v) / len(v) for k, v in agg.items()}
print(json.dumps(out, indent=1))
