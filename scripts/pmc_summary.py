"""Average rocprofv3 PMC counters per extract_kernel launch under a directory."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
out = {}
for f in sorted(glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True)):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'extract_kernel' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    tag = os.path.relpath(os.path.dirname(f), root)
    out[tag] = {k: sum(v) / len(v) for k, v in agg.items()}
print(json.dumps(out, indent=1))
