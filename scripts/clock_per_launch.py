"""Per-launch duration and effective engine clock of one kernel from a
rocprofv3 --pmc GRBM_GUI_ACTIVE counter-collection CSV:
clock = GRBM_GUI_ACTIVE / 8 XCDs / (End - Start).
    python scripts/clock_per_launch.py DIR KERNEL_SUBSTRING
prints a JSON summary (median duration, median clock, first/last launches)."""
import csv
import glob
import json
import os
import statistics
import sys

root, kern = sys.argv[1], sys.argv[2]
rows = []
for f in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r['Kernel_Name'] and r['Counter_Name'] == 'GRBM_GUI_ACTIVE':
            d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-6
            rows.append((int(r['Dispatch_Id']), d, float(r['Counter_Value']) / 8 / (d * 1e-3) / 1e9))
rows.sort()
ds = [r[1] for r in rows]
cs = [r[2] for r in rows]
print(json.dumps({'launches': len(rows), 'median_ms': statistics.median(ds) if ds else None,
                  'median_ghz': statistics.median(cs) if cs else None,
                  'last20_ms': statistics.median(ds[-20:]) if ds else None,
                  'last20_ghz': statistics.median(cs[-20:]) if cs else None}))
