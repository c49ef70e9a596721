#!/usr/bin/env python3
"""Per-kernel mean of each SQ counter over the dispatches in rocprofv3
counter_collection CSVs (tools/jobs/pmc_layer.sh)."""
import csv
import sys
from collections import defaultdict

sums = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
for path in sys.argv[1:]:
    with open(path, newline="") as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"].split("(")[0][-70:]
            c = r["Counter_Name"]
            sums[k][c] += float(r["Counter_Value"])
            disp[k][c].add(r["Dispatch_Id"])
for k in sums:
    print(k)
    for c in sorted(sums[k]):
        n = max(1, len(disp[k][c]))
        print(f"   {c:28s} {sums[k][c] / n:16.0f}")
