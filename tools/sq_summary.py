#!/usr/bin/env python3
"""Per-kernel averages of the SQ / SQC counters collected by tools/gpu_sqpmc.sh
(rocprofv3 counter_collection.csv), over the dispatches with the largest grid
of each kernel (the bench's timed workload)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    out = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        grid = defaultdict(int)
        for r in rows:
            grid[r["Kernel_Name"]] = max(grid[r["Kernel_Name"]], int(r.get("Grid_Size", 0) or 0))
        per = defaultdict(lambda: defaultdict(float))
        for r in rows:
            k = r["Kernel_Name"]
            if int(r.get("Grid_Size", 0) or 0) != grid[k]:
                continue
            per[(k, r.get("Dispatch_Id", ""))][r["Counter_Name"]] += float(r["Counter_Value"])
        for (k, _), cs in per.items():
            for c, v in cs.items():
                m = re.search(r"(k0_tables|k2_place<[^>]*>|k3_winner|copyBuffer)", k)
                acc[m.group(1) if m else k[:40]][c].append(v)
    for k, cs in acc.items():
        print(k)
        for c in sorted(cs):
            vals = cs[c]
            print("   %-28s %14.1f  (%d dispatches)" % (c, sum(vals) / len(vals), len(vals)))


if __name__ == "__main__":
    main()
