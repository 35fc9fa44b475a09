#!/usr/bin/env python3
"""Per-launch HBM traffic of the planner kernels from rocprofv3 PMC passes.

  python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json>

<fetch_dir> / <write_dir> are the `-d` directories of two separate
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` runs of the same bench
command (one TCC block cannot hold both counters).  Per the gfx950 recipe of
MI355X_MICROARCH.md §HBM and cdna_hip_programming.md §7 (traffic pricing):
both counters are KiB, and FETCH_SIZE reports half the bytes of a wide
coalesced read, so

  traffic_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024

averaged over each kernel's launches (the first two dropped as warm-up when
there are more than four).  Writes {kernel key: bytes per launch, "_raw":
{...}}; bench.py puts the dominant kernel's entry into roofline.traffic.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KEYS = {"k2_place": "k2_placement", "k2_node": "k2_placement", "k0_tables": "k0_tables", "k0_incremental": "k0_tables",
        "k3_winner": "k3_winner"}


def kernel_key(name):
    for frag, key in KEYS.items():
        if frag in name:
            return key
    return None


def per_launch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under %s" % d)
    by_dispatch = defaultdict(float)
    kname = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                key = kernel_key(row.get("Kernel_Name", ""))
                if key is None:
                    continue
                disp = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                by_dispatch[disp] += float(row["Counter_Value"])  # summed over dimensions
                kname[disp] = key
    out = defaultdict(list)
    for disp in sorted(by_dispatch, key=lambda x: (x[0], int(x[1]) if str(x[1]).isdigit() else 0)):
        out[kname[disp]].append(by_dispatch[disp])
    return out


def main():
    fetch_dir, write_dir, path = sys.argv[1:4]
    fetch = per_launch(fetch_dir, "FETCH_SIZE")
    write = per_launch(write_dir, "WRITE_SIZE")
    res = {"_raw": {}, "measured_at_head": os.environ.get("SR_SOURCE_HEAD", "unknown"),
           "command": os.environ.get("SR_PMC_COMMAND", "bench.py (see tools/gpu_round.sh)")}
    for key in sorted(set(fetch) | set(write)):
        f = fetch.get(key, [])
        w = write.get(key, [])
        f_s = f[2:] if len(f) > 4 else f
        w_s = w[2:] if len(w) > 4 else w
        fk = sum(f_s) / len(f_s) if f_s else 0.0
        wk = sum(w_s) / len(w_s) if w_s else 0.0
        res[key] = int(round((2.0 * fk + wk) * 1024))
        res["_raw"][key] = {"FETCH_SIZE_KiB_avg": round(fk, 3), "WRITE_SIZE_KiB_avg": round(wk, 3),
                            "launches_fetch": len(f), "launches_write": len(w),
                            "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 B (gfx950 FETCH_SIZE halving)"}
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
