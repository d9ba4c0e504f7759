#!/usr/bin/env python3
"""HBM bytes per dispatch from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE) of any command -- e.g. tools/refbench.py -- in dispatch order,
with consecutive dispatches of the same kernel and the same byte counts
(within 2%) collapsed into one line.  Same gfx950 corrections as
tools/pmc_traffic.py (KiB; FETCH_SIZE x 2)."""
import csv
import glob
import json
import os
import re
import sys


def read(d, counter):
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "").replace("(anonymous namespace)::", "")
            name = re.sub(r"^void ", "", name)
            name = name[: name.index("(")] if "(" in name else name
            rows[int(row["Dispatch_Id"])] = (name, float(row["Counter_Value"]))
    return [rows[k] for k in sorted(rows)]


def main():
    fetch, write = read(sys.argv[1], "FETCH_SIZE"), read(sys.argv[2], "WRITE_SIZE")
    runs = []
    for (name, f), (name2, w) in zip(fetch, write):
        f, w = f * 2048, w * 1024
        if name != name2:
            raise SystemExit("passes dispatched different kernels")
        last = runs[-1] if runs else None
        if (last and last["kernel"] == name and abs(last["fetch_bytes"] - f) <= 0.02 * f + 4096
                and abs(last["write_bytes"] - w) <= 0.02 * w + 4096):
            last["dispatches"] += 1
            continue
        runs.append({"kernel": name, "dispatches": 1, "fetch_bytes": int(f), "write_bytes": int(w)})
    for r in runs:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
