#!/usr/bin/env python3
"""Mean of every counter per (kernel, grid size) over the dispatches of one or
more rocprofv3 --pmc output directories.  Raw counter values, no
corrections (the HBM byte corrections live in tools/pmc_traffic.py)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main():
    vals = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                name = row.get("Kernel_Name", "").replace("(anonymous namespace)::", "")
                name = re.sub(r"^void ", "", name)
                name = name[: name.index("(")] if "(" in name else name
                grid = int(float(row.get("Grid_Size", row.get("Grid_Size_X", 0)) or 0))
                vals[(name, grid)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for (name, grid), cs in sorted(vals.items()):
        if not name.startswith("xrs::"):
            continue
        print(json.dumps({"kernel": name, "grid_threads": grid,
                          **{c: round(sum(v) / len(v), 1) for c, v in sorted(cs.items())}}))


if __name__ == "__main__":
    main()
