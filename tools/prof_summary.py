#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV per (kernel, grid size): the bench's
timed launches are separated from its setup launches by grid size.

    python tools/prof_summary.py profiles/r01_kernel_trace.csv
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"xrs::\(anonymous namespace\)::(\w+<[^>]*>)", name)
    return m.group(1) if m else name.split("(")[0][:48]


def main(path):
    groups = defaultdict(list)
    for r in csv.DictReader(open(path)):
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        groups[(short(r["Kernel_Name"]), int(r["Grid_Size_X"]))].append(dur)
    print(f"{'kernel':44s} {'grid':>10s} {'calls':>5s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s}")
    for (k, g), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:44s} {g:10d} {len(v):5d} {sum(v)/len(v):9.1f} {min(v):9.1f} {max(v):9.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
