#!/usr/bin/env python3
"""Per-kernel PMC summary of rocprofv3 ``--pmc ... --output-format csv`` outputs: mean counter value per dispatch
for kernels whose name matches a substring.  Usage: python tools/pmc_summary.py CSV [CSV...] --match kmeans_v"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    for path in a.csv:
        acc = collections.defaultdict(list)
        for row in csv.DictReader(open(path)):
            name = row.get("Kernel_Name", "")
            if a.match not in name:
                continue
            acc[(name[:70], row["Counter_Name"], row["Dispatch_Id"])].append(float(row["Counter_Value"]))
        per = collections.defaultdict(list)
        for (name, ctr, _), vals in acc.items():
            per[(name, ctr)].append(sum(vals))
        print(f"== {path}")
        for (name, ctr), vals in sorted(per.items()):
            print(f"  {name:70s} {ctr:28s} {sum(vals) / len(vals):14.4e}  (n={len(vals)})")


if __name__ == "__main__":
    main()
