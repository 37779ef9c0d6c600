"""Mean per-dispatch value of every counter in a rocprofv3 --pmc run, per kernel.

usage: pmc_sum.py <run_dir> [kernel_substring]
Prints one line per (kernel, counter): dispatches and mean value.  SQ_*_CYCLES and
SQ_WAIT_* count quad-cycles on gfx950 (MI355X_MICROARCH.md, per-instruction table).
"""
import collections
import csv
import sys


def main():
    rdir = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = collections.defaultdict(list)
    with open(f"{rdir}/run_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"]
            if sub in k:
                acc[(k.split("(")[0][:60], row["Counter_Name"])].append(float(row["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(f"{k:60s} {c:24s} n={len(v):3d} mean={sum(v) / len(v):.6g}")


if __name__ == "__main__":
    main()
