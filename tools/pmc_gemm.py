"""Summarise rocprofv3 --pmc passes of a decode-GEMM probe run (tools only).

    rocprofv3 --pmc <8 SQ counters> -d <dir> -o passA --output-format csv -- python tools/gemm_probe.py ...
    python tools/pmc_gemm.py <dir> <kernel-substring> [<kernel-substring> ...] > summary.jsonl

Prints, per kernel substring, the median over its dispatches of every counter found
(values are device totals per dispatch).
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def main():
    d, subs = sys.argv[1], sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            for s in subs:
                if s in r.get("Kernel_Name", ""):
                    vals[s][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for s in subs:
        out = {"kernel": s}
        for c, xs in sorted(vals[s].items()):
            out[c] = statistics.median(xs)
            out.setdefault("dispatches", len(xs))
        print(json.dumps(out))


if __name__ == "__main__":
    main()
