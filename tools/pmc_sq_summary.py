"""Per-wave SQ counters of one kernel family from rocprofv3 --pmc CSVs (tools only).

    python tools/pmc_sq_summary.py <kernel substring> <dir> [<dir> ...] > out.jsonl

Each <dir> holds one rocprofv3 run (``*counter_collection.csv``, optionally
``*kernel_trace.csv`` from the same run): per kernel name, the median over dispatches of
each counter, divided by SQ_WAVES (per-wave instructions / quad-cycles), and the median
kernel duration from the trace.  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count
quad-cycles (MI355X_MICROARCH.md).
"""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys


def main():
    key, dirs = sys.argv[1], sys.argv[2:]
    for d in dirs:
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(files[0])):
            if key in r["Kernel_Name"]:
                vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        durs = collections.defaultdict(list)
        for tr in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(tr)):
                if key in r["Kernel_Name"]:
                    durs[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for k, cs in vals.items():
            med = {c: statistics.median(v) for c, v in cs.items()}
            waves = med.get("SQ_WAVES") or 1.0
            print(json.dumps({"run": os.path.basename(os.path.normpath(d)), "kernel": (re.search(r"\w+<[^>]*>|\w+(?=\()", k.replace("(anonymous namespace)::", "")) or [k])[0],
                              "dispatches": max(len(v) for v in cs.values()),
                              "duration_us_median": round(statistics.median(durs[k]), 3) if durs[k] else None,
                              "waves": waves,
                              "per_wave": {c: round(v / waves, 1) for c, v in sorted(med.items()) if c != "SQ_WAVES"}}))


if __name__ == "__main__":
    main()
