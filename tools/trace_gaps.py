"""Timeline of the last K dispatches of one kernel in a rocprofv3 kernel trace (tools only).

    python tools/trace_gaps.py <rocprof-output-dir> <kernel-substring> <K>

Prints per-launch duration and the gap to the previous launch's end (us), then
the span first-start -> last-end, the summed durations and the summed gaps:
separates what a K-step replay spends in kernels from what it spends between them.
"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    root, sub, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = []
    for path in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            rows += [r for r in csv.DictReader(f) if sub in r.get("Kernel_Name", "")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-k:]
    st = [int(r["Start_Timestamp"]) / 1e3 for r in rows]
    en = [int(r["End_Timestamp"]) / 1e3 for r in rows]
    dur = [e - s for s, e in zip(st, en)]
    gaps = [st[i] - en[i - 1] for i in range(1, len(rows))]
    print(" ".join(f"{d:.2f}" for d in dur))
    print("gaps", " ".join(f"{g:.2f}" for g in gaps))
    print(json.dumps({"launches": len(rows), "span_us": en[-1] - st[0], "sum_dur_us": sum(dur),
                      "sum_gap_us": sum(gaps), "mean_dur_us": statistics.mean(dur),
                      "median_dur_us": statistics.median(dur),
                      "mean_gap_us": statistics.mean(gaps) if gaps else 0.0,
                      "span_per_launch_us": (en[-1] - st[0]) / len(rows)}))


if __name__ == "__main__":
    main()
