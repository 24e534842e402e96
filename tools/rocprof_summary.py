"""Summarise a rocprofv3 --kernel-trace --stats CSV run for one kernel (tools only).

    python tools/rocprof_summary.py <rocprof-output-dir> <kernel-name-substring> <out.json> [<stats-copy.csv>] [--last K]

Reads every *kernel_trace.csv under the directory, keeps the dispatches whose
kernel name contains the substring, and writes dispatch count, mean / median /
min / max duration (us), VGPR/SGPR/LDS and grid/workgroup sizes; optionally
copies the *kernel_stats.csv next to it.  ``--last K`` adds the same figures over
the last K dispatches (a bench's timed region) and their start-to-end span per launch.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys


def main():
    argv = sys.argv[1:]
    last = 0
    if "--last" in argv:
        i = argv.index("--last")
        last = int(argv[i + 1])
        del argv[i:i + 2]
    root, sub, out = argv[:3]
    rows = []
    for path in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if sub in r.get("Kernel_Name", ""):
                    rows.append(r)
    if not rows:
        raise SystemExit(f"no dispatch of a kernel matching {sub!r} under {root}")
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    r0 = rows[0]

    def field(*names):
        for n in names:
            if n in r0:
                return r0[n]
        return None

    res = {
        "source": f"rocprofv3 --kernel-trace --stats --output-format csv ({root})",
        "kernel": r0["Kernel_Name"],
        "dispatches": len(dur),
        "mean_us": statistics.fmean(dur),
        "median_us": statistics.median(dur),
        "min_us": min(dur),
        "max_us": max(dur),
        "vgpr": field("VGPR_Count", "Arch_VGPR_Count"),
        "sgpr": field("SGPR_Count"),
        "lds": field("LDS_Block_Size", "Group_Segment_Size"),
        "grid": field("Grid_Size", "Grid_Size_X"),
        "workgroup": field("Workgroup_Size", "Workgroup_Size_X"),
    }
    if last:
        tail = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))[-last:]
        td = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tail]
        span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
        res["timed_region"] = {"dispatches": len(td), "mean_us": statistics.fmean(td),
                               "median_us": statistics.median(td), "min_us": min(td), "max_us": max(td),
                               "span_per_launch_us": span / len(td)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    if len(argv) > 3:
        stats = glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)
        if stats:
            shutil.copy(stats[0], argv[3])


if __name__ == "__main__":
    main()
