"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into HBM bytes per launch.

    rocprofv3 --pmc FETCH_SIZE -d <dir> -o fetch --output-format csv -- python tools/pmc_probe.py
    rocprofv3 --pmc WRITE_SIZE -d <dir> -o write --output-format csv -- python tools/pmc_probe.py
    python tools/pmc_traffic.py <dir> profiles/r01/pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are in KiB (x1024).  They are separate passes because
FETCH_SIZE takes 3 of the 4 TCC counter slots and WRITE_SIZE 2
(MI355X_MICROARCH.md, rocprofv3 PMC slots).  gfx950 correction: the counters
are exact only for some access widths (FETCH_SIZE reads half of a 16 B/lane
stream), so each direction is scaled by a factor measured on a calibration
kernel with the dequant kernel's own access shape and a known byte count
(tools/pmc_calib.hip: 4 B/lane dword loads, 16 B/lane nt stores).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CALIB_BYTES = 1 << 30


def load(d, prefix, counter):
    files = glob.glob(os.path.join(d, "**", f"{prefix}*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no {prefix}*counter_collection.csv under {d}")
    vals = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def mean_for(vals, key):
    xs = [v for k, vs in vals.items() if key in k for v in vs]
    if not xs:
        raise SystemExit(f"no dispatches of {key}")
    return sum(xs) / len(xs), len(xs)


def main():
    d, out = sys.argv[1], sys.argv[2]
    m = int(os.environ.get("PMC_M", "4096"))
    n = int(os.environ.get("PMC_N", "4096"))
    fetch = load(d, "fetch", "FETCH_SIZE")
    write = load(d, "write", "WRITE_SIZE")
    cr, _ = mean_for(fetch, "calib_read_dword")
    cw, _ = mean_for(write, "calib_write_x4")
    rf = CALIB_BYTES / (cr * 1024.0)
    wf = CALIB_BYTES / (cw * 1024.0)
    # PMC_KERNEL: the kernel name to average (default the flat kernel; nf4_chunk for
    # tools/pmc_chunk.py's forms, whose shape PMC_CASE names)
    kname = os.environ.get("PMC_KERNEL", "nf4_flat_kernel")
    case = os.environ.get("PMC_CASE")
    if case:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from chunk_ab import SHAPES
        m, n, _ = SHAPES[case]
    kf, nf = mean_for(fetch, kname)
    kw, nw = mean_for(write, kname)
    fetch_b = kf * 1024.0 * rf
    write_b = kw * 1024.0 * wf
    N = m * n
    alg_r = N // 2 + N // 64 + 4 * ((N // 64 + 255) // 256)
    alg_w = 2 * N
    if case:  # tools/chunk_ab.py's algorithmic bytes (its frac): SURVEY 8(d) per element
        from bench_configs import alg_bytes
        alg_r = alg_bytes(m, n, 2) - 2 * N
    res = {"m": m, "n": n, "dtype": os.environ.get("PMC_DTYPE", "bf16"), "kernel": kname, "case": case,
           "fetch_kib_raw": kf, "write_kib_raw": kw, "dispatches": [nf, nw],
           "read_factor_dword_loads": rf, "write_factor_x4_nt_stores": wf,
           "hbm_read_bytes_per_launch": fetch_b, "hbm_write_bytes_per_launch": write_b,
           "hbm_bytes_per_launch": fetch_b + write_b,
           "algorithmic_read_bytes": alg_r, "algorithmic_write_bytes": alg_w,
           "read_over_algorithmic": fetch_b / alg_r, "write_over_algorithmic": write_b / alg_w,
           "traffic_over_algorithmic": (fetch_b + write_b) / (alg_r + alg_w)}
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
