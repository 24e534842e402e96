# round 6 session 34: rocprofv3 kernel trace of the Llama-3-8B decode pass at M = 1 on the
# final tree -- per-kernel statistics (the decode GEMV on o_proj / down_proj, the persistent
# kernel on the grouped q/k/v and gate/up launches).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_s34
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o pass -- \
    python3 -u tools/bench_gemm.py --ms 1 --no-bf16 --no-composite > $O/pass.out 2> $O/pass.err
cat $O/pass.out
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
cp "$f" $O/decode_pass_m1_kernel_stats.csv
python3 - "$O/decode_pass_m1_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1e3, 3))
PY
find $O/prof -name '*kernel_trace.csv' -delete
