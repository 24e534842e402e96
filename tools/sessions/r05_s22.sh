# round 5 session 22: per-wave phase stamps of the final kernel in bench.py's regime (last
# of 24 back-to-back launches; the boundary from the previous launch seen by the waves),
# and cold single launches for comparison
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s22
mkdir -p $O
test -f tools/_build/libnf4dq_stamps.so
timeout -k 10 300 python -u tools/flat_stamps.py --shape 4096,4096 --stream 24 --reps 12 > $O/flat_stamps_stream_4096.json 2> $O/stamps.err
cat $O/flat_stamps_stream_4096.json
timeout -k 10 300 python -u tools/flat_stamps.py --shape 4096,4096 --reps 12 > $O/flat_stamps_cold_4096.json 2>> $O/stamps.err
cat $O/flat_stamps_cold_4096.json
# the rocprof trace again, with a lead spin long enough for rocprofv3's slower submission
# (at 150 us/launch the last ~35 of 216 launches of session 21 trickled in with gaps)
bash tools/session.sh r05_s22 rocprof > $O/session.log 2>&1 || { tail -20 $O/session.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/rocprof_bench_summary.json'));print(d['timed_region'])"
tail -1 $O/bench_gaps.txt
