# round 5 session 42: the headline's launches over 1-4 independent streams (the reference
# harness's 3-stream pattern): how much of a dependent launch the boundary costs
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s42
mkdir -p $O
timeout -k 10 300 python -u tools/multistream_probe.py --streams 1,2,3,4 --steps 128 --rounds 7 > $O/multistream.jsonl 2> $O/err.txt
cat $O/multistream.jsonl
