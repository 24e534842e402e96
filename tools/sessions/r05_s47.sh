# round 5 session 47: after the past-end-wave fix in the chunk kernels -- the fuzz_api seed
# that faulted (61), the chunk tests, the full GPU suite
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s47
mkdir -p $O
timeout -k 10 300 python -u tools/fuzz_api.py --rounds 800 --seed 61 --seconds 200 > $O/fuzz_api_seed61.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz_api_seed61.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gputest.log.txt 2>&1
tail -2 $O/gputest.log.txt
