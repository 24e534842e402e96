# round 5 session 39: the chunk kernel's general forms (padded rows, unaligned packed
# pointer, n % 8 != 0 through the LDS-staged span) beside the flat and dense forms
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s39
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chunks.py -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider > $O/pytest.txt 2>&1
tail -2 $O/pytest.txt
timeout -k 10 400 python -u tools/chunk_ab.py --rounds 7 --cases flat_4096,chunk_4080,pad_4096,unal_4096,chunk_4090,chunk_4095 > $O/chunk_forms.jsonl 2> $O/err.txt
python -c "import json;[print(d['case'],d['us_median'],d['frac']) for d in map(json.loads,open('$O/chunk_forms.jsonl'))]"
