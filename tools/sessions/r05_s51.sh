# round 5 session 51: after merging the chunk kernel's staged-store instantiations -- chunk
# tests, a misaligned C-ABI dequant sweep
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_s51
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider > $O/pytest.txt 2>&1
tail -2 $O/pytest.txt
timeout -k 10 400 python -u tools/fuzz_dequant.py --cases 30000 --seed 83 --seconds 240 --abi-rate 0.6 > $O/fuzz_dequant.jsonl 2> $O/fuzz.err
tail -1 $O/fuzz_dequant.jsonl
