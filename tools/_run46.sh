# Per-set absmax placement at 8192^2: separate small allocations vs slices of one slab
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r46 && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/value_sensitivity.py > gpurun_out/r46/value_sensitivity.jsonl 2> gpurun_out/r46/vs.err || exit 1
cat gpurun_out/r46/value_sensitivity.jsonl
