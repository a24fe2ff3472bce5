#!/bin/bash
# Two workgroups per CU for the no-dX BPTT (HFREP_BWD_2WG): kernel tests on the new default, per-op A/B against the
# one-per-CU build (variants/bwd1wg), twice interleaved, then the headline bench on the new default.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
N=${1:-r05_bwd2wg}; OUT=gpurun_out/$N; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_runtime.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
bash scripts/gpu_ab_ops.sh $N/ab1 bfloat16 bwd,bwd_dx bwd1wg || exit 1
bash scripts/gpu_ab_ops.sh $N/ab2 bfloat16 bwd,bwd_dx bwd1wg || exit 1
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
