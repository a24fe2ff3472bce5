#!/bin/bash
# fwd4 tile-stride A/B (HFREP_FW4_STRIDE): kernel tests on the new default, per-op A/B against the
# KP + 8 build (variants/fw4old), twice interleaved, then the headline bench on the new default.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_fw4}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "lstm2 or fwd or tfwd" > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
bash scripts/gpu_ab_ops.sh ${1:-r05_fw4}/ab1 bfloat16 fwd,fwd_notape,tfwd fw4old || exit 1
bash scripts/gpu_ab_ops.sh ${1:-r05_fw4}/ab2 bfloat16 fwd,fwd_notape,tfwd fw4old || exit 1
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
