#!/bin/bash
# Vectorised sampler / Philox fill: their GPU tests + determinism, then the MLP and LSTM benches.
#   bash scripts/gpu_r06_misc.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r06_misc}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_runtime.py -x -v --timeout 240 --timeout-method thread \
  -k "rng or sampling or determinism or trainer_gradients" > $OUT/tests.txt 2>&1
rc=$?; tail -n 5 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for M in wgan_gp gan; do
  timeout -k 10 300 python -u bench.py --model $M --dtype bfloat16 --steps 8 --warmup 2 > $OUT/bench_$M.json 2> $OUT/bench_$M.err \
    || { tail $OUT/bench_$M.err; exit 1; }
  cut -c100-160 $OUT/bench_$M.json
done
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
