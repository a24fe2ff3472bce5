#!/bin/bash
# Round-6 fused MLP path: its GPU tests, then bench.py --model wgan_gp|gan in both dtypes.
#   bash scripts/gpu_r06_mlp.sh OUTNAME [skip-tests]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r06_mlpf}; mkdir -p $OUT; export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_mlp_fused_gpu.py -x -v --timeout 240 --timeout-method thread > $OUT/tests.txt 2>&1
  rc=$?; tail -n 30 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
fi
for M in wgan_gp gan; do
  for dt in bfloat16 float32; do
    timeout -k 10 300 python -u bench.py --model $M --dtype $dt --steps 5 --warmup 2 > $OUT/bench_${M}_$dt.json 2> $OUT/bench_${M}_$dt.err \
      || { tail $OUT/bench_${M}_$dt.err; exit 1; }
    cut -c1-200 $OUT/bench_${M}_$dt.json
  done
done
