#!/bin/bash
# wgrad3 split count by M: numerics of variants/<v>, then the reference preset (B = 32) and the bench-shape
# kernel timing, base vs variant.   bash profiles/archive_scripts/gpu_ab_w3s.sh <outdir> <variant>
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/$1; V=$2; mkdir -p $OUT
VL="$R/variants/$V/_hfrep_native.so"; test -f "$VL" || { echo "no $VL"; exit 1; }
HFREP_NATIVE_LIB="$VL" timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "wgrad" > $OUT/tests_$V.log 2>&1 || { tail -n 30 $OUT/tests_$V.log; exit 1; }
tail -n 1 $OUT/tests_$V.log
for L in base $V; do
  if [ $L = base ]; then unset HFREP_NATIVE_LIB; else export HFREP_NATIVE_LIB="$VL"; fi
  timeout -k 10 300 python -u scripts/bench_small.py --dtypes bfloat16,float32 --iters 200 > $OUT/small_$L.jsonl 2>&1 \
    || { tail -n 20 $OUT/small_$L.jsonl; exit 1; }
  timeout -k 10 200 python -u scripts/bench_wgrad.py --dtype bfloat16 --batch 262144 --iters 5 > $OUT/wgrad_$L.jsonl 2>&1 \
    || { tail -n 20 $OUT/wgrad_$L.jsonl; exit 1; }
  echo "== $L"; grep -h '^{' $OUT/small_$L.jsonl; grep -h '"kernel": "wgrad3"' $OUT/wgrad_$L.jsonl
done
