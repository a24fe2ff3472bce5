#!/bin/bash
# bf16 LSTM weight gradient (lstm_wgrad3): numerics of variants/<v> (HFREP_NATIVE_LIB), then base vs
# variant kernel timing and the bf16 step.
#   bash profiles/archive_scripts/gpu_ab_w3.sh <outdir> <variant>
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/$1; V=$2; mkdir -p $OUT
VL="$R/variants/$V/_hfrep_native.so"; test -f "$VL" || { echo "no $VL"; exit 1; }
HFREP_NATIVE_LIB="$VL" timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "wgrad" > $OUT/tests_$V.log 2>&1 || { tail -n 30 $OUT/tests_$V.log; exit 1; }
tail -n 1 $OUT/tests_$V.log
for L in base $V; do
  if [ $L = base ]; then unset HFREP_NATIVE_LIB; else export HFREP_NATIVE_LIB="$VL"; fi
  timeout -k 10 200 python -u scripts/bench_wgrad.py --dtype bfloat16 --batch 262144 --iters 5 > $OUT/wgrad_$L.jsonl 2>&1 \
    || { tail -n 20 $OUT/wgrad_$L.jsonl; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --dtype bfloat16 > $OUT/bench_$L.json 2> $OUT/bench_$L.err \
    || { tail $OUT/bench_$L.err; exit 1; }
  echo "== $L"; grep -h '"kernel": "wgrad3"' $OUT/wgrad_$L.jsonl; cat $OUT/bench_$L.json
done
