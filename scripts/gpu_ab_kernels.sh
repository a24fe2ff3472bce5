#!/bin/bash
# Per-call A/B of alternative library builds (variants/<name>, HFREP_NATIVE_LIB) on the fp32 LSTM ops at
# the bench shape, then the headline step for each.
#   bash scripts/gpu_ab_kernels.sh <outdir> <ops> <variant> [<variant> ...]   (ops: bench_lstm --only list)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/$1; OPS=$2; shift 2; mkdir -p $OUT
for V in base "$@"; do
  if [ $V = base ]; then unset HFREP_NATIVE_LIB
  else
    export HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so"
    test -f "$HFREP_NATIVE_LIB" || { echo "no $HFREP_NATIVE_LIB"; exit 1; }
  fi
  for K in 32 100; do
    timeout -k 10 200 python -u scripts/bench_lstm.py --dtype float32 --batch 262144 --K $K --iters 5 --only $OPS \
      > $OUT/lstm_${V}_K$K.jsonl 2>&1 || { tail -n 20 $OUT/lstm_${V}_K$K.jsonl; exit 1; }
  done
  echo "== $V"; grep -hv amdgpu.ids $OUT/lstm_${V}_K32.jsonl $OUT/lstm_${V}_K100.jsonl
done
if [ -n "$AB_BENCH" ]; then
  for V in base "$@"; do
    if [ $V = base ]; then unset HFREP_NATIVE_LIB; else export HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so"; fi
    timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --dtype float32 > $OUT/bench_$V.json 2> $OUT/bench_$V.err \
      || { tail $OUT/bench_$V.err; exit 1; }
    echo "== $V bench"; cat $OUT/bench_$V.json
  done
fi
