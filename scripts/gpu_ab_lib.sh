#!/bin/bash
# A/B of alternative builds of the native library (variants/<name>, loaded through HFREP_NATIVE_LIB)
# against the default one: the fp32 split kernels (BPTT + dX, input gradient, weight gradients) and the
# headline step (fp32 + bf16).
#   bash scripts/gpu_ab_lib.sh <outdir> <variant> [<variant> ...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for V in base "$@"; do
  if [ $V = base ]; then unset HFREP_NATIVE_LIB
  else
    export HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so"
    test -f "$HFREP_NATIVE_LIB" || { echo "no $HFREP_NATIVE_LIB"; exit 1; }
  fi
  for K in 32 100; do
    timeout -k 10 200 python -u scripts/bench_lstm.py --dtype float32 --batch 262144 --K $K --iters 5 --only bwd_dx,dgrad \
      > $OUT/lstm_${V}_K$K.jsonl 2>&1 || { tail -n 20 $OUT/lstm_${V}_K$K.jsonl; exit 1; }
  done
  timeout -k 10 200 python -u scripts/bench_wgrad.py --dtype float32 --batch 262144 --iters 5 > $OUT/wgrad_$V.jsonl 2>&1 \
    || { tail -n 20 $OUT/wgrad_$V.jsonl; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > $OUT/bench_$V.json 2> $OUT/bench_$V.err \
    || { tail $OUT/bench_$V.err; exit 1; }
  echo "== $V"; grep -hv amdgpu.ids $OUT/lstm_${V}_K32.jsonl $OUT/lstm_${V}_K100.jsonl; grep -h '"kernel"' $OUT/wgrad_$V.jsonl; cat $OUT/bench_$V.json
done
