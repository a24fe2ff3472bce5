#!/bin/bash
# Per-call A/B of library variants (variants/<name>, HFREP_NATIVE_LIB) on bench_lstm ops, no tests / bench.
#   bash scripts/gpu_ab_ops.sh OUTNAME DTYPE OPS VARIANT [VARIANT ...]   (OPS: bench_lstm --only list)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/$1; DT=$2; OPS=$3; shift 3; mkdir -p $OUT; export TMPDIR=/tmp
for V in base "$@"; do
  if [ $V = base ]; then unset HFREP_NATIVE_LIB; else export HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so"; fi
  for K in 32 100; do
    timeout -k 10 200 python -u scripts/bench_lstm.py --dtype $DT --batch 262144 --K $K --iters 10 --only $OPS \
      > $OUT/lstm_${V}_K$K.jsonl 2>&1 || { tail -n 20 $OUT/lstm_${V}_K$K.jsonl; exit 1; }
  done
  echo "== $V"; grep -hv amdgpu.ids $OUT/lstm_${V}_K*.jsonl
done
