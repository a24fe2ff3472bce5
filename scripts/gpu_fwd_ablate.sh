#!/bin/bash
# Timing-only ablations of the bf16 forward (HFREP_LSTM_DBG: 1 no tape stores, 2 no h stores, 4 no x loads,
# 256 tape stores to one L2-resident slot set) at the bench shape: what bounds lstm_fwd4.
#   bash scripts/gpu_fwd_ablate.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-fwd_ablate}; mkdir -p $OUT; export TMPDIR=/tmp
for D in 0 1 2 3 4 7 256; do
  for K in 32 100; do
    HFREP_LSTM_DBG=$D timeout -k 10 200 python -u scripts/bench_lstm.py --dtype bfloat16 --batch 262144 --K $K --iters 10 \
      --only fwd,tfwd > $OUT/fwd_dbg${D}_K$K.jsonl 2>&1 || { tail -n 20 $OUT/fwd_dbg${D}_K$K.jsonl; exit 1; }
  done
  echo "== dbg $D"; grep -hv amdgpu.ids $OUT/fwd_dbg${D}_K*.jsonl
done
