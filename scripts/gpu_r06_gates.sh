#!/bin/bash
# Gate-recompute bound (verdict r05 #2): per-call times of the bf16 recurrent kernels with the shipped
# library vs the timing-only HFREP_ABLATE_GATES=1 build (forward stores only the cell slot, reverse
# kernels skip the four gate-slot loads) at the bench shape.
#   bash scripts/gpu_r06_gates.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r06_gates}; mkdir -p $OUT; export TMPDIR=/tmp
for V in shipped nogates; do
  LIB=""; [ $V = nogates ] && LIB="$R/variants/nogates/_hfrep_native.so"
  for K in 32 100; do
    HFREP_NATIVE_LIB=$LIB timeout -k 10 300 python -u scripts/bench_lstm.py --dtype bfloat16 --batch 262144 --K $K --iters 10 \
      --only fwd,tfwd,bwd,tbwd,bwd_dx,tbwd_dx > $OUT/${V}_K$K.jsonl 2>&1 || { tail -n 20 $OUT/${V}_K$K.jsonl; exit 1; }
  done
  echo "== $V"; grep -hv amdgpu.ids $OUT/${V}_K*.jsonl
done
