#!/bin/bash
# Round-5 GPU pass 5 (after the BPTT switch to lstm_tbwd4<TG = false> and the lstm_bwd3 deletion): the bf16
# LSTM / trainer GPU tests, bf16 W-dist parity at the reference preset (3 seeds), then the first segment
# of the bf16 B = 32 768 parity run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_fifth}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "lstm2 or bf16 or lstm_fwd_bwd or slice_averages or lstm_tangent" > $OUT/tests_bf16.txt 2>&1
rc=$?; tail -n 4 $OUT/tests_bf16.txt; [ $rc -eq 0 ] || exit $rc
PARITY_TIMEOUT=300 bash scripts/gpu_parity.sh ${1:-r05_fifth} "bfloat16:32:123 bfloat16:32:124 bfloat16:32:125" || exit 1
PARITY_TIMEOUT=${SEG_TIMEOUT:-560} bash scripts/gpu_parity_seg.sh ${1:-r05_fifth} "bfloat16:32768:123:${SEG_STOP:-2700}"
