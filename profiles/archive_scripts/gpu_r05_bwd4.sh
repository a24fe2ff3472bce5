#!/bin/bash
# Round-5 A/B: the bf16 BPTT on lstm_tbwd4<TG = false> (HFREP_LSTM_BWD=4) vs lstm_bwd3 (=3): the bf16
# BPTT-touching GPU tests under impl 4, per-call times at the bench shape, the bench step and B = 32.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_bwd4}; mkdir -p $OUT; export TMPDIR=/tmp
HFREP_LSTM_BWD=4 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "lstm2 or bf16 or lstm_fwd_bwd or slice_averages or lstm_tangent" > $OUT/tests_bwd4.txt 2>&1
rc=$?; tail -n 4 $OUT/tests_bwd4.txt; [ $rc -le 1 ] || exit $rc
for I in 3 4; do
  for K in 32 100; do
    HFREP_LSTM_BWD=$I timeout -k 10 200 python -u scripts/bench_lstm.py --dtype bfloat16 --batch 262144 --K $K --iters 10 \
      --only bwd,bwd_dx > $OUT/lstm_bwd${I}_K$K.jsonl 2>&1 || { tail -n 20 $OUT/lstm_bwd${I}_K$K.jsonl; exit 1; }
  done
  echo "== impl $I"; grep -hv amdgpu.ids $OUT/lstm_bwd${I}_K*.jsonl
done
for I in 3 4; do
  HFREP_LSTM_BWD=$I timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --dtype bfloat16 > $OUT/bench_bwd$I.json 2> $OUT/bench_bwd$I.err \
    || { tail $OUT/bench_bwd$I.err; exit 1; }
  echo "== impl $I bench"; cat $OUT/bench_bwd$I.json
  HFREP_LSTM_BWD=$I timeout -k 10 300 python -u scripts/bench_small.py --iters 300 --dtypes bfloat16 > $OUT/small_bwd$I.jsonl 2>&1 \
    || { tail -n 20 $OUT/small_bwd$I.jsonl; exit 1; }
  grep -h '"ms' $OUT/small_bwd$I.jsonl
done
