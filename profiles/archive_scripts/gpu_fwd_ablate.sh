#!/bin/bash
# Timing-only ablations of the v4 forward (HFREP_LSTM_DBG bits, see csrc/lstm2.hip lstm_dbg()).
# usage: bash scripts/gpu_fwd_ablate.sh <tag> <batch>
set -e
tag=$1; B=${2:-262144}
out=gpurun_out/$tag; mkdir -p $out
for d in 0 1 2 4 6 7 256; do
  HFREP_LSTM_DBG=$d timeout -k 10 120 python scripts/bench_lstm.py --batch $B --only fwd,fwd_notape,tfwd --iters 5 \
    | sed "s/^{/{\"dbg\": $d, /" >> $out/ablate.jsonl
done
HFREP_LSTM_DBG=0 timeout -k 10 120 python scripts/bench_lstm.py --batch $B --act 1 --only fwd --iters 5 \
    | sed "s/^{/{\"dbg\": 0, \"act\": 1, /" >> $out/ablate.jsonl
