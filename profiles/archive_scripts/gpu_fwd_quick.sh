#!/bin/bash
# LSTM kernel GPU tests + recurrent-kernel microbench at 16k and 262k.  usage: bash scripts/gpu_fwd_quick.sh <tag>
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "lstm" --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for B in 16384 262144; do
  timeout -k 10 200 python scripts/bench_lstm.py --batch $B --only fwd,fwd_notape,tfwd,bwd,bwd_dx,tbwd,tbwd_dx --iters 5 >> $out/lstm.jsonl || exit 1
done
cat $out/lstm.jsonl
