#!/bin/bash
# Tape-store cache-policy experiment (B = 262144 forward / tangent forward timings).
mkdir -p gpurun_out/pol
# (the policy switch was a temporary HFREP_LSTM_DBG bit pair: 512 nt, 1024 sc1, 1536 sc0 sc1)
for d in 0 512 1024 1536 0; do HFREP_LSTM_DBG=$d timeout -k 10 120 python scripts/bench_lstm.py --batch 262144 --only fwd,tfwd --iters 5 | sed "s/^{/{\"dbg\": $d, /" >> gpurun_out/pol/pol.jsonl || exit 1; done
