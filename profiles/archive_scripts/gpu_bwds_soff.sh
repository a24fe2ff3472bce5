#!/bin/bash
# split BPTT with the tape offsets' uniform part in soffset: numerics tests, BPTT timing at B = 262144, bench
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-bwds_soff}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "split_bptt or lstmf or trainer_gradients or slice_averages" -q --timeout 200 \
  --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -n 30 $OUT/tests.txt; exit 1; }
tail -n 1 $OUT/tests.txt
for K in 32 100; do
  timeout -k 10 200 python scripts/bench_lstm.py --dtype float32 --batch 262144 --K $K --iters 5 --only bwd > $OUT/timing_K$K.log 2>&1 || { tail $OUT/timing_K$K.log; exit 1; }
  grep op $OUT/timing_K$K.log
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --dtype float32 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
