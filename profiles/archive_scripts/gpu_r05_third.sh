#!/bin/bash
# Round-5 third GPU pass: concurrency tests + reference-preset latency, the headline bench, the per-iteration
# HBM byte budget (bf16 + fp32) and DP overhead at equal total work on one GPU.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_third}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_runtime.py -k "concurrent or graph or determinism" -x -v \
  --timeout 200 --timeout-method thread > $OUT/tests_rt.txt 2>&1 || { tail -n 40 $OUT/tests_rt.txt; exit 1; }
tail -n 2 $OUT/tests_rt.txt
HFREP_CONCURRENT=1 timeout -k 10 300 python -u scripts/bench_small.py --iters 100 > $OUT/small_c1.jsonl 2>&1 \
  || { tail -n 20 $OUT/small_c1.jsonl; exit 1; }
grep -h dtype $OUT/small_c1.jsonl
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash scripts/pmc_step_bytes.sh ${1:-r05_third}/bytes bfloat16 float32 || exit 1
for dt in float32 bfloat16; do
  timeout -k 10 600 python -u scripts/bench_dp_shared.py --dtype $dt --steps 4 --warmup 2 > $OUT/dp_shared_$dt.jsonl 2> $OUT/dp_shared_$dt.err \
    || { tail -n 20 $OUT/dp_shared_$dt.err; exit 1; }
  cat $OUT/dp_shared_$dt.jsonl
done
