#!/bin/bash
# Round-4 first GPU pass: the fp32 split-kernel numerics (incl. the soffset BPTT), the whole GPU suite,
# the headline bench, an fp32 kernel table and the DP overlap timeline (1-rank RCCL, GradSync world 2).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r04_first}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lstmf or narrowf or tfwd_bitwise or linear or wgrad_fused" -q --timeout 200 \
  --timeout-method thread > $OUT/tests_split.txt 2>&1 || { tail -n 30 $OUT/tests_split.txt; exit 1; }
tail -n 2 $OUT/tests_split.txt
timeout -k 10 200 python -u scripts/bench_wgrad.py --dtype float32 --batch 262144 --iters 5 > $OUT/bench_wgrad.jsonl 2>&1 || { tail -n 20 $OUT/bench_wgrad.jsonl; exit 1; }
cat $OUT/bench_wgrad.jsonl
timeout -k 10 200 python -u scripts/bench_wgrad.py --dtype bfloat16 --batch 262144 --iters 5 > $OUT/bench_wgrad_bf16.jsonl 2>&1 || { tail -n 20 $OUT/bench_wgrad_bf16.jsonl; exit 1; }
cat $OUT/bench_wgrad_bf16.jsonl
timeout -k 10 200 python -u scripts/bench_small.py --iters 100 > $OUT/bench_small.jsonl 2>&1 || { tail -n 20 $OUT/bench_small.jsonl; exit 1; }
cat $OUT/bench_small.jsonl
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_all.txt 2>&1 \
  || { tail -n 30 $OUT/tests_all.txt; exit 1; }
tail -n 2 $OUT/tests_all.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o run -- python "$R/bench.py" --steps 3 --warmup 1 --dtype float32 > "$R/$OUT/prof.log" 2>&1 || { tail "$R/$OUT/prof.log"; exit 1; }
cd "$R" && python scripts/prof_summary.py $(find $OUT/prof -name "*kernel_stats.csv" | head -1) 40 > $OUT/kernel_summary.txt 2>&1; head -14 $OUT/kernel_summary.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/dp" -o run -- python "$R/scripts/dp_overlap_trace.py" > "$R/$OUT/dp.log" 2>&1 || { tail "$R/$OUT/dp.log"; exit 1; }
cd "$R" && python scripts/dp_overlap_summary.py $(find $OUT/dp -name "*kernel_trace.csv" | head -1) > $OUT/dp_overlap.txt 2>&1; cat $OUT/dp.log | grep dp_overlap; head -40 $OUT/dp_overlap.txt
