#!/bin/bash
# Round-6: (1) the bf16 tangent forward run to run at the headline batch B = 262 144 on the shipped build
# (act = tanh: lstm_fwd4<TAN>, the headline critic's path; act = sigmoid: lstm_tfwd2); (2) the bf16 sub-record
# at 262 144 vs 524 288 windows per GPU, same box.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r06_tanh_batch}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/dbg_tfwd4_diag.py 262144 4 > $OUT/tfwd_B262144.txt 2>&1 || { tail $OUT/tfwd_B262144.txt; exit 1; }
grep hd_ndiff $OUT/tfwd_B262144.txt | cut -c1-150
for B in 262144 524288 262144 524288; do
  timeout -k 10 400 python -u bench.py --dtype bfloat16 --batch-per-gpu $B --steps 8 --warmup 2 > $OUT/bench_bf16_$B.json 2> $OUT/bench_bf16_$B.err \
    || { tail $OUT/bench_bf16_$B.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_bf16_$B.json')); print($B, d['value'], d['ms_per_step'], d['peak_mem_gb_rank0'])"
  cat $OUT/bench_bf16_$B.json >> $OUT/bench_bf16_all.jsonl
done
