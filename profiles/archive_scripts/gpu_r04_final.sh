#!/bin/bash
# Round-4 closing GPU pass: whole GPU suite, headline bench, fp32 / bf16 kernel tables, the bf16
# autoencoder diagnosis (training vs evaluation precision).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r04_end}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_all.txt 2>&1 \
  || { tail -n 30 $OUT/tests_all.txt; exit 1; }
tail -n 2 $OUT/tests_all.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 python -u scripts/ae_bf16_diag.py --latents 1,4,8 --seeds 1,2 > $OUT/ae_bf16_diag.jsonl 2>&1 || { tail -n 20 $OUT/ae_bf16_diag.jsonl; exit 1; }
grep '"k"' $OUT/ae_bf16_diag.jsonl
for dt in float32 bfloat16; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$dt" -o run -- python "$R/bench.py" --steps 3 --warmup 1 --dtype $dt > "$R/$OUT/prof_$dt.log" 2>&1 || { tail "$R/$OUT/prof_$dt.log"; exit 1; }
  cd "$R" && python scripts/prof_summary.py $(find $OUT/prof_$dt -name "*kernel_stats.csv" | head -1) 40 > $OUT/kernel_summary_$dt.txt 2>&1; head -8 $OUT/kernel_summary_$dt.txt
done
