#!/bin/bash
# Round-4 main GPU pass: the whole GPU suite, the headline bench, fp32 and bf16 kernel tables and the
# DP overlap timeline (1-rank RCCL, GradSync world 2, bench shape).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r04_main}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_all.txt 2>&1 \
  || { tail -n 30 $OUT/tests_all.txt; exit 1; }
tail -n 2 $OUT/tests_all.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
for dt in float32 bfloat16; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$dt" -o run -- python "$R/bench.py" --steps 3 --warmup 1 --dtype $dt > "$R/$OUT/prof_$dt.log" 2>&1 || { tail "$R/$OUT/prof_$dt.log"; exit 1; }
  cd "$R" && python scripts/prof_summary.py $(find $OUT/prof_$dt -name "*kernel_stats.csv" | head -1) 40 > $OUT/kernel_summary_$dt.txt 2>&1; head -14 $OUT/kernel_summary_$dt.txt
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/dp" -o run -- python "$R/scripts/dp_overlap_trace.py" > "$R/$OUT/dp.log" 2>&1 || { tail "$R/$OUT/dp.log"; exit 1; }
cd "$R" && python scripts/dp_overlap_summary.py $(find $OUT/dp -name "*kernel_trace.csv" | head -1) > $OUT/dp_overlap.txt 2>&1; grep dp_overlap $OUT/dp.log; head -40 $OUT/dp_overlap.txt
