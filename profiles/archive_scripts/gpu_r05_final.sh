#!/bin/bash
# Round-5 closing GPU pass.  part "suite": the whole GPU suite + smoke; part "perf": the headline bench,
# fp32 / bf16 kernel tables and the bf16 HBM byte budget on the final kernels.
#   bash scripts/gpu_r05_final.sh OUTNAME suite|perf
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_final}; mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" = suite ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests_all.txt 2>&1
  rc=$?; tail -n 3 $OUT/tests_all.txt; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
  tail -n 1 $OUT/smoke.txt
  exit 0
fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python -u scripts/bench_small.py --iters 300 > $OUT/small.jsonl 2>&1 || { tail -n 20 $OUT/small.jsonl; exit 1; }
grep -h '"ms' $OUT/small.jsonl
for dt in float32 bfloat16; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$dt" -o run -- python "$R/bench.py" --steps 3 --warmup 1 --dtype $dt > "$R/$OUT/prof_$dt.log" 2>&1 || { tail "$R/$OUT/prof_$dt.log"; exit 1; }
  cd "$R" && python scripts/prof_summary.py $(find $OUT/prof_$dt -name "*kernel_stats.csv" | head -1) 40 > $OUT/kernel_summary_$dt.txt 2>&1; head -8 $OUT/kernel_summary_$dt.txt
done
bash scripts/pmc_step_bytes.sh ${1:-r05_final}/bytes bfloat16 || exit 1
