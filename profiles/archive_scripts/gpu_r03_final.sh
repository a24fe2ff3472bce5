#!/bin/bash
# Round-3 closing pass on one GPU: bitwise determinism (small and large batch), the whole GPU suite,
# smoke(), the headline bench, and rocprofv3 kernel tables of 3 fp32 and 3 bf16 iterations.
# usage: profiles/archive_scripts/gpu_r03_final.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r03_final}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python scripts/dbg_determinism.py 1 2 > $OUT/det_small.txt 2>&1 || { tail $OUT/det_small.txt; exit 1; }
timeout -k 10 300 python scripts/dbg_determinism.py 128 1 > $OUT/det_large.txt 2>&1 || { tail $OUT/det_large.txt; exit 1; }
echo "determinism: small $(grep -c False $OUT/det_small.txt) / large $(grep -c False $OUT/det_large.txt) rows with a False"
grep False $OUT/det_small.txt $OUT/det_large.txt | cut -c1-200
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_all.txt 2>&1 \
  || { tail -n 30 $OUT/tests_all.txt; exit 1; }
tail -n 1 $OUT/tests_all.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
grep smoke $OUT/smoke.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
for dt in float32 bfloat16; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$dt" -o run -- python "$R/bench.py" --steps 3 --warmup 1 --dtype $dt > "$R/$OUT/prof_$dt.log" 2>&1 || { tail "$R/$OUT/prof_$dt.log"; exit 1; }
  cd "$R" && python scripts/prof_summary.py $(find $OUT/prof_$dt -name "*kernel_stats.csv" | head -1) 45 > $OUT/kernel_summary_$dt.txt 2>&1; head -12 $OUT/kernel_summary_$dt.txt
done
