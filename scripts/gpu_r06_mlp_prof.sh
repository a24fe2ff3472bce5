#!/bin/bash
# Round-6 MLP profile (BASELINE configs 3 / 4): rocprofv3 kernel tables and TCC_EA0 byte totals of one
# timed iteration of bench.py --model gan|wgan_gp, fp32 and bf16.
#   bash scripts/gpu_r06_mlp_prof.sh OUTNAME [models...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r06_mlp}; shift; mkdir -p $OUT
export TMPDIR=/tmp
for M in ${@:-wgan_gp gan}; do
  for dt in bfloat16 float32; do
    timeout -k 10 300 python -u bench.py --model $M --dtype $dt --steps 5 --warmup 2 > $OUT/bench_${M}_$dt.json 2> $OUT/bench_${M}_$dt.err \
      || { tail $OUT/bench_${M}_$dt.err; exit 1; }
    cut -c1-160 $OUT/bench_${M}_$dt.json
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/kt_${M}_$dt" -o run -- \
      python "$R/bench.py" --model $M --dtype $dt --steps 1 --warmup 1 > "$R/$OUT/kt_${M}_$dt.log" 2>&1 \
      || { cd "$R"; echo "kernel trace $M $dt failed"; tail -5 "$OUT/kt_${M}_$dt.log"; exit 1; }
    cd "$R"
    f=$(ls $OUT/kt_${M}_$dt/*kernel_stats.csv $OUT/kt_${M}_$dt/*/*kernel_stats.csv 2>/dev/null | head -n 1)
    python scripts/prof_summary.py "$f" 30 > $OUT/kernel_summary_${M}_$dt.txt && head -n 12 $OUT/kernel_summary_${M}_$dt.txt
    cd /tmp
    timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
      --kernel-trace --output-format csv -d "$R/$OUT/by_${M}_$dt" -o run -- python "$R/bench.py" --model $M --dtype $dt \
      --steps 1 --warmup 1 > "$R/$OUT/by_${M}_$dt.log" 2>&1 || { cd "$R"; echo "PMC pass $M $dt failed"; exit 1; }
    cd "$R" && python scripts/step_bytes_summary.py $OUT/by_${M}_$dt 2 > $OUT/bytes_${M}_$dt.txt && head -n 3 $OUT/bytes_${M}_$dt.txt
    rm -rf $OUT/kt_${M}_$dt/*/*kernel_trace.csv $OUT/by_${M}_$dt
  done
done
