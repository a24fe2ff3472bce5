#!/bin/bash
# A/B of mlp_bt_colsum's threads per CU (HFREP_COLSUM_TPC) on config 4, both dtypes: bench + kernel table.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r06_colsum}; mkdir -p $OUT; export TMPDIR=/tmp
for tpc in 512 1024 2048; do
  for d in bfloat16 float32; do
    HFREP_COLSUM_TPC=$tpc timeout -k 10 200 python bench.py --model wgan_gp --dtype $d --steps 20 --warmup 3 \
      > $OUT/c4_${d}_$tpc.json 2> $OUT/err || { tail $OUT/err; exit 1; }
  done
  cd /tmp
  HFREP_COLSUM_TPC=$tpc timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/kt_$tpc" -o run -- \
    python "$R/bench.py" --model wgan_gp --dtype bfloat16 --steps 1 --warmup 1 > "$R/$OUT/kt_$tpc.log" 2>&1 || exit 1
  cd "$R"
  f=$(ls $OUT/kt_$tpc/*kernel_stats.csv $OUT/kt_$tpc/*/*kernel_stats.csv 2>/dev/null | head -n 1)
  python scripts/prof_summary.py "$f" 30 > $OUT/ks_$tpc.txt && grep -E "colsum|bcast" $OUT/ks_$tpc.txt
done
