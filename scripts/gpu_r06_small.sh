#!/bin/bash
# Small-kernel changes of the headline step (gp_coef, sampler, Philox): their GPU tests, then a
# rocprofv3 kernel table of one bf16 and one fp32 headline iteration.
#   bash scripts/gpu_r06_small.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r06_small}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_runtime.py -x -v --timeout 240 --timeout-method thread \
  -k "gp_coef or rng or sampling or determinism or trainer_gradients" > $OUT/tests.txt 2>&1
rc=$?; tail -n 3 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for dt in bfloat16 float32; do
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/kt_$dt" -o run -- \
    python "$R/bench.py" --dtype $dt --steps 2 --warmup 1 > "$R/$OUT/kt_$dt.log" 2>&1 \
    || { cd "$R"; echo "kernel trace $dt failed"; tail -5 "$OUT/kt_$dt.log"; exit 1; }
  cd "$R"
  f=$(ls $OUT/kt_$dt/*kernel_stats.csv $OUT/kt_$dt/*/*kernel_stats.csv 2>/dev/null | head -n 1)
  python scripts/prof_summary.py "$f" 45 > $OUT/kernel_summary_$dt.txt && head -n 6 $OUT/kernel_summary_$dt.txt
done
