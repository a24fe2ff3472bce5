#!/bin/bash
# Configs 3 / 4 bf16: the passes with in-kernel weight gradients (mlp_wgp_critic_w, mlp_gen_bwd_w) vs
# the operand path (HFREP_MLP_WGRAD_INKERNEL=0): fused-MLP GPU tests, bench A/B, rocprofv3 kernel table.
#   bash scripts/gpu_r06_wgpw.sh OUTNAME [skip-tests]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r06_wgpw}; mkdir -p $OUT; export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_mlp_fused_gpu.py -x -v --timeout 240 --timeout-method thread > $OUT/tests.txt 2>&1
  rc=$?; tail -n 30 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
fi
for M in wgan_gp gan; do
  for ik in 1 0; do
    HFREP_MLP_WGRAD_INKERNEL=$ik timeout -k 10 300 python -u bench.py --model $M --dtype bfloat16 --steps 8 --warmup 2 \
      > $OUT/bench_${M}_ik$ik.json 2> $OUT/bench_${M}_ik$ik.err || { tail $OUT/bench_${M}_ik$ik.err; exit 1; }
    cut -c1-220 $OUT/bench_${M}_ik$ik.json
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/kt" -o run -- \
  python "$R/bench.py" --model wgan_gp --dtype bfloat16 --steps 1 --warmup 1 > "$R/$OUT/kt.log" 2>&1 \
  || { cd "$R"; echo "kernel trace failed"; tail -5 "$OUT/kt.log"; exit 1; }
cd "$R"
f=$(ls $OUT/kt/*kernel_stats.csv $OUT/kt/*/*kernel_stats.csv 2>/dev/null | head -n 1)
python scripts/prof_summary.py "$f" 30 > $OUT/kernel_summary.txt && head -n 16 $OUT/kernel_summary.txt
