#!/bin/bash
# Round-5 second GPU pass: the P2P graph-capture test, tangent-reverse A/B, wgrad pair vs quad at K = 32,
# the per-iteration HBM byte budget (bf16 + fp32), and DP overhead at equal total work on one GPU.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_second}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_p2p_gpu.py -k graphed -x -v --timeout 200 --timeout-method thread \
  > $OUT/tests_graph.txt 2>&1 || { tail -n 40 $OUT/tests_graph.txt; exit 1; }
tail -n 2 $OUT/tests_graph.txt
bash scripts/gpu_ab_kernels.sh ${1:-r05_second}/ab_tb tbwd,tbwd_dx tbcg2 tbcg7 || exit 1
timeout -k 10 300 python -u scripts/bench_wgrad.py --dtype float32 --batch 262144 --iters 5 > $OUT/wgrad_f32.jsonl 2>&1 \
  || { tail -n 20 $OUT/wgrad_f32.jsonl; exit 1; }
cat $OUT/wgrad_f32.jsonl | grep -v amdgpu
bash scripts/pmc_step_bytes.sh ${1:-r05_second}/bytes bfloat16 float32 || exit 1
for dt in float32 bfloat16; do
  timeout -k 10 600 python -u scripts/bench_dp_shared.py --dtype $dt --steps 4 --warmup 2 > $OUT/dp_shared_$dt.jsonl 2> $OUT/dp_shared_$dt.err \
    || { tail -n 20 $OUT/dp_shared_$dt.err; exit 1; }
  cat $OUT/dp_shared_$dt.jsonl
done
