#!/bin/bash
# Round-5 second GPU pass: new GPU tests (P2P graph capture, small-batch stream overlap), tangent-reverse
# A/B, wgrad pair vs quad at K = 32, the sigmoid tangent-forward diagnosis builds, reference-preset latency.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_second}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_p2p_gpu.py tests/test_gpu_runtime.py -k "graphed or concurrent" -x -v \
  --timeout 200 --timeout-method thread > $OUT/tests_new.txt 2>&1 || { tail -n 40 $OUT/tests_new.txt; exit 1; }
tail -n 2 $OUT/tests_new.txt
for C in 0 1; do
  HFREP_CONCURRENT=$C timeout -k 10 300 python -u scripts/bench_small.py --iters 100 > $OUT/small_c$C.jsonl 2>&1 \
    || { tail -n 20 $OUT/small_c$C.jsonl; exit 1; }
  HFREP_CONCURRENT=$C timeout -k 10 300 python -u scripts/bench_small.py --iters 30 --no-graph > $OUT/small_eager_c$C.jsonl 2>&1 \
    || { tail -n 20 $OUT/small_eager_c$C.jsonl; exit 1; }
  grep -h dtype $OUT/small_c$C.jsonl $OUT/small_eager_c$C.jsonl
done
bash scripts/gpu_ab_kernels.sh ${1:-r05_second}/ab_tb tbwd,tbwd_dx tbcg2 tbcg7 || exit 1
timeout -k 10 300 python -u scripts/bench_wgrad.py --dtype float32 --batch 262144 --iters 5 > $OUT/wgrad_f32.jsonl 2>&1 \
  || { tail -n 20 $OUT/wgrad_f32.jsonl; exit 1; }
grep -v amdgpu $OUT/wgrad_f32.jsonl
for V in tf4sig tf4diag; do
  HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so" timeout -k 10 240 python -u scripts/dbg_tfwd4_diag.py > $OUT/diag_$V.txt 2>&1 \
    || { tail -n 30 $OUT/diag_$V.txt; exit 1; }
  grep -v amdgpu $OUT/diag_$V.txt | tail -n 40
done
