#!/bin/bash
# Uniform-branch build (wave index via readfirstlane): bitwise run-to-run checks of every LSTM
# layer op incl. the DX + generated-head tangent reverse and the two-step x prefetch forward,
# then the LSTM / trainer GPU tests and a bf16 bench with the re-enabled variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_det2; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 180 python -u scripts/dbg_determinism.py > $O/det_$i.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det_$i.txt; exit 1; }
done
cat $O/det_*.txt | grep -c "False" || true
timeout -k 10 180 python -u scripts/dbg_fwd_pf.py > $O/fwd_pf.txt 2>&1 || { echo PF_FAIL; tail -20 $O/fwd_pf.txt; exit 1; }
timeout -k 10 180 python -u scripts/dbg_tbwd_gen.py > $O/tbwd_gen.txt 2>&1 || { echo GEN_FAIL; tail -20 $O/tbwd_gen.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_runtime.py -x -v --timeout 120 --timeout-method thread \
    -k "lstm or determinism or trainer_gradients or head" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --dtype bfloat16 > $O/bench_bf16_262k.json 2> $O/bench.err && cat $O/bench_bf16_262k.json || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
