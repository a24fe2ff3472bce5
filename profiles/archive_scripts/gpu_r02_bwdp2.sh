#!/bin/bash
# role-split fp32 BPTT: numerics, A/B against the two-phase kernel, MFMA-busy counters of both
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=gpurun_out/r02_bwdp2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "lstmf or trainer_gradients_gpu_vs_cpu" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 2 1 2; do
  HFREP_LSTMF_BWD=$v timeout -k 10 120 python -u scripts/bench_lstm.py --dtype float32 --batch 32768 --K 100 --only bwd --iters 20 \
      | sed "s/^/{\"ver\": $v} /" >> $O/bwd_ab.txt || { echo AB_FAIL; exit 1; }
done
cat $O/bwd_ab.txt
cd /tmp
for v in 1 2; do
  HFREP_LSTMF_BWD=$v timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT \
      --output-format csv -d "$R/$O/pmc_v$v/p1" -o run -- python "$R/scripts/bench_lstm.py" --dtype float32 --batch 32768 --K 100 --iters 2 --only bwd > "$R/$O/pmc_v$v.log" 2>&1 || { echo PMC_FAIL; tail "$R/$O/pmc_v$v.log"; exit 1; }
  python "$R/scripts/pmc_summary.py" "$R/$O/pmc_v$v" > "$R/$O/pmc_v$v.txt"; grep -A10 lstmf_bwd "$R/$O/pmc_v$v.txt"
done
