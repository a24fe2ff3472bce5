#!/bin/bash
# fp32 LSTM dgrad kernel: numerics, timing vs hipBLASLt, MFMA-busy counters of both
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=gpurun_out/${1:-r02_dgrad}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "lstmf_dgrad or linear_dgrad" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u scripts/dgrad_fp32_bench.py 786432 6291456 > $O/bench.jsonl 2>&1 || { echo BENCH_FAIL; cat $O/bench.jsonl; exit 1; }
cat $O/bench.jsonl
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT \
    --output-format csv -d "$R/$O/pmc/p1" -o run -- python "$R/scripts/dgrad_fp32_bench.py" 6291456 > "$R/$O/pmc.log" 2>&1 || { echo PMC_FAIL; tail "$R/$O/pmc.log"; exit 1; }
python "$R/scripts/pmc_summary.py" "$R/$O/pmc" > "$R/$O/pmc.txt"; cat "$R/$O/pmc.txt"
