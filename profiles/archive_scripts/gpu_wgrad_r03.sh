#!/bin/bash
# fp32 split weight gradients: numerics tests, timing of impl 1 / 2 / 3 at the critic's 12.6 M rows,
# and one PMC pass (LDS bank conflicts, MFMA busy) over both split kernels.  usage: scripts/gpu_wgrad_r03.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-wgrad_r03}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lstmf_wgrad" -q --timeout 200 --timeout-method thread \
  > $OUT/tests.txt 2>&1 || { tail -n 30 $OUT/tests.txt; exit 1; }
tail -n 2 $OUT/tests.txt
timeout -k 10 300 python scripts/bench_wgrad.py --dtype float32 --batch 524288 --iters 5 > $OUT/timing.jsonl 2>&1 || { tail $OUT/timing.jsonl; exit 1; }
grep -v amdgpu.ids $OUT/timing.jsonl
cd /tmp
for impl in 2 3; do
  HFREP_LSTMF_WGRAD=$impl timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS \
    --output-format csv -d "$R/$OUT/p$impl" -o run -- python "$R/scripts/bench_lstm.py" --dtype float32 --batch 65536 --K 100 --iters 2 --only wgrad_tan \
    > "$R/$OUT/p$impl.log" 2>&1 || { echo "PMC pass $impl failed"; tail -20 "$R/$OUT/p$impl.log"; exit 1; }
done
cd "$R" && python scripts/pmc_summary.py $OUT > $OUT/summary.txt && grep -A9 "wgrad_q4\|wgrad_split" $OUT/summary.txt
