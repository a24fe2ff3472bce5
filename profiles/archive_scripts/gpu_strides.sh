#!/bin/bash
# Conflict-free plane strides (bwds / dgrad_s4 / fwds): split-kernel numerics, per-op timing at
# B = 262144 x T = 24 fp32, one PMC pass for the LDS conflict counters, then the headline bench.
# usage: scripts/gpu_strides.sh OUTNAME [--suite]   (--suite: the whole GPU test suite after the split tests)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-strides}; mkdir -p $OUT
export TMPDIR=/tmp
# MFMA result -> packed fp32 VALU consumer wait states (scripts/probes/mfma_pk_probe.hip, prebuilt in-tree)
timeout -k 10 120 scripts/probes/mfma_pk_probe 2048 64 > $OUT/mfma_pk.jsonl 2>&1 || { tail $OUT/mfma_pk.jsonl; exit 1; }
grep -v '"stale": \[0, 0, 0, 0\]' $OUT/mfma_pk.jsonl | head -40
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "split_forward or split_bptt or lstmf_dgrad or lstmf_wgrad" -q \
  --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -n 40 $OUT/tests.txt; exit 1; }
tail -n 1 $OUT/tests.txt
if [ "$2" == "--suite" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_all.txt 2>&1 \
    || { tail -n 30 $OUT/tests_all.txt; exit 1; }
  tail -n 2 $OUT/tests_all.txt
fi
for K in 32 100; do
  timeout -k 10 200 python scripts/bench_lstm.py --dtype float32 --batch 262144 --K $K --iters 5 \
    --only fwd,fwd_notape,tfwd,bwd,tbwd,dgrad,wgrad > $OUT/timing_K$K.log 2>&1 || { tail $OUT/timing_K$K.log; exit 1; }
  grep op $OUT/timing_K$K.log
done
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA \
  --output-format csv -d "$R/$OUT/p1" -o run -- python "$R/scripts/bench_lstm.py" --dtype float32 --batch 65536 --K 32 --iters 1 \
  --only fwd,bwd,dgrad > "$R/$OUT/p1.log" 2>&1 || { echo "PMC pass failed"; tail -20 "$R/$OUT/p1.log"; exit 1; }
cd "$R" && python scripts/pmc_summary.py $OUT > $OUT/pmc_summary.txt && grep -A7 "lstmf_" $OUT/pmc_summary.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
