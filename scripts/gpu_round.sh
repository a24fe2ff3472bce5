#!/bin/bash
# One GPU pass: kernel numerics of the fp32 split kernels, the full GPU suite, the headline bench and a
# rocprofv3 kernel table of 3 fp32 iterations.  usage: scripts/gpu_round.sh OUTNAME [--no-suite]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-round}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lstmf_wgrad or lstmf_dgrad or narrowf or split_bptt or split_forward" -q --timeout 200 \
  --timeout-method thread > $OUT/tests_split.txt 2>&1 || { tail -n 30 $OUT/tests_split.txt; exit 1; }
tail -n 2 $OUT/tests_split.txt
if [ "$2" != "--no-suite" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_all.txt 2>&1 \
    || { tail -n 30 $OUT/tests_all.txt; exit 1; }
  tail -n 2 $OUT/tests_all.txt
fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o run -- python "$R/bench.py" --steps 3 --warmup 1 --dtype float32 > "$R/$OUT/prof.log" 2>&1 || { tail "$R/$OUT/prof.log"; exit 1; }
cd "$R" && python scripts/prof_summary.py $(find $OUT/prof -name "*kernel_stats.csv" | head -1) 40 > $OUT/kernel_summary.txt 2>&1; head -30 $OUT/kernel_summary.txt
