#!/bin/bash
# MFMA result -> VALU read timing probe, then the fp32 step's kernel profile at B = 32768 and 262144
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_probe; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 ./scripts/probes/mfma_raw_probe 2048 64 > $O/mfma_raw.jsonl 2>&1 || { echo PROBE_FAIL; cat $O/mfma_raw.jsonl; exit 1; }
cat $O/mfma_raw.jsonl
bash scripts/gpu_prof_dtype.sh r02_probe/prof32k float32 32768 > /dev/null && tail -32 gpurun_out/r02_probe/prof32k/prof_summary.txt
timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --dtype float32 > $O/bench_fp32_262k.json 2> $O/bench.err && cat $O/bench_fp32_262k.json || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
