#!/bin/bash
# Round-5 first GPU pass: the P2P fail-loud / DP tests, then W-dist parity at the reference preset.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_first}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_p2p_gpu.py tests/test_gpu_rccl.py -x -v --timeout 200 --timeout-method thread \
  > $OUT/tests_dp.txt 2>&1 || { tail -n 40 $OUT/tests_dp.txt; exit 1; }
tail -n 3 $OUT/tests_dp.txt
timeout -k 10 300 python -u scripts/bench_fp3.py > $OUT/bench_fp3.jsonl 2>&1 || { tail -n 20 $OUT/bench_fp3.jsonl; exit 1; }
cat $OUT/bench_fp3.jsonl
bash scripts/gpu_parity.sh r05_parity "${2:-bfloat16:32:123 bfloat16:32:124 bfloat16:32:125 float32:32:123 float32:32:124 float32:32:125}"
