#!/bin/bash
# Round-5 third GPU pass: per-iteration HBM byte budget (bf16 + fp32) and DP overhead at equal total work.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_third}; mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/pmc_step_bytes.sh ${1:-r05_third}/bytes bfloat16 float32 || exit 1
for dt in float32 bfloat16; do
  timeout -k 10 600 python -u scripts/bench_dp_shared.py --dtype $dt --steps 4 --warmup 2 > $OUT/dp_shared_$dt.jsonl 2> $OUT/dp_shared_$dt.err \
    || { tail -n 20 $OUT/dp_shared_$dt.err; exit 1; }
  cat $OUT/dp_shared_$dt.jsonl
done
