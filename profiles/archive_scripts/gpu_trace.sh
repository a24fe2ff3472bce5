#!/bin/bash
# Timeline evidence: torch.profiler Chrome trace with the trainer's phase ranges, and a rocprofv3
# kernel + ROCTX marker trace of the same phases.   usage: bash scripts/gpu_trace.sh TAG [BATCH]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
TAG=${1:-trace}; B=${2:-16384}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 2 --warmup 2 --batch-per-gpu $B --profile-steps 1 --trace-out $OUT/torch_trace.json > $OUT/bench_trace.log 2> $OUT/torch_table.txt || { tail -20 $OUT/torch_table.txt; exit 1; }
tail -1 $OUT/bench_trace.log | cut -c1-200
export HFREP_TRACE=1
cd /tmp && timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d "$R/$OUT/roc" -o run --output-format csv -- python "$R/bench.py" --steps 1 --warmup 1 --batch-per-gpu $B > "$R/$OUT/roc.log" 2>&1 || { tail -20 "$R/$OUT/roc.log"; exit 1; }
cd "$R" && ls $OUT/roc | head
