#!/bin/bash
# first end-to-end GPU pass: smoke, batch sweep, kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
for B in 1024 4096 16384 65536; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --batch-per-gpu $B > gpurun_out/bench_B$B.log 2>&1 || { echo BENCH_FAIL $B; tail -30 gpurun_out/bench_B$B.log; exit 1; }
  tail -1 gpurun_out/bench_B$B.log
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --batch-per-gpu 16384 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
echo PROF_OK
