#!/bin/bash
# round-end rehearsal after the r02 fp32 fixes: full GPU suite, smoke, default bench, fp32 kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=r02_end bash scripts/gpu_r02_final.sh || exit 1
bash scripts/gpu_prof_dtype.sh r02_end/fp32 float32 262144 > /dev/null && head -32 gpurun_out/r02_end/fp32/prof_summary.txt
