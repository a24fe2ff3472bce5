#!/bin/bash
# All GPU tests, then bench + rocprofv3 kernel stats.   usage: bash scripts/gpu_full.sh TAG "B1 B2" PROF_B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-full}; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
bash scripts/gpu_bench_profile.sh "$TAG" "${2:-16384}" "${3:-16384}"
