#!/bin/bash
# Round-5 GPU pass 4: the batched autoencoder fit tests, then the B = 32768 parity segments.
# A test FAILURE (exit 1) still runs the parity; a crash / timeout / fault ends the call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_fourth}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ae_gpu.py > $OUT/tests_ae.txt 2>&1
rc=$?; tail -n 5 $OUT/tests_ae.txt
[ $rc -le 1 ] || exit $rc
PARITY_TIMEOUT=${PARITY_TIMEOUT:-700} bash scripts/gpu_parity_seg.sh ${1:-r05_fourth} "$2"
