#!/bin/bash
# the RCCL branch of the gradient sync (1-rank group), eager and captured in a hipGraph
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_rccl; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 280 --timeout-method thread -k bucketed > $O/tests_eager.log 2>&1 || { echo EAGER_FAIL; tail -40 $O/tests_eager.log; exit 1; }
tail -1 $O/tests_eager.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 280 --timeout-method thread -k in_graph > $O/tests_graph.log 2>&1 || { echo GRAPH_FAIL; tail -40 $O/tests_graph.log; exit 1; }
tail -1 $O/tests_graph.log
