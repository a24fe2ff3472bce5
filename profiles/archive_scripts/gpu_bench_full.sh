#!/bin/bash
# the driver's bench command at the default shape (fp32 headline + bf16 sub-record)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-bench_full}; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps ${2:-5} --warmup ${3:-2} > $O/bench.json 2> $O/bench.err && cat $O/bench.json || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
