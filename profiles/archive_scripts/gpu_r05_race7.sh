#!/bin/bash
# act = sigmoid tangent-forward drift, fingerprint trace build (variants/tf4trace): which value differs first
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_race7}; mkdir -p $OUT; export TMPDIR=/tmp
HFREP_NATIVE_LIB="$R/variants/tf4trace/_hfrep_native.so" timeout -k 10 300 python -u scripts/dbg_tfwd4_trace.py 32772 6 100 \
  > $OUT/trace_K100.txt 2>&1 || { tail -n 30 $OUT/trace_K100.txt; exit 1; }
cut -c1-600 $OUT/trace_K100.txt
