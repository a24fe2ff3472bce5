#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_race2}; mkdir -p $OUT
export TMPDIR=/tmp
for K in 100 32; do
  HFREP_NATIVE_LIB="$R/variants/tf4sig/_hfrep_native.so" timeout -k 10 200 python -u scripts/dbg_tfwd4_detail.py 32772 $K 3 \
    > $OUT/detail_K$K.txt 2>&1 || { tail -n 30 $OUT/detail_K$K.txt; exit 1; }
  grep -v amdgpu $OUT/detail_K$K.txt
done
