#!/bin/bash
# act = sigmoid tangent-forward drift vs a perturbation at the trace point (row half 1, rows 4 g + 2 / 3):
# tf4sig (as built, the positive control), tf4p1 (s_waitcnt vmcnt(0)), tf4p2 (dummy LDS write +
# lgkmcnt(0)), tf4p3 (64 s_nop cycles)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_race8}; mkdir -p $OUT; export TMPDIR=/tmp
for V in tf4sig tf4p1 tf4p2 tf4p3; do
  HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so" timeout -k 10 200 python -u scripts/dbg_tfwd4_diag.py 32772 5 \
    > $OUT/diag_$V.txt 2>&1 || { tail -n 30 $OUT/diag_$V.txt; exit 1; }
  echo "== $V"; grep -h '"B"' $OUT/diag_$V.txt | grep '"act": 1' | cut -c1-160
done
