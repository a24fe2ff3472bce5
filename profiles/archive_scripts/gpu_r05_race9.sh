#!/bin/bash
# act = sigmoid tangent-forward drift: does row 30 (31) carry the partner row's value? (variants tf4sig, tf4p2)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_race9}; mkdir -p $OUT; export TMPDIR=/tmp
for V in tf4sig tf4p2; do
  HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so" timeout -k 10 300 python -u scripts/dbg_tfwd4_rowswap.py 32772 6 100 \
    > $OUT/rowswap_$V.txt 2>&1 || { tail -n 30 $OUT/rowswap_$V.txt; exit 1; }
  echo "== $V"; tail -n 1 $OUT/rowswap_$V.txt
done
