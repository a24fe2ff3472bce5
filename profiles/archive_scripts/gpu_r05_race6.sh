#!/bin/bash
# act = sigmoid tangent-forward drift vs the cache policy of the primal-tape loads: as built (tf4sig),
# sc0 (tf4sc), sc0|sc1 (tf4sys); run-to-run diffs vs the first run and vs the previous run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_race6}; mkdir -p $OUT
export TMPDIR=/tmp
for V in tf4sig tf4sc tf4sys; do
  HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so" timeout -k 10 200 python -u scripts/dbg_tfwd4_diag.py 32772 5 \
    > $OUT/diag_$V.txt 2>&1 || { tail -n 30 $OUT/diag_$V.txt; exit 1; }
  echo "== $V"; grep -h '"B"' $OUT/diag_$V.txt | grep '"act": 1'
done
