#!/bin/bash
# act = sigmoid tangent-forward drift under the forward kernel's runtime ablation mask (HFREP_LSTM_DBG:
# 1 no tape store, 2 no h store, 4 no x_{t+1} load): which memory stream is involved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_race3}; mkdir -p $OUT
export TMPDIR=/tmp
for D in 0 4 3 7; do
  HFREP_LSTM_DBG=$D HFREP_NATIVE_LIB="$R/variants/tf4sig/_hfrep_native.so" timeout -k 10 200 python -u scripts/dbg_tfwd4_diag.py 32772 4 \
    > $OUT/diag_dbg$D.txt 2>&1 || { tail -n 30 $OUT/diag_dbg$D.txt; exit 1; }
  echo "== HFREP_LSTM_DBG=$D"; grep -h '"B"' $OUT/diag_dbg$D.txt | grep '"act": 1'
done
