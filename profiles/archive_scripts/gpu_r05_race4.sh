#!/bin/bash
# act = sigmoid tangent-forward drift: per-step unit groups of the differing rows, with and without the
# data wave's tape stores (HFREP_LSTM_DBG=1).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_race4}; mkdir -p $OUT
export TMPDIR=/tmp
for D in 0 1; do
  HFREP_LSTM_DBG=$D HFREP_NATIVE_LIB="$R/variants/tf4sig/_hfrep_native.so" timeout -k 10 200 python -u scripts/dbg_tfwd4_detail.py 32772 100 3 \
    > $OUT/detail_dbg$D.txt 2>&1 || { tail -n 30 $OUT/detail_dbg$D.txt; exit 1; }
  echo "== HFREP_LSTM_DBG=$D"; grep -v amdgpu $OUT/detail_dbg$D.txt | grep '"rep"\|per_step' | head -14
done
