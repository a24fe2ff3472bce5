#!/bin/bash
# act = sigmoid tangent-forward drift vs the data wave's tape stream: nt off (tf4nt0), the data wave waiting
# for its stores every step (tf4vm), and every step's tape stored to step 0's slots (HFREP_LSTM_DBG=256).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_race5}; mkdir -p $OUT
export TMPDIR=/tmp
for V in tf4nt0 tf4vm; do
  HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so" timeout -k 10 200 python -u scripts/dbg_tfwd4_diag.py 32772 4 \
    > $OUT/diag_$V.txt 2>&1 || { tail -n 30 $OUT/diag_$V.txt; exit 1; }
  echo "== $V"; grep -h '"B"' $OUT/diag_$V.txt | grep '"act": 1'
done
HFREP_LSTM_DBG=256 HFREP_NATIVE_LIB="$R/variants/tf4sig/_hfrep_native.so" timeout -k 10 200 python -u scripts/dbg_tfwd4_diag.py 32772 4 \
  > $OUT/diag_dbg256.txt 2>&1 || { tail -n 30 $OUT/diag_dbg256.txt; exit 1; }
echo "== tf4sig dbg 256"; grep -h '"B"' $OUT/diag_dbg256.txt | grep '"act": 1'
for V in tf4sig tf4nt0 tf4vm; do
  HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so" timeout -k 10 200 python -u scripts/bench_lstm.py --batch 262144 --K 100 --iters 5 --only fwd,tfwd \
    > $OUT/lstm_$V.jsonl 2>&1 || { tail -n 20 $OUT/lstm_$V.jsonl; exit 1; }
  echo "== $V"; grep -h '"op"' $OUT/lstm_$V.jsonl
done
