#!/bin/bash
# Round-5 race A/B: the act = sigmoid bf16 tangent forward on lstm_fwd4<TAN> as built (tf4sig) vs with
# 8 wait states forced after the tail MFMAs (tf4nop); run-to-run diffs at B = 32772.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_race}; mkdir -p $OUT
export TMPDIR=/tmp
for V in tf4sig tf4nop; do
  HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so" timeout -k 10 240 python -u scripts/dbg_tfwd4_diag.py 32772 6 > $OUT/diag_$V.txt 2>&1 \
    || { tail -n 30 $OUT/diag_$V.txt; exit 1; }
  grep -h '"B"' $OUT/diag_$V.txt
done
for V in tf4sig tf4nop; do
  HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so" timeout -k 10 200 python -u scripts/bench_lstm.py --batch 262144 --K 100 --iters 5 --only fwd,tfwd \
    > $OUT/lstm_$V.jsonl 2>&1 || { tail -n 20 $OUT/lstm_$V.jsonl; exit 1; }
  echo "== $V"; grep -h '"op"' $OUT/lstm_$V.jsonl
done
