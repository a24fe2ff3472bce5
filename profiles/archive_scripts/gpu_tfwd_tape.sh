#!/bin/bash
# bf16 tangent reverse run-to-run at B = 32772 (scripts/dbg_tfwd_tape.py), default library; where the dZ
# differences sit (row mod 32, step, gate, unit); act = 0 / 1 / 2; the v2 kernel (HFREP_LSTM_TBWD=2) at act 1
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-tfwd_tape}; mkdir -p $OUT
for a in "32772 32 1" "32772 32 0"; do
  timeout -k 10 200 python scripts/dbg_tfwd_tape.py $a 2 >> $OUT/log.txt 2>&1 || { tail $OUT/log.txt; exit 1; }
done
HFREP_LSTM_TBWD=2 timeout -k 10 200 python scripts/dbg_tfwd_tape.py 32772 32 1 2 >> $OUT/log_v2.txt 2>&1 || { tail $OUT/log_v2.txt; exit 1; }
grep -v amdgpu.ids $OUT/log.txt; echo "== v2"; grep -v amdgpu.ids $OUT/log_v2.txt
