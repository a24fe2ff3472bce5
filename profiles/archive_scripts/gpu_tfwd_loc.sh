#!/bin/bash
# Where the bf16 tangent forward (act = sigmoid, B = 32772) differs run to run: rows / steps / units of hd
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-tfwd_loc}; mkdir -p $OUT
for a in "32772 32 1" "32772 100 1"; do
  timeout -k 10 200 python scripts/dbg_tfwd_tape.py $a 4 >> $OUT/log.txt 2>&1 || { tail $OUT/log.txt; exit 1; }
done
grep -v amdgpu.ids $OUT/log.txt | grep "hd_\|'rep'" | cut -c1-400
