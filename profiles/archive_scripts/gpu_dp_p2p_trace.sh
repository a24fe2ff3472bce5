#!/bin/bash
# rocprofv3 kernel timeline of two-process DP training over the one-shot IPC all-reduce
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r04_dp_p2p}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/trace" -o run_%pid% -- python "$R/scripts/dp_p2p_trace.py" --batch 32768 > "$R/$OUT/trace.log" 2>&1 \
  || { tail -n 30 "$R/$OUT/trace.log"; exit 1; }
cd "$R"; grep '^{' $OUT/trace.log
for f in $(find $OUT/trace -name "*kernel_trace.csv"); do
  echo "== $f"; python scripts/dp_overlap_summary.py $f > $f.summary.txt 2>&1; head -n 12 $f.summary.txt; tail -n 1 $f.summary.txt
done
