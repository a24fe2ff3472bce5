#!/bin/bash
# Store-data hazard with an LDS read overwriting the data registers (scripts/probes/store_hazard_probe.hip modes 9 / 10)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-store_lds}; mkdir -p $OUT
timeout -k 10 120 scripts/probes/store_hazard_probe 1024 32 1 > $OUT/store_lds.jsonl 2>&1 || { tail $OUT/store_lds.jsonl; exit 1; }
timeout -k 10 120 scripts/probes/store_hazard_probe 4096 16 1 >> $OUT/store_lds.jsonl 2>&1 || { tail $OUT/store_lds.jsonl; exit 1; }
cat $OUT/store_lds.jsonl
