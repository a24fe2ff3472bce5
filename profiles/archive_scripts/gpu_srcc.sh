#!/bin/bash
# Cross-opcode MFMA SrcC forwarding probe (scripts/probes/mfma_srcc_probe.hip, prebuilt in-tree)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-srcc}; mkdir -p $OUT
timeout -k 10 120 scripts/probes/mfma_srcc_probe 2048 64 > $OUT/mfma_srcc.jsonl 2>&1 || { tail $OUT/mfma_srcc.jsonl; exit 1; }
cat $OUT/mfma_srcc.jsonl
