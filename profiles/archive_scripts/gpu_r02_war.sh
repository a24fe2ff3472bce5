#!/bin/bash
# MFMA source-operand overwrite timing probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_probe; mkdir -p $O
timeout -k 10 120 ./scripts/probes/mfma_war_probe 2048 64 > $O/mfma_war.jsonl 2>&1 || { echo PROBE_FAIL; cat $O/mfma_war.jsonl; exit 1; }
cat $O/mfma_war.jsonl
