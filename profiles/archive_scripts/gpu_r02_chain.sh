#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_probe; mkdir -p $O
timeout -k 10 120 ./scripts/probes/mfma_chain_probe 2400 2000 > $O/mfma_chain.jsonl 2>&1 || { echo PROBE_FAIL; cat $O/mfma_chain.jsonl; exit 1; }
cat $O/mfma_chain.jsonl
