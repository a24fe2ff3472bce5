#!/bin/bash
# Two quick diagnostics: the packed-consumer MFMA wait-state probe (scripts/probes/mfma_pk_probe.hip,
# prebuilt in-tree) and the aten-op audit of one fp32 / one bf16 training iteration on the device.
# usage: scripts/gpu_probe_audit.sh OUTNAME
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-probe_audit}; mkdir -p $OUT
timeout -k 10 120 scripts/probes/mfma_pk_probe 2048 64 > $OUT/mfma_pk.jsonl 2>&1 || { tail $OUT/mfma_pk.jsonl; exit 1; }
grep -c wait_states $OUT/mfma_pk.jsonl
timeout -k 10 300 python scripts/aten_audit.py --batch 4096 --dtype float32 > $OUT/aten_fp32.txt 2>&1 || { tail -20 $OUT/aten_fp32.txt; exit 1; }
timeout -k 10 300 python scripts/aten_audit.py --batch 4096 --dtype bfloat16 > $OUT/aten_bf16.txt 2>&1 || { tail -20 $OUT/aten_bf16.txt; exit 1; }
tail -25 $OUT/aten_fp32.txt; tail -3 $OUT/aten_bf16.txt
