#!/bin/bash
# Copy the newest parity checkpoints a GPU call brought back (gpurun_out/TAG/ckpt/<name>/) into the
# in-tree ./parity_ckpt/<name>/ that the next call resumes from.  usage: scripts/parity_ckpt_sync.sh TAG
set -e
cd "$(dirname "$0")/.."
for d in gpurun_out/$1/ckpt/*/; do
  name=$(basename "$d"); mkdir -p parity_ckpt/$name
  rm -f parity_ckpt/$name/state_*.pt; cp "$d"state_*.pt parity_ckpt/$name/
  ls parity_ckpt/$name
done
