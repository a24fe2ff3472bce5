#!/bin/bash
# W-dist parity runs (reference preset, 5000 iterations) with the current kernels.
#   usage: bash scripts/gpu_parity.sh TAG "dtype:batch:seed ..." [EPOCHS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-parity}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for spec in ${2:-"bfloat16:32:123"}; do
  IFS=: read dt b sd <<< "$spec"
  name=ref_${dt}_b${b}_s${sd}
  timeout -k 10 ${PARITY_TIMEOUT:-600} python -m hfrep parity --preset reference --model mtss_wgan_gp --graph --dtype $dt --epochs ${3:-5000} \
      --batch-size $b --seed $sd --no-save --quiet --log $OUT/${name}_train_log.jsonl --out $OUT/$name.json \
      > $OUT/$name.log 2>&1 || { echo "FAIL $name"; tail -20 $OUT/$name.log; exit 1; }
  echo "$name: $(cat $OUT/$name.json | head -c 400)"
done
