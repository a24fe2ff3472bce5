#!/bin/bash
# W-dist parity runs at the reference preset (5000 iterations), split over GPU calls: each spec trains
# to STOP with a checkpoint in ./parity_ckpt/<name> (in-tree, so it travels with the next call's
# snapshot after scripts/parity_ckpt_sync.sh) and resumes from it; the run that reaches 5000 reports
# W-dist.  usage: bash scripts/gpu_parity_seg.sh TAG "dtype:batch:seed:stop ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-parity_seg}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for spec in $2; do
  IFS=: read dt b sd stop <<< "$spec"
  name=ref_${dt}_b${b}_s${sd}
  CK=parity_ckpt/$name; mkdir -p $CK
  timeout -k 10 ${PARITY_TIMEOUT:-1000} python -m hfrep parity --preset reference --model mtss_wgan_gp --graph --dtype $dt \
      --batch-size $b --seed $sd --no-save --quiet --ckpt-dir $CK --resume auto --stop-at $stop \
      --log $OUT/${name}_to${stop}_train_log.jsonl --out $OUT/$name.json > $OUT/${name}_to${stop}.log 2>&1 \
      || { echo "FAIL $name"; tail -20 $OUT/${name}_to${stop}.log; exit 1; }
  mkdir -p $OUT/ckpt/$name && cp $CK/state_*.pt $OUT/ckpt/$name/
  echo "$name -> $stop: $(tail -n 1 $OUT/${name}_to${stop}.log | head -c 400)"
done
