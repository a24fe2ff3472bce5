#!/bin/bash
# Round-5 AE study with every (seed, latent) fit of a (dtype, panel) in ONE csrc/ae.hip launch: 30 seeds x
# fp32 / bf16 x real / augmented (compare locally: scripts/ae_compare.py against profiles/r04_ae).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_ae}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/ae_study.py --out $OUT --seeds ${2:-1-30} --dtypes float32,bfloat16 --device cuda > $OUT/study.log 2>&1 \
  || { tail -n 20 $OUT/study.log; exit 1; }
cat $OUT/study.log
