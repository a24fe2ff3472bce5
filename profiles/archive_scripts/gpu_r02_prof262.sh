#!/bin/bash
# the fp32 headline step's kernel profile at the bench shape + the GPU AE sweep wall time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_prof262; mkdir -p $O; export TMPDIR=/tmp
bash scripts/gpu_prof_dtype.sh r02_prof262/fp32 float32 262144 > /dev/null && head -30 gpurun_out/r02_prof262/fp32/prof_summary.txt
for dt in float32 bfloat16; do
  timeout -k 10 600 python -u -m hfrep replicate --method ae-sweep --latents 1-21 --seed 123 --device cuda --dtype $dt \
      --out $O/ae_sweep_cuda_${dt}.json > $O/ae_${dt}.log 2>&1 || { echo AE_FAIL; tail $O/ae_${dt}.log; exit 1; }
  grep -o '"elapsed_s": [0-9.]*' $O/ae_sweep_cuda_${dt}.json
done
