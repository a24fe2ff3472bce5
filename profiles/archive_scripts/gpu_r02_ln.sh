#!/bin/bash
# LayerNorm tangent kernels + LN-critic GP gradients, AE on the GPU (BASELINE config 2), GAN / WGAN-GP
# MLP configs (BASELINE configs 3 / 4) through bench.py at one GPU, and a GPU AE latent sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02_ln; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_ae_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "layernorm or trainer_gradients or ae_ or gan_eval" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for m in gan wgan_gp; do
  for dt in bfloat16 float32; do
    timeout -k 10 240 python -u bench.py --model $m --steps 5 --warmup 2 --dtype $dt > $O/bench_${m}_${dt}.json 2> $O/bench_${m}_${dt}.err \
      && cat $O/bench_${m}_${dt}.json || { echo BENCH_FAIL $m $dt; tail $O/bench_${m}_${dt}.err; exit 1; }
  done
done
for dt in float32 bfloat16; do
  timeout -k 10 600 python -u -m hfrep replicate --method ae-sweep --latents 1-21 --seed 123 --device cuda --dtype $dt \
      --out $O/ae_sweep_real_cuda_${dt}_s123.json > $O/ae_${dt}.log 2>&1 || { echo AE_FAIL $dt; tail -20 $O/ae_${dt}.log; exit 1; }
  echo "ae $dt done"
done
