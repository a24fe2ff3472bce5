#!/usr/bin/env bash
# Multi-seed AE replication study (real and generator-augmented panels), CPU fp32.
# usage: scripts/ae_seed_study.sh OUTDIR FIRST_SEED LAST_SEED [PARALLEL]
# Each seed: the reference production generator (.h5) draws 10 x 168 x 36 windows with that seed
# (autoencoder_v4.ipynb:1291), then one latent sweep k = 1..21 on real and one on augmented data.
set -euo pipefail
out=$1; s0=$2; s1=$3; par=${4:-6}
H5=${HFREP_H5:-/root/reference/GAN/trained_generator/MTTS_GAN_GP20220621_02-49-32.h5}
mkdir -p "$out"
export OMP_NUM_THREADS=1 MKL_NUM_THREADS=1
one() {
  s=$1
  python -m hfrep generate --ckpt "$H5" --n 10 --window 168 --seed "$s" --device cpu --out "$out/aug_s$s.npy" > /dev/null
  python -m hfrep replicate --method ae-sweep --latents 1-21 --seed "$s" --out "$out/sweep_real_cpu_fp32_s$s.json" > /dev/null
  python -m hfrep replicate --method ae-sweep --latents 1-21 --seed "$s" --augment "$out/aug_s$s.npy" \
    --out "$out/sweep_augmented_cpu_fp32_s$s.json" > /dev/null
  echo "seed $s done"
}
export -f one
export out H5
seq "$s0" "$s1" | xargs -P "$par" -I{} bash -c 'one {}'
