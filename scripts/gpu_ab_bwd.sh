#!/bin/bash
# A/B of the bf16 BPTT (lstm_tbwd4<TG = false>) between the default library and variant builds
# (variants/<name>, HFREP_NATIVE_LIB): the BPTT GPU tests on the default build, per-call times at the
# bench shape, the bf16 bench step and the B = 32 iteration for each.
#   bash scripts/gpu_ab_bwd.sh OUTNAME VARIANT [VARIANT ...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/$1; shift; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "lstm2 or bf16 or lstm_fwd_bwd or slice_averages" > $OUT/tests.txt 2>&1
rc=$?; tail -n 3 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for V in base "$@"; do
  if [ $V = base ]; then unset HFREP_NATIVE_LIB; else export HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so"; fi
  for K in 32 100; do
    timeout -k 10 200 python -u scripts/bench_lstm.py --dtype bfloat16 --batch 262144 --K $K --iters 10 --only bwd,bwd_dx \
      > $OUT/lstm_${V}_K$K.jsonl 2>&1 || { tail -n 20 $OUT/lstm_${V}_K$K.jsonl; exit 1; }
  done
  echo "== $V"; grep -hv amdgpu.ids $OUT/lstm_${V}_K*.jsonl
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --dtype bfloat16 > $OUT/bench_$V.json 2> $OUT/bench_$V.err \
    || { tail $OUT/bench_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$V.json')); print('bench', d['value'], d['ms_per_step'])"
  timeout -k 10 300 python -u scripts/bench_small.py --iters 300 --dtypes bfloat16 > $OUT/small_$V.jsonl 2>&1 \
    || { tail -n 20 $OUT/small_$V.jsonl; exit 1; }
  grep -h '"ms' $OUT/small_$V.jsonl
done
