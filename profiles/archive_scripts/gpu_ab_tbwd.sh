#!/bin/bash
# fp32 tangent reverse (lstmf_tbwdp_kernel): numerics, then base vs variants/<v> timing and the step.
#   bash profiles/archive_scripts/gpu_ab_tbwd.sh <outdir> <variant> [<variant> ...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/$1; shift; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "lstmf_fused_layer or persistent_multi_pass or tbwd or tangent" > $OUT/tests.log 2>&1 \
  || { tail -n 30 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
for V in base "$@"; do
  if [ $V = base ]; then unset HFREP_NATIVE_LIB
  else
    export HFREP_NATIVE_LIB="$R/variants/$V/_hfrep_native.so"
    test -f "$HFREP_NATIVE_LIB" || { echo "no $HFREP_NATIVE_LIB"; exit 1; }
  fi
  timeout -k 10 200 python -u scripts/bench_lstm.py --dtype float32 --batch 65536 --K 100 --iters 10 --only tbwd,tbwd_dx \
    > $OUT/lstm_$V.jsonl 2>&1 || { tail -n 20 $OUT/lstm_$V.jsonl; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > $OUT/bench_$V.json 2> $OUT/bench_$V.err \
    || { tail $OUT/bench_$V.err; exit 1; }
  echo "== $V"; grep -hv amdgpu.ids $OUT/lstm_$V.jsonl; cat $OUT/bench_$V.json
done
