#!/bin/bash
# Round-5 GPU pass 6: LayerNorm forward on the grid-stride two-row kernel (tests + per-call time; the
# previous build's numbers come from HFREP_NATIVE_LIB=variants/ln_old if present), then the second
# segment of the bf16 B = 32 768 parity run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_sixth}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm or trainer_gradients" \
  > $OUT/tests_ln.txt 2>&1
rc=$?; tail -n 3 $OUT/tests_ln.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/bench_ln.py > $OUT/ln_new.jsonl 2>&1 || { tail -n 20 $OUT/ln_new.jsonl; exit 1; }
if [ -f variants/ln_old/_hfrep_native.so ]; then
  HFREP_NATIVE_LIB=$R/variants/ln_old/_hfrep_native.so timeout -k 10 200 python -u scripts/bench_ln.py > $OUT/ln_old.jsonl 2>&1 \
    || { tail -n 20 $OUT/ln_old.jsonl; exit 1; }
fi
grep -h '"ms' $OUT/ln_*.jsonl
PARITY_TIMEOUT=${SEG_TIMEOUT:-700} bash scripts/gpu_parity_seg.sh ${1:-r05_sixth} "bfloat16:32768:123:5000"
