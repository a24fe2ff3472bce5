#!/bin/bash
# Round-6 BASELINE config 2 on the daily ETF matrix: its GPU tests, then the k = 1..21 daily sweep in fp32
# and bf16 (python -m hfrep replicate --method ae-sweep --freq daily).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r06_ae_daily}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ae_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -n 15 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for dt in float32 bfloat16; do
  timeout -k 10 600 python -u -m hfrep replicate --method ae-sweep --freq daily --latents 1-21 --device cuda --dtype $dt \
    --out $OUT/daily_$dt.json > $OUT/daily_$dt.log 2>&1 || { tail $OUT/daily_$dt.log; exit 1; }
  python -c "import json; d=json.load(open('$OUT/daily_$dt.json'))['ae_sweep_daily']; print('$dt', d['rows'], d['fit_s'], d['elapsed_s'], {k: round(v['OOS_r2'],3) for k, v in d['metrics'].items()})"
done
