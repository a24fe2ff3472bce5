#!/bin/bash
# Round-6 full pass: the whole GPU suite + smoke on the current tree, the headline bench (fp32 record + bf16
# sub-record) and the BASELINE config 3 / 4 benches.
#   bash scripts/gpu_r06_full.sh OUTNAME [skip-tests]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r06_full}; mkdir -p $OUT; export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests_all.txt 2>&1
  rc=$?; tail -n 3 $OUT/tests_all.txt; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/tests_all.txt | head; exit $rc; }
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
  tail -n 1 $OUT/smoke.txt
fi
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('headline', d['value'], d['ms_per_step'], d['bf16']['value'], d['bf16']['ms_per_step'])"
for M in wgan_gp gan; do
  timeout -k 10 300 python -u bench.py --model $M --steps 5 --warmup 2 > $OUT/bench_$M.json 2> $OUT/bench_$M.err || { tail $OUT/bench_$M.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$M.json')); print('$M', d['value'], d['ms_per_step'], d['bf16']['value'], d['bf16']['ms_per_step'])"
done
