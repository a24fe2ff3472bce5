#!/bin/bash
# Round-5 last GPU pass: whole GPU suite + smoke on the final tree, the BASELINE config 3 / 4 benches
# (vanilla GAN, MLP WGAN-GP) and the headline bench once more.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-r05_close}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests_all.txt 2>&1
rc=$?; tail -n 2 $OUT/tests_all.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
tail -n 1 $OUT/smoke.txt
for M in gan wgan_gp; do
  timeout -k 10 300 python -u bench.py --model $M --steps 5 --warmup 2 > $OUT/bench_$M.json 2> $OUT/bench_$M.err || { tail $OUT/bench_$M.err; exit 1; }
  cut -c1-200 $OUT/bench_$M.json
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['bf16']['value'], d['bf16']['ms_per_step'])"
timeout -k 10 300 python -u scripts/bench_small.py --iters 300 > $OUT/small.jsonl 2>&1 || { tail -n 20 $OUT/small.jsonl; exit 1; }
grep -h '"ms' $OUT/small.jsonl
