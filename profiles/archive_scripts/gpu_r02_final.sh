#!/bin/bash
# round-end rehearsal: full GPU suite, smoke(), the driver's default bench (fp32 headline + bf16
# sub-record at 262k), and a kernel profile of both dtypes at the bench shape
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT:-r02_final}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench.err && cat $O/bench_default.json || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
