#!/bin/bash
# After the cross-opcode SrcC fix (xdl_switch, csrc/lstm2.hip): the act = sigmoid tangent reverse run to run at
# B = 32772, the bitwise determinism script at small / large batch (default library and the DX + GEN variant),
# the whole GPU suite, then the headline bench (fp32 + bf16 sub-record).
# usage: scripts/gpu_xdl_fix.sh OUTNAME
set -o pipefail
R0="${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p $R0/gpurun_out/${1:-xdl_fix}; timeout -k 10 120 $R0/scripts/probes/mfma_srcc_probe 2048 64 > $R0/gpurun_out/${1:-xdl_fix}/mfma_srcc.jsonl 2>&1 || exit 1
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/${1:-xdl_fix}; mkdir -p $OUT
timeout -k 10 200 python scripts/dbg_tfwd_tape.py 32772 32 1 2 > $OUT/tbwd_act1.txt 2>&1 || { tail $OUT/tbwd_act1.txt; exit 1; }
grep "'rep'" $OUT/tbwd_act1.txt | sed 's/.hd_equal.*tbwd_same/ ... tbwd_same/'
timeout -k 10 300 python scripts/dbg_determinism.py 128 1 > $OUT/det_large.txt 2>&1 || { tail $OUT/det_large.txt; exit 1; }
echo "default lib, large: $(grep -c False $OUT/det_large.txt) rows with a False"
HFREP_NATIVE_LIB=$R/variants/dxgen/_hfrep_native.so HFREP_TBWD_DXGEN=1 timeout -k 10 300 python scripts/dbg_determinism.py 128 1 \
  > $OUT/det_large_dxgen.txt 2>&1 || { tail $OUT/det_large_dxgen.txt; exit 1; }
echo "dxgen lib, large: $(grep -c False $OUT/det_large_dxgen.txt) rows with a False"
HFREP_NATIVE_LIB=$R/variants/dxgen/_hfrep_native.so HFREP_TBWD_DXGEN=1 timeout -k 10 200 python scripts/dbg_determinism.py 1 3 \
  > $OUT/det_small_dxgen.txt 2>&1 || { tail $OUT/det_small_dxgen.txt; exit 1; }
echo "dxgen lib, small x3: $(grep -c False $OUT/det_small_dxgen.txt) rows with a False"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_all.txt 2>&1 \
  || { tail -n 30 $OUT/tests_all.txt; exit 1; }
tail -n 1 $OUT/tests_all.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
