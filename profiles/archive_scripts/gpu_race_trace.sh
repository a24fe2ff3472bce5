set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; OUT=gpurun_out/r03_race_trace; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp && HFREP_NATIVE_LIB=$R/variants/dxgen/_hfrep_native.so HFREP_TBWD_DXGEN=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python $R/scripts/dbg_tbwd_gen.py 32 > $R/$OUT/log.txt 2>&1 || { tail $R/$OUT/log.txt; exit 1; }
cd $R && grep -h tbwd $(find $OUT/prof -name "*kernel_stats.csv") | cut -c1-160
