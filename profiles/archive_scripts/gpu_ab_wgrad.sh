#!/bin/bash
# A/B of two native-library builds (ab_libs/a.so, b.so) on the weight-gradient microbench.
set -o pipefail
out=gpurun_out/${1:-ab_wgrad}; B=${2:-262144}; mkdir -p $out
for r in 1 2; do for v in a b; do
  HFREP_NATIVE_LIB=$PWD/ab_libs/$v.so timeout -k 10 150 python scripts/bench_wgrad.py --batch $B --iters 5 \
    | sed "s/^{/{\"lib\": \"$v\", /" >> $out/ab.jsonl || exit 1
done; done
cat $out/ab.jsonl
