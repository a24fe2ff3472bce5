#!/bin/bash
# A/B of two builds of the native library on the recurrent-kernel microbench (alternating runs).
# usage: bash scripts/gpu_ab_lstm.sh TAG "ops" [batch]
set -o pipefail
tag=$1; ops=${2:-fwd,tfwd,bwd,bwd_dx,tbwd,tbwd_dx}; B=${3:-262144}
out=gpurun_out/$tag; mkdir -p $out
for r in 1 2; do for v in a b; do
  HFREP_NATIVE_LIB=$PWD/ab_libs/$v.so timeout -k 10 150 python scripts/bench_lstm.py --batch $B --only $ops --iters 5 \
    | sed "s/^{/{\"lib\": \"$v\", /" >> $out/ab.jsonl || exit 1
done; done
python - "$out/ab.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); d[(r["op"], r["lib"])].append(r["ms"])
for op in sorted({k[0] for k in d}):
    a, b = min(d[(op, "a")]), min(d[(op, "b")])
    print(f"{op:10s} a {a:.3f} b {b:.3f} ({(b / a - 1) * 100:+.1f}%)")
PY
