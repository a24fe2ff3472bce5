#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/dbg; export TMPDIR=/tmp
for cfg in "$@"; do
  set -- $cfg
  HFREP_NATIVE_LIB=$PWD/ab_libs/old.so timeout -k 10 200 python scripts/dbg_ops.py $cfg > gpurun_out/dbg/old.log 2>&1 || { tail -20 gpurun_out/dbg/old.log; exit 1; }
  timeout -k 10 200 python scripts/dbg_ops.py $cfg > gpurun_out/dbg/new.log 2>&1 || { tail -20 gpurun_out/dbg/new.log; exit 1; }
  echo "== $cfg"; paste gpurun_out/dbg/old.log gpurun_out/dbg/new.log | grep -v amdgpu.ids
done
