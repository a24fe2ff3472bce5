#!/bin/bash
# Stage the reference's cleaned panel (CSV only) under assets/ so GPU runs see it: gpurun ships the
# working tree, and hfrep.data.io.data_root() searches <repo>/assets first.  Not committed.
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
SRC=${1:-/root/reference}
mkdir -p "$R/assets/cleaned_data"
for f in hfd.csv factor_etf_data.csv rf.csv; do cp "$SRC/cleaned_data/$f" "$R/assets/cleaned_data/$f"; done
echo "staged $(ls "$R/assets/cleaned_data" | tr '\n' ' ')"
