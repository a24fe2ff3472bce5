#!/bin/bash
# Stage the reference's cleaned panel (CSV only) under assets/ so GPU runs see it: gpurun ships the
# working tree, and hfrep.data.io.data_root() searches <repo>/assets first.  Not committed.
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
SRC=${1:-/root/reference}
mkdir -p "$R/assets/cleaned_data"
for f in hfd.csv factor_etf_data.csv rf.csv; do cp "$SRC/cleaned_data/$f" "$R/assets/cleaned_data/$f"; done
echo "staged $(ls "$R/assets/cleaned_data" | tr '\n' ' ')"
# name maps as JSON (read through the non-executing pickle reader, never unpickled)
PYTHONPATH="$R" python - "$SRC" "$R" <<'PY'
import json, os, sys
import hfrep
from hfrep.data.io import safe_pickle_load
src, dst = sys.argv[1], sys.argv[2]
for n in ("hfd_fullname", "factor_etf_name"):
    p = os.path.join(src, "cleaned_data", n + ".pkl")
    if os.path.exists(p):
        json.dump(safe_pickle_load(p), open(os.path.join(dst, "assets", "cleaned_data", n + ".json"), "w"), indent=1)
print("name maps staged")
PY
# the daily ETF excess-return matrix (BASELINE config 2: hfrep.data.cleaning.build_factor_etf_daily, all
# 22 factor columns) and its daily rf, built from the raw prices here: GPU boxes have no data/ directory
PYTHONPATH="$R" python - "$SRC" "$R" <<'PY'
import os, sys
import hfrep
from hfrep.data.cleaning import ETF_TICKERS, build_factor_etf_daily
src, dst = sys.argv[1], sys.argv[2]
ex, rf = build_factor_etf_daily(os.path.join(src, "data", "ETF_data.csv"),
                                os.path.join(src, "data", "F-F_Research_Data_Factors_daily.CSV"), tickers=ETF_TICKERS)
ex.to_csv(os.path.join(dst, "assets", "cleaned_data", "factor_etf_daily.csv"), float_format="%.17g")
rf.to_frame("RF").to_csv(os.path.join(dst, "assets", "cleaned_data", "rf_daily.csv"), float_format="%.17g")
print("daily panel staged", ex.shape)
PY
