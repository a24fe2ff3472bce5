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
