"""Compare two AE study directories (scripts/ae_study.py outputs): per (panel, dtype, seed) sweep the largest
absolute difference of every metric / Sharpe / turnover value, and the elapsed time of each run.

usage: python scripts/ae_compare.py NEW_DIR OLD_DIR [OLD_DIR2 ...]   (later dirs fill what earlier ones lack)
"""
import glob
import json
import os
import sys


def flat(d, pre=""):
    out = {}
    for k, v in d.items():
        if isinstance(v, dict):
            out.update(flat(v, f"{pre}{k}/"))
        elif isinstance(v, (int, float)):
            out[pre + k] = float(v)
    return out


def main():
    new, olds = sys.argv[1], sys.argv[2:]
    worst, n, exact, t_new, t_old = 0.0, 0, 0, 0.0, 0.0
    for p in sorted(glob.glob(os.path.join(new, "sweep_*.json"))):
        name = os.path.basename(p)
        q = next((os.path.join(o, name) for o in olds if os.path.exists(os.path.join(o, name))), None)
        if q is None:
            continue
        a, b = json.load(open(p))["ae_sweep"], json.load(open(q))["ae_sweep"]
        t_new += a.get("elapsed_s", 0.0)
        t_old += b.get("elapsed_s", 0.0)
        fa, fb = flat({k: a[k] for k in ("metrics", "sharpe_ante", "sharpe_post", "turnover")}), \
            flat({k: b[k] for k in ("metrics", "sharpe_ante", "sharpe_post", "turnover")})
        d = max((abs(fa[k] - fb[k]) for k in fa if k in fb and fa[k] == fa[k] and fb[k] == fb[k]), default=0.0)
        worst = max(worst, d)
        n += 1
        exact += d == 0.0
    print(json.dumps({"sweeps_compared": n, "bitwise_equal_sweeps": exact, "max_abs_diff": worst,
                      "elapsed_s_new_sum": round(t_new, 2), "elapsed_s_old_sum": round(t_old, 2)}))


if __name__ == "__main__":
    main()
