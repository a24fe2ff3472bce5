"""MFMA-busy / VALU-per-MFMA / LDS-conflict table from scripts/pmc_summary.py outputs.

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs) (the per-XCD GRBM counter);
LDS conflict = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS (extra cycles per LDS-active cycle).
usage: python scripts/pmc_table.py SUMMARY.txt [SUMMARY.txt ...]
"""
import re
import sys


def parse(path):
    out, name = {}, None
    for line in open(path):
        if not line.startswith(" ") and line.strip():
            name = line.strip()
            out[name] = {}
        elif name and line.strip():
            k, v = line.split()[:2]
            out[name][k] = float(v)
    return out


def main(paths):
    print("# kernel                                                            MFMA busy  VALU/MFMA  LDS conflict/LDS-active")
    for p in paths:
        for name, d in parse(p).items():
            if not name.startswith("hfrep::") or not d.get("SQ_INSTS_MFMA"):
                continue
            busy = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * d.get("GRBM_GUI_ACTIVE", 1) / 8)
            vm = d.get("SQ_INSTS_VALU", 0) / d["SQ_INSTS_MFMA"]
            lc = d.get("SQ_LDS_BANK_CONFLICT", 0) / max(d.get("SQ_ACTIVE_INST_LDS", 1), 1)
            print(f"{name[:66]:66s} {100 * busy:8.1f}%  {vm:9.2f}  {lc:8.2f}")


if __name__ == "__main__":
    main(sys.argv[1:])
