"""Static check of the gfx950 code objects for the buffer-store data hazard the compiler misses
(scripts/isa_store_hazard.py): a >8-byte MUBUF store with a register soffset whose data VGPRs the
next VALU instruction overwrites.  It corrupted a few fp32 BPTT dZ rows per 10^5 at the bench batch
before r02.  CPU only: hipcc cross-compiles every csrc/*.hip to assembly."""
import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "do-you-really-need-to-pay-2-20-hedge-fund-strategy-replication-via-machine-learning_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_no_buffer_store_data_hazard(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import isa_store_hazard

    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))

    # the SHIPPED kernel flags (-ffp-contract=fast, -munsafe-fp-atomics, -fPIC, ...): the hazard depends
    # on register allocation, so the scanned assembly must come from the same compile as the library
    from hfrep import build_native

    def asm(src):
        out = str(tmp_path / (os.path.basename(src) + ".s"))
        subprocess.run([HIPCC] + build_native.kernel_flags(src) + ["--cuda-device-only", "-S", src, "-o", out],
                       check=True, capture_output=True)
        return out

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        files = list(ex.map(asm, srcs))
    hits = [h for f in files for h in isa_store_hazard.scan(f)]
    assert not hits, "\n".join(f"{k[:60]}: {a} -> {b}" for k, a, b in hits)
    shutil.rmtree(tmp_path, ignore_errors=True)
