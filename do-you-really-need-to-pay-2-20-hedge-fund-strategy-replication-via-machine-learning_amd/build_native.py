"""Native build driver for the hfrep gfx950 kernel library.

Compiles every ``csrc/*.hip`` kernel translation unit with ``hipcc --offload-arch=gfx950``
and the torch op bindings (``csrc/bindings.cpp``), then links them IN-TREE into
``ops/_hfrep_native.so``.  The library registers ``torch.ops.hfrep.*`` when loaded with
``torch.ops.load_library`` (see ``ops/_native.py``).

No hipify, no torch JIT cache: the objects live under ``build/native`` and the shared object
lives next to the Python code so it travels with the repository snapshot to the GPU box.

Usage::

    python -m hfrep.build_native          # incremental
    python build_native.py --force        # full rebuild
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import json
import os
import re
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_SO = os.path.join(HERE, "ops", "_hfrep_native.so")
BUILD_DIR = os.path.join(os.path.dirname(HERE), "build", "native")
ARCH = os.environ.get("HFREP_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (expected /opt/rocm/bin/hipcc)")


def _torch_paths():
    import torch  # noqa: F401  (only for include/lib paths)
    from torch.utils import cpp_extension

    incs = cpp_extension.include_paths()
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return incs, libdir, abi


def _flags():
    incs, libdir, abi = _torch_paths()
    common = ["-O3", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-I{CSRC}"]
    kern = common + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-ffp-contract=fast"]
    bind = common + [f"--offload-arch={ARCH}", "-DUSE_ROCM", "-D__HIP_PLATFORM_AMD__", "-DTORCH_EXTENSION_NAME=hfrep_native",
                     "-DTORCH_API_INCLUDE_EXTENSION_H", "-Wno-unused-result", "-Wno-deprecated-declarations"]
    bind += [f"-I{p}" for p in incs] + [f"-I{sysconfig.get_paths()['include']}"]
    link = ["-shared", "-fPIC", f"--offload-arch={ARCH}", f"-L{libdir}", f"-Wl,-rpath,{libdir}",
            "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip"]
    return kern, bind, link


# per-translation-unit extra flags.  lstm_f32.hip: its split weight-gradient kernel runs one
# straight-line body per wave kind behind a switch on the wave index; SimplifyCFG's common-code
# sinking merged those bodies into one block with a run-time accumulator index, which moved the
# accumulators to scratch memory (80 B per lane at K = 32)
EXTRA_FLAGS = {"lstm_f32.hip": ["-mllvm", "-simplifycfg-sink-common=false"]}


def kernel_flags(src: str) -> list[str]:
    """The full hipcc flag list the library build uses for the kernel source ``src``."""
    return _flags()[0] + EXTRA_FLAGS.get(os.path.basename(src), [])


def _sources():
    hips = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    cpps = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".cpp"))
    headers = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h"))
    return hips, cpps, headers


def _digest(paths, extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    for p in paths:
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:20]


_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _local_headers(src: str) -> list[str]:
    """The csrc headers ``src`` includes, transitively (``#include "x.h"`` lines): a TU's stamp depends
    on exactly these, so a new header only rebuilds the TUs that include it."""
    seen, todo = [], [src]
    while todo:
        with open(todo.pop(), encoding="utf-8", errors="replace") as fh:
            text = fh.read()
        for name in _INC.findall(text):
            p = os.path.join(CSRC, name)
            if os.path.exists(p) and p not in seen:
                seen.append(p)
                todo.append(p)
    return sorted(seen)


def _compile(src, obj, flags, headers):
    stamp = obj + ".stamp"
    headers = [h for h in headers if h in set(_local_headers(src))]
    dig = _digest([src] + headers, " ".join(flags))
    if os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == dig:
        return obj, False
    cmd = [_hipcc()] + flags + ["-c", src, "-o", obj]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    with open(stamp, "w") as fh:
        fh.write(dig)
    return obj, True


def build(force: bool = False, jobs: int | None = None, verbose: bool = True, variant: str | None = None,
          extra: list[str] | None = None) -> str:
    """Build the library.  ``variant`` / ``extra``: an A/B build of the same sources with extra kernel
    flags (e.g. ``-DHFREP_TBWD_DXGEN=1``) into ``variants/<variant>/_hfrep_native.so`` (objects under
    ``build/native_<variant>``), loaded through ``HFREP_NATIVE_LIB``; the default build is untouched."""
    out_so = OUT_SO if not variant else os.path.join(os.path.dirname(HERE), "variants", variant, "_hfrep_native.so")
    bdir = BUILD_DIR if not variant else BUILD_DIR + "_" + variant
    os.makedirs(bdir, exist_ok=True)
    os.makedirs(os.path.dirname(out_so), exist_ok=True)
    kern, bind, link = _flags()
    kern = kern + list(extra or [])
    hips, cpps, headers = _sources()
    if force:
        for f in os.listdir(bdir):
            os.remove(os.path.join(bdir, f))
    jobs = jobs or min(8, os.cpu_count() or 4, 16)
    tasks = [(s, os.path.join(bdir, os.path.basename(s) + ".o"), kern + EXTRA_FLAGS.get(os.path.basename(s), []))
             for s in hips]
    tasks += [(s, os.path.join(bdir, os.path.basename(s) + ".o"), bind + list(extra or [])) for s in cpps]
    changed = False
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, o, f, headers) for s, o, f in tasks]
        objs = []
        for fut in futs:
            o, c = fut.result()
            objs.append(o)
            changed |= c
    OUT = out_so
    if changed or not os.path.exists(OUT) or force:
        tmp = OUT + ".tmp"
        cmd = [_hipcc()] + objs + link + ["-o", tmp]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
        os.replace(tmp, OUT)
        meta = {"arch": ARCH, "sources": [os.path.basename(s) for s in hips + cpps], "extra": list(extra or [])}
        with open(OUT + ".json", "w") as fh:
            json.dump(meta, fh)
        if verbose:
            print(f"[hfrep.build_native] linked {OUT} ({len(objs)} objects)")
    elif verbose:
        print(f"[hfrep.build_native] up to date: {OUT}")
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--variant", default=None, help="A/B build name (variants/<name>/_hfrep_native.so)")
    ap.add_argument("--extra", default="", help="extra kernel flags of the variant build (one string)")
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs, variant=a.variant, extra=a.extra.split() if a.extra else None)


if __name__ == "__main__":
    sys.exit(main())
