"""Data IO: CSV readers, data-root resolution and a *non-executing* pickle reader.

Reference behaviour: ``helper.read_csv`` (helper.py:18-23) parses ``Date`` and indexes by it;
``helper.dic_read`` (helper.py:26-29) is ``pickle.load``.  Unpickling untrusted files executes
code, so this framework reads ``.pkl`` files with :func:`safe_pickle_load`, an opcode
interpreter for the plain-data subset of the pickle protocol (dict/list/tuple/str/bytes/
numbers/bool/None, and ``numpy.ndarray`` payloads rebuilt from their raw bytes).  It never
imports or calls anything named inside the file; unknown globals raise ``ValueError``.
"""
from __future__ import annotations

import io
import json
import os
import pickletools
import struct
from typing import Any

import numpy as np
import pandas as pd

# ----------------------------------------------------------------------------------------
# data-root resolution
# ----------------------------------------------------------------------------------------
_REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def data_root() -> str | None:
    """Directory holding ``cleaned_data/`` and ``data/`` (reference layout).

    Search order: ``$HFREP_DATA_ROOT``, ``<repo>/assets``, ``/root/reference``.
    Returns ``None`` when no dataset is present (synthetic data is then the only source).
    """
    cands = [os.environ.get("HFREP_DATA_ROOT"), os.path.join(_REPO_ROOT, "assets"), "/root/reference"]
    for c in cands:
        if c and os.path.isdir(os.path.join(c, "cleaned_data")):
            return c
    return None


def require_data_root() -> str:
    r = data_root()
    if r is None:
        raise FileNotFoundError(
            "no dataset found: set HFREP_DATA_ROOT to a directory containing cleaned_data/ and data/"
        )
    return r


# ----------------------------------------------------------------------------------------
# CSV
# ----------------------------------------------------------------------------------------
def read_csv(loc: str, date: bool = True) -> pd.DataFrame:
    """``pd.read_csv`` with the ``Date`` column parsed and set as index (helper.py:18-23)."""
    df = pd.read_csv(loc)
    if date:
        df["Date"] = pd.to_datetime(df["Date"])
        df = df.set_index("Date")
    return df


# ----------------------------------------------------------------------------------------
# non-executing pickle reader
# ----------------------------------------------------------------------------------------
class _Global:
    __slots__ = ("module", "name")

    def __init__(self, module: str, name: str):
        self.module, self.name = module, name

    def key(self):
        return f"{self.module}.{self.name}"


class _Reduce:
    """A deferred ``callable(*args)`` whose callable is one of the whitelisted numpy rebuilders."""

    __slots__ = ("func", "args", "state")

    def __init__(self, func, args):
        self.func, self.args, self.state = func, args, None


_NUMPY_RECON = {"numpy.core.multiarray._reconstruct", "numpy._core.multiarray._reconstruct"}
_NUMPY_DTYPE = {"numpy.dtype"}
_NUMPY_SCALAR = {"numpy.core.multiarray.scalar", "numpy._core.multiarray.scalar"}
_NUMPY_NDARRAY = {"numpy.ndarray"}
_CODECS_ENCODE = {"_codecs.encode"}


def _finish(obj):
    """Materialise deferred numpy objects into real numpy values (data only)."""
    if isinstance(obj, _Reduce):
        k = obj.func.key()
        if k in _NUMPY_RECON:
            if obj.state is None:
                raise ValueError("ndarray pickle without state")
            st = obj.state
            # (version, shape, dtype, is_fortran, rawdata)
            _, shape, dt, fortran, raw = st
            dt = _finish(dt)
            if isinstance(raw, list):
                arr = np.array(raw, dtype=dt)
            else:
                arr = np.frombuffer(bytes(raw), dtype=dt).copy()
            arr = arr.reshape(tuple(shape), order="F" if fortran else "C")
            return arr
        if k in _NUMPY_DTYPE:
            name = obj.args[0]
            dt = np.dtype(name)
            if obj.state is not None:
                # state = (version, byteorder, subdescr, names, fields, elsize, alignment, flags)
                bo = obj.state[1]
                if bo in ("<", ">"):
                    dt = dt.newbyteorder(bo)
            return dt
        if k in _NUMPY_SCALAR:
            dt = _finish(obj.args[0])
            raw = obj.args[1]
            return np.frombuffer(bytes(raw), dtype=dt)[0]
        if k in _CODECS_ENCODE:
            s, enc = obj.args
            return s.encode(enc)
        raise ValueError(f"refusing to call {k} while reading a pickle")
    if isinstance(obj, dict):
        return {_finish(k): _finish(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_finish(v) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_finish(v) for v in obj)
    if isinstance(obj, _Global):
        raise ValueError(f"refusing bare global {obj.key()} in pickle")
    return obj


def safe_pickle_load(path_or_bytes) -> Any:
    """Interpret a pickle WITHOUT executing it.

    Supports protocol 0-5 data opcodes plus ``numpy.ndarray``/``numpy.dtype``/numpy scalar
    payloads (rebuilt from raw bytes).  Any other global raises ``ValueError``.
    """
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    stack: list = []
    marks: list = []
    memo: dict = {}

    def pop_mark():
        m = marks.pop()
        items = stack[m:]
        del stack[m:]
        return items

    for op, arg, _pos in pickletools.genops(io.BytesIO(data)):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            break
        if n == "MARK":
            marks.append(len(stack))
        elif n in ("EMPTY_DICT",):
            stack.append({})
        elif n == "DICT":
            items = pop_mark()
            stack.append({items[i]: items[i + 1] for i in range(0, len(items), 2)})
        elif n in ("EMPTY_LIST",):
            stack.append([])
        elif n == "LIST":
            stack.append(list(pop_mark()))
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n == "TUPLE1":
            stack[-1:] = [tuple(stack[-1:])]
        elif n == "TUPLE2":
            stack[-2:] = [tuple(stack[-2:])]
        elif n == "TUPLE3":
            stack[-3:] = [tuple(stack[-3:])]
        elif n in ("EMPTY_SET",):
            stack.append(set())
        elif n == "ADDITEMS":
            items = pop_mark()
            stack[-1].update(items)
        elif n == "FROZENSET":
            stack.append(frozenset(pop_mark()))
        elif n == "SETITEM":
            v = stack.pop(); k = stack.pop(); stack[-1][k] = v
        elif n == "SETITEMS":
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif n == "APPEND":
            v = stack.pop(); stack[-1].append(v)
        elif n == "APPENDS":
            items = pop_mark(); stack[-1].extend(items)
        elif n in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE", "SHORT_BINSTRING", "BINSTRING",
                   "STRING"):
            stack.append(arg)
        elif n in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8", "BYTEARRAY8"):
            stack.append(bytes(arg))
        elif n in ("BININT", "BININT1", "BININT2", "INT", "LONG", "LONG1", "LONG4", "BINFLOAT", "FLOAT"):
            stack.append(arg)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n in ("MEMOIZE",):
            memo[len(memo)] = stack[-1]
        elif n in ("PUT", "BINPUT", "LONG_BINPUT"):
            memo[arg] = stack[-1]
        elif n in ("GET", "BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif n == "GLOBAL":
            mod, name = arg.split(" ", 1)
            stack.append(_Global(mod, name))
        elif n == "STACK_GLOBAL":
            name = stack.pop(); mod = stack.pop()
            stack.append(_Global(mod, name))
        elif n == "REDUCE":
            args = stack.pop(); fn = stack.pop()
            if not isinstance(fn, _Global):
                raise ValueError("REDUCE on non-global")
            stack.append(_Reduce(fn, args))
        elif n == "BUILD":
            st = stack.pop()
            obj = stack[-1]
            if not isinstance(obj, _Reduce):
                raise ValueError("BUILD on unsupported object")
            obj.state = st
        elif n == "NEWOBJ":
            args = stack.pop(); cls = stack.pop()
            stack.append(_Reduce(cls, args))
        elif n == "POP":
            stack.pop()
        elif n == "POP_MARK":
            pop_mark()
        elif n == "DUP":
            stack.append(stack[-1])
        elif n == "NEXT_BUFFER" or n == "READONLY_BUFFER":
            raise ValueError("out-of-band buffers unsupported")
        else:
            raise ValueError(f"unsupported pickle opcode {n}")
    if len(stack) != 1:
        raise ValueError("malformed pickle")
    return _finish(stack[0])


def dic_read(loc: str) -> Any:
    """Safe replacement for ``helper.dic_read`` (helper.py:26-29)."""
    return safe_pickle_load(loc)


def dic_save(dic: Any, loc: str, verbose: bool = True) -> None:
    """``helper.dic_save`` (helper.py:155-162): pickle to ``loc`` then re-read as a check.

    Files written here are produced by this framework, so a standard pickle dump is used for
    format compatibility; the read-back goes through :func:`safe_pickle_load`.
    """
    import pickle

    with open(loc, "wb") as fh:
        pickle.dump(dic, fh, protocol=4)
    out = safe_pickle_load(loc)
    if verbose:
        print("stored dictionary:\n")
        print(out)


# ----------------------------------------------------------------------------------------
# cleaned dataset bundle
# ----------------------------------------------------------------------------------------
def load_cleaned(root: str | None = None) -> dict:
    """Load ``cleaned_data`` (hfd, factor_etf_data, rf, name maps) from the reference layout."""
    root = root or require_data_root()
    cd = os.path.join(root, "cleaned_data")
    out = {
        "hfd": read_csv(os.path.join(cd, "hfd.csv")),
        "factor_etf_data": read_csv(os.path.join(cd, "factor_etf_data.csv")),
        "rf": read_csv(os.path.join(cd, "rf.csv")),
    }
    for key, fname in (("hfd_fullname", "hfd_fullname"), ("factor_etf_name", "factor_etf_name")):
        js = os.path.join(cd, fname + ".json")
        pk = os.path.join(cd, fname + ".pkl")
        if os.path.exists(js):
            out[key] = json.load(open(js))
        elif os.path.exists(pk):
            out[key] = safe_pickle_load(pk)
        else:
            cols = out["hfd" if key == "hfd_fullname" else "factor_etf_data"].columns
            out[key] = {c: c for c in cols}
    out["all_data_name"] = {**out["factor_etf_name"], **out["hfd_fullname"]}
    return out


def load_daily_etf(root: str | None = None, tickers=None):
    """The DAILY ETF excess-return matrix and its daily rf (``cleaning.build_factor_etf_daily``), as
    ``(excess, rf_daily)`` DataFrame / Series: from ``cleaned_data/factor_etf_daily.csv`` +
    ``rf_daily.csv`` when staged there (GPU boxes: scripts/stage_reference_data.sh), otherwise built from
    the raw ``data/ETF_data.csv`` and the Fama-French daily file.  Default: all 22 factor columns (the 8
    CBOE option indices from the shipped raw prices)."""
    from .cleaning import ETF_TICKERS, build_factor_etf_daily

    tickers = list(tickers or ETF_TICKERS)
    root = root or require_data_root()
    cd = os.path.join(root, "cleaned_data")
    fx, fr = os.path.join(cd, "factor_etf_daily.csv"), os.path.join(cd, "rf_daily.csv")
    if os.path.exists(fx) and os.path.exists(fr):
        ex = read_csv(fx)
        return ex[[t for t in tickers if t in ex.columns]], read_csv(fr).iloc[:, 0]
    raw = os.path.join(root, "data")
    return build_factor_etf_daily(os.path.join(raw, "ETF_data.csv"), os.path.join(raw, "F-F_Research_Data_Factors_daily.CSV"),
                                  tickers=tickers)
