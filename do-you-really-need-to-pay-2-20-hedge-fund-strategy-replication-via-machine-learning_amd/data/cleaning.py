"""Raw -> cleaned data pipeline (reference part 1, ``data_cleaning+benchmark.ipynb``).

The reference notebook is missing from the snapshot (``.MISSING_LARGE_BLOBS:4``); its outputs
``cleaned_data/{hfd,factor_etf_data,rf}.csv`` are the golden files.  The transformations
below were recovered numerically:

* ``rf``   = log(1 + sum over the month of daily Fama-French RF / 100), month-end index;
* ``hfd``  = log(1 + NAVROR/100) - rf   (Credit Suisse HF index monthly returns, in %);
* ``factor_etf`` = log(P_m / P_{m-1}) - rf on the LAST available price of each month.

Sample window 1994-04-30 .. 2022-04-30 (337 months).  Eight CBOE option-index columns cannot
be regenerated from the shipped ``data/ETF_data.csv`` (the authors used a fuller price file,
``data/ETF_data_full.csv``, also missing); :func:`build_factor_etf` accepts an alternate price
frame for them (``overrides``).
"""
from __future__ import annotations

import os
import re

import numpy as np
import pandas as pd

START, END = "1994-04-30", "2022-04-30"

ETF_TICKERS = [
    "LUMSTRUU", "LT09STAT", "WGBI", "EMUSTRUU", "TWEXB", "SPGSCI_PM", "SPGSCI_Gra", "SPGSCI_O", "LCB1TRUU",
    "MSCI_EXUS", "MSCI_EM", "R1000", "R200", "FTSE_REIT", "VIX", "PUT", "PUTY", "CLL", "BFLY", "BXM", "BXY", "CLLZ",
]
# columns reproducible from the shipped raw price file (Q12)
REPRODUCIBLE_ETF = ETF_TICKERS[:14]


def _month_end_index(idx) -> pd.DatetimeIndex:
    return pd.DatetimeIndex(idx).to_period("M").to_timestamp(how="end").normalize()


def build_rf(ff_daily_csv: str, start: str = START, end: str = END) -> pd.DataFrame:
    """Monthly log risk-free rate from the Fama-French daily factor file (percent units)."""
    ff = pd.read_csv(ff_daily_csv, usecols=["Date", "RF"])
    ff["Date"] = pd.to_datetime(ff["Date"].astype(str), format="%Y%m%d")
    monthly = ff.set_index("Date")["RF"].groupby(pd.Grouper(freq="ME")).sum()
    rf = np.log(1.0 + monthly / 100.0)
    rf.index = _month_end_index(rf.index)
    out = rf.loc[start:end].to_frame("RF")
    out.index.name = "Date"
    return out


def _parse_pct(x):
    if isinstance(x, str):
        x = x.strip()
        if x == "":
            return np.nan
        return float(x.rstrip("%")) / 100.0
    return float(x) / 100.0 if x == x else np.nan


def build_hfd(navror_csv: str, rf: pd.DataFrame, start: str = START, end: str = END) -> pd.DataFrame:
    """Hedge-fund index excess log returns from ``data/NAVROR_full.csv`` (two header rows)."""
    raw = pd.read_csv(navror_csv, header=1, dtype=str)
    raw = raw.dropna(subset=["Date"])
    dates = pd.to_datetime(raw["Date"], format="%Y-%m-%d", errors="coerce")
    vals = raw.drop(columns=["Date"]).map(_parse_pct)
    vals.index = _month_end_index(dates)
    vals = vals.sort_index()
    logr = np.log1p(vals)
    out = logr.loc[start:end].sub(rf.loc[start:end, "RF"], axis=0)
    out.index.name = "Date"
    return out


_YMD = re.compile(r"^\d{4}[-/]\d{1,2}[-/]\d{1,2}$")


def _parse_mixed_date(s: str):
    s = s.strip()
    if not s:
        return pd.NaT
    if _YMD.match(s):
        return pd.to_datetime(s.replace("/", "-"), format="%Y-%m-%d", errors="coerce")
    return pd.to_datetime(s.replace("/", "-"), format="%d-%m-%Y", errors="coerce")


def read_etf_prices(etf_csv: str) -> dict[str, pd.Series]:
    """Parse the paired (date, price) column layout of ``data/ETF_data.csv``."""
    raw = pd.read_csv(etf_csv, header=None, dtype=str, skiprows=1, encoding="utf-8-sig")
    tickers = raw.iloc[0].tolist()
    body = raw.iloc[1:]
    out = {}
    for j in range(0, raw.shape[1] - 1, 2):
        name = tickers[j + 1] if isinstance(tickers[j + 1], str) else None
        if not name:
            continue
        d = body.iloc[:, j].dropna()
        p = pd.to_numeric(body.iloc[:, j + 1].loc[d.index], errors="coerce")
        dates = d.map(_parse_mixed_date)
        s = pd.Series(p.values, index=pd.DatetimeIndex(dates.values)).dropna()
        s = s[~s.index.isna()].sort_index()
        out[name.strip()] = s
    return out


def month_end_last(prices: pd.Series) -> pd.Series:
    m = prices.groupby(prices.index.to_period("M")).last()
    m.index = m.index.to_timestamp(how="end").normalize()
    return m


def build_factor_etf(etf_csv: str, rf: pd.DataFrame, tickers=ETF_TICKERS, overrides: dict | None = None,
                     start: str = START, end: str = END) -> pd.DataFrame:
    prices = read_etf_prices(etf_csv)
    if overrides:
        prices.update(overrides)
    cols = {}
    for t in tickers:
        if t not in prices:
            continue
        m = month_end_last(prices[t])
        cols[t] = np.log(m / m.shift(1))
    df = pd.DataFrame(cols)
    out = df.loc[start:end].sub(rf.loc[start:end, "RF"], axis=0)
    out.index.name = "Date"
    return out


def build_all(raw_dir: str, out_dir: str | None = None) -> dict:
    """Run the whole pipeline on a reference-layout ``data/`` directory."""
    rf = build_rf(os.path.join(raw_dir, "F-F_Research_Data_Factors_daily.CSV"))
    hfd = build_hfd(os.path.join(raw_dir, "NAVROR_full.csv"), rf)
    etf = build_factor_etf(os.path.join(raw_dir, "ETF_data.csv"), rf)
    res = {"rf": rf, "hfd": hfd, "factor_etf_data": etf}
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        for k, v in res.items():
            v.to_csv(os.path.join(out_dir, f"{k}.csv"))
    return res


def fama_french_monthly(ff_daily_csv: str, cols=("Mkt-RF", "SMB", "HML"), start: str = START,
                        end: str = END) -> pd.DataFrame:
    """Notebook cell 21/22 (autoencoder_v4.ipynb:645-651): daily % -> monthly sum -> log(x/100+1)."""
    ff = pd.read_csv(ff_daily_csv, usecols=["Date", *cols])
    ff["Date"] = pd.to_datetime(ff["Date"].astype(str), format="%Y%m%d")
    m = ff.set_index("Date").groupby(pd.Grouper(freq="ME")).sum()
    m = np.log(m / 100.0 + 1.0)
    m.index = _month_end_index(m.index)
    return m.loc[start:end]
