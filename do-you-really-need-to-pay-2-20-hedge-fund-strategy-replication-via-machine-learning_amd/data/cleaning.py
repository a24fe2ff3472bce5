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


def build_rf_daily(ff_daily_csv: str) -> pd.Series:
    """Daily log risk-free rate log(1 + RF / 100) on the Fama-French trading days."""
    ff = pd.read_csv(ff_daily_csv, usecols=["Date", "RF"])
    idx = pd.to_datetime(ff["Date"].astype(str), format="%Y%m%d")
    return pd.Series(np.log1p(ff["RF"].to_numpy(np.float64) / 100.0), index=pd.DatetimeIndex(idx), name="RF")


def build_factor_etf_daily(etf_csv: str, ff_daily_csv: str, tickers=REPRODUCIBLE_ETF, overrides: dict | None = None,
                           start: str = START, end: str = END):
    """DAILY excess log returns of the ETF / index factors (BASELINE config 2: the factor autoencoder on a
    daily ETF-return matrix).  Returns ``(excess, rf_daily)`` on one calendar.

    The calendar is every Fama-French trading day plus every day any selected index has a price, from
    the first day of ``start``'s month to ``end``.  For each index, L(d) = log of its last price on or
    before d, and the day's return is L(d) - L(previous calendar day); the first day's return is taken
    from the last price before the window (the month-end the monthly panel's first return starts from).
    An index without a price that day returns 0 and its next price carries the whole move, so the
    returns of a month always sum to log(P_last(m) / P_last(m - 1)), the monthly panel's price relative
    (``aggregate_daily_to_monthly`` reproduces ``factor_etf_data``; tests/test_data.py).  ``rf_daily`` =
    log(1 + RF / 100) on Fama-French days, 0 on the others.  Default tickers: the 14 columns the shipped
    raw prices reproduce."""
    prices = read_etf_prices(etf_csv)
    if overrides:
        prices.update(overrides)
    rf = build_rf_daily(ff_daily_csv)
    lo = pd.Timestamp(start).to_period("M").to_timestamp(how="start")
    hi = pd.Timestamp(end)
    days = set(rf.loc[lo:hi].index)
    logp = {}
    for t in tickers:
        if t not in prices:
            continue
        s = prices[t]
        s = s[~s.index.duplicated(keep="last")].sort_index()
        s = s[s > 0]
        logp[t] = np.log(s.astype(np.float64))
        days |= set(s.loc[lo:hi].index)
    cal = pd.DatetimeIndex(sorted(days))
    cols = {}
    for t, lp in logp.items():
        before = lp[lp.index < lo]
        if before.empty:
            continue
        L = lp.reindex(lp.index.union(cal)).ffill().reindex(cal)
        rel = L.diff()
        rel.iloc[0] = L.iloc[0] - before.iloc[-1]
        cols[t] = rel
    rf_cal = rf.reindex(cal).fillna(0.0)
    excess = pd.DataFrame(cols, index=cal).sub(rf_cal, axis=0)
    excess.index.name = "Date"
    rf_cal.index.name = "Date"
    return excess, rf_cal


def aggregate_daily_to_monthly(excess: pd.DataFrame, rf_daily: pd.Series, rf_monthly: pd.DataFrame) -> pd.DataFrame:
    """Monthly excess log returns from the daily panel: sum the day's price relatives (excess + daily rf)
    over each month, minus the monthly rf of ``build_rf`` -- the construction of ``factor_etf_data``."""
    rel = excess.add(rf_daily, axis=0)
    m = rel.groupby(rel.index.to_period("M")).sum()
    m.index = m.index.to_timestamp(how="end").normalize()
    out = m.reindex(rf_monthly.index).sub(rf_monthly["RF"], axis=0)
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
