"""Observatory clock corrections from TEMPO2-format clock files (optional):
observatory/clock_file.py:432-546 read_tempo2_clock_file and :143-188 ClockFile.evaluate
(linear interpolation in MJD, the end values beyond the ends with a warning).  A site's
corrections are the sum over its files (topo_obs.py clock_corrections without the GPS/BIPM
files, which are not bundled)."""
from __future__ import annotations

import re
import warnings
from functools import lru_cache
from typing import Dict, Sequence, Union

import numpy as np

from .observatory import get_observatory_name

_HDR = re.compile(r"#\s*(\S+)\s+(\S+)\s+(\d+)?(.*)")
_NUM = r"[-+]?(?:\d+(?:\.\d*)?|\.\d+)(?:[eEdD][-+]?\d+)?"
_ROW = re.compile(rf"\s*({_NUM})\s+({_NUM}) ?(.*)")


@lru_cache(maxsize=64)
def read_tempo2_clock_file(path: str, bogus_last_correction: bool = False):
    """(mjd [float], correction [s]) of a TEMPO2 clock file: the first line is the header
    (``# FROM TO [badness]``); '#' lines and lines that are not two numbers are comments;
    leading MJD-0 rows are dropped."""
    mjd, clk = [], []
    with open(path) as f:
        hdr = None
        for line in f:
            if hdr is None:
                if not _HDR.match(line):
                    raise ValueError(f"Header line must start with # and contain two time scales: {line!r}")
                hdr = line
                continue
            if line.startswith("#"):
                continue
            m = _ROW.match(line)
            if m is None:
                continue
            mjd.append(float(m.group(1).translate(str.maketrans("dD", "ee"))))
            clk.append(float(m.group(2).translate(str.maketrans("dD", "ee"))))
    if bogus_last_correction and mjd:
        mjd, clk = mjd[:-1], clk[:-1]
    while mjd and mjd[0] == 0:
        mjd, clk = mjd[1:], clk[1:]
    return np.array(mjd, dtype=np.float64), np.array(clk, dtype=np.float64)


def evaluate(path: str, mjd: np.ndarray, limits: str = "warn") -> np.ndarray:
    """ClockFile.evaluate (s)."""
    t, c = read_tempo2_clock_file(str(path))
    mjd = np.asarray(mjd, dtype=np.float64)
    if len(t) == 0:
        if limits == "error":
            raise ValueError(f"No data points in clock file '{path}'")
        warnings.warn(f"No data points in clock file '{path}'")
        return np.zeros_like(mjd)
    if np.any(mjd < t[0]) or np.any(mjd > t[-1]):
        if limits == "error":
            raise ValueError(f"Data points out of range in clock file '{path}'")
        warnings.warn(f"Data points out of range in clock file '{path}'")
    return np.interp(mjd, t, c)


def site_corrections(clock_files: Dict[str, Union[str, Sequence[str]]], obs: Sequence[str],
                     mjd: np.ndarray) -> np.ndarray:
    """Per-TOA clock correction (s): for each TOA, the sum of its site's files at its MJD."""
    obs = np.asarray(obs, dtype=object)
    out = np.zeros(len(obs))
    canon = {get_observatory_name(k): (v if isinstance(v, (list, tuple)) else [v]) for k, v in clock_files.items()}
    for site, files in canon.items():
        g = np.nonzero(obs == site)[0]
        for path in files:
            out[g] += evaluate(path, np.asarray(mjd)[g])
    return out
