"""tim-file reader: the reference's read_toa_file / _parse_TOA_line
(toa.py:441-858) -- Tempo2 ("FORMAT 1"), Princeton and Parkes lines, comments, and the
commands TIME, PHASE, EFAC, EQUAD, EMIN, EMAX, FMIN, FMAX, JUMP, SKIP/NOSKIP, INFO, INCLUDE,
MODE, FORMAT, END, with the reference's semantics (a command persists until changed, an
INCLUDEd file starts in "Unknown" format and inherits the other settings, EFAC/EQUAD
commands rescale the TOA error as it is read, JUMP blocks become -jump/-tim_jump flags,
TIME/PHASE become -to/-phase flags).

Each TOA is returned as a plain record: (imjd, fmjd) with the fraction as a float64 (the
reference parses "0.<digits>" with float(), toa.py:504-510), error (us), frequency (MHz;
0 -> inf), canonical site name, and its flag dict (strings, insertion ordered, including
the reference's implicit "format"/"name"/"ddm" entries).
"""
from __future__ import annotations

import gzip
import io
import os
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from .observatory import get_observatory_name

# toa.py:68-94
COMMANDS = ("DITHER", "EFAC", "EMAX", "EMAP", "EMIN", "EQUAD", "FMAX", "FMIN", "INCLUDE", "INFO", "JUMP",
            "MODE", "NOSKIP", "PHA1", "PHA2", "PHASE", "SEARCH", "SIGMA", "SIM", "SKIP", "TIME", "TRACK",
            "ZAWGT", "FORMAT", "END")
_RESERVED = ("error", "freq", "scale", "MJD", "flags", "obs", "name")


@dataclass
class TimTOA:
    imjd: int
    fmjd: float
    error_us: float
    freq_mhz: float
    obs: str
    flags: Dict[str, str] = field(default_factory=dict)


def line_format(line: str, fmt: str = "Unknown") -> str:
    """_toa_format (toa.py:441-468), the same tests in the same order."""
    if re.match(r"[0-9a-z@] ", line):
        return "Princeton"
    if line.startswith(("C ", "c ", "#", "CC ")):
        return "Comment"
    if line.upper().lstrip().startswith(COMMANDS):
        return "Command"
    if re.match(r"^\s*$", line):
        return "Blank"
    if re.match(r"^ ", line) and len(line) > 41 and line[41] == ".":
        return "Parkes"
    if len(line) > 80 or fmt == "Tempo2":
        return "Tempo2"
    if re.match(r"\S\S", line) and len(line) > 14 and line[14] == ".":
        return "ITOA"
    return "Unknown"


def _mjd_pair(s: str) -> Tuple[int, float]:
    if "." in s:
        ii, ff = s.split(".")
        return int(ii), float(f"0.{ff}")
    return int(s), 0.0


def parse_line(line: str, fmt: str = "Unknown"):
    """_parse_TOA_line (toa.py:471-558): (format, (imjd, fmjd) or None, record dict)."""
    kind = line_format(line, fmt)
    d: Dict[str, object] = {"format": kind}
    mjd = None
    if kind == "Princeton":
        d["obs"] = get_observatory_name(line[0].upper())
        d["freq"] = float(line[15:24])
        d["error"] = float(line[44:53])
        ii, ff = line[24:44].split(".")
        ii = int(ii)
        if ii < 40000:  # very old TOAs (tempo convention)
            ii += 39126
        mjd = (ii, float(f"0.{ff}"))
        try:
            d["ddm"] = str(float(line[68:78]))
        except ValueError:
            d["ddm"] = str(0.0)
    elif kind == "Tempo2":
        fields = line.split()
        d["name"] = fields[0]
        d["freq"] = float(fields[1])
        mjd = _mjd_pair(fields[2])
        d["error"] = float(fields[3])
        d["obs"] = get_observatory_name(fields[4].upper())
        rest = fields[5:]
        if len(rest) % 2:
            raise ValueError(f"Flags and flag-values should be given in pairs. The given flags are {' '.join(rest)}")
        for k, v in zip(rest[::2], rest[1::2]):
            key = k.lstrip("-")
            if key in _RESERVED:
                raise ValueError(f"TOA flag ({key}) will overwrite TOA parameter!")
            if not key:
                raise ValueError(f"The string {k!r} is not a valid flag")
            d[key] = v
    elif kind == "Command":
        d["Command"] = line.split()
    elif kind == "Parkes":
        d["name"] = line[1:25]
        d["freq"] = float(line[25:34])
        mjd = (int(line[34:41]), float(f"0.{line[42:55]}"))
        if float(line[55:62]) != 0:
            raise ValueError(f"Cannot interpret Parkes format with phaseoffset={float(line[55:62])} yet")
        d["error"] = float(line[63:71])
        d["obs"] = get_observatory_name(line[79].upper())
    elif kind == "ITOA":
        raise RuntimeError("TOA format 'ITOA' not implemented yet")
    elif kind not in ("Blank", "Comment"):
        raise RuntimeError(f"Unable to identify TOA format for line {line!r}, expecting {fmt}")
    return kind, mjd, d


def _new_state():
    return {"EFAC": 1.0, "EQUAD": 0.0, "EMIN": 0.0, "EMAX": np.inf, "FMIN": 0.0, "FMAX": np.inf, "INFO": None,
            "SKIP": False, "TIME": 0.0, "PHASE": 0.0, "PHA1": None, "PHA2": None, "MODE": 1, "JUMP": [False, 0],
            "FORMAT": "Unknown", "END": False}


def _open(path_or_file):
    if hasattr(path_or_file, "readlines"):
        return path_or_file, False
    p = str(path_or_file)
    if p.endswith(".gz"):
        return io.TextIOWrapper(gzip.open(p, "rb")), True
    return open(p, "r"), True


def read_tim(path_or_file, process_includes: bool = True, _state=None, _dir=None):
    """read_toa_file (toa.py:700-858): (list of TimTOA, commands [(fields, ntoas_before)])."""
    top = _state is None
    st = _new_state() if top else _state
    if _dir is None:
        _dir = os.path.dirname(str(path_or_file)) if not hasattr(path_or_file, "readlines") else "."
    f, close = _open(path_or_file)
    toas: List[TimTOA] = []
    commands = []
    try:
        lines = f.readlines()
    finally:
        if close:
            f.close()
    for line in lines:
        kind, mjd, d = parse_line(line, st["FORMAT"])
        if kind == "Command":
            cmdf = d["Command"]
            cmd = cmdf[0].upper()
            commands.append((cmdf, len(toas)))
            if cmd == "SKIP":
                st["SKIP"] = True
                continue
            if cmd == "NOSKIP":
                st["SKIP"] = False
                continue
            if cmd == "END":
                st["END"] = True
                break
            if cmd in ("TIME", "PHASE"):
                st[cmd] += float(cmdf[1])
            elif cmd in ("EMIN", "EMAX", "EQUAD"):
                st[cmd] = float(cmdf[1])  # us
            elif cmd in ("FMIN", "FMAX"):
                st[cmd] = float(cmdf[1])  # MHz
            elif cmd in ("EFAC", "PHA1", "PHA2"):
                st[cmd] = float(cmdf[1])
                if cmd in ("PHA1", "PHA2"):
                    d[cmd] = cmdf[1]
            elif cmd == "INFO":
                st[cmd] = cmdf[1]
            elif cmd == "FORMAT":
                if cmdf[1] == "1":
                    st[cmd] = "Tempo2"
            elif cmd == "JUMP":
                if st["JUMP"][0]:
                    st["JUMP"][0] = False
                    st["JUMP"][1] += 1
                else:
                    st["JUMP"][0] = True
            elif cmd == "INCLUDE" and process_includes:
                fmt = st["FORMAT"]
                st["FORMAT"] = "Unknown"
                inc = os.path.join(_dir, cmdf[1])
                cmdf[1] = inc
                more, more_cmds = read_tim(inc, process_includes, st, os.path.dirname(inc))
                toas.extend(more)
                commands.extend(more_cmds)
                st["FORMAT"] = fmt
            # MODE and unknown commands: ignored (the reference only warns)
            continue
        if st["SKIP"] or kind in ("Blank", "Unknown", "Comment"):
            continue
        if st["END"]:
            if top:
                break
            continue
        err = float(d.pop("error"))
        freq = float(d.pop("freq"))
        obs = d.pop("obs")
        if freq == 0.0:
            freq = np.inf
        if st["EMIN"] > err or st["EMAX"] < err or st["FMIN"] > freq or st["FMAX"] < freq:
            continue
        err = float(np.hypot(err * st["EFAC"], st["EQUAD"]))
        flags = {k: str(v) for k, v in d.items()}
        if st["INFO"]:
            flags["info"] = st["INFO"]
        if st["JUMP"][0]:
            flags["jump"] = str(st["JUMP"][1] + 1)
            flags["tim_jump"] = str(st["JUMP"][1] + 1)
        if st["PHASE"] != 0:
            flags["phase"] = str(st["PHASE"])
        if st["TIME"] != 0.0:
            flags["to"] = str(st["TIME"])
        toas.append(TimTOA(mjd[0], mjd[1], err, freq, obs, flags))
    return toas, commands
