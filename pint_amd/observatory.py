"""Observatory names (observatory/__init__.py get_observatory, observatory/topo_obs.py,
special_locations.py:277-303): canonical site name of a code or alias, case-insensitive, from
the site table pint_amd/data/observatories.json (oracle/refgen/gen_observatories.py)."""
from __future__ import annotations

import json
import os
from functools import lru_cache
from typing import Dict

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "observatories.json")


@lru_cache(maxsize=1)
def sites() -> Dict[str, dict]:
    with open(_DATA) as f:
        return json.load(f)


@lru_cache(maxsize=1)
def _alias_map() -> Dict[str, str]:
    m = {}
    for name, v in sites().items():
        m[name.lower()] = name
        for a in v.get("aliases") or []:
            m.setdefault(str(a).lower(), name)
    return m


def get_observatory_name(code) -> str:
    """get_observatory(code).name (parameter.py:79-91 _get_observatory_name)."""
    key = str(code).lower()
    try:
        return _alias_map()[key]
    except KeyError:
        raise KeyError(f"Observatory name '{code}' is not defined") from None
