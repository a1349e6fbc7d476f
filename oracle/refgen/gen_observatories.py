"""Site table for pint_amd (data, not code): names, aliases and ITRF positions of the
reference's observatory registry (observatories.json, observatory/special_locations.py:277-303).
Container only: writes pint_amd/data/observatories.json.  Usage: python3 gen_observatories.py"""
import json
import os

SRC = "/root/reference/src/pint/data/runtime/observatories.json"
OUT = os.path.join(os.path.dirname(__file__), "..", "..", "pint_amd", "data", "observatories.json")


def main():
    d = json.load(open(SRC))
    out = {}
    for name, v in d.items():
        al = [a for a in v.get("aliases", [])]
        for k in ("tempo_code", "itoa_code"):
            if v.get(k):
                al.append(v[k])
        out[name] = {"aliases": al, "itrf_xyz": v.get("itrf_xyz"), "special": None}
    # special locations (special_locations.py:277-303)
    out["barycenter"] = {"aliases": ["@", "ssb", "bary", "bat"], "itrf_xyz": None, "special": "barycenter"}
    out["geocenter"] = {"aliases": ["0", "o", "coe", "geo", "geo_nogps"], "itrf_xyz": None, "special": "geocenter"}
    out["geocenter_gps"] = {"aliases": ["geo_gps", "coe_gps"], "itrf_xyz": None, "special": "geocenter"}
    out["stl_geo"] = {"aliases": ["STL_GEO", "spacecraft"], "itrf_xyz": None, "special": "spacecraft"}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(len(out), "sites")


if __name__ == "__main__":
    main()
