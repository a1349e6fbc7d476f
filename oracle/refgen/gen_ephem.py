"""Compact Earth/Sun ephemeris table for the synthetic TOA generator (container only).

Samples the reference's offline ephemeris ("builtin" = erfa epv00, the ephemeris the
oracle recipe uses, solar_system_ephemerides.py objPosVel_wrt_SSB) daily over MJD
52900-58700 (TDB): Earth SSB position/velocity and Sun SSB position, in km and km/s.
The GPU box has no astropy/erfa, so pint_amd.simulation interpolates this table (cubic
Hermite) to place geocentric synthetic TOAs.  This is input-generation data, not an
oracle output.
"""
import os
import numpy as np
import erfa

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
AU_KM = 149597870.7
DAYSEC = 86400.0

mjd = np.arange(52900.0, 58701.0, 1.0)
jd1 = np.full_like(mjd, 2400000.5)
pvh, pvb = erfa.epv00(jd1, mjd)  # AU, AU/day; heliocentric and barycentric Earth
earth_pos = pvb["p"] * AU_KM
earth_vel = pvb["v"] * AU_KM / DAYSEC
sun_pos = (pvb["p"] - pvh["p"]) * AU_KM
out = os.path.join(REPO, "pint_amd", "data", "earth_ephem.npz")
os.makedirs(os.path.dirname(out), exist_ok=True)
np.savez_compressed(out, mjd=mjd, earth_pos_km=earth_pos, earth_vel_kms=earth_vel, sun_pos_km=sun_pos,
                    source=np.array("erfa.epv00 (astropy builtin ephemeris), TDB days, km, km/s"))
print("wrote", out, os.path.getsize(out))
