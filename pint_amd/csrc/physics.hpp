// physics.hpp — per-TOA timing-model evaluation for gfx950: delays, pulse phase (dd) and
// every design-matrix column, restated from the reference formulas (cited per function).
// One thread evaluates one TOA; parameters are wave-uniform (scalar loads).
#pragma once
#include "dd.hpp"
#include "../../include/pint_amd.h"

namespace pint {

// ---- constants (values as the reference's astropy/erfa constants; see
//      tests/golden/... constants and pint/__init__.py:67-102) ----------------------------
constexpr double C_KMS = 299792.458;              // c, km/s
constexpr double AU_KM = 149597870.7;             // astropy au
constexpr double KPC_KM = 3.0856775814913674e16;  // 1 kpc in km
constexpr double TSUN = 4.92549094830932e-06;     // GM_sun/c^3 (s), pint/__init__.py:80
// GM/c^3 of jupiter, saturn, venus, uranus, neptune: Tsun / (M_sun / M_planet) rounded once,
// as pint/__init__.py:84-90 forms them
__device__ __constant__ const double TPLANET[5] = {TSUN / 1047.3486, TSUN / 3497.898, TSUN / 408523.71, TSUN / 22902.98,
                               TSUN / 19412.24};
constexpr double DMCONST = 4149.377593360996;     // 1/2.41e-4 MHz^2 s cm^3/pc, :68
constexpr double DAYSEC = 86400.0;
constexpr double DJY = 365.25;
constexpr double ERFA_DC = 173.1446326742403;     // c in AU/day (erfa DC)
constexpr double DR2AS = 206264.80624709636;
constexpr double MAS_RAD = 4.84813681109536e-09;
constexpr double HA_RAD = 0.2617993877991494;
constexpr double DEG_RAD = 0.017453292519943295;
constexpr double MASYR_RADS = 1.5362818500441604e-16;  // (mas/yr) in rad/s
constexpr double YR_S = 31557600.0;
constexpr double TWO_PI = 6.283185307179586;
constexpr double PI_D = 3.141592653589793;
// reciprocals of the constants divided by per TOA (x / c -> x * (1/c): <= 1 ulp)
constexpr double INV_C_KMS = 1.0 / C_KMS;
constexpr double INV_AU_KM = 1.0 / AU_KM;
constexpr double INV_AUC = 1.0 / (AU_KM * C_KMS);
constexpr double INV_KPC_KM = 1.0 / KPC_KM;
constexpr double INV_DJY = 1.0 / DJY;
constexpr double INV_TWO_PI = 1.0 / TWO_PI;
// 1/k as double-double (hi correctly rounded, lo = 1/k - hi), k < 64: the Taylor-series
// divisions by small integers become multiplications (exact to ~1e-32 relative)
constexpr int NINV = 64;
__device__ __constant__ const double INV_HI[NINV] = {0.0, 1.0, 0.5, 0.3333333333333333, 0.25, 0.2, 0.16666666666666666, 0.14285714285714285, 0.125, 0.1111111111111111, 0.1, 0.09090909090909091, 0.08333333333333333, 0.07692307692307693, 0.07142857142857142, 0.06666666666666667, 0.0625, 0.058823529411764705, 0.05555555555555555, 0.05263157894736842, 0.05, 0.047619047619047616, 0.045454545454545456, 0.043478260869565216, 0.041666666666666664, 0.04, 0.038461538461538464, 0.037037037037037035, 0.03571428571428571, 0.034482758620689655, 0.03333333333333333, 0.03225806451612903, 0.03125, 0.030303030303030304, 0.029411764705882353, 0.02857142857142857, 0.027777777777777776, 0.02702702702702703, 0.02631578947368421, 0.02564102564102564, 0.025, 0.024390243902439025, 0.023809523809523808, 0.023255813953488372, 0.022727272727272728, 0.022222222222222223, 0.021739130434782608, 0.02127659574468085, 0.020833333333333332, 0.02040816326530612, 0.02, 0.0196078431372549, 0.019230769230769232, 0.018867924528301886, 0.018518518518518517, 0.01818181818181818, 0.017857142857142856, 0.017543859649122806, 0.017241379310344827, 0.01694915254237288, 0.016666666666666666, 0.01639344262295082, 0.016129032258064516, 0.015873015873015872};
__device__ __constant__ const double INV_LO[NINV] = {0.0, 0.0, 0.0, 1.850371707708594e-17, 0.0, -1.1102230246251566e-17, 9.25185853854297e-18, 7.93016446160826e-18, 0.0, 6.1679056923619804e-18, -5.551115123125783e-18, -2.523234146875356e-18, 4.625929269271485e-18, -4.270088556250602e-18, 3.96508223080413e-18, 9.251858538542971e-19, 0.0, 8.163404592832033e-19, 3.0839528461809902e-18, 2.921639538487254e-18, -2.7755575615628915e-18, 2.64338815386942e-18, -1.261617073437678e-18, 1.206764157201257e-18, 2.3129646346357427e-18, -8.326672684688674e-19, -2.135044278125301e-18, 2.05596856412066e-18, 1.982541115402065e-18, 4.785444071660157e-19, 4.625929269271486e-19, 8.953411488912552e-19, 0.0, -8.410780489584519e-19, 4.0817022964160166e-19, 8.921435019309293e-19, 1.5419764230904951e-18, -1.50030138462859e-18, 1.460819769243627e-18, 8.896017825522087e-19, -1.3877787807814458e-18, -8.46206573647223e-19, 1.32169407693471e-18, 3.2273925134452225e-19, -6.30808536718839e-19, -8.480870326997723e-19, 6.033820786006285e-19, 5.167261417803255e-19, 1.1564823173178713e-18, 1.6285159162231251e-18, -4.163336342344337e-19, 2.7211348642773444e-19, -1.0675221390626506e-18, 7.20073895688486e-19, 1.02798428206033e-18, 8.831319514063744e-19, 9.912705577010326e-19, 9.73879846162418e-19, 2.3927220358300787e-19, 5.880418562633244e-20, 2.312964634635743e-19, -8.531426931033477e-19, 4.476705744456276e-19, 8.8112938462314e-19};
PD double inv_int(int k) { return k < NINV ? INV_HI[k] : 1.0 / (double)k; }
PD dd dd_div_int(dd a, int k) { return k < NINV ? dd_mul(a, dd_make(INV_HI[k], INV_LO[k])) : dd_div_d(a, (double)k); }

PD double pval(const double* P, int o) { return P[o] + P[o + 1]; }
PD dd pdd(const double* P, int o) { return dd_make(P[o], P[o + 1]); }

// ------------------------------------------------------------------------------------
// erfa pmsafe/starpm/starpv restated (SOFA published algorithm; pyerfa 2.0.0 is the
// reference's third-party call at astrometry.py:513 and astropy apply_space_motion).
// Split in two: pm_setup() is everything that does not depend on the epoch (pmsafe's
// parallax override, starpv with its relativistic iteration) and runs once per instance
// (k_prep); pm_dir() is starpm's propagation to one TOA's epoch.
// ------------------------------------------------------------------------------------
struct PmState {
    double p[3], v1[3], tl1;
};

// the trigonometric values pm_setup starts from: cos/sin of ra, dec, ra2 = ra + pmr and
// dec2 = dec + pmd (independent: k_prep forms them on separate lanes, pm_setup_trig)
struct PmTrig {
    double cra, sra, cdec, sdec, cra2, sra2, cdec2, sdec2;
};

PD void pm_setup_trig(double pmr, double pmd, double px, const PmTrig& T, PmState& st);

PD void pm_setup(double ra, double dec, double pmr, double pmd, double px, PmState& st) {
    const double ra2 = ra + pmr, dec2 = dec + pmd;
    const PmTrig T = {cos(ra), sin(ra), cos(dec), sin(dec), cos(ra2), sin(ra2), cos(dec2), sin(dec2)};
    pm_setup_trig(pmr, pmd, px, T, st);
}

PD void pm_setup_trig(double pmr, double pmd, double px, const PmTrig& T, PmState& st) {
    // pmsafe: override parallax (PXMIN 5e-7 arcsec, F = 326)
    double a1[3] = {T.cra * T.cdec, T.sra * T.cdec, T.sdec};
    double b1[3] = {T.cra2 * T.cdec2, T.sra2 * T.cdec2, T.sdec2};
    double cx = a1[1] * b1[2] - a1[2] * b1[1];
    double cy = a1[2] * b1[0] - a1[0] * b1[2];
    double cz = a1[0] * b1[1] - a1[1] * b1[0];
    double ss = sqrt(cx * cx + cy * cy + cz * cz);
    double cs = a1[0] * b1[0] + a1[1] * b1[1] + a1[2] * b1[2];
    double px1a = px;
    // the separation pm = atan2(ss, cs) only enters as max(px, 326 pm); with cs > 0,
    // atan2(ss, cs) = atan(ss / cs) <= ss / cs, so when 326 ss / cs (with a rounding margin)
    // stays below px the override cannot apply and the atan2 chain is skipped
    if ((ss != 0.0 || cs != 0.0) && !(cs > 0.0 && 326.0 * (ss / cs) * (1.0 + 1e-12) < px1a)) {
        const double pm = 326.0 * atan2(ss, cs);
        if (px1a < pm) px1a = pm;
    }
    if (px1a < 5e-7) px1a = 5e-7;
    // starpv (rv = 0)
    double w = px1a >= 1e-7 ? px1a : 1e-7;
    double r = DR2AS / w;
    double rad = pmr / DJY, decd = pmd / DJY;
    double st_ = T.sra, ct = T.cra, sp = T.sdec, cp = T.cdec;
    double rcp = r * cp;
    double x = rcp * ct, y = rcp * st_;
    double rpd = r * decd;
    double ww = rpd * sp;  // - cp*rd with rd = 0
    double p[3] = {x, y, r * sp};
    double v[3] = {-y * rad - ww * ct, x * rad - ww * st_, rpd * cp};
    double vm = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (vm / ERFA_DC > 0.5) { v[0] = v[1] = v[2] = 0.0; }
    double pm_ = sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
    double xu[3] = {p[0] / pm_, p[1] / pm_, p[2] / pm_};
    double vsr = xu[0] * v[0] + xu[1] * v[1] + xu[2] * v[2];
    double usr[3] = {vsr * xu[0], vsr * xu[1], vsr * xu[2]};
    double ust[3] = {v[0] - usr[0], v[1] - usr[1], v[2] - usr[2]};
    double vst = sqrt(ust[0] * ust[0] + ust[1] * ust[1] + ust[2] * ust[2]);
    double betsr = vsr / ERFA_DC, betst = vst / ERFA_DC;
    double bett = betst, betr = betsr, d = 1.0, del = 0.0, od = 0.0, odel = 0.0, odd = 0.0, oddel = 0.0;
    for (int i = 0; i < 100; i++) {
        d = 1.0 + betr;
        double w2 = betr * betr + bett * bett;
        del = -w2 / (sqrt(1.0 - w2) + 1.0);
        betr = d * betsr + del;
        bett = d * betst;
        if (i > 0) {
            double dd_ = fabs(d - od), ddel = fabs(del - odel);
            if (i > 1 && dd_ >= odd && ddel >= oddel) break;
            odd = dd_;
            oddel = ddel;
        }
        od = d;
        odel = del;
    }
    double wr = (betsr != 0.0) ? d + del / betsr : 1.0;
    for (int k = 0; k < 3; k++) {
        st.p[k] = p[k];
        st.v1[k] = wr * usr[k] + d * ust[k];
    }
    st.tl1 = pm_ / ERFA_DC;
}

// starpm's propagation to dt_days, then pvstar -> (ra, dec) -> xyz_from_radec
// (astrometry.py:530), i.e. the unit vector of the propagated position.
PD void pm_dir(const PmState& st, double dt_days, double out[3]) {
    const double* p = st.p;
    const double* v1 = st.v1;
    const double tl1 = st.tl1;
    double q[3] = {p[0] + (dt_days + tl1) * v1[0], p[1] + (dt_days + tl1) * v1[1], p[2] + (dt_days + tl1) * v1[2]};
    double r2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2];
    double rdv = q[0] * v1[0] + q[1] * v1[1] + q[2] * v1[2];
    double v2 = v1[0] * v1[0] + v1[1] * v1[1] + v1[2] * v1[2];
    double c2mv2 = ERFA_DC * ERFA_DC - v2;
    double tl2 = (-rdv + sqrt(rdv * rdv + c2mv2 * r2)) / c2mv2;
    double s = dt_days + (tl1 - tl2);
    double p2[3] = {p[0] + s * v1[0], p[1] + s * v1[1], p[2] + s * v1[2]};
    double in = 1.0 / sqrt(p2[0] * p2[0] + p2[1] * p2[1] + p2[2] * p2[2]);
    out[0] = p2[0] * in;
    out[1] = p2[1] * in;
    out[2] = p2[2] * in;
}

// Ecliptic -> ICRS rotation (pulsar_ecliptic.py:70: rotation_matrix(obl, "x") is ICRS->ECL)
PD void ecl_to_icrs(double obl, const double e[3], double o[3]) {
    double c = cos(obl), s = sin(obl);
    o[0] = e[0];
    o[1] = c * e[1] - s * e[2];
    o[2] = s * e[1] + c * e[2];
}
PD void icrs_to_ecl(double obl, const double e[3], double o[3]) {
    double c = cos(obl), s = sin(obl);
    o[0] = e[0];
    o[1] = c * e[1] + s * e[2];
    o[2] = -s * e[1] + c * e[2];
}

// Per-instance constants of the astrometry (computed once by k_prep): the pulsar
// direction without proper motion, or the starpm state, and the position angles used by
// the design-matrix columns.  astrometry.py:469-528 AstrometryEquatorial.ssb_to_psb_xyz_ICRS;
// :71 base path + SkyCoord apply_space_motion for ecliptic models (sky_coordinate.py
// apply_space_motion -> erfa.pmsafe, 1-kpc dummy distance utils.py:2171).
struct InstConst {
    PmState pm;
    double L0[3];
    double posep;        // POSEPOCH (MJD) or 0
    double plon, plat;   // rad (RAJ in hourangle, ELONG/ELAT/DECJ in deg -> rad)
    double cplat, splat;
    double cplon, splon;
    double F0, iF0;
    double ipb_hi, ipb_lo;  // 1/(PB in s) in dd (binary models)
    int has_pm;
    int pad_;
};

PD void inst_setup(const pint_spec_t& S, const double* P, InstConst& C) {
    C.F0 = pval(P, S.o_F);
    C.iF0 = 1.0 / C.F0;
    C.has_pm = 0;
    C.L0[0] = 0.0; C.L0[1] = 0.0; C.L0[2] = 1.0;
    C.posep = S.o_POSEPOCH >= 0 ? pval(P, S.o_POSEPOCH) : 0.0;
    C.plon = C.plat = C.cplat = C.splat = 0.0;
    C.cplon = 1.0;
    C.splon = 0.0;
    C.ipb_hi = C.ipb_lo = 0.0;
    if (S.binary && S.o_bin[PINT_B_PB] >= 0) {
        dd ipb = dd_div(dd_make(1.0), dd_mul_d(pdd(P, S.o_bin[PINT_B_PB]), DAYSEC));
        C.ipb_hi = ipb.hi;
        C.ipb_lo = ipb.lo;
    }
    if (!S.astrometry) return;
    double lon = pval(P, S.o_lon), lat = pval(P, S.o_lat);
    double pml = S.o_pmlon >= 0 ? pval(P, S.o_pmlon) : 0.0;
    double pmb = S.o_pmlat >= 0 ? pval(P, S.o_pmlat) : 0.0;
    C.plon = lon * (S.astrometry == 1 ? HA_RAD : DEG_RAD);
    C.plat = lat * DEG_RAD;
    C.cplat = cos(C.plat);
    C.splat = sin(C.plat);
    C.cplon = cos(C.plon);
    C.splon = sin(C.plon);
    if (S.astrometry == 1) {
        double ra = lon * HA_RAD, dec = lat * DEG_RAD;
        C.L0[0] = cos(ra) * cos(dec);
        C.L0[1] = sin(ra) * cos(dec);
        C.L0[2] = sin(dec);
        if (pml == 0.0 && pmb == 0.0) return;
        double px_as = (S.o_px >= 0 ? pval(P, S.o_px) : 0.0) * 1e-3;
        pm_setup(ra, dec, pml * MAS_RAD / cos(dec), pmb * MAS_RAD, px_as, C.pm);
        C.has_pm = 1;
        return;
    }
    // ecliptic
    double l = lon * DEG_RAD, b = lat * DEG_RAD;
    double ue[3] = {cos(l) * cos(b), sin(l) * cos(b), sin(b)};
    ecl_to_icrs(S.obliquity, ue, C.L0);
    if (pml == 0.0 && pmb == 0.0) return;
    // tangential velocity (rad/yr at unit distance) in ecliptic, rotated to ICRS
    double el[3] = {-sin(l), cos(l), 0.0};
    double eb[3] = {-sin(b) * cos(l), -sin(b) * sin(l), cos(b)};
    double ve[3];
    for (int k = 0; k < 3; k++) ve[k] = pml * MAS_RAD * el[k] + pmb * MAS_RAD * eb[k];
    double u[3], v[3];
    ecl_to_icrs(S.obliquity, ue, u);
    ecl_to_icrs(S.obliquity, ve, v);
    double ra = atan2(u[1], u[0]);
    double dec = atan2(u[2], sqrt(u[0] * u[0] + u[1] * u[1]));
    double era[3] = {-sin(ra), cos(ra), 0.0};
    double edec[3] = {-sin(dec) * cos(ra), -sin(dec) * sin(ra), cos(dec)};
    double pmra_c = v[0] * era[0] + v[1] * era[1] + v[2] * era[2];
    double pmdec = v[0] * edec[0] + v[1] * edec[1] + v[2] * edec[2];
    pm_setup(ra, dec, pmra_c / cos(dec), pmdec, 1e-3 /* 1 kpc dummy */, C.pm);
    C.has_pm = 1;
}

// inst_setup_wave's operations by one thread, in the same order (so the same values): the
// lane-per-instance k_prep / k_apply of batches of small tables (grid points), where a wave
// sets up 64 instances at once instead of one
PD void inst_setup_seq(const pint_spec_t& S, const double* P, InstConst& C) {
    if (S.astrometry != 1) {
        inst_setup(S, P, C);
        return;
    }
    double sx[12];
    const double lon = pval(P, S.o_lon), lat = pval(P, S.o_lat);
    const double pml = S.o_pmlon >= 0 ? pval(P, S.o_pmlon) : 0.0;
    const double pmb = S.o_pmlat >= 0 ? pval(P, S.o_pmlat) : 0.0;
    const double ra = lon * HA_RAD, dec = lat * DEG_RAD;
    const bool pm = !(pml == 0.0 && pmb == 0.0);
    const double pmd = pmb * MAS_RAD;
    sx[0] = cos(ra);
    sx[1] = sin(ra);
    sx[2] = cos(dec);
    sx[3] = sin(dec);
    if (pm) {
        sx[10] = cos(dec + pmd);
        sx[11] = sin(dec + pmd);
    }
    if (S.binary && S.o_bin[PINT_B_PB] >= 0) {
        dd ipb = dd_div(dd_make(1.0), dd_mul_d(pdd(P, S.o_bin[PINT_B_PB]), DAYSEC));
        sx[4] = ipb.hi;
        sx[5] = ipb.lo;
    }
    const double cd = sx[2];
    const double pmr = pml * MAS_RAD / cd;
    if (pm) {
        const double ra2 = ra + pmr, d = ra2 - ra;
        if (fabs(d) < 1e-2) {
            const double d2 = d * d;
            const double sd = d * (1.0 - d2 * (1.0 / 6.0 - d2 * (1.0 / 120.0 - d2 * (1.0 / 5040.0))));
            const double cdl = 1.0 - d2 * (0.5 - d2 * (1.0 / 24.0 - d2 * (1.0 / 720.0 - d2 * (1.0 / 40320.0))));
            sx[8] = sx[0] * cdl - sx[1] * sd;
            sx[9] = sx[1] * cdl + sx[0] * sd;
        } else {
            sx[8] = cos(ra2);
            sx[9] = sin(ra2);
        }
    }
    C.F0 = pval(P, S.o_F);
    C.iF0 = 1.0 / C.F0;
    C.has_pm = 0;
    C.posep = S.o_POSEPOCH >= 0 ? pval(P, S.o_POSEPOCH) : 0.0;
    C.ipb_hi = C.ipb_lo = 0.0;
    if (S.binary && S.o_bin[PINT_B_PB] >= 0) {
        C.ipb_hi = sx[4];
        C.ipb_lo = sx[5];
    }
    C.plon = ra;
    C.plat = dec;
    C.cplat = sx[2];
    C.splat = sx[3];
    C.cplon = sx[0];
    C.splon = sx[1];
    C.L0[0] = sx[0] * sx[2];
    C.L0[1] = sx[1] * sx[2];
    C.L0[2] = sx[3];
    if (!pm) return;
    const double px_as = (S.o_px >= 0 ? pval(P, S.o_px) : 0.0) * 1e-3;
    const PmTrig T = {sx[0], sx[1], sx[2], sx[3], sx[8], sx[9], sx[10], sx[11]};
    pm_setup_trig(pmr, pmd, px_as, T, C.pm);
    C.has_pm = 1;
}

// inst_setup by the 64 lanes of one wave (k_prep, k_apply): the equatorial astrometry's
// independent transcendental calls -- cos/sin of RA, DEC and the proper-motion-displaced DEC,
// the double-double 1/PB -- on separate lanes, exchanged through
// `sx` (LDS, >= 8 doubles); lane 0 finishes (pmsafe's atan2, starpv's iteration).  The same
// expressions as inst_setup, so the same values; ecliptic models run inst_setup on lane 0.
// Every lane of the block's first wave must call it (lane = threadIdx.x); C is written by lane 0.
PD void inst_setup_wave(const pint_spec_t& S, const double* P, InstConst& C, double* sx, int lane) {
    if (S.astrometry != 1) {
        if (lane == 0) inst_setup(S, P, C);
        return;
    }
    const double lon = pval(P, S.o_lon), lat = pval(P, S.o_lat);
    const double pml = S.o_pmlon >= 0 ? pval(P, S.o_pmlon) : 0.0;
    const double pmb = S.o_pmlat >= 0 ? pval(P, S.o_pmlat) : 0.0;
    const double ra = lon * HA_RAD, dec = lat * DEG_RAD;
    const bool pm = !(pml == 0.0 && pmb == 0.0);
    const double pmd = pmb * MAS_RAD;
    // one cos and one sin per lane, of a per-lane angle (lane 0: RA, 1: DEC, 2: dec2 = DEC +
    // pmd, which does not depend on the other trig values): the calls are not divergent, so
    // the wave runs each once instead of once per lane's branch
    {
        const double ang = lane == 0 ? ra : (lane == 1 ? dec : dec + pmd);
        const double c = cos(ang), sn = sin(ang);
        if (lane < 2) {
            sx[2 * lane] = c;
            sx[2 * lane + 1] = sn;
        } else if (lane == 2 && pm) {
            sx[10] = c;
            sx[11] = sn;
        }
    }
    if (lane == 3 && S.binary && S.o_bin[PINT_B_PB] >= 0) {
        dd ipb = dd_div(dd_make(1.0), dd_mul_d(pdd(P, S.o_bin[PINT_B_PB]), DAYSEC));
        sx[4] = ipb.hi;
        sx[5] = ipb.lo;
    }
    // the exchange is within wave 0 (lanes 0..3 write, lane 0 reads): a wave-level barrier,
    // so a caller may run it on one wave while the block's other waves do other work
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane != 0) return;
    const double cd = sx[2];
    const double pmr = pml * MAS_RAD / cd;
    if (pm) {
        // cos/sin of ra2 = fl(ra + pmr) by angle addition from ra's: d = ra2 - ra is exact
        // (Sterbenz) and small, its sine and cosine are short Taylor series (a direct sincos
        // would need a second dependent transcendental phase); a large d takes sincos
        const double ra2 = ra + pmr, d = ra2 - ra;
        if (fabs(d) < 1e-2) {
            const double d2 = d * d;
            const double sd = d * (1.0 - d2 * (1.0 / 6.0 - d2 * (1.0 / 120.0 - d2 * (1.0 / 5040.0))));
            const double cdl = 1.0 - d2 * (0.5 - d2 * (1.0 / 24.0 - d2 * (1.0 / 720.0 - d2 * (1.0 / 40320.0))));
            sx[8] = sx[0] * cdl - sx[1] * sd;
            sx[9] = sx[1] * cdl + sx[0] * sd;
        } else {
            sx[8] = cos(ra2);
            sx[9] = sin(ra2);
        }
    }
    C.F0 = pval(P, S.o_F);
    C.iF0 = 1.0 / C.F0;
    C.has_pm = 0;
    C.posep = S.o_POSEPOCH >= 0 ? pval(P, S.o_POSEPOCH) : 0.0;
    C.ipb_hi = C.ipb_lo = 0.0;
    if (S.binary && S.o_bin[PINT_B_PB] >= 0) {
        C.ipb_hi = sx[4];
        C.ipb_lo = sx[5];
    }
    C.plon = ra;  // lon * HA_RAD
    C.plat = dec;
    C.cplat = sx[2];
    C.splat = sx[3];
    C.cplon = sx[0];
    C.splon = sx[1];
    C.L0[0] = sx[0] * sx[2];
    C.L0[1] = sx[1] * sx[2];
    C.L0[2] = sx[3];
    if (!pm) return;
    const double px_as = (S.o_px >= 0 ? pval(P, S.o_px) : 0.0) * 1e-3;
    const PmTrig T = {sx[0], sx[1], sx[2], sx[3], sx[8], sx[9], sx[10], sx[11]};
    pm_setup_trig(pmr, pmd, px_as, T, C.pm);
    C.has_pm = 1;
}

// Unit vector SSB->pulsar (ICRS) at TDB epoch `epoch_mjd`.
PD void psr_dir_icrs(const InstConst& C, double epoch_mjd, double L[3]) {
    if (C.has_pm) {
        pm_dir(C.pm, epoch_mjd - C.posep, L);
    } else {
        L[0] = C.L0[0];
        L[1] = C.L0[1];
        L[2] = C.L0[2];
    }
}

// ------------------------------------------------------------------------------------
// Binary models.  Base quantities are computed once per TOA; d_delay/d(param) per column.
// All derivatives are per SI unit of the parameter (s, rad, rad/s, ...), converted to the
// par-file unit by bin_unit_factor().
// ------------------------------------------------------------------------------------
struct BinState {
    // common
    double tt0;      // s (ttasc for ELL1)
    double orbits_frac, Phi;  // frac(orbits), orbital phase (rad)
    double floor_orbits;
    double PBs, PBDOT, XPBDOT, pb;  // PB (s), pbprime (s)
    double a1, A1DOT, ecc, EDOT;
    double TM2, SINI, GAMMA, DR, DTH, A0, B0;
    // ELL1
    double eps1, eps2, EPS1DOT, EPS2DOT, nhat;
    double R0, R1, R2;  // d_delayR_da1 and Phi derivatives (ELL1_model.py:221-315)
    double Dre, Drep, Drepp;
    // ELL1H (ELL1H_model.py): the H3 Shapiro delay's partials and d(stigma)/d(H3, H4)
    double hS_H3, hS_sig, hS_Phi, dsig_dH3, dsig_dH4;
    // DD
    double E, sinE, cosE, nu, k, omega, OMDOT_rs, er, eTheta, alpha, beta;
    // trigonometry shared by the delay and every derivative column (computed once)
    double s1, c1, s2, c2, s3, c3, s4, c4;                   // ELL1: sin/cos(k Phi)
    double snu, cnu, sw, cw, soPn, coPn, logNum, lgNum, sqTh, sqE;  // DD
    double ipb, iPBs;  // 1/pb (pbprime), 1/PBs
    double iomeE, isnu, ilogNum, isqTh, isqE;  // DD: 1/(1 - e cosE), 1/sin(nu), ...
    // DDK: the Kopeikin terms' d(a1), d(omega) (SI) and prtl_der("SINI", .) per KIN, KOM, T0
    double kA1[3], kOM[3], kSI[3];
    double delay;
    int status;
};

PD double bin_unit_factor(int pid) {
    switch (pid) {
        case PINT_B_PB: case PINT_B_T0: case PINT_B_TASC: return DAYSEC;
        case PINT_B_OM: return DEG_RAD;
        case PINT_B_OMDOT: return DEG_RAD / YR_S;
        case PINT_B_EPS1DOT: case PINT_B_EPS2DOT: return 1e-12;  // units 1e-12/s (binary_ell1.py:142)
        case PINT_B_KIN: case PINT_B_KOM: return DEG_RAD;
        default: return 1.0;
    }
}

PD double binp(const pint_spec_t& S, const double* P, int pid, double dflt = 0.0) {
    int o = S.o_bin[pid];
    return o >= 0 ? pval(P, o) : dflt;
}

// orbits (binary_orbits.py:98 OrbitPB.orbits) in dd; returns frac and floor
PD void orbit_phase(dd tt0, dd ipbs, double pbdot_sum, BinState& B) {
    dd x = dd_mul(tt0, ipbs);  // tt0 / PB with the per-instance dd reciprocal
    double xd = dd_to_d(x);
    dd orb = dd_add_d(x, -0.5 * pbdot_sum * xd * xd);
    dd fl = dd_floor(orb);
    B.floor_orbits = dd_to_d(fl);
    B.orbits_frac = dd_to_d(dd_sub(orb, fl));
    B.Phi = B.orbits_frac * TWO_PI;  // orbit_phase(): (orbits - floor)*2pi (binary_orbits.py:25)
}

// ---- ELL1H Shapiro delay (ELL1H_model.py, Freire & Wex 2010) ------------------------
// binary_ell1.py:383-405 picks the form: S.ell1h 1 = H3 alone (Eq. 19, stigma = 0), 2 = H3 + H4
// (Eq. 19, stigma = H4/H3, harmonics 3..NHARMS), 3 = H3 + STIGMA (the exact Eq. 29).  Eq. 19:
// -2 H3 sum_{k=3}^{N} c_k stigma^(k-3) b_k(k Phi), c_k = (-1)^pwr 2/k, odd k: sin, pwr = (k+1)/2,
// even k: cos, pwr = (k+2)/2 (ELL1H_model.py:90-140); sin/cos(k Phi) by rotation from k = 3.
// Returns the delay; sets its partials in H3, stigma and Phi (:238-330).
PD double ell1h_shapiro(const pint_spec_t& S, const double* P, BinState& B) {
    const double H3 = binp(S, P, PINT_B_H3);
    double sig = 0.0;
    B.dsig_dH3 = 0.0;
    B.dsig_dH4 = 0.0;
    if (S.ell1h == 2) {
        const double H4 = binp(S, P, PINT_B_H4);
        if (H3 != 0.0) {
            const double i3 = 1.0 / H3;
            sig = H4 * i3;
            B.dsig_dH3 = -H4 * i3 * i3;  // d_STIGMA_d_H3 (:283-297)
            B.dsig_dH4 = i3;             // d_STIGMA_d_H4 (:280)
        }
    } else if (S.ell1h == 3) {
        sig = binp(S, P, PINT_B_STIGMA);
    }
    if (S.ell1h == 3) {  // delayS_H3_STIGMA_exact and partials (:300-330)
        const double sP = B.s1, cP = B.c1;
        const double lg = 1.0 + sig * sig - 2.0 * sig * sP, L = log(lg), is = 1.0 / sig, il = 1.0 / lg;
        const double is2 = is * is, is3 = is2 * is;
        B.hS_H3 = -2.0 * is3 * L;
        B.hS_sig = -2.0 * H3 * is3 * is * (-3.0 * L + 2.0 * sig * (sig - sP) * il);
        B.hS_Phi = 4.0 * H3 * is2 * cP * il;
        return H3 * B.hS_H3;
    }
    const int N = S.ell1h == 1 ? 3 : S.nharms;
    const double s1 = B.s1, c1 = B.c1;
    double sk = B.s3, ck = B.c3;  // sin/cos(k Phi) from k = 3
    double pw = 1.0, pwm = 0.0;   // stigma^(k-3), stigma^(k-4)
    double f = 0.0, fs = 0.0, fp = 0.0;
    for (int k = 3; k <= N; k++) {
        const bool odd = k & 1;
        const int pwr = odd ? (k + 1) / 2 : (k + 2) / 2;
        const double c = ((pwr & 1) ? -2.0 : 2.0) / (double)k;
        const double b = odd ? sk : ck;
        const double db = odd ? (double)k * ck : -(double)k * sk;
        f += c * pw * b;
        fp += c * pw * db;
        if (k > 3) fs += c * (double)(k - 3) * pwm * b;
        pwm = pw;
        pw *= sig;
        const double sn = sk * c1 + ck * s1;
        ck = ck * c1 - sk * s1;
        sk = sn;
    }
    B.hS_H3 = -2.0 * f;
    B.hS_sig = -2.0 * H3 * fs;
    B.hS_Phi = -2.0 * H3 * fp;
    return H3 * B.hS_H3;
}

// ---- ELL1 (ELL1_model.py); H: ELL1H (binary_ell1.py:312, no M2/SINI, the H3 Shapiro delay)
template <bool H>
PD void ell1_setup(const pint_spec_t& S, const double* P, const InstConst& C, dd tdb, double acc_delay, BinState& B) {
    dd tasc = pdd(P, S.o_bin[PINT_B_TASC]);
    // ttasc = (t - TASC) in s with t = tdbld*day - acc_delay (pulsar_binary.py:398, ELL1_model.py:42)
    dd tt = dd_add_d(dd_mul_d(dd_sub(tdb, tasc), DAYSEC), -acc_delay);
    B.tt0 = dd_to_d(tt);
    dd PB = pdd(P, S.o_bin[PINT_B_PB]);
    dd PBs = dd_mul_d(PB, DAYSEC);
    B.PBs = dd_to_d(PBs);
    B.PBDOT = binp(S, P, PINT_B_PBDOT);
    B.XPBDOT = binp(S, P, PINT_B_XPBDOT);
    orbit_phase(tt, dd_make(C.ipb_hi, C.ipb_lo), B.PBDOT + B.XPBDOT, B);
    B.iPBs = C.ipb_hi + C.ipb_lo;
    B.pb = B.PBs + B.PBDOT * B.tt0;  // pbprime (binary_orbits.py:107)
    B.A1DOT = binp(S, P, PINT_B_A1DOT);
    B.a1 = binp(S, P, PINT_B_A1) + B.tt0 * B.A1DOT;
    B.EPS1DOT = binp(S, P, PINT_B_EPS1DOT) * 1e-12;  // par units 1e-12/s -> 1/s
    B.EPS2DOT = binp(S, P, PINT_B_EPS2DOT) * 1e-12;
    B.eps1 = binp(S, P, PINT_B_EPS1) + B.tt0 * B.EPS1DOT;
    B.eps2 = binp(S, P, PINT_B_EPS2) + B.tt0 * B.EPS2DOT;
    B.TM2 = H ? 0.0 : binp(S, P, PINT_B_M2) * TSUN;
    B.SINI = H ? 0.0 : binp(S, P, PINT_B_SINI);
    double Phi = B.Phi, e1 = B.eps1, e2 = B.eps2;
    // sin/cos(k Phi), k = 2..4, by the angle-addition identities from one sincos (a few
    // ulp of 1; they enter multiplied by a1 * eps <~ 1e-5 s)
    double s1, c1;
    sincos(Phi, &s1, &c1);
    const double s2 = 2.0 * s1 * c1, c2 = (c1 - s1) * (c1 + s1);
    const double s3 = s2 * c1 + c2 * s1, c3 = c2 * c1 - s2 * s1;
    const double s4 = 2.0 * s2 * c2, c4 = (c2 - s2) * (c2 + s2);
    B.s1 = s1; B.c1 = c1; B.s2 = s2; B.c2 = c2; B.s3 = s3; B.c3 = c3; B.s4 = s4; B.c4 = c4;
    double e1s = e1 * e1, e2s = e2 * e2;
    // d_delayR_da1 (ELL1_model.py:221-253)
    B.R0 = s1 + 0.5 * (e2 * s2 - e1 * c2) -
           (1.0 / 8) * (5 * e2s * s1 - 3 * e2s * s3 - 2 * e2 * e1 * c1 + 6 * e2 * e1 * c3 + 3 * e1s * s1 + 3 * e1s * s3) -
           (1.0 / 12) * (5 * e2s * e2 * s2 + 3 * e1s * e2 * s2 - 6 * e1 * e2s * c2 - 4 * e1s * e1 * c2 -
                         4 * e2s * e2 * s4 + 12 * e1s * e2 * s4 + 12 * e1 * e2s * c4 - 4 * e1s * e1 * c4);
    // d_d_delayR_dPhi_da1 (:255-284)
    B.R1 = c1 + e1 * s2 + e2 * c2 -
           (1.0 / 8) * (5 * e2s * c1 - 9 * e2s * c3 + 2 * e1 * e2 * s1 - 18 * e1 * e2 * s3 + 3 * e1s * c1 + 9 * e1s * c3) -
           (1.0 / 12) * (10 * e2s * e2 * c2 + 6 * e1s * e2 * c2 + 12 * e1 * e2s * s2 + 8 * e1s * e1 * s2 -
                         16 * e2s * e2 * c4 + 48 * e1s * e2 * c4 - 48 * e1 * e2s * s4 + 16 * e1s * e1 * s4);
    // d_dd_delayR_dPhi_da1 (:286-315)
    B.R2 = -s1 + 2 * e1 * c2 - 2 * e2 * s2 -
           (1.0 / 8) * (-5 * e2s * s1 + 27 * e2s * s3 + 2 * e1 * e2 * c1 - 54 * e1 * e2 * c3 - 3 * e1s * s1 - 27 * e1s * s3) -
           (1.0 / 12) * (-20 * e2s * e2 * s2 - 12 * e1s * e2 * s2 + 24 * e1 * e2s * c2 + 16 * e1s * e1 * c2 +
                         64 * e2s * e2 * s4 - 192 * e1s * e2 * s4 - 192 * e1 * e2s * c4 + 64 * e1s * e1 * c4);
    B.Dre = B.a1 * B.R0;  // delayR (:317)
    B.Drep = B.a1 * B.R1;  // Drep (:398)
    B.Drepp = B.a1 * B.R2;  // Drepp (:478)
    B.ipb = 1.0 / B.pb;
    B.nhat = TWO_PI * B.ipb;
    double nD = B.nhat * B.Drep;
    double delayI = B.Dre * (1 - nD + nD * nD + 0.5 * B.nhat * B.nhat * B.Dre * B.Drepp);  // :141-166
    double delayS;
    if (H) {
        B.lgNum = 0.0;
        delayS = ell1h_shapiro(S, P, B);  // ELL1Hdelay = delayI + delayS (ELL1H_model.py:78)
    } else {
        B.lgNum = log(1 - B.SINI * s1);
        delayS = -2 * B.TM2 * B.lgNum;  // :599-603
        B.hS_H3 = B.hS_sig = B.hS_Phi = B.dsig_dH3 = B.dsig_dH4 = 0.0;
    }
    B.delay = delayI + delayS;
    B.status = 0;
}

// d(ELL1 delay)/d(par) per SI unit (ELL1_model.py:637 d_ELL1delay_d_par -> :174, :325, :406,
// :483, :605).  The reference's chain rule is linear in the seeds (d a1, d Phi, d eps1,
// d eps2, d pb, d TM2, d SINI)/d(par) of prtl_der() (binary_generic.py:267), so the
// gradient over those seven primitives is formed once per TOA (ell1_grad) and every
// column is a dot product with its seed vector (ell1_deriv).
struct Ell1Grad {
    double a1, Phi, e1, e2, pb, TM2, SINI;
};

template <bool H>
PD void ell1_grad(const BinState& B, Ell1Grad& g) {
    double e1 = B.eps1, e2 = B.eps2, a1 = B.a1;
    double s1 = B.s1, c1 = B.c1, s2 = B.s2, c2 = B.c2, s3 = B.s3, c3 = B.c3, s4 = B.s4, c4 = B.c4;
    double e1s = e1 * e1, e2s = e2 * e2;
    double nhat = B.nhat, Dre = B.Dre, Drep = B.Drep, Drepp = B.Drepp;
    // d_Dre_d_par (:325-394)
    double dDre_de1 = a1 * (-0.5 * c2 - (1.0 / 8) * (-2 * e2 * c1 + 6 * e2 * c3 + 6 * e1 * s1 + 6 * e1 * s3) -
                            (1.0 / 12) * (6 * e1 * e2 * s2 - 6 * e2s * c2 - 12 * e1s * c2 + 24 * e1 * e2 * s4 +
                                          12 * e2s * c4 - 12 * e1s * c4));
    double dDre_de2 = a1 * (0.5 * s2 - (1.0 / 8) * (-2 * e1 * c1 + 6 * e1 * c3 + 10 * e2 * s1 - 6 * e2 * s3) -
                            (1.0 / 12) * (15 * e2s * s2 + 3 * e1s * s2 - 12 * e1 * e2 * c2 - 12 * e2s * s4 +
                                          12 * e1s * s4 + 24 * e1 * e2 * c4));
    // d_Drep_d_par (:406-476)
    double dDrep_de1 = a1 * (s2 - (1.0 / 8) * (6 * e1 * c1 + 18 * e1 * c3 + 2 * e2 * s1 - 18 * e2 * s3) -
                             (1.0 / 12) * (12 * e1 * e2 * c2 + 12 * e2s * s2 + 16 * e1s * s2 + 96 * e1 * e2 * c4 -
                                           48 * e2s * s4 + 48 * e1s * s4));
    double dDrep_de2 = a1 * (c2 - (1.0 / 8) * (2 * e1 * s1 - 18 * e1 * s3 + 10 * e2 * c1 - 18 * e2 * c3) -
                             (1.0 / 12) * (30 * e2s * c2 + 6 * e1s * c2 + 24 * e1 * e2 * s2 - 48 * e2s * c4 +
                                           48 * e1s * c4 - 96 * e1 * e2 * s4));
    // d_Drepp_d_par (:483-597)
    double dDrepp_dPhi =
        a1 * (-c1 - 4.0 * (e1 * s2 + e2 * c2) -
              (1.0 / 8) * (-5 * e2s * c1 + 81 * e2s * c3 - 2 * e1 * e2 * s1 + 162 * e1 * e2 * s3 - 3 * e1s * c1 - 81 * e1s * c3) -
              (1.0 / 12) * (-40 * e2s * e2 * c2 - 24 * e1s * e2 * c2 - 48 * e1 * e2s * s2 - 32 * e1s * e1 * s2 +
                            256 * e2s * e2 * c4 - 768 * e1s * e2 * c4 + 768 * e1 * e2s * s4 - 256 * e1s * e1 * s4));
    double dDrepp_de1 = a1 * (2.0 * c2 - (1.0 / 8) * (-6 * e1 * s1 - 54 * e1 * s3 + 2 * e2 * c1 - 54 * e2 * c3) -
                              (1.0 / 12) * (-24 * e1 * e2 * s2 + 24 * e2s * c2 + 48 * e1s * c2 - 384 * e1 * e2 * s4 -
                                            192 * e2s * c4 + 192 * e1s * c4));
    double dDrepp_de2 = a1 * (-2.0 * s2 - (1.0 / 8) * (2 * e1 * c1 - 54 * e1 * c3 - 10 * e2 * s1 + 54 * e2 * s3) -
                              (1.0 / 12) * (-60 * e2s * s2 - 12 * e1s * s2 + 48 * e1 * e2 * c2 + 192 * e2s * s4 -
                                            192 * e1s * s4 - 384 * e1 * e2 * c4));
    // d_delayI_d_par (:174-219)
    double nD = nhat * Drep;
    double dI_dDre = (1 - nD + nD * nD + 0.5 * nhat * nhat * Dre * Drepp) + Dre * 0.5 * nhat * nhat * Drepp;
    double dI_dDrep = -Dre * nhat + 2 * nD * nhat * Dre;
    double dI_dDrepp = 0.5 * (nhat * Dre) * (nhat * Dre);
    double dI_dnhat = Dre * (-Drep + 2 * nD * Drep + nhat * Dre * Drepp);
    // d_delayS_d_par (:605-631) -- note the reference's d_delayS_d_Phi omits cos(Phi) (:620)
    double lg = 1 - B.SINI * s1;
    g.a1 = dI_dDre * B.R0 + dI_dDrep * B.R1 + dI_dDrepp * B.R2;
    g.Phi = dI_dDre * Drep + dI_dDrep * Drepp + dI_dDrepp * dDrepp_dPhi +
            (H ? B.hS_Phi : (-2 * B.TM2 / lg * (-B.SINI)));
    g.e1 = dI_dDre * dDre_de1 + dI_dDrep * dDrep_de1 + dI_dDrepp * dDrepp_de1;
    g.e2 = dI_dDre * dDre_de2 + dI_dDrep * dDrep_de2 + dI_dDrepp * dDrepp_de2;
    g.pb = dI_dnhat * (-TWO_PI * B.ipb * B.ipb);
    g.TM2 = -2 * B.lgNum;
    g.SINI = -2 * B.TM2 / lg * (-s1);
}

PD double ell1_deriv(const BinState& B, const Ell1Grad& g, int pid) {
    const double tt0 = B.tt0, i2 = B.iPBs * B.iPBs;
    switch (pid) {
        case PINT_B_A1: return g.a1;
        case PINT_B_A1DOT: return g.a1 * tt0;
        case PINT_B_EPS1: return g.e1;
        case PINT_B_EPS1DOT: return g.e1 * tt0;
        case PINT_B_EPS2: return g.e2;
        case PINT_B_EPS2DOT: return g.e2 * tt0;
        case PINT_B_TASC:
            // d_Phi_d_TASC uses pb()=pbprime and pbdot() (ELL1_model.py:108)
            return g.e1 * (-B.EPS1DOT) + g.e2 * (-B.EPS2DOT) + g.Phi * ((B.PBDOT * tt0 * B.ipb - 1.0) * TWO_PI * B.ipb);
        case PINT_B_PB:
            return g.Phi * (TWO_PI * ((B.PBDOT + B.XPBDOT) * tt0 * tt0 * i2 * B.iPBs - tt0 * i2)) + g.pb;
        case PINT_B_PBDOT: return g.Phi * (-PI_D * tt0 * tt0 * i2) + g.pb * tt0;
        case PINT_B_XPBDOT: return g.Phi * (-PI_D * tt0 * tt0 * i2);
        case PINT_B_M2: return g.TM2 * TSUN;
        case PINT_B_SINI: return g.SINI;
        // ELL1H: d_delayS_d_par (ELL1H_model.py:326-359) through H3, stigma
        case PINT_B_H3: return B.hS_H3 + B.hS_sig * B.dsig_dH3;
        case PINT_B_H4: return B.hS_sig * B.dsig_dH4;
        case PINT_B_STIGMA: return B.hS_sig;
        default: return 0.0;
    }
}

// ---- DDK (DDK_model.py): Kopeikin corrections to DD's a1, omega and SINI -------------
// a1 = a1b (1 + dkin cot(kin)) (1 + cot(kin) P1), omega += K96 csc(kin) Bv tt0 - csc(kin) P2,
// SINI = sin(kin), kin = KIN + K96 A tt0 (:157-174, :233-252, :291-308, :399-414, :470-483,
// :526-584), A = -mu_l sin KOM + mu_b cos KOM, Bv = mu_l cos KOM + mu_b sin KOM (proper motion
// in the astrometry's frame, PMRA/PMDEC or PMELONG/PMELAT, rad/s), P1 = (dI0 sin KOM - dJ0 cos
// KOM)/d, P2 = (dI0 cos KOM + dJ0 sin KOM)/d with dI0, dJ0 the observatory position projected
// on the sky's east and north directions at the pulsar (Kopeikin 1995 Eqs. 15-16, :355-373) and
// d = 1 kpc / PX.  obs (km) and psr (unit) are in the astrometry's frame.  The derivative
// pieces per KIN, KOM, T0 follow d_a1_k_d_par / d_omega_k_d_par (:547-602) and
// d_SINI_d_{KIN,KOM,T0} as written (:176-195, incl. the T0 form without cos(kin) and the
// non-K96 forms in per-degree / per-day units).
PD void ddk_kopeikin(const pint_spec_t& S, const double* P, const double obs[3], const double psr[3], BinState& B) {
    const bool k96 = S.k96 != 0;
    const double mul = (S.o_pmlon >= 0 ? pval(P, S.o_pmlon) : 0.0) * MASYR_RADS;
    const double mub = (S.o_pmlat >= 0 ? pval(P, S.o_pmlat) : 0.0) * MASYR_RADS;
    const double KIN = binp(S, P, PINT_B_KIN) * DEG_RAD, KOM = binp(S, P, PINT_B_KOM) * DEG_RAD;
    double sK, cK;
    sincos(KOM, &sK, &cK);
    const double tt0 = B.tt0;
    const double A = -mul * sK + mub * cK, Bv = mul * cK + mub * sK;
    const double dkin = k96 ? A * tt0 : 0.0;
    double sk, ck;
    sincos(KIN + dkin, &sk, &ck);
    const double isk = 1.0 / sk, cot = ck * isk, isk2 = isk * isk;
    // psr_pos setter (:106-121)
    const double sl = psr[2], cl = cos(asin(sl)), icl = 1.0 / cl;
    const double slo = psr[1] * icl, clo = psr[0] * icl;
    const double dI0 = -obs[0] * slo + obs[1] * clo;
    const double dJ0 = -obs[0] * sl * clo - obs[1] * sl * slo + obs[2] * cl;
    const double ipx = (S.o_px >= 0 ? pval(P, S.o_px) : 0.0) * INV_KPC_KM;
    const double P1 = (dI0 * sK - dJ0 * cK) * ipx, P2 = (dI0 * cK + dJ0 * sK) * ipx;
    const double P3 = (-dI0 * sK + dJ0 * cK) * ipx;
    const double a1b = B.a1;
    const double a1p = k96 ? a1b + a1b * dkin * cot : a1b;
    B.a1 = a1p + a1p * cot * P1;
    B.omega += (k96 ? Bv * isk * tt0 : 0.0) - P2 * isk;
    B.SINI = sk;
    const double dk[3] = {1.0, k96 ? -Bv * tt0 : 0.0, k96 ? -A : 0.0};
    for (int j = 0; j < 3; j++) {
        // d_delta_a1_proper_motion_d_{KIN,KOM,T0} (:254-289)
        double dpm = 0.0;
        if (k96) dpm = (j == 0) ? -a1b * dkin * isk2 : a1b * dk[j] * (-dkin * isk2 + cot);
        const double da1p = (j == 2 ? -B.A1DOT : 0.0) + dpm;  // d_a1_k_d_par(., pm=K96, px=False)
        double dpx = (da1p * cot - a1p * dk[j] * isk2) * P1;  // d_delta_a1_parallax_d_* (:416-468)
        if (j == 1) dpx += a1p * cot * P2;
        B.kA1[j] = dpm + dpx;
        double dwpm = 0.0;  // d_delta_omega_proper_motion_d_* (:310-349)
        if (k96) {
            if (j == 0) dwpm = -ck * isk2 * Bv * tt0;
            else if (j == 1) dwpm = (-ck * isk2 * dk[1] * Bv + A * isk) * tt0;
            else dwpm = (-ck * isk2 * (-A) * tt0 - isk) * Bv;
        }
        double dwpx = ck * isk2 * dk[j] * P2;  // d_delta_omega_parallax_d_* (:485-524)
        if (j == 1) dwpx -= P3 * isk;
        B.kOM[j] = dwpm + dwpx;
    }
    B.kSI[0] = ck;
    B.kSI[1] = k96 ? -Bv * tt0 * ck : ck * (1.0 / DEG_RAD);
    B.kSI[2] = k96 ? -A : 1.0 / DAYSEC;
}

// ---- DD (DD_model.py, binary_generic.py) ------------------------------------------
template <bool K = false>
PD void ddm_setup(const pint_spec_t& S, const double* P, const InstConst& C, dd tdb, double acc_delay, BinState& B,
                  const double* kobs = nullptr, const double* kpsr = nullptr) {
    dd T0 = pdd(P, S.o_bin[PINT_B_T0]);
    dd tt = dd_add_d(dd_mul_d(dd_sub(tdb, T0), DAYSEC), -acc_delay);  // get_tt0 (binary_generic.py:372)
    B.tt0 = dd_to_d(tt);
    dd PB = pdd(P, S.o_bin[PINT_B_PB]);
    dd PBs = dd_mul_d(PB, DAYSEC);
    B.PBs = dd_to_d(PBs);
    B.PBDOT = binp(S, P, PINT_B_PBDOT);
    B.XPBDOT = binp(S, P, PINT_B_XPBDOT);
    orbit_phase(tt, dd_make(C.ipb_hi, C.ipb_lo), B.PBDOT + B.XPBDOT, B);
    B.iPBs = C.ipb_hi + C.ipb_lo;
    B.pb = B.PBs + B.PBDOT * B.tt0;
    B.A1DOT = binp(S, P, PINT_B_A1DOT);
    B.a1 = binp(S, P, PINT_B_A1) + B.tt0 * B.A1DOT;
    B.EDOT = binp(S, P, PINT_B_EDOT);
    B.ecc = binp(S, P, PINT_B_ECC) + B.tt0 * B.EDOT;
    B.TM2 = binp(S, P, PINT_B_M2) * TSUN;
    B.SINI = binp(S, P, PINT_B_SINI);
    B.GAMMA = binp(S, P, PINT_B_GAMMA);
    B.DR = binp(S, P, PINT_B_DR);
    B.DTH = binp(S, P, PINT_B_DTH);
    B.A0 = binp(S, P, PINT_B_A0);
    B.B0 = binp(S, P, PINT_B_B0);
    B.status = 0;
    double e = B.ecc, M = B.Phi;
    if (!(e >= 0.0 && e < 1.0)) { B.status = PINT_E_KEPLER; B.delay = 0; return; }
    // compute_eccentric_anomaly (binary_generic.py:337-370): Newton from E0 = M, tol 5e-15
    double U = M, sU, cU;
    int it = 0;
    sincos(U, &sU, &cU);
    double kU = U - e * sU - M;
    while (fabs(kU) > 5e-15 && it < 64) {
        U = U - kU / (1 - e * cU);
        sincos(U, &sU, &cU);
        kU = U - e * sU - M;
        it++;
    }
    if (fabs(kU) > 5e-15) B.status = PINT_E_KEPLER;
    B.E = U;
    B.sinE = sU;  // sin/cos of the converged U
    B.cosE = cU;
    // nu (binary_generic.py:538-549), unwrapped: 2*pi*orbits + nu - M = 2*pi*floor(orbits) + nu
    double nu = 2 * atan(sqrt((1.0 + e) / (1.0 - e)) * tan(U / 2.0));
    if (nu < 0) nu += TWO_PI;
    B.nu = TWO_PI * B.floor_orbits + nu;
    B.OMDOT_rs = binp(S, P, PINT_B_OMDOT) * (DEG_RAD / YR_S);
    B.ipb = 1.0 / B.pb;
    B.k = B.OMDOT_rs * B.pb * INV_TWO_PI;             // DD_model.py:76 k
    B.omega = binp(S, P, PINT_B_OM) * DEG_RAD + B.nu * B.k;  // :86
    if (K) ddk_kopeikin(S, P, kobs, kpsr, B);
    B.er = e * (1 + B.DR);
    B.eTheta = e * (1 + B.DTH);
    double sw, cw;
    sincos(B.omega, &sw, &cw);
    B.sw = sw;
    B.cw = cw;
    sincos(B.nu, &B.snu, &B.cnu);
    B.sqTh = sqrt(1 - B.eTheta * B.eTheta);
    B.sqE = sqrt(1 - e * e);
    B.alpha = B.a1 * sw;                                    // :223
    B.beta = B.a1 * B.sqTh * cw;                            // :275
    double sE = B.sinE, cE = B.cosE;
    double delayR = B.alpha * (cE - B.er) + B.beta * sE;    // :423
    B.Dre = delayR + B.GAMMA * sE;                          // :434 + delayE :786
    B.Drep = -B.alpha * sE + (B.beta + B.GAMMA) * cE;       // :470
    B.Drepp = -B.alpha * cE - (B.beta + B.GAMMA) * sE;      // :520
    B.iomeE = 1.0 / (1 - e * cE);
    B.isnu = 1.0 / B.snu;
    B.isqTh = 1.0 / B.sqTh;
    B.isqE = 1.0 / B.sqE;
    B.nhat = TWO_PI * B.ipb * B.iomeE;                      // :562
    double nH = B.nhat;
    double delayI = B.Dre * (1 - nH * B.Drep + (nH * B.Drep) * (nH * B.Drep) + 0.5 * nH * nH * B.Dre * B.Drepp -
                             0.5 * e * sE * B.iomeE * nH * nH * B.Dre * B.Drep);  // :602-646
    double logNum = 1 - e * cE - B.SINI * (sw * (cE - e) + B.sqE * cw * sE);
    B.logNum = logNum;
    B.lgNum = log(logNum);
    B.ilogNum = 1.0 / logNum;
    double delayS = -2 * B.TM2 * B.lgNum;                   // :700-720
    double oPn = B.omega + B.nu;
    sincos(oPn, &B.soPn, &B.coPn);
    double delayA = B.A0 * (B.soPn + e * sw) + B.B0 * (B.coPn + e * cw);  // :794-806
    B.delay = delayI + delayS + delayA;
}

template <bool K = false>
PD double ddm_deriv(const BinState& B, int pid) {
    const double e = B.ecc, sE = B.sinE, cE = B.cosE, tt0 = B.tt0;
    const double iP = B.iPBs, iP2 = iP * iP;
    const double iom = B.iomeE;  // 1 / (1 - e cosE)
    // ---- seeds (binary_generic.py / binary_orbits.py / DD_model.py) ----
    bool orbit_par = (pid == PINT_B_PB || pid == PINT_B_PBDOT || pid == PINT_B_XPBDOT || pid == PINT_B_T0);
    double d_ecc = 0, d_a1 = 0, d_M = 0, d_pb = 0;
    switch (pid) {
        case PINT_B_T0: d_ecc = -B.EDOT; d_a1 = -B.A1DOT;
            d_M = ((B.PBDOT - B.XPBDOT) * tt0 * iP - 1.0) * TWO_PI * iP;  // binary_orbits.py:114
            d_pb = -B.PBDOT; break;
        case PINT_B_ECC: d_ecc = 1; break;
        case PINT_B_EDOT: d_ecc = tt0; break;
        case PINT_B_A1: d_a1 = 1; break;
        case PINT_B_A1DOT: d_a1 = tt0; break;
        case PINT_B_PB: d_M = TWO_PI * ((B.PBDOT + B.XPBDOT) * tt0 * tt0 * iP2 * iP - tt0 * iP2);
            d_pb = 1; break;
        case PINT_B_PBDOT: d_M = -PI_D * tt0 * tt0 * iP2; d_pb = tt0; break;
        case PINT_B_XPBDOT: d_M = -PI_D * tt0 * tt0 * iP2; break;
        default: break;
    }
    // DDK: Kopeikin pieces of d_a1_d_par / d_omega_d_par / prtl_der("SINI", .)
    double k_a1 = 0.0, k_om = 0.0, k_si = (pid == PINT_B_SINI) ? 1.0 : 0.0;
    if (K) {
        const int j = pid == PINT_B_KIN ? 0 : (pid == PINT_B_KOM ? 1 : (pid == PINT_B_T0 ? 2 : -1));
        k_si = 0.0;
        if (j >= 0) {
            k_a1 = B.kA1[j];
            k_om = B.kOM[j];
            k_si = B.kSI[j];
        }
    }
    // E (binary_generic.py:397-448)
    double d_E_d_ECC = sE * iom;
    double d_E = 0;
    if (pid == PINT_B_T0) d_E = (d_M - B.EDOT * sE) * iom;
    else if (pid == PINT_B_ECC) d_E = d_E_d_ECC;
    else if (pid == PINT_B_EDOT) d_E = tt0 * d_E_d_ECC;
    else if (orbit_par) d_E = d_M * iom;
    // nu (binary_generic.py:451-624)
    double snu = B.snu, cnu = B.cnu;
    double d_nu_d_E = (1 + e * cnu) * iom * (sE * B.isnu);
    double d_nu_d_ecc = sE * sE * (iom * iom) * B.isnu;
    double d_nu = 0;
    if (pid == PINT_B_T0) d_nu = d_nu_d_ecc * (-B.EDOT) + d_nu_d_E * d_E;
    else if (pid == PINT_B_ECC) d_nu = d_nu_d_ecc + d_nu_d_E * d_E_d_ECC;
    else if (pid == PINT_B_EDOT) d_nu = tt0 * (d_nu_d_ecc + d_nu_d_E * d_E_d_ECC);
    else if (orbit_par) d_nu = d_nu_d_E * d_E;
    // omega (DD_model.py:88-133)
    double d_omega;
    if (pid == PINT_B_OM) d_omega = 1;
    else if (pid == PINT_B_OMDOT) d_omega = B.pb * INV_TWO_PI * B.nu;
    else if (orbit_par) d_omega = d_nu * B.k + d_pb * B.nu * B.OMDOT_rs * INV_TWO_PI;
    else d_omega = B.k * d_nu;
    d_omega += k_om;
    d_a1 += k_a1;  // alpha and d_beta_d_par; DD's d_beta_d_T0 keeps d_a1_d_T0 (DD_model.py:352)
    // er / eTheta (DD_model.py:149-205): d_ecc_d_par only for T0/ECC/EDOT; DR/DTH -> ecc
    double d_er = (pid == PINT_B_DR) ? e : d_ecc;
    double d_eTh = (pid == PINT_B_DTH) ? e : d_ecc;
    double sw = B.sw, cw = B.cw;
    double eTh = B.eTheta, sq = B.sqTh, isq = B.isqTh;
    // alpha (DD_model.py:225-246)
    double d_alpha = d_a1 * sw + B.a1 * cw * d_omega;
    // beta (DD_model.py:277-407): specific d_beta_d_X methods take precedence in prtl_der
    double d_beta;
    switch (pid) {
        case PINT_B_A1: d_beta = sq * cw; break;
        case PINT_B_A1DOT: d_beta = tt0 * sq * cw; break;
        case PINT_B_T0: d_beta = -B.A1DOT * sq * cw; break;
        case PINT_B_ECC: case PINT_B_EDOT: {
            double f = (pid == PINT_B_EDOT) ? tt0 : 1.0;
            d_beta = B.a1 * ((-eTh) * isq * cw * f - sq * sw * d_omega);
        } break;
        case PINT_B_DTH: d_beta = B.a1 * (-eTh) * isq * cw; break;
        default:
            d_beta = sq * cw * d_a1 + (-B.a1 * sq * sw) * d_omega + (B.a1 * (-eTh) * isq * cw) * d_eTh;
    }
    double d_gamma = (pid == PINT_B_GAMMA) ? 1.0 : 0.0;
    double alpha = B.alpha, beta = B.beta, G = B.GAMMA;
    // Dre, Drep, Drepp (DD_model.py:437-550)
    double dDre = alpha * (-d_er - d_E * sE) + (cE - B.er) * d_alpha + (d_beta + d_gamma) * sE + (beta + G) * cE * d_E;
    double dDrep = -sE * d_alpha - (alpha * cE + (beta + G) * sE) * d_E + cE * (d_beta + d_gamma);
    double dDrepp = -cE * d_alpha + (alpha * sE - (beta + G) * cE) * d_E - sE * (d_beta + d_gamma);
    // nhat (DD_model.py:564-590): uses prtl_der("PB") (1 only for PB)
    double dPB = (pid == PINT_B_PB) ? 1.0 : 0.0;
    double d_nhat = -TWO_PI * B.ipb * iom * (dPB * B.ipb - (cE * d_ecc - e * sE * d_E) * iom);
    // delayI (DD_model.py:648-698)
    double Dre = B.Dre, Drep = B.Drep, Drepp = B.Drepp, nH = B.nhat;
    double x = -0.5 * e * sE * iom;
    double dx = -sE * (0.5 * iom * iom) * d_ecc + e * (e - cE) * (0.5 * iom * iom) * d_E;
    double dI_dDre = 1 + (Drep * nH) * (Drep * nH) + Dre * Drepp * nH * nH + Drep * nH * (2 * Dre * nH * x - 1);
    double dI_dDrep = Dre * nH * (2 * Drep * nH + Dre * nH * x - 1);
    double dI_dDrepp = (Dre * nH) * (Dre * nH) / 2;
    double dI_dnhat = Dre * (-Drep + 2 * Drep * Drep * nH + nH * Dre * Drepp + 2 * x * nH * Dre * Drep);
    double dI_dx = (Dre * nH) * (Dre * nH) * Drep;
    double dI = dDre * dI_dDre + dDrep * dI_dDrep + dDrepp * dI_dDrepp + dx * dI_dx + d_nhat * dI_dnhat;
    // delayS (DD_model.py:722-784)
    double sq1 = B.sqE;
    double ilN = B.ilogNum;
    double d_TM2 = (pid == PINT_B_M2) ? TSUN : 0.0;
    double d_SINI = k_si;
    double TM2 = B.TM2;
    double dS = d_TM2 * (-2 * B.lgNum) +
                d_ecc * (-2 * TM2 * ilN * (-cE - B.SINI * (-e * cw * sE * B.isqE - sw))) +
                d_E * (-2 * TM2 * ilN * (e * sE - B.SINI * (sq1 * cE * cw - sE * sw))) +
                d_omega * (2 * TM2 * ilN * B.SINI * ((cE - e) * cw - sq1 * sE * sw)) +
                d_SINI * (-2 * TM2 * ilN * (-sq1 * cw * sE - (cE - e) * sw));
    // delayA (DD_model.py:808-848)
    const double soPn = B.soPn, coPn = B.coPn;
    double dA;
    if (pid == PINT_B_A0) dA = e * sw + soPn;
    else if (pid == PINT_B_B0) dA = e * cw + coPn;
    else
        dA = d_omega * (B.A0 * (coPn + e * cw) - B.B0 * (soPn + e * sw)) +
             d_nu * (B.A0 * coPn - B.B0 * soPn) + d_ecc * (B.A0 * sw + B.B0 * cw);
    return dI + dS + dA;
}

// ---- BT (BT_model.py, Blandford & Teukolsky 1976) -----------------------------------
// delay = (delayL1 + delayL2) * delayR with delayL1 = a1 sin(w) (cosE - e), delayL2 =
// (a1 cos(w) sqrt(1 - e^2) + GAMMA) sinE, delayR = 1 - 2 pi (a1 cos(w) sqrt(1-e^2) cosE -
// a1 sin(w) sinE) / ((1 - e cosE) pb'), w = OM + OMDOT tt0 (binary_generic.py:631).
// Kepler's equation as in DD.  B.Dre = L1 + L2, B.R0 = delayR.
PD void bt_setup(const pint_spec_t& S, const double* P, const InstConst& C, dd tdb, double acc_delay, BinState& B) {
    dd T0 = pdd(P, S.o_bin[PINT_B_T0]);
    dd tt = dd_add_d(dd_mul_d(dd_sub(tdb, T0), DAYSEC), -acc_delay);  // get_tt0 (binary_generic.py:372)
    B.tt0 = dd_to_d(tt);
    dd PBs = dd_mul_d(pdd(P, S.o_bin[PINT_B_PB]), DAYSEC);
    B.PBs = dd_to_d(PBs);
    B.PBDOT = binp(S, P, PINT_B_PBDOT);
    B.XPBDOT = binp(S, P, PINT_B_XPBDOT);
    orbit_phase(tt, dd_make(C.ipb_hi, C.ipb_lo), B.PBDOT + B.XPBDOT, B);
    B.iPBs = C.ipb_hi + C.ipb_lo;
    B.pb = B.PBs + B.PBDOT * B.tt0;
    B.A1DOT = binp(S, P, PINT_B_A1DOT);
    B.a1 = binp(S, P, PINT_B_A1) + B.tt0 * B.A1DOT;
    B.EDOT = binp(S, P, PINT_B_EDOT);
    B.ecc = binp(S, P, PINT_B_ECC) + B.tt0 * B.EDOT;
    B.GAMMA = binp(S, P, PINT_B_GAMMA);
    B.status = 0;
    const double e = B.ecc, M = B.Phi;
    if (!(e >= 0.0 && e < 1.0)) { B.status = PINT_E_KEPLER; B.delay = 0; return; }
    double U = M, sU, cU;
    int it = 0;
    sincos(U, &sU, &cU);
    double kU = U - e * sU - M;
    while (fabs(kU) > 5e-15 && it < 64) {
        U = U - kU / (1 - e * cU);
        sincos(U, &sU, &cU);
        kU = U - e * sU - M;
        it++;
    }
    if (fabs(kU) > 5e-15) B.status = PINT_E_KEPLER;
    B.E = U;
    B.sinE = sU;
    B.cosE = cU;
    B.OMDOT_rs = binp(S, P, PINT_B_OMDOT) * (DEG_RAD / YR_S);
    B.omega = binp(S, P, PINT_B_OM) * DEG_RAD + B.OMDOT_rs * B.tt0;
    sincos(B.omega, &B.sw, &B.cw);
    B.sqE = sqrt(1 - e * e);
    B.ipb = 1.0 / B.pb;
    B.iomeE = 1.0 / (1 - e * cU);
    const double L1 = B.a1 * B.sw * (cU - e);
    const double L2 = (B.a1 * B.cw * B.sqE + B.GAMMA) * sU;
    const double num = B.a1 * B.cw * B.sqE * cU - B.a1 * B.sw * sU;
    B.R0 = 1.0 - TWO_PI * num * B.iomeE * B.ipb;
    B.Dre = L1 + L2;
    B.delay = B.Dre * B.R0;
}

// d_BTdelay_d_par = delayR (d_delayL1_d_par + d_delayL2_d_par) (BT_model.py:258): delayR's own
// derivatives are ignored, d_delayL1_d_ECC carries +a1 sin(w) (:189, as the reference has
// it), d_delayL*_d_T0 goes through E only (:212-216); other orbit parameters through E.
PD double bt_deriv(const BinState& B, int pid) {
    const double e = B.ecc, sE = B.sinE, cE = B.cosE, tt0 = B.tt0, a1 = B.a1;
    const double sw = B.sw, cw = B.cw, sq = B.sqE, iom = B.iomeE;
    const double iP = B.iPBs, iP2 = iP * iP;
    const double dL1_dE = -a1 * sw * sE;
    const double dL2_dE = (a1 * cw * sq + B.GAMMA) * cE;
    const double dE_dECC = sE * iom;
    double dL1 = 0.0, dL2 = 0.0, dE = 0.0;
    switch (pid) {
        case PINT_B_A1: case PINT_B_A1DOT: {
            const double f = (pid == PINT_B_A1DOT) ? tt0 : 1.0;
            dL1 = f * sw * (cE - e);
            dL2 = f * cw * sq * sE;
        } break;
        case PINT_B_OM: case PINT_B_OMDOT: {
            const double f = (pid == PINT_B_OMDOT) ? tt0 : 1.0;
            dL1 = f * a1 * cw * (cE - e);
            dL2 = -f * a1 * sw * sq * sE;
        } break;
        case PINT_B_ECC: case PINT_B_EDOT: {
            const double f = (pid == PINT_B_EDOT) ? tt0 : 1.0;
            dL1 = f * (a1 * sw + dL1_dE * dE_dECC);
            dL2 = f * (-a1 * cw * e * sE / sq + dL2_dE * dE_dECC);
        } break;
        case PINT_B_GAMMA: dL2 = sE; break;
        case PINT_B_T0:
            dE = (((B.PBDOT - B.XPBDOT) * tt0 * iP - 1.0) * TWO_PI * iP - B.EDOT * sE) * iom;
            break;
        case PINT_B_PB: dE = TWO_PI * ((B.PBDOT + B.XPBDOT) * tt0 * tt0 * iP2 * iP - tt0 * iP2) * iom; break;
        case PINT_B_PBDOT: case PINT_B_XPBDOT: dE = -PI_D * tt0 * tt0 * iP2 * iom; break;
        default: break;
    }
    if (dE != 0.0) {
        dL1 = dL1_dE * dE;
        dL2 = dL2_dE * dE;
    }
    return B.R0 * (dL1 + dL2);
}

// ------------------------------------------------------------------------------------
// Per-TOA evaluation
// ------------------------------------------------------------------------------------
struct ToaRow {
    dd tdb;
    double freq;
    double pos[3], vel[3], sun[3];
    const double* planet;  // 15: observatory -> jupiter, saturn, venus, uranus, neptune (km), or null
    uint32_t flags;
    uint64_t jmask;
    int dmx_a, dmx_b;
    const int32_t* dmx_x;  // PsrDev::dmx_x (bins beyond the first two), entries [dmx_x0, dmx_x1)
    int dmx_x0, dmx_x1;
};

struct EvalOut {
    dd phase;        // spindown + jump phase (cycles)
    double delay;    // total delay (s)
    double fdt;      // spin frequency at dt incl. delay (for d_phase_d_delay)
    double ftaylor;  // spin frequency at dt without delay (residuals.py:295-310)
    double dmc;      // value of this TOA's DMX design-matrix entries (compact layout)
    double inv_f2;   // 1 / f_bary^2 (MHz^-2): PLDMNoise's basis scale (1400 MHz)^2 / f_bary^2
    int status;
};

// taylor_horner (utils.py:419) with coefficients [0, F0, F1, ...] in dd
PD dd spin_phase(const pint_spec_t& S, const double* P, dd dt) {
    int m = S.nf;
    dd r = pdd(P, S.o_F + 2 * (m - 1));
    for (int j = m - 1; j >= 1; j--) {
        r = dd_add(dd_div_int(dd_mul(r, dt), j + 1), pdd(P, S.o_F + 2 * (j - 1)));
    }
    return dd_mul(r, dt);
}
// taylor_horner_deriv(dt, [0, F0, ...], 1) in double
PD double spin_freq(const pint_spec_t& S, const double* P, double dt) {
    int m = S.nf;
    double r = pval(P, S.o_F + 2 * (m - 1));
    for (int j = m - 1; j >= 1; j--) r = r * dt * inv_int(j) + pval(P, S.o_F + 2 * (j - 1));
    return r;
}

// Column runs (built by pint_add_pulsar from spec.col_kind/col_index): consecutive
// design-matrix columns of one kind with consecutive indices, so the row loop walks ~15
// runs with tight per-kind inner loops instead of a switch per column.
struct ColRun {
    int kind, col0, cnt, idx0;
    int dcol0;  // column in the compact fit layout (DMX columns are not stored there: -1)
    int pad_[3];
};

// Evaluate one TOA.  If Mb != nullptr, writes the design-matrix row r (column-major,
// leading dimension ld, column c at Mb + c*ld) for columns 0..ncol-1
// (timing_model.py:2164-2173).  compact: the fit layout, where the DMX columns (1 on the
// bin's TOAs times one per-TOA value, o.dmc) are not stored and the other columns are
// packed (ColRun.dcol0).
// The parameter-side state eval_toa forms before the spin phase: everything but the spin
// phase, the spin frequencies and the chain factor that scales the design-matrix row depends
// on the TOA and the non-spin parameters only.  A grid whose points differ in spin
// parameters alone shares it across its points (k_eval_head / k_eval_spin).
struct EvalHead {
    double delay;                          // total delay (s)
    double gLON, gLAT, gPMLON, gPMLAT, gPX;  // astrometric geometry without the chain factor
    double inv_f2, dt_yr_dm, logf;
};
constexpr int EVAL_HEAD_W = 9;  // doubles of an EvalHead row

// eval_toa after the delay: the spin frequency at dt (dt0 - delay) and at dt0, the chain
// factor of the design matrix
struct EvalSpin {
    dd dt;
    double dtd, chain;
};
PD void eval_spin_a(const pint_spec_t& S, const double* P, const InstConst& C, const ToaRow& t, double delay,
                    EvalOut& o, EvalSpin& sp) {
    o.delay = delay;
    dd dt0 = dd_mul_d(dd_sub(t.tdb, pdd(P, S.o_PEPOCH)), DAYSEC);
    sp.dt = dd_add_d(dt0, -delay);
    sp.dtd = dd_to_d(sp.dt);
    o.fdt = spin_freq(S, P, sp.dtd);
    o.ftaylor = spin_freq(S, P, dd_to_d(dt0));
    sp.chain = o.fdt * C.iF0;  // M = -(d_phase_d_delay * d_delay_d_p)/F0, d_phase_d_delay = -F(dt)
}

// eval_toa's spindown phase, jumps and PhaseOffset, then the design-matrix row but for the
// binary columns (written by eval_toa while the binary state is live)
template <int BIN>
PD void eval_spin_b(const pint_spec_t& S, const double* P, const InstConst& C, const ToaRow& t, const EvalHead& h,
                    const EvalSpin& sp, EvalOut& o, double* Mb, unsigned r, long ld, const ColRun* runs, int nrun,
                    bool compact) {
    const double chain = sp.chain, dtd = sp.dtd;
    // ---- spindown phase (spindown.py:124-155) + jumps (jump.py:119-136) ----
    dd ph = spin_phase(S, P, sp.dt);
    if (S.njump > 0 && t.jmask) {
        dd F0 = pdd(P, S.o_F);
        for (int k = 0; k < S.njump; k++)
            if ((t.jmask >> k) & 1ull) ph = dd_add(ph, dd_mul(dd_make(pval(P, S.o_JUMP + 2 * k)), F0));
    }
    // PhaseOffset.offset_phase (phase_offset.py): -PHOFF on the TOAs, nothing on the TZR TOA
    // (row ld = n)
    if (S.o_PHOFF >= 0 && r < (unsigned)ld) ph = dd_sub(ph, pdd(P, S.o_PHOFF));
    o.phase = ph;
    if (!Mb) return;
    // ---- design matrix row (timing_model.py:2073-2175) ----
    const double iF0 = C.iF0;
    const double dt_yr_dm = h.dt_yr_dm, logf = h.logf;
    // the astrometric geometry formed above, times the chain factor
    const double gLON = h.gLON * chain;
    const double gLAT = h.gLAT * chain;
    const double gPMLON = h.gPMLON * chain;
    const double gPMLAT = h.gPMLAT * chain;
    const double gPX = h.gPX * chain;
    const double dmc = chain * DMCONST * h.inv_f2;
    o.dmc = dmc;
    for (int u = 0; u < nrun; u++) {
        const ColRun R = runs[u];
        if (compact && R.kind == PINT_COL_DMX) continue;
        double* colp = Mb + (long)(compact ? R.dcol0 : R.col0) * ld;
        switch (R.kind) {
            case PINT_COL_OFFSET: colp[r] = iF0; break;
            case PINT_COL_F: {  // d_phase_d_F (spindown.py:207): -dt^(k+1)/(k+1)! / F0
                double v = 1.0;
                for (int j = 1; j <= R.idx0; j++) v = v * dtd * inv_int(j);
                for (int j = 0; j < R.cnt; j++, colp += ld) {
                    v = v * dtd * inv_int(R.idx0 + j + 1);
                    colp[r] = -v * iF0;
                }
            } break;
            case PINT_COL_JUMP:  // jump.py:138
                for (int j = 0; j < R.cnt; j++, colp += ld) colp[r] = ((t.jmask >> (R.idx0 + j)) & 1ull) ? -1.0 : 0.0;
                break;
            case PINT_COL_LON: colp[r] = gLON; break;
            case PINT_COL_LAT: colp[r] = gLAT; break;
            case PINT_COL_PMLON: colp[r] = gPMLON; break;
            case PINT_COL_PMLAT: colp[r] = gPMLAT; break;
            case PINT_COL_PX: colp[r] = gPX; break;
            case PINT_COL_DM: {  // d_dm_d_DMs (dispersion_model.py:253) * DMconst / bfreq^2
                double v = 1.0;
                for (int j = 1; j <= R.idx0; j++) v = v * dt_yr_dm * inv_int(j);
                for (int j = 0; j < R.cnt; j++, colp += ld) {
                    if (j > 0) v = v * dt_yr_dm * inv_int(R.idx0 + j);
                    colp[r] = dmc * v;
                }
            } break;
            case PINT_COL_DMX:  // d_dm_d_DMX (:684): 1 on the bin's TOAs
                for (int j = 0; j < R.cnt; j++, colp += ld) {
                    const int idx = R.idx0 + j;
                    bool in = t.dmx_a == idx || t.dmx_b == idx;
                    for (int k = t.dmx_x0; k < t.dmx_x1; k++) in |= t.dmx_x[k] == idx;
                    colp[r] = in ? dmc : 0.0;
                }
                break;
            case PINT_COL_FD: {  // d_delay_FD_d_FDX (frequency_dependent.py:103): logf^(k+1)
                double v = 1.0;
                for (int j = 0; j <= R.idx0; j++) v *= logf;
                for (int j = 0; j < R.cnt; j++, colp += ld) {
                    if (j > 0) v *= logf;
                    colp[r] = chain * v;
                }
            } break;
            case PINT_COL_BIN:  // written with the binary state above
                if (BIN == 0)
                    for (int j = 0; j < R.cnt; j++, colp += ld) colp[r] = 0.0;
                break;
            default:
                for (int j = 0; j < R.cnt; j++, colp += ld) colp[r] = 0.0;
        }
    }
}

// eval_toa up to the binary model: the astrometric (Roemer, parallax), Solar-system Shapiro,
// dispersion (DM Taylor series, DMX) delays, the barycentric frequency, FD (formed, added
// after the binary delay), and the astrometric design-matrix geometry without the chain factor
struct EvalPre {
    EvalHead h;  // h.delay: the delay so far (without FD: acc_delay of the binary model)
    double fd;
    double L[3];
};
PD void eval_pre(const pint_spec_t& S, const double* P, const InstConst& C, const ToaRow& t, EvalOut& o, bool wantM,
                 EvalPre& pre) {
    o.status = 0;
    o.dmc = 0.0;
    double delay = 0.0;
    // ---- astrometry: solar_system_geometric_delay (astrometry.py:155-184) ----
    double L[3] = {0, 0, 1};
    double tdb_f = dd_to_d(t.tdb);
    bool has_pos = (t.flags & 2u) != 0;
    bool is_bary = (t.flags & 1u) != 0;
    double rr = 0.0, re_dot_L = 0.0;
    double px_mas = S.o_px >= 0 ? pval(P, S.o_px) : 0.0;
    if (S.astrometry) {
        psr_dir_icrs(C, tdb_f, L);
        rr = t.pos[0] * t.pos[0] + t.pos[1] * t.pos[1] + t.pos[2] * t.pos[2];
        re_dot_L = t.pos[0] * L[0] + t.pos[1] * L[1] + t.pos[2] * L[2];
        if (has_pos) {
            double d = -re_dot_L * INV_C_KMS;
            if (px_mas != 0.0) {
                // r^2/L with L = kpc/PX: rr * PX / kpc
                d += (0.5 * (rr * px_mas * INV_KPC_KM) * (1.0 - re_dot_L * re_dot_L / rr)) * INV_C_KMS;
            }
            delay += d;
        }
    }
    // ---- solar system Shapiro (solar_system_shapiro.py:59-124): the Sun, and with
    //      PLANET_SHAPIRO (shapiro == 2) the five planets of :112 summed in that order ----
    if (S.shapiro && !is_bary) {
        double rs = sqrt(t.sun[0] * t.sun[0] + t.sun[1] * t.sun[1] + t.sun[2] * t.sun[2]);
        double rct = t.sun[0] * L[0] + t.sun[1] * L[1] + t.sun[2] * L[2];
        double ds = -2.0 * TSUN * log((rs - rct) * INV_AU_KM);
        if (S.shapiro == 2) {
#pragma unroll 1
            for (int q = 0; q < 5; q++) {
                const double x = t.planet[3 * q], y = t.planet[3 * q + 1], z = t.planet[3 * q + 2];
                const double rp = sqrt(x * x + y * y + z * z);
                const double rcp = x * L[0] + y * L[1] + z * L[2];
                ds += -2.0 * TPLANET[q] * log((rp - rcp) * INV_AU_KM);
            }
        }
        delay += ds;
    }
    // ---- barycentric radio frequency (astrometry.py:359-364) ----
    double bfreq = t.freq;
    if (S.astrometry) {
        double vdl = t.vel[0] * L[0] + t.vel[1] * L[1] + t.vel[2] * L[2];
        bfreq = t.freq * (1.0 - vdl * INV_C_KMS);
    }
    double inv_f2 = 1.0 / (bfreq * bfreq);
    o.inv_f2 = inv_f2;
    // ---- DispersionDM (dispersion_model.py:217-234) ----
    double dt_yr_dm = 0.0;
    if (S.ndm > 0) {
        bool any = false;
        for (int k = 1; k < S.ndm; k++) any |= (pval(P, S.o_DM + 2 * k) != 0.0);
        if (S.o_DMEPOCH >= 0) {
            dd dtd = dd_sub(t.tdb, pdd(P, S.o_DMEPOCH));
            dt_yr_dm = dd_to_d(dtd) * INV_DJY;
        }
        double x = any ? dt_yr_dm : 0.0;
        double dm = pval(P, S.o_DM + 2 * (S.ndm - 1));
        for (int k = S.ndm - 1; k >= 1; k--) dm = dm * x * inv_int(k) + pval(P, S.o_DM + 2 * (k - 1));
        delay += dm * DMCONST * inv_f2;
    }
    // ---- DMX (dispersion_model.py:659-678) ----
    if (S.ndmx > 0) {
        double dmx = 0.0;
        if (t.dmx_a >= 0) dmx += pval(P, S.o_DMX + 2 * t.dmx_a);
        if (t.dmx_b >= 0) dmx += pval(P, S.o_DMX + 2 * t.dmx_b);
        for (int k = t.dmx_x0; k < t.dmx_x1; k++) dmx += pval(P, S.o_DMX + 2 * t.dmx_x[k]);
        delay += dmx * DMCONST * inv_f2;
    }
    // ---- FD (frequency_dependent.py:70-101): formed here, added after the binary delay (the
    //      sum keeps the reference's order) so that the binary columns can be written as soon
    //      as the binary state exists ----
    double logf = 0.0;  // used by FD and its columns only
    double fd = 0.0;
    if (S.nfd > 0) {
        logf = log(bfreq * 1e-3);
        if (!isfinite(logf)) logf = 0.0;
        for (int k = S.nfd; k >= 1; k--) fd = fd * logf + pval(P, S.o_FD + 2 * (k - 1));
        fd *= logf;
    }
    // ---- astrometric design-matrix geometry (astrometry.py:186-212 get_d_delay_quantities),
    //      formed here without the chain factor so that the TOA's position, velocity and Sun
    //      vectors and the pulsar direction die before the binary state is set up (the
    //      binary columns are written while that state is live: the register peak) ----
    double gLON = 0, gLAT = 0, gPMLON = 0, gPMLAT = 0, gPX = 0;
    if (wantM && S.astrometry) {
        // Earth direction angles (era, edec) of the SSB->observatory vector enter only as
        // cos(edec) sin(plon - era), cos(edec) cos(plon - era) and sin(edec): formed from
        // the vector itself, cos(edec) cos(era) = x/r etc. (no atan2/sin/cos per TOA)
        double u[3] = {t.pos[0], t.pos[1], t.pos[2]};
        if (S.astrometry == 2) {
            // earth ecliptic lon/lat via ICRS->PulsarEcliptic (astrometry.py:1034-1055)
            double ue[3] = {u[0], u[1], u[2]};
            icrs_to_ecl(S.obliquity, ue, u);
        }
        const double r_km = sqrt(rr);
        const double ir = r_km > 0.0 ? 1.0 / r_km : 0.0;
        const double ced_sdl = (C.splon * u[0] - C.cplon * u[1]) * ir;
        const double ced_cdl = (C.cplon * u[0] + C.splon * u[1]) * ir;
        const double sed = u[2] * ir;
        const double te_s = S.o_POSEPOCH >= 0 ? dd_to_d(dd_mul_d(dd_sub(t.tdb, pdd(P, S.o_POSEPOCH)), DAYSEC)) : 0.0;
        const double rc = r_km * INV_C_KMS;
        // d_delay_astrometry_d_RAJ / _ELONG, _DECJ / _ELAT, PM partials x te (astrometry.py:536-627, 1067-1170)
        gLON = rc * (ced_sdl * C.cplat) * (S.astrometry == 1 ? HA_RAD : DEG_RAD);
        gLAT = rc * (ced_cdl * C.splat - sed * C.cplat) * DEG_RAD;
        gPMLON = rc * ced_sdl * te_s * MASYR_RADS;
        gPMLAT = rc * (ced_cdl * C.splat - C.cplat * sed) * te_s * MASYR_RADS;
        // d_delay_astrometry_d_PX (astrometry.py:219-249)
        gPX = 0.5 * ((rr - re_dot_L * re_dot_L) * INV_AUC) * MAS_RAD;
    }
    pre.h = {delay, gLON, gLAT, gPMLON, gPMLAT, gPX, inv_f2, dt_yr_dm, logf};
    pre.fd = fd;
    pre.L[0] = L[0];
    pre.L[1] = L[1];
    pre.L[2] = L[2];
}

// the shared head of a spin-only grid (k_eval_head): eval_toa's operations up to the spin part
PD void eval_head(const pint_spec_t& S, const double* P, const InstConst& C, const ToaRow& t, EvalHead& h) {
    EvalOut o;
    EvalPre pre;
    eval_pre(S, P, C, t, o, true, pre);
    h = pre.h;
    if (S.nfd > 0) h.delay += pre.fd;
}

template <int BIN>
PD void eval_toa(const pint_spec_t& S, const double* P, const InstConst& C, const ToaRow& t, EvalOut& o,
                 double* Mb, unsigned r, long ld, const ColRun* runs, int nrun, bool compact) {
    EvalPre pre;
    eval_pre(S, P, C, t, o, Mb != nullptr, pre);
    double delay = pre.h.delay;
    const double* L = pre.L;
    const double fd = pre.fd;
    const double inv_f2 = pre.h.inv_f2, dt_yr_dm = pre.h.dt_yr_dm, logf = pre.h.logf;
    const double gLON = pre.h.gLON, gLAT = pre.h.gLAT, gPMLON = pre.h.gPMLON, gPMLAT = pre.h.gPMLAT, gPX = pre.h.gPX;
    // ---- binary (pulsar_binary.py:457, acc_delay = delay so far) ----
    BinState B;
    B.status = 0;
    if (BIN == 1 || BIN == 3) {
        ell1_setup<BIN == 3>(S, P, C, t.tdb, delay, B);
        delay += B.delay;
    } else if (BIN == 2) {
        ddm_setup(S, P, C, t.tdb, delay, B);
        delay += B.delay;
        if (B.status) o.status = B.status;
    } else if (BIN == 4) {
        bt_setup(S, P, C, t.tdb, delay, B);
        delay += B.delay;
        if (B.status) o.status = B.status;
    } else if (BIN == 5) {
        // obs_pos / psr_pos in the astrometry's frame (pulsar_binary.py:398-416)
        double ko[3] = {t.pos[0], t.pos[1], t.pos[2]}, kp[3] = {L[0], L[1], L[2]};
        if (S.astrometry == 2) {
            icrs_to_ecl(S.obliquity, t.pos, ko);
            icrs_to_ecl(S.obliquity, L, kp);
        }
        ddm_setup<true>(S, P, C, t.tdb, delay, B, ko, kp);
        delay += B.delay;
        if (B.status) o.status = B.status;
    }
    if (S.nfd > 0) delay += fd;
    EvalSpin sp;
    eval_spin_a(S, P, C, t, delay, o, sp);
    const double chain = sp.chain;
    // ---- the binary columns of the design-matrix row, while the binary state is live (it
    //      then dies: ~80 doubles fewer in registers through the phase and the other columns) ----
    if (Mb && BIN != 0) {
        Ell1Grad eg;
        if (BIN == 1 || BIN == 3) ell1_grad<BIN == 3>(B, eg);
        for (int u = 0; u < nrun; u++) {
            const ColRun R = runs[u];
            if (R.kind != PINT_COL_BIN) continue;
            double* colp = Mb + (long)(compact ? R.dcol0 : R.col0) * ld;
            for (int j = 0; j < R.cnt; j++, colp += ld) {
                const int pid = S.col_index[R.col0 + j];
                double d = 0.0;
                if (BIN == 1 || BIN == 3) d = ell1_deriv(B, eg, pid);
                if (BIN == 2) d = ddm_deriv(B, pid);
                if (BIN == 4) d = bt_deriv(B, pid);
                if (BIN == 5) d = ddm_deriv<true>(B, pid);
                colp[r] = chain * d * bin_unit_factor(pid);
            }
        }
    }
    const EvalHead h = {delay, gLON, gLAT, gPMLON, gPMLAT, gPX, inv_f2, dt_yr_dm, logf};
    eval_spin_b<BIN>(S, P, C, t, h, sp, o, Mb, r, ld, runs, nrun, compact);
}

}  // namespace pint
