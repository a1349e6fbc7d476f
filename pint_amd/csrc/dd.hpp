// dd.hpp — double-double arithmetic (pairs of FP64) used where the reference computes in
// numpy longdouble (80-bit x87): pulse phase (spindown.py:141 via utils.py:419
// taylor_horner), dt = (tdbld - PEPOCH)*86400 - delay (spindown.py:124), binary tt0 / orbit
// count (binary_generic.py:372, binary_orbits.py:98).  dd carries ~106 mantissa bits, a
// superset of longdouble's 64, so the restated values are at least as precise as the
// reference's (SURVEY.md §0 finding 3).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#define PD __host__ __device__ __forceinline__
// Error-free transformations must not be contracted: hipcc's device default is
// -ffp-contract=fast, which would fuse the product inside two_prod with a later add
// (after inlining) and destroy the exact error term.  Every dd routine opts out.
#define DD_NOCONTRACT _Pragma("clang fp contract(off)")

struct dd {
    double hi, lo;
};

PD dd dd_make(double h, double l = 0.0) { dd r; r.hi = h; r.lo = l; return r; }

PD dd two_sum(double a, double b) {
    DD_NOCONTRACT
    double s = a + b;
    double bb = s - a;
    double e = (a - (s - bb)) + (b - bb);
    return dd_make(s, e);
}
PD dd quick_two_sum(double a, double b) {
    DD_NOCONTRACT
    double s = a + b;
    double e = b - (s - a);
    return dd_make(s, e);
}
PD dd two_prod(double a, double b) {
    DD_NOCONTRACT
    double p = a * b;
    double e = fma(a, b, -p);
    return dd_make(p, e);
}
PD dd dd_add(dd a, dd b) {
    DD_NOCONTRACT
    dd s = two_sum(a.hi, b.hi);
    dd t = two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = quick_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return quick_two_sum(s.hi, s.lo);
}
PD dd dd_neg(dd a) { return dd_make(-a.hi, -a.lo); }
PD dd dd_sub(dd a, dd b) { return dd_add(a, dd_neg(b)); }
PD dd dd_add_d(dd a, double b) {
    DD_NOCONTRACT
    dd s = two_sum(a.hi, b);
    s.lo += a.lo;
    return quick_two_sum(s.hi, s.lo);
}
PD dd dd_mul(dd a, dd b) {
    DD_NOCONTRACT
    dd p = two_prod(a.hi, b.hi);
    p.lo += a.hi * b.lo + a.lo * b.hi;
    return quick_two_sum(p.hi, p.lo);
}
PD dd dd_mul_d(dd a, double b) {
    DD_NOCONTRACT
    dd p = two_prod(a.hi, b);
    p.lo += a.lo * b;
    return quick_two_sum(p.hi, p.lo);
}
PD dd dd_div_d(dd a, double b) {
    DD_NOCONTRACT
    double q1 = a.hi / b;
    dd p = two_prod(q1, b);
    dd r = dd_sub(a, p);
    double q2 = r.hi / b;
    p = two_prod(q2, b);
    r = dd_sub(r, p);
    double q3 = r.hi / b;
    dd q = quick_two_sum(q1, q2);
    return dd_add_d(q, q3);
}
PD dd dd_div(dd a, dd b) {
    DD_NOCONTRACT
    double q1 = a.hi / b.hi;
    dd r = dd_sub(a, dd_mul_d(b, q1));
    double q2 = r.hi / b.hi;
    r = dd_sub(r, dd_mul_d(b, q2));
    double q3 = r.hi / b.hi;
    dd q = quick_two_sum(q1, q2);
    return dd_add_d(q, q3);
}
PD double dd_to_d(dd a) { return a.hi + a.lo; }
// floor of a dd value, as a dd (exact integer)
PD dd dd_floor(dd a) {
    DD_NOCONTRACT
    double fh = floor(a.hi);
    if (fh == a.hi) {
        double fl = floor(a.lo);
        return quick_two_sum(fh, fl);
    }
    return dd_make(fh, 0.0);
}
// nearest integer with ties going up, i.e. frac in [-0.5, 0.5) (phase.py:73-87)
PD dd dd_round_half_up(dd a) { return dd_floor(dd_add_d(a, 0.5)); }
