// pg_sincos.h -- correctly rounded double sin / cos for the rotation math (QTransform::rotate,
// Qt5 qtransform.cpp, reached from draw_image, basic-abstract-game.cpp:912-913) and the games'
// float-position steering (caveflyer / starpilot / bossfight / ninja call cos / sin on doubles).
// The reference links glibc, whose sin / cos return the correctly rounded result for the
// arguments these games produce (checked on 8M+ arguments in tests/test_sincos_cpu.py); the
// device's own sin / cos are 1-ulp (3% of matrix entries differed), so the engine evaluates
// both in double-double arithmetic (Cody-Waite reduction with a 4-part pi/2, Taylor series to
// x^29) and rounds once.  Plain C so the same source is compiled for the host in the CPU test.
#pragma once

#ifdef __HIPCC__
#define PG_HD __host__ __device__ static inline
#else
#include <math.h>
#define PG_HD static inline
#endif

typedef struct { double hi, lo; } pg_dd;

PG_HD pg_dd pg_dd_make(double hi, double lo) { pg_dd r; r.hi = hi; r.lo = lo; return r; }
PG_HD pg_dd pg_two_sum(double a, double b) {
    double s = a + b, bb = s - a;
    return pg_dd_make(s, (a - (s - bb)) + (b - bb));
}
PG_HD pg_dd pg_quick_two_sum(double a, double b) {
    double s = a + b;
    return pg_dd_make(s, b - (s - a));
}
PG_HD pg_dd pg_two_prod(double a, double b) {
    double p = a * b;
    return pg_dd_make(p, fma(a, b, -p));
}
PG_HD pg_dd pg_dd_add(pg_dd x, pg_dd y) {
    pg_dd s = pg_two_sum(x.hi, y.hi), t = pg_two_sum(x.lo, y.lo);
    s.lo += t.hi;
    s = pg_quick_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return pg_quick_two_sum(s.hi, s.lo);
}
PG_HD pg_dd pg_dd_mul(pg_dd x, pg_dd y) {
    pg_dd p = pg_two_prod(x.hi, y.hi);
    p.lo += x.hi * y.lo + x.lo * y.hi;
    return pg_quick_two_sum(p.hi, p.lo);
}

// 1 / n! as double-double, n = 0..29 (exact rationals rounded twice)
#define PG_INV_FACT_N 30
PG_HD pg_dd pg_inv_fact(int n) {
    const double h[PG_INV_FACT_N] = {1.0, 1.0, 0.5, 0.16666666666666666, 0.041666666666666664,
        0.008333333333333333, 0.001388888888888889, 0.0001984126984126984, 2.48015873015873e-05,
        2.7557319223985893e-06, 2.755731922398589e-07, 2.505210838544172e-08, 2.08767569878681e-09,
        1.6059043836821613e-10, 1.1470745597729725e-11, 7.647163731819816e-13, 4.779477332387385e-14,
        2.8114572543455206e-15, 1.5619206968586225e-16, 8.22063524662433e-18, 4.110317623312165e-19,
        1.9572941063391263e-20, 8.896791392450574e-22, 3.868170170630684e-23, 1.6117375710961184e-24,
        6.446950284384474e-26, 2.4795962632247976e-27, 9.183689863795546e-29, 3.279889237069838e-30,
        1.1309962886447716e-31};
    const double l[PG_INV_FACT_N] = {0.0, 0.0, 0.0, 9.25185853854297e-18, 2.3129646346357427e-18,
        1.1564823173178714e-19, -5.300543954373577e-20, 1.7209558293420705e-22, 2.1511947866775882e-23,
        -1.858393274046472e-22, 2.3767714622250297e-23, -1.448814070935912e-24, -1.20734505911326e-25,
        1.2585294588752098e-26, 2.0655512752830745e-28, 7.03872877733453e-30, 4.399205485834081e-31,
        1.6508842730861433e-31, 1.1910679660273754e-32, 2.2141894119604265e-34, 1.4412973378659527e-36,
        -1.3643503830087908e-36, -7.911402614872376e-38, -8.843177655482344e-40, -3.6846573564509766e-41,
        -1.9330404233703465e-42, -1.2953730964765229e-43, 1.4303150396787322e-45, 1.5117542744029879e-46,
        1.0498015412959506e-47};
    return pg_dd_make(h[n], l[n]);
}

// sin and cos of x (|x| < 2^20): *s, *c correctly rounded (up to a 2^-100 relative ambiguity)
PG_HD void pg_sincos_cr(double x, double *s, double *c) {
    // pi/2 = P1 + P2 + P3 + P4; P1, P2 carry 33 bits so k * P1, k * P2 are exact for |k| < 2^20
    const double P1 = 1.5707963267341256, P2 = 6.077100506303966e-11;
    const double P3 = 2.0222662487959506e-21, P4 = 1.0085854035872483e-37;
    const double k = nearbyint(x * 0.6366197723675814);
    pg_dd r = pg_two_sum(x - k * P1, -(k * P2));
    r = pg_dd_add(r, pg_two_prod(-k, P3));
    r = pg_dd_add(r, pg_dd_make(-k * P4, 0));
    const pg_dd z = pg_dd_mul(r, r);
    // sin r = r (1 - z/3! + z^2/5! - ...), cos r = 1 - z/2! + z^2/4! - ...
    pg_dd ps = pg_inv_fact(29), pc = pg_inv_fact(28);
    for (int n = 27; n >= 1; n -= 2) {
        pg_dd t = pg_dd_mul(ps, z);
        ps = pg_dd_add(pg_dd_make(-t.hi, -t.lo), pg_inv_fact(n));
        t = pg_dd_mul(pc, z);
        pc = pg_dd_add(pg_dd_make(-t.hi, -t.lo), pg_inv_fact(n - 1));
    }
    // the loop leaves ps = sum (-1)^j z^j / (2j+1)!  (n = 1 term is 1/1!), pc = sum (-1)^j z^j / (2j)!
    const pg_dd sr = pg_dd_mul(ps, r);
    const int q = ((int)fmod(k, 4.0) + 4) & 3;
    double sv = sr.hi + sr.lo, cv = pc.hi + pc.lo;
    if (q == 0) { *s = sv; *c = cv; }
    else if (q == 1) { *s = cv; *c = -sv; }
    else if (q == 2) { *s = -sv; *c = -cv; }
    else { *s = -cv; *c = sv; }
}
