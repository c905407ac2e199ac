// pg_libm.h -- the C-library math the reference's arithmetic depends on, restated for the device.
//
// (1) pg_atan2f: glibc 2.35's atan2f (sysdeps/ieee754/flt-32/e_atan2f.c + s_atanf.c, the fdlibm
// algorithm with glibc's pi / pi_lo constants), operation by operation in float -- bit-identical to
// the library on 40M+ random arguments and every special case (tests/test_libm_cpu.py).
// Entity::face_direction calls it (entity.cpp:86: std::atan2(float, float) = atan2f).
//
// (2) pg_sincos_cr: correctly rounded double sin / cos for the rotation math (QTransform::rotate,
// Qt5 qtransform.cpp, reached from draw_image, basic-abstract-game.cpp:912-913) and the games'
// float-position steering (caveflyer / starpilot / bossfight / ninja call cos / sin on doubles).
// The reference links glibc, whose sin / cos return the correctly rounded result for the
// arguments these games produce except ~0.15% (off by 1 ulp; tests/test_libm_cpu.py); the
// device's own sin / cos are 1-ulp (3% of matrix entries differed), so the engine evaluates
// both in double-double arithmetic (Cody-Waite reduction with a 4-part pi/2, Taylor series to
// x^29) and rounds once.  Plain C so the same source is compiled for the host in the CPU test.
#pragma once

#ifdef __HIPCC__
#define PG_HD __host__ __device__ static inline
#else
#include <math.h>
#include <stdint.h>
#include <string.h>
#define PG_HD static inline
#endif

PG_HD uint32_t pg_fbits(float f) {
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    return u;
}
PG_HD float pg_bitsf(uint32_t u) {
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}

// s_atanf.c (fdlibm): atan(x) in float with a 4-interval argument reduction
PG_HD float pg_atanf(float x) {
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    const float aT[11] = {3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                          9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                          4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f};
    const int32_t hx = (int32_t)pg_fbits(x), ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) { // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) { // |x| < 0.4375
        if (ix < 0x31000000) return x; // |x| < 2^-29
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000) { // |x| < 1.1875
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    const float z = x * x, w = z * z;
    const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}

// e_atan2f.c (fdlibm, glibc constants pi = 0x40490fdb, pi_lo = -0x1.777a5cp-24)
PG_HD float pg_atan2f(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)pg_fbits(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)pg_fbits(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return pg_atanf(y); // x = 1
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        if (m <= 1) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000 || iy == 0x7f800000) return atan2f(y, x); // infinities: never drawn
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = pg_atanf(fabsf(y / x));
    if (m == 0) return z;
    if (m == 1) return pg_bitsf(pg_fbits(z) ^ 0x80000000u);
    if (m == 2) return pi - (z - pi_lo);
    return (z - pi_lo) - pi;
}

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
