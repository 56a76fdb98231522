/*
 * mh_math.h -- the project's own double-precision transcendentals, compiled unchanged for the
 * device (hipcc, gfx950) and the host (the product's host code, and gcc for the test oracle).
 *
 * The reference computes its transcendentals with CUDA's libdevice (Kernel.cu:173 atan2, :187
 * atan2f, :277 cosf, :712 exp; cuRAND's Box-Muller log / sin / cos behind curand_normal,
 * :605,608,641). Neither libdevice nor cuRAND exists in this image, so any faithful library is
 * as close to the reference as any other -- but the device and the oracle must use the SAME one,
 * or a 1-ulp difference between two libraries (OCML on the device, glibc on the host) can flip a
 * float rounding and fork a chain. Everything here is built only from IEEE-754 operations that
 * are correctly rounded on both sides (+, -, *, /, fma, integer and bit manipulation, exact
 * int <-> double conversions), evaluated in a fixed order (compile with -ffp-contract=off), so
 * host and device return the same bits for every input by construction. tests/test_gpu_math.py
 * checks that exhaustively on MI355X for the 32-bit domains the chains use.
 *
 * The algorithms are fdlibm's (Sun Microsystems, 1993; the FreeBSD msun revisions): argument
 * reduction by ln2 / pi/2 with extra-precise constants, and the published minimax polynomials.
 * Each is within 1 ulp of the exact result (tests/test_math.py measures them against 256-bit
 * arithmetic). Branches select between exact alternatives where fdlibm has shortcuts, so a
 * wavefront rarely diverges.
 *
 * Functions: mh_log, mh_exp, mh_sincos / mh_sin / mh_cos (any finite double: Cody-Waite
 * reduction below 2^20 pi/2, Payne-Hanek with a 1280-bit table of 2/pi above), mh_atan2.
 *
 * fdlibm's notice, preserved as its licence asks (the constants, polynomial coefficients and
 * algorithms below derive from e_log.c, e_exp.c, k_sin.c, k_cos.c, e_rem_pio2.c, k_rem_pio2.c,
 * s_atan.c and e_atan2.c):
 *
 *   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
 *
 *   Developed at SunPro, a Sun Microsystems, Inc. business.
 *   Permission to use, copy, modify, and distribute this
 *   software is freely granted, provided that this notice
 *   is preserved.
 */
#ifndef MH_MATH_H_
#define MH_MATH_H_

#include <stdint.h>

#if defined(__HIP__)
#define MH_MATH_FN static inline __host__ __device__ __attribute__((always_inline))
#define MH_MATH_TABLE static constexpr
#else
#define MH_MATH_FN static inline __attribute__((always_inline))
#define MH_MATH_TABLE static const
#endif
/* A select whose condition varies between lanes: evaluated as a select, never as a branch (clang
 * otherwise turns chains of such ternaries into divergent control flow on the GPU). */
#if defined(__clang__)
#define MH_SEL(c) __builtin_unpredictable(c)
#else
#define MH_SEL(c) (c)
#endif

/* ---- bit access ---------------------------------------------------------------------------- */

MH_MATH_FN uint64_t mh_dbits(double x) {
    uint64_t u;
    __builtin_memcpy(&u, &x, 8);
    return u;
}
MH_MATH_FN double mh_bitsd(uint64_t u) {
    double x;
    __builtin_memcpy(&x, &u, 8);
    return x;
}
MH_MATH_FN uint32_t mh_hiword(double x) { return (uint32_t)(mh_dbits(x) >> 32); }
/* 2^k for -1022 <= k <= 1023, exactly */
MH_MATH_FN double mh_pow2(int k) { return mh_bitsd((uint64_t)(k + 1023) << 52); }
/* the canonical quiet NaN (x86 and AMDGPU differ in the sign of the NaN an invalid operation
 * produces; every NaN returned here is this one) */
MH_MATH_FN double mh_nan(void) { return mh_bitsd(0x7FF8000000000000ull); }

/* ---- log (fdlibm e_log.c) -------------------------------------------------------------------
 * x = 2^k (1 + f), sqrt(2)/2 <= 1 + f < sqrt(2); log(1 + f) = f - hfsq + s (hfsq + R(z)),
 * s = f / (2 + f), z = s^2, R a degree-14 minimax polynomial in s (|error| < 2^-58.45). fdlibm's
 * k == 0 and |f| < 2^-20 shortcuts return the same value as the general formula up to rounding
 * symmetry (x - y == -(y - x)), so they are not taken; its two final forms are both computed
 * and the one fdlibm picks is selected. */
MH_MATH_FN double mh_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    const uint64_t u0 = mh_dbits(x);
    const int32_t hx0 = (int32_t)(u0 >> 32);
    if (hx0 < 0 || hx0 >= 0x7FF00000 || (u0 & 0x7FFFFFFFFFFFFFFFull) == 0) {
        if ((u0 & 0x7FFFFFFFFFFFFFFFull) == 0) return -mh_bitsd(0x7FF0000000000000ull);
        if (hx0 < 0) return mh_nan();
        return (u0 & 0x000FFFFFFFFFFFFFull) || hx0 > 0x7FF00000 ? mh_nan() : x;
    }
    const int sub = hx0 < 0x00100000;            /* subnormal: scale up by 2^54 */
    x = sub ? x * 18014398509481984.0 : x;
    const uint64_t u = mh_dbits(x);
    int32_t hx = (int32_t)(u >> 32);
    int k = (sub ? -54 : 0) + (hx >> 20) - 1023;
    hx &= 0x000FFFFF;
    const int32_t i = (hx + 0x95F64) & 0x100000;
    /* normalise x or x / 2 into [sqrt(2)/2, sqrt(2)) */
    x = mh_bitsd(((uint64_t)(uint32_t)(hx | (i ^ 0x3FF00000)) << 32) | (u & 0xFFFFFFFFull));
    k += i >> 20;
    const double f = x - 1.0;
    const double s = f / (2.0 + f);
    const double dk = (double)k;
    const double z = s * s;
    const double w = z * z;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    const double R = t2 + t1;
    const int32_t sel = (hx - 0x6147A) | (0x6B851 - hx);
    const double hfsq = 0.5 * f * f;
    const double a = dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    const double b = dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
    return sel > 0 ? a : b;
}

/* ---- exp (fdlibm e_exp.c) -------------------------------------------------------------------
 * x = k ln2 + r, |r| <= ln2 / 2 (ln2 in two parts, so hi - lo is r to ~2^-85); exp(r) from the
 * degree-5 Remez approximation R(r^2) of r (e^r + 1) / (e^r - 1) (|error| < 2^-59; Horner with
 * fused multiply-adds), then 2^k. */
MH_MATH_FN double mh_exp(double x) {
    const double o_threshold = 7.09782712893383973096e+02, u_threshold = -7.45133219101941108420e+02;
    const double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
                 invln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    const uint64_t u = mh_dbits(x);
    const uint32_t hx = (uint32_t)(u >> 32) & 0x7FFFFFFFu;
    const int xsb = (int)(u >> 63);
    if (hx >= 0x40862E42u) {                     /* |x| >= 709.78...: inf, NaN, overflow... */
        if (hx >= 0x7FF00000u) {
            if ((u & 0x000FFFFFFFFFFFFFull) || hx > 0x7FF00000u) return mh_nan();
            return xsb ? 0.0 : x;                /* exp(-inf) = 0, exp(+inf) = inf */
        }
        if (x > o_threshold) return mh_bitsd(0x7FF0000000000000ull);
        if (x < u_threshold) return 0.0;
    }
    /* the reduction x = k ln2 + (hi - lo): none for |x| <= ln2 / 2, k = +-1 below 1.5 ln2,
     * k = nearest(x / ln2) above (t * ln2HI is exact there) */
    const int red = hx > 0x3FD62E42u, near1 = hx < 0x3FF0A2B2u;
    const int kn = (int)(invln2 * x + (xsb ? -0.5 : 0.5));
    const int k = !red ? 0 : near1 ? 1 - xsb - xsb : kn;
    const double tk = (double)kn;
    /* (every arm computed beforehand: a ternary with computed arms becomes a branch) */
    const double hp = x + ln2HI, hm = x - ln2HI, hk = x - tk * ln2HI, lk = tk * ln2LO;
    const double h1 = MH_SEL(xsb) ? hp : hm, l1 = MH_SEL(xsb) ? -ln2LO : ln2LO;
    const double h2 = MH_SEL(near1) ? h1 : hk, l2 = MH_SEL(near1) ? l1 : lk;
    const double hi = MH_SEL(red) ? h2 : x, lo = MH_SEL(red) ? l2 : 0.0;
    const double rr = hi - lo;
    const double r = MH_SEL(red) ? rr : x;
    const double t = r * r;
    const double c = __builtin_fma(-t, __builtin_fma(t, __builtin_fma(t, __builtin_fma(t, __builtin_fma(t, P5, P4), P3), P2), P1), r);
    const double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    /* y 2^k: in one step for -1021 <= k < 1024, else in two */
    const double pa = mh_pow2(k < 1023 ? k : 1023), pb = mh_pow2(k + 1000 > -1022 ? k + 1000 : -1022);
    const double fa = MH_SEL(k >= -1021) ? pa : pb;
    const double f1 = MH_SEL(k == 1024) ? 2.0 : fa;
    const double fb = MH_SEL(k >= -1021) ? 1.0 : mh_pow2(-1000);
    const double f2 = MH_SEL(k == 1024) ? mh_pow2(1023) : fb;
    const double e = (y * f1) * f2, e1 = 1.0 + x;
    return MH_SEL(hx < 0x3E300000u) ? e1 : e;    /* |x| < 2^-28 */
}

/* ---- sin and cos ------------------------------------------------------------------------------ */

/* fdlibm k_sin.c / k_cos.c (FreeBSD revision): sin and cos of x + y, |x + y| <= ~pi/4, y the
 * tail of the reduced argument. Minimax polynomials, |error| < 2^-58, evaluated with fused
 * multiply-adds (round 4: fewer operations; the same on both sides, as fma is correctly rounded). */
MH_MATH_FN double mh_ksin(double x, double y) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double z = x * x;
    const double v = z * x;
    const double r = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, S6, S5), S4), S3), S2);
    return x - __builtin_fma(-v, S1, __builtin_fma(z, __builtin_fma(-v, r, 0.5 * y), -y));
}
MH_MATH_FN double mh_kcos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = x * x;
    const double w = z * z;
    const double r = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, C3, C2), C1),
                                   (w * w) * __builtin_fma(z, __builtin_fma(z, C6, C5), C4));
    const double hz = 0.5 * z;
    const double w1 = 1.0 - hz;
    return w1 + (((1.0 - w1) - hz) + __builtin_fma(z, r, -(x * y)));
}

/* 2/pi to 1280 bits: word k holds bits 32k+1 .. 32k+32 after the binary point (generated with
 * 1600-bit arithmetic; tests/test_math.py re-derives it). */
MH_MATH_TABLE uint32_t mh_two_over_pi[40] = {
    0xA2F9836Eu, 0x4E441529u, 0xFC2757D1u, 0xF534DDC0u, 0xDB629599u, 0x3C439041u, 0xFE5163ABu,
    0xDEBBC561u, 0xB7246E3Au, 0x424DD2E0u, 0x06492EEAu, 0x09D1921Cu, 0xFE1DEB1Cu, 0xB129A73Eu,
    0xE88235F5u, 0x2EBB4484u, 0xE99C7026u, 0xB45F7E41u, 0x3991D639u, 0x835339F4u, 0x9C845F8Bu,
    0xBDF9283Bu, 0x1FF897FFu, 0xDE05980Fu, 0xEF2F118Bu, 0x5A0A6D1Fu, 0x6D367ECFu, 0x27CB09B7u,
    0x4F463F66u, 0x9E5FEA2Du, 0x7527BAC7u, 0xEBE5F17Bu, 0x3D0739F7u, 0x8A5292EAu, 0x6BFB5FB1u,
    0x1F8D5D08u, 0x56033046u, 0xFC7B6BABu, 0xF0CFBC20u, 0x9AF4361Du};

/* Word j of 2/pi's bits, zero outside the table (j < 0: the bits before the binary point). */
MH_MATH_FN uint32_t mh_2opi_word(int j) { return j >= 0 && j < 40 ? mh_two_over_pi[j] : 0u; }

/* Payne-Hanek reduction of a finite |x| >= 2^20: x = n pi/2 + (y0 + y1), |y0 + y1| <= pi/4;
 * returns n mod 4. With |x| = M 2^E (M the 53-bit mantissa), bit i of 2/pi (weight 2^-i)
 * contributes M 2^(E - i), a multiple of 4 for i <= E - 2; so x 2/pi mod 4 is M times the 192
 * bits i = E - 1 .. E + 190 (zero for i <= 0), shifted right by 192 -- the bits below the window
 * contribute < 2^-137. The fraction is taken to 128 bits and multiplied by pi/2 in
 * double-double. Every index below is static except the table's, so nothing goes to scratch. */
MH_MATH_FN int mh_rem_pio2_large(double x, double* y0, double* y1) {
    const double PIO2_HI = 1.57079632679489655800e+00, PIO2_LO = 6.12323399573676603587e-17;
    const uint64_t u = mh_dbits(x);
    const uint64_t M = (u & 0x000FFFFFFFFFFFFFull) | 0x0010000000000000ull;
    const int E = (int)((u >> 52) & 0x7FF) - 1075;   /* |x| = M 2^E, E >= -32 */
    const int im1 = E - 2;                           /* (first bit i0 = E - 1) - 1 */
    const int w0 = im1 >> 5, s = im1 & 31;           /* (floor division) */
    const uint32_t W0 = mh_2opi_word(w0), W1 = mh_2opi_word(w0 + 1), W2 = mh_2opi_word(w0 + 2),
                   W3 = mh_2opi_word(w0 + 3), W4 = mh_2opi_word(w0 + 4), W5 = mh_2opi_word(w0 + 5),
                   W6 = mh_2opi_word(w0 + 6);
#define MH_FUNNEL(a, b) (s ? (uint32_t)(((a) << s) | ((b) >> (32 - s))) : (a))
    /* the window G, least significant word first */
    const uint32_t g0 = MH_FUNNEL(W5, W6), g1 = MH_FUNNEL(W4, W5), g2 = MH_FUNNEL(W3, W4),
                   g3 = MH_FUNNEL(W2, W3), g4 = MH_FUNNEL(W1, W2), g5 = MH_FUNNEL(W0, W1);
#undef MH_FUNNEL
    const uint32_t m0 = (uint32_t)M, m1 = (uint32_t)(M >> 32);
    /* P = M G (245 bits) in 32-bit limbs, schoolbook: row m0, then row m1 one limb up; only
     * limbs 0..5 are needed. x 2/pi = P 2^(E - i0 - 191) = P 2^-190: bits 190, 191 are n mod 4,
     * bits 62..189 the fraction. */
    uint64_t t;
    t = (uint64_t)m0 * g0;                uint32_t p0 = (uint32_t)t;
    t = (uint64_t)m0 * g1 + (t >> 32);    uint32_t p1 = (uint32_t)t;
    t = (uint64_t)m0 * g2 + (t >> 32);    uint32_t p2 = (uint32_t)t;
    t = (uint64_t)m0 * g3 + (t >> 32);    uint32_t p3 = (uint32_t)t;
    t = (uint64_t)m0 * g4 + (t >> 32);    uint32_t p4 = (uint32_t)t;
    t = (uint64_t)m0 * g5 + (t >> 32);    uint32_t p5 = (uint32_t)t;
    t = (uint64_t)m1 * g0 + p1;              p1 = (uint32_t)t;
    t = (uint64_t)m1 * g1 + p2 + (t >> 32);  p2 = (uint32_t)t;
    t = (uint64_t)m1 * g2 + p3 + (t >> 32);  p3 = (uint32_t)t;
    t = (uint64_t)m1 * g3 + p4 + (t >> 32);  p4 = (uint32_t)t;
    t = (uint64_t)m1 * g4 + p5 + (t >> 32);  p5 = (uint32_t)t;
    const uint64_t H = ((uint64_t)p5 << 32) | p4, Mi = ((uint64_t)p3 << 32) | p2,
                   Lo = ((uint64_t)p1 << 32) | p0;
    int q = (int)(H >> 62);
    uint64_t f1 = (H << 2) | (Mi >> 62), f2 = (Mi << 2) | (Lo >> 62);
    int neg = 0;
    if (f1 >> 63) {                                  /* fraction >= 1/2: n + 1, fraction - 1 */
        q = (q + 1) & 3;
        neg = 1;
        f1 = ~f1;
        f2 = ~f2 + 1u;
        if (f2 == 0) f1 += 1u;
    }
    if (f1 == 0) {                                   /* (unreachable for finite doubles: the
                                                        closest one to a multiple of pi/2 is
                                                        ~2^-61 away) */
        *y0 = 0.0;
        *y1 = 0.0;
        return q;
    }
    const int z = __builtin_clzll(f1);
    if (z) {
        f1 = (f1 << z) | (f2 >> (64 - z));
        f2 <<= z;
    }
    const double hi = (double)(f1 >> 11) * mh_pow2(-53 - z);
    const double lo = (double)(((f1 & 0x7FFu) << 42) | (f2 >> 22)) * mh_pow2(-106 - z);
    const double ph = hi * PIO2_HI;
    double pe = __builtin_fma(hi, PIO2_HI, -ph);
    pe = pe + (hi * PIO2_LO + lo * PIO2_HI);
    double r0 = ph + pe;
    double r1 = pe - (r0 - ph);
    if (neg) {
        r0 = -r0;
        r1 = -r1;
    }
    if (u >> 63) {
        r0 = -r0;
        r1 = -r1;
        q = (4 - q) & 3;
    }
    *y0 = r0;
    *y1 = r1;
    return q;
}

/* Reduction of |x| <= 2^20 pi/2 (fdlibm e_rem_pio2.c's "medium" case): x = n pi/2 + (y0 + y1),
 * returns n mod 4. n = nearest(x 2/pi) and pi/2 in 33 + 33 + 33 + 53 bits, the second and third
 * terms used only when the first cancels more than 16 / 49 bits. */
MH_MATH_FN int mh_rem_pio2_medium(double x, double* y0, double* y1) {
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                 pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
                 pio2_3t = 8.47842766036889956997e-32;
    const uint32_t ix = mh_hiword(x) & 0x7FFFFFFFu;
    double fn = x * invpio2 + 6755399441055744.0;    /* round to nearest integer (|.| < 2^51) */
    fn = fn - 6755399441055744.0;
    const int n = (int)fn;
    double r = x - fn * pio2_1;                      /* exact */
    double w = fn * pio2_1t;
    double y = r - w;
    const int j = (int)(ix >> 20);
    int i = j - (int)((mh_hiword(y) >> 20) & 0x7FF);
    if (i > 16) {
        double t = r;
        w = fn * pio2_2;
        r = t - w;
        w = fn * pio2_2t - ((t - r) - w);
        y = r - w;
        i = j - (int)((mh_hiword(y) >> 20) & 0x7FF);
        if (i > 49) {
            t = r;
            w = fn * pio2_3;
            r = t - w;
            w = fn * pio2_3t - ((t - r) - w);
            y = r - w;
        }
    }
    *y0 = y;
    *y1 = (r - y) - w;
    return n & 3;
}

/* sin and cos of the reduced argument in quadrant n */
MH_MATH_FN void mh_sincos_q(int n, double y0, double y1, double* s, double* c) {
    const double ks = mh_ksin(y0, y1), kc = mh_kcos(y0, y1);
    const double nks = -ks, nkc = -kc;
    const double s01 = MH_SEL(n == 0) ? ks : kc, s23 = MH_SEL(n == 2) ? nks : nkc;
    const double c01 = MH_SEL(n == 0) ? kc : nks, c23 = MH_SEL(n == 2) ? nkc : ks;
    *s = MH_SEL(n < 2) ? s01 : s23;
    *c = MH_SEL(n < 2) ? c01 : c23;
}

/* sin and cos of |x| <= 2^20 pi/2: the Box-Muller angles, which lie in (0, 2 pi] (the same values
 * mh_sincos returns there, without the large-argument code). */
MH_MATH_FN void mh_sincos_medium(double x, double* s, double* c) {
    double y0, y1;
    const int n = mh_rem_pio2_medium(x, &y0, &y1);
    mh_sincos_q(n, y0, y1, s, c);
}

MH_MATH_FN void mh_sincos(double x, double* s, double* c) {
    const uint32_t ix = mh_hiword(x) & 0x7FFFFFFFu;
    if (ix >= 0x7FF00000u) {  /* inf, NaN */
        *s = mh_nan();
        *c = mh_nan();
        return;
    }
    double y0, y1;
    /* the medium reduction always (of 0 above its range), the large one only where needed */
    int n = mh_rem_pio2_medium(ix > 0x413921FBu ? 0.0 : x, &y0, &y1);
    if (ix > 0x413921FBu) n = mh_rem_pio2_large(x, &y0, &y1);
    mh_sincos_q(n, y0, y1, s, c);
}

MH_MATH_FN double mh_sin(double x) {
    double s, c;
    mh_sincos(x, &s, &c);
    return s;
}

MH_MATH_FN double mh_cos(double x) {
    double s, c;
    mh_sincos(x, &s, &c);
    return c;
}

/* ---- atan2 (fdlibm s_atan.c, e_atan2.c) ----------------------------------------------------
 * atan(|t|): the argument reduced to |t'| < 7/16 against atan(0.5), atan(1), atan(1.5) or
 * pi/2 (each in two parts), then t' - t' (s1 + s2), an odd degree-23 minimax polynomial.
 * fdlibm's five-way branch is written as selects of the one division's numerator and
 * denominator (t' = t / 1 exactly for |t| < 7/16), so a wavefront computes one reduction
 * whatever mix of ranges its lanes hold; the values are fdlibm's. */
MH_MATH_FN double mh_atan(double x) {
    const double atanhi0 = 4.63647609000806093515e-01, atanhi1 = 7.85398163397448278999e-01,
                 atanhi2 = 9.82793723247329054082e-01, atanhi3 = 1.57079632679489655800e+00;
    const double atanlo0 = 2.26987774529616870924e-17, atanlo1 = 3.06161699786838301793e-17,
                 atanlo2 = 1.39033110312309984516e-17, atanlo3 = 6.12323399573676603587e-17;
    const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
                 aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
                 aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
                 aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
                 aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
                 aT10 = 1.62858201153657823623e-02;
    const uint64_t u = mh_dbits(x);
    const uint32_t ix = (uint32_t)(u >> 32) & 0x7FFFFFFFu;
    const int neg = (int)(u >> 63);
    if (ix >= 0x7FF00000u && (ix > 0x7FF00000u || (u & 0xFFFFFFFFull))) return mh_nan();
    const double ax = __builtin_fabs(x);
    /* id: -1 below 7/16, 0 below 11/16, 1 below 19/16, 2 below 39/16, 3 above */
    const int id = ix < 0x3FDC0000u ? -1 : ix < 0x3FE60000u ? 0 : ix < 0x3FF30000u ? 1
                 : ix < 0x40038000u ? 2 : 3;
    const double num = id < 0 ? x : id == 0 ? 2.0 * ax - 1.0 : id == 1 ? ax - 1.0
                     : id == 2 ? ax - 1.5 : -1.0;
    const double den = id < 0 ? 1.0 : id == 0 ? 2.0 + ax : id == 1 ? ax + 1.0
                     : id == 2 ? 1.0 + 1.5 * ax : ax;
    const double t = num / den;
    const double hi = id < 0 ? 0.0 : id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
    const double lo = id < 0 ? 0.0 : id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
    const double z = t * t;
    const double w = z * z;
    const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    const double small = t - t * (s1 + s2);               /* |x| < 7/16 (t == x) */
    const double r = hi - ((t * (s1 + s2) - lo) - t);
    const double big = neg ? -r : r;
    return ix < 0x3E400000u ? x                           /* |x| < 2^-27 */
         : ix >= 0x44100000u ? (neg ? -(atanhi3 + atanlo3) : atanhi3 + atanlo3)  /* >= 2^66 */
         : id < 0 ? small : big;
}

/* atan(a / b) for finite a, b > 0 (hm: the larger high word), with one division: fdlibm's
 * reduction of t = a / b, (t - c) / (1 + c t), applied to the operands as (a - c b) / (b + c a)
 * (exact numerators by Sterbenz for c = 1/2, 1; one fma rounding for c = 3/2), then fdlibm's
 * polynomial (Horner with fused multiply-adds) and atanhi/atanlo. The interval of t is chosen by comparing a with multiples of b
 * (either interval is accurate near a boundary). Operands near overflow or in the subnormal
 * range are scaled by a power of two first, which leaves the ratio unchanged. */
MH_MATH_FN double mh_atan_ratio(double a, double b, uint32_t hm) {
    const double atanhi0 = 4.63647609000806093515e-01, atanhi1 = 7.85398163397448278999e-01,
                 atanhi2 = 9.82793723247329054082e-01, atanhi3 = 1.57079632679489655800e+00;
    const double atanlo0 = 2.26987774529616870924e-17, atanlo1 = 3.06161699786838301793e-17,
                 atanlo2 = 1.39033110312309984516e-17, atanlo3 = 6.12323399573676603587e-17;
    const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
                 aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
                 aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
                 aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
                 aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
                 aT10 = 1.62858201153657823623e-02;
    const double sc = hm >= 0x7FC00000u ? 0.25 : hm < 0x00300000u ? 0x1p54 : 1.0;
    a = a * sc;
    b = b * sc;
    /* id: -1 for t below 7/16, 0 below 11/16, 1 below 19/16, 2 below 39/16, 3 above (the
     * products are monotonic in the constant, so the comparisons can be summed);
     * num = na a - nb b, den = nb a + na b (na in {0, 1}: the products are exact) */
    const int id = -1 + (a >= 0.4375 * b) + (a >= 0.6875 * b) + (a >= 1.1875 * b) + (a >= 2.4375 * b);
    const int e3 = id == 3;
    const double nb = MH_SEL(e3) ? 1.0 : 0.5 * (double)(id + 1);  /* 0, 1/2, 1, 3/2, 1 */
    const double na = MH_SEL(e3) ? 0.0 : 1.0;
    const double t = __builtin_fma(-nb, b, na * a) / __builtin_fma(nb, a, na * b);
    /* (every arm a value computed beforehand: a ternary with computed arms becomes a branch) */
    const double h0 = MH_SEL(id < 0) ? 0.0 : atanhi0, h1 = MH_SEL(id < 2) ? atanhi1 : atanhi2;
    const double h2 = MH_SEL(id < 3) ? h1 : atanhi3, hi = MH_SEL(id < 1) ? h0 : h2;
    const double l0 = MH_SEL(id < 0) ? 0.0 : atanlo0, l1 = MH_SEL(id < 2) ? atanlo1 : atanlo2;
    const double l2 = MH_SEL(id < 3) ? l1 : atanlo3, lo = MH_SEL(id < 1) ? l0 : l2;
    const double z = t * t;
    const double w = z * z;
    const double s1 = z * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, aT10, aT8), aT6), aT4), aT2), aT0);
    const double s2 = w * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, aT9, aT7), aT5), aT3), aT1);
    const double q = s1 + s2;
    const double rs = __builtin_fma(-t, q, t), rb = hi - (__builtin_fma(t, q, -lo) - t);
    return MH_SEL(id < 0) ? rs : rb;
}

/* atan2 (e_atan2.c): the special operands (NaN, zeros, infinities) on a branch of their own;
 * the general case as selects over atan(|y / x|). (fdlibm's x == 1 shortcut, atan(y), returns
 * the general case's value -- for |y| > 2^60 both round to pi/2 -- so it is not taken.) */
MH_MATH_FN double mh_atan2(double y, double x) {
    const double pi_o_4 = 7.8539816339744827900e-01, pi_o_2 = 1.5707963267948965580e+00,
                 pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
    const uint64_t ux = mh_dbits(x), uy = mh_dbits(y);
    const uint32_t ix = (uint32_t)(ux >> 32) & 0x7FFFFFFFu, iy = (uint32_t)(uy >> 32) & 0x7FFFFFFFu;
    const uint32_t lx = (uint32_t)ux, ly = (uint32_t)uy;
    const int m = (int)(uy >> 63) | ((int)(ux >> 63) << 1);  /* 2 sign(x) + sign(y) */
    if (ix >= 0x7FF00000u || iy >= 0x7FF00000u || (ix | lx) == 0 || (iy | ly) == 0) {
        if ((ix | ((lx | (0u - lx)) >> 31)) > 0x7FF00000u ||
            (iy | ((ly | (0u - ly)) >> 31)) > 0x7FF00000u)
            return mh_nan();                     /* x or y is NaN */
        if ((iy | ly) == 0) {                    /* y == 0 */
            if (m < 2) return y;                 /* atan(+-0, +anything) = +-0 */
            return m == 2 ? pi : -pi;            /* atan(+-0, -anything) = +-pi */
        }
        if ((ix | lx) == 0) return (m & 1) ? -pi_o_2 : pi_o_2;
        if (ix == 0x7FF00000u) {                 /* x is +-inf */
            if (iy == 0x7FF00000u) {
                switch (m) {
                    case 0: return pi_o_4;
                    case 1: return -pi_o_4;
                    case 2: return 3.0 * pi_o_4;
                    default: return -3.0 * pi_o_4;
                }
            }
            switch (m) {
                case 0: return 0.0;
                case 1: return -0.0;
                case 2: return pi;
                default: return -pi;
            }
        }
        return (m & 1) ? -pi_o_2 : pi_o_2;       /* y is +-inf */
    }
    const int k = ((int)iy - (int)ix) >> 20;
    const int big = k > 60;                                  /* |y / x| > 2^60 */
    const int tiny = !big && (ux >> 63) && k < -60;          /* 0 > |y| / x > -2^-60 */
    const double at = mh_atan_ratio(__builtin_fabs(y), __builtin_fabs(x), ix > iy ? ix : iy);
    const double zt = MH_SEL(tiny) ? 0.0 : at;
    const double z = MH_SEL(big) ? pi_o_2 + 0.5 * pi_lo : zt;
    const int mm = big ? (m & 1) : m;
    const double zn = -z, zl = z - pi_lo;
    const double q2 = pi - zl, q3 = zl - pi;
    const double r01 = MH_SEL(mm == 0) ? z : zn, r23 = MH_SEL(mm == 2) ? q2 : q3;
    return MH_SEL(mm < 2) ? r01 : r23;
}

/* ---- the float functions of the reference ----------------------------------------------------
 * atan2f in phi (Kernel.cu:187) and cosf in FocalPointCosts (:277): the double function
 * rounded once to float (the correctly rounded float value but in ~2^-29 of cases). */
MH_MATH_FN float mh_atan2_f32(float y, float x) { return (float)mh_atan2((double)y, (double)x); }
MH_MATH_FN float mh_cos_f32(float x) { return (float)mh_cos((double)x); }

/* ---- arguments of the sampled numerics checks (tests/test_gpu_math.py) -------------------------
 * The device diagnostic (mh_debug_math) and the oracle generate the same argument i of each
 * sampled check from this counter-based generator, so nothing is transferred to the device. */
MH_MATH_FN uint64_t mh_mix64(uint64_t z) {  /* splitmix64's finaliser */
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
/* A float in [0, w): the coordinates of a synthetic room of width w. */
MH_MATH_FN float mh_arg_coord(uint64_t h, float w) { return (float)(h >> 40) * 0x1p-24f * w; }
/* The (y, x) argument pair i of atan2 sample `kind`: 0, theta's and phi's float differences of
 * two room coordinates (Kernel.cu:173,187, rooms of width 20 and 40: configs 3 and 5); 1, any two
 * float bit patterns. */
MH_MATH_FN void mh_arg_atan2(uint64_t i, int kind, float* y, float* x) {
    const uint64_t a = mh_mix64(i * 4 + 1), b = mh_mix64(i * 4 + 2), c = mh_mix64(i * 4 + 3),
                   d = mh_mix64(i * 4 + 4);
    if (kind == 0) {
        const float w = (a & 1) ? 40.0f : 20.0f;
        *y = mh_arg_coord(a, w) - mh_arg_coord(b, w);
        *x = mh_arg_coord(c, w) - mh_arg_coord(d, w);
    } else {
        uint32_t by = (uint32_t)a, bx = (uint32_t)c;
        __builtin_memcpy(y, &by, 4);
        __builtin_memcpy(x, &bx, 4);
    }
}
/* The exp argument i of Accept (Kernel.cu:712): BETA (star - cur) with cur a float total of
 * magnitude up to 2^15 and star = cur + d, |d| = 2^U(-24, 7) (kind 0); any double from a float
 * pair's difference (kind 1). */
MH_MATH_FN double mh_arg_exp(uint64_t i, int kind) {
    const uint64_t a = mh_mix64(i * 2 + 11), b = mh_mix64(i * 2 + 12);
    if (kind == 0) {
        const float cur = ((float)(a >> 40) * 0x1p-24f - 0.5f) * 65536.0f;
        const int e = (int)((b >> 58) % 31u) - 24;
        float d = (float)((b >> 20) & 0xFFFFFu) * 0x1p-20f * (float)mh_pow2(e);
        d = (b & 1) ? -d : d;
        const float star = cur + d;
        return 2.0 * ((double)star - (double)cur);
    }
    const float p = ((float)(a >> 40) * 0x1p-24f - 0.5f) * 2048.0f;
    const float q = ((float)(b >> 40) * 0x1p-24f - 0.5f) * 2048.0f;
    return (double)p - (double)q;
}

/* Accept's decision u < min(1, (float)exp(x)) (Kernel.cu:712), the reference's way: x >= 0
 * gives a threshold of exactly 1, x < -24 one below every uniform either stream draws (>= 2^-33),
 * otherwise the double exp rounded to float. The device decides most draws with an fp32 screen
 * instead (mh_common.h accept_u); the probe below checks the two agree. */
MH_MATH_FN int mh_accept_exact(float u, double x) {
    if (x >= 0.0) return u < 1.0f;
    if (x < -24.0) return 0;
    const float e = (float)mh_exp(x);
    return u < (e < 1.0f ? e : 1.0f);
}

/* Arguments of the accept probe: a (0, 1] uniform as rocRAND converts a word, and x = BETA
 * (star - cur) either within 1e-4 of log(u) (three in four: the band the screen must resolve
 * exactly) or anywhere in [-30, 2]. */
MH_MATH_FN void mh_arg_accept(uint64_t i, float* u, double* x) {
    const uint64_t a = mh_mix64(i * 2 + 21), b = mh_mix64(i * 2 + 22);
    *u = (float)(uint32_t)a * 0x1p-32f + 0x1p-33f;
    if ((b & 3u) != 0u) {
        const double t = ((double)(int32_t)(uint32_t)(b >> 32) * 0x1p-31) * 1e-4;
        *x = mh_log((double)*u) + t;
    } else {
        *x = (double)(b >> 11) * 0x1p-53 * 32.0 - 30.0;
    }
}

/* The numerics checks: probe `fn` at argument index i, the results as doubles (float results
 * widened exactly) in out[0] (and out[1] for the sincos probes). Exhaustive probes take i over
 * all 2^32 values; sampled ones over any range. */
enum {
    MH_PROBE_BM_LOG = 0,     /* log(a 2^-32 + 2^-33), Box-Muller's radius (mh_common.h) */
    MH_PROBE_BM_SINCOS = 1,  /* sincos(2pi (b 2^-32 + 2^-33)), Box-Muller's angle */
    MH_PROBE_COS_F32 = 2,    /* cosf of the float with bit pattern i (FocalPoint, Kernel.cu:277) */
    MH_PROBE_XW_LOG = 3,     /* (float)log((double)u), u = x 2^-32 + 2^-33 in float (cuRAND's) */
    MH_PROBE_XW_SINCOS = 4,  /* sincos((double)v), v = fmaf(y, 2^-32 2pi, half of that) */
    MH_PROBE_ATAN2_ROOM = 5, /* double atan2 of room coordinate differences (theta, :173) */
    MH_PROBE_ATAN2_BITS = 6, /* double atan2 of any two floats */
    MH_PROBE_ATAN2F_ROOM = 7,/* atan2f of room coordinate differences (phi, :187) */
    MH_PROBE_ATAN2F_BITS = 8,
    MH_PROBE_EXP_ACCEPT = 9, /* exp(BETA (star - cur)) (Accept, :712) */
    MH_PROBE_EXP_ANY = 10,
    MH_PROBE_ACCEPT = 11,    /* Accept's decision, 1 or 0 (the device: its fp32 screen, :712) */
    MH_PROBE_COUNT = 12
};
MH_MATH_FN int mh_probe_width(int fn) {
    return fn == MH_PROBE_BM_SINCOS || fn == MH_PROBE_XW_SINCOS ? 2 : 1;
}
MH_MATH_FN void mh_math_probe(int fn, uint64_t i, double* out) {
    const uint32_t w = (uint32_t)i;
    float y, x;
    switch (fn) {
        case MH_PROBE_BM_LOG:
            out[0] = mh_log((double)w * 0x1p-32 + 0x1p-33);
            break;
        case MH_PROBE_BM_SINCOS:
            mh_sincos_medium(6.283185307179586 * ((double)w * 0x1p-32 + 0x1p-33), &out[0], &out[1]);
            break;
        case MH_PROBE_COS_F32: {
            float v;
            __builtin_memcpy(&v, &w, 4);
            out[0] = (double)mh_cos_f32(v);
            break;
        }
        case MH_PROBE_XW_LOG:
            out[0] = (double)(float)mh_log((double)((float)w * 0x1p-32f + 0x1p-32f * 0.5f));
            break;
        case MH_PROBE_XW_SINCOS: {
            const float k = 0x1p-32f * 6.2831855f;
            mh_sincos_medium((double)__builtin_fmaf((float)w, k, k * 0.5f), &out[0], &out[1]);
            break;
        }
        case MH_PROBE_ATAN2_ROOM:
        case MH_PROBE_ATAN2_BITS:
            mh_arg_atan2(i, fn == MH_PROBE_ATAN2_BITS, &y, &x);
            out[0] = mh_atan2((double)y, (double)x);
            break;
        case MH_PROBE_ATAN2F_ROOM:
        case MH_PROBE_ATAN2F_BITS:
            mh_arg_atan2(i, fn == MH_PROBE_ATAN2F_BITS, &y, &x);
            out[0] = (double)mh_atan2_f32(y, x);
            break;
        case MH_PROBE_EXP_ACCEPT:
        case MH_PROBE_EXP_ANY:
            out[0] = mh_exp(mh_arg_exp(i, fn == MH_PROBE_EXP_ANY));
            break;
        case MH_PROBE_ACCEPT: {
            float u;
            double xa;
            mh_arg_accept(i, &u, &xa);
            out[0] = mh_accept_exact(u, xa) ? 1.0 : 0.0;
            break;
        }
        default:
            out[0] = mh_nan();
            break;
    }
}

#endif /* MH_MATH_H_ */
