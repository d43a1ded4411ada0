/*
 * mz_detmath.h — the numerics contract shared by the HIP engine (device code,
 * hipcc/gfx950) and the CPU oracle (gcc).  Every function here is built only
 * from IEEE-754 operations that are correctly rounded on both x86-64 and
 * gfx950 (+ - * / sqrt fma, exact conversions, comparisons), evaluated in a
 * fixed order with floating-point contraction disabled.  Host and device
 * therefore produce bit-identical results, which is what lets the GPU MCTS
 * reproduce the oracle's tree indices and actions bit-exactly.
 *
 * Contents
 *   - det_expf / det_tanhf / det_logf (f32 results), det_exp / det_log (f64)
 *     — accuracy ≤ 2 ulp vs libm (tested in tests/test_detmath.py);
 *   - Philox4x32-10 counter-based RNG and the stream layout of the engine;
 *   - the Gamma / Dirichlet sampler used by add_exploration_noise!
 *     (reference: src/SelfPlay.jl:102-109, Distributions 0.25.6 Dirichlet).
 *
 * Both compilers must be invoked with -ffp-contract=off (see Makefiles); the
 * pragmas below repeat that for clang.
 */
#ifndef MZ_DETMATH_H
#define MZ_DETMATH_H

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define MZ_HD __host__ __device__ __forceinline__
#else
#define MZ_HD static inline
#endif

#ifdef __clang__
#pragma clang fp contract(off)
#endif

/* ------------------------------------------------------------------ bits */
MZ_HD float mz_u2f(uint32_t u) { union { uint32_t u; float f; } c; c.u = u; return c.f; }
MZ_HD uint32_t mz_f2u(float f) { union { uint32_t u; float f; } c; c.f = f; return c.u; }
MZ_HD double mz_u2d(uint64_t u) { union { uint64_t u; double d; } c; c.u = u; return c.d; }
MZ_HD uint64_t mz_d2u(double d) { union { uint64_t u; double d; } c; c.d = d; return c.u; }

/* 2^k as a float for k in [-126, 127] (normal range only). */
MZ_HD float mz_pow2f(int k) { return mz_u2f((uint32_t)(k + 127) << 23); }
/* 2^k as a double for k in [-1022, 1023]. */
MZ_HD double mz_pow2d(int k) { return mz_u2d((uint64_t)(k + 1023) << 52); }

/* round-half-even to an integral value: rintf/rint are exact IEEE operations
 * in the default rounding mode on both targets (v_rndne_f32/f64, SSE/libm). */
MZ_HD float mz_rintf(float x) { return rintf(x); }
MZ_HD double mz_rint(double x) { return rint(x); }

/* ------------------------------------------------------------- det_expf
 * exp(x) in f32: k = rint(x·log2e), r = x − k·ln2 (two-constant Cody-Waite,
 * fmaf), degree-7 Taylor in Horner/fmaf form, scaled by 2^k in two exact
 * steps so that subnormal results round the same way on both targets.   */
MZ_HD float det_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283935546875f) return INFINITY;
    if (x < -103.97208404541016f) return 0.0f;
    float kf = mz_rintf(x * 1.44269502162933349609375f);
    float r = fmaf(-kf, 0.693145751953125f, x);
    r = fmaf(-kf, 1.428606765330187045e-06f, r);
    float p = 1.98412698412698412698e-04f;          /* 1/5040 */
    p = fmaf(p, r, 1.38888888888888888889e-03f);    /* 1/720  */
    p = fmaf(p, r, 8.33333333333333333333e-03f);    /* 1/120  */
    p = fmaf(p, r, 4.16666666666666666667e-02f);    /* 1/24   */
    p = fmaf(p, r, 1.66666666666666666667e-01f);    /* 1/6    */
    p = fmaf(p, r, 0.5f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    int k = (int)kf;
    int k1 = k / 2, k2 = k - k1;
    return (p * mz_pow2f(k1)) * mz_pow2f(k2);
}

/* -------------------------------------------------------------- det_exp */
MZ_HD double det_exp(double x) {
    if (x != x) return x;
    if (x > 709.782712893384) return INFINITY;
    if (x < -745.1332191019412) return 0.0;
    double kd = mz_rint(x * 1.4426950408889634074);
    double r = fma(-kd, 6.93147180369123816490e-01, x);
    r = fma(-kd, 1.90821492927058770002e-10, r);
    /* Taylor to degree 13 (|r| <= 0.3466: truncation < 5e-18) */
    double p = 1.0 / 6227020800.0;       /* 1/13! */
    p = fma(p, r, 1.0 / 479001600.0);    /* 1/12! */
    p = fma(p, r, 1.0 / 39916800.0);
    p = fma(p, r, 1.0 / 3628800.0);
    p = fma(p, r, 1.0 / 362880.0);
    p = fma(p, r, 1.0 / 40320.0);
    p = fma(p, r, 1.0 / 5040.0);
    p = fma(p, r, 1.0 / 720.0);
    p = fma(p, r, 1.0 / 120.0);
    p = fma(p, r, 1.0 / 24.0);
    p = fma(p, r, 1.0 / 6.0);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    int k = (int)kd;
    int k1 = k / 2, k2 = k - k1;
    return (p * mz_pow2d(k1)) * mz_pow2d(k2);
}

/* -------------------------------------------------------------- det_log
 * log(x), x > 0: x = m·2^e with m in [1/sqrt2, sqrt2), s = (m−1)/(m+1),
 * log m = 2·atanh(s) by its odd series (|s| <= 0.1716, 14 terms).          */
MZ_HD double det_log(double x) {
    if (x != x) return x;
    if (x < 0.0) return NAN;
    if (x == 0.0) return -INFINITY;
    if (x == INFINITY) return x;
    int eadj = 0;
    if (x < 2.2250738585072014e-308) { x = x * 18014398509481984.0; eadj = -54; } /* 2^54 */
    uint64_t u = mz_d2u(x);
    int e = (int)((u >> 52) & 0x7ff) - 1023 + eadj;
    double m = mz_u2d((u & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL); /* [1,2) */
    if (m > 1.4142135623730951) { m = m * 0.5; e = e + 1; }
    double s = (m - 1.0) / (m + 1.0);
    double s2 = s * s;
    double p = 1.0 / 29.0;
    p = fma(p, s2, 1.0 / 27.0);
    p = fma(p, s2, 1.0 / 25.0);
    p = fma(p, s2, 1.0 / 23.0);
    p = fma(p, s2, 1.0 / 21.0);
    p = fma(p, s2, 1.0 / 19.0);
    p = fma(p, s2, 1.0 / 17.0);
    p = fma(p, s2, 1.0 / 15.0);
    p = fma(p, s2, 1.0 / 13.0);
    p = fma(p, s2, 1.0 / 11.0);
    p = fma(p, s2, 1.0 / 9.0);
    p = fma(p, s2, 1.0 / 7.0);
    p = fma(p, s2, 1.0 / 5.0);
    p = fma(p, s2, 1.0 / 3.0);
    double ls = (2.0 * s) * (s2 * p);           /* 2 s^3 (1/3 + ...) */
    double ed = (double)e;
    double lo = fma(ed, 1.90821492927058770002e-10, ls);
    return fma(ed, 6.93147180369123816490e-01, 2.0 * s + lo);
}

MZ_HD float det_logf(float x) { return (float)det_log((double)x); }

/* tanh in f32 (round 6; rounds 1-5 evaluated (e^{2|x|} − 1)/(e^{2|x|} + 1) in
 * f64, ~1 k cycles of dependent f64 work on the search's read-out path):
 *   |x| < 2^-12          x (tanh(x) rounds to x);
 *   |x| < 0.55           x + x³·P(x²), P of degree 4 fitted to the relative
 *                        error of tanh on [0, 0.55] (tools/fit_tanhf.py), Horner;
 *   |x| < 9.5            (1 − e)/(1 + e), e = det_expf(−2|x|) (no cancellation:
 *                        e ≤ e^{-1.1});
 *   else                 ±1.
 * Exhaustive over every f32 in [2^-12, 9.5] (tools/fit_tanhf.py): 0 ulp for
 * 87 %, 1 ulp for 13 %, 2 ulp for 3 inputs against tanh in f64 rounded to f32. */
MZ_HD float det_tanhf(float xf) {
    if (xf != xf) return xf;
    float ax = fabsf(xf), r;
    if (ax < 0.000244140625f) return xf;
    if (ax < 0.55f) {
        float s = ax * ax;
        float p = -0.006275205872952938f;
        p = fmaf(p, s, 0.021072300150990486f);
        p = fmaf(p, s, -0.053852442651987076f);
        p = fmaf(p, s, 0.13332587480545044f);
        p = fmaf(p, s, -0.33333316445350647f);
        r = fmaf(ax * s, p, ax);
    } else if (ax < 9.5f) {
        float e = det_expf(-2.0f * ax);
        r = (1.0f - e) / (1.0f + e);
    } else {
        r = 1.0f;
    }
    return xf < 0.0f ? -r : r;
}

/* Flux relu = max(0, x) (Julia max: +0 for ±0 input) */
MZ_HD float mz_relu(float x) { return x > 0.0f ? x : 0.0f; }

/* ------------------------------------------------------------- Philox4x32-10 */
typedef struct { uint32_t v[4]; } mz_u32x4;

MZ_HD uint32_t mz_mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
}

MZ_HD mz_u32x4 mz_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                         uint32_t k0, uint32_t k1) {
    for (int i = 0; i < 10; ++i) {
        uint32_t hi0, hi1;
        uint32_t lo0 = mz_mulhilo(0xD2511F53u, c0, &hi0);
        uint32_t lo1 = mz_mulhilo(0xCD9E8D57u, c2, &hi1);
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n1 = lo1;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        uint32_t n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    mz_u32x4 r; r.v[0] = c0; r.v[1] = c1; r.v[2] = c2; r.v[3] = c3;
    return r;
}

/* RNG stream purposes (counter word c3).  Counter layout:
 *   c0 = draw index within the stream, c1 = global game / sample id,
 *   c2 = step (move counter for search; learner step for replay sampling),
 *   c3 = purpose.  key = 64-bit seed.                                    */
enum {
    MZ_RNG_NOISE = 1,      /* Dirichlet root noise, SelfPlay.jl:104          */
    MZ_RNG_TIE = 2,        /* select_child tie-break, SelfPlay.jl:164         */
    MZ_RNG_ACTION = 3,     /* select_action categorical, SelfPlay.jl:299,303  */
    MZ_RNG_GAME = 4,       /* sample_n_games, ReplayBuffer.jl:102             */
    MZ_RNG_POS = 5,        /* sample_position, ReplayBuffer.jl:80             */
    MZ_RNG_ABSORB = 6,     /* absorbing-state action, ReplayBuffer.jl:46      */
    MZ_RNG_OPPONENT = 7,   /* random opponent, select_opponent_action :321    */
    MZ_RNG_ENV = 8,        /* synthetic Atari-like env: reset key, step      */
    MZ_RNG_FRAME = 9       /* synthetic Atari-like env: frame bytes of a key */
};

MZ_HD uint32_t mz_rng_u32(uint64_t seed, uint32_t purpose, uint32_t id, uint32_t step, uint32_t idx) {
    return mz_philox(idx, id, step, purpose, (uint32_t)seed, (uint32_t)(seed >> 32)).v[0];
}

/* uniform integer in [0, n) by 32x32 multiply-high (n >= 1) */
MZ_HD uint32_t mz_rng_below(uint32_t r, uint32_t n) {
    return (uint32_t)(((uint64_t)r * (uint64_t)n) >> 32);
}

/* sequential stream for rejection samplers */
typedef struct { uint64_t seed; uint32_t purpose, id, step, idx; } mz_stream;

MZ_HD double mz_stream_uniform_open(mz_stream* s) {   /* (0,1), 53 bits */
    mz_u32x4 r = mz_philox(s->idx, s->id, s->step, s->purpose, (uint32_t)s->seed, (uint32_t)(s->seed >> 32));
    s->idx += 1;
    uint64_t m = ((uint64_t)(r.v[0] >> 5) << 26) | (uint64_t)(r.v[1] >> 6);  /* 53 bits */
    return ((double)m + 0.5) * 1.1102230246251565404e-16;                  /* 2^-53 */
}

/* standard normal, Marsaglia polar method (first variate only) */
MZ_HD double mz_stream_normal(mz_stream* s) {
    for (;;) {
        double u1 = 2.0 * mz_stream_uniform_open(s) - 1.0;
        double u2 = 2.0 * mz_stream_uniform_open(s) - 1.0;
        double q = u1 * u1 + u2 * u2;
        if (q >= 1.0 || q == 0.0) continue;
        return u1 * sqrt((-2.0 * det_log(q)) / q);
    }
}

/* Gamma(alpha, 1): Marsaglia–Tsang; alpha < 1 boosted by U^(1/alpha)
 * (the GammaIPSampler construction of Distributions.jl).                 */
MZ_HD double mz_stream_gamma(mz_stream* s, double alpha) {
    double a = alpha < 1.0 ? alpha + 1.0 : alpha;
    double d = a - 1.0 / 3.0;
    double c = 1.0 / sqrt(9.0 * d);
    double g;
    for (;;) {
        double z = mz_stream_normal(s);
        double v = 1.0 + c * z;
        if (v <= 0.0) continue;
        v = v * v * v;
        double u = mz_stream_uniform_open(s);
        double z2 = z * z;
        if (u < 1.0 - 0.0331 * (z2 * z2)) { g = d * v; break; }
        if (det_log(u) < 0.5 * z2 + d * (1.0 - v + det_log(v))) { g = d * v; break; }
    }
    if (alpha < 1.0) {
        double u = mz_stream_uniform_open(s);
        g = g * det_exp(det_log(u) / alpha);
    }
    return g;
}

/* Component i (0-based, ascending legal-action order; reference: Dict key
 * order, SelfPlay.jl:103) of Dirichlet(n, alpha) before normalisation:
 * Float32(Gamma(alpha, 1)) drawn from its OWN stream (NOISE, game, step,
 * idx = i << 24 + draw), so the n components are independent and a device
 * lane draws each (Julia's global-RNG draw order is not reproducible
 * anyway, quirk Q6).                                                      */
MZ_HD float mz_dirichlet_gamma(uint64_t seed, uint32_t game, uint32_t step, int i, float alpha) {
    mz_stream s; s.seed = seed; s.purpose = MZ_RNG_NOISE; s.id = game; s.step = step;
    s.idx = (uint32_t)i << 24;
    return (float)mz_stream_gamma(&s, (double)alpha);
}

/* Dirichlet(n, alpha) noise into out[0..n) as f32.  As in
 * Distributions._rand!: x_i = Float32(gamma_i); x .*= inv(sum(x)), the sum
 * taken in ascending i.                                                    */
MZ_HD void mz_dirichlet(uint64_t seed, uint32_t game, uint32_t step, int n, float alpha, float* out) {
    float sum = 0.0f;
    for (int i = 0; i < n; ++i) {
        out[i] = mz_dirichlet_gamma(seed, game, step, i, alpha);
        sum = sum + out[i];
    }
    float inv = 1.0f / sum;
    for (int i = 0; i < n; ++i) out[i] = out[i] * inv;
}

#endif /* MZ_DETMATH_H */
