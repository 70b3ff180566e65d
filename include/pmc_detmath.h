/*
 * pmc_detmath.h -- deterministic scalar math shared by the HIP kernels (device) and the
 * C oracle (host).  Every function here is built only from IEEE-754 basic operations
 * (+ - * / sqrt, correctly rounded on both gfx950 and x86-64) and integer/bit operations,
 * so the same source produces bit-identical results on the GPU and on the CPU as long as
 * both sides are compiled with floating-point contraction disabled (-ffp-contract=off).
 *
 * Contents
 *   - Philox4x32-10 counter-based RNG (Salmon et al. 2011, Random123).  Replaces the
 *     reference's cuRAND XORWOW stream (curand_init(1234,id,0), subsweep.h:256-259 /
 *     start.cu:532), which is re-seeded on every launch.
 *   - uniform / normal / exponential variates on fixed counter slots.
 *   - det_log (fdlibm-style log, double) and det_sincos_2pi (octant reduction + Taylor).
 *   - the Lennard-Jones pair energy (subsweep.h:90-103 semantics, see pmc_pair_energy).
 *   - cell-index and sweep-plan helpers (colour order, shift axis / distance).
 *
 * This header is C99 (for the oracle, gcc) and HIP C++ (for the kernels, hipcc).
 */
#ifndef PMC_DETMATH_H
#define PMC_DETMATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define PMC_HD static inline __host__ __device__
#else
#define PMC_HD static inline
#endif

/* ------------------------------------------------------------------------------------- */
/* bit casts                                                                             */
/* ------------------------------------------------------------------------------------- */
PMC_HD uint64_t pmc_dbits(double x) { uint64_t u; __builtin_memcpy(&u, &x, 8); return u; }
PMC_HD double pmc_bitsd(uint64_t u) { double x; __builtin_memcpy(&x, &u, 8); return x; }
PMC_HD uint32_t pmc_fbits(float x) { uint32_t u; __builtin_memcpy(&u, &x, 4); return u; }
PMC_HD float pmc_bitsf(uint32_t u) { float x; __builtin_memcpy(&x, &u, 4); return x; }

/* ------------------------------------------------------------------------------------- */
/* Philox4x32-10                                                                         */
/* ------------------------------------------------------------------------------------- */
#define PMC_PHILOX_M0 0xD2511F53u
#define PMC_PHILOX_M1 0xCD9E8D57u
#define PMC_PHILOX_W0 0x9E3779B9u
#define PMC_PHILOX_W1 0xBB67AE85u

typedef struct { uint32_t v[4]; } pmc_u32x4;

PMC_HD pmc_u32x4 pmc_philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                   uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)PMC_PHILOX_M0 * (uint64_t)c0;
        uint64_t p1 = (uint64_t)PMC_PHILOX_M1 * (uint64_t)c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += PMC_PHILOX_W0; k1 += PMC_PHILOX_W1;
    }
    pmc_u32x4 out;
    out.v[0] = c0; out.v[1] = c1; out.v[2] = c2; out.v[3] = c3;
    return out;
}

/* Counter-slot tags (SURVEY Appendix A "RNG slots"). Counter = (idx, cell_id, sweep, tag). */
#define PMC_TAG_MOVE    0u  /* idx = move m: 4 words -> 3 normals (two Box-Muller pairs)     */
#define PMC_TAG_ACCEPT  1u  /* idx = move m: word 0 -> exponential acceptance threshold      */
#define PMC_TAG_SHUFFLE 2u  /* idx = slot i: word 0 -> Fisher-Yates index in [0, i]         */
#define PMC_TAG_PLAN    3u  /* host sweep plan, cell_id = 0xFFFFFFFF                          */

/* Uniform in (0,1): (k + 1/2) * 2^-23 with k the top 23 bits; exactly representable. */
PMC_HD float pmc_u01(uint32_t w) { return (float)((w >> 9) * 2u + 1u) * 0x1p-24f; }

/* Unbiased-enough bounded integer in [0, range) (multiply-shift, exact integer math). */
PMC_HD uint32_t pmc_bounded(uint32_t w, uint32_t range) {
    return (uint32_t)(((uint64_t)w * (uint64_t)range) >> 32);
}

/* ------------------------------------------------------------------------------------- */
/* det_log: natural log of a positive normal double (fdlibm e_log.c algorithm)           */
/* ------------------------------------------------------------------------------------- */
PMC_HD double pmc_det_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    uint64_t b = pmc_dbits(x);
    int e = (int)((b >> 52) & 0x7ff) - 1023;
    double m = pmc_bitsd((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull); /* [1,2) */
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }                      /* exact */
    double f = m - 1.0;                                                         /* exact */
    double hfsq = 0.5 * f * f;
    double s = f / (2.0 + f);
    double z = s * s;
    double w = z * z;
    double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    double R = t2 + t1;
    double dk = (double)e;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

/* sin / cos of 2*pi*u for u in [0,1) given as a float (so 4u is exact). */
PMC_HD void pmc_det_sincos_2pi(float u, float* s_out, float* c_out) {
    float t = 4.0f * u;              /* exact */
    int q = (int)t;                  /* quadrant 0..3 */
    float r = t - (float)q;          /* exact, [0,1) */
    int comp = r > 0.5f;
    float a = comp ? (1.0f - r) : r; /* exact (Sterbenz), [0, 0.5] */
    double x = (double)a * 1.5707963267948966;   /* [0, pi/4] */
    double x2 = x * x;
    /* Taylor to x^15 / x^16: truncation error < 3e-14 on [0, pi/4] */
    double sp = 1.0 + x2 * (-1.0 / 6.0 + x2 * (1.0 / 120.0 + x2 * (-1.0 / 5040.0
              + x2 * (1.0 / 362880.0 + x2 * (-1.0 / 39916800.0 + x2 * (1.0 / 6227020800.0
              + x2 * (-1.0 / 1307674368000.0)))))));
    double sx = x * sp;
    double cx = 1.0 + x2 * (-0.5 + x2 * (1.0 / 24.0 + x2 * (-1.0 / 720.0 + x2 * (1.0 / 40320.0
              + x2 * (-1.0 / 3628800.0 + x2 * (1.0 / 479001600.0 + x2 * (-1.0 / 87178291200.0
              + x2 * (1.0 / 20922789888000.0))))))));
    double sr = comp ? cx : sx;      /* sin(r*pi/2) */
    double cr = comp ? sx : cx;      /* cos(r*pi/2) */
    double so, co;
    if (q == 0)      { so = sr;  co = cr;  }
    else if (q == 1) { so = cr;  co = -sr; }
    else if (q == 2) { so = -sr; co = -cr; }
    else             { so = -cr; co = sr;  }
    *s_out = (float)so;
    *c_out = (float)co;
}

/* Three standard normals for one trial move (two Box-Muller pairs, fourth value dropped).
 * Replaces curand_normal x3 in make_move (subsweep.h:60-71). */
PMC_HD void pmc_move_normals(pmc_u32x4 w, float* g0, float* g1, float* g2) {
    float u0 = pmc_u01(w.v[0]), u1 = pmc_u01(w.v[1]);
    float u2 = pmc_u01(w.v[2]), u3 = pmc_u01(w.v[3]);
    float r0 = __builtin_sqrtf((float)(-2.0 * pmc_det_log((double)u0)));
    float r2 = __builtin_sqrtf((float)(-2.0 * pmc_det_log((double)u2)));
    float s1, c1, s3, c3;
    pmc_det_sincos_2pi(u1, &s1, &c1);
    pmc_det_sincos_2pi(u3, &s3, &c3);
    *g0 = r0 * c1;
    *g1 = r0 * s1;
    *g2 = r2 * c3;
}

/* Acceptance threshold T = -log(u), u in (0,1).  Metropolis test of accept_move
 * (subsweep.h:209-216: accept if dE<0 else if u < exp(-beta dE)) is evaluated as
 * beta*dE < T in double; beta*dE is exact in double (24x24-bit product). */
PMC_HD double pmc_accept_threshold(pmc_u32x4 w) {
    return -pmc_det_log((double)pmc_u01(w.v[0]));
}

/* ------------------------------------------------------------------------------------- */
/* Lennard-Jones pair energy, epsilon = sigma_LJ = 1, truncated (not shifted) at w.       */
/* Reference: calculate_pair_energy (subsweep.h:90-103): r = sqrtf(r2); 0 if r > w;       */
/* else 4(r^-12 - r^-6).  Here r > w is tested as r2 > rc2 where rc2 is the largest float */
/* whose correctly rounded sqrtf is <= w (pmc_cutoff_r2), i.e. the same predicate without */
/* the sqrt; r^-6 is (1/r2)^3 with IEEE division instead of the approximate __powf.       */
/* r2 is floored at 1e-4 so overlapping particles give a huge finite energy, never NaN.   */
/* ------------------------------------------------------------------------------------- */
#define PMC_R2_MIN 1.0e-4f

PMC_HD float pmc_r2(float dx, float dy, float dz) {
    float r2 = dx * dx + dy * dy;
    return r2 + dz * dz;
}

PMC_HD float pmc_lj_from_r2(float r2, float rc2) {
    float rr = r2 < PMC_R2_MIN ? PMC_R2_MIN : r2;
    float inv = 1.0f / rr;
    float p6 = inv * inv * inv;
    float e = 4.0f * (p6 * p6 - p6);
    return r2 <= rc2 ? e : 0.0f;
}

/* Fixed-point energy unit for observables: 2^-32 (order-independent int64 sums). */
#define PMC_FIX_SCALE 4294967296.0
#define PMC_FIX_CLAMP 1073741824.0 /* |E| clamped to 2^30 before conversion */
PMC_HD int64_t pmc_to_fixed(double e) {
    if (e > PMC_FIX_CLAMP) e = PMC_FIX_CLAMP;
    if (e < -PMC_FIX_CLAMP) e = -PMC_FIX_CLAMP;
    double v = e * PMC_FIX_SCALE;                 /* exact (power of two) */
    /* round half away from zero, integer arithmetic after truncation */
    double t = (double)(int64_t)v;                /* truncate toward zero */
    double fr = v - t;                            /* exact */
    int64_t r = (int64_t)t;
    if (fr >= 0.5) r += 1;
    else if (fr <= -0.5) r -= 1;
    return r;
}

/* ------------------------------------------------------------------------------------- */
/* Sweep plan: colour order + shift (f, d), replicated on every rank (no broadcast).      */
/* Reference: FY_Shuffle + itoa (start.cu:34-44,153-157), f/d (kernel.cu:683-684).        */
/* ------------------------------------------------------------------------------------- */
typedef struct {
    int order[8]; /* colour ids; colour -> offset via pmc_colour_offset */
    int f;        /* shift axis 0..2 */
    float d;      /* shift distance in (-w/2, w/2), never 0 */
} pmc_sweep_plan_t;

PMC_HD void pmc_colour_offset(int colour, int off[3]) {
    /* itoa (start.cu:153-157): r[2] = n%2, r[1] = (n/2)%2, r[0] = (n/4)%2 */
    off[2] = colour % 2;
    off[1] = (colour / 2) % 2;
    off[0] = (colour / 4) % 2;
}

PMC_HD pmc_sweep_plan_t pmc_plan_for_sweep(uint64_t seed, uint32_t sweep, float w) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    pmc_u32x4 a = pmc_philox4x32_10(0u, 0xFFFFFFFFu, sweep, PMC_TAG_PLAN, k0, k1);
    pmc_u32x4 b = pmc_philox4x32_10(1u, 0xFFFFFFFFu, sweep, PMC_TAG_PLAN, k0, k1);
    uint32_t words[8] = {a.v[0], a.v[1], a.v[2], a.v[3], b.v[0], b.v[1], b.v[2], b.v[3]};
    pmc_sweep_plan_t p;
    for (int i = 0; i < 8; ++i) p.order[i] = i;
    /* standard Fisher-Yates (fixes D1: the reference swaps a[n-i] and reseeds from time()) */
    for (int i = 7; i > 0; --i) {
        uint32_t j = pmc_bounded(words[7 - i], (uint32_t)(i + 1));
        int t = p.order[i]; p.order[i] = p.order[j]; p.order[j] = t;
    }
    p.f = (int)pmc_bounded(words[7], 3u);
    pmc_u32x4 c = pmc_philox4x32_10(2u, 0xFFFFFFFFu, sweep, PMC_TAG_PLAN, k0, k1);
    float u = pmc_u01(c.v[0]);
    p.d = u * w - w / 2.0f;
    return p;
}

/* ------------------------------------------------------------------------------------- */
/* Host-only: cutoff in r^2 equivalent to the reference's sqrtf(r2) > w test.            */
/* ------------------------------------------------------------------------------------- */
#include <math.h>
static inline float pmc_cutoff_r2(float w) {
    float x = w * w;
    while (sqrtf(x) > w) x = nextafterf(x, 0.0f);
    for (;;) {
        float nx = nextafterf(x, 2.0f * x + 1.0f);
        if (sqrtf(nx) > w) break;
        x = nx;
    }
    return x;
}

#endif /* PMC_DETMATH_H */
