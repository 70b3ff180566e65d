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
 *   - pmc_logf (fdlibm-style log) and pmc_det_sincos_2pi (octant reduction + Taylor), float.
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
#define PMC_TAG_SHUFFLE 2u  /* idx = i >> 2: word i & 3 -> Fisher-Yates index of slot i in [0, i] */
#define PMC_TAG_PLAN    3u  /* host sweep plan, cell_id = 0xFFFFFFFF                          */

/* Uniform in (0,1): (k + 1/2) * 2^-23 with k the top 23 bits; exactly representable. */
PMC_HD float pmc_u01(uint32_t w) { return (float)((w >> 9) * 2u + 1u) * 0x1p-24f; }

/* Unbiased-enough bounded integer in [0, range) (multiply-shift, exact integer math). */
PMC_HD uint32_t pmc_bounded(uint32_t w, uint32_t range) {
    return (uint32_t)(((uint64_t)w * (uint64_t)range) >> 32);
}

/* ------------------------------------------------------------------------------------- */
/* pmc_logf: natural log of a positive normal float (fdlibm e_logf.c reduction: m in        */
/* (sqrt(1/2), sqrt(2)], s = f/(2+f), log(1+f) = 2s(1 + s^2/3 + ... + s^8/9)); ~2 ulp.     */
/* The division is pmc_recip (defined below), so every op is an IEEE op or an fma.         */
/* ------------------------------------------------------------------------------------- */
PMC_HD float pmc_recip(float x);

PMC_HD float pmc_logf(float x) {
    const float ln2_hi = 6.9313812256e-01f;   /* 0x3f317180: trailing zero bits, e*ln2_hi exact */
    const float ln2_lo = 9.0580006145e-06f;   /* 0x3717f7d1 */
    uint32_t b = pmc_fbits(x);
    int e = (int)(b >> 23) - 127;
    float m = pmc_bitsf((b & 0x007FFFFFu) | 0x3F800000u);  /* [1,2) */
    if (m > 1.41421356f) { m = m * 0.5f; e += 1; }            /* exact */
    float f = m - 1.0f;                                       /* exact */
    float s = f * pmc_recip(2.0f + f);
    float z = s * s;
    float P = 1.0f + z * (0.333333343f + z * (0.2f + z * (0.142857149f + z * 0.111111112f)));
    float r = (2.0f * s) * P;
    float de = (float)e;
    return de * ln2_hi + (r + de * ln2_lo);
}

/* sin / cos of 2*pi*u for u in [0,1) given as a float (so 4u is exact): octant reduction, then
 * Taylor polynomials on [0, pi/4] (truncation < 2e-9); float ops only. */
PMC_HD void pmc_det_sincos_2pi(float u, float* s_out, float* c_out) {
    float t = 4.0f * u;              /* exact */
    int q = (int)t;                  /* quadrant 0..3 */
    float r = t - (float)q;          /* exact, [0,1) */
    int comp = r > 0.5f;
    float a = comp ? (1.0f - r) : r; /* exact (Sterbenz), [0, 0.5] */
    float x = a * 1.57079637f;       /* [0, pi/4] */
    float x2 = x * x;
    float sp = 1.0f + x2 * (-0.166666672f + x2 * (8.33333377e-03f + x2 * (-1.98412701e-04f
               + x2 * 2.75573188e-06f)));
    float sx = x * sp;
    float cx = 1.0f + x2 * (-0.5f + x2 * (4.16666679e-02f + x2 * (-1.38888892e-03f
               + x2 * (2.48015876e-05f + x2 * -2.75573192e-07f))));
    float sr = comp ? cx : sx;       /* sin(r*pi/2) */
    float cr = comp ? sx : cx;       /* cos(r*pi/2) */
    /* quadrant q: (sin, cos) = (sr, cr), (cr, -sr), (-sr, -cr), (-cr, sr) -- as selects and
     * sign flips (no branches; identical values) */
    float ua = (q & 1) ? cr : sr;
    float ub = (q & 1) ? sr : cr;
    *s_out = (q & 2) ? -ua : ua;
    *c_out = ((q + 1) & 2) ? -ub : ub;
}

/* Box-Muller radius sqrt(-2 log u) (sqrtf is correctly rounded on both targets). */
PMC_HD float pmc_bm_radius(float u) { return __builtin_sqrtf(-2.0f * pmc_logf(u)); }

/* Three standard normals for one trial move (two Box-Muller pairs, fourth value dropped).
 * Replaces curand_normal x3 in make_move (subsweep.h:60-71). */
PMC_HD void pmc_move_normals(pmc_u32x4 w, float* g0, float* g1, float* g2) {
    float r0 = pmc_bm_radius(pmc_u01(w.v[0]));
    float r2 = pmc_bm_radius(pmc_u01(w.v[2]));
    float s1, c1, s3, c3;
    pmc_det_sincos_2pi(pmc_u01(w.v[1]), &s1, &c1);
    pmc_det_sincos_2pi(pmc_u01(w.v[3]), &s3, &c3);
    *g0 = r0 * c1;
    *g1 = r0 * s1;
    *g2 = r2 * c3;
}

/* Acceptance threshold T = -log(u), u in (0,1).  Metropolis test of accept_move
 * (subsweep.h:209-216: accept if dE<0 else if u < exp(-beta dE)) is evaluated as
 * (double)beta*(double)dE < (double)T; the product is exact in double. */
PMC_HD float pmc_accept_threshold(pmc_u32x4 w) { return -pmc_logf(pmc_u01(w.v[0])); }

/* ------------------------------------------------------------------------------------- */
/* Lennard-Jones pair energy, epsilon = sigma_LJ = 1, truncated (not shifted) at w.       */
/* Reference: calculate_pair_energy (subsweep.h:90-103): r = sqrtf(r2); 0 if r > w;       */
/* else 4(r^-12 - r^-6).  Here r > w is tested as r2 > rc2 where rc2 is the largest float */
/* whose correctly rounded sqrtf is <= w (pmc_cutoff_r2), i.e. the same predicate without */
/* the sqrt; r^-6 is (1/r2)^3 with IEEE division instead of the approximate __powf.       */
/* r2 is floored at 1e-4 so overlapping particles give a huge finite energy, never NaN.   */
/* ------------------------------------------------------------------------------------- */
#define PMC_R2_MIN 1.0e-4f

/* r2 = fma(dz, dz, fma(dy, dy, dx*dx)): one multiply and two fused multiply-adds (v_mul +
 * 2 v_fma on gfx950, vmulss + 2 vfmadd on x86-64-v3), each a single IEEE rounding, so host and
 * device agree bit for bit.  Round-to-nearest is symmetric under negation, so
 * pmc_r2_neg = -pmc_r2 exactly (the kernels list old-position terms negated at no cost). */
PMC_HD float pmc_r2(float dx, float dy, float dz) {
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}
PMC_HD float pmc_r2_neg(float dx, float dy, float dz) {
    return __builtin_fmaf(-dz, dz, __builtin_fmaf(-dy, dy, (-dx) * dx));
}

/* Reciprocal by three Newton-Raphson steps from a bit-trick seed (max seed error 5.1%,
 * then 2.6e-3, 6.6e-6, 4.4e-11 before float rounding: ~1 ulp).  Only integer ops and fused
 * multiply-adds (IEEE, single rounding on both gfx950 v_fma_f32 and x86 vfmadd), so the result
 * is bit-identical on host and device -- and cheaper on CDNA than a correctly rounded division
 * (v_div_scale x2 + v_rcp + 4 fma + v_div_fmas + v_div_fixup). */
PMC_HD float pmc_recip(float x) {
    float y = pmc_bitsf(0x7EF311C3u - pmc_fbits(x));
    float e = __builtin_fmaf(-x, y, 1.0f);
    y = __builtin_fmaf(y, e, y);
    e = __builtin_fmaf(-x, y, 1.0f);
    y = __builtin_fmaf(y, e, y);
    e = __builtin_fmaf(-x, y, 1.0f);
    y = __builtin_fmaf(y, e, y);
    return y;
}

/* Quarter pair energy u = r^-12 - r^-6 (e = 4u).  Scaling by 4 is exact in binary floating
 * point, so sums of 4u equal 4 * (sums of u) bit for bit: the kernels accumulate u and apply the
 * factor 4 once per lane. */
PMC_HD float pmc_lj4_from_r2(float r2, float rc2) {
    float rr = __builtin_fmaxf(r2, PMC_R2_MIN);
    float inv = pmc_recip(rr);
    float p6 = inv * inv * inv;
    float u = p6 * p6 - p6;
    return r2 <= rc2 ? u : 0.0f;
}

PMC_HD float pmc_lj_from_r2(float r2, float rc2) { return 4.0f * pmc_lj4_from_r2(r2, rc2); }

/* Signed quarter pair energy of a listed term (the caller has already applied the cutoff):
 * r2s = +r2 for a new-position term, -r2 for an old-position term (sign bit set, -0 included).
 * Returns +u(r2) resp. -u(r2) bit for bit, u as in pmc_lj4_from_r2: round-to-nearest is
 * symmetric, so (inv*inv)*(-inv) = -p6 and (-p6)*p6 - (-p6) = -(p6*p6 - p6) exactly.  Costs one
 * bit-select over the unsigned form (|r2s| and |p6s| are free source modifiers on gfx950). */
PMC_HD float pmc_lj4_signed_m(float r2s, float r2min) {   /* r2min == PMC_R2_MIN */
    float a = __builtin_fabsf(r2s);
    float rr = a < r2min ? r2min : a;   /* = fmaxf for non-NaN; one compare + select, no canonicalize */
    float inv = pmc_recip(rr);
    float invs = __builtin_copysignf(inv, r2s);
    float p6s = (inv * inv) * invs;
    return p6s * __builtin_fabsf(p6s) - p6s;
}
PMC_HD float pmc_lj4_signed(float r2s) { return pmc_lj4_signed_m(r2s, PMC_R2_MIN); }

/* Conservative partner filter (staging): squared distance from a staged partner to the own
 * cell's closed box [lo, hi] (each side padded by PMC_BOX_PAD).  A partner with
 * d2 > rc2 * (1 + 2^-13) is farther than the cutoff from every position a particle of the cell
 * can take, so its pair energy is exactly 0 for every trial move and it is not staged. */
#define PMC_BOX_PAD 1.0e-3f
PMC_HD float pmc_box_d2(float x, float y, float z, const float lo[3], const float hi[3]) {
    /* fmaxf (maxNum): identical on both targets for non-NaN inputs; the sign of a zero is
     * irrelevant after squaring */
    float tx = __builtin_fmaxf(__builtin_fmaxf(lo[0] - x, x - hi[0]), 0.0f);
    float ty = __builtin_fmaxf(__builtin_fmaxf(lo[1] - y, y - hi[1]), 0.0f);
    float tz = __builtin_fmaxf(__builtin_fmaxf(lo[2] - z, z - hi[2]), 0.0f);
    return pmc_r2(tx, ty, tz);
}

/* Staging order of the neighbour partners (spec, kernels and oracle): in stencil order, first
 * slots [0, H) of every neighbour cell, then slots [H, n) of the cells holding more than H, with
 * H = nslot/2 for nslot >= 16 else nslot (nslot = smallest power of two >= max(nmax, 8)). */
PMC_HD int pmc_stage_split(int nmax) {
    int nslot = 8;
    while (nslot < nmax) nslot <<= 1;
    return nslot >= 16 ? nslot / 2 : nslot;
}

/* own-cell closed box padded by PMC_BOX_PAD: lb = c*w - L/2.0f (start.cu:129), ub = lb + w */
PMC_HD void pmc_cell_box(int cx, int cy, int cz, float w, float Lx, float Ly, float Lz, float lo[3],
                         float hi[3]) {
    float lbx = (float)cx * w - Lx / 2.0f, lby = (float)cy * w - Ly / 2.0f, lbz = (float)cz * w - Lz / 2.0f;
    lo[0] = lbx - PMC_BOX_PAD; hi[0] = (lbx + w) + PMC_BOX_PAD;
    lo[1] = lby - PMC_BOX_PAD; hi[1] = (lby + w) + PMC_BOX_PAD;
    lo[2] = lbz - PMC_BOX_PAD; hi[2] = (lbz + w) + PMC_BOX_PAD;
}

/* filter threshold: rc2 * (1 + 2^-13) */
PMC_HD float pmc_filter_r2(float rc2) { return rc2 * 1.0001220703125f; }

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

/* pmc_to_fixed((double)f) for a float f, in integer arithmetic only (no f64 ops: the GPU energy
 * kernel converts every pair term): f = m * 2^(ex-150), so f * 2^32 = m * 2^(ex-118); exact left
 * shift, or a right shift rounding half away from zero (the magnitude rounds, the sign is
 * reapplied: pmc_to_fixed is symmetric).  |f| > 2^30 clamps to +-2^62 as pmc_to_fixed does;
 * zeros and subnormals (< 2^-126, so |f * 2^32| < 0.5) give 0.  Finite f only. */
PMC_HD int64_t pmc_to_fixed_f32(float f) {
    /* branch-free (selects only): the GPU kernel converts a 64-lane block of terms at once */
    const uint32_t b = pmc_fbits(f);
    const uint32_t ex = (b >> 23) & 0xFFu;
    const uint32_t man = b & 0x7FFFFFu;
    const uint32_t m = man | 0x800000u;            /* ex == 0 (zero/subnormal) rounds to 0 below */
    const int sh = (int)ex - 118;
    const int sl = sh < 0 ? 0 : (sh > 39 ? 39 : sh);
    const int sr = sh >= 0 ? 1 : (-sh > 25 ? 25 : -sh);
    const uint64_t left = (uint64_t)m << sl;
    /* magnitude m * 2^-sr rounded half away from zero = floor(m / 2^sr + 1/2); m < 2^24, so
     * sr = 25 gives 0 for every smaller exponent too */
    const uint64_t right = (uint64_t)((m + (1u << (sr - 1))) >> sr);
    uint64_t q = sh >= 0 ? left : right;
    q = (ex > 157u || (ex == 157u && man != 0u)) ? ((uint64_t)1 << 62) : q;
    return (b >> 31) ? -(int64_t)q : (int64_t)q;
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

/* Colour order (spec v9).  Default: grouped by z parity -- the 4 colours of one z parity
 * (offset[2] = colour % 2, itoa start.cu:153-157), then the 4 of the other; which parity goes
 * first from word 0, each group Fisher-Yates-shuffled (words 1-3 and 4-6).  Every colour phase is
 * a Metropolis update that preserves the Boltzmann distribution, so any order is a valid sweep;
 * this one lets a z-slab decomposition exchange halos twice per sweep instead of up to 8 times
 * ("colour grouping by z-parity").  PMC_PLAN_FULL_SHUFFLE: one Fisher-Yates over all 8
 * (the reference's FY_Shuffle, start.cu:34-44, made standard and Philox-driven). */
#define PMC_PLAN_FULL_SHUFFLE 1u
PMC_HD pmc_sweep_plan_t pmc_plan_for_sweep_ex(uint64_t seed, uint32_t sweep, float w, uint32_t flags) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    pmc_u32x4 a = pmc_philox4x32_10(0u, 0xFFFFFFFFu, sweep, PMC_TAG_PLAN, k0, k1);
    pmc_u32x4 b = pmc_philox4x32_10(1u, 0xFFFFFFFFu, sweep, PMC_TAG_PLAN, k0, k1);
    uint32_t words[8] = {a.v[0], a.v[1], a.v[2], a.v[3], b.v[0], b.v[1], b.v[2], b.v[3]};
    pmc_sweep_plan_t p;
    if (flags & PMC_PLAN_FULL_SHUFFLE) {
        for (int i = 0; i < 8; ++i) p.order[i] = i;
        /* standard Fisher-Yates (fixes D1: the reference swaps a[n-i] and reseeds from time()) */
        for (int i = 7; i > 0; --i) {
            uint32_t j = pmc_bounded(words[7 - i], (uint32_t)(i + 1));
            int t = p.order[i]; p.order[i] = p.order[j]; p.order[j] = t;
        }
    } else {
        const int p0 = (int)pmc_bounded(words[0], 2u);
        for (int i = 0; i < 4; ++i) {
            p.order[i] = 2 * i + p0;
            p.order[4 + i] = 2 * i + (1 - p0);
        }
        for (int i = 3; i > 0; --i) {
            uint32_t j = pmc_bounded(words[4 - i], (uint32_t)(i + 1));        /* words 1..3 */
            int t = p.order[i]; p.order[i] = p.order[j]; p.order[j] = t;
        }
        for (int i = 3; i > 0; --i) {
            uint32_t j = pmc_bounded(words[7 - i], (uint32_t)(i + 1));        /* words 4..6 */
            int t = p.order[4 + i]; p.order[4 + i] = p.order[4 + j]; p.order[4 + j] = t;
        }
    }
    p.f = (int)pmc_bounded(words[7], 3u);
    pmc_u32x4 c = pmc_philox4x32_10(2u, 0xFFFFFFFFu, sweep, PMC_TAG_PLAN, k0, k1);
    float u = pmc_u01(c.v[0]);
    p.d = u * w - w / 2.0f;
    return p;
}
PMC_HD pmc_sweep_plan_t pmc_plan_for_sweep(uint64_t seed, uint32_t sweep, float w) {
    return pmc_plan_for_sweep_ex(seed, sweep, w, 0u);
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
