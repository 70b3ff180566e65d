// pmc_kernels.hip -- hand-written CDNA4 (gfx950) kernels for the checkerboard Metropolis hot path.
//
// Reference semantics: subsweep.h (root, "Version I": thread per cell) for the call surface and
// move rules; the LDS-staging design of CUDA-Parallel-MC/CUDA-Parallel-MC/kernel.cu:209-435
// ("Version II": block per cell) re-targeted to ONE 64-lane wavefront per cell visit (the main
// launch gives a wave two cells of the colour, visited one after the other, sharing their
// stencil-table and random-number passes):
//   * the cell's 27-cell stencil (own cell first, shuffled; then the 26 neighbours in
//     get_neighbors order, subsweep.h:119-137) is staged once into LDS (SoA x/y/z), with the
//     periodic image (apply_PBC, subsweep.h:139-151) folded into the staged coordinates;
//   * per trial move the lanes test old and new distances of the partners (lane = partner index
//     mod 64), evaluate the pair energies of the compacted in-cutoff pairs, and the wave reduces
//     dE with DPP row operations (no barrier); accept/reject is wave-uniform and in-kernel;
//   * Philox4x32-10 counter slots give every (sweep, cell, move) its own random numbers, so
//     results are independent of launch geometry and identical to the CPU oracle.
// No MFMA: this is not a dense contraction (pair energies are gathered, cut-off, divided).
//
// Build with -ffp-contract=off: every float/double op must stay a single IEEE op (the oracle,
// compiled by gcc with the same flag, reproduces the results bit for bit).
#include <hip/hip_ext.h>

#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "pmc_internal.h"
#include "../../include/pmc_detmath.h"

namespace pmc {

#ifndef PMC_MOVE_PRIO
#define PMC_MOVE_PRIO 2    // wave priority of the moves (their serial tail one above); 0: no s_setprio
#endif
#ifndef PMC_VISIT_PRIO
#define PMC_VISIT_PRIO 1   // wave priority of the shuffle, staging and write-back (see visit_cell)
#endif
#ifndef PMC_BOUNDARY_PB
#define PMC_BOUNDARY_PB 1   // slab boundary-plane launches: wave priority one level up (rank sweep -0.6% at 8 ranks, -1.2% at 4)
#endif
#ifndef PMC_BITOP3
#define PMC_BITOP3 1   // Philox key/word xors as one v_bitop3_b32 (sweep -0.3%, profiles/r03h_ab.txt)
#endif

#ifdef PMC_STAMPS
// Analysis build only (-DPMC_STAMPS, tools/stamps.py): per-wave s_memtime stamps at the section
// boundaries of a main-launch cell visit, written by lane 0 with vector stores.
__device__ unsigned long long* g_stamps = nullptr;
#define PMC_STAMP(k)                                                                              \
    do {                                                                                          \
        if (LCAP == kMainCap && g_stamps && lane == 0)                                            \
            g_stamps[(size_t)t * 16 + (k)] = __builtin_amdgcn_s_memtime();                        \
    } while (0)
#else
#define PMC_STAMP(k) \
    do {             \
    } while (0)
#endif

namespace {

__device__ __forceinline__ float as_f(int v) { return __builtin_bit_cast(float, v); }
__device__ __forceinline__ int as_i(float v) { return __builtin_bit_cast(int, v); }

__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Wave-wide float sum in a FIXED order, the xor butterfly 1, 2, 4, 8, 16, 32 the oracle replays
// (oracle/pmc_oracle.c subsweep_cell), delivered to an SGPR.  In-row steps: quad_perm DPP for xor 1
// and 2, then mirror patterns for xor 4 / 8 (after the previous steps all lanes of a quad, resp.
// half-row, hold equal values, so l^7 / l^15 supply the same operand as l^4 / l^8); every lane of
// row r then holds the row sum r_r.  Across rows, gfx9's row_bcast:15 (rows 1 and 3 add lane 15 of
// the row below: r1+r0, r3+r2) and row_bcast:31 (rows 2 and 3 add lane 31) leave (r3+r2)+(r1+r0)
// in lane 63 -- the butterfly's (r0+r1)+(r2+r3) bit for bit, as float addition is commutative.
// No LDS; only lane 63's value is meaningful (read into an SGPR).
__device__ __forceinline__ float wave_sum_fixed_order_s(float v) {
    v = v + as_f(__builtin_amdgcn_update_dpp(0, as_i(v), 0xB1, 0xF, 0xF, true));   // quad_perm 1,0,3,2
    v = v + as_f(__builtin_amdgcn_update_dpp(0, as_i(v), 0x4E, 0xF, 0xF, true));   // quad_perm 2,3,0,1
    v = v + as_f(__builtin_amdgcn_update_dpp(0, as_i(v), 0x141, 0xF, 0xF, true));  // row_half_mirror
    v = v + as_f(__builtin_amdgcn_update_dpp(0, as_i(v), 0x140, 0xF, 0xF, true));  // row_mirror
    // row-masked DPP adds written directly (the builtins above would not fuse a row-masked DPP
    // move into the add); s_nop 1 = the two wait states between a VALU write and a DPP read
    asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(v));
    asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf" : "+v"(v));
    return as_f(__builtin_amdgcn_readlane(as_i(v), 63));
}

// number of set bits of the 64-lane mask m below this lane (+ add)
__device__ __forceinline__ int mbcnt64_add(unsigned long long m, int add) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)add));
}
__device__ __forceinline__ int mbcnt64(unsigned long long m) { return mbcnt64_add(m, 0); }

// pmc_lj4_signed_m with the r2 floor as ONE v_max_f32 (|r2s| is a free source modifier; the
// compiler's fmaxf would add canonicalizing maxes, the C form a compare + select): identical
// values for the non-NaN inputs of the term list (max(|r2s|, r2min) == (|r2s| < r2min ? r2min :
// |r2s|)).
__device__ __forceinline__ float lj4_signed_max(float r2s, float r2min) {
    float rr;
    asm("v_max_f32_e64 %0, |%1|, %2" : "=v"(rr) : "v"(r2s), "s"(r2min));
    const float inv = pmc_recip(rr);
    const float invs = __builtin_copysignf(inv, r2s);
    const float p6s = (inv * inv) * invs;
    return p6s * __builtin_fabsf(p6s) - p6s;
}

__device__ __forceinline__ uint32_t bit_of(uint32_t m, int lane) { return (m >> (lane & 31)) & 1u; }

// Stencil lane masks: lane k = 9*hx + 3*hy + hz < 27; Neg[a] has the lanes whose offset along
// axis a is -1 (h == 1), Pos[a] those with +1 (h == 2).
constexpr uint32_t stencil_mask(int axis, int h) {
    uint32_t m = 0;
    for (int l = 0; l < 27; ++l) {
        const int hh = axis == 0 ? l / 9 : (axis == 1 ? (l / 3) % 3 : l % 3);
        if (hh == h) m |= 1u << l;
    }
    return m;
}
__device__ constexpr uint32_t kStencilNeg[3] = {stencil_mask(0, 1), stencil_mask(1, 1), stencil_mask(2, 1)};
__device__ constexpr uint32_t kStencilPos[3] = {stencil_mask(0, 2), stencil_mask(1, 2), stencil_mask(2, 2)};

// Staging lanes per stencil cell: slots [0, HS) of every neighbour are staged in the main passes
// (loaded with the visit's single HBM round trip); slots [HS, nmax) -- only cells holding more than
// HS particles, ~1.6% of cells at 4.77 per cell -- in overflow passes.  Half the lanes per cell of
// the full row for nmax >= 16: 4 main passes instead of 7 at nmax = 16.  The staged order (all
// cells' low slots, then the overflow cells' high slots) is part of the spec the oracle follows.
__host__ __device__ constexpr int stage_split(int nslot) { return nslot >= 16 ? nslot / 2 : nslot; }

// lanes of staging pass q whose stencil cell k = 1 + q*CPP + lane/NSLOT is < 27
template <int NSLOT>
__device__ constexpr unsigned long long stage_lane_mask(int q) {
    constexpr int CPP = kWave / NSLOT;
    unsigned long long m = 0;
    for (int l = 0; l < kWave; ++l)
        if (1 + q * CPP + l / NSLOT < 27) m |= 1ull << l;
    return m;
}

// Loads from the disk buffer.  OFF32 (buffer < 4 GiB): 32-bit byte offsets -> global_load with an
// SGPR base and a VGPR offset (no 64-bit address math per load); else 64-bit element addressing.
// ld3 / st3: a slot's x, y, z (dstep = lay_dim: the floats between dimensions) from ONE pointer, so
// the three accesses are provably adjacent (the packed layout: one dwordx3 access) or at immediate
// offsets (the reference rows), instead of three 32-bit offsets the compiler cannot combine.
template <int OFF32> struct DiskAddr;
template <> struct DiskAddr<1> {
    static constexpr uint32_t kUnit = 4;   // offsets in bytes
    __device__ static __forceinline__ const float* at(const float* b, uint32_t off) {
        return (const float*)((const char*)b + (uint64_t)off);
    }
    __device__ static __forceinline__ float* at(float* b, uint32_t off) { return (float*)((char*)b + (uint64_t)off); }
    __device__ static __forceinline__ float ld(const float* b, uint32_t off) { return *at(b, off); }
    __device__ static __forceinline__ void st(float* b, uint32_t off, float v) { *at(b, off) = v; }
    __device__ static __forceinline__ void ld3(const float* b, uint32_t off, uint32_t dstep, float& x, float& y,
                                               float& z) {
        const float* q = at(b, off);
        x = q[0];
        y = q[dstep];
        z = q[2 * dstep];
    }
    __device__ static __forceinline__ void st3(float* b, uint32_t off, uint32_t dstep, float x, float y, float z) {
        float* q = at(b, off);
        q[0] = x;
        q[dstep] = y;
        q[2 * dstep] = z;
    }
};
template <> struct DiskAddr<0> {
    static constexpr uint32_t kUnit = 1;   // offsets in floats
    __device__ static __forceinline__ float ld(const float* b, uint32_t off) { return b[(uint64_t)off]; }
    __device__ static __forceinline__ void st(float* b, uint32_t off, float v) { b[(uint64_t)off] = v; }
    __device__ static __forceinline__ void ld3(const float* b, uint32_t off, uint32_t dstep, float& x, float& y,
                                               float& z) {
        const float* q = b + (uint64_t)off;
        x = q[0];
        y = q[dstep];
        z = q[2 * dstep];
    }
    __device__ static __forceinline__ void st3(float* b, uint32_t off, uint32_t dstep, float x, float y, float z) {
        float* q = b + (uint64_t)off;
        q[0] = x;
        q[dstep] = y;
        q[2 * dstep] = z;
    }
};

// Philox4x32-10 with the host-computed key schedule (bit-identical to pmc_philox4x32_10: round
// r uses key (k0 + r*W0, k1 + r*W1)); fully unrolled, the keys are SGPR operands.
__device__ __forceinline__ pmc_u32x4 philox_sched(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                  const DevGeom& g) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)PMC_PHILOX_M0 * (uint64_t)c0;
        const uint64_t p1 = (uint64_t)PMC_PHILOX_M1 * (uint64_t)c2;
#if PMC_BITOP3
        // gfx950's three-input bitwise op (truth table 0x96 = a ^ b ^ c): one VALU per word
        uint32_t n0, n2;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n0) : "v"((uint32_t)(p1 >> 32)), "v"(c1), "s"(g.rk0[r]));
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n2) : "v"((uint32_t)(p0 >> 32)), "v"(c3), "s"(g.rk1[r]));
#else
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ g.rk0[r];
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ g.rk1[r];
#endif
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
    }
    pmc_u32x4 out;
    out.v[0] = c0; out.v[1] = c1; out.v[2] = c2; out.v[3] = c3;
    return out;
}

// The same Philox with the round keys formed on the fly from (k0, k1) -- for the RARE paths inside
// a visit (moves beyond the first chunk, more than 16 own particles).  The key words are laundered
// through an empty asm in the rare block itself, so the compiler cannot hoist the schedule out of
// it: the 20 round-key SGPRs of philox_sched then need not stay live across the move loop, where
// they pushed other loop values into SGPR spills (v_writelane / v_readlane per move).
#ifndef PMC_RARE_KEYS
#define PMC_RARE_KEYS 1
#endif
__device__ __forceinline__ pmc_u32x4 philox_rare(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                 const DevGeom& g) {
#if PMC_RARE_KEYS
    uint32_t k0 = g.k0, k1 = g.k1;
    asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)PMC_PHILOX_M0 * (uint64_t)c0;
        const uint64_t p1 = (uint64_t)PMC_PHILOX_M1 * (uint64_t)c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
        k0 += PMC_PHILOX_W0;
        k1 += PMC_PHILOX_W1;
    }
    pmc_u32x4 out;
    out.v[0] = c0; out.v[1] = c1; out.v[2] = c2; out.v[3] = c3;
    return out;
#else
    return philox_sched(c0, c1, c2, c3, g);
#endif
}

// exact n / d for 32-bit n (Granlund-Montgomery round-up method; magic from make_udiv_magic)
__device__ __forceinline__ uint32_t udiv_magic(uint32_t n, UDivMagic m) {
    const uint32_t hi = __umulhi(n, m.mul);
    return (hi + ((n - hi) >> m.sh1)) >> m.sh2;
}

// Acceptance by one float compare.  accept_move (subsweep.h:209-216; the spec's form, kept by the
// oracle) accepts when beta*dE < T in double, and the product of two floats is exact in double.
// The moves reduce s = dE/4, so for beta > 0 that is b4 * s < T with b4 = 4*(double)beta (24
// significant bits: b4 * s is exact too), i.e. s <= F with F the largest float whose product with
// b4 is below T.  F from the estimate T * (1/b4) (within one float ulp of T/b4), then one ulp step
// either way, checked exactly; the parking lanes do this once per move, off the moves' serial
// path.  beta == 0 (normalise rejects beta < 0): 0 < T always, as F = +inf gives for the finite s
// the r2 floor guarantees.
__device__ __forceinline__ float accept_bound(float T, const DevGeom& g) {
    if (!(g.beta > 0.0f)) return __builtin_inff();
    const double Td = (double)T;
    const double b4 = 4.0 * (double)g.beta;
    const float f = (float)(Td * g.inv_b4);                        // >= 0 (T > 0), maybe +inf
    const float up = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, f) + 1u);
    const float dn = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, f) - 1u);
    const bool f_ok = (double)f * b4 < Td;                          // false for +inf
    const bool up_ok = (double)up * b4 < Td;                        // false for NaN (f = +inf)
    return f_ok ? (up_ok ? up : f) : dn;
}

// storage index of local cell (x, y, zl)
__device__ __forceinline__ int64_t sidx(const DevGeom& g, int x, int y, int zl) {
    return (int64_t)x + (int64_t)g.cps_x * ((int64_t)y + (int64_t)g.cps_y * (int64_t)(zl + g.halo));
}

// ------------------------------------------------------------------------------------------
// subsweep: one colour phase, one wave per cell visit (subsweep_kernel, subsweep.h:240-300)
//
// Per cell visit (one wave; two per wave in the main launch, see subsweep_pair):
//   1. stencil table: lane k < 27 computes stencil cell k's storage offset and periodic image
//      and loads its count; every global load of the visit is issued at once (counts, the 26
//      neighbours' half rows -- a 64 B row sits inside one 128 B line -- and the own rows): one
//      HBM round trip per visit;
//   2. RNG while the loads fly (Philox counters per cell, move, slot; RNG spec above
//      rng_chunk_single): Box-Muller moves, -log u thresholds, Fisher-Yates words, the moves'
//      variates parked in LDS;
//   3. stage the neighbours into LDS, keeping (ballot + mbcnt compaction) only partners within
//      the cutoff of the own cell's box -- the others contribute exactly 0 -- then the own cell
//      (shuffled) after them;
//   4. n_M moves: per block of 64 partners, lane l computes the new- and old-position r2 of
//      partner 64*block + l; the pairs within the cutoff (about 1 in 5) are compacted by
//      ballot + mbcnt into an LDS term list (new terms, then old terms with the sign bit set),
//      and only those reach the reciprocal -- term t on lane t % 64; one fixed-order
//      DPP reduction gives dE; accept in-kernel, wave-uniformly;
//   5. write back the own cell; one atomic per counter per wave.
// LDS per wave (capacity lcap): x, y, z rows of `stride` = subsweep_stride(lcap) slots, then the
// term list (2 * lcap + 64 floats; the extra 64 hold the kPad entries after the list, so a pass
// reads a full 64-lane block without a lane mask).  Row slots past the last partner hold +inf ("far"), as
// does the moving particle's own slot during its move, so no lane mask is needed in the moves.
// ------------------------------------------------------------------------------------------
// Returns false (and leaves the cell untouched) when the cell's staged partners do not fit the
// LDS capacity `cap`; the caller queues it for the full-capacity fallback launch.
// MIRROR (slab boundary planes): the written-back rows also go to `mirror` -- mirror_mode 0: the
// packed colour buffer of the halo exchange (row ta + tb*cps_x/2), 1: a plane (row x + cps_x*y;
// the periodic single-rank halo).  Empty cells write nothing (their count stays 0).
#ifndef PMC_CELLS_PER_WAVE
#define PMC_CELLS_PER_WAVE 2   // main launch: cells visited per wave (1: the single-cell prologue)
#endif

// Overflow queue header (ints): [kOvfCount] queued cells, [kOvfDone] fallback workgroups done;
// entries from kOvfHead.  Zero between launches (the fallback's last workgroup resets it).
constexpr int kOvfCount = 0, kOvfDone = 1;

// Visiting order of the main launch (speed only: cells of a colour are independent).  Colour cell
// index t = ta + hx*(tb + hy*tc) (the stats slot and the overflow queue's entry); the main launch
// visits position p in groups of PMC_ZGROUP colour planes: x fastest, then the planes of the group,
// then y, then the group (cell_geo with zlog = log2 PMC_ZGROUP).  A stencil row of a
// plane between two colour planes is read by both of them; with x, y, z order those reads lie a
// whole colour plane of cells apart (more than an XCD's L2 holds), within a group they lie one row
// of cells apart.  With the XCD-aware block order an XCD's contiguous range is whole groups (at
// 128^3: 64 colour planes, 16 groups of 4, two per XCD).  Fabric reads per launch at 128^3/1e7:
// 835 MB in plain order, 497 MB in groups of 4; phase -0.5..1%, 256^3 box -2.3%; groups of 16
// were 15% slower at the same traffic (profiles/r02x_zgroup_ab.txt).  Ranges whose plane count
// PMC_ZGROUP does not divide keep the plain order.
#ifndef PMC_ZGROUP
#define PMC_ZGROUP 4
#endif
constexpr int ilog2_exact(int v) { return v <= 1 ? 0 : 1 + ilog2_exact(v >> 1); }
static_assert((PMC_ZGROUP & (PMC_ZGROUP - 1)) == 0, "PMC_ZGROUP must be a power of two");
constexpr int kZGroupLog = ilog2_exact(PMC_ZGROUP);

// Wave-uniform geometry of one cell visit: position p -> (ta, tb, tc) by host-computed magic
// division (SALU only; zlog = 0: the plain order, p = t), the colour cell index t, the cell's
// storage index, its global id (the RNG counter) and whether its stencil crosses a box face.
struct CellGeo {
    int t, ta, tb, x, y, zl, zg0;
    uint32_t c, id;
    bool edge;
};

// With zlog, a range whose colour-plane count ncz the group size does not divide ends in a short
// group of ncz % G planes (same order inside it: x, then its planes, then y).
__device__ __forceinline__ CellGeo cell_geo(const DevGeom& g, int p, int cz0, int ox, int oy, int oz,
                                            int zlog = 0, int ncz = 0, int czs = 1) {
    CellGeo cg;
    const int hx = g.cps_x >> 1, hy = g.cps_y >> 1;
    const uint32_t q1 = udiv_magic((uint32_t)p, g.div_ncx);     // p / hx: row of the visiting order
    cg.ta = p - (int)q1 * hx;
    int tcr;                                                     // colour plane in the range
    if (zlog == 0) {
        const uint32_t q2 = udiv_magic(q1, g.div_ncy);           // plane
        cg.tb = (int)q1 - (int)q2 * hy;
        tcr = (int)q2 * czs;                                     // (czs: colour planes czs apart)
    } else {
        const uint32_t lim = (uint32_t)(ncz >> zlog) * (uint32_t)hy << zlog;   // rows of the full groups
        if (q1 < lim) {
            const uint32_t q3 = q1 >> zlog;
            const uint32_t q2 = udiv_magic(q3, g.div_ncy);       // group
            cg.tb = (int)q3 - (int)q2 * hy;
            tcr = ((int)q2 << zlog) + (int)(q1 & ((1u << zlog) - 1u));
        } else {                                                 // the short last group: gl planes
            const uint32_t r = q1 - lim;
            const uint32_t gl = (uint32_t)ncz & ((1u << zlog) - 1u);   // 1..3 (PMC_ZGROUP <= 4)
            const uint32_t tb = gl == 1u ? r : (gl == 2u ? r >> 1 : (uint32_t)(((uint64_t)r * 0xAAAAAAABull) >> 33));
            cg.tb = (int)tb;
            tcr = ((ncz >> zlog) << zlog) + (int)(r - tb * gl);
        }
    }
    cg.t = zlog ? cg.ta + hx * (cg.tb + hy * tcr) : p;
    const int tc = cz0 + tcr;                              // colour plane (z = 2*tc + oz)
    cg.x = 2 * cg.ta + ox;
    cg.y = 2 * cg.tb + oy;
    cg.zl = 2 * tc + oz;
    cg.zg0 = g.z0 + cg.zl;
    // a halo plane visited redundantly (two-plane halos, launch_subsweep_plane) may lie across the
    // periodic z boundary: its global plane, cell id and cell centre are the owner's
    cg.zg0 += cg.zg0 < 0 ? g.cps_z : 0;
    cg.zg0 -= cg.zg0 >= g.cps_z ? g.cps_z : 0;
    const int plane = g.cps_x * g.cps_y;
    cg.c = (uint32_t)(cg.x + g.cps_x * cg.y + plane * (cg.zl + g.halo));
    cg.id = (uint32_t)cg.x + (uint32_t)g.cps_x * ((uint32_t)cg.y + (uint32_t)g.cps_y * (uint32_t)cg.zg0);
    cg.edge = cg.x == 0 || cg.x == g.cps_x - 1 || cg.y == 0 || cg.y == g.cps_y - 1 || cg.zg0 == 0 ||
              cg.zg0 == g.cps_z - 1;
    return cg;
}

// Stencil table of the cell on lanes hb + k, k < 27 (own cell first, then get_neighbors order,
// subsweep.h:119-137; lane k = 9*hx + 3*hy + hz, h = 0, 1, 2 -> offset 0, -1, +1): storage cell and
// periodic image (apply_PBC, subsweep.h:139-151).  `edge` is wave-uniform over both halves (the
// wrapped arithmetic is exact for interior cells too).
struct StencilLane {
    uint32_t kc;
    float sx, sy, sz;
};

__device__ __forceinline__ StencilLane stencil_lane(const DevGeom& g, const CellGeo& cg, int k, bool edge) {
    const int dx = (int)bit_of(kStencilPos[0], k) - (int)bit_of(kStencilNeg[0], k);
    const int dy = (int)bit_of(kStencilPos[1], k) - (int)bit_of(kStencilNeg[1], k);
    const int dz = (int)bit_of(kStencilPos[2], k) - (int)bit_of(kStencilNeg[2], k);
    const int plane = g.cps_x * g.cps_y;
    StencilLane sl;
    sl.sx = sl.sy = sl.sz = 0.0f;
    if (!edge) {
        sl.kc = cg.c + (uint32_t)(dx + g.cps_x * dy + plane * dz);   // (storage is contiguous across halos)
    } else {
        // periodic wrap as selects (no exec-mask branches)
        const int nx0 = cg.x + dx, ny0 = cg.y + dy, zgn = cg.zg0 + dz;
        const int nx = nx0 + (nx0 < 0 ? g.cps_x : 0) - (nx0 >= g.cps_x ? g.cps_x : 0);
        const int ny = ny0 + (ny0 < 0 ? g.cps_y : 0) - (ny0 >= g.cps_y ? g.cps_y : 0);
        sl.sx = nx0 < 0 ? -g.Lx : (nx0 >= g.cps_x ? g.Lx : 0.0f);
        sl.sy = ny0 < 0 ? -g.Ly : (ny0 >= g.cps_y ? g.Ly : 0.0f);
        sl.sz = zgn < 0 ? -g.Lz : (zgn >= g.cps_z ? g.Lz : 0.0f);
        const int nz0 = cg.zl + dz;
        const int nzl = g.halo ? nz0 : nz0 + (nz0 < 0 ? g.cps_z : 0) - (nz0 >= g.cps_z ? g.cps_z : 0);
        sl.kc = (uint32_t)(nx + g.cps_x * ny + plane * (nzl + g.halo));
    }
    return sl;
}

// The visit's single HBM round trip: lanes load half rows (slots [0, HS)) of the 26 neighbours
// (NP passes, CPP cells per pass; row offsets from the stencil lanes hb + k) and the own rows.
template <int NSLOT, int NMC, int OFF32>
struct VisitLoads {
    static constexpr int HS = stage_split(NSLOT);
    static constexpr int CPP = kWave / HS;
    static constexpr int NP = (26 + CPP - 1) / CPP;
    float vx[NP], vy[NP], vz[NP];
    float ownx, owny, ownz;
    __device__ __forceinline__ void issue(const DevGeom& g, const float* __restrict__ disk, const CellGeo& cg,
                                          uint32_t k_off, int hb) {
        const int lane = threadIdx.x & (kWave - 1);
        const int nm = NMC > 0 ? NMC : g.nmax;
        const int p = lane & (HS - 1);
        const int kk = lane / HS;
        const int pp = p < nm ? p : 0;
        const uint32_t pp_off = (uint32_t)pp * lay_slot() * DiskAddr<OFF32>::kUnit;
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const int k = 1 + q * CPP + kk;
            const uint32_t off = (uint32_t)__shfl((int)k_off, hb + (k < 27 ? k : 26)) + pp_off;
            DiskAddr<OFF32>::ld3(disk, off, lay_dim(nm), vx[q], vy[q], vz[q]);
        }
        const int l = lane < nm ? lane : 0;
        const float* own = disk + (uint64_t)cg.c * (uint32_t)(3 * nm);   // wave-uniform base
        ownx = own[(uint32_t)l * lay_slot()];
        owny = own[lay_dim(nm) + (uint32_t)l * lay_slot()];
        ownz = own[2u * lay_dim(nm) + (uint32_t)l * lay_slot()];
    }
};

// Random numbers (RNG spec, include/pmc_detmath.h tags): move m -> Philox(m, id, sweep, MOVE):
// (w0, w1) Box-Muller pair A -> d0 = s R cos, d1 = s R sin; (w2, w3) pair B -> d2 = s R cos;
// acceptance threshold of move m -> -log u(Philox(m, id, sweep, ACCEPT).w0); Fisher-Yates word of
// slot i -> Philox(i >> 2, id, sweep, SHUFFLE).w[i & 3].  Every (cell, move, slot) has its own
// counter, so the lane mapping below is free: one cell per wave (16 moves per chunk) or two cells per
// wave (10 moves each in the first chunk) give the same numbers.
//
// Parking: move j of the current chunk keeps (d0, d1) at y-row tail pair j and (d2, T) at z-row
// tail pair j (slots [lcap4, lcap4 + 32): never staged, read by the moves only as "far" partners'
// don't-care values), so a move takes its randoms with two broadcast LDS reads.

// Single-cell RNG chunk: moves m0..m0+15 -- lanes 0-15 MOVE call (pair A), 16-31 ACCEPT call,
// 32-47 the MOVE call again (pair B from its words 2, 3: no cross-lane traffic) -- parked.
__device__ __forceinline__ void rng_chunk_single(const DevGeom& g, uint32_t id, uint32_t sweep, int m0,
                                                 float* py_, float* pz_, int lcap4) {
    const int lane = threadIdx.x & (kWave - 1);
    const int j = lane & 15;
    const uint32_t tag = (lane & 48) == 16 ? PMC_TAG_ACCEPT : PMC_TAG_MOVE;
    const pmc_u32x4 w = philox_rare((uint32_t)(m0 + j), id, sweep, tag, g);
    const uint32_t wl = lane < 32 ? w.v[0] : w.v[2];
    const uint32_t ws = lane < 32 ? w.v[1] : w.v[3];
    const float lg = pmc_logf(pmc_u01(wl));
    const float R = __builtin_sqrtf(-2.0f * lg);
    float sn, cs;
    pmc_det_sincos_2pi(pmc_u01(ws), &sn, &cs);
    const float G0 = (R * cs) * g.sigma;   // lanes 0-15: d0 of move m0+j; 32-47: d2
    const float G1 = (R * sn) * g.sigma;   // lanes 0-15: d1
    const float TT = accept_bound(-lg, g);    // lanes 16-31: T's acceptance bound
    if (lane < 16) *(float2*)(py_ + lcap4 + 2 * j) = make_float2(G0, G1);
    else if (lane < 48) pz_[lcap4 + 2 * j + (lane < 32 ? 1 : 0)] = lane < 32 ? TT : G0;
}

// Fisher-Yates indices of slots 0-63 (lane i: slot i): SHUFFLE calls 0-15 on lanes 0-15, their
// 4 words through LDS scratch `tmp` (64 floats; the term list area, free outside the moves).
__device__ __forceinline__ int fy_words_single(const DevGeom& g, uint32_t id, uint32_t sweep, float* tmp) {
    const int lane = threadIdx.x & (kWave - 1);
    const pmc_u32x4 w = philox_rare((uint32_t)(lane & 15), id, sweep, PMC_TAG_SHUFFLE, g);
    if (lane < 16) *(uint4*)(tmp + 4 * lane) = make_uint4(w.v[0], w.v[1], w.v[2], w.v[3]);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const uint32_t wi = *(const uint32_t*)(tmp + lane);
    return (int)pmc_bounded(wi, (uint32_t)(lane + 1));
}

// One cell visit after its prologue (stencil table + loads issued on lanes hb.., FY words jv on
// lanes hb + i, first_len moves parked): shuffle, staging, moves, write-back.
// Returns false (and leaves the cell untouched) when the cell's staged partners do not fit the
// LDS capacity `cap`; the caller queues it for the full-capacity fallback launch.
// MIRROR (slab boundary planes): the written-back rows also go to `mirror` -- mirror_mode 0: the
// packed colour buffer of the halo exchange (row ta + tb*cps_x/2), 1: a plane (row x + cps_x*y;
// the periodic single-rank halo).  Empty cells write nothing (their count stays 0).
template <int NSLOT, int NMC, int LCAP, int OFF32, bool MIRROR, int PB = 0, int QK = 0>
__device__ __forceinline__ bool visit_cell(const DevGeom& g, float* __restrict__ disk, uint32_t sweep,
                                           unsigned long long* __restrict__ stats, float* __restrict__ px_,
                                           int lcap_rt, int cap, int t, const CellGeo& cg, int hb, int k_cnt,
                                           uint32_t k_off, float k_sx, float k_sy, float k_sz,
                                           const VisitLoads<NSLOT, NMC, OFF32>& ld, int jv, int fy_have,
                                           int first_len, float* __restrict__ mirror, int mirror_mode) {
    constexpr int HS = stage_split(NSLOT);        // staging lanes per stencil cell (main passes)
    constexpr int CPP = kWave / HS;               // stencil cells staged per pass
    constexpr int NP = (26 + CPP - 1) / CPP;      // main staging passes over the 26 neighbours
    const int lane = threadIdx.x & (kWave - 1);
    const int nm = NMC > 0 ? NMC : g.nmax;        // compile-time for the common nmax
    const int lcap = LCAP > 0 ? LCAP : lcap_rt;            // layout capacity (>= cap)
    const int stride = subsweep_stride(lcap);              // compile-time -> LDS offset immediates
    const int lcap4 = (lcap + 3) & ~3;                     // per-move randoms at rows' tails (16 B aligned)
    float* py_ = px_ + stride;
    float* pz_ = py_ + stride;
    float* buf = pz_ + stride;                  // term list: signed r2 values
    const int ta = cg.ta, tb = cg.tb, x = cg.x, y = cg.y, zg0 = cg.zg0;
    const uint32_t c = cg.c, id = cg.id;
    const bool edge = cg.edge;
    const int p = lane & (HS - 1);
    const int kk = lane / HS;
    const float (&vx)[NP] = ld.vx;
    const float (&vy)[NP] = ld.vy;
    const float (&vz)[NP] = ld.vz;
    const float ownx = ld.ownx, owny = ld.owny, ownz = ld.ownz;
    // single-cell RNG chunk: moves m0..m0+15 (lanes 0-15 MOVE, 16-31 ACCEPT, 32-47 pair B), parked
    auto rng_single = [&](int m0) { rng_chunk_single(g, id, sweep, m0, py_, pz_, lcap4); };
    // (PB: the slab boundary launches run one level higher: the halo exchange waits for them)
    constexpr int kVisitPrio = PMC_VISIT_PRIO + PB > 3 ? 3 : PMC_VISIT_PRIO + PB;
    constexpr int kMovePrio = PMC_MOVE_PRIO == 0 ? 0 : (PMC_MOVE_PRIO + PB > 3 ? 3 : PMC_MOVE_PRIO + PB);
    constexpr int kTailPrio = PMC_MOVE_PRIO == 0 ? 0 : (PMC_MOVE_PRIO + 1 + PB > 3 ? 3 : PMC_MOVE_PRIO + 1 + PB);
    if (kVisitPrio) __builtin_amdgcn_s_setprio(kVisitPrio);
    const int n_own = __builtin_amdgcn_readlane(k_cnt, hb);    // lane hb = own cell
    if (n_own == 0) return true;                                // subsweep.h:252-253
    PMC_STAMP(4);
    // slot i's Fisher-Yates index sits on lane jb + i (the prologue's layout: the cell's half)
    int jb = hb;
    if (n_own > fy_have) {                         // rare: slots beyond the prologue's, on lane i
        jv = fy_words_single(g, id, sweep, buf);
        jb = 0;
    }

    // ---- Fisher-Yates shuffle of the own cell (random_shuffle, subsweep.h:50-58; fixes R1) ---
    int perm;
    if (QK & PMC_FLAG_QUIRK_R1) {
        // quirk R1 (pmc.h): random_int is always 0 (subsweep.h:38-40), so random_shuffle swaps slot i
        // with slot 0 for i = n-1 .. 0 -- the rotation slot l <- particle (l + 1) mod n
        perm = lane + 1 < n_own ? lane + 1 : 0;
    } else if (n_own <= 16) {
        // the permutation as 16 nibbles of one 64-bit scalar: each swap is a few SALU ops on
        // SGPRs (no VGPR read-modify-write chain through v_readlane), one VALU unpack at the end
        uint64_t P = 0xFEDCBA9876543210ull;
        for (int i = n_own - 1; i > 0; --i) {
            const uint32_t j = (uint32_t)__builtin_amdgcn_readlane(jv, jb + i);
            const uint32_t si = 4u * (uint32_t)i, sj = 4u * j;
            const uint64_t d = ((P >> si) ^ (P >> sj)) & 15u;   // a[i] ^ a[j]
            P ^= (d << si) | (d << sj);                        // swap (d == 0 when i == j)
        }
        perm = (int)((P >> (4u * (uint32_t)(lane & 15))) & 15u);
    } else {
        perm = lane;
        for (int i = n_own - 1; i > 0; --i) {
            const int j = __builtin_amdgcn_readlane(jv, jb + i);
            const int vi = __builtin_amdgcn_readlane(perm, i);
            const int vj = __builtin_amdgcn_readlane(perm, j);
            perm = lane == i ? vj : (lane == j ? vi : perm);
        }
    }

    PMC_STAMP(5);
    // ---- 3. stage the own cell (shuffled) into slots [0, n_own), then the neighbours --------
    // (filtered, compacted) after it (spec v11; v10 staged the own cell after the neighbours).
    // Own slot i holds particle i of the shuffled order, so a moving particle's slot is always
    // in the first 64-partner block and the moves leave it out of their term lists by one mask
    // bit (no LDS store to park it at +inf and restore it).
    {
        const float sxo = as_f(__shfl(as_i(ownx), perm));
        const float syo = as_f(__shfl(as_i(owny), perm));
        const float szo = as_f(__shfl(as_i(ownz), perm));
        if (lane < n_own) {
            px_[lane] = sxo + 0.0f;
            py_[lane] = syo + 0.0f;
            pz_[lane] = szo + 0.0f;
        }
    }
    float blo[3], bhi[3];
    pmc_cell_box(x, y, zg0, g.w, g.Lx, g.Ly, g.Lz, blo, bhi);
    int S_nb = n_own;   // next free slot
    // interior waves skip the image adds (an add of +0 changes nothing downstream -- staged
    // coordinates only enter differences that are squared)
    // append the lanes of `valid` whose partner passes the box filter, in lane order
    auto append = [&](float ux, float uy, float uz, unsigned long long valid) {
        const unsigned long long mk = __builtin_amdgcn_ballot_w64(pmc_box_d2(ux, uy, uz, blo, bhi) <= g.rc2f) & valid;
        const int nk = wave_uniform(__popcll(mk));
        // otherwise the cell goes to the fallback; exec-masked stores of the kept lanes
        if (S_nb + nk <= cap && __builtin_amdgcn_inverse_ballot_w64(mk)) {
            float* dst = px_ + S_nb + mbcnt64(mk);
            dst[0] = ux;
            dst[stride] = uy;
            dst[2 * stride] = uz;
        }
        S_nb += nk;
    };
    auto stage = [&](auto with_image) {
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const int k = 1 + q * CPP + kk;
            const int ks = k < 27 ? k : 26;
            const int cnt = __shfl(k_cnt, hb + ks);
            float ux = vx[q], uy = vy[q], uz = vz[q];
            if constexpr (decltype(with_image)::value) {
                ux = ux + __shfl(k_sx, hb + ks);
                uy = uy + __shfl(k_sy, hb + ks);
                uz = uz + __shfl(k_sz, hb + ks);
            }
            // lanes of stencil cells k < 27 (compile-time per pass), slot < count, box filter
            const unsigned long long live = stage_lane_mask<HS>(q);
            append(ux, uy, uz, __builtin_amdgcn_ballot_w64(p < cnt) & live);
        }
        if constexpr (HS < NSLOT) {
            // overflow passes: slots [HS, nmax) of the neighbours holding more than HS particles,
            // in stencil order, CPP cells per pass (lane group j: the j-th remaining cell); loads
            // issued here (the rare case pays its own round trip)
            unsigned long long ovm = __builtin_amdgcn_ballot_w64(lane >= hb + 1 && lane < hb + 27 && k_cnt > HS);
            while (ovm) {
                int ks = hb + 26, ncell = 0;
                for (; ncell < CPP && ovm; ++ncell) {
                    const int kb = (int)__builtin_ctzll(ovm);
                    ovm &= ovm - 1ull;
                    ks = kk == ncell ? kb : ks;
                }
                const int cnt = __shfl(k_cnt, ks);
                const int ps = HS + p;                                    // slot in the row
                const uint32_t off = (uint32_t)__shfl((int)k_off, ks) +
                                     (uint32_t)(ps < nm ? ps : 0) * lay_slot() * DiskAddr<OFF32>::kUnit;
                float ux, uy, uz;
                DiskAddr<OFF32>::ld3(disk, off, lay_dim(nm), ux, uy, uz);
                if constexpr (decltype(with_image)::value) {
                    ux = ux + __shfl(k_sx, ks);
                    uy = uy + __shfl(k_sy, ks);
                    uz = uz + __shfl(k_sz, ks);
                }
                append(ux, uy, uz, __builtin_amdgcn_ballot_w64(kk < ncell && ps < cnt));
            }
        }
    };
    if (edge) stage(std::true_type{});
    else stage(std::false_type{});
    PMC_STAMP(6);
    S_nb = wave_uniform(S_nb);   // keep it scalar past the divergent stores (structurizer joins)
    if (S_nb > cap) return false;                               // -> full-capacity fallback
    const int K = S_nb;
    // slots [K, roundup64(K)) are read by the last 64-lane block of every move: make them "far"
    // (+inf -> r2 = inf, never listed).  roundup64(K) <= stride; the clamp keeps every lane's
    // store inside the x row.
    const float kFar = __builtin_inff();
    const float kPad = 1.0e30f;
    px_[(K + lane) < stride ? K + lane : stride - 1] = kFar;

    PMC_STAMP(7);
    // cell centre for out_of_bound (subsweep.h:73-88): c*w - L/2 + w/2 in float
    const float hw = g.w / 2.0f;
    const float cxf = (float)x * g.w - g.Lx / 2.0f + hw;
    const float cyf = (float)y * g.w - g.Ly / 2.0f + hw;
    const float czf = (float)zg0 * g.w - g.Lz / 2.0f + hw;
    const float rc2 = g.rc2;
    const float nrc2 = -g.rc2;
    // PMC_R2_MIN through an SGPR: v_max_f32 |r2s|, s takes it with the free |.| modifier (a
    // literal operand would force a second max)
    const float r2min = as_f(wave_uniform(as_i(g.r2min)));

    double de_cell = 0.0;   // sum of the accepted moves' s = dE/4 (x4 at the end: exact)
    int n_acc = 0, n_ev = 0;
    int i = 0;
    // ---- 4. trial moves --------------------------------------------------------------------
    // The number of 64-partner blocks per move is fixed for the visit: the move loop is
    // instantiated per block count (1-4 at the main capacity), so each move runs straight-line
    // block code with no per-move loop or bound tests (the full-capacity launches keep the loop).
    auto move_loop = [&](auto nb_c) {
    constexpr int NB = decltype(nb_c)::value;
    unsigned long long pend = 0;                       // in-cell moves of the current round
    int sp_l = 0;                                      // lane j: row slot of the round's move j
    for (int m0 = 0; m0 < g.n_moves; m0 += (m0 == 0 ? first_len : 16)) {
        if (m0 > 0) rng_single(m0);
        const int clen = m0 == 0 ? first_len : 16;
        const int mend = wave_uniform((g.n_moves - m0) < clen ? (g.n_moves - m0) : clen);
        float* mvs = py_ + lcap4;                          // this chunk's move slots (y / z tails)
        // Rounds of up to n_own consecutive moves: moves cycle through the shuffled particles
        // (i = m mod n_own, subsweep.h:284-296), so the moves of a round touch different
        // particles and each one's trial position depends only on its particle's current
        // position.  Lane j forms move r0 + j's trial position and its out_of_bound test
        // (subsweep.h:73-88) in parallel, parks (qx, qy | qz) over the move's (d0, d1 | d2), and
        // only the in-cell moves run one after the other, in order.  Same arithmetic, same order
        // of state updates as one move at a time: bit for bit.
        for (int r0 = 0; r0 < mend;) {
            const int L = wave_uniform((mend - r0) < n_own ? (mend - r0) : n_own);
            {
                const int jl = lane < L ? lane : 0;
                const int pj = (i + jl) >= n_own ? i + jl - n_own : i + jl;
                float* slot = mvs + 2 * (r0 + jl);
                const float2 mva = *(const float2*)slot;            // (d0, d1)
                const int sp = pj;                                  // own slot = particle
                const float d2 = slot[stride];                      // d2 (z tail)
                const float qx = px_[sp] + mva.x;                   // make_move: x + g * sigma
                const float qy = py_[sp] + mva.y;
                const float qz = pz_[sp] + d2;
                // (d > hw || d < -hw) == (|d| > hw) for non-NaN d; |d| is a free source modifier
                const bool out = (__builtin_fabsf(qx - cxf) > hw) || (__builtin_fabsf(qy - cyf) > hw) ||
                                 (__builtin_fabsf(qz - czf) > hw);
                if (lane < L) {
                    *(float2*)slot = make_float2(qx, qy);
                    slot[stride] = qz;
                }
                pend = __builtin_amdgcn_ballot_w64(!out) & ((1ull << L) - 1ull);
                sp_l = sp;                                          // lane j: move j's row slot
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
            while (pend) {
                const int j = (int)__builtin_ctzll(pend);
                asm volatile("s_bitset0_b64 %0, %1" : "+s"(pend) : "s"(j));   // pend &= ~(1 << j)
                const int si = __builtin_amdgcn_readlane(sp_l, j);  // slot = particle of move j (< 64)
                const float* slot = mvs + 2 * (r0 + j);
                const float2 qa = *(const float2*)slot;             // (qx, qy)
                const float2 qb = *(const float2*)(slot + stride);  // (qz, T)
                const float qx = qa.x, qy = qa.y, qz = qb.x, Fm = qb.y;   // Fm: T's acceptance bound
                const float xi = px_[si], yi = py_[si], zi = pz_[si];
                ++n_ev;
                // the moving particle is left out of its own term list: its lane in block 0
                const unsigned long long sbit = 1ull << si;
                // 4a. term list: per block of 64 partners, the new-position terms within the
                // cutoff, then the old-position ones (sign bit set), compacted by ballot+mbcnt.
                // ~80% of staged pairs lie beyond rc for a given position; they are exactly 0
                // and never reach the reciprocal.
                int C = 0;   // wave-uniform
                // list one block's terms: the new-position ones within the cutoff, then the
                // old-position ones (negated r2, sign bit set), compacted by ballot + mbcnt
                auto list = [&](float r2n, float r2on, unsigned long long excl) {
                    const unsigned long long mn = __builtin_amdgcn_ballot_w64(r2n <= rc2) & ~excl;
                    const unsigned long long mo = __builtin_amdgcn_ballot_w64(r2on >= nrc2) & ~excl;
                    const int cn = C + __popcll(mn);
                    // exec-masked stores (2 SALU each) beat a select into a discard slot (one
                    // half-rate v_cndmask per list on gfx950); packed f32 for the distances
                    // (lo/hi = two blocks) measured 5% slower (v_pk_*_f32 issue at half rate)
                    if (__builtin_amdgcn_inverse_ballot_w64(mn)) buf[mbcnt64_add(mn, C)] = r2n;
                    if (__builtin_amdgcn_inverse_ballot_w64(mo)) buf[mbcnt64_add(mo, cn)] = r2on;
                    C = cn + __popcll(mo);
                };
                auto block = [&](int base, unsigned long long excl) {
                    // slots >= K hold +inf in x: their r2 is inf, never listed; the moving slot
                    // (block 0) is cleared from the masks by excl
                    const int k = base + lane;
                    const float xj = px_[k], yj = py_[k], zj = pz_[k];
                    // old-position term computed negated (= -r2o bit for bit, pmc_r2_neg):
                    // listed with its sign bit set at no extra instruction
                    list(pmc_r2(qx - xj, qy - yj, qz - zj), pmc_r2_neg(xi - xj, yi - yj, zi - zj), excl);
                };
                if constexpr (NB > 0) {
#pragma unroll
                    for (int b = 0; b < NB - 1; ++b) block(b * kWave, b == 0 ? sbit : 0ull);
                    const unsigned long long xl = NB == 1 ? sbit : 0ull;   // the moving slot (block 0)
                    block((NB - 1) * kWave, xl);
                } else {
                    block(0, sbit);
                    for (int base = kWave; base < K; base += kWave) block(base, 0ull);
                }
                // 4b. energies of the listed terms: term t on lane t % 64, ascending t.  The 64
                // slots after the list get kPad (r2 = 1e30: inv^3 underflows to +0, so the term
                // is exactly +0 and adding it leaves a lane's sum unchanged) -- no lane mask.
                // the serial tail (energy pass, reduction, accept) one priority level above
                // the rest of the moves (same-box A/B: phase -0.5%, profiles/r03pr_priority_ab.txt)
                if (kTailPrio) __builtin_amdgcn_s_setprio(kTailPrio);
                buf[C + lane] = kPad;
                // the first pass unconditionally (C == 0 reads only kPad: +0), the rest looped.  (A
                // lane sum may start at -0 where the oracle's starts 0 + -0 = +0: zeros of either
                // sign leave every nonzero sum, the accept test and de_cell unchanged.)
                float acc = lj4_signed_max(buf[lane], r2min);
                for (int t0 = kWave; t0 < C; t0 += kWave) acc = acc + lj4_signed_max(buf[t0 + lane], r2min);
                // quarter energies u are accumulated and reduced: s = dE/4.  Scaling by 4 is exact,
                // so dE = 4s equals the oracle's sum of the 4u, bit for bit, in any association
                const float sq = wave_sum_fixed_order_s(acc);           // SGPR
                const bool acc_mv = sq <= Fm;                            // accept_move, subsweep.h:209-216
                if (kMovePrio) __builtin_amdgcn_s_setprio(kMovePrio);
                if (acc_mv) {
                    px_[si] = qx;
                    py_[si] = qy;
                    pz_[si] = qz;
                    ++n_acc;
                    de_cell = de_cell + (double)sq;
                }
            }
            i += L;
            if (i >= n_own) i -= n_own;
            r0 += L;
        }
    }
    };
    // Wave priority by section (s_setprio): the moves at 2, the rest of the visit (shuffle, staging,
    // write-back) at 1, the prologue (stencil table, loads, RNG) at 0.  The moves' serial chains
    // (term list -> energy pass -> DPP reduction -> accept) then win VALU arbitration over waves
    // that are staging, and both over waves whose RNG pass overlaps their loads (same-box A/B,
    // profiles/r03pr_priority_ab.txt: sweep -0.5%; moves at 1 alone -0.3%; staging above the moves
    // +1.2%)
    if (kMovePrio) __builtin_amdgcn_s_setprio(kMovePrio);
    if constexpr (LCAP == kMainCap) {
        const int nb = (K + kWave - 1) / kWave;                 // 1..4 (K <= cap <= 224)
        if (nb <= 1) move_loop(std::integral_constant<int, 1>{});
        else if (nb == 2) move_loop(std::integral_constant<int, 2>{});
        else if (nb == 3) move_loop(std::integral_constant<int, 3>{});
        else move_loop(std::integral_constant<int, 4>{});
    } else {
        move_loop(std::integral_constant<int, 0>{});
    }

    if (kMovePrio) __builtin_amdgcn_s_setprio(kVisitPrio);
    PMC_STAMP(8);
    // ---- 5. write back the own cell in shuffled order (cpy_D_sh_to_Disk, subsweep.h:29-36) ----
    if (lane < n_own) {
        using A = DiskAddr<OFF32>;
        const uint32_t off = (c * (uint32_t)(3 * nm) + (uint32_t)lane * lay_slot()) * A::kUnit;
        A::st3(disk, off, lay_dim(nm), px_[lane], py_[lane], pz_[lane]);
        if constexpr (MIRROR) {
            const uint32_t r = mirror_mode == 0 ? (uint32_t)ta + (uint32_t)tb * (uint32_t)(g.cps_x >> 1)
                                                : (uint32_t)x + (uint32_t)g.cps_x * (uint32_t)y;
            float* m = mirror + (size_t)r * (3 * nm) + (uint32_t)lane * lay_slot();
            m[0] = px_[lane];
            m[lay_dim(nm)] = py_[lane];
            m[2u * lay_dim(nm)] = pz_[lane];
        }
    }
    // fixed-point conversion only when something was accepted (pmc_to_fixed(0) == 0)
    const int64_t de_fix = n_acc ? pmc_to_fixed(4.0 * de_cell) : 0;
    if (PMC_STATS_LANES ? lane < kStatCounters : lane == 0) {
        const int slot = t & (kStatSlots - 1);
#if PMC_STATS_LANES
        // lane k adds counter k: one no-return atomic instruction, 32 contiguous bytes
        const int64_t v = lane == 0 ? de_fix : (lane == 1 ? n_acc : (lane == 2 ? g.n_moves : n_ev));
        atomicAdd(&stats[stat_index(lane, slot)], (unsigned long long)v);
#else
        atomicAdd(&stats[stat_index(0, slot)], (unsigned long long)de_fix);
        atomicAdd(&stats[stat_index(1, slot)], (unsigned long long)n_acc);
        atomicAdd(&stats[stat_index(2, slot)], (unsigned long long)g.n_moves);
        atomicAdd(&stats[stat_index(3, slot)], (unsigned long long)n_ev);
#endif
    }
    PMC_STAMP(9);
    return true;
}

// The single-cell prologue: stencil table on lanes 0-26, the visit's loads, then one RNG pass
// (moves 0-15 and FY words of slots 0-63) while the loads fly.
template <int NSLOT, int NMC, int LCAP, int OFF32, bool MIRROR = false, int PB = 0, int QK = 0>
__device__ __forceinline__ bool subsweep_wave(const DevGeom& g, float* __restrict__ disk,
                                              const int16_t* __restrict__ ncnt, int ox, int oy, int oz,
                                              uint32_t sweep, unsigned long long* __restrict__ stats,
                                              float* __restrict__ px_, int lcap_rt, int cap, int t,
                                              int cz0, float* __restrict__ mirror = nullptr,
                                              int mirror_mode = 0, int czs = 1, int zlog = 0, int ncz_z = 0) {
    const int lane = threadIdx.x & (kWave - 1);
    const int nm = NMC > 0 ? NMC : g.nmax;
    const int lcap = LCAP > 0 ? LCAP : lcap_rt;
    const int stride = subsweep_stride(lcap);
    const int lcap4 = (lcap + 3) & ~3;
    float* py_ = px_ + stride;
    float* pz_ = py_ + stride;
    float* buf = pz_ + stride;
    const CellGeo cg = cell_geo(g, t, cz0, ox, oy, oz, zlog, ncz_z, czs);
    // quirk R2 (pmc.h): curand_init(1234, id, 0) on every launch -- the sweep index leaves the counters
    if (QK & PMC_FLAG_QUIRK_R2) sweep = 0u;
    PMC_STAMP(0);
    const StencilLane sl = stencil_lane(g, cg, lane, cg.edge);
    const int k_cnt = ncnt[sl.kc];
    const uint32_t k_off = sl.kc * (uint32_t)(3 * nm) * DiskAddr<OFF32>::kUnit;   // bytes (OFF32) or floats
    PMC_STAMP(1);
    VisitLoads<NSLOT, NMC, OFF32> ld;
    ld.issue(g, disk, cg, k_off, 0);
    PMC_STAMP(2);
    rng_chunk_single(g, cg.id, sweep, 0, py_, pz_, lcap4);
    const int jv = fy_words_single(g, cg.id, sweep, buf);
    PMC_STAMP(3);
    if (PB) __builtin_amdgcn_s_setprio(PB);
    return visit_cell<NSLOT, NMC, LCAP, OFF32, MIRROR, PB, QK>(g, disk, sweep, stats, px_, lcap_rt, cap, t, cg, 0, k_cnt,
                                                       k_off, sl.sx, sl.sy, sl.sz, ld, jv, 64, 16, mirror,
                                                       mirror_mode);
}

// The two-cell prologue (main launch): cells tA (lanes 0-31) and tB (lanes 32-63) of one colour,
// never neighbours.  One stencil table for both (cell A's on lanes 0-26, B's on 32-58), one Philox
// pass and one log/sqrt/sincos pass for both cells' first 10 moves and Fisher-Yates slots 0-15:
//   Philox lane h + l:  l < 10 MOVE call l, 10 <= l < 20 ACCEPT call l-10, 20 <= l < 24 SHUFFLE call l-20
//   transform lane h + l:  l < 10 pair A of move l, 10 <= l < 20 pair B of move l-10,
//                          20 <= l < 30 -log u of move l-20
// (h = 0 for A, 32 for B).  Cell A is visited with its rows loaded up front; B's randoms wait in
// registers and its loads go out after A.
// LCAP = kMainCap for the main launch (overflowing cells go to `ovf`), 27*nmax for the slab
// boundary launch (full capacity: nothing overflows, ovf unused; MIRROR rows as visit_cell).
template <int NSLOT, int NMC, int LCAP, int OFF32, bool MIRROR = false>
__device__ __forceinline__ void subsweep_pair(const DevGeom& g, float* __restrict__ disk,
                                              const int16_t* __restrict__ ncnt, int ox, int oy, int oz,
                                              uint32_t sweep, unsigned long long* __restrict__ stats,
                                              float* __restrict__ px_, int lcap_rt, int cap, int pA, int pB, bool hasB,
                                              int cz0, int zlog, int ncz, int* __restrict__ ovf, float* __restrict__ mirror = nullptr,
                                              int mirror_mode = 0) {
    const int lane = threadIdx.x & (kWave - 1);
    const int nm = NMC > 0 ? NMC : g.nmax;
    const int lcap = LCAP > 0 ? LCAP : lcap_rt;
    const int stride = subsweep_stride(lcap);
    const int lcap4 = (lcap + 3) & ~3;
    float* py_ = px_ + stride;
    float* pz_ = py_ + stride;
    float* buf = pz_ + stride;
    const int h = lane & 32;                       // 0: cell A's half, 32: cell B's
    const int l = lane & 31;
    const CellGeo ca = cell_geo(g, pA, cz0, ox, oy, oz, zlog, ncz);
    const CellGeo cb = cell_geo(g, hasB ? pB : pA, cz0, ox, oy, oz, zlog, ncz);
    const int tA = ca.t, tB = cb.t;
    [[maybe_unused]] int t = tA;                   // (PMC_STAMP's cell index)
    PMC_STAMP(0);
    // ---- stencil tables of both cells, counts ----------------------------------------------
    CellGeo cl = ca;                               // this lane's cell (per-lane selects)
    cl.x = h ? cb.x : ca.x;
    cl.y = h ? cb.y : ca.y;
    cl.zl = h ? cb.zl : ca.zl;
    cl.zg0 = h ? cb.zg0 : ca.zg0;
    cl.c = h ? cb.c : ca.c;
    const StencilLane sl = stencil_lane(g, cl, l, ca.edge || cb.edge);
    const int k_cnt = ncnt[sl.kc];
    const uint32_t k_off = sl.kc * (uint32_t)(3 * nm) * DiskAddr<OFF32>::kUnit;
    PMC_STAMP(1);
    VisitLoads<NSLOT, NMC, OFF32> ld;
    ld.issue(g, disk, ca, k_off, 0);
    PMC_STAMP(2);
    // ---- one RNG pass for both cells ---------------------------------------------------------
    const uint32_t idl = h ? cb.id : ca.id;
    uint32_t idx, tag;
    if (l < 10) { idx = (uint32_t)l; tag = PMC_TAG_MOVE; }
    else if (l < 20) { idx = (uint32_t)(l - 10); tag = PMC_TAG_ACCEPT; }
    else { idx = (uint32_t)(l - 20); tag = PMC_TAG_SHUFFLE; }
    const pmc_u32x4 w = philox_sched(idx, idl, sweep, tag, g);
    // Fisher-Yates words of slots 0-15 of both cells through LDS (the term list area is free):
    // SHUFFLE call k's 4 words are slots 4k..4k+3; lane h + i takes slot i's
    if (l >= 20 && l < 24) *(uint4*)(buf + (h >> 1) + 4 * (l - 20)) = make_uint4(w.v[0], w.v[1], w.v[2], w.v[3]);
    // transform inputs: lanes l < 10 their own (w0, w1); 10-19 (w2, w3) of MOVE lane l-10;
    // 20-29 w0 of ACCEPT lane l-10
    const int src = h + (l < 10 ? l : l - 10);
    const uint32_t s0 = (uint32_t)__shfl((int)w.v[0], src);
    const uint32_t s2 = (uint32_t)__shfl((int)w.v[2], src);
    const uint32_t s3 = (uint32_t)__shfl((int)w.v[3], src);
    const uint32_t wl = l < 10 ? w.v[0] : (l < 20 ? s2 : s0);
    const uint32_t ws = l < 10 ? w.v[1] : s3;
    const float lg = pmc_logf(pmc_u01(wl));
    const float R = __builtin_sqrtf(-2.0f * lg);
    float sn, cs;
    pmc_det_sincos_2pi(pmc_u01(ws), &sn, &cs);
    const float G0 = (R * cs) * g.sigma;          // l < 10: d0; 10-19: d2
    const float G1 = (R * sn) * g.sigma;          // l < 10: d1
    const float TT = accept_bound(-lg, g);           // 20-29: T's acceptance bound
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int fyw = (int)*(const uint32_t*)(buf + (h >> 1) + (l & 15));
    const int jv = (int)pmc_bounded((uint32_t)fyw, (uint32_t)((l & 15) + 1));
    // park cell h's first 10 moves (h = 0 now, 32 before B's visit)
    auto park = [&](int hh) {
        const int j = l < 10 ? l : (l < 20 ? l - 10 : l - 20);
        if ((lane & 32) == hh && l < 30) {
            if (l < 10) *(float2*)(py_ + lcap4 + 2 * j) = make_float2(G0, G1);
            else pz_[lcap4 + 2 * j + (l < 20 ? 0 : 1)] = l < 20 ? G0 : TT;
        }
    };
    park(0);
    PMC_STAMP(3);
    if (!visit_cell<NSLOT, NMC, LCAP, OFF32, MIRROR>(g, disk, sweep, stats, px_, lcap, cap, tA, ca, 0, k_cnt, k_off,
                                                     sl.sx, sl.sy, sl.sz, ld, jv, 16, 10, mirror, mirror_mode)) {
        if (lane == 0 && ovf) ovf[kOvfHead + atomicAdd(&ovf[kOvfCount], 1)] = tA;
    }
    if (!hasB) return;
    t = tB;
    PMC_STAMP(0);
    PMC_STAMP(1);
    park(32);
    ld.issue(g, disk, cb, k_off, 32);
    PMC_STAMP(2);
    PMC_STAMP(3);
    if (!visit_cell<NSLOT, NMC, LCAP, OFF32, MIRROR>(g, disk, sweep, stats, px_, lcap, cap, tB, cb, 32, k_cnt,
                                                     k_off, sl.sx, sl.sy, sl.sz, ld, jv, 16, 10, mirror, mirror_mode)) {
        if (lane == 0 && ovf) ovf[kOvfHead + atomicAdd(&ovf[kOvfCount], 1)] = tB;
    }
}



// Main launch: one wave per cell of the colour; LDS layout for kMainCap partners, capacity `cap`
// (<= kMainCap) partners per wave (sized for the occupancy; a cell whose filtered stencil
// exceeds it is queued in ovf for the fallback).
// amdgpu_waves_per_eu(8): 8 waves per SIMD (what the 5 KiB LDS slots allow) also bounds the SGPRs
template <int NSLOT, int NMC, bool OFF32>
__global__ __launch_bounds__(kWave * kSubWaves) __attribute__((amdgpu_waves_per_eu(PMC_MAIN_WAVES, PMC_MAIN_WAVES))) void k_subsweep(DevGeom g, float* __restrict__ disk,
                                                                  const int16_t* __restrict__ ncnt,
                                                                  int ox, int oy, int oz, uint32_t sweep,
                                                                  unsigned long long* __restrict__ stats,
                                                                  int cap, int* __restrict__ ovf, int cz0, int ncz) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform -> SALU math
    float* px_ = smem + wv * lds_floats_per_wave(kMainCap);
    // XCD-aware block order: blocks b and b+8 share an XCD (round-robin dispatch), so give each
    // XCD a contiguous run of cells -> neighbouring stencils share that XCD's L2.  Speed only.
    uint32_t nblk = gridDim.x, b = blockIdx.x;
#ifndef PMC_NO_XCD_REMAP
    if ((nblk & 7u) == 0u) b = (b & 7u) * (nblk >> 3) + (b >> 3);
#endif
    const int total = (g.cps_x >> 1) * (g.cps_y >> 1) * ncz;
#if PMC_CELLS_PER_WAVE == 2
    // two cells per wave (shared stencil table and RNG pass): wave w takes the cells at positions
    // 2w and 2w+1 of the visiting order
    const int t = 2 * ((int)b * kSubWaves + wv);
    if (t >= total) return;
    // groups of PMC_ZGROUP colour planes, a short last group for a ragged count (PMC_ZGROUP <= 4;
    // larger groups only for counts they divide)
    const int zlog = (PMC_ZGROUP <= 4 || (ncz & ((1 << kZGroupLog) - 1)) == 0) ? kZGroupLog : 0;
    subsweep_pair<NSLOT, NMC, kMainCap, OFF32>(g, disk, ncnt, ox, oy, oz, sweep, stats, px_, kMainCap, cap, t, t + 1,
                                               t + 1 < total, cz0, zlog, ncz, ovf);
#else
    const int t = (int)b * kSubWaves + wv;
    if (t >= total) return;
    if (!subsweep_wave<NSLOT, NMC, kMainCap, OFF32>(g, disk, ncnt, ox, oy, oz, sweep, stats, px_, kMainCap, cap,
                                                t, cz0)) {
        if ((threadIdx.x & (kWave - 1)) == 0) ovf[kOvfHead + atomicAdd(&ovf[kOvfCount], 1)] = t;
    }
#endif
}

// Mixed main launch (PMC_MIXED_SINGLES=<s>, A/B switch): each XCD's contiguous run of cells is
// visited two cells per wave, except its last s cells, one per wave.  The hardware dispatches blocks
// in order, so the single-cell waves are the launch's last: the tail a launch spends draining its
// last round of wave slots is then half a two-cell wave lifetime.  Same cells, same visit: results
// bit-identical.  Grid: 8 * (pair_waves + singles) one-wave blocks (block b on XCD b % 8).
template <int NSLOT, int NMC, bool OFF32>
__global__ __launch_bounds__(kWave * kSubWaves) __attribute__((amdgpu_waves_per_eu(PMC_MAIN_WAVES, PMC_MAIN_WAVES))) void k_subsweep_mixed(
    DevGeom g, float* __restrict__ disk, const int16_t* __restrict__ ncnt, int ox, int oy, int oz, uint32_t sweep,
    unsigned long long* __restrict__ stats, int cap, int* __restrict__ ovf, int cz0, int ncz, int per_xcd, int pair_waves) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* px_ = smem;
    const int b = (int)blockIdx.x;
    const int base = (b & 7) * per_xcd;
    const int r = b >> 3;
    const int total = (g.cps_x >> 1) * (g.cps_y >> 1) * ncz;
    const int end = base + per_xcd < total ? base + per_xcd : total;
    const int zlog = (PMC_ZGROUP <= 4 || (ncz & ((1 << kZGroupLog) - 1)) == 0) ? kZGroupLog : 0;
    if (r < pair_waves) {
        const int p = base + 2 * r;
        if (p >= end) return;
        subsweep_pair<NSLOT, NMC, kMainCap, OFF32>(g, disk, ncnt, ox, oy, oz, sweep, stats, px_, kMainCap, cap, p, p + 1,
                                                   p + 1 < end, cz0, zlog, ncz, ovf);
    } else {
        const int p = base + 2 * pair_waves + (r - pair_waves);
        if (p >= end) return;
        if (!subsweep_wave<NSLOT, NMC, kMainCap, OFF32>(g, disk, ncnt, ox, oy, oz, sweep, stats, px_, kMainCap, cap, p,
                                                        cz0, nullptr, 0, 1, zlog, ncz)) {
            if ((threadIdx.x & (kWave - 1)) == 0)
                ovf[kOvfHead + atomicAdd(&ovf[kOvfCount], 1)] = cell_geo(g, p, cz0, ox, oy, oz, zlog, ncz).t;
        }
    }
}

// Boundary-plane launch of the slab driver: ONE cell per wave at the main launch's capacity (5 KiB
// of LDS per wave).  The boundary chain's launches are single colour planes that run beside the
// interior chains' launches and wait for their waves to retire; a boundary phase then takes about
// one wave lifetime, which one cell per wave halves (the two-cell waves of the main launch only pay
// off when a launch is many rounds of waves long).  Cells over the capacity go to the queue `ovf`,
// which the fallback launch after it visits.  Written-back rows may also go to `mirror`.
template <int NSLOT, int NMC, bool OFF32>
__global__ __launch_bounds__(kWave * kSubWaves) void k_subsweep_direct(DevGeom g, float* __restrict__ disk,
                                                                         const int16_t* __restrict__ ncnt,
                                                                         int ox, int oy, int oz, uint32_t sweep,
                                                                         unsigned long long* __restrict__ stats,
                                                                         int cap, int* __restrict__ ovf, int cz0,
                                                                         int ncz, float* __restrict__ mirror,
                                                                         int mirror_mode) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float* px_ = smem + wv * lds_floats_per_wave(kMainCap);
    const int total = (g.cps_x >> 1) * (g.cps_y >> 1) * ncz;
    const int t = (int)blockIdx.x * kSubWaves + wv;
    if (t >= total) return;
    bool ok;
    if (mirror)
        ok = subsweep_wave<NSLOT, NMC, kMainCap, OFF32, true, PMC_BOUNDARY_PB>(g, disk, ncnt, ox, oy, oz, sweep, stats, px_, kMainCap,
                                                             cap, t, cz0, mirror, mirror_mode);
    else
        ok = subsweep_wave<NSLOT, NMC, kMainCap, OFF32, false, PMC_BOUNDARY_PB>(g, disk, ncnt, ox, oy, oz, sweep, stats, px_, kMainCap, cap,
                                                       t, cz0);
    if (!ok && (threadIdx.x & (kWave - 1)) == 0) ovf[kOvfHead + atomicAdd(&ovf[kOvfCount], 1)] = t;
}

// Two colour planes czs apart in ONE boundary launch (the two-plane-halo schedule's first run: the
// boundary plane and the halo plane the neighbour owns, at opposite faces of the slab, so they never
// interact): one cell per wave at the main capacity, cells of plane 0 of the pair first; each plane's
// counters go to its own buffer (the redundant halo plane's to a scratch buffer).  Overflowing cells
// are queued for k_subsweep_fallback2.
template <int NSLOT, int NMC, bool OFF32>
__global__ __launch_bounds__(kWave * kSubWaves) void k_subsweep_direct2(DevGeom g, float* __restrict__ disk,
                                                                          const int16_t* __restrict__ ncnt,
                                                                          int ox, int oy, int oz, uint32_t sweep,
                                                                          unsigned long long* __restrict__ stats0,
                                                                          unsigned long long* __restrict__ stats1,
                                                                          int cap, int* __restrict__ ovf, int cz0, int czs) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float* px_ = smem + wv * lds_floats_per_wave(kMainCap);
    const int per_plane = (g.cps_x >> 1) * (g.cps_y >> 1);
    const int t = (int)blockIdx.x * kSubWaves + wv;
    if (t >= 2 * per_plane) return;
    unsigned long long* st = t < per_plane ? stats0 : stats1;
    const bool ok = subsweep_wave<NSLOT, NMC, kMainCap, OFF32, false, PMC_BOUNDARY_PB>(
        g, disk, ncnt, ox, oy, oz, sweep, st, px_, kMainCap, cap, t, cz0, nullptr, 0, czs);
    if (!ok && (threadIdx.x & (kWave - 1)) == 0) ovf[kOvfHead + atomicAdd(&ovf[kOvfCount], 1)] = t;
}

// Fallback launch: full capacity (27*nmax partners per wave), a fixed grid striding over the
// queued cells.  Cells of one colour are independent, so the order does not matter.
template <int NSLOT, int NMC, bool OFF32, bool MIRROR = false>
__global__ __launch_bounds__(kWave * kSubWaves) void k_subsweep_fallback(DevGeom g, float* __restrict__ disk,
                                                                           const int16_t* __restrict__ ncnt,
                                                                           int ox, int oy, int oz, uint32_t sweep,
                                                                           unsigned long long* __restrict__ stats,
                                                                           int* __restrict__ ovf, int cz0,
                                                                           float* __restrict__ mirror, int mirror_mode,
                                                                           int czs, unsigned long long* __restrict__ stats1) {
    // czs > 1: the queue of a two-plane launch (k_subsweep_direct2): planes czs apart, the second
    // plane's counters to stats1
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int full = 27 * (NMC > 0 ? NMC : g.nmax);
    const int per_plane = (g.cps_x >> 1) * (g.cps_y >> 1);
    float* px_ = smem + wv * lds_floats_per_wave(full);
    const int count = __builtin_amdgcn_readfirstlane(ovf[kOvfCount]);
    // nothing queued (the common case): nothing to clear either -- every workgroup reads the same
    // count, so either all of them take part in the done-counting below or none does (no atomic
    // round trip on the phase's critical path)
    if (count == 0) return;
    for (int e = (int)blockIdx.x * kSubWaves + wv; e < count; e += (int)gridDim.x * kSubWaves) {
        const int t = __builtin_amdgcn_readfirstlane(ovf[kOvfHead + e]);
        unsigned long long* st = (czs != 1 && t >= per_plane) ? stats1 : stats;
        (void)subsweep_wave<NSLOT, NMC, 27 * NMC, OFF32, MIRROR>(g, disk, ncnt, ox, oy, oz, sweep, st, px_, full,
                                                                 full, t, cz0, mirror, mirror_mode, czs);
    }
    // the queue is cleared for the next launch (no memset between launches; graph replays start
    // from a clean queue): a one-workgroup grid clears it itself; otherwise the last workgroup to
    // finish (every workgroup has read the count by then) does
    __syncthreads();   // every wave of the workgroup has read the count
    if (gridDim.x == 1) {
        if (threadIdx.x == 0 && count != 0) ovf[kOvfCount] = 0;
        return;
    }
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(&ovf[kOvfDone], 1) == (int)gridDim.x - 1) {
            ovf[kOvfCount] = 0;
            ovf[kOvfDone] = 0;
        }
    }
}

// Small launches (a colour phase of at most PMC_SMALL_LAUNCH cells, default 8192: boxes up to
// ~40^3): one cell per wave at full capacity (27*nmax partners, nothing overflows), so the phase is
// ONE launch -- no fallback launch after it -- and its waves live half as long as the main launch's
// two-cell waves.  Below a round of the chip's wave slots a phase lasts about one wave lifetime plus
// the launch, so both halve.  Same per-cell code as every other path: results bit-identical.
template <int NSLOT, int NMC, bool OFF32, int PB = 0, int QK = 0>
__global__ __launch_bounds__(kWave * kSubWaves) void k_subsweep_full(DevGeom g, float* __restrict__ disk,
                                                                       const int16_t* __restrict__ ncnt,
                                                                       int ox, int oy, int oz, uint32_t sweep,
                                                                       unsigned long long* __restrict__ stats,
                                                                       int cz0, int ncz) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int full = 27 * (NMC > 0 ? NMC : g.nmax);
    float* px_ = smem + wv * lds_floats_per_wave(full);
    const int total = (g.cps_x >> 1) * (g.cps_y >> 1) * ncz;
    const int t = (int)blockIdx.x * kSubWaves + wv;
    if (t >= total) return;
    (void)subsweep_wave<NSLOT, NMC, 27 * NMC, OFF32, false, PB, QK>(g, disk, ncnt, ox, oy, oz, sweep, stats, px_, full,
                                                                     full, t, cz0);
}


// colour phases of at most this many cells use k_subsweep_full (PMC_SMALL_LAUNCH; 0 disables it).
// Measured (profiles/r03sl_small_launch.txt): 16^3 0.122 -> 0.073 ms per sweep, 24^3 0.141 ->
// 0.087, 32^3 0.144 -> 0.098; larger launches are faster with the main kernel (48^3: 0.209 against
// 0.225, 64^3: 0.396 against 0.505), and so are the slab's boundary-plane launches, which share the
// chip with the interior chains (4-rank rehearsal 0.682 against 0.692 ms per rank sweep).
static int64_t env_cells(const char* name, int64_t dflt) {
    const char* v = std::getenv(name);
    return v ? (int64_t)std::atoll(v) : dflt;
}

// ------------------------------------------------------------------------------------------
// Small boxes: whole sweeps in ONE launch on ONE XCD (pmc_run_small).
//
// At 16^3 a colour phase is 512 cells: a sweep of 17 launches is dispatch-bound (~7.5 us each for
// a few us of work).  This kernel runs `count` sweeps (8 colour phases + shiftCells each) with P
// persistent one-wave workgroups and an in-kernel barrier where each kernel boundary was.  The
// launch has 8*P workgroups dealt round-robin over the 8 XCDs (tools/ubench/xcc_map.hip), and only
// those the XCC_ID register puts on XCD 0 stay: all P participants then share XCD 0's L2, which is the
// coherence point for them -- a barrier needs no L2 write-back, only (a) its stores completed
// (s_waitcnt vmcnt(0): the vector L1 is write-through), (b) an L2 atomic, (c) the vector L1
// invalidated afterwards (buffer_inv sc1; no buffer_wbl2).  (A grid barrier across the 8 XCDs must write back and
// invalidate each L2 -- round 2 measured that 3-6x slower than eager launches.)  More than P
// blocks on XCD 0 (a dispatch that is not round-robin) flags error bit 4.  Every cell
// visit uses the full-capacity LDS layout (27*nmax partners: no overflow queue), 9.9 KB per wave,
// 16 waves per CU: XCD 0 holds 512 participants.  Barrier waits give up after ~1 s of s_memrealtime
// (error flag value 8, bit 3) so a participant that never arrives cannot hang the GPU.
// ------------------------------------------------------------------------------------------
struct SmallPlans {
    int n;                          // sweeps in this launch
    uint32_t first;                 // sweep index of the first
    int order[kSmallSweeps][8];     // colour order
    int f[kSmallSweeps];            // shift axis
    float d[kSmallSweeps];          // shift distance
};

__device__ __forceinline__ bool small_barrier(unsigned* bar, unsigned target, uint32_t* flags) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if ((threadIdx.x & (kWave - 1)) == 0) __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();        // 100 MHz
    bool ok = true;
    while (true) {
        const unsigned v = __builtin_amdgcn_readfirstlane(
            (int)__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));   // L1 bypass, XCD 0's L2
        if ((int)(v - target) >= 0) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {
            ok = false;
            if ((threadIdx.x & (kWave - 1)) == 0) atomicOr(flags, 8u);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    // vector L1: drop stale lines.  (sc0, workgroup scope, is a no-op outside threadgroup-split
    // mode -- 8^3 read stale neighbour rows with it; sc1, agent scope, invalidates the L1 and only
    // MTYPE NC lines of the L2, none of which hipMalloc memory has.)
    asm volatile("buffer_inv sc1" ::: "memory");
    return ok;
}

// shiftCells of cells [c0, c0 + 64/NSLOT) (one cell per NSLOT-lane group), the arithmetic of k_shift
// (VS shiftCells.h:38-108, float s of the fixed copy) for one cell per lane group
template <int NSLOT>
__device__ __forceinline__ void shift_cells_wave(const DevGeom& g, const float* __restrict__ din,
                                                 const int16_t* __restrict__ nin, float* __restrict__ dout,
                                                 int16_t* __restrict__ nout, int f, float d, uint32_t* __restrict__ flags,
                                                 int c0, int ncells) {
    const int lane = threadIdx.x & (kWave - 1);
    const int p = lane & (NSLOT - 1);
    const int ci = c0 + lane / NSLOT;
    const bool live = ci < ncells;
    const int c = live ? ci : 0;
    const int nm = g.nmax;
    const float w = g.w;
    const int cps_f = f == 0 ? g.cps_x : (f == 1 ? g.cps_y : g.cps_z);
    const float Lf = f == 0 ? g.Lx : (f == 1 ? g.Ly : g.Lz);
    const int dir = (d <= 0) ? -1 : 1;
    const float s = w * (float)dir;
    const int x = c % g.cps_x, y = (c / g.cps_x) % g.cps_y, z = c / (g.cps_x * g.cps_y);
    const int cidf = f == 0 ? x : (f == 1 ? y : z);
    const float offset = (float)cidf * w - Lf / 2.0f;
    int nbg = cidf + dir;
    if (nbg < 0) nbg = cps_f - 1; else if (nbg >= cps_f) nbg = 0;
    const int nx = f == 0 ? nbg : x, ny = f == 1 ? nbg : y, nz = f == 2 ? nbg : z;
    const float offset_nb = (float)nbg * w - Lf / 2.0f;
    const int cnb = nx + g.cps_x * (ny + g.cps_y * nz);
    const int ncur = live ? (int)nin[c] : 0, nnb = live ? (int)nin[cnb] : 0;
    const int pp = p < nm ? p : 0;
    float own[3], nbv[3];
#pragma unroll
    for (int dim = 0; dim < 3; ++dim) {
        own[dim] = din[(uint64_t)c * (uint64_t)(3 * nm) + (uint64_t)(dim * lay_dim(nm) + pp * lay_slot())];
        nbv[dim] = din[(uint64_t)cnb * (uint64_t)(3 * nm) + (uint64_t)(dim * lay_dim(nm) + pp * lay_slot())];
    }
    const int gsh = lane & ~(NSLOT - 1);
    const unsigned long long gmask = NSLOT == 64 ? ~0ull : ((1ull << (NSLOT & 63)) - 1ull);
    const unsigned long long below = (1ull << p) - 1ull;
    const float xf = f == 0 ? own[0] : (f == 1 ? own[1] : own[2]);
    const float xfn = f == 0 ? nbv[0] : (f == 1 ? nbv[1] : nbv[2]);
    const float D = (xf - offset) - d;
    const float Dn = (xfn - offset_nb) - d;
    const bool keep = (p < ncur) && (D > 0 && D <= w);
    const bool take = (p < nnb) && !(Dn > 0 && Dn <= w);
    const unsigned long long km = (__ballot(keep) >> gsh) & gmask;
    const unsigned long long tm = (__ballot(take) >> gsh) & gmask;
    const int nk = __popcll(km);
    const int nnew = nk + __popcll(tm);
    const uint64_t ob = (uint64_t)c * (uint64_t)(3 * nm);
    if (keep) {
        const int dst = __popcll(km & below);
        if (dst < nm)
#pragma unroll
            for (int dim = 0; dim < 3; ++dim)
                dout[ob + (uint64_t)(dim * lay_dim(nm) + dst * lay_slot())] = (dim == f) ? D + offset : own[dim];
    }
    if (take) {
        const int dst = nk + __popcll(tm & below);
        if (dst < nm)
#pragma unroll
            for (int dim = 0; dim < 3; ++dim)
                dout[ob + (uint64_t)(dim * lay_dim(nm) + dst * lay_slot())] = (dim == f) ? ((Dn + offset) + s) : nbv[dim];
    }
    if (live && p == 0) {
        nout[c] = (int16_t)(nnew > nm ? nm : nnew);
        if (nnew > nm) atomicOr(flags, 1u);
    }
}

template <int NSLOT, int NMC, bool OFF32>
__global__ __launch_bounds__(kWave) void k_sweep_small(DevGeom g, float* __restrict__ disk0, int16_t* __restrict__ n0,
                                                      float* __restrict__ disk1, int16_t* __restrict__ n1,
                                                      unsigned long long* __restrict__ stats, uint32_t* __restrict__ flags,
                                                      unsigned* __restrict__ bar, SmallPlans plans) {
    // the dispatcher deals workgroups round-robin over the 8 XCDs, but from wherever the previous
    // launch left off: participate by the XCC_ID register, not by b % 8.  Consecutive blocks of one
    // XCD are 8 apart, so b / 8 numbers XCD 0's blocks 0..P-1.
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if ((xcc & 0xFu) != 0u) return;
    if ((int)(blockIdx.x >> 3) >= (int)(gridDim.x >> 3)) {   // (a 9th block on XCD 0: mapping broken)
        if ((threadIdx.x & (kWave - 1)) == 0) atomicOr(flags, 16u);
        return;
    }
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int full = 27 * NMC;
    const int P = (int)(gridDim.x >> 3), pid = (int)(blockIdx.x >> 3);
    const int per_colour = (g.cps_x >> 1) * (g.cps_y >> 1) * (g.cps_z >> 1);
    const int cells = g.cps_x * g.cps_y * g.cps_z;
    unsigned target = 0;
    float* dk[2] = {disk0, disk1};
    int16_t* nk[2] = {n0, n1};
    int cur = 0;
    for (int k = 0; k < plans.n; ++k) {
        const uint32_t sweep = plans.first + (uint32_t)k;
        for (int ph = 0; ph < 8; ++ph) {
            int o[3];
            pmc_colour_offset(plans.order[k][ph], o);
            for (int t = pid; t < per_colour; t += P)
                (void)subsweep_wave<NSLOT, NMC, full, OFF32>(g, dk[cur], nk[cur], o[0], o[1], o[2], sweep, stats, smem,
                                                             full, full, t, 0);
            target += (unsigned)P;
            if (!small_barrier(bar, target, flags)) return;
        }
        constexpr int CPW = kWave / NSLOT;
        for (int c0 = pid * CPW; c0 < cells; c0 += P * CPW)
            shift_cells_wave<NSLOT>(g, dk[cur], nk[cur], dk[cur ^ 1], nk[cur ^ 1], plans.f[k], plans.d[k], flags, c0, cells);
        target += (unsigned)P;
        if (!small_barrier(bar, target, flags)) return;
        cur ^= 1;
    }
}

// ------------------------------------------------------------------------------------------
// shiftCells: NSLOT lanes per cell, ballot compaction (shiftCells.h:28-144; float s of the fixed
// copy CUDA-Parallel-MC/CUDA-Parallel-MC/shiftCells.h:23-112).  Double-buffered.
// ------------------------------------------------------------------------------------------
#ifndef PMC_SHIFT_THREADS
#define PMC_SHIFT_THREADS 256   // k_shift workgroup size
#endif
constexpr int kShiftThreads = PMC_SHIFT_THREADS;
#ifndef PMC_SHIFT_LINES
#define PMC_SHIFT_LINES 1   // k_shift_run stores whole 64-B lines of each output record from LDS (0: per slot)
#endif
#ifndef PMC_SHIFT_RUN_LEN
#define PMC_SHIFT_RUN_LEN 4
#endif
constexpr int kShiftRun = PMC_SHIFT_RUN_LEN;   // k_shift_run: cells per lane group along the shift axis

// PMC_SHIFT_NT=1: the output rows as nontemporal stores (streamed past the L2, which then keeps
// the input rows the neighbour reads re-fetch)
__device__ __forceinline__ void shift_store(float* p, float v) {
#if PMC_SHIFT_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// OFF32 (buffer < 4 GiB, PMC_SHIFT_OFF32=1): 32-bit byte offsets from the SGPR bases (global_load /
// store with a VGPR offset), else 64-bit element addressing (default: the 32-bit form saves 170
// address instructions and 27 VGPRs but not time, profiles/r04_shift_counters.json)
template <int NSLOT, int U, int OFF32, bool S1 = false>
__global__ __launch_bounds__(kShiftThreads) void k_shift(DevGeom g, const float* __restrict__ din,
                                               const int16_t* __restrict__ nin, float* __restrict__ dout,
                                               int16_t* __restrict__ nout, int f, float d,
                                               uint32_t* __restrict__ flags, int zl0) {
    // grid: (ceil(cps_x / (CPB*U)), cps_y, planes); local plane zl = zl0 + blockIdx.z (zl0 = -1
    // takes the bottom halo plane of a slab: the slab driver shifts the halo planes it can compute
    // from its own data instead of receiving them).  NSLOT lanes per cell, CPB cells per block
    // along x per unrolled step j, U steps whose loads are all issued before any use (U times
    // the bytes in flight per wave: the kernel is latency-bound at one cell per lane group)
    constexpr int CPB = kShiftThreads / NSLOT;
    const int lane = threadIdx.x & (kWave - 1);
    const int p = threadIdx.x & (NSLOT - 1);
    // (the XCD-contiguous and y-chunked block orders measured no faster, profiles/r03o_shift_xcd_ab.txt,
    // r04 DESIGN section 6; removed in round 5)
    const int bx = (int)blockIdx.x, y = (int)blockIdx.y, zl = zl0 + (int)blockIdx.z;
    const int nm = g.nmax;
    const float w = g.w;
    const int cps_f = f == 0 ? g.cps_x : (f == 1 ? g.cps_y : g.cps_z);
    const float Lf = f == 0 ? g.Lx : (f == 1 ? g.Ly : g.Lz);
    const int dir = (d <= 0) ? -1 : 1;                     // VS shiftCells.h:38-44
    // quirk S1 (pmc.h): the root copy's int s[3] (shiftCells.h:31,105) truncates w*dir
    const float s = S1 ? (float)(int)(w * (float)dir) : w * (float)dir;
    const uint32_t plane = (uint32_t)g.cps_x * (uint32_t)g.cps_y;
    const int pp = p < nm ? p : 0;
    const int gsh = lane & ~(NSLOT - 1);
    const unsigned long long gmask = NSLOT == 64 ? ~0ull : ((1ull << (NSLOT & 63)) - 1ull);
    const unsigned long long below = (1ull << p) - 1ull;

    bool live[U];
    uint32_t c[U], cnbv[U];
    int ncur[U], nnb[U];
    float offset[U], offset_nb[U], own[U][3], nbv[U][3];
    // slot pp of cell c[j] and of its dir-neighbour (x, y, z: one dwordx3 each in the packed layout)
    auto load_slots = [&](int j) {
        if constexpr (OFF32) {
            const uint32_t oc = (c[j] * (uint32_t)(3 * nm) + (uint32_t)pp * lay_slot()) * 4u;
            const uint32_t on = (cnbv[j] * (uint32_t)(3 * nm) + (uint32_t)pp * lay_slot()) * 4u;
            DiskAddr<1>::ld3(din, oc, lay_dim(nm), own[j][0], own[j][1], own[j][2]);
            DiskAddr<1>::ld3(din, on, lay_dim(nm), nbv[j][0], nbv[j][1], nbv[j][2]);
        } else {
            const uint64_t oc = (uint64_t)c[j] * (uint64_t)(3 * nm) + (uint64_t)pp * lay_slot();
            const uint64_t on = (uint64_t)cnbv[j] * (uint64_t)(3 * nm) + (uint64_t)pp * lay_slot();
            own[j][0] = din[oc];
            own[j][1] = din[oc + lay_dim(nm)];
            own[j][2] = din[oc + 2 * lay_dim(nm)];
            nbv[j][0] = din[on];
            nbv[j][1] = din[on + lay_dim(nm)];
            nbv[j][2] = din[on + 2 * lay_dim(nm)];
        }
    };
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const int x = (bx * U + j) * CPB + (int)(threadIdx.x / NSLOT);
        live[j] = x < g.cps_x;
        const int xx = live[j] ? x : 0;
        int cidf = f == 0 ? xx : (f == 1 ? y : g.z0 + zl);
        if (cidf < 0) cidf += cps_f; else if (cidf >= cps_f) cidf -= cps_f;   // halo planes wrap
        offset[j] = (float)cidf * w - Lf / 2.0f;           // VS :46
        int nbg = cidf + dir;
        if (nbg < 0) nbg = cps_f - 1; else if (nbg >= cps_f) nbg = 0;
        int nx = xx, ny = y, nz = zl;
        if (f == 0) nx = nbg; else if (f == 1) ny = nbg; else nz = g.halo ? zl + dir : nbg;
        offset_nb[j] = (float)nbg * w - Lf / 2.0f;
        c[j] = (uint32_t)xx + (uint32_t)g.cps_x * (uint32_t)y + plane * (uint32_t)(zl + g.halo);
        const uint32_t cnb = (uint32_t)nx + (uint32_t)g.cps_x * (uint32_t)ny + plane * (uint32_t)(nz + g.halo);
        // one round trip: both counts and all six rows (a 64 B row sits inside one 128 B line)
        // unconditional loads (c, cnb are valid cells for dead lanes too: no branch, no wait)
        const int nc0 = OFF32 ? *(const int16_t*)((const char*)nin + (uint64_t)(c[j] * 2u)) : nin[c[j]];
        const int nn0 = OFF32 ? *(const int16_t*)((const char*)nin + (uint64_t)(cnb * 2u)) : nin[cnb];
        ncur[j] = live[j] ? nc0 : 0;
        nnb[j] = live[j] ? nn0 : 0;
        cnbv[j] = cnb;
        // every slot of both cells in the same round trip as the counts.  (Loading only slots [0, 8)
        // here and the rest after the counts when a cell of the wave holds more -- two of the packed
        // cell's three 64-B lines -- measured slower: 0.169 against 0.144 ms,
        // profiles/r05i_shift_half_ab.txt; so did loading only the occupied slots, r05h.)
        load_slots(j);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const float xf = f == 0 ? own[j][0] : (f == 1 ? own[j][1] : own[j][2]);
        const float xfn = f == 0 ? nbv[j][0] : (f == 1 ? nbv[j][1] : nbv[j][2]);
        const float D = (xf - offset[j]) - d;               // shortDisk - d
        const float Dn = (xfn - offset_nb[j]) - d;
        const bool keep = (p < ncur[j]) && (D > 0 && D <= w);
        const bool take = (p < nnb[j]) && !(Dn > 0 && Dn <= w);
        const unsigned long long km = (__ballot(keep) >> gsh) & gmask;
        const unsigned long long tm = (__ballot(take) >> gsh) & gmask;
        const int nk = __popcll(km);
        const int nnew = nk + __popcll(tm);
        // output slot `dst` of cell c[j] (element offset c*3nm + dst*lay_slot; dimension dim at +dim*lay_dim)
        auto out_at = [&](int dst) -> float* {
            const uint32_t e = (uint32_t)dst * lay_slot();
            if constexpr (OFF32)
                return (float*)((char*)dout + (uint64_t)((c[j] * (uint32_t)(3 * nm) + e) * 4u));
            else
                return dout + (uint64_t)c[j] * (uint64_t)(3 * nm) + (uint64_t)e;
        };
        if (keep) {
            const int dst = __popcll(km & below);
            if (dst < nm) {
                float* q = out_at(dst);
#pragma unroll
                for (int dim = 0; dim < 3; ++dim)
                    shift_store(q + dim * lay_dim(nm), (dim == f) ? D + offset[j] : own[j][dim]);
            }
        }
        if (take) {
            const int dst = nk + __popcll(tm & below);
            if (dst < nm) {
                float* q = out_at(dst);
#pragma unroll
                for (int dim = 0; dim < 3; ++dim)   // own offset (VS shiftCells.h:96)
                    shift_store(q + dim * lay_dim(nm), (dim == f) ? ((Dn + offset[j]) + s) : nbv[j][dim]);
            }
        }
        if (live[j] && p == 0) {
            if constexpr (OFF32)
                *(int16_t*)((char*)nout + (uint64_t)(c[j] * 2u)) = (int16_t)(nnew > nm ? nm : nnew);
            else
                nout[c[j]] = (int16_t)(nnew > nm ? nm : nnew);
            if (nnew > nm) atomicOr(flags, 1u);
        }
    }
}

// shiftCells along runs of the shift axis (launch_shift_planes; PMC_SHIFT_RUN=0: k_shift).  A lane
// group (NSLOT lanes, one per slot) takes R cells in a row along f; the dir-neighbour of cell j is
// cell j+dir of the same run -- already in registers -- except at the run's end, whose neighbour is
// one extra cell.  Each input cell is then read (R+1)/R times instead of twice (k_shift reads every
// cell as its own and again as its neighbour's neighbour, 128 B per cell each time), and the keep /
// take rule is k_shift's (VS shiftCells.h:46-102) cell for cell, so the output is the same bits.
// Lane groups: x fastest across a wave for f = 1, 2 (four neighbouring cells per wave load), runs
// along x for f = 0.  Range: local planes [zl0, zl0 + nzr), halo planes included as in k_shift.
template <int NSLOT, int R, int OFF32, bool S1 = false>
__global__ __launch_bounds__(kShiftThreads) void k_shift_run(DevGeom g, const float* __restrict__ din,
                                                             const int16_t* __restrict__ nin, float* __restrict__ dout,
                                                             int16_t* __restrict__ nout, int f, float d,
                                                             uint32_t* __restrict__ flags, int zl0, int nzr) {
    constexpr int LG = kShiftThreads / NSLOT;   // lane groups per block
    const int lane = threadIdx.x & (kWave - 1);
    const int p = threadIdx.x & (NSLOT - 1);
    const uint32_t G = blockIdx.x * (uint32_t)LG + threadIdx.x / NSLOT;
    const int nm = g.nmax;
    const float w = g.w;
    const int cps_f = f == 0 ? g.cps_x : (f == 1 ? g.cps_y : g.cps_z);
    const float Lf = f == 0 ? g.Lx : (f == 1 ? g.Ly : g.Lz);
    const int dir = (d <= 0) ? -1 : 1;                     // VS shiftCells.h:38-44
    // quirk S1 (pmc.h): the root copy's int s[3] (shiftCells.h:31,105) truncates w*dir
    const float s = S1 ? (float)(int)(w * (float)dir) : w * (float)dir;
    const int len = f == 0 ? g.cps_x : (f == 1 ? g.cps_y : nzr);   // cells along f in the range
    const uint32_t nruns = (uint32_t)((len + R - 1) / R);
    // lane group -> (run a, the two other coordinates)
    uint32_t a;
    int x = 0, y = 0, zr = 0;                              // zr: plane index within the range
    if (f == 0) {
        a = G % nruns;
        const uint32_t r = G / nruns;
        y = (int)(r % (uint32_t)g.cps_y);
        zr = (int)(r / (uint32_t)g.cps_y);
    } else if (f == 1) {
        x = (int)(G % (uint32_t)g.cps_x);
        const uint32_t r = G / (uint32_t)g.cps_x;
        a = r % nruns;
        zr = (int)(r / nruns);
    } else {
        x = (int)(G % (uint32_t)g.cps_x);
        const uint32_t r = G / (uint32_t)g.cps_x;
        y = (int)(r % (uint32_t)g.cps_y);
        a = r / (uint32_t)g.cps_y;
    }
    const bool group_live = f == 2 ? a < nruns : zr < nzr;
    if (!group_live) a = 0, zr = 0;                        // a valid cell to load from (nothing stored)
    const int f0 = (int)a * R;
    const int L = group_live ? (len - f0 < R ? len - f0 : R) : 0;   // live cells of the run
    const uint32_t plane = (uint32_t)g.cps_x * (uint32_t)g.cps_y;
    const int pp = p < nm ? p : 0;
    const int gsh = lane & ~(NSLOT - 1);
    const unsigned long long gmask = NSLOT == 64 ? ~0ull : ((1ull << (NSLOT & 63)) - 1ull);
    const unsigned long long below = (1ull << p) - 1ull;
    // cell j of the run: storage index and coordinate along f (cidf: global, wrapped for halo planes)
    auto cell_of = [&](int j, int& cidf) -> uint32_t {
        const int jj = j < L ? j : (L > 0 ? L - 1 : 0);
        int cx = x, cy = y, cz = zl0 + zr;
        if (f == 0) cx = f0 + jj; else if (f == 1) cy = f0 + jj; else cz = zl0 + f0 + jj;
        cidf = f == 0 ? cx : (f == 1 ? cy : g.z0 + cz);
        if (cidf < 0) cidf += cps_f; else if (cidf >= cps_f) cidf -= cps_f;
        return (uint32_t)cx + (uint32_t)g.cps_x * (uint32_t)cy + plane * (uint32_t)(cz + g.halo);
    };
    auto load3 = [&](uint32_t cell, float (&v)[3]) {
        if constexpr (OFF32) {
            const uint32_t o = (cell * (uint32_t)(3 * nm) + (uint32_t)pp * lay_slot()) * 4u;
            DiskAddr<1>::ld3(din, o, lay_dim(nm), v[0], v[1], v[2]);
        } else {
            const uint64_t o = (uint64_t)cell * (uint64_t)(3 * nm) + (uint64_t)pp * lay_slot();
            v[0] = din[o];
            v[1] = din[o + lay_dim(nm)];
            v[2] = din[o + 2 * lay_dim(nm)];
        }
    };
    auto count_of = [&](uint32_t cell) -> int {
        return OFF32 ? *(const int16_t*)((const char*)nin + (uint64_t)(cell * 2u)) : nin[cell];
    };
    uint32_t c[R];
    int cid[R], ncur[R];
    float own[R][3];
#if PMC_SHIFT_LINES
    __shared__ __attribute__((aligned(16))) float sh_rec[(kShiftThreads / NSLOT) * 3 * NSLOT];
    const bool lines = PMC_AOS && (3 * nm) % 4 == 0 && 3 * nm <= 4 * NSLOT;   // whole 16-B units per record
#endif
#pragma unroll
    for (int j = 0; j < R; ++j) {
        c[j] = cell_of(j, cid[j]);
        const int n0 = count_of(c[j]);
        ncur[j] = j < L ? n0 : 0;
        load3(c[j], own[j]);
    }
    // the extra cell: the dir-neighbour of the run's edge cell (its last live cell for dir > 0, its
    // first for dir < 0)
    const int je = dir > 0 ? (L > 0 ? L - 1 : 0) : 0;
    int cide;
    const uint32_t ce = cell_of(je, cide);
    int nbe = cide + dir;
    if (nbe < 0) nbe = cps_f - 1; else if (nbe >= cps_f) nbe = 0;
    uint32_t cx = ce;   // storage index of the extra cell
    {
        const int zl = (int)(ce / plane) - g.halo;
        const uint32_t rem = ce - (uint32_t)(zl + g.halo) * plane;
        int ex = (int)(rem % (uint32_t)g.cps_x), ey = (int)(rem / (uint32_t)g.cps_x), ez = zl;
        if (f == 0) ex = nbe; else if (f == 1) ey = nbe; else ez = g.halo ? zl + dir : nbe;
        cx = (uint32_t)ex + (uint32_t)g.cps_x * (uint32_t)ey + plane * (uint32_t)(ez + g.halo);
    }
    const int nne0 = count_of(cx);
    const int nne = L > 0 ? nne0 : 0;
    float ext[3];
    load3(cx, ext);
#pragma unroll
    for (int j = 0; j < R; ++j) {
        // the dir-neighbour: cell j + dir of the run when that is a live cell, else the extra one
        const int jn = j + dir;
        const bool in_run = jn >= 0 && jn < L;
        const int jl = j + 1 < R ? j + 1 : R - 1, jr = j > 0 ? j - 1 : 0;   // compile-time candidates
        float nbv[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) nbv[k] = in_run ? (dir > 0 ? own[jl][k] : own[jr][k]) : ext[k];
        const int nnb = in_run ? (dir > 0 ? ncur[jl] : ncur[jr]) : nne;
        int nbg = cid[j] + dir;
        if (nbg < 0) nbg = cps_f - 1; else if (nbg >= cps_f) nbg = 0;
        const float offset = (float)cid[j] * w - Lf / 2.0f;          // VS :46
        const float offset_nb = (float)nbg * w - Lf / 2.0f;
        const float xf = f == 0 ? own[j][0] : (f == 1 ? own[j][1] : own[j][2]);
        const float xfn = f == 0 ? nbv[0] : (f == 1 ? nbv[1] : nbv[2]);
        const float D = (xf - offset) - d;               // shortDisk - d
        const float Dn = (xfn - offset_nb) - d;
        const bool keep = (p < ncur[j]) && (D > 0 && D <= w);
        const bool take = (j < L) && (p < nnb) && !(Dn > 0 && Dn <= w);
        const unsigned long long km = (__ballot(keep) >> gsh) & gmask;
        const unsigned long long tm = (__ballot(take) >> gsh) & gmask;
        const int nk = __popcll(km);
        const int nnew = nk + __popcll(tm);
        auto out_at = [&](int dst) -> float* {
            const uint32_t e = (uint32_t)dst * lay_slot();
            if constexpr (OFF32)
                return (float*)((char*)dout + (uint64_t)((c[j] * (uint32_t)(3 * nm) + e) * 4u));
            else
                return dout + (uint64_t)c[j] * (uint64_t)(3 * nm) + (uint64_t)e;
        };
#if PMC_SHIFT_LINES
        if (lines) {
            // the output record assembled in LDS, then stored as whole 64-B lines (16-B units up to the
            // line that holds the last occupied slot): no partially written line reaches the memory side
            float* rec = sh_rec + (threadIdx.x / NSLOT) * (3 * NSLOT);
            // slots past the count go out as zeros (stale scratch there measured slower for the next
            // phases, profiles/r05x1_shift_lines_ab.txt)
            rec[3 * p] = 0.0f;
            rec[3 * p + 1] = 0.0f;
            rec[3 * p + 2] = 0.0f;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            if (keep) {
                const int dst = __popcll(km & below);
#pragma unroll
                for (int dim = 0; dim < 3; ++dim) rec[3 * dst + dim] = (dim == f) ? D + offset : own[j][dim];
            }
            if (take) {
                const int dst = nk + __popcll(tm & below);
                if (dst < nm) {
#pragma unroll
                    for (int dim = 0; dim < 3; ++dim) rec[3 * dst + dim] = (dim == f) ? ((Dn + offset) + s) : nbv[dim];
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            const int nw = nnew > nm ? nm : nnew;
            // whole lines counted from the record's start, capped at the record's own 3*nm/4 units: a
            // record that is not a whole number of lines (nm = 4, 8, 12, 20, ...) never spills into
            // the next cell's record or past the buffer
            int units = (12 * nw + 63) / 64 * 4;
            if (units > 3 * nm / 4) units = 3 * nm / 4;
            if (j < L && p < units) {
                const uint4 v = *reinterpret_cast<const uint4*>(rec + 4 * p);
                *reinterpret_cast<uint4*>(out_at(0) + 4 * p) = v;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   // the next cell reuses rec
        } else
#endif
        {
        if (keep) {
            const int dst = __popcll(km & below);
            if (dst < nm) {
                float* q = out_at(dst);
#pragma unroll
                for (int dim = 0; dim < 3; ++dim) shift_store(q + dim * lay_dim(nm), (dim == f) ? D + offset : own[j][dim]);
            }
        }
        if (take) {
            const int dst = nk + __popcll(tm & below);
            if (dst < nm) {
                float* q = out_at(dst);
#pragma unroll
                for (int dim = 0; dim < 3; ++dim)   // own offset (VS shiftCells.h:96)
                    shift_store(q + dim * lay_dim(nm), (dim == f) ? ((Dn + offset) + s) : nbv[dim]);
            }
        }
        }
        if (j < L && p == 0) {
            if constexpr (OFF32)
                *(int16_t*)((char*)nout + (uint64_t)(c[j] * 2u)) = (int16_t)(nnew > nm ? nm : nnew);
            else
                nout[c[j]] = (int16_t)(nnew > nm ? nm : nnew);
            if (nnew > nm) atomicOr(flags, 1u);
        }
    }
}

// ------------------------------------------------------------------------------------------
// init_r (start.cu:47-58 / kernel.cu:78-89) and assign (start.cu:87-146)
// ------------------------------------------------------------------------------------------
__global__ void k_init_r(DevGeom g, int64_t n_atoms, int64_t nc, float* __restrict__ r) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n_atoms) return;
    const int64_t ix = idx % nc, iy = (idx / nc) % nc, iz = idx / (nc * nc);
    const float Lzl = (float)g.nz_local * g.w;
    const float zc = ((float)g.z0 * g.w - g.Lz / 2.0f) + Lzl / 2.0f;
    const double fx = (double)((float)(2 * ix + 1) / (float)nc);
    const double fy = (double)((float)(2 * iy + 1) / (float)nc);
    const double fz = (double)((float)(2 * iz + 1) / (float)nc);
    r[idx] = (float)((double)g.Lx / 2.0 * (1.0 - fx));
    r[idx + n_atoms] = (float)((double)g.Ly / 2.0 * (1.0 - fy));
    r[idx + 2 * n_atoms] = (float)((double)zc + (double)Lzl / 2.0 * (1.0 - fz));
}

// half-open binning lb < x <= ub, lb = c*w - L/2.0f (start.cu:129-134); -1 if outside the box
__device__ int bin_axis(float xv, int cps, float w) {
    const float L = (float)cps * w;
    int c = (int)((xv + L / 2.0f) / w);
    if (c < 0) c = 0;
    if (c > cps - 1) c = cps - 1;
    for (int it = 0; it < 4; ++it) {
        const float lb = (float)c * w - L / 2.0f;
        const float ub = lb + w;
        if (xv <= lb) { if (c == 0) return -1; --c; }
        else if (xv > ub) { if (c == cps - 1) return -1; ++c; }
        else return c;
    }
    return -1;
}

__global__ void k_assign_count(DevGeom g, const float* __restrict__ r, int64_t n_atoms,
                               int32_t* __restrict__ tmp_cnt, int32_t* __restrict__ tmp_idx,
                               uint32_t* __restrict__ flags, int clip) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_atoms) return;
    const int cx = bin_axis(r[i], g.cps_x, g.w);
    const int cy = bin_axis(r[i + n_atoms], g.cps_y, g.w);
    const float zv = r[i + 2 * n_atoms];
    // clip 2 (pmc_init_lattice_planes): lattice rows above the periodic box are not part of it
    if (clip == 2 && zv > g.Lz / 2.0f) return;
    const int cz = bin_axis(zv, g.cps_z, g.w);
    if (cx < 0 || cy < 0 || cz < 0) {
        atomicOr(flags, 4u);
        return;
    }
    if (cz < g.z0 || cz >= g.z0 + g.nz_local) {   // another slab's particle
        if (!clip) atomicOr(flags, 4u);
        return;
    }
    const int64_t c = sidx(g, cx, cy, cz - g.z0);
    const int k = atomicAdd(&tmp_cnt[c], 1);
    if (k < g.nmax) tmp_idx[c * g.nmax + k] = (int32_t)i;
    else atomicOr(flags, 2u);
}

// per cell: order the slots by particle index (the reference scans particles in index order),
// then write the cell's rows.
__global__ void k_assign_fill(DevGeom g, const float* __restrict__ r, int64_t n_atoms,
                              const int32_t* __restrict__ tmp_cnt, const int32_t* __restrict__ tmp_idx,
                              float* __restrict__ disk, int16_t* __restrict__ n, int64_t cells, int ref_layout) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cells) return;
    const int nm = g.nmax;
    int cnt = tmp_cnt[c];
    if (cnt > nm) cnt = nm;
    int ids[64];
    for (int k = 0; k < cnt; ++k) {
        const int v = tmp_idx[c * nm + k];
        int j = k;
        while (j > 0 && ids[j - 1] > v) { ids[j] = ids[j - 1]; --j; }
        ids[j] = v;
    }
    for (int k = 0; k < cnt; ++k) {
        const int64_t i = ids[k];
        // (the reference layout for a caller's buffer, the state layout for the context's own)
        const int64_t ds = ref_layout ? nm : (int64_t)lay_dim(nm), ss = ref_layout ? 1 : (int64_t)lay_slot();
        disk[c * 3 * nm + k * ss] = r[i];
        disk[c * 3 * nm + ds + k * ss] = r[i + n_atoms];
        disk[c * 3 * nm + 2 * ds + k * ss] = r[i + 2 * n_atoms];
    }
    n[c] = (int16_t)cnt;
}

// ------------------------------------------------------------------------------------------
// total energy (calc_energy, kernel.cu:452-470) as a cell-list sum, fixed-point per pair
//
// One wave per owned cell.  The cell's stencil particles are staged into LDS (SoA, periodic image
// added, compacted by ballot + mbcnt) in three groups: the own cell, the "mutual" forward
// neighbours (owned, not wrapped, lexicographically after the cell: weight 2), and the directed
// ones (wrapped across the periodic box or in a halo plane: weight 1).  A pair of mutual cells
// gives bit-identical terms in both directions (xi - xj = -(xj - xi) exactly when no image is
// added), so it is evaluated once and counted twice; a pair across a wrap or a slab boundary is
// evaluated from each side like the oracle does (orc_energy: every directed pair, then x 0.5).  The
// per-pair fixed-point terms (pmc_to_fixed_f32 = pmc_to_fixed((double)e), integer-only) are
// summed in int64 -- exact in any order -- so the total equals the oracle's bit for bit.
// Lanes run over the flattened (own particle i, staged partner j) pairs.
// ------------------------------------------------------------------------------------------
// Per-lane stencil description of one cell (lane k < 27: stencil cell k) for k_energy.
struct EnergyStencil {
    int kc;            // storage cell
    float sx, sy, sz;  // periodic image
    int grp;           // 0 own, 1 mutual forward (weight 2), 2 directed (weight 1), 3 skipped
    int cnt;           // particles (0 for skipped cells); a load in flight until first used
    int x, y, zg;      // the cell (wave-uniform): its box filters the staged partners
};

// Per-lane constants of the stencil (lane k < 27): the storage offset of neighbour k from its cell
// (periodic wrap aside) and the group of an interior cell's neighbour k (0 own, 1 forward, 3
// backward; lanes >= 27: 3).  Computed once per wave.
struct EnergyLaneConst {
    int dk;
    int grp_in;
};

__device__ __forceinline__ EnergyLaneConst energy_lane_const(const DevGeom& g) {
    const int lane = threadIdx.x & (kWave - 1);
    const int k = lane < 27 ? lane : 0;
    const int dx = (int)bit_of(kStencilPos[0], k) - (int)bit_of(kStencilNeg[0], k);
    const int dy = (int)bit_of(kStencilPos[1], k) - (int)bit_of(kStencilNeg[1], k);
    const int dz = (int)bit_of(kStencilPos[2], k) - (int)bit_of(kStencilNeg[2], k);
    const bool forward = dz > 0 || (dz == 0 && (dy > 0 || (dy == 0 && dx > 0)));
    EnergyLaneConst lc;
    lc.dk = dx + g.cps_x * (dy + g.cps_y * dz);
    lc.grp_in = lane >= 27 ? 3 : (k == 0 ? 0 : (forward ? 1 : 3));
    return lc;
}

__device__ __forceinline__ EnergyStencil energy_stencil(const DevGeom& g, const int16_t* __restrict__ ncnt,
                                                        uint32_t t, const EnergyLaneConst& lc) {
    const int lane = threadIdx.x & (kWave - 1);
    // t is wave-uniform: scalar magic division (host-computed divisors)
    const uint32_t q1 = udiv_magic(t, g.div_cx);          // t / cps_x
    const uint32_t zq = udiv_magic(t, g.div_plane);       // t / (cps_x * cps_y)
    const int x = (int)(t - q1 * (uint32_t)g.cps_x);
    const int zl = (int)zq;
    const int y = (int)(q1 - zq * (uint32_t)g.cps_y);
    EnergyStencil e;
    e.x = x;
    e.y = y;
    e.zg = g.z0 + zl;
    // interior cell (no neighbour wrapped or in a halo plane): every neighbour is mutual, the
    // storage cells are plain offsets (same values as the general path below)
    if (x >= 1 && x <= g.cps_x - 2 && y >= 1 && y <= g.cps_y - 2 && zl >= 1 && zl <= g.nz_local - 2 &&
        e.zg >= 1 && e.zg <= g.cps_z - 2) {
        e.kc = (int)t + g.cps_x * g.cps_y * g.halo + lc.dk;
        e.sx = e.sy = e.sz = 0.0f;
        e.grp = lc.grp_in;
        e.cnt = e.grp < 3 ? (int)ncnt[e.kc] : 0;
        return e;
    }
    const int k = lane < 27 ? lane : 0;
    // lane k = 9*hx + 3*hy + hz, h = 0, 1, 2 -> offset 0, -1, +1 (the subsweep's stencil masks)
    const int dx = (int)bit_of(kStencilPos[0], k) - (int)bit_of(kStencilNeg[0], k);
    const int dy = (int)bit_of(kStencilPos[1], k) - (int)bit_of(kStencilNeg[1], k);
    const int dz = (int)bit_of(kStencilPos[2], k) - (int)bit_of(kStencilNeg[2], k);
    // periodic wrap as selects, 32-bit storage index (< 2^31 storage cells, normalise)
    const int nx0 = x + dx, ny0 = y + dy, zg = g.z0 + zl + dz, nz0 = zl + dz;
    const int nx = nx0 + (nx0 < 0 ? g.cps_x : 0) - (nx0 >= g.cps_x ? g.cps_x : 0);
    const int ny = ny0 + (ny0 < 0 ? g.cps_y : 0) - (ny0 >= g.cps_y ? g.cps_y : 0);
    e.sx = nx0 < 0 ? -g.Lx : (nx0 >= g.cps_x ? g.Lx : 0.0f);
    e.sy = ny0 < 0 ? -g.Ly : (ny0 >= g.cps_y ? g.Ly : 0.0f);
    e.sz = zg < 0 ? -g.Lz : (zg >= g.cps_z ? g.Lz : 0.0f);
    const int nzl = g.halo ? nz0 : nz0 + (nz0 < 0 ? g.cps_z : 0) - (nz0 >= g.cps_z ? g.cps_z : 0);
    e.kc = nx + g.cps_x * (ny + g.cps_y * (nzl + g.halo));
    const bool wrapped = e.sx != 0.0f || e.sy != 0.0f || e.sz != 0.0f;
    const bool halo_nb = nzl < 0 || nzl >= g.nz_local;
    const bool mutual = !wrapped && !halo_nb;
    const bool forward = dz > 0 || (dz == 0 && (dy > 0 || (dy == 0 && dx > 0)));
    e.grp = lane >= 27 ? 3 : (k == 0 ? 0 : (mutual ? (forward ? 1 : 3) : 2));
    e.cnt = e.grp < 3 ? (int)ncnt[e.kc] : 0;
    return e;
}

// fixed-point term of a mutual pair (weight 2), r2 <= rc2 already tested: 2 * pmc_to_fixed((double)
// pmc_lj_from_r2(r2, rc2)) bit for bit
__device__ __forceinline__ int64_t energy_term_w2(float r2, float r2min) {
    const float rr = r2 < r2min ? r2min : r2;
    const float inv = pmc_recip(rr);
    const float p6 = inv * inv * inv;
    return 2 * pmc_to_fixed_f32(4.0f * (p6 * p6 - p6));
}

// fixed-point term of a listed pair: r2s = +r2 (weight 1) or -r2 (weight 2), r2 <= rc2 already
// tested; the value is pmc_to_fixed((double)pmc_lj_from_r2(r2, rc2)) bit for bit
__device__ __forceinline__ int64_t energy_term(float r2s, float r2min) {
    const float r2 = __builtin_fabsf(r2s);
    const float rr = r2 < r2min ? r2min : r2;
    const float inv = pmc_recip(rr);
    const float p6 = inv * inv * inv;
    const int64_t e = pmc_to_fixed_f32(4.0f * (p6 * p6 - p6));
    return __builtin_signbit(r2s) ? 2 * e : e;
}

// One wave per kEnergyCells consecutive owned cells.  Per cell: the stencil particles are staged
// into LDS in three groups -- the own cell (all its slots first), the "mutual" forward neighbours
// (owned, not wrapped, lexicographically after the cell: weight 2) and the directed ones (wrapped
// across the periodic box or in a halo plane: weight 1); mutual backward neighbours are skipped.
// A pair of mutual cells gives bit-identical terms in both directions (xi - xj = -(xj - xi)
// exactly when no image is added), so it is evaluated once and counted twice; a pair across a
// wrap or a slab boundary is evaluated from each side, as the oracle does (orc_energy: every
// directed pair, then x 0.5).  Lanes run over the flattened pairs (own particle i, staged j > i);
// the pairs inside the cutoff (about one in five) are listed in an LDS ring and only those are
// converted: pmc_to_fixed_f32 per pair (= pmc_to_fixed((double)e)), int64 sums -- exact in any
// order, so the total equals the oracle's bit for bit.  The next cell's rows are loaded while
// the current cell's pairs run (the kernel is otherwise latency-bound: two dependent HBM round
// trips per cell).
#ifndef PMC_ENERGY_CELLS
#define PMC_ENERGY_CELLS 16
#endif
constexpr int kEnergyCells = PMC_ENERGY_CELLS;
// edge cells per wave (MODE 1): at 128^3 the ~98k edge cells are well under one round of the chip's
// wave slots at 16 per wave, so the launch lasts one long wave lifetime; shorter waves spread them
#ifndef PMC_ENERGY_EDGE_CELLS
#define PMC_ENERGY_EDGE_CELLS 4
#endif
constexpr int kEdgeCells = PMC_ENERGY_EDGE_CELLS;
// own particles per pair-loop step (1 or 2: two broadcast particles share the loop control, the
// ring accounting and the drain test)
#ifndef PMC_ENERGY_STEP
#define PMC_ENERGY_STEP 1
#endif
constexpr int kEnergyRing = PMC_ENERGY_STEP == 2 ? 256 : 128;

// k_energy_rows: one wave per row segment of kESeg cells along x; the 9 neighbouring rows of the
// segment (kESeg + 2 cells each) are staged once, kECap particles at most
// Segment length and staging capacity keep a wave's LDS within 5 KiB (8 waves per SIMD; round 3's
// 8-cell segments with 384 staged particles took 6.5 KiB: 6 waves per SIMD).  At 128^3/1e7 a
// 6-cell segment stages 186 particles on average; the near-lattice start peaks at 281.
#ifndef PMC_ENERGY_SEG
#define PMC_ENERGY_SEG 6
#endif
constexpr int kESeg = PMC_ENERGY_SEG;
constexpr int kERows = 5;                   // the rows of an interior cell's half shell
constexpr int kEStaged = kERows * (kESeg + 2);   // staged cells per segment (< 64: one lane each)
static_assert(kEStaged < 64, "one lane per staged cell");
// staged particles per segment: 288 at 6-cell segments with the 128-entry ring (the 5 KiB budget
// below; the near-lattice start of the configs peaks at 281 per segment, so a box a few percent
// denser than 4.77 per cell queues some segments for MODE 2), 240 with PMC_ENERGY_STEP=2's 256-entry
// ring, 384 at 8-cell segments (6.5 KiB)
constexpr int kECap = kESeg == 6 ? (kEnergyRing == 128 ? 288 : 240) : 384;
constexpr int kEList = 14 * 16;             // a cell's filtered partner list (indices into the staging)
#ifndef PMC_ENERGY_OWN_LDS
#define PMC_ENERGY_OWN_LDS 1   // pair loop: own particle from LDS (1) or by v_readlane (0)
#endif

// A cell is an "edge" cell for the energy when a stencil neighbour is wrapped across the periodic
// box or lies in a halo plane (slab mode): its pairs with that neighbour are directed (weight 1,
// evaluated from each side).  Every other cell's neighbours are all mutual, and k_energy_rows takes
// it (half shell, weight 2).
__device__ __forceinline__ bool energy_edge_cell(const DevGeom& g, int x, int y, int zl) {
    const int zg = g.z0 + zl;
    return x == 0 || x == g.cps_x - 1 || y == 0 || y == g.cps_y - 1 || zg == 0 || zg == g.cps_z - 1 ||
           (g.halo && (zl == 0 || zl == g.nz_local - 1));
}

// Cell-list energy, one wave per group of cells.  MODE 0: every owned cell, kEnergyCells
// consecutive cells per wave; 1: only the edge cells among them (k_energy_rows takes the rest);
// 2: the interior cells of the row segments k_energy_rows could not stage (its queue `segq`:
// [0] count, then segment ids), a fixed grid striding over the queue.
template <int NSLOT, bool OFF32, int MODE>
__global__ __launch_bounds__(kWave) void k_energy(DevGeom g, const float* __restrict__ disk,
                                                  const int16_t* __restrict__ ncnt,
                                                  unsigned long long* __restrict__ acc, uint32_t total_cells,
                                                  const int* __restrict__ segq, UDivMagic div_nsx) {
    extern __shared__ __attribute__((aligned(16))) float esm[];
    constexpr int HS = NSLOT >= 16 ? 8 : NSLOT;       // staging lanes per cell (slots [0, HS))
    constexpr int CPP = kWave / HS;                   // cells per staging pass
    constexpr int NPMAX = (27 + CPP - 1) / CPP;
    const int lane = threadIdx.x;
    const int nm = g.nmax;
    const int cap = 27 * nm;
    float* ex_ = esm;
    float* ey_ = esm + cap;
    float* ez_ = esm + 2 * cap;
    float* ring = esm + 3 * cap;                      // ring of listed pairs (signed r2)
    int* inv_l = (int*)(ring + kEnergyRing);          // list entry -> stencil lane (32 ints)
    const int p = lane % HS;
    const int ee = lane / HS;
    const float rc2 = g.rc2;
    const float r2min = g.r2min;
    long long sum = 0;

    // cells of this wave: base + the set bits of `todo` (ascending)
    auto cell_xyz = [&](uint32_t t, int* x, int* y, int* zl) {
        const uint32_t q1 = udiv_magic(t, g.div_cx);
        const uint32_t zq = udiv_magic(t, g.div_plane);
        *x = (int)(t - q1 * (uint32_t)g.cps_x);
        *zl = (int)zq;
        *y = (int)(q1 - zq * (uint32_t)g.cps_y);
    };
    const EnergyLaneConst lc = energy_lane_const(g);
    // the wave's cells: ncl of them, pop() returns the next cell id (wave-uniform)
    auto run_cells = [&](int ncl, auto pop) {
    if (ncl == 0) return;
    // staged-cell list of the cell whose rows are in flight: entry -> stencil lane in inv_l,
    // its group masks; rows in registers
    float vx[NPMAX], vy[NPMAX], vz[NPMAX];
    bool vact[NPMAX];
    unsigned long long m0 = 0, m1 = 0, m2 = 0;
    int n0 = 0, n1 = 0, ncells = 0;
    auto issue_rows = [&](const EnergyStencil& st) {
        m0 = __builtin_amdgcn_ballot_w64(st.grp == 0 && st.cnt > 0);
        m1 = __builtin_amdgcn_ballot_w64(st.grp == 1 && st.cnt > 0);
        m2 = __builtin_amdgcn_ballot_w64(st.grp == 2 && st.cnt > 0);
        n0 = __popcll(m0);
        n1 = __popcll(m1);
        ncells = n0 + n1 + __popcll(m2);
        const int pos = st.grp == 0 ? mbcnt64(m0) : (st.grp == 1 ? n0 + mbcnt64(m1) : n0 + n1 + mbcnt64(m2));
        if (st.grp < 3 && st.cnt > 0) inv_l[pos] = lane;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const int npass = (ncells + CPP - 1) / CPP;
        const bool edge = __builtin_amdgcn_ballot_w64(st.sx != 0.0f || st.sy != 0.0f || st.sz != 0.0f) != 0;
#pragma unroll
        for (int q = 0; q < NPMAX; ++q) {
            vact[q] = false;
            if (q < npass) {
                const int e = q * CPP + ee;
                const int src = inv_l[e < ncells ? e : 0];
                const int c_cnt = __shfl(st.cnt, src);
                const int c_idx = __shfl(st.kc, src);
                vact[q] = e < ncells && p < c_cnt;
                if (vact[q]) {
                    using DA = DiskAddr<OFF32>;
                    const uint32_t off = ((uint32_t)c_idx * (uint32_t)(3 * nm) + (uint32_t)p * lay_slot()) * DA::kUnit;
                    DA::ld3(disk, off, lay_dim(nm), vx[q], vy[q], vz[q]);
                }
                if (edge) {   // periodic images (a +0 add changes no difference: interior cells skip it)
                    // (cross-lane reads outside the branch: an inactive source lane supplies nothing)
                    const float isx = __shfl(st.sx, src), isy = __shfl(st.sy, src), isz = __shfl(st.sz, src);
                    vx[q] = vx[q] + isx;
                    vy[q] = vy[q] + isy;
                    vz[q] = vz[q] + isz;
                }
            }
        }
    };

    EnergyStencil cur = energy_stencil(g, ncnt, pop(), lc);
    issue_rows(cur);
    EnergyStencil nxt = cur;
    if (ncl > 1) nxt = energy_stencil(g, ncnt, pop(), lc);
    for (int c = 0; c < ncl; ++c) {
        // ---- stage cell c from the rows in registers: own cell (all slots), weight-2 cells,
        //      then weight-1 cells (each group: main slots, then the fuller cells' slots [HS, n))
        // partners farther than the cutoff from every point of the own cell's (padded) box
        // contribute exactly 0 to every pair with an own particle: not staged (the subsweep's
        // conservative filter, pmc_box_d2); own particles always are
        float blo[3], bhi[3];
        pmc_cell_box(cur.x, cur.y, cur.zg, g.w, g.Lx, g.Ly, g.Lz, blo, bhi);
        auto near = [&](float ux, float uy, float uz) { return pmc_box_d2(ux, uy, uz, blo, bhi) <= g.rc2f; };
        int S = 0;
        auto put = [&](bool act, float ux, float uy, float uz) {
            const unsigned long long am = __builtin_amdgcn_ballot_w64(act);
            if (act) {
                const int dst = S + mbcnt64(am);
                ex_[dst] = ux;
                ey_[dst] = uy;
                ez_[dst] = uz;
            }
            S += __popcll(am);
        };
        auto overflow = [&](unsigned long long mg, bool filter) {
            if constexpr (HS < NSLOT) {
                unsigned long long ov = __builtin_amdgcn_ballot_w64(((mg >> (lane & 63)) & 1ull) && cur.cnt > HS);
                while (ov) {
                    int ks = 0, nc = 0;
                    for (; nc < CPP && ov; ++nc) {
                        const int kb = (int)__builtin_ctzll(ov);
                        ov &= ov - 1ull;
                        ks = ee == nc ? kb : ks;
                    }
                    const int c_cnt = __shfl(cur.cnt, ks);
                    const int c_idx = __shfl(cur.kc, ks);
                    const float isx = __shfl(cur.sx, ks), isy = __shfl(cur.sy, ks), isz = __shfl(cur.sz, ks);
                    const int ps = HS + p;
                    const bool act = ee < nc && ps < c_cnt;
                    float ux = 0.0f, uy = 0.0f, uz = 0.0f;
                    if (act) {
                        using DA = DiskAddr<OFF32>;
                        const uint32_t off = ((uint32_t)c_idx * (uint32_t)(3 * nm) + (uint32_t)ps * lay_slot()) * DA::kUnit;
                        DA::ld3(disk, off, lay_dim(nm), ux, uy, uz);
                        ux = ux + isx;
                        uy = uy + isy;
                        uz = uz + isz;
                    }
                    put(act && (!filter || near(ux, uy, uz)), ux, uy, uz);
                }
            }
        };
        const int n_own = __builtin_amdgcn_readfirstlane(cur.cnt);   // lane 0 = own cell (entry 0)
        const int e0 = n0 + n1;
        // staged ranges: [0, n_own) own | main slots of the other cells in list order (weight-2
        // cells first: [n_own, A)) | overflow slots of weight-2 cells [B, C) | of weight-1 cells
        put(vact[0] && ee == 0, vx[0], vy[0], vz[0]);                 // own main slots
        overflow(m0, false);                                          // own slots [HS, n)
        int A = S;
#pragma unroll
        for (int q = 0; q < NPMAX; ++q) {
            const int e = q * CPP + ee;
            if (q * CPP < ncells) {
                const bool keep = vact[q] && e >= 1 && near(vx[q], vy[q], vz[q]);
                A += __popcll(__builtin_amdgcn_ballot_w64(keep && e < e0));
                put(keep, vx[q], vy[q], vz[q]);
            }
        }
        const int B = S;
        overflow(m1, true);
        const int C2 = S;
        overflow(m2, true);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // ---- the next cell's rows go out now and arrive while this cell's pairs run
        if (c + 1 < ncl) {
            cur = nxt;
            issue_rows(cur);
            if (c + 2 < ncl) nxt = energy_stencil(g, ncnt, pop(), lc);
        }
        if (n_own == 0) continue;
        // ---- pairs (i, j): lane j holds staged partner j (blocks of 64), own particle i < n_own
        //      (staged first: lane i of block 0) broadcast by readlane.  Own-own pairs once, j > i,
        //      weight 2: r2(xi - xj) and r2(xj - xi) are the same bits (the oracle's two directed
        //      terms, weight 1 each, sum to the same fixed-point value)
        constexpr int RM = kEnergyRing - 1;
        int head = 0, C = 0;   // ring: entries [head, head + C) mod kEnergyRing
        auto drain = [&](int lim) {
            if (lane < lim) sum += energy_term(ring[(head + lane) & RM], r2min);
            head = (head + 64) & RM;
            C -= lim;
        };
        const float ox = ex_[lane], oy = ey_[lane], oz = ez_[lane];   // block 0 (own at lanes < n_own)
        auto block = [&](int jb, auto first_c) {
            constexpr bool kFirst = decltype(first_c)::value;
            const int j = jb + lane;
            const bool vj = j < S;
            const int jj = vj ? j : 0;
            float xj = ox, yj = oy, zj = oz;
            if constexpr (!kFirst) {
                xj = ex_[jj];
                yj = ey_[jj];
                zj = ez_[jj];
            }
            const bool w2 = jj < A || (jj >= B && jj < C2);   // own (j > i), mutual forward
            const uint32_t sgn = w2 ? 0x80000000u : 0u;       // weight 2: listed with the sign bit set
            // partners j < S; in block 0 the lanes j > i (lanes 0..n_own-1 are all valid, so
            // clearing the lowest set bit each step drops lane i)
            unsigned long long vm = __builtin_amdgcn_ballot_w64(vj);
#if PMC_ENERGY_STEP == 2
            for (int i = 0; i < n_own; i += 2) {
                const bool two = i + 1 < n_own;   // wave-uniform
                const float xa = as_f(__builtin_amdgcn_readlane(as_i(ox), i));
                const float ya = as_f(__builtin_amdgcn_readlane(as_i(oy), i));
                const float za = as_f(__builtin_amdgcn_readlane(as_i(oz), i));
                const float xb = as_f(__builtin_amdgcn_readlane(as_i(ox), i + 1));
                const float yb = as_f(__builtin_amdgcn_readlane(as_i(oy), i + 1));
                const float zb = as_f(__builtin_amdgcn_readlane(as_i(oz), i + 1));
                const float r2a = pmc_r2(xa - xj, ya - yj, za - zj);
                const float r2b = pmc_r2(xb - xj, yb - yj, zb - zj);
                if constexpr (kFirst) vm &= vm - 1ull;
                const unsigned long long ima = __builtin_amdgcn_ballot_w64(r2a <= rc2) & vm;
                if constexpr (kFirst) vm &= vm - 1ull;
                const unsigned long long imb = two ? __builtin_amdgcn_ballot_w64(r2b <= rc2) & vm : 0ull;
                const int ca = __popcll(ima);
                if (__builtin_amdgcn_inverse_ballot_w64(ima))
                    ring[(head + C + mbcnt64(ima)) & RM] = as_f(as_i(r2a) | (int)sgn);
                if (__builtin_amdgcn_inverse_ballot_w64(imb))
                    ring[(head + C + ca + mbcnt64(imb)) & RM] = as_f(as_i(r2b) | (int)sgn);
                C += ca + __popcll(imb);   // C < 64 + 128 <= ring size
                while (C >= 64) drain(64);
            }
#else
            for (int i = 0; i < n_own; ++i) {
                const float xi = as_f(__builtin_amdgcn_readlane(as_i(ox), i));
                const float yi = as_f(__builtin_amdgcn_readlane(as_i(oy), i));
                const float zi = as_f(__builtin_amdgcn_readlane(as_i(oz), i));
                const float r2 = pmc_r2(xi - xj, yi - yj, zi - zj);
                if constexpr (kFirst) vm &= vm - 1ull;
                const unsigned long long im = __builtin_amdgcn_ballot_w64(r2 <= rc2) & vm;
                if (__builtin_amdgcn_inverse_ballot_w64(im))
                    ring[(head + C + mbcnt64(im)) & RM] = as_f(as_i(r2) | (int)sgn);
                C += __popcll(im);
                if (C >= 64) drain(64);
            }
#endif
        };
        block(0, std::true_type{});
        for (int jb = kWave; jb < S; jb += kWave) block(jb, std::false_type{});
        if (C > 0) drain(C);
    }
    };   // run_cells
    if constexpr (MODE == 2) {
        // queued row segments (k_energy_rows): their interior cells, kESeg consecutive cells in x
        const int nq = __builtin_amdgcn_readfirstlane(segq[0]);
        for (int k = (int)blockIdx.x; k < nq; k += (int)gridDim.x) {
            const uint32_t seg = (uint32_t)__builtin_amdgcn_readfirstlane(segq[1 + k]);
            const uint32_t row = udiv_magic(seg, div_nsx);
            const uint32_t x0 = (seg - row * (uint32_t)((g.cps_x + kESeg - 1) / kESeg)) * (uint32_t)kESeg;
            const uint32_t base = row * (uint32_t)g.cps_x + x0;
            int x, y, zl;
            cell_xyz(base + (uint32_t)lane, &x, &y, &zl);
            unsigned long long todo = __builtin_amdgcn_ballot_w64(lane < kESeg && x0 + (uint32_t)lane < (uint32_t)g.cps_x &&
                                                                  !energy_edge_cell(g, x, y, zl));
            run_cells(__popcll(todo), [&]() -> uint32_t {
                const int b = (int)__builtin_ctzll(todo);
                todo &= todo - 1ull;
                return base + (uint32_t)b;
            });
        }
    } else if constexpr (MODE == 1) {
        // the edge cells, enumerated densely: planes zl = 0 and nz-1 whole, then per middle plane
        // the rows y = 0 and cps_y-1 and the cells x = 0 and cps_x-1 of the rows between
        const uint32_t P = (uint32_t)g.cps_x * (uint32_t)g.cps_y;
        const uint32_t M = 2u * (uint32_t)g.cps_x + 2u * (uint32_t)(g.cps_y - 2);
        const uint32_t k0 = blockIdx.x * (uint32_t)kEdgeCells;
        const int ncl = (int)(total_cells - k0 < (uint32_t)kEdgeCells ? total_cells - k0 : (uint32_t)kEdgeCells);
        uint32_t k = k0;
        run_cells(ncl, [&]() -> uint32_t {
            const uint32_t kk = k++;
            uint32_t zl, x, y;
            if (kk < 2u * P) {
                zl = kk < P ? 0u : (uint32_t)g.nz_local - 1u;
                const uint32_t tin = kk < P ? kk : kk - P;
                y = udiv_magic(tin, g.div_cx);
                x = tin - y * (uint32_t)g.cps_x;
            } else {
                const uint32_t k1 = kk - 2u * P;
                const uint32_t pl = k1 / M;                        // (SALU: once per cell)
                const uint32_t r = k1 - pl * M;
                zl = 1u + pl;
                if (r < 2u * (uint32_t)g.cps_x) {
                    y = r < (uint32_t)g.cps_x ? 0u : (uint32_t)g.cps_y - 1u;
                    x = r < (uint32_t)g.cps_x ? r : r - (uint32_t)g.cps_x;
                } else {
                    const uint32_t r2 = r - 2u * (uint32_t)g.cps_x;
                    y = 1u + (r2 >> 1);
                    x = (r2 & 1u) ? (uint32_t)g.cps_x - 1u : 0u;
                }
            }
            return x + (uint32_t)g.cps_x * (y + (uint32_t)g.cps_y * zl);
        });
    } else {
        const uint32_t t0 = blockIdx.x * (uint32_t)kEnergyCells;
        const int ncl = (int)(total_cells - t0 < (uint32_t)kEnergyCells ? total_cells - t0 : (uint32_t)kEnergyCells);
        uint32_t t = t0;
        run_cells(ncl, [&]() -> uint32_t { return t++; });
    }
    // wave sum (int64, exact in any order), one atomic per wave
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    if (lane == 0 && sum != 0) atomicAdd(&acc[blockIdx.x & (kStatSlots - 1)], (unsigned long long)sum);
}

// Cell-list energy of the interior cells (no wrapped or halo neighbour: every pair mutual), one wave
// per row segment of kESeg cells along x.  An interior cell's half shell lies in five rows: its own
// row (the cell and its +x neighbour) and the rows (y+1, z), (y-1..y+1, z+1) (cells x-1..x+1).  These
// five rows over x0-1 .. x0+SL are staged ONCE for the segment: counts first, their exclusive prefix
// gives every staged cell its start in LDS, then the rows go straight to those starts (no
// compaction, no image: an interior cell's neighbours are never wrapped).  Per own cell the half
// shell is five contiguous staged ranges, walked as one flattened index and filtered through the
// own cell's box (pmc_box_d2, as the subsweep: a dropped partner's energy is exactly 0) into a
// partner list, own particles first (own-own pairs j > i).  Every pair is mutual, weight 2 (the
// oracle's two directed terms are the same bits); the fixed-point terms are summed in int64, exact in
// any order, so interior + edge cells (k_energy MODE 1) + queued segments (MODE 2) equal orc_energy
// bit for bit.  A segment holding more than `cap` particles is queued for MODE 2.
template <int NSLOT, bool OFF32>
__global__ __launch_bounds__(kWave) void k_energy_rows(DevGeom g, const float* __restrict__ disk,
                                                       const int16_t* __restrict__ ncnt,
                                                       unsigned long long* __restrict__ acc, int* __restrict__ segq,
                                                       UDivMagic div_nsx, UDivMagic div_cy, int cap) {
    extern __shared__ __attribute__((aligned(16))) float rsm[];
    float* ex_ = rsm;
    float* ey_ = rsm + kECap;
    float* ez_ = rsm + 2 * kECap;
    float* ring = rsm + 3 * kECap;                    // listed pairs (signed r2), kEnergyRing
    uint16_t* lst = (uint16_t*)(ring + kEnergyRing);  // the own cell's partners (staged indices)
    int2* rec = (int2*)(lst + kEList);                // staged cell: storage index, start | count << 16
    const int lane = threadIdx.x;
    const int nm = g.nmax;
    const int nsx = (g.cps_x + kESeg - 1) / kESeg;
    const uint32_t seg = blockIdx.x;
    const uint32_t row = udiv_magic(seg, div_nsx);    // y + cps_y * zl
    const int x0 = (int)(seg - row * (uint32_t)nsx) * kESeg;
    const uint32_t zq = udiv_magic(row, div_cy);
    const int zl = (int)zq, y = (int)(row - zq * (uint32_t)g.cps_y);
    const int zg = g.z0 + zl;
    // a segment on a y or z face (or next to a halo plane) holds edge cells only: k_energy MODE 1
    if (y == 0 || y == g.cps_y - 1 || zg == 0 || zg == g.cps_z - 1 || (g.halo && (zl == 0 || zl == g.nz_local - 1)))
        return;
    const int SL = g.cps_x - x0 < kESeg ? g.cps_x - x0 : kESeg;
    const int W = SL + 2, E = kERows * W;             // E < 64: one lane per staged cell
    // ---- staged cell e = r*W + q (lane e): row r in {(0,0), (+1,0), (-1,+1), (0,+1), (+1,+1)} as
    //      (dy, dz), cell x = x0 - 1 + q; cells outside [0, cps_x) neighbour edge cells only: not
    //      staged (count 0)
    const int r = (int)(((uint32_t)lane * ((65536u + (uint32_t)W - 1u) / (uint32_t)W)) >> 16);   // lane / W
    const int q = lane - r * W;
    const int dy = ((585 >> (2 * r)) & 3) - 1, dz = r >= 2 ? 1 : 0;
    const int xs = x0 - 1 + q;
    const bool st = lane < E && xs >= 0 && xs < g.cps_x;
    const int sidx = st ? xs + g.cps_x * (y + dy + g.cps_y * (zl + dz + g.halo)) : 0;
    const int cnt = st ? (int)ncnt[sidx] : 0;
    int inc = cnt;                                    // inclusive prefix of the counts over e
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int u = __shfl_up(inc, (unsigned)d);
        inc += lane >= d ? u : 0;
    }
    const int total = __builtin_amdgcn_readlane(inc, 63);
    // (never at equilibrium densities; nmax > 16: a cell's 14-cell list could exceed kEList)
    if (total > cap || 14 * nm > kEList) {   // the per-cell kernel (MODE 2) takes the segment
        if (lane == 0) segq[1 + atomicAdd(&segq[0], 1)] = (int)seg;
        return;
    }
    const int start = inc - cnt;                      // lane E: the total
    rec[lane] = make_int2(sidx, start | (cnt << 16));
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // ---- stage: slots [0, HS) of CPP cells per pass, then the fuller cells' slots [HS, n)
    constexpr int HS = NSLOT >= 16 ? 8 : NSLOT;
    constexpr int CPP = kWave / HS;
    using DA = DiskAddr<OFF32>;
    const int p = lane % HS, ce = lane / HS;
    for (int e0 = 0; e0 < E; e0 += CPP) {
        const int e = e0 + ce;
        const int2 rc = rec[e < E ? e : E];
        const int c_n = rc.y >> 16, c_s = rc.y & 0xffff;
        if (e < E && p < c_n) {
            const uint32_t off = ((uint32_t)rc.x * (uint32_t)(3 * nm) + (uint32_t)p * lay_slot()) * DA::kUnit;
            DA::ld3(disk, off, lay_dim(nm), ex_[c_s + p], ey_[c_s + p], ez_[c_s + p]);
        }
    }
    if constexpr (HS < NSLOT) {
        unsigned long long ov = __builtin_amdgcn_ballot_w64(cnt > HS);
        while (ov) {
            int ks = 0, nc = 0;
            for (; nc < CPP && ov; ++nc) {
                const int kb = (int)__builtin_ctzll(ov);
                ov &= ov - 1ull;
                ks = ce == nc ? kb : ks;
            }
            const int2 rc = rec[ks];
            const int c_n = rc.y >> 16, c_s = rc.y & 0xffff;
            for (int ps = HS + p; ps < NSLOT; ps += HS) {
                if (ce < nc && ps < c_n) {
                    const uint32_t off = ((uint32_t)rc.x * (uint32_t)(3 * nm) + (uint32_t)ps * lay_slot()) * DA::kUnit;
                    DA::ld3(disk, off, lay_dim(nm), ex_[c_s + ps], ey_[c_s + ps], ez_[c_s + ps]);
                }
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // staged cell e's start (e <= E) as a scalar
    auto st_of = [&](int e) -> int { return __builtin_amdgcn_readlane(start, e); };
    const float rc2 = g.rc2, r2min = g.r2min;
    long long sum = 0;
    constexpr int RM = kEnergyRing - 1;
    for (int s = 0; s < SL; ++s) {
        const int x = x0 + s;
        if (x == 0 || x == g.cps_x - 1) continue;       // edge cell (MODE 1)
        const int eo = s + 1;                            // own cell: row 0
        const int sA = st_of(eo), sA1 = st_of(eo + 1), eA = st_of(eo + 2);
        const int n_own = sA1 - sA;
        if (n_own == 0) continue;
        // ranges: A = own cell + its +x neighbour; B..E = cells x-1..x+1 of rows 1..4
        const int sB = st_of(W + s), eB = st_of(W + s + 3);
        const int sC = st_of(2 * W + s), eC = st_of(2 * W + s + 3);
        const int sD = st_of(3 * W + s), eD = st_of(3 * W + s + 3);
        const int sE = st_of(4 * W + s), eE = st_of(4 * W + s + 3);
        const int P1 = eA - sA, P2 = P1 + (eB - sB), P3 = P2 + (eC - sC), P4 = P3 + (eD - sD);
        const int T = P4 + (eE - sE);
        // the partner list: own particles first (unfiltered: the j > i pairs), then the others
        // within the cutoff of the own cell's (padded) box
        float blo[3], bhi[3];
        pmc_cell_box(x, y, zg, g.w, g.Lx, g.Ly, g.Lz, blo, bhi);
        if (lane < n_own) lst[lane] = (uint16_t)(sA + lane);
        int S = n_own;
        for (int jb = 0; jb < T; jb += kWave) {
            const int j = jb + lane;
            const int src = j < P1 ? sA + j : (j < P2 ? sB + (j - P1) : (j < P3 ? sC + (j - P2) :
                            (j < P4 ? sD + (j - P3) : sE + (j - P4))));
            const int sj = j < T ? src : 0;
            const bool keep = j >= n_own && j < T && pmc_box_d2(ex_[sj], ey_[sj], ez_[sj], blo, bhi) <= g.rc2f;
            const unsigned long long mk = __builtin_amdgcn_ballot_w64(keep);
            if (keep) lst[S + mbcnt64(mk)] = (uint16_t)sj;
            S += __popcll(mk);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#if !PMC_ENERGY_OWN_LDS
        const float ox = lane < n_own ? ex_[sA + lane] : 0.0f;
        const float oy = lane < n_own ? ey_[sA + lane] : 0.0f;
        const float oz = lane < n_own ? ez_[sA + lane] : 0.0f;
#endif
        int head = 0, C = 0;
        auto drain = [&](int lim) {
            if (lane < lim) sum += energy_term_w2(ring[(head + lane) & RM], r2min);
            head = (head + 64) & RM;
            C -= lim;
        };
        // one 64-partner block against every own particle i (broadcast by v_readlane); in block 0
        // the own slots j <= i are left out by a running mask (bit i cleared per step): the pairs
        // j > i of the own cell.  Every listed pair is mutual (weight 2: no sign bit).
        auto pairs = [&](int jb, auto first) {
            const int j = jb + lane;
            const int sj = lst[j < S ? j : 0];
            const float xj = ex_[sj], yj = ey_[sj], zj = ez_[sj];
            unsigned long long vm = __builtin_amdgcn_ballot_w64(j < S);
            unsigned long long bit = 1ull;                // own slot i (block 0)
            for (int i = 0; i < n_own; ++i) {
#if PMC_ENERGY_OWN_LDS
                // own particle i broadcast from the staging (uniform address: one LDS read per
                // coordinate) instead of three v_readlane
                const float xi = ex_[sA + i], yi = ey_[sA + i], zi = ez_[sA + i];
#else
                const float xi = as_f(__builtin_amdgcn_readlane(as_i(ox), i));
                const float yi = as_f(__builtin_amdgcn_readlane(as_i(oy), i));
                const float zi = as_f(__builtin_amdgcn_readlane(as_i(oz), i));
#endif
                const float r2 = pmc_r2(xi - xj, yi - yj, zi - zj);
                if constexpr (decltype(first)::value) {
                    vm &= ~bit;
                    bit <<= 1;
                }
                const unsigned long long im = __builtin_amdgcn_ballot_w64(r2 <= rc2) & vm;
                if (__builtin_amdgcn_inverse_ballot_w64(im)) ring[(head + C + mbcnt64(im)) & RM] = r2;
                C += __popcll(im);
                if (C >= 64) drain(64);
            }
        };
        // the pair loop above the staging of other waves (A/B: -0.7%, profiles/r03pr_priority_ab.txt)
        __builtin_amdgcn_s_setprio(1);
        pairs(0, std::true_type{});
        for (int jb = kWave; jb < S; jb += kWave) pairs(jb, std::false_type{});
        __builtin_amdgcn_s_setprio(0);
        if (C > 0) drain(C);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    if (lane == 0 && sum != 0) atomicAdd(&acc[blockIdx.x & (kStatSlots - 1)], (unsigned long long)sum);
}

// ------------------------------------------------------------------------------------------
// self-test of the deterministic math on the device (compared bitwise with the host oracle)
// ------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------
// halo exchange (slab driver): the cells of one colour (x % 2 == ox, y % 2 == oy) of one plane --
// the only cells a colour phase changes -- as (cps_y/2)*(cps_x/2) packed rows of 3*nmax floats.
// mode 0: plane -> packed, 1: packed -> plane, 2: plane -> plane (single-rank periodic halo).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_colour_rows(const float* __restrict__ src, float* __restrict__ dst,
                                                     int cps_x, int cps_y, int row, int ox, int oy, int mode) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int hx = cps_x >> 1;
    const int64_t total = (int64_t)hx * (cps_y >> 1) * row;
    if (i >= total) return;
    const int f = (int)(i % row);
    const int64_t j = i / row;
    const int64_t cell = (2 * (j / hx) + oy) * cps_x + 2 * (j % hx) + ox;
    const int64_t pidx = cell * row + f;
    if (mode == 0) dst[i] = src[pidx];
    else if (mode == 1) dst[pidx] = src[i];
    else dst[pidx] = src[pidx];
}

__global__ void k_selftest(const uint32_t* __restrict__ words, int count, float* __restrict__ out_f,
                           double* __restrict__ out_d, float rc2) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    pmc_u32x4 w;
    for (int k = 0; k < 4; ++k) w.v[k] = words[4 * i + k];
    float g0, g1, g2;
    pmc_move_normals(w, &g0, &g1, &g2);
    // pair energy for a separation derived from the words: components in (-2.5, 2.5)
    const float dx = pmc_u01(w.v[1]) * 5.0f - 2.5f;
    const float dy = pmc_u01(w.v[2]) * 5.0f - 2.5f;
    const float dz = pmc_u01(w.v[3]) * 5.0f - 2.5f;
    out_f[4 * i + 0] = g0;
    out_f[4 * i + 1] = g1;
    out_f[4 * i + 2] = g2;
    out_f[4 * i + 3] = pmc_lj_from_r2(pmc_r2(dx, dy, dz), rc2);
    out_d[2 * i + 0] = (double)pmc_accept_threshold(w);
    out_d[2 * i + 1] = (double)pmc_to_fixed((double)out_f[4 * i + 3]);
}

// Reference layout <-> state layout (pmc_internal.h, PMC_AOS): element e of cell c, e = d*nmax + s in
// the reference, d + 3*s in the packed layout.  One thread per float, coalesced on the destination.
__global__ void k_relayout(const float* __restrict__ src, float* __restrict__ dst, int64_t total, int nm,
                           int to_state) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int64_t row = 3 * (int64_t)nm;
    const int64_t c = i / row;
    const int e = (int)(i - c * row);
    int d, sl;                                      // (dimension, slot) of destination element e
    if (to_state) { d = (int)(e % 3); sl = e / 3; }  // destination packed, source reference
    else { d = e / nm; sl = e - d * nm; }            // destination reference, source packed
    const int es = to_state ? d * nm + sl : 3 * sl + d;
    dst[i] = src[c * row + es];
}

// Strong-scaling rehearsal only (PMC_XFER_DELAY_US): one wave that keeps the exchange stream busy
// for `ticks` of the 100 MHz real-time counter after a halo exchange -- the xGMI transfer time and
// RCCL latency a one-GPU rehearsal does not see.  Bounded by the tick count (no memory access).
__global__ void k_spin(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

}  // namespace

hipError_t launch_relayout(const float* src, float* dst, int64_t cells, int nmax, int to_state, hipStream_t st) {
    const int64_t total = cells * 3 * (int64_t)nmax;
    if (total <= 0) return hipSuccess;
    if (!PMC_AOS) return hipMemcpyAsync(dst, src, sizeof(float) * (size_t)total, hipMemcpyDeviceToDevice, st);
    hipLaunchKernelGGL(k_relayout, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, src, dst, total, nmax,
                       to_state);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// HBM probe (pmc_hbm_probe): the rate this GPU actually delivers, beside the
// 8 TB/s spec.  Streaming 16-B loads (and stores), several independent per lane in flight
// over a buffer far larger than the caches (MALL 256 MB): read -- each block folds its words into one
// xor written at the end (nothing else written); copy -- read + write the same amount.  U loads in
// flight per lane before their use.
// ------------------------------------------------------------------------------------------
template <int U>
__global__ void __launch_bounds__(256) k_hbm_read(const uint4* __restrict__ src, uint64_t n, uint32_t* __restrict__ sink) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        uint32_t v[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {   // nontemporal: streamed past the caches (fastest, profiles/r06h)
            const uint32_t* q = reinterpret_cast<const uint32_t*>(src + i + u * stride);
#pragma unroll
            for (int w = 0; w < 4; ++w) v[u][w] = __builtin_nontemporal_load(q + w);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
    }
    for (; i < n; i += stride) {
        const uint4 a = src[i];
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;   // (keeps the loads; practically never stores)
}

// copy: each workgroup streams its own contiguous chunk (faster than grid-stride for copies, r06h)
template <int U>
__global__ void __launch_bounds__(256) k_hbm_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n) {
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += U * 256) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < b1) v[u] = src[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < b1) dst[i + u * 256] = v[u];
    }
}

// kind 0 read, 1 copy; unroll 4 or 8 loads in flight per lane
hipError_t launch_hbm_probe(int kind, int unroll, const void* src, void* dst, uint64_t bytes, uint32_t* sink,
                            int blocks, hipStream_t st) {
    const uint64_t n = bytes / 16;
    const uint4* a = (const uint4*)src;
    if (kind == 0) {
        if (unroll == 8) hipLaunchKernelGGL(k_hbm_read<8>, dim3(blocks), dim3(256), 0, st, a, n, sink);
        else hipLaunchKernelGGL(k_hbm_read<4>, dim3(blocks), dim3(256), 0, st, a, n, sink);
    } else {
        if (unroll == 8) hipLaunchKernelGGL(k_hbm_copy<8>, dim3(blocks), dim3(256), 0, st, a, (uint4*)dst, n);
        else hipLaunchKernelGGL(k_hbm_copy<4>, dim3(blocks), dim3(256), 0, st, a, (uint4*)dst, n);
    }
    return hipGetLastError();
}

hipError_t launch_spin(double us, hipStream_t st) {
    const uint64_t ticks = us > 0.0 ? (uint64_t)(us * 100.0) : 0;   // s_memrealtime: 100 MHz
    if (ticks > 100000000ull) return hipErrorInvalidValue;          // at most 1 s
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(kWave), 0, st, ticks);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// IPC halo transport (pmc_slab_init_ipc): the slab driver's point-to-point messages between rank
// processes of one node (or several processes on one GPU), through IPC-mapped peer buffers and
// per-rank sequence flags in uncached device memory -- no host round trip per exchange.  Exchange k
// on the exchange stream is ONE launch, k_xfer<true>: block 0 publishes ready[me] = k (every
// earlier kernel of the stream has ended: its writes are released); every block waits until
// ready[p] >= k for each peer p this rank receives from, and until pulled[p] >= k' for each peer
// that read this rank's buffers in the previous exchange k' (so this exchange and everything after
// it may overwrite them); then pulls its share of every message from the peer's buffer into ours;
// the last block to finish stores pulled[me] = k.  PMC_IPC_FUSED=0 splits it into k_xfer_flag (the
// signal and the waits) and k_xfer<false> (the copy), whose reads then follow the command
// processor's kernel-start acquire rather than the shader's.  k_xfer_flag alone (no signal) settles
// the last exchange's "pulled" before host-visible points (pmc_slab_finish, copies, teardown).
// Waits give up after `timeout` ticks of the 100 MHz real-time counter and set error-flag bit 9
// (value 512) instead of hanging the GPU.
// ------------------------------------------------------------------------------------------
namespace {

__device__ __forceinline__ uint64_t flag_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void flag_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one thread: every w.flag[i] >= w.target[i] (false on timeout, after setting error bit 9)
__device__ __forceinline__ bool flags_wait(const XferFlags& w, uint64_t timeout, uint32_t* err) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < w.n; ++i) {
        while (flag_load(w.flag[i]) < w.target[i]) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
                atomicOr(err, 512u);
                return false;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    return true;
}

// Publish ready = seq for a peer on ANOTHER GPU to pull this rank's buffers.  The planes were written
// by earlier kernels, whose end-of-kernel release is only guaranteed to reach agent scope: dirty lines
// may sit in any of the 8 XCDs' L2s, invisible to a peer reading this GPU's HBM over xGMI.  So every
// block's thread 0 first writes back its XCD's L2 (system-scope release: buffer_wbl2 sc0 sc1) and
// checks in (count, and the XCC_ID bit in a mask); block 0 waits for all blocks, then stores the flag.
// The grid has >= 8 blocks: the dispatcher deals them round-robin over the XCDs, and the mask proves
// that every XCD wrote back (error bit 10, value 1024, if one did not).  wb[0]: count, wb[2]: mask.
__device__ __forceinline__ void publish_ready(uint64_t* ready, uint64_t seq, unsigned* wb, uint64_t timeout,
                                              uint32_t* err) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    __hip_atomic_fetch_or(wb + 2, 1u << (xcc & 7u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_fetch_add(wb, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (blockIdx.x != 0) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(wb, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < gridDim.x) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
            atomicOr(err, 512u);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    if (__hip_atomic_load(wb + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0xFFu) atomicOr(err, 1024u);
    __hip_atomic_store(wb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(wb + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    flag_store(ready, seq);
}

// mine: publish ready (grid >= 8, publish_ready) then wait for w; no mine: wait only (one block)
__global__ void __launch_bounds__(kWave) k_xfer_flag(uint64_t* mine, uint64_t seq, XferFlags w, uint64_t timeout,
                                                      uint32_t* err, unsigned* wb) {
    if (threadIdx.x != 0) return;
    if (mine) publish_ready(mine, seq, wb, timeout, err);
    if (blockIdx.x == 0) (void)flags_wait(w, timeout, err);
}

template <class U>
__device__ __forceinline__ void xfer_units(const XferSeg& s, int shift) {
    const U* __restrict__ src = reinterpret_cast<const U*>(s.src);
    U* __restrict__ dst = reinterpret_cast<U*>(s.dst);
    const uint64_t n = s.bytes >> shift;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // four independent loads in flight per lane before their stores
    for (; i + 3 * stride < n; i += 4 * stride) {
        const U a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

// WAIT (the one-launch form, PMC_IPC_FUSED): block 0 publishes ready[me] = seq and every block's
// thread 0 waits for w itself (system-scope acquire loads: the fence after the satisfied load
// invalidates the CU's L1 and the XCD's non-coherent L2 lines -- the peer's buffer as seen through
// its mapping: NC for another GPU's memory; this GPU's own memory is kept coherent across the XCDs'
// L2s by the cache probes of the PTE C-bit, AMDGPU memory model, gfx942 family) before the block's
// threads read past the workgroup barrier.  Grid <= 64 blocks: waiting blocks hold wave slots, and
// several rank processes may share one GPU.
constexpr unsigned kXferMinBlocks = 8;   // publish_ready: one block per XCD at least

template <bool WAIT>
__global__ void __launch_bounds__(256) k_xfer(XferCopy cp, uint64_t* pulled, uint64_t seq, unsigned* done,
                                               XferFlags w, uint64_t* ready, uint64_t timeout, uint32_t* err) {
    // A wait that timed out (this launch's, or k_xfer_flag's before a split copy) leaves error bit 9
    // set: the block then copies nothing -- the peer's buffer may be mid-write -- and "pulled" is not
    // published, so no peer overwrites buffers this rank has not read; from then on every exchange of
    // this rank and its peers times out too, and pmc_slab_finish / the observables report the error.
    __shared__ int go;
    if (threadIdx.x == 0) {
        bool ok = true;
        if constexpr (WAIT) {
            publish_ready(ready, seq, done + 2, timeout, err);
            ok = flags_wait(w, timeout, err);
        }
        go = ok && (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 512u) == 0;
    }
    __syncthreads();
    if (go) {
        for (int k = 0; k < cp.n; ++k) {
            const XferSeg& s = cp.seg[k];
            switch (s.shift) {
                case 4: xfer_units<uint4>(s, 4); break;
                case 3: xfer_units<uint2>(s, 3); break;
                case 2: xfer_units<uint32_t>(s, 2); break;
                case 1: xfer_units<uint16_t>(s, 1); break;
                default: xfer_units<uint8_t>(s, 0); break;
            }
        }
    }
    __syncthreads();                      // every load of this block has returned (its stores used them)
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
        if (prev == gridDim.x - 1) {
            __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 512u) == 0)
                flag_store(pulled, seq);
        }
    }
}

}  // namespace

hipError_t launch_xfer_flag(uint64_t* mine, uint64_t seq, const XferFlags& w, uint64_t timeout_ticks, uint32_t* err,
                            hipStream_t st) {
    if (w.n < 0 || w.n > kXferMax) return hipErrorInvalidValue;   // (seq: the value stored to mine)
    if (mine) return hipErrorInvalidValue;   // wait only (a ready flag is published by launch_xfer's grid)
    hipLaunchKernelGGL(k_xfer_flag, dim3(1), dim3(kWave), 0, st, mine, seq, w, timeout_ticks, err, (unsigned*)nullptr);
    return hipGetLastError();
}

hipError_t launch_xfer(const XferCopy& cp, const XferFlags& w, uint64_t* ready, uint64_t* pulled, uint64_t seq,
                       unsigned* done, uint64_t timeout_ticks, uint32_t* err, hipStream_t st) {
    if (cp.n < 0 || cp.n > kXferMax || w.n < 0 || w.n > kXferMax || !ready || !pulled || !done)
        return hipErrorInvalidValue;
    uint64_t units = 0;   // 16-B units of the largest segment set the grid: ~4 per lane
    for (int k = 0; k < cp.n; ++k) {
        const XferSeg& s = cp.seg[k];
        if (s.shift < 0 || s.shift > 4 || (s.bytes & ((1ull << s.shift) - 1)) ||
            (((uintptr_t)s.src | (uintptr_t)s.dst) & ((1ull << s.shift) - 1)))
            return hipErrorInvalidValue;
        units += (s.bytes + 15) / 16;
    }
    // PMC_IPC_FUSED=0: the wait as a launch of its own before the copy (the copy's reads then follow
    // the command processor's kernel-start acquire instead of the shader's)
    static const bool fused = [] {
        const char* v = std::getenv("PMC_IPC_FUSED");
        return !(v && std::atoi(v) == 0);
    }();
    const uint64_t want = (units + 1023) / 1024;
    if (fused) {
        const unsigned blocks = (unsigned)(want < kXferMinBlocks ? kXferMinBlocks : want > 64 ? 64 : want);
        hipLaunchKernelGGL(k_xfer<true>, dim3(blocks), dim3(256), 0, st, cp, pulled, seq, done, w, ready, timeout_ticks,
                           err);
    } else {
        hipLaunchKernelGGL(k_xfer_flag, dim3(kXferMinBlocks), dim3(kWave), 0, st, ready, seq, w, timeout_ticks, err,
                           done + 2);
        const unsigned blocks = (unsigned)(want < 1 ? 1 : want > 256 ? 256 : want);
        hipLaunchKernelGGL(k_xfer<false>, dim3(blocks), dim3(256), 0, st, cp, pulled, seq, done, w, ready,
                           timeout_ticks, err);
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
// hipLaunchKernelGGL, or with dispatch-packet timing events when tm is given
template <class K, class... A>
static void launch_k(K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t st, const LaunchTiming* tm, A... args) {
    // the argument block is packed from these types: the host-only geometry must be sliced first
    static_assert(!(std::is_same<A, HostGeom>::value || ...), "pass the DevGeom part of a HostGeom");
    if (tm && tm->start) hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, st, tm->start, tm->stop, 0u, args...);
    else hipLaunchKernelGGL(kernel, grid, block, lds, st, args...);
}

// Grid of the overflow launch (it strides over the queue).  The queue is empty in almost every
// phase (a cell overflows the main launch's LDS capacity only if its filtered stencil holds more
// than kMainCap partners); the launch costs the same ~5 us of dispatch with 1, 8 or 64 workgroups
// (kernel trace, tools/strong_trace.sh), so 8 (one per XCD) spread a crowded queue at no cost.
// PMC_FALLBACK_BLOCKS=n overrides (n = 1: no completion atomics at all).
static unsigned fallback_blocks() {
    static const unsigned n = [] {
        const char* v = std::getenv("PMC_FALLBACK_BLOCKS");
        const int k = v ? std::atoi(v) : 8;
        return (unsigned)(k > 0 ? k : 1);
    }();
    return n;
}
int subsweep_capacity(const DevGeom& g) {
    // Partners per wave held in LDS by the main launch.  Sized so a wave needs at most 5 KiB of
    // LDS (-> 32 waves/CU, the hardware limit): 3 floats per partner (x, y, z) + 2 term-list
    // entries + row tails (kMainCap = 224).  The filtered stencil holds ~98 partners at n = 4.77 per
    // cell; larger ones use the fallback.
    const int full = 27 * g.nmax;
    // test hook: PMC_SUBSWEEP_CAP forces a (small) capacity so the fallback path is exercised
    static const int forced = [] {
        const char* e = std::getenv("PMC_SUBSWEEP_CAP");
        return e ? std::atoi(e) : 0;
    }();
    if (forced > 0) return forced < full ? forced : full;
    return kMainCap < full ? kMainCap : full;
}

template <int NSLOT, int NMC, bool OFF32>
static void launch_direct_t(const DevGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz, uint32_t sweep,
                            unsigned long long* stats, int* ovf, int cz0, int ncz, float* mirror, int mode,
                            hipStream_t st, const LaunchTiming* tm);

template <int NSLOT, int NMC, bool OFF32>
static void launch_subsweep_t(const DevGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz,
                              uint32_t sweep, unsigned long long* stats, int* ovf, int cz0, int ncz,
                              hipStream_t st, const LaunchTiming* tm, bool solo) {
    const int64_t total = (int64_t)(g.cps_x / 2) * (g.cps_y / 2) * ncz;
    const int64_t waves = (total + PMC_CELLS_PER_WAVE - 1) / PMC_CELLS_PER_WAVE;
    const int64_t blocks = (waves + kSubWaves - 1) / kSubWaves;
    const int cap = subsweep_capacity(g);
    const int full = 27 * g.nmax;
    static const int64_t small_cells = env_cells("PMC_SMALL_LAUNCH", 8192);
    if (total <= small_cells) {   // one launch, one full-capacity cell per wave (k_subsweep_full)
        const size_t lds_full = sizeof(float) * (size_t)lds_floats_per_wave(full) * kSubWaves;
        launch_k(k_subsweep_full<NSLOT, NMC, OFF32>, dim3((unsigned)((total + kSubWaves - 1) / kSubWaves)),
                 dim3(kWave * kSubWaves), lds_full, st, tm, g, disk, n, ox, oy, oz, sweep, stats, cz0, ncz);
        return;
    }
    // PMC_DIRECT_CELLS=<n> (default 0: off): phases of at most n cells as one cell per wave at the
    // main capacity (the slab boundary launch's form) -- half-length waves, more of them, for phases
    // of a few rounds of the chip's wave slots (A/B switch)
    static const int64_t direct_cells = env_cells("PMC_DIRECT_CELLS", 0);
    if (total <= direct_cells) {
        launch_direct_t<NSLOT, NMC, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, nullptr, 0, st, tm);
        return;
    }
    size_t lds = sizeof(float) * (size_t)lds_floats_per_wave(kMainCap) * kSubWaves;
    // Solo launches (nothing else on the GPU) of at most two rounds of the chip's wave slots (<= 32768
    // cells: 16384 two-cell waves) end in single-cell waves, 1/8 of each XCD's cells
    // (k_subsweep_mixed): config 2's phase -3.7% (profiles/r06m_mixed_tail_ab.txt).  Launches beside
    // another chain drain their tails under its work (4-rank rehearsal +1.9% with them) and keep
    // k_subsweep.  PMC_MIXED_SINGLES=<n> forces n
    // single-cell waves per XCD on every launch, 0 turns it off (A/B switch).
    static const int64_t mixed_env = env_cells("PMC_MIXED_SINGLES", -1);
    const int64_t mixed = mixed_env >= 0 ? mixed_env : ((solo && total <= 32768) ? (total + 63) / 64 : 0);
    if (mixed > 0 && kSubWaves == 1 && PMC_CELLS_PER_WAVE == 2) {
        const int per_xcd = (int)((total + 7) / 8);
        const int singles = (int)(mixed < per_xcd ? mixed : per_xcd);
        const int pair_waves = (per_xcd - singles) / 2;
        const int waves_xcd = pair_waves + (per_xcd - 2 * pair_waves);
        launch_k(k_subsweep_mixed<NSLOT, NMC, OFF32>, dim3(8u * (unsigned)waves_xcd), dim3(kWave), lds, st, tm, g, disk,
                 n, ox, oy, oz, sweep, stats, cap, ovf, cz0, ncz, per_xcd, pair_waves);
    } else
    launch_k(k_subsweep<NSLOT, NMC, OFF32>, dim3((unsigned)blocks), dim3(kWave * kSubWaves), lds, st, tm, g, disk, n,
             ox, oy, oz, sweep, stats, cap, ovf, cz0, ncz);
    if (cap < full) {
        const size_t lds_full = sizeof(float) * (size_t)lds_floats_per_wave(full) * kSubWaves;
        hipLaunchKernelGGL((k_subsweep_fallback<NSLOT, NMC, OFF32>), dim3(fallback_blocks()), dim3(kWave * kSubWaves), lds_full, st,
                           g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, (float*)nullptr, 0, 1, stats);
    }
}

template <int NSLOT, int NMC, bool OFF32>
static void launch_direct_t(const DevGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz, uint32_t sweep,
                            unsigned long long* stats, int* ovf, int cz0, int ncz, float* mirror, int mode,
                            hipStream_t st, const LaunchTiming* tm) {
    const int64_t total = (int64_t)(g.cps_x / 2) * (g.cps_y / 2) * ncz;
    const int64_t blocks = (total + kSubWaves - 1) / kSubWaves;   // one cell per wave
    const int cap = subsweep_capacity(g);
    const int full = 27 * g.nmax;
    // PMC_BOUNDARY_FULL=1: the boundary plane at full capacity (27*nmax partners, 9.9 KiB of LDS per
    // wave): nothing can overflow, so a phase is ONE launch -- no fallback launch on the exchange
    // stream, whose chain (boundary phases -> exchange -> next run's boundary phases) is the sweep's
    // critical path once the exchange takes xGMI time
    static const bool bfull = env_cells("PMC_BOUNDARY_FULL", 0) == 1;
    if (bfull && !mirror) {
        const size_t lds_full = sizeof(float) * (size_t)lds_floats_per_wave(full) * kSubWaves;
        launch_k(k_subsweep_full<NSLOT, NMC, OFF32, PMC_BOUNDARY_PB>, dim3((unsigned)blocks), dim3(kWave * kSubWaves),
                 lds_full, st, tm, g, disk, n, ox, oy, oz, sweep, stats, cz0, ncz);
        return;
    }
    const size_t lds = sizeof(float) * (size_t)lds_floats_per_wave(kMainCap) * kSubWaves;
    launch_k(k_subsweep_direct<NSLOT, NMC, OFF32>, dim3((unsigned)blocks), dim3(kWave * kSubWaves), lds, st, tm, g,
             disk, n, ox, oy, oz, sweep, stats, cap, ovf, cz0, ncz, mirror, mode);
    if (cap < full) {
        const size_t lds_full = sizeof(float) * (size_t)lds_floats_per_wave(full) * kSubWaves;
        if (mirror)
            hipLaunchKernelGGL((k_subsweep_fallback<NSLOT, NMC, OFF32, true>), dim3(fallback_blocks()),
                               dim3(kWave * kSubWaves), lds_full, st, g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0,
                               mirror, mode, 1, stats);
        else
            hipLaunchKernelGGL((k_subsweep_fallback<NSLOT, NMC, OFF32>), dim3(fallback_blocks()),
                               dim3(kWave * kSubWaves), lds_full, st, g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0,
                               (float*)nullptr, 0, 1, stats);
    }
}

// Quirks R1/R2 (pmc.h): every colour phase through the full-capacity one-cell-per-wave kernel,
// instantiated with the quirk bits (the corrected-semantics kernels are not touched by them)
template <int NSLOT, int NMC, bool OFF32, int QK>
static void launch_quirk_t(const DevGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz, uint32_t sweep,
                           unsigned long long* stats, int cz0, int ncz, hipStream_t st, const LaunchTiming* tm) {
    const int64_t total = (int64_t)(g.cps_x / 2) * (g.cps_y / 2) * ncz;
    const int full = 27 * g.nmax;
    const size_t lds_full = sizeof(float) * (size_t)lds_floats_per_wave(full) * kSubWaves;
    launch_k(k_subsweep_full<NSLOT, NMC, OFF32, 0, QK>, dim3((unsigned)((total + kSubWaves - 1) / kSubWaves)),
             dim3(kWave * kSubWaves), lds_full, st, tm, g, disk, n, ox, oy, oz, sweep, stats, cz0, ncz);
}
template <bool OFF32, int QK>
static void launch_quirk_q(const DevGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz, uint32_t sweep,
                           unsigned long long* stats, int cz0, int ncz, hipStream_t st, const LaunchTiming* tm) {
    if (g.nmax == 16) launch_quirk_t<16, 16, OFF32, QK>(g, disk, n, ox, oy, oz, sweep, stats, cz0, ncz, st, tm);
    else if (g.nmax == 32) launch_quirk_t<32, 32, OFF32, QK>(g, disk, n, ox, oy, oz, sweep, stats, cz0, ncz, st, tm);
    else if (g.nslot == 8) launch_quirk_t<8, 0, OFF32, QK>(g, disk, n, ox, oy, oz, sweep, stats, cz0, ncz, st, tm);
    else if (g.nslot == 16) launch_quirk_t<16, 0, OFF32, QK>(g, disk, n, ox, oy, oz, sweep, stats, cz0, ncz, st, tm);
    else if (g.nslot == 32) launch_quirk_t<32, 0, OFF32, QK>(g, disk, n, ox, oy, oz, sweep, stats, cz0, ncz, st, tm);
    else launch_quirk_t<64, 0, OFF32, QK>(g, disk, n, ox, oy, oz, sweep, stats, cz0, ncz, st, tm);
}
constexpr uint32_t kQuirksRng = PMC_FLAG_QUIRK_R1 | PMC_FLAG_QUIRK_R2;
template <bool OFF32>
static void launch_quirk_n(const HostGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz, uint32_t sweep,
                           unsigned long long* stats, int cz0, int ncz, hipStream_t st, const LaunchTiming* tm) {
    const DevGeom& kg = g;
    switch (g.quirks & kQuirksRng) {
        case PMC_FLAG_QUIRK_R1:
            launch_quirk_q<OFF32, PMC_FLAG_QUIRK_R1>(kg, disk, n, ox, oy, oz, sweep, stats, cz0, ncz, st, tm); break;
        case PMC_FLAG_QUIRK_R2:
            launch_quirk_q<OFF32, PMC_FLAG_QUIRK_R2>(kg, disk, n, ox, oy, oz, sweep, stats, cz0, ncz, st, tm); break;
        default:
            launch_quirk_q<OFF32, kQuirksRng>(kg, disk, n, ox, oy, oz, sweep, stats, cz0, ncz, st, tm); break;
    }
}

template <bool OFF32>
static void launch_direct_n(const DevGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz, uint32_t sweep,
                            unsigned long long* stats, int* ovf, int cz0, int ncz, float* mirror, int mode, hipStream_t st, const LaunchTiming* tm) {
    if (g.nmax == 16) launch_direct_t<16, 16, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, mirror, mode, st, tm);
    else if (g.nmax == 32) launch_direct_t<32, 32, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, mirror, mode, st, tm);
    else if (g.nslot == 8) launch_direct_t<8, 0, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, mirror, mode, st, tm);
    else if (g.nslot == 16) launch_direct_t<16, 0, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, mirror, mode, st, tm);
    else if (g.nslot == 32) launch_direct_t<32, 0, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, mirror, mode, st, tm);
    else launch_direct_t<64, 0, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, mirror, mode, st, tm);
}

template <bool OFF32>
static void launch_subsweep_n(const DevGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz,
                              uint32_t sweep, unsigned long long* stats, int* ovf, int cz0, int ncz,
                              hipStream_t st, const LaunchTiming* tm, bool solo) {
    if (g.nmax == 16) launch_subsweep_t<16, 16, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, st, tm, solo);
    else if (g.nmax == 32) launch_subsweep_t<32, 32, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, st, tm, solo);
    else if (g.nslot == 8) launch_subsweep_t<8, 0, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, st, tm, solo);
    else if (g.nslot == 16) launch_subsweep_t<16, 0, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, st, tm, solo);
    else if (g.nslot == 32) launch_subsweep_t<32, 0, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, st, tm, solo);
    else launch_subsweep_t<64, 0, OFF32>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, st, tm, solo);
}

// a timed launch with nothing to visit (a chain whose planes hold no plane of the colour): its
// events are recorded anyway (zero duration), so the caller's timing entry stays valid
static hipError_t skip_launch(hipStream_t st, const LaunchTiming* tm) {
    if (tm && tm->start) {
        hipError_t e = hipEventRecord(tm->start, st);
        if (e == hipSuccess) e = hipEventRecord(tm->stop, st);
        return e;
    }
    return hipSuccess;
}

hipError_t launch_subsweep_boundary(const HostGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz,
                                    uint32_t sweep, unsigned long long* stats, int* ovf, int zl_begin, int zl_end,
                                    float* mirror, int mirror_mode, hipStream_t st, const LaunchTiming* tm) {
    auto ceil_half = [](int v) { return v <= 0 ? 0 : (v + 1) / 2; };
    const int nczc = g.nz_local / 2;
    int cz0 = ceil_half(zl_begin - oz), cz1 = ceil_half(zl_end - oz);
    if (cz1 > nczc) cz1 = nczc;
    if (cz1 <= cz0) return skip_launch(st, tm);
    const int64_t bytes = (int64_t)g.cps_x * g.cps_y * (g.nz_local + 2 * g.halo) * 3 * g.nmax * 4;
    if (g.quirks & kQuirksRng) {   // (no mirror rows: pmc_slab_sweep turns the direct halo off with R1/R2)
        if (mirror) return hipErrorInvalidValue;
        if (bytes < ((int64_t)1 << 32)) launch_quirk_n<true>(g, disk, n, ox, oy, oz, sweep, stats, cz0, cz1 - cz0, st, tm);
        else launch_quirk_n<false>(g, disk, n, ox, oy, oz, sweep, stats, cz0, cz1 - cz0, st, tm);
        return hipGetLastError();
    }
    if (bytes < ((int64_t)1 << 32)) launch_direct_n<true>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, cz1 - cz0, mirror, mirror_mode, st, tm);
    else launch_direct_n<false>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, cz1 - cz0, mirror, mirror_mode, st, tm);
    return hipGetLastError();
}

template <int NSLOT, int NMC, bool OFF32>
static void launch_direct2_t(const DevGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz, uint32_t sweep,
                             unsigned long long* stats0, unsigned long long* stats1, int* ovf, int cz0, int czs,
                             hipStream_t st, const LaunchTiming* tm) {
    const int64_t total = 2 * (int64_t)(g.cps_x / 2) * (g.cps_y / 2);
    const int64_t blocks = (total + kSubWaves - 1) / kSubWaves;
    const int cap = subsweep_capacity(g);
    const int full = 27 * g.nmax;
    const size_t lds = sizeof(float) * (size_t)lds_floats_per_wave(kMainCap) * kSubWaves;
    launch_k(k_subsweep_direct2<NSLOT, NMC, OFF32>, dim3((unsigned)blocks), dim3(kWave * kSubWaves), lds, st, tm, g,
             disk, n, ox, oy, oz, sweep, stats0, stats1, cap, ovf, cz0, czs);
    if (cap < full) {
        const size_t lds_full = sizeof(float) * (size_t)lds_floats_per_wave(full) * kSubWaves;
        hipLaunchKernelGGL((k_subsweep_fallback<NSLOT, NMC, OFF32>), dim3(fallback_blocks()), dim3(kWave * kSubWaves),
                           lds_full, st, g, disk, n, ox, oy, oz, sweep, stats0, ovf, cz0, (float*)nullptr, 0, czs, stats1);
    }
}

hipError_t launch_subsweep_planes2(const DevGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz,
                                   uint32_t sweep, unsigned long long* stats0, unsigned long long* stats1, int* ovf,
                                   int zl0, int zl1, hipStream_t st, const LaunchTiming* tm) {
    // planes zl0 < zl1 of colour parity oz (halo planes included), at least one plane apart
    if (zl1 <= zl0 + 1 || ((zl0 - oz) & 1) || ((zl1 - oz) & 1)) return hipErrorInvalidValue;
    for (int zl : {zl0, zl1})
        if (zl - 1 < -g.halo || zl + 1 > g.nz_local - 1 + g.halo) return hipErrorInvalidValue;
    const int cz0 = (zl0 - oz) >> 1, czs = (zl1 - zl0) >> 1;
    const int64_t bytes = (int64_t)g.cps_x * g.cps_y * (g.nz_local + 2 * g.halo) * 3 * g.nmax * 4;
    const bool off32 = bytes < ((int64_t)1 << 32);
    auto go = [&](auto off) {
        constexpr bool O = decltype(off)::value;
        if (g.nmax == 16) launch_direct2_t<16, 16, O>(g, disk, n, ox, oy, oz, sweep, stats0, stats1, ovf, cz0, czs, st, tm);
        else if (g.nmax == 32) launch_direct2_t<32, 32, O>(g, disk, n, ox, oy, oz, sweep, stats0, stats1, ovf, cz0, czs, st, tm);
        else if (g.nslot == 8) launch_direct2_t<8, 0, O>(g, disk, n, ox, oy, oz, sweep, stats0, stats1, ovf, cz0, czs, st, tm);
        else if (g.nslot == 16) launch_direct2_t<16, 0, O>(g, disk, n, ox, oy, oz, sweep, stats0, stats1, ovf, cz0, czs, st, tm);
        else if (g.nslot == 32) launch_direct2_t<32, 0, O>(g, disk, n, ox, oy, oz, sweep, stats0, stats1, ovf, cz0, czs, st, tm);
        else launch_direct2_t<64, 0, O>(g, disk, n, ox, oy, oz, sweep, stats0, stats1, ovf, cz0, czs, st, tm);
    };
    if (off32) go(std::true_type{});
    else go(std::false_type{});
    return hipGetLastError();
}

hipError_t launch_subsweep_plane(const HostGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz,
                                 uint32_t sweep, unsigned long long* stats, int* ovf, int zl, hipStream_t st,
                                 const LaunchTiming* tm) {
    // one colour plane z = zl (parity oz) of storage, halo planes included (-halo .. nz_local-1+halo):
    // the boundary launch's per-cell path (main capacity + fallback), colour plane cz = (zl - oz) / 2
    if (((zl - oz) & 1) || zl < -g.halo || zl > g.nz_local - 1 + g.halo) return hipErrorInvalidValue;
    // the visit reads planes zl - 1 .. zl + 1, which must be stored
    if (g.halo && (zl - 1 < -g.halo || zl + 1 > g.nz_local - 1 + g.halo)) return hipErrorInvalidValue;
    const int cz = (zl - oz) >> 1;   // arithmetic shift: floor, so zl = -1 (oz = 1) gives -1
    const int64_t bytes = (int64_t)g.cps_x * g.cps_y * (g.nz_local + 2 * g.halo) * 3 * g.nmax * 4;
    if (g.quirks & kQuirksRng) {
        if (bytes < ((int64_t)1 << 32)) launch_quirk_n<true>(g, disk, n, ox, oy, oz, sweep, stats, cz, 1, st, tm);
        else launch_quirk_n<false>(g, disk, n, ox, oy, oz, sweep, stats, cz, 1, st, tm);
        return hipGetLastError();
    }
    if (bytes < ((int64_t)1 << 32)) launch_direct_n<true>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz, 1, nullptr, 0, st, tm);
    else launch_direct_n<false>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz, 1, nullptr, 0, st, tm);
    return hipGetLastError();
}

hipError_t launch_subsweep(const HostGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz,
                           uint32_t sweep, unsigned long long* stats, int* ovf, int zl_begin, int zl_end,
                           hipStream_t st, const LaunchTiming* tm, bool solo) {
    // colour planes z = 2*cz + oz inside [zl_begin, zl_end)
    auto ceil_half = [](int v) { return v <= 0 ? 0 : (v + 1) / 2; };
    const int nczc = g.nz_local / 2;
    int cz0 = ceil_half(zl_begin - oz), cz1 = ceil_half(zl_end - oz);
    if (cz1 > nczc) cz1 = nczc;
    if (cz1 <= cz0) return skip_launch(st, tm);
    const int ncz = cz1 - cz0;
    // 32-bit byte offsets when the disk buffer is below 4 GiB (every single-GPU 256^3 config)
    // (test hook: PMC_FORCE_ADDR64 takes the 64-bit path for any size)
    static const bool force64 = std::getenv("PMC_FORCE_ADDR64") != nullptr;
    const int64_t bytes = (int64_t)g.cps_x * g.cps_y * (g.nz_local + 2 * g.halo) * 3 * g.nmax * 4;
    if (g.quirks & kQuirksRng) {
        if (!force64 && bytes < ((int64_t)1 << 32)) launch_quirk_n<true>(g, disk, n, ox, oy, oz, sweep, stats, cz0, ncz, st, tm);
        else launch_quirk_n<false>(g, disk, n, ox, oy, oz, sweep, stats, cz0, ncz, st, tm);
        return hipGetLastError();
    }
    if (!force64 && bytes < ((int64_t)1 << 32)) launch_subsweep_n<true>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, st, tm, solo);
    else launch_subsweep_n<false>(g, disk, n, ox, oy, oz, sweep, stats, ovf, cz0, ncz, st, tm, solo);
    return hipGetLastError();
}

// Participants of k_sweep_small for a box (0: the box does not qualify -- nmax != 16, a slab, or
// a colour phase over 4 cells per participant).  XCD 0 holds 512 waves of the 9.9 KB layout.
int small_sweep_participants(const HostGeom& g) {
    if (g.nmax != 16 || g.halo || g.quirks) return 0;   // (quirks: the eager path)
    const int64_t per_colour = (int64_t)(g.cps_x / 2) * (g.cps_y / 2) * (g.cps_z / 2);
    if (per_colour > 4 * 512) return 0;
    return per_colour < 512 ? (int)per_colour : 512;
}

hipError_t launch_sweep_small(const HostGeom& g, float* disk0, int16_t* n0, float* disk1, int16_t* n1, int cur,
                              unsigned long long* stats, uint32_t* flags, unsigned* bar, uint64_t seed,
                              uint32_t first, int count, uint32_t plan_flags, hipStream_t st) {
    const int P = small_sweep_participants(g);
    if (P == 0) return hipErrorInvalidValue;
    const size_t lds = sizeof(float) * (size_t)lds_floats_per_wave(27 * 16);
    const bool off32 = (int64_t)g.cps_x * g.cps_y * g.cps_z * 3 * g.nmax * 4 < ((int64_t)1 << 32);
    if (!off32) return hipErrorInvalidValue;
    for (int done = 0; done < count;) {
        SmallPlans sp;
        std::memset(&sp, 0, sizeof(sp));
        sp.n = count - done < kSmallSweeps ? count - done : kSmallSweeps;
        sp.first = first + (uint32_t)done;
        for (int k = 0; k < sp.n; ++k) {
            const pmc_sweep_plan_t plan = pmc_plan_for_sweep_ex(seed, sp.first + (uint32_t)k, g.w, plan_flags);
            for (int c = 0; c < 8; ++c) sp.order[k][c] = plan.order[c];
            sp.f[k] = plan.f;
            sp.d[k] = plan.d;
        }
        hipError_t e = hipMemsetAsync(bar, 0, sizeof(unsigned), st);
        if (e != hipSuccess) return e;
        float* d0 = cur == 0 ? disk0 : disk1;
        float* d1 = cur == 0 ? disk1 : disk0;
        int16_t* m0 = cur == 0 ? n0 : n1;
        int16_t* m1 = cur == 0 ? n1 : n0;
        const DevGeom& kg = g;
        hipLaunchKernelGGL((k_sweep_small<16, 16, true>), dim3(8u * (unsigned)P), dim3(kWave), lds, st, kg, d0, m0, d1,
                           m1, stats, flags, bar, sp);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (sp.n & 1) cur ^= 1;
        done += sp.n;
    }
    return hipSuccess;
}

hipError_t launch_shift(const HostGeom& g, const float* din, const int16_t* nin, float* dout,
                        int16_t* nout, int f, float d, uint32_t* flags, hipStream_t st, const LaunchTiming* tm) {
    return launch_shift_planes(g, din, nin, dout, nout, f, d, flags, 0, g.nz_local, st, tm);
}

hipError_t launch_shift_planes(const HostGeom& g, const float* din, const int16_t* nin, float* dout,
                               int16_t* nout, int f, float d, uint32_t* flags, int zl_begin, int zl_end,
                               hipStream_t st, const LaunchTiming* tm) {
    if (zl_begin < -g.halo || zl_end > g.nz_local + g.halo || zl_end <= zl_begin) return hipErrorInvalidValue;
    if (f == 2 && g.halo) {   // along z each plane reads its dir-neighbour, which must be stored
        const int dir = (d <= 0) ? -1 : 1;
        if (zl_begin + dir < -g.halo || zl_end - 1 + dir > g.nz_local - 1 + g.halo) return hipErrorInvalidValue;
    }
#ifndef PMC_SHIFT_U
#define PMC_SHIFT_U 8
#endif
    constexpr int U = PMC_SHIFT_U;   // cells per lane group, loads hoisted
    const int cpb = kShiftThreads / g.nslot;
    const unsigned gxs = (unsigned)((g.cps_x + cpb * U - 1) / (cpb * U));
    const dim3 grid(gxs, (unsigned)g.cps_y, (unsigned)(zl_end - zl_begin));
    const dim3 block(kShiftThreads);
    const int z0 = zl_begin;
    // 32-bit byte offsets when the storage is below 4 GiB (PMC_SHIFT_OFF32=0: the 64-bit form).  With
    // the reference rows it measured no faster (0.203-0.204 against 0.199-0.203 ms,
    // profiles/r04q_shift_off32_ab.txt); with the packed layout 0.146-0.147 against 0.151-0.153 ms
    // (profiles/r05h_shift_variants_ab.txt), so it is the default now
    static const bool off32_env = env_cells("PMC_SHIFT_OFF32", 1) != 0;
    const int64_t bytes = (int64_t)g.cps_x * g.cps_y * (g.nz_local + 2 * g.halo) * 3 * g.nmax * 4;
    const bool off32 = off32_env && bytes < ((int64_t)1 << 32);
    // PMC_SHIFT_RUN (default 1): runs of kShiftRun cells along the shift axis per lane group (k_shift_run)
    static const bool run_env = env_cells("PMC_SHIFT_RUN", 1) != 0;
    const int nzr = zl_end - zl_begin;
    const int len = f == 0 ? g.cps_x : (f == 1 ? g.cps_y : nzr);
    const int64_t runs = (int64_t)((len + kShiftRun - 1) / kShiftRun) *
                         (f == 0 ? (int64_t)g.cps_y * nzr : (f == 1 ? (int64_t)g.cps_x * nzr : (int64_t)g.cps_x * g.cps_y));
    const int64_t lgs = kShiftThreads / g.nslot;
    const dim3 rgrid((unsigned)((runs + lgs - 1) / lgs));
    const DevGeom& kg = g;   // the kernels' argument block
    auto go = [&](auto ns, auto s1) {
        constexpr int NS = decltype(ns)::value;
        constexpr bool S1 = decltype(s1)::value;
        if (run_env) {
            if (off32) launch_k(k_shift_run<NS, kShiftRun, 1, S1>, rgrid, block, 0, st, tm, kg, din, nin, dout, nout, f, d, flags, z0, nzr);
            else launch_k(k_shift_run<NS, kShiftRun, 0, S1>, rgrid, block, 0, st, tm, kg, din, nin, dout, nout, f, d, flags, z0, nzr);
            return;
        }
        if (off32) launch_k(k_shift<NS, U, 1, S1>, grid, block, 0, st, tm, kg, din, nin, dout, nout, f, d, flags, z0);
        else launch_k(k_shift<NS, U, 0, S1>, grid, block, 0, st, tm, kg, din, nin, dout, nout, f, d, flags, z0);
    };
    // quirk S1 (pmc.h): the integer offset -- its own instantiations, the default kernels unchanged
    auto by_slot = [&](auto s1) {
        switch (g.nslot) {
            case 8: go(std::integral_constant<int, 8>{}, s1); break;
            case 16: go(std::integral_constant<int, 16>{}, s1); break;
            case 32: go(std::integral_constant<int, 32>{}, s1); break;
            default: go(std::integral_constant<int, 64>{}, s1); break;
        }
    };
    if (g.quirks & PMC_FLAG_QUIRK_S1) by_slot(std::true_type{});
    else by_slot(std::false_type{});
    return hipGetLastError();
}

hipError_t launch_init_r(const DevGeom& g, int64_t n_atoms, int64_t n_cube, float* r, hipStream_t st) {
    if (n_atoms <= 0) return hipSuccess;
    dim3 grid((unsigned)((n_atoms + 255) / 256)), block(256);
    hipLaunchKernelGGL(k_init_r, grid, block, 0, st, g, n_atoms, n_cube, r);
    return hipGetLastError();
}

hipError_t launch_assign(const DevGeom& g, const float* r, int64_t n_atoms, float* disk, int16_t* n,
                         int32_t* tmp_cnt, int32_t* tmp_idx, uint32_t* flags, hipStream_t st, int clip,
                         int ref_layout) {
    const int64_t cells = (int64_t)g.cps_x * g.cps_y * (g.nz_local + 2 * g.halo);
    hipError_t e = hipMemsetAsync(tmp_cnt, 0, sizeof(int32_t) * (size_t)cells, st);
    if (e != hipSuccess) return e;
    if (n_atoms > 0) {
        dim3 grid((unsigned)((n_atoms + 255) / 256)), block(256);
        hipLaunchKernelGGL(k_assign_count, grid, block, 0, st, g, r, n_atoms, tmp_cnt, tmp_idx, flags, clip);
    }
    dim3 grid2((unsigned)((cells + 255) / 256)), block2(256);
    hipLaunchKernelGGL(k_assign_fill, grid2, block2, 0, st, g, r, n_atoms, tmp_cnt, tmp_idx, disk, n, cells,
                       ref_layout);
    return hipGetLastError();
}

size_t energy_segments(const DevGeom& g) {
    return (size_t)((g.cps_x + kESeg - 1) / kESeg) * (size_t)g.cps_y * (size_t)g.nz_local;
}

// segq: int[1 + energy_segments(g)], zeroed by the caller before the launches (on st).  Interior
// cells by row segments (k_energy_rows), edge cells (k_energy MODE 1), then the segments the rows
// kernel queued (MODE 2, normally none).  PMC_ENERGY_LEGACY=1: MODE 0 alone (every cell per cell).
hipError_t launch_energy(const DevGeom& g, const float* disk, const int16_t* n,
                         unsigned long long* acc, int* segq, hipStream_t st) {
    const int64_t total = (int64_t)g.cps_x * g.cps_y * g.nz_local;   // owned cells
    const size_t lds = sizeof(float) * (3 * 27 * (size_t)g.nmax + kEnergyRing + 32);
    dim3 grid((unsigned)((total + kEnergyCells - 1) / kEnergyCells)), block(kWave);
    const uint32_t tc = (uint32_t)total;
    // 32-bit byte offsets below 4 GiB of disk (every single-GPU 256^3 box), else element offsets
    const int64_t bytes = (int64_t)g.cps_x * g.cps_y * (g.nz_local + 2 * g.halo) * 3 * g.nmax * 4;
    const bool off32 = bytes < ((int64_t)1 << 32);
    static const bool legacy = [] {
        const char* v = std::getenv("PMC_ENERGY_LEGACY");
        return v && std::atoi(v) == 1;
    }();
    // test hook: PMC_ENERGY_ROWS_CAP lowers the staging capacity (0: every segment queued, MODE 2)
    static const int cap = [] {
        const char* v = std::getenv("PMC_ENERGY_ROWS_CAP");
        const int k = v ? std::atoi(v) : kECap;
        return k < 0 ? 0 : (k > kECap ? kECap : k);
    }();
    const int nsx = (g.cps_x + kESeg - 1) / kESeg;
    const UDivMagic div_nsx = make_udiv_magic((uint32_t)nsx), div_cy = make_udiv_magic((uint32_t)g.cps_y);
    // edge cells (energy_edge_cell): planes 0 and nz_local-1 whole, the rim of every plane between
    // (every plane's first and last plane coincide with the slab's halo-neighbour or box-face planes)
    const int64_t n_edge = 2 * (int64_t)g.cps_x * g.cps_y +
                           (int64_t)(g.nz_local - 2) * (2 * (int64_t)g.cps_x + 2 * (int64_t)(g.cps_y - 2));
    const size_t lds_rows = sizeof(float) * (3 * kECap + kEnergyRing) + sizeof(uint16_t) * kEList + sizeof(int2) * 64;
    static_assert(sizeof(float) * (3 * kECap + kEnergyRing) + sizeof(uint16_t) * kEList + sizeof(int2) * 64 <= 5120 || kESeg != 6,
                  "energy rows: 8 waves per SIMD");   // (holds for both ring sizes, kECap above)
    const dim3 grid_rows((unsigned)energy_segments(g));
    // The rows kernel stages a cell's half-shell partner list of at most kEList entries: with nmax >
    // 16 it could overflow, and every segment would be queued for MODE 2 -- run the per-cell kernel
    // over every cell instead (MODE 0, ~total/16 waves).  MODE 2's grid covers the queue's worst case
    // up to the chip's wave slots (blocks past the queue length exit at once): a dense box that
    // queues many segments keeps the whole chip (a fixed 64-wave grid was ~100x slower then).
    const bool per_cell = legacy || 14 * g.nmax > kEList;
    const unsigned seg_total = (unsigned)energy_segments(g);
    const dim3 grid_q(seg_total < 8192u ? (seg_total > 0u ? seg_total : 1u) : 8192u);
    auto go = [&](auto k0, auto k1, auto k2, auto kr) {
        if (per_cell) {
            hipLaunchKernelGGL(k0, grid, block, lds, st, g, disk, n, acc, tc, segq, div_nsx);
            return;
        }
        hipLaunchKernelGGL(kr, grid_rows, block, lds_rows, st, g, disk, n, acc, segq, div_nsx, div_cy, cap);
        hipLaunchKernelGGL(k1, dim3((unsigned)((n_edge + kEdgeCells - 1) / kEdgeCells)), block, lds, st, g, disk, n,
                           acc, (uint32_t)n_edge, segq, div_nsx);
        hipLaunchKernelGGL(k2, grid_q, block, lds, st, g, disk, n, acc, tc, segq, div_nsx);
    };
#define PMC_ENERGY_GO(NS, O32) go(k_energy<NS, O32, 0>, k_energy<NS, O32, 1>, k_energy<NS, O32, 2>, k_energy_rows<NS, O32>)
    switch (g.nslot) {
        case 8: off32 ? PMC_ENERGY_GO(8, true) : PMC_ENERGY_GO(8, false); break;
        case 16: off32 ? PMC_ENERGY_GO(16, true) : PMC_ENERGY_GO(16, false); break;
        case 32: off32 ? PMC_ENERGY_GO(32, true) : PMC_ENERGY_GO(32, false); break;
        default: off32 ? PMC_ENERGY_GO(64, true) : PMC_ENERGY_GO(64, false); break;
    }
#undef PMC_ENERGY_GO
    return hipGetLastError();
}


hipError_t launch_colour_rows(const DevGeom& g, const float* src, float* dst, int colour, int mode, hipStream_t st) {
    int o[3];
    pmc_colour_offset(colour, o);
    const int row = 3 * g.nmax;
    const int64_t total = (int64_t)(g.cps_x / 2) * (g.cps_y / 2) * row;
    dim3 grid((unsigned)((total + 255) / 256)), block(256);
    hipLaunchKernelGGL(k_colour_rows, grid, block, 0, st, src, dst, g.cps_x, g.cps_y, row, o[0], o[1], mode);
    return hipGetLastError();
}

hipError_t launch_selftest(const uint32_t* words, int count, float* out_f, double* out_d, float rc2,
                           hipStream_t st) {
    dim3 grid((unsigned)((count + 255) / 256)), block(256);
    hipLaunchKernelGGL(k_selftest, grid, block, 0, st, words, count, out_f, out_d, rc2);
    return hipGetLastError();
}

}  // namespace pmc

#ifdef PMC_STAMPS
extern "C" int pmc_debug_stamps(size_t n_cells, unsigned long long* host_out) {
    static unsigned long long* buf = nullptr;
    static size_t cap = 0;
    if (host_out == nullptr) {   // enable (allocate + zero) for n_cells colour cells
        if (n_cells > cap) {
            if (buf) (void)hipFree(buf);
            if (hipMalloc(&buf, n_cells * 16 * sizeof(unsigned long long)) != hipSuccess) return -2;
            cap = n_cells;
        }
        if (hipMemset(buf, 0, n_cells * 16 * sizeof(unsigned long long)) != hipSuccess) return -2;
        return hipMemcpyToSymbol(HIP_SYMBOL(pmc::g_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -2;
    }
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpy(host_out, buf, n_cells * 16 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return -2;
    unsigned long long* null = nullptr;   // disable
    return hipMemcpyToSymbol(HIP_SYMBOL(pmc::g_stamps), &null, sizeof(null)) == hipSuccess ? 0 : -2;
}
#endif
