// pmc_kernels.hip -- hand-written CDNA4 (gfx950) kernels for the checkerboard Metropolis hot path.
//
// Reference semantics: subsweep.h (root, "Version I": thread per cell) for the call surface and
// move rules; the LDS-staging design of CUDA-Parallel-MC/CUDA-Parallel-MC/kernel.cu:209-435
// ("Version II": block per cell) re-targeted to ONE 64-lane wavefront per cell:
//   * the cell's 27-cell stencil (own cell first, shuffled; then the 26 neighbours in
//     get_neighbors order, subsweep.h:119-137) is staged once into LDS (SoA x/y/z), with the
//     periodic image (apply_PBC, subsweep.h:139-151) folded into the staged coordinates;
//   * per trial move every lane evaluates old and new pair energies of its partners
//     (lane = partner index mod 64) and the wave reduces dE with DPP / swizzle (no LDS, no
//     barrier); accept/reject is wave-uniform and in-kernel;
//   * Philox4x32-10 counter slots give every (sweep, cell, move) its own random numbers, so
//     results are independent of launch geometry and identical to the CPU oracle.
// No MFMA: this is not a dense contraction (pair energies are gathered, cut-off, divided).
//
// Build with -ffp-contract=off: every float/double op must stay a single IEEE op (the oracle,
// compiled by gcc with the same flag, reproduces the results bit for bit).
#include "pmc_internal.h"
#include "../../include/pmc_detmath.h"

namespace pmc {

namespace {

__device__ __forceinline__ float as_f(int v) { return __builtin_bit_cast(float, v); }
__device__ __forceinline__ int as_i(float v) { return __builtin_bit_cast(int, v); }

// Wave-wide float sum with a FIXED xor-butterfly order (1,2,4,8,16,32).  Every lane ends with
// the same bits; the oracle replays exactly this tree (oracle/pmc_oracle.c subsweep_cell).
// Mirror DPP patterns are used for the xor-4 / xor-8 steps: after the previous steps all lanes of
// a quad (resp. half-row) hold equal values, so l^7 / l^15 supply the same operand as l^4 / l^8.
__device__ __forceinline__ float wave_sum_fixed_order(float v) {
    v = v + as_f(__builtin_amdgcn_mov_dpp(as_i(v), 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
    v = v + as_f(__builtin_amdgcn_mov_dpp(as_i(v), 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
    v = v + as_f(__builtin_amdgcn_mov_dpp(as_i(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = v + as_f(__builtin_amdgcn_mov_dpp(as_i(v), 0x140, 0xF, 0xF, false));  // row_mirror
    v = v + as_f(__builtin_amdgcn_ds_swizzle(as_i(v), 0x401F));               // xor 16 (in 32)
    float a = as_f(__builtin_amdgcn_readlane(as_i(v), 0));
    float b = as_f(__builtin_amdgcn_readlane(as_i(v), 32));
    return a + b;                                                             // xor 32
}

__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// storage index of local cell (x, y, zl)
__device__ __forceinline__ int64_t sidx(const DevGeom& g, int x, int y, int zl) {
    return (int64_t)x + (int64_t)g.cps_x * ((int64_t)y + (int64_t)g.cps_y * (int64_t)(zl + g.halo));
}

// ------------------------------------------------------------------------------------------
// subsweep: one colour phase, one wave per cell (subsweep_kernel, subsweep.h:240-300)
// ------------------------------------------------------------------------------------------
template <int NSLOT>
__global__ __launch_bounds__(kWave * kSubWaves) void k_subsweep(DevGeom g, float* __restrict__ disk,
                                                                  const int16_t* __restrict__ ncnt,
                                                                  int ox, int oy, int oz, uint32_t sweep,
                                                                  unsigned long long* __restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int CPP = kWave / NSLOT;            // stencil cells staged per pass
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x >> 6;
    const int nm = g.nmax;
    const int cap = 27 * nm;
    float* xs = smem + wv * 3 * cap;
    float* ys = xs + cap;
    float* zs = ys + cap;

    // XCD-aware block order: blocks b and b+8 share an XCD (round-robin dispatch), so give each
    // XCD a contiguous run of cells -> neighbouring stencils share that XCD's L2.  Speed only.
    uint32_t nblk = gridDim.x, b = blockIdx.x;
    if ((nblk & 7u) == 0u) b = (b & 7u) * (nblk >> 3) + (b >> 3);
    const int ncx = g.cps_x >> 1, ncy = g.cps_y >> 1, ncz = g.nz_local >> 1;
    const int64_t total = (int64_t)ncx * ncy * ncz;
    const int64_t t = (int64_t)b * kSubWaves + wv;
    if (t >= total) return;
    const int ta = wave_uniform((int)(t % ncx));
    const int tb = wave_uniform((int)((t / ncx) % ncy));
    const int tc = wave_uniform((int)(t / ((int64_t)ncx * ncy)));
    const int x = 2 * ta + ox, y = 2 * tb + oy, zl = 2 * tc + oz;
    const int64_t c = sidx(g, x, y, zl);
    const int n_own = wave_uniform(ncnt[c]);
    if (n_own == 0) return;                                   // subsweep.h:252-253
    const uint32_t id = (uint32_t)x + (uint32_t)g.cps_x * ((uint32_t)y + (uint32_t)g.cps_y * (uint32_t)(g.z0 + zl));

    // ---- stencil table: lane k < 27 describes stencil cell k ------------------------------
    int k_cnt = 0, k_idx = 0;
    float k_sx = 0.0f, k_sy = 0.0f, k_sz = 0.0f;
    if (lane < 27) {
        const int hx = lane / 9, hy = (lane / 3) % 3, hz = lane % 3;   // {0,-1,+1} order
        const int dx = hx == 0 ? 0 : (hx == 1 ? -1 : 1);
        const int dy = hy == 0 ? 0 : (hy == 1 ? -1 : 1);
        const int dz = hz == 0 ? 0 : (hz == 1 ? -1 : 1);
        int nx = x + dx, ny = y + dy;
        if (nx < 0) { nx += g.cps_x; k_sx = -g.Lx; } else if (nx >= g.cps_x) { nx -= g.cps_x; k_sx = g.Lx; }
        if (ny < 0) { ny += g.cps_y; k_sy = -g.Ly; } else if (ny >= g.cps_y) { ny -= g.cps_y; k_sy = g.Ly; }
        const int zg = g.z0 + zl + dz;
        if (zg < 0) k_sz = -g.Lz; else if (zg >= g.cps_z) k_sz = g.Lz;
        const int nzl = g.halo ? zl + dz : (zl + dz + g.cps_z) % g.cps_z;
        k_idx = (int)sidx(g, nx, ny, nzl);
        k_cnt = ncnt[k_idx];
    }
    // inclusive scan of counts -> staged base of each stencil cell
    int incl = k_cnt;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
        int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    const int S = __builtin_amdgcn_readlane(incl, 26);        // staged partners incl. own cell
    const int k_base = incl - k_cnt;

    const uint32_t k0 = g.k0, k1 = g.k1;

    // ---- Fisher-Yates shuffle of the own cell (random_shuffle, subsweep.h:50-58; fixes R1) ----
    int perm = lane;
    {
        int jv = 0;
        if (lane >= 1 && lane < n_own) {
            pmc_u32x4 wv4 = pmc_philox4x32_10((uint32_t)lane, id, sweep, PMC_TAG_SHUFFLE, k0, k1);
            jv = (int)pmc_bounded(wv4.v[0], (uint32_t)(lane + 1));
        }
        for (int i = n_own - 1; i > 0; --i) {
            const int j = __builtin_amdgcn_readlane(jv, i);
            const int vi = __builtin_amdgcn_readlane(perm, i);
            const int vj = __builtin_amdgcn_readlane(perm, j);
            perm = lane == i ? vj : (lane == j ? vi : perm);
        }
    }

    // ---- stage the 27-cell stencil into LDS (cpy_to_Dsh, subsweep.h:18-27; kernel.cu:269-278) --
    {
        const int p = lane & (NSLOT - 1);
        const int kk = lane / NSLOT;
        for (int q = 0; q < (27 + CPP - 1) / CPP; ++q) {
            const int k = q * CPP + kk;
            const int ks = k < 27 ? k : 26;
            const int cnt = __shfl(k_cnt, ks);
            const int base = __shfl(k_base, ks);
            const int idx = __shfl(k_idx, ks);
            const float sx = __shfl(k_sx, ks), sy = __shfl(k_sy, ks), sz = __shfl(k_sz, ks);
            if (k < 27 && p < cnt) {
                const int src = (k == 0) ? perm : p;          // k==0 only in lanes 0..NSLOT-1
                const float* cell = disk + (int64_t)idx * 3 * nm;
                const float vx = cell[src] + sx;
                const float vy = cell[nm + src] + sy;
                const float vz = cell[2 * nm + src] + sz;
                xs[base + p] = vx;
                ys[base + p] = vy;
                zs[base + p] = vz;
            }
        }
    }

    // cell centre for out_of_bound (subsweep.h:73-88): c*w - L/2 + w/2 in float
    const float hw = g.w / 2.0f;
    const float cxf = (float)x * g.w - g.Lx / 2.0f + hw;
    const float cyf = (float)y * g.w - g.Ly / 2.0f + hw;
    const float czf = (float)(g.z0 + zl) * g.w - g.Lz / 2.0f + hw;
    const double beta_d = (double)g.beta;

    int64_t de_fix = 0;
    int n_acc = 0, n_ev = 0;
    int i = 0;
    for (int m0 = 0; m0 < g.n_moves; m0 += kWave) {
        // per-move random numbers, one move per lane (make_move's curand_normal x3 and
        // accept_move's curand_uniform, subsweep.h:60-71,212)
        float G0 = 0.0f, G1 = 0.0f, G2 = 0.0f;
        double T = 0.0;
        const int mm = m0 + lane;
        if (mm < g.n_moves) {
            pmc_u32x4 wm = pmc_philox4x32_10((uint32_t)mm, id, sweep, PMC_TAG_MOVE, k0, k1);
            pmc_move_normals(wm, &G0, &G1, &G2);
            pmc_u32x4 wa = pmc_philox4x32_10((uint32_t)mm, id, sweep, PMC_TAG_ACCEPT, k0, k1);
            T = pmc_accept_threshold(wa);
        }
        const uint64_t Tb = __builtin_bit_cast(uint64_t, T);
        const int Tlo = (int)(uint32_t)Tb, Thi = (int)(uint32_t)(Tb >> 32);
        const int mend = (g.n_moves - m0) < kWave ? (g.n_moves - m0) : kWave;
        for (int ml = 0; ml < mend; ++ml) {
            const float g0 = as_f(__builtin_amdgcn_readlane(as_i(G0), ml));
            const float g1 = as_f(__builtin_amdgcn_readlane(as_i(G1), ml));
            const float g2 = as_f(__builtin_amdgcn_readlane(as_i(G2), ml));
            const uint32_t tl = (uint32_t)__builtin_amdgcn_readlane(Tlo, ml);
            const uint32_t th = (uint32_t)__builtin_amdgcn_readlane(Thi, ml);
            const double Tm = __builtin_bit_cast(double, ((uint64_t)th << 32) | tl);
            const float xi = xs[i], yi = ys[i], zi = zs[i];
            const float px = xi + g0 * g.sigma;
            const float py = yi + g1 * g.sigma;
            const float pz = zi + g2 * g.sigma;
            const float ddx = px - cxf, ddy = py - cyf, ddz = pz - czf;
            const bool out = (ddx > hw) || (ddx < -hw) || (ddy > hw) || (ddy < -hw) || (ddz > hw) ||
                             (ddz < -hw);
            if (!out) {
                ++n_ev;
                float acc = 0.0f;
                for (int j0 = 0; j0 < S; j0 += kWave) {
                    const int j = j0 + lane;
                    const bool valid = (j < S) && (j != i);
                    const int jr = j < S ? j : 0;
                    const float xj = xs[jr], yj = ys[jr], zj = zs[jr];
                    const float eo = pmc_lj_from_r2(pmc_r2(xi - xj, yi - yj, zi - zj), g.rc2);
                    const float en = pmc_lj_from_r2(pmc_r2(px - xj, py - yj, pz - zj), g.rc2);
                    const float dd = en - eo;
                    acc = acc + (valid ? dd : 0.0f);
                }
                const float dE = wave_sum_fixed_order(acc);
                if (beta_d * (double)dE < Tm) {                 // accept_move, subsweep.h:209-216
                    if (lane == 0) { xs[i] = px; ys[i] = py; zs[i] = pz; }
                    ++n_acc;
                    de_fix += pmc_to_fixed((double)dE);
                }
            }
            i += 1;
            if (i >= n_own) i = 0;
        }
    }

    // ---- write back the own cell in shuffled order (cpy_D_sh_to_Disk, subsweep.h:29-36) ----
    if (lane < n_own) {
        float* cell = disk + c * 3 * nm;
        cell[lane] = xs[lane];
        cell[nm + lane] = ys[lane];
        cell[2 * nm + lane] = zs[lane];
    }
    if (lane == 0) {
        const int slot = (int)(t & (kStatSlots - 1));
        atomicAdd(&stats[0 * kStatSlots + slot], (unsigned long long)de_fix);
        atomicAdd(&stats[1 * kStatSlots + slot], (unsigned long long)n_acc);
        atomicAdd(&stats[2 * kStatSlots + slot], (unsigned long long)g.n_moves);
        atomicAdd(&stats[3 * kStatSlots + slot], (unsigned long long)n_ev);
    }
}

// ------------------------------------------------------------------------------------------
// shiftCells: NSLOT lanes per cell, ballot compaction (shiftCells.h:28-144; float s of the fixed
// copy CUDA-Parallel-MC/CUDA-Parallel-MC/shiftCells.h:23-112).  Double-buffered.
// ------------------------------------------------------------------------------------------
template <int NSLOT>
__global__ __launch_bounds__(256) void k_shift(DevGeom g, const float* __restrict__ din,
                                               const int16_t* __restrict__ nin, float* __restrict__ dout,
                                               int16_t* __restrict__ nout, int f, float d,
                                               uint32_t* __restrict__ flags) {
    constexpr int CPB = 256 / NSLOT;
    const int lane = threadIdx.x & (kWave - 1);
    const int p = threadIdx.x & (NSLOT - 1);
    const int64_t t = (int64_t)blockIdx.x * CPB + threadIdx.x / NSLOT;
    const int64_t total = (int64_t)g.cps_x * g.cps_y * g.nz_local;
    const bool live = t < total;
    const int nm = g.nmax;
    const float w = g.w;

    int x = 0, y = 0, zl = 0;
    if (live) {
        x = (int)(t % g.cps_x);
        y = (int)((t / g.cps_x) % g.cps_y);
        zl = (int)(t / ((int64_t)g.cps_x * g.cps_y));
    }
    const int cps_f = f == 0 ? g.cps_x : (f == 1 ? g.cps_y : g.cps_z);
    const float Lf = f == 0 ? g.Lx : (f == 1 ? g.Ly : g.Lz);
    const int dir = (d <= 0) ? -1 : 1;                     // shiftCells.h:46-53
    const float s = w * (float)dir;
    const int cidf = f == 0 ? x : (f == 1 ? y : g.z0 + zl);
    const float offset = (float)cidf * w - Lf / 2.0f;     // :55
    int nbg = cidf + dir;
    if (nbg < 0) nbg = cps_f - 1; else if (nbg >= cps_f) nbg = 0;
    int nx = x, ny = y, nz = zl;
    if (f == 0) nx = nbg; else if (f == 1) ny = nbg; else nz = g.halo ? zl + dir : nbg;
    const float offset_nb = (float)nbg * w - Lf / 2.0f;
    const int64_t c = sidx(g, x, y, zl);
    const int64_t cnb = sidx(g, nx, ny, nz);

    int ncur = 0, nnb = 0;
    if (live) { ncur = nin[c]; nnb = nin[cnb]; }
    float D = 0.0f, Dn = 0.0f;
    bool keep = false, take = false;
    if (p < ncur) {
        D = (din[c * 3 * nm + f * nm + p] - offset) - d;   // shortDisk - d
        keep = D > 0 && D <= w;
    }
    if (p < nnb) {
        Dn = (din[cnb * 3 * nm + f * nm + p] - offset_nb) - d;
        take = !(Dn > 0 && Dn <= w);
    }
    const unsigned long long bk = __ballot(keep);
    const unsigned long long bt = __ballot(take);
    const int gsh = lane & ~(NSLOT - 1);
    const unsigned long long gmask = NSLOT == 64 ? ~0ull : ((1ull << NSLOT) - 1ull);
    const unsigned long long km = (bk >> gsh) & gmask;
    const unsigned long long tm = (bt >> gsh) & gmask;
    const unsigned long long below = (1ull << p) - 1ull;
    const int nk = __popcll(km);
    const int nnew = nk + __popcll(tm);
    if (keep) {
        const int dst = __popcll(km & below);
        if (dst < nm) {
#pragma unroll
            for (int dim = 0; dim < 3; ++dim)
                dout[c * 3 * nm + dim * nm + dst] = (dim == f) ? D + offset : din[c * 3 * nm + dim * nm + p];
        }
    }
    if (take) {
        const int dst = nk + __popcll(tm & below);
        if (dst < nm) {
#pragma unroll
            for (int dim = 0; dim < 3; ++dim)
                dout[c * 3 * nm + dim * nm + dst] =
                    (dim == f) ? ((Dn + offset) + s) : din[cnb * 3 * nm + dim * nm + p];
        }
    }
    if (live && p == 0) {
        nout[c] = (int16_t)(nnew > nm ? nm : nnew);
        if (nnew > nm) atomicOr(flags, 1u);
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
                               uint32_t* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_atoms) return;
    const int cx = bin_axis(r[i], g.cps_x, g.w);
    const int cy = bin_axis(r[i + n_atoms], g.cps_y, g.w);
    const int cz = bin_axis(r[i + 2 * n_atoms], g.cps_z, g.w);
    if (cx < 0 || cy < 0 || cz < 0 || cz < g.z0 || cz >= g.z0 + g.nz_local) {
        atomicOr(flags, 4u);
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
                              float* __restrict__ disk, int16_t* __restrict__ n, int64_t cells) {
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
        disk[c * 3 * nm + k] = r[i];
        disk[c * 3 * nm + nm + k] = r[i + n_atoms];
        disk[c * 3 * nm + 2 * nm + k] = r[i + 2 * n_atoms];
    }
    n[c] = (int16_t)cnt;
}

// ------------------------------------------------------------------------------------------
// total energy (calc_energy, kernel.cu:452-470) as a cell-list sum, fixed-point per pair
// ------------------------------------------------------------------------------------------
template <int NSLOT>
__global__ __launch_bounds__(256) void k_energy(DevGeom g, const float* __restrict__ disk,
                                                const int16_t* __restrict__ ncnt,
                                                unsigned long long* __restrict__ acc) {
    constexpr int CPB = 256 / NSLOT;
    const int p = threadIdx.x & (NSLOT - 1);
    const int64_t t = (int64_t)blockIdx.x * CPB + threadIdx.x / NSLOT;
    const int64_t total = (int64_t)g.cps_x * g.cps_y * g.nz_local;
    long long sum = 0;
    if (t < total) {
        const int nm = g.nmax;
        const int x = (int)(t % g.cps_x), y = (int)((t / g.cps_x) % g.cps_y);
        const int zl = (int)(t / ((int64_t)g.cps_x * g.cps_y));
        const int64_t c = sidx(g, x, y, zl);
        if (p < ncnt[c]) {
            const float xi = disk[c * 3 * nm + p], yi = disk[c * 3 * nm + nm + p], zi = disk[c * 3 * nm + 2 * nm + p];
            for (int k = 0; k < 27; ++k) {
                const int hx = k / 9, hy = (k / 3) % 3, hz = k % 3;
                const int dx = hx == 0 ? 0 : (hx == 1 ? -1 : 1);
                const int dy = hy == 0 ? 0 : (hy == 1 ? -1 : 1);
                const int dz = hz == 0 ? 0 : (hz == 1 ? -1 : 1);
                int nx = x + dx, ny = y + dy;
                float sx = 0.0f, sy = 0.0f, sz = 0.0f;
                if (nx < 0) { nx += g.cps_x; sx = -g.Lx; } else if (nx >= g.cps_x) { nx -= g.cps_x; sx = g.Lx; }
                if (ny < 0) { ny += g.cps_y; sy = -g.Ly; } else if (ny >= g.cps_y) { ny -= g.cps_y; sy = g.Ly; }
                const int zg = g.z0 + zl + dz;
                if (zg < 0) sz = -g.Lz; else if (zg >= g.cps_z) sz = g.Lz;
                const int nzl = g.halo ? zl + dz : (zl + dz + g.cps_z) % g.cps_z;
                const int64_t cb = sidx(g, nx, ny, nzl);
                const int cnt = ncnt[cb];
                for (int q = 0; q < cnt; ++q) {
                    if (k == 0 && q == p) continue;
                    const float xj = disk[cb * 3 * nm + q] + sx;
                    const float yj = disk[cb * 3 * nm + nm + q] + sy;
                    const float zj = disk[cb * 3 * nm + 2 * nm + q] + sz;
                    sum += pmc_to_fixed((double)pmc_lj_from_r2(pmc_r2(xi - xj, yi - yj, zi - zj), g.rc2));
                }
            }
        }
    }
    // wave sum (int64, exact in any order), one atomic per wave
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(&acc[blockIdx.x & (kStatSlots - 1)], (unsigned long long)sum);
}

// ------------------------------------------------------------------------------------------
// self-test of the deterministic math on the device (compared bitwise with the host oracle)
// ------------------------------------------------------------------------------------------
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
    out_d[2 * i + 0] = pmc_accept_threshold(w);
    out_d[2 * i + 1] = (double)pmc_to_fixed((double)out_f[4 * i + 3]);
}

}  // namespace

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
hipError_t launch_subsweep(const DevGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz,
                           uint32_t sweep, unsigned long long* stats, hipStream_t st) {
    const int64_t total = (int64_t)(g.cps_x / 2) * (g.cps_y / 2) * (g.nz_local / 2);
    const int64_t blocks = (total + kSubWaves - 1) / kSubWaves;
    const size_t lds = sizeof(float) * 3 * 27 * (size_t)g.nmax * kSubWaves;
    dim3 grid((unsigned)blocks), block(kWave * kSubWaves);
    switch (g.nslot) {
        case 8: hipLaunchKernelGGL(k_subsweep<8>, grid, block, lds, st, g, disk, n, ox, oy, oz, sweep, stats); break;
        case 16: hipLaunchKernelGGL(k_subsweep<16>, grid, block, lds, st, g, disk, n, ox, oy, oz, sweep, stats); break;
        case 32: hipLaunchKernelGGL(k_subsweep<32>, grid, block, lds, st, g, disk, n, ox, oy, oz, sweep, stats); break;
        default: hipLaunchKernelGGL(k_subsweep<64>, grid, block, lds, st, g, disk, n, ox, oy, oz, sweep, stats); break;
    }
    return hipGetLastError();
}

hipError_t launch_shift(const DevGeom& g, const float* din, const int16_t* nin, float* dout,
                        int16_t* nout, int f, float d, uint32_t* flags, hipStream_t st) {
    const int64_t total = (int64_t)g.cps_x * g.cps_y * g.nz_local;
    const int cpb = 256 / g.nslot;
    dim3 grid((unsigned)((total + cpb - 1) / cpb)), block(256);
    switch (g.nslot) {
        case 8: hipLaunchKernelGGL(k_shift<8>, grid, block, 0, st, g, din, nin, dout, nout, f, d, flags); break;
        case 16: hipLaunchKernelGGL(k_shift<16>, grid, block, 0, st, g, din, nin, dout, nout, f, d, flags); break;
        case 32: hipLaunchKernelGGL(k_shift<32>, grid, block, 0, st, g, din, nin, dout, nout, f, d, flags); break;
        default: hipLaunchKernelGGL(k_shift<64>, grid, block, 0, st, g, din, nin, dout, nout, f, d, flags); break;
    }
    return hipGetLastError();
}

hipError_t launch_init_r(const DevGeom& g, int64_t n_atoms, int64_t n_cube, float* r, hipStream_t st) {
    if (n_atoms <= 0) return hipSuccess;
    dim3 grid((unsigned)((n_atoms + 255) / 256)), block(256);
    hipLaunchKernelGGL(k_init_r, grid, block, 0, st, g, n_atoms, n_cube, r);
    return hipGetLastError();
}

hipError_t launch_assign(const DevGeom& g, const float* r, int64_t n_atoms, float* disk, int16_t* n,
                         int32_t* tmp_cnt, int32_t* tmp_idx, uint32_t* flags, hipStream_t st) {
    const int64_t cells = (int64_t)g.cps_x * g.cps_y * (g.nz_local + 2 * g.halo);
    hipError_t e = hipMemsetAsync(tmp_cnt, 0, sizeof(int32_t) * (size_t)cells, st);
    if (e != hipSuccess) return e;
    if (n_atoms > 0) {
        dim3 grid((unsigned)((n_atoms + 255) / 256)), block(256);
        hipLaunchKernelGGL(k_assign_count, grid, block, 0, st, g, r, n_atoms, tmp_cnt, tmp_idx, flags);
    }
    dim3 grid2((unsigned)((cells + 255) / 256)), block2(256);
    hipLaunchKernelGGL(k_assign_fill, grid2, block2, 0, st, g, r, n_atoms, tmp_cnt, tmp_idx, disk, n, cells);
    return hipGetLastError();
}

hipError_t launch_energy(const DevGeom& g, const float* disk, const int16_t* n,
                         unsigned long long* acc, hipStream_t st) {
    const int64_t total = (int64_t)g.cps_x * g.cps_y * g.nz_local;
    const int cpb = 256 / g.nslot;
    dim3 grid((unsigned)((total + cpb - 1) / cpb)), block(256);
    switch (g.nslot) {
        case 8: hipLaunchKernelGGL(k_energy<8>, grid, block, 0, st, g, disk, n, acc); break;
        case 16: hipLaunchKernelGGL(k_energy<16>, grid, block, 0, st, g, disk, n, acc); break;
        case 32: hipLaunchKernelGGL(k_energy<32>, grid, block, 0, st, g, disk, n, acc); break;
        default: hipLaunchKernelGGL(k_energy<64>, grid, block, 0, st, g, disk, n, acc); break;
    }
    return hipGetLastError();
}

hipError_t launch_selftest(const uint32_t* words, int count, float* out_f, double* out_d, float rc2,
                           hipStream_t st) {
    dim3 grid((unsigned)((count + 255) / 256)), block(256);
    hipLaunchKernelGGL(k_selftest, grid, block, 0, st, words, count, out_f, out_d, rc2);
    return hipGetLastError();
}

}  // namespace pmc
