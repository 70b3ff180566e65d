/*
 * pmc_oracle.c -- CPU oracle (TEST INFRASTRUCTURE ONLY; see pmc_oracle.h for the contract).
 *
 * Plain sequential C restatement of the corrected-mode algorithm.
 * Compiled with gcc -ffp-contract=off so every float/double operation is a single IEEE
 * operation in source order, identical to the HIP kernels built with the same flag.
 * OpenMP (orc_set_threads > 0) parallelises only over the independent cells of one colour
 * phase / of the shift; results are identical for any thread count.
 */
#include "pmc_oracle.h"
#include "../include/pmc_detmath.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static int g_threads = 0;

int orc_set_threads(int nthreads) {
    g_threads = nthreads < 0 ? 0 : nthreads;
    return g_threads;
}

/* ------------------------------------------------------------------------------------- */
/* parameters / geometry                                                                 */
/* ------------------------------------------------------------------------------------- */
int orc_params_check(pmc_params* p) {
    if (p->cps_y == 0) p->cps_y = p->cps_x;
    if (p->cps_z == 0) p->cps_z = p->cps_x;
    if (p->nz_local == 0) p->nz_local = p->cps_z;
    if (p->cps_x < 4 || p->cps_y < 4 || p->cps_z < 4) return PMC_ERR_ARG;
    if ((p->cps_x | p->cps_y | p->cps_z | p->nz_local | p->z0) & 1) return PMC_ERR_ARG;
    if (p->nmax < 1 || p->nmax > 64 || p->n_moves < 0) return PMC_ERR_ARG;
    if (p->halo != 0 && p->halo != 1) return PMC_ERR_ARG;
    if (p->flags & ~(PMC_FLAG_FULL_SHUFFLE | PMC_FLAG_QUIRKS)) return PMC_ERR_ARG;
    if (p->halo == 2 && (p->flags & (PMC_FLAG_QUIRK_R1 | PMC_FLAG_QUIRK_R2))) return PMC_ERR_ARG;
    if (!p->halo && (p->nz_local != p->cps_z || p->z0 != 0)) return PMC_ERR_ARG;
    if (p->z0 < 0 || p->z0 + p->nz_local > p->cps_z) return PMC_ERR_ARG;
    if (!(p->beta >= 0.0f) || isinf(p->beta)) return PMC_ERR_ARG;
    return PMC_OK;
}

int64_t orc_storage_cells(const pmc_params* p) {
    return (int64_t)p->cps_x * p->cps_y * (p->nz_local + 2 * p->halo);
}

float orc_cutoff_r2(float w) { return pmc_cutoff_r2(w); }

/* storage index of local cell (x, y, zl), zl in [-halo, nz_local-1+halo] */
static inline int64_t sidx(const pmc_params* p, int x, int y, int zl) {
    return (int64_t)x + (int64_t)p->cps_x * ((int64_t)y + (int64_t)p->cps_y * (zl + p->halo));
}

/* global cell id (RNG counter word), get_cell_index (subsweep.h:14-16) on global coords */
static inline uint32_t gid(const pmc_params* p, int x, int y, int zl) {
    return (uint32_t)x + (uint32_t)p->cps_x * ((uint32_t)y + (uint32_t)p->cps_y * (uint32_t)(p->z0 + zl));
}

typedef struct { int64_t idx; float sx, sy, sz; } nbref;

/* neighbour (x+dx, y+dy, zl+dz) with its periodic image shift.  apply_PBC (subsweep.h:139-151)
 * subtracts/adds L per pair when |other-the| > 2w; for cells (CPS >= 4) that is the image of
 * the whole neighbour cell, applied here once per staged cell: staged = x + (+-L or 0). */
static inline nbref nb_of(const pmc_params* p, int x, int y, int zl, int dx, int dy, int dz) {
    float Lx = (float)p->cps_x * p->w, Ly = (float)p->cps_y * p->w, Lz = (float)p->cps_z * p->w;
    nbref r;
    int nx = x + dx, ny = y + dy;
    r.sx = 0.0f; r.sy = 0.0f; r.sz = 0.0f;
    if (nx < 0) { nx += p->cps_x; r.sx = -Lx; } else if (nx >= p->cps_x) { nx -= p->cps_x; r.sx = Lx; }
    if (ny < 0) { ny += p->cps_y; r.sy = -Ly; } else if (ny >= p->cps_y) { ny -= p->cps_y; r.sy = Ly; }
    int zg = p->z0 + zl + dz;
    if (zg < 0) r.sz = -Lz; else if (zg >= p->cps_z) r.sz = Lz;
    int nzl;
    if (p->halo) nzl = zl + dz;
    else nzl = (zl + dz + p->cps_z) % p->cps_z;
    r.idx = sidx(p, nx, ny, nzl);
    return r;
}

/* the 26 neighbour offsets in get_neighbors order (subsweep.h:119-137): x slowest over
 * {0,-1,+1}, then y, then z, skipping (0,0,0); the own cell is staged first (kernel.cu:241-278) */
static void stencil_offsets(int off[27][3]) {
    static const int h[3] = {0, -1, 1};
    int k = 0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            for (int l = 0; l < 3; ++l) {
                off[k][0] = h[i]; off[k][1] = h[j]; off[k][2] = h[l];
                ++k;
            }
    /* k == 27 and entry 0 is (0,0,0) */
}

/* ------------------------------------------------------------------------------------- */
/* init_r / assign                                                                       */
/* ------------------------------------------------------------------------------------- */
static int64_t icbrt_ceil(int64_t n) {
    int64_t k = 0;
    while (k * k * k < n) ++k;
    return k;
}

int orc_init_r(const pmc_params* p, int64_t n_atoms, float* r) {
    /* init_r (start.cu:47-58) with the index < N guard of kernel.cu:83:
     * r = L/2.0 * (1.0 - float(2i+1)/N_cube), evaluated in double, stored as float. */
    int64_t nc = icbrt_ceil(n_atoms);
    float Lx = (float)p->cps_x * p->w, Ly = (float)p->cps_y * p->w, Lz = (float)p->cps_z * p->w;
    float Lzl = (float)p->nz_local * p->w;
    float zc = ((float)p->z0 * p->w - Lz / 2.0f) + Lzl / 2.0f;   /* 0 for the whole box */
    for (int64_t idx = 0; idx < n_atoms; ++idx) {
        int64_t ix = idx % nc, iy = (idx / nc) % nc, iz = idx / (nc * nc);
        double fx = (double)((float)(2 * ix + 1) / (float)nc);
        double fy = (double)((float)(2 * iy + 1) / (float)nc);
        double fz = (double)((float)(2 * iz + 1) / (float)nc);
        r[idx] = (float)((double)Lx / 2.0 * (1.0 - fx));
        r[idx + n_atoms] = (float)((double)Ly / 2.0 * (1.0 - fy));
        r[idx + 2 * n_atoms] = (float)((double)zc + (double)Lzl / 2.0 * (1.0 - fz));
    }
    return PMC_OK;
}

/* cell along one axis by the reference's half-open rule lb < x <= ub with
 * lb = c*w - L/2.0f (start.cu:129-134); -1 if outside (-L/2, L/2] */
static int bin_axis(float x, int cps, float w) {
    float L = (float)cps * w;
    int c = (int)((x + L / 2.0f) / w);
    if (c < 0) c = 0;
    if (c > cps - 1) c = cps - 1;
    for (int it = 0; it < 4; ++it) {
        float lb = (float)c * w - L / 2.0f;
        float ub = lb + w;
        if (x <= lb) { if (c == 0) return -1; --c; }
        else if (x > ub) { if (c == cps - 1) return -1; ++c; }
        else return c;
    }
    return -1;
}

int orc_assign(const pmc_params* p, const float* r, int64_t n_atoms, float* disk, int16_t* n) {
    int64_t cells = orc_storage_cells(p);
    int nm = p->nmax;
    int rc = PMC_OK;
    for (int64_t c = 0; c < cells; ++c) n[c] = 0;
    for (int64_t i = 0; i < n_atoms; ++i) {
        int cx = bin_axis(r[i], p->cps_x, p->w);
        int cy = bin_axis(r[i + n_atoms], p->cps_y, p->w);
        int cz = bin_axis(r[i + 2 * n_atoms], p->cps_z, p->w);
        if (cx < 0 || cy < 0 || cz < 0 || cz < p->z0 || cz >= p->z0 + p->nz_local) {
            rc = PMC_ERR_RANGE;
            continue;
        }
        int64_t c = sidx(p, cx, cy, cz - p->z0);
        int k = n[c];
        if (k >= nm) { rc = PMC_ERR_OVERFLOW; continue; }
        disk[c * 3 * nm + k] = r[i];
        disk[c * 3 * nm + nm + k] = r[i + n_atoms];
        disk[c * 3 * nm + 2 * nm + k] = r[i + 2 * n_atoms];
        n[c] = (int16_t)(k + 1);
    }
    return rc;
}

/* ------------------------------------------------------------------------------------- */
/* subsweep                                                                              */
/* ------------------------------------------------------------------------------------- */
static void subsweep_cell(const pmc_params* p, float* disk, const int16_t* n, int x, int y, int zl,
                          uint32_t sweep, float rc2, float* px_, float* py_, float* pz_,
                          int64_t* de, int64_t* acc, int64_t* tri, int64_t* ev) {
    const int nm = p->nmax;
    const int64_t c = sidx(p, x, y, zl);
    const int n_own = n[c];
    if (n_own == 0) return;                       /* subsweep.h:252-253 */
    const uint32_t id = gid(p, x, y, zl);
    const uint32_t k0 = (uint32_t)p->seed, k1 = (uint32_t)(p->seed >> 32);
    const float Lx = (float)p->cps_x * p->w, Ly = (float)p->cps_y * p->w, Lz = (float)p->cps_z * p->w;
    /* quirk R2 (curand_init(1234, id, 0) every launch, subsweep.h:256-259): the same numbers at every visit */
    if (p->flags & PMC_FLAG_QUIRK_R2) sweep = 0;

    /* shuffle (random_shuffle, subsweep.h:50-58; proper Fisher-Yates, fixes R1) */
    int perm[64];
    for (int s = 0; s < n_own; ++s) perm[s] = s;
    if (p->flags & PMC_FLAG_QUIRK_R1) {
        /* quirk R1: random_int is always 0 (subsweep.h:38-40), so slot i swaps with slot 0 for i = n-1
         * down to 0 -- the rotation slot l <- particle (l + 1) mod n */
        for (int s = 0; s < n_own; ++s) perm[s] = s + 1 < n_own ? s + 1 : 0;
    } else
    for (int i = n_own - 1; i > 0; --i) {
        /* slot i's word: word i & 3 of SHUFFLE call i >> 2 (RNG spec v8, include/pmc_detmath.h) */
        pmc_u32x4 w = pmc_philox4x32_10((uint32_t)(i >> 2), id, sweep, PMC_TAG_SHUFFLE, k0, k1);
        int j = (int)pmc_bounded(w.v[i & 3], (uint32_t)(i + 1));
        int t = perm[i]; perm[i] = perm[j]; perm[j] = t;
    }

    /* stage the own cell in shuffled order (cpy_to_Dsh, subsweep.h:18-27) into slots [0, n_own),
     * then the 26 neighbour cells (get_neighbors order, subsweep.h:119-137; global reads of
     * calculate_energy_in_neighbors :153-172 done once, Version II ldisk staging kernel.cu:269-278),
     * keeping only partners within the cutoff of the own cell's box (their pair energy is
     * otherwise exactly 0).  Spec v11: own cell first (v10 staged it after the neighbours). */
    for (int s = 0; s < n_own; ++s) {
        px_[s] = disk[c * 3 * nm + perm[s]] + 0.0f;
        py_[s] = disk[c * 3 * nm + nm + perm[s]] + 0.0f;
        pz_[s] = disk[c * 3 * nm + 2 * nm + perm[s]] + 0.0f;
    }
    int off[27][3];
    stencil_offsets(off);
    float lo[3], hi[3];
    pmc_cell_box(x, y, p->z0 + zl, p->w, Lx, Ly, Lz, lo, hi);
    const float rcf = pmc_filter_r2(rc2);
    int S = n_own;
    /* staging order (pmc_stage_split): slots [0, H) of every neighbour in stencil order, then
     * slots [H, n) of the neighbours holding more than H particles, in stencil order */
    const int H = pmc_stage_split(nm);
    for (int round = 0; round < 2; ++round) {
        for (int k = 1; k < 27; ++k) {
            nbref b = nb_of(p, x, y, zl, off[k][0], off[k][1], off[k][2]);
            int cnt = n[b.idx];
            const int q0 = round ? H : 0;
            const int q1 = round ? cnt : (cnt < H ? cnt : H);
            for (int q = q0; q < q1; ++q) {
                float vx = disk[b.idx * 3 * nm + q] + b.sx;
                float vy = disk[b.idx * 3 * nm + nm + q] + b.sy;
                float vz = disk[b.idx * 3 * nm + 2 * nm + q] + b.sz;
                if (pmc_box_d2(vx, vy, vz, lo, hi) <= rcf) {
                    px_[S] = vx; py_[S] = vy; pz_[S] = vz;
                    ++S;
                }
            }
        }
    }
    const int K = S;

    /* cell centre (out_of_bound, subsweep.h:73-88): c*w - L/2 + w/2 in float */
    const float hw = p->w / 2.0f;
    const float cxf = (float)x * p->w - Lx / 2.0f + hw;
    const float cyf = (float)y * p->w - Ly / 2.0f + hw;
    const float czf = (float)(p->z0 + zl) * p->w - Lz / 2.0f + hw;

    double de_cell = 0.0;
    int i = 0;
    for (int m = 0; m < p->n_moves; ++m) {
        /* make_move (subsweep.h:60-71): p = x + normal*sigma */
        pmc_u32x4 wm = pmc_philox4x32_10((uint32_t)m, id, sweep, PMC_TAG_MOVE, k0, k1);
        float g0, g1, g2;
        pmc_move_normals(wm, &g0, &g1, &g2);
        pmc_u32x4 wa = pmc_philox4x32_10((uint32_t)m, id, sweep, PMC_TAG_ACCEPT, k0, k1);
        float T = pmc_accept_threshold(wa);
        float xi = px_[i], yi = py_[i], zi = pz_[i];
        float qx = xi + g0 * p->sigma;
        float qy = yi + g1 * p->sigma;
        float qz = zi + g2 * p->sigma;
        ++*tri;
        float ddx = qx - cxf, ddy = qy - cyf, ddz = qz - czf;
        int out = (ddx > hw) || (ddx < -hw) || (ddy > hw) || (ddy < -hw) || (ddz > hw) || (ddz < -hw);
        if (!out) {
            ++*ev;
            /* energies (calculate_old/new_energy, subsweep.h:175-191): dE = sum over partners
             * k != i of e(new) - e(old).  Term list (the kernel's compaction, spec v6): for each
             * block of 64 staged partners (own cell first, neighbours after) append the new
             * terms with r2 <= rc2 in ascending k, then the old terms with r2 <= rc2 in
             * ascending k (pairs beyond the cutoff are exactly 0 and are not listed).  Term t is
             * summed by lane t%64 in ascending t as +u (new) / -u (old), u the quarter energy;
             * v = 4 * lane sum; dE = xor butterfly 1,2,...,32 over the 64 lanes. */
            float part[64];
            for (int l = 0; l < 64; ++l) part[l] = 0.0f;
            int t = 0;
            for (int base = 0; base < K; base += 64) {
                const int kend = base + 64 < K ? base + 64 : K;
                for (int pass = 0; pass < 2; ++pass) {
                    const float sx = pass ? xi : qx, sy = pass ? yi : qy, sz = pass ? zi : qz;
                    for (int k = base; k < kend; ++k) {
                        if (k == i) continue;
                        const float r2 = pmc_r2(sx - px_[k], sy - py_[k], sz - pz_[k]);
                        if (r2 <= rc2) {
                            part[t & 63] = part[t & 63] + pmc_lj4_signed(pass ? -r2 : r2);
                            ++t;
                        }
                    }
                }
            }
            float lane[64];
            for (int l = 0; l < 64; ++l) lane[l] = 4.0f * part[l];
            for (int mask = 1; mask < 64; mask <<= 1) {
                float t[64];
                for (int l = 0; l < 64; ++l) t[l] = lane[l] + lane[l ^ mask];
                for (int l = 0; l < 64; ++l) lane[l] = t[l];
            }
            const float dE = lane[0];
            /* accept_move (subsweep.h:209-216) as beta*dE < -log(u) */
            if ((double)p->beta * (double)dE < (double)T) {
                px_[i] = qx; py_[i] = qy; pz_[i] = qz;   /* :219-223 */
                ++*acc;
                de_cell = de_cell + (double)dE;
            }
        }
        i += 1;
        if (i >= n_own) i = 0;
    }
    *de += pmc_to_fixed(de_cell);
    /* cpy_D_sh_to_Disk (subsweep.h:29-36): write back in shuffled order */
    for (int s = 0; s < n_own; ++s) {
        disk[c * 3 * nm + s] = px_[s];
        disk[c * 3 * nm + nm + s] = py_[s];
        disk[c * 3 * nm + 2 * nm + s] = pz_[s];
    }
}

void orc_subsweep(const pmc_params* p, float* disk, const int16_t* n, int ox, int oy, int oz,
                  uint32_t sweep, pmc_stats* st) {
    orc_subsweep_range(p, disk, n, ox, oy, oz, sweep, 0, p->nz_local, st);
}

/* the cells of the colour in local planes [zl_begin, zl_end) */
void orc_subsweep_range(const pmc_params* p, float* disk, const int16_t* n, int ox, int oy, int oz,
                        uint32_t sweep, int zl_begin, int zl_end, pmc_stats* st) {
    const float rc2 = pmc_cutoff_r2(p->w);
    const int ncx = p->cps_x / 2, ncy = p->cps_y / 2;
    int cz0 = zl_begin - oz <= 0 ? 0 : (zl_begin - oz + 1) / 2;
    int cz1 = zl_end - oz <= 0 ? 0 : (zl_end - oz + 1) / 2;
    if (cz1 > p->nz_local / 2) cz1 = p->nz_local / 2;
    if (cz1 <= cz0) return;
    const int ncz = cz1 - cz0;
    const int64_t total = (int64_t)ncx * ncy * ncz;
    const int cap = 27 * p->nmax;
    int64_t de = 0, acc = 0, tri = 0, ev = 0;
#ifdef _OPENMP
#pragma omp parallel num_threads(g_threads > 0 ? g_threads : 1) if (g_threads > 0) \
    reduction(+ : de, acc, tri, ev)
#endif
    {
        float* buf = (float*)malloc(sizeof(float) * 3 * (size_t)cap);
        float *xs = buf, *ys = buf + cap, *zs = buf + 2 * cap;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
        for (int64_t t = 0; t < total; ++t) {
            int a = (int)(t % ncx), b = (int)((t / ncx) % ncy), cz = (int)(t / ((int64_t)ncx * ncy));
            subsweep_cell(p, disk, n, 2 * a + ox, 2 * b + oy, 2 * (cz0 + cz) + oz, sweep, rc2, xs, ys, zs,
                          &de, &acc, &tri, &ev);
        }
        free(buf);
    }
    if (st) {
        st->de_fixed += de; st->accepted += acc; st->trials += tri; st->evaluated += ev;
    }
}

/* ------------------------------------------------------------------------------------- */
/* shiftCells                                                                            */
/* ------------------------------------------------------------------------------------- */
int orc_shift_cells(const pmc_params* p, const float* din, const int16_t* nin, float* dout,
                    int16_t* nout, int f, float d) {
    return orc_shift_cells_planes(p, din, nin, dout, nout, f, d, 0, p->nz_local);
}

/* The same over local planes [zl_begin, zl_end); a slab's halo planes (-1, nz_local) take the
 * periodic global index of the plane they copy (the slab driver shifts the halo planes it can
 * compute from its own data, pmc_shift_slab). */
int orc_shift_cells_planes(const pmc_params* p, const float* din, const int16_t* nin, float* dout,
                           int16_t* nout, int f, float d, int zl_begin, int zl_end) {
    /* the planes must be stored, and along z in a slab each plane's dir-neighbour too (a halo
     * plane on the +dir side cannot be computed locally: it is received) -- found by the
     * sanitizer build (asan_main.c), which reads past the storage otherwise */
    if (f < 0 || f > 2 || zl_begin < -p->halo || zl_end > p->nz_local + p->halo || zl_end < zl_begin) return -1;
    if (f == 2 && p->halo) {
        const int dir = (d <= 0) ? -1 : 1;
        if (zl_begin + dir < -1 || zl_end - 1 + dir > p->nz_local) return -1;
    }
    const int nm = p->nmax;
    const float w = p->w;
    const int cps[3] = {p->cps_x, p->cps_y, p->cps_z};
    const float Lf = (float)cps[f] * w;
    const int dir = (d <= 0) ? -1 : 1;               /* VS shiftCells.h:38-44 */
    /* float s (VS copy :28, :83-85); quirk S1: the root copy's int s[3] (shiftCells.h:31,105) */
    const float s = (p->flags & PMC_FLAG_QUIRK_S1) ? (float)(int)(w * (float)dir) : w * (float)dir;
    const int64_t total = (int64_t)p->cps_x * p->cps_y * (zl_end - zl_begin);
    int over = 0;
#ifdef _OPENMP
#pragma omp parallel for num_threads(g_threads > 0 ? g_threads : 1) if (g_threads > 0) \
    reduction(+ : over) schedule(static)
#endif
    for (int64_t t = 0; t < total; ++t) {
        int x = (int)(t % p->cps_x), y = (int)((t / p->cps_x) % p->cps_y);
        int zl = zl_begin + (int)(t / ((int64_t)p->cps_x * p->cps_y));
        int cid[3] = {x, y, p->z0 + zl};
        if (cid[2] < 0) cid[2] += p->cps_z; else if (cid[2] >= p->cps_z) cid[2] -= p->cps_z;
        int64_t c = sidx(p, x, y, zl);
        float offset = (float)cid[f] * w - Lf / 2.0f;   /* VS :46 */
        /* neighbour in direction of f (VS :73-88) */
        int nb[3] = {x, y, zl};
        int nbg = cid[f] + dir;
        if (nbg < 0) nbg = cps[f] - 1; else if (nbg >= cps[f]) nbg = 0;
        if (f < 2) nb[f] = nbg;
        else nb[2] = p->halo ? zl + dir : nbg;
        int64_t cnb = sidx(p, nb[0], nb[1], nb[2]);
        float offset_nb = (float)nbg * w - Lf / 2.0f;
        int ncur = nin[c], nnb = nin[cnb];
        int nnew = 0;
        for (int i = 0; i < ncur; ++i) {                 /* VS :52-71 */
            float D = (din[c * 3 * nm + f * nm + i] - offset) - d;
            if (D > 0 && D <= w) {
                if (nnew < nm)
                    for (int dim = 0; dim < 3; ++dim)
                        dout[c * 3 * nm + dim * nm + nnew] =
                            (dim == f) ? D + offset : din[c * 3 * nm + dim * nm + i];
                ++nnew;
            }
        }
        for (int i = 0; i < nnb; ++i) {                  /* VS :90-102 */
            float D = (din[cnb * 3 * nm + f * nm + i] - offset_nb) - d;
            if (!(D > 0 && D <= w)) {
                if (nnew < nm)
                    for (int dim = 0; dim < 3; ++dim)
                        dout[c * 3 * nm + dim * nm + nnew] =
                            (dim == f) ? (D + offset) + s : din[cnb * 3 * nm + dim * nm + i];
                ++nnew;
            }
        }
        if (nnew > nm) { ++over; nnew = nm; }
        nout[c] = (int16_t)nnew;
    }
    return over;
}

/* ------------------------------------------------------------------------------------- */
/* energy                                                                                */
/* ------------------------------------------------------------------------------------- */
double orc_energy(const pmc_params* p, const float* disk, const int16_t* n) {
    const int nm = p->nmax;
    const float rc2 = pmc_cutoff_r2(p->w);
    int off[27][3];
    stencil_offsets(off);
    const int64_t total = (int64_t)p->cps_x * p->cps_y * p->nz_local;
    int64_t sum = 0;
#ifdef _OPENMP
#pragma omp parallel for num_threads(g_threads > 0 ? g_threads : 1) if (g_threads > 0) \
    reduction(+ : sum) schedule(static)
#endif
    for (int64_t t = 0; t < total; ++t) {
        int x = (int)(t % p->cps_x), y = (int)((t / p->cps_x) % p->cps_y);
        int zl = (int)(t / ((int64_t)p->cps_x * p->cps_y));
        int64_t c = sidx(p, x, y, zl);
        for (int i = 0; i < n[c]; ++i) {
            float xi = disk[c * 3 * nm + i], yi = disk[c * 3 * nm + nm + i], zi = disk[c * 3 * nm + 2 * nm + i];
            for (int k = 0; k < 27; ++k) {
                nbref b = nb_of(p, x, y, zl, off[k][0], off[k][1], off[k][2]);
                for (int q = 0; q < n[b.idx]; ++q) {
                    if (k == 0 && q == i) continue;
                    float xj = disk[b.idx * 3 * nm + q] + b.sx;
                    float yj = disk[b.idx * 3 * nm + nm + q] + b.sy;
                    float zj = disk[b.idx * 3 * nm + 2 * nm + q] + b.sz;
                    sum += pmc_to_fixed((double)pmc_lj_from_r2(pmc_r2(xi - xj, yi - yj, zi - zj), rc2));
                }
            }
        }
    }
    return (double)sum / PMC_FIX_SCALE * 0.5;
}

/* ------------------------------------------------------------------------------------- */
/* driver loop (start.cu:237-260)                                                        */
/* ------------------------------------------------------------------------------------- */
int orc_run(const pmc_params* p, float* disk, int16_t* n, float* sdisk, int16_t* sn,
            uint32_t first, int nsweeps, pmc_stats* st) {
    if (p->halo) return PMC_ERR_ARG;
    int64_t cells = orc_storage_cells(p);
    int over = 0;
    for (int k = 0; k < nsweeps; ++k) {
        uint32_t s = first + (uint32_t)k;
        pmc_sweep_plan_t plan = pmc_plan_for_sweep_ex(p->seed, s, p->w, p->flags);
        for (int c = 0; c < 8; ++c) {
            int o[3];
            pmc_colour_offset(plan.order[c], o);
            orc_subsweep(p, disk, n, o[0], o[1], o[2], s, st);
        }
        over += orc_shift_cells(p, disk, n, sdisk, sn, plan.f, plan.d);
        memcpy(disk, sdisk, sizeof(float) * 3 * (size_t)p->nmax * (size_t)cells);
        memcpy(n, sn, sizeof(int16_t) * (size_t)cells);
    }
    return over ? PMC_ERR_OVERFLOW : PMC_OK;
}

/* orc_run with the energy trace of kernel.cu:643,695 (calc_energy after every sweep there): the
 * cell-list energy after every `every`-th sweep into trace[nsweeps / every] -- one C call for the
 * statistical tests' long chains */
int orc_run_trace(const pmc_params* p, float* disk, int16_t* n, float* sdisk, int16_t* sn,
                  uint32_t first, int nsweeps, int every, double* trace, pmc_stats* st) {
    if (every < 1) return PMC_ERR_ARG;
    int rc = PMC_OK;
    for (int k = 0; k + every <= nsweeps; k += every) {
        const int r = orc_run(p, disk, n, sdisk, sn, first + (uint32_t)k, every, st);
        if (r) rc = r;
        trace[k / every] = orc_energy(p, disk, n);
    }
    return rc;
}

/* ------------------------------------------------------------------------------------- */
/* primitives for tests                                                                  */
/* ------------------------------------------------------------------------------------- */
void orc_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    pmc_u32x4 r = pmc_philox4x32_10(ctr[0], ctr[1], ctr[2], ctr[3], key[0], key[1]);
    for (int i = 0; i < 4; ++i) out[i] = r.v[i];
}
float orc_logf(float x) { return pmc_logf(x); }
float orc_recip(float x) { return pmc_recip(x); }
void orc_det_sincos_2pi(float u, float* s, float* c) { pmc_det_sincos_2pi(u, s, c); }
void orc_move_normals(const uint32_t w[4], float g[3]) {
    pmc_u32x4 v;
    for (int i = 0; i < 4; ++i) v.v[i] = w[i];
    pmc_move_normals(v, &g[0], &g[1], &g[2]);
}
float orc_pair_energy(float dx, float dy, float dz, float rc2) {
    return pmc_lj_from_r2(pmc_r2(dx, dy, dz), rc2);
}
void orc_sweep_plan(uint64_t seed, uint32_t sweep, float w, int order[8], int* f, float* d) {
    orc_sweep_plan_ex(seed, sweep, w, 0u, order, f, d);
}

void orc_sweep_plan_ex(uint64_t seed, uint32_t sweep, float w, uint32_t flags, int order[8], int* f, float* d) {
    pmc_sweep_plan_t pl = pmc_plan_for_sweep_ex(seed, sweep, w, flags);
    for (int i = 0; i < 8; ++i) order[i] = pl.order[i];
    *f = pl.f;
    *d = pl.d;
}
int64_t orc_to_fixed(double e) { return pmc_to_fixed(e); }
int64_t orc_to_fixed_f32(float f) { return pmc_to_fixed_f32(f); }
