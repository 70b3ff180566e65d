/*
 * asan_main.c -- sanitizer driver for the CPU oracle (TEST INFRASTRUCTURE ONLY; SURVEY.md 5:
 * "ASan/UBSan on the CPU oracle").  Built by `make -C oracle sanitize` with
 * -fsanitize=address,undefined and run by tests/test_oracle.py: whole-box sweeps with both colour
 * orders, a slab context (halo planes, plane-range subsweeps and shifts over halo planes), odd
 * rectangular boxes, nmax 8 (overflowing assign/shift must be reported, not written past the row),
 * the energy, and the exported primitives.  The reference's own undefined behaviour that motivates
 * it: __syncthreads in a divergent branch (subsweep.h:26,252-253) and dir[-1] / cid[-1] from
 * f = rand()%3 - 1 (start.cu:251 + shiftCells.h:45); the oracle must have none of its own.
 * Exit status 0 = clean (the sanitizers abort on the first finding).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pmc_oracle.h"

static pmc_params make(int cx, int cy, int cz, int nmax, uint32_t flags) {
    pmc_params p;
    memset(&p, 0, sizeof(p));
    p.cps_x = cx; p.cps_y = cy; p.cps_z = cz; p.nmax = nmax; p.n_moves = 10;
    p.w = 2.5f; p.beta = 0.3f; p.sigma = 0.5f; p.seed = 1234; p.flags = flags;
    return p;
}

static int whole_box(int cx, int cy, int cz, int nmax, int64_t atoms, int sweeps, uint32_t flags) {
    pmc_params p = make(cx, cy, cz, nmax, flags);
    if (orc_params_check(&p)) return 1;
    const int64_t cells = orc_storage_cells(&p);
    float* r = malloc(sizeof(float) * 3 * (size_t)atoms);
    float* disk = calloc((size_t)cells * 3 * (size_t)nmax, sizeof(float));
    float* sdisk = calloc((size_t)cells * 3 * (size_t)nmax, sizeof(float));
    int16_t* n = calloc((size_t)cells, sizeof(int16_t));
    int16_t* sn = calloc((size_t)cells, sizeof(int16_t));
    orc_init_r(&p, atoms, r);
    int rc = orc_assign(&p, r, atoms, disk, n);
    pmc_stats st;
    memset(&st, 0, sizeof(st));
    int over = 0;
    if (rc == 0) {
        double e0 = orc_energy(&p, disk, n);
        over = orc_run(&p, disk, n, sdisk, sn, 3, sweeps, &st);
        double e1 = orc_energy(&p, disk, n);
        printf("box %dx%dx%d nmax %d atoms %lld flags %u: E %.6f -> %.6f, accepted %lld / %lld, over %d\n", cx, cy,
               cz, nmax, (long long)atoms, flags, e0, e1, (long long)st.accepted, (long long)st.trials, over);
    } else {
        printf("box %dx%dx%d nmax %d atoms %lld: assign rc %d (reported, nothing written past a row)\n", cx, cy, cz,
               nmax, (long long)atoms, rc);
    }
    free(r); free(disk); free(sdisk); free(n); free(sn);
    return 0;
}

static int slab(void) {
    /* rank 1 of a 2-slab 8x8x8 box: planes 4..7 owned, halo planes 3 and 0 (periodic) */
    pmc_params p = make(8, 8, 8, 16, 0);
    p.halo = 1; p.nz_local = 4; p.z0 = 4;
    if (orc_params_check(&p)) return 1;
    const int64_t cells = orc_storage_cells(&p);
    float* disk = calloc((size_t)cells * 3 * 16, sizeof(float));
    float* dout = calloc((size_t)cells * 3 * 16, sizeof(float));
    int16_t* n = calloc((size_t)cells, sizeof(int16_t));
    int16_t* nout = calloc((size_t)cells, sizeof(int16_t));
    /* fill every storage plane (halos too) from a whole-box lattice */
    pmc_params w = make(8, 8, 8, 16, 0);
    orc_params_check(&w);
    const int64_t wc = orc_storage_cells(&w);
    float* r = malloc(sizeof(float) * 3 * 1500);
    float* wd = calloc((size_t)wc * 3 * 16, sizeof(float));
    int16_t* wn = calloc((size_t)wc, sizeof(int16_t));
    orc_init_r(&w, 1500, r);
    if (orc_assign(&w, r, 1500, wd, wn)) return 1;
    const int64_t plane = 64;
    for (int zl = -1; zl <= 4; ++zl) {
        const int zg = (4 + zl + 8) % 8;
        memcpy(disk + (size_t)(zl + 1) * plane * 48, wd + (size_t)zg * plane * 48, sizeof(float) * plane * 48);
        memcpy(n + (size_t)(zl + 1) * plane, wn + (size_t)zg * plane, sizeof(int16_t) * plane);
    }
    pmc_stats st;
    memset(&st, 0, sizeof(st));
    for (int colour = 0; colour < 8; ++colour)
        orc_subsweep_range(&p, disk, n, colour / 4 % 2, colour / 2 % 2, colour % 2, 7, 0, 4, &st);
    int over = 0;
    for (int f = 0; f < 3; ++f)
        for (int sgn = -1; sgn <= 1; sgn += 2) {
            /* the planes pmc_shift_slab shifts locally: along x/y every stored plane, along z all but
             * the halo on the +dir side; the whole storage along z must be refused */
            const int z0 = (f == 2 && sgn < 0) ? 0 : -1, z1 = (f == 2 && sgn > 0) ? 4 : 5;
            over += orc_shift_cells_planes(&p, disk, n, dout, nout, f, 0.9f * sgn, z0, z1);
            if (f == 2 && orc_shift_cells_planes(&p, disk, n, dout, nout, f, 0.9f * sgn, -1, 5) != -1) return 1;
        }
    double e = orc_energy(&p, disk, n);
    printf("slab: accepted %lld / %lld, E %.6f, shift over %d\n", (long long)st.accepted, (long long)st.trials, e, over);
    free(disk); free(dout); free(n); free(nout); free(r); free(wd); free(wn);
    return 0;
}

int main(void) {
    int bad = 0;
    orc_set_threads(0);
    bad |= whole_box(8, 8, 8, 16, 2000, 4, 0);
    bad |= whole_box(8, 8, 8, 16, 2000, 4, 1);
    bad |= whole_box(10, 6, 14, 16, 2000, 3, 0);     /* odd colour counts */
    bad |= whole_box(4, 4, 4, 10, 64, 20, 0);        /* the reference's N = 64 box, nmax 10 */
    bad |= whole_box(4, 4, 4, 8, 600, 2, 0);         /* assign overflows nmax: reported */
    bad |= whole_box(6, 6, 6, 8, 1400, 10, 0);       /* crowded: shift overflow path */
    bad |= slab();
    uint32_t ctr[4] = {1, 2, 3, 4}, key[2] = {5, 6}, out[4];
    orc_philox(ctr, key, out);
    float g[3];
    orc_move_normals(out, g);
    int order[8], f;
    float d;
    orc_sweep_plan_ex(1234, 9, 2.5f, 0u, order, &f, &d);
    printf("primitives: %08x %f %f %f %d %f %lld %lld\n", out[0], g[0], g[1], g[2], f, d,
           (long long)orc_to_fixed(-3.25), (long long)orc_to_fixed_f32(1e-30f));
    printf(bad ? "FAIL\n" : "clean\n");
    return bad;
}
