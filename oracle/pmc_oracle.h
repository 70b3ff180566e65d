/*
 * pmc_oracle.h -- CPU oracle for the checkerboard Metropolis subsweep + shiftCells hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library, and only as the checker / the timed CPU baseline -- never as a
 * product code path.  It is a plain-C, sequential restatement (optionally OpenMP over the
 * independent cells of one colour) of the reference algorithm as specified in SURVEY.md
 * Appendix A ("corrected mode"); each function cites the reference lines it follows.
 *
 * Parity pinning: see oracle/README.md and DESIGN.md section "Oracle".  The reference cannot
 * be built here (CUDA + cuRAND absent; building it would need stand-in headers, which this
 * project does not write), so the oracle is pinned by the reference's own data file
 * CUDA-Parallel-MC/CUDA-Parallel-MC/dumpR3.txt (lattice + energy function), by the lattice
 * energies derived from its definitions, by published Philox KATs and by statistical known
 * answers of <E> from an independent textbook Metropolis code (tools/textbook_mc.c,
 * tests/golden/known_answers.json: N=64 and N=305 particles in L=10, the configs' density).  The cuRAND XORWOW trajectory of the
 * reference is intentionally not reproduced (parity unpinned for the exact stream).
 */
#ifndef PMC_ORACLE_H
#define PMC_ORACLE_H

#include <stdint.h>
#include "../include/pmc.h"

#ifdef __cplusplus
extern "C" {
#endif

int orc_params_check(pmc_params* p);                 /* normalise defaults, validate */
int64_t orc_storage_cells(const pmc_params* p);
float orc_cutoff_r2(float w);
int orc_set_threads(int nthreads);                    /* 0 -> serial */

/* init_r (start.cu:47-58, kernel.cu:78-89) */
int orc_init_r(const pmc_params* p, int64_t n_atoms, float* r);
/* assign (start.cu:87-146) */
int orc_assign(const pmc_params* p, const float* r, int64_t n_atoms, float* disk, int16_t* n);
/* subsweep_kernel (subsweep.h:240-300) -- one colour phase */
void orc_subsweep(const pmc_params* p, float* disk, const int16_t* n, int ox, int oy, int oz,
                  uint32_t sweep, pmc_stats* st);
void orc_subsweep_range(const pmc_params* p, float* disk, const int16_t* n, int ox, int oy, int oz,
                        uint32_t sweep, int zl_begin, int zl_end, pmc_stats* st);
/* shiftCells (CUDA-Parallel-MC/CUDA-Parallel-MC/shiftCells.h:23-112) -- returns overflow count */
int orc_shift_cells(const pmc_params* p, const float* din, const int16_t* nin, float* dout,
                    int16_t* nout, int f, float d);
/* over local planes [zl_begin, zl_end) (halo planes included); -1 for a range outside the storage
 * or, along z in a slab, one whose dir-neighbour plane is not stored */
int orc_shift_cells_planes(const pmc_params* p, const float* din, const int16_t* nin, float* dout,
                           int16_t* nout, int f, float d, int zl_begin, int zl_end);
/* calc_energy (kernel.cu:452-470) as a cell-list sum over owned cells */
double orc_energy(const pmc_params* p, const float* disk, const int16_t* n);
/* whole-box driver loop (start.cu:237-260): nsweeps sweeps from `first`; state ends in
 * (disk, n) -- scratch buffers of the same size are used for the shift ping-pong */
int orc_run(const pmc_params* p, float* disk, int16_t* n, float* sdisk, int16_t* sn,
            uint32_t first, int nsweeps, pmc_stats* st);

/* orc_run recording the cell-list energy after every `every`-th sweep (trace[nsweeps / every]) */
int orc_run_trace(const pmc_params* p, float* disk, int16_t* n, float* sdisk, int16_t* sn,
                  uint32_t first, int nsweeps, int every, double* trace, pmc_stats* st);

/* exported primitives for unit tests */
void orc_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
float orc_logf(float x);
float orc_recip(float x);
void orc_det_sincos_2pi(float u, float* s, float* c);
void orc_move_normals(const uint32_t w[4], float g[3]);
float orc_pair_energy(float dx, float dy, float dz, float rc2);
void orc_sweep_plan(uint64_t seed, uint32_t sweep, float w, int order[8], int* f, float* d);
void orc_sweep_plan_ex(uint64_t seed, uint32_t sweep, float w, uint32_t flags, int order[8], int* f, float* d);
int64_t orc_to_fixed(double e);
int64_t orc_to_fixed_f32(float f);

#ifdef __cplusplus
}
#endif
#endif
