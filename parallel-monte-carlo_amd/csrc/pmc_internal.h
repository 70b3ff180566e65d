// pmc_internal.h -- shared between the kernel TU (pmc_kernels.hip) and the host API TU
// (pmc_api.hip).  Not part of the public C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pmc.h"

namespace pmc {

constexpr int kWave = 64;          // CDNA wavefront
// Waves per subsweep workgroup.  One: each wave is its own workgroup (5 KiB of LDS), so a CU
// refills a retiring wave's slot at once instead of when all waves of its workgroup are done;
// measured 2% faster per phase than 4 (and 6% faster than 8) at 128^3 / 1e7 (tools/bench_ab.sh).
#ifndef PMC_SUBWAVES
#define PMC_SUBWAVES 1
#endif
constexpr int kSubWaves = PMC_SUBWAVES;
#ifndef PMC_STAT_SLOTS
#define PMC_STAT_SLOTS 1024
#endif
constexpr int kStatSlots = PMC_STAT_SLOTS;   // stats accumulator slots per counter (contention spread)
static_assert((kStatSlots & (kStatSlots - 1)) == 0, "stats slots: a power of two");
// subsweep LDS per wave for a partner capacity lcap: x, y, z rows of `stride` slots
// (stride = lcap rounded up to 64 with >= 32 slots of tail: the tail is the discard target of the
// staging stores and the "far" fill past the last partner), then a term list of 2*lcap + 64.
__host__ __device__ constexpr int subsweep_stride(int lcap) { return (lcap + 32 + 63) / 64 * 64; }
__host__ __device__ constexpr int lds_floats_per_wave(int lcap) { return 3 * subsweep_stride(lcap) + 2 * lcap + 64; }
#ifndef PMC_MAIN_CAP
#define PMC_MAIN_CAP 224
#endif
#ifndef PMC_MAIN_WAVES
#define PMC_MAIN_WAVES 8   // main launch: waves per SIMD the LDS slot and the register budget are sized for
#endif
constexpr int kMainCap = PMC_MAIN_CAP;   // main launch: lds_floats_per_wave(224) * 4 B = 5120 B (32 waves/CU)
constexpr int kMainWaves = PMC_MAIN_WAVES;
static_assert(lds_floats_per_wave(kMainCap) * 4 * 4 * kMainWaves <= 160 * 1024, "main-launch LDS per wave");
constexpr int kStatCounters = 4;    // de_fixed, accepted, trials, evaluated
// Stats layout.  PMC_STATS_LANES = 1: slot-major, the 4 counters of a slot adjacent (32 B), so a
// cell's four counter adds are ONE wave instruction on lanes 0-3 (one 32-B memory-side atomic
// request instead of four single-lane ones).  0: counter-major, one single-lane atomic per counter.
#ifndef PMC_STATS_LANES
#define PMC_STATS_LANES 1
#endif
__host__ __device__ constexpr int stat_index(int counter, int slot) {
    return PMC_STATS_LANES ? slot * kStatCounters + counter : counter * kStatSlots + slot;
}
// Cell layout of the context's state buffers (disk): cell c holds 3*nmax floats at c*3*nmax in both
// layouts; slot s of dimension d sits at
//   PMC_AOS = 0: d*nmax + s  -- the reference's rows x[nmax], y[nmax], z[nmax] (start.cu:188);
//   PMC_AOS = 1: 3*s + d     -- x, y, z per slot: a cell's occupied slots are one contiguous run
//                               (4.8 particles = 58 B: one 64-B line instead of parts of three rows).
// The ABI's reference-layout buffers (pmc_copy_in/out, pmc_subsweep, pmc_shift_cells, pmc_assign)
// are converted at the boundary (launch_relayout); the context's own state is always this layout.
#ifndef PMC_AOS
#define PMC_AOS 1
#endif
__host__ __device__ constexpr uint32_t lay_dim(int nm) { return PMC_AOS ? 1u : (uint32_t)nm; }   // between dimensions
__host__ __device__ constexpr uint32_t lay_slot() { return PMC_AOS ? 3u : 1u; }                  // between slots
constexpr int kSmallSweeps = 32;   // k_sweep_small: sweep plans per launch (pmc_run_small checks each launch)
constexpr int kOvfHead = 2;        // ints of the subsweep overflow-queue header (pmc_kernels.hip)

// Unsigned division by an invariant d: n / d = (hi + ((n - hi) >> sh1)) >> sh2, hi = umulhi(n, mul)
// (Granlund & Montgomery 1994, round-up variant; exact for every 32-bit n).
struct UDivMagic {
    uint32_t mul, sh1, sh2;
};
inline UDivMagic make_udiv_magic(uint32_t d) {
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < d) ++l;                 // ceil(log2 d)
    UDivMagic m;
    m.mul = (uint32_t)((((1ull << l) - d) << 32) / d + 1);
    m.sh1 = l < 1 ? l : 1;
    m.sh2 = l > 1 ? l - 1 : 0;
    return m;
}

// Flattened kernel parameters (passed by value).
struct DevGeom {
    int cps_x, cps_y, cps_z, nz_local, z0, halo, nmax, n_moves;
    int nslot;                     // power of two >= nmax (lanes per cell in shift/energy)
    float w, beta, sigma, Lx, Ly, Lz, rc2;
    float rc2f;                    // staging filter threshold (pmc_filter_r2)
    float r2min;                   // PMC_R2_MIN (passed as data so the kernel keeps it in an SGPR)
    double inv_b4;                 // 1 / (4*(double)beta), 0 for beta == 0 (accept_bound's estimate)
    UDivMagic div_ncx, div_ncy;    // division by cps_x/2 and cps_y/2 (subsweep cell decode)
    UDivMagic div_cx, div_plane;   // division by cps_x and cps_x*cps_y (energy cell decode)
    uint32_t rk0[10], rk1[10];     // Philox round keys k + r*W (kernel arguments -> SGPRs, no key adds)
    uint32_t k0, k1;
};

// The host's copy: the kernel arguments plus what only the launchers read.  (The quirk bits select
// kernel instantiations; keeping them out of DevGeom keeps every kernel's argument block unchanged.)
struct HostGeom : DevGeom {
    uint32_t quirks = 0;           // PMC_FLAG_QUIRK_* of pmc_params.flags (0: the corrected semantics)
};

// Optional timing of one kernel launch: start/stop events carried by the dispatch packet itself
// (hipExtLaunchKernelGGL: no extra barrier packets between kernels, unlike hipEventRecord).
struct LaunchTiming {
    hipEvent_t start = nullptr, stop = nullptr;
};

// Launchers (pmc_kernels.hip).  All asynchronous on `st`.
// ovf: int[1 + cells_per_colour] scratch (overflow queue for the full-capacity fallback)
// only cells in local planes [zl_begin, zl_end) of the colour are visited
// solo: the launch has the GPU to itself (no concurrent chain): a short one ends in single-cell waves
hipError_t launch_subsweep(const HostGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz,
                           uint32_t sweep, unsigned long long* stats, int* ovf, int zl_begin, int zl_end,
                           hipStream_t st, const LaunchTiming* tm = nullptr, bool solo = false);
// the slab driver's boundary planes: full LDS capacity (no overflow queue), every written-back row
// also stored to `mirror` (mirror_mode 0: packed colour rows ta + tb*cps_x/2, 1: plane rows;
// mirror may be null)
hipError_t launch_subsweep_boundary(const HostGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz,
                                    uint32_t sweep, unsigned long long* stats, int* ovf, int zl_begin, int zl_end,
                                    float* mirror, int mirror_mode, hipStream_t st,
                                    const LaunchTiming* tm = nullptr);
// one colour plane zl of the storage, halo planes included (the two-plane-halo slab schedule
// visits the neighbour's boundary plane redundantly; its cell ids and centres are the owner's):
// the boundary path, one cell per wave + fallback on `ovf`
hipError_t launch_subsweep_plane(const HostGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz,
                                 uint32_t sweep, unsigned long long* stats, int* ovf, int zl, hipStream_t st,
                                 const LaunchTiming* tm = nullptr);
// two colour planes zl0 < zl1 of one parity in ONE launch (the two-plane-halo schedule's first run:
// the boundary plane and the halo plane at the opposite face); plane zl0's counters to stats0, zl1's
// to stats1
hipError_t launch_subsweep_planes2(const DevGeom& g, float* disk, const int16_t* n, int ox, int oy, int oz,
                                   uint32_t sweep, unsigned long long* stats0, unsigned long long* stats1, int* ovf,
                                   int zl0, int zl1, hipStream_t st, const LaunchTiming* tm = nullptr);
int subsweep_capacity(const DevGeom& g);
// whole sweeps of a small whole box in one launch on XCD 0 (k_sweep_small); bar: one unsigned of
// scratch; cur: the current buffer of the (disk, n) pairs; returns hipErrorInvalidValue when the box
// does not qualify (small_sweep_participants == 0)
int small_sweep_participants(const HostGeom& g);
hipError_t launch_sweep_small(const HostGeom& g, float* disk0, int16_t* n0, float* disk1, int16_t* n1, int cur,
                              unsigned long long* stats, uint32_t* flags, unsigned* bar, uint64_t seed,
                              uint32_t first, int count, uint32_t plan_flags, hipStream_t st);
hipError_t launch_shift(const HostGeom& g, const float* din, const int16_t* nin, float* dout,
                        int16_t* nout, int f, float d, uint32_t* flags, hipStream_t st,
                        const LaunchTiming* tm = nullptr);
// the same over local planes [zl_begin, zl_end), halo planes included (-halo .. nz_local+halo)
hipError_t launch_shift_planes(const HostGeom& g, const float* din, const int16_t* nin, float* dout,
                               int16_t* nout, int f, float d, uint32_t* flags, int zl_begin, int zl_end,
                               hipStream_t st, const LaunchTiming* tm);
hipError_t launch_init_r(const DevGeom& g, int64_t n_atoms, int64_t n_cube, float* r, hipStream_t st);
// ref_layout = 1: disk is a caller's buffer in the reference layout (pmc_assign); 0: the state layout
hipError_t launch_assign(const DevGeom& g, const float* r, int64_t n_atoms, float* disk, int16_t* n,
                         int32_t* tmp_cnt, int32_t* tmp_idx, uint32_t* flags, hipStream_t st, int clip = 0,
                         int ref_layout = 0);
// segq: int[1 + energy_segments(g)] scratch, zeroed on st before the call
size_t energy_segments(const DevGeom& g);
hipError_t launch_energy(const DevGeom& g, const float* disk, const int16_t* n,
                         unsigned long long* acc, int* segq, hipStream_t st);
// the cells of one colour of one plane: mode 0 plane -> packed buffer, 1 packed -> plane,
// 2 plane -> plane; (cps_x/2)*(cps_y/2)*3*nmax floats
hipError_t launch_colour_rows(const DevGeom& g, const float* src, float* dst, int colour, int mode, hipStream_t st);
// reference layout <-> the state layout (PMC_AOS) of `cells` cells: to_state = 1: ref -> state, 0: state ->
// ref (src != dst; a no-op copy when the layouts agree)
hipError_t launch_relayout(const float* src, float* dst, int64_t cells, int nmax, int to_state, hipStream_t st);
// rehearsal only: a one-wave kernel that occupies `st` for `us` microseconds (injected exchange delay)
hipError_t launch_spin(double us, hipStream_t st);
// pmc_hbm_probe: kind 0 streams `bytes` of src (reads only), 1 copies src -> dst; unroll 4 or 8
hipError_t launch_hbm_probe(int kind, int unroll, const void* src, void* dst, uint64_t bytes, uint32_t* sink,
                            int blocks, hipStream_t st);
// IPC halo transport (pmc_kernels.hip, pmc_slab_init_ipc): sequence flags and the pull copy
constexpr int kXferMax = 16;       // flags waited on / segments copied per launch (peers <= 16)
struct XferFlags {
    const uint64_t* flag[kXferMax];
    uint64_t target[kXferMax];     // wait until *flag[i] >= target[i]
    int n;
};
struct XferSeg {
    const void* src;
    void* dst;
    uint64_t bytes;
    int shift;                     // log2 of the copy unit (1..16 B): divides src, dst and bytes
};
struct XferCopy {
    XferSeg seg[kXferMax];
    int n;
};
// mine (may be null) := seq, then wait until every w.flag[i] >= w.target[i] (timeout: error flag 512)
hipError_t launch_xfer_flag(uint64_t* mine, uint64_t seq, const XferFlags& w, uint64_t timeout_ticks, uint32_t* err,
                            hipStream_t st);
// one exchange (two launches): *ready := seq and wait for w; then copy every segment, the last block
// storing *pulled = seq
hipError_t launch_xfer(const XferCopy& cp, const XferFlags& w, uint64_t* ready, uint64_t* pulled, uint64_t seq,
                       unsigned* done, uint64_t timeout_ticks, uint32_t* err, hipStream_t st);
hipError_t launch_selftest(const uint32_t* words, int count, float* out_f, double* out_d,
                           float rc2, hipStream_t st);

}  // namespace pmc
