// pmc_api.hip -- host side of the C ABI declared in include/pmc.h.
//
// Replaces the reference's host driver (start.cu:169-272 / kernel.cu:566-709): device
// allocation, kernel launches, the MC step loop and the energy/acceptance observables.  All work
// is asynchronous on the context stream; only the *_read / copy / synchronize calls block.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <cstring>
#include <string>
#include <unistd.h>
#include <utility>
#include <vector>

#include "pmc_internal.h"
#include "../../include/pmc_detmath.h"

using namespace pmc;

struct pmc_slab;   // multi-GPU slab driver state (pmc_slab_init)

struct pmc_ctx {
    pmc_slab* slab = nullptr;
    pmc_params P;
    HostGeom G;
    int64_t cells = 0;              // storage cells (incl. halo planes)
    float* disk[2] = {nullptr, nullptr};
    int16_t* n[2] = {nullptr, nullptr};
    bool own_state = false;
    int cur = 0;
    unsigned long long* stats = nullptr;   // kStatCounters * kStatSlots
    unsigned long long* eacc = nullptr;    // kStatSlots (energy)
    int* segq = nullptr;                   // energy: queue of row segments over the staging capacity
    uint32_t* flags = nullptr;
    int* ovf = nullptr;                    // subsweep overflow queue (1 + cells per colour)
    int* ovf_aux = nullptr;                // second queue: launches on a caller stream (pmc_phase_range_on)
    int* ovf_b = nullptr;                  // third queue: the slab driver's boundary chain
    int* ovf_aux2 = nullptr;               // fourth queue: the slab driver's third interior chain
    size_t ovf_bytes = 0;
    // two-plane halos: the shifted send planes (planes 0, 1 then nz-2, nz-1, with their counts)
    float* send_d = nullptr;
    int16_t* send_n = nullptr;
    // IPC halo transport (pmc_slab_ipc_handle / pmc_slab_init_ipc): sequence flags, reduction slots
    // (uncached device memory other rank processes map), and the exchange count -- monotonic over
    // the context's life, so a re-attached slab driver keeps agreeing with its peers' flags
    uint64_t* xflags = nullptr;
    int xflags_kind = 0;                   // 1 uncached, 2 fine-grained, 3 hipMalloc
    uint64_t xseq = 0;
    int32_t* tmp_cnt = nullptr;
    int32_t* tmp_idx = nullptr;
    float* d_r = nullptr;
    int64_t r_cap = 0;
    // reference-layout staging for the ABI's caller buffers and host copies (PMC_AOS: the state is
    // packed, the boundary converts; allocated on first use)
    float* conv[2] = {nullptr, nullptr};
    // whole-box sweeps in plane chains (enqueue_sweep): chains 1.. streams and overflow queues (chain 0:
    // the context stream and ovf), the chains' "previous run" events [chain][parity], and the context
    // stream's "sweep start" event
    hipStream_t hs[PMC_SWEEP_MAX_CHAINS - 1] = {};
    int* ovf_ch[PMC_SWEEP_MAX_CHAINS - 1] = {};
    hipEvent_t ev_c[PMC_SWEEP_MAX_CHAINS][2] = {};
    hipEvent_t ev_s = nullptr;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipGraphExec_t graph_exec = nullptr;
    // per-launch kernel timing (pmc_timing): dispatch-packet events, (start, stop) pairs in use
    bool timing = false;
    bool timing_paused = false;           // pmc_timing_pause: events off without collecting
    std::vector<hipEvent_t> tev;
    std::vector<int> tkind;                // 0 subsweep (interior / context stream), 1 shift, 2 subsweep (boundary / caller stream)
    std::vector<int64_t> tphase;           // colour phase of a timed launch split over plane chains (-1: none)
    int64_t phase_seq = 0;                 // next phase id (enqueue_sweep_chains)
    double span_ms = 0.0;                  // pmc_timing_kinds: summed spans of those phases (pmc_timing_phase_spans)
    int span_n = 0;
    uint32_t graph_first = 0;
    int graph_count = 0;
    int graph_cur = -1;
};

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return PMC_ERR_HIP;
}

#define PMC_HIP(call)                                   \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) return hip_fail(e_, #call); \
    } while (0)

int normalise(pmc_params* p) {
    if (p->cps_y == 0) p->cps_y = p->cps_x;
    if (p->cps_z == 0) p->cps_z = p->cps_x;
    if (p->nz_local == 0) p->nz_local = p->cps_z;
    if (p->cps_x < 4 || p->cps_y < 4 || p->cps_z < 4) return fail(PMC_ERR_ARG, "cells per side must be >= 4");
    if ((p->cps_x | p->cps_y | p->cps_z | p->nz_local | p->z0) & 1)
        return fail(PMC_ERR_ARG, "cells per side, nz_local and z0 must be even (checkerboard)");
    if (p->nmax < 1 || p->nmax > 64) return fail(PMC_ERR_ARG, "nmax must be in 1..64");
    if (p->n_moves < 0) return fail(PMC_ERR_ARG, "n_moves must be >= 0");
    if (p->halo < 0 || p->halo > 2) return fail(PMC_ERR_ARG, "halo must be 0, 1 or 2");
    if (p->halo == 2 && (p->flags & PMC_FLAG_FULL_SHUFFLE))
        return fail(PMC_ERR_ARG, "two-plane halos need the grouped colour order (two runs per sweep)");
    if (p->flags & ~(PMC_FLAG_FULL_SHUFFLE | PMC_FLAG_QUIRKS)) return fail(PMC_ERR_ARG, "unknown flags");
    if (p->halo == 2 && (p->flags & (PMC_FLAG_QUIRK_R1 | PMC_FLAG_QUIRK_R2)))
        return fail(PMC_ERR_ARG, "quirks R1/R2 run the full-capacity path, which two-plane halos do not use");
    if (!p->halo && (p->nz_local != p->cps_z || p->z0 != 0))
        return fail(PMC_ERR_ARG, "halo == 0 requires the whole box (nz_local == cps_z, z0 == 0)");
    if (p->z0 < 0 || p->z0 + p->nz_local > p->cps_z) return fail(PMC_ERR_ARG, "slab outside the box");
    if (!(p->w > 0.0f) || !(p->sigma >= 0.0f)) return fail(PMC_ERR_ARG, "w must be > 0, sigma >= 0");
    if (!(p->beta >= 0.0f) || std::isinf(p->beta)) return fail(PMC_ERR_ARG, "beta must be finite and >= 0");
    const int64_t cells = (int64_t)p->cps_x * p->cps_y * (p->nz_local + 2 * p->halo);
    if (cells * 3 * p->nmax >= ((int64_t)1 << 32)) return fail(PMC_ERR_ARG, "box too large (2^32 coordinate slots per context)");
    if ((int64_t)p->cps_x * p->cps_y * p->cps_z > 0xFFFFFFFFll) return fail(PMC_ERR_ARG, "more than 2^32 cells");
    if (cells >= ((int64_t)1 << 31)) return fail(PMC_ERR_ARG, "more than 2^31 storage cells");
    return PMC_OK;
}

HostGeom make_geom(const pmc_params& p) {
    HostGeom g;
    g.cps_x = p.cps_x; g.cps_y = p.cps_y; g.cps_z = p.cps_z;
    g.nz_local = p.nz_local; g.z0 = p.z0; g.halo = p.halo;
    g.nmax = p.nmax; g.n_moves = p.n_moves;
    g.nslot = 8;
    while (g.nslot < p.nmax) g.nslot <<= 1;
    g.w = p.w; g.beta = p.beta; g.sigma = p.sigma;
    g.Lx = (float)p.cps_x * p.w;
    g.Ly = (float)p.cps_y * p.w;
    g.Lz = (float)p.cps_z * p.w;
    g.rc2 = pmc_cutoff_r2(p.w);
    g.rc2f = pmc_filter_r2(g.rc2);
    g.r2min = PMC_R2_MIN;
    g.inv_b4 = p.beta > 0.0f ? 1.0 / (4.0 * (double)p.beta) : 0.0;   // the acceptance bound's estimate
    g.div_ncx = make_udiv_magic((uint32_t)(p.cps_x / 2));
    g.div_ncy = make_udiv_magic((uint32_t)(p.cps_y / 2));
    g.div_cx = make_udiv_magic((uint32_t)p.cps_x);
    g.div_plane = make_udiv_magic((uint32_t)p.cps_x * (uint32_t)p.cps_y);
    g.k0 = (uint32_t)p.seed;
    g.k1 = (uint32_t)(p.seed >> 32);
    g.quirks = p.flags & PMC_FLAG_QUIRKS;
    for (int r = 0; r < 10; ++r) {
        g.rk0[r] = g.k0 + (uint32_t)r * PMC_PHILOX_W0;
        g.rk1[r] = g.k1 + (uint32_t)r * PMC_PHILOX_W1;
    }
    return g;
}

int64_t icbrt_ceil(int64_t n) {
    int64_t k = (int64_t)std::cbrt((double)n);
    while (k > 0 && (k - 1) * (k - 1) * (k - 1) >= n) --k;
    while (k * k * k < n) ++k;
    return k;
}

size_t disk_bytes(const pmc_ctx* c) { return sizeof(float) * 3 * (size_t)c->P.nmax * (size_t)c->cells; }
size_t n_bytes(const pmc_ctx* c) { return sizeof(int16_t) * (size_t)c->cells; }

// a caller's device buffer that is one of the context's own state buffers (state layout already)
bool is_state_buffer(const pmc_ctx* c, const float* p) { return p == c->disk[0] || p == c->disk[1]; }

// staging buffer k (storage-sized, reference layout <-> state layout conversions)
hipError_t ensure_conv(pmc_ctx* c, int k) {
    return c->conv[k] ? hipSuccess : hipMalloc(&c->conv[k], disk_bytes(c));
}

void free_state(pmc_ctx* c) {
    if (c->own_state) {
        for (int b = 0; b < 2; ++b) {
            if (c->disk[b]) (void)hipFree(c->disk[b]);
            if (c->n[b]) (void)hipFree(c->n[b]);
        }
    }
    c->disk[0] = c->disk[1] = nullptr;
    c->n[0] = c->n[1] = nullptr;
    c->own_state = false;
}

void drop_graph(pmc_ctx* c) {
    if (c->graph_exec) (void)hipGraphExecDestroy(c->graph_exec);
    c->graph_exec = nullptr;
    c->graph_count = 0;
}

void drop_slab(pmc_ctx* c);
int slab_join(pmc_ctx* c);   // slab driver streams -> context stream (defined with the driver)
bool slab_is_ipc(const pmc_ctx* c);          // an IPC-transport slab driver is attached
int slab_pending_zdir(const pmc_ctx* c);     // a deferred z-shift halo exchange is outstanding

// the next timing slot when pmc_timing is on (nullptr otherwise): events ride on the launch's
// dispatch packet (hipExtLaunchKernelGGL), no extra packets in the stream
const LaunchTiming* next_timing(pmc_ctx* c, int kind, LaunchTiming* lt, int64_t phase = -1) {
    if (!c->timing || c->timing_paused) return nullptr;
    const size_t k = c->tkind.size();
    while (c->tev.size() < 2 * (k + 1)) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        c->tev.push_back(e);
    }
    c->tkind.push_back(kind);
    c->tphase.push_back(phase);
    lt->start = c->tev[2 * k];
    lt->stop = c->tev[2 * k + 1];
    return lt;
}

// Whole-box sweep in plane chains (PMC_SWEEP_CHAINS = 1, 2 (default) or 4): chain j runs the planes
// [b_j, b_{j+1}), b_j = 2*((j*nz)/(2*chains)) (even borders), chain 0 on the context stream, the others
// on streams of their own.  As in the slab driver (pmc_slab_sweep), the 8 phases form runs of equal z
// parity q; in a run only parity-q planes change, each reading its own plane and the parity 1-q planes
// next to it, which no phase of the run writes -- so the chains are independent for a whole run, and
// each chain's launch tails overlap the others' work.  At a run boundary each chain waits for its two
// neighbours' previous runs (the planes next to its borders, the periodic one included: plane 0 and
// plane nz-1 are neighbours).  shiftCells joins the chains on the context stream; the other streams
// start each sweep after it.  Cells of a colour are independent, so any split of a phase gives the
// same result bit for bit.
int chain_count(const pmc_ctx* c) {
    static const int env = [] {
        const char* v = std::getenv("PMC_SWEEP_CHAINS");
        return v ? std::atoi(v) : 2;
    }();
    if (c->P.halo) return 1;
    for (int n = env >= PMC_SWEEP_MAX_CHAINS ? PMC_SWEEP_MAX_CHAINS : env; n > 1; n /= 2)
        if (c->P.nz_local >= 4 * n) return n;   // chains of >= 4 planes
    return 1;
}
int chain_border(int nz, int n, int j) { return 2 * ((j * nz) / (2 * n)); }

int enqueue_sweep_chains(pmc_ctx* c, uint32_t sweep, const pmc_sweep_plan_t& plan, int n) {
    if (!c->ev_s) {
        for (auto& r : c->ev_c)
            for (auto& e : r) PMC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        PMC_HIP(hipEventCreateWithFlags(&c->ev_s, hipEventDisableTiming));
    }
    for (int j = 1; j < n; ++j) {
        if (!c->hs[j - 1]) PMC_HIP(hipStreamCreateWithFlags(&c->hs[j - 1], hipStreamNonBlocking));
        if (!c->ovf_ch[j - 1]) {   // chain j's overflow queue
            PMC_HIP(hipMalloc(&c->ovf_ch[j - 1], c->ovf_bytes));
            PMC_HIP(hipMemsetAsync(c->ovf_ch[j - 1], 0, c->ovf_bytes, c->stream));
        }
    }
    const int nz = c->P.nz_local;
    hipStream_t st[PMC_SWEEP_MAX_CHAINS];
    int* ovf[PMC_SWEEP_MAX_CHAINS];
    st[0] = c->stream;
    ovf[0] = c->ovf;
    for (int j = 1; j < n; ++j) {
        st[j] = c->hs[j - 1];
        ovf[j] = c->ovf_ch[j - 1];
    }
    // the other streams after everything issued on the context stream so far (the previous shift)
    PMC_HIP(hipEventRecord(c->ev_s, c->stream));
    for (int j = 1; j < n; ++j) PMC_HIP(hipStreamWaitEvent(st[j], c->ev_s, 0));
    int k = 0, q = 0;
    while (k < 8) {
        q = plan.order[k] % 2;
        int k1 = k;
        while (k1 < 8 && plan.order[k1] % 2 == q) ++k1;
        for (int j = 0; j < n; ++j) {
            if (k > 0) {   // the neighbours' previous runs (one neighbour when there are two chains)
                const int lo = (j + n - 1) % n, hi = (j + 1) % n;
                PMC_HIP(hipStreamWaitEvent(st[j], c->ev_c[lo][1 - q], 0));
                if (hi != lo) PMC_HIP(hipStreamWaitEvent(st[j], c->ev_c[hi][1 - q], 0));
            }
            for (int kk = k; kk < k1; ++kk) {
                int o[3];
                pmc_colour_offset(plan.order[kk], o);
                LaunchTiming lt;
                hipError_t e = launch_subsweep(c->G, c->disk[c->cur], c->n[c->cur], o[0], o[1], o[2], sweep, c->stats,
                                               ovf[j], chain_border(nz, n, j), chain_border(nz, n, j + 1), st[j],
                                               next_timing(c, 0, &lt, c->phase_seq + kk));
                if (e != hipSuccess) return hip_fail(e, "subsweep launch");
            }
            PMC_HIP(hipEventRecord(c->ev_c[j][q], st[j]));
        }
        k = k1;
    }
    c->phase_seq += 8;
    for (int j = 1; j < n; ++j)   // shiftCells reads every plane: each chain's last run
        PMC_HIP(hipStreamWaitEvent(c->stream, c->ev_c[j][q], 0));
    LaunchTiming lt;
    hipError_t e = launch_shift(c->G, c->disk[c->cur], c->n[c->cur], c->disk[c->cur ^ 1], c->n[c->cur ^ 1],
                                plan.f, plan.d, c->flags, c->stream, next_timing(c, 1, &lt));
    if (e != hipSuccess) return hip_fail(e, "shift launch");
    c->cur ^= 1;
    return PMC_OK;
}

int enqueue_sweep(pmc_ctx* c, uint32_t sweep, bool chains = true) {
    const pmc_sweep_plan_t plan = pmc_plan_for_sweep_ex(c->P.seed, sweep, c->P.w, c->P.flags);
    const int n = chains ? chain_count(c) : 1;
    if (n > 1) return enqueue_sweep_chains(c, sweep, plan, n);
    for (int k = 0; k < 8; ++k) {
        int o[3];
        pmc_colour_offset(plan.order[k], o);
        LaunchTiming lt;
        hipError_t e = launch_subsweep(c->G, c->disk[c->cur], c->n[c->cur], o[0], o[1], o[2], sweep,
                                       c->stats, c->ovf, 0, c->P.nz_local, c->stream, next_timing(c, 0, &lt), true);
        if (e != hipSuccess) return hip_fail(e, "subsweep launch");
    }
    LaunchTiming lt;
    hipError_t e = launch_shift(c->G, c->disk[c->cur], c->n[c->cur], c->disk[c->cur ^ 1], c->n[c->cur ^ 1],
                                plan.f, plan.d, c->flags, c->stream, next_timing(c, 1, &lt));
    if (e != hipSuccess) return hip_fail(e, "shift launch");
    c->cur ^= 1;
    return PMC_OK;
}

// The planes a slab context's shiftCells covers after the 8 phases (local [*zl0, *zl1), halo
// planes included) and which halo is left to receive (0 none, +1 top, -1 bottom): shiftCells
// moves particles between a plane and its neighbour in direction dir along f, so along x/y every
// halo plane is computable from the halo copy itself, along z the halo on the -dir side takes
// particles from the owned plane next to it and the other needs the neighbour's new plane.
int slab_shift_planes(int nz, const pmc_sweep_plan_t& plan, int* zl0, int* zl1) {
    const int dir = plan.d <= 0.0f ? -1 : 1;   // k_shift / shiftCells.h:46-53
    *zl0 = -1;
    *zl1 = nz + 1;
    if (plan.f != 2) return 0;
    if (dir > 0) *zl1 = nz;
    else *zl0 = 0;
    return dir;
}

}  // namespace

extern "C" {

const char* pmc_last_error(void) { return g_err.c_str(); }

// error reporting for the host-only I/O functions (pmc_io.cpp); internal, not in pmc.h
int pmc_io_fail(int code, const char* msg) { return fail(code, msg); }

int pmc_create(const pmc_params* params, pmc_ctx** out) {
    if (!params || !out) return fail(PMC_ERR_ARG, "null argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(PMC_ERR_NODEV, "no HIP device");
    pmc_params p = *params;
    int rc = normalise(&p);
    if (rc) return rc;
    pmc_ctx* c = new pmc_ctx();
    c->P = p;
    c->G = make_geom(p);
    c->cells = (int64_t)p.cps_x * p.cps_y * (p.nz_local + 2 * p.halo);
    auto cleanup = [&](int code) { pmc_destroy(c); return code; };
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess)
        return cleanup(hip_fail(e, "hipStreamCreate"));
    c->own_stream = true;
    c->own_state = true;
    for (int b = 0; b < 2; ++b) {
        if ((e = hipMalloc(&c->disk[b], disk_bytes(c))) != hipSuccess) return cleanup(hip_fail(e, "hipMalloc disk"));
        if ((e = hipMalloc(&c->n[b], n_bytes(c))) != hipSuccess) return cleanup(hip_fail(e, "hipMalloc n"));
        if ((e = hipMemsetAsync(c->disk[b], 0, disk_bytes(c), c->stream)) != hipSuccess) return cleanup(hip_fail(e, "hipMemset"));
        if ((e = hipMemsetAsync(c->n[b], 0, n_bytes(c), c->stream)) != hipSuccess) return cleanup(hip_fail(e, "hipMemset"));
    }
    const size_t sb = sizeof(unsigned long long) * kStatCounters * kStatSlots;
    if ((e = hipMalloc(&c->stats, sb)) != hipSuccess) return cleanup(hip_fail(e, "hipMalloc stats"));
    if ((e = hipMemsetAsync(c->stats, 0, sb, c->stream)) != hipSuccess) return cleanup(hip_fail(e, "hipMemset"));
    if ((e = hipMalloc(&c->eacc, sizeof(unsigned long long) * kStatSlots)) != hipSuccess)
        return cleanup(hip_fail(e, "hipMalloc eacc"));
    if ((e = hipMalloc(&c->flags, 16)) != hipSuccess) return cleanup(hip_fail(e, "hipMalloc flags"));
    {
        // (at least two colour planes: a two-plane boundary launch, launch_subsweep_planes2, queues
        // cells of two planes even when the slab has only one colour plane per parity)
        const size_t per_colour = (size_t)(p.cps_x / 2) * (p.cps_y / 2) * (size_t)(p.nz_local / 2 > 2 ? p.nz_local / 2 : 2);
        // header (queue length, done counter: zero between launches) + one entry per cell
        const size_t ob = sizeof(int) * (kOvfHead + per_colour);
        if ((e = hipMalloc(&c->ovf, ob)) != hipSuccess) return cleanup(hip_fail(e, "hipMalloc ovf"));
        if ((e = hipMemsetAsync(c->ovf, 0, ob, c->stream)) != hipSuccess) return cleanup(hip_fail(e, "hipMemset"));
        c->ovf_bytes = ob;
    }
    if ((e = hipMemsetAsync(c->flags, 0, 16, c->stream)) != hipSuccess) return cleanup(hip_fail(e, "hipMemset"));
    // Every zeroing above runs on the context stream and is complete before the context is
    // returned.  (It used to be hipMemset on the null stream, which a hipStreamNonBlocking stream
    // does not wait for and which may still be queued when hipMemset returns: with the null stream
    // busy -- torch's default stream, RCCL set-up work -- the zeroing of n could land after
    // init_lattice's assign had written the counts on the context stream, and a fresh context read
    // back all-zero counts.  tests/test_gpu_parity.py::test_create_ordered_after_busy_null_stream.)
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return cleanup(hip_fail(e, "hipStreamSynchronize"));
    if ((e = hipEventCreate(&c->ev0)) != hipSuccess) return cleanup(hip_fail(e, "hipEventCreate"));
    if ((e = hipEventCreate(&c->ev1)) != hipSuccess) return cleanup(hip_fail(e, "hipEventCreate"));
    *out = c;
    return PMC_OK;
}

void pmc_destroy(pmc_ctx* c) {
    if (!c) return;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    drop_slab(c);
    drop_graph(c);
    free_state(c);
    if (c->stats) (void)hipFree(c->stats);
    if (c->eacc) (void)hipFree(c->eacc);
    if (c->segq) (void)hipFree(c->segq);
    if (c->flags) (void)hipFree(c->flags);
    if (c->ovf) (void)hipFree(c->ovf);
    if (c->ovf_aux) (void)hipFree(c->ovf_aux);
    if (c->ovf_b) (void)hipFree(c->ovf_b);
    if (c->ovf_aux2) (void)hipFree(c->ovf_aux2);
    for (void* m : {(void*)c->send_d, (void*)c->send_n, (void*)c->xflags, (void*)c->conv[0], (void*)c->conv[1]})
        if (m) (void)hipFree(m);
    if (c->tmp_cnt) (void)hipFree(c->tmp_cnt);
    if (c->tmp_idx) (void)hipFree(c->tmp_idx);
    if (c->d_r) (void)hipFree(c->d_r);
    for (hipEvent_t e : c->tev) (void)hipEventDestroy(e);
    for (hipStream_t h : c->hs)
        if (h) {
            (void)hipStreamSynchronize(h);
            (void)hipStreamDestroy(h);
        }
    for (int* q : c->ovf_ch)
        if (q) (void)hipFree(q);
    for (auto& r : c->ev_c)
        for (hipEvent_t e : r)
            if (e) (void)hipEventDestroy(e);
    if (c->ev_s) (void)hipEventDestroy(c->ev_s);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int pmc_set_stream(pmc_ctx* c, void* stream) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    PMC_HIP(hipStreamSynchronize(c->stream));
    drop_graph(c);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    c->stream = (hipStream_t)stream;
    c->own_stream = false;
    return PMC_OK;
}

int pmc_get_stream(pmc_ctx* c, void** stream) {
    if (!c || !stream) return fail(PMC_ERR_ARG, "null argument");
    *stream = (void*)c->stream;
    return PMC_OK;
}

int pmc_device_count(int* count) {
    if (!count) return fail(PMC_ERR_ARG, "null argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        *count = 0;
        return fail(PMC_ERR_NODEV, "no HIP device");
    }
    *count = ndev;
    return PMC_OK;
}

int pmc_attach_state(pmc_ctx* c, float* disk0, int16_t* n0, float* disk1, int16_t* n1) {
    if (!c || !disk0 || !n0 || !disk1 || !n1) return fail(PMC_ERR_ARG, "null argument");
    if (slab_is_ipc(c)) return fail(PMC_ERR_ARG, "pmc_attach_state: the IPC transport's peers map the current buffers");
    PMC_HIP(hipStreamSynchronize(c->stream));
    drop_graph(c);
    free_state(c);
    c->disk[0] = disk0; c->n[0] = n0;
    c->disk[1] = disk1; c->n[1] = n1;
    c->cur = 0;
    return PMC_OK;
}

int pmc_state(pmc_ctx* c, float** disk, int16_t** n) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    if (disk) *disk = c->disk[c->cur];
    if (n) *n = c->n[c->cur];
    return PMC_OK;
}

int64_t pmc_storage_cells(const pmc_ctx* c) { return c ? c->cells : -1; }

int pmc_state_layout(const pmc_ctx* c, int* layout) {
    if (!c || !layout) return fail(PMC_ERR_ARG, "null argument");
    *layout = PMC_AOS ? PMC_LAYOUT_PACKED : PMC_LAYOUT_REFERENCE;
    return PMC_OK;
}

int pmc_init_r(pmc_ctx* c, int64_t n_atoms, float* d_r) {
    if (!c || !d_r || n_atoms < 0) return fail(PMC_ERR_ARG, "bad argument");
    hipError_t e = launch_init_r(c->G, n_atoms, icbrt_ceil(n_atoms), d_r, c->stream);
    return e == hipSuccess ? PMC_OK : hip_fail(e, "init_r launch");
}

int pmc_assign(pmc_ctx* c, const float* d_r, int64_t n_atoms, float* d_disk, int16_t* d_n) {
    if (!c || !d_disk || !d_n || (n_atoms > 0 && !d_r)) return fail(PMC_ERR_ARG, "bad argument");
    if (!c->tmp_cnt) {
        PMC_HIP(hipMalloc(&c->tmp_cnt, sizeof(int32_t) * (size_t)c->cells));
        PMC_HIP(hipMalloc(&c->tmp_idx, sizeof(int32_t) * (size_t)c->cells * (size_t)c->P.nmax));
    }
    PMC_HIP(hipMemsetAsync(c->flags, 0, 16, c->stream));
    hipError_t e = launch_assign(c->G, d_r, n_atoms, d_disk, d_n, c->tmp_cnt, c->tmp_idx, c->flags, c->stream, 0,
                                 is_state_buffer(c, d_disk) ? 0 : 1);
    if (e != hipSuccess) return hip_fail(e, "assign launch");
    uint32_t fl = 0;
    PMC_HIP(hipMemcpyAsync(&fl, c->flags, 4, hipMemcpyDeviceToHost, c->stream));
    PMC_HIP(hipStreamSynchronize(c->stream));
    if (fl & 4u) return fail(PMC_ERR_RANGE, "assign: particle outside the owned box");
    if (fl & 2u) return fail(PMC_ERR_OVERFLOW, "assign: cell occupancy exceeds nmax");
    return PMC_OK;
}

int pmc_subsweep_range(pmc_ctx* c, float* d_disk, const int16_t* d_n, const int offset[3], uint32_t sweep,
                       int zl_begin, int zl_end) {
    if (!c || !d_disk || !d_n || !offset) return fail(PMC_ERR_ARG, "bad argument");
    for (int k = 0; k < 3; ++k)
        if (offset[k] != 0 && offset[k] != 1) return fail(PMC_ERR_ARG, "offset must be in {0,1}^3");
    if (zl_begin < 0 || zl_end > c->P.nz_local || zl_begin > zl_end)
        return fail(PMC_ERR_ARG, "plane range outside the owned planes");
    // a caller's reference-layout buffer runs through the staging buffer in the state layout
    const bool conv = PMC_AOS && !is_state_buffer(c, d_disk);
    float* run = d_disk;
    if (conv) {
        PMC_HIP(ensure_conv(c, 0));
        PMC_HIP(launch_relayout(d_disk, c->conv[0], c->cells, c->P.nmax, 1, c->stream));
        run = c->conv[0];
    }
    LaunchTiming lt;
    hipError_t e = launch_subsweep(c->G, run, d_n, offset[0], offset[1], offset[2], sweep, c->stats, c->ovf,
                                   zl_begin, zl_end, c->stream, next_timing(c, 0, &lt), !c->slab);
    if (e == hipSuccess && conv) e = launch_relayout(c->conv[0], d_disk, c->cells, c->P.nmax, 0, c->stream);
    return e == hipSuccess ? PMC_OK : hip_fail(e, "subsweep launch");
}

int pmc_subsweep(pmc_ctx* c, float* d_disk, const int16_t* d_n, const int offset[3], uint32_t sweep) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    return pmc_subsweep_range(c, d_disk, d_n, offset, sweep, 0, c->P.nz_local);
}

int pmc_shift_cells(pmc_ctx* c, const float* din, const int16_t* nin, float* dout, int16_t* nout, int f,
                    float d) {
    if (!c || !din || !nin || !dout || !nout) return fail(PMC_ERR_ARG, "null buffer");
    if (f < 0 || f > 2) return fail(PMC_ERR_ARG, "f must be 0, 1 or 2 (reference draws -1..1: start.cu:251)");
    if (din == dout || nin == nout) return fail(PMC_ERR_ARG, "shift is double-buffered: in != out");
    // caller buffers in the reference layout run through the staging buffers in the state layout
    const bool cin = PMC_AOS && !is_state_buffer(c, din), cout = PMC_AOS && !is_state_buffer(c, dout);
    const float* rin = din;
    float* rout = dout;
    if (cin) {
        PMC_HIP(ensure_conv(c, 0));
        PMC_HIP(launch_relayout(din, c->conv[0], c->cells, c->P.nmax, 1, c->stream));
        rin = c->conv[0];
    }
    if (cout) {
        PMC_HIP(ensure_conv(c, 1));
        rout = c->conv[1];
    }
    LaunchTiming lt;
    hipError_t e = launch_shift(c->G, rin, nin, rout, nout, f, d, c->flags, c->stream, next_timing(c, 1, &lt));
    if (e == hipSuccess && cout) e = launch_relayout(rout, dout, c->cells, c->P.nmax, 0, c->stream);
    return e == hipSuccess ? PMC_OK : hip_fail(e, "shift launch");
}

int pmc_sweep_plan(uint64_t seed, uint32_t sweep, float w, int order[8], int* f, float* d) {
    return pmc_sweep_plan_ex(seed, sweep, w, 0u, order, f, d);
}

int pmc_sweep_plan_ex(uint64_t seed, uint32_t sweep, float w, uint32_t flags, int order[8], int* f, float* d) {
    if (!order || !f || !d) return fail(PMC_ERR_ARG, "null argument");
    if (flags & ~(PMC_FLAG_FULL_SHUFFLE | PMC_FLAG_QUIRKS)) return fail(PMC_ERR_ARG, "unknown plan flags");
    const pmc_sweep_plan_t plan = pmc_plan_for_sweep_ex(seed, sweep, w, flags);
    for (int k = 0; k < 8; ++k) order[k] = plan.order[k];
    *f = plan.f;
    *d = plan.d;
    return PMC_OK;
}

int pmc_init_lattice(pmc_ctx* c, int64_t n_atoms) {
    if (!c || n_atoms < 0) return fail(PMC_ERR_ARG, "bad argument");
    if (n_atoms > c->r_cap) {
        if (c->d_r) PMC_HIP(hipFree(c->d_r));
        c->d_r = nullptr;
        PMC_HIP(hipMalloc(&c->d_r, sizeof(float) * 3 * (size_t)(n_atoms > 0 ? n_atoms : 1)));
        c->r_cap = n_atoms;
    }
    int rc = pmc_init_r(c, n_atoms, c->d_r);
    if (rc) return rc;
    PMC_HIP(hipMemsetAsync(c->n[c->cur], 0, n_bytes(c), c->stream));
    return pmc_assign(c, c->d_r, n_atoms, c->disk[c->cur], c->n[c->cur]);
}

int pmc_init_lattice_planes(pmc_ctx* c, int64_t n_atoms_lattice, int32_t lattice_cps_z) {
    if (!c || n_atoms_lattice < 0) return fail(PMC_ERR_ARG, "bad argument");
    if (lattice_cps_z == 0) lattice_cps_z = c->P.cps_z;
    if (lattice_cps_z < c->P.cps_z) return fail(PMC_ERR_ARG, "lattice box lower than the simulation box");
    if (n_atoms_lattice > c->r_cap) {
        if (c->d_r) PMC_HIP(hipFree(c->d_r));
        c->d_r = nullptr;
        PMC_HIP(hipMalloc(&c->d_r, sizeof(float) * 3 * (size_t)(n_atoms_lattice > 0 ? n_atoms_lattice : 1)));
        c->r_cap = n_atoms_lattice;
    }
    // init_r over the lattice box cps_x x cps_y x lattice_cps_z, bottom-aligned with the periodic
    // box (z from -Lz/2): k_init_r's slab form with z0 = 0 and nz_local = lattice_cps_z.  With
    // lattice_cps_z == cps_z the offset is exactly 0 and these are a whole-box context's floats.
    DevGeom gg = c->G;
    gg.z0 = 0;
    gg.nz_local = lattice_cps_z;
    hipError_t e = launch_init_r(gg, n_atoms_lattice, icbrt_ceil(n_atoms_lattice), c->d_r, c->stream);
    if (e != hipSuccess) return hip_fail(e, "init_r launch");
    PMC_HIP(hipMemsetAsync(c->n[c->cur], 0, n_bytes(c), c->stream));
    if (!c->tmp_cnt) {
        PMC_HIP(hipMalloc(&c->tmp_cnt, sizeof(int32_t) * (size_t)c->cells));
        PMC_HIP(hipMalloc(&c->tmp_idx, sizeof(int32_t) * (size_t)c->cells * (size_t)c->P.nmax));
    }
    PMC_HIP(hipMemsetAsync(c->flags, 0, 16, c->stream));
    // assign keeps the owned planes' particles (clip 1: other slabs' particles are skipped;
    // clip 2: also the lattice rows above the periodic box)
    e = launch_assign(c->G, c->d_r, n_atoms_lattice, c->disk[c->cur], c->n[c->cur], c->tmp_cnt, c->tmp_idx,
                      c->flags, c->stream, lattice_cps_z > c->P.cps_z ? 2 : 1);
    if (e != hipSuccess) return hip_fail(e, "assign launch");
    uint32_t fl = 0;
    PMC_HIP(hipMemcpyAsync(&fl, c->flags, 4, hipMemcpyDeviceToHost, c->stream));
    PMC_HIP(hipStreamSynchronize(c->stream));
    if (fl & 4u) return fail(PMC_ERR_RANGE, "assign: particle outside the box");
    if (fl & 2u) return fail(PMC_ERR_OVERFLOW, "assign: cell occupancy exceeds nmax");
    return PMC_OK;
}

int pmc_init_lattice_global(pmc_ctx* c, int64_t n_atoms_total) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    return pmc_init_lattice_planes(c, n_atoms_total, c->P.cps_z);
}

int pmc_phase_range(pmc_ctx* c, int colour, uint32_t sweep, int zl_begin, int zl_end) {
    if (!c || colour < 0 || colour > 7) return fail(PMC_ERR_ARG, "bad argument");
    int o[3];
    pmc_colour_offset(colour, o);
    return pmc_subsweep_range(c, c->disk[c->cur], c->n[c->cur], o, sweep, zl_begin, zl_end);
}

int pmc_phase_range_on(pmc_ctx* c, int colour, uint32_t sweep, int zl_begin, int zl_end, void* stream) {
    if (!c || colour < 0 || colour > 7) return fail(PMC_ERR_ARG, "bad argument");
    if (zl_begin < 0 || zl_end > c->P.nz_local || zl_begin > zl_end)
        return fail(PMC_ERR_ARG, "plane range outside the owned planes");
    hipStream_t st = (hipStream_t)stream;
    if (st == c->stream) return pmc_phase_range(c, colour, sweep, zl_begin, zl_end);
    if (!c->ovf_aux) {   // the aux launches' own overflow queue (concurrent with the context stream's)
        PMC_HIP(hipMalloc(&c->ovf_aux, c->ovf_bytes));
        PMC_HIP(hipMemsetAsync(c->ovf_aux, 0, c->ovf_bytes, c->stream));   // ordered before st's launches:
        PMC_HIP(hipStreamSynchronize(c->stream));                         // st does not wait for c->stream
    }
    int o[3];
    pmc_colour_offset(colour, o);
    LaunchTiming lt;
    hipError_t e = launch_subsweep(c->G, c->disk[c->cur], c->n[c->cur], o[0], o[1], o[2], sweep, c->stats,
                                   c->ovf_aux, zl_begin, zl_end, st, next_timing(c, 2, &lt));
    return e == hipSuccess ? PMC_OK : hip_fail(e, "subsweep launch");
}

int pmc_phase(pmc_ctx* c, int colour, uint32_t sweep) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    return pmc_phase_range(c, colour, sweep, 0, c->P.nz_local);
}

int pmc_shift(pmc_ctx* c, uint32_t sweep) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    const pmc_sweep_plan_t plan = pmc_plan_for_sweep_ex(c->P.seed, sweep, c->P.w, c->P.flags);
    int rc = pmc_shift_cells(c, c->disk[c->cur], c->n[c->cur], c->disk[c->cur ^ 1], c->n[c->cur ^ 1], plan.f,
                             plan.d);
    if (rc) return rc;
    c->cur ^= 1;
    return PMC_OK;
}

int pmc_shift_slab(pmc_ctx* c, uint32_t sweep, int* halo_recv) {
    if (!c || !halo_recv) return fail(PMC_ERR_ARG, "null argument");
    if (c->P.halo != 1) return fail(PMC_ERR_ARG, "pmc_shift_slab needs a slab context (halo = 1)");
    const pmc_sweep_plan_t plan = pmc_plan_for_sweep_ex(c->P.seed, sweep, c->P.w, c->P.flags);
    int zl0, zl1;
    *halo_recv = slab_shift_planes(c->P.nz_local, plan, &zl0, &zl1);
    LaunchTiming lt;
    hipError_t e = launch_shift_planes(c->G, c->disk[c->cur], c->n[c->cur], c->disk[c->cur ^ 1], c->n[c->cur ^ 1],
                                       plan.f, plan.d, c->flags, zl0, zl1, c->stream, next_timing(c, 1, &lt));
    if (e != hipSuccess) return hip_fail(e, "shift launch");
    c->cur ^= 1;
    return PMC_OK;
}

int pmc_sweep(pmc_ctx* c, uint32_t sweep) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    if (c->P.halo) return fail(PMC_ERR_ARG, "pmc_sweep needs the whole box; slabs use pmc_phase/pmc_shift + halo exchange");
    return enqueue_sweep(c, sweep);
}

int pmc_run_graph(pmc_ctx* c, uint32_t first, int count) {
    if (!c || count < 0) return fail(PMC_ERR_ARG, "bad argument");
    if (c->P.halo) return fail(PMC_ERR_ARG, "graph replay needs the whole box");
    if (count == 0) return PMC_OK;
    // The sweep plan (colour order, f, d) differs per sweep and is baked into kernel arguments,
    // so the captured graph covers exactly sweeps [first, first+count) from the current buffer.
    if (!(c->graph_exec && c->graph_first == first && c->graph_count == count && c->graph_cur == c->cur)) {
        drop_graph(c);
        hipGraph_t graph = nullptr;
        const int cur0 = c->cur;
        const bool timing = c->timing;   // no per-launch events inside a graph
        c->timing = false;
        PMC_HIP(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
        int rc = PMC_OK;
        for (int k = 0; k < count && rc == PMC_OK; ++k) rc = enqueue_sweep(c, first + (uint32_t)k, false);
        hipError_t e = hipStreamEndCapture(c->stream, &graph);
        c->cur = cur0;
        c->timing = timing;
        if (rc) { if (graph) (void)hipGraphDestroy(graph); return rc; }
        if (e != hipSuccess) return hip_fail(e, "hipStreamEndCapture");
        e = hipGraphInstantiate(&c->graph_exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (e != hipSuccess) return hip_fail(e, "hipGraphInstantiate");
        c->graph_first = first;
        c->graph_count = count;
        c->graph_cur = cur0;
    }
    PMC_HIP(hipGraphLaunch(c->graph_exec, c->stream));
    if (count & 1) c->cur ^= 1;
    return PMC_OK;
}

// sum over the context's owned cells of the fixed-point pair terms (k_energy; the energy is half of
// it, scaled by 2^-32): exact, and exactly additive over slabs
int energy_fixed(pmc_ctx* c, int64_t* fixed) {
    // the energy reads both halos: a z shift's deferred halo exchange must be flushed first, and the
    // flush is collective (pmc_slab_finish / pmc_slab_observables do it on every rank)
    if (slab_pending_zdir(c))
        return fail(PMC_ERR_ARG, "pmc_energy: a slab halo exchange is pending (call pmc_slab_finish first)");
    if (int rj = slab_join(c)) return rj;
    PMC_HIP(hipMemsetAsync(c->eacc, 0, sizeof(unsigned long long) * kStatSlots, c->stream));
    if (!c->segq) PMC_HIP(hipMalloc(&c->segq, sizeof(int) * (1 + energy_segments(c->G))));
    PMC_HIP(hipMemsetAsync(c->segq, 0, sizeof(int), c->stream));
    hipError_t e = launch_energy(c->G, c->disk[c->cur], c->n[c->cur], c->eacc, c->segq, c->stream);
    if (e != hipSuccess) return hip_fail(e, "energy launch");
    std::vector<unsigned long long> h(kStatSlots);
    PMC_HIP(hipMemcpyAsync(h.data(), c->eacc, sizeof(unsigned long long) * kStatSlots, hipMemcpyDeviceToHost,
                           c->stream));
    PMC_HIP(hipStreamSynchronize(c->stream));
    unsigned long long s = 0;
    for (auto v : h) s += v;
    *fixed = (int64_t)s;
    return PMC_OK;
}

int pmc_energy(pmc_ctx* c, double* e_out) {
    if (!c || !e_out) return fail(PMC_ERR_ARG, "bad argument");
    int64_t f = 0;
    if (int rc = energy_fixed(c, &f)) return rc;
    *e_out = (double)f / PMC_FIX_SCALE * 0.5;
    return PMC_OK;
}

int pmc_stats_read(pmc_ctx* c, pmc_stats* out, int reset) {
    if (!c || !out) return fail(PMC_ERR_ARG, "bad argument");
    if (int rj = slab_join(c)) return rj;
    std::vector<unsigned long long> h((size_t)kStatCounters * kStatSlots);
    PMC_HIP(hipMemcpyAsync(h.data(), c->stats, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost,
                           c->stream));
    PMC_HIP(hipStreamSynchronize(c->stream));
    unsigned long long s[kStatCounters] = {0, 0, 0, 0};
    for (int k = 0; k < kStatCounters; ++k)
        for (int i = 0; i < kStatSlots; ++i) s[k] += h[(size_t)stat_index(k, i)];
    out->de_fixed = (int64_t)s[0];
    out->accepted = (int64_t)s[1];
    out->trials = (int64_t)s[2];
    out->evaluated = (int64_t)s[3];
    if (reset) {
        PMC_HIP(hipMemsetAsync(c->stats, 0, sizeof(unsigned long long) * h.size(), c->stream));
        PMC_HIP(hipStreamSynchronize(c->stream));
    }
    return PMC_OK;
}

int pmc_error_flags(pmc_ctx* c, uint32_t* flags, int reset) {
    if (!c || !flags) return fail(PMC_ERR_ARG, "bad argument");
    if (int rj = slab_join(c)) return rj;
    PMC_HIP(hipMemcpyAsync(flags, c->flags, 4, hipMemcpyDeviceToHost, c->stream));
    if (reset) PMC_HIP(hipMemsetAsync(c->flags, 0, 16, c->stream));
    PMC_HIP(hipStreamSynchronize(c->stream));
    return PMC_OK;
}

int pmc_run_small(pmc_ctx* c, uint32_t first, int count) {
    if (!c || count < 0) return fail(PMC_ERR_ARG, "bad argument");
    if (small_sweep_participants(c->G) == 0)
        return fail(PMC_ERR_ARG, "pmc_run_small: the box does not qualify (whole box, nmax 16, <= 2048 cells per colour, no quirk flags)");
    if (count == 0) return PMC_OK;
    const unsigned P = (unsigned)small_sweep_participants(c->G);
    // one launch per kSmallSweeps sweeps; after each, the barrier counter (flags word 2; word 0 holds
    // the error bits) must show every participant at every one of the launch's 9 barriers per sweep.
    // A launch none of whose workgroups ran on XCD 0 (the kernel's participation test) does nothing
    // and reaches no barrier: without this check the context would flip to the stale buffer.
    for (int done = 0; done < count;) {
        const int n = count - done < kSmallSweeps ? count - done : kSmallSweeps;
        hipError_t e = launch_sweep_small(c->G, c->disk[0], c->n[0], c->disk[1], c->n[1], c->cur, c->stats, c->flags,
                                          (unsigned*)(c->flags + 2), c->P.seed, first + (uint32_t)done, n, c->P.flags,
                                          c->stream);
        if (e != hipSuccess) return hip_fail(e, "small-box sweep launch");
        uint32_t w[3] = {0, 0, 0};
        PMC_HIP(hipMemcpyAsync(w, c->flags, sizeof w, hipMemcpyDeviceToHost, c->stream));
        PMC_HIP(hipStreamSynchronize(c->stream));
        if (w[0] & 8u) return fail(PMC_ERR_HIP, "small-box sweep: a barrier timed out (participants not co-resident)");
        if (w[0] & 16u) return fail(PMC_ERR_HIP, "small-box sweep: the launch was not dealt round-robin over the XCDs");
        if (w[2] != 9u * P * (unsigned)n) {
            w[0] |= 32u;
            PMC_HIP(hipMemcpyAsync(c->flags, &w[0], sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
            PMC_HIP(hipStreamSynchronize(c->stream));
            return fail(PMC_ERR_HIP, "small-box sweep: no workgroup of the launch ran on XCD 0 (state unchanged)");
        }
        if (n & 1) c->cur ^= 1;
        done += n;
    }
    return PMC_OK;
}

// pmc_start runs every box with eager launches: since small colour phases run as one full-capacity
// launch each (k_subsweep_full, 9 launches per sweep), they beat pmc_run_small's single launch on
// XCD 0 at every size (8^3: 0.070 against 0.110 ms per sweep, 16^3: 0.072 against 0.513 ms,
// profiles/r03sm_small_box.txt; round 3 had picked pmc_run_small for <= 64 cells per colour against
// the 17-launch sweep).  PMC_SMALL=1 restores that choice; pmc_run_small stays callable.
static bool use_small(const pmc_ctx* c) {
    static const bool on = [] {
        const char* v = std::getenv("PMC_SMALL");
        return v && std::atoi(v) == 1;
    }();
    const int64_t per_colour = (int64_t)(c->P.cps_x / 2) * (c->P.cps_y / 2) * (c->P.cps_z / 2);
    return on && small_sweep_participants(c->G) > 0 && per_colour <= 64;
}

int pmc_start_ex(pmc_ctx* c, uint32_t first, int mc_passes, int flags, pmc_result* out) {
    if (!c || mc_passes < 0) return fail(PMC_ERR_ARG, "bad argument");
    if (c->P.halo) return fail(PMC_ERR_ARG, "pmc_start drives the whole box; use the slab driver for halo mode");
    const bool energies = !(flags & PMC_START_NO_ENERGY);
    pmc_result r;
    std::memset(&r, 0, sizeof(r));
    r.e_initial = r.e_final = std::nan("");
    pmc_stats s0;
    int rc = pmc_stats_read(c, &s0, 0);
    if (rc) return rc;
    if (energies && (rc = pmc_energy(c, &r.e_initial))) return rc;
    PMC_HIP(hipEventRecord(c->ev0, c->stream));
    if (use_small(c) && !c->timing) {
        if ((rc = pmc_run_small(c, first, mc_passes))) return rc;
    } else {
        for (int k = 0; k < mc_passes; ++k) {
            rc = enqueue_sweep(c, first + (uint32_t)k);
            if (rc) return rc;
        }
    }
    PMC_HIP(hipEventRecord(c->ev1, c->stream));
    PMC_HIP(hipEventSynchronize(c->ev1));
    float ms = 0.0f;
    PMC_HIP(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    r.seconds = ms * 1e-3;
    if (energies && (rc = pmc_energy(c, &r.e_final))) return rc;
    pmc_stats s1;
    rc = pmc_stats_read(c, &s1, 0);
    if (rc) return rc;
    r.stats.de_fixed = s1.de_fixed - s0.de_fixed;
    r.stats.accepted = s1.accepted - s0.accepted;
    r.stats.trials = s1.trials - s0.trials;
    r.stats.evaluated = s1.evaluated - s0.evaluated;
    r.sweeps = mc_passes;
    uint32_t fl = 0;
    rc = pmc_error_flags(c, &fl, 0);
    if (rc) return rc;
    if (out) *out = r;
    if (fl & 1u) return fail(PMC_ERR_OVERFLOW, "shiftCells: cell occupancy exceeded nmax");
    if (fl & 8u) return fail(PMC_ERR_HIP, "small-box sweep: a barrier timed out (participants not co-resident)");
    if (fl & 16u) return fail(PMC_ERR_HIP, "small-box sweep: the launch was not dealt round-robin over the XCDs");
    if (fl & 32u) return fail(PMC_ERR_HIP, "small-box sweep: no workgroup of the launch ran on XCD 0");
    return PMC_OK;
}

int pmc_start(pmc_ctx* c, uint32_t first, int mc_passes, pmc_result* out) {
    return pmc_start_ex(c, first, mc_passes, 0, out);
}

int pmc_copy_out(pmc_ctx* c, float* h_disk, int16_t* h_n) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    if (int rj = slab_join(c)) return rj;
    if (h_disk) {   // the reference layout (PMC_AOS: converted on the device first)
        const float* src = c->disk[c->cur];
        if (PMC_AOS) {
            PMC_HIP(ensure_conv(c, 0));
            PMC_HIP(launch_relayout(src, c->conv[0], c->cells, c->P.nmax, 0, c->stream));
            src = c->conv[0];
        }
        PMC_HIP(hipMemcpyAsync(h_disk, src, disk_bytes(c), hipMemcpyDeviceToHost, c->stream));
    }
    if (h_n) PMC_HIP(hipMemcpyAsync(h_n, c->n[c->cur], n_bytes(c), hipMemcpyDeviceToHost, c->stream));
    PMC_HIP(hipStreamSynchronize(c->stream));
    return PMC_OK;
}

int pmc_copy_in(pmc_ctx* c, const float* h_disk, const int16_t* h_n) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    if (int rj = slab_join(c)) return rj;
    if (h_disk) {   // from the reference layout (PMC_AOS: converted on the device)
        if (PMC_AOS) {
            PMC_HIP(ensure_conv(c, 0));
            PMC_HIP(hipMemcpyAsync(c->conv[0], h_disk, disk_bytes(c), hipMemcpyHostToDevice, c->stream));
            PMC_HIP(launch_relayout(c->conv[0], c->disk[c->cur], c->cells, c->P.nmax, 1, c->stream));
        } else {
            PMC_HIP(hipMemcpyAsync(c->disk[c->cur], h_disk, disk_bytes(c), hipMemcpyHostToDevice, c->stream));
        }
    }
    if (h_n) PMC_HIP(hipMemcpyAsync(c->n[c->cur], h_n, n_bytes(c), hipMemcpyHostToDevice, c->stream));
    PMC_HIP(hipStreamSynchronize(c->stream));
    return PMC_OK;
}

int pmc_synchronize(pmc_ctx* c) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    if (int rj = slab_join(c)) return rj;
    PMC_HIP(hipStreamSynchronize(c->stream));
    return PMC_OK;
}

int pmc_plane_span(const pmc_ctx* c, int z_local, size_t* disk_off, size_t* disk_b, size_t* n_off,
                   size_t* n_b) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    const int lo = -c->P.halo, hi = c->P.nz_local - 1 + c->P.halo;
    if (z_local < lo || z_local > hi) return fail(PMC_ERR_ARG, "plane outside storage");
    const size_t plane_cells = (size_t)c->P.cps_x * (size_t)c->P.cps_y;
    const size_t pidx = (size_t)(z_local + c->P.halo);
    if (disk_off) *disk_off = pidx * plane_cells * 3 * (size_t)c->P.nmax * sizeof(float);
    if (disk_b) *disk_b = plane_cells * 3 * (size_t)c->P.nmax * sizeof(float);
    if (n_off) *n_off = pidx * plane_cells * sizeof(int16_t);
    if (n_b) *n_b = plane_cells * sizeof(int16_t);
    return PMC_OK;
}

int pmc_selftest_detmath(const uint32_t* h_words, int count, float* h_out_f, double* h_out_d) {
    if (!h_words || !h_out_f || !h_out_d || count < 0) return fail(PMC_ERR_ARG, "bad argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(PMC_ERR_NODEV, "no HIP device");
    if (count == 0) return PMC_OK;
    uint32_t* dw = nullptr;
    float* df = nullptr;
    double* dd = nullptr;
    PMC_HIP(hipMalloc(&dw, sizeof(uint32_t) * 4 * (size_t)count));
    PMC_HIP(hipMalloc(&df, sizeof(float) * 4 * (size_t)count));
    PMC_HIP(hipMalloc(&dd, sizeof(double) * 2 * (size_t)count));
    PMC_HIP(hipMemcpy(dw, h_words, sizeof(uint32_t) * 4 * (size_t)count, hipMemcpyHostToDevice));
    hipError_t e = launch_selftest(dw, count, df, dd, pmc_cutoff_r2(2.5f), nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(h_out_f, df, sizeof(float) * 4 * (size_t)count, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(h_out_d, dd, sizeof(double) * 2 * (size_t)count, hipMemcpyDeviceToHost);
    (void)hipFree(dw);
    (void)hipFree(df);
    (void)hipFree(dd);
    return e == hipSuccess ? PMC_OK : hip_fail(e, "selftest");
}

int pmc_hbm_probe(uint64_t bytes, int reps, double* read_gbs, double* copy_gbs) {
    if (!read_gbs || !copy_gbs || reps < 1 || bytes < ((uint64_t)1 << 24)) return fail(PMC_ERR_ARG, "bad argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(PMC_ERR_NODEV, "no HIP device");
    bytes &= ~(uint64_t)4095;
    int dev = 0, cus = 0;
    PMC_HIP(hipGetDevice(&dev));
    PMC_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int ncu = cus > 0 ? cus : 256;
    void *a = nullptr, *b = nullptr, *sink = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t e = hipMalloc(&a, bytes);
    if (e == hipSuccess) e = hipMalloc(&b, bytes);
    if (e == hipSuccess) e = hipMalloc(&sink, sizeof(uint32_t) * (size_t)ncu * 32);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipMemsetAsync(a, 0x5a, bytes, st);
    // best over the shapes that measured fastest (tools/ubench/hbm_stream.hip, profiles/r06h_hbm_stream.txt):
    // 2 / 8 / 32 workgroups of 256 per CU, 8 nontemporal loads in flight per lane (read), 4 or 8 per
    // lane in per-workgroup chunks (copy)
    double best[2] = {0.0, 0.0};
    for (int cfg = 0; cfg < 12 && e == hipSuccess; ++cfg) {
        const int kind = cfg / 6, unroll = kind == 0 || (cfg / 3) % 2 ? 8 : 4;
        const int blocks = ncu * (cfg % 3 == 0 ? 2 : (cfg % 3 == 1 ? 8 : 32));
        e = launch_hbm_probe(kind, unroll, a, b, bytes, (uint32_t*)sink, blocks, st);   // warm-up
        for (int r = 0; r < reps && e == hipSuccess; ++r) {
            e = hipEventRecord(e0, st);
            if (e == hipSuccess) e = launch_hbm_probe(kind, unroll, a, b, bytes, (uint32_t*)sink, blocks, st);
            if (e == hipSuccess) e = hipEventRecord(e1, st);
            if (e == hipSuccess) e = hipEventSynchronize(e1);
            float ms = 0.0f;
            if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
            const double gbs = (kind == 0 ? 1.0 : 2.0) * (double)bytes / ((double)ms * 1e-3) / 1e9;
            if (e == hipSuccess && ms > 0.0f && gbs > best[kind]) best[kind] = gbs;
        }
    }
    if (st) (void)hipStreamSynchronize(st);
    for (void* p : {a, b, sink})
        if (p) (void)hipFree(p);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
    if (e != hipSuccess) return hip_fail(e, "hbm probe");
    *read_gbs = best[0];
    *copy_gbs = best[1];
    return PMC_OK;
}

}  // extern "C"

// ---- trajectory dump / restart (kernel.cu:497-536; pmc_io.cpp holds the host formats) ----------
namespace {

// owned cells of the storage (slab mode skips the halo planes)
void owned_range(const pmc_ctx* c, int64_t* first, int64_t* count) {
    const int64_t plane = (int64_t)c->P.cps_x * c->P.cps_y;
    *first = plane * c->P.halo;
    *count = plane * c->P.nz_local;
}

}  // namespace

int pmc_get_params(const pmc_ctx* c, pmc_params* out) {
    if (!c || !out) return fail(PMC_ERR_ARG, "bad argument");
    *out = c->P;
    return PMC_OK;
}

int pmc_stats_write(pmc_ctx* c, const pmc_stats* in) {
    if (!c || !in) return fail(PMC_ERR_ARG, "bad argument");
    if (int rj = slab_join(c)) return rj;
    std::vector<unsigned long long> h((size_t)kStatCounters * kStatSlots, 0ull);
    h[stat_index(0, 0)] = (unsigned long long)in->de_fixed;
    h[stat_index(1, 0)] = (unsigned long long)in->accepted;
    h[stat_index(2, 0)] = (unsigned long long)in->trials;
    h[stat_index(3, 0)] = (unsigned long long)in->evaluated;
    PMC_HIP(hipMemcpyAsync(c->stats, h.data(), sizeof(unsigned long long) * h.size(), hipMemcpyHostToDevice, c->stream));
    PMC_HIP(hipStreamSynchronize(c->stream));
    return PMC_OK;
}

int pmc_dump_frame(pmc_ctx* c, const char* path, int append, int64_t timestep) {
    if (!c || !path) return fail(PMC_ERR_ARG, "bad argument");
    std::vector<float> disk((size_t)c->cells * 3 * (size_t)c->P.nmax);
    std::vector<int16_t> n((size_t)c->cells);
    int rc = pmc_copy_out(c, disk.data(), n.data());
    if (rc) return rc;
    int64_t first, count, atoms = 0;
    owned_range(c, &first, &count);
    const float* d0 = disk.data() + (size_t)first * 3 * (size_t)c->P.nmax;
    if ((rc = pmc_disk_to_r(d0, n.data() + first, count, c->P.nmax, nullptr, 0, &atoms))) return rc;
    std::vector<float> r((size_t)atoms * 3);
    if ((rc = pmc_disk_to_r(d0, n.data() + first, count, c->P.nmax, r.data(), atoms, &atoms))) return rc;
    // the reference writes -L/2 .. L/2 on every axis (kernel.cu:523-524); global box in slab mode
    const float lo[3] = {-c->G.Lx / 2.0f, -c->G.Ly / 2.0f, -c->G.Lz / 2.0f};
    const float hi[3] = {c->G.Lx / 2.0f, c->G.Ly / 2.0f, c->G.Lz / 2.0f};
    return pmc_write_dump(path, append, timestep, r.data(), atoms, atoms, lo, hi);
}

int pmc_save_snapshot(pmc_ctx* c, const char* path, uint32_t next_sweep) {
    if (!c || !path) return fail(PMC_ERR_ARG, "bad argument");
    std::vector<float> disk((size_t)c->cells * 3 * (size_t)c->P.nmax);
    std::vector<int16_t> n((size_t)c->cells);
    int rc = pmc_copy_out(c, disk.data(), n.data());
    if (rc) return rc;
    pmc_stats st;
    if ((rc = pmc_stats_read(c, &st, 0))) return rc;
    int64_t first, count;
    owned_range(c, &first, &count);
    return pmc_snapshot_write(path, &c->P, next_sweep, &st, disk.data() + (size_t)first * 3 * (size_t)c->P.nmax,
                              n.data() + first, count);
}

int pmc_load_snapshot(pmc_ctx* c, const char* path, uint32_t* next_sweep) {
    if (!c || !path) return fail(PMC_ERR_ARG, "bad argument");
    const pmc_params& p = c->P;
    int64_t first, count;
    owned_range(c, &first, &count);
    std::vector<float> disk((size_t)c->cells * 3 * (size_t)p.nmax, 0.0f);
    std::vector<int16_t> n((size_t)c->cells, 0);
    // one open file: header and payload; the reader rejects an nmax other than ours before
    // writing into the buffers (sized for our nmax)
    pmc_params q;
    std::memset(&q, 0, sizeof(q));
    q.nmax = p.nmax;
    uint32_t sw = 0;
    pmc_stats st;
    int rc = pmc_snapshot_read(path, &q, &sw, &st, disk.data() + (size_t)first * 3 * (size_t)p.nmax,
                               n.data() + first, count);
    if (rc) return rc;
    if (q.cps_x != p.cps_x || q.cps_y != p.cps_y || q.cps_z != p.cps_z || q.nz_local != p.nz_local || q.z0 != p.z0 ||
        q.halo != p.halo || q.nmax != p.nmax || q.n_moves != p.n_moves || q.w != p.w || q.beta != p.beta ||
        q.sigma != p.sigma || q.seed != p.seed || q.flags != p.flags)
        return fail(PMC_ERR_ARG, "pmc_load_snapshot: snapshot parameters differ from the context's");
    if ((rc = pmc_copy_in(c, disk.data(), n.data()))) return rc;   // halo planes: zero until exchanged
    if ((rc = pmc_stats_write(c, &st))) return rc;
    if (next_sweep) *next_sweep = sw;
    return PMC_OK;
}

// =========================================================================================
// Multi-GPU slab driver: one process per GPU, each owning a z-slab of the box
// plus one halo plane below and above; halos travel over RCCL (xGMI) point-to-point.
// The whole sweep schedule runs here, in C: per colour phase a handful of HIP/RCCL calls and no
// Python, so the host stays ahead of the GPU even for thin (strong-scaling) slabs.
// =========================================================================================
#include <dlfcn.h>
#include <rccl/rccl.h>   // types and signatures only: librccl is dlopen'ed by soname, so a
                         // process that already holds one (torch's) shares that instance

namespace {

struct Rccl {
    bool tried = false, ok = false;
    std::string err;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;   // observables (pmc_slab_observables)
};

Rccl& rccl() {
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    const char* path = std::getenv("PMC_RCCL_LIB");
    void* h = dlopen(path && *path ? path : "librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        r.err = std::string("dlopen librccl: ") + dlerror();
        return r;
    }
    auto sym = [&](const char* name) { return dlsym(h, name); };
    r.get_unique_id = (decltype(r.get_unique_id))sym("ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))sym("ncclCommInitRank");
    r.comm_destroy = (decltype(r.comm_destroy))sym("ncclCommDestroy");
    r.send = (decltype(r.send))sym("ncclSend");
    r.recv = (decltype(r.recv))sym("ncclRecv");
    r.group_start = (decltype(r.group_start))sym("ncclGroupStart");
    r.group_end = (decltype(r.group_end))sym("ncclGroupEnd");
    r.error_string = (decltype(r.error_string))sym("ncclGetErrorString");
    r.all_reduce = (decltype(r.all_reduce))sym("ncclAllReduce");
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.send && r.recv && r.group_start &&
           r.group_end && r.error_string;
    if (!r.ok) r.err = "librccl lacks a required symbol";
    return r;
}

int nccl_fail(ncclResult_t e, const char* what) {
    return fail(PMC_ERR_HIP, std::string(what) + ": " + rccl().error_string(e));
}

#define PMC_NCCL(call)                                    \
    do {                                                  \
        ncclResult_t r_ = (call);                         \
        if (r_ != ncclSuccess) return nccl_fail(r_, #call); \
    } while (0)

}  // namespace

// ---- halo transports --------------------------------------------------------------------------
// Every halo exchange of the slab driver is a list of point-to-point messages (sends and receives
// of byte ranges, with ncclSend/ncclRecv matching: the k-th send from rank a to rank b fills the
// k-th receive on b from a) issued on the aux stream.  Two transports carry them:
//   * RCCL (one process per GPU, the product multi-GPU path): one ncclGroupStart/End per list;
//   * an in-process group (pmc_local_group): W slab contexts of ONE process, one host thread per
//     rank, device-to-device copies ordered by HIP events and a host barrier -- the same schedule,
//     peers and message lists as RCCL, so W ranks run on one GPU ("a local-copy halo
//     transport behind the same interface as the RCCL transport");
//   * IPC (pmc_slab_init_ipc): one process per rank on one node -- one per GPU, or several on one
//     GPU -- each mapping its peers' state buffers and flags (hipIpcOpenMemHandle over xGMI); the
//     receiver pulls every message straight from the sender's buffer with its own copy kernel,
//     ordered by per-rank sequence flags in device memory (pmc_kernels.hip, k_xfer_*): no host
//     round trip, no proxy thread, no RCCL channel set-up per message.
// A single rank without either keeps its periodic halos by local copies (no messages at all).
struct XferMsg {
    void* buf;
    size_t bytes;
    int peer;
    // receives: where the sender's source lies, named by the SAME buffer and offset in this rank's
    // own memory -- every rank has the identical layout and ping-pong index (symmetric buffers), so
    // the IPC transport maps it to the peer's copy (pmc_slab_init_ipc)
    const void* sym = nullptr;
};

struct pmc_local_group {
    struct Slot {
        hipEvent_t ready = nullptr;    // the rank's aux stream after its send buffers were written
        hipEvent_t pulled = nullptr;   // ... after its receives (copies from the peers' buffers)
        std::vector<XferMsg> sends, recvs;
        bool joined = false;
        uint64_t red[5] = {0, 0, 0, 0, 0};   // observables of the rank (pmc_slab_observables)
    };
    int world = 0;
    int timeout_ms = 120000;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    bool broken = false;
    std::vector<Slot> slot;
};

namespace {

// host barrier of the in-process group; PMC_ERR_HIP when a rank failed or the wait timed out (a
// rank that never arrives must not hang the others: the group is marked broken)
int group_barrier(pmc_local_group* g) {
    std::unique_lock<std::mutex> lk(g->m);
    if (g->broken) return fail(PMC_ERR_HIP, "local group: another rank failed");
    const uint64_t gen = g->generation;
    if (++g->arrived == g->world) {
        g->arrived = 0;
        ++g->generation;
        g->cv.notify_all();
        return PMC_OK;
    }
    const bool ok = g->cv.wait_for(lk, std::chrono::milliseconds(g->timeout_ms),
                                   [&] { return g->generation != gen || g->broken; });
    if (!ok || g->broken) {
        g->broken = true;
        g->cv.notify_all();
        return fail(PMC_ERR_HIP, ok ? "local group: another rank failed" : "local group: barrier timed out");
    }
    return PMC_OK;
}

void group_break(pmc_local_group* g) {
    std::lock_guard<std::mutex> lk(g->m);
    g->broken = true;
    g->cv.notify_all();
}

}  // namespace

// IPC transport: the symmetric buffers a peer maps, and the layout of the flags buffer (u64 slots;
// each flag on its own 128-B line)
constexpr int kIpcBufs = 7;               // disk[0], disk[1], n[0], n[1], send_d, send_n, xflags
constexpr int kFlagReady = 0, kFlagPulled = 16, kFlagDone = 32, kFlagRed = 48, kFlagGather = 64;
constexpr size_t kFlagBytes = sizeof(uint64_t) * (kFlagGather + 8 * kXferMax);

struct pmc_slab {
    int rank = 0, world = 1, below = 0, above = 0;
    ncclComm_t comm = nullptr;            // RCCL transport
    pmc_local_group* group = nullptr;     // in-process transport (not owned)
    hipStream_t aux = nullptr;            // halo exchanges ("T")
    hipStream_t hi[2] = {nullptr, nullptr};   // interior chains 1 and 2 (chain 0 runs on the context stream)
    int chains = 2;                       // interior plane chains (streams running subsweeps): 1, 2 or 3
    hipEvent_t ev_i = nullptr, ev_b = nullptr, ev_t = nullptr;
    hipEvent_t ev_x = nullptr;            // T after its latest exchange
    static constexpr int kB = 3;          // chain index of the boundary chain (T)
    hipEvent_t ev_run[4][2] = {};         // [interior chain 0..2, boundary][parity]
    std::vector<hipEvent_t*> run_events() {
        std::vector<hipEvent_t*> v;
        for (auto& r : ev_run)
            for (auto& e : r) v.push_back(&e);
        return v;
    }
    std::vector<XferMsg> sends, recvs;    // the exchange being assembled
    // two-plane halos (pmc_params.halo = 2, slab_sweep_h2): the shifted send planes (the context's:
    // planes 0, 1 then nz-2, nz-1, with their counts) and the counters the redundant visits of the
    // neighbour's boundary plane add to (never read)
    float* send_d = nullptr;
    int16_t* send_n = nullptr;
    unsigned long long* stats_scratch = nullptr;
    hipEvent_t ev_hp = nullptr;           // T after a boundary plane it shifted itself
    // a z-shift's halo plane not yet exchanged (deferred, PMC_SLAB_DEFER_Z): 0 none, else the shift direction;
    // the exchange of sweep `pending_sweep`'s first run carries it (same messages plus the counts)
    int pending_zdir = 0;
    uint32_t pending_sweep = 0;
    // IPC transport: every peer's symmetric buffers (disk0, disk1, n0, n1, send_d, send_n, flags)
    // mapped into this process (this rank's own pointers for itself)
    bool ipc = false;
    struct IpcPeer {
        void* base[kIpcBufs] = {};
        std::vector<void*> opened;        // hipIpcOpenMemHandle mappings to close
    };
    std::vector<IpcPeer> peers;
    uint64_t ipc_timeout = 0;             // wait limit, ticks of the 100 MHz real-time counter
    // the latest exchange whose readers may still be pulling from this rank's buffers: the next
    // exchange waits for their "pulled" (so does ipc_settle, before host-visible points)
    uint64_t pend_seq = 0;
    std::vector<int> pend_readers;
    bool messages() const { return comm != nullptr || group != nullptr || ipc; }
};

namespace {

int ipc_settle(pmc_ctx* c);   // IPC transport: wait for the latest exchange's readers (on aux)

bool slab_is_ipc(const pmc_ctx* c) { return c->slab && c->slab->ipc; }
int slab_pending_zdir(const pmc_ctx* c) { return c->slab ? c->slab->pending_zdir : 0; }

void drop_slab(pmc_ctx* c) {
    pmc_slab* s = c->slab;
    if (!s) return;
    (void)ipc_settle(c);   // (IPC: no peer still pulls from the buffers about to be freed)
    if (s->aux) (void)hipStreamSynchronize(s->aux);
    if (s->comm && rccl().ok) (void)rccl().comm_destroy(s->comm);
    if (s->group) {
        std::lock_guard<std::mutex> lk(s->group->m);
        s->group->slot[s->rank].joined = false;
    }
    if (s->aux) (void)hipStreamDestroy(s->aux);
    for (hipStream_t h : s->hi)
        if (h) (void)hipStreamSynchronize(h);
    if (s->stats_scratch) (void)hipFree(s->stats_scratch);   // (the send planes are the context's)
    for (pmc_slab::IpcPeer& pr : s->peers)
        for (void* m : pr.opened) (void)hipIpcCloseMemHandle(m);
    for (hipEvent_t e : {s->ev_i, s->ev_b, s->ev_t, s->ev_x, s->ev_hp})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t* e : s->run_events())
        if (*e) (void)hipEventDestroy(*e);
    for (hipStream_t h : s->hi)
        if (h) (void)hipStreamDestroy(h);
    delete s;
    c->slab = nullptr;
}

// Interior plane chains of a slab of nz planes: chain j covers planes [zs[j], zs[j+1]) of the
// interior [1, nz-1); every inner border is even (a parity-q run of a chain then ends at the same
// side of each border).  Two chains split at 2*(nz/4), three at the even planes nearest 1/3 and
// 2/3 of the interior; degenerate splits of thin slabs fold into fewer chains.  Returns the count.

int slab_split(int chains, int nz, int zs[4]) {
    zs[0] = 1;
    zs[1] = zs[2] = zs[3] = nz - 1;
    if (chains == 2) {
        zs[1] = 2 * (nz / 4);
    } else if (chains == 3) {
        zs[1] = 2 * ((1 + (nz - 2) / 3 + 1) / 2);
        zs[2] = 2 * ((1 + 2 * (nz - 2) / 3 + 1) / 2);
    }
    int m = 1;
    for (int j = 1; j < chains; ++j)
        if (zs[j] >= 2 && zs[j] > zs[m - 1] && zs[j] < nz - 1) zs[m++] = zs[j];
    for (int j = m; j < 4; ++j) zs[j] = nz - 1;
    return m;
}

// order the context stream after all work of the slab driver's other streams (before the state, the
// halos or the statistics are read on it)
int slab_join(pmc_ctx* c) {
    pmc_slab* s = c->slab;
    if (!s) return PMC_OK;
    if (int rc = ipc_settle(c)) return rc;   // IPC: the peers are done reading this rank's buffers
    for (hipStream_t st : {s->aux, s->hi[0], s->hi[1]}) {
        if (!st) continue;
        hipError_t e = hipEventRecord(s->ev_b, st);
        if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, s->ev_b, 0);
        if (e != hipSuccess) return hip_fail(e, "slab join");
    }
    return PMC_OK;
}

// queue one message of the current exchange
void xfer_send(pmc_slab* s, const void* buf, size_t bytes, int peer) {
    s->sends.push_back({const_cast<void*>(buf), bytes, peer});
}
void xfer_recv(pmc_slab* s, void* buf, size_t bytes, int peer, const void* sym) {
    s->recvs.push_back({buf, bytes, peer, sym});
}

// this rank's symmetric buffers, in the order of pmc_slab::IpcPeer::base
void ipc_local_bufs(const pmc_ctx* c, const void* base[kIpcBufs], size_t bytes[kIpcBufs]) {
    const size_t db = sizeof(float) * 3 * (size_t)c->P.nmax * (size_t)c->cells, nb = sizeof(int16_t) * (size_t)c->cells;
    const size_t pf = (size_t)c->P.cps_x * c->P.cps_y * 3 * c->P.nmax, pc = (size_t)c->P.cps_x * c->P.cps_y;
    const void* b[kIpcBufs] = {c->disk[0], c->disk[1], c->n[0], c->n[1], c->send_d, c->send_n, c->xflags};
    const size_t z[kIpcBufs] = {db, db, nb, nb, c->send_d ? 4 * pf * sizeof(float) : 0,
                                c->send_n ? 4 * pc * sizeof(int16_t) : 0, c->xflags ? kFlagBytes : 0};
    for (int i = 0; i < kIpcBufs; ++i) {
        base[i] = b[i];
        bytes[i] = b[i] ? z[i] : 0;
    }
}

// the peer's copy of this rank's symmetric address `sym` (nullptr if `sym` lies in none of them)
const void* ipc_translate(const pmc_ctx* c, const pmc_slab* s, int peer, const void* sym, size_t bytes) {
    const void* base[kIpcBufs];
    size_t size[kIpcBufs];
    ipc_local_bufs(c, base, size);
    const uintptr_t a = (uintptr_t)sym;
    for (int i = 0; i < kIpcBufs; ++i) {
        const uintptr_t b = (uintptr_t)base[i];
        if (b && a >= b && a + bytes <= b + size[i] && s->peers[(size_t)peer].base[i])
            return (const char*)s->peers[(size_t)peer].base[i] + (a - b);
    }
    return nullptr;
}

int xfer_seg(XferCopy& cp, const void* src, void* dst, size_t bytes) {
    if (cp.n >= kXferMax) return fail(PMC_ERR_ARG, "IPC transport: too many messages in one exchange");
    int sh = 4;
    while (sh > 0 && ((((uintptr_t)src | (uintptr_t)dst | (uintptr_t)bytes) & ((1u << sh) - 1)) != 0)) --sh;
    cp.seg[cp.n++] = {src, dst, (uint64_t)bytes, sh};
    return PMC_OK;
}

void xfer_flag_add(XferFlags& w, const uint64_t* f, uint64_t target) {
    for (int i = 0; i < w.n; ++i)
        if (w.flag[i] == f) {
            if (target > w.target[i]) w.target[i] = target;
            return;
        }
    w.flag[w.n] = f;
    w.target[w.n++] = target;
}

const uint64_t* ipc_peer_flags(const pmc_slab* s, int p) {
    return reinterpret_cast<const uint64_t*>(s->peers[(size_t)p].base[kIpcBufs - 1]);
}

// the waits on the previous exchange's readers (pulled >= its sequence number), then none pending
void ipc_take_pending(pmc_slab* s, XferFlags& w) {
    for (int p : s->pend_readers) xfer_flag_add(w, ipc_peer_flags(s, p) + kFlagPulled, s->pend_seq);
    s->pend_readers.clear();
    s->pend_seq = 0;
}

// exchange k over IPC: ONE launch on aux (k_xfer): ready[me] = k; wait for the senders' ready >= k
// and for the previous exchange's readers' pulled; pull every message from the peer's buffer; the
// last block stores pulled[me] = k.  This exchange's readers are waited for by the next exchange or
// by ipc_settle, whichever comes first: nothing before either overwrites what they read (the sent
// planes of buffer cur are rewritten only by a later sweep's shift, after more exchanges).
int ipc_run(pmc_ctx* c, const std::vector<XferMsg>& sends, const std::vector<XferMsg>& recvs) {
    pmc_slab* s = c->slab;
    const uint64_t seq = ++c->xseq;
    XferFlags w{};
    XferCopy cp{};
    ipc_take_pending(s, w);
    for (const XferMsg& m : recvs) {
        const void* src = m.sym ? ipc_translate(c, s, m.peer, m.sym, m.bytes) : nullptr;
        if (!src) return fail(PMC_ERR_ARG, "IPC transport: a receive's source is not in a symmetric buffer");
        if (int rc = xfer_seg(cp, src, m.buf, m.bytes)) return rc;
        xfer_flag_add(w, ipc_peer_flags(s, m.peer) + kFlagReady, seq);
    }
    for (const XferMsg& m : sends)
        if (std::find(s->pend_readers.begin(), s->pend_readers.end(), m.peer) == s->pend_readers.end())
            s->pend_readers.push_back(m.peer);
    s->pend_seq = seq;
    hipError_t e = launch_xfer(cp, w, c->xflags + kFlagReady, c->xflags + kFlagPulled, seq,
                               reinterpret_cast<unsigned*>(c->xflags + kFlagDone), s->ipc_timeout, c->flags, s->aux);
    return e == hipSuccess ? PMC_OK : hip_fail(e, "IPC halo exchange");
}

// the readers of the latest exchange are done (a wait launch on aux) -- before the host or the
// context stream may read or overwrite this rank's buffers, and before teardown
int ipc_settle(pmc_ctx* c) {
    pmc_slab* s = c->slab;
    if (!s || !s->ipc || s->pend_readers.empty()) return PMC_OK;
    XferFlags w{};
    ipc_take_pending(s, w);
    hipError_t e = launch_xfer_flag(nullptr, 0, w, s->ipc_timeout, c->flags, s->aux);
    return e == hipSuccess ? PMC_OK : hip_fail(e, "IPC settle");
}

// carry the queued messages on the aux stream (RCCL group, IPC pulls, or the in-process group's copies)
int xfer_run(pmc_ctx* c) {
    pmc_slab* s = c->slab;
    std::vector<XferMsg> sends, recvs;
    sends.swap(s->sends);
    recvs.swap(s->recvs);
    if (s->ipc) return ipc_run(c, sends, recvs);
    if (s->comm) {
        Rccl& R = rccl();
        PMC_NCCL(R.group_start());
        for (const XferMsg& m : sends) PMC_NCCL(R.send(m.buf, m.bytes, ncclUint8, m.peer, s->comm, s->aux));
        for (const XferMsg& m : recvs) PMC_NCCL(R.recv(m.buf, m.bytes, ncclUint8, m.peer, s->comm, s->aux));
        PMC_NCCL(R.group_end());
        return PMC_OK;
    }
    pmc_local_group* g = s->group;
    if (!g) return fail(PMC_ERR_ARG, "slab exchange without a transport");
    pmc_local_group::Slot& me = g->slot[s->rank];
    // 1. publish the send list and an event after the work that wrote the send buffers
    hipError_t e = hipEventRecord(me.ready, s->aux);
    if (e != hipSuccess) { group_break(g); return hip_fail(e, "hipEventRecord"); }
    {
        std::lock_guard<std::mutex> lk(g->m);
        me.sends = sends;
        me.recvs = recvs;
    }
    int rc = group_barrier(g);
    if (rc) return rc;
    // 2. pull: the k-th receive from peer p copies p's k-th send to this rank (RCCL matching)
    std::vector<int> taken(g->world, 0);
    for (const XferMsg& m : recvs) {
        const pmc_local_group::Slot& src = g->slot[m.peer];
        const XferMsg* hit = nullptr;
        int k = 0;
        for (const XferMsg& sm : src.sends)
            if (sm.peer == s->rank && k++ == taken[m.peer]) { hit = &sm; break; }
        if (!hit || hit->bytes != m.bytes) {
            group_break(g);
            return fail(PMC_ERR_ARG, "local group: unmatched or mis-sized halo message");
        }
        ++taken[m.peer];
        if ((e = hipStreamWaitEvent(s->aux, src.ready, 0)) != hipSuccess ||
            (e = hipMemcpyAsync(m.buf, hit->buf, m.bytes, hipMemcpyDeviceToDevice, s->aux)) != hipSuccess) {
            group_break(g);
            return hip_fail(e, "local group: halo copy");
        }
    }
    if ((e = hipEventRecord(me.pulled, s->aux)) != hipSuccess) { group_break(g); return hip_fail(e, "hipEventRecord"); }
    // every send must be received (the slots are stable between the two barriers: a rank publishes
    // its next lists only after the second one)
    std::vector<char> readers(g->world, 0);
    for (const XferMsg& m : sends) {
        if (readers[m.peer]) continue;
        readers[m.peer] = 1;
        int want = 0, got = 0;
        for (const XferMsg& x : sends) want += x.peer == m.peer;
        for (const XferMsg& x : g->slot[m.peer].recvs) got += x.peer == s->rank;
        if (want != got) {
            group_break(g);
            return fail(PMC_ERR_ARG, "local group: a halo message was not received");
        }
    }
    if ((rc = group_barrier(g))) return rc;
    // 3. every peer that read this rank's buffers is done before the aux stream writes them again
    //    (RCCL's send completes the same way); a peer re-records `pulled` only after the next
    //    exchange's first barrier, which this rank has not reached yet
    for (int p = 0; p < g->world; ++p) {
        if (!readers[p]) continue;
        if ((e = hipStreamWaitEvent(s->aux, g->slot[p].pulled, 0)) != hipSuccess) {
            group_break(g);
            return hip_fail(e, "hipStreamWaitEvent");
        }
    }
    return PMC_OK;
}

size_t plane_floats(const pmc_ctx* c) { return (size_t)c->P.cps_x * c->P.cps_y * 3 * c->P.nmax; }
size_t plane_cells(const pmc_ctx* c) { return (size_t)c->P.cps_x * c->P.cps_y; }

// the two-plane-halo send buffer (4 planes and their counts), context-owned: the IPC transport
// exports it before the slab driver attaches
hipError_t ensure_send_planes(pmc_ctx* c) {
    hipError_t e = hipSuccess;
    if (!c->send_d) e = hipMalloc(&c->send_d, 4 * plane_floats(c) * sizeof(float));
    if (e == hipSuccess && !c->send_n) e = hipMalloc(&c->send_n, 4 * plane_cells(c) * sizeof(int16_t));
    return e;
}
// storage plane of local plane z (-halo .. -1 bottom halos, nz_local .. nz_local-1+halo top halos)
float* disk_plane(pmc_ctx* c, int z) { return c->disk[c->cur] + (size_t)(z + c->P.halo) * plane_floats(c); }
int16_t* n_plane(pmc_ctx* c, int z) { return c->n[c->cur] + (size_t)(z + c->P.halo) * plane_cells(c); }


// Strong-scaling rehearsal (PMC_XFER_DELAY_US, microseconds, default 0): after every halo exchange
// the exchange stream T is held busy for that long by a one-wave spin kernel -- the xGMI time and
// RCCL latency of a real exchange (3.1 MB each way per run at 128^2 cells per plane), which a
// one-GPU rehearsal does not pay.  Never set in production runs.
double xfer_delay_us() {
    static const double us = [] {
        const char* v = std::getenv("PMC_XFER_DELAY_US");
        return v ? std::atof(v) : 0.0;
    }();
    return us;
}

int inject_delay(pmc_slab* s) {
    const double us = xfer_delay_us();
    if (us <= 0.0) return PMC_OK;
    hipError_t e = launch_spin(us, s->aux);
    return e == hipSuccess ? PMC_OK : hip_fail(e, "injected exchange delay");
}

// End of a run of colour phases of z parity p (spec v9 groups the 8 phases of a sweep into two
// runs): during the run only the owned planes of parity p changed, and the one of them another rank
// holds as a halo is the boundary plane P_p (plane 0 for p = 0, nz-1 for p = 1).  It goes whole
// (every colour of the run touched it; counts do not change in a subsweep) to the neighbour that
// holds it -- the rank below for p = 0, above for p = 1 -- and the matching halo H_p (top for p = 0,
// bottom for p = 1) comes from the other side: one message each way, straight from and into the
// state buffer (no packing).  The next run (parity 1-p) is the first to read H_p.  A single rank
// without messages copies its own plane into its periodic halo.  On aux.
int slab_exchange_run(pmc_ctx* c, int p, bool with_counts = false, bool rows_written = false) {
    pmc_slab* s = c->slab;
    const int nz = c->P.nz_local;
    const size_t pf = plane_floats(c), pc = plane_cells(c);
    const int src = p == 0 ? 0 : nz - 1, dst = p == 0 ? nz : -1;
    if (!s->messages()) {
        // (rows_written: the boundary launches already wrote the rows into the halo: direct halo)
        if (!rows_written)
            PMC_HIP(hipMemcpyAsync(disk_plane(c, dst), disk_plane(c, src), pf * 4, hipMemcpyDeviceToDevice, s->aux));
        if (with_counts)
            PMC_HIP(hipMemcpyAsync(n_plane(c, dst), n_plane(c, src), pc * 2, hipMemcpyDeviceToDevice, s->aux));
        return inject_delay(s);
    }
    const int to = p == 0 ? s->below : s->above, from = p == 0 ? s->above : s->below;
    xfer_send(s, disk_plane(c, src), pf * 4, to);
    if (with_counts) xfer_send(s, n_plane(c, src), pc * 2, to);
    xfer_recv(s, disk_plane(c, dst), pf * 4, from, disk_plane(c, src));
    if (with_counts) xfer_recv(s, n_plane(c, dst), pc * 2, from, n_plane(c, src));
    if (int rc = xfer_run(c)) return rc;
    return inject_delay(s);
}

// both halos with their counts, halo (1 or 2) planes deep: the owned planes [0, h) go down and
// [nz-h, nz) up, the halos [nz, nz+h) come from above and [-h, 0) from below.  Sources: the state
// buffer (initialisation, restart) or, with from_send, the send buffer T shifted them into
// (two-plane halos after shiftCells: the interior chains may already be rewriting planes 1 and
// nz-2 of the state).  On aux.
int slab_exchange_full(pmc_ctx* c, bool from_send = false) {
    pmc_slab* s = c->slab;
    const int nz = c->P.nz_local, h = c->P.halo;
    const size_t pf = plane_floats(c), pc = plane_cells(c);
    const float* lo_d = from_send ? s->send_d : disk_plane(c, 0);
    const float* hi_d = from_send ? s->send_d + (size_t)h * pf : disk_plane(c, nz - h);
    const int16_t* lo_n = from_send ? s->send_n : n_plane(c, 0);
    const int16_t* hi_n = from_send ? s->send_n + (size_t)h * pc : n_plane(c, nz - h);
    const size_t db = (size_t)h * pf * 4, nb = (size_t)h * pc * 2;
    if (!s->messages()) {
        PMC_HIP(hipMemcpyAsync(disk_plane(c, nz), lo_d, db, hipMemcpyDeviceToDevice, s->aux));
        PMC_HIP(hipMemcpyAsync(n_plane(c, nz), lo_n, nb, hipMemcpyDeviceToDevice, s->aux));
        PMC_HIP(hipMemcpyAsync(disk_plane(c, -h), hi_d, db, hipMemcpyDeviceToDevice, s->aux));
        PMC_HIP(hipMemcpyAsync(n_plane(c, -h), hi_n, nb, hipMemcpyDeviceToDevice, s->aux));
        return PMC_OK;
    }
    // per peer, sends and receives match in issue order: (planes, counts) down, then up
    // (counts travel as bytes: RCCL has no 16-bit integer type)
    xfer_send(s, lo_d, db, s->below);
    xfer_send(s, lo_n, nb, s->below);
    xfer_send(s, hi_d, db, s->above);
    xfer_send(s, hi_n, nb, s->above);
    xfer_recv(s, disk_plane(c, nz), db, s->above, lo_d);
    xfer_recv(s, n_plane(c, nz), nb, s->above, lo_n);
    xfer_recv(s, disk_plane(c, -h), db, s->below, hi_d);
    xfer_recv(s, n_plane(c, -h), nb, s->below, hi_n);
    return xfer_run(c);
}

// after a shift along z in direction dir: the halo on the +dir side takes the neighbour's new
// plane next to it (the -dir side was shifted locally), on aux
int slab_exchange_zplane(pmc_ctx* c, int dir) {
    pmc_slab* s = c->slab;
    const int nz = c->P.nz_local;
    const size_t pf = plane_floats(c), pc = plane_cells(c);
    const int src = dir > 0 ? 0 : nz - 1, dst = dir > 0 ? nz : -1;   // my plane -> the -dir rank's halo
    if (!s->messages()) {
        PMC_HIP(hipMemcpyAsync(disk_plane(c, dst), disk_plane(c, src), pf * 4, hipMemcpyDeviceToDevice, s->aux));
        PMC_HIP(hipMemcpyAsync(n_plane(c, dst), n_plane(c, src), pc * 2, hipMemcpyDeviceToDevice, s->aux));
        return inject_delay(s);
    }
    const int to = dir > 0 ? s->below : s->above, from = dir > 0 ? s->above : s->below;
    xfer_send(s, disk_plane(c, src), pf * 4, to);
    xfer_send(s, n_plane(c, src), pc * 2, to);
    xfer_recv(s, disk_plane(c, dst), pf * 4, from, disk_plane(c, src));
    xfer_recv(s, n_plane(c, dst), pc * 2, from, n_plane(c, src));
    if (int rc = xfer_run(c)) return rc;
    return inject_delay(s);
}

// A deferred z-shift halo exchange (PMC_SLAB_DEFER_Z) issued now, on T (collective: every rank
// defers and flushes at the same calls).
int slab_flush_z(pmc_ctx* c) {
    pmc_slab* s = c->slab;
    if (!s || !s->pending_zdir) return PMC_OK;
    const int dir = s->pending_zdir;
    s->pending_zdir = 0;
    if (int rc = slab_exchange_zplane(c, dir)) return rc;
    // IPC: the plane it sent may be the next run's boundary plane (rewritten in place before any
    // later exchange waits for this one's readers): settle now -- this path is off the sweep's
    // critical path (a flush before a non-consecutive sweep or a host-visible call)
    return ipc_settle(c);
}

}  // namespace

extern "C" {

int pmc_comm_unique_id(unsigned char id[128]) {
    if (!id) return fail(PMC_ERR_ARG, "null argument");
    Rccl& R = rccl();
    if (!R.ok) return fail(PMC_ERR_HIP, R.err);
    ncclUniqueId u;
    PMC_NCCL(R.get_unique_id(&u));
    static_assert(sizeof(u) == 128, "ncclUniqueId size");
    std::memcpy(id, &u, 128);
    return PMC_OK;
}

}  // extern "C"

namespace {

// common part of pmc_slab_init / pmc_slab_init_local: streams, events, overflow queue, buffers
int slab_attach(pmc_ctx* c, int rank, int world, bool messages) {
    if (!c || world < 1 || rank < 0 || rank >= world) return fail(PMC_ERR_ARG, "bad argument");
    if (c->P.halo < 1) return fail(PMC_ERR_ARG, "pmc_slab_init needs a slab context (halo = 1 or 2)");
    if (c->P.nz_local < 2 || c->P.z0 != rank * c->P.nz_local || c->P.cps_z != world * c->P.nz_local)
        return fail(PMC_ERR_ARG, "slab geometry must be z0 = rank*nz_local, cps_z = world*nz_local");
    PMC_HIP(hipStreamSynchronize(c->stream));
    drop_slab(c);
    pmc_slab* s = new pmc_slab();
    c->slab = s;
    s->rank = rank;
    s->world = world;
    s->below = (rank + world - 1) % world;
    s->above = (rank + 1) % world;
    hipError_t e;
    // the boundary chain (T) is the critical path of a sweep when its small launches wait for the
    // interior chains' waves to retire: its queue gets the higher dispatch priority
    // (PMC_SLAB_PRIORITY=0 disables)
    static const bool prio = [] {
        const char* v = std::getenv("PMC_SLAB_PRIORITY");
        return !(v && std::atoi(v) == 0);
    }();
    int lo_p = 0, hi_p = 0;
    if (prio) (void)hipDeviceGetStreamPriorityRange(&lo_p, &hi_p);
    if ((e = hipStreamCreateWithPriority(&s->aux, hipStreamNonBlocking, prio ? hi_p : 0)) != hipSuccess) {
        drop_slab(c);
        return hip_fail(e, "hipStreamCreate");
    }
    std::vector<hipEvent_t*> evs = {&s->ev_i, &s->ev_b, &s->ev_t, &s->ev_x, &s->ev_hp};
    for (hipEvent_t* ev : s->run_events()) evs.push_back(ev);
    for (hipEvent_t* ev : evs)
        if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) {
            drop_slab(c);
            return hip_fail(e, "hipEventCreate");
        }
    // Interior planes in `chains` chains on as many streams (chain 0 on the context stream);
    // PMC_SLAB_CHAINS = 1, 2 or 3 (default 2).  With the exchange stream that is at most 4 streams,
    // the box's GPU_MAX_HW_QUEUES: every chain keeps a hardware queue of its own.
    {
        static const int forced = [] {
            const char* v = std::getenv("PMC_SLAB_CHAINS");
            return v ? std::atoi(v) : 0;
        }();
        s->chains = forced >= 1 && forced <= 3 ? forced : 2;
    }
    // two-plane halos: at most 2 interior chains
    if (c->P.halo == 2) {
        if (s->chains > 2) s->chains = 2;
        const size_t sb = sizeof(unsigned long long) * kStatCounters * kStatSlots;
        if ((e = ensure_send_planes(c)) != hipSuccess || (e = hipMalloc(&s->stats_scratch, sb)) != hipSuccess ||
            (e = hipMemsetAsync(s->stats_scratch, 0, sb, c->stream)) != hipSuccess) {
            drop_slab(c);
            return hip_fail(e, "hipMalloc (two-plane halos)");
        }
    }
    s->send_d = c->send_d;
    s->send_n = c->send_n;
    for (int j = 0; j + 1 < s->chains; ++j)
        if ((e = hipStreamCreateWithFlags(&s->hi[j], hipStreamNonBlocking)) != hipSuccess) {
            drop_slab(c);
            return hip_fail(e, "hipStreamCreate");
        }
    // every "latest" event starts recorded (waits on them are no-ops until real work records them)
    std::vector<hipEvent_t*> latest = {&s->ev_x};
    for (hipEvent_t* ev : s->run_events()) latest.push_back(ev);
    for (hipEvent_t* ev : latest)
        if ((e = hipEventRecord(*ev, c->stream)) != hipSuccess) {
            drop_slab(c);
            return hip_fail(e, "hipEventRecord");
        }
    // overflow queues of the other interior chains and the boundary chain (they run beside the
    // context stream's)
    for (int** q : {&c->ovf_aux, &c->ovf_b, &c->ovf_aux2})
        if (!*q && ((e = hipMalloc(q, c->ovf_bytes)) != hipSuccess ||
                    (e = hipMemsetAsync(*q, 0, c->ovf_bytes, c->stream)) != hipSuccess)) {
            drop_slab(c);
            return hip_fail(e, "hipMalloc overflow queue");
        }
    // the queues' zeroing and the initial event records complete before any stream uses them
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) {
        drop_slab(c);
        return hip_fail(e, "hipStreamSynchronize");
    }
    (void)messages;   // halo messages go straight from and into the state buffers
    return PMC_OK;
}

}  // namespace

extern "C" {

int pmc_slab_init(pmc_ctx* c, int rank, int world, const unsigned char* id) {
    if (!id && world != 1) return fail(PMC_ERR_ARG, "more than one rank needs an RCCL unique id");
    if (id && !rccl().ok) return fail(PMC_ERR_HIP, rccl().err);
    int rc = slab_attach(c, rank, world, id != nullptr);
    if (rc || !id) return rc;
    pmc_slab* s = c->slab;
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    ncclResult_t r = rccl().comm_init_rank(&s->comm, world, u, rank);
    if (r != ncclSuccess) {
        s->comm = nullptr;
        rc = nccl_fail(r, "ncclCommInitRank");
        drop_slab(c);
        return rc;
    }
    return PMC_OK;
}

int pmc_local_group_create(int world, pmc_local_group** out) {
    if (!out || world < 1) return fail(PMC_ERR_ARG, "bad argument");
    *out = nullptr;
    pmc_local_group* g = new pmc_local_group();
    g->world = world;
    g->slot.resize((size_t)world);
    for (auto& sl : g->slot) {
        hipError_t e;
        if ((e = hipEventCreateWithFlags(&sl.ready, hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&sl.pulled, hipEventDisableTiming)) != hipSuccess) {
            pmc_local_group_destroy(g);
            return hip_fail(e, "hipEventCreate");
        }
    }
    const char* t = std::getenv("PMC_LOCAL_GROUP_TIMEOUT_MS");
    if (t && std::atoi(t) > 0) g->timeout_ms = std::atoi(t);
    *out = g;
    return PMC_OK;
}

void pmc_local_group_destroy(pmc_local_group* g) {
    if (!g) return;
    for (auto& sl : g->slot) {
        if (sl.ready) (void)hipEventDestroy(sl.ready);
        if (sl.pulled) (void)hipEventDestroy(sl.pulled);
    }
    delete g;
}

int pmc_slab_init_local(pmc_ctx* c, int rank, pmc_local_group* g) {
    if (!c || !g || rank < 0 || rank >= g->world) return fail(PMC_ERR_ARG, "bad argument");
    {
        std::lock_guard<std::mutex> lk(g->m);
        if (g->slot[rank].joined) return fail(PMC_ERR_ARG, "local group: rank already attached");
    }
    int rc = slab_attach(c, rank, g->world, true);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g->m);
    g->slot[rank].joined = true;
    c->slab->group = g;
    return PMC_OK;
}

// ---- IPC transport ---------------------------------------------------------------------------
namespace {

constexpr uint32_t kIpcMagic = 0x49434d50u;   // "PMCI"
constexpr uint32_t kIpcVersion = 1;
struct IpcBlob {
    uint32_t magic, version;
    uint64_t token;                     // (pid << 32) ^ context address: the exporting process + context
    int32_t pid, device;
    int32_t cps_x, cps_y, nz_local, halo, nmax, world_hint;
    struct Buf {
        hipIpcMemHandle_t handle;
        uint64_t offset, bytes;         // the buffer inside the exported allocation
    } buf[kIpcBufs];
};
static_assert(sizeof(IpcBlob) <= PMC_IPC_HANDLE_BYTES, "IPC blob size");

uint64_t ipc_token(const pmc_ctx* c) { return ((uint64_t)(uint32_t)getpid() << 32) ^ (uint64_t)(uintptr_t)c; }

// the flags buffer: uncached device memory (every flag access goes to memory: other processes and
// other GPUs see it without cache maintenance), else fine-grained, else plain -- the first kind
// whose IPC export works
int ensure_xflags(pmc_ctx* c) {
    if (c->xflags) return PMC_OK;
    const unsigned kinds[2] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained};
    for (int k = 0; k < 3 && !c->xflags; ++k) {
        void* p = nullptr;
        hipError_t e = k < 2 ? hipExtMallocWithFlags(&p, kFlagBytes, kinds[k]) : hipMalloc(&p, kFlagBytes);
        if (e != hipSuccess) continue;
        hipIpcMemHandle_t h;
        if (hipIpcGetMemHandle(&h, p) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipFree(p);
            continue;
        }
        c->xflags = (uint64_t*)p;
        c->xflags_kind = k + 1;
    }
    if (!c->xflags) return fail(PMC_ERR_HIP, "IPC transport: no exportable device memory for the flags");
    PMC_HIP(hipMemsetAsync(c->xflags, 0, kFlagBytes, c->stream));
    PMC_HIP(hipStreamSynchronize(c->stream));
    return PMC_OK;
}

}  // namespace

int pmc_slab_ipc_handle(pmc_ctx* c, unsigned char* blob) {
    if (!c || !blob) return fail(PMC_ERR_ARG, "null argument");
    if (c->P.halo < 1) return fail(PMC_ERR_ARG, "pmc_slab_ipc_handle needs a slab context (halo = 1 or 2)");
    if (int rc = ensure_xflags(c)) return rc;
    if (c->P.halo == 2) PMC_HIP(ensure_send_planes(c));
    IpcBlob b;
    std::memset(&b, 0, sizeof b);
    b.magic = kIpcMagic;
    b.version = kIpcVersion;
    b.token = ipc_token(c);
    b.pid = (int32_t)getpid();
    PMC_HIP(hipGetDevice(&b.device));
    b.cps_x = c->P.cps_x;
    b.cps_y = c->P.cps_y;
    b.nz_local = c->P.nz_local;
    b.halo = c->P.halo;
    b.nmax = c->P.nmax;
    const void* base[kIpcBufs];
    size_t bytes[kIpcBufs];
    ipc_local_bufs(c, base, bytes);
    for (int i = 0; i < kIpcBufs; ++i) {
        if (!base[i]) continue;
        void* alloc = nullptr;
        size_t asize = 0;
        PMC_HIP(hipMemGetAddressRange(&alloc, &asize, const_cast<void*>(base[i])));
        PMC_HIP(hipIpcGetMemHandle(&b.buf[i].handle, alloc));
        b.buf[i].offset = (uint64_t)((uintptr_t)base[i] - (uintptr_t)alloc);
        b.buf[i].bytes = bytes[i];
    }
    std::memset(blob, 0, PMC_IPC_HANDLE_BYTES);
    std::memcpy(blob, &b, sizeof b);
    return PMC_OK;
}

int pmc_slab_init_ipc(pmc_ctx* c, int rank, int world, const unsigned char* blobs) {
    if (!c || !blobs || world < 1 || rank < 0 || rank >= world) return fail(PMC_ERR_ARG, "bad argument");
    if (world > kXferMax) return fail(PMC_ERR_ARG, "IPC transport: at most 16 ranks");
    std::vector<IpcBlob> bl((size_t)world);
    for (int p = 0; p < world; ++p) {
        std::memcpy(&bl[(size_t)p], blobs + (size_t)p * PMC_IPC_HANDLE_BYTES, sizeof(IpcBlob));
        const IpcBlob& b = bl[(size_t)p];
        if (b.magic != kIpcMagic || b.version != kIpcVersion)
            return fail(PMC_ERR_ARG, "IPC transport: not a pmc_slab_ipc_handle blob");
        if (b.cps_x != c->P.cps_x || b.cps_y != c->P.cps_y || b.nz_local != c->P.nz_local || b.halo != c->P.halo ||
            b.nmax != c->P.nmax)
            return fail(PMC_ERR_ARG, "IPC transport: the ranks' slab geometries differ");
    }
    if (!c->xflags || bl[(size_t)rank].token != ipc_token(c))
        return fail(PMC_ERR_ARG, "IPC transport: blob[rank] is not this context's pmc_slab_ipc_handle");
    int rc = slab_attach(c, rank, world, true);
    if (rc) return rc;
    pmc_slab* s = c->slab;
    s->peers.assign((size_t)world, pmc_slab::IpcPeer{});
    const void* mine[kIpcBufs];
    size_t mine_bytes[kIpcBufs];
    ipc_local_bufs(c, mine, mine_bytes);
    for (int p = 0; p < world; ++p) {
        const IpcBlob& b = bl[(size_t)p];
        pmc_slab::IpcPeer& pr = s->peers[(size_t)p];
        if (b.token == ipc_token(c)) {            // this context itself (a one-rank IPC rehearsal)
            for (int i = 0; i < kIpcBufs; ++i) pr.base[i] = const_cast<void*>(mine[i]);
            continue;
        }
        if (b.pid == (int32_t)getpid()) {
            drop_slab(c);
            return fail(PMC_ERR_ARG, "IPC transport: two ranks in one process (use pmc_slab_init_local)");
        }
        std::vector<std::pair<std::string, void*>> seen;   // one mapping per exported allocation
        for (int i = 0; i < kIpcBufs; ++i) {
            if (!b.buf[i].bytes) continue;
            if (b.buf[i].bytes != mine_bytes[i]) {
                drop_slab(c);
                return fail(PMC_ERR_ARG, "IPC transport: a peer's buffer sizes differ");
            }
            const std::string key(reinterpret_cast<const char*>(&b.buf[i].handle), sizeof(hipIpcMemHandle_t));
            void* m = nullptr;
            for (auto& kv : seen)
                if (kv.first == key) m = kv.second;
            if (!m) {
                hipError_t e = hipIpcOpenMemHandle(&m, b.buf[i].handle, hipIpcMemLazyEnablePeerAccess);
                if (e != hipSuccess) {
                    drop_slab(c);
                    return hip_fail(e, "hipIpcOpenMemHandle (IPC transport)");
                }
                pr.opened.push_back(m);
                seen.emplace_back(key, m);
            }
            pr.base[i] = (char*)m + b.buf[i].offset;
        }
        if (!pr.base[kIpcBufs - 1]) {
            drop_slab(c);
            return fail(PMC_ERR_ARG, "IPC transport: a peer exported no flags");
        }
    }
    static const double timeout_s = [] {
        const char* v = std::getenv("PMC_IPC_TIMEOUT_S");
        const double t = v ? std::atof(v) : 0.0;
        return t > 0.0 ? t : 60.0;
    }();
    s->ipc_timeout = (uint64_t)(timeout_s * 1e8);
    s->ipc = true;
    return PMC_OK;
}

int pmc_slab_exchange(pmc_ctx* c) {
    if (!c || !c->slab) return fail(PMC_ERR_ARG, "no slab driver (pmc_slab_init)");
    pmc_slab* s = c->slab;
    s->pending_zdir = 0;   // both halos with their counts below: a deferred z exchange is subsumed
    // everything before (state set up on the context stream, earlier sweeps on all three streams)
    // is ordered before the exchange and before every stream's next work
    int rc = slab_join(c);
    if (rc) return rc;
    PMC_HIP(hipEventRecord(s->ev_i, c->stream));
    PMC_HIP(hipStreamWaitEvent(s->aux, s->ev_i, 0));
    for (hipStream_t h : {s->hi[0], s->hi[1]})
        if (h) PMC_HIP(hipStreamWaitEvent(h, s->ev_i, 0));
    if ((rc = slab_exchange_full(c))) return rc;
    // IPC: the sent planes are rewritten in place by the next sweep's first runs (boundary and, with
    // two-plane halos, interior chains on other streams) before any later exchange: settle now
    if ((rc = ipc_settle(c))) return rc;
    PMC_HIP(hipEventRecord(s->ev_t, s->aux));
    PMC_HIP(hipStreamWaitEvent(c->stream, s->ev_t, 0));
    for (hipStream_t h : {s->hi[0], s->hi[1]})
        if (h) PMC_HIP(hipStreamWaitEvent(h, s->ev_t, 0));
    PMC_HIP(hipEventRecord(s->ev_x, s->aux));
    for (hipEvent_t* ev : s->run_events()) PMC_HIP(hipEventRecord(*ev, s->aux));
    return PMC_OK;
}

}  // extern "C"

namespace {

// Two-plane halos (pmc_params.halo = 2): ONE exchange per sweep, after shiftCells, instead of one
// per run.  A rank stores two halo planes on each side.  In a sweep's first run (parity a) the
// halo plane of parity a -- the neighbour's boundary plane P_a, top halo nz for a = 0, bottom halo
// -1 for a = 1 -- is visited here as well, redundantly, in the same launches as our boundary plane
// P_a on T (k_subsweep_direct2: the two planes lie at opposite faces): its cells read only
// our boundary plane and the second halo plane beyond it, which no phase of that run changes, and
// its random numbers, cell centre and staging are the owner's (global cell ids), so the result is
// the owner's bit for bit (its counters go to a scratch buffer: the owner counts them).  The second
// run's boundary plane P_b reads exactly that halo, so no exchange is needed between the runs.
// After the two runs the other halos are stale; shiftCells of the owned planes needs only the
// halo on its dir side along z, which is the fresh one unless (a = 0 and dir < 0) or (a = 1 and
// dir > 0): then ONE plane is exchanged first (slab_exchange_run of the second run's parity) and T
// shifts the plane that reads it.  T also shifts the four planes the neighbours need (0, 1, nz-2,
// nz-1) into a send buffer -- the interior chains may rewrite planes 1 and nz-2 while the exchange
// is in flight -- and exchanges all four halo planes with their counts.  The next sweep's interior
// chains read no halo, so they start right after the shift; only T (its boundary and halo planes)
// waits for the exchange.  Streams: S + one interior stream, T.
int slab_sweep_h2(pmc_ctx* c, uint32_t sweep) {
    pmc_slab* s = c->slab;
    hipStream_t S = c->stream, T = s->aux;
    const int nz = c->P.nz_local;
    int zs[4];
    const int nc = slab_split(s->chains, nz, zs);   // <= 2 chains
    hipStream_t ist[2] = {S, s->hi[0]};
    int* iovf[2] = {c->ovf, c->ovf_aux};
    const pmc_sweep_plan_t plan = pmc_plan_for_sweep_ex(c->P.seed, sweep, c->P.w, c->P.flags);
    const int a = plan.order[0] % 2, b = 1 - a;
    for (int k = 1; k < 8; ++k)
        if (plan.order[k] % 2 != (k < 4 ? a : b))
            return fail(PMC_ERR_ARG, "two-plane halos need the grouped colour order (two runs per sweep)");
    constexpr int kB = pmc_slab::kB, kR = 2;             // ev_run rows: chains 0-1, the halo plane, T
    const int pa = a == 0 ? 0 : nz - 1, pb = b == 0 ? 0 : nz - 1;   // boundary planes of the runs
    const int za = a == 0 ? nz : -1;                     // the halo plane T also visits in run a
    auto phases = [&](hipStream_t st, int* ovf, unsigned long long* stats, int z0, int z1, int k0, int k1,
                      bool plane) -> int {
        for (int kk = k0; kk < k1; ++kk) {
            int o[3];
            pmc_colour_offset(plan.order[kk], o);
            LaunchTiming lt;
            hipError_t le = plane ? launch_subsweep_plane(c->G, c->disk[c->cur], c->n[c->cur], o[0], o[1], o[2], sweep,
                                                          stats, ovf, z0, st, stats == c->stats ? next_timing(c, 2, &lt) : nullptr)
                                  : launch_subsweep(c->G, c->disk[c->cur], c->n[c->cur], o[0], o[1], o[2], sweep, stats,
                                                    ovf, z0, z1, st, next_timing(c, 0, &lt));
            if (le != hipSuccess) return hip_fail(le, "subsweep launch");
        }
        return PMC_OK;
    };
    auto owner = [&](int z) {
        if (z == 0 || z == nz - 1) return kB;
        if (z == za) return kR;
        int j = 0;
        while (j + 1 < nc && z >= zs[j + 1]) ++j;
        return j;
    };
    // run b waits for the run-a owners of the planes next to the ones a chain writes
    auto waits_b = [&](int chain, int z0, int z1, hipStream_t st) -> int {
        bool need[4] = {false, false, false, false};
        for (int z = z0; z < z1; ++z) {
            if ((z & 1) != b) continue;
            for (int zn : {z - 1, z + 1})
                if (zn >= -1 && zn <= nz && owner(zn) != chain && (zn >= 0 && zn < nz ? true : zn == za))
                    need[owner(zn)] = true;
        }
        for (int j = 0; j < 4; ++j)
            if (need[j]) PMC_HIP(hipStreamWaitEvent(st, s->ev_run[j][a], 0));
        return PMC_OK;
    };
    int rc;
    // ---- run a: T the boundary plane and the halo plane of parity a as ONE launch per phase
    // (k_subsweep_direct2: the two planes lie at opposite faces), the interior chains --------------
    // (round 4 also had the halo plane on a stream of its own: slower, removed)
    {
        const int z0 = pa < za ? pa : za, z1 = pa < za ? za : pa;
        unsigned long long* s0 = z0 == pa ? c->stats : s->stats_scratch;
        unsigned long long* s1 = z0 == pa ? s->stats_scratch : c->stats;
        for (int kk = 0; kk < 4; ++kk) {
            int o[3];
            pmc_colour_offset(plan.order[kk], o);
            LaunchTiming lt;
            hipError_t le = launch_subsweep_planes2(c->G, c->disk[c->cur], c->n[c->cur], o[0], o[1], o[2], sweep, s0, s1,
                                                    c->ovf_b, z0, z1, T, next_timing(c, 2, &lt));
            if (le != hipSuccess) return hip_fail(le, "subsweep launch (two planes)");
        }
        PMC_HIP(hipEventRecord(s->ev_run[kB][a], T));
        PMC_HIP(hipEventRecord(s->ev_run[kR][a], T));      // (the halo plane is T's too)
    }
    for (int j = 0; j < nc; ++j) {
        if (zs[j + 1] > zs[j] && (rc = phases(ist[j], iovf[j], c->stats, zs[j], zs[j + 1], 0, 4, false))) return rc;
        PMC_HIP(hipEventRecord(s->ev_run[j][a], ist[j]));
    }
    // ---- run b: T the other boundary plane (it reads R's halo plane), the interior chains -------
    if ((rc = waits_b(kB, pb, pb + 1, T))) return rc;
    if ((rc = phases(T, c->ovf_b, c->stats, pb, pb + 1, 4, 8, true))) return rc;
    PMC_HIP(hipEventRecord(s->ev_run[kB][b], T));
    for (int j = 0; j < nc; ++j) {
        if ((rc = waits_b(j, zs[j], zs[j + 1], ist[j]))) return rc;
        if (zs[j + 1] > zs[j] && (rc = phases(ist[j], iovf[j], c->stats, zs[j], zs[j + 1], 4, 8, false))) return rc;
        PMC_HIP(hipEventRecord(s->ev_run[j][b], ist[j]));
    }
    // ---- shiftCells --------------------------------------------------------------------------
    const int dir = plan.d <= 0.0f ? -1 : 1;
    const bool stale = plan.f == 2 && ((a == 0 && dir < 0) || (a == 1 && dir > 0));
    const int hp = dir < 0 ? 0 : nz - 1;                 // (stale) the plane that reads the stale halo
    // T: the stale halo first (the neighbour's second-run boundary plane), then the send planes
    if (stale && (rc = slab_exchange_run(c, b))) return rc;
    for (int j = 0; j < nc; ++j) PMC_HIP(hipStreamWaitEvent(T, s->ev_run[j][b], 0));
    PMC_HIP(hipStreamWaitEvent(T, s->ev_run[kR][a], 0));
    // S: every owned plane (but hp when T shifts it), after every chain, R and T's second run
    for (int j = 1; j < nc; ++j) PMC_HIP(hipStreamWaitEvent(S, s->ev_run[j][b], 0));
    PMC_HIP(hipStreamWaitEvent(S, s->ev_run[kR][a], 0));
    PMC_HIP(hipStreamWaitEvent(S, s->ev_run[kB][b], 0));
    float* dn = c->disk[c->cur ^ 1];
    int16_t* nn = c->n[c->cur ^ 1];
    const float* din = c->disk[c->cur];
    const int16_t* nin = c->n[c->cur];
    LaunchTiming lts;
    hipError_t e = launch_shift_planes(c->G, din, nin, dn, nn, plan.f, plan.d, c->flags, stale && hp == 0 ? 1 : 0,
                                       stale && hp == nz - 1 ? nz - 1 : nz, S, next_timing(c, 1, &lts));
    if (e != hipSuccess) return hip_fail(e, "shift launch");
    if (stale) {
        e = launch_shift_planes(c->G, din, nin, dn, nn, plan.f, plan.d, c->flags, hp, hp + 1, T, nullptr);
        if (e != hipSuccess) return hip_fail(e, "shift launch (boundary)");
        PMC_HIP(hipEventRecord(s->ev_hp, T));
    }
    // the send planes: shiftCells of planes [0, 2) and [nz-2, nz) again, into the send buffer (the
    // kernel addresses its output by storage plane: the base is offset so plane 0 / nz-2 lands at
    // the buffer's start / third plane) -- IPC: after the previous sweep's readers pulled from it
    if ((rc = ipc_settle(c))) return rc;
    {
        const int h = c->P.halo;
        const ptrdiff_t pf = (ptrdiff_t)plane_floats(c), pc = (ptrdiff_t)plane_cells(c);
        for (int part = 0; part < 2; ++part) {
            const int z0 = part == 0 ? 0 : nz - 2;
            float* bd = reinterpret_cast<float*>(reinterpret_cast<uintptr_t>(s->send_d) +
                                                 (uintptr_t)((2 * part - z0 - h) * pf * (ptrdiff_t)sizeof(float)));
            int16_t* bn = reinterpret_cast<int16_t*>(reinterpret_cast<uintptr_t>(s->send_n) +
                                                     (uintptr_t)((2 * part - z0 - h) * pc * (ptrdiff_t)sizeof(int16_t)));
            e = launch_shift_planes(c->G, din, nin, bd, bn, plan.f, plan.d, c->flags, z0, z0 + 2, T, nullptr);
            if (e != hipSuccess) return hip_fail(e, "shift launch (send planes)");
        }
    }
    c->cur ^= 1;
    // ---- the sweep's exchange: all four halo planes with their counts, from the send buffer ----
    if ((rc = slab_exchange_full(c, true))) return rc;
    if ((rc = inject_delay(s))) return rc;
    PMC_HIP(hipEventRecord(s->ev_x, T));
    // the next sweep: the interior chains after the shift (they read no halo), T and R after it too
    // (their planes read the shifted owned planes); R also after the exchange (ev_x, next run a);
    // the chain next to a boundary plane T shifted also after that
    PMC_HIP(hipEventRecord(s->ev_i, S));
    for (int j = 1; j < nc; ++j) PMC_HIP(hipStreamWaitEvent(ist[j], s->ev_i, 0));
    PMC_HIP(hipStreamWaitEvent(T, s->ev_i, 0));
    if (stale) {
        const int zn = hp == 0 ? 1 : nz - 2;              // the owned plane next to hp
        const int j = owner(zn);
        if (zn >= 0 && zn < nz && j < nc) PMC_HIP(hipStreamWaitEvent(ist[j], s->ev_hp, 0));
    }
    return PMC_OK;
}

}  // namespace

extern "C" {

#ifndef PMC_SLAB_INTERLEAVE
#define PMC_SLAB_INTERLEAVE 1   // pmc_slab_sweep issues a run phase by phase across the chains (0: chain by chain)
#endif
int pmc_slab_sweep(pmc_ctx* c, uint32_t sweep) {
    if (!c || !c->slab) return fail(PMC_ERR_ARG, "no slab driver (pmc_slab_init)");
    if (c->P.halo == 2) return slab_sweep_h2(c, sweep);
    pmc_slab* s = c->slab;
    hipStream_t S = c->stream, T = s->aux;
    const int nz = c->P.nz_local;
    // interior planes [1, nz-1) in nc chains: chain j = planes [zs[j], zs[j+1]) on stream ist[j]
    // (chain 0 on the context stream S); every inner border zs[j] is even, so every parity-q run
    // of a chain ends at the same side of each border
    int zs[4];
    const int nc = slab_split(s->chains, nz, zs);
    hipStream_t ist[3] = {S, s->hi[0], s->hi[1]};
    int* iovf[3] = {c->ovf, c->ovf_aux, c->ovf_aux2};
    const pmc_sweep_plan_t plan = pmc_plan_for_sweep_ex(c->P.seed, sweep, c->P.w, c->P.flags);
    int rc;
    // a deferred z-shift halo exchange: carried by this sweep's first run exchange when this is the
    // sweep it was deferred to (the first run's boundary plane does not read that halo), else now
    bool merge_z = false;
    if (s->pending_zdir) {
        if (sweep == s->pending_sweep) merge_z = true;
        else if ((rc = slab_flush_z(c))) return rc;
    }
    // The 8 colour phases form runs of equal z parity q (two runs of 4 with the default plan).  In a
    // run only the planes of parity q change, each reading its own plane and the parity 1-q planes
    // next to it, which no phase of the run writes and no halo of the run changes: every plane's
    // chain of phases is independent of the other planes' for the whole run.  So each run is
    // nc + 1 independent chains of launches:
    //   interior chain j (stream ist[j]; j = 0 on the context stream S): the run's phases on the
    //     interior planes [zs[j], zs[j+1]);
    //   B (exchange stream T): the run's phases on the boundary plane P_q (plane 0 for q = 0, nz-1
    //     for q = 1) -- the only plane of the run that reads a halo (H_{1-q}, received by T at the end
    //     of the previous run) and that another rank holds as a halo -- then the exchange: P_q whole to
    //     the neighbour holding it, H_q from the other side (slab_exchange_run), one message each way.
    // The chains' launch gaps and tails overlap each other's work, and the exchange overlaps them.
    // The chains synchronise only at run boundaries, where a run's reads cross a chain border (the
    // borders are even: a parity-q plane next to a border reads the plane across it, which the other
    // chain wrote in its previous run of parity 1-q): each waits for the owner chain's previous run
    // (an event per chain and parity; border_waits derives the set from the plane ownership, so any
    // number of interior chains, or none, works the same way).  Those are also the only readers of
    // the planes a run overwrites, so the same waits order every overwrite after its readers.  Cells
    // of a colour are independent, so any split of a phase gives the whole-box result bit for bit
    // (the GPU tests compare every world size and chain count with the oracle's whole box).
    constexpr int kB = pmc_slab::kB;
    int k = 0;
    // One rank without messages (the periodic single-rank slab, the strong-scaling rehearsal):
    // PMC_SLAB_DIRECT_HALO=1 lets the boundary launches write each row they store into the halo
    // plane that holds its periodic image as well (mirror mode 1), so the run's exchange copies
    // nothing -- the one-GPU form of device-initiated halo writes
    static const bool direct_halo_env = [] {
        const char* v = std::getenv("PMC_SLAB_DIRECT_HALO");
        return v && std::atoi(v) == 1;
    }();
    // (not with quirks R1/R2: their full-capacity path writes no mirror rows)
    const bool direct_halo = direct_halo_env && !s->messages() &&
                             !(c->P.flags & (PMC_FLAG_QUIRK_R1 | PMC_FLAG_QUIRK_R2));
    auto phases = [&](hipStream_t st, int* ovf, int z0, int z1, int k0, int k1, bool boundary) -> int {
        float* mir = nullptr;
        if (boundary && direct_halo) mir = disk_plane(c, z0 == 0 ? nz : -1);   // plane 0 -> top halo, nz-1 -> bottom
        for (int kk = k0; kk < k1; ++kk) {
            int o[3];
            pmc_colour_offset(plan.order[kk], o);
            LaunchTiming lt;
            hipError_t le = boundary
                ? launch_subsweep_boundary(c->G, c->disk[c->cur], c->n[c->cur], o[0], o[1], o[2], sweep, c->stats,
                                           ovf, z0, z1, mir, mir ? 1 : 0, st, next_timing(c, 2, &lt))
                : launch_subsweep(c->G, c->disk[c->cur], c->n[c->cur], o[0], o[1], o[2], sweep, c->stats, ovf, z0,
                                  z1, st, next_timing(c, 0, &lt));   // every interior chain: kind 0
            if (le != hipSuccess) return hip_fail(le, "subsweep launch");
        }
        return PMC_OK;
    };
    // owner chain of owned plane z; the planes a chain writes in a run of parity q and the other
    // chains owning a plane next to one of them (those it waits for; halos are T's own business)
    auto owner = [&](int z) {
        if (z == 0 || z == nz - 1) return kB;
        int j = 0;
        while (j + 1 < nc && z >= zs[j + 1]) ++j;
        return j;
    };
    auto border_waits = [&](int chain, int z0, int z1, int q, hipStream_t st, int parity) -> int {
        bool need[4] = {false, false, false, false};
        for (int z = z0; z < z1; ++z) {
            if ((z & 1) != q) continue;
            for (int zn : {z - 1, z + 1})
                if (zn >= 0 && zn < nz && owner(zn) != chain) need[owner(zn)] = true;
        }
        for (int j = 0; j < 4; ++j)
            if (need[j]) PMC_HIP(hipStreamWaitEvent(st, s->ev_run[j][parity], 0));
        return PMC_OK;
    };
    while (k < 8) {
        const int q = plan.order[k] % 2;                          // itoa: offset[2] = colour % 2
        int k1 = k;
        while (k1 < 8 && plan.order[k1] % 2 == q) ++k1;           // run [k, k1)
        const int p = 1 - q;                                      // parity of the previous run
        // the sweep's first run needs no border waits: the previous sweep's shift joined every
        // chain, and the other streams wait for it (a stream wait costs a barrier packet on the
        // critical path)
        const bool first = k == 0;
        // B, then the exchange -- issued first: the boundary chain (its phases, the exchange, the
        // next run's phases) is the sweep's critical path, so its work reaches the GPU first.  (The
        // issue order inside a run does not change the dependencies: every wait refers to events of
        // the previous run.)
        // (PMC_SLAB_B_FIRST=0: the interior chains first, round 3's order, for A/B)
        static const bool b_first = [] {
            const char* v = std::getenv("PMC_SLAB_B_FIRST");
            return !(v && std::atoi(v) == 0);
        }();
        auto boundary = [&]() -> int {
            const int zb = q == 0 ? 0 : nz - 1;
            int r;
            if (!first && (r = border_waits(kB, zb, zb + 1, q, T, p))) return r;
            if ((r = phases(T, c->ovf_b, zb, zb + 1, k, k1, true))) return r;
            PMC_HIP(hipEventRecord(s->ev_run[kB][q], T));
            if ((r = slab_exchange_run(c, q, merge_z, direct_halo))) return r;
            merge_z = false;
            s->pending_zdir = 0;
            return PMC_OK;
        };
#if PMC_SLAB_INTERLEAVE
        // Issue order phase by phase across the chains (B's phase, then each interior chain's), B's
        // exchange right after its last phase.  The host issues a rank sweep in about the time the
        // GPU runs it (8 ranks: 16-plane slabs), so chain by chain (B's 4 phases and exchange, then
        // all of L, then all of U) left the last chain's first launch ~10 API calls behind the
        // others' every run (kernel trace: U started as L's run was ending, profiles/r06a_*).
        if (!first) {
            const int zb = q == 0 ? 0 : nz - 1;
            if ((rc = border_waits(kB, zb, zb + 1, q, T, p))) return rc;
            for (int j = 0; j < nc; ++j)
                if ((rc = border_waits(j, zs[j], zs[j + 1], q, ist[j], p))) return rc;
        }
        for (int kk = k; kk < k1; ++kk) {
            const int zb = q == 0 ? 0 : nz - 1;
            if ((rc = phases(T, c->ovf_b, zb, zb + 1, kk, kk + 1, true))) return rc;
            if (kk == k1 - 1) {
                PMC_HIP(hipEventRecord(s->ev_run[kB][q], T));
                if ((rc = slab_exchange_run(c, q, merge_z, direct_halo))) return rc;
                merge_z = false;
                s->pending_zdir = 0;
            }
            for (int j = 0; j < nc; ++j)
                if (zs[j + 1] > zs[j] && (rc = phases(ist[j], iovf[j], zs[j], zs[j + 1], kk, kk + 1, false))) return rc;
        }
        for (int j = 0; j < nc; ++j) PMC_HIP(hipEventRecord(s->ev_run[j][q], ist[j]));
        (void)b_first;
        (void)boundary;
#else
        if (b_first && (rc = boundary())) return rc;
        for (int j = 0; j < nc; ++j) {
            if (!first && (rc = border_waits(j, zs[j], zs[j + 1], q, ist[j], p))) return rc;
            if (zs[j + 1] > zs[j] && (rc = phases(ist[j], iovf[j], zs[j], zs[j + 1], k, k1, false))) {
                return rc;
            }
            PMC_HIP(hipEventRecord(s->ev_run[j][q], ist[j]));
        }
        if (!b_first && (rc = boundary())) return rc;
#endif
        k = k1;
    }
    // after the 8 phases both halo planes are exact copies of the neighbours' planes, so
    // every halo plane whose new content depends only on planes this rank holds is shifted here,
    // bit-identical to its owner's result.  Along x or y that is both halo planes (no exchange at
    // all); along z in direction dir, the halo on the -dir side (it takes particles from the owned
    // plane next to it), and the other one is received: one plane with its counts, one direction.
    int zl0, zl1;
    const int dir = slab_shift_planes(nz, plan, &zl0, &zl1);
    // Split shift (default; PMC_SLAB_SPLIT_SHIFT=0 off; shifts along x or y): of all the shift's output planes
    // only the halo H_q the LAST run's exchange fills reads that exchange (along x/y an output plane
    // reads only itself).  The context stream S shifts every other plane as soon as the interior
    // chains and the boundary chain's last phases are done -- not waiting for the exchange -- and T
    // shifts H_q after it: the exchange leaves the sweep's critical path (it matters once the
    // exchange takes xGMI time: PMC_XFER_DELAY_US rehearsals).  The next sweep's interior chains
    // read no halo; T, which runs the next boundary phases, is in order after its own part.
    static const bool split_env = [] {   // default on (PMC_SLAB_SPLIT_SHIFT=0: off)
        const char* v = std::getenv("PMC_SLAB_SPLIT_SHIFT");
        return !(v && std::atoi(v) == 0);
    }();
    const int q_last = plan.order[7] % 2;
    const int hq = q_last == 0 ? nz : -1;                    // the halo the last exchange fills
    const bool split = split_env && plan.f != 2 && hq >= zl0 && hq < zl1;
    for (int j = 1; j < nc; ++j) {
        PMC_HIP(hipEventRecord(s->ev_b, ist[j]));
        PMC_HIP(hipStreamWaitEvent(S, s->ev_b, 0));
    }
    LaunchTiming lts;
    hipError_t e;
    if (split) {
        // S after B's last phases (ev_run[kB][q_last]: recorded on T after every earlier exchange)
        PMC_HIP(hipStreamWaitEvent(S, s->ev_run[kB][q_last], 0));
        const int a0 = hq == -1 ? 0 : zl0, a1 = hq == -1 ? zl1 : nz;
        e = launch_shift_planes(c->G, c->disk[c->cur], c->n[c->cur], c->disk[c->cur ^ 1], c->n[c->cur ^ 1], plan.f,
                                plan.d, c->flags, a0, a1, S, next_timing(c, 1, &lts));
        if (e != hipSuccess) return hip_fail(e, "shift launch");
        e = launch_shift_planes(c->G, c->disk[c->cur], c->n[c->cur], c->disk[c->cur ^ 1], c->n[c->cur ^ 1], plan.f,
                                plan.d, c->flags, hq, hq + 1, T, nullptr);
        if (e != hipSuccess) return hip_fail(e, "shift launch (halo)");
    } else {
        // shiftCells reads every plane and both halos: the other chains and T joined into S
        PMC_HIP(hipEventRecord(s->ev_x, T));
        PMC_HIP(hipStreamWaitEvent(S, s->ev_x, 0));
        e = launch_shift_planes(c->G, c->disk[c->cur], c->n[c->cur], c->disk[c->cur ^ 1], c->n[c->cur ^ 1], plan.f,
                                plan.d, c->flags, zl0, zl1, S, next_timing(c, 1, &lts));
        if (e != hipSuccess) return hip_fail(e, "shift launch");
    }
    c->cur ^= 1;
    // the other chains and T continue after the shift (it rewrote every plane); the z halo arrives
    // on T, overlapping the next sweep's first interior launches (they read no halo).  The next
    // sweep's first run waits for nothing else (no border waits), so no "previous run" event is
    // recorded here.
    PMC_HIP(hipEventRecord(s->ev_i, S));
    for (int j = 1; j < nc; ++j) PMC_HIP(hipStreamWaitEvent(ist[j], s->ev_i, 0));
    PMC_HIP(hipStreamWaitEvent(T, s->ev_i, 0));
    // After a shift along z in direction dir the halo on the +dir side is received: the neighbour's
    // new plane next to it (plane 0 of the rank above for dir > 0, its top plane nz-1 of the rank
    // below for dir < 0) -- exactly the plane that neighbour sends as the boundary plane of its
    // run of parity 0 (dir > 0) or 1 (dir < 0) after that run.  Default on (PMC_SLAB_DEFER_Z=0: off): when the next
    // sweep's first run is that parity, its boundary plane reads only the other halo (the
    // interior chains read none), so this exchange is skipped and the first run's exchange brings
    // the plane -- with its counts -- one run later: one exchange (xGMI latency) less on the
    // exchange stream's chain.  Any other next call flushes it first (slab_flush_z).
    static const bool defer_env = [] {   // default on (PMC_SLAB_DEFER_Z=0: off)
        const char* v = std::getenv("PMC_SLAB_DEFER_Z");
        return !(v && std::atoi(v) == 0);
    }();
    if (dir != 0) {
        const pmc_sweep_plan_t next = pmc_plan_for_sweep_ex(c->P.seed, sweep + 1, c->P.w, c->P.flags);
        const int q_next = next.order[0] % 2;
        if (defer_env && q_next == (dir > 0 ? 0 : 1)) {
            s->pending_zdir = dir;
            s->pending_sweep = sweep + 1;
        } else if ((rc = slab_exchange_zplane(c, dir))) {
            return rc;
        }
    }
    PMC_HIP(hipEventRecord(s->ev_x, T));
    return PMC_OK;
}

int pmc_slab_layout(pmc_ctx* c, int* n_chains, int borders[4]) {
    if (!c || !c->slab || !n_chains || !borders) return fail(PMC_ERR_ARG, "no slab driver (pmc_slab_init)");
    // (two-plane halos run at most 2 interior chains, slab_sweep_h2)
    *n_chains = slab_split(c->P.halo == 2 && c->slab->chains > 2 ? 2 : c->slab->chains, c->P.nz_local, borders);
    return PMC_OK;
}

int pmc_slab_finish(pmc_ctx* c) {
    if (!c || !c->slab) return fail(PMC_ERR_ARG, "no slab driver (pmc_slab_init)");
    if (int rc = slab_flush_z(c)) return rc;
    if (int rc = slab_join(c)) return rc;
    if (c->slab->ipc) {
        // a timed-out IPC wait (error bit 9) means some halo was not copied: the run is void
        PMC_HIP(hipStreamSynchronize(c->stream));
        uint32_t fl = 0;
        PMC_HIP(hipMemcpy(&fl, c->flags, 4, hipMemcpyDeviceToHost));
        if (fl & 512u) return fail(PMC_ERR_HIP, "IPC transport: a peer did not arrive (wait timed out, error flag 512)");
        if (fl & 1024u) return fail(PMC_ERR_HIP, "IPC transport: an XCD's L2 was not written back before ready (error flag 1024)");
    }
    return PMC_OK;
}

int pmc_slab_observables(pmc_ctx* c, int with_energy, pmc_stats* out, double* e_out) {
    if (!c || !c->slab || !out || (with_energy && !e_out)) return fail(PMC_ERR_ARG, "bad argument");
    pmc_slab* s = c->slab;
    if (int rc = slab_flush_z(c)) return rc;   // the energy reads both halos
    pmc_stats st;
    if (int rc = pmc_stats_read(c, &st, 0)) return rc;
    int64_t ef = 0;
    if (with_energy)
        if (int rc = energy_fixed(c, &ef)) return rc;
    // two's-complement sums: exact for the signed fields as 64-bit unsigned sums
    uint64_t v[5] = {(uint64_t)st.de_fixed, (uint64_t)st.accepted, (uint64_t)st.trials, (uint64_t)st.evaluated,
                     (uint64_t)ef};
    if (s->comm) {
        Rccl& R = rccl();
        if (!R.all_reduce) return fail(PMC_ERR_HIP, "librccl lacks ncclAllReduce");
        void* d = nullptr;
        PMC_HIP(hipMalloc(&d, sizeof v));
        // every copy on aux, the stream the all-reduce runs on (no null-stream work in between)
        hipError_t e = hipMemcpyAsync(d, v, sizeof v, hipMemcpyHostToDevice, s->aux);
        if (e != hipSuccess) { (void)hipFree(d); return hip_fail(e, "observables copy"); }
        ncclResult_t r = R.all_reduce(d, d, 5, ncclUint64, ncclSum, s->comm, s->aux);
        if (r != ncclSuccess) { (void)hipFree(d); return nccl_fail(r, "ncclAllReduce"); }
        e = hipMemcpyAsync(v, d, sizeof v, hipMemcpyDeviceToHost, s->aux);
        if (e == hipSuccess) e = hipStreamSynchronize(s->aux);
        (void)hipFree(d);
        if (e != hipSuccess) return hip_fail(e, "observables all-reduce");
    } else if (s->ipc) {
        // every rank's five sums into its flags buffer; each rank pulls all of them (one exchange:
        // ready, pull, pulled -- the sequence numbers of the halo exchanges continue)
        if (int rc = ipc_settle(c)) return rc;     // (nobody still reads the reduction slot)
        const uint64_t seq = ++c->xseq;
        XferFlags w{};
        XferCopy cp{};
        for (int p = 0; p < s->world; ++p) {
            const uint64_t* pf = ipc_peer_flags(s, p);
            if (int rc = xfer_seg(cp, pf + kFlagRed, c->xflags + kFlagGather + 8 * p, sizeof v)) return rc;
            if (p != s->rank) {
                xfer_flag_add(w, pf + kFlagReady, seq);
                s->pend_readers.push_back(p);
            }
        }
        s->pend_seq = seq;
        PMC_HIP(hipMemcpyAsync(c->xflags + kFlagRed, v, sizeof v, hipMemcpyHostToDevice, s->aux));
        PMC_HIP(launch_xfer(cp, w, c->xflags + kFlagReady, c->xflags + kFlagPulled, seq,
                            reinterpret_cast<unsigned*>(c->xflags + kFlagDone), s->ipc_timeout, c->flags, s->aux));
        if (int rc = ipc_settle(c)) return rc;
        std::vector<uint64_t> h((size_t)8 * s->world);
        PMC_HIP(hipMemcpyAsync(h.data(), c->xflags + kFlagGather, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost,
                               s->aux));
        PMC_HIP(hipStreamSynchronize(s->aux));
        uint32_t fl = 0;
        PMC_HIP(hipMemcpy(&fl, c->flags, 4, hipMemcpyDeviceToHost));
        if (fl & 512u) return fail(PMC_ERR_HIP, "IPC transport: a peer did not arrive (wait timed out, error flag 512)");
        for (int k = 0; k < 5; ++k) {
            v[k] = 0;
            for (int p = 0; p < s->world; ++p) v[k] += h[(size_t)8 * p + k];
        }
    } else if (s->group) {
        pmc_local_group* g = s->group;
        {
            std::lock_guard<std::mutex> lk(g->m);
            for (int k = 0; k < 5; ++k) g->slot[s->rank].red[k] = v[k];
        }
        if (int rc = group_barrier(g)) return rc;   // every rank's values are in
        uint64_t t[5] = {0, 0, 0, 0, 0};
        {
            std::lock_guard<std::mutex> lk(g->m);
            for (const auto& sl : g->slot)
                for (int k = 0; k < 5; ++k) t[k] += sl.red[k];
        }
        if (int rc = group_barrier(g)) return rc;   // every rank has read them
        for (int k = 0; k < 5; ++k) v[k] = t[k];
    }
    out->de_fixed = (int64_t)v[0];
    out->accepted = (int64_t)v[1];
    out->trials = (int64_t)v[2];
    out->evaluated = (int64_t)v[3];
    if (with_energy) *e_out = (double)(int64_t)v[4] / PMC_FIX_SCALE * 0.5;
    return PMC_OK;
}

int pmc_timing_kinds(pmc_ctx* c, int enable, double ms[3], int count[3]) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    double a[3] = {0.0, 0.0, 0.0};
    int na[3] = {0, 0, 0};
    if (!c->tkind.empty()) {
        PMC_HIP(hipStreamSynchronize(c->stream));
        if (c->slab) PMC_HIP(hipStreamSynchronize(c->slab->aux));
        if (c->slab)
            for (hipStream_t h : c->slab->hi)
                if (h) PMC_HIP(hipStreamSynchronize(h));
        for (hipStream_t h : c->hs)
            if (h) PMC_HIP(hipStreamSynchronize(h));
        for (size_t k = 0; k < c->tkind.size(); ++k) {
            float t = 0.0f;
            PMC_HIP(hipEventElapsedTime(&t, c->tev[2 * k], c->tev[2 * k + 1]));
            a[c->tkind[k]] += t;
            ++na[c->tkind[k]];
        }
        // colour phases split over plane chains: the chains' launches run concurrently and a chain starts
        // its next phase while the others finish theirs, so per-launch times do not add up to the sweep.
        // The phases' time is the span of each sweep's subsweep launches, from the first start to the
        // last stop (launch gaps inside the sweep included, shiftCells not), over its 8 phases
        c->span_ms = 0.0;
        c->span_n = 0;
        for (size_t k = 0; k < c->tkind.size(); ++k) {
            if (c->tphase[k] < 0) continue;
            const int64_t sw = c->tphase[k] / 8;
            bool first = true;
            for (size_t j = 0; j < k; ++j) first = first && !(c->tphase[j] >= 0 && c->tphase[j] / 8 == sw);
            if (!first) continue;
            float lo = 1e30f, hi = -1e30f;
            for (size_t j = k; j < c->tkind.size(); ++j) {
                if (c->tphase[j] < 0 || c->tphase[j] / 8 != sw) continue;
                float t0 = 0.0f, t1 = 0.0f;
                PMC_HIP(hipEventElapsedTime(&t0, c->tev[0], c->tev[2 * j]));
                PMC_HIP(hipEventElapsedTime(&t1, c->tev[0], c->tev[2 * j + 1]));
                lo = t0 < lo ? t0 : lo;
                hi = t1 > hi ? t1 : hi;
            }
            c->span_ms += hi - lo;
            c->span_n += 8;
        }
    }
    for (int k = 0; k < 3; ++k) {
        if (ms) ms[k] = a[k];
        if (count) count[k] = na[k];
    }
    c->tkind.clear();
    c->tphase.clear();
    c->timing = enable != 0;
    c->timing_paused = false;
    return PMC_OK;
}

int pmc_timing_phase_spans(pmc_ctx* c, double* span_ms, int* n_phases) {
    if (!c || !span_ms || !n_phases) return fail(PMC_ERR_ARG, "null argument");
    *span_ms = c->span_ms;
    *n_phases = c->span_n;
    return PMC_OK;
}

int pmc_sweep_layout(pmc_ctx* c, int* n_chains, int borders[PMC_SWEEP_MAX_CHAINS + 1]) {
    if (!c || !n_chains || !borders) return fail(PMC_ERR_ARG, "null argument");
    const int nz = c->P.nz_local;
    *n_chains = chain_count(c);
    for (int j = 0; j <= PMC_SWEEP_MAX_CHAINS; ++j) borders[j] = j <= *n_chains ? chain_border(nz, *n_chains, j) : nz;
    return PMC_OK;
}

int pmc_timing_pause(pmc_ctx* c, int paused) {
    if (!c) return fail(PMC_ERR_ARG, "null ctx");
    c->timing_paused = paused != 0;
    return PMC_OK;
}

int pmc_timing(pmc_ctx* c, int enable, double* subsweep_ms, int* n_subsweep, double* shift_ms, int* n_shift) {
    double ms[3];
    int cnt[3];
    int rc = pmc_timing_kinds(c, enable, ms, cnt);
    if (rc) return rc;
    if (subsweep_ms) *subsweep_ms = ms[0];
    if (n_subsweep) *n_subsweep = cnt[0];
    if (shift_ms) *shift_ms = ms[1];
    if (n_shift) *n_shift = cnt[1];
    return PMC_OK;
}

int pmc_slab_timing(pmc_ctx* c, int enable, double* subsweep_ms, int* n_subsweep, double* shift_ms,
                    int* n_shift) {
    if (!c || !c->slab) return fail(PMC_ERR_ARG, "no slab driver (pmc_slab_init)");
    return pmc_timing(c, enable, subsweep_ms, n_subsweep, shift_ms, n_shift);
}

}  // extern "C"
