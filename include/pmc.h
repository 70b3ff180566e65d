/*
 * pmc.h -- C ABI of the MI355X-native checkerboard Monte Carlo hot path.
 *
 * Drop-in boundary for qingye3/parallel-monte-carlo (reference at /root/reference, read-only).
 * The reference has no library or FFI; its call surface is the three __global__ entry points
 * plus the `start` driver, all sharing the `disk`/`n` layout:
 *
 *   disk : float[cells][3][nmax]  -- cell c at c*3*nmax: x[nmax], y[nmax], z[nmax]
 *          (start.cu:188, indexing subsweep.h:20-24 / start.cu:291-300)
 *   n    : int16_t[cells]         -- particles per cell (start.cu:187)
 *   r    : float[3*N]             -- SoA positions x[N], y[N], z[N] (start.cu:186, :54-56)
 *   cell index = x + y*CPS + z*CPS^2  (get_cell_index, subsweep.h:14-16)
 *
 * Every entry point below cites the reference symbol it replaces.  Device pointers a caller passes
 * (pmc_subsweep, pmc_shift_cells, pmc_assign) and host arrays (pmc_copy_in/out, snapshots) are in
 * the reference layout.  The context's OWN state (pmc_state, pmc_attach_state) is in the state
 * layout pmc_state_layout reports: the reference rows, or x, y, z packed per slot (a cell's
 * occupied slots one contiguous run); the entry points convert at the boundary.  A cell holds
 * 3*nmax floats at cell*3*nmax in both.  All functions return PMC_OK (0) or a negative
 * pmc_status; they never print and never exit (the reference printf's and continues,
 * start.cu:213-216).  One host thread per context; all work is enqueued on the context's
 * stream (default: a stream created by pmc_create, or the one given to pmc_set_stream).
 */
#ifndef PMC_H
#define PMC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    PMC_OK = 0,
    PMC_ERR_ARG = -1,        /* invalid argument / parameter combination */
    PMC_ERR_HIP = -2,        /* HIP runtime error (see pmc_last_error) */
    PMC_ERR_OVERFLOW = -3,   /* a cell would hold more than nmax particles (reference: unchecked,
                                shiftCells.h:90,121 -- SURVEY Appendix B S3) */
    PMC_ERR_RANGE = -4,      /* a particle lies outside the (local) box in pmc_assign */
    PMC_ERR_NODEV = -5       /* no HIP device available */
} pmc_status;

/* Runtime parameters (the reference uses compile-time #defines, start.cu:14-24). */
typedef struct pmc_params {
    int32_t cps_x;      /* cells per side along x (cellsPerSide); even, >= 4 */
    int32_t cps_y;      /* cells along y (0 -> cps_x); even, >= 4 */
    int32_t cps_z;      /* GLOBAL cells along z (0 -> cps_x); even, >= 4 */
    int32_t nz_local;   /* z-planes owned by this context (0 -> cps_z); even */
    int32_t z0;         /* global z index of the first owned plane; even */
    int32_t halo;       /* 0: storage holds the whole periodic box (nz_local == cps_z);
                           1: slab mode, one halo plane below and above the owned planes;
                           2: slab mode with two halo planes per side (the slab driver's
                              one-exchange-per-sweep schedule; needs the grouped colour order) */
    int32_t nmax;       /* particle slots per cell (nmax), 1..64 */
    int32_t n_moves;    /* trial moves per cell visit (n_M) */
    float w;            /* cell width == LJ cutoff rc (w); box L = cps * w */
    float beta;         /* inverse temperature (beta) */
    float sigma;        /* Gaussian trial-move width (sigma) */
    uint32_t flags;     /* PMC_FLAG_*: 0 = defaults */
    uint64_t seed;      /* Philox key; the reference seeds cuRAND with 1234 (subsweep.h:259) */
} pmc_params;
/* pmc_params.flags: colour order of a sweep.  Default (0): grouped by z parity (4 colours of one
 * parity, then the other 4; spec v9, pmc_detmath.h); PMC_FLAG_FULL_SHUFFLE: one shuffle of all 8
 * colours (the reference's FY_Shuffle, start.cu:34-44). */
#define PMC_FLAG_FULL_SHUFFLE 1u
/* Reference quirks (off by default: the build runs the corrected semantics).
 * Each reproduces one behaviour of the root reference on top of the build's own RNG and ordering:
 *   PMC_FLAG_QUIRK_R1 -- random_int (subsweep.h:38-40) is always 0, so random_shuffle (:50-58) swaps
 *                        every slot with slot 0: the own cell is visited in the fixed rotation
 *                        slot l <- particle (l + 1) mod n instead of a random permutation;
 *   PMC_FLAG_QUIRK_R2 -- curand_init(1234, id, 0) on every launch (subsweep.h:256-259): a cell draws the
 *                        same random numbers at every visit (the sweep index is left out of the
 *                        Philox counters);
 *   PMC_FLAG_QUIRK_S1 -- int s[3] (shiftCells.h:31,105): the offset added to particles taken from the
 *                        neighbour cell is (int)(w*dir), -2 / +2 at w = 2.5, instead of w*dir.
 * With R1 or R2 every colour phase runs the full-capacity one-cell-per-wave kernel (a comparison
 * mode, not a fast path); two-plane halos and the persistent small-box kernel refuse them. */
#define PMC_FLAG_QUIRK_R1 2u
#define PMC_FLAG_QUIRK_R2 4u
#define PMC_FLAG_QUIRK_S1 8u
#define PMC_FLAG_QUIRKS (PMC_FLAG_QUIRK_R1 | PMC_FLAG_QUIRK_R2 | PMC_FLAG_QUIRK_S1)

/* Observables accumulated by the subsweep kernels (reference: kernel.cu:228,413-415 --
 * accept_counter and d_Eblocks; the reference never reports acceptance). */
typedef struct pmc_stats {
    int64_t de_fixed;   /* sum of accepted dE, fixed point 2^-32 energy units */
    int64_t accepted;   /* accepted trial moves */
    int64_t trials;     /* all trial moves, including out-of-cell rejections */
    int64_t evaluated;  /* trial moves that passed out_of_bound and had energies evaluated */
} pmc_stats;

/* Result of pmc_start (the reference main prints the energy trace, kernel.cu:695). */
typedef struct pmc_result {
    pmc_stats stats;    /* totals over the run */
    double e_initial;   /* total energy before the run (cell-list, pmc_energy) */
    double e_final;     /* total energy after the run */
    double seconds;     /* device time of the run (HIP events) */
    int64_t sweeps;     /* MC sweeps executed */
} pmc_result;

typedef struct pmc_ctx pmc_ctx;

/* ---- context ---------------------------------------------------------------------- */
/* Allocate device state (disk/n ping-pong pair, stats slots) on the current HIP device.
 * Replaces the cudaMalloc block of main (start.cu:197-205). */
int pmc_create(const pmc_params* params, pmc_ctx** out);
void pmc_destroy(pmc_ctx* ctx);
/* Enqueue all further work on `stream` (a hipStream_t; NULL = the null stream). */
int pmc_set_stream(pmc_ctx* ctx, void* stream);
/* The stream the context enqueues on (a hipStream_t), for ordering caller work against it. */
int pmc_get_stream(pmc_ctx* ctx, void** stream);
/* Use caller-owned device buffers as the context state instead of its own (e.g. torch
 * tensors for RCCL halo exchange).  Each disk buffer holds storage_cells*3*nmax floats in the
 * state layout (pmc_state_layout), each n buffer storage_cells int16; buffer 0 is the current
 * state. */
int pmc_attach_state(pmc_ctx* ctx, float* disk0, int16_t* n0, float* disk1, int16_t* n1);
/* Current state buffers (device pointers, state layout), storage geometry. */
int pmc_state(pmc_ctx* ctx, float** disk, int16_t** n);
int64_t pmc_storage_cells(const pmc_ctx* ctx);
/* Layout of the state buffers: slot s of dimension d of a cell at float d*nmax + s
 * (PMC_LAYOUT_REFERENCE, start.cu:188) or 3*s + d (PMC_LAYOUT_PACKED). */
#define PMC_LAYOUT_REFERENCE 0
#define PMC_LAYOUT_PACKED 1
int pmc_state_layout(const pmc_ctx* ctx, int* layout);
/* Last error message of this thread ("" if none). */
const char* pmc_last_error(void);
/* HIP devices visible to this process; PMC_ERR_NODEV (and *count = 0) when there is none.  Lets a
 * launcher's rank process fail before it touches a device it does not have. */
int pmc_device_count(int* count);

/* ---- reference kernels ------------------------------------------------------------- */
/* init_r (start.cu:47-58; index<N guard of kernel.cu:78-89): simple-cubic lattice of
 * n_atoms particles into d_r[3*n_atoms] (SoA), N_cube = ceil(cbrt(n_atoms)) computed
 * exactly (fixes start.cu:208 truncation).  In slab mode the lattice fills the owned slab. */
int pmc_init_r(pmc_ctx* ctx, int64_t n_atoms, float* d_r);
/* assign (start.cu:87-146): bin d_r into d_disk/d_n with the reference's half-open rule
 * lb < x <= ub, particles of a cell in ascending index order.  Returns PMC_ERR_OVERFLOW if a
 * cell exceeds nmax, PMC_ERR_RANGE if a particle is outside the owned box. */
int pmc_assign(pmc_ctx* ctx, const float* d_r, int64_t n_atoms, float* d_disk, int16_t* d_n);
/* subsweep_kernel (subsweep.h:240-300): one checkerboard colour phase, offset = (ox,oy,oz)
 * in {0,1}^3 (start.cu:241-245).  `sweep` is the RNG counter (sweep index).  d_disk: the reference
 * layout (converted through a staging buffer when the state layout is packed), or one of the
 * context's own state buffers. */
int pmc_subsweep(pmc_ctx* ctx, float* d_disk, const int16_t* d_n, const int offset[3],
                 uint32_t sweep);
/* shiftCells (shiftCells.h:28-144; semantics of the fixed copy
 * CUDA-Parallel-MC/CUDA-Parallel-MC/shiftCells.h:23-112): shift the cell grid along axis
 * f by d and re-bin.  Double-buffered: reads (d_disk_in,d_n_in), writes (d_disk_out,d_n_out)
 * (the reference's in-place update is only race-free inside one block, shiftCells.h:135-143). */
int pmc_shift_cells(pmc_ctx* ctx, const float* d_disk_in, const int16_t* d_n_in,
                    float* d_disk_out, int16_t* d_n_out, int f, float d);

/* ---- driver (start.cu:169-272 main loop, kernel.cu:652-701) ------------------------- */
/* Initialise the context state from a lattice of n_atoms particles (init_r + assign). */
int pmc_init_lattice(pmc_ctx* ctx, int64_t n_atoms);
/* Strong-scaling start state (BASELINE config 4): the lattice of n_atoms_total particles over the
 * WHOLE periodic box (init_r as for a whole-box context), of which this slab keeps the particles
 * of its owned planes (assign, start.cu:87-146, restricted to z0 <= cz < z0 + nz_local).  The
 * owned planes equal the same planes of a whole-box pmc_init_lattice, slot for slot.  With no
 * slab (z0 = 0, nz_local = cps_z) it is pmc_init_lattice. */
int pmc_init_lattice_global(pmc_ctx* ctx, int64_t n_atoms_total);
/* The reference lattice of n_atoms_lattice particles over a TALLER box of cps_x x cps_y x
 * lattice_cps_z cells (init_r, kernel.cu:78-89), bottom-aligned with the periodic box; the rows
 * inside the box's planes [0, cps_z) are kept, this slab keeping its owned planes.  The config-5
 * weak-scaling start (bench.py --config 5): N ranks of 256x256x32 cells hold exactly the planes
 * they hold in the 8-rank 256^3 / 8e7 box.  lattice_cps_z == cps_z (or 0) is
 * pmc_init_lattice_global. */
int pmc_init_lattice_planes(pmc_ctx* ctx, int64_t n_atoms_lattice, int32_t lattice_cps_z);
/* One full MC sweep on the context state: colour order from the sweep plan, 8 subsweeps,
 * shiftCells, buffer swap (start.cu:237-260).  Asynchronous. */
int pmc_sweep(pmc_ctx* ctx, uint32_t sweep);
/* One colour phase (colour id 0..7, itoa start.cu:153-157) / the sweep plan's shiftCells on the
 * context state (any mode; the slab driver interleaves these with halo exchange). */
int pmc_phase(pmc_ctx* ctx, int colour, uint32_t sweep);
int pmc_shift(pmc_ctx* ctx, uint32_t sweep);
/* Slab contexts (halo = 1) after the 8 phases of a sweep, when both halo planes are exact copies
 * of the neighbours' boundary planes: the sweep plan's shiftCells over the owned planes AND every
 * halo plane whose new content depends only on planes this rank holds (along x/y both halos, along
 * z in direction dir the one on the -dir side; VS shiftCells.h:38-108 applied to the halo copies, the
 * same float operations as the plane's owner), then the buffer swap.  *halo_recv tells the caller
 * which halo still has to be received: 0 none, +1 the top halo (local plane nz_local) from the rank
 * above's new plane 0, -1 the bottom halo (plane -1) from the rank below's new top plane.  The C
 * slab driver (pmc_slab_sweep) does the same internally. */
int pmc_shift_slab(pmc_ctx* ctx, uint32_t sweep, int* halo_recv);
/* Restrict a colour phase to the cells in local planes [zl_begin, zl_end) (0 <= .. <= nz_local).
 * Cells of one colour are independent, so splitting a phase into ranges in any order gives the
 * same result; the slab driver runs the halo-free interior while boundary planes travel. */
int pmc_subsweep_range(pmc_ctx* ctx, float* d_disk, const int16_t* d_n, const int offset[3],
                       uint32_t sweep, int zl_begin, int zl_end);
int pmc_phase_range(pmc_ctx* ctx, int colour, uint32_t sweep, int zl_begin, int zl_end);
/* pmc_phase_range launched on `stream` (a hipStream_t; NULL = the default stream) instead of the
 * context stream, with its own overflow queue, so it may run concurrently with a context-stream
 * launch of the same colour on other planes (the slab driver's boundary planes beside the
 * interior).  The caller orders the two streams between phases. */
int pmc_phase_range_on(pmc_ctx* ctx, int colour, uint32_t sweep, int zl_begin, int zl_end, void* stream);
/* ---- multi-GPU slab driver (one process per GPU; RCCL over xGMI) -------------------------
 * Replaces the reference's single-GPU main loop (start.cu:237-260) for a box split into z-slabs:
 * rank r owns planes [r*nz_local, (r+1)*nz_local) of a cps_x x cps_y x (world*nz_local) periodic
 * box (context created with halo = 1, z0 = r*nz_local) plus a halo plane below and above.  The
 * whole sweep schedule runs in C.  The 8 colour phases of a sweep form runs of equal z parity q (two
 * runs of 4 with the default order); each run is independent launch chains: the interior planes
 * in 1-3 chains (PMC_SLAB_CHAINS, default 2: the context stream and one or two more streams) and
 * the boundary plane of parity q on the exchange stream, which then sends that whole plane to the
 * neighbour holding it as a halo and receives the opposite halo (one RCCL send/recv each way per
 * run) while the interior chains run.
 * After shiftCells only a z shift needs one more plane (with its counts) from one side.  Every rank
 * derives the sweep plan itself and RNG counters use global cell ids, so any world size
 * reproduces the single-GPU run bit for bit.  librccl is dlopen'ed ("librccl.so.1", or the path
 * in PMC_RCCL_LIB).
 * Contexts created with halo = 2 run a different schedule with ONE exchange per sweep: the first
 * run also visits the neighbour's boundary plane of its parity (a halo plane) redundantly, on a
 * stream of its own (its counters are not added: the owner counts them), so the second run needs no
 * exchange; after shiftCells the four planes next to the slab's faces travel with their counts
 * (and, for a z shift whose dir-side halo is the stale one, one plane before it).  Same results bit
 * for bit; DESIGN.md section 6 has the measurements (slower than halo = 1 on one GPU). */
/* rank 0: a fresh RCCL unique id (128 bytes) to broadcast to the other ranks */
int pmc_comm_unique_id(unsigned char id[128]);
/* Attach the slab driver: create the RCCL communicator (collective over the world ranks; id from
 * rank 0), the auxiliary stream and the halo buffers.  id = NULL with world = 1: no RCCL, the
 * periodic halos are local copies. */
int pmc_slab_init(pmc_ctx* ctx, int rank, int world, const unsigned char* id);
/* In-process halo transport: `world` slab contexts of ONE process (e.g. W slabs on one GPU), one
 * host thread per rank.  The slab driver issues exactly the messages it gives RCCL (same peers,
 * same order, same ncclSend/ncclRecv matching); each becomes a device-to-device copy on the
 * receiver's aux stream, ordered by HIP events and a host barrier per exchange.  Every rank must
 * call the collective functions (pmc_slab_exchange, pmc_slab_sweep) from its own thread.  A rank
 * that fails, or a barrier that waits longer than PMC_LOCAL_GROUP_TIMEOUT_MS (default 120000),
 * breaks the group: every later exchange returns PMC_ERR_HIP.  Destroy the contexts before the
 * group. */
typedef struct pmc_local_group pmc_local_group;
int pmc_local_group_create(int world, pmc_local_group** out);
void pmc_local_group_destroy(pmc_local_group* group);
/* pmc_slab_init with the in-process transport: rank `rank` of group->world. */
int pmc_slab_init_local(pmc_ctx* ctx, int rank, pmc_local_group* group);
/* IPC transport: one PROCESS per rank on one node (one per GPU over xGMI, or several on one GPU),
 * without RCCL.  Each rank exports its symmetric buffers -- the disk/n ping-pong pair, the
 * two-plane-halo send planes, a flags buffer in uncached device memory -- with
 * pmc_slab_ipc_handle; the caller gathers the world's blobs in rank order (any host collective,
 * e.g. a gloo all_gather) and passes them to pmc_slab_init_ipc, which maps every peer's buffers
 * (hipIpcOpenMemHandle).  An exchange is then three launches on the exchange stream and no host
 * round trip: publish a sequence number and wait for the senders' (k_xfer_flag), pull every
 * message straight from the sender's buffer (k_xfer_copy), wait until the readers have pulled.
 * The messages, peers and matching are exactly RCCL's.  A wait that exceeds PMC_IPC_TIMEOUT_S
 * (default 60 s) gives up and sets error flag bit 9 (512) instead of hanging the GPU.  The state
 * buffers must not change afterwards (pmc_attach_state fails on an IPC slab).  The blob holding
 * this context itself (a one-rank rehearsal: world = 1) maps nothing.  Replaces, like
 * pmc_slab_init, the single-GPU loop start.cu:237-260. */
#define PMC_IPC_HANDLE_BYTES 1024
int pmc_slab_ipc_handle(pmc_ctx* ctx, unsigned char blob[PMC_IPC_HANDLE_BYTES]);
/* blobs: world * PMC_IPC_HANDLE_BYTES bytes, rank r's blob at r * PMC_IPC_HANDLE_BYTES; collective
 * in the sense that every rank must call it before the first exchange. */
int pmc_slab_init_ipc(pmc_ctx* ctx, int rank, int world, const unsigned char* blobs);
/* Refill both halo planes and their counts from the neighbours (after init_lattice, copy_in or
 * load_snapshot).  Collective. */
int pmc_slab_exchange(pmc_ctx* ctx);
/* One full sweep (8 colour phases with halo exchange + shiftCells + halo refresh).  Asynchronous;
 * collective (every rank calls it with the same sweep index). */
int pmc_slab_sweep(pmc_ctx* ctx, uint32_t sweep);
/* Order the context stream after the outstanding exchanges (before reading state or halos).  With
 * the IPC transport it also synchronises and returns PMC_ERR_HIP when a wait timed out (error bit 9):
 * a timed-out exchange copies nothing and the run's state is void. */
int pmc_slab_finish(pmc_ctx* ctx);
/* The interior chains of pmc_slab_sweep: *n_chains chains, chain j over local planes
 * [borders[j], borders[j+1]) (borders[0] = 1, borders[*n_chains] = nz_local - 1). */
int pmc_slab_layout(pmc_ctx* ctx, int* n_chains, int borders[4]);
/* Observables of the whole box (one sum over the ranks per report): the four counters
 * (pmc_stats_read without reset) and, with with_energy, the cell-list energy (pmc_energy), each
 * summed over all ranks in fixed point -- exact, equal to a one-GPU run's -- through the slab's
 * transport (one RCCL all-reduce, or the in-process group).  Collective: every rank calls it.
 * Reference: kernel.cu:415 (accept_counter), kernel.cu:452-470 (calc_energy). */
int pmc_slab_observables(pmc_ctx* ctx, int with_energy, pmc_stats* out, double* e_out);
/* Sum of the HIP-event durations of the subsweep and shift launches since the last call
 * (synchronizes), then switch per-launch events on (enable = 1) or off.  The events ride on the
 * kernels' own dispatch packets (no extra packets between launches); graph replays and the
 * overflow (fallback) launches are not timed.  pmc_timing reports the kind-[0] subsweep launches and
 * the shift launches; pmc_slab_timing is the same call, requiring the slab driver.
 * pmc_timing_kinds splits by kind: [0] subsweep launches of whole colour phases or of a slab's
 * interior planes (the slab driver's interior chains, pmc_slab_layout: one launch per chain and
 * phase, running concurrently), [1] shiftCells, [2] the slab driver's boundary-plane launches and
 * pmc_phase_range_on launches (other streams: they overlap [0], durations do not add). */
int pmc_timing(pmc_ctx* ctx, int enable, double* subsweep_ms, int* n_subsweep, double* shift_ms, int* n_shift);
int pmc_timing_kinds(pmc_ctx* ctx, int enable, double ms[3], int count[3]);
/* Colour phases that pmc_sweep splits over plane chains (pmc_sweep_layout) run as concurrent
 * launches, a chain starting its next phase while the others finish theirs: the last pmc_timing /
 * pmc_timing_kinds call also summed, per timed sweep, the span of its subsweep launches (first start
 * to last stop: the 8 phases with the gaps between them, shiftCells excluded); this returns that sum
 * and the number of phases it covers (8 per sweep). */
int pmc_timing_phase_spans(pmc_ctx* ctx, double* span_ms, int* n_phases);
/* pmc_sweep's plane chains (whole box): *n_chains (1, 2 or 4: PMC_SWEEP_CHAINS, default 2; fewer when
 * the box has under 4 planes per chain), chain j over local planes [borders[j], borders[j+1]) (entries
 * past n_chains: nz).  More than one chain: each colour phase is one launch per chain, on streams of
 * their own; the chains' launch tails overlap (the runs of equal z parity make them independent; the
 * slab driver's rule, pmc_slab_sweep). */
#define PMC_SWEEP_MAX_CHAINS 4
int pmc_sweep_layout(pmc_ctx* ctx, int* n_chains, int borders[PMC_SWEEP_MAX_CHAINS + 1]);
/* Pause (paused = 1) or resume the per-launch events of pmc_timing without collecting them (no
 * synchronization): a caller times a sample of its launches, e.g. every k-th sweep, and the events'
 * own cost (about 1.3% of a sweep when every launch carries them) shrinks with the sample. */
int pmc_timing_pause(pmc_ctx* ctx, int paused);
int pmc_slab_timing(pmc_ctx* ctx, int enable, double* subsweep_ms, int* n_subsweep, double* shift_ms,
                    int* n_shift);
/* The per-sweep plan every rank replicates (no broadcast): colour order (FY_Shuffle + itoa,
 * start.cu:34-44,153-157, reseeded from time() in the reference) and the shift axis/distance
 * (kernel.cu:683-684), all from the host Philox stream keyed by `seed`. */
int pmc_sweep_plan(uint64_t seed, uint32_t sweep, float w, int order[8], int* f, float* d);
int pmc_sweep_plan_ex(uint64_t seed, uint32_t sweep, float w, uint32_t flags, int order[8], int* f, float* d);
/* mc_passes sweeps starting at sweep index `first_sweep` (the `start` driver). */
int pmc_start(pmc_ctx* ctx, uint32_t first_sweep, int mc_passes, pmc_result* out);
/* pmc_start with flags: PMC_START_NO_ENERGY skips the two cell-list energies (e_initial/e_final
 * are NaN), for drivers that evaluate the energy once per interval themselves. */
#define PMC_START_NO_ENERGY 1
int pmc_start_ex(pmc_ctx* ctx, uint32_t first_sweep, int mc_passes, int flags, pmc_result* out);
/* Record the sweep loop (pmc_sweep for sweeps first..first+count-1) as a hipGraph and
 * replay it; identical results to calling pmc_sweep in a loop. */
int pmc_run_graph(pmc_ctx* ctx, uint32_t first_sweep, int count);
/* Small boxes (whole box, nmax 16, at most 2048 cells per colour, e.g. 16^3): sweeps
 * first..first+count-1 as ONE launch per 32 sweeps on one XCD, in-kernel barriers where the 17
 * launches of a sweep were (start.cu:242-249's per-phase launch + synchronize); identical results
 * to pmc_sweep in a loop.  PMC_ERR_ARG for a box that does not qualify.  One XCD is an eighth of the
 * chip: slower than per-phase launches (16^3: 0.513 against 0.072 ms per sweep), so pmc_start does
 * not use it by default (PMC_SMALL=1 in the environment: for boxes of at most 64 cells per colour).
 * Error flags bit 3 (value 8): a barrier timed out; bit 4 (value 16): the launch's blocks were not
 * dealt round-robin over the XCDs; bit 5 (value 32): no workgroup of the launch ran on XCD 0. */
int pmc_run_small(pmc_ctx* ctx, uint32_t first_sweep, int count);

/* ---- observables ------------------------------------------------------------------- */
/* Total LJ energy of the owned cells' particles (calc_energy, kernel.cu:452-470, as an
 * O(N) cell-list sum; pairs across the slab boundary count half on each side).  A slab context
 * must be flushed first after pmc_slab_sweep (pmc_slab_finish): a z shift's halo plane may still be
 * pending, and that flush is collective, so pmc_energy refuses (PMC_ERR_ARG) instead of doing it. */
int pmc_energy(pmc_ctx* ctx, double* e_out);
/* Read and optionally reset the accumulated subsweep statistics (synchronises). */
int pmc_stats_read(pmc_ctx* ctx, pmc_stats* out, int reset);
/* Device error flags (bit 0: shift overflow, bit 1: assign overflow, bit 2: assign range, bits 3-4:
 * pmc_run_small; bit 9: an IPC-transport wait timed out; bit 10: the IPC sender's L2 write-back did
 * not cover all 8 XCDs);
 * synchronises; `reset` clears them. */
int pmc_error_flags(pmc_ctx* ctx, uint32_t* flags, int reset);

/* ---- host mirrors ------------------------------------------------------------------ */
int pmc_copy_out(pmc_ctx* ctx, float* h_disk, int16_t* h_n);
int pmc_copy_in(pmc_ctx* ctx, const float* h_disk, const int16_t* h_n);
int pmc_synchronize(pmc_ctx* ctx);

/* ---- slab decomposition support (multi-GPU, halo == 1) ----------------------------- */
/* Byte offsets/sizes of a storage z-plane (local z in [-1, nz_local]) inside the disk and
 * n buffers, for point-to-point halo exchange by the caller (RCCL). */
int pmc_plane_span(const pmc_ctx* ctx, int z_local, size_t* disk_off, size_t* disk_bytes,
                   size_t* n_off, size_t* n_bytes);

/* ---- diagnostics ------------------------------------------------------------------ */
/* Evaluate the deterministic math of pmc_detmath.h on the device for `count` Philox word
 * quadruples (h_words[4*count]): h_out_f[4*count] = 3 trial-move normals + one LJ pair energy,
 * h_out_d[2*count] = acceptance threshold + fixed-point energy.  Used by the parity tests to pin
 * host == device bit equality of every transcendental the kernels use. */
int pmc_selftest_detmath(const uint32_t* h_words, int count, float* h_out_f, double* h_out_d);
/* The HBM rate this GPU delivers (beside the 8 TB/s spec): best of `reps`
 * passes of a streaming read of `bytes` (16-B loads, nothing written) and of a copy of `bytes`
 * (read + write counted), GB/s; two buffers of `bytes` (>= 16 MiB) on the current device. */
int pmc_hbm_probe(uint64_t bytes, int reps, double* read_gbs, double* copy_gbs);

/* ---- trajectory dump / restart ---------------------------------- */
/* The reference's visualisation path is host code: disk_to_r + create_dump
 * (CUDA-Parallel-MC/CUDA-Parallel-MC/kernel.cu:497-536), LAMMPS-style text for OVITO.  It has
 * no reader and no checkpoint; the reader and the binary snapshot below are the restart path.
 * The host-only functions need no GPU. */
/* disk_to_r (kernel.cu:500-510): particles of `cells` cells in cell order, then slot order, into
 * h_r[3*stride] (SoA: x at [0,stride), y at [stride,2*stride), z after).  h_r == NULL only counts.
 * *count = particles found; PMC_ERR_ARG if they exceed stride or a count is outside [0, nmax]. */
int pmc_disk_to_r(const float* h_disk, const int16_t* h_n, int64_t cells, int32_t nmax, float* h_r,
                  int64_t stride, int64_t* count);
/* One frame in create_dump's format (kernel.cu:521-535): "ITEM: TIMESTEP \n<t>\n ITEM: NUMBER OF
 * ATOMS ... ITEM: BOX BOUNDS ... ITEM: ATOMS id type x y z ix iy iz", coordinates "%f", ids 1..n.
 * append = 0 truncates the file. */
int pmc_write_dump(const char* path, int append, int64_t timestep, const float* h_r, int64_t stride,
                   int64_t n_atoms, const float box_lo[3], const float box_hi[3]);
/* Read frame `frame` (0-based) of such a file into h_r[3*stride] by atom id; h_r == NULL reads the
 * header only (timestep, n_atoms, box).  PMC_ERR_RANGE if the file has fewer frames. */
int pmc_read_dump(const char* path, int64_t frame, int64_t* timestep, float* h_r, int64_t stride,
                  int64_t* n_atoms, float box_lo[3], float box_hi[3]);
/* Binary snapshot "PMCSNAP1": parameters, the next sweep index (the whole RNG state: Philox
 * counters are (sweep, cell, move)), the accumulated statistics, and every occupied slot's
 * exact float bits; FNV-1a checksum; written to path.tmp then renamed.  h_disk/h_n hold `cells`
 * cells in the reference layout (pmc_snapshot_read zero-fills unused slots; h_disk == h_n == NULL
 * reads the header only). */
int pmc_snapshot_write(const char* path, const pmc_params* params, uint32_t next_sweep,
                       const pmc_stats* stats, const float* h_disk, const int16_t* h_n, int64_t cells);
/* pmc_snapshot_read: with h_disk/h_n, params is required and params->nmax must be the nmax the
 * buffers were sized for (cells*3*nmax floats): a snapshot with another nmax is refused before
 * anything is written (PMC_ERR_ARG); on return *params holds the snapshot's parameters.  Header and
 * payload come from one open file. */
int pmc_snapshot_read(const char* path, pmc_params* params, uint32_t* next_sweep, pmc_stats* stats,
                      float* h_disk, int16_t* h_n, int64_t cells);
/* Context wrappers (owned cells; slab mode: this rank's planes, halos must be exchanged after a
 * load).  pmc_dump_frame writes the current state as one frame with box -L/2..L/2 per axis. */
int pmc_get_params(const pmc_ctx* ctx, pmc_params* out);
int pmc_stats_write(pmc_ctx* ctx, const pmc_stats* in);
int pmc_dump_frame(pmc_ctx* ctx, const char* path, int append, int64_t timestep);
int pmc_save_snapshot(pmc_ctx* ctx, const char* path, uint32_t next_sweep);
/* Restores state + statistics; PMC_ERR_ARG if the snapshot's parameters differ from the ctx's. */
int pmc_load_snapshot(pmc_ctx* ctx, const char* path, uint32_t* next_sweep);

/* ---- environment switches read by the library (none is needed in production) ----------
 * Operational:      PMC_IPC_TIMEOUT_S (IPC wait limit, default 60), PMC_LOCAL_GROUP_TIMEOUT_MS,
 *                   PMC_RCCL_LIB (librccl path; SlabDriver sets torch's).
 * Schedule A/B:     PMC_SWEEP_CHAINS, PMC_SLAB_CHAINS, PMC_SLAB_PRIORITY, PMC_SLAB_B_FIRST,
 *                   PMC_SLAB_SPLIT_SHIFT, PMC_SLAB_DEFER_Z, PMC_SLAB_DIRECT_HALO, PMC_BOUNDARY_FULL,
 *                   PMC_IPC_FUSED, PMC_SMALL, PMC_SMALL_LAUNCH, PMC_DIRECT_CELLS, PMC_FALLBACK_BLOCKS,
 *                   PMC_SHIFT_RUN, PMC_SHIFT_OFF32, PMC_ENERGY_LEGACY, PMC_ENERGY_ROWS_CAP: every
 *                   setting gives the same bits (the GPU tests run the non-default ones); DESIGN.md
 *                   records which were measured and why the default won.
 * Test hooks:       PMC_SUBSWEEP_CAP (forces the overflow-queue fallback), PMC_FORCE_ADDR64 (64-bit
 *                   addressing below 4 GiB).
 * Timing only:      PMC_XFER_DELAY_US (a one-GPU rehearsal's stand-in for xGMI time per exchange;
 *                   changes no result). */

#ifdef __cplusplus
}
#endif

#endif /* PMC_H */
