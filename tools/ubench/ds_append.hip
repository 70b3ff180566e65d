// ds_append as the term-list compaction primitive (gfx950 microbenchmark).
//  1. semantics: under an exec mask, does ds_append return base + (active lanes below this lane)
//     -- the same index as mbcnt -- and advance the LDS counter by the active count?  65536 masks
//     (random, sparse, empty, full) on 256 waves.
//  2. throughput: a compaction loop shaped like the subsweep's per-block term listing (two masks per
//     block, exec-masked ds_write of one float per listed lane) with mbcnt (v_mbcnt_lo/hi + base) vs
//     ds_append, at 8 waves per SIMD, timed with HIP events.
// Build: hipcc --offload-arch=gfx950 -O3 -o ds_append ds_append.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) int lds_int;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_sem(const unsigned* masks_lo, const unsigned* masks_hi, int n, int* bad) {
    __shared__ int ctr[4];
    const int lane = threadIdx.x & 63;
    int nbad = 0;
    for (int it = 0; it < n; ++it) {
        if (lane == 0) ctr[0] = 100 * it;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const unsigned long long m = ((unsigned long long)masks_hi[it] << 32) | masks_lo[it];
        const bool on = (m >> lane) & 1ull;
        int v = -1;
        if (on) v = __builtin_amdgcn_ds_append((lds_int*)&ctr[0]);
        const int expect = 100 * it + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        if (on && v != expect) ++nbad;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const int tot = ctr[0];
        if (lane == 0 && tot != 100 * it + __popcll(m)) ++nbad;
    }
    atomicAdd(bad, nbad);
}

// per wave: REPS blocks; each block lists the lanes with a < t (new) then b >= -t (old)
template <bool APPEND>
__global__ __launch_bounds__(64) void k_tp(const float* in, int reps, float t, float* out) {
    extern __shared__ float sm[];
    float* buf = sm + 1;                 // list (sm[0]: the append counter)
    const int lane = threadIdx.x;
    float a = in[blockIdx.x * 64 + lane], b = -a;
    float acc = 0.0f;
    int C = 0;
    for (int r = 0; r < reps; ++r) {
        a = a * 1.0001f + 0.37f; if (a > 1.0f) a -= 2.0f;
        b = b * 0.9999f - 0.29f; if (b < -1.0f) b += 2.0f;
        const unsigned long long mn = __builtin_amdgcn_ballot_w64(a <= t);
        const unsigned long long mo = __builtin_amdgcn_ballot_w64(b >= -t);
        if constexpr (APPEND) {
            if ((r & 7) == 0) { if (lane == 0) ((int*)sm)[0] = 0; C = 0; }
            if (a <= t) buf[__builtin_amdgcn_ds_append((lds_int*)sm) & 255] = a;
            if (b >= -t) buf[__builtin_amdgcn_ds_append((lds_int*)sm) & 255] = b;
        } else {
            if ((r & 7) == 0) C = 0;
            const int cn = C + __popcll(mn);
            if (__builtin_amdgcn_inverse_ballot_w64(mn))
                buf[(int)__builtin_amdgcn_mbcnt_hi((unsigned)(mn >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mn, (unsigned)C)) & 255] = a;
            if (__builtin_amdgcn_inverse_ballot_w64(mo))
                buf[(int)__builtin_amdgcn_mbcnt_hi((unsigned)(mo >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mo, (unsigned)cn)) & 255] = b;
            C = cn + __popcll(mo);
        }
        if ((r & 7) == 7) acc += buf[lane];
    }
    out[blockIdx.x * 64 + lane] = acc + (float)C;
}

int main() {
    const int n = 1 << 16;
    std::vector<unsigned> lo(n), hi(n);
    unsigned s = 12345;
    for (int i = 0; i < n; ++i) {
        s = s * 1664525u + 1013904223u; lo[i] = s;
        s = s * 1664525u + 1013904223u; hi[i] = s;
        if (i % 7 == 0) lo[i] &= s >> 3;
        if (i % 11 == 0) hi[i] = 0;
    }
    lo[1] = hi[1] = 0; lo[2] = hi[2] = 0xFFFFFFFFu; lo[3] = 1; hi[3] = 0x80000000u;
    unsigned *dlo, *dhi; int* dbad;
    CK(hipMalloc(&dlo, n * 4)); CK(hipMalloc(&dhi, n * 4)); CK(hipMalloc(&dbad, 4));
    CK(hipMemcpy(dlo, lo.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dhi, hi.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(dbad, 0, 4));
    hipLaunchKernelGGL(k_sem, dim3(256), dim3(64), 0, 0, dlo, dhi, n, dbad);
    CK(hipDeviceSynchronize());
    int bad = -1;
    CK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
    printf("semantics: %d mismatches in %d masks x 256 waves (0: ds_append == base + mbcnt, lane order)\n", bad, n);

    const int waves = 256 * 4 * 8 * 4;   // 4 rounds of 8 waves on every SIMD
    float *din, *dout;
    CK(hipMalloc(&din, waves * 64 * 4)); CK(hipMalloc(&dout, waves * 64 * 4));
    std::vector<float> h(waves * 64);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 2000) / 1000.0f - 1.0f;
    CK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int reps = 2048;
    const size_t lds = 4 * 1280;         // 5 KiB per wave: 8 waves per SIMD, as the subsweep
    for (int pass = 0; pass < 3; ++pass) {
        for (int ap = 0; ap < 2; ++ap) {
            CK(hipEventRecord(e0));
            if (ap) hipLaunchKernelGGL(k_tp<true>, dim3(waves), dim3(64), lds, 0, din, reps, -0.6f, dout);
            else hipLaunchKernelGGL(k_tp<false>, dim3(waves), dim3(64), lds, 0, din, reps, -0.6f, dout);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0; CK(hipEventElapsedTime(&ms, e0, e1));
            printf("pass %d %-9s %.3f ms  (%.2f ns per block per wave-slot)\n", pass, ap ? "ds_append" : "mbcnt", ms,
                   ms * 1e6 / ((double)reps * waves / (256 * 4 * 8)));
        }
    }
    return 0;
}
