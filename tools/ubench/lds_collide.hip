// Which lane's value lands when several lanes of ONE ds_write_b32 hit the same LDS address?
// Compaction pattern of the subsweep term list: lane l writes at C + mbcnt(mask) for random masks
// (non-listed lanes share the slot of the next listed lane above them).  Counts, over many random
// masks and offsets, how often the slot holds the highest writer's value.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/lds_collide tools/ubench/lds_collide.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k(const unsigned long long* masks, const int* offs, int n, int* bad, int* total) {
    __shared__ float buf[256 * 4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float* b = buf + wv * 256;
    for (int it = blockIdx.x * 4 + wv; it < n; it += gridDim.x * 4) {
        const unsigned long long m = masks[it];
        const int C = offs[it];
        for (int i = lane; i < 256; i += 64) b[i] = -1.0f;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const int pos = C + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        const bool listed = (m >> lane) & 1ull;
        b[pos] = listed ? (float)lane : 1000.0f + (float)lane;   // every lane writes
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // lane l checks: if listed, slot pos must hold l
        const bool wrong = listed && b[pos] != (float)lane;
        const unsigned long long wm = __builtin_amdgcn_ballot_w64(wrong);
        if (lane == 0) {
            if (wm) atomicAdd(bad, 1);
            atomicAdd(total, 1);
        }
    }
}

int main() {
    const int n = 1 << 20;
    unsigned long long* hm = (unsigned long long*)malloc(n * 8);
    int* ho = (int*)malloc(n * 4);
    srand(7);
    for (int i = 0; i < n; ++i) {
        unsigned long long m = 0;
        const int dens = rand() % 100;   // listed density 0-99 %
        for (int l = 0; l < 64; ++l)
            if (rand() % 100 < dens) m |= 1ull << l;
        hm[i] = m;
        ho[i] = rand() % 128;
    }
    unsigned long long* dm;
    int *dof, *dbad;
    hipMalloc(&dm, n * 8);
    hipMalloc(&dof, n * 4);
    hipMalloc(&dbad, 8);
    hipMemcpy(dm, hm, n * 8, hipMemcpyHostToDevice);
    hipMemcpy(dof, ho, n * 4, hipMemcpyHostToDevice);
    hipMemset(dbad, 0, 8);
    hipLaunchKernelGGL(k, dim3(2048), dim3(256), 0, 0, dm, dof, n, dbad, dbad + 1);
    int r[2];
    hipMemcpy(r, dbad, 8, hipMemcpyDeviceToHost);
    printf("{\"trials\": %d, \"listed_lane_lost\": %d}\n", r[1], r[0]);
    return r[0] != 0;
}
