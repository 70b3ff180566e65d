// HBM streaming-rate exploration (round 6): read-only and copy kernels over 2 GiB with different
// grid shapes, loads in flight and load flavours, to size pmc_hbm_probe (bench.py's achievable peak).
//   hipcc --offload-arch=gfx950 -O3 -o hbm_stream tools/ubench/hbm_stream.hip && ./hbm_stream
#include <hip/hip_runtime.h>
#include <cstdio>

template <int U, bool NT>
__global__ __launch_bounds__(256) void rd(const uint4* __restrict__ s, uint64_t n, unsigned* sink) {
    const uint64_t st = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned acc = 0;
    for (; i + (U - 1) * st < n; i += U * st) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) {
                v[u].x = __builtin_nontemporal_load(&s[i + u * st].x);
                v[u].y = __builtin_nontemporal_load(&s[i + u * st].y);
                v[u].z = __builtin_nontemporal_load(&s[i + u * st].z);
                v[u].w = __builtin_nontemporal_load(&s[i + u * st].w);
            } else {
                v[u] = s[i + u * st];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345u) sink[blockIdx.x] = acc;
}

// contiguous chunk per block (each block sweeps its own range)
template <int U>
__global__ __launch_bounds__(256) void rd_chunk(const uint4* __restrict__ s, uint64_t n, unsigned* sink) {
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    unsigned acc = 0;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += U * 256) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = (i + u * 256 < b1) ? s[i + u * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345u) sink[blockIdx.x] = acc;
}

template <int U>
__global__ __launch_bounds__(256) void cp(const uint4* __restrict__ s, uint4* __restrict__ d, uint64_t n) {
    const uint64_t st = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * st < n; i += U * st) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = s[i + u * st];
#pragma unroll
        for (int u = 0; u < U; ++u) d[i + u * st] = v[u];
    }
}

template <int U>
__global__ __launch_bounds__(256) void cp_chunk(const uint4* __restrict__ s, uint4* __restrict__ d, uint64_t n) {
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += U * 256) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + u * 256 < b1) v[u] = s[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + u * 256 < b1) d[i + u * 256] = v[u];
    }
}

int main() {
    const uint64_t bytes = 2ull << 30, n = bytes / 16;
    uint4 *a, *b;
    unsigned* sink;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMalloc(&sink, 1 << 20);
    hipMemset(a, 1, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto time = [&](const char* name, int bl, auto fn, double mult) {
        fn();
        hipDeviceSynchronize();
        float best = 1e9f;
        for (int r = 0; r < 8; ++r) {
            hipEventRecord(e0);
            fn();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        printf("%-14s blocks/CU %3d  %7.1f GB/s\n", name, bl, mult * bytes / (best * 1e-3) / 1e9);
    };
    for (int bl : {2, 4, 8, 16, 32}) {
        const int g = 256 * bl;
        time("read U4", bl, [&] { rd<4, false><<<g, 256>>>(a, n, sink); }, 1.0);
        time("read U8", bl, [&] { rd<8, false><<<g, 256>>>(a, n, sink); }, 1.0);
        time("read U16", bl, [&] { rd<16, false><<<g, 256>>>(a, n, sink); }, 1.0);
        time("read U8 nt", bl, [&] { rd<8, true><<<g, 256>>>(a, n, sink); }, 1.0);
        time("read chunk U8", bl, [&] { rd_chunk<8><<<g, 256>>>(a, n, sink); }, 1.0);
        time("copy U4", bl, [&] { cp<4><<<g, 256>>>(a, b, n); }, 2.0);
        time("copy U8", bl, [&] { cp<8><<<g, 256>>>(a, b, n); }, 2.0);
        time("copy chunk U4", bl, [&] { cp_chunk<4><<<g, 256>>>(a, b, n); }, 2.0);
    }
    time("hipMemcpyD2D", 0, [&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); }, 2.0);
    return 0;
}
