// Micro-benchmark: issue cost of the VALU instructions the RNG and the accept test use, on one
// MI355X (gfx950).  Each lane runs 8 independent chains of one instruction kind; the grid holds
// 8 waves per SIMD on every CU.  Prints cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 4096;

#define CHAINS 8
template <int K>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
    uint32_t x[CHAINS];
    float f[CHAINS];
    unsigned long long msk = 0x5555aaaa5555aaaaull + seed;
    double d[CHAINS];
    for (int c = 0; c < CHAINS; ++c) {
        x[c] = seed + threadIdx.x * 7919u + c * 104729u;
        f[c] = 1.0f + (float)x[c] * 1e-9f;
        d[c] = 1.0 + (double)x[c] * 1e-12;
    }
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if constexpr (K == 0) { asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(x[(c + 1) % CHAINS])); }
            if constexpr (K == 1) { uint64_t p, cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p), "=s"(cc) : "v"(x[c]), "s"(0xD2511F53u)); x[c] = (uint32_t)(p >> 32); }
            if constexpr (K == 2) { asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[c]) : "s"(0xD2511F53u)); }
            if constexpr (K == 3) { asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[c]) : "s"(0xD2511F53u)); }
            if constexpr (K == 4) { asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[c]) : "s"(0x511F53u)); }
            if constexpr (K == 5) { asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x[c]) : "s"(0x511F53u)); }
            if constexpr (K == 6) { asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(f[c])); }
            if constexpr (K == 7) { asm volatile("v_sqrt_f32 %0, %0" : "+v"(f[c])); }
            if constexpr (K == 8) { asm volatile("v_fma_f64 %0, %0, %0, 1.0" : "+v"(d[c])); }
            if constexpr (K == 9) { asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[c]) : "v"(f[c])); }
            if constexpr (K == 10) { asm volatile("v_mul_f64 %0, %0, %0" : "+v"(d[c])); }
            if constexpr (K == 11) { asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(f[c])); }
            if constexpr (K == 12) { asm volatile("v_log_f32 %0, %0" : "+v"(f[c])); }
            if constexpr (K == 13) { asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(f[c])); }
            if constexpr (K == 14) { uint32_t sv; asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(sv) : "v"(x[c])); x[c] ^= sv; }
            if constexpr (K == 15) { asm volatile("v_mbcnt_lo_u32_b32 %0, %1, %0" : "+v"(x[c]) : "s"(0x12345u)); }
            if constexpr (K == 16) { asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(d[c])); }
            if constexpr (K == 17) { asm volatile("v_pk_add_f32 %0, %0, %0" : "+v"(d[c])); }
            if constexpr (K == 18) { asm volatile("v_pk_mul_f32 %0, %0, %0" : "+v"(d[c])); }
            if constexpr (K == 19) { asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[c]) : "v"(x[(c+1)%CHAINS]), "s"(msk)); }
            if constexpr (K == 20) { asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(x[c]) : "v"(x[(c+1)%CHAINS])); }
            if constexpr (K == 21) { asm volatile("v_bfi_b32 %0, %0, %1, %0" : "+v"(x[c]) : "v"(x[(c+1)%CHAINS])); }
            if constexpr (K == 22) { asm volatile("v_max3_f32 %0, %0, %0, 1.0" : "+v"(f[c])); }
            if constexpr (K == 23) { asm volatile("v_cmp_gt_f32 vcc, %0, 1.0" :: "v"(f[c]) : "vcc"); }
            if constexpr (K == 24) { asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(x[(c+1)%CHAINS])); }
            if constexpr (K == 25) { asm volatile("v_sub_f32 %0, %0, %1" : "+v"(f[c]) : "v"(f[(c+1)%CHAINS])); }
            if constexpr (K == 26) { asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f[c]) : "v"(f[(c+1)%CHAINS])); }
            if constexpr (K == 27) { asm volatile("v_lshlrev_b32 %0, 2, %0" : "+v"(x[c])); }
            if constexpr (K == 28) { asm volatile("v_cmp_gt_f32_e64 %0, %1, 1.0" : "=s"(msk) : "v"(f[c])); }
            if constexpr (K == 29) { asm volatile("v_mov_b32 %0, %1" : "=v"(x[c]) : "v"(x[(c+1)%CHAINS])); }
            if constexpr (K == 30) { asm volatile("v_add3_u32 %0, %0, %1, 7" : "+v"(x[c]) : "v"(x[(c+1)%CHAINS])); }
            if constexpr (K == 31) { asm volatile("v_med3_f32 %0, %0, %1, 1.0" : "+v"(f[c]) : "v"(f[(c+1)%CHAINS])); }
            if constexpr (K == 32) { asm volatile("v_cvt_f32_i32 %0, %1" : "=v"(f[c]) : "v"(x[c])); }
            if constexpr (K == 33) { asm volatile("v_xad_u32 %0, %0, %1, 3" : "+v"(x[c]) : "v"(x[(c+1)%CHAINS])); }
            if constexpr (K == 34) { asm volatile("v_sub_f32_e64 %0, |%0|, %1" : "+v"(f[c]) : "v"(f[(c+1)%CHAINS])); }
            if constexpr (K == 35) { asm volatile("v_max_f32 %0, %0, %1" : "+v"(f[c]) : "v"(f[(c+1)%CHAINS])); }
        }
    }
    uint32_t acc = 0;
    for (int c = 0; c < CHAINS; ++c) acc ^= x[c] ^ __float_as_uint(f[c]) ^ (uint32_t)__double_as_longlong(d[c]) ^ (uint32_t)msk;
    if (acc == 0x12345678u) out[0] = acc;
}

template <int K>
float run(uint32_t* out, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k<K>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    hipEventRecord(a);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k<K>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms / 3;
}

int main() {
    hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const double clk = p.clockRate * 1e3;   // Hz
    const int blocks = cus * 8;              // 8 blocks x 4 waves = 32 waves/CU = 8 per SIMD
    uint32_t* out; hipMalloc(&out, 4);
    const char* names[] = {"v_xor_b32", "v_mad_u64_u32", "v_mul_hi_u32", "v_mul_lo_u32", "v_mul_u32_u24",
                           "v_mul_hi_u32_u24", "v_fma_f32", "v_sqrt_f32", "v_fma_f64", "v_cvt_f64_f32",
                           "v_mul_f64", "v_cvt_f32_u32", "v_log_f32", "v_add_f32_dpp", "v_readfirstlane(+nop)", "v_mbcnt_lo", "v_pk_fma_f32", "v_pk_add_f32", "v_pk_mul_f32", "v_cndmask_b32", "v_lshl_add_u32", "v_bfi_b32", "v_max3_f32", "v_cmp_gt_f32(vcc)", "v_add_u32", "v_sub_f32", "v_mul_f32", "v_lshlrev_b32", "v_cmp_gt_f32_e64(sgpr)", "v_mov_b32", "v_add3_u32", "v_med3_f32", "v_cvt_f32_i32", "v_xad_u32", "v_sub_f32 |abs|", "v_max_f32"};
    float ms[36];
    ms[0] = run<0>(out, blocks); ms[1] = run<1>(out, blocks); ms[2] = run<2>(out, blocks); ms[3] = run<3>(out, blocks);
    ms[4] = run<4>(out, blocks); ms[5] = run<5>(out, blocks); ms[6] = run<6>(out, blocks); ms[7] = run<7>(out, blocks);
    ms[8] = run<8>(out, blocks); ms[9] = run<9>(out, blocks); ms[10] = run<10>(out, blocks); ms[11] = run<11>(out, blocks);
    ms[12] = run<12>(out, blocks); ms[13] = run<13>(out, blocks); ms[14] = run<14>(out, blocks); ms[15] = run<15>(out, blocks);
    ms[16] = run<16>(out, blocks); ms[17] = run<17>(out, blocks); ms[18] = run<18>(out, blocks); ms[19] = run<19>(out, blocks);
    ms[20] = run<20>(out, blocks); ms[21] = run<21>(out, blocks); ms[22] = run<22>(out, blocks); ms[23] = run<23>(out, blocks);
    ms[24] = run<24>(out, blocks); ms[25] = run<25>(out, blocks); ms[26] = run<26>(out, blocks); ms[27] = run<27>(out, blocks);
    ms[28] = run<28>(out, blocks); ms[29] = run<29>(out, blocks); ms[30] = run<30>(out, blocks); ms[31] = run<31>(out, blocks);
    ms[32] = run<32>(out, blocks); ms[33] = run<33>(out, blocks); ms[34] = run<34>(out, blocks); ms[35] = run<35>(out, blocks);
    const double wave_insts_per_simd = (double)blocks * 4 / (cus * 4) * ITERS * CHAINS;
    printf("CUs %d clock %.0f MHz\n", cus, clk / 1e6);
    for (int i = 0; i < 36; ++i)
        printf("%-22s %8.3f ms  %6.2f cycles per wave-instruction per SIMD\n", names[i], ms[i],
               ms[i] * 1e-3 * clk / wave_insts_per_simd);
    return 0;
}
