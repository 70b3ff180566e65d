// Probe of the HW_ID / XCC_ID register fields on gfx950 (hardware wave-slot identity), used to size
// the subsweep's per-wave-slot overflow scratch.  Prints the max of each field and the number of
// distinct slots seen while a grid of one-wave workgroups (5 KiB LDS each: 32 waves per CU) runs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <vector>

__global__ __launch_bounds__(64) void k(unsigned* out, int spin) {
    extern __shared__ float sm[];
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    sm[threadIdx.x] = (float)hw;
    long long t0 = clock64();
    while (clock64() - t0 < spin) {}
    if (threadIdx.x == 0) { out[2 * blockIdx.x] = hw; out[2 * blockIdx.x + 1] = xcc + (unsigned)sm[1] * 0u; }
}

int main() {
    const int nb = 65536;
    unsigned* d;
    hipMalloc(&d, sizeof(unsigned) * 2 * nb);
    hipLaunchKernelGGL(k, dim3(nb), dim3(64), 5120, 0, d, 20000);
    hipDeviceSynchronize();
    std::vector<unsigned> h(2 * nb);
    hipMemcpy(h.data(), d, sizeof(unsigned) * 2 * nb, hipMemcpyDeviceToHost);
    unsigned mx[8] = {0};
    std::set<unsigned long long> slots;
    for (int i = 0; i < nb; ++i) {
        unsigned hw = h[2 * i], xcc = h[2 * i + 1] & 0xF;
        unsigned f[7] = {hw & 0xF, (hw >> 4) & 3, (hw >> 8) & 0xF, (hw >> 12) & 1, (hw >> 13) & 7, (hw >> 16) & 0xF, xcc};
        for (int j = 0; j < 7; ++j) mx[j] = f[j] > mx[j] ? f[j] : mx[j];
        slots.insert(((unsigned long long)xcc << 32) | (hw & 0xFFFF));
    }
    printf("max wave %u simd %u cu %u sh %u se %u tg %u xcc %u; distinct (xcc, hw[15:0]) %zu\n", mx[0], mx[1],
           mx[2], mx[3], mx[4], mx[5], mx[6], slots.size());
    return 0;
}
