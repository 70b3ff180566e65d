// Which XCD (HW_REG_XCC_ID) runs workgroup b: the dispatch order the XCD-aware block remap and a
// single-XCD persistent launch rely on.  Prints the XCC of blocks 0..31 and, over a 4096-block grid,
// how many blocks with b % 8 == k ran on XCC k.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k(unsigned* out) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (threadIdx.x == 0) out[blockIdx.x] = xcc & 0xF;
}
int main() {
    const int nb = 4096;
    unsigned* d;
    if (hipMalloc(&d, sizeof(unsigned) * nb) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(nb), dim3(64), 0, 0, d);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    std::vector<unsigned> h(nb);
    if (hipMemcpy(h.data(), d, sizeof(unsigned) * nb, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("xcc of blocks 0..31:");
    for (int i = 0; i < 32; ++i) printf(" %u", h[i]);
    int match = 0;
    for (int i = 0; i < nb; ++i) match += h[i] == (unsigned)(i % 8);
    printf("\nblocks with xcc == b %% 8: %d of %d\n", match, nb);
    return 0;
}
