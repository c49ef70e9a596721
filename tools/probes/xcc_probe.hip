// Records the XCC (XCD) id each workgroup of a 1-D grid runs on, for a
// sequence of launches of different sizes on one stream: is block i on XCD
// (block 0's XCD + i) % 8, and does block 0 land on the same XCD in every
// launch?  (Decides whether a batch-major XCD remap keeps a batch item's
// activations in one XCD's L2 from one kernel to the next.)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void xcc_kernel(int* out) {
    if (threadIdx.x == 0) {
        // s_getreg_b32 hwreg(HW_REG_XCC_ID = 20, offset 0, size 4)
        const int id = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15;
        out[blockIdx.x] = id;
    }
}

int main() {
    const int grids[] = {1024, 1024, 256, 1000, 1024, 37, 512, 2048, 256, 256, 96, 1024};
    const int n = sizeof(grids) / sizeof(grids[0]);
    int* d;
    hipMalloc(&d, 4096 * sizeof(int) * n);
    for (int l = 0; l < n; ++l) hipLaunchKernelGGL(xcc_kernel, dim3(grids[l]), dim3(256), 0, 0, d + 4096 * l);
    hipDeviceSynchronize();
    std::vector<int> h(4096 * n);
    hipMemcpy(h.data(), d, h.size() * sizeof(int), hipMemcpyDeviceToHost);
    for (int l = 0; l < n; ++l) {
        const int* x = h.data() + 4096 * l;
        int rr = 0;
        for (int i = 0; i < grids[l]; ++i) rr += x[i] == (x[0] + i) % 8;
        printf("launch %2d grid %5d: block0 xcc %d, blocks on (xcc0+i)%%8: %d/%d; first 16:", l, grids[l], x[0], rr,
               grids[l]);
        for (int i = 0; i < 16 && i < grids[l]; ++i) printf(" %d", x[i]);
        printf("\n");
    }
    hipFree(d);
    return 0;
}
