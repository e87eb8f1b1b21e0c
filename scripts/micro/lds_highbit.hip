// Does a DS read honour address bits above the LDS size?  Lane l reads word l at byte address
// 4 l | 0x80000000 (and | 0x00040000), against the plain read.  Prints the first mismatches.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) float lf;
__global__ void k(float *out) {
    __shared__ float s[64];
    const int l = threadIdx.x;
    s[l] = 1.0f + l;
    __syncthreads();
    const unsigned a = (unsigned)(size_t)(const lf *)&s[l];  // this lane's word's LDS byte address
    out[l] = *reinterpret_cast<const lf *>(a);
    out[64 + l] = *reinterpret_cast<const lf *>(a | 0x80000000u);
    out[128 + l] = *reinterpret_cast<const lf *>(a | 0x00040000u);
}
int main() {
    float *d, h[192];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int same31 = 0, same18 = 0;
    for (int l = 0; l < 64; ++l) {
        same31 += h[64 + l] == h[l];
        same18 += h[128 + l] == h[l];
    }
    printf("plain[5]=%g bit31[5]=%g bit18[5]=%g  lanes equal: bit31 %d/64, bit18 %d/64\n", h[5], h[69], h[133], same31, same18);
    return 0;
}
