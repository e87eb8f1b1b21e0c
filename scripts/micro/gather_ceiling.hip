// gather_ceiling.hip -- measured ceilings for the partitioned instance's access pattern (config 5,
// DESIGN.md §5.1): uniformly random 4-byte gathers from a table, and uniformly random 4-byte
// scatter stores into one, one thread per access, coalesced index stream -- the roofline the
// clause / variable kernels are compared with (they are bound by random 4-byte accesses, not by
// streamed bytes).  Prints one JSON line per (kind, table size): accesses per second.
//   hipcc --offload-arch=gfx950 -O3 -o gather_ceiling gather_ceiling.hip && ./gather_ceiling
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

__global__ __launch_bounds__(256) void k_gather3(const float *__restrict__ tab, const uint32_t *__restrict__ idx,
                                                 float *__restrict__ out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // three independent gathers per thread, as a clause's three voltages
    const uint32_t a = __builtin_nontemporal_load(&idx[3 * i]), b = __builtin_nontemporal_load(&idx[3 * i + 1]),
                   c = __builtin_nontemporal_load(&idx[3 * i + 2]);
    const float x = tab[a], y = tab[b], z = tab[c];
    __builtin_nontemporal_store(x + y + z, &out[i]);
}

__global__ __launch_bounds__(256) void k_scatter3(float *__restrict__ tab, const uint32_t *__restrict__ idx, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t a = __builtin_nontemporal_load(&idx[3 * i]), b = __builtin_nontemporal_load(&idx[3 * i + 1]),
                   c = __builtin_nontemporal_load(&idx[3 * i + 2]);
    tab[a] = 1.0f;
    tab[b] = 2.0f;
    tab[c] = 3.0f;
}

static uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main() {
    const int64_t n = 4200000;  // threads = config 5's clauses; 3 accesses each
    std::vector<uint32_t> h(3 * n);
    float *dout;
    uint32_t *didx;
    CK(hipMalloc(&dout, n * 4));
    CK(hipMalloc(&didx, 3 * n * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int64_t sizes[] = {1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20};  // table entries (x4 bytes)
    for (int64_t entries : sizes) {
        for (int64_t i = 0; i < 3 * n; ++i) h[i] = (uint32_t)(mix((uint64_t)i * 7 + (uint64_t)entries) % (uint64_t)entries);
        float *tab;
        CK(hipMalloc(&tab, entries * 4));
        CK(hipMemset(tab, 0, entries * 4));
        CK(hipMemcpy(didx, h.data(), 3 * n * 4, hipMemcpyHostToDevice));
        const unsigned grid = (unsigned)((n + 255) / 256);
        for (int kind = 0; kind < 2; ++kind) {
            for (int w = 0; w < 3; ++w) {  // warmup
                if (kind == 0) hipLaunchKernelGGL(k_gather3, dim3(grid), dim3(256), 0, 0, tab, didx, dout, n);
                else hipLaunchKernelGGL(k_scatter3, dim3(grid), dim3(256), 0, 0, tab, didx, n);
            }
            const int reps = 20;
            CK(hipEventRecord(e0, 0));
            for (int r = 0; r < reps; ++r) {
                if (kind == 0) hipLaunchKernelGGL(k_gather3, dim3(grid), dim3(256), 0, 0, tab, didx, dout, n);
                else hipLaunchKernelGGL(k_scatter3, dim3(grid), dim3(256), 0, 0, tab, didx, n);
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / reps;
            std::printf("{\"kind\": \"%s\", \"table_bytes\": %lld, \"accesses\": %lld, \"us_per_launch\": %.2f, "
                        "\"G_accesses_per_s\": %.1f}\n",
                        kind == 0 ? "gather4B" : "scatter4B", (long long)(entries * 4), (long long)(3 * n), us,
                        3.0 * n / us / 1e3);
        }
        CK(hipFree(tab));
    }
    return 0;
}
