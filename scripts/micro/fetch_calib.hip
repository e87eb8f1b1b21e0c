// fetch_calib.hip -- what rocprofv3's FETCH_SIZE / WRITE_SIZE (and the TCC_EA0 request counters they
// are derived from) count on gfx950, per access width and per cache level (VERDICT r4 "Next #2").
// Every dispatch moves a KNOWN number of bytes in one access shape; scripts/fetch_calib_report.py
// divides each counter-derived byte figure by that number.  Shapes (the product kernels' own):
//   read4 / read8 / read16   coalesced streaming reads, 4 / 8 / 16 B per lane, 1 GiB (> the 256 MiB
//                            Infinity Cache), after a 1 GiB flush write: every byte from HBM once
//   read16_mall_cold/_warm   64 MiB read twice back to back: the second read is served by the Infinity
//                            Cache (64 MiB > the 32 MiB of L2), so equal counts mean the L2-side
//                            counters include Infinity-Cache hits
//   rows256                  random 256-B rows (64 lanes x 4 B: k_step's voltage rows), each row of a
//                            1 GiB table once
//   rows512                  random 512-B rows (64 lanes x 8 B: k_step's clause-memory rows), 1 GiB
//   gather4_l2               12.6 M random 4-B reads from a 4 MiB table (config 5's voltage gathers)
//   gather4_hbm              12.6 M random 4-B reads from a 1 GiB table
//   write4 / write8 / write16  coalesced streaming stores, 1 GiB
//   rows256_write            random 256-B row stores, each row of a 1 GiB table once
// One JSON line per dispatch on stdout: name, bytes, microseconds (HIP events).
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip && ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float hsum(float x) { return x; }
__device__ __forceinline__ float hsum(f2 x) { return x.x + x.y; }
__device__ __forceinline__ float hsum(f4 x) { return x.x + x.y + x.z + x.w; }

// The buffers hold zeros, so the sink store never happens; the compiler cannot know that.
template <typename T, int TAG>
__global__ __launch_bounds__(256) void k_read(const T *__restrict__ p, int64_t n, float *sink) {
    float acc = 0.f;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) acc += hsum(p[i]);
    if (acc == 1234.5f) sink[threadIdx.x] = acc;
}

template <typename T, int TAG>
__global__ __launch_bounds__(256) void k_write(T *__restrict__ p, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = T(0.f);
}

// wave-granular random rows: row r of the visit order is (r * mult) % nrows (mult odd, nrows a power
// of two: a bijection), each of a row's 64 lanes reads one element of type T (256 or 512 B per row)
template <typename T, int TAG>
__global__ __launch_bounds__(256) void k_rows(const T *__restrict__ p, int64_t nrows, uint64_t mult, float *sink) {
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x / 64);
    const int lane = threadIdx.x & 63;
    float acc = 0.f;
    for (int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); r < nrows; r += waves) {
        const int64_t row = (int64_t)(((uint64_t)r * mult) & (uint64_t)(nrows - 1));
        acc += hsum(p[row * 64 + lane]);
    }
    if (acc == 1234.5f) sink[threadIdx.x] = acc;
}

template <int TAG>
__global__ __launch_bounds__(256) void k_rows_write(float *__restrict__ p, int64_t nrows, uint64_t mult) {
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x / 64);
    const int lane = threadIdx.x & 63;
    for (int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); r < nrows; r += waves) {
        const int64_t row = (int64_t)(((uint64_t)r * mult) & (uint64_t)(nrows - 1));
        p[row * 64 + lane] = 0.f;
    }
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// uniformly random 4-B reads (each lane its own address)
template <int TAG>
__global__ __launch_bounds__(256) void k_gather4(const float *__restrict__ p, uint32_t mask, int64_t accesses, float *sink) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < accesses; i += stride)
        acc += p[mix((uint32_t)i * 2654435761U + TAG) & mask];
    if (acc == 1234.5f) sink[threadIdx.x] = acc;
}

struct Timer {
    hipEvent_t a, b;
    Timer() {
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
    }
};

static void report(const char *name, double bytes, float ms, const char *note) {
    std::printf("{\"name\": \"%s\", \"bytes\": %.0f, \"us\": %.2f, \"GBps\": %.1f, \"note\": \"%s\"}\n", name, bytes,
                ms * 1e3, bytes / (ms * 1e-3) / 1e9, note);
    std::fflush(stdout);
}

int main() {
    const int64_t GiB = 1ll << 30, MiB = 1ll << 20;
    float *big = nullptr, *flush = nullptr, *small = nullptr, *sink = nullptr;
    CK(hipMalloc(&big, GiB));
    CK(hipMalloc(&flush, GiB));
    CK(hipMalloc(&small, 64 * MiB));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(big, 0, GiB));
    CK(hipMemset(small, 0, 64 * MiB));
    CK(hipDeviceSynchronize());
    const dim3 grid(256 * 16), block(256);  // 16 workgroups of 4 waves per CU
    Timer t;
    float ms = 0.f;
#define RUN(name, bytes, note, ...)                                      \
    do {                                                                 \
        CK(hipEventRecord(t.a));                                         \
        __VA_ARGS__;                                                     \
        CK(hipGetLastError());                                           \
        CK(hipEventRecord(t.b));                                         \
        CK(hipEventSynchronize(t.b));                                    \
        CK(hipEventElapsedTime(&ms, t.a, t.b));                          \
        report(name, (double)(bytes), ms, note);                         \
    } while (0)
    // the flush: 1 GiB of 16-B stores to another buffer evicts the Infinity Cache (k_write<f4, 0>)
#define FLUSH() RUN("flush", GiB, "1 GiB of 16-B stores to another buffer", hipLaunchKernelGGL((k_write<f4, 0>), grid, block, 0, 0, (f4 *)flush, GiB / 16))

    FLUSH();
    RUN("read16", GiB, "coalesced 16 B/lane, 1 GiB, cold", hipLaunchKernelGGL((k_read<f4, 1>), grid, block, 0, 0, (const f4 *)big, GiB / 16, sink));
    FLUSH();
    RUN("read8", GiB, "coalesced 8 B/lane, 1 GiB, cold", hipLaunchKernelGGL((k_read<f2, 1>), grid, block, 0, 0, (const f2 *)big, GiB / 8, sink));
    FLUSH();
    RUN("read4", GiB, "coalesced 4 B/lane, 1 GiB, cold", hipLaunchKernelGGL((k_read<float, 1>), grid, block, 0, 0, (const float *)big, GiB / 4, sink));
    FLUSH();
    RUN("read16_mall_cold", 64 * MiB, "coalesced 16 B/lane, 64 MiB, cold", hipLaunchKernelGGL((k_read<f4, 2>), grid, block, 0, 0, (const f4 *)small, 64 * MiB / 16, sink));
    RUN("read16_mall_warm", 64 * MiB, "the same 64 MiB again (Infinity-Cache resident, larger than the L2s)", hipLaunchKernelGGL((k_read<f4, 3>), grid, block, 0, 0, (const f4 *)small, 64 * MiB / 16, sink));
    RUN("read4_mall_warm", 64 * MiB, "the same 64 MiB again, 4 B/lane", hipLaunchKernelGGL((k_read<float, 3>), grid, block, 0, 0, (const float *)small, 64 * MiB / 4, sink));
    FLUSH();
    RUN("rows256", GiB, "random 256-B rows (64 lanes x 4 B), each row of 1 GiB once, cold", hipLaunchKernelGGL((k_rows<float, 1>), grid, block, 0, 0, (const float *)big, GiB / 256, 0x9E3779B97F4A7C15ull, sink));
    FLUSH();
    RUN("rows512", GiB, "random 512-B rows (64 lanes x 8 B), each row of 1 GiB once, cold", hipLaunchKernelGGL((k_rows<f2, 1>), grid, block, 0, 0, (const f2 *)big, GiB / 512, 0x9E3779B97F4A7C15ull, sink));
    FLUSH();
    const int64_t G = 12600000;
    RUN("gather4_l2", 4 * G, "12.6 M random 4-B reads from a 4 MiB table (bytes = 4 per access)", hipLaunchKernelGGL((k_gather4<1>), grid, block, 0, 0, (const float *)big, (uint32_t)(MiB - 1), G, sink));
    FLUSH();
    RUN("gather4_hbm", 4 * G, "12.6 M random 4-B reads from a 1 GiB table (bytes = 4 per access)", hipLaunchKernelGGL((k_gather4<2>), grid, block, 0, 0, (const float *)big, (uint32_t)(GiB / 4 - 1), G, sink));
    FLUSH();
    RUN("write16", GiB, "coalesced 16 B/lane stores, 1 GiB", hipLaunchKernelGGL((k_write<f4, 1>), grid, block, 0, 0, (f4 *)big, GiB / 16));
    RUN("write8", GiB, "coalesced 8 B/lane stores, 1 GiB", hipLaunchKernelGGL((k_write<f2, 1>), grid, block, 0, 0, (f2 *)big, GiB / 8));
    RUN("write4", GiB, "coalesced 4 B/lane stores, 1 GiB", hipLaunchKernelGGL((k_write<float, 1>), grid, block, 0, 0, (float *)big, GiB / 4));
    RUN("rows256_write", GiB, "random 256-B row stores, each row of 1 GiB once", hipLaunchKernelGGL((k_rows_write<1>), grid, block, 0, 0, big, GiB / 256, 0x9E3779B97F4A7C15ull));
    CK(hipDeviceSynchronize());
    CK(hipFree(big));
    CK(hipFree(flush));
    CK(hipFree(small));
    CK(hipFree(sink));
    return 0;
}
