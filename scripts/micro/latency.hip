// latency.hip -- the latencies the B = 1 latency kernels (k_solo_fast, k_solo_cv) are
// made of, on one workgroup of NT threads (s_memtime cycles per operation, one JSON line each):
//   add_f64 / mul_f64 / min_f64    a dependent chain of that instruction (16 per unrolled round)
//   add_f64_x3                      three independent chains interleaved (the fold of 3 variables)
//   ds_read_b32_chain               a dependent LDS pointer chase (address = loaded value)
//   ds_read_b128_x12                12 independent 16-byte reads per lane from random blocks (80-byte
//                                   stride, conflicts as in k_solo_cv), then their sum: per round (the
//                                   next round's addresses wait for the sum)
//   ds_read_b128_x12_bcast          the same 12 reads all from one block (broadcast)
//   ds_read_b128_x12_Kway           the same reads with exactly K distinct blocks on each bank set of a
//                                   16-lane group (1: conflict-free)
//   handoff                         ds_write, s_waitcnt, s_barrier, ds_read of another lane's word: per
//                                   round (the exchange k_solo_cv does twice per adaptive step)
//   hipcc --offload-arch=gfx950 -O3 -o latency latency.hip && ./latency
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

constexpr int ROUNDS = 256;

__device__ __forceinline__ long long now() {
    long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

template <int KIND>
__global__ __launch_bounds__(512) void k_lat(double *sink, long long *cyc, double a, int salt) {
    __shared__ __attribute__((aligned(16))) double lds[8192];
    const int l = threadIdx.x;
    for (int i = l; i < 8192; i += blockDim.x) lds[i] = (double)(i % 7) * 1e-3;
    __shared__ int ptr[1024];
    for (int i = l; i < 1024; i += blockDim.x) ptr[i] = (i * 389 + 17) % 1024;
    __syncthreads();
    double x = a + l, y = a - l, z = a * 0.5 + l;
    int p = l;
    long long t0 = now();
    for (int r = 0; r < ROUNDS; ++r) {
        if constexpr (KIND == 0) {
#pragma unroll
            for (int u = 0; u < 16; ++u) x = x + a;
        } else if constexpr (KIND == 1) {
#pragma unroll
            for (int u = 0; u < 16; ++u) x = x * a;
        } else if constexpr (KIND == 2) {
#pragma unroll
            for (int u = 0; u < 16; ++u) x = fmin(x, a + u);
        } else if constexpr (KIND == 3) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                x = x + a;
                y = y + a;
                z = z + a;
            }
        } else if constexpr (KIND == 4) {
#pragma unroll
            for (int u = 0; u < 16; ++u) p = ptr[(p + salt) & 1023];
        } else if constexpr (KIND == 5 || KIND == 6) {
            typedef double TV __attribute__((ext_vector_type(2)));
            TV s = {0.0, 0.0};
            TV t[12];
            const int dep = x > 1e300 ? 1 : 0;  // the round's reads wait for the previous round's sum
#pragma unroll
            for (int j = 0; j < 12; ++j) {
                const int blk = (KIND == 5 ? ((l * 37 + j * 11 + r * 5 + salt) % 100) : 0) + dep;
                t[j] = *reinterpret_cast<const TV *>(lds + blk * 10 + (j & 3) * 2);
            }
#pragma unroll
            for (int j = 0; j < 12; ++j) s = s + t[j];
            x = x + s.x + s.y;
        } else if constexpr (KIND >= 10) {  // 12 reads per round, (KIND - 10)-way conflicts per 16-lane group
            constexpr int K = KIND - 10, S = 16 / K;
            typedef double TV __attribute__((ext_vector_type(2)));
            TV s = {0.0, 0.0};
            TV t[12];
            const int dep = x > 1e300 ? 1 : 0;
            const int blk = (l % 16) % S + 16 * ((l % 16) / S) + 16 * dep;
#pragma unroll
            for (int j = 0; j < 12; ++j) t[j] = *reinterpret_cast<const TV *>(lds + blk * 10 + (j & 3) * 2);
#pragma unroll
            for (int j = 0; j < 12; ++j) s = s + t[j];
            x = x + s.x + s.y;
        } else if constexpr (KIND == 7) {
            lds[4096 + l] = x;
            __syncthreads();
            x = x + lds[4096 + (l + 64 + salt) % blockDim.x];
            __syncthreads();
        }
    }
    long long t1 = now();
    if (l == 0) cyc[0] = t1 - t0;
    sink[l] = x + y + z + p;
}

template <int KIND> int run(const char *name, int nt, int per_round) {
    double *sink;
    long long *cyc, h = 0;
    CK(hipMalloc(&sink, 1024 * 8));
    CK(hipMalloc(&cyc, 8));
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_lat<KIND>, dim3(1), dim3(nt), 0, 0, sink, cyc, 1.0000001, 0);
        CK(hipDeviceSynchronize());
    }
    CK(hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost));
    printf("{\"kind\": \"%s\", \"threads\": %d, \"cycles_per_op\": %.2f}\n", name, nt,
           (double)h / ROUNDS / per_round);
    CK(hipFree(sink));
    CK(hipFree(cyc));
    return 0;
}

int main() {
    for (int nt : {64, 192}) {
        if (run<0>("add_f64", nt, 16) || run<1>("mul_f64", nt, 16) || run<2>("min_f64", nt, 16) ||
            run<3>("add_f64_x3", nt, 16) || run<4>("ds_read_b32_chain", nt, 16) ||
            run<5>("ds_read_b128_x12_round", nt, 1) || run<6>("ds_read_b128_x12_bcast_round", nt, 1) ||
            run<7>("handoff_round", nt, 2) || run<11>("ds_read_b128_x12_1way_round", nt, 1) ||
            run<12>("ds_read_b128_x12_2way_round", nt, 1) || run<14>("ds_read_b128_x12_4way_round", nt, 1) ||
            run<18>("ds_read_b128_x12_8way_round", nt, 1) || run<26>("ds_read_b128_x12_16way_round", nt, 1))
            return 1;
    }
    return 0;
}
