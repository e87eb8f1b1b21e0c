// row_ceiling.hip -- measured ceilings for config 4's access shape (VERDICT r2 "Next
// #2"): the FUSED step (k_step, kernels.hpp) of B = 1024 replicas of a random 3-SAT instance with
// n = 50 000, m = 210 000, stripped of its arithmetic.  16 groups of 64 replicas, replica-innermost:
// a voltage row is 256 B (V[g][i][64], 205 MB in all), a clause-memory row 512 B (C[g][c][64][2],
// 1.72 GB).  A wave owns 16 consecutive variables of one group and walks their incidences in
// variable-major order (the reference's fold order), issuing 8 incidences' loads before using them.
// Per incidence it gathers the clause's voltage rows and memory row exactly as k_step does; the
// clause's first literal stores the memory row to the other buffer, and every variable's voltage
// row is stored once.  Variants (one JSON line each, microseconds per step):
//   fused      k_step's loads: 3 voltage rows + the memory row per incidence
//   other_v    the two OTHER voltage rows only (the own row is the wave's current variable)
//   owner_mem  3 voltage rows, the memory row only at the owning incidence (a design that reads
//              each clause's memories once -- the best any re-layout of the memory reads could do)
//   owner_min  2 voltage rows + the memory row at the owner only
//   owner_tt   a realisable owner-only design (round 4): 3 voltage rows; the owning
//              incidence reads the memory row, stores it and stores the clause's product row
//              tt = xl xs (256 B, a buffer of its own); the other two incidences read that product
//              row (written by the previous step's owner) instead of the memory row
//   owner_tt_min  the same with the two OTHER voltage rows only
//   stream     the compulsory bytes as one coalesced read + write pass over v and the memories
//              (SURVEY.md §8d's 3.85 GB per step: the HBM-streaming floor)
//   hipcc --offload-arch=gfx950 -O3 -o row_ceiling row_ceiling.hip && ./row_ceiling
#include <hip/hip_runtime.h>

#include <algorithm>
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

constexpr int N = 50000, M = 210000, G = 16, W = 64, ROWS = 16, RB = 8;

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

struct alignas(16) Inc {
    int32_t x, y, z, w;  // clause << 2 | own position, the clause's three variables
};

template <bool OWNV, bool MEMALL, bool TT = false>
__global__ __launch_bounds__(256) void k_rows(const Inc *__restrict__ inc, const int32_t *__restrict__ vptr,
                                              const float *__restrict__ V, float *__restrict__ Vn,
                                              const f2 *__restrict__ CM, f2 *__restrict__ CMn,
                                              const float *__restrict__ TTr = nullptr, float *__restrict__ TTw = nullptr) {
    const int wave = (int)(blockIdx.x * 4 + (threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int tiles = (N + ROWS - 1) / ROWS;
    // XCD-aware like k_step's xmode 1: group g's waves on blocks b with b % 8 == g % 8
    const int b = (int)blockIdx.x, x = b & 7, k = b >> 3, bpg = (tiles + 3) / 4;
    const int g = x + 8 * (k / bpg), tb = k % bpg;
    if (g >= G) return;
    const int tile = tb * 4 + (int)(threadIdx.x >> 6);
    if (tile >= tiles) return;
    (void)wave;
    const int i0 = tile * ROWS, i1 = min(i0 + ROWS, N);
    const int P0 = vptr[i0], P1 = vptr[i1];
    const float *Vg = V + (size_t)g * N * W + lane;
    const f2 *Cg = CM + (size_t)g * M * W + lane;
    f2 *Cn = CMn + (size_t)g * M * W + lane;
    float acc = 0.0f;
    int cur = i0;
    for (int p0 = P0; p0 < P1; p0 += RB) {
        Inc r[RB];
#pragma unroll
        for (int j = 0; j < RB; ++j) r[j] = inc[min(p0 + j, P1 - 1)];
        float a[RB][3];
        f2 mm[RB];
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            const int own = r[j].x & 3;
            a[j][0] = (OWNV || own != 0) ? Vg[(size_t)r[j].y * W] : 0.0f;
            a[j][1] = (OWNV || own != 1) ? Vg[(size_t)r[j].z * W] : 0.0f;
            a[j][2] = (OWNV || own != 2) ? Vg[(size_t)r[j].w * W] : 0.0f;
            mm[j] = (MEMALL || own == 0) ? __builtin_nontemporal_load(&Cg[(size_t)(r[j].x >> 2) * W])
                                         : f2{0.0f, 0.0f};
            if (TT && own != 0) mm[j].x = TTr[(size_t)g * M * W + (size_t)(r[j].x >> 2) * W + lane];
        }
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            if (p0 + j >= P1) break;
            acc += a[j][0] + a[j][1] + a[j][2] + mm[j].x;
            if ((r[j].x & 3) == 0) {
                f2 o = mm[j];
                o.y += acc;
                __builtin_nontemporal_store(o, &Cn[(size_t)(r[j].x >> 2) * W]);
                if (TT) TTw[(size_t)g * M * W + (size_t)(r[j].x >> 2) * W + lane] = o.x * o.y;
            }
        }
        // voltage rows of the variables finished so far (one store per variable, as k_step)
        while (cur < i1 && vptr[cur + 1] <= min(p0 + RB, P1)) {
            __builtin_nontemporal_store(acc, &Vn[(size_t)g * N * W + (size_t)cur * W + lane]);
            ++cur;
        }
    }
    for (; cur < i1; ++cur) __builtin_nontemporal_store(acc, &Vn[(size_t)g * N * W + (size_t)cur * W + lane]);
}

// the compulsory bytes once: v and the memories read and written, coalesced (16 B per lane)
__global__ __launch_bounds__(256) void k_stream(const f4 *__restrict__ a, f4 *__restrict__ b, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        f4 v = __builtin_nontemporal_load(&a[i]);
        v.x += 1.0f;
        __builtin_nontemporal_store(v, &b[i]);
    }
}

static uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main() {
    // random 3-SAT: three distinct variables per clause
    std::vector<int32_t> cv(3 * (size_t)M);
    for (int c = 0; c < M; ++c) {
        uint64_t s = (uint64_t)c * 3;
        for (int j = 0; j < 3; ++j) {
            int v;
            do v = (int)(mix(s++ * 0x100000001ull + 3) % N);
            while ((j > 0 && v == cv[3 * c]) || (j > 1 && v == cv[3 * c + 1]));
            cv[3 * c + j] = v;
        }
    }
    // variable-major incidences sorted by (variable, clause)
    std::vector<int32_t> deg(N + 1, 0);
    for (int32_t v : cv) deg[v + 1]++;
    std::vector<int32_t> vptr(N + 1, 0);
    for (int i = 0; i < N; ++i) vptr[i + 1] = vptr[i] + deg[i + 1];
    std::vector<Inc> incs(3 * (size_t)M);
    std::vector<int32_t> fill(vptr.begin(), vptr.end() - 1);
    for (int c = 0; c < M; ++c)
        for (int j = 0; j < 3; ++j) incs[fill[cv[3 * c + j]]++] = Inc{c << 2 | j, cv[3 * c], cv[3 * c + 1], cv[3 * c + 2]};

    Inc *dinc;
    int32_t *dvptr;
    float *V0, *V1;
    f2 *C0, *C1;
    const size_t vbytes = (size_t)G * N * W * 4, cbytes = (size_t)G * M * W * 8;
    CK(hipMalloc(&dinc, incs.size() * sizeof(Inc)));
    CK(hipMalloc(&dvptr, vptr.size() * 4));
    CK(hipMalloc(&V0, vbytes));
    CK(hipMalloc(&V1, vbytes));
    CK(hipMalloc(&C0, cbytes));
    CK(hipMalloc(&C1, cbytes));
    CK(hipMemcpy(dinc, incs.data(), incs.size() * sizeof(Inc), hipMemcpyHostToDevice));
    CK(hipMemcpy(dvptr, vptr.data(), vptr.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(V0, 0, vbytes));
    CK(hipMemset(V1, 0, vbytes));
    CK(hipMemset(C0, 0, cbytes));
    CK(hipMemset(C1, 0, cbytes));
    float *T0, *T1;
    CK(hipMalloc(&T0, cbytes / 2));
    CK(hipMalloc(&T1, cbytes / 2));
    CK(hipMemset(T0, 0, cbytes / 2));
    CK(hipMemset(T1, 0, cbytes / 2));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int tiles = (N + ROWS - 1) / ROWS, bpg = (tiles + 3) / 4;
    const dim3 grid((unsigned)(G * bpg)), block(256);
    const double alg_bytes = (8.0 * N + 16.0 * M) * G * W;  // SURVEY.md §8d per step
    auto run = [&](const char *name, auto launch) -> int {
        for (int w = 0; w < 3; ++w) launch(w & 1);
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) launch(r & 1);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        std::printf("{\"variant\": \"%s\", \"us_per_step\": %.1f, \"algorithmic_TBps\": %.2f}\n", name, us,
                    alg_bytes / us / 1e6);
        return 0;
    };
#define ROWS_LAUNCH(OWNV, MEMALL)                                                                                \
    [&](int par) {                                                                                               \
        hipLaunchKernelGGL((k_rows<OWNV, MEMALL>), grid, block, 0, 0, dinc, dvptr, par ? V1 : V0, par ? V0 : V1, \
                           par ? C1 : C0, par ? C0 : C1);                                                        \
    }
    if (run("fused", ROWS_LAUNCH(true, true))) return 1;
    if (run("other_v", ROWS_LAUNCH(false, true))) return 1;
    if (run("owner_mem", ROWS_LAUNCH(true, false))) return 1;
    if (run("owner_min", ROWS_LAUNCH(false, false))) return 1;
#define TT_LAUNCH(OWNV)                                                                                         \
    [&](int par) {                                                                                               \
        hipLaunchKernelGGL((k_rows<OWNV, false, true>), grid, block, 0, 0, dinc, dvptr, par ? V1 : V0,          \
                           par ? V0 : V1, par ? C1 : C0, par ? C0 : C1, par ? T1 : T0, par ? T0 : T1);         \
    }
    if (run("owner_tt", TT_LAUNCH(true))) return 1;
    if (run("owner_tt_min", TT_LAUNCH(false))) return 1;
    if (run("stream", [&](int par) {
            const int64_t v4 = (int64_t)(vbytes / 16), c4 = (int64_t)(cbytes / 16);
            hipLaunchKernelGGL(k_stream, dim3(4096), block, 0, 0, (const f4 *)(par ? V1 : V0),
                               (f4 *)(par ? V0 : V1), v4);
            hipLaunchKernelGGL(k_stream, dim3(4096), block, 0, 0, (const f4 *)(par ? C1 : C0),
                               (f4 *)(par ? C0 : C1), c4);
        }))
        return 1;
    return 0;
}
