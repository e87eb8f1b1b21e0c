// quarter_rows.hip -- the access-pattern ceiling of a config-4 FUSED step laid out for the L2 (round 5,
// VERDICT r4 "Next #3"): k_step (kernels.hpp) stripped of its arithmetic, in two layouts.
//   w64       today's layout: 16 groups of 64 replicas, a voltage row = 256 B (V[g][i][64], 12.8 MB a
//             group, two groups per XCD: 25.6 MB against a 4 MiB L2), a wave = one variable's
//             incidences x 64 replicas, 8 incidences' loads in flight (k_step's RB = 4, double-buffered)
//   q16       64 groups of 16 replicas: a voltage row = 64 B and a group's table 3.2 MB, which FITS an
//             XCD's L2.  A wave = 4 incidences of one variable x 16 replicas (quarter q of the wave takes
//             incidence p + q), so the records, voltage rows and memory rows stay one per quarter; the
//             4 incidences' terms are added in the reference's order through 3 cross-quarter shuffles.
//             XCD x steps groups x, x + 8, ... one after another (a group at a time per L2):
//               q16_1  one launch per step, blocks ordered so XCD x's blocks take its groups in turn
//               q16_8  eight launches per step, launch k = groups 8k .. 8k + 7 (one per XCD)
// The memory rows are read per incidence (3 per clause, as k_step) with non-temporal loads and the owner
// stores them; every variable's voltage row is stored once.  Microseconds per step of 1024 replicas,
// one JSON line per variant; algorithmic TB/s = SURVEY.md §8d's 3.85 GB / the step time.
//   hipcc --offload-arch=gfx950 -O3 -o quarter_rows quarter_rows.hip && ./quarter_rows
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

constexpr int N = 50000, M = 210000, B = 1024, ROWS = 16, RB = 8;

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

struct alignas(16) Inc {
    int32_t x, y, z, w;  // clause << 2 | own position, the clause's three variables
};

// W = 64: k_step's loads (row_ceiling.hip's `fused`)
__global__ __launch_bounds__(256) void k_w64(const Inc *__restrict__ inc, const int32_t *__restrict__ vptr,
                                             const float *__restrict__ V, float *__restrict__ Vn,
                                             const f2 *__restrict__ CM, f2 *__restrict__ CMn) {
    constexpr int W = 64, G = B / W;
    const int lane = threadIdx.x & 63;
    const int tiles = (N + ROWS - 1) / ROWS;
    const int b = (int)blockIdx.x, x = b & 7, k = b >> 3, bpg = (tiles + 3) / 4;
    const int g = x + 8 * (k / bpg), tb = k % bpg;
    if (g >= G) return;
    const int tile = tb * 4 + (int)(threadIdx.x >> 6);
    if (tile >= tiles) return;
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
            a[j][0] = Vg[(size_t)r[j].y * W];
            a[j][1] = Vg[(size_t)r[j].z * W];
            a[j][2] = Vg[(size_t)r[j].w * W];
            mm[j] = __builtin_nontemporal_load(&Cg[(size_t)(r[j].x >> 2) * W]);
        }
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            if (p0 + j >= P1) break;
            acc += a[j][0] + a[j][1] + a[j][2] + mm[j].x;
            if ((r[j].x & 3) == 0) {
                f2 o = mm[j];
                o.y += acc;
                __builtin_nontemporal_store(o, &Cn[(size_t)(r[j].x >> 2) * W]);
            }
        }
        while (cur < i1 && vptr[cur + 1] <= min(p0 + RB, P1)) {
            __builtin_nontemporal_store(acc, &Vn[(size_t)g * N * W + (size_t)cur * W + lane]);
            ++cur;
        }
    }
    for (; cur < i1; ++cur) __builtin_nontemporal_store(acc, &Vn[(size_t)g * N * W + (size_t)cur * W + lane]);
}

// W = 16, quarter waves.  g0: first group of this launch; per_xcd: groups each XCD steps in turn.
template <bool NT_V>
__global__ __launch_bounds__(256) void k_q16(const Inc *__restrict__ inc, const int32_t *__restrict__ vptr,
                                             const float *__restrict__ V, float *__restrict__ Vn,
                                             const f2 *__restrict__ CM, f2 *__restrict__ CMn, int g0,
                                             int per_xcd) {
    constexpr int W = 16, G = B / W, RQ = RB / 4;  // RQ quads of 4 incidences in flight
    const int lane = threadIdx.x & 63, q = lane >> 4, rr = lane & 15;
    const int tiles = (N + ROWS - 1) / ROWS;
    const int b = (int)blockIdx.x, x = b & 7, k = b >> 3, bpg = (tiles + 3) / 4;
    const int slot = k / bpg, tb = k % bpg;
    if (slot >= per_xcd) return;
    const int g = g0 + x + 8 * slot;
    if (g >= G) return;
    const int tile = tb * 4 + (int)(threadIdx.x >> 6);
    if (tile >= tiles) return;
    const int i0 = tile * ROWS, i1 = min(i0 + ROWS, N);
    const int P0 = vptr[i0], P1 = vptr[i1];
    const float *Vg = V + (size_t)g * N * W + rr;
    const f2 *Cg = CM + (size_t)g * M * W + rr;
    f2 *Cn = CMn + (size_t)g * M * W + rr;
    float acc = 0.0f;
    int cur = i0;
    for (int p0 = P0; p0 < P1; p0 += RB) {
        Inc r[RQ];
#pragma unroll
        for (int j = 0; j < RQ; ++j) r[j] = inc[min(p0 + 4 * j + q, P1 - 1)];  // one record per quarter
        float a[RQ][3];
        f2 mm[RQ];
#pragma unroll
        for (int j = 0; j < RQ; ++j) {
            if (NT_V) {
                a[j][0] = __builtin_nontemporal_load(&Vg[(size_t)r[j].y * W]);
                a[j][1] = __builtin_nontemporal_load(&Vg[(size_t)r[j].z * W]);
                a[j][2] = __builtin_nontemporal_load(&Vg[(size_t)r[j].w * W]);
            } else {
                a[j][0] = Vg[(size_t)r[j].y * W];
                a[j][1] = Vg[(size_t)r[j].z * W];
                a[j][2] = Vg[(size_t)r[j].w * W];
            }
            mm[j] = __builtin_nontemporal_load(&Cg[(size_t)(r[j].x >> 2) * W]);
        }
#pragma unroll
        for (int j = 0; j < RQ; ++j) {
            const bool live = p0 + 4 * j + q < P1;
            const float t = live ? a[j][0] + a[j][1] + a[j][2] + mm[j].x : 0.0f;
            // the four incidences' terms in order, gathered onto quarter 0 (replica rr of each quarter)
            acc += __shfl(t, rr);  // the left fold of system.rs:80, incidence by incidence
            acc += __shfl(t, rr + 16);
            acc += __shfl(t, rr + 32);
            acc += __shfl(t, rr + 48);
            if (live && (r[j].x & 3) == 0) {
                f2 o = mm[j];
                o.y += acc;
                __builtin_nontemporal_store(o, &Cn[(size_t)(r[j].x >> 2) * W]);
            }
        }
        while (cur < i1 && vptr[cur + 1] <= min(p0 + RB, P1)) {
            if (q == 0) __builtin_nontemporal_store(acc, &Vn[(size_t)g * N * W + (size_t)cur * W + rr]);
            ++cur;
        }
    }
    for (; cur < i1; ++cur)
        if (q == 0) __builtin_nontemporal_store(acc, &Vn[(size_t)g * N * W + (size_t)cur * W + rr]);
}

static uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main() {
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
    const size_t vbytes = (size_t)B * N * 4, cbytes = (size_t)B * M * 8;  // the same bytes in either layout
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
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int tiles = (N + ROWS - 1) / ROWS, bpg = (tiles + 3) / 4;
    const double alg_bytes = (8.0 * N + 16.0 * M) * B;  // SURVEY.md §8d per step
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
        std::fflush(stdout);
        return 0;
    };
    const dim3 block(256);
    if (run("w64", [&](int par) {
            hipLaunchKernelGGL(k_w64, dim3((unsigned)(16 * bpg)), block, 0, 0, dinc, dvptr, par ? V1 : V0,
                               par ? V0 : V1, par ? C1 : C0, par ? C0 : C1);
        }))
        return 1;
    for (int nt = 0; nt < 2; ++nt) {
        auto k1 = nt ? k_q16<true> : k_q16<false>;
        if (run(nt ? "q16_1_ntv" : "q16_1", [&](int par) {  // one launch: XCD x steps its 8 groups in turn
                hipLaunchKernelGGL(k1, dim3((unsigned)(64 * bpg)), block, 0, 0, dinc, dvptr, par ? V1 : V0,
                                   par ? V0 : V1, par ? C1 : C0, par ? C0 : C1, 0, 8);
            }))
            return 1;
        if (run(nt ? "q16_8_ntv" : "q16_8", [&](int par) {  // eight launches, one group per XCD each
                for (int l = 0; l < 8; ++l)
                    hipLaunchKernelGGL(k1, dim3((unsigned)(8 * bpg)), block, 0, 0, dinc, dvptr, par ? V1 : V0,
                                       par ? V0 : V1, par ? C1 : C0, par ? C0 : C1, 8 * l, 1);
            }))
            return 1;
    }
    return 0;
}
