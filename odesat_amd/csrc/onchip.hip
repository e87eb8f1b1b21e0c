// onchip.hip -- ODESAT_ALG_ONCHIP: the fixed-step integrator with a replica's whole state on one CU
// (onchip.hpp).  Reference: /root/reference/src/system.rs:25-97 (compute_derivatives, update_state)
// and :141-154 (euler_step_fixed), driven by simulate / simulate_inter (:156-359).
//
// Same clause tiles as the RESIDENT kernel (resident.hpp): no two clauses of a
// tile share a variable and every variable's tiles increase in the reference's clause order, so
// the lanes of a tile add their terms straight into dv (LDS) and every dv[i] is the reference's
// left fold over (clause, literal), bit for bit.  What changes is where the clause memories live:
// lane l owns clause slot l of every tile, so its memories form a per-lane array indexed by the
// tile number.  The first TR tiles keep theirs in VGPRs (the tile sequence is expanded at compile
// time, so the index is static), the remaining tiles in LDS next to v and dv.  A step then moves
// no state through the memory hierarchy at all; the only per-step reads are the 8-byte literal
// records (slot-major, L2-resident and shared by every CU).
//
// Exactness of the short arithmetic (the host launches this kernel only on "in-range" states:
// v in [-1, 1], xs in [-1, 1], xl in [1, 1e30], |zeta| <= 1e6 -- every state after one step is, by
// the clamps of system.rs:94-96; otherwise the first step of the call runs RESIDENT):
//   * vals are finite and non-NaN, so the strict-< min / second-min scan of :43-57 is exactly
//     min3 / med3 (ties give second = min, as the scan does);
//   * q * v with q = +-1 is a sign flip (v ^ signmask), and tt * (0.5 q sel) = +-((0.5 tt) sel)
//     (a product by 0.5 or by +-1 is exact; |tt| >= 1e-3 and sel >= 2^-24 or 0, so nothing is
//     subnormal);
//   * the rigidity term R (:73-80) only fires with mn = 0 = val_j, i.e. v_j = q_j, where it is
//     0.5 (q - v) = +0, and tr * (+0) is a signed zero for finite tr; adding it can only turn a -0
//     term into +0, and dv (which starts at +0 and is never -0) absorbs either identically.  So R
//     is omitted.
// The formula must have three distinct variables per clause (the host checks), so a clause's three
// dv updates are independent.  Empty slots of a partial tile point at per-lane-bank sink words
// (v = 1.0, so the slot's C = 0 never reports unsat; its dv sink is never read).
#pragma clang fp contract(off)

#include "onchip.hpp"

#include <climits>
#include <utility>

#include "../../include/odesat.h"

namespace onchip {
namespace {

struct Slot {  // one lane's literal record for one tile
    uint32_t lo, hi;
};

struct Pend {  // a clause's three dv terms (LDS byte addresses of v; dv is at +DV), applied one tile later
    uint32_t a0, a1, a2;
    float d0, d1, d2;
};

typedef const __attribute__((address_space(1))) uint64_t grec;  // global: counts in vmcnt only

// Records of tile t (uniform base, per-lane offset: the SGPR-base form of global_load).
__device__ __forceinline__ Slot load_rec(const grec *rec, int t, int lane) {
    const grec *base = rec + (size_t)t * NTH;
    const uint64_t r = base[lane];
    return Slot{(uint32_t)r, (uint32_t)(r >> 32)};
}

typedef __attribute__((address_space(3))) float lfloat;
__device__ __forceinline__ float lds_f(uint32_t byte_addr, uint32_t off) {
    return *reinterpret_cast<const lfloat *>(byte_addr + off);
}
__device__ __forceinline__ void lds_st(uint32_t byte_addr, uint32_t off, float x) {
    *reinterpret_cast<lfloat *>(byte_addr + off) = x;
}

// One clause (system.rs:43-88): C, the three dv terms into P, the sat test, and the memory update
// in place (:84-85, :94-95).
__device__ __forceinline__ void clause(const Args &a, const Slot &S, float2 &mem, float h, Pend &P, float &cmax) {
    P.a0 = S.lo & 0xffffu;
    P.a1 = S.lo >> 16;
    P.a2 = S.hi & 0xffffu;
    const uint32_t s0 = S.hi & 0x80000000u, s1 = (S.hi << 1) & 0x80000000u, s2 = (S.hi << 2) & 0x80000000u;
    const float v0 = lds_f(P.a0, 0), v1 = lds_f(P.a1, 0), v2 = lds_f(P.a2, 0);
    const float val0 = 1.0f - __uint_as_float(__float_as_uint(v0) ^ s0);  // 1 - q v  (:47)
    const float val1 = 1.0f - __uint_as_float(__float_as_uint(v1) ^ s1);
    const float val2 = 1.0f - __uint_as_float(__float_as_uint(v2) ^ s2);
    const float mn = fminf(fminf(val0, val1), val2);                // min (:49-55)
    const float sec = __builtin_amdgcn_fmed3f(val0, val1, val2);     // second min, ties -> min
    const float C = 0.5f * mn;                                       // :60
    const float xs = mem.x, xl = mem.y;
    const float ht = 0.5f * (xl * xs);
    P.d0 = __uint_as_float(__float_as_uint(ht * (val0 != mn ? mn : sec)) ^ s0);  // xl xs G (:64-70, :80)
    P.d1 = __uint_as_float(__float_as_uint(ht * (val1 != mn ? mn : sec)) ^ s1);
    P.d2 = __uint_as_float(__float_as_uint(ht * (val2 != mn ? mn : sec)) ^ s2);
    cmax = fmaxf(cmax, C);  // :88 -- unsat iff max C >= gamma (C is never NaN here)
    asm volatile("" : "+v"(cmax));  // fold now: deferred, it would keep every tile's C live
    const float dxs = 20.0f * (xs + 0.001f) * (C - 0.25f);      // :84
    const float dxl = 5.0f * (C - 0.05f);                       // :85
    mem.x = fminf(fmaxf(xs + h * dxs, 0.001f), 1.0f - 0.001f);  // :94
    mem.y = fminf(fmaxf(xl + h * dxl, 1.0f), a.xl_max);         // :95
    asm volatile("" : "+v"(mem.x), "+v"(mem.y));  // update now: sunk into later tiles it keeps C live
}

// :80 for one clause: dv[i_j] += d_j (three distinct variables: independent updates)
__device__ __forceinline__ void apply(uint32_t DV, const Pend &P) {
    const float o0 = lds_f(P.a0, DV), o1 = lds_f(P.a1, DV), o2 = lds_f(P.a2, DV);
    lds_st(P.a0, DV, o0 + P.d0);
    lds_st(P.a1, DV, o1 + P.d1);
    lds_st(P.a2, DV, o2 + P.d2);
}

// Register tile T of the pass (static T, so mr[] stays in VGPRs): terms of tile T+1 (ring slot
// (T+1) % 4, refilled with tile T+5), apply tile T's terms P, barrier.  All TR register tiles run
// (tiles past the last one are empty): an early exit would join TR paths after the sequence, and
// the copies that merge mr[] there double its VGPR footprint.
template <int TR, int T>
__device__ __forceinline__ void reg_tile(const Args &a, const grec *rec, uint32_t DV, float2 *memL,
                                         float2 (&mr)[TR], Slot (&ring)[4], Pend &P, float h, int lane, float &cmax) {
    Pend Q;
    if constexpr (T + 1 < TR) {
        clause(a, ring[(T + 1) % 4], mr[T + 1], h, Q, cmax);
    } else {
        float2 m = make_float2(0.0f, 0.0f);
        if (a.tl > 0) m = memL[lane];
        clause(a, ring[(T + 1) % 4], m, h, Q, cmax);
        if (a.tl > 0) memL[lane] = m;
    }
    apply(DV, P);
    ring[(T + 1) % 4] = load_rec(rec, T + 5, lane);
    __builtin_amdgcn_sched_barrier(0);  // a tile's work stays between its barriers
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
    P = Q;
}

template <int TR, int... Ts>
__device__ __forceinline__ void reg_tiles(std::integer_sequence<int, Ts...>, const Args &a, const grec *rec,
                                          uint32_t DV, float2 *memL, float2 (&mr)[TR], Slot (&ring)[4], Pend &P,
                                          float h, int lane, float &cmax) {
    (reg_tile<TR, Ts>(a, rec, DV, memL, mr, ring, P, h, lane, cmax), ...);
}

// One RHS pass + memory update over every tile; ends with a barrier (dv complete).
template <int TR>
__device__ __forceinline__ void pass(const Args &a, uint32_t DV, float2 *memL, float2 (&mr)[TR], float h, int lane,
                                     float &cmax) {
    // an opaque copy of the record pointer per pass keeps the record loads inside the step loop
    // (hoisted out of it they would pin hundreds of VGPRs)
    const grec *rec = (const grec *)a.rec;
    asm volatile("" : "+s"(rec));
    Slot ring[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) ring[s] = load_rec(rec, s, lane);
    Pend P;
    clause(a, ring[0], mr[0], h, P, cmax);
    ring[0] = load_rec(rec, 4, lane);
    reg_tiles<TR>(std::make_integer_sequence<int, TR>{}, a, rec, DV, memL, mr, ring, P, h, lane, cmax);
    // LDS tiles [TR, TR + tl): tl is a multiple of 4 (the host pads the tiling)
    const int NT = TR + a.tl;
    const int last = a.tl - 1;
    for (int t0 = TR; t0 < NT; t0 += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = t0 + u;
            Pend Q;
            const int lt = min(t + 1 - TR, last);
            float2 m = memL[lt * NTH + lane];
            clause(a, ring[(u + 1) % 4], m, h, Q, cmax);
            memL[lt * NTH + lane] = m;
            apply(DV, P);
            ring[(u + 1) % 4] = load_rec(rec, t + 5, lane);
            __syncthreads();
            P = Q;
        }
    }
}

typedef const __attribute__((address_space(4))) int32_t cint32;

// Load (in) or store the register tiles' memories from / to the replica's clause memories.
template <int TR, int... Js>
__device__ __forceinline__ void mem_io(std::integer_sequence<int, Js...>, const cint32 *tc, int nt, float2 *CM,
                                       float2 (&mr)[TR], int lane, bool in) {
    auto one = [&](auto J) {
        constexpr int j = decltype(J)::value;
        const int c0 = tc[min(j, nt)], c1 = tc[min(j + 1, nt)];
        const int c = c0 + lane;
        if (in) mr[j] = c < c1 ? CM[c] : make_float2(0.0f, 0.0f);
        else if (c < c1) CM[c] = mr[j];
    };
    (one(std::integral_constant<int, Js>{}), ...);
}

// LDS map (floats): v[n2] at 0 (v[n .. n2) = sink words, 1.0), dv[n2] at n2 (byte offset DV),
// two unsat flags, then tl tiles of memories [tl][NTH] float2.
template <int TR>
__global__ __launch_bounds__(NTH) void k_onchip(Args a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int g = blockIdx.x, lane = threadIdx.x;
    int act = a.act[g];
    if (!act) return;  // frozen replica (uniform)
    if (a.stop_mode == ODESAT_STOP_ANY && *a.stop < a.step0) return;  // an earlier step stopped every replica
    const bool p = __builtin_amdgcn_readfirstlane((int)a.par[g]) != 0;
    float *V = (p ? a.v1 : a.v0) + (size_t)g * a.n;
    float2 *CM = reinterpret_cast<float2 *>((p ? a.c1 : a.c0) + (size_t)g * a.m * 2);
    const int n2 = a.n + SINKS;
    float *vL = smem, *dvL = smem + n2;
    int *unsL = reinterpret_cast<int *>(smem + 2 * n2);
    float2 *memL = reinterpret_cast<float2 *>(smem + 2 * n2 + 2);
    const uint32_t DV = (uint32_t)(4 * n2);
    int64_t sat = a.sat_step[g], done = a.steps_done[g];
    const cint32 *tc = (const cint32 *)a.tc;

    for (int i = lane; i < n2; i += NTH) {
        vL[i] = i < a.n ? V[i] : 1.0f;
        dvL[i] = 0.0f;  // :33
    }
    float2 mr[TR];
    mem_io<TR>(std::make_integer_sequence<int, TR>{}, tc, a.ntiles, CM, mr, lane, true);
    for (int t = 0; t < a.tl; ++t) {
        const int c0 = tc[min(TR + t, a.ntiles)], c1 = tc[min(TR + t + 1, a.ntiles)];
        const int c = c0 + lane;
        memL[t * NTH + lane] = c < c1 ? CM[c] : make_float2(0.0f, 0.0f);
    }
    if (lane == 0) {
        unsL[0] = 0;
        unsL[1] = 0;
    }
    __syncthreads();

    const float h = a.dt;
    for (int k = 0; k < a.nsteps; ++k) {  // euler_step_fixed (system.rs:141-154)
        float cmax = 0.0f;
        pass<TR>(a, DV, memL, mr, h, lane, cmax);
        if (!(cmax < 0.25f)) unsL[k & 1] = 1;
        for (int i = lane; i < a.n; i += NTH) {  // :96, dv restarts at 0 (:33)
            const float d = dvL[i];
            dvL[i] = 0.0f;
            vL[i] = fminf(fmaxf(vL[i] + h * d, -1.0f), 1.0f);
        }
        if (lane == 0) unsL[(k + 1) & 1] = 0;  // read by everyone before this step's first barrier
        __syncthreads();
        done += 1;
        if (unsL[k & 1] == 0) {  // allsat before the update; the step was still taken (:148-152)
            const int step = a.step0 + k;
            if (sat < 0) sat = step;
            if (a.stop_mode == ODESAT_STOP_ANY && lane == 0) atomicMin(a.stop, step);  // simulate_inter (:291)
            if (a.stop_mode == ODESAT_STOP_EACH) {                                      // simulate (:193)
                act = 0;
                break;
            }
        }
    }

    for (int i = lane; i < a.n; i += NTH) V[i] = vL[i];  // written by this lane in the last update
    {   // opaque copies: the store addresses are recomputed here instead of being kept live (two
        // VGPRs per tile) across the step loop from the loads above
        float2 *CMs = CM;
        const cint32 *tcs = tc;
        asm volatile("" : "+s"(CMs), "+s"(tcs));
        mem_io<TR>(std::make_integer_sequence<int, TR>{}, tcs, a.ntiles, CMs, mr, lane, false);
    }
    for (int t = 0; t < a.tl; ++t) {  // this lane's own LDS slots: no barrier needed
        const int c0 = tc[min(TR + t, a.ntiles)], c1 = tc[min(TR + t + 1, a.ntiles)];
        const int c = c0 + lane;
        if (c < c1) CM[c] = memL[t * NTH + lane];
    }
    if (lane == 0) {
        a.act[g] = (uint8_t)act;
        a.sat_step[g] = sat;
        a.steps_done[g] = done;
    }
}

template <int TR> hipError_t launch_t(const Args &a, int G, size_t lds, hipStream_t stream) {
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_onchip<TR>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL((k_onchip<TR>), dim3((unsigned)G), dim3(NTH), lds, stream, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch(int tr, const Args &a, int G, size_t lds, hipStream_t stream) {
    switch (tr) {
#define ONCHIP_CASE(N) \
    case N: return launch_t<N>(a, G, lds, stream);
        ONCHIP_CASE(8) ONCHIP_CASE(16) ONCHIP_CASE(24) ONCHIP_CASE(32) ONCHIP_CASE(40) ONCHIP_CASE(48)
        ONCHIP_CASE(56) ONCHIP_CASE(64) ONCHIP_CASE(72) ONCHIP_CASE(80) ONCHIP_CASE(88) ONCHIP_CASE(96)
#undef ONCHIP_CASE
        default: return hipErrorInvalidValue;
    }
}

}  // namespace onchip
