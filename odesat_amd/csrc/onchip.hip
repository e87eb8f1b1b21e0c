// onchip.hip -- ODESAT_ALG_ONCHIP: the fixed-step integrator with a replica's whole state on one CU
// (onchip.hpp).  Reference: /root/reference/src/system.rs:25-97 (compute_derivatives, update_state)
// and :141-154 (euler_step_fixed), driven by simulate / simulate_inter (:156-359).
//
// Same clause tiles as the RESIDENT kernel (resident.hpp): no two clauses of a
// tile share a variable and every variable's tiles increase in the reference's clause order, so
// the lanes of a tile add their terms straight into dv (LDS) and every dv[i] is the reference's
// left fold over (clause, literal), bit for bit.  The tiles are wave-paired (odesat_hip.hip
// pair_tiles): a barrier follows every second tile only, and a clause that depends on a clause of
// the same pair sits in the same wave, whose LDS operations complete in issue order.  What changes is where the clause memories live:
// lane l owns clause slot l of every tile, so its memories form a per-lane array indexed by the
// tile number.  The first TR tiles keep theirs in VGPRs (the tile sequence is expanded at compile
// time, so the index is static), the remaining tiles in LDS next to v and dv.  A step then moves
// no state through the memory hierarchy at all; the only per-step reads are the literal records
// (slot-major, L2-resident and shared by every CU): 12 bytes per clause slot for fixed steps, one
// word per literal (ONCHIP_REC12, onchip.hpp), for both passes of an adaptive step too.
//
// Exactness of the short arithmetic (the host launches this kernel only on "in-range" states:
// v in [-1, 1], xs in [-1, 1], xl in [1, 1e30], |zeta| <= 1e6 -- every state after one step is, by
// the clamps of system.rs:94-96; otherwise the first step of the call runs RESIDENT):
//   * vals are finite and non-NaN, so the strict-< min / second-min scan of :43-57 gives the
//     smallest and the second smallest value (ties give second = min), and the value literal j's
//     term selects is the min of the other two literals' values (see Front);
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
#include "devattr.hpp"

#include <climits>
#include <utility>

#include "../../include/odesat.h"

namespace onchip {
namespace {

// Diagnostic build only (-DONCHIP_STAMPS=1|2, scripts/build_variant.sh): per wave, s_memtime stamps
// split each tile step into the barrier wait and the work before it (2: and the dv read-modify-write
// at its start); the sums go to g_onchip_stamps, read by odesat_onchip_stamps.  Each stamp drains the
// wave's LDS operations, so read the SHARES, never the build's run time.  In the product build
// Stamps is empty and every stamp call vanishes.
#ifdef ONCHIP_STAMPS
struct Stamps {
    uint64_t last, bar, work, rmw, tiles;
};
__device__ unsigned long long g_onchip_stamps[4096 * 16 * 4];
__device__ __forceinline__ uint64_t memtime() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#else
struct Stamps {};
#endif
// Diagnostic build only (-DONCHIP_ADA_STAMPS): the adaptive step of workgroup 0 split by s_memtime into
// pass 1, the first voltage phase (+ its barrier), pass 2, the second voltage phase with the error
// terms, and the step's closing barrier with the dt update; per wave sums in g_onchip_ada_stamps[w][5]
// (read by odesat_onchip_ada_stamps; scripts/onchip_ada_stamps.py).  Each stamp drains the wave's LDS
// operations, so the segments include that drain.
#ifdef ONCHIP_ADA_STAMPS
__device__ unsigned long long g_onchip_ada_stamps[8 * 5];
__device__ __forceinline__ uint64_t ada_memtime() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define ADA_STAMP(acc)                      \
    do {                                    \
        const uint64_t t_ = ada_memtime();  \
        (acc) += t_ - ada_last;             \
        ada_last = t_;                      \
    } while (0)
#else
#define ADA_STAMP(acc) do {} while (0)
#endif
// Diagnostic build only (-DONCHIP_PHASES): per workgroup, wave 0 records s_memrealtime (100 MHz)
// at kernel start, after the state load (its barrier), after the step loop and at the end, into
// g_onchip_phases[g][4] (read by odesat_onchip_phases).
// g_onchip_clk holds s_memtime (shader clock) at the same points: their ratio is the effective clock.
#ifdef ONCHIP_PHASES
__device__ unsigned long long g_onchip_phases[4096 * 4];
__device__ unsigned long long g_onchip_clk[4096 * 4];
#define ONCHIP_PHASE(i)                                                                                   \
    do {                                                                                                  \
        if (threadIdx.x == 0 && blockIdx.x < 4096) {                                                      \
            uint64_t t_, c_;                                                                              \
            asm volatile("s_memrealtime %0\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_), "=s"(c_)::"memory"); \
            g_onchip_phases[blockIdx.x * 4 + (i)] = t_;                                                   \
            g_onchip_clk[blockIdx.x * 4 + (i)] = c_;                                                      \
        }                                                                                                 \
    } while (0)
#else
#define ONCHIP_PHASE(i) do {} while (0)
#endif

struct Slot {  // one lane's literal record for one tile
    uint32_t lo, hi;
};
#if ONCHIP_REC12
struct SlotF {  // the fixed-step kernel's 12-byte record: one word per literal (address | sign << 31)
    uint32_t w0, w1, w2;
};
#else
typedef Slot SlotF;
#endif

struct Pend {  // a clause's three dv terms (LDS byte addresses of v; dv is at +DVC), applied one tile later
    uint32_t a0, a1, a2;
    float d0, d1, d2;
};

struct Gath {  // a clause's gathered inputs: LDS byte addresses of its voltages, sign word(s), voltages
    uint32_t a0, a1, a2;
#if ONCHIP_REC12
    uint32_t s0, s1, s2;  // the literals' record words (sign at bit 31)
#else
    uint32_t hi;
#endif
    float v0, v1, v2;
};

// The records are read with buffer loads: the resource (SGPRs) holds the base, the per-lane offset
// lane * (8 or 12) is one VGPR for the whole launch and the tile offset a scalar, so a ring refill
// costs no vector instruction.
struct Recs {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t voff;  // lane * record bytes
    uint32_t soff;  // opaque 0 (see pass())
};
__device__ __forceinline__ Slot load_rec(const Recs &R, int t) {
    typedef int i2 __attribute__((ext_vector_type(2)));
    const i2 r = __builtin_amdgcn_raw_buffer_load_b64(R.rsrc, R.voff, R.soff + (uint32_t)t * (NTH * 8), 0);
    return Slot{(uint32_t)r.x, (uint32_t)r.y};
}
#if ONCHIP_REC12
constexpr uint32_t RECF_BYTES = 12;
__device__ __forceinline__ SlotF load_recf(const Recs &R, int t) {
    typedef int i3 __attribute__((ext_vector_type(3)));
    const i3 r = __builtin_amdgcn_raw_buffer_load_b96(R.rsrc, R.voff, R.soff + (uint32_t)t * (NTH * 12), 0);
    return SlotF{(uint32_t)r.x, (uint32_t)r.y, (uint32_t)r.z};
}
#else
constexpr uint32_t RECF_BYTES = 8;
__device__ __forceinline__ SlotF load_recf(const Recs &R, int t) { return load_rec(R, t); }
#endif

typedef __attribute__((address_space(3))) float lfloat;
__device__ __forceinline__ float lds_f(uint32_t byte_addr) { return *reinterpret_cast<const lfloat *>(byte_addr); }
__device__ __forceinline__ void lds_st(uint32_t byte_addr, float x) { *reinterpret_cast<lfloat *>(byte_addr) = x; }
typedef __attribute__((address_space(3))) float2 lfloat2;
__device__ __forceinline__ float2 *lds_f2(uint32_t byte_addr) { return (float2 *)(reinterpret_cast<lfloat2 *>(byte_addr)); }
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) f4v lf4v;
__device__ __forceinline__ f4v lds_f4(uint32_t byte_addr) { return *reinterpret_cast<const lf4v *>(byte_addr); }
__device__ __forceinline__ void lds_st4(uint32_t byte_addr, f4v x) { *reinterpret_cast<lf4v *>(byte_addr) = x; }

// The clause's three voltages (system.rs:46-48): LDS reads issued here, consumed by front().
__device__ __forceinline__ void gather(const SlotF &S, Gath &G) {
#if ONCHIP_REC12
    G.a0 = S.w0 & 0xffffu;
    G.a1 = S.w1 & 0xffffu;
    G.a2 = S.w2 & 0xffffu;
    G.s0 = S.w0;
    G.s1 = S.w1;
    G.s2 = S.w2;
#else
    G.a0 = S.lo & 0xffffu;
    G.a1 = S.lo >> 16;
    G.a2 = S.hi & 0xffffu;
    G.hi = S.hi;
#endif
    G.v0 = lds_f(G.a0);
    G.v1 = lds_f(G.a1);
    G.v2 = lds_f(G.a2);
}

// One clause (system.rs:43-88), in two halves that run one tile step apart (so a step interleaves
// two independent halves of two tiles).  Exact rewritten forms (C = mn / 2 exactly):
//   C < gamma  <=>  mn < 0.5, so cmax folds the bits of mn (mn >= +0 orders as its bits);
//   C - 0.25 = 0.5 (mn - 0.5) and C - 0.05 = 0.5 (mn - 0.1) (0.05f is exactly 0.1f / 2), so
//   h dxs = (h/2) round(A (mn - 0.5)) with A = 20 (xs + eps), and dxl = 2.5 (mn - 0.1);
//   xl xs G_j = +-round((xl xs / 2) sel_j) = +-round(xl xs sel_j) / 2 with sel_j = mn or sec: the
//   terms are accumulated unhalved (dv2 = 2 dv, also exact), and the update uses h/2 (:96);
//   the clamps are med3 (finite arguments: the host requires a finite dt).
// Scalings by 0.5 / 2 / 2.5 / +-1 are exact here (no subnormals: |A| >= 0.02, |mn - c| >= 2^-26 or 0,
// |xl xs sel| >= 6e-11 or 0).
//   the term of literal j selects (val_j != mn ? mn : sec) (:64-70), which for finite values is
//   exactly the min of the OTHER two literal values: the min when some other literal attains it,
//   the second smallest (the scan's `sec`, ties included) when j does -- so sel_j = min(val_k, val_l)
//   needs no compare and no select.
//   the sign q_j of literal j's term rides on its selected value (q tt sel = tt (q sel): a sign
//   flip, exact), so the second half needs no sign word.
struct Front {  // first half: the min (:49-55) and each literal's signed selected value
    uint32_t a0, a1, a2;
    float sel0, sel1, sel2, mn;
};

__device__ __forceinline__ void front(const Gath &G, Front &F) {
    F.a0 = G.a0;
    F.a1 = G.a1;
    F.a2 = G.a2;
#if ONCHIP_REC12
    const uint32_t s0 = G.s0 & 0x80000000u, s1 = G.s1 & 0x80000000u, s2 = G.s2 & 0x80000000u;
#else
    const uint32_t s0 = G.hi & 0x80000000u, s1 = (G.hi << 1) & 0x80000000u, s2 = (G.hi << 2) & 0x80000000u;
#endif
    const float val0 = 1.0f - __uint_as_float(__float_as_uint(G.v0) ^ s0);  // 1 - q v  (:47)
    const float val1 = 1.0f - __uint_as_float(__float_as_uint(G.v1) ^ s1);
    const float val2 = 1.0f - __uint_as_float(__float_as_uint(G.v2) ^ s2);
    const float sel2 = fminf(val0, val1);
    F.sel0 = __uint_as_float(__float_as_uint(fminf(val1, val2)) ^ s0);
    F.sel1 = __uint_as_float(__float_as_uint(fminf(val0, val2)) ^ s1);
    F.sel2 = __uint_as_float(__float_as_uint(sel2) ^ s2);
    F.mn = fminf(sel2, val2);  // min (:49-55)
}

// Second half: the three dv terms into Q, the sat fold and the memory update in place
// (:60-88, :94-95).
// (UPD = false: the terms and the sat fold only, the memories left as they are -- the adaptive
// step's first pass, pass1.)
template <bool UPD = true>
__device__ __forceinline__ void back(const Args &a, const Front &F, float2 &mem, float h, float hh, Pend &Q,
                                     uint32_t &cmax) {
    const float mn = F.mn;
    const float xs = mem.x, xl = mem.y;
    const float tt = xl * xs;
    Q.a0 = F.a0;
    Q.a1 = F.a1;
    Q.a2 = F.a2;
    Q.d0 = tt * F.sel0;  // 2 xl xs G (:64-70, :80), the sign q in sel
    Q.d1 = tt * F.sel1;
    Q.d2 = tt * F.sel2;
    cmax = max(cmax, __float_as_uint(mn));  // :88 -- unsat iff max mn >= 0.5
    asm volatile("" : "+v"(cmax));          // fold now: deferred, it would keep every tile's mn live
    if constexpr (!UPD) return;
    const float dxs2 = (20.0f * (xs + 0.001f)) * (mn - 0.5f);  // 2 dxs (:84)
    const float dxl = 2.5f * (mn - 0.1f);                       // :85
    mem.x = __builtin_amdgcn_fmed3f(xs + hh * dxs2, 0.001f, 1.0f - 0.001f);  // :94
    mem.y = __builtin_amdgcn_fmed3f(xl + h * dxl, 1.0f, a.xl_max);           // :95
    asm volatile("" : "+v"(mem.x), "+v"(mem.y));  // update now: sunk into later tiles it keeps mn live
}

// Split barriers between the pairs of register tiles (ONCHIP_SPLITBAR, round 4): instead of a
// workgroup barrier after the second tile of a pair, each wave adds 1 to an LDS counter right after
// that tile's dv writes, and waits -- polling the counter -- only before the NEXT pair's first dv
// read-modify-write.  The independent work of the tile (the gathers of tile t+3, the halves of tiles
// t+1 and t+2) runs between the two, so a wave that finished early no longer idles at a barrier.
// Ordering: a wave's LDS operations are performed in issue order, so a counter increment is performed
// after that wave's dv writes; a wave that has read the counter at its target issues its dv reads
// after that read returned, i.e. after every wave's writes of the pair.
// ONCHIP_SPLITBAR is a mask: 1 = the fixed-step kernel, 2 = the adaptive one.  Measured (round 4,
// profiles/r04i_splitbar_ab.txt): adaptive 2.5-3.5 % faster, fixed 2-3 % slower -- the default is the
// adaptive kernel only.
#ifndef ONCHIP_SPLITBAR
#define ONCHIP_SPLITBAR 2
#endif
#ifndef ONCHIP_POLL_SLEEP  // s_sleep between polls (0: none)
#define ONCHIP_POLL_SLEEP 1
#endif
#define POLL_STR2(x) #x
#define POLL_STR(x) POLL_STR2(x)
typedef __attribute__((address_space(3))) uint32_t lu32;
// (The counter is one word per wave -- the number of pairs it has signalled -- written by all of the
// wave's lanes (one address: no lane branch, which would cost the unrolled tile code its registers);
// a waiting wave's lane l reads wave l % 8's word and the wave proceeds once every word is at the
// target.)
__device__ __forceinline__ void pair_signal(uint32_t cnt, uint32_t ep) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    *reinterpret_cast<volatile lu32 *>(cnt + 4u * (threadIdx.x >> 6)) = ep;
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}
// The poll is one inline-assembly loop, invisible to the compiler's control flow: a loop in the
// unrolled tile sequence cost it 40-65 spilled VGPRs.  (All 64 lanes are active here.)  It gives up
// after `limit` polls (2^22, ~0.1 s; the experiment knob ONCHIP_POLL_LIMIT lowers it for the test of
// this path), so a broken count can never hang the GPU.  Giving up stores a nonzero word in the fault
// slots after the counters (the lane's counter address + 32: no register beyond the loop's own),
// which the kernel reports to the host at its end: the call then fails instead of returning results
// that raced.
__device__ __forceinline__ void pair_wait(uint32_t cnt, uint32_t target, uint32_t limit) {
    static_assert(WAVES == 8, "the asm's fault slot (offset:32 = 8 counters) and tid & 7 assume 8 waves");
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t addr = cnt + 4u * (threadIdx.x & 7);
    uint32_t tmp, it;
    uint64_t msk;
    asm volatile(
        "s_mov_b32 %2, 0\n"
        "L_pw%=:\n\t"
        "ds_read_b32 %0, %3\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_cmp_ge_u32_e64 %1, %0, %4\n\t"
        "s_cmp_eq_u64 %1, exec\n\t"
        "s_cbranch_scc1 L_pd%=\n\t"
        "s_add_u32 %2, %2, 1\n\t"
        "s_cmp_gt_u32 %2, %5\n\t"
        "s_cbranch_scc1 L_pt%=\n\t"
#if ONCHIP_POLL_SLEEP > 0
        "s_sleep " POLL_STR(ONCHIP_POLL_SLEEP) "\n\t"
#endif
        "s_branch L_pw%=\n"
        "L_pt%=:\n\t"
        "v_mov_b32 %0, 1\n\t"
        "ds_write_b32 %3, %0 offset:32\n"
        "L_pd%=:"
        : "=&v"(tmp), "=&s"(msk), "=&s"(it)
#ifdef ONCHIP_POLL_CONST  // A/B: the limit as an immediate (one SGPR less in the adaptive kernel)
        : "v"(addr), "s"(target), "i"(0x400000)
#else
        : "v"(addr), "s"(target), "s"(limit)
#endif
        : "memory", "scc");
    __builtin_amdgcn_sched_barrier(0);
}

// One tile step.  In flight: P = tile t's dv terms, Fn = tile t+1's first half, Gn = tile t+2's
// gathered voltages, ring = the records of tiles t+3 .. t+6.  The critical chain of a step is tile
// t's dv read-modify-write (:80; three distinct variables per clause, so the updates are
// independent): its reads go out first and the writes right after they return.  The voltage
// gathers of tile t+3 follow (v is constant during a pass), then tile t+1's second half and tile
// t+2's first half -- independent, so they interleave -- while the writes and the gathers drain.
// After the second tile of a pair (bar), the barrier orders the pair's dv updates against the next
// pair's; inside a pair the same-wave order suffices (see the header).
template <bool SPL = false, uint32_t DVO = DVC, bool UPD = true>
__device__ __forceinline__ void tile_step(const Args &a, const Recs &R, SlotF &slot3, float2 &mem1, Pend &P, Front &Fn,
                                          Gath &Gn, int t, float h, float hh, uint32_t &cmax, Stamps &S, bool bar,
                                          bool first = false, uint32_t cnt = 0, uint32_t *ep = nullptr) {
    if (SPL && first) pair_wait(cnt, *ep, a.poll_limit);  // every wave's dv writes of the previous pair are performed
    const float o0 = lds_f(P.a0 + DVO), o1 = lds_f(P.a1 + DVO), o2 = lds_f(P.a2 + DVO);
    lds_st(P.a0 + DVO, o0 + P.d0);
    lds_st(P.a1 + DVO, o1 + P.d1);
    lds_st(P.a2 + DVO, o2 + P.d2);
    __builtin_amdgcn_sched_barrier(0);
    if (SPL && bar) pair_signal(cnt, ++*ep);
#if defined(ONCHIP_STAMPS) && ONCHIP_STAMPS == 2
    const uint64_t t_rmw = memtime();
    S.rmw += t_rmw - S.last;
#endif
    Gath G3;
    gather(slot3, G3);
    slot3 = load_recf(R, t + 7);
    __builtin_amdgcn_sched_barrier(0);
    back<UPD>(a, Fn, mem1, h, hh, P, cmax);  // P <- tile t+1's terms (tile t's were written above)
    front(Gn, Fn);                      // Fn <- tile t+2's first half
    __builtin_amdgcn_sched_barrier(0);  // a tile's work stays between its barriers
#ifdef ONCHIP_STAMPS
    const uint64_t t_pre = memtime();
    S.work += t_pre - S.last;
#endif
    if (bar && !SPL) __syncthreads();  // static: only after the second tile of a pair
    __builtin_amdgcn_sched_barrier(0);
#ifdef ONCHIP_STAMPS
    S.last = memtime();
    S.bar += S.last - t_pre;
    S.tiles += 1;
#endif
    Gn = G3;
}

// LDS byte address of this lane's slot in LDS memory tile lt (onchip.hpp, Lds).
__device__ __forceinline__ uint32_t mem_addr(const Args &a, int lt, int lane) {
    const uint32_t base = (uint32_t)lt < a.lds.gap_tiles ? a.lds.gap_base + (uint32_t)lt * TILE_LDS
                                                         : a.lds.after_base + ((uint32_t)lt - a.lds.gap_tiles) * TILE_LDS;
    return base + (uint32_t)lane * 8u;
}

// Register tile T of the pass (static T, so mr[] stays in VGPRs).  All TR register tiles run
// (tiles past the last one are empty): an early exit would join TR paths after the sequence, and
// the copies that merge mr[] there double its VGPR footprint.
template <int TR, int OFF, int T>
__device__ __forceinline__ void reg_tile(const Args &a, const Recs &R, float2 (&mr)[TR], SlotF (&ring)[4], Pend &P,
                                         Front &Fn, Gath &Gn, float h, float hh, int lane, uint32_t &cmax, Stamps &S,
                                         uint32_t cnt, uint32_t *ep) {
    constexpr bool bar = ((T + OFF) & 1) != 0;  // wave-paired tiles: a barrier after the second of a pair
    constexpr bool first = T > 0 && ((T - 1 + OFF) & 1) != 0;  // the first tile of a pair after another pair
    constexpr bool SPL = (ONCHIP_SPLITBAR & 1) != 0;
    if constexpr (T + 1 < TR) {
        tile_step<SPL>(a, R, ring[(T + 3) % 4], mr[T + 1], P, Fn, Gn, T, h, hh, cmax, S, bar, first, cnt, ep);
    } else {  // tile TR is the first LDS tile (if any)
        float2 m = make_float2(0.0f, 0.0f);
        if (a.tl > 0) m = *lds_f2(mem_addr(a, 0, lane));
        tile_step<SPL>(a, R, ring[(T + 3) % 4], m, P, Fn, Gn, T, h, hh, cmax, S, bar, first, cnt, ep);
        if (a.tl > 0) *lds_f2(mem_addr(a, 0, lane)) = m;
    }
}

template <int TR, int OFF, int... Ts>
__device__ __forceinline__ void reg_tiles(std::integer_sequence<int, Ts...>, const Args &a, const Recs &R,
                                          float2 (&mr)[TR], SlotF (&ring)[4], Pend &P, Front &Fn, Gath &Gn, float h,
                                          float hh, int lane, uint32_t &cmax, Stamps &S, uint32_t cnt, uint32_t *ep) {
    (reg_tile<TR, OFF, Ts>(a, R, mr, ring, P, Fn, Gn, h, hh, lane, cmax, S, cnt, ep), ...);
}

// One RHS pass + memory update over every tile; ends with a barrier (dv complete).
template <int TR, int OFF>
__device__ __forceinline__ void pass(const Args &a, float2 (&mr)[TR], float h, int lane, uint32_t &cmax, Stamps &S,
                                     uint32_t cnt, uint32_t &ep) {
    Recs R;
#if ONCHIP_REC12
    R.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)a.rec12, 0, (int)a.rec12_bytes, 0x00020000);
#else
    R.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)a.rec, 0, (int)a.rec_bytes, 0x00020000);
#endif
    R.voff = (uint32_t)lane * RECF_BYTES;
    // an opaque zero per pass keeps the record loads inside the step loop (hoisted out of it they
    // would pin hundreds of VGPRs)
    R.soff = 0u;
    asm volatile("" : "+s"(R.soff));
    const float hh = 0.5f * h;
    SlotF ring[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) ring[s] = load_recf(R, s);
    Pend P;
    Gath G0, G1, Gn;
    gather(ring[0], G0);
    ring[0] = load_recf(R, 4);
    gather(ring[1], G1);
    ring[1] = load_recf(R, 5);
    gather(ring[2], Gn);
    ring[2] = load_recf(R, 6);
    Front F0, Fn;
    front(G0, F0);
    front(G1, Fn);
    back(a, F0, mr[0], h, hh, P, cmax);
    reg_tiles<TR, OFF>(std::make_integer_sequence<int, TR>{}, a, R, mr, ring, P, Fn, Gn, h, hh, lane, cmax, S, cnt, &ep);
    // LDS tiles [TR, TR + tl): tl is a multiple of 4 (the host pads the tiling); they keep plain barriers
    if ((ONCHIP_SPLITBAR & 1) && a.tl > 0) __syncthreads();
    const int NT = TR + a.tl;
    const int last = a.tl - 1;
    for (int t0 = TR; t0 < NT; t0 += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = t0 + u;
            // the step's second half works on tile t + 1; after the last tile there is none, and
            // its (discarded) update must not land on the last tile's memories
            const int lt = t + 1 - TR;
            const uint32_t ma = mem_addr(a, min(lt, last), lane);
            float2 m = *lds_f2(ma);
            tile_step(a, R, ring[(u + 3) % 4], m, P, Fn, Gn, t, h, hh, cmax, S, ((u + OFF) & 1) != 0);  // TR is even
            if (lt <= last) *lds_f2(ma) = m;
        }
    }
    if constexpr (OFF == 1 || (ONCHIP_SPLITBAR & 1)) __syncthreads();  // the last tile (TR + tl - 1, odd) ends no pair
}

// ------------------------------------------------------------------------------------------------
// Adaptive steps (system.rs:111-139, onchip.hpp's ADA_* map).  Pass 1 is the RHS at y (terms with
// y's memories, which stay in the registers: pass1 below, the fixed pass's tile step); pass 2 the RHS
// at the half step.  Each pass is its own unrolled code instance (round 5; until then one instance
// served both under a uniform flag, on the assumption that two would not share the instruction cache
// -- measured, the split is 14 % faster).  In pass 2 each clause gathers its voltages from H and from A
// (y: their min is pass 1's C, recomputed instead of stored), rebuilds its memories' full-step clone
// and first half step from y's memories and that C (:124-128), takes the second half step (:130) and
// its max_error terms (:101-108).  The arithmetic is k_resident's / k_wave's in the
// exact rewritten forms of the header (h dxs = (h/2) (2 dxs), (h/2) dxs = (h/4) (2 dxs), ...).
// Empty slots compute on stand-in memories (0.001, 1): their literals sit at sink words (v = 1.0, so
// mn = 0 in both passes), where xs = 0.001 and xl = 1 are fixed points of both clamped half steps and
// of the full step -- so their error terms are exactly 0 and need no mask.

// Pass 2's records: the 12-byte form, as pass 1 (round 5: +1.2 % on the adaptive leg against the 8-byte
// form, profiles/r05ai_ab_p2r12.txt, at 10 spilled VGPRs instead of 1; 0 = the 8-byte form, A/B only).
#ifndef ONCHIP_ADA_P2_REC12
#define ONCHIP_ADA_P2_REC12 1
#endif
#if ONCHIP_ADA_P2_REC12 && ONCHIP_REC12
typedef SlotF SlotA;
constexpr uint32_t RECA_BYTES = 12;
__device__ __forceinline__ SlotA load_recA(const Recs &R, int t) { return load_recf(R, t); }
struct GathA {  // a clause's gathered inputs: the literals' record words, voltages from H and from A (y)
    uint32_t w0, w1, w2;
    float v0, v1, v2, y0, y1, y2;
};
#else
typedef Slot SlotA;
constexpr uint32_t RECA_BYTES = 8;
__device__ __forceinline__ SlotA load_recA(const Recs &R, int t) { return load_rec(R, t); }
struct GathA {  // a clause's gathered inputs: addresses, sign word, voltages from H and from A (y)
    uint32_t a0, a1, a2, hi;
    float v0, v1, v2, y0, y1, y2;
};
#endif

struct FrontA {  // the min at H and each literal's signed selected value (see Front); the min at y
    uint32_t a0, a1, a2;
    float sel0, sel1, sel2, mn, mn1;
};

#if ONCHIP_ADA_P2_REC12 && ONCHIP_REC12
__device__ __forceinline__ void gatherA(const SlotA &S, GathA &G) {
    G.w0 = S.w0;
    G.w1 = S.w1;
    G.w2 = S.w2;
    const uint32_t a0 = S.w0 & 0xffffu, a1 = S.w1 & 0xffffu, a2 = S.w2 & 0xffffu;
    G.v0 = lds_f(a0 + ADA_H);
    G.v1 = lds_f(a1 + ADA_H);
    G.v2 = lds_f(a2 + ADA_H);
    G.y0 = lds_f(a0);
    G.y1 = lds_f(a1);
    G.y2 = lds_f(a2);
}
#else
__device__ __forceinline__ void gatherA(const SlotA &S, GathA &G) {
    G.a0 = S.lo & 0xffffu;
    G.a1 = S.lo >> 16;
    G.a2 = S.hi & 0xffffu;
    G.hi = S.hi;
    G.v0 = lds_f(G.a0 + ADA_H);
    G.v1 = lds_f(G.a1 + ADA_H);
    G.v2 = lds_f(G.a2 + ADA_H);
    G.y0 = lds_f(G.a0);
    G.y1 = lds_f(G.a1);
    G.y2 = lds_f(G.a2);
}
#endif

__device__ __forceinline__ void frontA(const GathA &G, FrontA &F) {
#if ONCHIP_ADA_P2_REC12 && ONCHIP_REC12
    F.a0 = G.w0 & 0xffffu;
    F.a1 = G.w1 & 0xffffu;
    F.a2 = G.w2 & 0xffffu;
    const uint32_t s0 = G.w0 & 0x80000000u, s1 = G.w1 & 0x80000000u, s2 = G.w2 & 0x80000000u;
#else
    F.a0 = G.a0;
    F.a1 = G.a1;
    F.a2 = G.a2;
    const uint32_t s0 = G.hi & 0x80000000u, s1 = (G.hi << 1) & 0x80000000u, s2 = (G.hi << 2) & 0x80000000u;
#endif
    const float val0 = 1.0f - __uint_as_float(__float_as_uint(G.v0) ^ s0);  // 1 - q v  (:47)
    const float val1 = 1.0f - __uint_as_float(__float_as_uint(G.v1) ^ s1);
    const float val2 = 1.0f - __uint_as_float(__float_as_uint(G.v2) ^ s2);
    const float sel2 = fminf(val0, val1);
    F.sel0 = __uint_as_float(__float_as_uint(fminf(val1, val2)) ^ s0);  // the sign q rides on sel (see Front)
    F.sel1 = __uint_as_float(__float_as_uint(fminf(val0, val2)) ^ s1);
    F.sel2 = __uint_as_float(__float_as_uint(sel2) ^ s2);
    F.mn = fminf(sel2, val2);
    // pass 1's 2 C (:60) from the voltages at y
    const float y0 = 1.0f - __uint_as_float(__float_as_uint(G.y0) ^ s0);
    const float y1 = 1.0f - __uint_as_float(__float_as_uint(G.y1) ^ s1);
    const float y2 = 1.0f - __uint_as_float(__float_as_uint(G.y2) ^ s2);
    F.mn1 = fminf(fminf(y0, y1), y2);
}

__device__ __forceinline__ void backA(const Args &a, const FrontA &F, float2 &mem, float h, float hh, float hq,
                                      Pend &Q, float &e) {
    const float xs = mem.x, xl = mem.y;  // y's memories
    // the full-step clone and the first half step of the memories (:124-128) from pass 1's C
    const float mn1 = F.mn1;
    const float dxs1 = (20.0f * (xs + 0.001f)) * (mn1 - 0.5f);  // 2 dxs (:84)
    const float dxl1 = 2.5f * (mn1 - 0.1f);                      // :85
    const float xs_f = __builtin_amdgcn_fmed3f(xs + hh * dxs1, 0.001f, 1.0f - 0.001f);
    const float xl_f = __builtin_amdgcn_fmed3f(xl + h * dxl1, 1.0f, a.xl_max);
    const float xs_t = __builtin_amdgcn_fmed3f(xs + hq * dxs1, 0.001f, 1.0f - 0.001f);  // the half step's memories
    const float xl_t = __builtin_amdgcn_fmed3f(xl + hh * dxl1, 1.0f, a.xl_max);
    // the RHS at the half step
    const float mn = F.mn;
    const float tt = xl_t * xs_t;
    Q.a0 = F.a0;
    Q.a1 = F.a1;
    Q.a2 = F.a2;
    Q.d0 = tt * F.sel0;  // 2 xl xs G (:64-70, :80), the sign q in sel
    Q.d1 = tt * F.sel1;
    Q.d2 = tt * F.sel2;
    // second half step (:130) and its max_error terms (:132)
    const float dxs2 = (20.0f * (xs_t + 0.001f)) * (mn - 0.5f);
    const float dxl2 = 2.5f * (mn - 0.1f);
    const float xs_n = __builtin_amdgcn_fmed3f(xs_t + hq * dxs2, 0.001f, 1.0f - 0.001f);
    const float xl_n = __builtin_amdgcn_fmed3f(xl_t + hh * dxl2, 1.0f, a.xl_max);
    e = fmaxf(e, fmaxf(fabsf(xs_f - xs_n), fabsf(xl_f - xl_n)));
    mem.x = xs_n;
    mem.y = xl_n;
    asm volatile("" : "+v"(mem.x), "+v"(mem.y), "+v"(e));
}

__device__ __forceinline__ void tile_stepA(const Args &a, const Recs &R, SlotA &slot3, float2 &mem1, Pend &P,
                                           FrontA &Fn, GathA &Gn, int t, float h, float hh, float hq, float &e,
                                           bool bar, bool first, uint32_t cnt, uint32_t &ep) {
    constexpr bool SPL = (ONCHIP_SPLITBAR & 2) != 0;
    if (SPL && first) pair_wait(cnt, ep, a.poll_limit);  // (split barriers: see tile_step)
    const float o0 = lds_f(P.a0 + ADA_D), o1 = lds_f(P.a1 + ADA_D), o2 = lds_f(P.a2 + ADA_D);
    lds_st(P.a0 + ADA_D, o0 + P.d0);
    lds_st(P.a1 + ADA_D, o1 + P.d1);
    lds_st(P.a2 + ADA_D, o2 + P.d2);
    __builtin_amdgcn_sched_barrier(0);
    if (SPL && bar) pair_signal(cnt, ++ep);
    GathA G3;
    gatherA(slot3, G3);
    slot3 = load_recA(R, t + 7);
    __builtin_amdgcn_sched_barrier(0);
    backA(a, Fn, mem1, h, hh, hq, P, e);
    frontA(Gn, Fn);
    __builtin_amdgcn_sched_barrier(0);
    if (bar && !SPL) __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
    Gn = G3;
}

// Register tile T of pass 2; the pass's last tile ends no pair (pass2 closes with a barrier).
template <int TR, int OFF, int T>
__device__ __forceinline__ void reg_tileA(const Args &a, const Recs &R, float2 (&mr)[TR], SlotA (&ring)[4], Pend &P,
                                          FrontA &Fn, GathA &Gn, float h, float hh, float hq, float &e, uint32_t cnt,
                                          uint32_t &ep) {
    constexpr bool bar = ((T + OFF) & 1) != 0 && T + 1 < TR;
    constexpr bool first = T > 0 && ((T - 1 + OFF) & 1) != 0;  // the first tile of a pair after another pair
    if constexpr (T + 1 < TR) {
        tile_stepA(a, R, ring[(T + 3) % 4], mr[T + 1], P, Fn, Gn, T, h, hh, hq, e, bar, first, cnt, ep);
    } else {  // the (empty) tile after the last: stand-in memories (zero error terms), nothing stored
        float2 m = make_float2(0.001f, 1.0f);
        tile_stepA(a, R, ring[(T + 3) % 4], m, P, Fn, Gn, T, h, hh, hq, e, bar, first, cnt, ep);
    }
}

template <int TR, int OFF, int... Ts>
__device__ __forceinline__ void reg_tilesA(std::integer_sequence<int, Ts...>, const Args &a, const Recs &R,
                                           float2 (&mr)[TR], SlotA (&ring)[4], Pend &P, FrontA &Fn, GathA &Gn, float h,
                                           float hh, float hq, float &e, uint32_t cnt, uint32_t &ep) {
    (reg_tileA<TR, OFF, Ts>(a, R, mr, ring, P, Fn, Gn, h, hh, hq, e, cnt, ep), ...);
}

// Pass 2 of an adaptive step over every tile (all in registers): the RHS at the half step (H) into D
// and the memories' second half step, with their error terms.  Ends with a barrier.
template <int TR, int OFF>
__device__ __forceinline__ void pass2(const Args &a, float2 (&mr)[TR], float h, int lane, float &e, uint32_t cnt,
                                      uint32_t &ep) {
    Recs R;
#if ONCHIP_ADA_P2_REC12 && ONCHIP_REC12
    R.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)a.rec12, 0, (int)a.rec12_bytes, 0x00020000);
#else
    R.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)a.rec, 0, (int)a.rec_bytes, 0x00020000);
#endif
    R.voff = (uint32_t)lane * RECA_BYTES;
    R.soff = 0u;
    asm volatile("" : "+s"(R.soff));
    const float hh = 0.5f * h, hq = 0.25f * h;
    SlotA ring[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) ring[s] = load_recA(R, s);
    Pend P;
    GathA G0, G1, Gn;
    gatherA(ring[0], G0);
    ring[0] = load_recA(R, 4);
    gatherA(ring[1], G1);
    ring[1] = load_recA(R, 5);
    gatherA(ring[2], Gn);
    ring[2] = load_recA(R, 6);
    FrontA F0, Fn;
    frontA(G0, F0);
    frontA(G1, Fn);
    backA(a, F0, mr[0], h, hh, hq, P, e);
    reg_tilesA<TR, OFF>(std::make_integer_sequence<int, TR>{}, a, R, mr, ring, P, Fn, Gn, h, hh, hq, e, cnt, ep);
    __syncthreads();
}

// Diagnostic builds only (-DONCHIP_ADA_SKIP=1 | 2, scripts/build_variant.sh; results are wrong): the
// adaptive step without its second / first pass, so that PMC counters of the full build minus those of
// a skip build give one pass's share.
#ifndef ONCHIP_ADA_SKIP
#define ONCHIP_ADA_SKIP 0
#endif
// Pass 1 takes plain barriers, as the fixed pass does: split barriers in pass 1 cost 2.7 %
// (profiles/r05final2_ab_p1plain.txt; 1 = split barriers, A/B only).  Pass 2 keeps its split barriers.
#ifndef ONCHIP_ADA_P1_SPL
#define ONCHIP_ADA_P1_SPL 0
#endif
// The adaptive step's first pass: the fixed pass's tile step with the dv terms into D and no memory
// update -- the 12-byte records, one gather per literal.
template <int TR, int OFF, int T>
__device__ __forceinline__ void reg_tile1(const Args &a, const Recs &R, float2 (&mr)[TR], SlotF (&ring)[4], Pend &P,
                                          Front &Fn, Gath &Gn, uint32_t &cmax, Stamps &S, uint32_t cnt, uint32_t *ep) {
    constexpr bool bar = ((T + OFF) & 1) != 0 && T + 1 < TR;  // (as reg_tileA: pass1 closes with a barrier)
    constexpr bool first = T > 0 && ((T - 1 + OFF) & 1) != 0;
    constexpr bool SPL = (ONCHIP_SPLITBAR & 2) != 0 && ONCHIP_ADA_P1_SPL;
    if constexpr (T + 1 < TR) {
        tile_step<SPL, ADA_D, false>(a, R, ring[(T + 3) % 4], mr[T + 1], P, Fn, Gn, T, 0.0f, 0.0f, cmax, S, bar, first,
                                     cnt, ep);
    } else {  // the (empty) tile after the last: its terms are never applied
        float2 m = make_float2(0.001f, 1.0f);
        tile_step<SPL, ADA_D, false>(a, R, ring[(T + 3) % 4], m, P, Fn, Gn, T, 0.0f, 0.0f, cmax, S, bar, first, cnt, ep);
    }
}

template <int TR, int OFF, int... Ts>
__device__ __forceinline__ void reg_tiles1(std::integer_sequence<int, Ts...>, const Args &a, const Recs &R,
                                           float2 (&mr)[TR], SlotF (&ring)[4], Pend &P, Front &Fn, Gath &Gn,
                                           uint32_t &cmax, Stamps &S, uint32_t cnt, uint32_t *ep) {
    (reg_tile1<TR, OFF, Ts>(a, R, mr, ring, P, Fn, Gn, cmax, S, cnt, ep), ...);
}

// Pass 1 of an adaptive step: the RHS at y (A) into D, the unsat flag at `flag` (:88).  Ends with a
// barrier.
template <int TR, int OFF>
__device__ __forceinline__ void pass1(const Args &a, float2 (&mr)[TR], int lane, uint32_t flag, uint32_t cnt,
                                      uint32_t &ep) {
    Recs R;
#if ONCHIP_REC12
    R.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)a.rec12, 0, (int)a.rec12_bytes, 0x00020000);
#else
    R.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)a.rec, 0, (int)a.rec_bytes, 0x00020000);
#endif
    R.voff = (uint32_t)lane * RECF_BYTES;
    R.soff = 0u;
    asm volatile("" : "+s"(R.soff));
    uint32_t cmax = 0u;
    Stamps S{};
    SlotF ring[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) ring[s] = load_recf(R, s);
    Pend P;
    Gath G0, G1, Gn;
    gather(ring[0], G0);
    ring[0] = load_recf(R, 4);
    gather(ring[1], G1);
    ring[1] = load_recf(R, 5);
    gather(ring[2], Gn);
    ring[2] = load_recf(R, 6);
    Front F0, Fn;
    front(G0, F0);
    front(G1, Fn);
    back<false>(a, F0, mr[0], 0.0f, 0.0f, P, cmax);
    reg_tiles1<TR, OFF>(std::make_integer_sequence<int, TR>{}, a, R, mr, ring, P, Fn, Gn, cmax, S, cnt, &ep);
    if (!(__uint_as_float(cmax) < 0.5f)) lds_st(flag, 1.0f);
    __syncthreads();
}

typedef const __attribute__((address_space(4))) int32_t cint32;

// The state moves through HBM once per launch, read once and written once: non-temporal (aux nt),
// so the launch's 770 MB stream (config 2, B = 1024) does not evict the clause records every CU
// re-reads from L2 at the next round's first pass.  ONCHIP_STATE_AUX=0: default policy (A/B).
#ifndef ONCHIP_STATE_AUX
#define ONCHIP_STATE_AUX 2
#endif
template <typename P> __device__ __forceinline__ P ld_state(const P *p) {
    if constexpr (ONCHIP_STATE_AUX != 0) return __builtin_nontemporal_load(p);
    else return *p;
}
template <typename P> __device__ __forceinline__ void st_state(P *p, P x) {
    if constexpr (ONCHIP_STATE_AUX != 0) __builtin_nontemporal_store(x, p);
    else *p = x;
}
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2 ld_state(const float2 *p) {
    const f2v x = ld_state(reinterpret_cast<const f2v *>(p));
    return make_float2(x.x, x.y);
}
__device__ __forceinline__ void st_state(float2 *p, float2 x) {
    f2v y;
    y.x = x.x;
    y.y = x.y;
    st_state(reinterpret_cast<f2v *>(p), y);
}
// The replica's clause memories as a buffer resource (m float2 records): tile j's slot of lane l is
// the byte offset 8 (tc[j] + l), checked against the range as a whole (the VGPR offset: the scalar
// offset is not range-checked), so a slot past the replica's memories reads 0 and stores nothing.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mem_rsrc(float *base, int m) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, 8 * m, 0x00020000);
}

// Load the register tiles' memories.  The start of this wave's clauses in tile j is a scalar load
// at a static offset of the padded wave table (tcw = tc + wave; a tile past the last one starts at
// m), so the compiler batches them into wide scalar loads.  The loads are unconditional: a slot past the end of the memories reads 0 (buffer
// range check), any other empty slot reads the next tile's clause -- neither is used, since an
// empty slot's literals point at the sink words (its terms go to the dv sinks) and its update is
// not stored.
// Adaptive launches: every empty slot of a register tile gets the stand-in memories (0.001, 1) (see
// backA), once per launch.
template <int TR, int... Js>
__device__ __forceinline__ void mem_standins(std::integer_sequence<int, Js...>, const cint32 *tcw, int wl,
                                             float2 (&mr)[TR]) {
    auto one = [&](auto J) {
        constexpr int j = decltype(J)::value;
        const bool empty = wl >= tcw[j * WAVES + 1] - tcw[j * WAVES];
        mr[j].x = empty ? 0.001f : mr[j].x;
        mr[j].y = empty ? 1.0f : mr[j].y;
    };
    (one(std::integral_constant<int, Js>{}), ...);
}

template <int TR, int... Js>
__device__ __forceinline__ void mem_load(std::integer_sequence<int, Js...>, const cint32 *tcw,
                                         __amdgpu_buffer_rsrc_t rs, uint32_t lane8, float2 (&mr)[TR]) {
    typedef int i2 __attribute__((ext_vector_type(2)));
    auto one = [&](auto J) {
        constexpr int j = decltype(J)::value;
        const i2 r = __builtin_amdgcn_raw_buffer_load_b64(rs, lane8 + 8u * (uint32_t)tcw[j * WAVES], 0, ONCHIP_STATE_AUX);
        mr[j] = make_float2(__int_as_float(r.x), __int_as_float(r.y));
    };
    (one(std::integral_constant<int, Js>{}), ...);
}

// Store them back, 8 tiles at a time (the last group may be shorter): the group's wave bounds are
// loaded together (scalar loads, no wait per tile); a lane whose slot of tile j holds no clause
// stores out of the buffer's range, which drops the store.
template <int TR, int... Gs>
__device__ __forceinline__ void mem_store(std::integer_sequence<int, Gs...>, const cint32 *tcw,
                                          __amdgpu_buffer_rsrc_t rs, int lane, const float2 (&mr)[TR]) {
    typedef int i2 __attribute__((ext_vector_type(2)));
    auto group = [&](auto G) {
        constexpr int j0 = decltype(G)::value * 8;
        constexpr int cnt = TR - j0 < 8 ? TR - j0 : 8;
        int b[8], e[8];
#pragma unroll
        for (int k = 0; k < cnt; ++k) {
            b[k] = tcw[(j0 + k) * WAVES];
            e[k] = tcw[(j0 + k) * WAVES + 1];
        }
#pragma unroll
        for (int k = 0; k < cnt; ++k) {
            const uint32_t vo = lane < e[k] - b[k] ? 8u * (uint32_t)(b[k] + lane) : 0x80000000u;
            i2 r;
            r.x = __float_as_int(mr[j0 + k].x);
            r.y = __float_as_int(mr[j0 + k].y);
            __builtin_amdgcn_raw_buffer_store_b64(r, rs, vo, 0, ONCHIP_STATE_AUX);
        }
    };
    (group(std::integral_constant<int, Gs>{}), ...);
}

// The kernel declares no static LDS, so dynamic LDS -- and the records' byte addresses -- start at 0.
template <int TR, int OFF, bool ADA>
__global__ __launch_bounds__(NTH) void k_onchip(Args a) {
    const int g = blockIdx.x, lane = threadIdx.x;
    const int wl = lane & 63;  // slot of this lane in its wave's share of a tile
    ONCHIP_PHASE(0);
    if (lane == 0) io_begin_store<float>(a.io, g, a.act, a.sat_step, a.steps_done, a.dtr, ADA, a.stop);
    int act = io_active(a.io, a.act, g);
    if (!act) return;  // frozen replica (uniform)
    if (a.stop_mode == ODESAT_STOP_ANY && *a.stop < a.step0) return;  // an earlier step stopped every replica
    const bool p = __builtin_amdgcn_readfirstlane((int)a.par[g]) != 0;
    float *V = (p ? a.v1 : a.v0) + (size_t)g * a.n;
    float2 *CM = reinterpret_cast<float2 *>((p ? a.c1 : a.c0) + (size_t)g * a.m * 2);
    // out of place (a.oop, STOP_ANY launches of several steps): the final state goes to the other
    // buffer and par flips, so the launch's starting state survives for a replay
    const bool q = a.oop ? !p : p;
    const int n2 = a.n + SINKS;
    constexpr uint32_t DV = ADA ? ADA_D : DVC;
    // two unsat flags (adaptive: after A's sinks, then the waves' error words)
    const uint32_t UNS = ADA ? 4u * (uint32_t)n2 : DVC + 4u * (uint32_t)n2;
    int64_t sat = io_sat(a.io, a.sat_step, g), done = io_done(a.io, a.steps_done, g);
    const cint32 *tcw = (const cint32 *)a.tc + __builtin_amdgcn_readfirstlane(lane >> 6);  // this wave's starts

    // The clause memories first: their loads (one per register tile and lane) stay in flight while v
    // streams into LDS behind them.
    const int mlast = a.m - 1;
    float2 mr[TR];
    mem_load<TR>(std::make_integer_sequence<int, TR>{}, tcw, mem_rsrc((p ? a.c1 : a.c0) + (size_t)g * a.m * 2, a.m),
                 8u * (uint32_t)wl, mr);
    {   // v (sinks = 1.0) into LDS, dv = 0 (:33): the loads of a pass issued together, then the stores
        if ((a.n & 3) == 0) {  // 16 bytes per access (V, v, dv and H are 16-byte aligned; n + SINKS % 4 == 0)
            constexpr int U = 4;
            const int n4 = n2 >> 2, nv4 = a.n >> 2;
            for (int q0 = lane; q0 < n4; q0 += NTH * U) {
                f4v x[U];
#pragma unroll
                for (int u = 0; u < U; ++u) x[u] = ld_state(reinterpret_cast<const f4v *>(V) + min(q0 + u * NTH, nv4 - 1));
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int q = q0 + u * NTH;
                    if (q < n4) {
                        const f4v one4 = {1.0f, 1.0f, 1.0f, 1.0f};
                        lds_st4(16u * q, q < nv4 ? x[u] : one4);
                        lds_st4(16u * q + DV, f4v{0.0f, 0.0f, 0.0f, 0.0f});
                        if (ADA && q >= nv4) lds_st4(16u * q + ADA_H, one4);  // H's sinks (pass 2 gathers them)
                    }
                }
            }
        } else {
            constexpr int U = 16;
            for (int i0 = lane; i0 < n2; i0 += NTH * U) {
                float x[U];
#pragma unroll
                for (int u = 0; u < U; ++u) x[u] = ld_state(&V[min(i0 + u * NTH, a.n - 1)]);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int i = i0 + u * NTH;
                    if (i < n2) {
                        lds_st(4u * i, i < a.n ? x[u] : 1.0f);
                        lds_st(4u * i + DV, 0.0f);
                        if (ADA && i >= a.n) lds_st(4u * i + ADA_H, 1.0f);  // H's sinks (pass 2 gathers them)
                    }
                }
            }
        }
    }
    if constexpr (ADA) mem_standins<TR>(std::make_integer_sequence<int, TR>{}, tcw, wl, mr);
    for (int t = 0; t < a.tl; ++t) {
        const int c0 = tcw[(TR + t) * WAVES];
        *lds_f2(mem_addr(a, t, lane)) = ld_state(&CM[min(c0 + wl, mlast)]);  // (empty slots: as mem_io)
    }
    // the waves' pair counts (split barriers): after the unsat flags (adaptive: and the error words)
    const uint32_t CNT = UNS + 8u + (ADA ? 4u * WAVES : 0u);
    if (lane < 2) lds_st(UNS + 4u * lane, 0.0f);
    if ((ONCHIP_SPLITBAR & (ADA ? 2 : 1)) && lane < 2 * WAVES) lds_st(CNT + 4u * lane, 0.0f);  // + the fault slots
    __syncthreads();
    ONCHIP_PHASE(1);
    uint32_t ep = 0u;  // the pairs every wave has signalled so far

    const float h = a.dt, hh = 0.5f * a.dt;
    Stamps S{};
    float dtr = ADA ? io_dt<float>(a.io, a.dtr, g) : a.dt;
    if constexpr (ADA) {
#ifdef ONCHIP_ADA_STAMPS
        uint64_t ada_st[5] = {0, 0, 0, 0, 0};
        uint64_t ada_last = ada_memtime();
#endif
        for (int k = 0; k < a.nsteps; ++k) {  // euler_step (system.rs:111-139)
            const float hk = dtr, hhk = 0.5f * dtr, hqk = 0.25f * dtr;
            const uint32_t flag = UNS + 4u * (k & 1);
            float e = 0.0f;
#if ONCHIP_ADA_SKIP == 2  // diagnostic build (results wrong): no pass 1, every step takes pass 2
            if (lane == 0) lds_st(flag, 1.0f);
            __syncthreads();
#else
            pass1<TR, OFF>(a, mr, lane, flag, CNT, ep);  // the RHS at y into D, the unsat flag
#endif
            ADA_STAMP(ada_st[0]);
            const bool uns = lds_f(flag) != 0.0f;  // uniform
            if (!uns) {  // an allsat replica takes no step (:122): drop pass 1's terms
                for (int i = lane; i < a.n; i += NTH) lds_st(4u * i + ADA_D, 0.0f);
            } else {
                // full-step clone and first half step (:124-128), four variables per LDS access (A, D,
                // H and F are 16-byte aligned), then the n % 4 last ones
                for (int i4 = lane; i4 < (a.n >> 2); i4 += NTH) {
                    const uint32_t o = 16u * (uint32_t)i4;
                    const f4v d2 = lds_f4(o + ADA_D), y = lds_f4(o);
                    lds_st4(o + ADA_D, f4v{0.0f, 0.0f, 0.0f, 0.0f});
                    f4v vf, vh;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        vf[u] = __builtin_amdgcn_fmed3f(y[u] + hhk * d2[u], -1.0f, 1.0f);
                        vh[u] = __builtin_amdgcn_fmed3f(y[u] + hqk * d2[u], -1.0f, 1.0f);
                    }
                    lds_st4(o + ADA_F, vf);
                    lds_st4(o + ADA_H, vh);
                }
                for (int i = (a.n & ~3) + lane; i < a.n; i += NTH) {
                    const float d2 = lds_f(4u * i + ADA_D), y = lds_f(4u * i);
                    lds_st(4u * i + ADA_D, 0.0f);
                    lds_st(4u * i + ADA_F, __builtin_amdgcn_fmed3f(y + hhk * d2, -1.0f, 1.0f));
                    lds_st(4u * i + ADA_H, __builtin_amdgcn_fmed3f(y + hqk * d2, -1.0f, 1.0f));
                }
                __syncthreads();
                ADA_STAMP(ada_st[1]);
#if ONCHIP_ADA_SKIP != 1  // (diagnostic build 1: no pass 2)
                pass2<TR, OFF>(a, mr, hk, lane, e, CNT, ep);  // the RHS at the half step, the memories' step
#endif
                ADA_STAMP(ada_st[2]);
                // second half step (:130), max_error (:101-108); the same lane ownership as the final
                // store below
                for (int i4 = lane; i4 < (a.n >> 2); i4 += NTH) {
                    const uint32_t o = 16u * (uint32_t)i4;
                    const f4v d2 = lds_f4(o + ADA_D), vh = lds_f4(o + ADA_H), vf = lds_f4(o + ADA_F);
                    lds_st4(o + ADA_D, f4v{0.0f, 0.0f, 0.0f, 0.0f});
                    f4v vn;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        vn[u] = __builtin_amdgcn_fmed3f(vh[u] + hqk * d2[u], -1.0f, 1.0f);
                        e = fmaxf(e, fabsf(vf[u] - vn[u]));
                    }
                    lds_st4(o, vn);
                }
                for (int i = (a.n & ~3) + lane; i < a.n; i += NTH) {
                    const float d2 = lds_f(4u * i + ADA_D);
                    lds_st(4u * i + ADA_D, 0.0f);
                    const float vn = __builtin_amdgcn_fmed3f(lds_f(4u * i + ADA_H) + hqk * d2, -1.0f, 1.0f);
                    e = fmaxf(e, fabsf(lds_f(4u * i + ADA_F) - vn));
                    lds_st(4u * i, vn);
                }
                uint32_t eb = __float_as_uint(e);  // non-negative: the bits order as the values
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) eb = max(eb, (uint32_t)__shfl_xor((int)eb, off, 64));
                if ((lane & 63) == 0) lds_st(UNS + 8u + 4u * (uint32_t)(lane >> 6), __uint_as_float(eb));
                ADA_STAMP(ada_st[3]);
            }
            if (lane == 0) lds_st(UNS + 4u * ((k + 1) & 1), 0.0f);  // read by everyone after this step's first pass
            __syncthreads();
            if (uns) {  // :133-135 dt <- clamp(dt * sqrt(tol / err), 2^-7, 1e3)
                uint32_t eb = 0u;
#pragma unroll
                for (int w = 0; w < WAVES; ++w) eb = max(eb, __float_as_uint(lds_f(UNS + 8u + 4u * w)));
                dtr = fmaxf(fminf(dtr * sqrtf(a.tol / __uint_as_float(eb)), 1e3f), 0.0078125f);
            }
            ADA_STAMP(ada_st[4]);
            done += 1;
            if (!uns) {  // allsat: no step taken (:122)
                const int step = a.step0 + k;
                if (sat < 0) sat = step;
                if (a.stop_mode == ODESAT_STOP_ANY && lane == 0) atomicMin(a.stop, step);  // simulate_inter (:291)
                if (a.stop_mode == ODESAT_STOP_EACH) {                                      // simulate (:193)
                    act = 0;
                    break;
                }
            }
        }
#ifdef ONCHIP_ADA_STAMPS
        if ((lane & 63) == 0 && g == 0)
            for (int i = 0; i < 5; ++i) g_onchip_ada_stamps[(lane >> 6) * 5 + i] = ada_st[i];
#endif
    } else
    for (int k = 0; k < a.nsteps; ++k) {  // euler_step_fixed (system.rs:141-154)
        uint32_t cmax = 0u;
#ifdef ONCHIP_STAMPS
        S.last = memtime();
#endif
        pass<TR, OFF>(a, mr, h, lane, cmax, S, CNT, ep);
        if (!(__uint_as_float(cmax) < 0.5f)) lds_st(UNS + 4u * (k & 1), 1.0f);
        // :96 (h dv = (h/2) dv2), dv restarts at 0 (:33): four variables per lane and access (v and dv
        // are 16-byte aligned), then the n % 4 last ones
        for (int i4 = lane; i4 < (a.n >> 2); i4 += NTH) {
            const uint32_t o = 16u * (uint32_t)i4;
            const f4v d2 = lds_f4(o + DVC);
            lds_st4(o + DVC, f4v{0.0f, 0.0f, 0.0f, 0.0f});
            f4v v = lds_f4(o);
            v.x = __builtin_amdgcn_fmed3f(v.x + hh * d2.x, -1.0f, 1.0f);
            v.y = __builtin_amdgcn_fmed3f(v.y + hh * d2.y, -1.0f, 1.0f);
            v.z = __builtin_amdgcn_fmed3f(v.z + hh * d2.z, -1.0f, 1.0f);
            v.w = __builtin_amdgcn_fmed3f(v.w + hh * d2.w, -1.0f, 1.0f);
            lds_st4(o, v);
        }
        for (int i = (a.n & ~3) + lane; i < a.n; i += NTH) {
            const float d2 = lds_f(4u * i + DVC);
            lds_st(4u * i + DVC, 0.0f);
            lds_st(4u * i, __builtin_amdgcn_fmed3f(lds_f(4u * i) + hh * d2, -1.0f, 1.0f));
        }
        if (lane == 0) lds_st(UNS + 4u * ((k + 1) & 1), 0.0f);  // read by everyone before this step's first barrier
        __syncthreads();
        done += 1;
        if (lds_f(UNS + 4u * (k & 1)) == 0.0f) {  // allsat before the update; the step was still taken (:148-152)
            const int step = a.step0 + k;
            if (sat < 0) sat = step;
            if (a.stop_mode == ODESAT_STOP_ANY && lane == 0) atomicMin(a.stop, step);  // simulate_inter (:291)
            if (a.stop_mode == ODESAT_STOP_EACH) {                                      // simulate (:193)
                act = 0;
                break;
            }
        }
    }

    ONCHIP_PHASE(2);
    float *Vo = (q ? a.v1 : a.v0) + (size_t)g * a.n;
    // written by this lane in the last update (four variables per lane, then the tail)
    for (int i4 = lane; i4 < (a.n >> 2); i4 += NTH) {
        const f4v v = lds_f4(16u * (uint32_t)i4);
        st_state(&Vo[4 * i4], v.x);
        st_state(&Vo[4 * i4 + 1], v.y);
        st_state(&Vo[4 * i4 + 2], v.z);
        st_state(&Vo[4 * i4 + 3], v.w);
    }
    for (int i = (a.n & ~3) + lane; i < a.n; i += NTH) st_state(&Vo[i], lds_f(4u * i));
    {   // opaque copies: the store addresses are recomputed here instead of being kept live (two
        // VGPRs per tile) across the step loop from the loads above
        float2 *CMs = reinterpret_cast<float2 *>((q ? a.c1 : a.c0) + (size_t)g * a.m * 2);
        const cint32 *tcs = tcw;
        asm volatile("" : "+s"(CMs), "+s"(tcs));
        mem_store<TR>(std::make_integer_sequence<int, (TR + 7) / 8>{}, tcs, mem_rsrc(reinterpret_cast<float *>(CMs), a.m), wl, mr);
        for (int t = 0; t < a.tl; ++t) {  // this lane's own LDS slots: no barrier needed
            const int c0 = tcw[(TR + t) * WAVES], c1 = tcw[(TR + t) * WAVES + 1];
            const int c = c0 + wl;
            if (c < c1) st_state(&CMs[c], *lds_f2(mem_addr(a, t, lane)));
        }
    }
#ifdef ONCHIP_STAMPS
    if ((lane & 63) == 0 && g < 4096) {
        unsigned long long *o = g_onchip_stamps + ((size_t)g * 16 + lane / 64) * 4;
        o[0] = S.bar;
        o[1] = S.work;
        o[2] = S.rmw;
        o[3] = S.tiles;
    }
#endif
    ONCHIP_PHASE(3);
    // a split-barrier wait that gave up (EP_TIMEOUT): the dv updates may have raced, so the call must
    // fail -- the fault word beside the stop word, read by the host after the call (ODESAT_EDEVICE)
    // (the fault slots after the pair counts; every wave's store to them precedes the steps' last barrier)
    // (compared as a word: pair_wait stores the integer 1, a denormal that a flushing build would read as 0)
    if ((ONCHIP_SPLITBAR & (ADA ? 2 : 1)) && lane < WAVES && __float_as_uint(lds_f(CNT + 4u * (WAVES + lane))) != 0u)
        atomicOr(reinterpret_cast<unsigned *>(a.stop + 1), 1u);
    if (lane == 0) {
        if (a.oop) a.par[g] = (uint8_t)q;
        a.act[g] = (uint8_t)act;
        a.sat_step[g] = sat;
        a.steps_done[g] = done;
        if (ADA) a.dtr[g] = dtr;
        io_mirror<float>(a.io, g, sat, done, dtr, ADA);
    }
}

}  // namespace

bool split_barriers(bool adaptive) { return (ONCHIP_SPLITBAR & (adaptive ? 2 : 1)) != 0; }

namespace {

template <int TR, int OFF, bool ADA> hipError_t launch_t(const Args &a, int G, size_t lds, hipStream_t stream) {
    hipError_t e = odesat::ensure_max_lds(reinterpret_cast<const void *>(&k_onchip<TR, OFF, ADA>), (int)LDS_MAX);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_onchip<TR, OFF, ADA>), dim3((unsigned)G), dim3(NTH), lds, stream, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch(int tr, int off, const Args &a, int G, size_t lds, hipStream_t stream, bool adaptive) {
    switch (tr) {
#ifdef ONCHIP_ONLY_TR  // experiments: one shape (scripts/build_variant.sh style quick builds)
#define ONCHIP_CASE(N)                                                                                  \
    case N:                                                                                             \
        if constexpr (N == ONCHIP_ONLY_TR) {                                                            \
            if (adaptive) return off ? launch_t<N, 1, true>(a, G, lds, stream) : launch_t<N, 0, true>(a, G, lds, stream); \
            return off ? launch_t<N, 1, false>(a, G, lds, stream) : launch_t<N, 0, false>(a, G, lds, stream); \
        } else return hipErrorInvalidValue;
#else
#define ONCHIP_CASE(N)                                                                                  \
    case N:                                                                                             \
        if (adaptive) return off ? launch_t<N, 1, true>(a, G, lds, stream) : launch_t<N, 0, true>(a, G, lds, stream); \
        return off ? launch_t<N, 1, false>(a, G, lds, stream) : launch_t<N, 0, false>(a, G, lds, stream);
#endif
        ONCHIP_CASE(8) ONCHIP_CASE(16) ONCHIP_CASE(24) ONCHIP_CASE(32) ONCHIP_CASE(40) ONCHIP_CASE(48)
        ONCHIP_CASE(56) ONCHIP_CASE(64) ONCHIP_CASE(66) ONCHIP_CASE(68) ONCHIP_CASE(70) ONCHIP_CASE(72)
        ONCHIP_CASE(74) ONCHIP_CASE(76) ONCHIP_CASE(78) ONCHIP_CASE(80) ONCHIP_CASE(82) ONCHIP_CASE(84)
        ONCHIP_CASE(86) ONCHIP_CASE(88) ONCHIP_CASE(90) ONCHIP_CASE(92) ONCHIP_CASE(94) ONCHIP_CASE(96)
#undef ONCHIP_CASE
        default: return hipErrorInvalidValue;
    }
}

}  // namespace onchip

#ifdef ONCHIP_STAMPS
// Diagnostic build only: copy out the per-(replica, wave) stamp sums {barrier wait, work, dv RMW,
// tiles} of the last launches (replicas < 4096, 16 wave slots each).
extern "C" int odesat_onchip_stamps(unsigned long long *out, int count) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(onchip::g_onchip_stamps), sizeof(unsigned long long) * (size_t)count, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

#ifdef ONCHIP_PHASES
// Diagnostic build only: the per-workgroup phase stamps of the last launch (4096 x 4, s_memrealtime).
extern "C" int odesat_onchip_phases(unsigned long long *out, int count) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(onchip::g_onchip_phases), sizeof(unsigned long long) * (size_t)count, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int odesat_onchip_clk(unsigned long long *out, int count) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(onchip::g_onchip_clk), sizeof(unsigned long long) * (size_t)count, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

#ifdef ONCHIP_ADA_STAMPS
// Diagnostic build only: workgroup 0's adaptive-step segment sums of the last launch (8 waves x 5).
extern "C" int odesat_onchip_ada_stamps(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(onchip::g_onchip_ada_stamps), sizeof(unsigned long long) * 40, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
