// onchip.hpp -- host interface of the on-chip integrator (onchip.hip, ODESAT_ALG_ONCHIP).
//
// One workgroup (512 threads, one per CU) owns ONE replica for a launch of many fixed Euler
// steps, with its whole state on the CU: voltages v[n] and accumulators dv[n] in LDS, clause
// memories (xs, xl) in VGPRs (the first TR tiles) and LDS (the remaining tl tiles).  Per step
// nothing but the clause records (8 B per clause, L2-resident, shared by every CU) is read from
// the memory hierarchy; HBM sees the state once at launch start and once at launch end.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>

#include "callio.hpp"

namespace onchip {

constexpr int NTH = 512;           // threads per workgroup = tile capacity in clauses
constexpr int WAVES = NTH / 64;    // slots [64 w, 64 w + 64) of a tile are wave w's
constexpr int TILE_LDS = NTH * 8;  // LDS bytes of one LDS-resident tile of memories (float2 per lane)
constexpr int SINKS = 32;          // sink words after v and after dv (empty slots of lane l use l % 32)
constexpr uint32_t DVC = 65520;    // LDS byte offset of dv[0] from v[0], 16-byte aligned: the ds instructions' 16-bit
                                   // immediate offset, so one address VGPR serves v and dv
constexpr int MAX_N = (int)(DVC / 4) - SINKS;  // v and its sinks below DVC
constexpr size_t LDS_MAX = 160 * 1024;

// LDS map (bytes): v[n + SINKS] at 0 (sinks = 1.0), memory tiles in the gap up to DVC, 2 dv[n +
// SINKS] (twice dv: see onchip.hip) at DVC, two unsat flags, the waves' pair counts (ONCHIP_SPLITBAR),
// then the remaining memory tiles.
struct Lds {
    uint32_t gap_base, gap_tiles, after_base, after_tiles;
};
inline Lds lds_map(int64_t n) {
    Lds L;
    const uint32_t vend = (uint32_t)(4 * (n + SINKS));
    L.gap_base = (vend + 7u) & ~7u;
    L.gap_tiles = L.gap_base < DVC ? (DVC - L.gap_base) / TILE_LDS : 0;
    L.after_base = ((DVC + vend + 8u + 8u * WAVES) + 7u) & ~7u;  // after dv: two unsat flags, the waves' pair counts, the fault slots
    L.after_tiles = L.after_base < LDS_MAX ? (uint32_t)((LDS_MAX - L.after_base) / TILE_LDS) : 0;
    return L;
}
inline size_t lds_bytes(int64_t n, int tl) {
    const Lds L = lds_map(n);
    const uint32_t after = tl > (int)L.gap_tiles ? (uint32_t)tl - L.gap_tiles : 0u;
    return (size_t)L.after_base + (size_t)after * TILE_LDS;
}
inline int tl_max(int64_t n) {
    const Lds L = lds_map(n);
    return (int)(L.gap_tiles + L.after_tiles) / 4 * 4;
}

// Adaptive steps (system.rs:111-139) keep four voltage arrays in LDS and every tile's memories in
// VGPRs (no LDS tiles): A = the step's starting voltages y (and then its result), D = 2 dv (within
// the ds instructions' 16-bit immediate of A, as DVC), H = the half step, F = the full-step clone,
// n + SINKS floats each; A's region also holds the unsat flags and the waves' error words.
constexpr uint32_t ADA_D = 40960, ADA_H = 81920, ADA_F = 122880;
constexpr int ADA_FLAGS = 2 + 3 * WAVES;  // two unsat flags, the waves' error words, their pair counts, the fault slots
constexpr int ADA_MAX_N = (int)(ADA_D / 4) - SINKS - ADA_FLAGS;

struct Args {
    const uint64_t *rec; // [tiles][NTH] slot-major clause records (make_rec), padded with empty tiles
    uint32_t rec_bytes;
    const uint32_t *rec12;  // ONCHIP_REC12: the same records in 12 bytes (make_rec12), [tiles][NTH][3]
    uint32_t rec12_bytes;
    const int32_t *tc;   // wave starts: wave w of tile t holds internal clauses [tc[8t+w], tc[8t+w+1]) in
                         // its lanes 0.. (the rest of its slots are empty); padded with m to at least
                         // 8 (TR + tl) + 1 entries (constant memory reads at static offsets)
    float *v0, *v1;      // voltages, [B][n] (par selects the buffer holding the current state)
    float *c0, *c1;      // clause memories, [B][m][2] (xs, xl), internal clause order
    uint8_t *par;        // [B] (flipped by an out-of-place launch)
    uint8_t *act;        // [B] replica still stepping
    int64_t *sat_step, *steps_done;
    int32_t *stop;       // first stop step (STOP_ANY), INT_MAX = none
    int32_t n, m, ntiles, tl;  // tiles [0, TR) live in VGPRs, [TR, TR + tl) in LDS
    int32_t step0, nsteps, stop_mode;
    int32_t oop;         // 1: write the final state to the other buffer and flip par (replayable launch)
    float dt, xl_max;
    Lds lds;
    float *dtr;          // [B] per-replica adaptive dt (adaptive launches)
    float tol;           // adaptive tolerance, as the solver's f32
    CallIO io;           // per-call bookkeeping (callio.hpp)
    uint32_t poll_limit; // split-barrier polls before a wait gives up and reports the fault (onchip.hip)
};

// Register-tile counts compiled (template instantiations; VGPRs ~ 50 + 2 TR, ~245 at TR = 96).
// Every launch runs all TR register tiles (an empty one costs as much as a full one: a barrier and
// the whole tile code), so the host picks the smallest TR >= the tiles that hold clauses -- in steps
// of 2 where real instances land (config 2: 90 tiles, k_onchip<90>) -- else TR = 96 plus LDS tiles
// for the rest.  A branch that skipped the empty tiles instead costs every tile a join (register
// copies and a vmcnt(0) wait on the record ring).
constexpr int TR_CHOICES[] = {8, 16, 24, 32, 40, 48, 56, 64, 66, 68, 70, 72, 74, 76, 78, 80,
                              82, 84, 86, 88, 90, 92, 94, 96};
constexpr int TR_MAX = 96;

// Record of one clause slot (8 bytes): lo = a0 | a1 << 16, hi = a2 | neg0 << 31 | neg1 << 30 |
// neg2 << 29, with a_j = 4 * var_j the LDS byte address of the literal's voltage; an empty slot
// (all three literals at its lane's sink word) also has REC_EMPTY in hi.
constexpr uint32_t REC_EMPTY = 1u << 28;
inline uint64_t make_rec(uint32_t a0, uint32_t a1, uint32_t a2, bool n0, bool n1, bool n2) {
    const uint32_t lo = a0 | (a1 << 16);
    const uint32_t hi = a2 | (n0 ? 0x80000000u : 0u) | (n1 ? 0x40000000u : 0u) | (n2 ? 0x20000000u : 0u);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
// 12-byte records (the fixed-step kernel; ONCHIP_REC12=0 builds the 8-byte form, A/B: 12 bytes are
// ~2 % faster, profiles/r03_rec12_ab.txt): one word per literal, its 16-bit LDS
// address and its sign at bit 31, so no literal's sign needs a shift (both passes of the adaptive
// kernel read them too since round 5: ONCHIP_ADA_P2_REC12, onchip.hip)
#ifndef ONCHIP_REC12
#define ONCHIP_REC12 1
#endif
inline void make_rec12(uint32_t a0, uint32_t a1, uint32_t a2, bool n0, bool n1, bool n2, uint32_t *w) {
    w[0] = a0 | (n0 ? 0x80000000u : 0u);
    w[1] = a1 | (n1 ? 0x80000000u : 0u);
    w[2] = a2 | (n2 ? 0x80000000u : 0u);
}

// Launch over replicas [0, G) on `stream`; tr must be one of TR_CHOICES, off (0 / 1) the pair offset
// of the wave-paired tiles (a barrier after tile t iff t + off is odd).  adaptive: euler_step with
// per-replica dt (a.dtr, a.tol); needs a.tl == 0 and n <= ADA_MAX_N, and LDS_MAX bytes of LDS.
hipError_t launch(int tr, int off, const Args &a, int G, size_t lds, hipStream_t stream, bool adaptive = false);
// The launch's kernel may wait on split barriers (ONCHIP_SPLITBAR, onchip.hip), whose bounded wait
// reports a timeout in the fault word stop[1]: the host then checks that word after the call.
bool split_barriers(bool adaptive);

}  // namespace onchip
