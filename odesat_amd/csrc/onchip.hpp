// onchip.hpp -- host interface of the on-chip integrator (onchip.hip, ODESAT_ALG_ONCHIP).
//
// One workgroup (512 threads, one per CU) owns ONE replica for a launch of many fixed Euler
// steps, with its whole state on the CU: voltages v[n] and accumulators dv[n] in LDS, clause
// memories (xs, xl) in VGPRs (the first TR tiles) and LDS (the remaining TL tiles).  Per step
// nothing but the clause topology (8 B per clause, L2-resident, shared by every CU) is read
// from the memory hierarchy; HBM sees the state once at launch start and once at launch end.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace onchip {

constexpr int NTH = 512;           // threads per workgroup = tile capacity in clauses
constexpr int TILE_LDS = NTH * 8;  // LDS bytes of one LDS-resident tile of memories (float2 per lane)
constexpr int SINKS = 32;          // sink words after v and after dv (empty slots of lane l use l % 32)
constexpr int MAX_N = 16352;       // 4 (n + SINKS) < 65536: LDS byte addresses fit the 16-bit record fields
constexpr size_t LDS_MAX = 160 * 1024;

struct Args {
    const uint64_t *rec; // [tiles][NTH] slot-major clause records (make_rec), padded with empty tiles
    const int32_t *tc;   // [ntiles + 1] first internal clause of each tile (constant memory reads)
    float *v0, *v1;      // voltages, [B][n] (par selects the buffer holding the current state)
    float *c0, *c1;      // clause memories, [B][m][2] (xs, xl), internal clause order
    const uint8_t *par;  // [B]
    uint8_t *act;        // [B] replica still stepping
    int64_t *sat_step, *steps_done;
    int32_t *stop;       // first stop step (STOP_ANY), INT_MAX = none
    int32_t n, m, ntiles, tl;  // tiles [0, TR) live in VGPRs, [TR, TR + tl) in LDS
    int32_t step0, nsteps, stop_mode;
    float dt, zeta, xl_max;
};

// Register-tile counts compiled (template instantiations; VGPRs ~ 54 + 2 TR, 248 at TR = 96).
// Every launch runs all TR register tiles (the empty ones cost a barrier each), so the host picks
// the smallest TR >= ntiles, else TR = 96 plus LDS tiles for the rest.
constexpr int TR_CHOICES[] = {8, 16, 24, 32, 40, 48, 56, 64, 72, 80, 88, 96};
constexpr int TR_MAX = 96;

// LDS bytes of a launch: v and dv with their sinks, two flags, tl tiles of memories.
inline size_t lds_bytes(int64_t n, int tl) { return (size_t)8 * (n + SINKS) + 8 + (size_t)tl * TILE_LDS; }

// Record of one clause slot (8 bytes): lo = a0 | a1 << 16, hi = a2 | neg0 << 31 | neg1 << 30 |
// neg2 << 29, with a_j = 4 * var_j the LDS byte address of the literal's voltage.
inline uint64_t make_rec(uint32_t a0, uint32_t a1, uint32_t a2, bool n0, bool n1, bool n2) {
    const uint32_t lo = a0 | (a1 << 16);
    const uint32_t hi = a2 | (n0 ? 0x80000000u : 0u) | (n1 ? 0x40000000u : 0u) | (n2 ? 0x20000000u : 0u);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Launch over replicas [0, G) on `stream`; tr must be one of TR_CHOICES.
hipError_t launch(int tr, const Args &a, int G, size_t lds, hipStream_t stream);

}  // namespace onchip
