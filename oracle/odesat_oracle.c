/*
 * odesat_oracle.c -- CPU restatement of /root/reference/src/system.rs (TEST INFRASTRUCTURE ONLY;
 * see odesat_oracle.h for the parity status).  Built by oracle/Makefile into
 * oracle/build/libodesat_oracle.so; loaded only by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.
 */
#include "odesat_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- f64: the reference's own precision ---- */
#define R double
#define P oc64_
#define FMIN fmin
#define FMAX fmax
#define FABS fabs
#define FSQRT sqrt
#include "oracle_body.inc"
#undef R
#undef P
#undef FMIN
#undef FMAX
#undef FABS
#undef FSQRT

/* ---- f32: same expressions, every constant and operation in f32 ---- */
#define R float
#define P oc32_
#define FMIN fminf
#define FMAX fmaxf
#define FABS fabsf
#define FSQRT sqrtf
#include "oracle_body.inc"
#undef R
#undef P
#undef FMIN
#undef FMAX
#undef FABS
#undef FSQRT

/* splitmix64 finaliser (Steele, Lea, Flood 2014); identical on the GPU (odesat_hip.hip). */
static uint64_t oc_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

uint64_t oc_hash3(uint64_t seed, uint64_t replica, uint64_t var) {
    uint64_t h = oc_mix64(seed + 0x9E3779B97F4A7C15ULL);
    h = oc_mix64(h ^ (replica * 0xD1B54A32D192ED03ULL + 0x632BE59BD9B4E019ULL));
    h = oc_mix64(h ^ (var * 0x8CB92BA72F3D8DD7ULL + 0x9E3779B97F4A7C15ULL));
    return h;
}

double oc_init_voltage(uint64_t seed, uint64_t replica, uint64_t var) {
    /* rand 0.8 Standard f64: (x >> 11) * 2^-53, then main.rs:171 `* 2.0 - 1.0` */
    const double u = (double)(oc_hash3(seed, replica, var) >> 11) * (1.0 / 9007199254740992.0);
    return u * 2.0 - 1.0;
}

void oc_init_voltages(uint64_t seed, int64_t r0, int64_t B, int64_t n, double *v) {
    for (int64_t b = 0; b < B; ++b)
        for (int64_t i = 0; i < n; ++i)
            v[b * n + i] = oc_init_voltage(seed, (uint64_t)(r0 + b), (uint64_t)i);
}
