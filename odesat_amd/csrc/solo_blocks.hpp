// solo_blocks.hpp -- the term-block geometry shared by k_solo_fast / k_solo_cv (wave.hpp) and the host's
// bank model of k_solo_cv's layout search (cv_layout.cpp), so that the search optimises the blocks the
// kernel actually reads.
#pragma once

#include <cstddef>

#include <hip/hip_runtime.h>

// a variable's terms sit in a padded block of SOLO_DPAD slots (wave.hpp, k_solo_fast)
constexpr int SOLO_DPAD = 8;
// k_solo_cv: slots between consecutive blocks (SOLO_DPAD, then 16 bytes of the block's own)
__host__ __device__ constexpr int solo_cv_bs(size_t tsize) { return SOLO_DPAD + 16 / (int)tsize; }
// 16-byte reads per padded block
__host__ __device__ constexpr int solo_dpad_reads(size_t tsize) { return SOLO_DPAD / (16 / (int)tsize); }
