// Device helpers of the dataflow executor (dataflow.hip): control-word constants,
// DPP group sums, tagged granules and wave-uniform reductions.
#pragma once

#include <hip/hip_runtime.h>

#include "common.h"

namespace ana {

typedef __attribute__((address_space(1))) unsigned int gu32;
typedef int v4i __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

constexpr uint64_t kTimeoutTicks = 500000000ull;  // 5 s of the 100 MHz s_memrealtime clock
constexpr uint64_t kProgressTicks = 50000000ull;  // re-read the progress counter every 0.5 s
constexpr int kHeads = 8;                          // ticket shards
constexpr int kChunk = 64;                         // matches per ticket = one per lane
constexpr int kWavesPerBlock = 4;
// byte offset past every buffer the executor reads through a resource (the
// launcher checks the roster and the links stay below it): a load there returns 0
constexpr int kOutOfRange = 0x7fffffc0;

// sum over the G lanes of a group, result in every lane of the group.
// Power-of-two groups up to a DPP row (16 lanes): a butterfly of DPP lane moves
// (quad_perm xor 1, xor 2, row_half_mirror, row_mirror), one VALU op per step with
// no LDS round trip -- the previous bpermute butterfly put 15 dependent LDS
// trips into every rated batch.  After the two quad steps every lane of a quad
// holds the quad sum, so a mirror (lane i <-> 7-i, or 15-i) lands in the
// other half and completes the next level.  Wider power-of-two groups finish
// with xor shuffles; other sizes (G = 2K lanes, no idle lanes per match) use a
// bpermute tree to the group's first lane and a broadcast.
template <int Ctrl>
__device__ __forceinline__ float dpp_mov(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), Ctrl, 0xf, 0xf, true));
}
template <int G>
__device__ __forceinline__ float group_sum(float x, int j, int gbase) {
  if constexpr ((G & (G - 1)) == 0) {
    if constexpr (G >= 2) x += dpp_mov<0xb1>(x);   // quad_perm [1,0,3,2]
    if constexpr (G >= 4) x += dpp_mov<0x4e>(x);   // quad_perm [2,3,0,1]
    if constexpr (G >= 8) x += dpp_mov<0x141>(x);  // row_half_mirror
    if constexpr (G >= 16) x += dpp_mov<0x140>(x); // row_mirror
#pragma unroll
    for (int off = 16; off < G; off <<= 1) x += __shfl_xor(x, off);
    return x;
  } else {
#pragma unroll
    for (int off = 1; off < G; off <<= 1) {
      const float y = __shfl(x, (gbase + j + off) & 63);
      if (j + off < G && (j & (2 * off - 1)) == 0) x += y;
    }
    return __shfl(x, gbase);
  }
}

// {mu, tag A, sigma, tag B}: the tag words let a reader verify that the write it
// depends on has landed.  Shared granule: A = epoch | per-mode write counters << 8
// (6 x 4 bits), B = the match that reads it next.  Mode granule: A = epoch,
// B = that mode's write counter after this write (1..15, cyclic).
__device__ __forceinline__ v4i granule(float mu, uint32_t a, float sig, uint32_t b) {
  v4i v;
  v.x = __float_as_int(mu);
  v.y = (int)a;
  v.z = __float_as_int(sig);
  v.w = (int)b;
  return v;
}

// a value every lane holds identically, marked wave-uniform for the compiler
// (values built from shuffles are otherwise assumed divergent, which drags the
// chunk bookkeeping into vector registers)
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// OR over the 64 lanes, in every lane: DPP within rows of 16, then the 4 rows
__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xb1, 0xf, 0xf, true);   // quad_perm [1,0,3,2]
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4e, 0xf, 0xf, true);   // quad_perm [2,3,0,1]
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xf, 0xf, true);  // row_half_mirror
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xf, 0xf, true);  // row_mirror
  return (uint32_t)(__builtin_amdgcn_readlane((int)x, 0) | __builtin_amdgcn_readlane((int)x, 16) |
                    __builtin_amdgcn_readlane((int)x, 32) | __builtin_amdgcn_readlane((int)x, 48));
}

}  // namespace ana
