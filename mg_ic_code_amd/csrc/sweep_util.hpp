// sweep_util.hpp -- device helpers shared by the GSRB sweep kernels
// (smoother.hip, smoother_tb.hip).  Header-only, device code.
#pragma once

#include <hip/hip_runtime.h>

#include "mgic_core.hpp"

namespace mgic {
namespace kern {
namespace sweep {

// ParseBC's ghost value for a domain face (SetBCs.cpp:49-131 -> DiriBC /
// NeumBC order 1, BcMode in mgic_core.hpp): the image of the adjacent cell
template <class T>
__device__ __forceinline__ T ghost_of(int mode, T c, T near) {
  return mode == kBcDirichlet ? (c - near) : (mode == kBcNeumannHom ? near : near + c);
}

// q ? x : y as an integer bit select: a "cond ? arr1[i] : arr0[i]" on
// register arrays is otherwise turned into a select of two stack addresses
// and lowered to scratch memory.  Exact (no arithmetic on the values).
__device__ __forceinline__ double bsel(int q, double x, double y) {
  // per 32-bit half, so each half is one v_bitop3 / v_bfi
  const unsigned m = 0u - (unsigned)(q & 1);
  const unsigned long long xb = (unsigned long long)__double_as_longlong(x);
  const unsigned long long yb = (unsigned long long)__double_as_longlong(y);
  const unsigned lo = ((unsigned)xb & m) | ((unsigned)yb & ~m);
  const unsigned hi = ((unsigned)(xb >> 32) & m) | ((unsigned)(yb >> 32) & ~m);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ float bsel(int q, float x, float y) {
  const unsigned m = 0u - (unsigned)(q & 1);
  return __uint_as_float((__float_as_uint(x) & m) | (__float_as_uint(y) & ~m));
}

// Stores whose instruction count does not depend on the lane: raw buffer
// stores through a resource over `base`, where a lane that must not store
// passes kDrop as its byte offset (past the range: the hardware drops it).
// vmcnt counts loads and stores together in issue order, so with a static
// store count a later wait for loads issued BEFORE the stores is vmcnt(n
// stores) instead of vmcnt(0) -- which would also wait for the stores.
constexpr unsigned kDrop = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t store_rsrc(void *base) {
  return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
}
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
// CP: cache-policy bits (0 plain; 2 = nt; 16 = sc1)
template <int CP = 0>
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, double2 v, unsigned off) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, off, 0, CP);
}
template <int CP = 0>
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, double v, unsigned off) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, off, 0, CP);
}
template <int CP = 0>
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, float2 v, unsigned off) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, off, 0, CP);
}
template <int CP = 0>
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, float v, unsigned off) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, CP);
}

// XCD-aware workgroup -> tile order: blocks are dealt round-robin over the
// 8 XCDs, so give each XCD a contiguous range of tiles (neighbouring tiles
// share halo lines in that XCD's L2)
__device__ __forceinline__ int xcd_tile(int bid, int nblocks) {
  const int q8 = nblocks / 8, r8 = nblocks % 8;
  const int xcd = bid % 8, i8 = bid / 8;
  return xcd * q8 + min(xcd, r8) + i8;
}

// Round-major variant (w = workgroups resident per XCD): in each dispatch
// round the 8 XCDs take 8 consecutive runs of w tiles of the logical order,
// so the bands that border each other run at the same time on neighbouring
// XCDs -- the halo rows they share are read twice at nearly the same moment
// (the second read from the Infinity Cache) instead of one dispatch round
// apart (twice from HBM).  Blocks past the last whole round keep xcd_tile's
// contiguous ranges over what is left.
__device__ __forceinline__ int round_tile(int bid, int nblocks, int w) {
  const int full = w > 0 ? nblocks / (8 * w) * (8 * w) : 0;
  if (bid < full) {
    const int xcd = bid % 8, i8 = bid / 8;
    return (i8 / w) * (8 * w) + xcd * w + i8 % w;
  }
  return full + xcd_tile(bid - full, nblocks - full);
}

}  // namespace sweep
}  // namespace kern
}  // namespace mgic
