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

// XCD-aware workgroup -> tile order: blocks are dealt round-robin over the
// 8 XCDs, so give each XCD a contiguous range of tiles (neighbouring tiles
// share halo lines in that XCD's L2)
__device__ __forceinline__ int xcd_tile(int bid, int nblocks) {
  const int q8 = nblocks / 8, r8 = nblocks % 8;
  const int xcd = bid % 8, i8 = bid / 8;
  return xcd * q8 + min(xcd, r8) + i8;
}

}  // namespace sweep
}  // namespace kern
}  // namespace mgic
