// mgic_core.hpp -- core types of the MI355X-native multigrid library.
//
// Box / ProblemDomain / DisjointBoxLayout / FArrayBox counterparts of the
// Chombo types the reference operator is written against
// (Source/VariableCoeffPoissonOperator.H:25-170), laid out for HBM:
//   * every field at a level shares one geometry: 1 ghost layer, rows padded
//     so the first valid cell of every row sits on a 128-byte line
//     (kRowAlign doubles), i fastest, fp64;
//   * a LevelData owns one allocation per local box and a device-side table
//     of valid-lo pointers, so batched kernels (exchange, BLAS-1) need no
//     host round trip and stay capturable in a hipGraph.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace mgic {

constexpr int kGhost = 4;     // ghost depth allocated: 1 for the stencils (CH_assert(ghostVect >=
                              // Unit), .cpp:279) + 1 for the fused sweep's halo (shell exchange)
                              // + 2 for the deep halo (two sweeps per 4-deep shell exchange)
constexpr int kRowAlign = 16; // doubles: 128-byte rows

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

enum ErrCode { kOk = 0, kBadArg = -1, kHipErr = -2, kRcclErr = -3, kState = -4 };

#define MGIC_HIP(x)                                                                   \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess)                                                             \
      throw ::mgic::Error(::mgic::kHipErr, std::string("HIP error ") +                \
                                               hipGetErrorString(e_) + " in " #x);    \
  } while (0)

#define MGIC_CHECK(cond, msg)                                                         \
  do {                                                                                \
    if (!(cond)) throw ::mgic::Error(::mgic::kBadArg, msg);                           \
  } while (0)

inline int floordiv(int i, int r) { return i >= 0 ? i / r : -((-i + r - 1) / r); }

// Cell-centred inclusive box (Chombo Box, cell-centred, IntVect lo/hi).
struct Box {
  int lo[3] = {0, 0, 0};
  int hi[3] = {-1, -1, -1};
  static Box make(const int *lohi) {
    Box b;
    for (int d = 0; d < 3; ++d) {
      b.lo[d] = lohi[d];
      b.hi[d] = lohi[3 + d];
    }
    return b;
  }
  bool empty() const { return hi[0] < lo[0] || hi[1] < lo[1] || hi[2] < lo[2]; }
  int size(int d) const { return hi[d] - lo[d] + 1; }
  long ncells() const { return empty() ? 0 : (long)size(0) * size(1) * size(2); }
  bool contains(const Box &o) const {
    for (int d = 0; d < 3; ++d)
      if (o.lo[d] < lo[d] || o.hi[d] > hi[d]) return false;
    return true;
  }
  Box intersect(const Box &o) const {
    Box r;
    for (int d = 0; d < 3; ++d) {
      r.lo[d] = lo[d] > o.lo[d] ? lo[d] : o.lo[d];
      r.hi[d] = hi[d] < o.hi[d] ? hi[d] : o.hi[d];
    }
    return r;
  }
  Box shifted(const int *s) const {
    Box r = *this;
    for (int d = 0; d < 3; ++d) {
      r.lo[d] += s[d];
      r.hi[d] += s[d];
    }
    return r;
  }
  Box coarsened(int r) const {
    Box c;
    for (int d = 0; d < 3; ++d) {
      c.lo[d] = floordiv(lo[d], r);
      c.hi[d] = floordiv(hi[d], r);
    }
    return c;
  }
  bool coarsenable(int r) const {
    for (int d = 0; d < 3; ++d)
      if (floordiv(lo[d], r) * r != lo[d] || floordiv(hi[d] + 1, r) * r != hi[d] + 1) return false;
    return true;
  }
  // adjCellBox(*this, dir, side, 1): the 1-deep slab just outside a face
  Box adj_cell(int dir, int side) const {
    Box r = *this;
    if (side == 0) r.lo[dir] = r.hi[dir] = lo[dir] - 1;
    else r.lo[dir] = r.hi[dir] = hi[dir] + 1;
    return r;
  }
  bool operator==(const Box &o) const {
    for (int d = 0; d < 3; ++d)
      if (lo[d] != o.lo[d] || hi[d] != o.hi[d]) return false;
    return true;
  }
};

// Memory geometry of one box's fab (all fields at a level share it).
struct FabGeom {
  Box valid;
  int nx = 0, ny = 0, nz = 0;
  long sy = 0, sz = 0;   // strides in doubles (sx = 1)
  long origin = 0;       // offset of valid-lo inside the allocation
  long total = 0;        // doubles in the allocation
  static FabGeom make(const Box &v) {
    FabGeom g;
    g.valid = v;
    g.nx = v.size(0);
    g.ny = v.size(1);
    g.nz = v.size(2);
    const long xoff = kRowAlign; // ghost at xoff-1
    g.sy = ((xoff + g.nx + kGhost + kRowAlign - 1) / kRowAlign) * kRowAlign;
    g.sz = g.sy * (g.ny + 2 * kGhost);
    g.origin = g.sz * kGhost + g.sy * kGhost + xoff;
    g.total = g.sz * (g.nz + 2 * kGhost) + kRowAlign;
    return g;
  }
  long offset(int i, int j, int k) const {  // global cell -> offset from valid-lo
    return (long)(i - valid.lo[0]) + (long)(j - valid.lo[1]) * sy + (long)(k - valid.lo[2]) * sz;
  }
};

// One rectangular copy between fabs and/or contiguous buffers.
// src/dst >= 0: local box index into a pointer table; -1: the buffer.
struct CopyItem {
  int src, dst;
  long soff, doff;
  long ssy, ssz, dsy, dsz;
  int nx, ny, nz, pad;
};

// Per-face boundary handling folded into the stencil kernels.
// Face order: (x lo, x hi, y lo, y hi, z lo, z hi).
enum BcMode : int {
  kBcMemory = 0,     // ghost holds exchanged data (internal / periodic face)
  kBcDirichlet = 1,  // ghost = c - near            (c = 2*value; DiriBC order 1)
  kBcNeumannHom = 2, // ghost = near
  kBcNeumann = 3,    // ghost = near + c            (c = isign*dx*value)
  // homogeneous QuadCFInterp ghost of an AMR level's coarse-fine face:
  // ((8/15)*0 + (2/3)*near) + (-0.2)*next (k_cf_interp<true>); the 3D-block
  // sweep kernel only (it refills these ghosts between its colour passes)
  kBcCFHom = 4
};

struct BoxArgs {
  int nx, ny, nz;
  int glo[3];
  long sy, sz;
  int bcm[6];
  double bcc[6];
};

struct StencilCoefs {
  double alpha, beta, dx;
  double dxinv;    // 1/(dx*dx)            (.ChF:89)
  double lamshift; // 2*3*beta/(dx*dx)     (.cpp:240)
  // bCoef is one value everywhere (set_b_coef writes 1, SetLevelData.cpp:
  // 330-340, and averaging keeps it): kernels use bval instead of loading
  // the field -- the same operand, so bit-identical, 8 B/cell less traffic
  int bconst = 0;
  double bval = 1.0;
  // every lambda of the level (1 / (alpha a + 6 beta / dx^2), .cpp:234-243)
  // lies in [2^-500, 2^500] in magnitude, one sign: the two-sweep kernel may
  // form 1 / x with the division's own instruction sequence minus its
  // scale / fix-up steps, which are identities there (the same bits);
  // rcp_fast32: the same for the fp32 sweeps (|lambda| in [2^-60, 2^60])
  int rcp_fast = 0;
  int rcp_fast32 = 0;
};

}  // namespace mgic
