// kernels.hip -- gfx950 (CDNA4) kernels of the multigrid V-cycle hot path.
//
// Arithmetic restates Source/VariableCoeffPoissonOperatorF.ChF statement by
// statement (cited per kernel); the library is built with
// -ffp-contract=off so every result is bit-identical to the CPU oracle.
// These are HBM-streaming stencils (~0.3 flop/byte): no MFMA, 64-wide
// wavefronts along x so every wave touches whole 128-byte lines.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "kernels.hpp"

namespace mgic {
namespace kern {

namespace {

constexpr int TX = 64;  // one wavefront along x
constexpr int TY = 4;   // 4 waves per block

template <class T>
__device__ __forceinline__ T ghost_of(int mode, T c, T near) {
  // DiriBC order 1: 2*value - near (c = 2*value); NeumBC: near (+ isign*dx*value)
  return mode == kBcDirichlet ? (c - near) : (mode == kBcNeumannHom ? near : near + c);
}

// reduction operator: sums (KIND < 3) and maxima (KIND >= 3, also of |x|)
template <int KIND>
__device__ __forceinline__ double red_op(double a, double b) {
  if constexpr (KIND >= 3) return a > b ? a : b;
  else return a + b;
}

// element type traits for the fp32 (mixed-precision) variants: a lane pair
// is one 16-B (double) / 8-B (float) access; the stencil constants are
// rounded to T once (identity for double)
template <class T> struct Vec2;
template <> struct Vec2<double> { using type = double2; };
template <> struct Vec2<float> { using type = float2; };
template <class T> using V2 = typename Vec2<T>::type;
template <class T>
struct SC {
  T alpha, beta, dxinv, bval;
  __device__ explicit SC(const StencilCoefs &s)
      : alpha((T)s.alpha), beta((T)s.beta), dxinv((T)s.dxinv), bval((T)s.bval) {}
};

// 7-point Laplacian (.ChF:111-120) with the domain BC folded in: a ghost on
// a domain face is the BC image of the adjacent valid cell, which is the
// centre cell itself -- exactly what ParseBC would have written there
// before this pass (SetBCs.cpp:49-131).
__device__ __forceinline__ double lap7(const double *__restrict__ u, long idx, double c, int i,
                                       int j, int k, const BoxArgs &g) {
  double xm = u[idx - 1], xp = u[idx + 1];
  double ym = u[idx - g.sy], yp = u[idx + g.sy];
  double zm = u[idx - g.sz], zp = u[idx + g.sz];
  if (i == 0 && g.bcm[0]) xm = ghost_of(g.bcm[0], g.bcc[0], c);
  if (i == g.nx - 1 && g.bcm[1]) xp = ghost_of(g.bcm[1], g.bcc[1], c);
  if (j == 0 && g.bcm[2]) ym = ghost_of(g.bcm[2], g.bcc[2], c);
  if (j == g.ny - 1 && g.bcm[3]) yp = ghost_of(g.bcm[3], g.bcc[3], c);
  if (k == 0 && g.bcm[4]) zm = ghost_of(g.bcm[4], g.bcc[4], c);
  if (k == g.nz - 1 && g.bcm[5]) zp = ghost_of(g.bcm[5], g.bcc[5], c);
  const double tx = (xp + xm) - 2.0 * c;
  const double ty = (yp + ym) - 2.0 * c;
  const double tz = (zp + zm) - 2.0 * c;
  return (tx + ty) + tz;
}

template <bool LAM_MEM, bool BC>
__global__ __launch_bounds__(256) void k_gsrb(double *__restrict__ u,
                                              const double *__restrict__ rhs,
                                              const double *__restrict__ a,
                                              const double *__restrict__ b,
                                              const double *__restrict__ lam, const BoxArgs g,
                                              const StencilCoefs s, int colour) {
  const int p = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (j >= g.ny) return;
  // cells with (i+j+k) % 2 == redBlack in global indices (.ChF:98-106)
  const int i = 2 * p + ((g.glo[0] + g.glo[1] + j + g.glo[2] + k + colour) & 1);
  if (i >= g.nx) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  const double uc = u[idx];
  const double av = a[idx];
  double lofdpsi = s.alpha * av * uc;           // .ChF:107-108
  double ldpsi = lap7(u, idx, uc, i, j, k, g);  // .ChF:111-120
  ldpsi = ldpsi * s.dxinv * (BC ? s.bval : b[idx]);  // .ChF:122
  lofdpsi = lofdpsi - s.beta * ldpsi;           // .ChF:124
  double l;
  if (LAM_MEM) l = lam[idx];
  else l = 1.0 / (av * s.alpha + s.lamshift);   // .cpp:234-243
  u[idx] = uc - l * (lofdpsi - rhs[idx]);       // .ChF:127-128
}

template <bool BC>
__global__ __launch_bounds__(256) void k_apply_op(double *__restrict__ lu,
                                                  const double *__restrict__ u,
                                                  const double *__restrict__ a,
                                                  const double *__restrict__ b, const BoxArgs g,
                                                  const StencilCoefs s) {
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= g.nx || j >= g.ny) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  const double uc = u[idx];
  const double lof = s.alpha * a[idx] * uc;                     // .ChF:211-212
  double ldpsi = lap7(u, idx, uc, i, j, k, g);                   // .ChF:216-225
  ldpsi = ldpsi * s.dxinv * s.beta * (BC ? s.bval : b[idx]);     // .ChF:227
  lu[idx] = lof - ldpsi;                                         // .ChF:229
}

template <bool BC>
__global__ __launch_bounds__(256) void k_residual(double *__restrict__ r,
                                                  const double *__restrict__ u,
                                                  const double *__restrict__ rhs,
                                                  const double *__restrict__ a,
                                                  const double *__restrict__ b, const BoxArgs g,
                                                  const StencilCoefs s) {
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= g.nx || j >= g.ny) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  const double uc = u[idx];
  const double res = rhs[idx] - s.alpha * a[idx] * uc;           // .ChF:314-316
  double ldpsi = lap7(u, idx, uc, i, j, k, g);                   // .ChF:320-329
  ldpsi = ldpsi * s.dxinv * s.beta * (BC ? s.bval : b[idx]);     // .ChF:331
  r[idx] = res + ldpsi;                                          // .ChF:333
}

// z-streaming residual: a thread owns one (i, j) column of a z chunk and
// carries u(k-1), u(k) in registers; u(k+1) is the only new u load per cell
// (the x/y neighbours come from L1/L2, loaded as centres by the neighbours).
// Same expressions as k_residual.
template <bool BC, class RT>
__global__ __launch_bounds__(256) void k_residual_z(RT *__restrict__ r,
                                                    const double *__restrict__ u,
                                                    const double *__restrict__ rhs,
                                                    const double *__restrict__ a,
                                                    const double *__restrict__ b, const BoxArgs g,
                                                    const StencilCoefs s, int kc) {
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k0 = blockIdx.z * kc, k1 = min(k0 + kc, g.nz);
  if (i >= g.nx || j >= g.ny) return;
  const long col = (long)i + (long)j * g.sy;
  const bool fx0 = i == 0 && g.bcm[0], fx1 = i == g.nx - 1 && g.bcm[1];
  const bool fy0 = j == 0 && g.bcm[2], fy1 = j == g.ny - 1 && g.bcm[3];
  double um = u[col + (long)(k0 - 1) * g.sz];  // ghost plane -1 is allocated
  double uc = u[col + (long)k0 * g.sz];
  for (int k = k0; k < k1; ++k) {
    const long idx = col + (long)k * g.sz;
    const double up = u[idx + g.sz];  // plane nz (ghost) when k = nz - 1
    double xm = u[idx - 1], xp = u[idx + 1], ym = u[idx - g.sy], yp = u[idx + g.sy];
    double zm = um, zp = up;
    if (fx0) xm = ghost_of(g.bcm[0], g.bcc[0], uc);
    if (fx1) xp = ghost_of(g.bcm[1], g.bcc[1], uc);
    if (fy0) ym = ghost_of(g.bcm[2], g.bcc[2], uc);
    if (fy1) yp = ghost_of(g.bcm[3], g.bcc[3], uc);
    if (k == 0 && g.bcm[4]) zm = ghost_of(g.bcm[4], g.bcc[4], uc);
    if (k == g.nz - 1 && g.bcm[5]) zp = ghost_of(g.bcm[5], g.bcc[5], uc);
    const double res = rhs[idx] - s.alpha * a[idx] * uc;           // .ChF:314-316
    const double tx = (xp + xm) - 2.0 * uc;
    const double ty = (yp + ym) - 2.0 * uc;
    const double tz = (zp + zm) - 2.0 * uc;
    double ldpsi = (tx + ty) + tz;                                  // .ChF:320-329
    ldpsi = ldpsi * s.dxinv * s.beta * (BC ? s.bval : b[idx]);     // .ChF:331
    r[idx] = (RT)(res + ldpsi);  // .ChF:333 (RT = float: the fp64 residual rounded once)
    um = uc;
    uc = up;
  }
}

// One thread per coarse cell; the 8 fine children are visited in the
// Fortran k,j,i order so the accumulation res = 0 + t1 + ... + t8
// (.cpp:177 + .ChF:431-432) rounds exactly like the reference.  The two
// children of a fine row are one 16-B load per array (fine boxes start on
// even cells and the valid-lo is 128-B aligned); all loads are issued
// unconditionally (ghost addresses are always allocated) and the domain BC
// is folded afterwards, as in lap7.
template <class T>
__device__ __forceinline__ V2<T> ld2(const T *__restrict__ p) {
  return *reinterpret_cast<const V2<T> *>(p);
}

// k_residual_z on x-pairs: a thread owns columns (2i, 2i+1) of a z chunk, so
// u, rhs, a (and b) are one 16-B load per pair and the x neighbours inside
// the pair come from registers (xl, xr: the cells either side).  Rows are
// padded and the valid-lo 16-B aligned (FabGeom), so the pair's second cell
// is always allocated; at an odd nx the last pair writes its first cell
// only.  Same expressions, per cell, as k_residual.
// non-temporal forms (NT bit 0: rhs / aCoef / bCoef loads, read once per
// launch; bit 1: the residual stores): stream them past L2 so u's halo rows,
// which the neighbouring blocks re-read, stay resident.  Defaults
// MGIC_RESIDUAL_NT = 3, MGIC_RESTRICT_NT = 1 (512^3 residual 827 -> 789 us,
// V-cycle +0.9%, A/B over three rounds on one box)
template <class T> struct NTV2;
template <> struct NTV2<double> { typedef double type __attribute__((ext_vector_type(2))); };
template <> struct NTV2<float> { typedef float type __attribute__((ext_vector_type(2))); };
template <bool NT, class T>
__device__ __forceinline__ V2<T> ld2n(const T *__restrict__ p) {
  if constexpr (NT) {
    const typename NTV2<T>::type v =
        __builtin_nontemporal_load(reinterpret_cast<const typename NTV2<T>::type *>(p));
    V2<T> w;
    w.x = v.x;
    w.y = v.y;
    return w;
  } else {
    return *reinterpret_cast<const V2<T> *>(p);
  }
}
template <bool NT, class T>
__device__ __forceinline__ void st2n(T *__restrict__ p, const V2<T> &w) {
  if constexpr (NT) {
    typename NTV2<T>::type v;
    v.x = w.x;
    v.y = w.y;
    __builtin_nontemporal_store(v, reinterpret_cast<typename NTV2<T>::type *>(p));
  } else {
    *reinterpret_cast<V2<T> *>(p) = w;
  }
}

// NRM: also the block's max |r| over the cells it writes into
// partials[linear block id] (AMRMultiGrid's per-iteration max norm, normType
// 0, taken while r is in registers instead of a second pass over it; a max
// is exact, so it equals the separate norm bit for bit)
template <bool BC, class RT, int NT = 0, bool NRM = false>
__global__ __launch_bounds__(256) void k_residual_z2(RT *__restrict__ r,
                                                     const double *__restrict__ u,
                                                     const double *__restrict__ rhs,
                                                     const double *__restrict__ a,
                                                     const double *__restrict__ b, const BoxArgs g,
                                                     const StencilCoefs s, int kc,
                                                     double *__restrict__ partials = nullptr) {
  const int i = 2 * (blockIdx.x * TX + threadIdx.x);
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k0 = blockIdx.z * kc, k1 = min(k0 + kc, g.nz);
  double nmax = 0.0;  // the identity of max |x|
  if (i < g.nx && j < g.ny) {
    const long col = (long)i + (long)j * g.sy;
    const bool two = i + 1 < g.nx;
    const bool fx0 = i == 0 && g.bcm[0];
    const bool fx1a = i == g.nx - 1 && g.bcm[1], fx1b = i + 1 == g.nx - 1 && g.bcm[1];
    const bool fy0 = j == 0 && g.bcm[2], fy1 = j == g.ny - 1 && g.bcm[3];
    double2 um = ld2(u + col + (long)(k0 - 1) * g.sz);  // ghost plane -1 is allocated
    double2 uc = ld2(u + col + (long)k0 * g.sz);
    for (int k = k0; k < k1; ++k) {
      const long idx = col + (long)k * g.sz;
      const double2 up = ld2(u + idx + g.sz);  // plane nz (ghost) when k = nz - 1
      const double xl = u[idx - 1], xr = u[idx + 2];
      const double2 ym = ld2(u + idx - g.sy), yp = ld2(u + idx + g.sy);
      const double2 rv = ld2n<NT & 1>(rhs + idx), av = ld2n<NT & 1>(a + idx);
      const double2 bv = BC ? make_double2(s.bval, s.bval) : ld2n<NT & 1>(b + idx);
      auto cell = [&](double c, double xm, double xp, double ymv, double ypv, double zm, double zp,
                      double rr, double aa, double bb, bool bxm, bool bxp) {
        if (bxm) xm = ghost_of(g.bcm[0], g.bcc[0], c);
        if (bxp) xp = ghost_of(g.bcm[1], g.bcc[1], c);
        if (fy0) ymv = ghost_of(g.bcm[2], g.bcc[2], c);
        if (fy1) ypv = ghost_of(g.bcm[3], g.bcc[3], c);
        if (k == 0 && g.bcm[4]) zm = ghost_of(g.bcm[4], g.bcc[4], c);
        if (k == g.nz - 1 && g.bcm[5]) zp = ghost_of(g.bcm[5], g.bcc[5], c);
        const double res = rr - s.alpha * aa * c;            // .ChF:314-316
        const double tx = (xp + xm) - 2.0 * c;
        const double ty = (ypv + ymv) - 2.0 * c;
        const double tz = (zp + zm) - 2.0 * c;
        double ldpsi = (tx + ty) + tz;                       // .ChF:320-329
        ldpsi = ldpsi * s.dxinv * s.beta * bb;               // .ChF:331
        return (RT)(res + ldpsi);                            // .ChF:333
      };
      const RT r0 = cell(uc.x, xl, uc.y, ym.x, yp.x, um.x, up.x, rv.x, av.x, bv.x, fx0, fx1a);
      const RT r1 = cell(uc.y, uc.x, xr, ym.y, yp.y, um.y, up.y, rv.y, av.y, bv.y, false, fx1b);
      if (two) {
        V2<RT> w;
        w.x = r0;
        w.y = r1;
        st2n<(NT & 2) != 0>(r + idx, w);
      } else {
        r[idx] = r0;
      }
      if constexpr (NRM) {
        nmax = red_op<3>(nmax, fabs((double)r0));
        if (two) nmax = red_op<3>(nmax, fabs((double)r1));
      }
      um = uc;
      uc = up;
    }
  }
  if constexpr (NRM) {
    __shared__ double sm[TY];
    for (int o = 32; o > 0; o >>= 1) nmax = red_op<3>(nmax, __shfl_xor(nmax, o, 64));
    if (threadIdx.x == 0) sm[threadIdx.y] = nmax;
    __syncthreads();
    if (threadIdx.x == 0 && threadIdx.y == 0) {
      double m = sm[0];
      for (int w = 1; w < TY; ++w) m = red_op<3>(m, sm[w]);
      partials[blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)] = m;
    }
  }
}

// one coarse cell of restrictResidual
template <class T, bool BC, int NT>
__device__ __forceinline__ void restrict_cell(T *__restrict__ rc, const BoxArgs &cg,
                                              const T *__restrict__ u, const T *__restrict__ rhs,
                                              const T *__restrict__ a, const T *__restrict__ b,
                                              const BoxArgs &fg, const SC<T> &s, int accumulate,
                                              int ci, int cj, int ck) {
  const T denom = (T)(2 * 2 * 2);  // .ChF:402
  const long cidx = (long)ci + (long)cj * cg.sy + (long)ck * cg.sz;
  T sum = accumulate ? rc[cidx] : (T)0;
  const int i0 = 2 * ci;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = 2 * cj + jj, k = 2 * ck + kk;
      const long row = (long)i0 + (long)j * fg.sy + (long)k * fg.sz;
      const V2<T> c = ld2(u + row);
      const V2<T> ym = ld2(u + row - fg.sy), yp = ld2(u + row + fg.sy);
      const V2<T> zm = ld2(u + row - fg.sz), zp = ld2(u + row + fg.sz);
      const T xl = u[row - 1], xr = u[row + 2];
      const V2<T> rv = ld2n<NT & 1>(rhs + row), av = ld2n<NT & 1>(a + row);
      V2<T> bv;
      if (BC) bv.x = bv.y = s.bval;
      else bv = ld2n<NT & 1>(b + row);
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = i0 + ii;
        const T uc = ii ? c.y : c.x;
        T vxm = ii ? c.x : xl, vxp = ii ? xr : c.y;
        T vym = ii ? ym.y : ym.x, vyp = ii ? yp.y : yp.x;
        T vzm = ii ? zm.y : zm.x, vzp = ii ? zp.y : zp.x;
        if (i == 0 && fg.bcm[0]) vxm = ghost_of(fg.bcm[0], (T)fg.bcc[0], uc);
        if (i == fg.nx - 1 && fg.bcm[1]) vxp = ghost_of(fg.bcm[1], (T)fg.bcc[1], uc);
        if (j == 0 && fg.bcm[2]) vym = ghost_of(fg.bcm[2], (T)fg.bcc[2], uc);
        if (j == fg.ny - 1 && fg.bcm[3]) vyp = ghost_of(fg.bcm[3], (T)fg.bcc[3], uc);
        if (k == 0 && fg.bcm[4]) vzm = ghost_of(fg.bcm[4], (T)fg.bcc[4], uc);
        if (k == fg.nz - 1 && fg.bcm[5]) vzp = ghost_of(fg.bcm[5], (T)fg.bcc[5], uc);
        const T tx = (vxp + vxm) - (T)2 * uc;
        const T ty = (vyp + vym) - (T)2 * uc;
        const T tz = (vzp + vzm) - (T)2 * uc;
        T ldpsi = (tx + ty) + tz;                                  // .ChF:416-425
        T lofdpsi = s.alpha * (ii ? av.y : av.x) * uc;            // .ChF:411-412
        ldpsi = ldpsi * s.dxinv * s.beta * (ii ? bv.y : bv.x);         // .ChF:427
        lofdpsi = lofdpsi - ldpsi;                                      // .ChF:429
        sum = sum + ((ii ? rv.y : rv.x) - lofdpsi) / denom;             // .ChF:431-432
      }
    }
  rc[cidx] = sum;
}

// XCD-aware tile order for the LDS-staged streaming kernels: consecutive
// workgroup ids go round-robin to the 8 XCDs, so in the dispatch order a
// tile's x / y neighbours run on other XCDs and share none of their halo
// rows through an L2.  In bands of S tiles: every group of 8 S ids takes 8
// consecutive bands of the logical x-fastest order, one per XCD, so an XCD
// streams runs of S neighbouring tiles (its L2 shares their halo rows) while
// the 8 XCDs stay on neighbouring bands (the concurrent streams stay close
// in memory, as in the dispatch order); ids past the last whole group keep
// their place.  S = 0: the dispatch order.
__device__ __forceinline__ unsigned xcd_order(unsigned bid, unsigned nb, unsigned S) {
  if (S == 0) return bid;
  const unsigned G = 8 * S, full = nb / G * G;
  if (bid >= full) return bid;
  const unsigned g = bid / G, j = bid - g * G;
  return g * G + (j % 8) * S + j / 8;
}
// (x, y, z) tile of this workgroup: lg.w == 0, the 3D grid as launched;
// else a 1D grid of lg.x * lg.y * lg.z ids in bands of lg.w tiles
__device__ __forceinline__ uint3 tile_of(const uint4 lg) {
  if (lg.w == 0) return make_uint3(blockIdx.x, blockIdx.y, blockIdx.z);
  const unsigned L = xcd_order(blockIdx.x, gridDim.x, lg.w);
  return make_uint3(L % lg.x, (L / lg.x) % lg.y, L / (lg.x * lg.y));
}

// k_residual_z2 with the u planes staged in LDS: the workgroup's 128 x 4
// cells of a plane plus their one-cell halo (6 rows x 132 columns) go to a
// 4-slot LDS ring, each row loaded once with 16-B loads (the next plane
// prefetched into registers), one barrier per plane; rhs / aCoef / bCoef
// and r stream as in k_residual_z2.  Same grid, same cells per thread, same
// expressions, so the same bits and the same norm partials.
constexpr int kRlCols = 132, kRlRows = 6, kRlPairs = kRlRows * kRlCols / 2;  // 396
template <bool BC, class RT, int NT = 0, bool NRM = false>
__global__ __launch_bounds__(256) void k_residual_zl(RT *__restrict__ r,
                                                     const double *__restrict__ u,
                                                     const double *__restrict__ rhs,
                                                     const double *__restrict__ a,
                                                     const double *__restrict__ b, const BoxArgs g,
                                                     const StencilCoefs s, int kc,
                                                     double *__restrict__ partials = nullptr,
                                                     const uint4 lg = uint4{0, 0, 0, 0}) {
  __shared__ double Ls[4][kRlRows][kRlCols];
  const uint3 bt = tile_of(lg);
  const int tid = threadIdx.x + TX * threadIdx.y;
  const int x0 = 2 * (int)bt.x * TX, y0 = (int)bt.y * TY;
  const int i = x0 + 2 * threadIdx.x, j = y0 + threadIdx.y;
  const int k0 = (int)bt.z * kc, k1 = min(k0 + kc, g.nz);
  // pair q of the staged plane: row q / 66 (cell y0 - 1 + row), pair q % 66
  // (cells x0 - 2 + 2 m, +1); clamped into the allocated ghosts (a clamped
  // pair is never read)
  long poff[2];
  int pl[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int q = tid + 256 * h;
    const int rr = q / (kRlCols / 2), m = q - rr * (kRlCols / 2);
    int y = min(y0 - 1 + rr, g.ny + 1), x = min(x0 - 2 + 2 * m, g.nx & ~1);
    // a ghost of a DOMAIN face is staged but replaced by its image (cell):
    // pairs / rows wholly outside the box load an in-box one instead (no
    // ghost line from HBM; the same for the ghost planes in fetch)
    if (g.bcm[0] && x < 0) x = 0;
    if (g.bcm[1] && x >= g.nx) x = (g.nx - 2) & ~1;
    if (g.bcm[2] && y < 0) y = 0;
    if (g.bcm[3] && y >= g.ny) y = g.ny - 1;
    poff[h] = (long)x + (long)y * g.sy;
    pl[h] = q < kRlPairs ? rr * kRlCols + 2 * m : -1;
  }
  V2<double> pre[2];
  const int pzlo = g.bcm[4] ? 0 : -1, pzhi = g.bcm[5] ? g.nz - 1 : g.nz + 1;
  auto fetch = [&](int k) {
    const double *p = u + (long)min(max(k, pzlo), pzhi) * g.sz;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (pl[h] >= 0) pre[h] = ld2(p + poff[h]);
  };
  auto put = [&](int k) {
    double *dst = &Ls[k & 3][0][0];
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (pl[h] >= 0) *reinterpret_cast<V2<double> *>(dst + pl[h]) = pre[h];
  };
  fetch(k0 - 1);
  put(k0 - 1);
  fetch(k0);
  put(k0);
  fetch(k0 + 1);
  put(k0 + 1);
  fetch(k0 + 2);
  __syncthreads();
  double nmax = 0.0;  // the identity of max |x|
  const bool act = i < g.nx && j < g.ny;
  const long col = (long)i + (long)j * g.sy;
  const bool two = i + 1 < g.nx;
  const bool fx0 = i == 0 && g.bcm[0];
  const bool fx1a = i == g.nx - 1 && g.bcm[1], fx1b = i + 1 == g.nx - 1 && g.bcm[1];
  const bool fy0 = j == 0 && g.bcm[2], fy1 = j == g.ny - 1 && g.bcm[3];
  const int lr = threadIdx.y + 1, lc = 2 * threadIdx.x + 2;
  for (int k = k0; k < k1; ++k) {
    put(k + 2);  // (slot of plane k - 2, last read in the previous step)
    if (k + 3 < k1 + 2) fetch(k + 3);
    if (act) {
      const double *Lk = &Ls[k & 3][0][0], *Lm = &Ls[(k - 1) & 3][0][0], *Lp = &Ls[(k + 1) & 3][0][0];
      const long idx = col + (long)k * g.sz;
      const double2 uc = *reinterpret_cast<const double2 *>(Lk + lr * kRlCols + lc);
      const double2 um = *reinterpret_cast<const double2 *>(Lm + lr * kRlCols + lc);
      const double2 up = *reinterpret_cast<const double2 *>(Lp + lr * kRlCols + lc);
      const double xl = Lk[lr * kRlCols + lc - 1], xr = Lk[lr * kRlCols + lc + 2];
      const double2 ym = *reinterpret_cast<const double2 *>(Lk + (lr - 1) * kRlCols + lc);
      const double2 yp = *reinterpret_cast<const double2 *>(Lk + (lr + 1) * kRlCols + lc);
      const double2 rv = ld2n<NT & 1>(rhs + idx), av = ld2n<NT & 1>(a + idx);
      const double2 bv = BC ? make_double2(s.bval, s.bval) : ld2n<NT & 1>(b + idx);
      auto cell = [&](double c, double xm, double xp, double ymv, double ypv, double zm, double zp,
                      double rr, double aa, double bb, bool bxm, bool bxp) {
        if (bxm) xm = ghost_of(g.bcm[0], g.bcc[0], c);
        if (bxp) xp = ghost_of(g.bcm[1], g.bcc[1], c);
        if (fy0) ymv = ghost_of(g.bcm[2], g.bcc[2], c);
        if (fy1) ypv = ghost_of(g.bcm[3], g.bcc[3], c);
        if (k == 0 && g.bcm[4]) zm = ghost_of(g.bcm[4], g.bcc[4], c);
        if (k == g.nz - 1 && g.bcm[5]) zp = ghost_of(g.bcm[5], g.bcc[5], c);
        const double res = rr - s.alpha * aa * c;            // .ChF:314-316
        const double tx = (xp + xm) - 2.0 * c;
        const double ty = (ypv + ymv) - 2.0 * c;
        const double tz = (zp + zm) - 2.0 * c;
        double ldpsi = (tx + ty) + tz;                       // .ChF:320-329
        ldpsi = ldpsi * s.dxinv * s.beta * bb;               // .ChF:331
        return (RT)(res + ldpsi);                            // .ChF:333
      };
      const RT r0 = cell(uc.x, xl, uc.y, ym.x, yp.x, um.x, up.x, rv.x, av.x, bv.x, fx0, fx1a);
      const RT r1 = cell(uc.y, uc.x, xr, ym.y, yp.y, um.y, up.y, rv.y, av.y, bv.y, false, fx1b);
      if (two) {
        V2<RT> w;
        w.x = r0;
        w.y = r1;
        st2n<(NT & 2) != 0>(r + idx, w);
      } else {
        r[idx] = r0;
      }
      if constexpr (NRM) {
        nmax = red_op<3>(nmax, fabs((double)r0));
        if (two) nmax = red_op<3>(nmax, fabs((double)r1));
      }
    }
    __syncthreads();
  }
  if constexpr (NRM) {
    __shared__ double sm[TY];
    for (int o = 32; o > 0; o >>= 1) nmax = red_op<3>(nmax, __shfl_xor(nmax, o, 64));
    if (threadIdx.x == 0) sm[threadIdx.y] = nmax;
    __syncthreads();
    if (threadIdx.x == 0 && threadIdx.y == 0) {
      double m = sm[0];
      for (int w = 1; w < TY; ++w) m = red_op<3>(m, sm[w]);
      const unsigned gx = lg.w ? lg.x : gridDim.x, gy = lg.w ? lg.y : gridDim.y;
      partials[bt.x + gx * (bt.y + gy * bt.z)] = m;
    }
  }
}

template <class T, bool BC, int NT = 0>
__global__ __launch_bounds__(256) void k_restrict(T *__restrict__ rc, const BoxArgs cg,
                                                  const T *__restrict__ u,
                                                  const T *__restrict__ rhs,
                                                  const T *__restrict__ a,
                                                  const T *__restrict__ b, const BoxArgs fg,
                                                  const StencilCoefs s64, int accumulate) {
  const SC<T> s(s64);
  const int ci = blockIdx.x * TX + threadIdx.x;
  const int cj = blockIdx.y * TY + threadIdx.y;
  if (ci >= cg.nx || cj >= cg.ny) return;
  restrict_cell<T, BC, NT>(rc, cg, u, rhs, a, b, fg, s, accumulate, ci, cj, blockIdx.z);
}

// The restriction with the fine u planes staged in LDS (the default): a
// workgroup owns 64 x 4 coarse columns over a chunk of coarse planes; the
// four fine planes a coarse plane reads (2k-1 .. 2k+2) sit in a 4-slot LDS
// ring of 10 x 132 doubles (the tile's 8 fine rows and 128 fine columns with
// their halo), each loaded from global memory once with 16-B loads and the
// next two prefetched into registers while the current plane is summed.  rhs
// and aCoef stream from global memory as in k_restrict.  Per coarse cell the
// expressions and order of restrict_cell, so the same bits.  Loading every
// fine row once into LDS instead of five times per lane through the L1 (c,
// y -+ 1, z -+ 1) is what pays: k_restrict's L1 sent the L2 twice its
// compulsory bytes and stalled on pending requests two thirds of the time
// (profiles/r05q_stream_pmc.txt); short chunks (2 coarse planes) keep the
// grid large, longer ones re-read fewer halo planes but ran slower.
constexpr int kRzCols = 132, kRzRows = 10, kRzPairs = kRzRows * kRzCols / 2;  // 660
template <class T, bool BC, int NT, bool PRE = false>
__global__ __launch_bounds__(256) void k_restrict_zl(T *__restrict__ rc, const BoxArgs cg,
                                                     const T *__restrict__ u,
                                                     const T *__restrict__ rhs,
                                                     const T *__restrict__ a,
                                                     const T *__restrict__ b, const BoxArgs fg,
                                                     const StencilCoefs s64, int accumulate, int kc,
                                                     int ntx, int nty, int xcd = 0) {
  __shared__ T Ls[4][kRzRows][kRzCols];
  const SC<T> s(s64);
  const int ntile = ntx * nty;
  // xcd > 0: bands of xcd tiles in the x-fastest, chunk-slowest order; < 0:
  // bands of -xcd in the chunk-fastest order (a tile's z chunks together)
  const int bid = (int)xcd_order(blockIdx.x, gridDim.x, (unsigned)(xcd < 0 ? -xcd : xcd));
  const int nch = (int)gridDim.x / ntile;
  const int tile = xcd < 0 ? bid / nch : bid % ntile, chunk = xcd < 0 ? bid % nch : bid / ntile;
  const int cx0 = (tile % ntx) * TX, cy0 = (tile / ntx) * 4;
  const int k0 = chunk * kc, k1 = min(k0 + kc, cg.nz);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ci = cx0 + lane, cj = cy0 + w;
  const bool act = ci < cg.nx && cj < cg.ny;
  // the staged plane: fine rows 2 cy0 - 1 .. 2 cy0 + 8, columns 2 cx0 - 2 ..
  // 2 cx0 + 129, as 660 16-B pairs; pair q of lane tid + 256 i (clamped into
  // the allocated ghosts: what a clamped pair holds is never read)
  const int fx0 = 2 * cx0 - 2, fy0 = 2 * cy0 - 1;
  long poff[3];
  int pl[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int q = tid + 256 * i;
    const int r = q / (kRzCols / 2), m = q - r * (kRzCols / 2);
    int y = min(fy0 + r, fg.ny + 1), x = min(fx0 + 2 * m, fg.nx);
    // (domain-face ghosts are replaced by their images: no ghost line, as
    // in k_residual_zl)
    if (fg.bcm[0] && x < 0) x = 0;
    if (fg.bcm[1] && x >= fg.nx) x = (fg.nx - 2) & ~1;
    if (fg.bcm[2] && y < 0) y = 0;
    if (fg.bcm[3] && y >= fg.ny) y = fg.ny - 1;
    poff[i] = (long)x + (long)y * fg.sy;
    pl[i] = q < kRzPairs ? r * kRzCols + 2 * m : -1;
  }
  const int pzlo = fg.bcm[4] ? 0 : -1, pzhi = fg.bcm[5] ? fg.nz - 1 : fg.nz + 1;
  auto plane_ptr = [&](int k) { return u + (long)min(max(k, pzlo), pzhi) * fg.sz; };
  V2<T> pre[2][3];
  auto fetch = [&](int k, int h) {
    const T *p = plane_ptr(k);
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (pl[i] >= 0) pre[h][i] = ld2(p + poff[i]);
  };
  auto put = [&](int k, int h) {
    T *dst = &Ls[k & 3][0][0];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (pl[i] >= 0) *reinterpret_cast<V2<T> *>(dst + pl[i]) = pre[h][i];
  };
  fetch(2 * k0 - 1, 0);
  fetch(2 * k0, 1);
  put(2 * k0 - 1, 0);
  put(2 * k0, 1);
  fetch(2 * k0 + 1, 0);
  fetch(2 * k0 + 2, 1);
  put(2 * k0 + 1, 0);
  put(2 * k0 + 2, 1);
  __syncthreads();
  const T denom = (T)(2 * 2 * 2);  // .ChF:402
  // PRE (constant bCoef): the rhs / aCoef rows of coarse plane ck + 1 are
  // loaded while plane ck is summed (software pipelined: the waves keep a
  // plane's worth of loads in flight instead of waiting for each plane's)
  V2<T> crv[4], cav[4];
  auto cload = [&](int ck, V2<T>(&rv_)[4], V2<T>(&av_)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kk = q >> 1, jj = q & 1;
      const long row = (long)(2 * ci) + (long)(2 * cj + jj) * fg.sy + (long)(2 * ck + kk) * fg.sz;
      rv_[q] = ld2n<NT & 1>(rhs + row);
      av_[q] = ld2n<NT & 1>(a + row);
    }
  };
  if (PRE && act) cload(k0, crv, cav);
  for (int ck = k0; ck < k1; ++ck) {
    const bool more = ck + 1 < k1;
    if (more) {
      fetch(2 * ck + 3, 0);
      fetch(2 * ck + 4, 1);
    }
    V2<T> nrv[4], nav[4];
    if (PRE && act && more) cload(ck + 1, nrv, nav);
    if (act) {
      const long cidx = (long)ci + (long)cj * cg.sy + (long)ck * cg.sz;
      T sum = accumulate ? rc[cidx] : (T)0;
      const int i0 = 2 * ci;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int j = 2 * cj + jj, k = 2 * ck + kk;
          const int r = 2 * w + jj + 1, cx = 2 * lane + 2;
          const T *Lk = &Ls[k & 3][0][0], *Lm = &Ls[(k - 1) & 3][0][0],
                       *Lp = &Ls[(k + 1) & 3][0][0];
          const V2<T> c = *reinterpret_cast<const V2<T> *>(Lk + r * kRzCols + cx);
          const V2<T> ym = *reinterpret_cast<const V2<T> *>(Lk + (r - 1) * kRzCols + cx);
          const V2<T> yp = *reinterpret_cast<const V2<T> *>(Lk + (r + 1) * kRzCols + cx);
          const V2<T> zm = *reinterpret_cast<const V2<T> *>(Lm + r * kRzCols + cx);
          const V2<T> zp = *reinterpret_cast<const V2<T> *>(Lp + r * kRzCols + cx);
          const T xl = Lk[r * kRzCols + cx - 1], xr = Lk[r * kRzCols + cx + 2];
          const long row = (long)i0 + (long)j * fg.sy + (long)k * fg.sz;
          const V2<T> rv = PRE ? crv[kk * 2 + jj] : ld2n<NT & 1>(rhs + row);
          const V2<T> av = PRE ? cav[kk * 2 + jj] : ld2n<NT & 1>(a + row);
          V2<T> bv;
          if (BC) bv.x = bv.y = s.bval;
          else bv = ld2n<NT & 1>(b + row);
#pragma unroll
          for (int ii = 0; ii < 2; ++ii) {
            const int i = i0 + ii;
            const T uc = ii ? c.y : c.x;
            T vxm = ii ? c.x : xl, vxp = ii ? xr : c.y;
            T vym = ii ? ym.y : ym.x, vyp = ii ? yp.y : yp.x;
            T vzm = ii ? zm.y : zm.x, vzp = ii ? zp.y : zp.x;
            if (i == 0 && fg.bcm[0]) vxm = ghost_of(fg.bcm[0], (T)fg.bcc[0], uc);
            if (i == fg.nx - 1 && fg.bcm[1]) vxp = ghost_of(fg.bcm[1], (T)fg.bcc[1], uc);
            if (j == 0 && fg.bcm[2]) vym = ghost_of(fg.bcm[2], (T)fg.bcc[2], uc);
            if (j == fg.ny - 1 && fg.bcm[3]) vyp = ghost_of(fg.bcm[3], (T)fg.bcc[3], uc);
            if (k == 0 && fg.bcm[4]) vzm = ghost_of(fg.bcm[4], (T)fg.bcc[4], uc);
            if (k == fg.nz - 1 && fg.bcm[5]) vzp = ghost_of(fg.bcm[5], (T)fg.bcc[5], uc);
            const T tx = (vxp + vxm) - (T)2 * uc;
            const T ty = (vyp + vym) - (T)2 * uc;
            const T tz = (vzp + vzm) - (T)2 * uc;
            T ldpsi = (tx + ty) + tz;                                  // .ChF:416-425
            T lofdpsi = s.alpha * (ii ? av.y : av.x) * uc;            // .ChF:411-412
            ldpsi = ldpsi * s.dxinv * s.beta * (ii ? bv.y : bv.x);         // .ChF:427
            lofdpsi = lofdpsi - ldpsi;                                      // .ChF:429
            sum = sum + ((ii ? rv.y : rv.x) - lofdpsi) / denom;             // .ChF:431-432
          }
        }
      rc[cidx] = sum;
    }
    if (PRE && more) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        crv[q] = nrv[q];
        cav[q] = nav[q];
      }
    }
    if (more) {
      __syncthreads();  // every lane is done with planes 2ck-1, 2ck
      put(2 * ck + 3, 0);
      put(2 * ck + 4, 1);
      __syncthreads();
    }
  }
}

struct ProlongArgs {
  int avail_lo[3], avail_hi[3];
};

// One thread per coarse cell, updating its 2x2x2 fine children with two
// 16-B read-modify-writes per fine row.  Linear (type 1): per direction the
// slope is taken on the child's side when that coarse neighbour exists
// (interior, or an exchanged ghost across a box / periodic face), else on the
// other side; e = c0 + dx-term + dy-term + dz-term in that order.  The six
// neighbour loads are unconditional (coarse ghosts are always allocated).
template <class T, int TYPE>
__global__ __launch_bounds__(256) void k_prolong(T *__restrict__ uf, const BoxArgs fg,
                                                 const T *__restrict__ ec, const BoxArgs cg,
                                                 const ProlongArgs pa) {
  const int ci = blockIdx.x * TX + threadIdx.x;
  const int cj = blockIdx.y * TY + threadIdx.y;
  const int ck = blockIdx.z;
  if (ci >= cg.nx || cj >= cg.ny) return;
  const long cidx = (long)ci + (long)cj * cg.sy + (long)ck * cg.sz;
  const T c0 = ec[cidx];
  T dlo[3] = {(T)0, (T)0, (T)0}, dhi[3] = {(T)0, (T)0, (T)0};  // slope for lower / upper child
  bool ok[3] = {false, false, false};
  if (TYPE == 1) {
    const long cs[3] = {1, cg.sy, cg.sz};
    const int ic[3] = {ci, cj, ck};
    const int cn[3] = {cg.nx, cg.ny, cg.nz};
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const T lo = ec[cidx - cs[d]], hi = ec[cidx + cs[d]];
      const bool has_lo = (ic[d] > 0) || pa.avail_lo[d];
      const bool has_hi = (ic[d] < cn[d] - 1) || pa.avail_hi[d];
      ok[d] = has_lo || has_hi;
      const T sl_hi = hi - c0, sl_lo = c0 - lo;
      dhi[d] = (has_hi ? sl_hi : sl_lo) * (T)0.25;    // upper child: +0.25 * slope
      dlo[d] = (!has_lo ? sl_hi : sl_lo) * (T)-0.25;  // lower child: -0.25 * slope
    }
  }
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const long row = (long)(2 * ci) + (long)(2 * cj + jj) * fg.sy + (long)(2 * ck + kk) * fg.sz;
      V2<T> v = ld2(uf + row);
      T e0 = c0, e1 = c0;
      if (TYPE == 1) {
        if (ok[0]) {
          e0 = e0 + dlo[0];
          e1 = e1 + dhi[0];
        }
        if (ok[1]) {
          const T t = jj ? dhi[1] : dlo[1];
          e0 = e0 + t;
          e1 = e1 + t;
        }
        if (ok[2]) {
          const T t = kk ? dhi[2] : dlo[2];
          e0 = e0 + t;
          e1 = e1 + t;
        }
      }
      v.x = v.x + e0;
      v.y = v.y + e1;
      *reinterpret_cast<V2<T> *>(uf + row) = v;
    }
}

__global__ __launch_bounds__(256) void k_lambda(double *__restrict__ lam,
                                                const double *__restrict__ a, const BoxArgs g,
                                                const StencilCoefs s) {
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= g.nx || j >= g.ny) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  double v = a[idx];   // copy   (.cpp:234)
  v = v * s.alpha;     // mult   (.cpp:235)
  v = v + s.lamshift;  // plus   (.cpp:240)
  lam[idx] = 1.0 / v;  // invert (.cpp:243)
}

// [Chombo] AverageF.ChF AVERAGE / AVERAGEHARMONIC: the ratio^3 children of a
// coarse cell summed in the k,j,i order of the refinement box, times
// refScale = 1/ratio^3 (harmonic: reciprocals summed, result inverted).
__global__ __launch_bounds__(256) void k_average(double *__restrict__ c, const BoxArgs cg,
                                                 const double *__restrict__ f, const BoxArgs fg,
                                                 int ratio, int harmonic) {
  const int I = blockIdx.x * TX + threadIdx.x;
  const int J = blockIdx.y * TY + threadIdx.y;
  const int K = blockIdx.z;
  if (I >= cg.nx || J >= cg.ny) return;
  const double refScale = 1.0 / (ratio * ratio * ratio);
  double sum = 0.0;
  for (int kk = 0; kk < ratio; ++kk)
    for (int jj = 0; jj < ratio; ++jj)
      for (int ii = 0; ii < ratio; ++ii) {
        const double v = f[(long)(ratio * I + ii) + (long)(ratio * J + jj) * fg.sy +
                           (long)(ratio * K + kk) * fg.sz];
        sum = sum + (harmonic ? 1.0 / v : v);
      }
  c[(long)I + (long)J * cg.sy + (long)K * cg.sz] =
      harmonic ? 1.0 / (sum * refScale) : sum * refScale;
}

__global__ void k_fill_bc_face(double *__restrict__ u, const BoxArgs g, int face) {
  const int dir = face >> 1, side = face & 1;
  const int n[3] = {g.nx, g.ny, g.nz};
  const int d1 = dir == 0 ? 1 : 0, d2 = dir == 2 ? 1 : 2;
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  const int bb = blockIdx.y;
  if (a >= n[d1] || bb >= n[d2]) return;
  int c[3];
  c[dir] = side == 0 ? 0 : n[dir] - 1;
  c[d1] = a;
  c[d2] = bb;
  const long s[3] = {1, g.sy, g.sz};
  const long near = (long)c[0] + (long)c[1] * g.sy + (long)c[2] * g.sz;
  const long gh = near + (side == 0 ? -s[dir] : s[dir]);
  u[gh] = ghost_of(g.bcm[face], g.bcc[face], u[near]);
}

// BLAS-1 kinds are template parameters: every launch compiles to one
// straight-line body (no runtime switch inside the cell loop).
template <int KIND>
__global__ __launch_bounds__(256) void k_blas(double *__restrict__ x, const double *__restrict__ y,
                                              const double *__restrict__ z, double s, double t,
                                              const BoxArgs g) {
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= g.nx || j >= g.ny) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  if constexpr (KIND == 0) x[idx] = y[idx];                    // assign / copy
  else if constexpr (KIND == 1) x[idx] = x[idx] + s * y[idx];  // incr (FArrayBox::plus(src, scale))
  else if constexpr (KIND == 2) x[idx] = x[idx] * s;           // scale (FArrayBox::mult(scale))
  else if constexpr (KIND == 3) x[idx] = x[idx] * y[idx];      // mult (FArrayBox::mult(src))
  else if constexpr (KIND == 4) x[idx] = s * y[idx] + t * z[idx];  // axby
  else if constexpr (KIND == 6) x[idx] = y[idx] * z[idx];      // copy y, then mult by z (one pass)
  else x[idx] = s;                                             // setVal
}

constexpr int RB = 256;

// identity of the reduction: 0 for sums and max|x|, -inf for max x / max -x
template <int KIND>
__device__ __forceinline__ double red_init() {
  if constexpr (KIND >= 4) return -__builtin_huge_val();
  else return 0.0;
}

template <int KIND>
__device__ __forceinline__ double red_term(const double *__restrict__ x,
                                           const double *__restrict__ y, long idx) {
  const double v = x[idx];
  if constexpr (KIND == 0) return v * y[idx];
  else if constexpr (KIND == 2) return v * v;
  else if constexpr (KIND == 4) return v;
  else if constexpr (KIND == 5) return -v;
  else return fabs(v);
}

// one wave per (j, k) row, lanes along i (coalesced 512-B rows, four
// independent accumulators per lane), block partials through LDS.  Rows are
// dealt round-robin to the waves of the grid; no per-element index division.
template <int KIND>
__global__ __launch_bounds__(RB) void k_reduce_partial(const double *__restrict__ x,
                                                       const double *__restrict__ y,
                                                       const BoxArgs g,
                                                       double *__restrict__ partials) {
  __shared__ double sm[RB];
  constexpr int W = RB / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nrows = g.ny * g.nz;
  double a0 = red_init<KIND>(), a1 = a0, a2 = a0, a3 = a0;
  for (int r = blockIdx.x * W + wave; r < nrows; r += gridDim.x * W) {
    const int k = r / g.ny, j = r - k * g.ny;
    const long base = (long)j * g.sy + (long)k * g.sz;
    int i = lane;
    for (; i + 192 < g.nx; i += 256) {
      a0 = red_op<KIND>(a0, red_term<KIND>(x, y, base + i));
      a1 = red_op<KIND>(a1, red_term<KIND>(x, y, base + i + 64));
      a2 = red_op<KIND>(a2, red_term<KIND>(x, y, base + i + 128));
      a3 = red_op<KIND>(a3, red_term<KIND>(x, y, base + i + 192));
    }
    for (; i < g.nx; i += 64) a0 = red_op<KIND>(a0, red_term<KIND>(x, y, base + i));
  }
  sm[threadIdx.x] = red_op<KIND>(red_op<KIND>(a0, a1), red_op<KIND>(a2, a3));
  __syncthreads();
  for (int w = RB / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) sm[threadIdx.x] = red_op<KIND>(sm[threadIdx.x], sm[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) partials[blockIdx.x] = sm[0];
}

// ---- BiCGStab's vector updates fused with the reductions that follow them
// (BiCGStabSolver, restated in op.cpp).  Each element is computed with the
// same expressions as the separate assign / scale / incr passes (bit-identical
// results), and the partial sums use k_reduce_partial's row-to-wave deal and
// accumulators, so a fused norm equals the separate one bit for bit.
// s = r + ca*v; e = e + cb*pt; partials of the norm kind KIND of s
template <int KIND>
__global__ __launch_bounds__(RB) void k_axpy2_reduce(double *__restrict__ s,
                                                     const double *__restrict__ r,
                                                     const double *__restrict__ v, double ca,
                                                     double *__restrict__ e,
                                                     const double *__restrict__ pt, double cb,
                                                     const BoxArgs g,
                                                     double *__restrict__ partials) {
  __shared__ double sm[RB];
  constexpr int W = RB / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nrows = g.ny * g.nz;
  double acc[4] = {red_init<KIND>(), red_init<KIND>(), red_init<KIND>(), red_init<KIND>()};
  auto one = [&](long idx, int q) {
    const double sv = r[idx] + ca * v[idx];  // S = R; S += ca V
    s[idx] = sv;
    e[idx] = e[idx] + cb * pt[idx];          // E += cb PT
    acc[q] = red_op<KIND>(acc[q], red_term<KIND>(s, nullptr, idx));
  };
  for (int row = blockIdx.x * W + wave; row < nrows; row += gridDim.x * W) {
    const int k = row / g.ny, j = row - k * g.ny;
    const long base = (long)j * g.sy + (long)k * g.sz;
    int i = lane;
    for (; i + 192 < g.nx; i += 256) {
      one(base + i, 0);
      one(base + i + 64, 1);
      one(base + i + 128, 2);
      one(base + i + 192, 3);
    }
    for (; i < g.nx; i += 64) one(base + i, 0);
  }
  sm[threadIdx.x] = red_op<KIND>(red_op<KIND>(acc[0], acc[1]), red_op<KIND>(acc[2], acc[3]));
  __syncthreads();
  for (int w = RB / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) sm[threadIdx.x] = red_op<KIND>(sm[threadIdx.x], sm[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) partials[blockIdx.x] = sm[0];
}

// the partials of dot(t, s) and dot(t, t) in one pass
__global__ __launch_bounds__(RB) void k_dot2(const double *__restrict__ t,
                                             const double *__restrict__ s, const BoxArgs g,
                                             double *__restrict__ pts, double *__restrict__ ptt) {
  __shared__ double sm[2][RB];
  constexpr int W = RB / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nrows = g.ny * g.nz;
  double a[4] = {0.0, 0.0, 0.0, 0.0}, b[4] = {0.0, 0.0, 0.0, 0.0};
  auto one = [&](long idx, int q) {
    const double tv = t[idx];
    a[q] = a[q] + tv * s[idx];
    b[q] = b[q] + tv * tv;
  };
  for (int row = blockIdx.x * W + wave; row < nrows; row += gridDim.x * W) {
    const int k = row / g.ny, j = row - k * g.ny;
    const long base = (long)j * g.sy + (long)k * g.sz;
    int i = lane;
    for (; i + 192 < g.nx; i += 256) {
      one(base + i, 0);
      one(base + i + 64, 1);
      one(base + i + 128, 2);
      one(base + i + 192, 3);
    }
    for (; i < g.nx; i += 64) one(base + i, 0);
  }
  sm[0][threadIdx.x] = (a[0] + a[1]) + (a[2] + a[3]);
  sm[1][threadIdx.x] = (b[0] + b[1]) + (b[2] + b[3]);
  __syncthreads();
  for (int w = RB / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      sm[0][threadIdx.x] = sm[0][threadIdx.x] + sm[0][threadIdx.x + w];
      sm[1][threadIdx.x] = sm[1][threadIdx.x] + sm[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    pts[blockIdx.x] = sm[0][0];
    ptt[blockIdx.x] = sm[1][0];
  }
}

// p = ((p * beta) + c * v) + 1.0 * r  (scale(P, beta); incr(P, V, c); incr(P, R, 1))
__global__ __launch_bounds__(256) void k_bicg_p(double *__restrict__ p,
                                                const double *__restrict__ v,
                                                const double *__restrict__ r, double beta,
                                                double c, const BoxArgs g) {
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= g.nx || j >= g.ny) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  double t = p[idx] * beta;
  t = t + c * v[idx];
  p[idx] = t + 1.0 * r[idx];
}

template <int KIND>
__global__ __launch_bounds__(RB) void k_reduce_final(const double *__restrict__ p, int n,
                                                     double *__restrict__ out, const HostPub pub) {
  __shared__ double sm[RB];
  double acc = red_init<KIND>();
  for (int t = threadIdx.x; t < n; t += RB) acc = red_op<KIND>(acc, p[t]);
  sm[threadIdx.x] = acc;
  __syncthreads();
  for (int w = RB / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) sm[threadIdx.x] = red_op<KIND>(sm[threadIdx.x], sm[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = sm[0];
    publish(pub, sm[0]);
  }
}

// max-type kinds (3, 4, 5): any order gives the same result, so a wide
// block with four independent loads in flight per thread (the single 256-
// thread loop above is latency bound: 16 K residual partials took 25 us)
template <int KIND>
__global__ __launch_bounds__(1024) void k_reduce_final_wide(const double *__restrict__ p, int n,
                                                           double *__restrict__ out,
                                                           const HostPub pub) {
  static_assert(KIND >= 3, "order-independent reductions only");
  __shared__ double sm[16];
  double a0 = red_init<KIND>(), a1 = a0, a2 = a0, a3 = a0;
  int t = threadIdx.x;
  for (; t + 3 * 1024 < n; t += 4 * 1024) {
    a0 = red_op<KIND>(a0, p[t]);
    a1 = red_op<KIND>(a1, p[t + 1024]);
    a2 = red_op<KIND>(a2, p[t + 2048]);
    a3 = red_op<KIND>(a3, p[t + 3072]);
  }
  for (; t < n; t += 1024) a0 = red_op<KIND>(a0, p[t]);
  double acc = red_op<KIND>(red_op<KIND>(a0, a1), red_op<KIND>(a2, a3));
  for (int o = 32; o > 0; o >>= 1) acc = red_op<KIND>(acc, __shfl_xor(acc, o, 64));
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = sm[0];
    for (int w = 1; w < 16; ++w) m = red_op<KIND>(m, sm[w]);
    out[0] = m;
    publish(pub, m);
  }
}

__global__ void k_publish(const double *__restrict__ v, const HostPub pub) {
  if (threadIdx.x == 0) publish(pub, *v);
}

template <class T>
__global__ __launch_bounds__(256) void k_copy_items(const CopyItem *__restrict__ items,
                                                    T *const *__restrict__ src_tab,
                                                    const T *__restrict__ src_buf,
                                                    T *const *__restrict__ dst_tab,
                                                    T *__restrict__ dst_buf) {
  const CopyItem it = items[blockIdx.y];
  const T *src = (it.src >= 0 ? src_tab[it.src] : src_buf) + it.soff;
  T *dst = (it.dst >= 0 ? dst_tab[it.dst] : dst_buf) + it.doff;
  // pairs when every row of the item starts 2-element aligned on both sides
  // (x slabs of the ghost shell are 2 wide at even offsets: one 16-B access
  // per row instead of two strided 8-B ones); 32-bit index math (an item is
  // a face slab, far below 2^31 elements)
  const bool pairs = ((it.nx | it.soff | it.doff | it.ssy | it.ssz | it.dsy | it.dsz) & 1) == 0 &&
                     ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) &
                      (2 * sizeof(T) - 1)) == 0;
  const unsigned w = pairs ? (unsigned)it.nx / 2 : (unsigned)it.nx;
  const unsigned n = w * (unsigned)it.ny * (unsigned)it.nz, ny = (unsigned)it.ny;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
    const unsigned r = t / w, i = t - r * w;
    const unsigned k = r / ny, j = r - k * ny;
    const long so = (long)j * it.ssy + (long)k * it.ssz, d = (long)j * it.dsy + (long)k * it.dsz;
    if (pairs) {
      using V = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
      reinterpret_cast<V *>(dst + d)[i] = reinterpret_cast<const V *>(src + so)[i];
    } else {
      dst[d + i] = src[so + i];
    }
  }
}

// ---- input generator: SetLevelData.cpp / SetBinaryBH.H / MyPhiFunction.H
__device__ double bh_phi(const BhParams &p, double x, double y, double z) {
  const double r2 = x * x + y * y + z * z;  // MyPhiFunction.H:15
  return p.phi_amplitude * exp(-r2 / p.phi_wavelength);
}
__device__ double bh_loc(int iv, double dx, double domlen) { return ((double)iv + 0.5) * dx - domlen / 2.0; }
__device__ double bh_Aij(int i, int j, double r1, double r2, const double *n1, const double *n2,
                         const double *J1, const double *J2, const double *P1, const double *P2) {
  // SetBinaryBH.H:24-53
  auto eps = [](int a, int b, int c) -> double {
    if (a == 0 && b == 1 && c == 2) return 1.0;
    if (a == 1 && b == 2 && c == 0) return 1.0;
    if (a == 2 && b == 0 && c == 1) return 1.0;
    if (a == 0 && b == 2 && c == 1) return -1.0;
    if (a == 2 && b == 1 && c == 0) return -1.0;
    if (a == 1 && b == 0 && c == 2) return -1.0;
    return 0.0;
  };
  double Aij = 1.5 / r1 / r1 * (n1[i] * P1[j] + n1[j] * P1[i]) +
               1.5 / r2 / r2 * (n2[i] * P2[j] + n2[j] * P2[i]);
  for (int k = 0; k < 3; k++) {
    Aij += 1.5 / r1 / r1 * (n1[i] * n1[j] - (double)(i == j)) * P1[k] * n1[k] +
           1.5 / r2 / r2 * (n2[i] * n2[j] - (double)(i == j)) * P2[k] * n2[k];
    for (int l = 0; l < 3; l++) {
      Aij += -3.0 / r1 / r1 / r1 * (eps(i, l, k) * n1[j] + eps(j, l, k) * n1[i]) * n1[l] * J1[k] -
             3.0 / r2 / r2 / r2 * (eps(i, l, k) * n2[j] + eps(j, l, k) * n2[i]) * n2[l] * J2[k];
    }
  }
  return Aij;
}

// set_a_coef + set_rhs (SetLevelData.cpp:73-127, :281-325); psi == nullptr:
// psi = 1 everywhere (NL iteration 0), else psi read with its ghost layer
// INTEGRAND: set_constant_K_integrand (SetLevelData.cpp:131-180) into acoef
// instead (m taken at K = 0, rhs untouched)
template <bool INTEGRAND>
__global__ __launch_bounds__(256) void k_binary_bh(double *__restrict__ acoef,
                                                   double *__restrict__ rhs,
                                                   const double *__restrict__ psi,
                                                   const BoxArgs g, double dx, const BhParams p) {
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= g.nx || j >= g.ny) return;
  const int iv[3] = {g.glo[0] + i, g.glo[1] + j, g.glo[2] + k};
  double loc[3];
  for (int d = 0; d < 3; ++d) loc[d] = bh_loc(iv[d], dx, p.domlen[d]);
  double rho_grad = 0.0;  // GETRHOGRADPHIF, SetLevelDataF.ChF:65-103
  for (int d0 = 0; d0 < 3; ++d0) {
    double lp[3], lm[3];
    for (int d = 0; d < 3; ++d) {
      lp[d] = bh_loc(iv[d] + (d == d0), dx, p.domlen[d]);
      lm[d] = bh_loc(iv[d] - (d == d0), dx, p.domlen[d]);
    }
    const double dphidx = 0.5 / dx * (+bh_phi(p, lp[0], lp[1], lp[2]) - bh_phi(p, lm[0], lm[1], lm[2]));
    rho_grad = rho_grad + 0.5 * dphidx * dphidx;
  }
  double l1[3] = {loc[0] - p.off1, loc[1], loc[2]}, l2[3] = {loc[0] - p.off2, loc[1], loc[2]};
  const double r1 = sqrt(l1[0] * l1[0] + l1[1] * l1[1] + l1[2] * l1[2]);
  const double r2 = sqrt(l2[0] * l2[0] + l2[1] * l2[1] + l2[2] * l2[2]);
  const double n1[3] = {l1[0] / r1, l1[1] / r1, l1[2] / r1};
  const double n2[3] = {l2[0] / r2, l2[1] / r2, l2[2] / r2};
  const double J1[3] = {0.0, 0.0, p.spin1}, J2[3] = {0.0, 0.0, p.spin2};
  const double P1[3] = {0.0, p.mom1, 0.0}, P2[3] = {0.0, p.mom2, 0.0};
  const double A11 = bh_Aij(0, 0, r1, r2, n1, n2, J1, J2, P1, P2);
  const double A22 = bh_Aij(1, 1, r1, r2, n1, n2, J1, J2, P1, P2);
  const double A33 = bh_Aij(2, 2, r1, r2, n1, n2, J1, J2, P1, P2);
  const double A12 = bh_Aij(0, 1, r1, r2, n1, n2, J1, J2, P1, P2);
  const double A13 = bh_Aij(0, 2, r1, r2, n1, n2, J1, J2, P1, P2);
  const double A23 = bh_Aij(1, 2, r1, r2, n1, n2, J1, J2, P1, P2);
  const double A2 = pow(A11, 2.0) + pow(A22, 2.0) + pow(A33, 2.0) + 2 * pow(A12, 2.0) +
                    2 * pow(A13, 2.0) + 2 * pow(A23, 2.0);  // SetLevelData.cpp:312-317
  const double rho = 0.5 * 0.0 * 0.0 + 0.0;
  const double K = INTEGRAND ? 0.0 : p.constant_K;  // set_m_value(.., 0.0) for the integrand
  const double m = (2.0 / 3.0) * (K * K) - 16.0 * M_PI * p.G_Newton * rho;
  const double psi_bh = p.m1 / r1 + p.m2 / r2;  // SetBinaryBH.H:85-99
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  const double psi_c = psi ? psi[idx] : 1.0;
  const double psi_0 = psi_c + psi_bh;  // SetLevelData.cpp:319-320
  double lap = 0.0;  // GETLAPLACIANPSIF, SetLevelDataF.ChF:15-58 (2nd order)
  const long st[3] = {1, g.sy, g.sz};
  for (int d0 = 0; d0 < 3; ++d0) {
    const double pm = psi ? psi[idx - st[d0]] : 1.0, pp = psi ? psi[idx + st[d0]] : 1.0;
    lap = lap + 1.0 / dx / dx * (+1.0 * pm - 2.0 * psi_c + 1.0 * pp);
  }
  if (INTEGRAND) {  // SetLevelData.cpp:174-177
    acoef[idx] = -1.5 * m + 1.5 * A2 * pow(psi_0, -12.0) +
                 24.0 * M_PI * p.G_Newton * rho_grad * pow(psi_0, -4.0) +
                 12.0 * lap * pow(psi_0, -5.0);
    return;
  }
  acoef[idx] = -0.625 * m * pow(psi_0, 4.0) - A2 * pow(psi_0, -8.0) +
               2.0 * M_PI * p.G_Newton * rho_grad;  // SetLevelData.cpp:321-322
  rhs[idx] = 0.125 * m * pow(psi_0, 5.0) - 0.125 * A2 * pow(psi_0, -7.0) -
             2.0 * M_PI * p.G_Newton * rho_grad * psi_0 - lap;  // SetLevelData.cpp:121-124
}

// GETLAPLACIANPSIF (SetLevelDataF.ChF:15-58), 2nd-order branch, and
// GETRHOGRADPHIF (:65-103): undivided-difference loops over `box` with the
// operand's ghost layer read as is (no BC)
__global__ __launch_bounds__(256) void k_lap_psi(double *__restrict__ l,
                                                 const double *__restrict__ psi, const BoxArgs g,
                                                 double dx) {
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= g.nx || j >= g.ny) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  const long st[3] = {1, g.sy, g.sz};
  double acc = 0.0;
  for (int d0 = 0; d0 < 3; ++d0) {
    const double d2 = 1.0 / dx / dx * (+1.0 * psi[idx - st[d0]] - 2.0 * psi[idx] +
                                       1.0 * psi[idx + st[d0]]);
    acc = acc + d2;
  }
  l[idx] = acc;
}

__global__ __launch_bounds__(256) void k_rho_grad_phi(double *__restrict__ r,
                                                      const double *__restrict__ phi,
                                                      const BoxArgs g, double dx) {
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= g.nx || j >= g.ny) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  const long st[3] = {1, g.sy, g.sz};
  double acc = 0.0;
  for (int d0 = 0; d0 < 3; ++d0) {
    const double dphidx = 0.5 / dx * (+phi[idx + st[d0]] - phi[idx - st[d0]]);
    acc = acc + 0.5 * dphidx * dphidx;
  }
  r[idx] = acc;
}

// ---- output: the components WriteOutput.H writes, for
// planes [k0, k0 + nk) of a valid box, component-major and i fastest (the
// FArrayBox order of the HDF5 "data:datatype=0" chunk of that box)
// KIND 0: set_output_data (SetLevelData.cpp:343-396), the 31 GRChombo
//         variables (GRChomboUserVariables.hpp order) from psi
// KIND 1: output_solver_data's tempData (WriteOutput.H:84-100): dpsi, rhs and
//         the 8 multigrid_vars (psi, A11_0 .. A33_0, phi_0; the A_ij_0 and
//         phi_0 of set_initial_conditions, SetLevelData.cpp:31-72)
template <int KIND>
__global__ __launch_bounds__(256) void k_output_vars(double *__restrict__ out,
                                                     const double *__restrict__ psi,
                                                     const double *__restrict__ dpsi,
                                                     const double *__restrict__ rhs,
                                                     const BoxArgs g, int k0, int nk, double dx,
                                                     const BhParams p) {
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= g.nx || j >= g.ny) return;
  const int iv[3] = {g.glo[0] + i, g.glo[1] + j, g.glo[2] + k0 + k};
  double loc[3];
  for (int d = 0; d < 3; ++d) loc[d] = bh_loc(iv[d], dx, p.domlen[d]);
  double l1[3] = {loc[0] - p.off1, loc[1], loc[2]}, l2[3] = {loc[0] - p.off2, loc[1], loc[2]};
  const double r1 = sqrt(l1[0] * l1[0] + l1[1] * l1[1] + l1[2] * l1[2]);
  const double r2 = sqrt(l2[0] * l2[0] + l2[1] * l2[1] + l2[2] * l2[2]);
  const double n1[3] = {l1[0] / r1, l1[1] / r1, l1[2] / r1};
  const double n2[3] = {l2[0] / r2, l2[1] / r2, l2[2] / r2};
  const double J1[3] = {0.0, 0.0, p.spin1}, J2[3] = {0.0, 0.0, p.spin2};
  const double P1[3] = {0.0, p.mom1, 0.0}, P2[3] = {0.0, p.mom2, 0.0};
  const double A11 = bh_Aij(0, 0, r1, r2, n1, n2, J1, J2, P1, P2);  // SetBinaryBH.H:77-82
  const double A22 = bh_Aij(1, 1, r1, r2, n1, n2, J1, J2, P1, P2);
  const double A33 = bh_Aij(2, 2, r1, r2, n1, n2, J1, J2, P1, P2);
  const double A12 = bh_Aij(0, 1, r1, r2, n1, n2, J1, J2, P1, P2);
  const double A13 = bh_Aij(0, 2, r1, r2, n1, n2, J1, J2, P1, P2);
  const double A23 = bh_Aij(1, 2, r1, r2, n1, n2, J1, J2, P1, P2);
  const double phi0 = bh_phi(p, loc[0], loc[1], loc[2]);  // MyPhiFunction.H
  const long idx = (long)i + (long)j * g.sy + (long)(k0 + k) * g.sz;
  const double psi_c = psi[idx];
  const long V = (long)g.nx * g.ny * nk;
  double *o = out + (long)i + (long)g.nx * (j + (long)g.ny * k);
  if (KIND == 1) {
    const double v[10] = {dpsi[idx], rhs[idx], psi_c, A11, A12, A13, A22, A23, A33, phi0};
#pragma unroll
    for (int c = 0; c < 10; ++c) o[c * V] = v[c];
    return;
  }
  const double psi_bh = p.m1 / r1 + p.m2 / r2;      // SetBinaryBH.H:85-99
  const double chi = pow(psi_c + psi_bh, -4.0);      // SetLevelData.cpp:381-383
  const double factor = pow(chi, 1.5);               // :384
  double v[31];
#pragma unroll
  for (int c = 0; c < 31; ++c) v[c] = 0.0;           // :358-361
  v[1] = v[4] = v[6] = 1.0;                          // h11, h22, h33 (:365-367)
  v[18] = 1.0;                                       // lapse (:368)
  v[7] = p.constant_K;                               // K (:371)
  v[0] = chi;
  v[25] = phi0;                                      // phi (:387)
  v[8] = A11 * factor;                               // A11 .. A33 (:388-393)
  v[9] = A12 * factor;
  v[10] = A13 * factor;
  v[11] = A22 * factor;
  v[12] = A23 * factor;
  v[13] = A33 * factor;
#pragma unroll
  for (int c = 0; c < 31; ++c) o[c * V] = v[c];
}

inline dim3 grid_cells(int nx, int ny, int nz) {
  return dim3((unsigned)((nx + TX - 1) / TX), (unsigned)((ny + TY - 1) / TY), (unsigned)nz);
}
const dim3 kBlock(TX, TY, 1);

inline void check_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(kHipErr, std::string("kernel launch: ") + hipGetErrorString(e));
}

// the LDS-staged residual (MGIC_RESIDUAL_XCD) and restriction
// (MGIC_RESTRICT_XCD) in XCD bands of S tiles (xcd_order above; 0: the
// dispatch order; the restriction's S < 0: chunk-fastest bands of -S).
// The residual takes bands of 16 tiles (4 y rows of the 512^3 plane): its
// HBM fetch 4.34 -> 3.41 GB per 512^3 launch, 0.782 -> 0.732 ms, 256^3
// 0.093 -> 0.081 ms, V-cycle +0.3..0.7% (profiles/r05ad_xcd_bands_ab.txt).  The
// fp64 restriction takes bands of 16 with 4-plane chunks: HBM fetch 3.84 ->
// 3.41 GB per 512^3 launch (1.19x -> 1.06x the compulsory reads) at the
// same time (profiles/r05ah_restrict_chunk_band.txt: it is not bound by its
// HBM bytes); the fp32 one keeps the dispatch order (MGIC_RESTRICT_F_XCD)
// MGIC_RESTRICT_PRE (mask, 1 fp64 / 2 fp32, default 1): the LDS-staged
// restriction with constant bCoef loads the next coarse plane's rhs / aCoef
// rows while it sums the current one; 0 loads them per plane (A/Bs).  fp64:
// 0.638 -> 0.615 ms at 512^3; fp32 (two coarse planes per workgroup): 1024^3
// mixed V-cycle 31.05 -> 31.50 ms, so off (profiles/r06zh_restrict_f_pre_ab.txt)
static int restrict_pre() {
  static const int v = [] {
    const char *e = getenv("MGIC_RESTRICT_PRE");
    return e ? atoi(e) : 1;
  }();
  return v;
}
static int residual_xcd() {
  static const int v = [] {
    const char *e = getenv("MGIC_RESIDUAL_XCD");
    return e ? atoi(e) : 16;
  }();
  return v;
}
static int restrict_xcd() {
  static const int v = [] {
    const char *e = getenv("MGIC_RESTRICT_XCD");
    return e ? atoi(e) : 16;
  }();
  return v;
}
static int restrict_f_xcd() {
  static const int v = [] {
    const char *e = getenv("MGIC_RESTRICT_F_XCD");
    return e ? atoi(e) : 0;
  }();
  return v;
}
// a 3D tile grid as launched: itself, or 1D with its logical shape in lg
inline dim3 xcd_grid(const dim3 &g, uint4 &lg) {
  if (residual_xcd() <= 0) {
    lg = uint4{0, 0, 0, 0};
    return g;
  }
  lg = uint4{g.x, g.y, g.z, (unsigned)residual_xcd()};
  return dim3(g.x * g.y * g.z);
}

// fp64 -> fp32 over the valid region grown by `grow` (coefficients of the
// mixed-precision V-cycle); and a float box copy
__global__ __launch_bounds__(256) void k_to_float(float *__restrict__ d, const double *__restrict__ s,
                                                  const BoxArgs g, int grow) {
  const int i = blockIdx.x * TX + threadIdx.x - grow;
  const int j = blockIdx.y * TY + threadIdx.y - grow;
  const int k = (int)blockIdx.z - grow;
  if (i >= g.nx + grow || j >= g.ny + grow) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  d[idx] = (float)s[idx];
}

__global__ __launch_bounds__(256) void k_incr_f(double *__restrict__ x, const float *__restrict__ y,
                                                const BoxArgs g) {
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= g.nx || j >= g.ny) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  x[idx] = x[idx] + (double)y[idx];
}

__global__ __launch_bounds__(256) void k_copy_f(float *__restrict__ d, const float *__restrict__ s,
                                                const BoxArgs g) {
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= g.nx || j >= g.ny) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  d[idx] = s[idx];
}

// ---- coarse-fine interpolation ([Chombo] QuadCFInterp, restated) ---------
// A ghost cell g of a fine box face that is not a domain face takes the
// quadratic through (normal coordinate, fine cells h from the face = 0):
//   phi* at -h (the centre of the coarse cell that holds g, tangentially
//           interpolated to g's position), f1 at h/2, f2 at 3h/2,
// evaluated at -h/2:  g = 8/15 phi* + 2/3 f1 - 1/5 f2   (ratio 2).
// phi* = c0 + sum_t (x_t d1_t + x_t^2/2 d2_t) + x_1 x_2 d12 with x_t = +-1/4
// (the fine cell's offset in coarse cells), centred differences where both
// tangential coarse neighbours are usable (inside the domain or periodic, not
// covered by the fine level), one-sided first differences (d2 = 0) where one
// is, nothing where none is; the mixed term needs all four diagonals.
// Homogeneous (HOM): phi* = 0 (a zero coarse correction).
__device__ __forceinline__ bool cf_covered(int x, int y, int z, const CFArgs &c) {
  for (int n = 0; n < c.ncov; ++n) {
    const int *b = c.cov + 6 * n;
    if (x >= b[0] && x <= b[3] && y >= b[1] && y <= b[4] && z >= b[2] && z <= b[5]) return true;
  }
  return false;
}

__device__ __forceinline__ bool cf_usable(int p[3], const CFArgs &c) {
  int q[3];
  for (int d = 0; d < 3; ++d) {
    q[d] = p[d];
    const int n = c.cdom_hi[d] - c.cdom_lo[d] + 1;
    if (q[d] < c.cdom_lo[d] || q[d] > c.cdom_hi[d]) {
      if (!c.periodic[d]) return false;
      q[d] = c.cdom_lo[d] + ((q[d] - c.cdom_lo[d]) % n + n) % n;
    }
  }
  return !cf_covered(q[0], q[1], q[2], c);
}

template <bool HOM>
__global__ __launch_bounds__(256) void k_cf_interp(double *__restrict__ u,
                                                   const double *__restrict__ cs, const BoxArgs g,
                                                   const CFArgs c) {
  const int dir = c.face >> 1, side = c.face & 1;
  const int d0 = dir == 0 ? 1 : 0, d1 = dir == 2 ? 1 : 2;
  const int n[3] = {g.nx, g.ny, g.nz};
  const int a0 = (int)(blockIdx.x * blockDim.x + threadIdx.x), a1 = (int)blockIdx.y;
  if (a0 >= n[d0] || a1 >= n[d1]) return;
  int l[3];  // local fine index of the ghost
  l[dir] = side ? n[dir] : -1;
  l[d0] = a0;
  l[d1] = a1;
  const long st[3] = {1, g.sy, g.sz};
  const long gi = (long)l[0] + (long)l[1] * g.sy + (long)l[2] * g.sz;
  const long in = side ? -st[dir] : st[dir];  // one cell into the box
  const double f1 = u[gi + in], f2 = u[gi + 2 * in];
  double ps = 0.0;
  if (!HOM) {
    int gf[3], gc[3];
    for (int d = 0; d < 3; ++d) {
      gf[d] = c.flo[d] + l[d];
      gc[d] = gf[d] >= 0 ? gf[d] / 2 : -((-gf[d] + 1) / 2);  // floor(gf / 2)
    }
    auto at = [&](int x, int y, int z) {
      return cs[(long)(x - c.clo[0]) + (long)(y - c.clo[1]) * c.csy + (long)(z - c.clo[2]) * c.csz];
    };
    const double c0 = at(gc[0], gc[1], gc[2]);
    const int td[2] = {d0, d1};
    double d1v[2], d2v[2], xt[2];
    bool okp[2], okm[2];
    for (int t = 0; t < 2; ++t) {
      const int d = td[t];
      xt[t] = (gf[d] - 2 * gc[d]) ? 0.25 : -0.25;
      int pp[3] = {gc[0], gc[1], gc[2]}, pm[3] = {gc[0], gc[1], gc[2]};
      pp[d] += 1;
      pm[d] -= 1;
      okp[t] = cf_usable(pp, c);
      okm[t] = cf_usable(pm, c);
      const double vp = okp[t] ? at(pp[0], pp[1], pp[2]) : 0.0;
      const double vm = okm[t] ? at(pm[0], pm[1], pm[2]) : 0.0;
      if (okp[t] && okm[t]) {
        d1v[t] = (vp - vm) * 0.5;
        d2v[t] = (vp - 2.0 * c0) + vm;
      } else if (okp[t]) {
        d1v[t] = vp - c0;
        d2v[t] = 0.0;
      } else if (okm[t]) {
        d1v[t] = c0 - vm;
        d2v[t] = 0.0;
      } else {
        d1v[t] = 0.0;
        d2v[t] = 0.0;
      }
    }
    double d12 = 0.0;
    {
      bool all = true;
      double v[4];
      int q = 0;
      for (int s1 = -1; s1 <= 1; s1 += 2)
        for (int s0 = -1; s0 <= 1; s0 += 2) {
          int p[3] = {gc[0], gc[1], gc[2]};
          p[d0] += s0;
          p[d1] += s1;
          const bool ok = cf_usable(p, c);
          all = all && ok;
          v[q++] = ok ? at(p[0], p[1], p[2]) : 0.0;
        }
      // v: (-,-), (+,-), (-,+), (+,+) in (d0, d1)
      if (all) d12 = (((v[3] - v[2]) - v[1]) + v[0]) * 0.25;
    }
    ps = c0;
    for (int t = 0; t < 2; ++t) ps = ps + (xt[t] * d1v[t] + 0.5 * (xt[t] * xt[t]) * d2v[t]);
    ps = ps + (xt[0] * xt[1]) * d12;
  }
  u[gi] = ((8.0 / 15.0) * ps + (2.0 / 3.0) * f1) + (-0.2) * f2;
}

// ---- BiCGStab on the device (the bottom solver's loop without host
// readbacks; op.cpp BiCGStabSolver::solve_device).  The scalars the host loop
// branches on live in a BicgState in device memory: the last block of each
// reduction launch (told by an agent-scope counter) finishes the partials with
// k_reduce_final's loop and tree, evaluates the host loop's tests in the same
// order and writes alpha / omega / beta, or stops the solve (done = 1, with
// its reason); every later launch of the batch returns at once.  Each vector
// update fuses the reductions and the preCond scaling that follow it in the
// host loop, with the same per-element expressions and k_reduce_partial's
// row-to-wave deal and accumulators, so every value is the host loop's bit
// for bit.

// The launch's last block to arrive, by counters sharded per XCD (block b
// runs on XCD b % 8): one word takes ~88 atomic adds per us, so 2048 blocks
// on one counter cost ~23 us; on eight shards of 256 about 3.  Thread 0 has
// stored this block's partials write-through (sc1, agent scope) and waits for
// them before its add (MI355X_MICROARCH.md's counter hand-off); the last
// adder of a shard adds to the top counter, and the last adder there resets
// it and acquires at agent scope before its block reads the partials.  cnt:
// nine counters, each on a 128-B line of its own (32 words apart), zero
// between launches.
constexpr int kBicgCntStride = 32, kBicgCntWords = 9 * kBicgCntStride;
static_assert(4 * kBicgCntWords == kBicgCounterWords, "counter block size");
__device__ __forceinline__ bool bicg_last_block(unsigned int *cnt, unsigned int nb) {
  __shared__ int last;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned int g = blockIdx.x & 7u;
    const unsigned int ng = (nb + 7u - g) / 8u;  // blocks of shard g
    const unsigned int groups = nb < 8u ? nb : 8u;
    unsigned int *sh = cnt + kBicgCntStride * (1 + g);
    int l = 0;
    if (__hip_atomic_fetch_add(sh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1) {
      __hip_atomic_store(sh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
          groups - 1) {
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        l = 1;
      }
    }
    last = l;
  }
  __syncthreads();
  return last != 0;
}

__device__ __forceinline__ void bicg_store_part(double *p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p),
                     (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// k_reduce_final<KIND>'s loop and tree over n partials, in the last block
// (the first 8 * RB partials loaded together, then added in the loop's
// order); the result in every thread
template <int KIND>
__device__ double bicg_final(const double *parts, int n, double *sm) {
  double v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int t = threadIdx.x + q * RB;
    v[q] = t < n ? parts[t] : 0.0;
  }
  double acc = red_init<KIND>();
#pragma unroll
  for (int q = 0; q < 8; ++q)
    if ((int)threadIdx.x + q * RB < n) acc = red_op<KIND>(acc, v[q]);
  for (int t = threadIdx.x + 8 * RB; t < n; t += RB) acc = red_op<KIND>(acc, parts[t]);
  sm[threadIdx.x] = acc;
  __syncthreads();
  for (int w = RB / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) sm[threadIdx.x] = red_op<KIND>(sm[threadIdx.x], sm[threadIdx.x + w]);
    __syncthreads();
  }
  const double r = sm[0];
  __syncthreads();
  return r;
}

// the block's partial of reduction KIND (k_reduce_partial's tree) -> parts[blockIdx.x]
template <int KIND>
__device__ void bicg_block_part(const double acc[4], double *sm, double *parts, int lb) {
  sm[threadIdx.x] = red_op<KIND>(red_op<KIND>(acc[0], acc[1]), red_op<KIND>(acc[2], acc[3]));
  __syncthreads();
  for (int w = RB / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) sm[threadIdx.x] = red_op<KIND>(sm[threadIdx.x], sm[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) bicg_store_part(parts + lb, sm[0]);
  __syncthreads();
}

// norm_of (op.cpp): max / sum norms as reduced, the 2-norm's square root
__device__ __forceinline__ double bicg_norm_of(int nt, double x) {
  return nt == 1 || nt == 0 ? x : sqrt(x);
}

__device__ __forceinline__ void bicg_stop(BicgState *st, int reason) {
  st->done = 1;
  st->reason = reason;
}

// The logical block whose rows (and partial) a block takes: its own index, or
// (BicgState::xr, a grid of whole groups of 8) the XCD-contiguous deal --
// block b runs on XCD b % 8 and takes logical block (b % 8) (nb / 8) + b / 8,
// so an XCD streams a contiguous slab of planes (its L2 holds the y / z
// neighbours of its rows).  The partials stay indexed by logical block, so
// the sums, and every value, are the same either way.
__device__ __forceinline__ int bicg_lblock(const BicgState *st) {
  const int b = blockIdx.x, nb = gridDim.x;
  if (!st->xr || (nb & 7)) return b;
  return (b & 7) * (nb >> 3) + (b >> 3);
}

// k_reduce_partial's row-to-wave deal: for every cell, in that deal's order,
// v = ld(i, j, k, idx) then op(v, i, j, k, idx, q), q = the lane's
// accumulator.  Rows of at most 128 cells (the bottom's boxes) give a lane at
// most two cells per row, both into accumulator 0: two rows are taken at
// once, every load of the four cells issued before the first op, so each
// lane keeps four cells' loads in flight (the ops, and so every sum, still
// run in the deal's order).
template <class LD, class OP>
__device__ __forceinline__ void bicg_rows(const BoxArgs &g, int lb, LD &&ld, OP &&op) {
  constexpr int W = RB / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nrows = g.ny * g.nz;
  const int stride = gridDim.x * W;
  if (g.nx <= 128) {
    const bool c0 = lane < g.nx, c1 = lane + 64 < g.nx;
    for (int row = lb * W + wave; row < nrows; row += 2 * stride) {
      const int rowb = row + stride;
      const bool rb = rowb < nrows;
      const int k = row / g.ny, j = row - k * g.ny;
      const int kb = rb ? rowb / g.ny : k, jb = rb ? rowb - kb * g.ny : j;
      const long base = (long)j * g.sy + (long)k * g.sz;
      const long baseb = (long)jb * g.sy + (long)kb * g.sz;
      decltype(ld(0, 0, 0, 0L)) v0{}, v1{}, v2{}, v3{};
      if (c0) v0 = ld(lane, j, k, base + lane);
      if (c1) v1 = ld(lane + 64, j, k, base + lane + 64);
      if (rb && c0) v2 = ld(lane, jb, kb, baseb + lane);
      if (rb && c1) v3 = ld(lane + 64, jb, kb, baseb + lane + 64);
      if (c0) op(v0, lane, j, k, base + lane, 0);
      if (c1) op(v1, lane + 64, j, k, base + lane + 64, 0);
      if (rb && c0) op(v2, lane, jb, kb, baseb + lane, 0);
      if (rb && c1) op(v3, lane + 64, jb, kb, baseb + lane + 64, 0);
    }
    return;
  }
  auto f = [&](int i, int j, int k, long idx, int q) { op(ld(i, j, k, idx), i, j, k, idx, q); };
  for (int row = lb * W + wave; row < nrows; row += stride) {
    const int k = row / g.ny, j = row - k * g.ny;
    const long base = (long)j * g.sy + (long)k * g.sz;
    int i = lane;
    for (; i + 192 < g.nx; i += 256) {
      f(i, j, k, base + i, 0);
      f(i + 64, j, k, base + i + 64, 1);
      f(i + 128, j, k, base + i + 128, 2);
      f(i + 192, j, k, base + i + 192, 3);
    }
    for (; i < g.nx; i += 64) f(i, j, k, base + i, 0);
  }
}

// VCCOMPUTEOP3D at one cell (k_apply_op's expressions, lap7's BC images),
// split into its loads and its arithmetic for bicg_rows
struct BicgSten {
  double c, xm, xp, ym, yp, zm, zp, av, bv;
};
template <bool BC>
__device__ __forceinline__ BicgSten bicg_sten_load(const double *__restrict__ u,
                                                   const double *__restrict__ a,
                                                   const double *__restrict__ b, long idx,
                                                   const BoxArgs &g) {
  BicgSten v;
  v.c = u[idx];
  v.xm = u[idx - 1];
  v.xp = u[idx + 1];
  v.ym = u[idx - g.sy];
  v.yp = u[idx + g.sy];
  v.zm = u[idx - g.sz];
  v.zp = u[idx + g.sz];
  v.av = a[idx];
  v.bv = BC ? 0.0 : b[idx];
  return v;
}
template <bool BC>
__device__ __forceinline__ double bicg_sten_apply(BicgSten v, int i, int j, int k,
                                                  const BoxArgs &g, const StencilCoefs &s) {
  const double c = v.c;
  if (i == 0 && g.bcm[0]) v.xm = ghost_of(g.bcm[0], g.bcc[0], c);
  if (i == g.nx - 1 && g.bcm[1]) v.xp = ghost_of(g.bcm[1], g.bcc[1], c);
  if (j == 0 && g.bcm[2]) v.ym = ghost_of(g.bcm[2], g.bcc[2], c);
  if (j == g.ny - 1 && g.bcm[3]) v.yp = ghost_of(g.bcm[3], g.bcc[3], c);
  if (k == 0 && g.bcm[4]) v.zm = ghost_of(g.bcm[4], g.bcc[4], c);
  if (k == g.nz - 1 && g.bcm[5]) v.zp = ghost_of(g.bcm[5], g.bcc[5], c);
  const double tx = (v.xp + v.xm) - 2.0 * c;
  const double ty = (v.yp + v.ym) - 2.0 * c;
  const double tz = (v.zp + v.zm) - 2.0 * c;
  const double lap = (tx + ty) + tz;                  // lap7
  const double lof = s.alpha * v.av * c;              // .ChF:211-212
  const double ldpsi = lap * s.dxinv * s.beta * (BC ? s.bval : v.bv);  // .ChF:227
  return lof - ldpsi;                                 // .ChF:229
}

// P = R (first iteration after a (re)start) or ((P*beta) + c*V) + 1.0*R,
// c = (-beta)*omega (bicgP); W = P * lambda (preCond's first pass)
__global__ __launch_bounds__(256) void k_bicgd_p(BicgState *__restrict__ st,
                                                double *__restrict__ p, double *__restrict__ w,
                                                const double *__restrict__ v,
                                                const double *__restrict__ r,
                                                const double *__restrict__ lam, const BoxArgs g) {
  if (st->done) return;
  const int i = blockIdx.x * TX + threadIdx.x;
  const int j = blockIdx.y * TY + threadIdx.y;
  const int k = blockIdx.z;
  if (i >= g.nx || j >= g.ny) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  double pv;
  if (st->init) {
    pv = r[idx];
  } else {
    const double beta = st->beta, c = (-beta) * st->omega;
    double t = p[idx] * beta;
    t = t + c * v[idx];
    pv = t + 1.0 * r[idx];
  }
  p[idx] = pv;
  w[idx] = pv * lam[idx];
}

// V = L(PT); <RT, V>; last block: m, alpha (or a restart / stop)
template <bool BC>
__global__ __launch_bounds__(RB) void k_bicgd_apply_dot(BicgState *__restrict__ st,
                                                       double *__restrict__ v,
                                                       const double *__restrict__ pt,
                                                       const double *__restrict__ rt,
                                                       const double *__restrict__ a,
                                                       const double *__restrict__ b,
                                                       const BoxArgs g, const StencilCoefs s,
                                                       double *__restrict__ parts,
                                                       unsigned int *__restrict__ cnt) {
  __shared__ double sm[RB];
  if (st->done) return;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  struct L {
    BicgSten u;
    double rt;
  };
  const int lb = bicg_lblock(st);
  bicg_rows(
      g, lb,
      [&](int, int, int, long idx) { return L{bicg_sten_load<BC>(pt, a, b, idx, g), rt[idx]}; },
      [&](const L &x, int i, int j, int k, long idx, int q) {
        const double vv = bicg_sten_apply<BC>(x.u, i, j, k, g, s);
        v[idx] = vv;
        acc[q] = acc[q] + x.rt * vv;
      });
  bicg_block_part<0>(acc, sm, parts, lb);
  if (!bicg_last_block(cnt, gridDim.x)) return;
  const double m = bicg_final<0>(parts, gridDim.x, sm);
  if (threadIdx.x == 0) {
    st->m = m;
    st->init = 0;
    if (fabs(m) > st->small * fabs(st->rho1)) st->alpha = st->rho1 / m;
    else bicg_stop(st, st->restarts >= st->num_restarts ? kBicgRestartLimit : kBicgRestart);
  }
}

// S = R + (-alpha) V; |S| (norm kind NK); W = S * lambda; last block: the
// half-step stop test.  E += alpha PT is left pending (epend) for k_bicgd_r.
template <int NK>
__global__ __launch_bounds__(RB) void k_bicgd_s(BicgState *__restrict__ st,
                                               double *__restrict__ s, double *__restrict__ w,
                                               const double *__restrict__ r,
                                               const double *__restrict__ v,
                                               const double *__restrict__ lam, const BoxArgs g,
                                               double *__restrict__ parts,
                                               unsigned int *__restrict__ cnt) {
  __shared__ double sm[RB];
  if (st->done) return;
  const double ca = -st->alpha;
  double acc[4] = {red_init<NK>(), red_init<NK>(), red_init<NK>(), red_init<NK>()};
  struct L {
    double r, v, lam;
  };
  const int lb = bicg_lblock(st);
  bicg_rows(
      g, lb, [&](int, int, int, long idx) { return L{r[idx], v[idx], lam[idx]}; },
      [&](const L &x, int, int, int, long idx, int q) {
        const double sv = x.r + ca * x.v;
        s[idx] = sv;
        w[idx] = sv * x.lam;
        acc[q] = red_op<NK>(acc[q], NK == 2 ? sv * sv : fabs(sv));
      });
  bicg_block_part<NK>(acc, sm, parts, lb);
  if (!bicg_last_block(cnt, gridDim.x)) return;
  const double x = bicg_final<NK>(parts, gridDim.x, sm);
  if (threadIdx.x == 0) {
    const double nrm = bicg_norm_of(st->nt, x);
    st->nrm = nrm;
    st->epend = 1;
    if (nrm <= st->eps * st->init_norm || nrm <= st->reps) bicg_stop(st, kBicgHalf);
  }
}

// <T, S> and <T, T> of T = L(ST), T not stored (k_bicgd_r recomputes it,
// the same expressions on the same inputs); last block: omega (or the
// tt == 0 stop)
template <bool BC>
__global__ __launch_bounds__(RB) void k_bicgd_apply_dot2(BicgState *__restrict__ st,
                                                        const double *__restrict__ stv,
                                                        const double *__restrict__ s,
                                                        const double *__restrict__ a,
                                                        const double *__restrict__ b,
                                                        const BoxArgs g, const StencilCoefs sc,
                                                        double *__restrict__ parts_ts,
                                                        double *__restrict__ parts_tt,
                                                        unsigned int *__restrict__ cnt) {
  __shared__ double sm[RB];
  if (st->done) return;
  double aa[4] = {0.0, 0.0, 0.0, 0.0}, bb[4] = {0.0, 0.0, 0.0, 0.0};
  struct L {
    BicgSten u;
    double s;
  };
  const int lb = bicg_lblock(st);
  bicg_rows(
      g, lb,
      [&](int, int, int, long idx) { return L{bicg_sten_load<BC>(stv, a, b, idx, g), s[idx]}; },
      [&](const L &x, int i, int j, int k, long, int q) {
        const double tv = bicg_sten_apply<BC>(x.u, i, j, k, g, sc);
        aa[q] = aa[q] + tv * x.s;
        bb[q] = bb[q] + tv * tv;
      });
  bicg_block_part<0>(aa, sm, parts_ts, lb);
  bicg_block_part<0>(bb, sm, parts_tt, lb);
  if (!bicg_last_block(cnt, gridDim.x)) return;
  const double ts = bicg_final<0>(parts_ts, gridDim.x, sm);
  const double tt = bicg_final<0>(parts_tt, gridDim.x, sm);
  if (threadIdx.x == 0) {
    st->ts = ts;
    st->tt = tt;
    if (tt == 0.0) bicg_stop(st, kBicgTt0);
    else st->omega = ts / tt;
  }
}

// R = S + (-omega) T with T = L(ST) recomputed; E = (E + alpha PT) + omega
// ST; |R| (kind NK) and <RT, R>; last block: the omega == 0 stop, then the
// loop's head -- its test, it += 1, rho1 = <RT, R>, the rho1 == 0 stop and
// beta
template <int NK, bool BC>
__global__ __launch_bounds__(RB) void k_bicgd_r(BicgState *__restrict__ st,
                                               double *__restrict__ r, double *__restrict__ e,
                                               const double *__restrict__ s,
                                               const double *__restrict__ a,
                                               const double *__restrict__ b,
                                               const StencilCoefs sc,
                                               const double *__restrict__ pt,
                                               const double *__restrict__ stv,
                                               const double *__restrict__ rt, const BoxArgs g,
                                               double *__restrict__ parts_n,
                                               double *__restrict__ parts_d,
                                               unsigned int *__restrict__ cnt) {
  __shared__ double sm[RB];
  if (st->done) return;
  const double alpha = st->alpha, omega = st->omega, ca = -omega;
  double an[4] = {red_init<NK>(), red_init<NK>(), red_init<NK>(), red_init<NK>()};
  double ad[4] = {0.0, 0.0, 0.0, 0.0};
  struct L {
    BicgSten u;
    double s, e, pt, rt;
  };
  const int lb = bicg_lblock(st);
  bicg_rows(
      g, lb,
      [&](int, int, int, long idx) {
        return L{bicg_sten_load<BC>(stv, a, b, idx, g), s[idx], e[idx], pt[idx], rt[idx]};
      },
      [&](const L &x, int i, int j, int k, long idx, int q) {
        const double tv = bicg_sten_apply<BC>(x.u, i, j, k, g, sc);
        const double rv = x.s + ca * tv;
        r[idx] = rv;
        const double e1 = x.e + alpha * x.pt;
        e[idx] = e1 + omega * x.u.c;  // (x.u.c: ST at the cell)
        an[q] = red_op<NK>(an[q], NK == 2 ? rv * rv : fabs(rv));
        ad[q] = ad[q] + x.rt * rv;
      });
  bicg_block_part<NK>(an, sm, parts_n, lb);
  bicg_block_part<0>(ad, sm, parts_d, lb);
  if (!bicg_last_block(cnt, gridDim.x)) return;
  const double x = bicg_final<NK>(parts_n, gridDim.x, sm);
  const double rho_next = bicg_final<0>(parts_d, gridDim.x, sm);
  if (threadIdx.x == 0) {
    const double nrm = bicg_norm_of(st->nt, x);
    st->nrm = nrm;
    st->rho_next = rho_next;
    st->epend = 0;
    if (omega == 0.0) {
      bicg_stop(st, kBicgOmega0);
    } else if (!(st->it < st->imax && nrm > st->eps * st->init_norm && nrm > st->reps)) {
      bicg_stop(st, kBicgStop);
    } else {
      st->it += 1;
      st->rho2 = st->rho1;
      st->rho1 = rho_next;
      if (rho_next == 0.0) bicg_stop(st, kBicgRho0);
      else st->beta = (st->rho1 / st->rho2) * (st->alpha / st->omega);
    }
  }
}

// the state into pinned host memory, then the sequence number the host spins on
__global__ void k_bicgd_publish(const BicgState *__restrict__ st, BicgState *host,
                               unsigned long long *seq, unsigned long long seqv) {
  if (threadIdx.x != 0) return;
  constexpr int nw = (int)(sizeof(BicgState) / 4);
  const unsigned int *src = reinterpret_cast<const unsigned int *>(st);
  unsigned int *dst = reinterpret_cast<unsigned int *>(host);
  for (int t = 0; t < nw; ++t)
    __hip_atomic_store(dst + t, src[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(seq, seqv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace

void gsrb_pass(double *u, const double *rhs, const double *a, const double *b, const double *lam,
               const BoxArgs &g, const StencilCoefs &s, int colour, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  const int npairs = (g.nx + 1) / 2;
  const dim3 grid((unsigned)((npairs + TX - 1) / TX), (unsigned)((g.ny + TY - 1) / TY),
                  (unsigned)g.nz);
  if (lam) {
    if (s.bconst) k_gsrb<true, true><<<grid, kBlock, 0, st>>>(u, rhs, a, b, lam, g, s, colour);
    else k_gsrb<true, false><<<grid, kBlock, 0, st>>>(u, rhs, a, b, lam, g, s, colour);
  } else {
    if (s.bconst) k_gsrb<false, true><<<grid, kBlock, 0, st>>>(u, rhs, a, b, nullptr, g, s, colour);
    else k_gsrb<false, false><<<grid, kBlock, 0, st>>>(u, rhs, a, b, nullptr, g, s, colour);
  }
  check_launch();
}

void apply_op(double *lu, const double *u, const double *a, const double *b, const BoxArgs &g,
              const StencilCoefs &s, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  if (s.bconst) k_apply_op<true><<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st>>>(lu, u, a, b, g, s);
  else k_apply_op<false><<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st>>>(lu, u, a, b, g, s);
  check_launch();
}

// the fp64 residual on LDS-staged u planes (k_residual_zl) in 32-plane
// chunks: 512^3 0.800 -> 0.775 ms, 256^3 0.100 -> 0.092, V-cycle +0.4%
// (profiles/r05s_residual_lds_ab.txt); MGIC_RESIDUAL_ZL=0: k_residual_z2
static bool residual_lds() {
  static const bool v = [] {
    const char *e = getenv("MGIC_RESIDUAL_ZL");
    return !(e && atoi(e) == 0);
  }();
  return v;
}

static int residual_kc_env();

void residual(double *r, const double *u, const double *rhs, const double *a, const double *b,
              const BoxArgs &g, const StencilCoefs &s, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  const int mode = residual_kc_env();
  static const int pairs = [] {
    const char *e = getenv("MGIC_RESIDUAL_PAIRS");
    return e ? atoi(e) : 1;
  }();
  if (mode > 0 && pairs) {  // z-streaming on x-pairs, chunks of `mode` planes
    const int kc = mode < g.nz ? mode : g.nz;
    dim3 grid = grid_cells((g.nx + 1) / 2, g.ny, g.nz);
    grid.z = (unsigned)((g.nz + kc - 1) / kc);
    static const int nt = [] {
      const char *e = getenv("MGIC_RESIDUAL_NT");
      return e ? atoi(e) : 3;
    }();
#define MGIC_RZ2(N)                                                                        \
  do {                                                                                     \
    if (residual_lds()) {                                                                  \
      uint4 lg;                                                                            \
      const dim3 xg = xcd_grid(grid, lg);                                                  \
      if (s.bconst) k_residual_zl<true, double, N><<<xg, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc, nullptr, lg); \
      else k_residual_zl<false, double, N><<<xg, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc, nullptr, lg);         \
    } else if (s.bconst) k_residual_z2<true, double, N><<<grid, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc); \
    else k_residual_z2<false, double, N><<<grid, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc);         \
  } while (0)
    switch (nt & 3) {
      case 1: MGIC_RZ2(1); break;
      case 2: MGIC_RZ2(2); break;
      case 3: MGIC_RZ2(3); break;
      default: MGIC_RZ2(0); break;
    }
#undef MGIC_RZ2
  } else if (mode > 0) {  // z-streaming, chunks of `mode` planes
    const int kc = mode < g.nz ? mode : g.nz;
    dim3 grid = grid_cells(g.nx, g.ny, g.nz);
    grid.z = (unsigned)((g.nz + kc - 1) / kc);
    if (s.bconst) k_residual_z<true, double><<<grid, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc);
    else k_residual_z<false, double><<<grid, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc);
  } else if (s.bconst) {
    k_residual<true><<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st>>>(r, u, rhs, a, b, g, s);
  } else {
    k_residual<false><<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st>>>(r, u, rhs, a, b, g, s);
  }
  check_launch();
}

// z chunk of the fp64 residual (MGIC_RESIDUAL_KC): 16 planes for both forms
// (LDS-staged: 0.749 -> 0.737 ms at 512^3 against 32 with the XCD bands,
// V-cycle +0.6%, profiles/r06zq_residual_chunk_ab.jsonl; the max-norm
// partials are order-free, so the norm is the same whatever the chunk)
static int residual_kc_env() {
  static const int mode = [] {
    const char *e = getenv("MGIC_RESIDUAL_KC");
    return e ? atoi(e) : 16;
  }();
  return mode;
}

long residual_norm_blocks(const BoxArgs &g) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return 0;
  const int mode = residual_kc_env();
  if (mode <= 0) return 0;
  const int kc = mode < g.nz ? mode : g.nz;
  const dim3 grid = grid_cells((g.nx + 1) / 2, g.ny, g.nz);
  return (long)grid.x * grid.y * ((g.nz + kc - 1) / kc);
}

void residual_norm(double *r, const double *u, const double *rhs, const double *a, const double *b,
                   const BoxArgs &g, const StencilCoefs &s, double *partials, hipStream_t st) {
  if (residual_norm_blocks(g) <= 0) throw Error(kBadArg, "residual_norm: streaming residual off");
  const int mode = residual_kc_env();
  const int kc = mode < g.nz ? mode : g.nz;
  dim3 grid = grid_cells((g.nx + 1) / 2, g.ny, g.nz);
  grid.z = (unsigned)((g.nz + kc - 1) / kc);
  // the default streams of residual() (MGIC_RESIDUAL_NT = 3: rhs / aCoef
  // loads and r stores non-temporal)
  if (residual_lds()) {
    uint4 lg;
    const dim3 xg = xcd_grid(grid, lg);
    if (s.bconst)
      k_residual_zl<true, double, 3, true><<<xg, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc, partials, lg);
    else
      k_residual_zl<false, double, 3, true><<<xg, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc, partials, lg);
  } else if (s.bconst)
    k_residual_z2<true, double, 3, true><<<grid, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc, partials);
  else
    k_residual_z2<false, double, 3, true><<<grid, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc, partials);
  check_launch();
}

void restrict_residual(double *rc, const BoxArgs &cg, const double *u, const double *rhs,
                       const double *a, const double *b, const BoxArgs &fg, const StencilCoefs &s,
                       hipStream_t st, bool accumulate) {
  if (cg.nx <= 0 || cg.ny <= 0 || cg.nz <= 0) return;
  static const int nt = [] {
    const char *e = getenv("MGIC_RESTRICT_NT");
    return e ? atoi(e) : 1;
  }();
  // MGIC_RESTRICT_NT bit 0: non-temporal rhs / aCoef / bCoef loads, for
  // every bCoef kind (the same switch in restrict_residual_f)
  const int accu = accumulate ? 1 : 0;
  // k_restrict_zl, two coarse planes per workgroup (MGIC_RESTRICT_ZL: the
  // chunk; 0 = k_restrict).  512^3: 0.706 -> 0.641 ms, 256^3 equal, V-cycle
  // +1.4% (chunks 1 .. 32 measured, profiles/r05r_restrict_lds_ab.txt); 4
  // planes in XCD bands since (restrict_xcd above)
  static const int zl = [] {
    const char *e = getenv("MGIC_RESTRICT_ZL");
    return e ? atoi(e) : 4;
  }();
  if (zl > 0 && (nt & 1) && fg.nx == 2 * cg.nx && fg.ny == 2 * cg.ny && fg.nz == 2 * cg.nz) {
    const int ntx = (cg.nx + TX - 1) / TX, nty = (cg.ny + 3) / 4;
    const int kc = zl < cg.nz ? zl : cg.nz;
    const int nb = ntx * nty * ((cg.nz + kc - 1) / kc);
    if (s.bconst && (restrict_pre() & 1))
      k_restrict_zl<double, true, 1, true><<<nb, 256, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, accu, kc,
                                                               ntx, nty, restrict_xcd());
    else if (s.bconst)
      k_restrict_zl<double, true, 1><<<nb, 256, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, accu, kc, ntx, nty,
                                                         restrict_xcd());
    else
      k_restrict_zl<double, false, 1><<<nb, 256, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, accu, kc, ntx, nty,
                                                          restrict_xcd());
    check_launch();
    return;
  }
  const dim3 grid = grid_cells(cg.nx, cg.ny, cg.nz);
  if (s.bconst && (nt & 1))
    k_restrict<double, true, 1><<<grid, kBlock, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, accu);
  else if (s.bconst)
    k_restrict<double, true><<<grid, kBlock, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, accu);
  else if (nt & 1)
    k_restrict<double, false, 1><<<grid, kBlock, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, accu);
  else
    k_restrict<double, false><<<grid, kBlock, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, accu);
  check_launch();
}

void prolong(double *uf, const BoxArgs &fg, const double *ec, const BoxArgs &cg,
             const int avail_lo[3], const int avail_hi[3], int type, hipStream_t st) {
  if (fg.nx <= 0 || fg.ny <= 0 || fg.nz <= 0) return;
  ProlongArgs pa;
  for (int d = 0; d < 3; ++d) {
    pa.avail_lo[d] = avail_lo[d];
    pa.avail_hi[d] = avail_hi[d];
  }
  MGIC_CHECK(fg.nx == 2 * cg.nx && fg.ny == 2 * cg.ny && fg.nz == 2 * cg.nz,
             "prolong: fine box must be the coarse box refined by 2");
  if (type == 1)
    k_prolong<double, 1><<<grid_cells(cg.nx, cg.ny, cg.nz), kBlock, 0, st>>>(uf, fg, ec, cg, pa);
  else
    k_prolong<double, 0><<<grid_cells(cg.nx, cg.ny, cg.nz), kBlock, 0, st>>>(uf, fg, ec, cg, pa);
  check_launch();
}

void lambda(double *lam, const double *a, const BoxArgs &g, const StencilCoefs &s,
            hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  k_lambda<<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st>>>(lam, a, g, s);
  check_launch();
}

void average(double *c, const BoxArgs &cg, const double *f, const BoxArgs &fg, int ratio,
             int harmonic, hipStream_t st) {
  if (cg.nx <= 0 || cg.ny <= 0 || cg.nz <= 0) return;
  k_average<<<grid_cells(cg.nx, cg.ny, cg.nz), kBlock, 0, st>>>(c, cg, f, fg, ratio, harmonic);
  check_launch();
}

void fill_bc(double *u, const BoxArgs &g, hipStream_t st) {
  const int n[3] = {g.nx, g.ny, g.nz};
  for (int face = 0; face < 6; ++face) {
    if (!g.bcm[face]) continue;
    const int dir = face >> 1;
    const int d1 = dir == 0 ? 1 : 0, d2 = dir == 2 ? 1 : 2;
    const dim3 grid((unsigned)((n[d1] + 255) / 256), (unsigned)n[d2], 1);
    k_fill_bc_face<<<grid, dim3(256, 1, 1), 0, st>>>(u, g, face);
    check_launch();
  }
}

static long reduce_blocks(const BoxArgs &g) {
  // (MGIC_RED_MAXBLK: a lower cap, for A/Bs; the host loop and the device
  // loop both size their partials here, so they stay bit-identical)
  static const long cap = [] {
    const char *e = getenv("MGIC_RED_MAXBLK");
    const long v = e ? atol(e) : 0;
    return v >= 8 && v <= kMaxPartsPerBox ? v : (long)kMaxPartsPerBox;
  }();
  long nb = ((long)g.ny * g.nz + RB / 64 - 1) / (RB / 64);  // one wave per row at most
  return nb > cap ? cap : nb;
}

void blas(int kind, double *x, const double *y, const double *z, double s, double t,
          const BoxArgs &g, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  const dim3 grid = grid_cells(g.nx, g.ny, g.nz);
  switch (kind) {
    case 0: k_blas<0><<<grid, kBlock, 0, st>>>(x, y, z, s, t, g); break;
    case 1: k_blas<1><<<grid, kBlock, 0, st>>>(x, y, z, s, t, g); break;
    case 2: k_blas<2><<<grid, kBlock, 0, st>>>(x, y, z, s, t, g); break;
    case 3: k_blas<3><<<grid, kBlock, 0, st>>>(x, y, z, s, t, g); break;
    case 4: k_blas<4><<<grid, kBlock, 0, st>>>(x, y, z, s, t, g); break;
    case 5: k_blas<5><<<grid, kBlock, 0, st>>>(x, y, z, s, t, g); break;
    case 6: k_blas<6><<<grid, kBlock, 0, st>>>(x, y, z, s, t, g); break;
    default: throw Error(kBadArg, "blas: bad kind");
  }
  check_launch();
}

int reduce_partial(int kind, const double *x, const double *y, const BoxArgs &g,
                   double *partials, hipStream_t st) {
  const long ncell = (long)g.nx * g.ny * g.nz;
  if (ncell <= 0) return 0;
  const long nb = reduce_blocks(g);
  const dim3 grid((unsigned)nb), block(RB);
  switch (kind) {
    case 0: k_reduce_partial<0><<<grid, block, 0, st>>>(x, y, g, partials); break;
    case 1: k_reduce_partial<1><<<grid, block, 0, st>>>(x, y, g, partials); break;
    case 2: k_reduce_partial<2><<<grid, block, 0, st>>>(x, y, g, partials); break;
    case 3: k_reduce_partial<3><<<grid, block, 0, st>>>(x, y, g, partials); break;
    case 4: k_reduce_partial<4><<<grid, block, 0, st>>>(x, y, g, partials); break;
    case 5: k_reduce_partial<5><<<grid, block, 0, st>>>(x, y, g, partials); break;
    default: throw Error(kBadArg, "reduce: bad kind");
  }
  check_launch();
  return (int)nb;
}

void reduce_final(int kind, const double *partials, int n, double *out, hipStream_t st,
                  const HostPub &pub) {
  switch (kind) {
    case 0: k_reduce_final<0><<<1, RB, 0, st>>>(partials, n, out, pub); break;
    case 1: k_reduce_final<1><<<1, RB, 0, st>>>(partials, n, out, pub); break;
    case 2: k_reduce_final<2><<<1, RB, 0, st>>>(partials, n, out, pub); break;
    case 3: k_reduce_final_wide<3><<<1, 1024, 0, st>>>(partials, n, out, pub); break;
    case 4: k_reduce_final_wide<4><<<1, 1024, 0, st>>>(partials, n, out, pub); break;
    case 5: k_reduce_final_wide<5><<<1, 1024, 0, st>>>(partials, n, out, pub); break;
    default: throw Error(kBadArg, "reduce: bad kind");
  }
  check_launch();
}

void publish_result(const double *d_val, const HostPub &pub, hipStream_t st) {
  if (!pub.val) return;
  k_publish<<<1, 64, 0, st>>>(d_val, pub);
  check_launch();
}

int axpy2_reduce(int kind, double *s, const double *r, const double *v, double ca, double *e,
                 const double *pt, double cb, const BoxArgs &g, double *partials,
                 hipStream_t st) {
  if ((long)g.nx * g.ny * g.nz <= 0) return 0;
  const long nb = reduce_blocks(g);
  const dim3 grid((unsigned)nb), block(RB);
  switch (kind) {
    case 1: k_axpy2_reduce<1><<<grid, block, 0, st>>>(s, r, v, ca, e, pt, cb, g, partials); break;
    case 2: k_axpy2_reduce<2><<<grid, block, 0, st>>>(s, r, v, ca, e, pt, cb, g, partials); break;
    case 3: k_axpy2_reduce<3><<<grid, block, 0, st>>>(s, r, v, ca, e, pt, cb, g, partials); break;
    default: throw Error(kBadArg, "axpy2_reduce: bad kind");
  }
  check_launch();
  return (int)nb;
}

int dot2_partial(const double *t, const double *s, const BoxArgs &g, double *pts, double *ptt,
                 hipStream_t st) {
  if ((long)g.nx * g.ny * g.nz <= 0) return 0;
  const long nb = reduce_blocks(g);
  k_dot2<<<dim3((unsigned)nb), dim3(RB), 0, st>>>(t, s, g, pts, ptt);
  check_launch();
  return (int)nb;
}

void bicg_p(double *p, const double *v, const double *r, double beta, double c, const BoxArgs &g,
            hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  k_bicg_p<<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st>>>(p, v, r, beta, c, g);
  check_launch();
}


// Blocks per item (grid.y = item): sized for the largest item at
// copy_ept() elements per thread, so the many small items (edges, corners of
// a ghost shell) do not each launch the largest item's share of empty blocks
int copy_ept() {
  static const int ept = [] {
    const char *e = getenv("MGIC_COPY_EPT");
    const int v = e ? atoi(e) : 4;
    return v > 0 ? v : 1;
  }();
  return ept;
}
void copy_items(const CopyItem *d_items, int nitems, long max_cells, double *const *src_tab,
                const double *src_buf, double *const *dst_tab, double *dst_buf, hipStream_t st) {
  if (nitems <= 0 || max_cells <= 0) return;
  const long per = 256L * copy_ept();
  long bx = (max_cells + per - 1) / per;
  if (bx > 1024) bx = 1024;
  k_copy_items<double><<<dim3((unsigned)bx, (unsigned)nitems), dim3(256), 0, st>>>(
      d_items, src_tab, src_buf, dst_tab, dst_buf);
  check_launch();
}

void binary_bh_coefs(double *acoef, double *rhs, const double *psi, const BoxArgs &g, double dx,
                     const BhParams &p, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  k_binary_bh<false><<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st>>>(acoef, rhs, psi, g, dx, p);
  check_launch();
}

void constant_k_integrand(double *out, const double *psi, const BoxArgs &g, double dx,
                          const BhParams &p, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  k_binary_bh<true><<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st>>>(out, nullptr, psi, g, dx, p);
  check_launch();
}

void lap_psi(double *l, const double *psi, const BoxArgs &g, double dx, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  k_lap_psi<<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st>>>(l, psi, g, dx);
  check_launch();
}

void rho_grad_phi(double *r, const double *phi, const BoxArgs &g, double dx, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  k_rho_grad_phi<<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st>>>(r, phi, g, dx);
  check_launch();
}

void output_vars(int kind, double *out, const double *psi, const double *dpsi, const double *rhs,
                 const BoxArgs &g, int k0, int nk, double dx, const BhParams &p, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || nk <= 0) return;
  if (kind == 0)
    k_output_vars<0><<<grid_cells(g.nx, g.ny, nk), kBlock, 0, st>>>(out, psi, dpsi, rhs, g, k0, nk,
                                                                    dx, p);
  else
    k_output_vars<1><<<grid_cells(g.nx, g.ny, nk), kBlock, 0, st>>>(out, psi, dpsi, rhs, g, k0, nk,
                                                                    dx, p);
  check_launch();
}

// x += y over the valid box grown by `grow` cells (set_update_psi0 adds over
// the whole FAB, SetLevelData.cpp:236-256; one ghost layer is all the
// stencils read)
__global__ __launch_bounds__(256) void k_incr_grown(double *__restrict__ x,
                                                    const double *__restrict__ y, const BoxArgs g,
                                                    int grow) {
  const int i = (int)(blockIdx.x * TX + threadIdx.x) - grow;
  const int j = (int)(blockIdx.y * TY + threadIdx.y) - grow;
  const int k = (int)blockIdx.z - grow;
  if (i >= g.nx + grow || j >= g.ny + grow) return;
  const long idx = (long)i + (long)j * g.sy + (long)k * g.sz;
  x[idx] = x[idx] + y[idx];
}

void incr_grown(double *x, const double *y, const BoxArgs &g, int grow, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  k_incr_grown<<<grid_cells(g.nx + 2 * grow, g.ny + 2 * grow, g.nz + 2 * grow), kBlock, 0, st>>>(
      x, y, g, grow);
  check_launch();
}


// ---- fp32 (mixed-precision V-cycle) variants -------------------------------
void residual_to_f(float *r, const double *u, const double *rhs, const double *a, const double *b,
                   const BoxArgs &g, const StencilCoefs &s, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  // k_residual_zl<float> in 16-plane chunks by default (MGIC_RESIDUAL_F_ZL;
  // 0: k_residual_z2): 1024^3 mixed V-cycle 33.4 -> 32.8 ms
  // (profiles/r05u_residual_f_lds_ab.txt)
  static const int fzl = [] {
    const char *e = getenv("MGIC_RESIDUAL_F_ZL");
    return e ? atoi(e) : 16;
  }();
  const int kc0 = fzl > 0 ? fzl : 16;
  const int kc = kc0 < g.nz ? kc0 : g.nz;
  dim3 grid = grid_cells((g.nx + 1) / 2, g.ny, g.nz);
  grid.z = (unsigned)((g.nz + kc - 1) / kc);
  static const int nt = [] {  // as residual(): MGIC_RESIDUAL_NT, default 3
    const char *e = getenv("MGIC_RESIDUAL_NT");
    return e ? atoi(e) : 3;
  }();
  // every value of MGIC_RESIDUAL_NT & 3, for both bCoef kinds, as residual()
#define MGIC_RZ2F(N)                                                                        \
  do {                                                                                      \
    if (fzl > 0) {                                                                          \
      uint4 lg;                                                                             \
      const dim3 xg = xcd_grid(grid, lg);                                                   \
      if (s.bconst) k_residual_zl<true, float, N><<<xg, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc, nullptr, lg); \
      else k_residual_zl<false, float, N><<<xg, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc, nullptr, lg);         \
    } else if (s.bconst) k_residual_z2<true, float, N><<<grid, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc); \
    else k_residual_z2<false, float, N><<<grid, kBlock, 0, st>>>(r, u, rhs, a, b, g, s, kc);         \
  } while (0)
  switch (nt & 3) {
    case 1: MGIC_RZ2F(1); break;
    case 2: MGIC_RZ2F(2); break;
    case 3: MGIC_RZ2F(3); break;
    default: MGIC_RZ2F(0); break;
  }
#undef MGIC_RZ2F
  check_launch();
}

void restrict_residual_f(float *rc, const BoxArgs &cg, const float *u, const float *rhs,
                         const float *a, const float *b, const BoxArgs &fg, const StencilCoefs &s,
                         hipStream_t st) {
  if (cg.nx <= 0 || cg.ny <= 0 || cg.nz <= 0) return;
  static const int nt = [] {  // as restrict_residual(): MGIC_RESTRICT_NT, default 1
    const char *e = getenv("MGIC_RESTRICT_NT");
    return e ? atoi(e) : 1;
  }();
  // k_restrict_zl<float>, two coarse planes per workgroup (MGIC_RESTRICT_F_ZL;
  // 0: k_restrict): 1024^3 mixed V-cycle 32.6 -> 32.0 ms, FMG 45.4 -> 44.1
  // (profiles/r05v_restrict_f_lds_ab.txt)
  static const int fzl = [] {
    const char *e = getenv("MGIC_RESTRICT_F_ZL");
    return e ? atoi(e) : 2;
  }();
  if (fzl > 0 && (nt & 1) && fg.nx == 2 * cg.nx && fg.ny == 2 * cg.ny && fg.nz == 2 * cg.nz) {
    const int ntx = (cg.nx + TX - 1) / TX, nty = (cg.ny + 3) / 4;
    const int kc = fzl < cg.nz ? fzl : cg.nz;
    const int nb = ntx * nty * ((cg.nz + kc - 1) / kc);
    if (s.bconst && (restrict_pre() & 2))
      k_restrict_zl<float, true, 1, true><<<nb, 256, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, 0, kc, ntx,
                                                              nty, restrict_f_xcd());
    else if (s.bconst)
      k_restrict_zl<float, true, 1><<<nb, 256, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, 0, kc, ntx, nty,
                                                        restrict_f_xcd());
    else
      k_restrict_zl<float, false, 1><<<nb, 256, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, 0, kc, ntx, nty,
                                                         restrict_f_xcd());
    check_launch();
    return;
  }
  const dim3 grid = grid_cells(cg.nx, cg.ny, cg.nz);
  if (s.bconst && (nt & 1))
    k_restrict<float, true, 1><<<grid, kBlock, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, 0);
  else if (s.bconst)
    k_restrict<float, true><<<grid, kBlock, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, 0);
  else if (nt & 1)
    k_restrict<float, false, 1><<<grid, kBlock, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, 0);
  else
    k_restrict<float, false><<<grid, kBlock, 0, st>>>(rc, cg, u, rhs, a, b, fg, s, 0);
  check_launch();
}

void prolong_f(float *uf, const BoxArgs &fg, const float *ec, const BoxArgs &cg,
               const int avail_lo[3], const int avail_hi[3], int type, hipStream_t st) {
  if (fg.nx <= 0 || fg.ny <= 0 || fg.nz <= 0) return;
  ProlongArgs pa;
  for (int d = 0; d < 3; ++d) {
    pa.avail_lo[d] = avail_lo[d];
    pa.avail_hi[d] = avail_hi[d];
  }
  MGIC_CHECK(fg.nx == 2 * cg.nx && fg.ny == 2 * cg.ny && fg.nz == 2 * cg.nz,
             "prolong: fine box must be the coarse box refined by 2");
  if (type == 1)
    k_prolong<float, 1><<<grid_cells(cg.nx, cg.ny, cg.nz), kBlock, 0, st>>>(uf, fg, ec, cg, pa);
  else
    k_prolong<float, 0><<<grid_cells(cg.nx, cg.ny, cg.nz), kBlock, 0, st>>>(uf, fg, ec, cg, pa);
  check_launch();
}

void copy_items_f(const CopyItem *d_items, int nitems, long max_cells, float *const *src_tab,
                  const float *src_buf, float *const *dst_tab, float *dst_buf, hipStream_t st) {
  if (nitems <= 0 || max_cells <= 0) return;
  const long per = 256L * copy_ept();
  long bx = (max_cells + per - 1) / per;
  if (bx > 1024) bx = 1024;
  k_copy_items<float><<<dim3((unsigned)bx, (unsigned)nitems), dim3(256), 0, st>>>(
      d_items, src_tab, src_buf, dst_tab, dst_buf);
  check_launch();
}

void to_float(float *d, const double *s, const BoxArgs &g, int grow, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  k_to_float<<<grid_cells(g.nx + 2 * grow, g.ny + 2 * grow, g.nz + 2 * grow), kBlock, 0, st>>>(
      d, s, g, grow);
  check_launch();
}

void cf_interp(double *u, const double *coarse_stage, const BoxArgs &g, const CFArgs &c,
               bool homogeneous, hipStream_t st) {
  const int dir = c.face >> 1;
  const int n[3] = {g.nx, g.ny, g.nz};
  const int d0 = dir == 0 ? 1 : 0, d1 = dir == 2 ? 1 : 2;
  if (n[dir] < 2) throw Error(kBadArg, "cf_interp: a box needs 2 cells normal to a CF face");
  const dim3 grid((unsigned)((n[d0] + 255) / 256), (unsigned)n[d1]);
  if (homogeneous) k_cf_interp<true><<<grid, 256, 0, st>>>(u, coarse_stage, g, c);
  else k_cf_interp<false><<<grid, 256, 0, st>>>(u, coarse_stage, g, c);
  check_launch();
}

void incr_f(double *x, const float *y, const BoxArgs &g, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  k_incr_f<<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st>>>(x, y, g);
  check_launch();
}

void copy_f(float *d, const float *s, const BoxArgs &g, hipStream_t st) {
  if (g.nx <= 0 || g.ny <= 0 || g.nz <= 0) return;
  k_copy_f<<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st>>>(d, s, g);
  check_launch();
}


// ---- BiCGStab on the device: launchers (kernels above; the reductions use
// reduce_blocks(g) blocks, as the host loop's partials do)
int bicg_dev_parts(const BoxArgs &g) { return (int)reduce_blocks(g); }

void bicg_dev_p(BicgState *st, double *p, double *w, const double *v, const double *r,
                const double *lam, const BoxArgs &g, hipStream_t st_) {
  k_bicgd_p<<<grid_cells(g.nx, g.ny, g.nz), kBlock, 0, st_>>>(st, p, w, v, r, lam, g);
  check_launch();
}

void bicg_dev_apply_dot(BicgState *st, double *v, const double *pt, const double *rt,
                        const double *a, const double *b, const BoxArgs &g, const StencilCoefs &s,
                        double *parts, unsigned int *cnt, hipStream_t st_) {
  const dim3 grid((unsigned)reduce_blocks(g)), block(RB);
  cnt += 0 * kBicgCntWords;
  if (s.bconst) k_bicgd_apply_dot<true><<<grid, block, 0, st_>>>(st, v, pt, rt, a, b, g, s, parts, cnt);
  else k_bicgd_apply_dot<false><<<grid, block, 0, st_>>>(st, v, pt, rt, a, b, g, s, parts, cnt);
  check_launch();
}

void bicg_dev_s(BicgState *st, double *s, double *w, const double *r, const double *v,
                const double *lam, const BoxArgs &g, int norm_kind, double *parts,
                unsigned int *cnt, hipStream_t st_) {
  const dim3 grid((unsigned)reduce_blocks(g)), block(RB);
  cnt += 1 * kBicgCntWords;
  switch (norm_kind) {
    case 1: k_bicgd_s<1><<<grid, block, 0, st_>>>(st, s, w, r, v, lam, g, parts, cnt); break;
    case 2: k_bicgd_s<2><<<grid, block, 0, st_>>>(st, s, w, r, v, lam, g, parts, cnt); break;
    case 3: k_bicgd_s<3><<<grid, block, 0, st_>>>(st, s, w, r, v, lam, g, parts, cnt); break;
    default: throw Error(kBadArg, "bicg_dev_s: bad norm kind");
  }
  check_launch();
}

void bicg_dev_apply_dot2(BicgState *st, const double *stv, const double *s, const double *a,
                         const double *b, const BoxArgs &g, const StencilCoefs &sc,
                         double *parts_ts, double *parts_tt, unsigned int *cnt, hipStream_t st_) {
  const dim3 grid((unsigned)reduce_blocks(g)), block(RB);
  cnt += 2 * kBicgCntWords;
  if (sc.bconst)
    k_bicgd_apply_dot2<true><<<grid, block, 0, st_>>>(st, stv, s, a, b, g, sc, parts_ts, parts_tt,
                                                      cnt);
  else
    k_bicgd_apply_dot2<false><<<grid, block, 0, st_>>>(st, stv, s, a, b, g, sc, parts_ts, parts_tt,
                                                       cnt);
  check_launch();
}

void bicg_dev_r(BicgState *st, double *r, double *e, const double *s, const double *a,
                const double *b, const StencilCoefs &sc, const double *pt, const double *stv,
                const double *rt, const BoxArgs &g, int norm_kind, double *parts_n,
                double *parts_d, unsigned int *cnt, hipStream_t st_) {
  const dim3 grid((unsigned)reduce_blocks(g)), block(RB);
  cnt += 3 * kBicgCntWords;
#define MGIC_BICG_R(K, BC)                                                                   \
  k_bicgd_r<K, BC><<<grid, block, 0, st_>>>(st, r, e, s, a, b, sc, pt, stv, rt, g, parts_n,  \
                                            parts_d, cnt)
  switch (norm_kind * 2 + (sc.bconst ? 1 : 0)) {
    case 2: MGIC_BICG_R(1, false); break;
    case 3: MGIC_BICG_R(1, true); break;
    case 4: MGIC_BICG_R(2, false); break;
    case 5: MGIC_BICG_R(2, true); break;
    case 6: MGIC_BICG_R(3, false); break;
    case 7: MGIC_BICG_R(3, true); break;
    default: throw Error(kBadArg, "bicg_dev_r: bad norm kind");
  }
#undef MGIC_BICG_R
  check_launch();
}

void bicg_dev_publish(const BicgState *st, BicgState *host, unsigned long long *seq,
                      unsigned long long seqv, hipStream_t st_) {
  k_bicgd_publish<<<1, 64, 0, st_>>>(st, host, seq, seqv);
  check_launch();
}

}  // namespace kern
}  // namespace mgic
