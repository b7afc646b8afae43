// smoother.hip -- fused red+black GSRB sweep for gfx950.
//
// One launch performs both colour passes of levelGSRB
// (Source/VariableCoeffPoissonOperator.cpp:290-331; arithmetic of
// GSRBHELMHOLTZVC3D, VariableCoeffPoissonOperatorF.ChF:56-139) on a box whose
// six faces are all domain faces with a folded BC (one box per level).
//
// Design (HBM-bound stencil, ~0.3 flop/B, no MFMA):
//   * a workgroup owns a TX x TY tile of (x, y) and streams a chunk of z
//     planes through a 4-slot LDS ring holding the tile plus a 2-cell halo;
//   * at step p it loads plane p+1, updates the RED cells of plane p on the
//     tile grown by one (the ring the black pass needs), then updates the
//     BLACK cells of plane p-1 and writes plane p-1 of the tile;
//   * out of place (u_in -> u_out): every workgroup reads only old values,
//     so overlapping halos never race; the caller alternates buffers;
//   * per sweep HBM traffic ~ read u, rhs, a, b + write u = 40 B/cell,
//     against 2 x 40 B/cell for two separate colour passes; lambda is
//     recomputed in registers, bit-identical to resetLambda.
// Results are bit-identical to two gsrb_pass launches (same expressions,
// -ffp-contract=off).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.hpp"

namespace mgic {
namespace kern {

namespace {

__device__ __forceinline__ double ghost_of(int mode, double c, double near) {
  return mode == kBcDirichlet ? (c - near) : (mode == kBcNeumannHom ? near : near + c);
}

constexpr int kThreads = 256;

// q ? x : y as an integer bit select: a "cond ? arr1[i] : arr0[i]" on
// register arrays is otherwise turned into a select of two stack addresses
// and lowered to scratch memory.  Exact (no arithmetic on the values).
__device__ __forceinline__ double bsel(int q, double x, double y) {
  const long long m = -(long long)(q & 1);
  return __longlong_as_double((__double_as_longlong(x) & m) | (__double_as_longlong(y) & ~m));
}

template <int TX, int TY>
__global__ __launch_bounds__(kThreads) void k_gsrb_fused(double *__restrict__ uo,
                                                         const double *__restrict__ ui,
                                                         const double *__restrict__ rhs,
                                                         const double *__restrict__ a,
                                                         const double *__restrict__ b,
                                                         const BoxArgs g, const StencilCoefs s,
                                                         int kc) {
  constexpr int LW = TX + 4, LH = TY + 4, LP = LW * LH;
  constexpr int HW = (TX + 2) / 2;     // red cells per ring row
  constexpr int NRED = HW * (TY + 2);  // red cells per ring plane
  __shared__ double U[4 * LP];

  const int x0 = blockIdx.x * TX, y0 = blockIdx.y * TY;
  const int z0 = blockIdx.z * kc;
  const int z1 = min(z0 + kc, g.nz);
  const int tid = threadIdx.x;
  const int gsum = g.glo[0] + g.glo[1] + g.glo[2];
  const long sy = g.sy, sz = g.sz;

  auto load = [&](int p) {
    if (p < 0 || p >= g.nz) return;
    double *S = U + (p & 3) * LP;
    const double *src = ui + (long)p * sz;
    for (int c = tid; c < LP; c += kThreads) {
      const int ly = c / LW, lx = c - ly * LW;
      const int gx = x0 - 2 + lx, gy = y0 - 2 + ly;
      if (gx >= 0 && gx < g.nx && gy >= 0 && gy < g.ny) S[c] = src[gx + gy * sy];
    }
  };

  // one GSRB update of cell (gx, gy, p) whose current value is uc, with
  // the neighbour values taken from the LDS planes (BC folded at faces)
  auto update = [&](const double *S, const double *Sm, const double *Sp, int ci, int gx, int gy,
                    int p, double uc) -> double {
    double xm = S[ci - 1], xp = S[ci + 1];
    double ym = S[ci - LW], yp = S[ci + LW];
    double zm = Sm[ci], zp = Sp[ci];
    if (gx == 0) xm = ghost_of(g.bcm[0], g.bcc[0], uc);
    if (gx == g.nx - 1) xp = ghost_of(g.bcm[1], g.bcc[1], uc);
    if (gy == 0) ym = ghost_of(g.bcm[2], g.bcc[2], uc);
    if (gy == g.ny - 1) yp = ghost_of(g.bcm[3], g.bcc[3], uc);
    if (p == 0) zm = ghost_of(g.bcm[4], g.bcc[4], uc);
    if (p == g.nz - 1) zp = ghost_of(g.bcm[5], g.bcc[5], uc);
    const double tx = (xp + xm) - 2.0 * uc;
    const double ty = (yp + ym) - 2.0 * uc;
    const double tz = (zp + zm) - 2.0 * uc;
    const double lap = (tx + ty) + tz;                          // .ChF:111-120
    const long idx = (long)gx + (long)gy * sy + (long)p * sz;
    const double av = a[idx];
    double lofdpsi = s.alpha * av * uc;                         // .ChF:107-108
    const double ldpsi = lap * s.dxinv * b[idx];                // .ChF:122
    lofdpsi = lofdpsi - s.beta * ldpsi;                         // .ChF:124
    const double lam = 1.0 / (av * s.alpha + s.lamshift);      // .cpp:234-243
    return uc - lam * (lofdpsi - rhs[idx]);                     // .ChF:127-128
  };

  load(z0 - 2);
  load(z0 - 1);
  for (int p = z0 - 1; p <= z1; ++p) {
    load(p + 1);
    __syncthreads();
    // RED (pass 0) on plane p over the tile grown by one cell
    if (p >= 0 && p < g.nz) {
      double *S = U + (p & 3) * LP;
      const double *Sm = U + ((p - 1) & 3) * LP;
      const double *Sp = U + ((p + 1) & 3) * LP;
      for (int c = tid; c < NRED; c += kThreads) {
        const int ry = c / HW, m = c - ry * HW;
        const int gy = y0 - 1 + ry;
        const int q = (x0 - 1 + gy + p + gsum) & 1;  // (gx+gy+p) even <=> red
        const int gx = x0 - 1 + 2 * m + q;
        if (gx < 0 || gx >= g.nx || gy < 0 || gy >= g.ny) continue;
        const int ci = (ry + 1) * LW + (gx - x0 + 2);
        S[ci] = update(S, Sm, Sp, ci, gx, gy, p, S[ci]);
      }
    }
    __syncthreads();
    // BLACK (pass 1) on plane k = p-1 over the tile, then store the plane
    const int k = p - 1;
    if (k >= z0 && k < z1) {
      const double *S = U + (k & 3) * LP;
      const double *Sm = U + ((k - 1) & 3) * LP;
      const double *Sp = U + ((k + 1) & 3) * LP;
      double *dst = uo + (long)k * sz;
      for (int c = tid; c < TX * TY; c += kThreads) {
        const int ty = c / TX, tx = c - ty * TX;
        const int gx = x0 + tx, gy = y0 + ty;
        if (gx >= g.nx || gy >= g.ny) continue;
        const int ci = (ty + 2) * LW + tx + 2;
        double v = S[ci];
        if ((gx + gy + k + gsum) & 1) v = update(S, Sm, Sp, ci, gx, gy, k, v);
        dst[gx + gy * sy] = v;
      }
    }
    __syncthreads();
  }
}

// v2: same algorithm, software-pipelined.  Plane p+2 of u and the
// rhs/aCoef/bCoef values of the next red and black cells are fetched into
// registers one step ahead; a 5-slot ring lets the next plane be stored
// while the black pass still reads the oldest one, so a step needs two
// barriers instead of three.
template <int TX, int TY, int NT>
__global__ __launch_bounds__(NT) void k_gsrb_fused2(double *__restrict__ uo,
                                                    const double *__restrict__ ui,
                                                    const double *__restrict__ rhs,
                                                    const double *__restrict__ a,
                                                    const double *__restrict__ b,
                                                    const BoxArgs g, const StencilCoefs s, int kc) {
  constexpr int LW = TX + 4, LH = TY + 4, LP = LW * LH;
  constexpr int HW = (TX + 2) / 2;
  constexpr int NRED = HW * (TY + 2);
  constexpr int NL = (LP + NT - 1) / NT;
  constexpr int NR = (NRED + NT - 1) / NT;
  constexpr int NB = (TX * TY + NT - 1) / NT;
  __shared__ double U[5 * LP];

  const int x0 = blockIdx.x * TX, y0 = blockIdx.y * TY;
  const int z0 = blockIdx.z * kc;
  const int z1 = min(z0 + kc, g.nz);
  const int tid = threadIdx.x;
  const int gsum = g.glo[0] + g.glo[1] + g.glo[2];
  const long sy = g.sy, sz = g.sz;
  auto slot = [](int p) { return ((p % 5) + 5) % 5; };

  double pu[NL];
  double rr[NR], ra[NR], rb[NR];
  double br[NB], ba[NB], bb[NB];

  auto fetch_u = [&](int p) {
    if (p < 0 || p >= g.nz) return;
    const double *src = ui + (long)p * sz;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = tid + i * NT;
      const int ly = c / LW, lx = c - ly * LW;
      const int gx = x0 - 2 + lx, gy = y0 - 2 + ly;
      if (c < LP && gx >= 0 && gx < g.nx && gy >= 0 && gy < g.ny) pu[i] = src[gx + gy * sy];
    }
  };
  auto put_u = [&](int p) {
    if (p < 0 || p >= g.nz) return;
    double *S = U + slot(p) * LP;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = tid + i * NT;
      const int ly = c / LW, lx = c - ly * LW;
      const int gx = x0 - 2 + lx, gy = y0 - 2 + ly;
      if (c < LP && gx >= 0 && gx < g.nx && gy >= 0 && gy < g.ny) S[c] = pu[i];
    }
  };
  // red cell i of plane p: (gx, gy) or gx = -1 when outside
  auto red_cell = [&](int i, int p, int &gx, int &gy) {
    const int c = tid + i * NT;
    const int ry = c / HW, m = c - ry * HW;
    gy = y0 - 1 + ry;
    gx = x0 - 1 + 2 * m + ((x0 - 1 + gy + p + gsum) & 1);
    if (c >= NRED || gx < 0 || gx >= g.nx || gy < 0 || gy >= g.ny) gx = -1;
  };
  auto fetch_red = [&](int p) {
    if (p < 0 || p >= g.nz) return;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      int gx, gy;
      red_cell(i, p, gx, gy);
      if (gx >= 0) {
        const long idx = (long)gx + (long)gy * sy + (long)p * sz;
        rr[i] = rhs[idx];
        ra[i] = a[idx];
        rb[i] = b[idx];
      }
    }
  };
  auto fetch_black = [&](int k) {
    if (k < z0 || k >= z1) return;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c = tid + i * NT;
      const int ty = c / TX, tx = c - ty * TX;
      const int gx = x0 + tx, gy = y0 + ty;
      if (c < TX * TY && gx < g.nx && gy < g.ny) {
        const long idx = (long)gx + (long)gy * sy + (long)k * sz;
        br[i] = rhs[idx];
        ba[i] = a[idx];
        bb[i] = b[idx];
      }
    }
  };
  auto update = [&](const double *S, const double *Sm, const double *Sp, int ci, int gx, int gy,
                    int p, double uc, double rv, double av, double bv) -> double {
    double xm = S[ci - 1], xp = S[ci + 1];
    double ym = S[ci - LW], yp = S[ci + LW];
    double zm = Sm[ci], zp = Sp[ci];
    if (gx == 0) xm = ghost_of(g.bcm[0], g.bcc[0], uc);
    if (gx == g.nx - 1) xp = ghost_of(g.bcm[1], g.bcc[1], uc);
    if (gy == 0) ym = ghost_of(g.bcm[2], g.bcc[2], uc);
    if (gy == g.ny - 1) yp = ghost_of(g.bcm[3], g.bcc[3], uc);
    if (p == 0) zm = ghost_of(g.bcm[4], g.bcc[4], uc);
    if (p == g.nz - 1) zp = ghost_of(g.bcm[5], g.bcc[5], uc);
    const double tx = (xp + xm) - 2.0 * uc;
    const double ty = (yp + ym) - 2.0 * uc;
    const double tz = (zp + zm) - 2.0 * uc;
    const double lap = (tx + ty) + tz;                       // .ChF:111-120
    double lofdpsi = s.alpha * av * uc;                      // .ChF:107-108
    const double ldpsi = lap * s.dxinv * bv;                 // .ChF:122
    lofdpsi = lofdpsi - s.beta * ldpsi;                      // .ChF:124
    const double lam = 1.0 / (av * s.alpha + s.lamshift);   // .cpp:234-243
    return uc - lam * (lofdpsi - rv);                        // .ChF:127-128
  };

  // prologue: planes z0-2, z0-1 in LDS, plane z0 in registers, coefficients
  // of red(z0-1) and black(z0) in registers
  fetch_u(z0 - 2);
  put_u(z0 - 2);
  fetch_u(z0 - 1);
  put_u(z0 - 1);
  fetch_u(z0);
  fetch_red(z0 - 1);
  fetch_black(z0);
  for (int p = z0 - 1; p <= z1; ++p) {
    put_u(p + 1);
    fetch_u(p + 2);
    __syncthreads();
    if (p >= 0 && p < g.nz) {  // RED on plane p, tile + 1 ring
      double *S = U + slot(p) * LP;
      const double *Sm = U + slot(p - 1) * LP;
      const double *Sp = U + slot(p + 1) * LP;
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        int gx, gy;
        red_cell(i, p, gx, gy);
        if (gx < 0) continue;
        const int ci = (gy - y0 + 2) * LW + (gx - x0 + 2);
        S[ci] = update(S, Sm, Sp, ci, gx, gy, p, S[ci], rr[i], ra[i], rb[i]);
      }
    }
    fetch_red(p + 1);
    __syncthreads();
    const int k = p - 1;
    if (k >= z0 && k < z1) {  // BLACK on plane k, tile; store plane k
      const double *S = U + slot(k) * LP;
      const double *Sm = U + slot(k - 1) * LP;
      const double *Sp = U + slot(k + 1) * LP;
      double *dst = uo + (long)k * sz;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int c = tid + i * NT;
        const int ty = c / TX, tx = c - ty * TX;
        const int gx = x0 + tx, gy = y0 + ty;
        if (c >= TX * TY || gx >= g.nx || gy >= g.ny) continue;
        const int ci = (ty + 2) * LW + tx + 2;
        double v = S[ci];
        if ((gx + gy + k + gsum) & 1) v = update(S, Sm, Sp, ci, gx, gy, k, v, br[i], ba[i], bb[i]);
        dst[gx + gy * sy] = v;
      }
    }
    fetch_black(p);
  }
}

// v4: colour-split LDS planes + x-pairs + XCD-aware tile order.
//  * A lane owns a pair of cells (x = 2m, 2m+1 of the region): one red and
//    one black cell per plane.  Global traffic is 16-byte double2 loads and
//    stores, and every rhs/aCoef/bCoef line is fetched once per plane: the
//    pair's coefficients are loaded one step ahead for the red update of
//    its red cell and kept in registers for its black cell one step later.
//  * LDS holds each plane as two colour arrays RED[r][m], BLK[r][m]: every
//    neighbour of a red cell is BLK[r][m-1..m+1], BLK[r+-1][m] or the same
//    m in the planes above/below (the colour flips with y and z), so the
//    reads are unit-stride across lanes (no bank conflicts) and the parity
//    is uniform along a row.
//  * Tiles are numbered x, then y, then z-chunk and handed out so that each
//    XCD (blockIdx % 8 share an L2) works on a contiguous band: vertical
//    neighbours, whose halos overlap, share an L2 and run at the same time.
template <int TX, int TY, int NT>
__global__ __launch_bounds__(NT) void k_gsrb_fused4(double *__restrict__ uo,
                                                    const double *__restrict__ ui,
                                                    const double *__restrict__ rhs,
                                                    const double *__restrict__ a,
                                                    const double *__restrict__ b,
                                                    const BoxArgs g, const StencilCoefs s, int kc,
                                                    int ntx, int nty, int nblocks) {
  static_assert(TX % 2 == 0, "TX must be even");
  constexpr int PW = TX / 2 + 2;      // pairs per region row: x in [x0-2, x0+TX+2)
  constexpr int LH = TY + 4;          // region rows: y in [y0-2, y0+TY+2)
  constexpr int CP = PW * LH;         // pairs per colour plane
  constexpr int NLP = CP;             // pairs loaded per plane
  constexpr int NRP = PW * (TY + 2);  // pairs on the ring rows y0-1 .. y0+TY
  constexpr int NL = (NLP + NT - 1) / NT;
  constexpr int NP = (NRP + NT - 1) / NT;
  __shared__ double R[5 * CP];
  __shared__ double B[5 * CP];

  // XCD-aware, bijective block -> tile map
  const int bid = blockIdx.x;
  const int q8 = nblocks / 8, r8 = nblocks % 8;
  const int xcd = bid % 8, i8 = bid / 8;
  const int L = xcd * q8 + min(xcd, r8) + i8;
  const int tx_ = L % ntx, ty_ = (L / ntx) % nty, tz_ = L / (ntx * nty);
  const int x0 = tx_ * TX, y0 = ty_ * TY;
  const int z0 = tz_ * kc;
  const int z1 = min(z0 + kc, g.nz);
  const int tid = threadIdx.x;
  const int gsum = g.glo[0] + g.glo[1] + g.glo[2];
  const long sy = g.sy, sz = g.sz;
  auto slot = [](int p) { return ((p % 5) + 5) % 5; };
  // red element (0/1) of the pairs of region row gy at plane p; pairs
  // start at even x, so this is uniform along the row
  auto redq = [&](int gy, int p) { return (x0 + gy + p + gsum) & 1; };

  // element 0 / element 1 of each pair kept as separate scalars: selecting
  // an element of a double2 by a runtime parity is lowered to scratch
  double pu0[NL], pu1[NL];
  double cr0[NP], cr1[NP], ca0[NP], ca1[NP], cb0[NP], cb1[NP];  // plane p (red now)
  double nr0[NP], nr1[NP], na0[NP], na1[NP], nb0[NP], nb1[NP];  // plane p+1 (prefetch)
  double kr[NP], ka[NP], kb[NP];                                // black elements of plane p-1

  auto ld2 = [&](const double *base, int gx, long off) -> double2 {
    if (gx + 1 < g.nx) return *reinterpret_cast<const double2 *>(base + off);
    double2 v;
    v.x = base[off];
    v.y = 0.0;
    return v;
  };
  auto fetch_u = [&](int p) {
    if (p < 0 || p >= g.nz) return;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = tid + i * NT;
      const int r = c / PW, m = c - r * PW;
      const int gx = x0 - 2 + 2 * m, gy = y0 - 2 + r;
      if (c < NLP && gx >= 0 && gx < g.nx && gy >= 0 && gy < g.ny) {
        const double2 v = ld2(ui, gx, (long)gx + (long)gy * sy + (long)p * sz);
        pu0[i] = v.x;
        pu1[i] = v.y;
      }
    }
  };
  auto put_u = [&](int p) {
    if (p < 0 || p >= g.nz) return;
    double *Rs = R + slot(p) * CP, *Bs = B + slot(p) * CP;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = tid + i * NT;
      const int r = c / PW, m = c - r * PW;
      const int gx = x0 - 2 + 2 * m, gy = y0 - 2 + r;
      if (c < NLP && gx >= 0 && gx < g.nx && gy >= 0 && gy < g.ny) {
        const int q = redq(gy, p);
        Rs[c] = q ? pu1[i] : pu0[i];
        Bs[c] = q ? pu0[i] : pu1[i];
      }
    }
  };
  auto fetch_c = [&](int p, double *r0, double *r1, double *a0, double *a1, double *b0,
                     double *b1) {
    if (p < 0 || p >= g.nz) return;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int c = tid + i * NT;
      const int rr = c / PW, m = c - rr * PW;
      const int gx = x0 - 2 + 2 * m, gy = y0 - 1 + rr;
      if (c < NRP && gx >= 0 && gx < g.nx && gy >= 0 && gy < g.ny) {
        const long off = (long)gx + (long)gy * sy + (long)p * sz;
        const double2 vr = ld2(rhs, gx, off), va = ld2(a, gx, off), vb = ld2(b, gx, off);
        r0[i] = vr.x;
        r1[i] = vr.y;
        a0[i] = va.x;
        a1[i] = va.y;
        b0[i] = vb.x;
        b1[i] = vb.y;
      }
    }
  };
  // GSRB update of a cell with value uc and the six neighbour values
  auto upd = [&](double uc, double xm, double xp, double ym, double yp, double zm, double zp,
                 int gx, int gy, int p, double rv, double av, double bv) -> double {
    if (gx == 0) xm = ghost_of(g.bcm[0], g.bcc[0], uc);
    if (gx == g.nx - 1) xp = ghost_of(g.bcm[1], g.bcc[1], uc);
    if (gy == 0) ym = ghost_of(g.bcm[2], g.bcc[2], uc);
    if (gy == g.ny - 1) yp = ghost_of(g.bcm[3], g.bcc[3], uc);
    if (p == 0) zm = ghost_of(g.bcm[4], g.bcc[4], uc);
    if (p == g.nz - 1) zp = ghost_of(g.bcm[5], g.bcc[5], uc);
    const double tx = (xp + xm) - 2.0 * uc;
    const double ty = (yp + ym) - 2.0 * uc;
    const double tz = (zp + zm) - 2.0 * uc;
    const double lap = (tx + ty) + tz;                       // .ChF:111-120
    double lofdpsi = s.alpha * av * uc;                      // .ChF:107-108
    const double ldpsi = lap * s.dxinv * bv;                 // .ChF:122
    lofdpsi = lofdpsi - s.beta * ldpsi;                      // .ChF:124
    const double lam = 1.0 / (av * s.alpha + s.lamshift);   // .cpp:234-243
    return uc - lam * (lofdpsi - rv);                        // .ChF:127-128
  };

  fetch_u(z0 - 2);
  put_u(z0 - 2);
  fetch_u(z0 - 1);
  put_u(z0 - 1);
  fetch_u(z0);
  fetch_c(z0 - 1, cr0, cr1, ca0, ca1, cb0, cb1);
  for (int p = z0 - 1; p <= z1; ++p) {
    put_u(p + 1);
    fetch_u(p + 2);
    fetch_c(p + 1, nr0, nr1, na0, na1, nb0, nb1);
    __syncthreads();
    // RED cells of plane p on the ring rows (x in [x0-1, x0+TX])
    if (p >= 0 && p < g.nz) {
      double *Rs = R + slot(p) * CP;
      const double *Bs = B + slot(p) * CP;
      const double *Bm = B + slot(p - 1) * CP;
      const double *Bp = B + slot(p + 1) * CP;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int c = tid + i * NT;
        const int rr = c / PW, m = c - rr * PW;
        const int gy = y0 - 1 + rr;
        const int q = redq(gy, p);
        const int gx = x0 - 2 + 2 * m + q;
        if (c < NRP && gx >= x0 - 1 && gx <= x0 + TX && gx >= 0 && gx < g.nx && gy >= 0 &&
            gy < g.ny) {
          const int ci = (rr + 1) * PW + m;
          const double xm = q ? Bs[ci] : Bs[ci - 1];
          const double xp = q ? Bs[ci + 1] : Bs[ci];
          Rs[ci] = upd(Rs[ci], xm, xp, Bs[ci - PW], Bs[ci + PW], Bm[ci], Bp[ci], gx, gy, p,
                       q ? cr1[i] : cr0[i], q ? ca1[i] : ca0[i], q ? cb1[i] : cb0[i]);
        }
      }
    }
    __syncthreads();
    // BLACK cells of plane k = p-1 on the tile; store the tile's pairs
    const int k = p - 1;
    if (k >= z0 && k < z1) {
      const double *Rs = R + slot(k) * CP;
      const double *Bs = B + slot(k) * CP;
      const double *Rm = R + slot(k - 1) * CP;
      const double *Rp = R + slot(k + 1) * CP;
      double *dst = uo + (long)k * sz;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int c = tid + i * NT;
        const int rr = c / PW, m = c - rr * PW;
        const int gy = y0 - 1 + rr;
        const int gx0 = x0 - 2 + 2 * m;
        if (c >= NRP || rr < 1 || rr > TY || m < 1 || m > TX / 2 || gx0 >= g.nx || gy >= g.ny)
          continue;
        const int qr = redq(gy, k), qb = 1 - qr;  // black element of the pair
        const int gx = gx0 + qb;
        const int ci = (rr + 1) * PW + m;
        const double red = Rs[ci];
        double blk = Bs[ci];
        if (gx < g.nx) {
          const double xm = qb ? Rs[ci] : Rs[ci - 1];
          const double xp = qb ? Rs[ci + 1] : Rs[ci];
          blk = upd(blk, xm, xp, Rs[ci - PW], Rs[ci + PW], Rm[ci], Rp[ci], gx, gy, k, kr[i], ka[i],
                    kb[i]);
        }
        if (gx0 + 1 < g.nx) {
          double2 w;
          w.x = qb ? red : blk;
          w.y = qb ? blk : red;
          *reinterpret_cast<double2 *>(dst + gx0 + (long)gy * sy) = w;
        } else {
          dst[gx0 + (long)gy * sy] = qb ? red : blk;
        }
      }
    }
    // rotate coefficients: keep plane p's black elements, advance plane p+1
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int c = tid + i * NT;
      const int rr = c / PW;
      const int qb = 1 - redq(y0 - 1 + rr, p);
      kr[i] = qb ? cr1[i] : cr0[i];
      ka[i] = qb ? ca1[i] : ca0[i];
      kb[i] = qb ? cb1[i] : cb0[i];
      cr0[i] = nr0[i];
      cr1[i] = nr1[i];
      ca0[i] = na0[i];
      ca1[i] = na1[i];
      cb0[i] = nb0[i];
      cb1[i] = nb1[i];
    }
  }
}

// v5: v4 with (1) the domain BC folded into the LDS planes when a plane is
// loaded -- a ghost next to a domain face is only ever read by the valid
// cell it mirrors, and always as f(old value of that cell) (DiriBC/NeumBC,
// SetBCs.cpp), so it is written once per plane and the update has no face
// tests -- and (2) all per-thread index arithmetic hoisted out of the z loop.
// LAMREAD reads the stored lambda instead of recomputing 1/(alpha a + shift).
template <int TX, int TY, int NT, bool LAMREAD>
__global__ __launch_bounds__(NT) void k_gsrb_fused5(double *__restrict__ uo,
                                                    const double *__restrict__ ui,
                                                    const double *__restrict__ rhs,
                                                    const double *__restrict__ a,
                                                    const double *__restrict__ b,
                                                    const double *__restrict__ lamp,
                                                    const BoxArgs g, const StencilCoefs s, int kc,
                                                    int ntx, int nty, int nblocks) {
  static_assert(TX % 2 == 0, "TX must be even");
  constexpr int PW = TX / 2 + 2;
  constexpr int LH = TY + 4;
  constexpr int CP = PW * LH;
  constexpr int NRP = PW * (TY + 2);
  constexpr int NL = (CP + NT - 1) / NT;
  constexpr int NP = (NRP + NT - 1) / NT;
  __shared__ double R[5 * CP];
  __shared__ double B[5 * CP];

  const int bid = blockIdx.x;
  const int q8 = nblocks / 8, r8 = nblocks % 8;
  const int xcd = bid % 8, i8 = bid / 8;
  const int L = xcd * q8 + min(xcd, r8) + i8;
  const int tx_ = L % ntx, ty_ = (L / ntx) % nty, tz_ = L / (ntx * nty);
  const int x0 = tx_ * TX, y0 = ty_ * TY;
  const int z0 = tz_ * kc;
  const int z1 = min(z0 + kc, g.nz);
  const int tid = threadIdx.x;
  const long sy = g.sy, sz = g.sz;
  const int nx = g.nx, ny = g.ny, nz = g.nz;
  auto slot = [](int p) { return ((p % 5) + 5) % 5; };
  const int q0 = (x0 + g.glo[0] + g.glo[1] + g.glo[2]) & 1;

  // ---- loop-invariant per-thread geometry
  // load slots: region pair (r, m); flags: fast = both elements and the row
  // inside the box (one double2 load)
  long loff[NL];
  int lgy[NL], lgx[NL], lok[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int c = tid + i * NT;
    const int r = c / PW, m = c - r * PW;
    lgx[i] = x0 - 2 + 2 * m;
    lgy[i] = y0 - 2 + r;
    loff[i] = (long)lgx[i] + (long)lgy[i] * sy;
    lok[i] = c < CP;
  }
  // ring slots: pair (rr, m) on rows y0-1 .. y0+TY
  long roff[NP];
  int rgy[NP], rgx0[NP], rci[NP], rflag[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int c = tid + i * NT;
    const int rr = c / PW, m = c - rr * PW;
    rgy[i] = y0 - 1 + rr;
    rgx0[i] = x0 - 2 + 2 * m;
    roff[i] = (long)rgx0[i] + (long)rgy[i] * sy;
    rci[i] = (rr + 1) * PW + m;
    const bool inrow = c < NRP && rgy[i] >= 0 && rgy[i] < ny;
    // bit0: coefficients to load (pair start inside), bit1: black-on-tile slot
    rflag[i] = (inrow && rgx0[i] >= 0 && rgx0[i] < nx ? 1 : 0) |
               (inrow && rr >= 1 && rr <= TY && m >= 1 && m <= TX / 2 && rgx0[i] < nx ? 2 : 0);
  }

  double pu0[NL], pu1[NL];
  double cr0[NP], cr1[NP], ca0[NP], ca1[NP], cb0[NP], cb1[NP], cl0[NP], cl1[NP];
  double nr0[NP], nr1[NP], na0[NP], na1[NP], nb0[NP], nb1[NP], nl0[NP], nl1[NP];
  double kr[NP], ka[NP], kb[NP], kl[NP];

  // value of region element (gx, gy) of plane p with the domain BC applied
  // to the first ghost layer (anything further out is never read)
  auto elem = [&](int gx, int gy, int p) -> double {
    const bool ix = gx >= 0 && gx < nx, iy = gy >= 0 && gy < ny, iz = p >= 0 && p < nz;
    const long pz = (long)p * sz;
    if (ix && iy && iz) return ui[(long)gx + (long)gy * sy + pz];
    if (iy && iz && gx == -1) return ghost_of(g.bcm[0], g.bcc[0], ui[(long)gy * sy + pz]);
    if (iy && iz && gx == nx) return ghost_of(g.bcm[1], g.bcc[1], ui[(long)(nx - 1) + (long)gy * sy + pz]);
    if (ix && iz && gy == -1) return ghost_of(g.bcm[2], g.bcc[2], ui[(long)gx + pz]);
    if (ix && iz && gy == ny) return ghost_of(g.bcm[3], g.bcc[3], ui[(long)gx + (long)(ny - 1) * sy + pz]);
    if (ix && iy && p == -1) return ghost_of(g.bcm[4], g.bcc[4], ui[(long)gx + (long)gy * sy]);
    if (ix && iy && p == nz)
      return ghost_of(g.bcm[5], g.bcc[5], ui[(long)gx + (long)gy * sy + (long)(nz - 1) * sz]);
    return 0.0;
  };
  auto fetch_u = [&](int p) {
    if (p < -1 || p > nz) return;
    const bool pin = p >= 0 && p < nz;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      if (!lok[i]) continue;
      if (pin && lgy[i] >= 0 && lgy[i] < ny && lgx[i] >= 0 && lgx[i] + 1 < nx) {
        const double2 v = *reinterpret_cast<const double2 *>(ui + loff[i] + (long)p * sz);
        pu0[i] = v.x;
        pu1[i] = v.y;
      } else {
        pu0[i] = elem(lgx[i], lgy[i], p);
        pu1[i] = elem(lgx[i] + 1, lgy[i], p);
      }
    }
  };
  auto put_u = [&](int p) {
    if (p < -1 || p > nz) return;
    double *Rs = R + slot(p) * CP, *Bs = B + slot(p) * CP;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      if (!lok[i]) continue;
      const int c = tid + i * NT;
      const int q = (q0 + lgy[i] + p) & 1;  // red element of the pair
      Rs[c] = bsel(q, pu1[i], pu0[i]);
      Bs[c] = bsel(q, pu0[i], pu1[i]);
    }
  };
  auto fetch_c = [&](int p, double *r0, double *r1, double *a0, double *a1, double *b0,
                     double *b1, double *l0, double *l1) {
    if (p < 0 || p >= nz) return;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      if (!(rflag[i] & 1)) continue;
      // the pair is 16-B aligned and its second element is at most the
      // ghost column x = nx, which every fab allocates: always one double2
      // load (a value past the box is never used)
      const long off = roff[i] + (long)p * sz;
      const double2 vr = *reinterpret_cast<const double2 *>(rhs + off);
      const double2 va = *reinterpret_cast<const double2 *>(a + off);
      const double2 vb = *reinterpret_cast<const double2 *>(b + off);
      r0[i] = vr.x; r1[i] = vr.y;
      a0[i] = va.x; a1[i] = va.y;
      b0[i] = vb.x; b1[i] = vb.y;
      if (LAMREAD) {
        const double2 vl = *reinterpret_cast<const double2 *>(lamp + off);
        l0[i] = vl.x; l1[i] = vl.y;
      }
    }
  };
  auto upd = [&](double uc, double xm, double xp, double ym, double yp, double zm, double zp,
                 double rv, double av, double bv, double lv) -> double {
    const double tx = (xp + xm) - 2.0 * uc;
    const double ty = (yp + ym) - 2.0 * uc;
    const double tz = (zp + zm) - 2.0 * uc;
    const double lap = (tx + ty) + tz;                                     // .ChF:111-120
    double lofdpsi = s.alpha * av * uc;                                    // .ChF:107-108
    const double ldpsi = lap * s.dxinv * bv;                               // .ChF:122
    lofdpsi = lofdpsi - s.beta * ldpsi;                                    // .ChF:124
    const double lam = LAMREAD ? lv : 1.0 / (av * s.alpha + s.lamshift);  // .cpp:234-243
    return uc - lam * (lofdpsi - rv);                                      // .ChF:127-128
  };

  fetch_u(z0 - 2);
  put_u(z0 - 2);
  fetch_u(z0 - 1);
  put_u(z0 - 1);
  fetch_u(z0);
  fetch_c(z0 - 1, cr0, cr1, ca0, ca1, cb0, cb1, cl0, cl1);
  for (int p = z0 - 1; p <= z1; ++p) {
    put_u(p + 1);
    fetch_u(p + 2);
    fetch_c(p + 1, nr0, nr1, na0, na1, nb0, nb1, nl0, nl1);
    __syncthreads();
    if (p >= 0 && p < nz) {  // RED cells of plane p on the ring
      double *Rs = R + slot(p) * CP;
      const double *Bs = B + slot(p) * CP;
      const double *Bm = B + slot(p - 1) * CP;
      const double *Bp = B + slot(p + 1) * CP;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int q = (q0 + rgy[i] + p) & 1;
        const int gx = rgx0[i] + q;
        if (!(rflag[i] & 1) || gx < x0 - 1 || gx > x0 + TX || gx >= nx) continue;
        const int ci = rci[i];
        const double xm = q ? Bs[ci] : Bs[ci - 1];
        const double xp = q ? Bs[ci + 1] : Bs[ci];
        Rs[ci] = upd(Rs[ci], xm, xp, Bs[ci - PW], Bs[ci + PW], Bm[ci], Bp[ci],
                     bsel(q, cr1[i], cr0[i]), bsel(q, ca1[i], ca0[i]), bsel(q, cb1[i], cb0[i]),
                     bsel(q, cl1[i], cl0[i]));
      }
    }
    __syncthreads();
    const int k = p - 1;
    if (k >= z0 && k < z1) {  // BLACK cells of plane k on the tile + store
      const double *Rs = R + slot(k) * CP;
      const double *Bs = B + slot(k) * CP;
      const double *Rm = R + slot(k - 1) * CP;
      const double *Rp = R + slot(k + 1) * CP;
      double *dst = uo + (long)k * sz;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        if (!(rflag[i] & 2)) continue;
        const int qb = 1 - ((q0 + rgy[i] + k) & 1);
        const int gx = rgx0[i] + qb;
        const int ci = rci[i];
        const double red = Rs[ci];
        double blk = Bs[ci];
        if (gx < nx) {
          const double xm = qb ? Rs[ci] : Rs[ci - 1];
          const double xp = qb ? Rs[ci + 1] : Rs[ci];
          blk = upd(blk, xm, xp, Rs[ci - PW], Rs[ci + PW], Rm[ci], Rp[ci], kr[i], ka[i], kb[i], kl[i]);
        }
        if (rgx0[i] + 1 < nx) {
          double2 w;
          w.x = qb ? red : blk;
          w.y = qb ? blk : red;
          *reinterpret_cast<double2 *>(dst + roff[i]) = w;
        } else {
          dst[roff[i]] = qb ? red : blk;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int qb = 1 - ((q0 + rgy[i] + p) & 1);
      kr[i] = bsel(qb, cr1[i], cr0[i]);
      ka[i] = bsel(qb, ca1[i], ca0[i]);
      kb[i] = bsel(qb, cb1[i], cb0[i]);
      kl[i] = bsel(qb, cl1[i], cl0[i]);
      cr0[i] = nr0[i]; cr1[i] = nr1[i];
      ca0[i] = na0[i]; ca1[i] = na1[i];
      cb0[i] = nb0[i]; cb1[i] = nb1[i];
      cl0[i] = nl0[i]; cl1[i] = nl1[i];
    }
  }
}

// v6: branch-free streaming.  The domain BC of the six faces is written into
// the input's ghost layer by one small launch before the sweep (a ghost is
// the BC image of the cell it touches, and that cell keeps its input value
// until its own colour is updated, so one fill serves both colour passes).
// Every global load is then unconditional, at an address clamped into the
// allocation: no divergent branch sits between issuing a load and the next
// plane, so the loads of plane p+2 (u) and p+1 (rhs, a, b) stay in flight
// across the red and black updates of planes p and p-1.
template <int TX, int TY, int NT>
struct Fused6 {
  static_assert(TX % 2 == 0, "TX must be even");
  static constexpr int PW = TX / 2 + 2;      // pairs per region row (x0-2 .. x0+TX+1)
  static constexpr int LH = TY + 4;          // region rows y0-2 .. y0+TY+1
  static constexpr int CP = PW * LH;         // pairs per plane
  static constexpr int NRP = PW * (TY + 2);  // ring pairs (rows y0-1 .. y0+TY)
  static constexpr int NL = (CP + NT - 1) / NT;
  static constexpr int NP = (NRP + NT - 1) / NT;
};

// One tile (x0, y0) of the box, planes [z0, z1): R/B are the 5-plane LDS
// rings (5 * CP doubles each) holding the red / black element of each pair.
template <int TX, int TY, int NT>
__device__ __forceinline__ void fused6_segment(double *__restrict__ R, double *__restrict__ B,
                                               double *__restrict__ uo,
                                               const double *__restrict__ ui,
                                               const double *__restrict__ rhs,
                                               const double *__restrict__ a,
                                               const double *__restrict__ b, const BoxArgs &g,
                                               const StencilCoefs &s, int x0, int y0, int z0,
                                               int z1) {
  using F = Fused6<TX, TY, NT>;
  constexpr int PW = F::PW, CP = F::CP, NRP = F::NRP, NL = F::NL, NP = F::NP;
  const int tid = threadIdx.x;
  const long sy = g.sy, sz = g.sz;
  const int nx = g.nx, ny = g.ny, nz = g.nz;
  const int xpmax = nx & ~1;  // last pair start that can hold a needed element
  const int q0 = (x0 + g.glo[0] + g.glo[1] + g.glo[2]) & 1;
  auto slot = [](int p) { return ((p % 5) + 5) % 5; };
  auto clampi = [](int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); };

  // region pairs owned by this thread (loads + LDS stores)
  long loff[NL];
  int lgy[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int c = tid + i * NT;
    const int r = c / PW, m = c - r * PW;
    lgy[i] = y0 - 2 + r;
    const int gx = min(x0 - 2 + 2 * m, xpmax);
    loff[i] = c < CP ? (long)gx + (long)clampi(lgy[i], -1, ny) * sy : 0;
  }
  // ring pairs owned by this thread (coefficient loads, red/black updates)
  long roff[NP], rcoff[NP];
  int rgy[NP], rgx0[NP], rci[NP], rrow[NP], rtile[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int c = tid + i * NT;
    const int rr = c / PW, m = c - rr * PW;
    rgy[i] = y0 - 1 + rr;
    rgx0[i] = x0 - 2 + 2 * m;
    roff[i] = (long)rgx0[i] + (long)rgy[i] * sy;
    rcoff[i] = c < NRP ? (long)min(rgx0[i], xpmax) + (long)clampi(rgy[i], -1, ny) * sy : 0;
    rci[i] = (rr + 1) * PW + m;
    rrow[i] = c < NRP && rgy[i] >= 0 && rgy[i] < ny;
    rtile[i] = rrow[i] && rr >= 1 && rr <= TY && m >= 1 && m <= TX / 2 && rgx0[i] < nx;
  }
  const int gxlo = max(x0 - 1, 0), gxhi = min(x0 + TX, nx - 1);  // red ring extent

  double pu0[NL], pu1[NL];
  double cr0[NP], cr1[NP], ca0[NP], ca1[NP], cb0[NP], cb1[NP];
  double nr0[NP], nr1[NP], na0[NP], na1[NP], nb0[NP], nb1[NP];
  double kr[NP], ka[NP], kb[NP];

  auto fetch_u = [&](int p) {
    const long pz = (long)clampi(p, -1, nz) * sz;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const double2 v = *reinterpret_cast<const double2 *>(ui + loff[i] + pz);
      pu0[i] = v.x;
      pu1[i] = v.y;
    }
  };
  auto put_u = [&](int p) {
    double *Rs = R + slot(p) * CP, *Bs = B + slot(p) * CP;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = tid + i * NT;
      if (NL * NT > CP && c >= CP) continue;
      const int q = (q0 + lgy[i] + p) & 1;  // 1: the red element is the second
      Rs[c] = bsel(q, pu1[i], pu0[i]);
      Bs[c] = bsel(q, pu0[i], pu1[i]);
    }
  };
  auto fetch_c = [&](int p) {
    const long pz = (long)clampi(p, 0, nz - 1) * sz;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const long off = rcoff[i] + pz;
      const double2 vr = *reinterpret_cast<const double2 *>(rhs + off);
      const double2 va = *reinterpret_cast<const double2 *>(a + off);
      const double2 vb = *reinterpret_cast<const double2 *>(b + off);
      nr0[i] = vr.x; nr1[i] = vr.y;
      na0[i] = va.x; na1[i] = va.y;
      nb0[i] = vb.x; nb1[i] = vb.y;
    }
  };
  auto upd = [&](double uc, double xm, double xp, double ym, double yp, double zm, double zp,
                 double rv, double av, double bv) -> double {
    const double tx = (xp + xm) - 2.0 * uc;
    const double ty = (yp + ym) - 2.0 * uc;
    const double tz = (zp + zm) - 2.0 * uc;
    const double lap = (tx + ty) + tz;                     // .ChF:111-120
    double lofdpsi = s.alpha * av * uc;                    // .ChF:107-108
    const double ldpsi = lap * s.dxinv * bv;               // .ChF:122
    lofdpsi = lofdpsi - s.beta * ldpsi;                    // .ChF:124
    const double lam = 1.0 / (av * s.alpha + s.lamshift);  // .cpp:234-243
    return uc - lam * (lofdpsi - rv);                      // .ChF:127-128
  };

  fetch_u(z0 - 2);
  put_u(z0 - 2);
  fetch_u(z0 - 1);
  put_u(z0 - 1);
  fetch_u(z0);
  fetch_c(z0 - 1);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    cr0[i] = nr0[i]; cr1[i] = nr1[i];
    ca0[i] = na0[i]; ca1[i] = na1[i];
    cb0[i] = nb0[i]; cb1[i] = nb1[i];
  }
  for (int p = z0 - 1; p <= z1; ++p) {
    put_u(p + 1);
    fetch_u(p + 2);
    fetch_c(p + 1);
    __syncthreads();
    if (p >= 0 && p < nz) {  // RED cells of plane p on the ring
      double *Rs = R + slot(p) * CP;
      const double *Bs = B + slot(p) * CP;
      const double *Bm = B + slot(p - 1) * CP;
      const double *Bp = B + slot(p + 1) * CP;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int q = (q0 + rgy[i] + p) & 1;
        const int gx = rgx0[i] + q;
        if (!rrow[i] || gx < gxlo || gx > gxhi) continue;
        const int ci = rci[i];
        const double xm = q ? Bs[ci] : Bs[ci - 1];
        const double xp = q ? Bs[ci + 1] : Bs[ci];
        Rs[ci] = upd(Rs[ci], xm, xp, Bs[ci - PW], Bs[ci + PW], Bm[ci], Bp[ci],
                     bsel(q, cr1[i], cr0[i]), bsel(q, ca1[i], ca0[i]), bsel(q, cb1[i], cb0[i]));
      }
    }
    __syncthreads();
    const int k = p - 1;
    if (k >= z0 && k < z1) {  // BLACK cells of plane k on the tile + store
      const double *Rs = R + slot(k) * CP;
      const double *Bs = B + slot(k) * CP;
      const double *Rm = R + slot(k - 1) * CP;
      const double *Rp = R + slot(k + 1) * CP;
      double *dst = uo + (long)k * sz;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        if (!rtile[i]) continue;
        const int qb = 1 - ((q0 + rgy[i] + k) & 1);  // 1: the black element is the second
        const int gx = rgx0[i] + qb;
        const int ci = rci[i];
        const double red = Rs[ci];
        double blk = Bs[ci];
        if (gx < nx) {
          const double xm = qb ? Rs[ci] : Rs[ci - 1];
          const double xp = qb ? Rs[ci + 1] : Rs[ci];
          blk = upd(blk, xm, xp, Rs[ci - PW], Rs[ci + PW], Rm[ci], Rp[ci], kr[i], ka[i], kb[i]);
        }
        if (rgx0[i] + 1 < nx) {
          double2 w;
          w.x = bsel(qb, red, blk);
          w.y = bsel(qb, blk, red);
          *reinterpret_cast<double2 *>(dst + roff[i]) = w;
        } else {
          dst[roff[i]] = bsel(qb, red, blk);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NP; ++i) {  // plane p's black coefficients wait one step
      const int qb = 1 - ((q0 + rgy[i] + p) & 1);
      kr[i] = bsel(qb, cr1[i], cr0[i]);
      ka[i] = bsel(qb, ca1[i], ca0[i]);
      kb[i] = bsel(qb, cb1[i], cb0[i]);
      cr0[i] = nr0[i]; cr1[i] = nr1[i];
      ca0[i] = na0[i]; ca1[i] = na1[i];
      cb0[i] = nb0[i]; cb1[i] = nb1[i];
    }
  }
}

template <int TX, int TY, int NT>
__global__ __launch_bounds__(NT) void k_gsrb_fused6(double *__restrict__ uo,
                                                    const double *__restrict__ ui,
                                                    const double *__restrict__ rhs,
                                                    const double *__restrict__ a,
                                                    const double *__restrict__ b,
                                                    const BoxArgs g, const StencilCoefs s, int kc,
                                                    int ntx, int nty, int nblocks) {
  using F = Fused6<TX, TY, NT>;
  __shared__ double R[5 * F::CP];  // red element of every pair, 5-plane ring
  __shared__ double B[5 * F::CP];  // black element
  const int bid = blockIdx.x;      // XCD-aware: consecutive tiles on one XCD
  const int q8 = nblocks / 8, r8 = nblocks % 8;
  const int xcd = bid % 8, i8 = bid / 8;
  const int L = xcd * q8 + min(xcd, r8) + i8;
  const int tx_ = L % ntx, ty_ = (L / ntx) % nty, tz_ = L / (ntx * nty);
  const int z0 = tz_ * kc;
  fused6_segment<TX, TY, NT>(R, B, uo, ui, rhs, a, b, g, s, tx_ * TX, ty_ * TY, z0,
                             min(z0 + kc, g.nz));
}

// v7: persistent.  Exactly as many workgroups as fit on the chip at once;
// the (slab, tile, plane) units are dealt out in equal contiguous ranges
// (a range may span tiles), so no partial last round of workgroups idles
// most of the CUs.  Slabs of zs planes keep the tiles in flight together
// at similar z (shared halos in L2).
template <int TX, int TY, int NT>
__global__ __launch_bounds__(NT) void k_gsrb_fused7(double *__restrict__ uo,
                                                    const double *__restrict__ ui,
                                                    const double *__restrict__ rhs,
                                                    const double *__restrict__ a,
                                                    const double *__restrict__ b,
                                                    const BoxArgs g, const StencilCoefs s, int zs,
                                                    int ntx, int nty, int nblocks) {
  using F = Fused6<TX, TY, NT>;
  __shared__ double R[5 * F::CP];
  __shared__ double B[5 * F::CP];
  const int bid = blockIdx.x;
  const int q8 = nblocks / 8, r8 = nblocks % 8;
  const int xcd = bid % 8, i8 = bid / 8;
  const long L = xcd * q8 + min(xcd, r8) + i8;
  const long T = (long)ntx * nty;
  const long W = T * g.nz;
  const int nfull = g.nz / zs, rem = g.nz - nfull * zs;
  long u = L * W / nblocks;
  const long end = (L + 1) * W / nblocks;
  while (u < end) {
    long t;
    int z, len;
    if (u < (long)nfull * T * zs) {
      const long sl = u / (T * zs), r = u - sl * T * zs;
      t = r / zs;
      const int zi = (int)(r - t * zs);
      z = (int)sl * zs + zi;
      len = zs - zi;
    } else {
      const long r = u - (long)nfull * T * zs;
      t = r / rem;
      const int zi = (int)(r - t * rem);
      z = nfull * zs + zi;
      len = rem - zi;
    }
    if ((long)len > end - u) len = (int)(end - u);
    const int tx_ = (int)(t % ntx), ty_ = (int)(t / ntx);
    fused6_segment<TX, TY, NT>(R, B, uo, ui, rhs, a, b, g, s, tx_ * TX, ty_ * TY, z, z + len);
    u += len;
    __syncthreads();  // the next segment refills the rings
  }
}

// All six face ghost layers of one box in one launch (faces with a BC only;
// each face writes its own ghost cells, edges and corners are untouched).
__global__ void k_fill_bc_faces(double *__restrict__ u, const BoxArgs g) {
  const int face = blockIdx.z;
  if (!g.bcm[face]) return;
  const int dir = face >> 1, side = face & 1;
  const int n0 = dir == 0 ? g.ny : g.nx;  // fastest in-face direction
  const int n1 = dir == 2 ? g.ny : g.nz;
  const int a0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int a1 = blockIdx.y;
  if (a0 >= n0 || a1 >= n1) return;
  int c[3];
  c[dir] = side == 0 ? 0 : (dir == 0 ? g.nx : dir == 1 ? g.ny : g.nz) - 1;
  c[dir == 0 ? 1 : 0] = a0;
  c[dir == 2 ? 1 : 2] = a1;
  const long st = dir == 0 ? 1 : dir == 1 ? g.sy : g.sz;
  const long near = (long)c[0] + (long)c[1] * g.sy + (long)c[2] * g.sz;
  u[near + (side == 0 ? -st : st)] = ghost_of(g.bcm[face], g.bcc[face], u[near]);
}

}  // namespace

bool gsrb_sweep_fused_supported(const BoxArgs &g) {
  for (int f = 0; f < 6; ++f)
    if (g.bcm[f] == kBcMemory) return false;  // needs every face BC-folded
  return g.nx > 0 && g.ny > 0 && g.nz > 0;
}

template <class K>
static void launch_fused(K kern_fn, int TX, int TY, int NT, double *u_out, const double *u_in,
                         const double *rhs, const double *a, const double *b, const BoxArgs &g,
                         const StencilCoefs &s, hipStream_t st) {
  const int tiles = ((g.nx + TX - 1) / TX) * ((g.ny + TY - 1) / TY);
  int kc = g.nz;  // z-chunk: enough workgroups to fill 256 CUs several times over
  while (kc > 16 && (long)tiles * ((g.nz + kc - 1) / kc) < 4096) kc = (kc + 1) / 2;
  const dim3 grid((unsigned)((g.nx + TX - 1) / TX), (unsigned)((g.ny + TY - 1) / TY),
                  (unsigned)((g.nz + kc - 1) / kc));
  kern_fn<<<grid, dim3(NT), 0, st>>>(u_out, u_in, rhs, a, b, g, s, kc);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(kHipErr, std::string("fused sweep launch: ") + hipGetErrorString(e));
}

template <int TX, int TY, int NT>
static void launch_fused4(double *u_out, const double *u_in, const double *rhs, const double *a,
                          const double *b, const BoxArgs &g, const StencilCoefs &s, hipStream_t st) {
  const int ntx = (g.nx + TX - 1) / TX, nty = (g.ny + TY - 1) / TY;
  int kc = g.nz;
  while (kc > 16 && (long)ntx * nty * ((g.nz + kc - 1) / kc) < 3072) kc = (kc + 1) / 2;
  const int ntz = (g.nz + kc - 1) / kc;
  const int nblocks = ntx * nty * ntz;
  k_gsrb_fused4<TX, TY, NT><<<dim3((unsigned)nblocks), dim3(NT), 0, st>>>(u_out, u_in, rhs, a, b, g,
                                                                          s, kc, ntx, nty, nblocks);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(kHipErr, std::string("fused sweep launch: ") + hipGetErrorString(e));
}

template <int TX, int TY, int NT, bool LAMREAD>
static void launch_fused5(double *u_out, const double *u_in, const double *rhs, const double *a,
                          const double *b, const double *lam, const BoxArgs &g,
                          const StencilCoefs &s, hipStream_t st) {
  const int ntx = (g.nx + TX - 1) / TX, nty = (g.ny + TY - 1) / TY;
  int kc = g.nz;
  while (kc > 16 && (long)ntx * nty * ((g.nz + kc - 1) / kc) < 3072) kc = (kc + 1) / 2;
  const int ntz = (g.nz + kc - 1) / kc;
  const int nblocks = ntx * nty * ntz;
  k_gsrb_fused5<TX, TY, NT, LAMREAD><<<dim3((unsigned)nblocks), dim3(NT), 0, st>>>(
      u_out, u_in, rhs, a, b, lam, g, s, kc, ntx, nty, nblocks);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(kHipErr, std::string("fused sweep launch: ") + hipGetErrorString(e));
}

template <int TX, int TY, int NT>
static void launch_fused6(double *u_out, double *u_in, const double *rhs, const double *a,
                          const double *b, const BoxArgs &g, const StencilCoefs &s, hipStream_t st) {
  const int m = g.nx > g.ny ? g.nx : g.ny;
  const int m1 = g.ny > g.nz ? g.ny : g.nz;
  k_fill_bc_faces<<<dim3((unsigned)((m + 255) / 256), (unsigned)m1, 6), dim3(256), 0, st>>>(u_in, g);
  const int ntx = (g.nx + TX - 1) / TX, nty = (g.ny + TY - 1) / TY;
  int kc = g.nz;
  while (kc > 16 && (long)ntx * nty * ((g.nz + kc - 1) / kc) < 3072) kc = (kc + 1) / 2;
  const int ntz = (g.nz + kc - 1) / kc;
  const int nblocks = ntx * nty * ntz;
  k_gsrb_fused6<TX, TY, NT><<<dim3((unsigned)nblocks), dim3(NT), 0, st>>>(u_out, u_in, rhs, a, b, g,
                                                                          s, kc, ntx, nty, nblocks);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(kHipErr, std::string("fused sweep launch: ") + hipGetErrorString(e));
}

template <int TX, int TY, int NT>
static void launch_fused7(double *u_out, double *u_in, const double *rhs, const double *a,
                          const double *b, const BoxArgs &g, const StencilCoefs &s, hipStream_t st) {
  static const int slots = [] {
    int dev = 0, ncu = 0, per = 0;
    MGIC_HIP(hipGetDevice(&dev));
    MGIC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    MGIC_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_gsrb_fused7<TX, TY, NT>, NT, 0));
    return (per > 0 ? per : 1) * ncu;
  }();
  static const int zs_env = [] {
    const char *e = getenv("MGIC_FUSED_ZS");
    return e ? atoi(e) : 0;
  }();
  const int m = g.nx > g.ny ? g.nx : g.ny;
  const int m1 = g.ny > g.nz ? g.ny : g.nz;
  k_fill_bc_faces<<<dim3((unsigned)((m + 255) / 256), (unsigned)m1, 6), dim3(256), 0, st>>>(u_in, g);
  const int ntx = (g.nx + TX - 1) / TX, nty = (g.ny + TY - 1) / TY;
  const long units = (long)ntx * nty * g.nz;
  const int zs = zs_env > 0 && zs_env < g.nz ? zs_env : g.nz;
  // at least ~8 planes per workgroup, else the ring prologue dominates
  long nb = slots;
  if (nb > units / 8) nb = units / 8 > 0 ? units / 8 : 1;
  const int nblocks = (int)nb;
  k_gsrb_fused7<TX, TY, NT><<<dim3((unsigned)nblocks), dim3(NT), 0, st>>>(u_out, u_in, rhs, a, b, g,
                                                                          s, zs, ntx, nty, nblocks);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(kHipErr, std::string("fused sweep launch: ") + hipGetErrorString(e));
}

static int fused_variant() {
  static int v = [] {
    const char *e = getenv("MGIC_FUSED_VARIANT");
    return e ? atoi(e) : 15;
  }();
  return v;
}

void gsrb_sweep_fused(double *u_out, double *u_in, const double *rhs, const double *a,
                      const double *b, const double *lam, const BoxArgs &g, const StencilCoefs &s,
                      hipStream_t st) {
  switch (fused_variant()) {
    case 0: launch_fused(k_gsrb_fused<64, 8>, 64, 8, kThreads, u_out, u_in, rhs, a, b, g, s, st); break;
    case 2: launch_fused(k_gsrb_fused2<64, 16, 512>, 64, 16, 512, u_out, u_in, rhs, a, b, g, s, st); break;
    case 3: launch_fused(k_gsrb_fused2<64, 4, 256>, 64, 4, 256, u_out, u_in, rhs, a, b, g, s, st); break;
    case 4: launch_fused(k_gsrb_fused2<128, 8, 512>, 128, 8, 512, u_out, u_in, rhs, a, b, g, s, st); break;
    case 5: launch_fused4<60, 12, 256>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 6: launch_fused4<60, 8, 256>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 7: launch_fused4<124, 6, 256>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 8: launch_fused4<60, 28, 512>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 9: launch_fused4<28, 12, 128>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 10: launch_fused5<60, 12, 256, false>(u_out, u_in, rhs, a, b, nullptr, g, s, st); break;
    case 11: launch_fused5<60, 12, 256, true>(u_out, u_in, rhs, a, b, lam, g, s, st); break;
    case 12: launch_fused5<60, 8, 256, false>(u_out, u_in, rhs, a, b, nullptr, g, s, st); break;
    case 13: launch_fused5<124, 6, 256, false>(u_out, u_in, rhs, a, b, nullptr, g, s, st); break;
    case 14: launch_fused6<60, 12, 256>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 15: launch_fused6<60, 8, 256>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 16: launch_fused6<124, 6, 256>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 17: launch_fused6<60, 28, 512>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 18: launch_fused6<124, 12, 512>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 19: launch_fused6<28, 12, 128>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 20: launch_fused7<60, 12, 256>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 21: launch_fused7<60, 8, 256>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 22: launch_fused7<124, 12, 512>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 23: launch_fused7<60, 28, 512>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 24: launch_fused7<124, 6, 256>(u_out, u_in, rhs, a, b, g, s, st); break;
    case 1: launch_fused(k_gsrb_fused2<64, 8, 256>, 64, 8, 256, u_out, u_in, rhs, a, b, g, s, st); break;
    default: launch_fused6<60, 8, 256>(u_out, u_in, rhs, a, b, g, s, st); break;
  }
}

}  // namespace kern
}  // namespace mgic
