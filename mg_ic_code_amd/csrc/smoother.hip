// smoother.hip -- fused red+black GSRB sweep for gfx950.
//
// One launch performs both colour passes of levelGSRB
// (Source/VariableCoeffPoissonOperator.cpp:290-331; arithmetic of
// GSRBHELMHOLTZVC3D, VariableCoeffPoissonOperatorF.ChF:56-139) on one box:
// domain faces take the BC on the fly, exchanged faces read a 2-deep ghost
// shell (see gsrb_sweep_fused in kernels.hpp).  Results are bit-identical to two per-colour k_gsrb launches (same
// expressions, -ffp-contract=off).
//
// Design (HBM-bound stencil, ~0.3 flop/B, no MFMA):
//   * a workgroup owns a TX x TY (x, y) tile and streams a chunk of z planes
//     through a 5-plane LDS ring holding the tile plus a 2-cell halo; red
//     and black elements of each x-pair live in separate LDS arrays (R, B),
//     so every LDS access is stride-1 and a pair is one 16-B global load;
//   * at step p: store plane p+1 (loaded last step) into the ring, issue the
//     loads of u plane p+2 and rhs/a/b plane p+1, update the RED cells of
//     plane p on the tile grown by one (the ring the black pass reads), then
//     the BLACK cells of plane p-1 on the tile, and store plane p-1;
//   * out of place (u_in -> u_out): every workgroup reads only old values, so
//     overlapping halos never race; the caller alternates two buffers;
//   * lambda is recomputed in registers (bit-identical to resetLambda), so
//     the compulsory traffic is 40 B/cell (u, rhs, a, b in, u out) against
//     2 x 48 B/cell for two per-colour passes.
//
// What the earlier variants taught (git history has them):
//   * a z-streaming kernel with conditional (bounds / BC) loads was latency
//     bound at ~1.45 ms / 512^3 sweep: loads whose results merge at a join
//     point got an s_waitcnt vmcnt(0) right after issue, so nothing stayed in
//     flight across the barriers.  Hence unconditional clamped loads here and
//     the BC applied as planes enter LDS (ghost pairs load the cells they
//     image and transform them; an earlier separate fill launch cost ~4%);
//   * `cond ? arr1[i] : arr0[i]` on register arrays (and runtime-indexed
//     double2 elements) is lowered to scratch: use bsel() on scalars;
//   * a persistent grid (exactly one wave of workgroups, equal contiguous
//     ranges) removed the tail but lost the L2 halo sharing of neighbouring
//     tiles running together and was slower; the XCD-aware tile order below
//     keeps neighbouring tiles on one XCD.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.hpp"
#include "sweep_util.hpp"

namespace mgic {
namespace kern {

namespace {

using sweep::bsel;
using sweep::ghost_of;

// element type traits: a lane pair is one 16-B (double) / 8-B (float) load
template <class T> struct Vec2;
template <> struct Vec2<double> { using type = double2; };
template <> struct Vec2<float> { using type = float2; };
template <class T> using V2 = typename Vec2<T>::type;
template <class T>
__device__ __forceinline__ V2<T> mk2(T x, T y) {
  V2<T> v;
  v.x = x;
  v.y = y;
  return v;
}

// the stencil constants in the element type (fp32 sweeps round each once;
// for double this is the identity, so the fp64 kernels are unchanged)
template <class T>
struct SC {
  T alpha, beta, dxinv, lamshift, bval;
  __device__ explicit SC(const StencilCoefs &s)
      : alpha((T)s.alpha), beta((T)s.beta), dxinv((T)s.dxinv), lamshift((T)s.lamshift),
        bval((T)s.bval) {}
};

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
template <class T, int TX, int TY, int NT, bool ZIN, bool BC, bool ACC>
__device__ __forceinline__ void fused6_segment(T *__restrict__ R, T *__restrict__ B,
                                               T *__restrict__ uo,
                                               double *__restrict__ acc,
                                               const T *__restrict__ ui,
                                               const T *__restrict__ rhs,
                                               const T *__restrict__ a,
                                               const T *__restrict__ b, const BoxArgs &g,
                                               const StencilCoefs &s64, int x0, int y0, int z0,
                                               int z1) {
  using F = Fused6<TX, TY, NT>;
  const SC<T> s(s64);
  constexpr int PW = F::PW, CP = F::CP, NRP = F::NRP, NL = F::NL, NP = F::NP;
  const int tid = threadIdx.x;
  const long sy = g.sy, sz = g.sz;
  const int nx = g.nx, ny = g.ny, nz = g.nz;
  // last pair start that can hold a needed element (x <= nx + 1); a pair
  // past the row end reads the next row's padding or the allocation slack
  const int xpmax = (nx + 1) & ~1;
  // the red ring extends onto ghost layer 1 across exchanged faces (the
  // neighbours' red values there are recomputed from the 2-deep shell)
  const int rxlo = g.bcm[0] ? 0 : -1, rxhi = g.bcm[1] ? nx - 1 : nx;
  const int rylo = g.bcm[2] ? 0 : -1, ryhi = g.bcm[3] ? ny - 1 : ny;
  const int rzlo = g.bcm[4] ? 0 : -1, rzhi = g.bcm[5] ? nz - 1 : nz;
  const int q0 = (x0 + g.glo[0] + g.glo[1] + g.glo[2]) & 1;
  auto slot = [](int p) { return ((p % 5) + 5) % 5; };
  auto clampi = [](int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); };

  // region pairs owned by this thread (loads + LDS stores).  The domain BC
  // is applied on the way into LDS: a pair holding a BC-face ghost loads
  // the cells the ghost images instead and transforms them (lbc), so the
  // ghost takes exactly the value ParseBC would write before the pass --
  // including along exchanged faces, whose shell cells are loaded as they
  // are.  Cells that are ghosts of two BC faces (never read) get garbage.
  long loff[NL];
  int lgy[NL], lbc[NL], lym[NL];
  T lyc[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int c = tid + i * NT;
    const int r = c / PW, m = c - r * PW;
    lgy[i] = y0 - 2 + r;
    const int ps = x0 - 2 + 2 * m;  // first x of the pair
    int gx = min(ps, xpmax), bx = 0, gy = clampi(lgy[i], -2, ny + 1), by = 0;
    if (g.bcm[0] && ps == -2) {  // (-2, -1) <- image of (0): load (0, 1)
      gx = 0;
      bx = 1;
    } else if (g.bcm[1] && ps == nx) {  // (nx, nx+1) <- image of nx-1: load (nx-2, nx-1)
      gx = nx - 2;
      bx = 2;
    } else if (g.bcm[1] && ps == nx - 1) {  // (nx-1, nx): element 1 <- image of element 0
      bx = 3;
    }
    if (g.bcm[2] && lgy[i] == -1) {
      gy = 0;
      by = 1;
    } else if (g.bcm[3] && lgy[i] == ny) {
      gy = ny - 1;
      by = 2;
    }
    lbc[i] = c < CP ? bx | (by << 2) : 0;
    loff[i] = c < CP ? (long)gx + (long)gy * sy : 0;
    // the y-face BC of the pair, static indices only: g.bcm[1 + by] with a
    // per-lane index puts BoxArgs in memory and costs a dependent load +
    // vmcnt(0) per pair inside the z loop
    lym[i] = by == 1 ? g.bcm[2] : by == 2 ? g.bcm[3] : 0;
    lyc[i] = (T)(by == 1 ? g.bcc[2] : g.bcc[3]);
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
    rrow[i] = c < NRP && rgy[i] >= rylo && rgy[i] <= ryhi;
    rtile[i] = c < NRP && rgy[i] >= 0 && rgy[i] < ny && rr >= 1 && rr <= TY && m >= 1 &&
               m <= TX / 2 && rgx0[i] < nx;
  }
  const int gxlo = max(x0 - 1, rxlo), gxhi = min(x0 + TX, rxhi);  // red ring extent

  T pu0[NL], pu1[NL];
  T cr0[NP], cr1[NP], ca0[NP], ca1[NP], cb0[NP], cb1[NP];
  T nr0[NP], nr1[NP], na0[NP], na1[NP], nb0[NP], nb1[NP];
  T kr[NP], ka[NP], kb[NP];
  double an0[NP], an1[NP], ak0[NP], ak1[NP];  // ACC: acc pairs of planes p and p-1

  auto fetch_u = [&](int p) {
    // a BC-face ghost plane loads the plane it images
    const int pp = (g.bcm[4] && p == -1) ? 0 : (g.bcm[5] && p == nz) ? nz - 1 : clampi(p, -2, nz + 1);
    const long pz = (long)pp * sz;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      if (ZIN) {  // the input is identically +0 (a freshly zeroed correction)
        pu0[i] = (T)0;
        pu1[i] = (T)0;
      } else {
        const V2<T> v = *reinterpret_cast<const V2<T> *>(ui + loff[i] + pz);
        pu0[i] = v.x;
        pu1[i] = v.y;
      }
    }
  };
  auto put_u = [&](int p) {
    T *Rs = R + slot(p) * CP, *Bs = B + slot(p) * CP;
    const int zf = (g.bcm[4] && p == -1) ? 4 : (g.bcm[5] && p == nz) ? 5 : -1;
    const int zmode = zf == 4 ? g.bcm[4] : g.bcm[5];  // uniform; static indices
    const T zc = (T)(zf == 4 ? g.bcc[4] : g.bcc[5]);
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = tid + i * NT;
      if (NL * NT > CP && c >= CP) continue;
      T u0 = pu0[i], u1 = pu1[i];
      if (!ZIN) {  // BC images (a zero input images to zero: homogeneous BC)
        const int bx = lbc[i] & 3, by = lbc[i] >> 2;
        if (by) {
          u0 = ghost_of(lym[i], lyc[i], u0);
          u1 = ghost_of(lym[i], lyc[i], u1);
        }
        if (bx == 1) u1 = ghost_of(g.bcm[0], (T)g.bcc[0], u0);
        else if (bx == 2) u0 = ghost_of(g.bcm[1], (T)g.bcc[1], u1);
        else if (bx == 3) u1 = ghost_of(g.bcm[1], (T)g.bcc[1], u0);
        if (zf >= 0) {
          u0 = ghost_of(zmode, zc, u0);
          u1 = ghost_of(zmode, zc, u1);
        }
      }
      const int q = (q0 + lgy[i] + p) & 1;  // 1: the red element is the second
      Rs[c] = bsel(q, u1, u0);
      Bs[c] = bsel(q, u0, u1);
    }
  };
  auto fetch_c = [&](int p) {
    const long pz = (long)clampi(p, -1, nz) * sz;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const long off = rcoff[i] + pz;
      const V2<T> vr = *reinterpret_cast<const V2<T> *>(rhs + off);
      const V2<T> va = *reinterpret_cast<const V2<T> *>(a + off);
      const V2<T> vb = BC ? mk2<T>(s.bval, s.bval)
                            : *reinterpret_cast<const V2<T> *>(b + off);
      nr0[i] = vr.x; nr1[i] = vr.y;
      na0[i] = va.x; na1[i] = va.y;
      nb0[i] = vb.x; nb1[i] = vb.y;
    }
  };
  auto fetch_acc = [&](int p) {  // the sum field, one step ahead of its store
    const long pz = (long)clampi(p, 0, nz - 1) * sz;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const double2 v = *reinterpret_cast<const double2 *>(acc + rcoff[i] + pz);
      an0[i] = v.x;
      an1[i] = v.y;
    }
  };
  auto upd = [&](T uc, T xm, T xp, T ym, T yp, T zm, T zp,
                 T rv, T av, T bv) -> T {
    const T tx = (xp + xm) - (T)2 * uc;
    const T ty = (yp + ym) - (T)2 * uc;
    const T tz = (zp + zm) - (T)2 * uc;
    const T lap = (tx + ty) + tz;                     // .ChF:111-120
    T lofdpsi = s.alpha * av * uc;                    // .ChF:107-108
    const T ldpsi = lap * s.dxinv * bv;               // .ChF:122
    lofdpsi = lofdpsi - s.beta * ldpsi;                    // .ChF:124
    const T lam = (T)1 / (av * s.alpha + s.lamshift);  // .cpp:234-243
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
  if (ACC) fetch_acc(z0 - 1);
  for (int p = z0 - 1; p <= z1; ++p) {
    put_u(p + 1);
    fetch_u(p + 2);
    fetch_c(p + 1);
    if (ACC) {
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        ak0[i] = an0[i];
        ak1[i] = an1[i];
      }
      fetch_acc(p);
    }
    __syncthreads();
    if (p >= rzlo && p <= rzhi) {  // RED cells of plane p on the ring
      T *Rs = R + slot(p) * CP;
      const T *Bs = B + slot(p) * CP;
      const T *Bm = B + slot(p - 1) * CP;
      const T *Bp = B + slot(p + 1) * CP;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int q = (q0 + rgy[i] + p) & 1;
        const int gx = rgx0[i] + q;
        if (!rrow[i] || gx < gxlo || gx > gxhi) continue;
        const int ci = rci[i];
        const T xm = q ? Bs[ci] : Bs[ci - 1];
        const T xp = q ? Bs[ci + 1] : Bs[ci];
        Rs[ci] = upd(Rs[ci], xm, xp, Bs[ci - PW], Bs[ci + PW], Bm[ci], Bp[ci],
                     bsel(q, cr1[i], cr0[i]), bsel(q, ca1[i], ca0[i]), bsel(q, cb1[i], cb0[i]));
      }
    }
    __syncthreads();
    const int k = p - 1;
    if (k >= z0 && k < z1) {  // BLACK cells of plane k on the tile + store
      const T *Rs = R + slot(k) * CP;
      const T *Bs = B + slot(k) * CP;
      const T *Rm = R + slot(k - 1) * CP;
      const T *Rp = R + slot(k + 1) * CP;
      T *dst = uo + (long)k * sz;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        if (!rtile[i]) continue;
        const int qb = 1 - ((q0 + rgy[i] + k) & 1);  // 1: the black element is the second
        const int gx = rgx0[i] + qb;
        const int ci = rci[i];
        const T red = Rs[ci];
        T blk = Bs[ci];
        if (gx < nx) {
          const T xm = qb ? Rs[ci] : Rs[ci - 1];
          const T xp = qb ? Rs[ci + 1] : Rs[ci];
          blk = upd(blk, xm, xp, Rs[ci - PW], Rs[ci + PW], Rm[ci], Rp[ci], kr[i], ka[i], kb[i]);
        }
        V2<T> w;
        w.x = bsel(qb, red, blk);
        w.y = bsel(qb, blk, red);
        if (ACC) {  // acc += the swept value (incr, scale 1), u_out not written
          double *ad = acc + (long)k * sz + roff[i];
          if (rgx0[i] + 1 < nx) {
            double2 t;
            t.x = ak0[i] + (double)w.x;
            t.y = ak1[i] + (double)w.y;
            *reinterpret_cast<double2 *>(ad) = t;
          } else {
            ad[0] = ak0[i] + (double)w.x;
          }
        } else if (rgx0[i] + 1 < nx) {
          *reinterpret_cast<V2<T> *>(dst + roff[i]) = w;
        } else {
          dst[roff[i]] = w.x;
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

template <class T, int TX, int TY, int NT, bool ZIN, bool BC, bool ACC>
__global__ __launch_bounds__(NT) void k_gsrb_fused6(T *__restrict__ uo,
                                                    double *__restrict__ acc,
                                                    const T *__restrict__ ui,
                                                    const T *__restrict__ rhs,
                                                    const T *__restrict__ a,
                                                    const T *__restrict__ b,
                                                    const BoxArgs g, const StencilCoefs s, int kc,
                                                    int ntx, int nty, int nblocks) {
  using F = Fused6<TX, TY, NT>;
  __shared__ T R[5 * F::CP];  // red element of every pair, 5-plane ring
  __shared__ T B[5 * F::CP];  // black element
  const int bid = blockIdx.x;      // XCD-aware: consecutive tiles on one XCD
  const int q8 = nblocks / 8, r8 = nblocks % 8;
  const int xcd = bid % 8, i8 = bid / 8;
  const int L = xcd * q8 + min(xcd, r8) + i8;
  const int tx_ = L % ntx, ty_ = (L / ntx) % nty, tz_ = L / (ntx * nty);
  const int z0 = tz_ * kc;
  fused6_segment<T, TX, TY, NT, ZIN, BC, ACC>(R, B, uo, acc, ui, rhs, a, b, g, s, tx_ * TX,
                                           ty_ * TY, z0, min(z0 + kc, g.nz));
}

// ---- small levels: one 3D block per workgroup, no streaming ---------------
// On a coarse level (<= 128^3 per box) the streaming kernel is latency bound:
// a workgroup walks kc + 5 pipeline steps, each waiting on one global load,
// so a 64^3 sweep costs as much as a 128^3 one.  Here a workgroup loads its
// whole TX x TY x TZ tile plus the 2-cell u halo into LDS at once (all loads
// in flight together), updates the RED cells of the tile grown by one, then
// the BLACK cells of the tile, and stores: one memory round trip per sweep.
// Same operands and expressions as k_gsrb_fused6 (bit-identical), same ring
// extension across exchanged faces, same ZIN/BC/ACC variants, out of place.
// The domain BC is applied to the LDS copy (no fill launch, u_in untouched).
// The halo re-reads (u 2.9x, rhs/a 2.1x at 32x8x4) hit L2/MALL: the whole
// level is cache resident at these sizes.
template <int TX, int TY, int TZ, int NT>
struct Blk {
  static_assert(TX % 2 == 0, "TX must be even");
  static constexpr int PW = TX / 2 + 2;          // pairs per region row (x0-2 .. x0+TX+1)
  static constexpr int LH = TY + 4;              // region rows y0-2 .. y0+TY+1
  static constexpr int CP = PW * LH;             // pairs per region plane
  static constexpr int NREG = CP * (TZ + 4);     // region planes z0-2 .. z0+TZ+1
  static constexpr int RH = TY + 2, RZ = TZ + 2;  // ring rows / planes
  static constexpr int NRP = PW * RH * RZ;
  static constexpr int NL = (NREG + NT - 1) / NT;
  static constexpr int NP = (NRP + NT - 1) / NT;
};

// One TX x TY x TZ tile at (x0, y0, z0) of the box; R/B: LDS of NREG
// elements each (Blk<..>::NREG).
template <class T, int TX, int TY, int TZ, int NT, bool ZIN, bool BC, bool ACC>
__device__ __forceinline__ void block_tile(T *__restrict__ R, T *__restrict__ B,
                                           T *__restrict__ uo, double *__restrict__ acc,
                                           const T *__restrict__ ui, const T *__restrict__ rhs,
                                           const T *__restrict__ a, const T *__restrict__ b,
                                           const BoxArgs &g, const StencilCoefs &s64, int x0,
                                           int y0, int z0) {
  using F = Blk<TX, TY, TZ, NT>;
  const SC<T> s(s64);
  constexpr int PW = F::PW, CP = F::CP, NREG = F::NREG, NRP = F::NRP, NL = F::NL, NP = F::NP;
  const int tid = threadIdx.x;
  const long sy = g.sy, sz = g.sz;
  const int nx = g.nx, ny = g.ny, nz = g.nz;
  const int xpmax = (nx + 1) & ~1;
  const int rxlo = g.bcm[0] ? 0 : -1, rxhi = g.bcm[1] ? nx - 1 : nx;
  const int rylo = g.bcm[2] ? 0 : -1, ryhi = g.bcm[3] ? ny - 1 : ny;
  const int rzlo = g.bcm[4] ? 0 : -1, rzhi = g.bcm[5] ? nz - 1 : nz;
  const int q0 = (x0 + g.glo[0] + g.glo[1] + g.glo[2]) & 1;
  auto clampi = [](int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); };

  // 1. issue every load: the u region (tile + 2) and the ring's rhs/a/b
  V2<T> v[NL];
  if (!ZIN) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = tid + i * NT;
      const int pz = c / CP, rem = c - pz * CP, r = rem / PW, m = rem - r * PW;
      const long off = (long)min(x0 - 2 + 2 * m, xpmax) + (long)clampi(y0 - 2 + r, -2, ny + 1) * sy +
                       (long)clampi(z0 - 2 + pz, -2, nz + 1) * sz;
      v[i] = *reinterpret_cast<const V2<T> *>(ui + (c < NREG ? off : 0));
    }
  }
  T cr[NP][2], ca[NP][2], cb[NP][2];
  double ac[NP][2];  // ACC: the sum field (fp64)
  int rgx0[NP], rgy[NP], rgz[NP], rci[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int c = tid + i * NT;
    const int rz = c / (PW * F::RH), rem = c - rz * (PW * F::RH), rr = rem / PW, m = rem - rr * PW;
    rgx0[i] = x0 - 2 + 2 * m;
    rgy[i] = y0 - 1 + rr;
    rgz[i] = c < NRP ? z0 - 1 + rz : -1000;  // -1000: no pair (fails every range test)
    rci[i] = ((rz + 1) * F::LH + rr + 1) * PW + m;
    const long off = c < NRP ? (long)min(rgx0[i], xpmax) + (long)clampi(rgy[i], -1, ny) * sy +
                                   (long)clampi(rgz[i], -1, nz) * sz
                             : 0;
    const V2<T> vr = *reinterpret_cast<const V2<T> *>(rhs + off);
    const V2<T> va = *reinterpret_cast<const V2<T> *>(a + off);
    const V2<T> vb = BC ? mk2<T>(s.bval, s.bval) : *reinterpret_cast<const V2<T> *>(b + off);
    cr[i][0] = vr.x; cr[i][1] = vr.y;
    ca[i][0] = va.x; ca[i][1] = va.y;
    cb[i][0] = vb.x; cb[i][1] = vb.y;
    if (ACC) {
      const long ao = (long)min(rgx0[i], xpmax) + (long)clampi(rgy[i], 0, ny - 1) * sy +
                      (long)clampi(rgz[i], 0, nz - 1) * sz;
      const double2 w = *reinterpret_cast<const double2 *>(acc + (c < NRP ? ao : 0));
      ac[i][0] = w.x; ac[i][1] = w.y;
    }
  }
  // 2. the u region into LDS, red / black split
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int c = tid + i * NT;
    if (NL * NT > NREG && c >= NREG) continue;
    const int pz = c / CP, rem = c - pz * CP, r = rem / PW;
    const int q = (q0 + y0 - 2 + r + z0 - 2 + pz) & 1;  // 1: the red element is the second
    const T u0 = ZIN ? (T)0 : v[i].x, u1 = ZIN ? (T)0 : v[i].y;
    R[c] = bsel(q, u1, u0);
    B[c] = bsel(q, u0, u1);
  }
  // the ghosts of the region's BC faces (cf_only: the coarse-fine faces),
  // from the LDS values
  const int n3[3] = {nx, ny, nz}, o3[3] = {x0 - 2, y0 - 2, z0 - 2};
  constexpr int E3[3] = {TX + 4, TY + 4, TZ + 4};  // region extent per direction
  auto lds = [&](int x, int y, int z) -> T * {  // the LDS slot of cell (x, y, z)
    const int rx = x - o3[0];
    const int idx = ((z - o3[2]) * F::LH + (y - o3[1])) * PW + (rx >> 1);
    const int red = (rx & 1) == ((q0 + y + z) & 1);
    return red ? &R[idx] : &B[idx];
  };
  auto fill_ghosts = [&](bool cf_only) {
    for (int face = 0; face < 6; ++face) {
      const int mode = g.bcm[face];
      if (!mode || (cf_only && mode != kBcCFHom)) continue;
      const int dir = face >> 1, side = face & 1;
      const int gc = side == 0 ? -1 : n3[dir];  // ghost coordinate along dir
      if (gc < o3[dir] || gc >= o3[dir] + E3[dir]) continue;  // face not in this region
      const int d0 = dir == 0 ? 1 : 0, d1 = dir == 2 ? 1 : 2;
      const int lo0 = max(g.bcm[2 * d0] ? 0 : -1, o3[d0]);
      const int hi0 = min(g.bcm[2 * d0 + 1] ? n3[d0] - 1 : n3[d0], o3[d0] + E3[d0] - 1);
      const int lo1 = max(g.bcm[2 * d1] ? 0 : -1, o3[d1]);
      const int hi1 = min(g.bcm[2 * d1 + 1] ? n3[d1] - 1 : n3[d1], o3[d1] + E3[d1] - 1);
      const int w0 = hi0 - lo0 + 1, cnt = w0 * (hi1 - lo1 + 1);
      for (int t = tid; t < cnt; t += NT) {
        int c[3];
        c[dir] = gc;
        c[d0] = lo0 + t % w0;
        c[d1] = lo1 + t / w0;
        T *gp = lds(c[0], c[1], c[2]);
        c[dir] = side == 0 ? 0 : n3[dir] - 1;
        const T f1 = *lds(c[0], c[1], c[2]);
        if (mode == kBcCFHom) {  // k_cf_interp<true>: ps = 0, f1, f2 one / two cells in
          c[dir] = side == 0 ? 1 : n3[dir] - 2;
          const T f2 = *lds(c[0], c[1], c[2]);
          *gp = ((T)(8.0 / 15.0) * (T)0 + (T)(2.0 / 3.0) * f1) + (T)(-0.2) * f2;
        } else {
          *gp = ghost_of(mode, (T)g.bcc[face], f1);
        }
      }
    }
  };
  // does the region reach a coarse-fine face? (uniform)
  bool cf_tile = false;
  for (int face = 0; face < 6; ++face) {
    const int gc = (face & 1) == 0 ? -1 : n3[face >> 1];
    cf_tile = cf_tile || (g.bcm[face] == kBcCFHom && gc >= o3[face >> 1] &&
                          gc < o3[face >> 1] + E3[face >> 1]);
  }
  // 2b. the domain BC, in LDS: each BC-face ghost of the region takes the
  // image of the cell it touches -- the values ParseBC writes before the
  // pass (same cells, including the extension onto exchanged faces' ghost
  // layers), so the input is never written and the sweep is one launch.  Only tiles touching a BC face (a workgroup-uniform test) pay.
  // (the region reaches the hi ghost at n once x0 + TX + 1 >= n)
  if (!ZIN && ((g.bcm[0] && x0 == 0) || (g.bcm[1] && x0 + TX + 1 >= nx) || (g.bcm[2] && y0 == 0) ||
               (g.bcm[3] && y0 + TY + 1 >= ny) || (g.bcm[4] && z0 == 0) ||
               (g.bcm[5] && z0 + TZ + 1 >= nz))) {
    __syncthreads();
    fill_ghosts(false);
  }
  auto upd = [&](T uc, T xm, T xp, T ym, T yp, T zm, T zp,
                 T rv, T av, T bv) -> T {
    const T tx = (xp + xm) - (T)2 * uc;
    const T ty = (yp + ym) - (T)2 * uc;
    const T tz = (zp + zm) - (T)2 * uc;
    const T lap = (tx + ty) + tz;                     // .ChF:111-120
    T lofdpsi = s.alpha * av * uc;                    // .ChF:107-108
    const T ldpsi = lap * s.dxinv * bv;               // .ChF:122
    lofdpsi = lofdpsi - s.beta * ldpsi;                    // .ChF:124
    const T lam = (T)1 / (av * s.alpha + s.lamshift);  // .cpp:234-243
    return uc - lam * (lofdpsi - rv);                      // .ChF:127-128
  };
  __syncthreads();
  // 3. RED cells of the ring (tile grown by one, clipped at BC faces)
  const int gxlo = max(x0 - 1, rxlo), gxhi = min(x0 + TX, rxhi);
  const int gylo = max(y0 - 1, rylo), gyhi = min(y0 + TY, ryhi);
  const int gzlo = max(z0 - 1, rzlo), gzhi = min(z0 + TZ, rzhi);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int q = (q0 + rgy[i] + rgz[i]) & 1;
    const int gx = rgx0[i] + q;
    if (gx < gxlo || gx > gxhi || rgy[i] < gylo || rgy[i] > gyhi || rgz[i] < gzlo || rgz[i] > gzhi)
      continue;
    const int ci = rci[i];
    const T xm = q ? B[ci] : B[ci - 1];
    const T xp = q ? B[ci + 1] : B[ci];
    R[ci] = upd(R[ci], xm, xp, B[ci - PW], B[ci + PW], B[ci - CP], B[ci + CP],
                bsel(q, cr[i][1], cr[i][0]), bsel(q, ca[i][1], ca[i][0]), bsel(q, cb[i][1], cb[i][0]));
  }
  __syncthreads();
  if (cf_tile) {  // homogeneousCFInterp again before the black pass (.cpp:296): red cells moved
    fill_ghosts(true);
    __syncthreads();
  }
  // 4. BLACK cells of the tile + store
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int gy = rgy[i], gz = rgz[i];
    if (rgx0[i] < x0 || rgx0[i] >= x0 + TX || rgx0[i] >= nx || gy < y0 || gy >= y0 + TY || gy >= ny ||
        gz < z0 || gz >= z0 + TZ || gz >= nz)
      continue;
    const int qb = 1 - ((q0 + gy + gz) & 1);  // 1: the black element is the second
    const int gx = rgx0[i] + qb;
    const int ci = rci[i];
    const T red = R[ci];
    T blk = B[ci];
    if (gx < nx) {
      const T xm = qb ? R[ci] : R[ci - 1];
      const T xp = qb ? R[ci + 1] : R[ci];
      blk = upd(blk, xm, xp, R[ci - PW], R[ci + PW], R[ci - CP], R[ci + CP], bsel(qb, cr[i][1], cr[i][0]),
                bsel(qb, ca[i][1], ca[i][0]), bsel(qb, cb[i][1], cb[i][0]));
    }
    V2<T> w;
    w.x = bsel(qb, red, blk);
    w.y = bsel(qb, blk, red);
    const long off = (long)rgx0[i] + (long)gy * sy + (long)gz * sz;
    if (ACC) {
      double2 t;
      t.x = ac[i][0] + (double)w.x;
      t.y = ac[i][1] + (double)w.y;
      if (rgx0[i] + 1 < nx) *reinterpret_cast<double2 *>(acc + off) = t;
      else acc[off] = t.x;
    } else if (rgx0[i] + 1 < nx) {
      *reinterpret_cast<V2<T> *>(uo + off) = w;
    } else {
      uo[off] = w.x;
    }
  }
}

template <class T, int TX, int TY, int TZ, int NT, bool ZIN, bool BC, bool ACC>
__global__ __launch_bounds__(NT) void k_gsrb_block(T *__restrict__ uo,
                                                   double *__restrict__ acc,
                                                   const T *__restrict__ ui,
                                                   const T *__restrict__ rhs,
                                                   const T *__restrict__ a,
                                                   const T *__restrict__ b,
                                                   const BoxArgs g, const StencilCoefs s64, int ntx,
                                                   int nty, int nblocks, int ox, int oy, int oz) {
  using F = Blk<TX, TY, TZ, NT>;
  __shared__ T R[F::NREG];  // red element of every region pair
  __shared__ T B[F::NREG];  // black element
  const int bid = blockIdx.x;  // XCD-aware: consecutive tiles on one XCD
  const int q8 = nblocks / 8, r8 = nblocks % 8;
  const int L = (bid % 8) * q8 + min(bid % 8, r8) + bid / 8;
  // tiles of the region starting at (ox, oy, oz); ox is even (16-B pairs)
  block_tile<T, TX, TY, TZ, NT, ZIN, BC, ACC>(R, B, uo, acc, ui, rhs, a, b, g, s64,
                                              ox + (L % ntx) * TX, oy + ((L / ntx) % nty) * TY,
                                              oz + (L / (ntx * nty)) * TZ);
}

// ---- last pre-smoothing sweep + restrictResidual in one pass -------------
// The streaming sweep carried one stage deeper so that the residual of the
// smoothed e can be restricted while its planes are still in LDS
// (restrictResidual, VariableCoeffPoissonOperator.cpp:151-194 with
// RESTRICTRESVC3D, .ChF:379-437): at step p the workgroup updates RED on
// plane p over the tile grown by two and restricts the residual of plane p-3
// (its neighbours p-4 .. p-2 are final), then updates BLACK on plane p-1
// over the tile grown by one (written back into LDS) and stores e on plane
// p-1.  The residual goes into the coarse cells of the tile -- one thread per coarse (x, y) cell, children
// summed in the Fortran k, j, i order.  rhs/a of the residual come from L2
// (the sweep loaded them two steps earlier), so the restriction adds no HBM
// reads: the separate restrict kernel (25 B/cell) disappears.  A 6-plane
// LDS ring (143 KB at 128x16).  Boxes whose faces are all domain faces (the
// exchanged-face case would need a 3-deep shell); bit-identical to
// gsrb_sweep_fused + restrict_residual.
template <int TX, int TY, int NT>
struct FRst {
  static_assert(TX % 2 == 0 && TY % 2 == 0, "even tiles");
  static_assert((TX / 2) * (TY / 2) == NT, "one thread per coarse (x, y) cell");
  static constexpr int PW = TX / 2 + 4;  // pairs x0-4 .. x0+TX+3
  static constexpr int LH = TY + 6;      // rows y0-3 .. y0+TY+2
  static constexpr int CP = PW * LH;
  static constexpr int NS = 6;           // LDS planes
  static constexpr int RW = TX / 2 + 2;  // ring pairs per row (x0-2 .. x0+TX+1)
  static constexpr int NRP = RW * (TY + 4);  // ring rows y0-2 .. y0+TY+1
  static constexpr int NL = (CP + NT - 1) / NT;
  static constexpr int NP = (NRP + NT - 1) / NT;
};

template <int TX, int TY, int NT, bool BC>
__global__ __launch_bounds__(NT) void k_gsrb_fused_rst(double *__restrict__ uo,
                                                       double *__restrict__ rc,
                                                       const double *__restrict__ ui,
                                                       const double *__restrict__ rhs,
                                                       const double *__restrict__ a,
                                                       const double *__restrict__ b,
                                                       const BoxArgs g, const StencilCoefs s,
                                                       const BoxArgs cg, int kc, int ntx, int nty,
                                                       int nblocks) {
  using F = FRst<TX, TY, NT>;
  constexpr int PW = F::PW, CP = F::CP, NS = F::NS, RW = F::RW, NRP = F::NRP, NL = F::NL,
                NP = F::NP;
  __shared__ double R[NS * CP];  // red element of every pair
  __shared__ double B[NS * CP];  // black element
  const int bid = blockIdx.x;    // XCD-aware tile order, as k_gsrb_fused6
  const int q8 = nblocks / 8, r8 = nblocks % 8;
  const int L = (bid % 8) * q8 + min(bid % 8, r8) + bid / 8;
  const int x0 = (L % ntx) * TX, y0 = ((L / ntx) % nty) * TY;
  const int z0 = (L / (ntx * nty)) * kc, z1 = min(z0 + kc, g.nz);
  const int tid = threadIdx.x;
  const long sy = g.sy, sz = g.sz;
  const int nx = g.nx, ny = g.ny, nz = g.nz;
  const int xpmax = (nx + 1) & ~1;
  const int q0 = (x0 + g.glo[0] + g.glo[1] + g.glo[2]) & 1;
  auto slot = [](int p) { return ((p % NS) + NS) % NS; };
  auto clampi = [](int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); };

  // region pairs: loads (BC images applied on entry, as k_gsrb_fused6)
  long loff[NL];
  int lgy[NL], lbc[NL], lym[NL];
  double lyc[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int c = tid + i * NT;
    const int r = c / PW, m = c - r * PW;
    lgy[i] = y0 - 3 + r;
    const int ps = x0 - 4 + 2 * m;
    int gx = clampi(ps, -2, xpmax), bx = 0, gy = clampi(lgy[i], -2, ny + 1), by = 0;
    if (g.bcm[0] && ps == -2) {
      gx = 0;
      bx = 1;
    } else if (g.bcm[1] && ps == nx) {
      gx = nx - 2;
      bx = 2;
    } else if (g.bcm[1] && ps == nx - 1) {
      bx = 3;
    }
    if (g.bcm[2] && lgy[i] == -1) {
      gy = 0;
      by = 1;
    } else if (g.bcm[3] && lgy[i] == ny) {
      gy = ny - 1;
      by = 2;
    }
    lbc[i] = c < CP ? bx | (by << 2) : 0;
    loff[i] = c < CP ? (long)gx + (long)gy * sy : 0;
    lym[i] = by == 1 ? g.bcm[2] : by == 2 ? g.bcm[3] : 0;  // static indices (fused6)
    lyc[i] = by == 1 ? g.bcc[2] : g.bcc[3];
  }
  // ring pairs (tile + 2): coefficient loads, red / black updates, stores
  long rcoff[NP];
  int rgy[NP], rgx0[NP], rci[NP], rfl[NP];  // rfl: 1 red row, 2 black row, 4 tile
  const int rxlo = max(x0 - 2, 0), rxhi = min(x0 + TX + 1, nx - 1);
  const int rylo = max(y0 - 2, 0), ryhi = min(y0 + TY + 1, ny - 1);
  const int bxlo = max(x0 - 1, 0), bxhi = min(x0 + TX, nx - 1);
  const int bylo = max(y0 - 1, 0), byhi = min(y0 + TY, ny - 1);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int c = tid + i * NT;
    const int rr = c / RW, mm = c - rr * RW;
    rgy[i] = y0 - 2 + rr;
    rgx0[i] = x0 - 2 + 2 * mm;
    rcoff[i] = c < NRP ? (long)clampi(rgx0[i], -2, xpmax) + (long)clampi(rgy[i], -1, ny) * sy : 0;
    rci[i] = (rr + 1) * PW + mm + 1;
    const int red = c < NRP && rgy[i] >= rylo && rgy[i] <= ryhi;
    const int blk = c < NRP && rgy[i] >= bylo && rgy[i] <= byhi;
    const int tile = c < NRP && rgy[i] >= y0 && rgy[i] < y0 + TY && rgy[i] < ny &&
                     rgx0[i] >= x0 && rgx0[i] < x0 + TX && rgx0[i] < nx;
    rfl[i] = red | (blk << 1) | (tile << 2);
  }
  // the coarse cell of this thread: fine pair (x0 + 2cx, +1), rows y0 + 2cy + {0, 1}
  const int cx = tid % (TX / 2), cy = tid / (TX / 2);
  const int fxr = x0 + 2 * cx, fyr = y0 + 2 * cy;
  const bool rown = fxr < nx && fyr < ny;
  const int cci = (2 * cy + 3) * PW + cx + 2;  // LDS index of the (fxr, fyr) pair
  const long frow = (long)min(fxr, xpmax) + (long)min(fyr, ny - 1) * sy;
  const bool xyface = (g.bcm[0] && x0 == 0) || (g.bcm[1] && x0 + TX >= nx) ||
                      (g.bcm[2] && y0 == 0) || (g.bcm[3] && y0 + TY >= ny);

  double pu0[NL], pu1[NL];
  double cr0[NP], cr1[NP], ca0[NP], ca1[NP], cb0[NP], cb1[NP];
  double nr0[NP], nr1[NP], na0[NP], na1[NP], nb0[NP], nb1[NP];
  double kr[NP], ka[NP], kb[NP];
  double2 qr[2], qa[2], qb[2];  // rhs/a/b of the residual plane, (fxr, fyr + jj)
  double2 wr[2], wa[2], wb[2];  // ... of the next residual plane (one step ahead)
  double sum = 0.0;

  auto fetch_u = [&](int p) {
    const int pp = (g.bcm[4] && p == -1) ? 0 : (g.bcm[5] && p == nz) ? nz - 1 : clampi(p, -2, nz + 1);
    const long pz = (long)pp * sz;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const double2 v = *reinterpret_cast<const double2 *>(ui + loff[i] + pz);
      pu0[i] = v.x;
      pu1[i] = v.y;
    }
  };
  auto put_u = [&](int p) {
    double *Rs = R + slot(p) * CP, *Bs = B + slot(p) * CP;
    const int zf = (g.bcm[4] && p == -1) ? 4 : (g.bcm[5] && p == nz) ? 5 : -1;
    const int zmode = zf == 4 ? g.bcm[4] : g.bcm[5];
    const double zc = zf == 4 ? g.bcc[4] : g.bcc[5];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = tid + i * NT;
      if (NL * NT > CP && c >= CP) continue;
      double u0 = pu0[i], u1 = pu1[i];
      const int bx = lbc[i] & 3, by = lbc[i] >> 2;
      if (by) {
        u0 = ghost_of(lym[i], lyc[i], u0);
        u1 = ghost_of(lym[i], lyc[i], u1);
      }
      if (bx == 1) u1 = ghost_of(g.bcm[0], g.bcc[0], u0);
      else if (bx == 2) u0 = ghost_of(g.bcm[1], g.bcc[1], u1);
      else if (bx == 3) u1 = ghost_of(g.bcm[1], g.bcc[1], u0);
      if (zf >= 0) {
        u0 = ghost_of(zmode, zc, u0);
        u1 = ghost_of(zmode, zc, u1);
      }
      const int q = (q0 + lgy[i] + p) & 1;
      Rs[c] = bsel(q, u1, u0);
      Bs[c] = bsel(q, u0, u1);
    }
  };
  auto fetch_c = [&](int p) {
    const long pz = (long)clampi(p, -1, nz) * sz;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const long off = rcoff[i] + pz;
      const double2 vr = *reinterpret_cast<const double2 *>(rhs + off);
      const double2 va = *reinterpret_cast<const double2 *>(a + off);
      const double2 vb = BC ? make_double2(s.bval, s.bval) : *reinterpret_cast<const double2 *>(b + off);
      nr0[i] = vr.x; nr1[i] = vr.y;
      na0[i] = va.x; na1[i] = va.y;
      nb0[i] = vb.x; nb1[i] = vb.y;
    }
  };
  auto fetch_q = [&](int k) {  // the residual plane's coefficients (L2: loaded by the sweep)
    const long pz = (long)clampi(k, 0, nz - 1) * sz;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const long off = frow + (long)(jj && fyr + 1 < ny ? sy : 0) + pz;
      wr[jj] = *reinterpret_cast<const double2 *>(rhs + off);
      wa[jj] = *reinterpret_cast<const double2 *>(a + off);
      wb[jj] = BC ? make_double2(s.bval, s.bval) : *reinterpret_cast<const double2 *>(b + off);
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

  fetch_u(z0 - 3);
  put_u(z0 - 3);
  fetch_u(z0 - 2);
  put_u(z0 - 2);
  fetch_u(z0 - 1);
  fetch_c(z0 - 2);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    cr0[i] = nr0[i]; cr1[i] = nr1[i];
    ca0[i] = na0[i]; ca1[i] = na1[i];
    cb0[i] = nb0[i]; cb1[i] = nb1[i];
  }
  for (int p = z0 - 2; p <= z1 + 2; ++p) {
    put_u(p + 1);
    fetch_u(p + 2);
    fetch_c(p + 1);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {  // plane p-3's (fetched last step)
      qr[jj] = wr[jj];
      qa[jj] = wa[jj];
      qb[jj] = wb[jj];
    }
    if (p - 2 >= z0 && p - 2 < z1) fetch_q(p - 2);
    __syncthreads();
    if (p >= 0 && p <= nz - 1 && p <= z1 + 1) {  // RED of plane p on the tile grown by two
      double *Rs = R + slot(p) * CP;
      const double *Bs = B + slot(p) * CP;
      const double *Bm = B + slot(p - 1) * CP;
      const double *Bp = B + slot(p + 1) * CP;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int q = (q0 + rgy[i] + p) & 1;
        const int gx = rgx0[i] + q;
        if (!(rfl[i] & 1) || gx < rxlo || gx > rxhi) continue;
        const int ci = rci[i];
        const double xm = q ? Bs[ci] : Bs[ci - 1];
        const double xp = q ? Bs[ci + 1] : Bs[ci];
        Rs[ci] = upd(Rs[ci], xm, xp, Bs[ci - PW], Bs[ci + PW], Bm[ci], Bp[ci],
                     bsel(q, cr1[i], cr0[i]), bsel(q, ca1[i], ca0[i]), bsel(q, cb1[i], cb0[i]));
      }
    }
    // residual of plane p-3 (final: its black was updated last step) -- it
    // reads planes p-4 .. p-2 while RED writes plane p
    const int kr3 = p - 3;
    if (kr3 >= z0 && kr3 < z1) {  // residual of plane p-3 into the coarse cell
      const double *Rs = R + slot(kr3) * CP, *Bs = B + slot(kr3) * CP;
      const double *Rm = R + slot(kr3 - 1) * CP, *Bm = B + slot(kr3 - 1) * CP;
      const double *Rp = R + slot(kr3 + 1) * CP, *Bp = B + slot(kr3 + 1) * CP;
      const double denom = 2 * 2 * 2;  // .ChF:402
      if ((kr3 & 1) == 0) sum = 0.0;  // rc zeroed first (.cpp:177)
      // the colour of a row is uniform over the workgroup (fyr even), so each
      // element comes from R or B by a uniform choice: element e of a pair
      // is red iff e == (q0 + row + plane) & 1
      // (the parity of row fyr + dr is that of y0 + dr: written with y0, the
      // choice is visibly uniform and selects a base address, not a value)
      auto el = [&](const double *Rp_, const double *Bp_, int ci, int e, int dr, int k) {
        return ((e == ((q0 + y0 + dr + k) & 1)) ? Rp_ : Bp_)[ci];
      };
      double v[4][2], zm[2][2], zp[2][2], xl[2], xr[2];
#pragma unroll
      for (int r = 0; r < 4; ++r)  // rows fyr-1 .. fyr+2 of plane k
#pragma unroll
        for (int e = 0; e < 2; ++e) v[r][e] = el(Rs, Bs, cci + (r - 1) * PW, e, r - 1, kr3);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int ci = cci + jj * PW;
        xl[jj] = el(Rs, Bs, ci - 1, 1, jj, kr3);
        xr[jj] = el(Rs, Bs, ci + 1, 0, jj, kr3);
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          zm[jj][e] = el(Rm, Bm, ci, e, jj, kr3 - 1);
          zp[jj][e] = el(Rp, Bp, ci, e, jj, kr3 + 1);
        }
      }
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int j = fyr + jj;
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const int i = fxr + ii;
          const double uc = v[jj + 1][ii];
          double vxm = ii ? v[jj + 1][0] : xl[jj];
          double vxp = ii ? xr[jj] : v[jj + 1][1];
          double vym = v[jj][ii], vyp = v[jj + 2][ii];
          double vzm = zm[jj][ii], vzp = zp[jj][ii];
          if (xyface) {  // only tiles on an x / y domain face (uniform)
            if (i == 0 && g.bcm[0]) vxm = ghost_of(g.bcm[0], g.bcc[0], uc);
            if (i == nx - 1 && g.bcm[1]) vxp = ghost_of(g.bcm[1], g.bcc[1], uc);
            if (j == 0 && g.bcm[2]) vym = ghost_of(g.bcm[2], g.bcc[2], uc);
            if (j == ny - 1 && g.bcm[3]) vyp = ghost_of(g.bcm[3], g.bcc[3], uc);
          }
          if (kr3 == 0 && g.bcm[4]) vzm = ghost_of(g.bcm[4], g.bcc[4], uc);
          if (kr3 == nz - 1 && g.bcm[5]) vzp = ghost_of(g.bcm[5], g.bcc[5], uc);
          const double tx = (vxp + vxm) - 2.0 * uc;
          const double ty = (vyp + vym) - 2.0 * uc;
          const double tz = (vzp + vzm) - 2.0 * uc;
          double ldpsi = (tx + ty) + tz;                                        // .ChF:416-425
          double lofdpsi = s.alpha * (ii ? qa[jj].y : qa[jj].x) * uc;          // .ChF:411-412
          ldpsi = ldpsi * s.dxinv * s.beta * (ii ? qb[jj].y : qb[jj].x);       // .ChF:427
          lofdpsi = lofdpsi - ldpsi;                                            // .ChF:429
          sum = sum + ((ii ? qr[jj].y : qr[jj].x) - lofdpsi) / denom;          // .ChF:431-432
        }
      }
      if ((kr3 & 1) == 1 && rown)
        rc[(long)(fxr >> 1) + (long)(fyr >> 1) * cg.sy + (long)(kr3 >> 1) * cg.sz] = sum;
    }
    __syncthreads();
    const int k = p - 1;
    if (k >= 0 && k <= nz - 1 && k >= z0 - 1 && k <= z1) {  // BLACK of plane k, tile + 1
      const double *Rs = R + slot(k) * CP;
      double *Bs = B + slot(k) * CP;
      const double *Rm = R + slot(k - 1) * CP;
      const double *Rp = R + slot(k + 1) * CP;
      double *dst = uo + (long)k * sz;
      const bool store = k >= z0 && k < z1;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        if (!(rfl[i] & 2)) continue;
        const int qb = 1 - ((q0 + rgy[i] + k) & 1);  // 1: the black element is the second
        const int gx = rgx0[i] + qb;
        const int ci = rci[i];
        const double red = Rs[ci];
        double blk = Bs[ci];
        if (gx >= bxlo && gx <= bxhi) {
          const double xm = qb ? Rs[ci] : Rs[ci - 1];
          const double xp = qb ? Rs[ci + 1] : Rs[ci];
          blk = upd(blk, xm, xp, Rs[ci - PW], Rs[ci + PW], Rm[ci], Rp[ci], kr[i], ka[i], kb[i]);
          Bs[ci] = blk;
        }
        if (store && (rfl[i] & 4)) {
          double2 w;
          w.x = bsel(qb, red, blk);
          w.y = bsel(qb, blk, red);
          const long off = (long)rgx0[i] + (long)rgy[i] * sy;
          if (rgx0[i] + 1 < nx) *reinterpret_cast<double2 *>(dst + off) = w;
          else dst[off] = w.x;
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

}  // namespace

// workgroups of kernel `k` the whole device holds at once
template <class K>
static int resident_slots(K k, int nt) {
  int dev = 0, ncu = 0, per = 0;
  MGIC_HIP(hipGetDevice(&dev));
  MGIC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  MGIC_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, nt, 0));
  return (per > 0 ? per : 1) * (ncu > 0 ? ncu : 1);
}

// z chunk per workgroup: a workgroup streams kc planes plus `overlap` planes
// of pipeline fill; minimise rounds(kc) * (kc + overlap), where rounds is
// the number of waves of workgroups on `slots` resident slots (a partial
// last round costs a full one)
static int choose_kc(int tiles, int nz, int slots, int overlap) {
  int best = nz;
  double best_cost = 1e300;
  for (int kc = nz; kc >= 8; --kc) {
    const long nb = (long)tiles * ((nz + kc - 1) / kc);
    const long rounds = (nb + slots - 1) / slots;
    const double cost = (double)rounds * (kc + overlap);
    if (cost < best_cost * 0.999) {
      best_cost = cost;
      best = kc;
    }
  }
  return best;
}

template <class T, int TX, int TY, int NT>
static void launch_fused6(T *u_out, T *u_in, const T *rhs, const T *a, const T *b,
                          const BoxArgs &g, const StencilCoefs &s, bool zero_in, double *acc,
                          hipStream_t st) {
  // the domain BC is applied as the planes enter LDS (no fill launch)
  const int ntx = (g.nx + TX - 1) / TX, nty = (g.ny + TY - 1) / TY;
  static const int slots = resident_slots(k_gsrb_fused6<T, TX, TY, NT, false, false, false>, NT);
  static const int kc_mode = [] {
    const char *e = getenv("MGIC_KC_MODE");
    return e ? atoi(e) : 0;
  }();
  int kc = g.nz;
  if (kc_mode == 1) {  // >= 3072 workgroups
    while (kc > 16 && (long)ntx * nty * ((g.nz + kc - 1) / kc) < 3072) kc = (kc + 1) / 2;
  } else if (kc_mode >= 16) {
    kc = kc_mode < g.nz ? kc_mode : g.nz;
  } else {
    kc = choose_kc(ntx * nty, g.nz, slots, 5);
  }
  const int ntz = (g.nz + kc - 1) / kc;
  const int nblocks = ntx * nty * ntz;
  const dim3 grid((unsigned)nblocks), block(NT);
#define MGIC_F6(Z, B, A)                                                                     \
  k_gsrb_fused6<T, TX, TY, NT, Z, B, A><<<grid, block, 0, st>>>(u_out, acc, u_in, rhs, a, b, g, \
                                                                s, kc, ntx, nty, nblocks)
  if (acc) {  // last sweep of a V-cycle at depth 0: phi += e in the same pass
    if (zero_in) throw Error(kBadArg, "fused sweep: accumulate on a zero input");
    if (s.bconst) MGIC_F6(false, true, true);
    else MGIC_F6(false, false, true);
  } else if (zero_in) {
    if (s.bconst) MGIC_F6(true, true, false);
    else MGIC_F6(true, false, false);
  } else {
    if (s.bconst) MGIC_F6(false, true, false);
    else MGIC_F6(false, false, false);
  }
#undef MGIC_F6
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(kHipErr, std::string("fused sweep launch: ") + hipGetErrorString(e));
}

static long block_max_cells();

// tile shape, for measurement (MGIC_FUSED_VARIANT): 0 = 128x16 / 512 threads
// (default: one 106 KB workgroup per CU, 1 KB contiguous rows, u halo 1.29x,
// coefficient ring 1.16x), 1 = 60x8 / 256 (4 workgroups per CU); a 256x8 /
// 512 variant measured 0.90 ms, 128x16 / 1024 threads (four waves per SIMD,
// 107 VGPRs) 0.93 ms, loads two steps ahead (three rotating register sets)
// 0.89 ms: neither more waves nor deeper prefetch moves it.  512^3 sweep: 0.89 / 1.05 ms; 256^3: 0.142 /
// 0.168 ms.
static int fused_variant() {
  static int v = [] {
    const char *e = getenv("MGIC_FUSED_VARIANT");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// the sweep on the tiles covering the region o + [0, e) of the box (the
// whole box, or a slab along one face); cells of those tiles outside the
// region are computed too (the same values)
template <class T, int TX, int TY, int TZ, int NT>
static void launch_block(T *u_out, T *u_in, const T *rhs, const T *a, const T *b,
                         const BoxArgs &g, const StencilCoefs &s, bool zero_in, double *acc,
                         hipStream_t st, const int *o = nullptr, const int *e = nullptr) {
  const int ox = o ? o[0] : 0, oy = o ? o[1] : 0, oz = o ? o[2] : 0;
  const int ex = e ? e[0] : g.nx, ey = e ? e[1] : g.ny, ez = e ? e[2] : g.nz;
  if (ox & 1) throw Error(kBadArg, "block sweep: odd x origin");
  const int ntx = (ex + TX - 1) / TX, nty = (ey + TY - 1) / TY, ntz = (ez + TZ - 1) / TZ;
  const int nblocks = ntx * nty * ntz;
  if (nblocks <= 0) return;
  const dim3 grid((unsigned)nblocks), block(NT);
#define MGIC_BK(Z, B, A)                                                                     \
  k_gsrb_block<T, TX, TY, TZ, NT, Z, B, A><<<grid, block, 0, st>>>(                          \
      u_out, acc, u_in, rhs, a, b, g, s, ntx, nty, nblocks, ox, oy, oz)
  if (acc) {
    if (zero_in) throw Error(kBadArg, "fused sweep: accumulate on a zero input");
    if (s.bconst) MGIC_BK(false, true, true);
    else MGIC_BK(false, false, true);
  } else if (zero_in) {
    if (s.bconst) MGIC_BK(true, true, false);
    else MGIC_BK(true, false, false);
  } else {
    if (s.bconst) MGIC_BK(false, true, false);
    else MGIC_BK(false, false, false);
  }
#undef MGIC_BK
  hipError_t err = hipGetLastError();
  if (err != hipSuccess)
    throw Error(kHipErr, std::string("block sweep launch: ") + hipGetErrorString(err));
}

// boxes of at most this many cells take the block kernel (MGIC_BLOCK_MAX_CELLS;
// 0 = never); MGIC_BLOCK_VARIANT picks its tile for measurement.  100^3: the
// 128^3 bottom of the 512^3 V-cycle runs its sweep pairs through the
// two-sweep kernel (two launches instead of four; V-cycle +0.1..0.6%, three
// rounds, round 3), while the 64^3-per-rank bottom of the 8-GPU split and its
// deep-halo grown boxes (68^3) keep the one-shot block kernel.  (Round 2's
// 132^3 kept the grown 128^3-per-rank boxes here: 20 us per sweep against 31
// streamed with single sweeps.)
static long block_max_cells() {
  static long v = [] {
    const char *e = getenv("MGIC_BLOCK_MAX_CELLS");
    return e ? atol(e) : 100L * 100 * 100;
  }();
  return v;
}

long gsrb_block_max_cells() { return block_max_cells(); }

static int block_variant() {
  static int v = [] {
    const char *e = getenv("MGIC_BLOCK_VARIANT");
    return e ? atoi(e) : 0;
  }();
  return v;
}

void gsrb_sweep_fused(double *u_out, double *u_in, const double *rhs, const double *a,
                      const double *b, const BoxArgs &g, const StencilCoefs &s, bool zero_in,
                      double *acc, int kind, hipStream_t st) {
  if (kind == 3 || (kind != 2 && (long)g.nx * g.ny * g.nz <= block_max_cells())) {
    // 32x8x4 / 256 threads: 64^3 0.0094 ms, 128^3 0.026 ms per sweep; 32x8x8
    // 0.0116 / 0.0278; 16x8x8, 16x8x4, 32x4x4 (128 threads) were slower still
    if (block_variant() == 1)
      launch_block<double, 32, 8, 8, 256>(u_out, u_in, rhs, a, b, g, s, zero_in, acc, st);
    else
      launch_block<double, 32, 8, 4, 256>(u_out, u_in, rhs, a, b, g, s, zero_in, acc, st);
    return;
  }
  if (fused_variant() == 1)
    launch_fused6<double, 60, 8, 256>(u_out, u_in, rhs, a, b, g, s, zero_in, acc, st);
  else if ((g.nx + 131) / 132 < (g.nx + 127) / 128)
    // a box just over a multiple of 128 wide (the deep halo's grown boxes,
    // 256 + 2..4): 132 x 17 tiles (114 KB LDS, same 3 loads / 3 updates per
    // thread) instead of a mostly empty third column of 128-wide tiles
    launch_fused6<double, 132, 17, 512>(u_out, u_in, rhs, a, b, g, s, zero_in, acc, st);
  else
    launch_fused6<double, 128, 16, 512>(u_out, u_in, rhs, a, b, g, s, zero_in, acc, st);
}

// fp32 sweeps (the mixed-precision V-cycle): the same kernels with float
// elements and 8-B pairs; acc (phi) stays fp64
void gsrb_sweep_fused_f(float *u_out, float *u_in, const float *rhs, const float *a,
                        const float *b, const BoxArgs &g, const StencilCoefs &s, bool zero_in,
                        double *acc, int kind, hipStream_t st) {
  // fp32 streaming tiles: 128x32 with 1024 threads (95 KB LDS, four waves
  // per SIMD): 4.03 ms per 1024^3 sweep against 4.31-4.39 for 128x16 / 512
  // (MGIC_FUSED_F_VARIANT=1), 128x32 / 512 and 256x16 / 512 (4.45, 4.39)
  static const int fv = [] {
    const char *e = getenv("MGIC_FUSED_F_VARIANT");
    return e ? atoi(e) : 0;
  }();
  if (kind == 3 || (kind != 2 && (long)g.nx * g.ny * g.nz <= block_max_cells()))
    launch_block<float, 32, 8, 4, 256>(u_out, u_in, rhs, a, b, g, s, zero_in, acc, st);
  else if (fv == 1)
    launch_fused6<float, 128, 16, 512>(u_out, u_in, rhs, a, b, g, s, zero_in, acc, st);
  else
    launch_fused6<float, 128, 32, 1024>(u_out, u_in, rhs, a, b, g, s, zero_in, acc, st);
}

template <int TX, int TY, int NT>
static void launch_fused_rst(double *u_out, double *u_in, const double *rhs, const double *a,
                             const double *b, const BoxArgs &g, const StencilCoefs &s, double *rc,
                             const BoxArgs &cg, hipStream_t st) {
  const int ntx = (g.nx + TX - 1) / TX, nty = (g.ny + TY - 1) / TY;
  static const int slots = resident_slots(k_gsrb_fused_rst<TX, TY, NT, false>, NT);
  int kc = choose_kc(ntx * nty, g.nz, slots, 6);
  kc += kc & 1;  // coarse planes never straddle two workgroups
  if (kc > g.nz) kc = g.nz;
  const int ntz = (g.nz + kc - 1) / kc;
  const int nblocks = ntx * nty * ntz;
  const dim3 grid((unsigned)nblocks), block(NT);
  if (s.bconst)
    k_gsrb_fused_rst<TX, TY, NT, true><<<grid, block, 0, st>>>(u_out, rc, u_in, rhs, a, b, g, s, cg,
                                                              kc, ntx, nty, nblocks);
  else
    k_gsrb_fused_rst<TX, TY, NT, false><<<grid, block, 0, st>>>(u_out, rc, u_in, rhs, a, b, g, s, cg,
                                                               kc, ntx, nty, nblocks);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    throw Error(kHipErr, std::string("fused sweep+restrict launch: ") + hipGetErrorString(e));
}

bool gsrb_sweep_fused_restrict_applies(const BoxArgs &g, const BoxArgs &cg, int kind) {
  static const int enabled = [] {
    const char *e = getenv("MGIC_FUSED_RESTRICT");
    return e ? atoi(e) : 1;
  }();
  if (!enabled || kind == 0 || kind == 3) return false;
  if (kind != 2 && (long)g.nx * g.ny * g.nz <= block_max_cells()) return false;  // block kernel
  for (int f = 0; f < 6; ++f)
    if (!g.bcm[f]) return false;  // exchanged faces would need a 3-deep shell
  if ((g.nx | g.ny | g.nz) & 1) return false;
  return cg.nx * 2 == g.nx && cg.ny * 2 == g.ny && cg.nz * 2 == g.nz;
}

void gsrb_sweep_fused_restrict(double *u_out, double *u_in, const double *rhs, const double *a,
                               const double *b, const BoxArgs &g, const StencilCoefs &s,
                               double *rc, const BoxArgs &cg, hipStream_t st) {
  launch_fused_rst<128, 16, 512>(u_out, u_in, rhs, a, b, g, s, rc, cg, st);
}

}  // namespace kern
}  // namespace mgic
