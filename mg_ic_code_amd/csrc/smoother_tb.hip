// smoother_tb.hip -- two red+black GSRB sweeps per launch (temporal blocking)
// for gfx950.
//
// Two consecutive levelGSRB calls (Source/VariableCoeffPoissonOperator.cpp:
// 290-331; arithmetic of GSRBHELMHOLTZVC3D, VariableCoeffPoissonOperatorF.
// ChF:56-139) on one box in one z-streaming launch, out of place (u_in ->
// u_out), bit-identical to four per-colour passes (same expressions,
// -ffp-contract=off).  Compulsory HBM traffic: u, rhs, aCoef read once and u
// written once per TWO sweeps (16 B/cell/sweep) against 32 for the single
// fused sweep.
//
// Pipeline.  A workgroup owns a TX x TY (x, y) tile and streams a chunk of
// z planes through an 8-slot LDS ring (red and black element of every x pair
// in separate arrays, so every LDS access is stride 1).  At step p it runs
// four colour passes on four planes, each on the tile grown by the cells the
// later passes read:
//     sweep-1 red   plane p     tile + 3
//     sweep-1 black plane p-1   tile + 2
//     sweep-2 red   plane p-3   tile + 1
//     sweep-2 black plane p-4   tile        -> stored
// (two barriers per step: the red passes, then the black ones)
// Every pass updates the ring array in place (red and black cells are
// disjoint), so one copy of each plane suffices.
//
// What makes it cheaper per cell than the single sweep run twice:
//   * a thread owns the same x pairs in all four passes, so each pair's
//     coefficients are prepared ONCE per plane -- rhs, alpha*a and lambda =
//     1/(alpha*a + 6 beta/dx^2) (.cpp:234-243, the one fp64 division) -- and
//     carried in registers, split into the red and the black element, to the
//     two passes that use them; the register sets rotate over a 4-step
//     unrolled loop, so nothing is moved;
//   * alpha = 1, beta = -1, bCoef = 1 (the reference's configuration,
//     Main_PoissonSolver.cpp:40, set_b_coef) is a specialisation that drops
//     three multiplications by exact constants (x*1 = x, x - (-1*y) = x + y
//     in IEEE arithmetic): 15 fp64 operations per cell update;
//   * the domain BC costs nothing in the passes of interior tiles: ghosts
//     enter the ring as ParseBC's images of the loaded cells, and since a
//     ghost is only ever read by the cell it images, a face cell's update
//     re-images its own ghosts (the value ParseBC writes before the next
//     colour pass); only tiles that reach an x / y domain face run that code.
// Exchanged faces (kBcMemory) read a 4-deep ghost shell of u and rhs/aCoef
// (the deep-halo exchange): the rings run onto the shell up to depth 3 and
// produce there exactly the neighbours' own values, as in the deep-halo
// schedule of op.cpp.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "kernels.hpp"
#include "sweep_util.hpp"

namespace mgic {
namespace kern {

namespace {

using sweep::bsel;

template <int N>
using IC = std::integral_constant<int, N>;

// Chosen variants (each measured A/B; the rejected ones were
// removed in round 4 -- their probe builds are in the git history):
//   kPF2: loads two steps ahead in the plain / ZIN launches (ACC: one);
//   SDY (steady step): the chunk's inner steps run a copy of the step without the z
//     range / face tests and plane clamps, with the coefficient sets copied
//     out of the load registers (reg_copy) and a static number of u loads per
//     step -- for fp32, zero-input and phi += e launches (the plain fp64
//     launch is bound by its memory traffic and keeps the generic step);
//   kZinShort: zero-input launches run sweep-1 red / black without the LDS
//     reads a zero input makes redundant;
//   kSkipOut: waves whose rows all lie outside the box skip every pass.
constexpr bool kPF2 = true;
constexpr bool kZinShort = true;
constexpr bool kSkipOut = true;

// Geometry.  Rows of the LDS ring are SHIFTED pairings: in row y of plane k
// pair m holds cells (X, X+1) with X = x0 - 6 + 2m + s, s = (x0 + y + k +
// sum(glo)) & 1, so the first element of every pair is RED ((i+j+k) even,
// GSRBHELMHOLTZVC3D's redBlack = 0) and the second BLACK.  No lane ever
// selects between its elements by colour: red values live in R, black ones
// in B, loaded and stored as 16-B pairs (8-B aligned in odd rows).  With the
// shift the neighbours are at fixed pair offsets:
//     red  (m):  x-1, x+1 = B[m-1], B[m];  y+-1, z+-1 = B[m-1+s] of that row / plane
//     black(m):  x-1, x+1 = R[m], R[m+1];  y+-1, z+-1 = R[m+s]
// (a neighbouring row or plane has the opposite shift).
template <int TX, int TY, int NT>
struct TB2 {
  static_assert(TX % 2 == 0, "TX must be even");
  static constexpr int PW = TX / 2 + 5;            // pairs per LDS row: X = x0-6+s .. x0+TX+2+s
  static constexpr int LH = TY + 8;                // LDS rows y0-4 .. y0+TY+3
  static constexpr int CP = PW * LH;               // pairs per plane
  static constexpr int SS = CP + 2 * PW + 2;       // slot stride: + a scratch row
  static constexpr int PAD = CP + PW + 1;          // write target of elements never updated
  static constexpr int NS = 8;                     // ring slots: planes p+1 .. p-5 live
  static constexpr int UW = PW - 1;                // update pairs per row: m = 1 .. PW-1
  static constexpr int NRP = UW * (TY + 6);        // update pairs: rows y0-3 .. y0+TY+2
  static constexpr int NL = (CP + NT - 1) / NT;
  static constexpr int NP = (NRP + NT - 1) / NT;
  static constexpr int RING = 2 * NS * SS + 2 * PW + 2;  // + what a PAD lane's reads overrun
  static constexpr int LDS_BYTES = RING * 8;
};

// a ParseBC ghost as one add: ghost_of(mode, c, v) == (sign ^ v) + gc
// exactly (c - v == c + (-v); v + (-0.0) == v for every v, signed zeros
// included), with sign/gc per domain face
// (built on the host, one per face, so the kernel holds no BC-mode logic)
template <class T>
struct TB2Ghosts {
  T c[6];
  unsigned sgn[6];  // 0x80000000: negate v (Dirichlet; the sign bit of T's top word)
};
template <class T>
TB2Ghosts<T> make_ghosts(const BoxArgs &g) {
  TB2Ghosts<T> r{};
  for (int f = 0; f < 6; ++f) {
    const int mode = g.bcm[f];
    r.sgn[f] = mode == kBcDirichlet ? 0x80000000u : 0u;
    r.c[f] = mode == kBcNeumannHom ? (T)-0.0 : (T)g.bcc[f];
  }
  return r;
}
__device__ __forceinline__ double ghost(const TB2Ghosts<double> &gg, int f, double v) {
  const long long b = __double_as_longlong(v) ^ ((long long)gg.sgn[f] << 32);
  return __longlong_as_double(b) + gg.c[f];
}
__device__ __forceinline__ float ghost(const TB2Ghosts<float> &gg, int f, float v) {
  return __uint_as_float(__float_as_uint(v) ^ gg.sgn[f]) + gg.c[f];
}

// the stencil constants rounded to T once (identity for double), as the
// single-sweep kernels' SC<T> (smoother.hip) and oracle/mixed.py do
template <class T>
struct TB2Coefs {
  T alpha, beta, dxinv, lamshift, bval;
  __device__ explicit TB2Coefs(const StencilCoefs &s)
      : alpha((T)s.alpha), beta((T)s.beta), dxinv((T)s.dxinv), lamshift((T)s.lamshift),
        bval((T)s.bval) {}
};
// A register copy the compiler cannot coalesce (steady steps, fp32): the
// coefficient sets are copied out of the in-flight load registers, so those
// keep one register per step parity across the unrolled loop's back edge --
// coalesced, the four steps' loads landed in four register sets and the back
// edge moved two of them, which waited (vmcnt) for loads issued in the same
// step and undid the two-step prefetch.
__device__ __forceinline__ double reg_copy(double x) { return x; }
__device__ __forceinline__ float reg_copy(float x) {
  float y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
  return y;
}
// 1.0 / d correctly rounded, for a normal d of moderate exponent: the
// instructions hipcc emits for an fp64 division with numerator 1 --
// v_div_scale (twice), v_rcp, two Newton steps, q = 1 * r, the remainder,
// v_div_fmas, v_div_fixup -- less the scale, the multiply by 1 and the
// fix-up, which return their input unchanged for |d| in [2^-500, 2^500]
// (StencilCoefs::rcp_fast, checked on the host over every lambda of the
// level): the same operations on the same values, so the same bits
// (.cpp:234-243), in 7 instructions instead of 11
__device__ __forceinline__ double rcp_div1(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(e, r, r);
}
// the fp32 form: hipcc's fp32 division with numerator 1 is v_div_scale
// (twice), v_rcp, one Newton step, q = 1 * r, two remainder / correction
// steps, v_div_fmas, v_div_fixup; without the scale, the multiply by 1 and the
// fix-up (identities for |d| in [2^-60, 2^60]: StencilCoefs::rcp_fast32), 7
// instructions instead of 11 on the same values
__device__ __forceinline__ float rcp_div1(float d) {
  const float r = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, r, 1.0f);
  const float r1 = __builtin_fmaf(e, r, r);
  const float e1 = __builtin_fmaf(-d, r1, 1.0f);
  const float q = __builtin_fmaf(e1, r1, r1);
  const float e2 = __builtin_fmaf(-d, q, 1.0f);
  return __builtin_fmaf(e2, r1, q);
}
template <class T> struct TB2Vec;
template <> struct TB2Vec<double> { using type = double2; };
template <> struct TB2Vec<float> { using type = float2; };

// One tile (x0, y0) of the box, planes [z0, z1).  FAST: alpha == 1, beta ==
// -1, bval == 1 (exact specialisation, see above), and lambda by rcp_div1;
// EM: the x (3) / y (12) domain faces the tile's rings reach (BC code
// compiled in for those; 0: an interior tile); UBC: every x / y domain face
// of the box has the same ghost rule (one ghost per update instead of one
// per face; without it EM is 15 and the faces come from ef).
template <class T, int TX, int TY, int NT, bool ZIN, bool ACC, bool FAST, int EM, bool UBC, bool TRIM>
__device__ __forceinline__ void tb2_tile(T *__restrict__ RB, T *__restrict__ uo, double *__restrict__ acc,
                                         const T *__restrict__ ui,
                                         const T *__restrict__ rhs,
                                         const T *__restrict__ a, const BoxArgs &g,
                                         const StencilCoefs &s64, const TB2Ghosts<T> &gg, int x0,
                                         int y0, int z0, int z1, int ef) {
  // (ACC: acc is the fp64 sum field whatever T; a float sweep adds (double)e)
  using F = TB2<TX, TY, NT>;
  using V = typename TB2Vec<T>::type;
  const TB2Coefs<T> s(s64);
  constexpr int PW = F::PW, CP = F::CP, SS = F::SS, UW = F::UW, NRP = F::NRP, NL = F::NL,
                NP = F::NP;
  const int nx = g.nx, ny = g.ny, nz = g.nz;
  const int tid = threadIdx.x;
  // The LDS ring, slot-interleaved: slot sl's red elements at RB + 2 sl SS,
  // its black ones SS further, so the other colour of a slot is a constant
  // byte offset away.  A lane's LDS accesses are a uniform slot base + one
  // of two loop-invariant lane offsets (cbm, coy) + a constant, which the
  // compiler folds into the ds instruction's offset field: one address add
  // per base instead of an index computation per access.
  constexpr unsigned ES = sizeof(T), SB = (unsigned)SS * ES;
  char *const RBc = reinterpret_cast<char *>(RB);
  auto slot_base = [&](int sl) { return RBc + (unsigned)sl * (2u * SB); };
  auto ldsp = [](char *base, unsigned off) { return base + off; };
  const long sy = g.sy, sz = g.sz;
  // the tile clipped to the box: ring levels are distances from it
  const int tx1 = min(x0 + TX, nx) - 1, ty1 = min(y0 + TY, ny) - 1;
  // updatable cells per direction: inside the box at a domain face; up to
  // depth 3 into the (4-deep) ghost shell at an exchanged face
  const int uxlo = g.bcm[0] ? 0 : -3, uxhi = g.bcm[1] ? nx - 1 : nx + 2;
  const int uylo = g.bcm[2] ? 0 : -3, uyhi = g.bcm[3] ? ny - 1 : ny + 2;
  const bool zdl = g.bcm[4] != 0, zdh = g.bcm[5] != 0;
  const int pstart = z0 - 3, pend = z1 + 3;
  // the shift s of a lane's row at plane pstart + t is (gsum + y + t) & 1
  const int gsum = g.glo[0] + g.glo[1] + g.glo[2] + x0 + pstart;
  // in-plane offsets are BYTE offsets from the plane's allocated corner
  // (x = -16, y = -4): non-negative 32-bit values, so every global access is
  // a uniform 64-bit plane base + a 32-bit lane offset
  const long corner = -16 - 4 * sy;
  auto clampi = [](int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); };
  // (steady steps: every plane they touch lies inside [-4, nz + 3], no clamp)
  auto plane_u = [&](const auto *f, int p) {
    return reinterpret_cast<const char *>(f + corner + (long)p * sz);
  };
  // corner of (clamped) plane p.  Beyond a z DOMAIN face no plane is read
  // but the ghost plane, which is loaded as the plane it images (fetch_u):
  // the fill / drain steps' loads there go to the face plane (L2 hits, no
  // ghost lines from HBM)
  const int pzlo = zdl ? 0 : -4, pzhi = zdh ? nz - 1 : nz + 3;
  auto plane = [&](const auto *f, int p) {
    return reinterpret_cast<const char *>(f + corner + (long)clampi(p, pzlo, pzhi) * sz);
  };
  // the lane offset is laundered per access: otherwise the compiler hoists
  // "array + lane offset" out of the z loop as 64-bit per-lane pointers (two
  // VGPRs each, for every array and offset variant) instead of using the
  // uniform plane base + 32-bit offset form
  auto at2 = [](const char *base, unsigned off) {
    asm volatile("" : "+v"(off));
    return *reinterpret_cast<const V *>(base + off);
  };
  // the fp64 sum field (ACC) at the byte offset of the same cell: offsets
  // scale by sizeof(double) / sizeof(T)
  constexpr unsigned kAccScale = (unsigned)(sizeof(double) / sizeof(T));
  auto at2d = [](const char *base, unsigned off) {
    asm volatile("" : "+v"(off));
    return *reinterpret_cast<const double2 *>(base + off);
  };
  auto boff = [&](int x, int y) {  // byte offset of cell (x, y) from the corner
    return (unsigned)(sizeof(T) * (16 + x + (long)(y + 4) * sy));
  };
  // ring slot of plane q (q >= pstart - 1 >= -4), and of plane q + j from
  // plane q's slot s0 (the steps derive every slot from one slot per step)
  auto es = [](int q) -> int { return q & 7; };
  auto eadd = [](int s0, int j) -> int { return (s0 + j) & 7; };
  // Load offset of pair (X, X+1) in row gy.  No pass reads a ghost element of
  // an x / y DOMAIN face (a face cell takes ghost(own value), see pass), so
  // (TRIM) the tiles that reach one (EM != 0) load no ghost line at all: a pair
  // wholly outside the box loads an in-box pair instead (its values are never
  // read), a row outside the box loads the face row, and the pair that
  // straddles the face loads the in-box pair next to it, its cell moved into
  // place after the load (sw 1: element 1 <- the loaded element 0, at x = 0;
  // sw 2: element 0 <- the loaded element 1, at x = nx - 1).  Interior tiles
  // never reach a ghost line.
  auto ld_off = [&](int X, int gy, int &sw) -> unsigned {
    sw = 0;
    int xl = clampi(X, -6, nx + 3), yl = clampi(gy, -4, ny + 3);
    // (x only where the x-face code is compiled in: swz moves the straddling
    // pair's cell, which a ring cell may read; likewise y)
    if constexpr (TRIM && (EM & 3) != 0) {
      if (g.bcm[0] && X < 0) {
        sw = X == -1 ? 1 : 0;
        xl = 0;
      }
      if (g.bcm[1] && X >= nx - 1) {
        sw = X == nx - 1 ? 2 : 0;
        xl = nx - 2;
      }
    }
    if constexpr (TRIM && (EM & 12) != 0) {
      if (g.bcm[2] && gy < 0) yl = 0;
      if (g.bcm[3] && gy > ny - 1) yl = ny - 1;
    }
    return boff(xl, yl);
  };
  // the pair's elements from a load at ld_off (sw as set there)
  auto swz = [](int sw, auto v) {
    if constexpr (TRIM && (EM & 3) != 0) {
      decltype(v) w;
      w.x = sw == 2 ? v.y : v.x;
      w.y = sw == 1 ? v.x : v.y;
      return w;
    } else {
      return v;
    }
  };
  // ---- loads of u (slot c = LDS pair index), per plane parity t ----------
  unsigned loff[2][NL];
  int lsw = 0;  // sw of (t, i) at bits 2 (t NL + i)
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int c = tid + i * NT;
    const int r = c / PW, m = c - r * PW;
    const int gy = y0 - 4 + r;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int X = x0 - 6 + 2 * m + ((gsum + gy + t) & 1);
      int sw;
      const unsigned o = ld_off(X, gy, sw);
      loff[t][i] = c < CP ? o : 0u;
      lsw |= (c < CP ? sw : 0) << (2 * (t * NL + i));
    }
  }
  // ---- update pairs: c = tid + i * NT -> row rr (y0-3+rr), pair m ---------
  // Each 32-lane half of a wave takes pairs 1..32 of one row (one row per
  // 32-lane LDS bank group: conflict-free reads); wave w holds rows w and
  // NR-1-w, so the inner rings' passes skip the waves of the outer rows
  // whole.  The rows' last UW-32 pairs go to the lanes after them.  Per
  // parity t: roff (global byte offset of the pair),
  // yzo (LDS index offset of the red element's y / z neighbours: s - 1; the
  // black one's is s), rinf (bits 0-3 / 4-7: domain faces the red / black
  // element borders; 8-9: store mask of the red / black element; 10-11: the
  // red / black element is ever updated -- ring level <= 3 and an updatable
  // cell).  A pass writes every lane's new value except for elements never
  // updated, which keep theirs: an element updated at ring W holds a value no
  // later pass reads once W falls below its level, so no pass needs the ring
  // test.
  static_assert(UW >= 32, "a row must fill a 32-lane group");
  constexpr int NR = TY + 6, MAIN = 32 * NR;
  static_assert(NR % 2 == 0 && MAIN <= NT * NP, "row pairing needs an even row count");
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave index (uniform)
  // the passes a wave skips whole: those of ring W < wthr.  A main wave whose
  // two rows both lie outside the box's updatable rows (a tile that overhangs
  // a y domain face, e.g. the last, 6-row tile row at 512 / 22) updates
  // nothing in any pass and skips them all (its elements keep their values,
  // which is what the passes would write; kSkipOut)
  int wthr = 3 - wv;
  if (kSkipOut && 2 * wv < NR) {
    const int ga = y0 - 3 + wv, gb = y0 - 3 + (NR - 1 - wv);
    if ((ga < uylo || ga > uyhi) && (gb < uylo || gb > uyhi)) wthr = 4;
  }
  wthr = __builtin_amdgcn_readfirstlane(wthr);
  // roff: the pair's load offset (ld_off; sw in rinf bits 12-13); its store
  // offset is roff moved back by the straddle shift (st_off)
  unsigned roff[2][NP];
  // cbm: byte offset of the element before the pair's (pair index c - 1);
  // coy[t]: of its y / z neighbour column minus one row (c + s - 1 - PW, s
  // the row's shift at parity t)
  unsigned cbm[NP], coy[2][NP];
  int rinf[2][NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int c = tid + i * NT, jt = c - MAIN;
    // wave w takes rows w and NR-1-w (one per 32-lane half), so the waves
    // of the outer rows -- idle in the inner rings' passes -- skip them whole
    // (with one pair per lane; NP > 1 keeps the mapping, not the skipping)
    const int rr = c < MAIN ? (((c >> 5) & 1) ? NR - 1 - (c >> 6) : (c >> 6)) : jt / (UW - 32);
    const int m = c < MAIN ? 1 + (c & 31) : 33 + jt - (jt / (UW - 32)) * (UW - 32);
    const int gy = y0 - 3 + rr;
    const bool row_ok = c < NRP;
    const int cix = row_ok ? (rr + 1) * PW + m : F::PAD;
    cbm[i] = (unsigned)(cix - 1) * ES;
    asm volatile("" : "+v"(cbm[i]));
    const int dy = gy < y0 ? y0 - gy : (gy > ty1 ? gy - ty1 : 0);
    const bool yok = row_ok && gy >= uylo && gy <= uyhi;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int sh = (gsum + gy + t) & 1;
      const int X = x0 - 6 + 2 * m + sh;
      int sw;
      const unsigned lo = ld_off(X, gy, sw);
      roff[t][i] = row_ok ? lo : 0u;
      if (!row_ok) sw = 0;
      coy[t][i] = (unsigned)(cix + sh - 1 - PW) * ES;
      // (opaque from here on: the compiler adds each use's constant in the
      // ds instruction's offset field instead of keeping lane offset +
      // constant combinations in registers)
      asm volatile("" : "+v"(coy[t][i]));
      int bits = 0;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int gx = X + e;
        const int dx = gx < x0 ? x0 - gx : (gx > tx1 ? gx - tx1 : 0);
        const bool upd_ok = yok && gx >= uxlo && gx <= uxhi && max(dx, dy) <= 3;
        bits |= (upd_ok ? 1 : 0) << (10 + e);
        const int f = ((g.bcm[0] && gx == 0) ? 1 : 0) | ((g.bcm[1] && gx == nx - 1) ? 2 : 0) |
                      ((g.bcm[2] && gy == 0) ? 4 : 0) | ((g.bcm[3] && gy == ny - 1) ? 8 : 0);
        bits |= (upd_ok ? f : 0) << (4 * e);
        const bool st = row_ok && gy >= y0 && gy <= ty1 && gx >= x0 && gx <= tx1;
        bits |= (st ? 1 : 0) << (8 + e);
      }
      rinf[t][i] = bits | (sw << 12);
    }
  }
  // z extent of each pass: the chunk grown by the pass's ring width,
  // clipped to the box at a domain face
  auto klo = [&](int w) { return zdl ? max(z0 - w, 0) : z0 - w; };
  auto khi = [&](int w) { return zdh ? min(z1 - 1 + w, nz - 1) : z1 - 1 + w; };
  int kl[4];
  unsigned kw[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    kl[w] = klo(w);
    kw[w] = (unsigned)(khi(w) - klo(w));
  }
  constexpr int kNone = -(1 << 28);
  const int zfl = zdl ? 0 : kNone, zfh = zdh ? nz - 1 : kNone;
  const int zgl = zdl ? -1 : kNone, zgh = zdh ? nz : kNone;

  // loads in flight, PF steps ahead (PF 1: u plane p+2 and rhs / aCoef of
  // plane p+1 while step p runs; PF 2: planes p+3 / p+2, one register set
  // per step parity)
  constexpr int PF = (kPF2 && !ACC) ? 2 : 1;
  // (SDY: the steady-state step, kSteady above)
  constexpr bool SDY = std::is_same<T, float>::value || ZIN || ACC;
  T pu0[PF][NL], pu1[PF][NL];
  T nr0[PF][NP], nr1[PF][NP], na0[PF][NP], na1[PF][NP];
  // coefficient sets (rhs, alpha*a, lambda): red of planes p .. p-3 (made
  // when the plane's pair arrives, last used by sweep-2 red three steps
  // later), black of planes p-1 .. p-4 (made one step later from rb / ab);
  // set J of the 4-step unrolled loop is made at step J and last used at
  // step J + 3
  T Rr[4][NP], Ra[4][NP], Rl[4][NP], Br[4][NP], Ba[4][NP], Bl[4][NP];
  T rb[NP], ab[NP];
  double ac0[NP], ac1[NP], an0[NP], an1[NP];  // ACC: acc pairs of planes p-4 / p-3
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    rb[i] = ab[i] = ac0[i] = ac1[i] = an0[i] = an1[i] = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) Rr[j][i] = Ra[j][i] = Rl[j][i] = Br[j][i] = Ba[j][i] = Bl[j][i] = 0.0;
  }

  // (sd: IC<1> in steady steps, which never meet a z face, a chunk end or a
  // clamped plane -- see the loop)
  auto fetch_u = [&](int t, int p, auto bc, auto sd) {
    constexpr int b = decltype(bc)::value;
    // a z ghost plane of a domain face loads the plane it images
    const char *pl = decltype(sd)::value ? plane_u(ui, p) : plane(ui, p == zgl ? 0 : p == zgh ? nz - 1 : p);
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      if (ZIN) {  // the input is identically +0 (a freshly zeroed correction)
        pu0[b][i] = 0.0;
        pu1[b][i] = 0.0;
      } else if (NL * NT <= CP || SDY || tid + i * NT < CP) {
        // (SDY: lanes past the plane load too -- from the plane's corner,
        // loff 0 -- and put skips them, so every step issues a static number
        // of loads and the waits for the loads of two steps ago do not also
        // wait for the previous step's stores)
        const V v = swz((lsw >> (2 * (t * NL + i))) & 3, at2(pl, loff[t][i]));
        pu0[b][i] = v.x;
        pu1[b][i] = v.y;
      }
    }
  };
  // a z ghost plane of a domain face, fetched as the plane it images ->
  // ParseBC's images.  (x / y ghosts are never stored: see pass.)
  auto image = [&](int p, auto bc, auto sd) {
    constexpr int b = decltype(bc)::value;
    if (!decltype(sd)::value && (p == zgl || p == zgh)) {
      const int zf = p == -1 ? 4 : 5;
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        pu0[b][i] = ghost(gg, zf, pu0[b][i]);
        pu1[b][i] = ghost(gg, zf, pu1[b][i]);
      }
    }
  };
  auto put = [&](int sl, auto bc) {  // into ring slot sl: red element -> R, black -> B
    constexpr int b = decltype(bc)::value;
    T *Rs = reinterpret_cast<T *>(slot_base(sl)), *Bs = Rs + SS;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      if (NL * NT > CP && tid + i * NT >= CP) continue;  // whole waves past the plane
      Rs[tid + i * NT] = pu0[b][i];
      Bs[tid + i * NT] = pu1[b][i];
    }
  };
  auto fetch_c = [&](int t, int p, auto bc, auto sd) {
    constexpr int b = decltype(bc)::value;
    constexpr bool SD = decltype(sd)::value;
    const char *pr = SD ? plane_u(rhs, p) : plane(rhs, p), *pa = SD ? plane_u(a, p) : plane(a, p);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int sw = (rinf[t][i] >> 12) & 3;
      const V vr = swz(sw, at2(pr, roff[t][i]));
      const V va = swz(sw, at2(pa, roff[t][i]));
      nr0[b][i] = vr.x;
      nr1[b][i] = vr.y;
      na0[b][i] = va.x;
      na1[b][i] = va.y;
    }
  };
  auto lam = [&](T aa) {  // .cpp:234-243 (a*alpha == alpha*a)
    if constexpr (FAST) return rcp_div1(aa + s.lamshift);
    else return (T)1 / (aa + s.lamshift);
  };
  auto upd = [&](T uc, T xm, T xp, T ym, T yp, T zm, T zp,
                 T rv, T aa, T lm) -> T {
    const T tx = (xp + xm) - (T)2 * uc;
    const T ty = (yp + ym) - (T)2 * uc;
    const T tz = (zp + zm) - (T)2 * uc;
    const T lap = (tx + ty) + tz;  // .ChF:111-120
    T lofdpsi = aa * uc;           // .ChF:107-108
    if (FAST) {
      lofdpsi = lofdpsi + lap * s.dxinv;  // .ChF:122-124 with bCoef 1, beta -1
    } else {
      const T ldpsi = lap * s.dxinv * s.bval;  // .ChF:122
      lofdpsi = lofdpsi - s.beta * ldpsi;           // .ChF:124
    }
    return uc - lm * (lofdpsi - rv);  // .ChF:127-128
  };
  // One colour pass on plane k (ring slot sl, parity t, coefficient set j)
  // over the ring of width W: every pair's LDS reads, then the update chains,
  // then the writes (the compiler cannot move one update's LDS accesses across
  // another's).  A ghost is read only by the cell it images, and ParseBC
  // fills it from that cell's value before every colour pass
  // (SetBCs.cpp:49-131), i.e. from the value the update starts from: an x / y
  // face cell takes its ghost neighbour as ghost(its own value) in registers
  // (branch-free selects), so x / y ghosts are never stored or loaded.  z
  // ghosts (face planes of z chunks only) are still written into the ring.
  // zc (ZIN launches only): 1 = sweep-1 red, 2 = sweep-1 black.  On a zero
  // input under homogeneous BCs (launch_tb2 checks) sweep-1 red sees u = 0
  // and six neighbours that are +-0 (loaded zeros, ParseBC's images of
  // them), so .ChF:107-128 reduce exactly to 0 - lam * (0 - rhs): lofdpsi
  // is +-0, (+-0 - rhs) == -rhs for rhs != 0 and +-0 otherwise, which gives
  // +0 either way.  Sweep-1 black starts from its own u = 0 (the constant
  // lets x - 2*0 fold to x, exact).  Both skip the LDS reads they no longer
  // need.
  auto pass = [&](auto zc, auto sd, bool red, int W, int t, int k, int sk, const T (&cr)[NP],
                  const T (&ca)[NP], const T (&cl)[NP]) {
    constexpr int ZC = decltype(zc)::value;
    constexpr bool SD = decltype(sd)::value;  // steady: k in range, not a z face plane
    if (!SD && (unsigned)(k - kl[W]) > kw[W]) return;  // uniform
    // rows beyond ring W (distance > W from the tile) are never read once
    // this pass is done, so waves holding only such rows skip it
    if (NP == 1 && W < wthr) return;  // (one pair per lane only)
    // slot bases (sk = es(k)) and the colours' offsets within a slot: X the
    // colour updated, N the other one; y / z neighbours of pair c are pair
    // c + o -+ PW (this plane) and c + o (planes k -+ 1), o = s - 1 (red) or
    // s (black)
    char *const Bk = slot_base(sk), *const Bm = slot_base(eadd(sk, -1)),
               *const Bp = slot_base(eadd(sk, 1));
    const unsigned XO = red ? 0u : SB, NO = red ? SB : 0u, RO = red ? 0u : ES;
    auto at = [](char *p, unsigned o) -> T & { return *reinterpret_cast<T *>(p + o); };
    char *a0[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) a0[i] = ldsp(Bk, cbm[i]);  // pair c - 1 of slot sk
    if constexpr (ZC == 1) {
      T v[NP];
#pragma unroll
      for (int i = 0; i < NP; ++i) v[i] = (T)0 - cl[i] * ((T)0 - cr[i]);
#pragma unroll
      for (int i = 0; i < NP; ++i) at(a0[i], XO + ES) = (rinf[t][i] >> 10) & 1 ? v[i] : (T)0;
      const bool zl = !SD && k == zfl, zh = !SD && k == zfh;
      if (zl || zh) {
        char *const Bz = zl ? Bm : Bp;
        const int zf = zl ? 4 : 5;
#pragma unroll
        for (int i = 0; i < NP; ++i) at(ldsp(Bz, coy[t][i]), NO + PW * ES) = ghost(gg, zf, v[i]);
      }
      return;
    }
    T uc[NP], xm[NP], xp[NP], ym[NP], yp[NP], zm[NP], zp[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      char *const a1 = ldsp(Bk, coy[t][i]);
      uc[i] = ZC == 2 ? (T)0 : at(a0[i], XO + ES);
      xm[i] = at(a0[i], NO + RO);       // N[c - 1] (red), N[c] (black)
      xp[i] = at(a0[i], NO + RO + ES);  // N[c], N[c + 1]
      ym[i] = at(a1, NO + RO);
      yp[i] = at(a1, NO + RO + 2 * PW * ES);
      zm[i] = at(ldsp(Bm, coy[t][i]), NO + RO + PW * ES);
      zp[i] = at(ldsp(Bp, coy[t][i]), NO + RO + PW * ES);
    }
    if constexpr (EM != 0) {
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int f = (rinf[t][i] >> (red ? 0 : 4)) & 15;
        if constexpr (UBC) {
          // one rule for every x / y domain face (gg slot 0): one ghost of
          // the cell's own value, selected into whichever neighbours it
          // images, for the directions whose faces the tile reaches
          const T gv = ghost(gg, 0, uc[i]);
          if constexpr ((EM & 3) != 0) {
            xm[i] = (f & 1) ? gv : xm[i];
            xp[i] = (f & 2) ? gv : xp[i];
          }
          if constexpr ((EM & 12) != 0) {
            ym[i] = (f & 4) ? gv : ym[i];
            yp[i] = (f & 8) ? gv : yp[i];
          }
        } else {
          // ef: the domain faces this tile's rings reach (uniform)
          if (ef & 1) xm[i] = (f & 1) ? ghost(gg, 0, uc[i]) : xm[i];
          if (ef & 2) xp[i] = (f & 2) ? ghost(gg, 1, uc[i]) : xp[i];
          if (ef & 4) ym[i] = (f & 4) ? ghost(gg, 2, uc[i]) : ym[i];
          if (ef & 8) yp[i] = (f & 8) ? ghost(gg, 3, uc[i]) : yp[i];
        }
      }
    }
    T v[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) v[i] = upd(uc[i], xm[i], xp[i], ym[i], yp[i], zm[i], zp[i], cr[i], ca[i], cl[i]);
#pragma unroll
    for (int i = 0; i < NP; ++i)
      at(a0[i], XO + ES) = (rinf[t][i] >> (red ? 10 : 11)) & 1 ? v[i] : uc[i];
    const bool zl = !SD && k == zfl, zh = !SD && k == zfh;
    if (zl || zh) {  // z ghosts of the face plane (every lane: an element
                     // never updated owns its ghost alone)
      char *const Bz = zl ? Bm : Bp;
      const int zf = zl ? 4 : 5;
#pragma unroll
      for (int i = 0; i < NP; ++i) at(ldsp(Bz, coy[t][i]), NO + RO + PW * ES) = ghost(gg, zf, v[i]);
    }
  };
  // plane k's tile cells -> u_out (or acc += them), from ring slot sl
  // Stores with a static instruction count (sweep::bstore): a lane's
  // elements outside the tile (or a plane outside the chunk) are dropped by
  // an out-of-range offset, so every step issues exactly NP * 2 stores with
  // no branch around them and the next step waits vmcnt(2) for its loads
  // instead of vmcnt(0), which would also wait for these stores.
  // the pair's store offset: its load offset, less the straddle shift
  auto st_off = [&](int t, int i) -> unsigned {
    unsigned o = roff[t][i];
    if constexpr (TRIM && (EM & 3) != 0) {
      const int sw = (rinf[t][i] >> 12) & 3;
      o = sw == 1 ? o - ES : (sw == 2 ? o + ES : o);
    }
    return o;
  };
  auto store = [&](int t, int k, int sl, auto sd) {  // sl = es(k)
    constexpr bool SD = decltype(sd)::value;
    const bool kin = SD || (k >= z0 && k < z1);  // uniform
    const int kk = SD ? k : clampi(k, z0, z1 - 1);
    char *dst = ACC ? reinterpret_cast<char *>(acc + corner + (long)kk * sz)
                    : reinterpret_cast<char *>(uo + corner + (long)kk * sz);
    const __amdgpu_buffer_rsrc_t rs = sweep::store_rsrc(dst);
    constexpr unsigned kDrop = sweep::kDrop;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int st = kin ? (rinf[t][i] >> 8) & 3 : 0;
      V w;
      char *const a = ldsp(slot_base(sl), cbm[i]);
      w.x = *reinterpret_cast<const T *>(a + ES);
      w.y = *reinterpret_cast<const T *>(a + SB + ES);
      if constexpr (ACC && !std::is_same<T, double>::value) {
        // phi += (double)e into the fp64 field (the fp32 sweeps of the mixed
        // V-cycle; smoother.hip's single sweep does the same)
        double2 d;
        d.x = ac0[i] + (double)w.x;
        d.y = ac1[i] + (double)w.y;
        const unsigned off = kAccScale * st_off(t, i);
        const unsigned o4 = st == 3 ? off : kDrop;
        const unsigned o2 = st == 1 ? off : (st == 2 ? off + (unsigned)sizeof(double) : kDrop);
        const double e = st == 1 ? d.x : d.y;
        sweep::bstore(rs, d, o4);
        sweep::bstore(rs, e, o2);
        continue;
      }
      if constexpr (ACC) {  // phi += e (incr, scale 1) in the same pass
        w.x = ac0[i] + w.x;
        w.y = ac1[i] + w.y;
      }
      const unsigned off = st_off(t, i);
      // both elements (st 3) as one pair store; a single one (st 1 / 2, the
      // tile's x edges) as an element store
      const unsigned o4 = st == 3 ? off : kDrop;
      const unsigned o2 = st == 1 ? off : (st == 2 ? off + (unsigned)sizeof(T) : kDrop);
      const T e = st == 1 ? w.x : w.y;
      sweep::bstore(rs, w, o4);
      sweep::bstore(rs, e, o2);
    }
  };
  // One pipeline step at plane p (t: its parity relative to pstart; ring
  // slots es(q)), two barriers:
  //   phase A: sweep-1 red of plane p (ring 3), sweep-2 red of plane p-3 (ring 1)
  //   phase B: sweep-1 black of plane p-1 (ring 2), sweep-2 black of plane
  //            p-4 (the tile) + its store
  // The two passes of a phase touch disjoint planes; phase A reads black
  // cells only, phase B red ones.  Live ring planes p+1 .. p-5; plane p+1 is
  // written over plane p-7.
  auto step = [&](auto tc, auto sd, int p) {
    // J: position in the 4-step unrolled loop; T / U: parity of p / of p +- 1;
    // coefficient sets live in slot J (made this step) .. slot J3 (made
    // three steps ago, last use), so no register moves between steps
    constexpr int J = decltype(tc)::value, PT = J & 1, PU = PT ^ 1;
    constexpr int J0 = J, J3 = (J + 1) & 3;
    constexpr int FB = PF == 2 ? (J & 1) : 0;  // in-flight register set consumed / refilled
    using ICF = IC<FB>;
    using SDC = decltype(sd);
    asm volatile("" : "+s"(p));  // opaque: plane-derived values are recomputed, not kept live
    // coefficient sets: black of plane p-1 from the raw black element, red
    // of plane p from its pair fetched last step (alpha * a, .ChF:107)
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      Br[J0][i] = rb[i];
      Ba[J0][i] = FAST ? ab[i] : s.alpha * ab[i];
      Bl[J0][i] = lam(Ba[J0][i]);
      Rr[J0][i] = reg_copy(nr0[FB][i]);
      Ra[J0][i] = FAST ? reg_copy(na0[FB][i]) : s.alpha * na0[FB][i];
      Rl[J0][i] = lam(Ra[J0][i]);
      rb[i] = reg_copy(nr1[FB][i]);
      ab[i] = reg_copy(na1[FB][i]);
    }
    const int E0 = es(p);  // this step's slots derive from this one
    image(p + 1, ICF{}, SDC{});
    put(eadd(E0, 1), ICF{});
    auto fc = [&] {
      if (PF == 2) fetch_c(PT, p + 2, ICF{}, SDC{});
      else fetch_c(PU, p + 1, ICF{}, SDC{});
    };
    auto fa = [&] {
      if constexpr (ACC) {
        const char *pl = SDC::value ? plane_u(acc, p - 3) : plane(acc, p - 3);
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          ac0[i] = an0[i];
          ac1[i] = an1[i];
          const double2 v = swz((rinf[PU][i] >> 12) & 3, at2d(pl, kAccScale * roff[PU][i]));
          an0[i] = v.x;
          an1[i] = v.y;
        }
      }
    };
    auto fu = [&] {
      if (PF == 2) fetch_u(PU, p + 3, ICF{}, SDC{});
      else fetch_u(PT, p + 2, ICF{}, SDC{});
    };
    // The step's global loads are issued in three places, not in one burst
    // (round 5): u of plane p+3 here, rhs / aCoef of plane p+2 between the
    // two red passes, acc at the start of the black phase.  All 16 waves of
    // all CUs issuing every load of a step at once filled the memory
    // pipeline's queues: the waves stalled at issue for most of the step's
    // first phase, the colour passes queued behind them (DESIGN.md 3,
    // "Spread load issue": 512^3 plain launch -4.5%, 256^3 -6%, V-cycle
    // +2.5%; the stores and other placements measured no better).
    fu();
    __syncthreads();
    pass(IC<(ZIN && kZinShort) ? 1 : 0>{}, SDC{}, true, 3, PT, p, E0, Rr[J0], Ra[J0], Rl[J0]);
    fc();
    pass(IC<0>{}, SDC{}, true, 1, PU, p - 3, eadd(E0, -3), Rr[J3], Ra[J3], Rl[J3]);
    __syncthreads();
    fa();
    pass(IC<(ZIN && kZinShort) ? 2 : 0>{}, SDC{}, false, 2, PU, p - 1, eadd(E0, -1), Br[J0], Ba[J0], Bl[J0]);
    pass(IC<0>{}, SDC{}, false, 0, PT, p - 4, eadd(E0, -4), Br[J3], Ba[J3], Bl[J3]);
    store(PT, p - 4, eadd(E0, -4), SDC{});
  };

  fetch_u(1, pstart - 1, IC<0>{}, IC<0>{});
  image(pstart - 1, IC<0>{}, IC<0>{});
  put(es(pstart - 1), IC<0>{});
  fetch_u(0, pstart, IC<0>{}, IC<0>{});
  image(pstart, IC<0>{}, IC<0>{});
  put(es(pstart), IC<0>{});
  fetch_u(1, pstart + 1, IC<0>{}, IC<0>{});
  fetch_c(0, pstart, IC<0>{}, IC<0>{});
  if (PF == 2) {
    fetch_u(0, pstart + 2, IC<PF - 1>{}, IC<0>{});
    fetch_c(1, pstart + 1, IC<PF - 1>{}, IC<0>{});
  }
  // (up to three steps past pend: their passes and stores fall outside every
  // range test, their loads are clamped)
  // Steady 4-step groups (SDY): steps p .. p+3 with z0 + 5 <= p and
  // p + 3 <= z1 - 4.  Every pass of such a step is inside its z range (the
  // tile pass needs p - 4 >= z0, the others less), none is on a domain face
  // plane (p - 4 >= 1 > 0, p <= nz - 4 < nz - 1), the loaded planes p + 2,
  // p + 3 are below z1 <= nz (no z ghost plane to image) and the stored plane
  // p - 4 lies in [z0, z1): their range tests, face tests and plane clamps are
  // compiled out.  pstart + 8 == z0 + 5, so the first steady group keeps the
  // 4-step alignment of the register sets.
  // (three loops: fill, steady, drain; the fill takes the first two groups)
  auto group = [&](auto sd, int p) {
    step(IC<0>{}, sd, p);
    step(IC<1>{}, sd, p + 1);
    step(IC<2>{}, sd, p + 2);
    step(IC<3>{}, sd, p + 3);
  };
  const int ssh = z1 - 7;
  int p = pstart;
  if (SDY) {
    for (; p < pstart + 8 && p <= pend; p += 4) group(IC<0>{}, p);
    for (; p <= ssh; p += 4) group(IC<1>{}, p);
  }
  for (; p <= pend; p += 4) group(IC<0>{}, p);
}


template <class T, int TX, int TY, int NT, bool ZIN, bool ACC, bool FAST, bool UBC, bool TRIM>
__global__ __launch_bounds__(NT) void k_gsrb_tb2(T *__restrict__ uo,
                                                 double *__restrict__ acc,
                                                 const T *__restrict__ ui,
                                                 const T *__restrict__ rhs,
                                                 const T *__restrict__ a,
                                                 const BoxArgs g, const StencilCoefs s,
                                                 const TB2Ghosts<T> gg, int kc, int ntx, int nty,
                                                 int nblocks, const int *__restrict__ skip,
                                                 int rw) {
  using F = TB2<TX, TY, NT>;
  __shared__ T RB[F::RING];  // per ring slot: the red element of every pair, then the black
  if (skip && *skip) return;  // a device-side solve has stopped (BicgState::done)
  // (rw: workgroups resident per XCD for the round-major order; 0: xcd_tile)
  const int L = rw > 0 ? sweep::round_tile(blockIdx.x, nblocks, rw) : sweep::xcd_tile(blockIdx.x, nblocks);
  const int x0 = (L % ntx) * TX, y0 = ((L / ntx) % nty) * TY;
  const int z0 = (L / (ntx * nty)) * kc;
  const int z1 = min(z0 + kc, g.nz);
  // uniform: the x / y domain faces the tile's rings (3 cells) reach
  const int ef = (g.bcm[0] && x0 <= 3 ? 1 : 0) | (g.bcm[1] && min(x0 + TX, g.nx) + 3 >= g.nx ? 2 : 0) |
                 (g.bcm[2] && y0 <= 3 ? 4 : 0) | (g.bcm[3] && min(y0 + TY, g.ny) + 3 >= g.ny ? 8 : 0);
#define MGIC_TILE(EM)                                                                             \
  tb2_tile<T, TX, TY, NT, ZIN, ACC, FAST, EM, UBC, TRIM>(RB, uo, acc, ui, rhs, a, g, s, gg, x0, y0,  \
                                                         z0, z1, ef)
  // (uniform) an x-face or a y-face tile runs only that direction's ghost code
  if (!ef) MGIC_TILE(0);
  else if (UBC && !(ef & 12)) MGIC_TILE(UBC ? 3 : 15);
  else if (UBC && !(ef & 3)) MGIC_TILE(UBC ? 12 : 15);
  else MGIC_TILE(15);
#undef MGIC_TILE
}

template <class T, int TX, int TY, int NT>
int tb2_resident_slots() {
  static const int slots = [] {
    int dev = 0, ncu = 0, per = 0;
    MGIC_HIP(hipGetDevice(&dev));
    MGIC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    MGIC_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per, k_gsrb_tb2<T, TX, TY, NT, false, false, true, true, false>, NT, 0));
    return (per > 0 ? per : 1) * (ncu > 0 ? ncu : 1);
  }();
  return slots;
}

// z chunk per workgroup: minimise rounds(kc) * (kc + pipeline fill), the
// fill being 7 steps rounded up with the chunk to the 2-step unroll.  Chunks
// go down to 4 planes (MGIC_TB2_KCMIN, for A/Bs): a 128^3 box of 12 tiles
// then takes 19 chunks of 7 (228 workgroups, one round) instead of 15 of 9
int tb2_choose_kc(int tiles, int nz, int slots) {
  static const int kc_min = [] {
    const char *e = getenv("MGIC_TB2_KCMIN");
    const int v = e ? atoi(e) : 4;
    return v < 1 ? 1 : v;
  }();
  int best = nz;
  double best_cost = 1e300;
  for (int kc = nz; kc >= kc_min; --kc) {
    const long nb = (long)tiles * ((nz + kc - 1) / kc);
    const long rounds = (nb + slots - 1) / slots;
    const double cost = (double)rounds * (double)(((kc + 7 + 1) / 2) * 2);
    if (cost < best_cost * 0.999) {
      best_cost = cost;
      best = kc;
    }
  }
  return best;
}

// the launch geometry of one two-sweep launch (tiles, z chunk, blocks)
template <class T, int TX, int TY, int NT>
struct TB2Geom {
  int ntx, nty, kc, nblocks;
  explicit TB2Geom(const BoxArgs &g) {
    ntx = (g.nx + TX - 1) / TX;
    nty = (g.ny + TY - 1) / TY;
    // the raw buffer stores address a plane with unsigned 32-bit byte offsets
    // and drop masked lanes at kDrop = 2^31: every in-plane offset must stay
    // below that, or valid stores would be dropped silently
    if ((double)(g.ny + 8) * (double)g.sy * sizeof(T) >= 2147483648.0)
      throw Error(kBadArg, "two-sweep launch: a plane exceeds the 2 GB buffer-offset range");
    static const int kc_env = [] {
      const char *e = getenv("MGIC_TB2_KC");
      return e ? atoi(e) : 0;
    }();
    kc = kc_env >= 1 ? (kc_env < g.nz ? kc_env : g.nz)
                     : tb2_choose_kc(ntx * nty, g.nz, tb2_resident_slots<T, TX, TY, NT>());
    nblocks = ntx * nty * ((g.nz + kc - 1) / kc);
  }
};

constexpr double kTrimMinCells = 160.0 * 160.0 * 160.0;

template <class T, int TX, int TY, int NT>
void launch_tb2(T *u_out, const T *u_in, const T *rhs, const T *a, const BoxArgs &g,
                const StencilCoefs &s, bool zero_in, double *acc, hipStream_t st,
                const int *skip = nullptr) {
  const TB2Geom<T, TX, TY, NT> G(g);
  const int ntx = G.ntx, nty = G.nty, kc = G.kc, nblocks = G.nblocks;
  // the fp32 ACC launch stores into the fp64 phi at twice the float offsets:
  // its planes must stay inside the buffer-offset range as doubles too
  if (acc && (double)(g.ny + 8) * (double)g.sy * sizeof(double) >= 2147483648.0)
    throw Error(kBadArg, "two-sweep launch: a phi plane exceeds the 2 GB buffer-offset range");
  const dim3 grid((unsigned)nblocks), block(NT);
  // FAST: the reference's constants (exact specialisation) and lambda in the
  // short reciprocal's range for T
  const bool fast = s.alpha == 1.0 && s.beta == -1.0 && s.bval == 1.0 &&
                    (std::is_same<T, double>::value ? s.rcp_fast : s.rcp_fast32);
  TB2Ghosts<T> gg = make_ghosts<T>(g);
  if (zero_in)  // the ZIN passes assume every ghost of a zero input is +-0
    for (int f = 0; f < 6; ++f)
      if (g.bcm[f] != kBcMemory && gg.c[f] != (T)0)
        throw Error(kBadArg, "two-sweep launch: zero input under an inhomogeneous BC");
  // UBC: the x / y domain faces share one ghost rule (the reference's
  // configuration: Dirichlet-0 everywhere); slot 0 then holds it
  bool ubc = true;
  int rep = -1;
  for (int f = 0; f < 4; ++f) {
    if (g.bcm[f] == kBcMemory) continue;
    if (rep < 0) rep = f;
    else ubc = ubc && gg.sgn[f] == gg.sgn[rep] &&
               std::memcmp(&gg.c[f], &gg.c[rep], sizeof(T)) == 0;  // (signed zeros differ)
  }
  if (ubc && rep > 0) {
    gg.sgn[0] = gg.sgn[rep];
    gg.c[0] = gg.c[rep];
  }
  // trim: the edge tiles skip the ghost lines of x / y domain faces (TRIM in
  // tb2_tile) -- on boxes large enough to stream from HBM (512^3 plain launch
  // 0.941 -> 0.911 ms, profiles/r06q_ghost_trim_ab.txt); on MALL-resident
  // ones (the 128^3 bottom) the straddle selects cost more than the lines
  // (MGIC_TB2_TRIM: a mask of launch kinds, for A/Bs; fp64 launches only)
  // the tile order: round-major (sweep::round_tile) when the grid has whole
  // dispatch rounds (MGIC_TB2_MAP: 0 xcd_tile, 1 round-major)
  static const int map_env = [] {
    const char *e = getenv("MGIC_TB2_MAP");
    return e ? atoi(e) : 1;
  }();
  const int rw = map_env == 1 ? tb2_resident_slots<T, TX, TY, NT>() / 8 : 0;
  static const int trim_mask = [] {
    const char *e = getenv("MGIC_TB2_TRIM");  // bits: 1 ZIN, 2 plain, 4 ACC; 8 any size
    return e ? atoi(e) : 7;
  }();
  // (fp64 only: the fp32 launch is not bound by its traffic, and the trimmed
  // one ran 4.87 against 4.59 ms at 1024^3)
  constexpr bool kDbl = std::is_same<T, double>::value;
  const int kind_bit = acc ? 4 : (zero_in ? 1 : 2);
  const bool trim = kDbl && fast && ubc && (trim_mask & kind_bit) &&
                    ((trim_mask & 8) || (double)g.nx * g.ny * g.nz >= kTrimMinCells);
#define MGIC_TB2(Z, A, FA)                                                                         \
  do {                                                                                             \
    if (ubc && FA && trim)                                                                         \
      k_gsrb_tb2<T, TX, TY, NT, Z, A, FA, true, FA && kDbl><<<grid, block, 0, st>>>(              \
          u_out, acc, u_in, rhs, a, g, s, gg, kc, ntx, nty, nblocks, skip, rw);                          \
    else if (ubc)                                                                                  \
      k_gsrb_tb2<T, TX, TY, NT, Z, A, FA, true, false><<<grid, block, 0, st>>>(                    \
          u_out, acc, u_in, rhs, a, g, s, gg, kc, ntx, nty, nblocks, skip, rw);                          \
    else                                                                                           \
      k_gsrb_tb2<T, TX, TY, NT, Z, A, FA, false, false><<<grid, block, 0, st>>>(                   \
          u_out, acc, u_in, rhs, a, g, s, gg, kc, ntx, nty, nblocks, skip, rw);                          \
  } while (0)
  if (acc) {
    if (zero_in) throw Error(kBadArg, "two-sweep launch: accumulate on a zero input");
    if (fast) MGIC_TB2(false, true, true);
    else MGIC_TB2(false, true, false);
  } else if (zero_in) {
    if (fast) MGIC_TB2(true, false, true);
    else MGIC_TB2(true, false, false);
  } else {
    if (fast) MGIC_TB2(false, false, true);
    else MGIC_TB2(false, false, false);
  }
#undef MGIC_TB2
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(kHipErr, std::string("two-sweep launch: ") + hipGetErrorString(e));
}

}  // namespace

bool gsrb_sweep_tb2_applies(const BoxArgs &g, const StencilCoefs &s, int kind) {
  if (!s.bconst || kind == 0 || kind == 3) return false;
  if (kind == 1 && (long)g.nx * g.ny * g.nz <= gsrb_block_max_cells()) return false;
  for (int f = 0; f < 6; ++f)  // the CF ghost rule of AMR levels is not folded here
    if (g.bcm[f] == kBcCFHom) return false;
  // a 4-deep shell must exist on every exchanged face; tiny boxes go to the
  // 3D-block kernel
  return g.nx >= 8 && g.ny >= 8 && g.nz >= 8;
}

// tile shape: a thread owns one x pair of the update region ((TX/2 + 4) x
// (TY + 6) pairs <= NT) and carries its coefficient sets in registers; 1024
// threads = four waves per SIMD at 128 VGPRs, 64 x 22 tiles (148 KB LDS).
// Measured and not kept: the same tile with 512 threads and two pairs each
// (1.79 vs 1.53 ms per 512^3 launch: fewer waves hide less of the pass
// latency); 58 x 22 (one u load per lane) 1.53 vs 1.36 ms -- a step costs
// about the same whatever the tile, so wide tiles win
void gsrb_sweep_tb2(double *u_out, const double *u_in, const double *rhs, const double *a,
                    const BoxArgs &g, const StencilCoefs &s, bool zero_in, double *acc,
                    hipStream_t st, const int *skip) {
  launch_tb2<double, 64, 22, 1024>(u_out, u_in, rhs, a, g, s, zero_in, acc, st, skip);
}

// fp32 (the mixed-precision V-cycle's smoother, BASELINE config C5): the same
// kernel on floats with the stencil constants rounded to float once, as the
// single-sweep fp32 kernel and oracle/mixed.py compute them (phi += e stays a
// separate fp64 sweep there)
void gsrb_sweep_tb2_f(float *u_out, const float *u_in, const float *rhs, const float *a,
                      const BoxArgs &g, const StencilCoefs &s, bool zero_in, double *acc,
                      hipStream_t st) {
  launch_tb2<float, 64, 22, 1024>(u_out, u_in, rhs, a, g, s, zero_in, acc, st);
}

}  // namespace kern
}  // namespace mgic
