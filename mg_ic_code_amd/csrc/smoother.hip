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

#include "kernels.hpp"

namespace mgic {
namespace kern {

namespace {

__device__ __forceinline__ double ghost_of(int mode, double c, double near) {
  return mode == kBcDirichlet ? (c - near) : (mode == kBcNeumannHom ? near : near + c);
}

constexpr int kThreads = 256;

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

constexpr int kTX = 64, kTY = 8;

}  // namespace

bool gsrb_sweep_fused_supported(const BoxArgs &g) {
  for (int f = 0; f < 6; ++f)
    if (g.bcm[f] == kBcMemory) return false;  // needs every face BC-folded
  return g.nx > 0 && g.ny > 0 && g.nz > 0;
}

void gsrb_sweep_fused(double *u_out, const double *u_in, const double *rhs, const double *a,
                      const double *b, const BoxArgs &g, const StencilCoefs &s, hipStream_t st) {
  const int tiles = ((g.nx + kTX - 1) / kTX) * ((g.ny + kTY - 1) / kTY);
  int kc = g.nz;  // z-chunk: enough workgroups to fill 256 CUs several times over
  while (kc > 16 && (long)tiles * ((g.nz + kc - 1) / kc) < 4096) kc = (kc + 1) / 2;
  const dim3 grid((unsigned)((g.nx + kTX - 1) / kTX), (unsigned)((g.ny + kTY - 1) / kTY),
                  (unsigned)((g.nz + kc - 1) / kc));
  k_gsrb_fused<kTX, kTY><<<grid, dim3(kThreads), 0, st>>>(u_out, u_in, rhs, a, b, g, s, kc);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(kHipErr, std::string("fused sweep launch: ") + hipGetErrorString(e));
}

}  // namespace kern
}  // namespace mgic
