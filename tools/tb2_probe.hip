// tb2_probe.hip -- diagnostic harness for the two-sweep kernel
// (smoother_tb.hip): launches k_gsrb_tb2 directly on an n^3 box and reports
// its time by HIP events and, with -DSTAMPS, s_memtime stamps taken by wave 0
// of a few workgroups at fixed points of each pipeline step (per-phase cycle
// breakdown).  Not part of the library; built by tools/build_probe.sh.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#ifdef STAMPS
#ifndef STAMP_T
#define STAMP_T 0  // the stamping thread (lane 0 of wave STAMP_T / 64)
#endif
__device__ unsigned long long g_stamps[4][64][12];
__device__ int g_probe_blocks[4];
#define TB2_STAMP(id, p)                                                              \
  do {                                                                                \
    if (threadIdx.x == STAMP_T) {                                                     \
      for (int w_ = 0; w_ < 4; ++w_)                                                  \
        if ((int)blockIdx.x == g_probe_blocks[w_] && (p) >= z0 + 40 && (p) < z0 + 104) \
          g_stamps[w_][(p) - z0 - 40][id] = __builtin_amdgcn_s_memtime();             \
    }                                                                                 \
  } while (0)
#endif

#ifdef DRIFT
// per-block progress: thread 0 stamps step p = z0 + 32k (k < 16) and the
// tile origin, so the host can see how far neighbouring tiles drift apart
__device__ unsigned long long g_drift[2048][16];
__device__ int g_tile[2048][4];  // x0, y0, z0, XCC the block ran on
#define TB2_STAMP(id, p)                                                              \
  do {                                                                                \
    if (id == 0 && threadIdx.x == 0 && (p) >= z0 && (p) < z0 + 512 && (((p) - z0) & 31) == 0) { \
      g_drift[blockIdx.x][((p) - z0) >> 5] = __builtin_amdgcn_s_memrealtime();           \
      unsigned xcc_;                                                                  \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc_));       \
      g_tile[blockIdx.x][0] = x0;                                                     \
      g_tile[blockIdx.x][1] = y0;                                                     \
      g_tile[blockIdx.x][2] = z0;                                                     \
      g_tile[blockIdx.x][3] = (int)xcc_;                                              \
    }                                                                                 \
  } while (0)
#endif

#include "../mg_ic_code_amd/csrc/smoother_tb.hip"

using namespace mgic;

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 512;
  const int zin = argc > 2 ? atoi(argv[2]) : 0;
  FabGeom geo = FabGeom::make(Box{{0, 0, 0}, {n - 1, n - 1, n - 1}});
  BoxArgs g{};
  g.nx = g.ny = g.nz = n;
  g.sy = geo.sy;
  g.sz = geo.sz;
  for (int f = 0; f < 6; ++f) {
    g.bcm[f] = argc > 3 && atoi(argv[3]) ? kBcMemory : kBcDirichlet;
    g.bcc[f] = 0.0;
  }
  StencilCoefs s{};
  s.alpha = 1.0;
  s.beta = -1.0;
  s.dx = 100.0 / n;
  s.dxinv = 1.0 / (s.dx * s.dx);
  s.lamshift = (2 * 3) * s.beta / (s.dx * s.dx);
  s.bconst = 1;
  s.bval = 1.0;
  std::vector<double *> f(4);
  std::vector<double> h(geo.total);
  for (int k = 0; k < 4; ++k) {
    MGIC_HIP(hipMalloc(&f[k], geo.total * sizeof(double)));
    for (long i = 0; i < geo.total; ++i)
      h[i] = k == 2 ? -1.0 - 0.5 * ((i * 2654435761u) % 1000) / 1000.0
                    : ((i * 40503u + k) % 2001) / 1000.0 - 1.0;
    MGIC_HIP(hipMemcpy(f[k], h.data(), geo.total * sizeof(double), hipMemcpyHostToDevice));
  }
  double *u_in = f[0] + geo.origin, *rhs = f[1] + geo.origin, *a = f[2] + geo.origin,
         *u_out = f[3] + geo.origin;
#ifdef STAMPS
  int blocks[4] = {0, 37, 300, 600};
  MGIC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_probe_blocks), blocks, sizeof(blocks)));
#endif
  hipEvent_t e0, e1;
  MGIC_HIP(hipEventCreate(&e0));
  MGIC_HIP(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w)
    kern::gsrb_sweep_tb2(u_out, u_in, rhs, a, g, s, zin, nullptr, nullptr);
  const int reps = 10;
  MGIC_HIP(hipEventRecord(e0, nullptr));
  for (int r = 0; r < reps; ++r)
    kern::gsrb_sweep_tb2(u_out, u_in, rhs, a, g, s, zin, nullptr, nullptr);
  MGIC_HIP(hipEventRecord(e1, nullptr));
  MGIC_HIP(hipEventSynchronize(e1));
  float ms = 0;
  MGIC_HIP(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double cells = (double)n * n * n;
  printf("{\"n\": %d, \"zin\": %d, \"ms_per_launch\": %.4f, \"compulsory_GBps\": %.1f}\n", n, zin,
         ms, (zin ? 24.0 : 32.0) * cells / (ms * 1e-3) / 1e9);
#ifdef STAMPS
  constexpr int kStamps = 9;  // TB2_STAMP ids 0..8 per step (smoother_tb.hip)
  static unsigned long long st[4][64][12];
  MGIC_HIP(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st)));
  for (int w = 0; w < 4; ++w) {
    double acc[12] = {0};
    int cnt = 0;
    for (int p = 0; p < 63; ++p) {
      if (!st[w][p][0] || !st[w][p + 1][0]) continue;
      for (int i = 0; i < kStamps - 1; ++i) acc[i] += (double)(st[w][p][i + 1] - st[w][p][i]);
      acc[kStamps - 1] += (double)(st[w][p + 1][0] - st[w][p][kStamps - 1]);
      ++cnt;
    }
    printf("block %d: %d steps; memtime ticks per step by phase:", blocks[w], cnt);
    double tot = 0;
    for (int i = 0; i < kStamps; ++i) {
      printf(" %.0f", cnt ? acc[i] / cnt : 0.0);
      tot += cnt ? acc[i] / cnt : 0.0;
    }
    printf("  total %.0f\n", tot);
  }
#endif
#ifdef DRIFT
  static unsigned long long dr[2048][16];
  static int tl[2048][4];
  MGIC_HIP(hipMemcpyFromSymbol(dr, HIP_SYMBOL(g_drift), sizeof(dr)));
  MGIC_HIP(hipMemcpyFromSymbol(tl, HIP_SYMBOL(g_tile), sizeof(tl)));
  // blocks of the last launch: those with a stamp at k = 0
  std::vector<int> bs;
  for (int b = 0; b < 2048; ++b)
    if (dr[b][0]) bs.push_back(b);
  {  // where the blocks ran: XCC against blockIdx % 8, neighbours sharing an XCC
    int same_rr = 0, xs = 0, xn = 0, ys = 0, yn = 0;
    double xlag = 0, ylag = 0;
    for (int b : bs) {
      same_rr += tl[b][3] == b % 8;
      for (int c : bs) {
        if (tl[c][2] != tl[b][2]) continue;
        const bool xnb = tl[c][1] == tl[b][1] && tl[c][0] == tl[b][0] + 64;
        const bool ynb = tl[c][0] == tl[b][0] && tl[c][1] == tl[b][1] + 22;
        const double st = fabs((double)dr[c][0] - (double)dr[b][0]);
        if (xnb) { ++xn; xs += tl[c][3] == tl[b][3]; xlag += st; }
        if (ynb) { ++yn; ys += tl[c][3] == tl[b][3]; ylag += st; }
      }
    }
    printf("XCC == blockIdx %% 8 for %d of %zu blocks; x-neighbours on one XCC %d of %d (start lag %.0f x10ns), "
           "y-neighbours %d of %d (start lag %.0f x10ns)\n",
           same_rr, bs.size(), xs, xn, xn ? xlag / xn : 0.0, ys, yn, yn ? ylag / yn : 0.0);
    for (int b = 0; b < 12 && b < (int)bs.size(); ++b)
      printf("  block %d: tile (%d, %d, %d) XCC %d\n", bs[b], tl[bs[b]][0], tl[bs[b]][1], tl[bs[b]][2], tl[bs[b]][3]);
  }
  {  // time over the first 128 steps, interior vs edge tiles
    double ti = 0, te = 0;
    int ni = 0, ne = 0;
    for (int b : bs) {
      if (!dr[b][4]) continue;
      const double d = (double)(dr[b][4] - dr[b][0]);
      const bool edge = tl[b][0] <= 3 || tl[b][0] + 64 + 3 >= n || tl[b][1] <= 3 || tl[b][1] + 22 + 3 >= n;
      if (edge) { te += d; ++ne; } else { ti += d; ++ni; }
    }
    printf("128 steps: interior tiles %.0f x10ns (%d), edge tiles %.0f x10ns (%d)\n", ni ? ti / ni : 0.0, ni,
           ne ? te / ne : 0.0, ne);
  }
  for (int k = 0; k < 16; ++k) {
    unsigned long long lo = ~0ull, hi = 0;
    double nb = 0;
    int nn = 0;
    for (int b : bs) {
      if (!dr[b][k]) continue;
      lo = dr[b][k] < lo ? dr[b][k] : lo;
      hi = dr[b][k] > hi ? dr[b][k] : hi;
      for (int c : bs)  // x neighbour (same y0, x0 + 64)
        if (tl[c][2] == tl[b][2] && tl[c][1] == tl[b][1] && tl[c][0] == tl[b][0] + 64 && dr[c][k]) {
          nb += dr[c][k] > dr[b][k] ? (double)(dr[c][k] - dr[b][k]) : (double)(dr[b][k] - dr[c][k]);
          ++nn;
        }
    }
    if (!hi) continue;
    printf("plane z0+%3d: %zu blocks, spread %llu x10ns, mean |x-neighbour lag| %.0f x10ns\n", 32 * k,
           bs.size(), hi - lo, nn ? nb / nn : 0.0);
  }
#endif
  return 0;
}
