// tb2_probe.hip -- timing harness for the two-sweep kernel (smoother_tb.hip):
// launches k_gsrb_tb2 directly on an n^3 box and reports its time by HIP
// events.  Not part of the library; built by tools/build_probe.sh.  (The
// round-2/3 decomposition probes -- parts of the step removed, per-phase
// stamps, tile drift -- hooked into the kernel through macros that were
// removed from the product in round 4; their results are in
// profiles/r03g_tb2_probes.txt and DESIGN.md 3, their code in git history.)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

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
  s.rcp_fast = argc > 4 ? atoi(argv[4]) : 1;  // 0: lambda by fp64 division (the generic path)
  std::vector<double *> f(4);
  std::vector<double> h(geo.total);
  // argv[5]: stagger the four arrays' bases by k * that many 128-B lines
  // (L2 set / channel placement experiment)
  const long stag = argc > 5 ? atol(argv[5]) : 0;
  std::vector<double *> alloc(4);
  for (int k = 0; k < 4; ++k) {
    MGIC_HIP(hipMalloc(&alloc[k], geo.total * sizeof(double) + 4096 * 128));
    f[k] = alloc[k] + k * stag * 16;
    for (long i = 0; i < geo.total; ++i)
      h[i] = k == 2 ? -1.0 - 0.5 * ((i * 2654435761u) % 1000) / 1000.0
                    : ((i * 40503u + k) % 2001) / 1000.0 - 1.0;
    MGIC_HIP(hipMemcpy(f[k], h.data(), geo.total * sizeof(double), hipMemcpyHostToDevice));
  }
  double *u_in = f[0] + geo.origin, *rhs = f[1] + geo.origin, *a = f[2] + geo.origin,
         *u_out = f[3] + geo.origin;
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
  printf("{\"n\": %d, \"zin\": %d, \"rcp_fast\": %d, \"ms_per_launch\": %.4f, "
         "\"compulsory_GBps\": %.1f}\n", n, zin, s.rcp_fast, ms,
         (zin ? 24.0 : 32.0) * cells / (ms * 1e-3) / 1e9);
  return 0;
}
