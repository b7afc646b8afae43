// fp64_lat.hip -- micro-measurement of gfx950 fp64 VALU dependent latency and
// issue rate (one wave; C independent add chains), s_memtime around an
// unrolled loop.  Diagnostic only.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int C>
__global__ void chain(double *out, unsigned long long *t, double x0, int iters) {
  double v[C];
#pragma unroll
  for (int c = 0; c < C; ++c) v[c] = x0 + threadIdx.x + c;
  const double d = out[0];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
#pragma unroll
      for (int c = 0; c < C; ++c) v[c] = v[c] + d;
    }
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) s += v[c];
  out[1 + threadIdx.x + blockIdx.x * blockDim.x] = s;
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) t[0] = t1 - t0;
}

template <int C>
void run(double *out, unsigned long long *t, int blocks, int threads) {
  const int iters = 256;
  chain<C><<<blocks, threads>>>(out, t, 1.0, iters);
  hipDeviceSynchronize();
  unsigned long long h = 0;
  hipMemcpy(&h, t, sizeof(h), hipMemcpyDeviceToHost);
  const double ops = (double)iters * 16 * C;
  printf("chains %2d  blocks %4d x %4d threads: %.2f cycles per dependent add (per wave), %.2f per add\n",
         C, blocks, threads, (double)h / (iters * 16), (double)h / ops);
}

int main() {
  double *out;
  unsigned long long *t;
  hipMalloc(&out, (1 << 22) * sizeof(double));
  hipMalloc(&t, 8);
  hipMemset(out, 0, 8);
  run<1>(out, t, 1, 64);
  run<2>(out, t, 1, 64);
  run<4>(out, t, 1, 64);
  run<8>(out, t, 1, 64);
  run<1>(out, t, 1, 256);
  run<4>(out, t, 1, 256);
  run<1>(out, t, 1, 512);
  run<2>(out, t, 1, 512);
  run<4>(out, t, 1, 512);
  run<8>(out, t, 1, 512);
  run<4>(out, t, 256, 512);
  return 0;
}
