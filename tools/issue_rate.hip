// issue_rate.hip -- micro-measurement of gfx950 instruction issue rates with
// 16 waves per CU (the two-sweep kernel's occupancy): independent scalar
// adds, independent fp64 vector adds, and both interleaved.  Reports cycles
// (s_memtime) per instruction per wave.  Diagnostic only (tools/).
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHK(x)                                                      \
  do {                                                              \
    hipError_t e_ = (x);                                            \
    if (e_ != hipSuccess) {                                         \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                \
      return 1;                                                     \
    }                                                               \
  } while (0)

// 8 independent scalar adds (s_add_u32 on 8 SGPRs)
#define S8                                                                              \
  asm volatile(                                                                         \
      "s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %2, %2, 1\n s_add_u32 %3, %3, 1\n" \
      "s_add_u32 %4, %4, 1\n s_add_u32 %5, %5, 1\n s_add_u32 %6, %6, 1\n s_add_u32 %7, %7, 1\n" \
      : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)::"scc")
// 8 independent fp64 vector adds
#define V8                                                                                    \
  asm volatile(                                                                               \
      "v_add_f64 %0, %0, %8\n v_add_f64 %1, %1, %8\n v_add_f64 %2, %2, %8\n v_add_f64 %3, %3, %8\n" \
      "v_add_f64 %4, %4, %8\n v_add_f64 %5, %5, %8\n v_add_f64 %6, %6, %8\n v_add_f64 %7, %7, %8\n" \
      : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)        \
      : "v"(d))

template <int MODE>
__global__ __launch_bounds__(1024) void k_rate(double *out, unsigned long long *t, int iters,
                                               double d) {
  unsigned s0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), s1 = 1, s2 = 2, s3 = 3, s4 = 4, s5 = 5, s6 = 6, s7 = 7;
  double v0 = threadIdx.x, v1 = 1, v2 = 2, v3 = 3, v4 = 4, v5 = 5, v6 = 6, v7 = 7;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) { S8; S8; S8; S8; }
    if (MODE == 1) { V8; V8; V8; V8; }
    if (MODE == 2) { S8; V8; S8; V8; S8; V8; S8; V8; }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) t[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] =
      v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + (double)(s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7);
}

template <int MODE>
int run(int blocks, int threads, const char *name, int ninstr) {
  double *out;
  unsigned long long *t;
  CHK(hipMalloc(&out, sizeof(double) * blocks * threads));
  CHK(hipMalloc(&t, sizeof(unsigned long long) * blocks * 16));
  CHK(hipMemset(t, 0, sizeof(unsigned long long) * blocks * 16));
  const int iters = 2000;
  k_rate<MODE><<<blocks, threads>>>(out, t, iters, 1e-9);
  k_rate<MODE><<<blocks, threads>>>(out, t, iters, 1e-9);
  CHK(hipDeviceSynchronize());
  static unsigned long long h[4096 * 16];
  CHK(hipMemcpy(h, t, sizeof(unsigned long long) * blocks * 16, hipMemcpyDeviceToHost));
  double s = 0;
  int n = 0;
  for (int i = 0; i < blocks * 16; ++i)
    if (h[i]) {
      s += (double)h[i];
      ++n;
    }
  const double per = s / n / ((double)iters * ninstr);
  printf("%-28s blocks %4d x %4d threads: %.2f cycles per instruction per wave (waves/SIMD %d)\n",
         name, blocks, threads, per, threads / 256 > 0 ? threads / 256 : 1);
  CHK(hipFree(out));
  CHK(hipFree(t));
  return 0;
}

int main() {
  for (int th : {64, 256, 512, 1024}) {
    run<0>(256, th, "scalar adds", 32);
    run<1>(256, th, "fp64 vector adds", 32);
    run<2>(256, th, "scalar + fp64 interleaved", 64);
  }
  return 0;
}
