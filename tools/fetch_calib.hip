// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE / TCC_EA0_RDREQ on
// gfx950 for the access shapes of the two-sweep kernel (measurement only;
// MI355X_MICROARCH.md: "other access widths are uncalibrated").  Each kernel
// reads a known number of distinct bytes once; run under
//   rocprofv3 --pmc FETCH_SIZE -- tools/fetch_calib
// and compare FETCH_SIZE (KiB) with the bytes printed here.
//   aligned   16 B per lane, waves on 1-KiB-aligned contiguous spans
//   shifted   the same, every wave's span starting 8 B into a line (the odd
//             rows of the kernel's shifted pairings)
//   halfline  each 128-B line read in its upper 64 B only (8 B per lane)
//   tilerows  the kernel's u rows: 37 pairs from x0-6, rows 4352 B apart,
//             16-B pair loads, even and odd shift alternating by row
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__global__ void k_aligned(const double2 *__restrict__ p, long n, double *out) {
  double acc = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    acc += p[i].x + p[i].y;
  if (acc == 12345.0) out[0] = acc;
}

__global__ void k_shifted(const char *__restrict__ base, long nwaves, double *out) {
  // wave w reads bytes [w * 1024 + 8, w * 1024 + 1032) as 64 lanes x 16 B
  double acc = 0;
  const int lane = threadIdx.x & 63;
  for (long w = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6; w < nwaves;
       w += ((long)gridDim.x * blockDim.x) >> 6) {
    const double *q = reinterpret_cast<const double *>(base + w * 1024 + 8 + 16 * lane);
    acc += q[0] + q[1];
  }
  if (acc == 12345.0) out[0] = acc;
}

__global__ void k_halfline(const double *__restrict__ p, long nlines, double *out) {
  // lane l of a wave reads double 8 + (l & 7) of line (wave's line base + l / 8)
  double acc = 0;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < nlines * 8;
       t += (long)gridDim.x * blockDim.x) {
    const long line = t >> 3;
    acc += p[line * 16 + 8 + (t & 7)];
  }
  if (acc == 12345.0) out[0] = acc;
}

__global__ void k_tilerows(const double *__restrict__ p, int nrows, int ntiles, long sy,
                           double *out) {
  // one wave per (row, tile): lanes 0..36 load the pair at x0 - 6 + 2m + s
  double acc = 0;
  const int lane = threadIdx.x & 63;
  const long wid = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nw = (long)nrows * ntiles;
  if (wid < nw && lane < 37) {
    const int row = (int)(wid / ntiles), tile = (int)(wid % ntiles);
    const int s = row & 1;
    const long x = 16 + (long)tile * 64 - 6 + 2 * lane + s;  // 16: the valid-lo offset
    const double *q = p + (long)row * sy + x;
    acc = q[0] + q[1];
  }
  if (acc == 12345.0) out[0] = acc;
}

int main() {
  const long bytes = 1L << 30;  // 1 GiB buffer
  char *buf = nullptr;
  double *out = nullptr;
  CK(hipMalloc(&buf, bytes + 4096));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 0, bytes + 4096));
  const dim3 g(4096), b(256);
  // a 512 MiB flush between kernels so no kernel reads another's lines from
  // the Infinity Cache
  char *flush = nullptr;
  CK(hipMalloc(&flush, 512L << 20));
  auto fl = [&] { CK(hipMemset(flush, 1, 512L << 20)); };
  fl();
  k_aligned<<<g, b>>>(reinterpret_cast<const double2 *>(buf), bytes / 16, out);
  CK(hipDeviceSynchronize());
  printf("aligned   distinct bytes %ld (%.1f KiB)\n", bytes, bytes / 1024.0);
  fl();
  const long nw = bytes / 1024 - 1;
  k_shifted<<<g, b>>>(buf, nw, out);
  CK(hipDeviceSynchronize());
  printf("shifted   distinct bytes %ld (%.1f KiB), lines touched %ld\n", nw * 1024, nw * 1024 / 1024.0,
         nw * 8 + 1);
  fl();
  const long nl = bytes / 128;
  k_halfline<<<g, b>>>(reinterpret_cast<const double *>(buf), nl, out);
  CK(hipDeviceSynchronize());
  printf("halfline  distinct bytes %ld (%.1f KiB), lines touched %ld\n", nl * 64, nl * 64 / 1024.0, nl);
  fl();
  // 512^3 rows: sy = 544 doubles, 8 tiles per row, 240000 rows
  const long sy = 544;
  const int ntiles = 8, nrows = (int)((bytes / 8 - 64) / sy);
  const int nwaves = nrows * ntiles;
  k_tilerows<<<(nwaves * 64 + 255) / 256, 256>>>(reinterpret_cast<const double *>(buf), nrows,
                                                   ntiles, sy, out);
  CK(hipDeviceSynchronize());
  // distinct: each row's cells x0-6 .. x0+67(+1) over its 8 tiles = cols 10 .. 16+512+4
  const long cells_row = (16 + 512 + 4 + 1) - 10;
  printf("tilerows  rows %d, distinct bytes %ld (%.1f KiB), data-line bytes %ld (%.1f KiB)\n", nrows,
         (long)nrows * cells_row * 8, nrows * cells_row * 8 / 1024.0, (long)nrows * 34 * 128,
         nrows * 34 * 128 / 1024.0);
  return 0;
}
