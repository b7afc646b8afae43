// ipc_probe.hip -- feasibility probe for the cross-process halo transport
// (measurement tool, not product code): two processes on ONE device (or one
// per device) map each other's buffers with hipIpcOpenMemHandle and hand off
// data with device-side flags.
//
//   ipc_probe <rank> <dir> <iters> <bytes> <device>
// Each rank publishes two IPC handles (data: 2 x bytes, double-buffered by
// iteration parity; flags: a 4 KB uncached page) as <dir>/h<rank>, waits for
// the peer's file, opens it, then runs <iters> iterations of
//   put:  write the pattern (iter, rank) into the peer's data slot, release,
//         flag_peer[rank] = iter (last block of the grid, ticket)
//   wait: poll flag_mine[peer] >= iter (bounded), acquire, check every word.
// Prints one JSON line: errors, timeouts, us per iteration.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "rank %d: %s failed: %s\n", g_rank, #x, hipGetErrorString(e_)); \
      exit(3);                                                                    \
    }                                                                             \
  } while (0)

static int g_rank = 0;

struct Handles {
  hipIpcMemHandle_t data, flags;
};

// flags page layout (unsigned long long words): [0..7] arrival flag per peer
// rank, [8] local ticket, [9] timeouts, [10] errors
// MODE 0: plain stores, every block releases at system scope before its ticket
// MODE 1: non-temporal stores, every block drains (vmcnt), the last block
//         releases once and signals
// MODE 2: system-scope relaxed atomic stores (sc0 sc1), drained, last block
//         releases once and signals
template <int MODE>
__global__ void k_put(double *__restrict__ peer_data, unsigned long long *peer_flags,
                      unsigned long long *my_flags, long n, int rank, unsigned long long iter) {
  double *slot = peer_data + (iter & 1) * n;
  const double v = (double)iter * 8.0 + rank;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < n; t += (long)gridDim.x * blockDim.x) {
    const double x = v + (double)(t & 7) * 0.125;
    if constexpr (MODE == 0) slot[t] = x;
    else if constexpr (MODE == 1) __builtin_nontemporal_store(x, slot + t);
    else __hip_atomic_store(slot + t, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if constexpr (MODE == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned long long t =
        __hip_atomic_fetch_add(&my_flags[8], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t + 1 == iter * gridDim.x) {  // last block of this launch
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&peer_flags[rank], iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// MODE 3: 16-B write-through buffer stores (sc0 sc1), every block drains and
// adds 1 to the peer's counter (no fence, no ticket); the consumer polls the
// counter up to iter * blocks and reads with 16-B sc0 sc1 buffer loads
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__global__ void k_put3(double *__restrict__ peer_data, unsigned long long *peer_flags, long n,
                       int rank, unsigned long long iter) {
  double *slot = peer_data + (iter & 1) * n;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(slot, (short)0, 0x7fffffff, 0x00020000);
  const double v = (double)iter * 8.0 + rank;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; 2 * t < n; t += (long)gridDim.x * blockDim.x) {
    double2 x;
    x.x = v + (double)((2 * t) & 7) * 0.125;
    x.y = v + (double)((2 * t + 1) & 7) * 0.125;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, x), rs, (unsigned)(16 * t), 0, 17);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(&peer_flags[rank], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_wait_check3(const double *__restrict__ my_data, unsigned long long *my_flags, long n,
                              int peer, unsigned long long iter) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    int good = 1;
    while (__hip_atomic_load(&my_flags[peer], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) <
           iter * gridDim.x) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > 200000000ull) {
        good = 0;
        break;
      }
    }
    ok = good;
    if (!good)
      __hip_atomic_fetch_add(&my_flags[9], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!ok) return;
  const double *slot = my_data + (iter & 1) * n;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(slot), (short)0, 0x7fffffff, 0x00020000);
  const double v = (double)iter * 8.0 + peer;
  unsigned long long bad = 0;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; 2 * t < n; t += (long)gridDim.x * blockDim.x) {
    const double2 x = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(16 * t), 0, 17));
    bad += x.x != v + (double)((2 * t) & 7) * 0.125;
    bad += x.y != v + (double)((2 * t + 1) & 7) * 0.125;
  }
  if (bad) __hip_atomic_fetch_add(&my_flags[10], bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_fill(double *__restrict__ d, long n, double v) {
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < n; t += (long)gridDim.x * blockDim.x)
    d[t] = v + (double)(t & 7) * 0.125;
}

__global__ void k_wait_check(const double *__restrict__ my_data, unsigned long long *my_flags, long n,
                             int peer, unsigned long long iter) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    int good = 1;
    while (__hip_atomic_load(&my_flags[peer], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < iter) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > 200000000ull) {  // 2 s at 100 MHz
        good = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ok = good;
    if (!good)
      __hip_atomic_fetch_add(&my_flags[9], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!ok) return;
  const double *slot = my_data + (iter & 1) * n;
  const double v = (double)iter * 8.0 + peer;
  unsigned long long bad = 0;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < n; t += (long)gridDim.x * blockDim.x)
    bad += slot[t] != v + (double)(t & 7) * 0.125;
  if (bad) __hip_atomic_fetch_add(&my_flags[10], bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int main(int argc, char **argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: ipc_probe rank dir iters bytes device\n");
    return 2;
  }
  g_rank = atoi(argv[1]);
  const std::string dir = argv[2];
  const int iters = atoi(argv[3]);
  const long bytes = atol(argv[4]);
  const int dev = atoi(argv[5]);
  const int mode = argc > 6 ? atoi(argv[6]) : 0;
  const int peer = 1 - g_rank;
  CK(hipSetDevice(dev));
  const long n = bytes / 8;
  double *data = nullptr;
  unsigned long long *flags = nullptr;
  CK(hipMalloc(&data, 2 * n * sizeof(double)));
  CK(hipMemset(data, 0, 2 * n * sizeof(double)));
  CK(hipExtMallocWithFlags((void **)&flags, 4096, hipDeviceMallocUncached));
  CK(hipMemset(flags, 0, 4096));
  CK(hipDeviceSynchronize());
  Handles h;
  CK(hipIpcGetMemHandle(&h.data, data));
  CK(hipIpcGetMemHandle(&h.flags, flags));
  {
    const std::string tmp = dir + "/h" + std::to_string(g_rank) + ".tmp";
    FILE *f = fopen(tmp.c_str(), "wb");
    fwrite(&h, sizeof h, 1, f);
    fclose(f);
    rename(tmp.c_str(), (dir + "/h" + std::to_string(g_rank)).c_str());
  }
  Handles ph;
  {
    const std::string pf = dir + "/h" + std::to_string(peer);
    FILE *f = nullptr;
    for (int t = 0; t < 3000 && !(f = fopen(pf.c_str(), "rb")); ++t)
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    if (!f) {
      fprintf(stderr, "rank %d: no peer handle\n", g_rank);
      return 4;
    }
    if (fread(&ph, sizeof ph, 1, f) != 1) return 4;
    fclose(f);
  }
  double *pdata = nullptr;
  unsigned long long *pflags = nullptr;
  const hipError_t e1 = hipIpcOpenMemHandle((void **)&pdata, ph.data, hipIpcMemLazyEnablePeerAccess);
  const hipError_t e2 = hipIpcOpenMemHandle((void **)&pflags, ph.flags, hipIpcMemLazyEnablePeerAccess);
  if (e1 != hipSuccess || e2 != hipSuccess) {
    printf("{\"rank\": %d, \"ipc_open\": \"%s / %s\"}\n", g_rank, hipGetErrorString(e1),
           hipGetErrorString(e2));
    return 5;
  }
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int blocks = (int)std::min<long>(1024, (n + 255) / 256);
  hipEvent_t ev[3];
  for (auto &e : ev) CK(hipEventCreate(&e));
  double put_ms = 0.0, wait_ms = 0.0;
  auto run = [&](int it0, int it1) {
    for (int it = it0; it <= it1; ++it) {
      CK(hipEventRecord(ev[0], st));
      if (mode == 3) {
        k_put3<<<blocks, 256, 0, st>>>(pdata, pflags, n, g_rank, (unsigned long long)it);
        CK(hipEventRecord(ev[1], st));
        k_wait_check3<<<blocks, 256, 0, st>>>(data, flags, n, peer, (unsigned long long)it);
        CK(hipEventRecord(ev[2], st));
        goto timing;
      }
      if (mode == 0) k_put<0><<<blocks, 256, 0, st>>>(pdata, pflags, flags, n, g_rank, (unsigned long long)it);
      else if (mode == 1) k_put<1><<<blocks, 256, 0, st>>>(pdata, pflags, flags, n, g_rank, (unsigned long long)it);
      else k_put<2><<<blocks, 256, 0, st>>>(pdata, pflags, flags, n, g_rank, (unsigned long long)it);
      CK(hipEventRecord(ev[1], st));
      k_wait_check<<<blocks, 256, 0, st>>>(data, flags, n, peer, (unsigned long long)it);
      CK(hipEventRecord(ev[2], st));
    timing:
      if (it % 16 == 0) {
        float a = 0, b = 0;
        CK(hipEventSynchronize(ev[2]));
        CK(hipEventElapsedTime(&a, ev[0], ev[1]));
        CK(hipEventElapsedTime(&b, ev[1], ev[2]));
        put_ms += a;
        wait_ms += b;
      }
    }
    CK(hipStreamSynchronize(st));
  };
  // baseline: the same stores into this process's own buffer, and into the
  // peer's mapped buffer without any flag
  float local_ms = 0, remote_ms = 0;
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipEventRecord(ev[0], st));
    for (int r = 0; r < 100; ++r) k_fill<<<blocks, 256, 0, st>>>(data, n, 1.0);
    CK(hipEventRecord(ev[1], st));
    for (int r = 0; r < 100; ++r) k_fill<<<blocks, 256, 0, st>>>(pdata + n * (r & 1), n, 1.0);
    CK(hipEventRecord(ev[2], st));
    CK(hipEventSynchronize(ev[2]));
    CK(hipEventElapsedTime(&local_ms, ev[0], ev[1]));
    CK(hipEventElapsedTime(&remote_ms, ev[1], ev[2]));
  }
  fprintf(stderr, "rank %d fill: local %.2f us, mapped peer %.2f us per launch\n", g_rank,
          local_ms * 10.0, remote_ms * 10.0);
  CK(hipStreamSynchronize(st));
  {  // host barrier (files) so no baseline store lands during the checked run
    fclose(fopen((dir + "/d" + std::to_string(g_rank)).c_str(), "wb"));
    const std::string pf = dir + "/d" + std::to_string(peer);
    FILE *f = nullptr;
    for (int t = 0; t < 3000 && !(f = fopen(pf.c_str(), "rb")); ++t)
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    if (!f) return 4;
    fclose(f);
  }
  run(1, 10);
  put_ms = wait_ms = 0.0;
  const auto t0 = std::chrono::steady_clock::now();
  run(11, 10 + iters);
  const auto t1 = std::chrono::steady_clock::now();
  unsigned long long hf[16];
  CK(hipMemcpy(hf, flags, sizeof hf, hipMemcpyDeviceToHost));
  const double us = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
  printf("{\"mode\": %d, \"rank\": %d, \"device\": %d, \"bytes\": %ld, \"iters\": %d, \"us_per_iter\": %.2f, "
         "\"timeouts\": %llu, \"errors\": %llu, \"flag_from_peer\": %llu, \"put_us\": %.2f, "
         "\"wait_check_us\": %.2f}\n",
         mode, g_rank, dev, bytes, iters, us, hf[9], hf[10], hf[peer], put_ms * 1e3 / (iters / 16),
         wait_ms * 1e3 / (iters / 16));
  CK(hipIpcCloseMemHandle(pdata));
  CK(hipIpcCloseMemHandle(pflags));
  return (hf[9] || hf[10]) ? 1 : 0;
}
