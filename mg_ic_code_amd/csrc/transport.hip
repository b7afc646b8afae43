// transport.hip -- kernels of the peer-mapped halo transport (transport.hpp).
//
// Hand-off protocol (MI355X_MICROARCH.md, inter-workgroup visibility, at
// system scope because the reader can be another process or another GPU):
//   producer: payload stored with system-scope (write-through) stores ->
//             every wave drains them (s_waitcnt vmcnt(0)) -> workgroup barrier
//             -> one lane takes a ticket -> the grid's last block releases at
//             system scope, drains, and raises each peer's counter;
//   consumer: one lane polls the counter (relaxed system-scope loads, s_sleep,
//             bounded) -> system-scope acquire -> vmcnt(0) -> barrier -> loads.
// tools/ipc_probe.hip measured the variants on one MI355X with two processes:
// plain stores with a single release lose words across XCDs; per-block
// releases are correct but 3x slower at 2-8 MB; write-through stores with one
// release are correct (0 errors in 6000 checked hand-offs) and the fastest.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "kernels.hpp"
#include "transport.hpp"

namespace mgic {
namespace kern {

namespace {

__device__ __forceinline__ unsigned long long ld_sys(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(unsigned long long *p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// bounded poll of *w >= v; false on timeout (recorded in *err) or when an
// earlier timeout of this rank is already recorded (fail fast, never hang)
__device__ bool ipc_wait(const unsigned long long *w, unsigned long long v,
                         unsigned long long *err) {
  if (ld_sys(w) >= v) return true;
  const unsigned long long t0 = wall_clock64();
  for (;;) {
    __builtin_amdgcn_s_sleep(1);
    if (ld_sys(w) >= v) return true;
    if (ld_sys(err) != 0) return false;
    if (wall_clock64() - t0 > kIpcTimeoutTicks) {
      __hip_atomic_fetch_add(err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
  }
}

// after every wave's stores are drained: the grid's last block raises the flags
__device__ __forceinline__ void ipc_finish(const IpcPeers &pp) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t =
        __hip_atomic_fetch_add(pp.ticket, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t + 1 == pp.ticket_end) {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int q = 0; q < pp.n; ++q) st_sys(pp.flag[q], pp.flag_val[q]);
    }
  }
}

template <class T>
__device__ __forceinline__ void st_wt(T *p, T v) {  // write-through (system scope)
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <class T>
__global__ __launch_bounds__(256) void k_ipc_put(const CopyItem *__restrict__ items,
                                                 T *const *__restrict__ src_tab, const IpcPeers pp) {
  const CopyItem it = items[blockIdx.y];
  const int p = it.pad;
  __shared__ int ok;
  if (threadIdx.x == 0) ok = ipc_wait(pp.wait[p], pp.wait_val[p], pp.err);  // slot free
  __syncthreads();
  if (ok) {
    const T *src = src_tab[it.src] + it.soff;
    T *dst = static_cast<T *>(pp.buf[p]) + it.doff;  // rows packed: dsy = nx, dsz = nx * ny
    const unsigned w = (unsigned)it.nx, ny = (unsigned)it.ny;
    const unsigned n = w * ny * (unsigned)it.nz;
    for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
      const unsigned r = t / w, i = t - r * w;
      const unsigned k = r / ny, j = r - k * ny;
      st_wt(dst + t, src[(long)j * it.ssy + (long)k * it.ssz + i]);
    }
  }
  ipc_finish(pp);
}

template <class T>
__global__ __launch_bounds__(256) void k_ipc_get(const CopyItem *__restrict__ items,
                                                 T *const *__restrict__ dst_tab, const IpcPeers pp) {
  const CopyItem it = items[blockIdx.y];
  const int p = it.pad;
  __shared__ int ok;
  if (threadIdx.x == 0) {
    ok = ipc_wait(pp.wait[p], pp.wait_val[p], pp.err);  // message delivered
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (ok) {
    const T *src = static_cast<const T *>(pp.buf[p]) + it.soff;
    T *dst = dst_tab[it.dst] + it.doff;
    const unsigned w = (unsigned)it.nx, ny = (unsigned)it.ny;
    const unsigned n = w * ny * (unsigned)it.nz;
    for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
      const unsigned r = t / w, i = t - r * w;
      const unsigned k = r / ny, j = r - k * ny;
      dst[(long)j * it.dsy + (long)k * it.dsz + i] = src[t];
    }
  }
  ipc_finish(pp);  // acknowledge the slot to each sender
}

__global__ void k_ipc_allreduce(double *val, int op, const IpcReduce r, unsigned long long *err) {
  if (threadIdx.x != 0) return;
  const unsigned long long bits = __double_as_longlong(*val);
  const int slot = kSigRedVal + r.parity * 1024 + r.rank * kSigStride;
  for (int q = 0; q < r.size; ++q) st_sys(r.sig[q] + slot, bits);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int q = 0; q < r.size; ++q) st_sys(r.sig[q] + kSigRedCnt + r.rank * kSigStride, r.count);
  unsigned long long *mine = r.sig[r.rank];
  bool ok = true;
  for (int q = 0; q < r.size && ok; ++q) ok = ipc_wait(mine + kSigRedCnt + q * kSigStride, r.count, err);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  if (!ok) return;
  double acc = __longlong_as_double(ld_sys(mine + kSigRedVal + r.parity * 1024));
  for (int q = 1; q < r.size; ++q) {
    const double v =
        __longlong_as_double(ld_sys(mine + kSigRedVal + r.parity * 1024 + q * kSigStride));
    acc = op == 1 ? (acc > v ? acc : v) : acc + v;
  }
  *val = acc;
}

inline void check_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(kHipErr, std::string("kernel launch: ") + hipGetErrorString(e));
}

}  // namespace

int ipc_grid_x(long max_cells) {
  // at most 64 blocks of 256 threads per item (4+ elements per thread on the
  // large faces): the spinning get blocks of one rank must leave room on a
  // shared device for the put blocks of another
  long bx = (max_cells + 1023) / 1024;
  if (bx < 1) bx = 1;
  if (bx > 64) bx = 64;
  return (int)bx;
}

template <class T>
static void put_t(const CopyItem *items, int nitems, long max_cells, T *const *src_tab,
                  const IpcPeers &pp, hipStream_t st) {
  if (nitems <= 0) return;
  k_ipc_put<T><<<dim3((unsigned)ipc_grid_x(max_cells), (unsigned)nitems), dim3(256), 0, st>>>(
      items, src_tab, pp);
  check_launch();
}
template <class T>
static void get_t(const CopyItem *items, int nitems, long max_cells, T *const *dst_tab,
                  const IpcPeers &pp, hipStream_t st) {
  if (nitems <= 0) return;
  k_ipc_get<T><<<dim3((unsigned)ipc_grid_x(max_cells), (unsigned)nitems), dim3(256), 0, st>>>(
      items, dst_tab, pp);
  check_launch();
}

void ipc_put(const CopyItem *items, int nitems, long max_cells, double *const *src_tab,
             const IpcPeers &pp, hipStream_t st) {
  put_t<double>(items, nitems, max_cells, src_tab, pp, st);
}
void ipc_put_f(const CopyItem *items, int nitems, long max_cells, float *const *src_tab,
               const IpcPeers &pp, hipStream_t st) {
  put_t<float>(items, nitems, max_cells, src_tab, pp, st);
}
void ipc_get(const CopyItem *items, int nitems, long max_cells, double *const *dst_tab,
             const IpcPeers &pp, hipStream_t st) {
  get_t<double>(items, nitems, max_cells, dst_tab, pp, st);
}
void ipc_get_f(const CopyItem *items, int nitems, long max_cells, float *const *dst_tab,
               const IpcPeers &pp, hipStream_t st) {
  get_t<float>(items, nitems, max_cells, dst_tab, pp, st);
}

void ipc_allreduce(double *val, int op, const IpcReduce &r, unsigned long long *err,
                   hipStream_t st) {
  k_ipc_allreduce<<<1, 64, 0, st>>>(val, op, r, err);
  check_launch();
}

}  // namespace kern
}  // namespace mgic
