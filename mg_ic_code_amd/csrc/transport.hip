// transport.hip -- kernels of the peer-mapped halo transport (transport.hpp).
//
// Hand-off protocol (MI355X_MICROARCH.md, inter-workgroup visibility, taken
// to system scope because the reader can be another process or another GPU):
//   producer block: payload stored write-through (sc0 sc1 buffer stores) ->
//                   s_waitcnt vmcnt(0) in every wave -> workgroup barrier ->
//                   one lane adds 1 to the consumer's counter (system scope);
//   consumer block: one lane polls the counter (relaxed system-scope loads,
//                   s_sleep, bounded) until it covers every block of the
//                   message -> workgroup barrier -> payload read with
//                   system-scope (sc0 sc1) loads, so no cached copy is used.
// tools/ipc_probe.hip measured the forms on one MI355X with two processes:
// plain stores behind a single release lose words across XCDs; a release per
// block is correct but 3x slower at 2-8 MB; write-through stores are correct
// and the fastest.
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
__device__ __forceinline__ void st_word(unsigned long long *p, unsigned long long v) {
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

// 16-B / 8-B / 4-B write-through (sc0 sc1) buffer stores and system-scope
// loads: cache policy 1 (sc0) | 16 (sc1)
constexpr int kSys = 17;
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void *base) {
  return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st_sys(__amdgpu_buffer_rsrc_t r, unsigned off, double2 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, off, 0, kSys);
}
__device__ __forceinline__ void st_sys(__amdgpu_buffer_rsrc_t r, unsigned off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, off, 0, kSys);
}
__device__ __forceinline__ void st_sys(__amdgpu_buffer_rsrc_t r, unsigned off, float2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, off, 0, kSys);
}
__device__ __forceinline__ void st_sys(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, kSys);
}
template <class V> __device__ __forceinline__ V ld_sys(__amdgpu_buffer_rsrc_t r, unsigned off);
template <> __device__ __forceinline__ double2 ld_sys<double2>(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSys));
}
template <> __device__ __forceinline__ double ld_sys<double>(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kSys));
}
template <> __device__ __forceinline__ float2 ld_sys<float2>(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kSys));
}
template <> __device__ __forceinline__ float ld_sys<float>(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kSys));
}

// after every wave's memory operations are drained, one lane counts the block
__device__ __forceinline__ void ipc_done(unsigned long long *count) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(count, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the element range [e0, e1) of an item this block moves, in pairs when every
// row starts 2-aligned on both sides (the shells' x slabs are 2 or 4 wide)
struct Share {
  bool pairs;
  unsigned w, ny, e0, e1;
};
template <class T>
__device__ __forceinline__ Share share(const CopyItem &it, int sub, const T *field, long foff,
                                       long fsy, long fsz, long moff) {
  Share s;
  s.pairs = ((it.nx | foff | fsy | fsz | moff) & 1) == 0 &&
            (reinterpret_cast<uintptr_t>(field) & (2 * sizeof(T) - 1)) == 0;
  s.w = s.pairs ? (unsigned)it.nx / 2 : (unsigned)it.nx;
  s.ny = (unsigned)it.ny;
  const unsigned n = s.w * s.ny * (unsigned)it.nz;
  const unsigned per = s.pairs ? (unsigned)kIpcBlockElems / 2 : (unsigned)kIpcBlockElems;
  s.e0 = (unsigned)sub * per;
  s.e1 = min(n, s.e0 + per);
  return s;
}

template <class T>
__global__ __launch_bounds__(256) void k_ipc_put(const CopyItem *__restrict__ items,
                                                 const IpcBlock *__restrict__ blocks,
                                                 T *const *__restrict__ src_tab, const IpcPeers pp) {
  using V = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
  const IpcBlock b = blocks[blockIdx.x];
  const CopyItem it = items[b.item];
  const int p = it.pad;
  __shared__ int ok;
  if (threadIdx.x == 0) ok = ipc_wait(pp.wait[p], pp.wait_val[p], pp.err);  // slot free
  __syncthreads();
  if (ok) {
    const T *src = src_tab[it.src] + it.soff;
    const Share s = share(it, b.sub, src_tab[it.src], it.soff, it.ssy, it.ssz, it.doff);
    const __amdgpu_buffer_rsrc_t r = rsrc(pp.buf[p]);
    for (unsigned t = s.e0 + threadIdx.x; t < s.e1; t += blockDim.x) {
      const unsigned q = t / s.w, i = t - q * s.w;
      const unsigned k = q / s.ny, j = q - k * s.ny;
      const long so = (long)j * it.ssy + (long)k * it.ssz;
      if (s.pairs)  // message rows are packed: pair t is elements 2t, 2t+1
        st_sys(r, (unsigned)((it.doff + 2 * (long)t) * sizeof(T)),
               reinterpret_cast<const V *>(src + so)[i]);
      else
        st_sys(r, (unsigned)((it.doff + (long)t) * sizeof(T)), src[so + i]);
    }
  }
  ipc_done(pp.count[p]);
}

template <class T>
__global__ __launch_bounds__(256) void k_ipc_get(const CopyItem *__restrict__ items,
                                                 const IpcBlock *__restrict__ blocks,
                                                 T *const *__restrict__ dst_tab, const IpcPeers pp) {
  using V = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
  const IpcBlock b = blocks[blockIdx.x];
  const CopyItem it = items[b.item];
  const int p = it.pad;
  __shared__ int ok;
  if (threadIdx.x == 0) ok = ipc_wait(pp.wait[p], pp.wait_val[p], pp.err);  // message complete
  __syncthreads();
  if (ok) {
    T *dst = dst_tab[it.dst] + it.doff;
    const Share s = share(it, b.sub, dst_tab[it.dst], it.doff, it.dsy, it.dsz, it.soff);
    const __amdgpu_buffer_rsrc_t r = rsrc(pp.buf[p]);
    for (unsigned t = s.e0 + threadIdx.x; t < s.e1; t += blockDim.x) {
      const unsigned q = t / s.w, i = t - q * s.w;
      const unsigned k = q / s.ny, j = q - k * s.ny;
      const long d = (long)j * it.dsy + (long)k * it.dsz;
      if (s.pairs)
        reinterpret_cast<V *>(dst + d)[i] =
            ld_sys<V>(r, (unsigned)((it.soff + 2 * (long)t) * sizeof(T)));
      else
        dst[d + i] = ld_sys<T>(r, (unsigned)((it.soff + (long)t) * sizeof(T)));
    }
  }
  ipc_done(pp.count[p]);  // acknowledge to the sender
}

__global__ void k_ipc_allreduce(double *val, int op, const IpcReduce r, unsigned long long *err) {
  if (threadIdx.x != 0) return;
  const unsigned long long bits = __double_as_longlong(*val);
  const int slot = kSigRedVal + r.parity * 1024 + r.rank * kSigStride;
  for (int q = 0; q < r.size; ++q) st_word(r.sig[q] + slot, bits);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int q = 0; q < r.size; ++q) st_word(r.sig[q] + kSigRedCnt + r.rank * kSigStride, r.count);
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

template <class T>
static void put_t(const CopyItem *items, const IpcBlock *blocks, int nblocks, T *const *src_tab,
                  const IpcPeers &pp, hipStream_t st) {
  if (nblocks <= 0) return;
  k_ipc_put<T><<<dim3((unsigned)nblocks), dim3(256), 0, st>>>(items, blocks, src_tab, pp);
  check_launch();
}
template <class T>
static void get_t(const CopyItem *items, const IpcBlock *blocks, int nblocks, T *const *dst_tab,
                  const IpcPeers &pp, hipStream_t st) {
  if (nblocks <= 0) return;
  k_ipc_get<T><<<dim3((unsigned)nblocks), dim3(256), 0, st>>>(items, blocks, dst_tab, pp);
  check_launch();
}

void ipc_put(const CopyItem *items, const IpcBlock *blocks, int nblocks, double *const *src_tab,
             const IpcPeers &pp, hipStream_t st) {
  put_t<double>(items, blocks, nblocks, src_tab, pp, st);
}
void ipc_put_f(const CopyItem *items, const IpcBlock *blocks, int nblocks, float *const *src_tab,
               const IpcPeers &pp, hipStream_t st) {
  put_t<float>(items, blocks, nblocks, src_tab, pp, st);
}
void ipc_get(const CopyItem *items, const IpcBlock *blocks, int nblocks, double *const *dst_tab,
             const IpcPeers &pp, hipStream_t st) {
  get_t<double>(items, blocks, nblocks, dst_tab, pp, st);
}
void ipc_get_f(const CopyItem *items, const IpcBlock *blocks, int nblocks, float *const *dst_tab,
               const IpcPeers &pp, hipStream_t st) {
  get_t<float>(items, blocks, nblocks, dst_tab, pp, st);
}

void ipc_allreduce(double *val, int op, const IpcReduce &r, unsigned long long *err,
                   hipStream_t st) {
  k_ipc_allreduce<<<1, 64, 0, st>>>(val, op, r, err);
  check_launch();
}

}  // namespace kern
}  // namespace mgic
