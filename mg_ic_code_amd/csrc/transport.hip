// transport.hip -- kernels of the peer-mapped halo transport (transport.hpp).
//
// Hand-off protocol (MI355X_MICROARCH.md, inter-workgroup visibility, taken
// to system scope because the reader can be another process or another GPU):
//   producer:  a block's payload stored write-through (sc0 sc1 buffer
//              stores) -> s_waitcnt vmcnt(0) in every wave -> workgroup
//              barrier -> one lane stores the message number into the
//              block's flag word in the consumer's page (system scope);
//   consumer:  the matching block's lane polls that flag (relaxed
//              system-scope loads, s_sleep, bounded) -> workgroup barrier ->
//              payload read with system-scope (sc0 sc1) loads, so no cached
//              copy is used.
// Each get block waits for its own put block only, so the two halves of an
// exchange overlap, and no two blocks poll or write the same word.
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
                         unsigned long long *err, unsigned long long timeout) {
  if (ld_sys(w) >= v) return true;
  const unsigned long long t0 = wall_clock64();
  for (;;) {
    __builtin_amdgcn_s_sleep(1);
    if (ld_sys(w) >= v) return true;
    if (ld_sys(err) != 0) return false;
    if (wall_clock64() - t0 > timeout) {
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

// the element range [e0, e1) of an item this block moves, in pairs when every
// row starts 2-aligned on both sides (the shells' x slabs are 2 or 4 wide)
struct Share {
  bool pairs;
  unsigned w, ny, e0, e1;
};
__device__ __forceinline__ Share share_of(const CopyItem &it, const IpcBlock &b, bool pairs) {
  Share s;
  s.pairs = pairs && (it.nx & 1) == 0;
  s.w = s.pairs ? (unsigned)it.nx / 2 : (unsigned)it.nx;
  s.ny = (unsigned)it.ny;
  const unsigned n = s.w * s.ny * (unsigned)it.nz;
  const unsigned sh = s.pairs ? 1 : 0;  // (block ranges are in elements, even for pairs)
  s.e0 = b.e0 >> sh;
  s.e1 = min(n, b.e1 >> sh);
  return s;
}
// a field region whose rows all start on a 16-B (double) / 8-B (float) pair
template <class T>
__device__ __forceinline__ bool pairable(const T *field, long off, long sy, long sz) {
  return ((off | sy | sz) & 1) == 0 &&
         (reinterpret_cast<uintptr_t>(field) & (2 * sizeof(T) - 1)) == 0;
}

// A block's share in passes of kU elements per thread, each pass issuing all
// its loads (at clamped indices, never conditional) before its stores: a load
// cannot move above an earlier store the compiler cannot prove disjoint, so a
// plain load/store loop would run one memory round trip per element.
constexpr int kU = 4;

// element offset of message element / pair t in a field region (rows of w)
struct Rows {
  unsigned w, ny;
  long sy, sz;
  __device__ __forceinline__ long at(unsigned t, unsigned scale) const {
    const unsigned q = t / w, i = t - q * w;
    const unsigned k = q / ny, j = q - k * ny;
    return (long)j * sy + (long)k * sz + (long)scale * i;
  }
};

// move a block's element range: load(t) for every t of a pass, then
// store(t, v) for the in-range ones
template <class V, class Load, class Store>
__device__ __forceinline__ void move_share(unsigned e0, unsigned e1, Load load, Store store) {
  for (unsigned base = e0 + threadIdx.x; base < e1; base += 256u * kU) {
    V v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) v[u] = load(min(base + 256u * u, e1 - 1));
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (base + 256u * u < e1) store(base + 256u * u, v[u]);
  }
}

// put: a block's share of one item, field -> peer's message slot (rows packed:
// pair t is message elements 2t, 2t+1)
template <class T>
__device__ __forceinline__ void put_share(const CopyItem &it, const IpcBlock &b,
                                          T *const *src_tab, const IpcPeers &pp, int p) {
  using V = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
  const T *src = src_tab[it.src] + it.soff;
  const Share s = share_of(it, b, pairable(src_tab[it.src], it.soff, it.ssy, it.ssz) &&
                                        (it.doff & 1) == 0);
  const Rows rw{s.w, s.ny, it.ssy, it.ssz};
  const __amdgpu_buffer_rsrc_t r = rsrc(pp.buf[p]);
  const long mo = it.doff;
  if (s.pairs)
    move_share<V>(s.e0, s.e1,
                  [&](unsigned t) { return *reinterpret_cast<const V *>(src + rw.at(t, 2)); },
                  [&](unsigned t, V v) { st_sys(r, (unsigned)((mo + 2 * (long)t) * sizeof(T)), v); });
  else
    move_share<T>(s.e0, s.e1, [&](unsigned t) { return src[rw.at(t, 1)]; },
                  [&](unsigned t, T v) { st_sys(r, (unsigned)((mo + (long)t) * sizeof(T)), v); });
}

// get: a block's share of one item, my message slot -> field ghosts
template <class T>
__device__ __forceinline__ void get_share(const CopyItem &it, const IpcBlock &b,
                                          T *const *dst_tab, const IpcPeers &pp, int p) {
  using V = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
  T *dst = dst_tab[it.dst] + it.doff;
  const Share s = share_of(it, b, pairable(dst_tab[it.dst], it.doff, it.dsy, it.dsz) &&
                                        (it.soff & 1) == 0);
  const Rows rw{s.w, s.ny, it.dsy, it.dsz};
  const __amdgpu_buffer_rsrc_t r = rsrc(pp.buf[p]);
  const long mo = it.soff;
  if (s.pairs)
    move_share<V>(s.e0, s.e1,
                  [&](unsigned t) { return ld_sys<V>(r, (unsigned)((mo + 2 * (long)t) * sizeof(T))); },
                  [&](unsigned t, V v) { *reinterpret_cast<V *>(dst + rw.at(t, 2)) = v; });
  else
    move_share<T>(s.e0, s.e1,
                  [&](unsigned t) { return ld_sys<T>(r, (unsigned)((mo + (long)t) * sizeof(T))); },
                  [&](unsigned t, T v) { dst[rw.at(t, 1)] = v; });
}

// A workgroup's wait for peer p's slot to be free, at most once per launch:
// the condition holds for the rest of the launch once met, so `passed`
// (uniform, bit p) remembers it.  A timed-out wait skips the copy; the block
// is still flagged, so no peer waits on this one in turn.
__device__ __forceinline__ bool wait_slot(const IpcPeers &pp, int p, unsigned &passed, int &ok) {
  if (passed >> p & 1u) return true;
  if (threadIdx.x == 0) ok = ipc_wait(pp.ack[p], pp.val[p], pp.err, pp.timeout);
  __syncthreads();
  const bool go = ok != 0;
  __syncthreads();  // (ok is rewritten by the next wait)
  if (go) passed |= 1u << p;
  return go;
}

// A get block's wait for its own flag: the sender's put block for the same
// message range has landed (one word per block, so no two blocks poll or
// write the same word)
__device__ __forceinline__ bool wait_block(const IpcPeers &pp, int p, int flag, int &ok) {
  if (threadIdx.x == 0) ok = ipc_wait(pp.flags[p] + flag, pp.seq[p], pp.err, pp.timeout);
  __syncthreads();
  const bool go = ok != 0;
  __syncthreads();
  return go;
}

// a put block's payload is drained from every wave, then one lane raises the
// block's flag in the receiver's page
__device__ __forceinline__ void flag_block(const IpcPeers &pp, int p, int flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) st_word(pp.flags[p] + flag, pp.seq[p]);
}

// after every wave's loads are drained, one lane adds the workgroup's
// consumed blocks per sender to the senders' acknowledgement counters (one
// atomic per sender and workgroup)
__device__ __forceinline__ void ack_blocks(unsigned *done, const IpcPeers &pp) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    for (int q = 0; q < pp.n; ++q)
      if (done[q])
        __hip_atomic_fetch_add(pp.ack[q], (unsigned long long)done[q], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
}

// local: a block's share of a same-rank copy, field -> field
template <class T>
__device__ __forceinline__ void local_share(const CopyItem &it, const IpcBlock &b,
                                            T *const *src_tab, T *const *dst_tab) {
  using V = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
  const T *src = src_tab[it.src] + it.soff;
  T *dst = dst_tab[it.dst] + it.doff;
  const Share s = share_of(it, b, pairable(src_tab[it.src], it.soff, it.ssy, it.ssz) &&
                                        pairable(dst_tab[it.dst], it.doff, it.dsy, it.dsz));
  const Rows rs{s.w, s.ny, it.ssy, it.ssz}, rd{s.w, s.ny, it.dsy, it.dsz};
  if (s.pairs)
    move_share<V>(s.e0, s.e1,
                  [&](unsigned t) { return *reinterpret_cast<const V *>(src + rs.at(t, 2)); },
                  [&](unsigned t, V v) { *reinterpret_cast<V *>(dst + rd.at(t, 2)) = v; });
  else
    move_share<T>(s.e0, s.e1, [&](unsigned t) { return src[rs.at(t, 1)]; },
                  [&](unsigned t, T v) { dst[rd.at(t, 1)] = v; });
}

// one exchange in one launch: virtual blocks [0, npu) put my messages (first,
// so the peers can start), [npu, npu + nlo) copy the same-rank regions, the
// rest get my messages.  The workgroups stride over the virtual blocks in
// ascending order, so a workgroup has done all its puts before its first
// get, and the grid is capped (Comm::ipc_grid_cap) so that every rank's
// exchange workgroups on a device fit on it at once: no get -- of a peer's
// message or of this launch's own self messages -- can hold the CU slot of
// a put that has not started, whatever order workgroups are dispatched in.
template <class T>
__global__ __launch_bounds__(256) void k_exchange(const CopyItem *__restrict__ put_items,
                                                  const CopyItem *__restrict__ loc_items,
                                                  const CopyItem *__restrict__ get_items,
                                                  const IpcBlock *__restrict__ blocks, int npu,
                                                  int nlo, int nall,
                                                  T *const *__restrict__ src_tab,
                                                  T *const *__restrict__ dst_tab,
                                                  const IpcPeers pput, const IpcPeers pget) {
  __shared__ int ok;
  __shared__ unsigned done_get[kMaxIpcPeers];  // blocks consumed per sender (lane 0 only)
  if (threadIdx.x == 0)
    for (int q = 0; q < kMaxIpcPeers; ++q) done_get[q] = 0;
  unsigned passed = 0;  // peers whose slot this workgroup has seen free (uniform)
  for (int v = blockIdx.x; v < nall; v += gridDim.x) {  // (uniform per workgroup)
    const IpcBlock b = blocks[v];
    if (v < npu) {
      const CopyItem &it = put_items[b.item];
      const int p = __builtin_amdgcn_readfirstlane(it.pad);
      if (wait_slot(pput, p, passed, ok)) put_share<T>(it, b, src_tab, pput, p);
      flag_block(pput, p, b.flag);
    } else if (v < npu + nlo) {
      local_share<T>(loc_items[b.item], b, src_tab, dst_tab);
    } else {
      const CopyItem &it = get_items[b.item];
      const int p = __builtin_amdgcn_readfirstlane(it.pad);
      if (wait_block(pget, p, b.flag, ok)) get_share<T>(it, b, dst_tab, pget, p);
      if (threadIdx.x == 0) ++done_get[p];
    }
  }
  ack_blocks(done_get, pget);
}

__global__ void k_ipc_allreduce(double *val, int op, const IpcReduce r, unsigned long long *err,
                                const HostPub pub) {
  if (threadIdx.x != 0) return;
  const unsigned long long bits = __double_as_longlong(*val);
  const int slot = kSigRedVal + r.parity * 1024 + r.rank * kSigStride;
  for (int q = 0; q < r.size; ++q) st_word(r.sig[q] + slot, bits);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int q = 0; q < r.size; ++q) st_word(r.sig[q] + kSigRedCnt + r.rank * kSigStride, r.count);
  unsigned long long *mine = r.sig[r.rank];
  bool ok = true;
  for (int q = 0; q < r.size && ok; ++q)
    ok = ipc_wait(mine + kSigRedCnt + q * kSigStride, r.count, err, r.timeout);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  if (!ok) {  // the error word (set) goes to the host with the sequence number
    publish(pub, __longlong_as_double(0x7ff8000000000000ll));
    return;
  }
  double acc = __longlong_as_double(ld_sys(mine + kSigRedVal + r.parity * 1024));
  for (int q = 1; q < r.size; ++q) {
    const double v =
        __longlong_as_double(ld_sys(mine + kSigRedVal + r.parity * 1024 + q * kSigStride));
    acc = op == 1 ? (acc > v ? acc : v) : acc + v;
  }
  *val = acc;
  publish(pub, acc);
}

inline void check_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(kHipErr, std::string("kernel launch: ") + hipGetErrorString(e));
}

}  // namespace

template <class T>
static void exchange_t(const CopyItem *put_items, const CopyItem *loc_items,
                       const CopyItem *get_items, const IpcBlock *blocks, int npu, int nlo, int nge,
                       T *const *src_tab, T *const *dst_tab, const IpcPeers &pput,
                       const IpcPeers &pget, int grid_cap, hipStream_t st) {
  const int n = npu + nlo + nge;
  if (n <= 0) return;
  const int g = grid_cap > 0 && grid_cap < n ? grid_cap : n;  // (the Comm always caps)
  k_exchange<T><<<dim3((unsigned)g), dim3(256), 0, st>>>(put_items, loc_items, get_items, blocks,
                                                         npu, nlo, n, src_tab,
                                                         dst_tab, pput, pget);
  check_launch();
}

void ipc_exchange(const CopyItem *put_items, const CopyItem *loc_items, const CopyItem *get_items,
                  const IpcBlock *blocks, int npu, int nlo, int nge,
                  double *const *src_tab, double *const *dst_tab, const IpcPeers &pput,
                  const IpcPeers &pget, int grid_cap, hipStream_t st) {
  exchange_t<double>(put_items, loc_items, get_items, blocks, npu, nlo, nge, src_tab, dst_tab,
                     pput, pget, grid_cap, st);
}
void ipc_exchange_f(const CopyItem *put_items, const CopyItem *loc_items,
                    const CopyItem *get_items, const IpcBlock *blocks, int npu, int nlo, int nge,
                    float *const *src_tab, float *const *dst_tab, const IpcPeers &pput,
                    const IpcPeers &pget, int grid_cap, hipStream_t st) {
  exchange_t<float>(put_items, loc_items, get_items, blocks, npu, nlo, nge, src_tab, dst_tab,
                    pput, pget, grid_cap, st);
}

void ipc_allreduce(double *val, int op, const IpcReduce &r, unsigned long long *err,
                   const HostPub &pub, hipStream_t st) {
  k_ipc_allreduce<<<1, 64, 0, st>>>(val, op, r, err, pub);
  check_launch();
}

}  // namespace kern
}  // namespace mgic
