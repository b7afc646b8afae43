// transport.hpp -- the cross-process halo transport (peer-mapped buffers and
// device-side counters), the second transport beside RCCL send/recv.
//
// Every rank maps, through hipIpcOpenMemHandle, every other rank's
//   * signal page: 64 KB of uncached device memory holding per-peer block
//     counters, acknowledgements, an error word and the allreduce slots;
//   * receive arena: size x 2 message buffers (double-buffered per sender).
// An exchange (CopyPlan) is then two launches and no host round trip:
//   put  -- each block copies its share of my boundary regions, with
//           write-through (system-scope) 16-B stores, straight into the
//           peer's arena slot; a workgroup drains its stores and adds its
//           blocks to the peer's counter for me before its first get;
//   get  -- each block waits until the sender's counter covers the whole
//           message, reads it with system-scope loads into my ghost cells;
//           the workgroup adds its blocks to the sender's acknowledgement
//           counter when it ends.
// Both sides split an item into blocks the same way (ipc_blocks), so the
// counters count blocks; they are cumulative per (sender, receiver) pair, so
// nothing is ever reset, and no ticket or last-block step is needed.  Every
// poll is bounded in time (MGIC_IPC_TIMEOUT_S, default 10 s) and records a
// timeout in the error word
// (Comm::ipc_check raises it on the host) instead of hanging the GPU.  The
// same kernels serve a single process with self messages (tests).
#pragma once

#include <hip/hip_runtime.h>

#include "mgic_core.hpp"

namespace mgic {
namespace kern {

constexpr int kMaxIpcPeers = 32;  // peers of one plan (26 neighbours in 3D + slack)
constexpr int kMaxIpcRanks = 64;  // ranks of one job (one node: 8 GPUs)

// signal page layout, in 64-bit words; every counter on its own 128-B line
constexpr int kSigStride = 16;
constexpr int kSigArr = 0;           // arr[r]: message blocks rank r has delivered to me
constexpr int kSigAck = 1024;        // ack[r]: blocks of my messages rank r has consumed
constexpr int kSigErr = 2064;        // timeouts observed by this rank
constexpr int kSigRedCnt = 3072;     // red_cnt[r]: allreduce contributions of rank r
constexpr int kSigRedVal = 4096;     // val[parity][r] at kSigRedVal + parity * 1024 + r * 16
constexpr int kSigWords = 8192;      // 64 KB

struct IpcPeers {
  int n;                                         // peers of this launch
  unsigned long long *err;                       // my error word
  unsigned long long timeout;                    // bound of every wait (100 MHz ticks)
  unsigned long long *count[kMaxIpcPeers];       // +1 per block when done (a peer's page)
  const unsigned long long *wait[kMaxIpcPeers];  // polled before a block copies (my page)
  unsigned long long wait_val[kMaxIpcPeers];
  void *buf[kMaxIpcPeers];                       // message slot: put -> peer arena, get -> mine
};

// one block of a put / get launch: its item and its share of the item
struct IpcBlock {
  int item, sub;
};
// elements per block: a job-wide constant (Comm::ipc_block_elems, checked
// equal on every rank at setup), so both sides of a message split alike
constexpr long kIpcBlockElemsDefault = 4096;
inline long ipc_blocks(long cells, long per) { return (cells + per - 1) / per; }

struct IpcReduce {
  int size, rank, parity;
  unsigned long long count;                    // this allreduce's number (1-based)
  unsigned long long timeout;                  // bound of every wait (100 MHz ticks)
  unsigned long long *sig[kMaxIpcRanks];       // every rank's signal page (mine at [rank])
};

// One exchange in one launch over the block table `blocks`: npu put blocks
// (items: src = local box, doff = offset in the peer's message, pad = peer
// index in pput), then nlo same-rank copy blocks (loc_items), then nge get
// blocks (items: dst = local box, soff = offset in the sender's message, pad =
// peer index in pget).  Every item is split into ipc_blocks(cells, per) blocks.
// At most grid_cap workgroups, striding over the blocks in ascending order
// (every workgroup's puts before its gets; see k_exchange and Comm).
void ipc_exchange(const CopyItem *put_items, const CopyItem *loc_items, const CopyItem *get_items,
                  const IpcBlock *blocks, int npu, int nlo, int nge, int per,
                  double *const *src_tab, double *const *dst_tab, const IpcPeers &pput,
                  const IpcPeers &pget, int grid_cap, hipStream_t st);
void ipc_exchange_f(const CopyItem *put_items, const CopyItem *loc_items,
                    const CopyItem *get_items, const IpcBlock *blocks, int npu, int nlo, int nge,
                    int per, float *const *src_tab, float *const *dst_tab, const IpcPeers &pput,
                    const IpcPeers &pget, int grid_cap, hipStream_t st);
// in-place allreduce of one device double over all ranks (op 0 sum, 1 max),
// reduced in rank order on every rank (identical results everywhere)
void ipc_allreduce(double *val, int op, const IpcReduce &r, unsigned long long *err,
                   hipStream_t st);

}  // namespace kern
}  // namespace mgic
