// transport.hpp -- the cross-process halo transport (peer-mapped buffers and
// device-side counters), the second transport beside RCCL send/recv.
//
// Every rank maps, through hipIpcOpenMemHandle, every other rank's
//   * signal page: uncached device memory holding per-peer acknowledgement
//     counters, an error word, the allreduce slots and, per (sender, slot
//     parity), one flag word per message block;
//   * receive arena: size x 2 message buffers (double-buffered per sender).
// An exchange (CopyPlan) is then one launch and no host round trip:
//   put  -- each block copies its share of my boundary regions, with
//           write-through (system-scope) 16-B stores, straight into the
//           peer's arena slot, drains them and stores the message number
//           into its flag in the peer's page;
//   get  -- each block waits for its own flag, reads its share with
//           system-scope loads into my ghost cells; the workgroup adds its
//           blocks to the sender's acknowledgement counter when it ends.
// Both sides split an item into blocks the same way (ipc_blocks) and number
// a message's blocks by their offset in the message, so block i's flag is the
// same word on both sides.  Flags hold message numbers and acknowledgements
// are cumulative per (sender, receiver) pair, so nothing is ever reset.  Every
// poll is bounded in time (MGIC_IPC_TIMEOUT_S, default 10 s) and records a
// timeout in the error word
// (Comm::ipc_check raises it on the host) instead of hanging the GPU.  The
// same kernels serve a single process with self messages (tests).
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "mgic_core.hpp"

namespace mgic {
namespace kern {

constexpr int kMaxIpcPeers = 32;  // peers of one plan (26 neighbours in 3D + slack)
constexpr int kMaxIpcRanks = 64;  // ranks of one job (one node: 8 GPUs)

// signal page layout, in 64-bit words; every counter on its own 128-B line
constexpr int kSigStride = 16;
constexpr int kSigAck = 1024;        // ack[r]: blocks of my messages rank r has consumed
constexpr int kSigErr = 2064;        // timeouts observed by this rank
constexpr int kSigRedCnt = 3072;     // red_cnt[r]: allreduce contributions of rank r
constexpr int kSigRedVal = 4096;     // val[parity][r] at kSigRedVal + parity * 1024 + r * 16
constexpr int kSigFlags = 8192;      // flags of sender r's slot q at kSigFlags + (2r + q) * kMaxMsgBlocks
constexpr int kMaxMsgBlocks = 16384; // blocks of one message
inline size_t sig_words(int size) { return (size_t)kSigFlags + (size_t)size * 2 * kMaxMsgBlocks; }

struct IpcPeers {
  int n;                                     // peers of this launch
  unsigned long long *err;                   // my error word
  unsigned long long timeout;                // bound of every wait (100 MHz ticks)
  unsigned long long *flags[kMaxIpcPeers];   // this message's block flags (the receiver's page)
  unsigned long long seq[kMaxIpcPeers];      // a landed block's flag value: message number + 1
  // put: my acknowledgement counter from the peer, polled until it reaches
  // val (the slot's previous message consumed); get: the sender's counter
  // for me, +1 per block consumed
  unsigned long long *ack[kMaxIpcPeers];
  unsigned long long val[kMaxIpcPeers];
  void *buf[kMaxIpcPeers];                   // message slot: put -> peer arena, get -> mine
};

// one block of an exchange launch: its item, its flag (its number within the
// message, by message offset; puts and gets) and its element range [e0, e1)
// of the item
struct IpcBlock {
  int item, flag;
  unsigned e0, e1;
};
// Elements per block of an item of `cells` elements: a power of two in
// [512, maxper] giving 16 to 32 blocks where it can, so that small messages spread
// over many workgroups; maxper is a job-wide constant (Comm::ipc_block_elems,
// checked equal on every rank at setup), so both sides of a message split alike
constexpr long kIpcBlockElemsDefault = 2048;
inline long ipc_item_per(long cells, long maxper) {
  long per = 512;
  // (doubling, clamped: a maxper that is not 512 * 2^k is still the cap)
  while (per < maxper && per * 32 <= cells) per = per * 2 < maxper ? per * 2 : maxper;
  return per;
}
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
// peer index in pget).  Every item is split into blocks of ipc_item_per elements.
// At most grid_cap workgroups, striding over the blocks in ascending order
// (every workgroup's puts before its gets; see k_exchange and Comm).
void ipc_exchange(const CopyItem *put_items, const CopyItem *loc_items, const CopyItem *get_items,
                  const IpcBlock *blocks, int npu, int nlo, int nge, double *const *src_tab,
                  double *const *dst_tab, const IpcPeers &pput,
                  const IpcPeers &pget, int grid_cap, hipStream_t st);
void ipc_exchange_f(const CopyItem *put_items, const CopyItem *loc_items,
                    const CopyItem *get_items, const IpcBlock *blocks, int npu, int nlo, int nge,
                    float *const *src_tab, float *const *dst_tab, const IpcPeers &pput,
                    const IpcPeers &pget, int grid_cap, hipStream_t st);
// in-place allreduce of one device double over all ranks (op 0 sum, 1 max),
// reduced in rank order on every rank (identical results everywhere)
// (pub: the result also published to the host, kernels.hpp)
void ipc_allreduce(double *val, int op, const IpcReduce &r, unsigned long long *err,
                   const HostPub &pub, hipStream_t st);

}  // namespace kern
}  // namespace mgic
