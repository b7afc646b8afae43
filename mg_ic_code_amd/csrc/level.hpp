// level.hpp -- layouts, level data and ghost exchange (the Chombo
// DisjointBoxLayout / LevelData<FArrayBox> / Copier layer the reference
// operator relies on), MI355X-first:
//   * one process per GPU; boxes are owned by ranks; a rank may own several
//     boxes (tests run a multi-box decomposition on one GPU through the same
//     code path);
//   * the exchange is a precomputed CopyPlan: one batched kernel for
//     same-rank copies and packing, one grouped RCCL send/recv per peer over
//     xGMI, one batched unpack kernel -- no host round trip, capturable.
#pragma once

#include <rccl/rccl.h>

#include <array>
#include <map>

#include "kernels.hpp"
#include "mgic_core.hpp"
#include "transport.hpp"

namespace mgic {

#define MGIC_NCCL(x)                                                                  \
  do {                                                                                \
    ncclResult_t r_ = (x);                                                            \
    if (r_ != ncclSuccess)                                                            \
      throw ::mgic::Error(::mgic::kRcclErr,                                           \
                          std::string("RCCL error ") + ncclGetErrorString(r_) + " in " #x); \
  } while (0)

// host control plane for the peer-mapped transport's setup: gather `nbytes`
// from every rank into out[size * nbytes] (rank order); 0 on success.  The
// host passes its own collective (MPI_Allgather for Chombo, gloo for Python).
typedef int (*HostAllgather)(const void *in, size_t nbytes, void *out, void *user);

// One process's view of the job: rank, size, transport (RCCL communicator or
// peer-mapped buffers, transport.hpp), stream.
class Comm {
 public:
  Comm(int rank, int size, const ncclUniqueId *id, bool force_rccl);
  // peer-mapped transport: no RCCL communicator; `allgather` is called once,
  // here (may be null when size == 1); arena_bytes: one message buffer per
  // (sender, parity), 0 = MGIC_IPC_ARENA_MB (default 64 MB)
  Comm(int rank, int size, HostAllgather allgather, void *user, size_t arena_bytes);
  // rank/size only, no device resources: host-side planning (the exchange
  // plans a rank would execute) on machines without a GPU
  static std::shared_ptr<Comm> host_only(int rank, int size);
  ~Comm();
  int rank() const { return rank_; }
  int size() const { return size_; }
  bool uses_rccl() const { return nccl_ != nullptr; }
  bool uses_ipc() const { return ipc_; }
  bool remote_ok() const { return nccl_ != nullptr || ipc_; }
  // route same-rank copies through RCCL self send/recv (tests the remote
  // path on one GPU)
  bool self_messages() const { return self_messages_; }
  void set_self_messages(bool v) { self_messages_ = v; }
  // exchanges with messages issued so far (CopyPlan::execute*, a measurement counter)
  unsigned long long exchanges() const { return exchanges_; }
  void count_exchange() { ++exchanges_; }
  ncclComm_t nccl() const { return nccl_; }
  hipStream_t stream() const { return stream_; }
  void set_stream(hipStream_t s) { stream_ = s; }
  // in-place allreduce of one device double (op: 0 sum, 1 max); pub: the
  // result also published to the host (host_pub)
  void allreduce(double *d_val, int op, const kern::HostPub &pub = kern::HostPub());
  // scratch for reductions (device partials + result, pinned host result)
  double *d_partials(int n);
  // reduction results (device) and their host copies (pinned): slots 0-1 for
  // the operators' reductions
  static constexpr int kResultSlots = 4;
  double *d_result() const { return d_result_; }
  double *h_result() const { return h_result_; }
  // a reduction's readback: the final kernel (or the allreduce) publishes
  // result `slot` into h_result(); `last` also publishes the transport's error
  // word and the sequence number wait_results() spins on
  kern::HostPub host_pub(int slot, bool last);
  // after the launch that publishes `p` is queued: its sequence number becomes
  // the one wait_results() waits for
  void commit_pub(const kern::HostPub &p);
  // until the last host_pub(…, true) result (or the one of `ticket`, a
  // last_ticket() value) has landed (host spin on pinned memory, no stream
  // synchronisation); raises a transport timeout
  void wait_results(hipStream_t st, unsigned long long ticket = 0);
  unsigned long long last_ticket() const { return pub_count_; }
  // staging word for a host -> device copy (synchronised by its caller)
  double *h_stage() const { return h_result_ + kResultSlots; }

  // ---- peer-mapped transport (transport.hpp)
  size_t ipc_arena_bytes() const { return arena_bytes_; }
  // workgroup cap of one exchange launch: the CUs of the GPU, split among
  // the ranks that share it (MGIC_IPC_GRID_CAP overrides); see the constructor
  int ipc_grid_cap() const { return grid_cap_; }
  // elements per exchange block (MGIC_IPC_BLOCK_ELEMS, a multiple of 512;
  // every rank must use the same, checked at setup)
  long ipc_block_elems() const { return block_elems_; }
  // bound of every device-side wait, in 100 MHz clock ticks
  // (MGIC_IPC_TIMEOUT_S seconds, default 10)
  unsigned long long ipc_timeout_ticks() const { return timeout_ticks_; }
  // device-side barrier over the signal pages (returns once every rank's
  // earlier stream work is done; raises if a wait timed out)
  void ipc_barrier();
  // my next message to `peer` (nblocks put blocks) into entry q of a put
  // launch's peer table: its slot in the peer's arena, its flags in the
  // peer's page and their value, the acknowledgement count that frees the slot
  void ipc_send(int peer, long nblocks, kern::IpcPeers &pp, int q);
  // my next message from `src` into entry q of a get launch's peer table: its
  // slot in my arena, its flags in my page and their value, the sender's
  // acknowledgement counter
  void ipc_recv(int src, kern::IpcPeers &pp, int q);
  unsigned long long *ipc_err() const { return sig_ + kern::kSigErr; }
  // raise if a transport wait of this rank timed out (synchronizes the stream)
  void ipc_check();
  // the same split around a caller's own synchronize: queue the read of the
  // error word, then (after the stream sync) raise
  void ipc_err_async(hipStream_t st);
  void ipc_err_raise() const;

 private:
  Comm() = default;
  int rank_ = 0, size_ = 1;
  bool self_messages_ = false;
  ncclComm_t nccl_ = nullptr;
  hipStream_t stream_ = nullptr;
  bool own_stream_ = false;
  double *d_partials_ = nullptr;
  int n_partials_ = 0;
  double *d_result_ = nullptr;
  // pinned, host-coherent: kResultSlots results, a staging word, the error
  // word and the published sequence number
  double *h_result_ = nullptr;
  unsigned long long *h_seq_ = nullptr;
  unsigned long long pub_count_ = 0;
  void alloc_host_block();
  unsigned long long exchanges_ = 0;
  bool ipc_ = false;
  int grid_cap_ = 0;
  long block_elems_ = kern::kIpcBlockElemsDefault;
  unsigned long long timeout_ticks_ = 1000000000ull;
  double *barrier_val_ = nullptr;
  unsigned long long *sig_ = nullptr;            // my signal page (uncached)
  char *arena_ = nullptr;                        // my receive arena: size x 2 x arena_bytes_
  size_t arena_bytes_ = 0;
  std::vector<unsigned long long *> peer_sig_;   // per rank (mine at [rank_])
  std::vector<char *> peer_arena_;
  std::vector<unsigned long long> sent_, recvd_;  // messages per peer so far
  // cumulative blocks sent per peer (after the last message / before it)
  std::vector<unsigned long long> sent_blocks_, sent_prev_;
  unsigned long long red_count_ = 0;
  unsigned long long *h_err_ = nullptr;          // pinned
};

// A precomputed set of rectangular copies between two LevelData layouts
// (possibly the same), split into same-rank copies and per-peer messages.
class CopyPlan {
 public:
  ~CopyPlan();
  void finalize_host();  // per-peer buffer offsets (host only)
  void finalize();       // + upload the item tables (RCCL / local copies)
  // + the peer-mapped transport's tables (on first use; per = elements per block)
  void finalize_ipc(long per);
  // the peer-mapped transport's host tables only (raises when the plan has
  // more peers than that transport takes: kern::kMaxIpcPeers)
  void finalize_ipc_host(long per);
  // after finalize_ipc_host: per put / get block {side (0 put, 1 get), peer
  // rank, flag, first message element, element count}
  std::vector<std::array<long long, 5>> ipc_block_rows() const;
  // src_tab / dst_tab: device tables of valid-lo pointers per local box
  void execute(Comm &comm, double *const *src_tab, double *const *dst_tab, hipStream_t st);
  // the same copies on fp32 fields (same element offsets; messages in floats)
  void execute_f(Comm &comm, float *const *src_tab, float *const *dst_tab, hipStream_t st);
  bool empty() const { return local_.empty() && pack_.empty() && unpack_.empty(); }

  std::vector<CopyItem> local_, pack_, unpack_;
  std::map<int, long> send_cnt_, recv_cnt_;  // per peer rank, doubles
  std::map<int, long> send_off_, recv_off_;
  long send_total_ = 0, recv_total_ = 0;

 private:
  template <class T>
  void execute_ipc(Comm &comm, T *const *src_tab, T *const *dst_tab, hipStream_t st);
  void alloc_buffers();
  CopyItem *d_local_ = nullptr, *d_pack_ = nullptr, *d_unpack_ = nullptr;
  // the peer-mapped transport's item tables: offsets within one peer's
  // message, pad = index into the plan's peer list
  CopyItem *d_ipc_pack_ = nullptr, *d_ipc_unpack_ = nullptr;
  kern::IpcBlock *d_xblocks_ = nullptr;  // put, local, get blocks of the one-launch exchange
  int n_put_blocks_ = 0, n_loc_blocks_ = 0, n_get_blocks_ = 0;
  long ipc_per_ = 0;  // elements per block of the tables above
  std::vector<int> send_peers_, recv_peers_;
  std::vector<long> send_blocks_, recv_blocks_;  // per peer of the lists above
  long max_local_ = 0, max_pack_ = 0, max_unpack_ = 0;
  double *sendbuf_ = nullptr, *recvbuf_ = nullptr;
  bool final_ = false, host_final_ = false, ipc_final_ = false, ipc_host_ = false;
  std::vector<CopyItem> ipc_pack_h_, ipc_unpack_h_;
  std::vector<kern::IpcBlock> xblocks_h_;
};

// DisjointBoxLayout + ProblemDomain + dx at one level.
class Grid {
 public:
  Grid(std::shared_ptr<Comm> comm, const Box &domain, const bool periodic[3], double dx,
       const std::vector<Box> &boxes, const std::vector<int> &owners);
  std::shared_ptr<Comm> comm;
  Box domain;
  bool periodic[3];
  double dx;
  std::vector<Box> boxes;    // global list
  std::vector<int> owners;   // rank per box
  std::vector<int> local;    // global indices of my boxes
  std::vector<FabGeom> geom; // per local box
  int nlocal() const { return (int)local.size(); }
  long max_cells_local() const;
  bool tiles_domain() const;  // boxes disjoint and covering the domain
  bool coarsenable(int r) const;
  std::shared_ptr<Grid> coarsened(int r) const;
  // face ghost exchange plan (exchangeDefine(grids, Unit) + trimEdges)
  CopyPlan &exchange_plan();
  // full 2-deep ghost shell (faces, edges, corners): what a fused sweep
  // needs to recompute the neighbours' red values on its own ghost layer
  CopyPlan &shell_plan(int depth = 2);
  bool has_memory_faces() const;  // some local box face is exchanged
  // BoxArgs of local box n with the face BC modes for (bc flags, value,
  // homogeneous); faces that are not domain faces (or are periodic) get
  // kBcMemory.
  BoxArgs box_args(int n, const int bc_lo[3], const int bc_hi[3], double bc_value,
                   bool homogeneous) const;
  BoxArgs box_args_plain(int n) const;  // all faces kBcMemory

 private:
  std::unique_ptr<CopyPlan> exchange_;
  std::map<int, std::unique_ptr<CopyPlan>> shell_;  // per depth
};

// Build a copy plan from src layout to dst layout.  dst regions: the valid
// box (with_valid) and/or its six 1-deep face slabs (with_faces); periodic
// images of src boxes are used in periodic directions.  Both layouts must
// live on the same domain index space.
// upload = false: host-side plan only (no device tables / buffers).
// shell > 0: instead of the 1-deep faces, the full ghost shell of that depth.
std::unique_ptr<CopyPlan> build_copy_plan(const Grid &src, const Grid &dst, bool with_valid,
                                          bool with_faces, bool upload = true, int shell = 0);

// LevelData<FArrayBox> with one component and one ghost layer.
class LevelData {
 public:
  explicit LevelData(std::shared_ptr<Grid> g);
  ~LevelData();
  LevelData(const LevelData &) = delete;
  LevelData &operator=(const LevelData &) = delete;
  std::shared_ptr<Grid> grid;
  std::vector<double *> base;  // allocation per local box
  std::vector<double *> p;     // valid-lo pointer per local box
  double **d_tab = nullptr;    // device copy of p
  double *ptr(int n) const { return p[n]; }
  void set_zero_all(hipStream_t st);  // valid + ghosts
  void exchange(hipStream_t st);
  void exchange_shell(hipStream_t st, int depth = 2);  // faces + edges + corners
};

// The same layout with fp32 elements (the mixed-precision V-cycle's
// corrections, right-hand sides and coefficients): identical FabGeom in
// elements, so every kernel offset and copy plan is shared with LevelData.
class LevelDataF {
 public:
  explicit LevelDataF(std::shared_ptr<Grid> g);
  ~LevelDataF();
  LevelDataF(const LevelDataF &) = delete;
  LevelDataF &operator=(const LevelDataF &) = delete;
  std::shared_ptr<Grid> grid;
  std::vector<float *> base;
  std::vector<float *> p;
  float **d_tab = nullptr;
  void exchange(hipStream_t st);
  void exchange_shell(hipStream_t st, int depth = 2);
};

}  // namespace mgic
