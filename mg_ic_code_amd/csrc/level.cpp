// level.cpp -- Comm, Grid, CopyPlan, LevelData (see level.hpp).
#include "level.hpp"

#include <cstdio>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <type_traits>

namespace mgic {

// ------------------------------------------------------------------ Comm
Comm::Comm(int rank, int size, const ncclUniqueId *id, bool force_rccl)
    : rank_(rank), size_(size) {
  MGIC_CHECK(size >= 1 && rank >= 0 && rank < size, "bad rank/size");
  MGIC_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  own_stream_ = true;
  if (size > 1 || force_rccl) {
    MGIC_CHECK(id != nullptr, "RCCL unique id required for size > 1");
    MGIC_NCCL(ncclCommInitRank(&nccl_, size, *id, rank));
  }
  MGIC_HIP(hipMalloc(&d_result_, kResultSlots * sizeof(double)));
  alloc_host_block();
}

// results, staging word, error word and sequence number in one pinned,
// host-coherent block: the GPU's stores reach the host without a copy
void Comm::alloc_host_block() {
  void *p = nullptr;
  MGIC_HIP(hipHostMalloc(&p, (kResultSlots + 3) * sizeof(double), hipHostMallocCoherent));
  h_result_ = static_cast<double *>(p);
  for (int i = 0; i < kResultSlots + 1; ++i) h_result_[i] = 0.0;
  h_err_ = reinterpret_cast<unsigned long long *>(h_result_ + kResultSlots + 1);
  h_seq_ = h_err_ + 1;
  *h_err_ = 0;
  *h_seq_ = 0;
}

kern::HostPub Comm::host_pub(int slot, bool last) {
  MGIC_CHECK(slot >= 0 && slot < kResultSlots, "result slot");
  kern::HostPub p;
  p.val = h_result_ + slot;
  if (last) {
    // the sequence number is taken here and committed (commit_pub) once the
    // publishing launch is queued: a launch that throws leaves the count as
    // it was, so later waits do not wait for a number that never comes
    p.seq = h_seq_;
    p.seqv = pub_count_ + 1;
    if (ipc_) {
      p.err_src = sig_ + kern::kSigErr;
      p.err_dst = h_err_;
    }
  }
  return p;
}

void Comm::commit_pub(const kern::HostPub &p) {
  if (p.seq) pub_count_ = p.seqv;
}

void Comm::wait_results(hipStream_t st, unsigned long long ticket) {
  const unsigned long long want = ticket ? ticket : pub_count_;
  for (unsigned long long i = 0;; ++i) {
    if (__atomic_load_n(h_seq_, __ATOMIC_ACQUIRE) >= want) break;
    if ((i & 1023) == 1023) {
      // a faulted or finished stream that never published: report, not spin
      const hipError_t e = hipStreamQuery(st);
      if (e == hipSuccess) {
        if (__atomic_load_n(h_seq_, __ATOMIC_ACQUIRE) >= want) break;
        throw Error(kState, "reduction result was not published");
      }
      if (e != hipErrorNotReady) MGIC_HIP(e);
      if (i > (1ull << 22)) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    __builtin_ia32_pause();
  }
  ipc_err_raise();
}

// the peer-mapped transport: signal page + receive arena per rank, mapped by
// every other rank (transport.hpp)
Comm::Comm(int rank, int size, HostAllgather allgather, void *user, size_t arena_bytes)
    : rank_(rank), size_(size) {
  MGIC_CHECK(size >= 1 && rank >= 0 && rank < size, "bad rank/size");
  MGIC_CHECK(size <= kern::kMaxIpcRanks, "peer-mapped transport: too many ranks");
  MGIC_CHECK(size == 1 || allgather != nullptr, "peer-mapped transport needs a host allgather");
  if (arena_bytes == 0) {
    const char *e = getenv("MGIC_IPC_ARENA_MB");
    arena_bytes = (size_t)(e ? atol(e) : 64) << 20;
  }
  arena_bytes_ = (arena_bytes + 255) & ~(size_t)255;
  MGIC_CHECK(arena_bytes_ < ((size_t)1 << 31), "transport arena buffer must stay below 2 GB "
                                               "(32-bit buffer offsets)");
  MGIC_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  own_stream_ = true;
  MGIC_HIP(hipMalloc(&d_result_, kResultSlots * sizeof(double)));
  alloc_host_block();
  // counters are polled across processes / devices: uncached memory
  MGIC_HIP(hipExtMallocWithFlags((void **)&sig_, sizeof(unsigned long long) * kern::sig_words(size),
                                 hipDeviceMallocUncached));
  MGIC_HIP(hipMemset(sig_, 0, sizeof(unsigned long long) * kern::sig_words(size)));
  MGIC_HIP(hipMalloc(&arena_, (size_t)size * 2 * arena_bytes_));
  MGIC_HIP(hipDeviceSynchronize());
  ipc_ = true;
  {
    const char *te = getenv("MGIC_IPC_TIMEOUT_S");
    const double s = te ? atof(te) : 10.0;
    // the 100 MHz constant clock (wall_clock64); at least 1 ms
    timeout_ticks_ = (unsigned long long)(std::max(s, 1e-3) * 1e8);
    const char *be = getenv("MGIC_IPC_BLOCK_ELEMS");
    if (be && atol(be) > 0) block_elems_ = atol(be);
    MGIC_CHECK(block_elems_ >= 512 && block_elems_ <= (1 << 20) && block_elems_ % 512 == 0,
               "MGIC_IPC_BLOCK_ELEMS must be a multiple of 512 in [512, 2^20]");
  }
  peer_sig_.assign(size, nullptr);
  peer_arena_.assign(size, nullptr);
  sent_.assign(size, 0);
  recvd_.assign(size, 0);
  sent_blocks_.assign(size, 0);
  sent_prev_.assign(size, 0);
  peer_sig_[rank] = sig_;
  peer_arena_[rank] = arena_;
  int colocated = 1;  // ranks on this GPU (this one included)
  if (size > 1) {
    colocated = 0;
    struct Rec {
      hipIpcMemHandle_t sig, arena;
      unsigned long long arena_bytes;
      long block_elems;
      int rank;
      int pci[3];  // domain, bus, device of this rank's GPU
    } mine{}, *all = nullptr;
    MGIC_HIP(hipIpcGetMemHandle(&mine.sig, sig_));
    MGIC_HIP(hipIpcGetMemHandle(&mine.arena, arena_));
    mine.arena_bytes = arena_bytes_;
    mine.block_elems = block_elems_;
    mine.rank = rank;
    {
      int dev = 0;
      MGIC_HIP(hipGetDevice(&dev));
      MGIC_HIP(hipDeviceGetAttribute(&mine.pci[0], hipDeviceAttributePciDomainID, dev));
      MGIC_HIP(hipDeviceGetAttribute(&mine.pci[1], hipDeviceAttributePciBusId, dev));
      MGIC_HIP(hipDeviceGetAttribute(&mine.pci[2], hipDeviceAttributePciDeviceId, dev));
    }
    std::vector<Rec> recs(size);
    all = recs.data();
    if (allgather(&mine, sizeof(Rec), all, user) != 0)
      throw Error(kState, "peer-mapped transport: host allgather failed");
    for (int r = 0; r < size; ++r)
      colocated += recs[r].pci[0] == mine.pci[0] && recs[r].pci[1] == mine.pci[1] &&
                   recs[r].pci[2] == mine.pci[2];
    for (int r = 0; r < size; ++r) {
      MGIC_CHECK(recs[r].rank == r && recs[r].arena_bytes == arena_bytes_ &&
                     recs[r].block_elems == block_elems_,
                 "peer-mapped transport: ranks disagree on the setup");
      if (r == rank) continue;
      void *ps = nullptr, *pa = nullptr;
      MGIC_HIP(hipIpcOpenMemHandle(&ps, recs[r].sig, hipIpcMemLazyEnablePeerAccess));
      MGIC_HIP(hipIpcOpenMemHandle(&pa, recs[r].arena, hipIpcMemLazyEnablePeerAccess));
      peer_sig_[r] = static_cast<unsigned long long *>(ps);
      peer_arena_[r] = static_cast<char *>(pa);
    }
  }
  // The exchange launch's grid (k_exchange): workgroups stride over the
  // virtual blocks in ascending order, puts first, so a workgroup has done
  // all its puts before its first get; and the grid is capped so that every
  // workgroup of every rank on this GPU can be resident at once.  Then no get
  // can hold a slot a put needs, whatever order the hardware dispatches
  // workgroups in.  Two workgroups per CU for one rank per GPU (a quarter of
  // what fits: 8 per CU at the kernel's 8 waves per SIMD; 512 measured 0.8%
  // faster than 256 on the 8-GPU share, profiles/r04l_exchange_cap_sweep.txt);
  // ranks sharing a GPU split half the CUs (r03i rehearsals).
  {
    int dev = 0, ncu = 0;
    MGIC_HIP(hipGetDevice(&dev));
    MGIC_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    ncu = std::max(ncu, 8);
    const char *ce = getenv("MGIC_IPC_GRID_CAP");
    grid_cap_ = ce && atoi(ce) > 0 ? atoi(ce)
                                   : (colocated > 1 ? std::max(8, ncu / (2 * colocated)) : 2 * ncu);
  }
}

void Comm::ipc_barrier() {
  if (!ipc_ || size_ == 1) return;
  // an allreduce over the signal pages completes on a rank only after every
  // rank has issued it, i.e. after every rank's earlier stream work (its
  // exchanges' puts into this rank's arena and acks into its page) is done
  if (!barrier_val_) MGIC_HIP(hipMalloc(&barrier_val_, sizeof(double)));
  MGIC_HIP(hipMemsetAsync(barrier_val_, 0, sizeof(double), stream_));
  allreduce(barrier_val_, 0);
  ipc_check();
}

void Comm::ipc_send(int peer, long nblocks, kern::IpcPeers &pp, int q) {
  const unsigned long long m = sent_[peer]++;  // my message number m to peer (0-based)
  const size_t slot = (size_t)rank_ * 2 + (m & 1);
  pp.buf[q] = peer_arena_[peer] + slot * arena_bytes_;
  pp.flags[q] = peer_sig_[peer] + kern::kSigFlags + slot * kern::kMaxMsgBlocks;
  pp.seq[q] = m + 1;
  // the slot last held message m - 2: wait until the peer has acknowledged
  // every block up to and including it (= the blocks sent before message m - 1)
  pp.ack[q] = sig_ + kern::kSigAck + peer * kern::kSigStride;
  pp.val[q] = sent_prev_[peer];
  sent_prev_[peer] = sent_blocks_[peer];
  sent_blocks_[peer] += (unsigned long long)nblocks;
}

void Comm::ipc_recv(int src, kern::IpcPeers &pp, int q) {
  const unsigned long long m = recvd_[src]++;
  const size_t slot = (size_t)src * 2 + (m & 1);
  pp.buf[q] = arena_ + slot * arena_bytes_;
  pp.flags[q] = sig_ + kern::kSigFlags + slot * kern::kMaxMsgBlocks;
  pp.seq[q] = m + 1;
  pp.ack[q] = peer_sig_[src] + kern::kSigAck + rank_ * kern::kSigStride;
  pp.val[q] = 0;
}

void Comm::ipc_err_async(hipStream_t st) {
  if (!ipc_) return;
  MGIC_HIP(hipMemcpyAsync(h_err_, sig_ + kern::kSigErr, sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, st));
}

void Comm::ipc_err_raise() const {
  if (ipc_ && *h_err_ != 0)
    throw Error(kState, "peer-mapped transport: a wait for a peer timed out (peer gone or the "
                        "ranks' exchange sequences differ)");
}

void Comm::ipc_check() {
  if (!ipc_) return;
  ipc_err_async(stream_);
  MGIC_HIP(hipStreamSynchronize(stream_));
  ipc_err_raise();
}

std::shared_ptr<Comm> Comm::host_only(int rank, int size) {
  MGIC_CHECK(size >= 1 && rank >= 0 && rank < size, "bad rank/size");
  std::shared_ptr<Comm> c(new Comm());
  c->rank_ = rank;
  c->size_ = size;
  return c;
}

Comm::~Comm() {
  if (nccl_) ncclCommDestroy(nccl_);
  if (ipc_) {
    // no rank unmaps or frees its arena / signal page while a peer may still
    // write into it: a collective barrier (every rank destroys its
    // communicator), bounded -- a peer that is gone times it
    // out after MGIC_IPC_TIMEOUT_S, which is reported on stderr.  It runs on
    // a stream of its own after this rank's work on every stream has drained:
    // the caller's stream (mgic_comm_set_stream) may be gone by now.
    if (*h_err_ == 0) {
      hipStream_t s = nullptr;
      const hipStream_t keep = stream_;
      try {
        MGIC_HIP(hipDeviceSynchronize());
        MGIC_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        stream_ = s;
        ipc_barrier();
      } catch (const std::exception &e) {
        fprintf(stderr, "mgic: rank %d: communicator teardown barrier: %s\n", rank_, e.what());
      }
      stream_ = keep;
      if (s) (void)hipStreamDestroy(s);
    }
    (void)hipDeviceSynchronize();
    for (int r = 0; r < size_; ++r) {
      if (r == rank_) continue;
      if (peer_sig_[r]) (void)hipIpcCloseMemHandle(peer_sig_[r]);
      if (peer_arena_[r]) (void)hipIpcCloseMemHandle(peer_arena_[r]);
    }
    if (sig_) (void)hipFree(sig_);
    if (arena_) (void)hipFree(arena_);
    if (barrier_val_) (void)hipFree(barrier_val_);
  }
  if (d_partials_) (void)hipFree(d_partials_);
  if (d_result_) (void)hipFree(d_result_);
  if (h_result_) (void)hipHostFree(h_result_);
  if (own_stream_ && stream_) (void)hipStreamDestroy(stream_);
}

double *Comm::d_partials(int n) {
  if (n > n_partials_) {
    if (d_partials_) MGIC_HIP(hipFree(d_partials_));
    n_partials_ = std::max(n, 4096);
    MGIC_HIP(hipMalloc(&d_partials_, sizeof(double) * (size_t)n_partials_));
  }
  return d_partials_;
}

void Comm::allreduce(double *d_val, int op, const kern::HostPub &pub) {
  if (size_ == 1) {
    kern::publish_result(d_val, pub, stream_);
    return;
  }
  if (ipc_) {
    kern::IpcReduce r{};
    r.size = size_;
    r.rank = rank_;
    r.count = ++red_count_;
    r.parity = (int)(r.count & 1);
    r.timeout = timeout_ticks_;
    for (int q = 0; q < size_; ++q) r.sig[q] = peer_sig_[q];
    kern::ipc_allreduce(d_val, op, r, ipc_err(), pub, stream_);
    return;
  }
  if (nccl_)
    MGIC_NCCL(ncclAllReduce(d_val, d_val, 1, ncclDouble, op == 1 ? ncclMax : ncclSum, nccl_, stream_));
  kern::publish_result(d_val, pub, stream_);
}

// ------------------------------------------------------------------ Grid
Grid::Grid(std::shared_ptr<Comm> c, const Box &dom, const bool per[3], double dx_,
           const std::vector<Box> &bx, const std::vector<int> &own)
    : comm(std::move(c)), domain(dom), dx(dx_), boxes(bx), owners(own) {
  MGIC_CHECK(boxes.size() == owners.size(), "boxes/owners size mismatch");
  for (int d = 0; d < 3; ++d) periodic[d] = per[d];
  for (size_t b = 0; b < boxes.size(); ++b) {
    MGIC_CHECK(!boxes[b].empty(), "empty box");
    MGIC_CHECK(domain.contains(boxes[b]), "box outside domain");
    MGIC_CHECK(owners[b] >= 0 && owners[b] < comm->size(), "bad owner rank");
    if (owners[b] == comm->rank()) {
      local.push_back((int)b);
      geom.push_back(FabGeom::make(boxes[b]));
    }
  }
}

long Grid::max_cells_local() const {
  long m = 0;
  for (auto &g : geom) m = std::max(m, g.valid.ncells());
  return m;
}

bool Grid::tiles_domain() const {
  long tot = 0;
  for (auto &b : boxes) tot += b.ncells();
  if (tot != domain.ncells()) return false;
  for (size_t a = 0; a < boxes.size(); ++a)
    for (size_t b = a + 1; b < boxes.size(); ++b)
      if (!boxes[a].intersect(boxes[b]).empty()) return false;
  return true;
}

bool Grid::coarsenable(int r) const {
  for (auto &b : boxes)
    if (!b.coarsenable(r)) return false;
  return true;
}

std::shared_ptr<Grid> Grid::coarsened(int r) const {
  std::vector<Box> cb;
  for (auto &b : boxes) cb.push_back(b.coarsened(r));
  return std::make_shared<Grid>(comm, domain.coarsened(r), periodic, dx * (double)r, cb, owners);
}

CopyPlan &Grid::exchange_plan() {
  if (!exchange_) exchange_ = build_copy_plan(*this, *this, false, true);
  return *exchange_;
}

CopyPlan &Grid::shell_plan(int depth) {
  MGIC_CHECK(depth >= 1 && depth <= kGhost, "shell depth exceeds the allocated ghosts");
  auto &p = shell_[depth];
  if (!p) p = build_copy_plan(*this, *this, false, false, true, depth);
  return *p;
}

bool Grid::has_memory_faces() const {
  for (int n = 0; n < nlocal(); ++n) {
    const Box &v = geom[n].valid;
    for (int d = 0; d < 3; ++d)
      if (periodic[d] || v.lo[d] != domain.lo[d] || v.hi[d] != domain.hi[d]) return true;
  }
  return false;
}

BoxArgs Grid::box_args_plain(int n) const {
  BoxArgs a{};
  const FabGeom &g = geom[n];
  a.nx = g.nx;
  a.ny = g.ny;
  a.nz = g.nz;
  a.sy = g.sy;
  a.sz = g.sz;
  for (int d = 0; d < 3; ++d) a.glo[d] = g.valid.lo[d];
  for (int f = 0; f < 6; ++f) {
    a.bcm[f] = kBcMemory;
    a.bcc[f] = 0.0;
  }
  return a;
}

BoxArgs Grid::box_args(int n, const int bc_lo[3], const int bc_hi[3], double bc_value,
                       bool homogeneous) const {
  BoxArgs a = box_args_plain(n);
  const Box &v = geom[n].valid;
  const double val = homogeneous ? 0.0 : bc_value;  // ParseValue (SetBCs.cpp:42-47)
  for (int dir = 0; dir < 3; ++dir) {
    if (periodic[dir]) continue;  // SetBCs.cpp:65
    for (int side = 0; side < 2; ++side) {
      const bool at_dom = side == 0 ? v.lo[dir] == domain.lo[dir] : v.hi[dir] == domain.hi[dir];
      if (!at_dom) continue;  // SetBCs.cpp:68, :98
      const int flag = side == 0 ? bc_lo[dir] : bc_hi[dir];
      const int f = 2 * dir + side;
      const int isign = side == 0 ? -1 : 1;
      if (flag == 0) {  // DiriBC, order 1
        a.bcm[f] = kBcDirichlet;
        a.bcc[f] = 2.0 * val;
      } else if (flag == 1) {  // NeumBC
        if (homogeneous) {
          a.bcm[f] = kBcNeumannHom;
        } else {
          a.bcm[f] = kBcNeumann;
          a.bcc[f] = (double)isign * dx * val;
        }
      } else if (flag == 2) {  // periodic flag on a non-periodic domain: no fill
        a.bcm[f] = kBcMemory;
      } else {
        throw Error(kBadArg, "bogus bc flag");  // MayDay::Error (SetBCs.cpp:94, :123)
      }
    }
  }
  return a;
}

// ------------------------------------------------------------------ CopyPlan
std::unique_ptr<CopyPlan> build_copy_plan(const Grid &src, const Grid &dst, bool with_valid,
                                          bool with_faces, bool upload, int shell) {
  auto plan = std::make_unique<CopyPlan>();
  const int me = dst.comm->rank();
  std::vector<int> sloc(src.boxes.size(), -1), dloc(dst.boxes.size(), -1);
  for (int n = 0; n < src.nlocal(); ++n) sloc[src.local[n]] = n;
  for (int n = 0; n < dst.nlocal(); ++n) dloc[dst.local[n]] = n;
  int len[3];
  for (int d = 0; d < 3; ++d) len[d] = dst.domain.size(d);
  const bool self_msg = dst.comm->self_messages() && dst.comm->remote_ok();
  for (size_t db = 0; db < dst.boxes.size(); ++db) {
    const Box &dv = dst.boxes[db];
    std::vector<Box> regions;
    if (with_valid) regions.push_back(dv);
    if (with_faces)
      for (int dir = 0; dir < 3; ++dir)
        for (int side = 0; side < 2; ++side) regions.push_back(dv.adj_cell(dir, side));
    if (shell > 0) {  // grow(dv, shell) \ dv as six disjoint slabs: the x slabs span
      // the grown y and z ranges, the y slabs the valid x and grown z, the z
      // slabs the valid x and y
      for (int dir = 0; dir < 3; ++dir)
        for (int side = 0; side < 2; ++side) {
          Box r = dv;
          for (int d = 0; d < 3; ++d)
            if (d > dir) {
              r.lo[d] -= shell;
              r.hi[d] += shell;
            }
          if (side == 0) {
            r.hi[dir] = dv.lo[dir] - 1;
            r.lo[dir] = dv.lo[dir] - shell;
          } else {
            r.lo[dir] = dv.hi[dir] + 1;
            r.hi[dir] = dv.hi[dir] + shell;
          }
          regions.push_back(r);
        }
    }
    const int od = dst.owners[db];
    for (const Box &R : regions) {
      for (size_t sb = 0; sb < src.boxes.size(); ++sb) {
        const int os = src.owners[sb];
        if (od != me && os != me) continue;
        for (int sz = -1; sz <= 1; ++sz)
          for (int sy = -1; sy <= 1; ++sy)
            for (int sx = -1; sx <= 1; ++sx) {
              if ((sx && !dst.periodic[0]) || (sy && !dst.periodic[1]) || (sz && !dst.periodic[2]))
                continue;
              const int sh[3] = {sx * len[0], sy * len[1], sz * len[2]};
              const Box X = R.intersect(src.boxes[sb].shifted(sh));
              if (X.empty()) continue;
              CopyItem it{};
              it.nx = X.size(0);
              it.ny = X.size(1);
              it.nz = X.size(2);
              const long n = X.ncells();
              if (od == me) {
                const FabGeom &g = dst.geom[dloc[db]];
                it.dst = dloc[db];
                it.doff = g.offset(X.lo[0], X.lo[1], X.lo[2]);
                it.dsy = g.sy;
                it.dsz = g.sz;
              }
              if (os == me) {
                const FabGeom &g = src.geom[sloc[sb]];
                it.src = sloc[sb];
                it.soff = g.offset(X.lo[0] - sh[0], X.lo[1] - sh[1], X.lo[2] - sh[2]);
                it.ssy = g.sy;
                it.ssz = g.sz;
              }
              if (od == me && os == me && !self_msg) {
                plan->local_.push_back(it);
                continue;
              }
              if (os == me) {  // send to od (possibly ourselves through RCCL)
                CopyItem p = it;
                p.dst = -1;
                p.pad = od;
                p.doff = plan->send_cnt_[od];
                p.dsy = it.nx;
                p.dsz = (long)it.nx * it.ny;
                plan->send_cnt_[od] += n;
                plan->pack_.push_back(p);
              }
              if (od == me) {  // receive from os
                CopyItem u = it;
                u.src = -1;
                u.pad = os;
                u.soff = plan->recv_cnt_[os];
                u.ssy = it.nx;
                u.ssz = (long)it.nx * it.ny;
                plan->recv_cnt_[os] += n;
                plan->unpack_.push_back(u);
              }
            }
      }
    }
  }
  if (upload)
    plan->finalize();
  else
    plan->finalize_host();
  return plan;
}

CopyPlan::~CopyPlan() {
  if (d_local_) (void)hipFree(d_local_);
  if (d_pack_) (void)hipFree(d_pack_);
  if (d_unpack_) (void)hipFree(d_unpack_);
  if (d_ipc_pack_) (void)hipFree(d_ipc_pack_);
  if (d_ipc_unpack_) (void)hipFree(d_ipc_unpack_);
  if (d_xblocks_) (void)hipFree(d_xblocks_);
  if (sendbuf_) (void)hipFree(sendbuf_);
  if (recvbuf_) (void)hipFree(recvbuf_);
}

static CopyItem *upload_items(const std::vector<CopyItem> &v, long &maxc) {
  maxc = 0;
  for (auto &it : v) maxc = std::max(maxc, (long)it.nx * it.ny * it.nz);
  if (v.empty()) return nullptr;
  CopyItem *d = nullptr;
  MGIC_HIP(hipMalloc(&d, sizeof(CopyItem) * v.size()));
  MGIC_HIP(hipMemcpy(d, v.data(), sizeof(CopyItem) * v.size(), hipMemcpyHostToDevice));
  return d;
}

void CopyPlan::finalize_host() {
  if (host_final_) return;
  long off = 0;
  for (auto &kv : send_cnt_) {
    send_off_[kv.first] = off;
    off += kv.second;
  }
  send_total_ = off;
  off = 0;
  for (auto &kv : recv_cnt_) {
    recv_off_[kv.first] = off;
    off += kv.second;
  }
  recv_total_ = off;
  for (auto &it : pack_) it.doff += send_off_[it.pad];
  for (auto &it : unpack_) it.soff += recv_off_[it.pad];
  host_final_ = true;
}

void CopyPlan::finalize() {
  if (final_) return;
  finalize_host();
  d_local_ = upload_items(local_, max_local_);
  d_pack_ = upload_items(pack_, max_pack_);
  d_unpack_ = upload_items(unpack_, max_unpack_);
  final_ = true;
}

// The peer-mapped transport's tables, built on the plan's first execution
// through that transport (an RCCL job never builds them, and the transport's
// peer limit binds only plans it executes): offsets within each peer's
// message, pad = the peer's index in send_peers_ / recv_peers_; one block
// table for the one-launch exchange: put blocks, then the same-rank copies,
// then get blocks, every item split into blocks of ipc_item_per(cells, per) -- the same
// split on the sending and the receiving side, so a message's blocks and their
// flags match
void CopyPlan::finalize_ipc_host(long per) {
  if (ipc_host_) {
    MGIC_CHECK(per == ipc_per_, "exchange plan: executed with two transport block sizes");
    return;
  }
  MGIC_CHECK(per >= 512 && per % 512 == 0, "transport block size must be a multiple of 512");
  ipc_per_ = per;
  finalize_host();
  ipc_pack_h_.clear();
  ipc_unpack_h_.clear();
  xblocks_h_.clear();
  send_peers_.clear();
  recv_peers_.clear();
  if (!pack_.empty() || !unpack_.empty()) {
    for (auto &kv : send_cnt_) send_peers_.push_back(kv.first);
    for (auto &kv : recv_cnt_) recv_peers_.push_back(kv.first);
    MGIC_CHECK((int)send_peers_.size() <= kern::kMaxIpcPeers &&
                   (int)recv_peers_.size() <= kern::kMaxIpcPeers,
               "exchange plan: too many peers for the peer-mapped transport");
    ipc_pack_h_ = pack_;
    ipc_unpack_h_ = unpack_;
    for (auto &it : ipc_pack_h_) {
      it.doff -= send_off_[it.pad];
      it.pad = (int)(std::find(send_peers_.begin(), send_peers_.end(), it.pad) - send_peers_.begin());
    }
    for (auto &it : ipc_unpack_h_) {
      it.soff -= recv_off_[it.pad];
      it.pad = (int)(std::find(recv_peers_.begin(), recv_peers_.end(), it.pad) - recv_peers_.begin());
    }
    // side: 0 puts (message offset doff), 1 same-rank copies (no flag), 2 gets
    // (message offset soff); a message's blocks are numbered (flag) in the
    // order of their first element in the message, the same on both sides
    auto add = [&](const std::vector<CopyItem> &v, size_t npeers, std::vector<long> *by_peer,
                   int side) {
      if (by_peer) by_peer->assign(npeers, 0);
      const size_t n0 = xblocks_h_.size();
      std::vector<std::vector<std::pair<long, size_t>>> order(npeers);  // (offset, block)
      for (size_t i = 0; i < v.size(); ++i) {
        const long cells = (long)v[i].nx * v[i].ny * v[i].nz;
        const long pi = kern::ipc_item_per(cells, per), nb = kern::ipc_blocks(cells, pi);
        const long mo = side == 0 ? v[i].doff : v[i].soff;
        for (long b = 0; b < nb; ++b) {
          if (side != 1) order[v[i].pad].push_back({mo + b * pi, xblocks_h_.size()});
          xblocks_h_.push_back({(int)i, -1, (unsigned)(b * pi), (unsigned)std::min(cells, (b + 1) * pi)});
        }
        if (by_peer) (*by_peer)[v[i].pad] += nb;
      }
      for (auto &o : order) {
        MGIC_CHECK((long)o.size() <= kern::kMaxMsgBlocks,
                   "exchange message has more blocks than the transport flags "
                   "(raise MGIC_IPC_BLOCK_ELEMS)");
        std::sort(o.begin(), o.end());
        for (size_t f = 0; f < o.size(); ++f) xblocks_h_[o[f].second].flag = (int)f;
      }
      return (int)(xblocks_h_.size() - n0);
    };
    n_put_blocks_ = add(ipc_pack_h_, send_peers_.size(), &send_blocks_, 0);
    n_loc_blocks_ = add(local_, 0, nullptr, 1);
    n_get_blocks_ = add(ipc_unpack_h_, recv_peers_.size(), &recv_blocks_, 2);
  }
  ipc_host_ = true;
}

std::vector<std::array<long long, 5>> CopyPlan::ipc_block_rows() const {
  std::vector<std::array<long long, 5>> rows;
  for (int v = 0; v < (int)xblocks_h_.size(); ++v) {
    if (v >= n_put_blocks_ && v < n_put_blocks_ + n_loc_blocks_) continue;
    const bool put = v < n_put_blocks_;
    const kern::IpcBlock &b = xblocks_h_[v];
    const CopyItem &it = put ? ipc_pack_h_[b.item] : ipc_unpack_h_[b.item];
    const int peer = put ? send_peers_[it.pad] : recv_peers_[it.pad];
    rows.push_back({put ? 0LL : 1LL, (long long)peer, (long long)b.flag,
                    (long long)(put ? it.doff : it.soff) + b.e0, (long long)(b.e1 - b.e0)});
  }
  return rows;
}

void CopyPlan::finalize_ipc(long per) {
  if (ipc_final_) return;
  finalize();
  finalize_ipc_host(per);
  if (!xblocks_h_.empty()) {
    long dummy = 0;
    d_ipc_pack_ = upload_items(ipc_pack_h_, dummy);
    d_ipc_unpack_ = upload_items(ipc_unpack_h_, dummy);
    MGIC_HIP(hipMalloc(&d_xblocks_, sizeof(kern::IpcBlock) * xblocks_h_.size()));
    MGIC_HIP(hipMemcpy(d_xblocks_, xblocks_h_.data(), sizeof(kern::IpcBlock) * xblocks_h_.size(),
                       hipMemcpyHostToDevice));
  }
  ipc_final_ = true;
}

template <class T>
void CopyPlan::execute_ipc(Comm &comm, T *const *src_tab, T *const *dst_tab, hipStream_t st) {
  finalize_ipc(comm.ipc_block_elems());
  const size_t cap = comm.ipc_arena_bytes() / sizeof(T);
  for (auto &kv : send_cnt_)
    MGIC_CHECK((size_t)kv.second <= cap, "exchange message exceeds the transport arena "
                                         "(raise MGIC_IPC_ARENA_MB)");
  kern::IpcPeers pput{}, pget{};
  pput.n = (int)send_peers_.size();
  pput.err = pget.err = comm.ipc_err();
  pput.timeout = pget.timeout = comm.ipc_timeout_ticks();
  for (int q = 0; q < pput.n; ++q)
    comm.ipc_send(send_peers_[q], send_blocks_[q], pput, q);
  pget.n = (int)recv_peers_.size();
  for (int q = 0; q < pget.n; ++q)
    comm.ipc_recv(recv_peers_[q], pget, q);
  if constexpr (std::is_same<T, double>::value)
    kern::ipc_exchange(d_ipc_pack_, d_local_, d_ipc_unpack_, d_xblocks_, n_put_blocks_,
                       n_loc_blocks_, n_get_blocks_, src_tab, dst_tab, pput,
                       pget, comm.ipc_grid_cap(), st);
  else
    kern::ipc_exchange_f(d_ipc_pack_, d_local_, d_ipc_unpack_, d_xblocks_, n_put_blocks_,
                         n_loc_blocks_, n_get_blocks_, src_tab, dst_tab, pput,
                         pget, comm.ipc_grid_cap(), st);
}

void CopyPlan::execute(Comm &comm, double *const *src_tab, double *const *dst_tab,
                       hipStream_t st) {
  const bool remote = send_total_ || recv_total_;
  if (remote) comm.count_exchange();
  if (remote && comm.uses_ipc()) {  // local copies included: one launch
    execute_ipc<double>(comm, src_tab, dst_tab, st);
    return;
  }
  if (!local_.empty())
    kern::copy_items(d_local_, (int)local_.size(), max_local_, src_tab, nullptr, dst_tab, nullptr, st);
  if (!remote) return;
  MGIC_CHECK(comm.remote_ok(), "remote copies need an RCCL communicator or the peer-mapped transport");
  alloc_buffers();
  if (!pack_.empty())
    kern::copy_items(d_pack_, (int)pack_.size(), max_pack_, src_tab, nullptr, nullptr, sendbuf_, st);
  MGIC_NCCL(ncclGroupStart());
  for (auto &kv : send_cnt_)
    MGIC_NCCL(ncclSend(sendbuf_ + send_off_[kv.first], (size_t)kv.second, ncclDouble, kv.first,
                       comm.nccl(), st));
  for (auto &kv : recv_cnt_)
    MGIC_NCCL(ncclRecv(recvbuf_ + recv_off_[kv.first], (size_t)kv.second, ncclDouble, kv.first,
                       comm.nccl(), st));
  MGIC_NCCL(ncclGroupEnd());
  if (!unpack_.empty())
    kern::copy_items(d_unpack_, (int)unpack_.size(), max_unpack_, nullptr, recvbuf_, dst_tab,
                     nullptr, st);
}

void CopyPlan::execute_f(Comm &comm, float *const *src_tab, float *const *dst_tab,
                         hipStream_t st) {
  const bool remote = send_total_ || recv_total_;
  if (remote) comm.count_exchange();
  if (remote && comm.uses_ipc()) {  // local copies included: one launch
    execute_ipc<float>(comm, src_tab, dst_tab, st);
    return;
  }
  if (!local_.empty())
    kern::copy_items_f(d_local_, (int)local_.size(), max_local_, src_tab, nullptr, dst_tab, nullptr, st);
  if (!remote) return;
  MGIC_CHECK(comm.remote_ok(), "remote copies need an RCCL communicator or the peer-mapped transport");
  alloc_buffers();
  float *sb = reinterpret_cast<float *>(sendbuf_), *rb = reinterpret_cast<float *>(recvbuf_);
  if (!pack_.empty())
    kern::copy_items_f(d_pack_, (int)pack_.size(), max_pack_, src_tab, nullptr, nullptr, sb, st);
  MGIC_NCCL(ncclGroupStart());
  for (auto &kv : send_cnt_)
    MGIC_NCCL(ncclSend(sb + send_off_[kv.first], (size_t)kv.second, ncclFloat, kv.first,
                       comm.nccl(), st));
  for (auto &kv : recv_cnt_)
    MGIC_NCCL(ncclRecv(rb + recv_off_[kv.first], (size_t)kv.second, ncclFloat, kv.first,
                       comm.nccl(), st));
  MGIC_NCCL(ncclGroupEnd());
  if (!unpack_.empty())
    kern::copy_items_f(d_unpack_, (int)unpack_.size(), max_unpack_, nullptr, rb, dst_tab,
                       nullptr, st);
}

void CopyPlan::alloc_buffers() {  // RCCL staging buffers, on first use
  if (send_total_ && !sendbuf_) MGIC_HIP(hipMalloc(&sendbuf_, sizeof(double) * (size_t)send_total_));
  if (recv_total_ && !recvbuf_) MGIC_HIP(hipMalloc(&recvbuf_, sizeof(double) * (size_t)recv_total_));
}

// ------------------------------------------------------------------ LevelData
LevelData::LevelData(std::shared_ptr<Grid> g) : grid(std::move(g)) {
  const int n = grid->nlocal();
  base.resize(n, nullptr);
  p.resize(n, nullptr);
  for (int i = 0; i < n; ++i) {
    const FabGeom &fg = grid->geom[i];
    MGIC_HIP(hipMalloc(&base[i], sizeof(double) * (size_t)fg.total));
    MGIC_HIP(hipMemset(base[i], 0, sizeof(double) * (size_t)fg.total));
    p[i] = base[i] + fg.origin;
  }
  MGIC_HIP(hipMalloc(&d_tab, sizeof(double *) * (size_t)std::max(n, 1)));
  if (n) MGIC_HIP(hipMemcpy(d_tab, p.data(), sizeof(double *) * (size_t)n, hipMemcpyHostToDevice));
}

LevelData::~LevelData() {
  for (double *b : base)
    if (b) (void)hipFree(b);
  if (d_tab) (void)hipFree(d_tab);
}

void LevelData::set_zero_all(hipStream_t st) {
  for (int i = 0; i < (int)base.size(); ++i)
    MGIC_HIP(hipMemsetAsync(base[i], 0, sizeof(double) * (size_t)grid->geom[i].total, st));
}

void LevelData::exchange(hipStream_t st) {
  CopyPlan &pl = grid->exchange_plan();
  if (pl.empty()) return;
  pl.execute(*grid->comm, d_tab, d_tab, st);
}

void LevelData::exchange_shell(hipStream_t st, int depth) {
  CopyPlan &pl = grid->shell_plan(depth);
  if (pl.empty()) return;
  pl.execute(*grid->comm, d_tab, d_tab, st);
}

// ------------------------------------------------------------------ LevelDataF
LevelDataF::LevelDataF(std::shared_ptr<Grid> g) : grid(std::move(g)) {
  const int n = grid->nlocal();
  base.resize(n, nullptr);
  p.resize(n, nullptr);
  for (int i = 0; i < n; ++i) {
    const FabGeom &fg = grid->geom[i];
    MGIC_HIP(hipMalloc(&base[i], sizeof(float) * (size_t)fg.total));
    MGIC_HIP(hipMemset(base[i], 0, sizeof(float) * (size_t)fg.total));
    p[i] = base[i] + fg.origin;
  }
  MGIC_HIP(hipMalloc(&d_tab, sizeof(float *) * (size_t)std::max(n, 1)));
  if (n) MGIC_HIP(hipMemcpy(d_tab, p.data(), sizeof(float *) * (size_t)n, hipMemcpyHostToDevice));
}

LevelDataF::~LevelDataF() {
  for (float *b : base)
    if (b) (void)hipFree(b);
  if (d_tab) (void)hipFree(d_tab);
}

void LevelDataF::exchange(hipStream_t st) {
  CopyPlan &pl = grid->exchange_plan();
  if (pl.empty()) return;
  pl.execute_f(*grid->comm, d_tab, d_tab, st);
}

void LevelDataF::exchange_shell(hipStream_t st, int depth) {
  CopyPlan &pl = grid->shell_plan(depth);
  if (pl.empty()) return;
  pl.execute_f(*grid->comm, d_tab, d_tab, st);
}

}  // namespace mgic
