// capi.cpp -- extern "C" boundary (include/mgic.h) over the C++ layer.
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>

#include "../../include/mgic.h"
#include "amr.hpp"
#include "mixed.hpp"
#include "op.hpp"

using namespace mgic;

struct mgic_comm_s {
  std::shared_ptr<Comm> c;
};
struct mgic_grid_s {
  std::shared_ptr<Grid> g;
};
struct mgic_field_s {
  std::shared_ptr<LevelData> f;
};
struct mgic_factory_s {
  VariableCoeffPoissonOperatorFactory f;
};
struct mgic_op_s {
  std::unique_ptr<VariableCoeffPoissonOperator> owned;
  VariableCoeffPoissonOperator *op = nullptr;
};
struct mgic_mg_s {
  AMRMultiGrid amg;
};
struct mgic_amr_s {
  AMRSolver amr;
};
struct mgic_mixed_s {
  MixedMultiGrid mm;
};
struct mgic_plan_s {
  std::shared_ptr<Grid> src, dst;
  std::unique_ptr<CopyPlan> plan;
};

namespace {
thread_local std::string g_err;

template <class F>
int guard(F &&f) {
  try {
    f();
    return MGIC_OK;
  } catch (const Error &e) {
    g_err = e.what();
    return e.code;
  } catch (const std::exception &e) {
    g_err = e.what();
    return MGIC_EUNKNOWN;
  } catch (...) {
    g_err = "unknown exception";
    return MGIC_EUNKNOWN;
  }
}

#define NEED(p) MGIC_CHECK((p) != nullptr, "null argument: " #p)

OpParams to_op(const mgic_op_params *p) {
  OpParams o;
  if (!p) return o;
  o.alpha = p->alpha;
  o.beta = p->beta;
  for (int d = 0; d < 3; ++d) {
    o.bc_lo[d] = p->bc_lo[d];
    o.bc_hi[d] = p->bc_hi[d];
  }
  o.bc_value = p->bc_value;
  o.coefficient_average_type = p->coefficient_average_type;
  o.prolong_type = p->prolong_type;
  o.relax_mode = p->relax_mode;
  o.fused_smoother = p->fused_smoother;
  o.deep_halo = p->deep_halo;
  return o;
}

MGParams to_mg(const mgic_mg_params *p) {
  MGParams m;
  if (!p) return m;
  m.max_depth = p->max_depth;
  m.n_pre = p->n_pre;
  m.n_post = p->n_post;
  m.n_bottom = p->n_bottom;
  m.bottom_solver = p->bottom_solver;
  m.cycles = p->cycles;
  m.agglomerate_below = p->agglomerate_below;
  m.bicg.imax = p->bicg_imax;
  m.bicg.eps = p->bicg_eps;
  m.bicg.reps = p->bicg_reps;
  m.bicg.small = p->bicg_small;
  m.bicg.numRestarts = p->bicg_restarts;
  m.bicg.normType = p->bicg_norm_type;
  return m;
}

// host contiguous <-> fab region copy through a device staging buffer
void box_transfer(LevelData &f, int n, double *host, bool upload, bool with_ghosts) {
  MGIC_CHECK(n >= 0 && n < f.grid->nlocal(), "bad local box index");
  const FabGeom &g = f.grid->geom[n];
  Box R = g.valid;
  if (with_ghosts)
    for (int d = 0; d < 3; ++d) {
      R.lo[d] -= 1;
      R.hi[d] += 1;
    }
  const long nc = R.ncells();
  const hipStream_t st = f.grid->comm->stream();
  double *dbuf = nullptr;
  CopyItem *ditem = nullptr;
  MGIC_HIP(hipMalloc(&dbuf, sizeof(double) * (size_t)nc));
  MGIC_HIP(hipMalloc(&ditem, sizeof(CopyItem)));
  CopyItem it{};
  it.nx = R.size(0);
  it.ny = R.size(1);
  it.nz = R.size(2);
  const long off = g.offset(R.lo[0], R.lo[1], R.lo[2]);
  if (upload) {
    it.src = -1;
    it.soff = 0;
    it.ssy = it.nx;
    it.ssz = (long)it.nx * it.ny;
    it.dst = n;
    it.doff = off;
    it.dsy = g.sy;
    it.dsz = g.sz;
  } else {
    it.dst = -1;
    it.doff = 0;
    it.dsy = it.nx;
    it.dsz = (long)it.nx * it.ny;
    it.src = n;
    it.soff = off;
    it.ssy = g.sy;
    it.ssz = g.sz;
  }
  try {
    MGIC_HIP(hipStreamSynchronize(st));
    MGIC_HIP(hipMemcpy(ditem, &it, sizeof(CopyItem), hipMemcpyHostToDevice));
    if (upload) {
      MGIC_HIP(hipMemcpy(dbuf, host, sizeof(double) * (size_t)nc, hipMemcpyHostToDevice));
      kern::copy_items(ditem, 1, nc, nullptr, dbuf, f.d_tab, nullptr, st);
      MGIC_HIP(hipStreamSynchronize(st));
    } else {
      kern::copy_items(ditem, 1, nc, f.d_tab, nullptr, nullptr, dbuf, st);
      MGIC_HIP(hipStreamSynchronize(st));
      MGIC_HIP(hipMemcpy(host, dbuf, sizeof(double) * (size_t)nc, hipMemcpyDeviceToHost));
    }
  } catch (...) {
    (void)hipFree(dbuf);
    (void)hipFree(ditem);
    throw;
  }
  MGIC_HIP(hipFree(dbuf));
  MGIC_HIP(hipFree(ditem));
}

mgic_field borrowed_field(LevelData *ld) {
  auto *h = new mgic_field_s;
  h->f = std::shared_ptr<LevelData>(ld, [](LevelData *) {});
  return h;
}
}  // namespace

extern "C" {

// 0.2.0 (round 5): mgic_op_params lost overlap_exchange and mgic_mg_params
// lost fused_residual in round 4 (struct layouts changed); agglomerated
// depths run on their owner rank only; mgic_abi_version added
MGIC_API const char *mgic_version(void) { return "mgic 0.2.0 (gfx950, fp64 + fp32 mixed)"; }
MGIC_API int mgic_abi_version(void) { return MGIC_ABI_VERSION; }
MGIC_API const char *mgic_last_error(void) { return g_err.c_str(); }

MGIC_API int mgic_set_device(int device) {
  return guard([&] { MGIC_HIP(hipSetDevice(device)); });
}
MGIC_API int mgic_get_device_count(int *count) {
  return guard([&] {
    NEED(count);
    MGIC_HIP(hipGetDeviceCount(count));
  });
}
MGIC_API int mgic_device_synchronize(void) {
  return guard([&] { MGIC_HIP(hipDeviceSynchronize()); });
}

MGIC_API void mgic_op_params_default(mgic_op_params *p) {
  if (!p) return;
  OpParams o;
  p->alpha = o.alpha;
  p->beta = o.beta;
  for (int d = 0; d < 3; ++d) {
    p->bc_lo[d] = o.bc_lo[d];
    p->bc_hi[d] = o.bc_hi[d];
  }
  p->bc_value = o.bc_value;
  p->coefficient_average_type = o.coefficient_average_type;
  p->prolong_type = o.prolong_type;
  p->relax_mode = o.relax_mode;
  p->fused_smoother = o.fused_smoother;
  p->deep_halo = o.deep_halo;
}

MGIC_API void mgic_mg_params_default(mgic_mg_params *p) {
  if (!p) return;
  MGParams m;
  p->max_depth = m.max_depth;
  p->n_pre = m.n_pre;
  p->n_post = m.n_post;
  p->n_bottom = m.n_bottom;
  p->bottom_solver = m.bottom_solver;
  p->cycles = m.cycles;
  p->agglomerate_below = m.agglomerate_below;
  p->bicg_imax = m.bicg.imax;
  p->bicg_eps = m.bicg.eps;
  p->bicg_reps = m.bicg.reps;
  p->bicg_small = m.bicg.small;
  p->bicg_restarts = m.bicg.numRestarts;
  p->bicg_norm_type = m.bicg.normType;
}

// ---------------------------------------------------------------- comm
MGIC_API int mgic_comm_unique_id(unsigned char id[MGIC_UNIQUE_ID_BYTES]) {
  return guard([&] {
    NEED(id);
    static_assert(sizeof(ncclUniqueId) == MGIC_UNIQUE_ID_BYTES, "unique id size");
    ncclUniqueId uid;
    MGIC_NCCL(ncclGetUniqueId(&uid));
    std::memcpy(id, &uid, sizeof(uid));
  });
}

MGIC_API int mgic_comm_create(int rank, int size, const unsigned char *id, int force_rccl,
                              mgic_comm *out) {
  return guard([&] {
    NEED(out);
    ncclUniqueId uid;
    const ncclUniqueId *pid = nullptr;
    if (id) {
      std::memcpy(&uid, id, sizeof(uid));
      pid = &uid;
    }
    auto *h = new mgic_comm_s;
    try {
      h->c = std::make_shared<Comm>(rank, size, pid, force_rccl != 0);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}
MGIC_API int mgic_comm_create_ipc(int rank, int size, mgic_allgather_fn allgather, void *user,
                                  size_t arena_bytes, mgic_comm *out) {
  return guard([&] {
    NEED(out);
    auto *h = new mgic_comm_s;
    try {
      h->c = std::make_shared<Comm>(rank, size, allgather, user, arena_bytes);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}
MGIC_API int mgic_comm_transport(mgic_comm c, int *transport) {
  return guard([&] {
    NEED(c);
    NEED(transport);
    *transport = c->c->uses_ipc() ? 2 : c->c->uses_rccl() ? 1 : 0;
  });
}
MGIC_API int mgic_comm_destroy(mgic_comm c) {
  return guard([&] { delete c; });
}
MGIC_API int mgic_comm_set_stream(mgic_comm c, void *s) {
  return guard([&] {
    NEED(c);
    c->c->set_stream((hipStream_t)s);
  });
}
MGIC_API int mgic_comm_get_stream(mgic_comm c, void **s) {
  return guard([&] {
    NEED(c);
    NEED(s);
    *s = (void *)c->c->stream();
  });
}
MGIC_API int mgic_comm_set_self_messages(mgic_comm c, int on) {
  return guard([&] {
    NEED(c);
    c->c->set_self_messages(on != 0);
  });
}
MGIC_API int mgic_comm_exchanges(mgic_comm c, unsigned long long *count) {
  return guard([&] {
    NEED(c);
    NEED(count);
    *count = c->c->exchanges();
  });
}
MGIC_API int mgic_comm_synchronize(mgic_comm c) {
  return guard([&] {
    NEED(c);
    MGIC_HIP(hipStreamSynchronize(c->c->stream()));
    c->c->ipc_check();
  });
}
MGIC_API int mgic_comm_rank(mgic_comm c, int *rank, int *size, int *uses_rccl) {
  return guard([&] {
    NEED(c);
    if (rank) *rank = c->c->rank();
    if (size) *size = c->c->size();
    if (uses_rccl) *uses_rccl = c->c->uses_rccl();
  });
}

// ---------------------------------------------------------------- grid
MGIC_API int mgic_grid_create(mgic_comm c, const int domain[6], const int periodic[3], double dx,
                              int nbox, const int *boxes, const int *owners, mgic_grid *out) {
  return guard([&] {
    NEED(c);
    NEED(domain);
    NEED(boxes);
    NEED(out);
    MGIC_CHECK(nbox >= 1, "nbox must be >= 1");
    MGIC_CHECK(dx > 0.0, "dx must be positive");
    bool per[3] = {false, false, false};
    if (periodic)
      for (int d = 0; d < 3; ++d) per[d] = periodic[d] != 0;
    std::vector<Box> bx;
    std::vector<int> own;
    for (int b = 0; b < nbox; ++b) {
      bx.push_back(Box::make(boxes + 6 * b));
      own.push_back(owners ? owners[b] : 0);
    }
    auto g = std::make_shared<Grid>(c->c, Box::make(domain), per, dx, bx, own);
    MGIC_CHECK(g->tiles_domain(), "boxes must be disjoint and tile the domain");
    *out = new mgic_grid_s{g};
  });
}
MGIC_API int mgic_plan_create(int rank, int size, const int domain[6], const int periodic[3],
                              int nsrc, const int *src_boxes, const int *src_owners, int ndst,
                              const int *dst_boxes, const int *dst_owners, int with_valid,
                              int with_faces, mgic_plan *out) {
  return guard([&] {
    NEED(domain);
    NEED(src_boxes);
    NEED(src_owners);
    NEED(dst_boxes);
    NEED(dst_owners);
    NEED(out);
    MGIC_CHECK(nsrc >= 1 && ndst >= 1, "empty layout");
    bool per[3] = {false, false, false};
    if (periodic)
      for (int d = 0; d < 3; ++d) per[d] = periodic[d] != 0;
    auto comm = Comm::host_only(rank, size);
    auto layout = [&](int nb, const int *bx, const int *own) {
      std::vector<Box> b;
      std::vector<int> o;
      for (int i = 0; i < nb; ++i) {
        b.push_back(Box::make(bx + 6 * i));
        o.push_back(own[i]);
      }
      return std::make_shared<Grid>(comm, Box::make(domain), per, 1.0, b, o);
    };
    auto p = std::make_unique<mgic_plan_s>();
    p->src = layout(nsrc, src_boxes, src_owners);
    p->dst = layout(ndst, dst_boxes, dst_owners);
    p->plan = build_copy_plan(*p->src, *p->dst, with_valid != 0, with_faces != 0, false);
    *out = p.release();
  });
}
MGIC_API int mgic_plan_create_shell(int rank, int size, const int domain[6],
                                    const int periodic[3], int nboxes, const int *boxes,
                                    const int *owners, int depth, mgic_plan *out) {
  return guard([&] {
    NEED(domain);
    NEED(boxes);
    NEED(owners);
    NEED(out);
    MGIC_CHECK(nboxes >= 1, "empty layout");
    MGIC_CHECK(depth >= 1 && depth <= kGhost, "shell depth exceeds the allocated ghosts");
    bool per[3] = {false, false, false};
    if (periodic)
      for (int d = 0; d < 3; ++d) per[d] = periodic[d] != 0;
    auto comm = Comm::host_only(rank, size);
    std::vector<Box> b;
    std::vector<int> o;
    for (int i = 0; i < nboxes; ++i) {
      b.push_back(Box::make(boxes + 6 * i));
      o.push_back(owners[i]);
    }
    auto p = std::make_unique<mgic_plan_s>();
    p->src = std::make_shared<Grid>(comm, Box::make(domain), per, 1.0, b, o);
    p->dst = p->src;
    p->plan = build_copy_plan(*p->src, *p->dst, false, false, false, depth);
    *out = p.release();
  });
}
MGIC_API int mgic_plan_check_transport(mgic_plan p, int transport) {
  return guard([&] {
    NEED(p);
    MGIC_CHECK(transport == 1 || transport == 2, "transport: 1 RCCL, 2 peer-mapped");
    if (transport == 2) p->plan->finalize_ipc_host(kern::kIpcBlockElemsDefault);
    else p->plan->finalize_host();
  });
}
MGIC_API int mgic_plan_destroy(mgic_plan p) {
  return guard([&] { delete p; });
}
MGIC_API int mgic_plan_sizes(mgic_plan p, int *n_local, int *n_pack, int *n_unpack, int *n_peers) {
  return guard([&] {
    NEED(p);
    std::map<int, int> peers;
    for (auto &kv : p->plan->send_cnt_) peers[kv.first] = 1;
    for (auto &kv : p->plan->recv_cnt_) peers[kv.first] = 1;
    if (n_local) *n_local = (int)p->plan->local_.size();
    if (n_pack) *n_pack = (int)p->plan->pack_.size();
    if (n_unpack) *n_unpack = (int)p->plan->unpack_.size();
    if (n_peers) *n_peers = (int)peers.size();
  });
}
MGIC_API int mgic_plan_ipc_blocks(mgic_plan p, int *n, long long *rows) {
  return mgic_plan_ipc_blocks_per(p, kern::kIpcBlockElemsDefault, n, rows);
}
MGIC_API int mgic_plan_ipc_blocks_per(mgic_plan p, long long block_elems, int *n,
                                      long long *rows) {
  return guard([&] {
    NEED(p);
    NEED(n);
    MGIC_CHECK(block_elems >= 512 && block_elems <= (1 << 20) && block_elems % 512 == 0,
               "block_elems must be a multiple of 512 in [512, 2^20]");
    p->plan->finalize_ipc_host((long)block_elems);
    const auto r = p->plan->ipc_block_rows();
    *n = (int)r.size();
    if (rows)
      for (size_t i = 0; i < r.size(); ++i)
        for (int c = 0; c < 5; ++c) rows[5 * i + c] = r[i][c];
  });
}

MGIC_API int mgic_plan_items(mgic_plan p, int which, long long *items) {
  return guard([&] {
    NEED(p);
    NEED(items);
    MGIC_CHECK(which >= 0 && which <= 2, "which must be 0 (local), 1 (pack) or 2 (unpack)");
    const auto &v = which == 0 ? p->plan->local_ : which == 1 ? p->plan->pack_ : p->plan->unpack_;
    for (size_t i = 0; i < v.size(); ++i) {
      const CopyItem &c = v[i];
      const long long row[12] = {c.src, c.dst, c.soff, c.doff, c.ssy, c.ssz,
                                 c.dsy, c.dsz, c.nx,   c.ny,   c.nz,  which == 0 ? -1 : c.pad};
      std::memcpy(items + 12 * i, row, sizeof(row));
    }
  });
}
MGIC_API int mgic_plan_peers(mgic_plan p, int *peers, long long *send_cnt, long long *send_off,
                             long long *recv_cnt, long long *recv_off) {
  return guard([&] {
    NEED(p);
    NEED(peers);
    std::map<int, int> all;
    for (auto &kv : p->plan->send_cnt_) all[kv.first] = 1;
    for (auto &kv : p->plan->recv_cnt_) all[kv.first] = 1;
    int i = 0;
    for (auto &kv : all) {
      const int r = kv.first;
      auto get = [r](const std::map<int, long> &m) {
        auto it = m.find(r);
        return it == m.end() ? 0LL : (long long)it->second;
      };
      peers[i] = r;
      if (send_cnt) send_cnt[i] = get(p->plan->send_cnt_);
      if (send_off) send_off[i] = get(p->plan->send_off_);
      if (recv_cnt) recv_cnt[i] = get(p->plan->recv_cnt_);
      if (recv_off) recv_off[i] = get(p->plan->recv_off_);
      ++i;
    }
  });
}
MGIC_API int mgic_plan_geom(mgic_plan p, int layout, int n, long long geom[4]) {
  return guard([&] {
    NEED(p);
    NEED(geom);
    const Grid &g = layout == 0 ? *p->src : *p->dst;
    MGIC_CHECK(n >= 0 && n < g.nlocal(), "local box index out of range");
    const FabGeom &f = g.geom[n];
    geom[0] = f.sy;
    geom[1] = f.sz;
    geom[2] = f.origin;
    geom[3] = f.total;
  });
}
MGIC_API int mgic_grid_destroy(mgic_grid g) {
  return guard([&] { delete g; });
}
MGIC_API int mgic_grid_num_local(mgic_grid g, int *n) {
  return guard([&] {
    NEED(g);
    NEED(n);
    *n = g->g->nlocal();
  });
}
MGIC_API int mgic_grid_local_box(mgic_grid g, int n, int lohi[6], int *gi) {
  return guard([&] {
    NEED(g);
    NEED(lohi);
    MGIC_CHECK(n >= 0 && n < g->g->nlocal(), "bad local box index");
    const Box &b = g->g->geom[n].valid;
    for (int d = 0; d < 3; ++d) {
      lohi[d] = b.lo[d];
      lohi[3 + d] = b.hi[d];
    }
    if (gi) *gi = g->g->local[n];
  });
}
MGIC_API int mgic_grid_coarsen(mgic_grid g, int ratio, mgic_grid *out) {
  return guard([&] {
    NEED(g);
    NEED(out);
    MGIC_CHECK(ratio >= 1 && g->g->coarsenable(ratio), "grid not coarsenable by ratio");
    *out = new mgic_grid_s{g->g->coarsened(ratio)};
  });
}

// ---------------------------------------------------------------- field
MGIC_API int mgic_field_create(mgic_grid g, mgic_field *out) {
  return guard([&] {
    NEED(g);
    NEED(out);
    *out = new mgic_field_s{std::make_shared<LevelData>(g->g)};
  });
}
MGIC_API int mgic_field_destroy(mgic_field f) {
  return guard([&] { delete f; });
}
MGIC_API int mgic_field_device_ptr(mgic_field f, int n, double **p, long strides[3]) {
  return guard([&] {
    NEED(f);
    MGIC_CHECK(n >= 0 && n < f->f->grid->nlocal(), "bad local box index");
    if (p) *p = f->f->p[n];
    if (strides) {
      strides[0] = 1;
      strides[1] = f->f->grid->geom[n].sy;
      strides[2] = f->f->grid->geom[n].sz;
    }
  });
}
MGIC_API int mgic_field_upload(mgic_field f, int n, const double *host, int with_ghosts) {
  return guard([&] {
    NEED(f);
    NEED(host);
    box_transfer(*f->f, n, const_cast<double *>(host), true, with_ghosts != 0);
  });
}
MGIC_API int mgic_field_download(mgic_field f, int n, double *host, int with_ghosts) {
  return guard([&] {
    NEED(f);
    NEED(host);
    box_transfer(*f->f, n, host, false, with_ghosts != 0);
  });
}
MGIC_API int mgic_field_set_val(mgic_field f, double v) {
  return guard([&] {
    NEED(f);
    LevelData &x = *f->f;
    for (int n = 0; n < x.grid->nlocal(); ++n)
      kern::blas(5, x.p[n], nullptr, nullptr, v, 0.0, x.grid->box_args_plain(n), x.grid->comm->stream());
  });
}
MGIC_API int mgic_field_set_zero(mgic_field f) {
  return guard([&] {
    NEED(f);
    f->f->set_zero_all(f->f->grid->comm->stream());
  });
}
MGIC_API int mgic_field_exchange(mgic_field f) {
  return guard([&] {
    NEED(f);
    f->f->exchange(f->f->grid->comm->stream());
  });
}
MGIC_API int mgic_field_copy_to(mgic_field src, mgic_field dst, int with_faces) {
  return guard([&] {
    NEED(src);
    NEED(dst);
    auto plan = build_copy_plan(*src->f->grid, *dst->f->grid, true, with_faces != 0);
    plan->execute(*dst->f->grid->comm, src->f->d_tab, dst->f->d_tab, dst->f->grid->comm->stream());
    MGIC_HIP(hipStreamSynchronize(dst->f->grid->comm->stream()));
  });
}
static kern::BhParams bh_params(const double bh[13]) {
  kern::BhParams p;
  for (int d = 0; d < 3; ++d) p.domlen[d] = bh[0];
  p.G_Newton = bh[1];
  p.phi_amplitude = bh[2];
  p.phi_wavelength = bh[3];
  p.m1 = bh[4];
  p.m2 = bh[5];
  p.spin1 = bh[6];
  p.spin2 = bh[7];
  p.off1 = bh[8];
  p.off2 = bh[9];
  p.mom1 = bh[10];
  p.mom2 = bh[11];
  p.constant_K = bh[12];
  return p;
}
MGIC_API int mgic_field_nl_coefs(mgic_field psi, mgic_field acoef, mgic_field rhs,
                                 const double bh[13]) {
  return guard([&] {
    NEED(acoef);
    NEED(rhs);
    NEED(bh);
    const Grid &g = *acoef->f->grid;
    if (psi) check_same_layout(g, *psi->f, "psi");
    check_same_layout(g, *rhs->f, "rhs");
    const kern::BhParams p = bh_params(bh);
    for (int n = 0; n < g.nlocal(); ++n)
      kern::binary_bh_coefs(acoef->f->p[n], rhs->f->p[n], psi ? psi->f->p[n] : nullptr,
                            g.box_args_plain(n), g.dx, p, g.comm->stream());
  });
}
MGIC_API int mgic_field_nl_integrand(mgic_field psi, mgic_field out, const double bh[13]) {
  return guard([&] {
    NEED(out);
    NEED(bh);
    const Grid &g = *out->f->grid;
    if (psi) check_same_layout(g, *psi->f, "psi");
    const kern::BhParams p = bh_params(bh);
    for (int n = 0; n < g.nlocal(); ++n)
      kern::constant_k_integrand(out->f->p[n], psi ? psi->f->p[n] : nullptr, g.box_args_plain(n),
                                 g.dx, p, g.comm->stream());
  });
}
// ---- output: WriteOutput.H's per-box components, and
// the layout queries the HDF5 writer (libmgic_io) needs
// a device staging buffer for results the caller wants on the host (grown on
// demand, freed at exit)
static void *scratch_device(size_t bytes) {
  struct Buf {
    void *p = nullptr;
    size_t n = 0;
    ~Buf() {
      if (p) (void)hipFree(p);
    }
  };
  static Buf b;
  if (bytes > b.n) {
    if (b.p) MGIC_HIP(hipFree(b.p));
    b.p = nullptr;
    b.n = 0;
    MGIC_HIP(hipMalloc(&b.p, bytes));
    b.n = bytes;
  }
  return b.p;
}
static void output_vars_capi(int kind, mgic_field psi, mgic_field dpsi, mgic_field rhs, int n,
                             int k0, int nk, const double bh[13], double *out, int on_device) {
  NEED(psi);
  NEED(bh);
  NEED(out);
  const LevelData &u = *psi->f;
  const Grid &g = *u.grid;
  if (kind == 1) {
    NEED(dpsi);
    NEED(rhs);
    check_same_layout(g, *dpsi->f, "dpsi");
    check_same_layout(g, *rhs->f, "rhs");
  }
  MGIC_CHECK(n >= 0 && n < g.nlocal(), "bad local box index");
  const FabGeom &fg = g.geom[n];
  MGIC_CHECK(k0 >= 0 && nk >= 1 && k0 + nk <= fg.nz, "plane range outside the box");
  const int nc = kind == 0 ? kern::kNumGRChomboVars : kern::kNumSolverVars;
  const size_t bytes = sizeof(double) * (size_t)nc * fg.nx * fg.ny * nk;
  const hipStream_t st = g.comm->stream();
  const BoxArgs a = g.box_args_plain(n);
  const kern::BhParams p = bh_params(bh);
  double *d = out;
  if (!on_device) d = static_cast<double *>(scratch_device(bytes));
  kern::output_vars(kind, d, u.p[n], kind ? dpsi->f->p[n] : nullptr, kind ? rhs->f->p[n] : nullptr,
                    a, k0, nk, g.dx, p, st);
  if (!on_device) {
    MGIC_HIP(hipMemcpyAsync(out, d, bytes, hipMemcpyDeviceToHost, st));
    MGIC_HIP(hipStreamSynchronize(st));
  }
}
MGIC_API int mgic_field_grchombo_vars(mgic_field psi, int n, int k0, int nk, const double bh[13],
                                      double *out, int out_on_device) {
  return guard([&] { output_vars_capi(0, psi, nullptr, nullptr, n, k0, nk, bh, out, out_on_device); });
}
MGIC_API int mgic_field_solver_vars(mgic_field dpsi, mgic_field rhs, mgic_field psi, int n, int k0,
                                    int nk, const double bh[13], double *out, int out_on_device) {
  return guard([&] { output_vars_capi(1, psi, dpsi, rhs, n, k0, nk, bh, out, out_on_device); });
}
MGIC_API int mgic_field_layout(mgic_field f, int domain[6], int periodic[3], double *dx, int *nbox,
                               int *rank, int *size) {
  return guard([&] {
    NEED(f);
    const Grid &g = *f->f->grid;
    for (int d = 0; d < 3; ++d) {
      if (domain) {
        domain[d] = g.domain.lo[d];
        domain[3 + d] = g.domain.hi[d];
      }
      if (periodic) periodic[d] = g.periodic[d] ? 1 : 0;
    }
    if (dx) *dx = g.dx;
    if (nbox) *nbox = (int)g.boxes.size();
    if (rank) *rank = g.comm->rank();
    if (size) *size = g.comm->size();
  });
}
MGIC_API int mgic_field_box(mgic_field f, int i, int lohi[6], int *owner, int *local_index) {
  return guard([&] {
    NEED(f);
    NEED(lohi);
    const Grid &g = *f->f->grid;
    MGIC_CHECK(i >= 0 && i < (int)g.boxes.size(), "bad box index");
    for (int d = 0; d < 3; ++d) {
      lohi[d] = g.boxes[i].lo[d];
      lohi[3 + d] = g.boxes[i].hi[d];
    }
    if (owner) *owner = g.owners[i];
    if (local_index) {
      *local_index = -1;
      for (int n = 0; n < g.nlocal(); ++n)
        if (g.local[n] == i) *local_index = n;
    }
  });
}
MGIC_API int mgic_field_barrier(mgic_field f) {
  return guard([&] {
    NEED(f);
    Comm &c = *f->f->grid->comm;
    c.allreduce(c.d_result(), 0);  // any collective orders the ranks
    MGIC_HIP(hipStreamSynchronize(c.stream()));
  });
}
MGIC_API int mgic_host_alloc(size_t bytes, void **out) {
  return guard([&] {
    NEED(out);
    *out = nullptr;
    MGIC_HIP(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
  });
}
MGIC_API int mgic_host_free(void *p) {
  return guard([&] {
    if (p) MGIC_HIP(hipHostFree(p));
  });
}
MGIC_API int mgic_field_binary_bh(mgic_field acoef, mgic_field rhs, const double bh[13]) {
  return mgic_field_nl_coefs(nullptr, acoef, rhs, bh);
}
MGIC_API int mgic_field_set_val_all(mgic_field f, double v) {
  return guard([&] {
    NEED(f);
    const Grid &g = *f->f->grid;
    for (int n = 0; n < g.nlocal(); ++n) {  // the valid box grown by every ghost layer
      BoxArgs a = g.box_args_plain(n);
      a.nx += 2 * kGhost;
      a.ny += 2 * kGhost;
      a.nz += 2 * kGhost;
      double *base = f->f->p[n] - kGhost * (1 + a.sy + a.sz);
      kern::blas(5, base, nullptr, nullptr, v, 0.0, a, g.comm->stream());
    }
  });
}

// ---------------------------------------------------------------- factory / op
MGIC_API int mgic_factory_define(mgic_grid g, const mgic_op_params *p, mgic_field a,
                                 mgic_field b, mgic_factory *out) {
  return guard([&] {
    NEED(g);
    NEED(a);
    NEED(b);
    NEED(out);
    auto *h = new mgic_factory_s;
    h->f.define(g->g, to_op(p), a->f, b->f);
    *out = h;
  });
}
MGIC_API int mgic_factory_destroy(mgic_factory f) {
  return guard([&] { delete f; });
}
MGIC_API int mgic_factory_mg_new_op(mgic_factory f, int depth, mgic_op *out) {
  int rc = 0;
  int st = guard([&] {
    NEED(f);
    NEED(out);
    MGIC_CHECK(depth >= 0, "depth must be >= 0");
    auto op = f->f.MGnewOp(depth);
    if (!op) {
      *out = nullptr;
      rc = 1;
      return;
    }
    auto *h = new mgic_op_s;
    h->op = op.get();
    h->owned = std::move(op);
    *out = h;
  });
  return st ? st : rc;
}
MGIC_API int mgic_factory_amr_new_op(mgic_factory f, mgic_op *out) {
  return guard([&] {
    NEED(f);
    NEED(out);
    auto *h = new mgic_op_s;
    h->owned = f->f.AMRnewOp();
    h->op = h->owned.get();
    *out = h;
  });
}
MGIC_API int mgic_factory_ref_to_finer(mgic_factory f, int *r) {
  return guard([&] {
    NEED(f);
    NEED(r);
    *r = f->f.refToFiner();
  });
}

#define OPGUARD(body)        \
  return guard([&] {         \
    NEED(op);                \
    VariableCoeffPoissonOperator &o = *op->op; \
    (void)o;                 \
    body;                    \
  })

MGIC_API int mgic_op_destroy(mgic_op op) {
  return guard([&] { delete op; });
}
MGIC_API int mgic_op_grid(mgic_op op, mgic_grid *out) {
  OPGUARD(NEED(out); *out = new mgic_grid_s{o.grid});
}
MGIC_API int mgic_op_coef(mgic_op op, int which, mgic_field *out) {
  OPGUARD({
    NEED(out);
    if (which == 0) *out = new mgic_field_s{o.m_aCoef};
    else if (which == 1) *out = new mgic_field_s{o.m_bCoef};
    else {
      o.resetLambda();
      MGIC_CHECK(o.m_lambda != nullptr, "lambda not defined");
      *out = borrowed_field(o.m_lambda.get());
    }
  });
}
MGIC_API int mgic_op_residual(mgic_op op, mgic_field lhs, mgic_field dpsi, mgic_field rhs, int h) {
  OPGUARD(NEED(lhs); NEED(dpsi); NEED(rhs); o.residualI(*lhs->f, *dpsi->f, *rhs->f, h != 0));
}
MGIC_API int mgic_op_apply_op(mgic_op op, mgic_field lhs, mgic_field dpsi, int h) {
  OPGUARD(NEED(lhs); NEED(dpsi); o.applyOpI(*lhs->f, *dpsi->f, h != 0));
}
MGIC_API int mgic_op_apply_op_no_boundary(mgic_op op, mgic_field lhs, mgic_field dpsi) {
  OPGUARD(NEED(lhs); NEED(dpsi); o.applyOpNoBoundary(*lhs->f, *dpsi->f));
}
MGIC_API int mgic_op_precond(mgic_op op, mgic_field cor, mgic_field res) {
  OPGUARD(NEED(cor); NEED(res); o.preCond(*cor->f, *res->f));
}
MGIC_API int mgic_op_relax(mgic_op op, mgic_field e, mgic_field r, int it) {
  OPGUARD(NEED(e); NEED(r); o.relax(*e->f, *r->f, it));
}
MGIC_API int mgic_op_level_gsrb(mgic_op op, mgic_field e, mgic_field r) {
  OPGUARD(NEED(e); NEED(r); o.levelGSRB(*e->f, *r->f));
}
MGIC_API int mgic_op_level_jacobi(mgic_op op, mgic_field e, mgic_field r) {
  OPGUARD(NEED(e); NEED(r); o.levelJacobi(*e->f, *r->f));
}
MGIC_API int mgic_op_restrict_residual(mgic_op op, mgic_field rc, mgic_field df, mgic_field rf) {
  OPGUARD(NEED(rc); NEED(df); NEED(rf); o.restrictResidual(*rc->f, *df->f, *rf->f));
}
MGIC_API int mgic_op_prolong_increment(mgic_op op, mgic_field phi, mgic_field cor) {
  OPGUARD(NEED(phi); NEED(cor); o.prolongIncrement(*phi->f, *cor->f));
}
MGIC_API int mgic_op_set_alpha_beta(mgic_op op, double a, double b) {
  OPGUARD(o.setAlphaAndBeta(a, b));
}
MGIC_API int mgic_op_set_coefs(mgic_op op, mgic_field a, mgic_field b, double alpha, double beta) {
  OPGUARD(NEED(a); NEED(b); o.setCoefs(a->f, b->f, alpha, beta));
}
MGIC_API int mgic_op_reset_lambda(mgic_op op) { OPGUARD(o.resetLambda()); }
MGIC_API int mgic_op_set_time(mgic_op op, double t) { OPGUARD(o.setTime(t)); }
MGIC_API int mgic_op_update_psi(mgic_op op, mgic_field psi, mgic_field dpsi) {
  return guard([&] {
    NEED(op);
    NEED(psi);
    NEED(dpsi);
    VariableCoeffPoissonOperator &o = *op->op;
    check_same_layout(*o.grid, *psi->f, "psi");
    check_same_layout(*o.grid, *dpsi->f, "dpsi");
    // set_update_psi0 (SetLevelData.cpp:236-256): dpsi ghosts from the
    // exchange (domain faces: the inhomogeneous BC image), psi += dpsi over
    // the valid cells and the ghost layer the stencils read
    dpsi->f->exchange(o.stream());
    o.fillBC(*dpsi->f, false);
    for (int n = 0; n < o.grid->nlocal(); ++n)
      kern::incr_grown(psi->f->p[n], dpsi->f->p[n], o.grid->box_args_plain(n), 1, o.stream());
  });
}
MGIC_API int mgic_op_fill_bc(mgic_op op, mgic_field u, int h) {
  OPGUARD(NEED(u); o.fillBC(*u->f, h != 0));
}
MGIC_API int mgic_op_set_to_zero(mgic_op op, mgic_field x) { OPGUARD(NEED(x); o.setToZero(*x->f)); }
MGIC_API int mgic_op_assign(mgic_op op, mgic_field l, mgic_field r) {
  OPGUARD(NEED(l); NEED(r); o.assignLocal(*l->f, *r->f));
}
MGIC_API int mgic_op_incr(mgic_op op, mgic_field l, mgic_field x, double s) {
  OPGUARD(NEED(l); NEED(x); o.incr(*l->f, *x->f, s));
}
MGIC_API int mgic_op_axby(mgic_op op, mgic_field l, mgic_field x, mgic_field y, double a, double b) {
  OPGUARD(NEED(l); NEED(x); NEED(y); o.axby(*l->f, *x->f, *y->f, a, b));
}
MGIC_API int mgic_op_scale(mgic_op op, mgic_field l, double s) { OPGUARD(NEED(l); o.scale(*l->f, s)); }
MGIC_API int mgic_op_dot(mgic_op op, mgic_field x, mgic_field y, double *out) {
  OPGUARD(NEED(x); NEED(y); NEED(out); *out = o.dotProduct(*x->f, *y->f));
}
MGIC_API int mgic_op_norm(mgic_op op, mgic_field x, int ord, double *out) {
  OPGUARD(NEED(x); NEED(out); *out = o.norm(*x->f, ord));
}
MGIC_API int mgic_op_bicgstab(mgic_op op, mgic_field phi, mgic_field rhs, int h,
                              const mgic_mg_params *p, int *iters) {
  OPGUARD({
    NEED(phi);
    NEED(rhs);
    BiCGStabSolver s;
    s.prm = to_mg(p).bicg;
    const int it = s.solve(o, *phi->f, *rhs->f, h != 0);
    if (iters) *iters = it;
  });
}

// ---------------------------------------------------------------- multigrid
MGIC_API int mgic_mg_create(mgic_factory f, const mgic_mg_params *p, mgic_mg *out) {
  return guard([&] {
    NEED(f);
    NEED(out);
    auto *h = new mgic_mg_s;
    try {
      h->amg.define(f->f, to_mg(p));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}
MGIC_API int mgic_mg_destroy(mgic_mg mg) {
  return guard([&] { delete mg; });
}
MGIC_API int mgic_mg_num_depths(mgic_mg mg, int *n) {
  return guard([&] {
    NEED(mg);
    NEED(n);
    *n = mg->amg.mg.depths();
  });
}
MGIC_API int mgic_mg_op(mgic_mg mg, int depth, mgic_op *out) {
  return guard([&] {
    NEED(mg);
    NEED(out);
    MGIC_CHECK(depth >= 0 && depth < mg->amg.mg.depths(), "bad depth");
    auto *h = new mgic_op_s;
    h->op = &mg->amg.mg.op(depth);
    *out = h;
  });
}
MGIC_API int mgic_mg_level_field(mgic_mg mg, int depth, int which, mgic_field *out) {
  return guard([&] {
    NEED(mg);
    NEED(out);
    MGIC_CHECK(depth >= 1 && depth < mg->amg.mg.depths(), "bad depth (internal fields exist for depth >= 1)");
    LevelData *ld = which == 0 ? mg->amg.mg.corr(depth) : mg->amg.mg.resid(depth);
    MGIC_CHECK(ld != nullptr, "field not allocated");
    *out = borrowed_field(ld);
  });
}
MGIC_API int mgic_mg_one_cycle(mgic_mg mg, mgic_field e, mgic_field r) {
  return guard([&] {
    NEED(mg);
    NEED(e);
    NEED(r);
    mg->amg.mg.oneCycle(*e->f, *r->f);
  });
}
MGIC_API int mgic_mg_iteration(mgic_mg mg, mgic_field phi, mgic_field rhs, mgic_field resid,
                               int norm_type, int h, double *norm) {
  return guard([&] {
    NEED(mg);
    NEED(phi);
    NEED(rhs);
    NEED(resid);
    const double v = mg->amg.iteration(*phi->f, *rhs->f, *resid->f, norm_type, h != 0);
    if (norm) *norm = v;
  });
}
MGIC_API int mgic_mg_iterations(mgic_mg mg, mgic_field phi, mgic_field rhs, mgic_field resid,
                                int count, int norm_type, int h, double *norms) {
  return guard([&] {
    NEED(mg);
    NEED(phi);
    NEED(rhs);
    NEED(resid);
    MGIC_CHECK(count >= 0, "count must be >= 0");
    mg->amg.iterations(*phi->f, *rhs->f, *resid->f, count, norm_type, h != 0, norms);
  });
}
MGIC_API int mgic_mg_init_residual(mgic_mg mg, mgic_field phi, mgic_field rhs, mgic_field resid,
                                   int norm_type, int h, double *norm) {
  return guard([&] {
    NEED(mg);
    NEED(phi);
    NEED(rhs);
    NEED(resid);
    const double v = mg->amg.initResidual(*phi->f, *rhs->f, *resid->f, norm_type, h != 0);
    if (norm) *norm = v;
  });
}

MGIC_API int mgic_mg_bottom_timer(mgic_mg mg, int on) {
  return guard([&] {
    NEED(mg);
    mg->amg.mg.bottom_timer(on != 0);
  });
}
MGIC_API int mgic_mg_bottom_ms(mgic_mg mg, double *ms, int *calls) {
  return guard([&] {
    NEED(mg);
    NEED(ms);
    *ms = mg->amg.mg.bottom_ms(calls);
  });
}
MGIC_API int mgic_mg_bottom_iters(mgic_mg mg, long long *iters, double *r0_min,
                                  double *r0_max) {
  return guard([&] {
    NEED(mg);
    NEED(iters);
    *iters = mg->amg.mg.bottom_iters(r0_min, r0_max);
  });
}
MGIC_API int mgic_mg_bottom_info(mgic_mg mg, int *device, int *iters, double *r0) {
  return guard([&] {
    NEED(mg);
    const BiCGStabSolver &b = mg->amg.mg.bottom;
    if (device) *device = b.last_device ? 1 : 0;
    if (iters) *iters = b.last_iters;
    if (r0) *r0 = b.last_init_norm;
  });
}
MGIC_API int mgic_mg_bottom_replay(mgic_mg mg, int n, double *ms, int *iters, double *r0,
                                   int *solves) {
  return guard([&] {
    NEED(mg);
    NEED(ms);
    NEED(iters);
    NEED(r0);
    MGIC_CHECK(n >= 0, "n must be >= 0");
    const int k = mg->amg.mg.bottom_replay(n, ms, iters, r0);
    if (solves) *solves = k;
  });
}
MGIC_API int mgic_mg_fmg(mgic_mg mg, mgic_field phi, mgic_field rhs, mgic_field resid,
                         int norm_type, int h, int ncycles, double *norm) {
  return guard([&] {
    NEED(mg);
    NEED(phi);
    NEED(rhs);
    NEED(resid);
    MGIC_CHECK(ncycles >= 1, "ncycles must be >= 1");
    const double v = mg->amg.fmg(*phi->f, *rhs->f, *resid->f, norm_type, h != 0, ncycles);
    if (norm) *norm = v;
  });
}

// ---------------------------------------------------------------- mixed precision
MGIC_API int mgic_mixed_create(mgic_factory f, const mgic_mg_params *p, mgic_mixed *out) {
  return guard([&] {
    NEED(f);
    NEED(out);
    auto *h = new mgic_mixed_s;
    try {
      h->mm.define(f->f, to_mg(p));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}
MGIC_API int mgic_mixed_destroy(mgic_mixed m) {
  return guard([&] { delete m; });
}
MGIC_API int mgic_mixed_num_depths(mgic_mixed m, int *n) {
  return guard([&] {
    NEED(m);
    NEED(n);
    *n = m->mm.depths();
  });
}
MGIC_API int mgic_mixed_init_residual(mgic_mixed m, mgic_field phi, mgic_field rhs,
                                      mgic_field resid, int norm_type, double *norm) {
  return guard([&] {
    NEED(m);
    NEED(phi);
    NEED(rhs);
    const double v = m->mm.initResidual(*phi->f, *rhs->f, resid ? resid->f.get() : nullptr, norm_type);
    if (norm) *norm = v;
  });
}
MGIC_API int mgic_mixed_iteration(mgic_mixed m, mgic_field phi, mgic_field rhs, mgic_field resid,
                                  int norm_type, double *norm) {
  return guard([&] {
    NEED(m);
    NEED(phi);
    NEED(rhs);
    const double v = m->mm.iteration(*phi->f, *rhs->f, resid ? resid->f.get() : nullptr, norm_type);
    if (norm) *norm = v;
  });
}
MGIC_API int mgic_mixed_fmg(mgic_mixed m, mgic_field phi, mgic_field rhs, mgic_field resid,
                            int norm_type, int ncycles, double *norm) {
  return guard([&] {
    NEED(m);
    NEED(phi);
    NEED(rhs);
    MGIC_CHECK(ncycles >= 1, "ncycles must be >= 1");
    const double v = m->mm.fmg(*phi->f, *rhs->f, resid ? resid->f.get() : nullptr, norm_type, ncycles);
    if (norm) *norm = v;
  });
}

// ---------------------------------------------------------------- AMR levels
MGIC_API int mgic_grid_create_patches(mgic_comm c, const int domain[6], const int periodic[3],
                                      double dx, int nbox, const int *boxes, const int *owners,
                                      mgic_grid *out) {
  return guard([&] {
    NEED(c);
    NEED(domain);
    NEED(boxes);
    NEED(out);
    MGIC_CHECK(nbox >= 1, "nbox must be >= 1");
    MGIC_CHECK(dx > 0.0, "dx must be positive");
    bool per[3] = {false, false, false};
    if (periodic)
      for (int d = 0; d < 3; ++d) per[d] = periodic[d] != 0;
    const Box dom = Box::make(domain);
    std::vector<Box> bx;
    std::vector<int> own;
    for (int b = 0; b < nbox; ++b) {
      bx.push_back(Box::make(boxes + 6 * b));
      MGIC_CHECK(!bx.back().empty() && dom.contains(bx.back()), "patch boxes must lie in the domain");
      own.push_back(owners ? owners[b] : 0);
    }
    for (int a = 0; a < nbox; ++a)
      for (int b = a + 1; b < nbox; ++b)
        MGIC_CHECK(bx[a].intersect(bx[b]).empty(), "patch boxes must be disjoint");
    *out = new mgic_grid_s{std::make_shared<Grid>(c->c, dom, per, dx, bx, own)};
  });
}

MGIC_API int mgic_amr_create(int nlevels, const mgic_grid *grids, const mgic_field *acoef,
                             const mgic_field *bcoef, const mgic_op_params *op,
                             const mgic_mg_params *base, mgic_amr *out) {
  return guard([&] {
    NEED(grids);
    NEED(acoef);
    NEED(bcoef);
    NEED(out);
    MGIC_CHECK(nlevels >= 1, "nlevels must be >= 1");
    std::vector<AMRLevelSpec> lv;
    for (int l = 0; l < nlevels; ++l) {
      NEED(grids[l]);
      NEED(acoef[l]);
      NEED(bcoef[l]);
      lv.push_back({grids[l]->g, acoef[l]->f, bcoef[l]->f});
    }
    auto *h = new mgic_amr_s;
    try {
      h->amr.define(lv, to_op(op), to_mg(base));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}
MGIC_API int mgic_amr_destroy(mgic_amr a) {
  return guard([&] { delete a; });
}
MGIC_API int mgic_amr_num_levels(mgic_amr a, int *n) {
  return guard([&] {
    NEED(a);
    NEED(n);
    *n = a->amr.numLevels();
  });
}
static void amr_level(mgic_amr a, int l, int lo) {
  MGIC_CHECK(l >= lo && l < a->amr.numLevels(), "bad AMR level");
}
MGIC_API int mgic_amr_level_op(mgic_amr a, int level, mgic_op *out) {
  return guard([&] {
    NEED(a);
    NEED(out);
    amr_level(a, level, 0);
    auto *h = new mgic_op_s;
    h->op = &a->amr.op(level);
    *out = h;
  });
}
MGIC_API int mgic_amr_cf_interp(mgic_amr a, int level, mgic_field u, mgic_field coarse) {
  return guard([&] {
    NEED(a);
    NEED(u);
    amr_level(a, level, 1);
    a->amr.cf(level).interp(*u->f, coarse ? coarse->f.get() : nullptr, a->amr.op(level).stream());
  });
}
MGIC_API int mgic_amr_average_down(mgic_amr a, int level, mgic_field coarse, mgic_field fine) {
  return guard([&] {
    NEED(a);
    NEED(coarse);
    NEED(fine);
    amr_level(a, level, 1);
    a->amr.cf(level).averageDown(*coarse->f, *fine->f, a->amr.op(level).stream());
  });
}
MGIC_API int mgic_amr_operator(mgic_amr a, int level, mgic_field lphi, mgic_field phi,
                               mgic_field phi_coarse, int h) {
  return guard([&] {
    NEED(a);
    NEED(lphi);
    NEED(phi);
    amr_level(a, level, 0);
    a->amr.AMROperator(level, *lphi->f, *phi->f, phi_coarse ? phi_coarse->f.get() : nullptr, h != 0);
  });
}
MGIC_API int mgic_amr_residual(mgic_amr a, int level, mgic_field r, mgic_field phi,
                               mgic_field phi_coarse, mgic_field rhs, int h) {
  return guard([&] {
    NEED(a);
    NEED(r);
    NEED(phi);
    NEED(rhs);
    amr_level(a, level, 0);
    a->amr.AMRResidual(level, *r->f, *phi->f, phi_coarse ? phi_coarse->f.get() : nullptr, *rhs->f,
                       h != 0);
  });
}
MGIC_API int mgic_amr_restrict(mgic_amr a, int level, mgic_field res_coarse, mgic_field res,
                               mgic_field corr, mgic_field corr_coarse) {
  return guard([&] {
    NEED(a);
    NEED(res_coarse);
    NEED(res);
    NEED(corr);
    amr_level(a, level, 1);
    a->amr.AMRRestrict(level, *res_coarse->f, *res->f, *corr->f,
                       corr_coarse ? corr_coarse->f.get() : nullptr);
  });
}
MGIC_API int mgic_amr_prolong(mgic_amr a, int level, mgic_field corr, mgic_field corr_coarse) {
  return guard([&] {
    NEED(a);
    NEED(corr);
    NEED(corr_coarse);
    amr_level(a, level, 1);
    a->amr.AMRProlong(level, *corr->f, *corr_coarse->f);
  });
}
MGIC_API int mgic_amr_update_residual(mgic_amr a, int level, mgic_field res, mgic_field corr,
                                      mgic_field corr_coarse) {
  return guard([&] {
    NEED(a);
    NEED(res);
    NEED(corr);
    amr_level(a, level, 1);
    a->amr.AMRUpdateResidual(level, *res->f, *corr->f, corr_coarse ? corr_coarse->f.get() : nullptr);
  });
}
static std::vector<LevelData *> amr_fields(mgic_amr a, const mgic_field *f) {
  std::vector<LevelData *> v;
  for (int l = 0; l < a->amr.numLevels(); ++l) {
    MGIC_CHECK(f[l] != nullptr, "null field");
    check_same_layout(*a->amr.op(l).grid, *f[l]->f, "AMR field");
    v.push_back(f[l]->f.get());
  }
  return v;
}
MGIC_API int mgic_amr_init_residual(mgic_amr a, const mgic_field *phi, const mgic_field *rhs,
                                    int norm_type, double *norm) {
  return guard([&] {
    NEED(a);
    NEED(phi);
    NEED(rhs);
    auto p = amr_fields(a, phi);
    const double v = a->amr.initResidual(p, amr_fields(a, rhs), norm_type);
    if (norm) *norm = v;
  });
}
MGIC_API int mgic_amr_iteration(mgic_amr a, const mgic_field *phi, const mgic_field *rhs,
                                int norm_type, double *norm) {
  return guard([&] {
    NEED(a);
    NEED(phi);
    NEED(rhs);
    auto p = amr_fields(a, phi);
    const double v = a->amr.iteration(p, amr_fields(a, rhs), norm_type);
    if (norm) *norm = v;
  });
}
MGIC_API int mgic_amr_residual_field(mgic_amr a, int level, mgic_field *out) {
  return guard([&] {
    NEED(a);
    NEED(out);
    amr_level(a, level, 0);
    *out = borrowed_field(&a->amr.residual(level));
  });
}

MGIC_API int mgic_amr_apply_op(mgic_amr a, const mgic_field *lhs, const mgic_field *x,
                               int homogeneous) {
  return guard([&] {
    NEED(a);
    NEED(lhs);
    NEED(x);
    auto l = amr_fields(a, lhs);
    auto v = amr_fields(a, x);
    a->amr.applyOp(l, v, homogeneous != 0);
  });
}
MGIC_API int mgic_amr_dot(mgic_amr a, const mgic_field *x, const mgic_field *y, double *out) {
  return guard([&] {
    NEED(a);
    NEED(x);
    NEED(y);
    NEED(out);
    *out = a->amr.compositeDot(amr_fields(a, x), amr_fields(a, y));
  });
}
MGIC_API int mgic_amr_norm(mgic_amr a, const mgic_field *x, int ord, double *out) {
  return guard([&] {
    NEED(a);
    NEED(x);
    NEED(out);
    MGIC_CHECK(ord >= 0 && ord <= 2, "norm order must be 0, 1 or 2");
    *out = a->amr.compositeNorm(amr_fields(a, x), ord);
  });
}
MGIC_API int mgic_amr_composite_norm(mgic_amr a, const mgic_field *x, int ord, double *out) {
  return guard([&] {
    NEED(a);
    NEED(x);
    NEED(out);
    MGIC_CHECK(ord >= 0 && ord <= 2, "norm order must be 0, 1 or 2");
    *out = a->amr.compositeNorm(amr_fields(a, x), ord);
  });
}
MGIC_API int mgic_amr_composite_sum(mgic_amr a, const mgic_field *x, double *out) {
  return guard([&] {
    NEED(a);
    NEED(x);
    NEED(out);
    *out = a->amr.compositeSum(amr_fields(a, x));
  });
}
MGIC_API int mgic_amr_precondition(mgic_amr a, const mgic_field *e, const mgic_field *r, int iters) {
  return guard([&] {
    NEED(a);
    NEED(e);
    NEED(r);
    MGIC_CHECK(iters >= 0, "iters must be >= 0");
    auto ev = amr_fields(a, e);
    a->amr.precondition(ev, amr_fields(a, r), iters);
  });
}
MGIC_API int mgic_amr_solve(mgic_amr a, const mgic_field *phi, const mgic_field *rhs,
                            const mgic_solve_params *p, int *iterations, double *final_norm) {
  return guard([&] {
    NEED(a);
    NEED(phi);
    NEED(rhs);
    SolveParams sp;
    if (p) {
      sp.num_mg_iterations = p->num_mg_iterations;
      sp.max_iterations = p->max_iterations;
      sp.tolerance = p->tolerance;
      sp.norm_type = p->norm_type;
    }
    MGIC_CHECK(sp.max_iterations >= 0 && sp.tolerance >= 0.0, "bad solve parameters");
    MGIC_CHECK(sp.norm_type >= 0 && sp.norm_type <= 2, "norm type must be 0, 1 or 2");
    auto pv = amr_fields(a, phi);
    double nrm = 0.0;
    const int it = a->amr.solve(pv, amr_fields(a, rhs), sp, &nrm);
    if (iterations) *iterations = it;
    if (final_norm) *final_norm = nrm;
  });
}
MGIC_API int mgic_mg_precondition(mgic_mg mg, mgic_field e, mgic_field r, int iters) {
  return guard([&] {
    NEED(mg);
    NEED(e);
    NEED(r);
    MGIC_CHECK(iters >= 0, "iters must be >= 0");
    mg->amg.precondition(*e->f, *r->f, iters);
  });
}
MGIC_API void mgic_solve_params_default(mgic_solve_params *p) {
  if (!p) return;
  SolveParams d;
  p->num_mg_iterations = d.num_mg_iterations;
  p->max_iterations = d.max_iterations;
  p->tolerance = d.tolerance;
  p->norm_type = d.norm_type;
}
MGIC_API int mgic_mg_solve(mgic_mg mg, mgic_field phi, mgic_field rhs, const mgic_solve_params *p,
                           int *iterations, double *final_norm) {
  return guard([&] {
    NEED(mg);
    NEED(phi);
    NEED(rhs);
    SolveParams sp;
    if (p) {
      sp.num_mg_iterations = p->num_mg_iterations;
      sp.max_iterations = p->max_iterations;
      sp.tolerance = p->tolerance;
      sp.norm_type = p->norm_type;
    }
    MGIC_CHECK(sp.max_iterations >= 0 && sp.tolerance >= 0.0, "bad solve parameters");
    double nrm = 0.0;
    const int it = mg->amg.solve(*phi->f, *rhs->f, sp, &nrm);
    if (iterations) *iterations = it;
    if (final_norm) *final_norm = nrm;
  });
}
MGIC_API int mgic_prof_smoother(int enable, long min_cells) {
  return guard([&] { prof_enable(enable != 0, min_cells, enable == 2 ? 2 : 1); });
}
MGIC_API int mgic_prof_smoother_read(int *launches, long *passes, double *total_ms) {
  return guard([&] {
    double t = 0.0;
    long np = 0;
    const int n = prof_read(&t, &np);
    if (launches) *launches = n;
    if (passes) *passes = np;
    if (total_ms) *total_ms = t;
  });
}

}  // extern "C"
