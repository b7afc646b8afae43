// op.cpp -- VariableCoeffPoissonOperator(+Factory), BiCGStabSolver,
// MultiGrid, AMRMultiGrid (see op.hpp).
#include "op.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace mgic {

// --------------------------------------------------------------- profiling
namespace {
// HIP events around the fine-level smoother launches (bench.py's roofline).
// mode 1: one event pair per launch.  mode 2: one pair per run of
// consecutive counted launches (a relax call), time / launches = the
// average launch: an event record between two kernels costs a ~5-10 us
// gap on this stack, which mode 1 adds to the timed V-cycle 16 times.
struct SmootherProf {
  int mode = 0;
  long min_cells = 0;
  std::vector<hipEvent_t> ev;
  size_t used = 0;
  bool open = false;
  long passes = 0;    // colour passes covered by the recorded launches
  long launches = 0;  // launches inside the recorded intervals
  hipStream_t st = nullptr;
} g_prof;

void prof_record(hipStream_t st) {
  if (g_prof.used + 1 > g_prof.ev.size()) {
    const size_t add = std::max<size_t>(256, g_prof.ev.size());
    for (size_t i = 0; i < add; ++i) {
      hipEvent_t e;
      MGIC_HIP(hipEventCreate(&e));
      g_prof.ev.push_back(e);
    }
  }
  MGIC_HIP(hipEventRecord(g_prof.ev[g_prof.used++], st));
}
}  // namespace

void prof_enable(bool on, long min_cells, int mode) {
  g_prof.mode = on ? mode : 0;
  g_prof.min_cells = min_cells;
  g_prof.used = 0;
  g_prof.open = false;
  g_prof.passes = 0;
  g_prof.launches = 0;
}

void prof_flush() {
  if (g_prof.mode == 2 && g_prof.open) {
    prof_record(g_prof.st);
    g_prof.open = false;
  }
}

void prof_mark(hipStream_t st, long ncells, bool begin, int passes) {
  if (!g_prof.mode) return;
  if (ncells < g_prof.min_cells) {  // an uncounted launch closes a mode-2 interval
    if (begin) prof_flush();
    return;
  }
  if (begin) {
    if (g_prof.open && g_prof.mode == 2 && st == g_prof.st) return;  // interval continues
    prof_flush();
    prof_record(st);
    g_prof.open = true;
    g_prof.st = st;
  } else if (g_prof.open) {
    g_prof.passes += passes;
    g_prof.launches += 1;
    if (g_prof.mode == 1) {
      prof_record(st);
      g_prof.open = false;
    }
  }
}

int prof_read(double *total_ms, long *passes) {
  prof_flush();
  double tot = 0.0;
  if (g_prof.used) MGIC_HIP(hipEventSynchronize(g_prof.ev[g_prof.used - 1]));
  for (size_t i = 0; i + 1 < g_prof.used; i += 2) {
    float ms = 0.f;
    MGIC_HIP(hipEventElapsedTime(&ms, g_prof.ev[i], g_prof.ev[i + 1]));
    tot += ms;
  }
  *total_ms = tot;
  if (passes) *passes = g_prof.passes;
  return (int)g_prof.launches;
}

// --------------------------------------------------------------- operator
int VariableCoeffPoissonOperator::s_maxCoarse = 2;
static int sweeps_per_launch();

void check_same_layout(const Grid &g, const LevelData &x, const char *what) {
  const Grid &h = *x.grid;
  bool ok = h.nlocal() == g.nlocal();
  for (int n = 0; ok && n < g.nlocal(); ++n)
    ok = h.geom[n].valid == g.geom[n].valid && h.geom[n].sy == g.geom[n].sy &&
         h.geom[n].sz == g.geom[n].sz;
  if (!ok) throw Error(kBadArg, std::string("layout mismatch: ") + what);
}

void VariableCoeffPoissonOperator::define(std::shared_ptr<Grid> g, const OpParams &p) {
  grid = std::move(g);
  prm = p;
  m_dx = grid->dx;
  m_alpha = p.alpha;
  m_beta = p.beta;
  m_lambdaNeedsResetting = true;
  build_args();
}

void VariableCoeffPoissonOperator::build_args() {
  args_hom_.clear();
  args_inhom_.clear();
  args_plain_.clear();
  for (int n = 0; n < grid->nlocal(); ++n) {
    args_hom_.push_back(grid->box_args(n, prm.bc_lo, prm.bc_hi, prm.bc_value, true));
    args_inhom_.push_back(grid->box_args(n, prm.bc_lo, prm.bc_hi, prm.bc_value, false));
    args_plain_.push_back(grid->box_args_plain(n));
  }
}

const BoxArgs &VariableCoeffPoissonOperator::args(int n, bool homogeneous) {
  return homogeneous ? args_hom_[n] : args_inhom_[n];
}

StencilCoefs VariableCoeffPoissonOperator::coefs() {
  resetLambda();  // lazy: lambda and the constant-b test follow coefficient changes
  StencilCoefs s;
  s.alpha = m_alpha;
  s.beta = m_beta;
  s.dx = m_dx;
  s.dxinv = 1.0 / (m_dx * m_dx);                    // .ChF:89
  s.lamshift = 2.0 * 3 * m_beta / (m_dx * m_dx);    // .cpp:240
  s.bconst = b_const_ ? 1 : 0;
  s.bval = b_val_;
  s.rcp_fast = rcp_fast_ ? 1 : 0;
  s.rcp_fast32 = rcp_fast32_ ? 1 : 0;
  return s;
}

void VariableCoeffPoissonOperator::residualI(LevelData &lhs, LevelData &dpsi,
                                             const LevelData &rhs, bool homogeneous) {
  check_same_layout(*grid, lhs, "residual lhs");
  check_same_layout(*grid, dpsi, "residual dpsi");
  check_same_layout(*grid, rhs, "residual rhs");
  const hipStream_t st = stream();
  dpsi.exchange(st);  // .cpp:48 (the BC of :43-45 is folded into the kernel)
  const StencilCoefs s = coefs();
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::residual(lhs.p[n], dpsi.p[n], rhs.p[n], m_aCoef->p[n], m_bCoef->p[n], args(n, homogeneous),
                   s, st);
}

double VariableCoeffPoissonOperator::residualNorm(LevelData &lhs, LevelData &dpsi,
                                                  const LevelData &rhs, bool homogeneous,
                                                  int normType) {
  double now = 0.0;
  const unsigned long long t = residualNormQueue(lhs, dpsi, rhs, homogeneous, normType, &now);
  return t ? residualNormTake(t) : now;
}

double VariableCoeffPoissonOperator::residualNormTake(unsigned long long ticket) {
  Comm &c = *grid->comm;
  c.wait_results(stream(), ticket);
  return c.h_result()[kNormSlot];
}

unsigned long long VariableCoeffPoissonOperator::residualNormQueue(LevelData &lhs, LevelData &dpsi,
                                                                   const LevelData &rhs,
                                                                   bool homogeneous, int normType,
                                                                   double *now) {
  long total = 0;
  bool fused = normType == 0;
  for (int n = 0; fused && n < grid->nlocal(); ++n) {
    const long nb = kern::residual_norm_blocks(args(n, homogeneous));
    fused = nb > 0;
    total += nb;
  }
  if (!fused) {
    residualI(lhs, dpsi, rhs, homogeneous);
    *now = normType >= 0 ? norm(lhs, normType) : -1.0;
    return 0;
  }
  check_same_layout(*grid, lhs, "residual lhs");
  check_same_layout(*grid, dpsi, "residual dpsi");
  check_same_layout(*grid, rhs, "residual rhs");
  Comm &c = *grid->comm;
  const hipStream_t st = stream();
  dpsi.exchange(st);  // .cpp:48
  const StencilCoefs s = coefs();
  double *parts = c.d_partials((int)std::max(1L, total));
  long off = 0;
  for (int n = 0; n < grid->nlocal(); ++n) {
    const BoxArgs &a = args(n, homogeneous);
    kern::residual_norm(lhs.p[n], dpsi.p[n], rhs.p[n], m_aCoef->p[n], m_bCoef->p[n], a, s,
                        parts + off, st);
    off += kern::residual_norm_blocks(a);
  }
  finish_reduce(3, parts, (int)total, kNormSlot);
  return c.last_ticket();
}

void VariableCoeffPoissonOperator::preCond(LevelData &cor, const LevelData &res) {
  resetLambda();  // .cpp:90
  const hipStream_t st = stream();
  // cor = res (:99), then cor *= lambda (:100), as one pass: res * lambda is
  // the same product (IEEE multiplication commutes)
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::blas(6, cor.p[n], res.p[n], m_lambda->p[n], 0.0, 0.0, args_plain_[n], st);
  relax(cor, res, 2);  // :103
}

bool VariableCoeffPoissonOperator::preCondFromScaledApplies() {
  if (prm.relax_mode != 1 || cf || !fusedSmootherApplies()) return false;
  if (grid->nlocal() != 1 || grid->has_memory_faces() || sweeps_per_launch() < 2) return false;
  const StencilCoefs s = coefs();
  // fusedRelax(cor, res, 2) is then exactly one two-sweep launch from cor
  return kern::gsrb_sweep_tb2_applies(args_hom_[0], s, prm.fused_smoother);
}

void VariableCoeffPoissonOperator::preCondFromScaled(LevelData &cor, const LevelData &w,
                                                     const LevelData &res, const int *skip) {
  const StencilCoefs s = coefs();  // resetLambda (.cpp:90)
  kern::gsrb_sweep_tb2(cor.p[0], w.p[0], res.p[0], m_aCoef->p[0], args_hom_[0], s, false, nullptr,
                       stream(), skip);
}

void VariableCoeffPoissonOperator::applyOpI(LevelData &lhs, LevelData &dpsi, bool homogeneous) {
  check_same_layout(*grid, lhs, "applyOp lhs");
  check_same_layout(*grid, dpsi, "applyOp dpsi");
  const hipStream_t st = stream();
  dpsi.exchange(st);  // .cpp:131 (BC of :115-117 folded)
  const StencilCoefs s = coefs();
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::apply_op(lhs.p[n], dpsi.p[n], m_aCoef->p[n], m_bCoef->p[n], args(n, homogeneous), s, st);
}

void VariableCoeffPoissonOperator::applyOpNoBoundary(LevelData &lhs, LevelData &dpsi) {
  const hipStream_t st = stream();
  dpsi.exchange(st);
  const StencilCoefs s = coefs();
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::apply_op(lhs.p[n], dpsi.p[n], m_aCoef->p[n], m_bCoef->p[n], args_plain_[n], s, st);
}

void VariableCoeffPoissonOperator::restrictResidual(LevelData &resC, LevelData &dpsiF,
                                                    const LevelData &rhsF, bool exchange) {
  const Grid &cg = *resC.grid;
  MGIC_CHECK(cg.nlocal() == grid->nlocal(), "restrictResidual: coarse layout mismatch");
  for (int n = 0; n < grid->nlocal(); ++n) {
    MGIC_CHECK(grid->geom[n].valid.coarsenable(2), "restrictResidual: fine box not coarsenable");
    MGIC_CHECK(cg.geom[n].valid == grid->geom[n].valid.coarsened(2),
               "restrictResidual: coarse box is not coarsen(fine box, 2)");
  }
  const hipStream_t st = stream();
  if (cf) cf_homogeneous(*cf, dpsiF, st);  // .cpp:156
  if (exchange || cf) dpsiF.exchange(st);  // .cpp:163 (BC of :158-161 folded, homogeneous)
  const StencilCoefs s = coefs();
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::restrict_residual(resC.p[n], cg.box_args_plain(n), dpsiF.p[n], rhsF.p[n], m_aCoef->p[n],
                            m_bCoef->p[n], args(n, true), s, st);
}

void VariableCoeffPoissonOperator::prolongIncrement(LevelData &phi, LevelData &corC) {
  if (prm.prolong_type == 1) corC.exchange(stream());
  prolongIncrementFilled(phi, corC);
}

void VariableCoeffPoissonOperator::prolongIncrementFilled(LevelData &phi, const LevelData &corC) {
  const Grid &cg = *corC.grid;
  MGIC_CHECK(cg.nlocal() == grid->nlocal(), "prolongIncrement: coarse layout mismatch");
  const hipStream_t st = stream();
  for (int n = 0; n < grid->nlocal(); ++n) {
    const Box &cb = cg.geom[n].valid;
    MGIC_CHECK(cb == grid->geom[n].valid.coarsened(2), "prolongIncrement: coarse box mismatch");
    int alo[3], ahi[3];
    for (int d = 0; d < 3; ++d) {
      alo[d] = cg.periodic[d] || cb.lo[d] > cg.domain.lo[d];
      ahi[d] = cg.periodic[d] || cb.hi[d] < cg.domain.hi[d];
    }
    kern::prolong(phi.p[n], args_plain_[n], corC.p[n], cg.box_args_plain(n), alo, ahi,
                  prm.prolong_type, st);
  }
}

void VariableCoeffPoissonOperator::setAlphaAndBeta(double alpha, double beta) {
  m_alpha = alpha;  // .cpp:196-203
  m_beta = beta;
  m_lambdaNeedsResetting = true;
}

void VariableCoeffPoissonOperator::setCoefs(std::shared_ptr<LevelData> a,
                                            std::shared_ptr<LevelData> b, double alpha,
                                            double beta) {
  check_same_layout(*grid, *a, "aCoef");
  check_same_layout(*grid, *b, "bCoef");
  m_alpha = alpha;  // .cpp:205-218
  m_beta = beta;
  m_aCoef = std::move(a);
  m_bCoef = std::move(b);
  m_lambdaNeedsResetting = true;
  coef_ghosts_ = false;
}

void VariableCoeffPoissonOperator::resetLambda() {
  if (!m_lambdaNeedsResetting) return;  // .cpp:222
  m_lambdaNeedsResetting = false;
  if (!m_lambda) m_lambda = std::make_unique<LevelData>(grid);
  // a gathered depth on a rank that does not hold it: nothing to compute
  // (it never runs a kernel or a reduction there)
  if (owner_local >= 0 && grid->comm->rank() != owner_local) return;
  // is bCoef one value everywhere?  (max b == min b over all ranks' boxes)
  const double bmax = reduce(4, *m_bCoef, nullptr), bmin = -reduce(5, *m_bCoef, nullptr);
  b_const_ = bmax == bmin && std::isfinite(bmax);
  b_val_ = b_const_ ? bmax : 1.0;
  rcp_fast_ = rcp_fast32_ = false;
  const StencilCoefs s = coefs();
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::lambda(m_lambda->p[n], m_aCoef->p[n], args_plain_[n], s, stream());
  // the range of lambda over every rank's cells (StencilCoefs::rcp_fast):
  // the denominators the sweeps meet, ghost cells included, are some rank's
  // valid cells
  static const int allow = [] {
    const char *e = getenv("MGIC_TB2_RCP");
    return e ? atoi(e) : 1;
  }();
  if (allow) {
    const double lmax = reduce(4, *m_lambda, nullptr), lmin = -reduce(5, *m_lambda, nullptr);
    // |lambda| in [2^-e, 2^e], one sign (a <= b, both > 0 in ok)
    auto within = [&](int e) {
      const double lo = std::ldexp(1.0, -e), hi = std::ldexp(1.0, e);
      auto ok = [&](double a, double b) { return a >= lo && b <= hi; };
      return std::isfinite(lmax) && std::isfinite(lmin) &&
             ((lmin > 0.0 && ok(lmin, lmax)) || (lmax < 0.0 && ok(-lmax, -lmin)));
    };
    rcp_fast_ = within(500);
    rcp_fast32_ = within(60);
  }
}

void VariableCoeffPoissonOperator::computeLambda() {
  if (!m_lambda) m_lambda = std::make_unique<LevelData>(grid);  // .cpp:258
  m_lambdaNeedsResetting = true;
  resetLambda();
}

void VariableCoeffPoissonOperator::setTime(double t) {
  m_time = t;  // .cpp:400-420 (no b-coefficient interpolator is set in this app)
  m_lambdaNeedsResetting = true;
}

// An AMR level whose boxes are isolated patches (no box face touches another
// box, no periodic images): every non-domain face is a coarse-fine face, so
// homogeneousCFInterp before each colour pass (.cpp:296) is a per-face ghost
// rule of the two cells next to it, which the 3D-block sweep applies in LDS
// at entry and again between its red and black passes (MGIC_CF_FUSED=0: the
// per-colour path).  Mixed faces (part CF, part fine-fine) stay per colour.
bool VariableCoeffPoissonOperator::cfFusedApplies() {
  if (cf_fused_ >= 0) return cf_fused_ == 1;
  static const int enabled = [] {
    const char *e = getenv("MGIC_CF_FUSED");
    return e ? atoi(e) : 1;
  }();
  bool ok = enabled && prm.fused_smoother != 0;
  for (int d = 0; d < 3; ++d) ok = ok && !grid->periodic[d];
  const std::vector<Box> &bx = grid->boxes;
  for (size_t i = 0; ok && i < bx.size(); ++i)
    for (size_t j = 0; ok && j < bx.size(); ++j) {
      if (i == j) continue;
      for (int d = 0; ok && d < 3; ++d) {  // box i grown by one across its d faces
        Box g = bx[i];
        g.lo[d] -= 1;
        g.hi[d] += 1;
        bool meet = true;
        for (int e = 0; e < 3; ++e)
          meet = meet && g.lo[e] <= bx[j].hi[e] && bx[j].lo[e] <= g.hi[e];
        ok = !meet;
      }
    }
  for (int n = 0; ok && n < grid->nlocal(); ++n) {
    const FabGeom &fg = grid->geom[n];
    ok = fg.nx % 2 == 0 && fg.valid.lo[0] % 2 == 0;  // the kernel's x pairs
  }
  args_cf_.clear();
  for (int n = 0; ok && n < grid->nlocal(); ++n) {
    BoxArgs a = args_hom_[n];
    for (int f = 0; f < 6; ++f)
      if (a.bcm[f] == kBcMemory) {
        a.bcm[f] = kBcCFHom;
        a.bcc[f] = 0.0;
      }
    args_cf_.push_back(a);
  }
  cf_fused_ = ok ? 1 : 0;
  return ok;
}

bool VariableCoeffPoissonOperator::fusedSmootherApplies() {
  if (cf) return cfFusedApplies();  // isolated patches only (see above)
  // Both colour passes of a sweep in one launch per box.  Faces on the
  // domain boundary fold the BC; exchanged faces (box or periodic
  // neighbours) get a 2-deep ghost shell before the sweep, from which the
  // kernel recomputes the neighbours' red values on its ghost layer -- the
  // values the reference's second exchange (.cpp:301, black pass) delivers.
  return prm.fused_smoother != 0;
}

// MGIC_SWEEPS_PER_LAUNCH: 2 (default) pairs consecutive sweeps in the
// temporally blocked kernel (smoother_tb.hip) where it applies; 1 one sweep
// per launch.  (Round 1's two-sweep kernels, selected by 3 / 4, ran no faster
// than the single sweep and were removed in round 3.)
static int sweeps_per_launch() {
  static const int v = [] {
    const char *e = getenv("MGIC_SWEEPS_PER_LAUNCH");
    return e ? std::max(1, std::min(2, atoi(e))) : 2;
  }();
  return v;
}

// Deep halo (deep_halo = 1): a 4-deep ghost shell feeds two sweeps.  The
// first sweeps the box grown by 2 across every exchanged face -- the
// neighbours' cells within 2 of the face, recomputed from the shell with the
// same expressions and inputs, so bit-identical to their own -- which leaves
// the result's 2-deep shell valid for the second sweep without an exchange.
// Half the exchanges of the 2-deep scheme for the same bytes (latency bound
// halos on coarse levels and small per-rank boxes).  rhs / aCoef / bCoef need
// the 4-deep shell too (the grown sweep's red ring reaches depth 3).
static constexpr int kDeepDepth = 4, kDeepGrow = 2;

bool VariableCoeffPoissonOperator::deepApplies() const {
  if (!prm.deep_halo || !grid->has_memory_faces() || !grid->tiles_domain()) return false;
  static const long max_cells = [] {  // deep_halo 2: only levels of boxes up to this size
    const char *e = getenv("MGIC_DEEP_MAX_CELLS");
    return e ? atol(e) : 128L * 128 * 128;
  }();
  // every shell cell must be some box's valid cell within one period
  for (const Box &b : grid->boxes) {
    if (prm.deep_halo == 2 && b.ncells() > max_cells) return false;
    for (int d = 0; d < 3; ++d)
      if (b.size(d) < kDeepDepth) return false;
  }
  return true;
}

void VariableCoeffPoissonOperator::rhsHalo(LevelData &r, hipStream_t st) const {
  if (deepApplies()) r.exchange_shell(st, kDeepDepth);
  else r.exchange(st);
}

// the box grown by `d` cells across every exchanged face (element offset of
// its lo corner from the valid-lo corner: negative)
static BoxArgs grow_exchanged(const BoxArgs &g, int d, long *off) {
  BoxArgs a = g;
  long o = 0;
  const long st[3] = {1, g.sy, g.sz};
  int *n[3] = {&a.nx, &a.ny, &a.nz};
  for (int k = 0; k < 3; ++k) {
    if (!g.bcm[2 * k]) {
      *n[k] += d;
      a.glo[k] -= d;
      o -= d * st[k];
    }
    if (!g.bcm[2 * k + 1]) *n[k] += d;
  }
  *off = o;
  return a;
}

bool VariableCoeffPoissonOperator::fusedRelax(LevelData &dpsi, const LevelData &rhs, int n,
                                              bool zero_in, LevelData *acc, int flags,
                                              LevelData *rst,
                                              const std::function<void()> *before_acc) {
  resetLambda();  // .cpp:283
  const hipStream_t st = stream();
  const StencilCoefs s = coefs();
  if (!sweep_tmp_) sweep_tmp_ = create();
  // AMR level > 0 (isolated patches): no exchanges, coarse-fine faces as
  // ghost rules, 3D-block kernel, no fused restriction / two-sweep launches
  const bool cfl = cf != nullptr;
  if (cfl) MGIC_CHECK(cfFusedApplies(), "fused sweep on a coarse-fine level it does not apply to");
  const std::vector<BoxArgs> &sargs = cfl ? args_cf_ : args_hom_;
  const int skind = cfl ? 3 : prm.fused_smoother;
  if (cfl) rst = nullptr;
  const bool halo = !cfl && grid->has_memory_faces();
  const bool deep_ok = halo && deepApplies();
  if (halo) {  // ghost layer 1 of rhs / aCoef / bCoef for the red ring on the halo
    if (!(flags & kRhsHaloReady)) rhsHalo(const_cast<LevelData &>(rhs), st);
    if (!coef_ghosts_) {
      if (deep_ok) {
        m_aCoef->exchange_shell(st, kDeepDepth);
        m_bCoef->exchange_shell(st, kDeepDepth);
      } else {
        m_aCoef->exchange(st);
        m_bCoef->exchange(st);
      }
      coef_ghosts_ = true;
    }
  }
  LevelData *src = &dpsi, *dst = sweep_tmp_.get();
  // two sweeps per launch (temporal blocking): on boxes with only domain
  // faces, or with exchanged faces in deep-halo mode (the kernel's rings run
  // onto the 4-deep shell, exchanged before every pair; rhs / coefficient
  // shells are 4 deep there too)
  const int spl = sweeps_per_launch();
  bool two = (!halo || (deep_ok && spl == 2)) && !cfl && spl >= 2 && n >= 2;
  for (int b = 0; two && b < grid->nlocal(); ++b)
    two = kern::gsrb_sweep_tb2_applies(args_hom_[b], s, prm.fused_smoother);
  const int per = two ? 2 : 1;
  // the pair also takes the phi += e sweep
  const bool pair_acc = two;
  const bool want_out = halo && (flags & kHaloOut) && !acc;
  // (overlapping the exchange with the sweep on a second stream, by
  // recomputed boundary slabs or a boundary-first split, measured slower
  // with both transports and was removed in round 4: DESIGN.md 6)
  const bool deep = deep_ok && per == 1;
  int vd = zero_in ? (1 << 20) : 0;  // deep: valid ghost-shell depth of src
  bool out_ready = false;            // deep: the last sweep left its face ghosts valid
  // the last sweep restricts too (single sweep kernel over every box) when
  // it is a single sweep: with pairs, a separate restriction is cheaper than
  // splitting the last pair
  bool restrict_last = rst != nullptr && !acc && !(zero_in && n == 1) && !halo &&
                       !(pair_acc && n % 2 == 0);
  if (restrict_last) {
    const Grid &cg = *rst->grid;
    restrict_last = cg.nlocal() == grid->nlocal();
    for (int b = 0; restrict_last && b < grid->nlocal(); ++b)
      restrict_last = cg.geom[b].valid == grid->geom[b].valid.coarsened(2) &&
                      kern::gsrb_sweep_fused_restrict_applies(args_hom_[b], cg.box_args_plain(b),
                                                              prm.fused_smoother);
  }
  for (int it = 0; it < n;) {
    const bool zin = zero_in && it == 0;
    // a pair, unless it would swallow a special last sweep (+ restriction,
    // phi += e)
    const int left = n - it;
    const int k = per == 2 && (left >= 3 || (left == 2 && !restrict_last && (!acc || pair_acc))) ? 2 : 1;
    const bool last = it + k == n;
    if (deep) {
      if (vd < 2) {
        src->exchange_shell(st, kDeepDepth);
        vd = kDeepDepth;
      }
    } else if (halo && !zin) {
      src->exchange_shell(st, k == 2 ? kDeepDepth : 2);
    }
    // deep: sweep the grown box when the shell allows it and the result's
    // ghosts are wanted (a later sweep, or the caller's face ghosts)
    const int grow = deep && vd >= kDeepDepth && !(last && acc) && (!last || want_out) ? kDeepGrow : 0;
    if (deep) {
      vd = grow;
      if (last) out_ready = grow > 0;
    }
    if (last && acc && before_acc) (*before_acc)();
    for (int b = 0; b < grid->nlocal(); ++b) {
      // the roofline instrumentation times the sweep kernels only (the
      // sweep+restriction launch moves other bytes)
      const long nc = last && restrict_last ? 0 : grid->geom[b].valid.ncells();
      prof_mark(st, nc, true, 2 * k);
      if (k == 2)  // two sweeps in one launch (temporal blocking), + phi += e
        kern::gsrb_sweep_tb2(dst->p[b], src->p[b], rhs.p[b], m_aCoef->p[b], args_hom_[b], s, zin,
                             last && acc ? acc->p[b] : nullptr, st);
      else if (last && restrict_last)  // + restrictResidual(rst, result, rhs)
        kern::gsrb_sweep_fused_restrict(dst->p[b], src->p[b], rhs.p[b], m_aCoef->p[b],
                                        m_bCoef->p[b], args_hom_[b], s, rst->p[b],
                                        rst->grid->box_args_plain(b), st);
      else if (grow) {
        long o = 0;
        const BoxArgs ga = grow_exchanged(args_hom_[b], grow, &o);
        kern::gsrb_sweep_fused(dst->p[b] + o, src->p[b] + o, rhs.p[b] + o, m_aCoef->p[b] + o,
                               m_bCoef->p[b] + o, ga, s, zin, nullptr, prm.fused_smoother, st);
      } else
        kern::gsrb_sweep_fused(dst->p[b], src->p[b], rhs.p[b], m_aCoef->p[b], m_bCoef->p[b],
                               sargs[b], s, zin, last && acc ? acc->p[b] : nullptr, skind, st);
      prof_mark(st, nc, false, 2 * k);
    }
    std::swap(src, dst);
    it += k;
  }
  prof_flush();  // the interval ends with the relax
  if (acc) return false;  // the last sweep went into acc; dpsi is scratch now
  if (src != &dpsi) {  // the result sits in the scratch buffer
    for (int b = 0; b < grid->nlocal(); ++b)
      kern::blas(0, dpsi.p[b], src->p[b], nullptr, 0.0, 0.0, args_plain_[b], st);
    if (want_out) dpsi.exchange(st);
  } else if (want_out && !out_ready) {
    dpsi.exchange(st);
  }
  return restrict_last;
}

void VariableCoeffPoissonOperator::relaxAccumulate(LevelData &e, const LevelData &r, int n,
                                                   LevelData &phi, int flags,
                                                   const std::function<void()> *before_acc) {
  if (n > 0 && prm.relax_mode == 1 && fusedSmootherApplies()) {
    check_same_layout(*grid, phi, "phi");
    fusedRelax(e, r, n, false, &phi, flags, nullptr, before_acc);
    return;
  }
  relax(e, r, n);
  if (before_acc) (*before_acc)();
  incr(phi, e, 1.0);
}

void VariableCoeffPoissonOperator::relaxFromZero(LevelData &e, const LevelData &r, int n,
                                                 int flags) {
  if (n > 0 && prm.relax_mode == 1 && fusedSmootherApplies()) {
    fusedRelax(e, r, n, true, nullptr, flags);
    return;
  }
  setToZero(e);
  relax(e, r, n);
  if (flags & kHaloOut) e.exchange(stream());
}

bool VariableCoeffPoissonOperator::relaxRestrict(LevelData &e, const LevelData &r, int n,
                                                 bool zero_in, int flags, LevelData &resC) {
  if (n > 0 && prm.relax_mode == 1 && fusedSmootherApplies()) {
    resetLambda();
    return fusedRelax(e, r, n, zero_in, nullptr, flags, &resC);
  }
  if (zero_in)
    relaxFromZero(e, r, n, flags);
  else
    relaxFlags(e, r, n, flags);
  return false;
}

void VariableCoeffPoissonOperator::relaxFlags(LevelData &e, const LevelData &r, int n,
                                              int flags) {
  if (n > 0 && prm.relax_mode == 1 && fusedSmootherApplies()) {
    fusedRelax(e, r, n, false, nullptr, flags);
    return;
  }
  relax(e, r, n);
  if (flags & kHaloOut) e.exchange(stream());
}

void VariableCoeffPoissonOperator::relax(LevelData &e, const LevelData &r, int iterations) {
  if (iterations <= 0) return;
  if (prm.relax_mode == 1 && fusedSmootherApplies()) {
    fusedRelax(e, r, iterations);
    return;
  }
  for (int it = 0; it < iterations; ++it) {
    switch (prm.relax_mode) {
      case 1: levelGSRB(e, r); break;
      case 4: levelJacobi(e, r); break;
      case 2: levelMultiColor(e, r); break;
      case 3: looseGSRB(e, r); break;
      case 5: overlapGSRB(e, r); break;
      default: levelGSRBLazy(e, r);
    }
  }
}

void VariableCoeffPoissonOperator::levelGSRB(LevelData &dpsi, const LevelData &rhs) {
  if (fusedSmootherApplies()) {
    fusedRelax(dpsi, rhs, 1);
    return;
  }
  resetLambda();  // .cpp:283
  const hipStream_t st = stream();
  const StencilCoefs s = coefs();
  for (int pass = 0; pass <= 1; ++pass) {  // .cpp:290
    if (cf) cf_homogeneous(*cf, dpsi, st);  // .cpp:296
    dpsi.exchange(st);                      // .cpp:301 (BC of :307-310 folded)
    for (int n = 0; n < grid->nlocal(); ++n) {
      const long nc = grid->geom[n].valid.ncells();
      prof_mark(st, nc, true, 1);
      kern::gsrb_pass(dpsi.p[n], rhs.p[n], m_aCoef->p[n], m_bCoef->p[n], nullptr, args_hom_[n], s,
                      pass, st);  // .cpp:313-330
      prof_mark(st, nc, false, 1);
    }
  }
}

void VariableCoeffPoissonOperator::levelJacobi(LevelData &dpsi, const LevelData &rhs) {
  resetLambda();  // .cpp:366
  if (!jac_tmp_) jac_tmp_ = create();
  residualI(*jac_tmp_, dpsi, rhs, true);  // .cpp:372
  const hipStream_t st = stream();
  for (int n = 0; n < grid->nlocal(); ++n) {
    kern::blas(3, jac_tmp_->p[n], m_lambda->p[n], nullptr, 0.0, 0.0, args_plain_[n], st);  // :377
    kern::blas(1, dpsi.p[n], jac_tmp_->p[n], nullptr, 0.5, 0.0, args_plain_[n], st);       // :381
  }
  dpsi.exchange(st);  // :384
}

void VariableCoeffPoissonOperator::levelMultiColor(LevelData &, const LevelData &) {
  throw Error(kState, "VariableCoeffPoissonOperator::levelMultiColor - Not implemented");
}
void VariableCoeffPoissonOperator::looseGSRB(LevelData &, const LevelData &) {
  throw Error(kState, "VariableCoeffPoissonOperator::looseGSRB - Not implemented");
}
void VariableCoeffPoissonOperator::overlapGSRB(LevelData &, const LevelData &) {
  throw Error(kState, "VariableCoeffPoissonOperator::overlapGSRB - Not implemented");
}
void VariableCoeffPoissonOperator::levelGSRBLazy(LevelData &, const LevelData &) {
  throw Error(kState, "VariableCoeffPoissonOperator::levelGSRBLazy - Not implemented");
}

void VariableCoeffPoissonOperator::fillBC(LevelData &u, bool homogeneous) {
  for (int n = 0; n < grid->nlocal(); ++n) kern::fill_bc(u.p[n], args(n, homogeneous), stream());
}

void VariableCoeffPoissonOperator::setToZero(LevelData &x) { x.set_zero_all(stream()); }

void VariableCoeffPoissonOperator::assignLocal(LevelData &lhs, const LevelData &rhs) {
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::blas(0, lhs.p[n], rhs.p[n], nullptr, 0.0, 0.0, args_plain_[n], stream());
}
void VariableCoeffPoissonOperator::incr(LevelData &lhs, const LevelData &x, double sc) {
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::blas(1, lhs.p[n], x.p[n], nullptr, sc, 0.0, args_plain_[n], stream());
}
void VariableCoeffPoissonOperator::axby(LevelData &lhs, const LevelData &x, const LevelData &y,
                                        double a, double b) {
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::blas(4, lhs.p[n], x.p[n], y.p[n], a, b, args_plain_[n], stream());
}
void VariableCoeffPoissonOperator::scale(LevelData &lhs, double sc) {
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::blas(2, lhs.p[n], nullptr, nullptr, sc, 0.0, args_plain_[n], stream());
}
void VariableCoeffPoissonOperator::mult(LevelData &lhs, const LevelData &x) {
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::blas(3, lhs.p[n], x.p[n], nullptr, 0.0, 0.0, args_plain_[n], stream());
}
void VariableCoeffPoissonOperator::setVal(LevelData &lhs, double v) {
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::blas(5, lhs.p[n], nullptr, nullptr, v, 0.0, args_plain_[n], stream());
}

// the final step of a reduction into result slot `slot`, published to the
// host by its last kernel (the final reduction on one rank, the allreduce on
// several); `last`: the readback's last result (Comm::wait_results)
void VariableCoeffPoissonOperator::finish_reduce(int kind, double *parts, int total, int slot,
                                                 bool last) {
  Comm &c = *grid->comm;
  const hipStream_t st = stream();
  double *res = c.d_result() + slot;
  // a gathered depth reduces on its owner alone (the rank-0 bottom solve:
  // no other rank joins its Krylov reductions)
  if (owner_local >= 0 && c.rank() != owner_local)
    throw Error(kState, "reduction on a gathered MG depth: it runs on its owner rank only");
  const kern::HostPub pub = c.host_pub(slot, last);
  const bool solo = c.size() == 1 || owner_local >= 0;
  if (total == 0) {  // no local cells: the identity of the reduction
    *c.h_stage() = kind >= 4 ? -HUGE_VAL : 0.0;
    MGIC_HIP(hipMemcpyAsync(res, c.h_stage(), sizeof(double), hipMemcpyHostToDevice, st));
    MGIC_HIP(hipStreamSynchronize(st));  // (the staging word is reused)
    c.allreduce(res, kind >= 3 ? 1 : 0, pub);
    c.commit_pub(pub);
    return;
  }
  kern::reduce_final(kind, parts, total, res, st, solo ? pub : kern::HostPub());
  if (!solo) c.allreduce(res, kind >= 3 ? 1 : 0, pub);
  c.commit_pub(pub);
}

double VariableCoeffPoissonOperator::reduce(int kind, const LevelData &x, const LevelData *y) {
  Comm &c = *grid->comm;
  const hipStream_t st = stream();
  double *parts = c.d_partials(std::max(1, grid->nlocal()) * kern::kMaxPartsPerBox);
  int total = 0;
  for (int n = 0; n < grid->nlocal(); ++n)
    total += kern::reduce_partial(kind, x.p[n], y ? y->p[n] : nullptr, args_plain_[n], parts + total, st);
  finish_reduce(kind, parts, total, 0);
  c.wait_results(st);
  return c.h_result()[0];
}

static int norm_kind(int ord) { return ord == 0 ? 3 : ord == 1 ? 1 : 2; }

double VariableCoeffPoissonOperator::axpy2Norm(LevelData &s, const LevelData &r, const LevelData &v,
                                               double ca, LevelData &e, const LevelData &pt,
                                               double cb, int ord) {
  Comm &c = *grid->comm;
  const hipStream_t st = stream();
  const int kind = norm_kind(ord);
  double *parts = c.d_partials(std::max(1, grid->nlocal()) * kern::kMaxPartsPerBox);
  int total = 0;
  for (int n = 0; n < grid->nlocal(); ++n)
    total += kern::axpy2_reduce(kind, s.p[n], r.p[n], v.p[n], ca, e.p[n], pt.p[n], cb,
                                args_plain_[n], parts + total, st);
  finish_reduce(kind, parts, total, 0);
  c.wait_results(st);
  const double x = c.h_result()[0];
  return kind == 2 ? std::sqrt(x) : x;
}

void VariableCoeffPoissonOperator::bicgP(LevelData &p, const LevelData &v, const LevelData &r,
                                         double beta, double cc) {
  for (int n = 0; n < grid->nlocal(); ++n)
    kern::bicg_p(p.p[n], v.p[n], r.p[n], beta, cc, args_plain_[n], stream());
}

void VariableCoeffPoissonOperator::dot2(const LevelData &t, const LevelData &s, double &ts,
                                        double &tt) {
  Comm &c = *grid->comm;
  const hipStream_t st = stream();
  const int cap = std::max(1, grid->nlocal()) * kern::kMaxPartsPerBox;
  double *parts = c.d_partials(2 * cap);
  int total = 0;
  for (int n = 0; n < grid->nlocal(); ++n) {
    const int k = kern::dot2_partial(t.p[n], s.p[n], args_plain_[n], parts + total,
                                     parts + cap + total, st);
    total += k;
  }
  finish_reduce(0, parts, total, 0, false);
  finish_reduce(0, parts + cap, total, 1, true);
  c.wait_results(st);
  ts = c.h_result()[0];
  tt = c.h_result()[1];
}

double VariableCoeffPoissonOperator::dotProduct(const LevelData &x, const LevelData &y) {
  return reduce(0, x, &y);
}

unsigned long long VariableCoeffPoissonOperator::dotProductQueue(const LevelData &x,
                                                                 const LevelData &y, int slot) {
  Comm &c = *grid->comm;
  double *parts = c.d_partials(std::max(1, grid->nlocal()) * kern::kMaxPartsPerBox);
  int total = 0;
  for (int n = 0; n < grid->nlocal(); ++n)
    total += kern::reduce_partial(0, x.p[n], y.p[n], args_plain_[n], parts + total, stream());
  finish_reduce(0, parts, total, slot);
  return c.last_ticket();
}

unsigned long long VariableCoeffPoissonOperator::axpy2NormQueue(LevelData &s, const LevelData &r,
                                                                const LevelData &v, double ca,
                                                                LevelData &e, const LevelData &pt,
                                                                double cb, int ord, int slot) {
  Comm &c = *grid->comm;
  double *parts = c.d_partials(std::max(1, grid->nlocal()) * kern::kMaxPartsPerBox);
  int total = 0;
  for (int n = 0; n < grid->nlocal(); ++n)
    total += kern::axpy2_reduce(norm_kind(ord), s.p[n], r.p[n], v.p[n], ca, e.p[n], pt.p[n], cb,
                                args_plain_[n], parts + total, stream());
  finish_reduce(norm_kind(ord), parts, total, slot);
  return c.last_ticket();
}

unsigned long long VariableCoeffPoissonOperator::dot2Queue(const LevelData &t, const LevelData &s) {
  Comm &c = *grid->comm;
  const int cap = std::max(1, grid->nlocal()) * kern::kMaxPartsPerBox;
  double *parts = c.d_partials(2 * cap);
  int total = 0;
  for (int n = 0; n < grid->nlocal(); ++n)
    total += kern::dot2_partial(t.p[n], s.p[n], args_plain_[n], parts + total, parts + cap + total,
                                stream());
  finish_reduce(0, parts, total, 0, false);
  finish_reduce(0, parts + cap, total, 1, true);
  return c.last_ticket();
}

double VariableCoeffPoissonOperator::result(int slot) const {
  return grid->comm->h_result()[slot];
}

double VariableCoeffPoissonOperator::norm(const LevelData &x, int ord) {
  if (ord == 0) return reduce(3, x, nullptr);
  if (ord == 1) return reduce(1, x, nullptr);
  return std::sqrt(reduce(2, x, nullptr));
}

// --------------------------------------------------------------- factory
void VariableCoeffPoissonOperatorFactory::define(std::shared_ptr<Grid> g, const OpParams &p,
                                                 std::shared_ptr<LevelData> a,
                                                 std::shared_ptr<LevelData> b) {
  grid = std::move(g);  // Factory.cpp:59-106 (one AMR level)
  prm = p;
  m_aCoef = std::move(a);
  m_bCoef = std::move(b);
  m_coefficient_average_type = p.coefficient_average_type;  // Factory.cpp:44-46
}

std::shared_ptr<LevelData> average_coef(const LevelData &fine, std::shared_ptr<Grid> cgrid,
                                        int ratio, int harmonic) {
  auto c = std::make_shared<LevelData>(cgrid);
  const hipStream_t st = fine.grid->comm->stream();
  for (int n = 0; n < cgrid->nlocal(); ++n)
    kern::average(c->p[n], cgrid->box_args_plain(n), fine.p[n], fine.grid->box_args_plain(n), ratio,
                  harmonic, st);
  return c;
}

std::unique_ptr<VariableCoeffPoissonOperator> VariableCoeffPoissonOperatorFactory::MGnewOp(
    int depth, bool) {
  const int coarsening = 1 << depth;  // Factory.cpp:161-166
  if (coarsening > 1 && !grid->coarsenable(coarsening * VariableCoeffPoissonOperator::s_maxCoarse))
    return nullptr;  // :168-172
  auto layout = depth == 0 ? grid : grid->coarsened(coarsening);
  auto op = std::make_unique<VariableCoeffPoissonOperator>();
  OpParams p = prm;
  p.coefficient_average_type = m_coefficient_average_type;
  op->define(layout, p);  // :189
  op->m_alpha = prm.alpha;
  op->m_beta = prm.beta;
  if (depth == 0) {  // :194-197
    op->m_aCoef = m_aCoef;
    op->m_bCoef = m_bCoef;
  } else {  // :198-227: CoarseAverage straight from the AMR level, ratio 2^depth
    const int harm = m_coefficient_average_type == 1;
    op->m_aCoef = average_coef(*m_aCoef, layout, coarsening, harm);
    op->m_bCoef = average_coef(*m_bCoef, layout, coarsening, harm);
  }
  op->computeLambda();  // :229
  return op;
}

std::unique_ptr<VariableCoeffPoissonOperator> VariableCoeffPoissonOperatorFactory::AMRnewOp() {
  auto op = std::make_unique<VariableCoeffPoissonOperator>();  // Factory.cpp:236-295
  op->define(grid, prm);
  op->m_alpha = prm.alpha;
  op->m_beta = prm.beta;
  op->m_aCoef = m_aCoef;
  op->m_bCoef = m_bCoef;
  op->computeLambda();
  return op;
}

// --------------------------------------------------------------- BiCGStab
int BiCGStabSolver::solve(VariableCoeffPoissonOperator &op, LevelData &phi, const LevelData &rhs,
                          bool hom) {
  last_device = deviceApplies(op);
  if (last_device) return solveDevice(op, phi, rhs, hom);
  auto &tv = temps_[op.grid.get()];
  if (tv.empty())
    for (int i = 0; i < 9; ++i) tv.push_back(op.create());
  LevelData &R = *tv[0], &RT = *tv[1], &E = *tv[2], &P = *tv[3], &PT = *tv[4], &S = *tv[5],
            &ST = *tv[6], &T = *tv[7], &V = *tv[8];
  const int nt = prm.normType;
  op.residual(R, phi, rhs, hom);
  op.assignLocal(RT, R);
  op.setToZero(E);
  op.setToZero(PT);
  op.setToZero(ST);
  op.setToZero(P);
  op.setToZero(V);
  double rho1 = 0.0, rho2 = 0.0, alpha = 0.0, beta = 0.0, omega = 0.0;
  const double init_norm = op.norm(R, nt);
  last_init_norm = init_norm;
  double nrm = init_norm;
  int it = 0, restarts = 0;
  bool init = true;
  // With op.preCond (the bottom solver) the host waits three times per
  // iteration instead of five: the second half-step's preconditioner,
  // applyOp and dot2 are queued behind the first half-step's norm, and the
  // next iteration's <RT, R> behind the second's, each pair read back at
  // once.  The queued work only writes temporaries (ST, T) or nothing, so an
  // iteration that stops on the norm discards it and every value is the
  // unpipelined loop's.  Slots: 2 = the norms, 0 / 1 = the dots.
  // (MGIC_BICG_PIPE=0: the unpipelined loop, read per solve; the parity test
  // compares the two bit for bit)
  const char *pe = getenv("MGIC_BICG_PIPE");
  const bool pipe = !precond && !(pe && atoi(pe) == 0);
  auto norm_of = [&](int slot) {
    const double x = op.result(slot);
    return nt == 1 || nt == 0 ? x : std::sqrt(x);
  };
  auto wait = [&](unsigned long long ticket) { op.grid->comm->wait_results(op.stream(), ticket); };
  bool have_rho = false;  // the next rho1, read back with the last norm (pipelined)
  double rho_next = 0.0;
  while (it < prm.imax && nrm > prm.eps * init_norm && nrm > prm.reps) {
    ++it;
    rho2 = rho1;
    rho1 = have_rho ? rho_next : op.dotProduct(RT, R);
    have_rho = false;
    if (rho1 == 0.0) break;
    if (init) {
      op.assignLocal(P, R);
      init = false;
    } else {
      beta = (rho1 / rho2) * (alpha / omega);
      op.bicgP(P, V, R, beta, -beta * omega);  // scale(P, beta); incr(P, V, -beta omega); incr(P, R, 1)
    }
    if (precond) precond(PT, P);
    else op.preCond(PT, P);
    op.applyOp(V, PT, true);  // writes every valid cell of V
    const double m = op.dotProduct(RT, V);
    if (std::fabs(m) > prm.small * std::fabs(rho1)) {
      alpha = rho1 / m;
      double ts = 0.0, tt = 0.0;
      if (pipe) {
        op.axpy2NormQueue(S, R, V, -alpha, E, PT, alpha, nt, 2);  // S = R - alpha V; E += alpha PT
        op.preCond(ST, S);
        op.applyOp(T, ST, true);
        wait(op.dot2Queue(T, S));
        nrm = norm_of(2);
        if (nrm <= prm.eps * init_norm || nrm <= prm.reps) break;
        ts = op.result(0);
        tt = op.result(1);
      } else {
        nrm = op.axpy2Norm(S, R, V, -alpha, E, PT, alpha, nt);  // S = R - alpha V; E += alpha PT
        if (nrm <= prm.eps * init_norm || nrm <= prm.reps) break;
        if (precond) precond(ST, S);
        else op.preCond(ST, S);
        op.applyOp(T, ST, true);
        op.dot2(T, S, ts, tt);
      }
      if (tt == 0.0) break;
      omega = ts / tt;
      if (pipe) {
        op.axpy2NormQueue(R, S, T, -omega, E, ST, omega, nt, 2);  // R = S - omega T; E += omega ST
        wait(op.dotProductQueue(RT, R, 0));  // <RT, R> of the next iteration
        nrm = norm_of(2);
        rho_next = op.result(0);
        have_rho = true;
        if (omega == 0.0) break;
      } else {
        nrm = op.axpy2Norm(R, S, T, -omega, E, ST, omega, nt);  // R = S - omega T; E += omega ST
        if (omega == 0.0) break;
      }
    } else {
      if (restarts >= prm.numRestarts) break;
      ++restarts;
      op.incr(phi, E, 1.0);
      op.residual(R, phi, rhs, hom);
      op.assignLocal(RT, R);
      op.setToZero(E);
      nrm = op.norm(R, nt);
      init = true;
    }
  }
  op.incr(phi, E, 1.0);
  last_iters = it;
  return it;
}


// ------------------------------------------------------ BiCGStab on the device
BiCGStabSolver::~BiCGStabSolver() {
  for (auto &kv : dev_) {
    DevWork &d = *kv.second;
    if (d.d_st) (void)hipFree(d.d_st);
    if (d.d_parts) (void)hipFree(d.d_parts);
    if (d.d_cnt) (void)hipFree(d.d_cnt);
    if (d.h_pub) (void)hipHostFree(d.h_pub);
    if (d.h_up) (void)hipHostFree(d.h_up);
  }
}

bool BiCGStabSolver::deviceApplies(VariableCoeffPoissonOperator &op) const {
  if (precond) return false;  // the outer solve's MG preconditioner: host loop
  const char *e = getenv("MGIC_BICG_DEVICE");
  if (e && atoi(e) == 0) return false;
  const Comm &c = *op.grid->comm;
  // one rank's reductions: a single rank, or a depth gathered onto this one
  if (!(c.size() == 1 || op.owner_local >= 0)) return false;
  if (op.grid->nlocal() != 1) return false;
  const int nt = prm.normType;
  return (nt == 0 || nt == 1 || nt == 2) && op.preCondFromScaledApplies();
}

BiCGStabSolver::DevWork &BiCGStabSolver::devWork(VariableCoeffPoissonOperator &op) {
  auto &slot = dev_[op.grid.get()];
  if (!slot) {
    auto d = std::make_unique<DevWork>();
    MGIC_HIP(hipMalloc(&d->d_st, sizeof(kern::BicgState)));
    MGIC_HIP(hipMemset(d->d_st, 0, sizeof(kern::BicgState)));
    const int np = kern::bicg_dev_parts(op.boxArgsPlain(0));
    MGIC_HIP(hipMalloc(&d->d_parts, 2 * (size_t)std::max(1, np) * sizeof(double)));
    MGIC_HIP(hipMalloc(&d->d_cnt, kern::kBicgCounterWords * sizeof(unsigned int)));
    MGIC_HIP(hipMemset(d->d_cnt, 0, kern::kBicgCounterWords * sizeof(unsigned int)));
    void *p = nullptr;
    // the published state, then the sequence number the host spins on
    MGIC_HIP(hipHostMalloc(&p, sizeof(kern::BicgState) + 64, hipHostMallocCoherent));
    d->h_pub = static_cast<kern::BicgState *>(p);
    std::memset(p, 0, sizeof(kern::BicgState) + 64);
    d->h_seq = reinterpret_cast<unsigned long long *>(static_cast<char *>(p) +
                                                      sizeof(kern::BicgState) + 56);
    MGIC_HIP(hipHostMalloc(&p, sizeof(kern::BicgState), hipHostMallocDefault));
    d->h_up = static_cast<kern::BicgState *>(p);
    slot = std::move(d);
  }
  return *slot;
}

// the reductions' XCD-contiguous row deal (kern::bicg_lblock; bit-identical
// either way, 174.3 vs 175.9 us per 128^3 iteration, profiles/
// r06m_bottom_deal_ab.txt): MGIC_BICG_XCD=0 turns it off
static int bicg_xcd_deal() {
  static const int v = [] {
    const char *e = getenv("MGIC_BICG_XCD");
    return e ? (atoi(e) != 0 ? 1 : 0) : 1;
  }();
  return v;
}

static int bicg_batch() {
  const char *e = getenv("MGIC_BICG_BATCH");
  const int b = e ? atoi(e) : 4;
  return std::max(1, std::min(64, b));
}

// The loop of solve() with the scalars on the device.  The host runs the
// loop's head at a (re)start -- its test, it += 1, rho1 = <RT, R> -- and
// uploads the state; then batches of whole iterations are queued, each
// ending in a published copy of the state, two batches ahead of the host's
// wait.  A stop inside an iteration makes every later launch return at once.
// On a stop the host completes E (+ alpha PT when the stop came after the
// S update), restarts on the host when the device asks for it, and finishes
// with phi += E, as solve() does.
int BiCGStabSolver::solveDevice(VariableCoeffPoissonOperator &op, LevelData &phi,
                                const LevelData &rhs, bool hom) {
  auto &tv = temps_[op.grid.get()];
  if (tv.empty())
    for (int i = 0; i < 9; ++i) tv.push_back(op.create());
  LevelData &R = *tv[0], &RT = *tv[1], &E = *tv[2], &P = *tv[3], &PT = *tv[4], &S = *tv[5],
            &ST = *tv[6], &T = *tv[7], &V = *tv[8];
  DevWork &dw = devWork(op);
  LevelData &W = T;  // res * lambda for the two-sweep launches (T itself is never stored)
  const hipStream_t st = op.stream();
  const int nt = prm.normType, nk = norm_kind(nt);
  op.residual(R, phi, rhs, hom);
  op.assignLocal(RT, R);
  op.setToZero(E);
  op.setToZero(PT);
  op.setToZero(ST);
  op.setToZero(P);
  op.setToZero(V);
  kern::BicgState h{};
  h.init_norm = op.norm(R, nt);
  h.nrm = h.init_norm;
  h.eps = prm.eps;
  h.reps = prm.reps;
  h.small = prm.small;
  h.imax = prm.imax;
  h.num_restarts = prm.numRestarts;
  h.nt = nt;
  h.init = 1;
  h.xr = bicg_xcd_deal();
  last_init_norm = h.init_norm;
  const BoxArgs &gp = op.boxArgsPlain(0), &gh = op.boxArgs(0, true);
  const StencilCoefs sc = op.stencil();
  const double *lam = op.m_lambda->p[0], *a = op.m_aCoef->p[0], *b = op.m_bCoef->p[0];
  const int np = kern::bicg_dev_parts(gp);
  double *pa = dw.d_parts, *pb = dw.d_parts + std::max(1, np);
  kern::BicgState *d = dw.d_st;
  unsigned int *cnt = dw.d_cnt;
  const int *skip = &d->done;
  const int nb = bicg_batch();
  auto batch = [&] {
    for (int i = 0; i < nb; ++i) {
      kern::bicg_dev_p(d, P.p[0], W.p[0], V.p[0], R.p[0], lam, gp, st);
      op.preCondFromScaled(PT, W, P, skip);
      kern::bicg_dev_apply_dot(d, V.p[0], PT.p[0], RT.p[0], a, b, gh, sc, pa, cnt, st);
      kern::bicg_dev_s(d, S.p[0], W.p[0], R.p[0], V.p[0], lam, gp, nk, pa, cnt, st);
      op.preCondFromScaled(ST, W, S, skip);
      kern::bicg_dev_apply_dot2(d, ST.p[0], S.p[0], a, b, gh, sc, pa, pb, cnt, st);
      kern::bicg_dev_r(d, R.p[0], E.p[0], S.p[0], a, b, sc, PT.p[0], ST.p[0], RT.p[0], gh, nk, pa,
                       pb, cnt, st);
    }
    kern::bicg_dev_publish(d, dw.h_pub, dw.h_seq, ++dw.seq, st);
    return dw.seq;
  };
  auto wait = [&](unsigned long long want) {
    for (unsigned long long i = 0;; ++i) {
      if (__atomic_load_n(dw.h_seq, __ATOMIC_ACQUIRE) >= want) return;
      if ((i & 1023) == 1023) {
        const hipError_t e = hipStreamQuery(st);
        if (e == hipSuccess) {
          if (__atomic_load_n(dw.h_seq, __ATOMIC_ACQUIRE) >= want) return;
          throw Error(kState, "device BiCGStab: state was not published");
        }
        if (e != hipErrorNotReady) MGIC_HIP(e);
      }
      __builtin_ia32_pause();
    }
  };
  for (;;) {
    // the loop's head on the host (solve(): while-test, ++it, rho1)
    if (!(h.it < prm.imax && h.nrm > prm.eps * h.init_norm && h.nrm > prm.reps)) break;
    ++h.it;
    h.rho2 = h.rho1;
    h.rho1 = op.dotProduct(RT, R);
    if (h.rho1 == 0.0) break;
    h.done = 0;
    h.reason = kern::kBicgRun;
    h.epend = 0;
    *dw.h_up = h;
    MGIC_HIP(hipMemcpyAsync(d, dw.h_up, sizeof(h), hipMemcpyHostToDevice, st));
    unsigned long long t1 = batch(), t2 = batch();
    for (;;) {
      wait(t1);
      if (__atomic_load_n(&dw.h_pub->done, __ATOMIC_ACQUIRE)) break;
      t1 = t2;
      t2 = batch();
    }
    h = *dw.h_pub;  // frozen once done: later batches skip and publish the same words
    if (h.epend) op.incr(E, PT, h.alpha);  // the stop came after S = R - alpha V
    if (h.reason != kern::kBicgRestart) break;
    ++h.restarts;  // |m| <= small |rho1|: restart (solve()'s else branch)
    op.incr(phi, E, 1.0);
    op.residual(R, phi, rhs, hom);
    op.assignLocal(RT, R);
    op.setToZero(E);
    h.nrm = op.norm(R, nt);
    h.init = 1;
  }
  op.incr(phi, E, 1.0);
  last_iters = h.it;
  return h.it;
}

// --------------------------------------------------------------- MultiGrid
static int min_box_side(const Grid &g) {
  int m = 1 << 30;
  for (auto &b : g.boxes)
    for (int d = 0; d < 3; ++d) m = std::min(m, b.size(d));
  return m;
}

void MultiGrid::define(VariableCoeffPoissonOperatorFactory &factory, const MGParams &p) {
  prm = p;
  bottom.prm = p.bicg;
  levels_.clear();
  {
    Level L0;
    L0.op = factory.MGnewOp(0);
    levels_.push_back(std::move(L0));
  }
  bool agg_chain = false;
  for (int d = 1;; ++d) {
    if (prm.max_depth >= 0 && d > prm.max_depth) break;
    Level L;
    if (!agg_chain) {
      auto op = factory.MGnewOp(d);
      if (!op) break;
      const bool do_agg = prm.agglomerate_below > 0 && op->grid->boxes.size() > 1 &&
                          min_box_side(*op->grid) < prm.agglomerate_below;
      if (!do_agg) {
        L.e = op->create();
        L.r = op->create();
        L.op = std::move(op);
      } else {
        // gather this depth onto one box owned by rank 0
        const Grid &dg = *op->grid;
        bool per[3] = {dg.periodic[0], dg.periodic[1], dg.periodic[2]};
        auto ag = std::make_shared<Grid>(dg.comm, dg.domain, per, dg.dx, std::vector<Box>{dg.domain},
                                         std::vector<int>{0});
        auto a = std::make_shared<LevelData>(ag);
        auto b = std::make_shared<LevelData>(ag);
        auto to_agg = build_copy_plan(dg, *ag, true, false);
        to_agg->execute(*dg.comm, op->m_aCoef->d_tab, a->d_tab, dg.comm->stream());
        to_agg->execute(*dg.comm, op->m_bCoef->d_tab, b->d_tab, dg.comm->stream());
        auto aop = std::make_unique<VariableCoeffPoissonOperator>();
        aop->define(ag, op->prm);
        aop->m_aCoef = a;
        aop->m_bCoef = b;
        aop->owner_local = 0;  // the bottom solve is rank 0's alone
        aop->computeLambda();
        L.r_stage = op->create();
        L.e_stage = op->create();
        L.restrict_plan = build_copy_plan(dg, *ag, true, false);
        L.prolong_plan = build_copy_plan(*ag, dg, true, true);
        L.e = aop->create();
        L.r = aop->create();
        L.op = std::move(aop);
        L.agg = true;
        L.owner = 0;
        agg_chain = true;
      }
    } else {
      const VariableCoeffPoissonOperator &prev = *levels_.back().op;
      if (!prev.grid->coarsenable(2 * VariableCoeffPoissonOperator::s_maxCoarse)) break;
      auto cg = prev.grid->coarsened(2);
      auto op = std::make_unique<VariableCoeffPoissonOperator>();
      op->define(cg, prev.prm);
      const int harm = prev.prm.coefficient_average_type == 1;
      if (factory.grid->coarsenable(1 << d)) {
        // same coefficients as MGnewOp(d) would give: average from the AMR
        // level, then gather
        auto dgrid = factory.grid->coarsened(1 << d);
        auto da = average_coef(*factory.m_aCoef, dgrid, 1 << d, harm);
        auto db = average_coef(*factory.m_bCoef, dgrid, 1 << d, harm);
        auto a = std::make_shared<LevelData>(cg);
        auto b = std::make_shared<LevelData>(cg);
        auto pl = build_copy_plan(*dgrid, *cg, true, false);
        pl->execute(*cg->comm, da->d_tab, a->d_tab, cg->comm->stream());
        pl->execute(*cg->comm, db->d_tab, b->d_tab, cg->comm->stream());
        MGIC_HIP(hipStreamSynchronize(cg->comm->stream()));
        op->m_aCoef = a;
        op->m_bCoef = b;
      } else {
        op->m_aCoef = average_coef(*prev.m_aCoef, cg, 2, harm);
        op->m_bCoef = average_coef(*prev.m_bCoef, cg, 2, harm);
      }
      op->owner_local = 0;
      op->computeLambda();
      L.e = op->create();
      L.r = op->create();
      L.op = std::move(op);
      L.owner = 0;
    }
    levels_.push_back(std::move(L));
  }
  MGIC_HIP(hipStreamSynchronize(levels_[0].op->stream()));
}

MultiGrid::~MultiGrid() {
  for (hipEvent_t ev : bt_ev_) (void)hipEventDestroy(ev);
}

void MultiGrid::bottom_timer(bool on) {
  bt_on_ = on;
  bt_used_ = 0;
  bt_iters_ = bt_solves_ = 0;
  bt_r0_min_ = bt_r0_max_ = 0.0;
}

long MultiGrid::bottom_iters(double *r0_min, double *r0_max) const {
  if (r0_min) *r0_min = bt_r0_min_;
  if (r0_max) *r0_max = bt_r0_max_;
  return bt_iters_;
}

int MultiGrid::bottom_replay(int n, double *ms, int *iters, double *r0) {
  *ms = 0.0;
  *iters = 0;
  *r0 = 0.0;
  const int d = (int)levels_.size() - 1;
  if (n <= 0 || !bt_filled_ || !runs(d)) return 0;
  VariableCoeffPoissonOperator &op = *levels_[d].op;
  LevelData &e = *levels_[d].e, &r = *levels_[d].r;
  const bool was_on = bt_on_;
  const size_t used0 = bt_used_;
  const long it0 = bt_iters_, sv0 = bt_solves_;
  const double lo0 = bt_r0_min_, hi0 = bt_r0_max_;
  bt_on_ = true;
  for (int i = 0; i < n; ++i) {
    op.setToZero(e);
    bottom_solve(op, e, r);
  }
  MGIC_HIP(hipEventSynchronize(bt_ev_[bt_used_ - 1]));
  for (size_t i = used0; i + 1 < bt_used_; i += 2) {
    float t = 0.f;
    MGIC_HIP(hipEventElapsedTime(&t, bt_ev_[i], bt_ev_[i + 1]));
    *ms += t;
  }
  *iters = bottom.last_iters;
  *r0 = bottom.last_init_norm;
  bt_used_ = used0;
  bt_on_ = was_on;
  bt_iters_ = it0;
  bt_solves_ = sv0;
  bt_r0_min_ = lo0;
  bt_r0_max_ = hi0;
  return n;
}

double MultiGrid::bottom_ms(int *calls) {
  double tot = 0.0;
  if (bt_used_) MGIC_HIP(hipEventSynchronize(bt_ev_[bt_used_ - 1]));
  for (size_t i = 0; i + 1 < bt_used_; i += 2) {
    float ms = 0.f;
    MGIC_HIP(hipEventElapsedTime(&ms, bt_ev_[i], bt_ev_[i + 1]));
    tot += ms;
  }
  if (calls) *calls = (int)(bt_used_ / 2);
  return tot;
}

// the bottom BiCGStab (Main_PoissonSolver.cpp:103-117), between events when
// the bottom timer is on
void MultiGrid::bottom_solve(VariableCoeffPoissonOperator &op, LevelData &e, LevelData &r) {
  auto mark = [&] {
    if (bt_used_ == bt_ev_.size()) {
      hipEvent_t ev;
      MGIC_HIP(hipEventCreate(&ev));
      bt_ev_.push_back(ev);
    }
    MGIC_HIP(hipEventRecord(bt_ev_[bt_used_++], op.stream()));
  };
  bt_filled_ = true;
  if (!bt_on_) {
    bottom.solve(op, e, r, true);
    return;
  }
  const size_t open = bt_used_;
  mark();
  try {
    bottom.solve(op, e, r, true);
  } catch (...) {
    bt_used_ = open;  // keep the start/end pairs aligned
    throw;
  }
  mark();
  const double r0 = bottom.last_init_norm;
  bt_r0_min_ = bt_solves_ ? std::min(bt_r0_min_, r0) : r0;
  bt_r0_max_ = bt_solves_ ? std::max(bt_r0_max_, r0) : r0;
  bt_iters_ += bottom.last_iters;
  ++bt_solves_;
}

void MultiGrid::cycle(int d, LevelData &e, LevelData &r, bool e_zero, LevelData *phi_acc,
                      bool halo_out, const std::function<void()> *before_phi) {
  VariableCoeffPoissonOperator &op = *levels_[d].op;
  const hipStream_t st = op.stream();
  // r's ghost layer once per level visit (the fused sweeps' red ring reads
  // it; r does not change between pre- and post-smoothing)
  int rf = 0;
  if (op.grid->has_memory_faces() && op.fusedSmootherApplies() && op.prm.relax_mode == 1) {
    op.rhsHalo(r, st);
    rf = kRhsHaloReady;
  }
  const int out = halo_out ? kHaloOut : 0;
  if (d == (int)levels_.size() - 1) {  // bottom
    if (prm.bottom_solver == 1) {
      if (e_zero) op.setToZero(e);
      bottom_solve(op, e, r);
      if (halo_out) e.exchange(st);
    } else if (e_zero) {
      op.relaxFromZero(e, r, prm.n_bottom, rf | out);
    } else {
      op.relaxFlags(e, r, prm.n_bottom, rf | out);
    }
    if (phi_acc) {
      if (before_phi) (*before_phi)();
      op.incr(*phi_acc, e, 1.0);
    }
    return;
  }
  // pre-smoothing leaves e's face ghosts exchanged for the restriction, or
  // restricts in its last sweep
  Level &N = levels_[d + 1];
  LevelData &rc = N.agg ? *N.r_stage : *N.r;
  if (!op.relaxRestrict(e, r, prm.n_pre, e_zero, rf | kHaloOut, rc)) {
    op.restrictResidual(rc, e, r, false);
  }
  if (N.agg) N.restrict_plan->execute(*op.grid->comm, N.r_stage->d_tab, N.r->d_tab, st);
  // coarse correction e_c = 0 (folded into its first sweep when possible);
  // its last relax exchanges e_c's ghosts for the linear prolongation
  // a gathered coarse depth runs on its owner only; the other ranks go on to
  // the scatter, whose receives wait (on the device) for the owner's result
  const bool coarse_out = !N.agg && op.prm.prolong_type == 1;
  if (runs(d + 1))
    for (int c = 0; c < prm.cycles; ++c)
      cycle(d + 1, *N.e, *N.r, c == 0, nullptr, coarse_out && c == prm.cycles - 1);
  if (!N.agg) {
    op.prolongIncrementFilled(e, *N.e);
  } else {
    N.prolong_plan->execute(*op.grid->comm, N.e->d_tab, N.e_stage->d_tab, st);
    op.prolongIncrementFilled(e, *N.e_stage);
  }
  if (phi_acc)  // phi += e folded into the last post-smoothing sweep
    op.relaxAccumulate(e, r, prm.n_post, *phi_acc, rf, before_phi);
  else
    op.relaxFlags(e, r, prm.n_post, rf | out);
}

void MultiGrid::fmg(LevelData &e0, LevelData &r0, LevelData &phi, int ncycles) {
  const int D = depths();
  auto E = [&](int d) -> LevelData & { return d == 0 ? e0 : *levels_[d].e; };
  auto Rr = [&](int d) -> LevelData & { return d == 0 ? r0 : *levels_[d].r; };
  if (D == 1) {  // one depth: the bottom solve is the whole cycle
    cycle(0, e0, r0, true, &phi);
    return;
  }
  // right-hand sides: r_{d+1} = restrictResidual of a zero correction; into
  // a gathered depth through its stage and the gather (every rank), below it
  // on the owner only
  for (int d = 0; d + 1 < D && runs(d); ++d) {
    Level &N = levels_[d + 1];
    const hipStream_t st = levels_[d].op->stream();
    levels_[d].op->setToZero(E(d));
    levels_[d].op->restrictResidual(N.agg ? *N.r_stage : Rr(d + 1), E(d), Rr(d), true);
    if (N.agg) N.restrict_plan->execute(*levels_[d].op->grid->comm, N.r_stage->d_tab, N.r->d_tab, st);
  }
  // coarsest depth from zero, then up with e_d = P e_{d+1} as the start
  if (runs(D - 1)) {
    VariableCoeffPoissonOperator &op = *levels_[D - 1].op;
    if (prm.bottom_solver == 1) {
      op.setToZero(E(D - 1));
      bottom_solve(op, E(D - 1), Rr(D - 1));
    } else {
      op.relaxFromZero(E(D - 1), Rr(D - 1), prm.n_bottom);
    }
  }
  for (int d = D - 2; d >= 0; --d) {
    Level &N = levels_[d + 1];
    VariableCoeffPoissonOperator &op = *levels_[d].op;
    if (N.agg) {  // scatter the gathered correction (every rank)
      N.prolong_plan->execute(*op.grid->comm, N.e->d_tab, N.e_stage->d_tab, op.stream());
    }
    if (!runs(d)) continue;
    op.setToZero(E(d));
    if (N.agg) op.prolongIncrementFilled(E(d), *N.e_stage);
    else op.prolongIncrement(E(d), E(d + 1));
    for (int c = 0; c < ncycles; ++c)
      cycle(d, E(d), Rr(d), false, d == 0 && c == ncycles - 1 ? &phi : nullptr);
  }
}

// --------------------------------------------------------------- AMRMultiGrid
void AMRMultiGrid::define(VariableCoeffPoissonOperatorFactory &factory, const MGParams &p) {
  mg.define(factory, p);
  corr_ = mg.op(0).create();
}

double AMRMultiGrid::iteration(LevelData &phi, const LevelData &rhs, LevelData &resid,
                               int normType, bool homogeneous) {
  VariableCoeffPoissonOperator &op0 = mg.op(0);
  mg.oneCycleFromZeroInto(*corr_, resid, phi);  // e = 0; oneCycle(e, r); phi += e
  return op0.residualNorm(resid, phi, rhs, homogeneous, normType);
}

void AMRMultiGrid::iterations(LevelData &phi, const LevelData &rhs, LevelData &resid, int count,
                              int normType, bool homogeneous, double *norms) {
  VariableCoeffPoissonOperator &op0 = mg.op(0);
  // iteration i's norm is taken (host) once iteration i+1's V-cycle has been
  // queued up to its first phi-writing launch -- the GPU runs that part while
  // the host waits -- and before that launch is queued
  int pending = -1;  // the iteration whose norm is not yet taken
  unsigned long long ticket = 0;
  double now = 0.0;
  const std::function<void()> take = [&] {
    if (pending < 0) return;
    const double v = ticket ? op0.residualNormTake(ticket) : now;
    if (norms) norms[pending] = v;
    pending = -1;
  };
  for (int i = 0; i < count; ++i) {
    mg.oneCycleFromZeroInto(*corr_, resid, phi, &take);
    take();  // (a V-cycle with no launch to hook)
    ticket = op0.residualNormQueue(resid, phi, rhs, homogeneous, normType, &now);
    pending = i;
  }
  take();
}

double AMRMultiGrid::fmg(LevelData &phi, const LevelData &rhs, LevelData &resid, int normType,
                         bool homogeneous, int ncycles) {
  VariableCoeffPoissonOperator &op0 = mg.op(0);
  mg.fmg(*corr_, resid, phi, ncycles);
  return op0.residualNorm(resid, phi, rhs, homogeneous, normType);
}

void AMRMultiGrid::precondition(LevelData &e, const LevelData &r, int iters) {
  VariableCoeffPoissonOperator &op0 = mg.op(0);
  if (!pre_resid_) pre_resid_ = op0.create();
  op0.setToZero(e);
  // e = 0, so the first residual r - L(0) (homogeneous BC) is r itself: the
  // first cycle runs on r (its ghosts are the only cells it writes); the
  // residual after the last cycle is not needed
  LevelData &r0 = const_cast<LevelData &>(r);
  for (int i = 0; i < iters; ++i) {
    if (i > 0) op0.residual(*pre_resid_, e, r, true);
    mg.oneCycleFromZeroInto(*corr_, i == 0 ? r0 : *pre_resid_, e);
  }
}

int AMRMultiGrid::solve(LevelData &phi, const LevelData &rhs, const SolveParams &p,
                        double *final_norm) {
  VariableCoeffPoissonOperator &op0 = mg.op(0);
  outer_.prm = mg.prm.bicg;  // reps, small, restarts: BiCGStabSolver defaults
  outer_.prm.imax = p.max_iterations;
  outer_.prm.eps = p.tolerance;
  outer_.prm.normType = p.norm_type;
  const int iters = std::max(1, p.num_mg_iterations);
  outer_.precond = [this, iters](LevelData &e, const LevelData &r) { precondition(e, r, iters); };
  const int it = outer_.solve(op0, phi, rhs, false);
  if (!pre_resid_) pre_resid_ = op0.create();
  op0.residual(*pre_resid_, phi, rhs, false);
  const double nrm = op0.norm(*pre_resid_, p.norm_type);
  if (final_norm) *final_norm = nrm;
  return it;
}

double AMRMultiGrid::initResidual(LevelData &phi, const LevelData &rhs, LevelData &resid,
                                  int normType, bool homogeneous) {
  VariableCoeffPoissonOperator &op0 = mg.op(0);
  return op0.residualNorm(resid, phi, rhs, homogeneous, normType);
}

}  // namespace mgic
