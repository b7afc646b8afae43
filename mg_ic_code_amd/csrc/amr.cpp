// amr.cpp -- AMR levels > 0: coarse-fine interface, AMRLevelOp multi-level
// operators, AMR V-cycle (see amr.hpp).
#include "amr.hpp"

#include <algorithm>
#include <cmath>

#include "kernels.hpp"

namespace mgic {

void cf_homogeneous(CFLevel &cf, LevelData &u, hipStream_t st) { cf.interp(u, nullptr, st); }

namespace {

bool coarsenable2(const Box &b) {
  for (int d = 0; d < 3; ++d)
    if ((b.lo[d] & 1) || ((b.hi[d] + 1) & 1)) return false;
  return true;
}

// is the box (clipped to the domain in non-periodic directions) covered by
// the union of the (disjoint) boxes?
bool covered_by(Box r, const Grid &g) {
  for (int d = 0; d < 3; ++d) {  // (periodic images: the in-domain part is checked)
    r.lo[d] = std::max(r.lo[d], g.domain.lo[d]);
    r.hi[d] = std::min(r.hi[d], g.domain.hi[d]);
  }
  long v = 0;
  for (const Box &b : g.boxes) v += r.intersect(b).ncells();
  return v == r.ncells();
}

}  // namespace

CFLevel::CFLevel(std::shared_ptr<Grid> f, std::shared_ptr<Grid> c)
    : fine(std::move(f)), coarse(std::move(c)) {
  for (int d = 0; d < 3; ++d) {
    MGIC_CHECK(fine->domain.lo[d] == 2 * coarse->domain.lo[d] &&
                   fine->domain.hi[d] + 1 == 2 * (coarse->domain.hi[d] + 1),
               "AMR: a level's domain must be the coarser domain refined by 2");
    MGIC_CHECK(fine->periodic[d] == coarse->periodic[d], "AMR: periodicity differs between levels");
  }
  std::vector<Box> cb;
  for (const Box &b : fine->boxes) {
    MGIC_CHECK(coarsenable2(b), "AMR: fine boxes must be coarsenable by 2");
    const Box c2 = b.coarsened(2);
    Box g = c2;
    for (int d = 0; d < 3; ++d) {
      g.lo[d] -= 1;
      g.hi[d] += 1;
    }
    MGIC_CHECK(covered_by(g, *coarse),
               "AMR: fine boxes are not properly nested in the coarser level (1 coarse cell)");
    for (int d = 0; d < 3; ++d)
      MGIC_CHECK(b.size(d) >= 2, "AMR: fine boxes need 2 cells in every direction");
    cb.push_back(c2);
  }
  bool per[3] = {coarse->periodic[0], coarse->periodic[1], coarse->periodic[2]};
  cfine = std::make_shared<Grid>(coarse->comm, coarse->domain, per, coarse->dx, cb, fine->owners);
  stage = std::make_unique<LevelData>(cfine);
  stage_plan = build_copy_plan(*coarse, *cfine, true, false, true, 1);
  down_plan = build_copy_plan(*cfine, *coarse, true, false, true, 0);
  ncov = (int)cb.size();
  std::vector<int> flat;
  for (const Box &b : cb)
    for (int d = 0; d < 6; ++d) flat.push_back(d < 3 ? b.lo[d] : b.hi[d - 3]);
  MGIC_HIP(hipMalloc(&d_cov, sizeof(int) * flat.size()));
  MGIC_HIP(hipMemcpy(d_cov, flat.data(), sizeof(int) * flat.size(), hipMemcpyHostToDevice));
}

CFLevel::~CFLevel() {
  if (d_cov) (void)hipFree(d_cov);
}

void CFLevel::interp(LevelData &u, const LevelData *crs, hipStream_t st) {
  if (crs) stage_plan->execute(*coarse->comm, crs->d_tab, stage->d_tab, st);
  for (int n = 0; n < fine->nlocal(); ++n) {
    const Box &b = fine->geom[n].valid;
    const Box &c = cfine->geom[n].valid;
    kern::CFArgs a{};
    for (int d = 0; d < 3; ++d) {
      a.flo[d] = b.lo[d];
      a.clo[d] = c.lo[d];
      a.cdom_lo[d] = coarse->domain.lo[d];
      a.cdom_hi[d] = coarse->domain.hi[d];
      a.periodic[d] = coarse->periodic[d] ? 1 : 0;
    }
    a.csy = cfine->geom[n].sy;
    a.csz = cfine->geom[n].sz;
    a.ncov = ncov;
    a.cov = d_cov;
    const BoxArgs g = fine->box_args_plain(n);
    for (int face = 0; face < 6; ++face) {
      const int dir = face >> 1, side = face & 1;
      const bool domain_face = !fine->periodic[dir] &&
                               (side ? b.hi[dir] == fine->domain.hi[dir] : b.lo[dir] == fine->domain.lo[dir]);
      if (domain_face) continue;  // the physical BC (folded into the stencil kernels)
      a.face = face;
      kern::cf_interp(u.p[n], stage->p[n], g, a, crs == nullptr, st);
    }
  }
}

void CFLevel::averageDown(LevelData &crs, const LevelData &f, hipStream_t st) {
  for (int n = 0; n < fine->nlocal(); ++n)
    kern::average(stage->p[n], cfine->box_args_plain(n), f.p[n], fine->box_args_plain(n), 2, 0, st);
  down_plan->execute(*coarse->comm, stage->d_tab, crs.d_tab, st);
}

void CFLevel::prolongConstant(LevelData &f, const LevelData &crs, hipStream_t st) {
  stage_plan->execute(*coarse->comm, crs.d_tab, stage->d_tab, st);
  const int a0[3] = {0, 0, 0};
  for (int n = 0; n < fine->nlocal(); ++n)
    kern::prolong(f.p[n], fine->box_args_plain(n), stage->p[n], cfine->box_args_plain(n), a0, a0, 0,
                  st);
}

void CFLevel::zeroCovered(LevelData &crs, hipStream_t st) {
  stage->set_zero_all(st);
  down_plan->execute(*coarse->comm, stage->d_tab, crs.d_tab, st);
}

// ------------------------------------------------------------------ solver
void AMRSolver::define(const std::vector<AMRLevelSpec> &levels, const OpParams &prm,
                       const MGParams &base) {
  MGIC_CHECK(!levels.empty(), "AMR: no levels");
  MGIC_CHECK(levels[0].grid->tiles_domain(), "AMR: level 0 must tile its domain");
  mgp_ = base;
  fac0_.define(levels[0].grid, prm, levels[0].a, levels[0].b);
  base_.define(fac0_, base);
  L_.clear();
  L_.resize(levels.size());
  for (size_t l = 0; l < levels.size(); ++l) {
    Level &V = L_[l];
    V.grid = levels[l].grid;
    if (l > 0) {
      MGIC_CHECK(std::abs(V.grid->dx * 2 - levels[l - 1].grid->dx) <= 1e-12 * V.grid->dx,
                 "AMR: dx must halve from level to level");
      V.cf = std::make_shared<CFLevel>(V.grid, levels[l - 1].grid);
      V.op = std::make_unique<VariableCoeffPoissonOperator>();
      V.op->define(V.grid, prm);  // AMRnewOp for ref > 0 (Factory.cpp:236-295)
      check_same_layout(*V.grid, *levels[l].a, "aCoef");
      check_same_layout(*V.grid, *levels[l].b, "bCoef");
      V.op->m_aCoef = levels[l].a;
      V.op->m_bCoef = levels[l].b;
      V.op->m_dxCrse = levels[l - 1].grid->dx;
      V.op->computeLambda();
      V.op->cf = V.cf;
    }
    V.corr = std::make_unique<LevelData>(V.grid);
    V.res = std::make_unique<LevelData>(V.grid);
    V.dcorr = std::make_unique<LevelData>(V.grid);
    V.tmp = std::make_unique<LevelData>(V.grid);
  }
}

void AMRSolver::AMROperator(int l, LevelData &Lphi, LevelData &phi, const LevelData *phiC,
                            bool hom) {
  VariableCoeffPoissonOperator &o = op(l);
  if (l > 0) L_[l].cf->interp(phi, phiC, o.stream());  // [Chombo] coarseFineInterp
  o.applyOpI(Lphi, phi, hom);                           // reflux: a no-op (.cpp:264-271)
}

void AMRSolver::AMRResidual(int l, LevelData &r, LevelData &phi, const LevelData *phiC,
                            const LevelData &rhs, bool hom) {
  VariableCoeffPoissonOperator &o = op(l);
  if (l > 0) L_[l].cf->interp(phi, phiC, o.stream());
  o.residualI(r, phi, rhs, hom);  // r = rhs - L(phi)
}

void AMRSolver::AMRRestrict(int l, LevelData &resC, const LevelData &res, LevelData &corr,
                            const LevelData *corrC) {
  MGIC_CHECK(l > 0, "AMRRestrict needs a coarser level");
  Level &V = L_[l];
  const hipStream_t st = V.op->stream();
  V.cf->interp(corr, corrC, st);
  V.op->residualI(*V.tmp, corr, res, true);  // res - L(corr), homogeneous physical BC
  V.cf->averageDown(resC, *V.tmp, st);       // CoarseAverage onto the covered cells
}

void AMRSolver::AMRProlong(int l, LevelData &corr, const LevelData &corrC) {
  MGIC_CHECK(l > 0, "AMRProlong needs a coarser level");
  L_[l].cf->prolongConstant(corr, corrC, L_[l].op->stream());
}

void AMRSolver::AMRUpdateResidual(int l, LevelData &res, LevelData &corr, const LevelData *corrC) {
  MGIC_CHECK(l > 0, "AMRUpdateResidual needs a coarser level");
  Level &V = L_[l];
  V.cf->interp(corr, corrC, V.op->stream());
  V.op->residualI(*V.tmp, corr, res, true);
  V.op->assignLocal(res, *V.tmp);
}

void AMRSolver::cycle(int l) {
  if (l == 0) {  // l_base: the level's own MultiGrid V-cycle from zero
    base_.oneCycleFromZero(*L_[0].corr, *L_[0].res);
    return;
  }
  Level &F = L_[l], &C = L_[l - 1];
  // downsweep: smooth (homogeneous CF), residual of the correction onto the
  // covered coarse cells
  F.op->relaxFromZero(*F.corr, *F.res, mgp_.n_pre);
  AMRRestrict(l, *C.res, *F.res, *F.corr, nullptr);
  cycle(l - 1);
  // upsweep: e += P(e_c), r -= L(e) with the CF ghosts of e from e_c, smooth
  // the rest and add
  AMRProlong(l, *F.corr, *C.corr);
  AMRUpdateResidual(l, *F.res, *F.corr, C.corr.get());
  F.op->relaxFromZero(*F.dcorr, *F.res, mgp_.n_post);
  F.op->incr(*F.corr, *F.dcorr, 1.0);
}

double AMRSolver::initResidual(std::vector<LevelData *> &phi, const std::vector<LevelData *> &rhs,
                               int normType) {
  const int n = numLevels();
  MGIC_CHECK((int)phi.size() == n && (int)rhs.size() == n, "AMR: one field per level");
  for (int l = 0; l < n; ++l)
    AMRResidual(l, *L_[l].res, *phi[l], l ? phi[l - 1] : nullptr, *rhs[l], false);
  for (int l = 1; l < n; ++l) L_[l].cf->zeroCovered(*L_[l - 1].res, op(l).stream());
  if (normType < 0) return -1.0;
  double m = 0.0;
  for (int l = 0; l < n; ++l) m = std::max(m, op(l).norm(*L_[l].res, normType));
  return m;
}

double AMRSolver::iteration(std::vector<LevelData *> &phi, const std::vector<LevelData *> &rhs,
                            int normType) {
  const int n = numLevels();
  cycle(n - 1);
  for (int l = 0; l < n; ++l) op(l).incr(*phi[l], *L_[l].corr, 1.0);
  for (int l = n - 1; l > 0; --l) L_[l].cf->averageDown(*phi[l - 1], *phi[l], op(l).stream());
  return initResidual(phi, rhs, normType);
}

// ------------------------------------------------ MultilevelLinearOp + BiCGStab
double AMRSolver::weight(int l) const {
  const double dx = L_[l].grid->dx;
  return dx * dx * dx;
}

void AMRSolver::zeroCovered(std::vector<LevelData *> &x) {
  for (int l = 1; l < numLevels(); ++l) L_[l].cf->zeroCovered(*x[l - 1], op(l).stream());
}

void AMRSolver::applyOp(std::vector<LevelData *> &lhs, std::vector<LevelData *> &x, bool hom) {
  const int n = numLevels();
  MGIC_CHECK((int)lhs.size() == n && (int)x.size() == n, "AMR: one field per level");
  for (int l = 0; l < n; ++l) AMROperator(l, *lhs[l], *x[l], l ? x[l - 1] : nullptr, hom);
  zeroCovered(lhs);
}

void AMRSolver::residual(std::vector<LevelData *> &r, std::vector<LevelData *> &phi,
                         const std::vector<LevelData *> &rhs, bool hom) {
  const int n = numLevels();
  MGIC_CHECK((int)r.size() == n && (int)phi.size() == n && (int)rhs.size() == n,
             "AMR: one field per level");
  for (int l = 0; l < n; ++l) AMRResidual(l, *r[l], *phi[l], l ? phi[l - 1] : nullptr, *rhs[l], hom);
  zeroCovered(r);
}

double AMRSolver::dotProduct(const std::vector<LevelData *> &x, const std::vector<LevelData *> &y) {
  double s = 0.0;
  for (int l = 0; l < numLevels(); ++l) s += weight(l) * op(l).dotProduct(*x[l], *y[l]);
  return s;
}

double AMRSolver::norm(const std::vector<LevelData *> &x, int ord) {
  double s = 0.0;
  for (int l = 0; l < numLevels(); ++l) {
    const double v = op(l).norm(*x[l], ord);
    if (ord == 0) s = std::max(s, v);
    else if (ord == 1) s += weight(l) * v;
    else s += weight(l) * (v * v);
  }
  return ord == 0 || ord == 1 ? s : std::sqrt(s);
}

std::vector<LevelData *> AMRSolver::masked(const std::vector<LevelData *> &x) {
  const int n = numLevels();
  MGIC_CHECK((int)x.size() == n, "AMR: one field per level");
  if ((int)mask_.size() != n - 1) {
    mask_.clear();
    for (int l = 0; l + 1 < n; ++l) mask_.push_back(op(l).create());
  }
  std::vector<LevelData *> m(x.begin(), x.end());
  for (int l = 0; l + 1 < n; ++l) {
    op(l).assignLocal(*mask_[l], *x[l]);
    L_[l + 1].cf->zeroCovered(*mask_[l], op(l).stream());
    m[l] = mask_[l].get();
  }
  return m;
}

double AMRSolver::compositeNorm(const std::vector<LevelData *> &x, int ord) {
  return norm(masked(x), ord);
}

double AMRSolver::compositeDot(const std::vector<LevelData *> &x,
                               const std::vector<LevelData *> &y) {
  return dotProduct(masked(x), y);
}

double AMRSolver::compositeSum(const std::vector<LevelData *> &x) {
  // computeSum: sum over the uncovered cells of every level, times dx_l^3
  // (the level sum as a dot product with a field of ones)
  std::vector<LevelData *> m = masked(x);
  std::vector<LevelData *> ones = bicgVec(9);
  double s = 0.0;
  for (int l = 0; l < numLevels(); ++l) {
    op(l).setVal(*ones[l], 1.0);
    s += weight(l) * op(l).dotProduct(*m[l], *ones[l]);
  }
  return s;
}

std::vector<LevelData *> AMRSolver::bicgVec(int i) {
  while ((int)bicg_.size() <= i) {
    std::vector<std::unique_ptr<LevelData>> v;
    for (int l = 0; l < numLevels(); ++l) v.push_back(op(l).create());
    bicg_.push_back(std::move(v));
  }
  std::vector<LevelData *> out;
  for (auto &f : bicg_[i]) out.push_back(f.get());
  return out;
}

void AMRSolver::precondition(std::vector<LevelData *> &e, const std::vector<LevelData *> &r,
                             int iters) {
  const int n = numLevels();
  MGIC_CHECK((int)e.size() == n && (int)r.size() == n, "AMR: one field per level");
  for (int l = 0; l < n; ++l) op(l).setToZero(*e[l]);
  for (int i = 0; i < iters; ++i) {
    // the first residual r - L(0) (homogeneous BCs) is r itself (covered
    // cells already zero); later ones are recomputed from e
    for (int l = 0; l < n; ++l) {
      if (i == 0) op(l).assignLocal(*L_[l].res, *r[l]);
      else AMRResidual(l, *L_[l].res, *e[l], l ? e[l - 1] : nullptr, *r[l], true);
    }
    if (i > 0)
      for (int l = 1; l < n; ++l) L_[l].cf->zeroCovered(*L_[l - 1].res, op(l).stream());
    cycle(n - 1);
    for (int l = 0; l < n; ++l) op(l).incr(*e[l], *L_[l].corr, 1.0);
    for (int l = n - 1; l > 0; --l) L_[l].cf->averageDown(*e[l - 1], *e[l], op(l).stream());
  }
}

int AMRSolver::solve(std::vector<LevelData *> &phi, const std::vector<LevelData *> &rhs,
                     const SolveParams &p, double *final_norm) {
  const int n = numLevels();
  MGIC_CHECK((int)phi.size() == n && (int)rhs.size() == n, "AMR: one field per level");
  BiCGStabParams prm = mgp_.bicg;  // reps, small, restarts: BiCGStabSolver defaults
  prm.imax = p.max_iterations;
  prm.eps = p.tolerance;
  prm.normType = p.norm_type;
  const int iters = std::max(1, p.num_mg_iterations);
  std::vector<LevelData *> R = bicgVec(0), RT = bicgVec(1), E = bicgVec(2), P = bicgVec(3),
                           PT = bicgVec(4), S = bicgVec(5), ST = bicgVec(6), T = bicgVec(7),
                           V = bicgVec(8);
  auto each = [&](auto f) {
    for (int l = 0; l < n; ++l) f(l, op(l));
  };
  const int nt = prm.normType;
  residual(R, phi, rhs, false);
  each([&](int l, VariableCoeffPoissonOperator &o) {
    o.assignLocal(*RT[l], *R[l]);
    o.setToZero(*E[l]);
    o.setToZero(*PT[l]);
    o.setToZero(*ST[l]);
    o.setToZero(*P[l]);
    o.setToZero(*V[l]);
  });
  double rho1 = 0.0, rho2 = 0.0, alpha = 0.0, beta = 0.0, omega = 0.0;
  const double init_norm = norm(R, nt);
  double nrm = init_norm;
  int it = 0, restarts = 0;
  bool init = true;
  while (it < prm.imax && nrm > prm.eps * init_norm && nrm > prm.reps) {
    ++it;
    rho2 = rho1;
    rho1 = dotProduct(RT, R);
    if (rho1 == 0.0) break;
    if (init) {
      each([&](int l, VariableCoeffPoissonOperator &o) { o.assignLocal(*P[l], *R[l]); });
      init = false;
    } else {
      beta = (rho1 / rho2) * (alpha / omega);
      each([&](int l, VariableCoeffPoissonOperator &o) {
        o.bicgP(*P[l], *V[l], *R[l], beta, -beta * omega);
      });
    }
    precondition(PT, P, iters);
    applyOp(V, PT, true);
    const double m = dotProduct(RT, V);
    if (std::fabs(m) > prm.small * std::fabs(rho1)) {
      alpha = rho1 / m;
      // S = R - alpha V; E += alpha PT (the level norms combined as norm())
      double s = 0.0;
      each([&](int l, VariableCoeffPoissonOperator &o) {
        const double v = o.axpy2Norm(*S[l], *R[l], *V[l], -alpha, *E[l], *PT[l], alpha, nt);
        s = nt == 0 ? std::max(s, v) : s + weight(l) * (nt == 1 ? v : v * v);
      });
      nrm = nt == 0 || nt == 1 ? s : std::sqrt(s);
      if (nrm <= prm.eps * init_norm || nrm <= prm.reps) break;
      precondition(ST, S, iters);
      applyOp(T, ST, true);
      double ts = 0.0, tt = 0.0;
      each([&](int l, VariableCoeffPoissonOperator &o) {
        double a = 0.0, b = 0.0;
        o.dot2(*T[l], *S[l], a, b);
        ts += weight(l) * a;
        tt += weight(l) * b;
      });
      if (tt == 0.0) break;
      omega = ts / tt;
      s = 0.0;
      each([&](int l, VariableCoeffPoissonOperator &o) {
        const double v = o.axpy2Norm(*R[l], *S[l], *T[l], -omega, *E[l], *ST[l], omega, nt);
        s = nt == 0 ? std::max(s, v) : s + weight(l) * (nt == 1 ? v : v * v);
      });
      nrm = nt == 0 || nt == 1 ? s : std::sqrt(s);
      if (omega == 0.0) break;
    } else {
      if (restarts >= prm.numRestarts) break;
      ++restarts;
      each([&](int l, VariableCoeffPoissonOperator &o) { o.incr(*phi[l], *E[l], 1.0); });
      residual(R, phi, rhs, false);
      each([&](int l, VariableCoeffPoissonOperator &o) {
        o.assignLocal(*RT[l], *R[l]);
        o.setToZero(*E[l]);
      });
      nrm = norm(R, nt);
      init = true;
    }
  }
  each([&](int l, VariableCoeffPoissonOperator &o) { o.incr(*phi[l], *E[l], 1.0); });
  if (final_norm) {
    residual(R, phi, rhs, false);
    *final_norm = norm(R, nt);
  }
  return it;
}

}  // namespace mgic
