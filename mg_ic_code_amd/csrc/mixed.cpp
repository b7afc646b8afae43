// mixed.cpp -- the mixed-precision V-cycle and FMG (see mixed.hpp).
#include "mixed.hpp"

#include "kernels.hpp"

namespace mgic {

// the deep-halo schedule's shell depth (op.cpp kDeepDepth)
static constexpr int kDeepShell = 4;

void MixedMultiGrid::define(VariableCoeffPoissonOperatorFactory &factory, const MGParams &p) {
  MGParams q = p;
  q.bottom_solver = 0;  // relax(n_bottom) at the coarsest depth
  mg.define(factory, q);
  lf_.clear();
  lf_.resize(mg.depths());
  for (int d = 0; d < mg.depths(); ++d) {
    VariableCoeffPoissonOperator &op = mg.op(d);
    const hipStream_t st = op.stream();
    LevelF &L = lf_[d];
    if (mg.agglomerated(d)) {  // every rank takes part in the gather / scatter
      L.r_stage = std::make_unique<LevelDataF>(mg.stage_grid(d));
      L.e_stage = std::make_unique<LevelDataF>(mg.stage_grid(d));
    }
    // (a gathered depth on another rank: empty fields, never touched)
    L.e = std::make_unique<LevelDataF>(op.grid);
    L.r = std::make_unique<LevelDataF>(op.grid);
    L.tmp = std::make_unique<LevelDataF>(op.grid);
    L.a = std::make_unique<LevelDataF>(op.grid);
    L.b = std::make_unique<LevelDataF>(op.grid);
    if (!mg.runs(d)) continue;
    L.s = op.stencil();
    L.halo = op.grid->has_memory_faces();
    L.deep = L.halo && op.deepApplies();
    // coefficients: the fp64 hierarchy (averaged in fp64) rounded once, with
    // the ghost layers the sweeps' rings read on exchanged faces (layer 1;
    // the 4-deep shell in deep-halo mode), exchanged first
    const int gd = L.deep ? kDeepShell : 1;
    if (L.deep) {
      op.m_aCoef->exchange_shell(st, kDeepShell);
      op.m_bCoef->exchange_shell(st, kDeepShell);
    } else {
      op.m_aCoef->exchange(st);
      op.m_bCoef->exchange(st);
    }
    for (int n = 0; n < op.grid->nlocal(); ++n) {
      const BoxArgs &g = op.boxArgs(n, true);
      kern::to_float(L.a->p[n], op.m_aCoef->p[n], g, gd, st);
      kern::to_float(L.b->p[n], op.m_bCoef->p[n], g, gd, st);
    }
  }
}

double MixedMultiGrid::residualF(LevelData &phi, const LevelData &rhs, LevelData *resid64,
                                 int normType) {
  VariableCoeffPoissonOperator &op = mg.op(0);
  const hipStream_t st = op.stream();
  phi.exchange(st);  // .cpp:48
  const StencilCoefs s = op.stencil();
  LevelDataF &r = *lf_[0].r;
  for (int n = 0; n < op.grid->nlocal(); ++n)
    kern::residual_to_f(r.p[n], phi.p[n], rhs.p[n], op.m_aCoef->p[n], op.m_bCoef->p[n],
                        op.boxArgs(n, false), s, st);
  if (normType < 0) return -1.0;
  MGIC_CHECK(resid64 != nullptr, "mixed V-cycle: a norm needs the fp64 residual field");
  op.residual(*resid64, phi, rhs, false);
  return op.norm(*resid64, normType);
}

double MixedMultiGrid::initResidual(LevelData &phi, const LevelData &rhs, LevelData *resid64,
                                    int normType) {
  return residualF(phi, rhs, resid64, normType);
}

double MixedMultiGrid::iteration(LevelData &phi, const LevelData &rhs, LevelData *resid64,
                                 int normType) {
  cycle(0, true, &phi, false);  // e = 0; oneCycle(e, r) in fp32; phi += e
  return residualF(phi, rhs, resid64, normType);
}

void MixedMultiGrid::relax(int d, LevelDataF &e, const LevelDataF &r, int n, bool zero_in,
                           LevelData *acc, bool halo_out) {
  VariableCoeffPoissonOperator &op = mg.op(d);
  const hipStream_t st = op.stream();
  LevelF &L = lf_[d];
  const int kind = op.prm.fused_smoother ? op.prm.fused_smoother : 1;
  if (n <= 0) {
    MGIC_CHECK(!acc, "mixed V-cycle: no sweep to fold phi += e into");
    if (zero_in)
      for (int b = 0; b < op.grid->nlocal(); ++b)
        MGIC_HIP(hipMemsetAsync(e.base[b], 0, sizeof(float) * (size_t)op.grid->geom[b].total, st));
    if (halo_out && L.halo) e.exchange(st);
    return;
  }
  LevelDataF *src = &e, *dst = L.tmp.get();
  if (acc && zero_in && n == 1) {  // a single sweep on a zero input: sweep, then phi += e
    for (int b = 0; b < op.grid->nlocal(); ++b) {
      kern::gsrb_sweep_fused_f(e.p[b], dst->p[b], r.p[b], L.a->p[b], L.b->p[b], op.boxArgs(b, true),
                               L.s, true, nullptr, kind, st);
      kern::incr_f(acc->p[b], e.p[b], op.boxArgs(b, true), st);
    }
    return;
  }
  // two sweeps per launch (the temporally blocked kernel, smoother_tb.hip)
  // on levels without exchanged faces, and on exchanged layouts in deep-halo
  // mode (a 4-deep shell before each pair: the kernel's rings run onto it);
  // the last pair folds phi += e into fp64 (round 5; a pair cannot start
  // from zero and accumulate, so that one case takes two single sweeps)
  bool two = (!L.halo || L.deep) && n >= 2;
  for (int b = 0; two && b < op.grid->nlocal(); ++b)
    two = kern::gsrb_sweep_tb2_applies(op.boxArgs(b, true), L.s, kind);
  for (int it = 0; it < n;) {
    const bool zin = zero_in && it == 0;
    const int left = n - it;
    const int k = two && left >= 2 && !(zin && left == 2 && acc) ? 2 : 1;
    const bool last = it + k == n;
    if (L.halo && !zin) src->exchange_shell(st, k == 2 ? kDeepShell : 2);
    for (int b = 0; b < op.grid->nlocal(); ++b) {
      const long nc = op.grid->geom[b].valid.ncells();
      prof_mark(st, nc, true, 2 * k);
      if (k == 2)
        kern::gsrb_sweep_tb2_f(dst->p[b], src->p[b], r.p[b], L.a->p[b], op.boxArgs(b, true), L.s,
                               zin, last && acc ? acc->p[b] : nullptr, st);
      else
        kern::gsrb_sweep_fused_f(dst->p[b], src->p[b], r.p[b], L.a->p[b], L.b->p[b],
                                 op.boxArgs(b, true), L.s, zin, last && acc ? acc->p[b] : nullptr,
                                 kind, st);
      prof_mark(st, nc, false, 2 * k);
    }
    std::swap(src, dst);
    it += k;
  }
  if (acc) return;
  if (src != &e)
    for (int b = 0; b < op.grid->nlocal(); ++b) kern::copy_f(e.p[b], src->p[b], op.boxArgs(b, true), st);
  if (halo_out && L.halo) e.exchange(st);
}

void MixedMultiGrid::prolongInto(int d) {
  VariableCoeffPoissonOperator &op = mg.op(d);
  const hipStream_t st = op.stream();
  LevelF &N = lf_[d + 1];
  // a gathered coarser depth: its correction scattered back onto this
  // layout coarsened (valid cells and face ghosts) first
  const bool agg = mg.agglomerated(d + 1);
  if (agg) mg.scatter_plan(d + 1).execute_f(*op.grid->comm, N.e->d_tab, N.e_stage->d_tab, st);
  const Grid &cg = agg ? *mg.stage_grid(d + 1) : *mg.op(d + 1).grid;
  LevelDataF &ec = agg ? *N.e_stage : *N.e;
  for (int n = 0; n < op.grid->nlocal(); ++n) {
    const Box &cb = cg.geom[n].valid;
    int alo[3], ahi[3];
    for (int k = 0; k < 3; ++k) {
      alo[k] = cg.periodic[k] || cb.lo[k] > cg.domain.lo[k];
      ahi[k] = cg.periodic[k] || cb.hi[k] < cg.domain.hi[k];
    }
    kern::prolong_f(lf_[d].e->p[n], op.boxArgs(n, true), ec.p[n], cg.box_args_plain(n),
                    alo, ahi, op.prm.prolong_type, st);
  }
}

void MixedMultiGrid::restrictInto(int d) {
  VariableCoeffPoissonOperator &op = mg.op(d);
  const hipStream_t st = op.stream();
  LevelF &L = lf_[d], &N = lf_[d + 1];
  const bool agg = mg.agglomerated(d + 1);
  const Grid &cg = agg ? *mg.stage_grid(d + 1) : *mg.op(d + 1).grid;
  LevelDataF &rc = agg ? *N.r_stage : *N.r;
  for (int n = 0; n < op.grid->nlocal(); ++n)
    kern::restrict_residual_f(rc.p[n], cg.box_args_plain(n), L.e->p[n], L.r->p[n], L.a->p[n],
                              L.b->p[n], op.boxArgs(n, true), L.s, st);
  if (agg) mg.gather_plan(d + 1).execute_f(*op.grid->comm, N.r_stage->d_tab, N.r->d_tab, st);
}

void MixedMultiGrid::cycle(int d, bool e_zero, LevelData *phi_acc, bool halo_out) {
  VariableCoeffPoissonOperator &op = mg.op(d);
  const hipStream_t st = op.stream();
  LevelF &L = lf_[d];
  // r's ghosts once per level visit (layer 1, or the 4-deep shell)
  if (L.halo) {
    if (L.deep) L.r->exchange_shell(st, kDeepShell);
    else L.r->exchange(st);
  }
  const MGParams &prm = mg.prm;
  if (d == mg.depths() - 1) {  // bottom: relax(n_bottom)
    relax(d, *L.e, *L.r, prm.n_bottom, e_zero, phi_acc, halo_out);
    return;
  }
  relax(d, *L.e, *L.r, prm.n_pre, e_zero, nullptr, true);
  restrictInto(d);
  // a gathered coarser depth runs on its owner only (the others wait for
  // the scatter); its face ghosts come with the scatter
  const bool agg = mg.agglomerated(d + 1);
  if (mg.runs(d + 1))
    for (int c = 0; c < prm.cycles; ++c)
      cycle(d + 1, c == 0, nullptr, !agg && op.prm.prolong_type == 1 && c == prm.cycles - 1);
  prolongInto(d);
  relax(d, *L.e, *L.r, prm.n_post, false, phi_acc, halo_out);
}

double MixedMultiGrid::fmg(LevelData &phi, const LevelData &rhs, LevelData *resid64,
                           int normType, int ncycles) {
  // the residual equation's right-hand side at every depth: r_{d+1} = R(r_d)
  // (restrictResidual of a zero correction)
  const int D = mg.depths();
  for (int d = 0; d + 1 < D && mg.runs(d); ++d) {
    VariableCoeffPoissonOperator &op = mg.op(d);
    const hipStream_t st = op.stream();
    LevelF &L = lf_[d];
    for (int b = 0; b < op.grid->nlocal(); ++b)
      MGIC_HIP(hipMemsetAsync(L.e->base[b], 0, sizeof(float) * (size_t)op.grid->geom[b].total, st));
    if (L.halo) L.r->exchange(st);
    restrictInto(d);
  }
  if (D == 1) {  // a single depth: the bottom relax is the whole solve
    relax(0, *lf_[0].e, *lf_[0].r, mg.prm.n_bottom, true, &phi, false);
    return residualF(phi, rhs, resid64, normType);
  }
  // coarsest: relax from zero (on its owner when gathered); then up: e_d =
  // P e_{d+1}, ncycles V-cycles
  if (mg.runs(D - 1)) {
    LevelF &B = lf_[D - 1];
    if (B.halo) {
      if (B.deep) B.r->exchange_shell(mg.op(D - 1).stream(), kDeepShell);
      else B.r->exchange(mg.op(D - 1).stream());
    }
    relax(D - 1, *B.e, *B.r, mg.prm.n_bottom, true, nullptr,
          !mg.agglomerated(D - 1) && mg.op(D - 1).prm.prolong_type == 1);
  }
  for (int d = D - 2; d >= 0; --d) {
    VariableCoeffPoissonOperator &op = mg.op(d);
    const hipStream_t st = op.stream();
    if (!mg.runs(d)) {  // a gathered depth held by another rank
      continue;
    }
    for (int b = 0; b < op.grid->nlocal(); ++b)
      MGIC_HIP(hipMemsetAsync(lf_[d].e->base[b], 0, sizeof(float) * (size_t)op.grid->geom[b].total, st));
    prolongInto(d);
    for (int c = 0; c < ncycles; ++c) {
      const bool last = d == 0 && c == ncycles - 1;
      cycle(d, false, last ? &phi : nullptr, d > 0 && c == ncycles - 1 && op.prm.prolong_type == 1);
    }
  }
  return residualF(phi, rhs, resid64, normType);
}

}  // namespace mgic
