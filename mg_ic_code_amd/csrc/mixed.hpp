// mixed.hpp -- mixed-precision V-cycle: fp32 smoother / fp64 residual
// (BASELINE config C5, SURVEY §8(a) a1 "C5 ... fp32 smoother", §8(d) "fp32
// smoother: 24 B/cell per pass").
//
// Iterative refinement around an fp32 V-cycle: the fine-level residual
// r = rhs - L(phi) is computed in fp64 (VCCOMPUTERES3D, .ChF:283-339) and
// rounded to fp32 once; the correction equation L e = r is then cycled
// entirely in fp32 -- GSRB sweeps (GSRBHELMHOLTZVC3D arithmetic in float),
// restrictResidual and prolongIncrement in float, coefficients rounded from
// the fp64 hierarchy (averaged in fp64 first) -- and phi += e accumulates in
// fp64, folded into the last post-smoothing sweep.  Same schedule as
// MultiGrid::cycle (pre-relax from zero, restrict, recurse, prolong,
// post-relax; relax(n_bottom) at the coarsest depth), same halo
// bookkeeping, same agglomeration (depths gathered onto rank 0, which alone
// relaxes them: the restriction is gathered and the correction scattered as
// fp32 messages) and, in deep-halo mode, the same schedule (two sweeps per
// 4-deep shell exchange, both in one two-sweep launch); no BiCGStab bottom
// (relax only).
//
// Also the full-multigrid (FMG) start the C5 config names: restrict the
// fine residual to every depth, relax at the coarsest, then at each finer
// depth prolong the coarser solution as the initial correction and run
// `ncycles` V-cycles on it; phi += e at the end.
#pragma once

#include "op.hpp"

namespace mgic {

class MixedMultiGrid {
 public:
  // builds the fp64 MultiGrid hierarchy (grids, averaged coefficients) from
  // the factory and the fp32 copies the cycle runs on
  void define(VariableCoeffPoissonOperatorFactory &factory, const MGParams &prm);
  // r32 = fp32(rhs - L(phi)); returns norm of the fp64 residual when
  // normType >= 0 (resid64 receives it; may be null otherwise)
  double initResidual(LevelData &phi, const LevelData &rhs, LevelData *resid64, int normType);
  // one fp32 V-cycle on the current residual, phi += e (fp64), then the
  // residual of the new phi as in initResidual
  double iteration(LevelData &phi, const LevelData &rhs, LevelData *resid64, int normType);
  // FMG from the current residual: phi += FMG(e), ncycles V-cycles per
  // depth; then the new residual as in initResidual
  double fmg(LevelData &phi, const LevelData &rhs, LevelData *resid64, int normType, int ncycles);
  int depths() const { return mg.depths(); }
  MultiGrid mg;  // the fp64 hierarchy (operators, grids, coefficients)

 private:
  struct LevelF {
    std::unique_ptr<LevelDataF> e, r, tmp, a, b;
    // the first gathered depth: the restriction before the gather and the
    // correction after the scatter, on the finer layout coarsened
    std::unique_ptr<LevelDataF> r_stage, e_stage;
    StencilCoefs s;
    bool halo = false;
    bool deep = false;  // exchanged faces in deep-halo mode (4-deep shells)
  };
  std::vector<LevelF> lf_;
  void cycle(int d, bool e_zero, LevelData *phi_acc, bool halo_out);
  void relax(int d, LevelDataF &e, const LevelDataF &r, int n, bool zero_in, LevelData *acc,
             bool halo_out);
  void prolongInto(int d);  // e[d] += P e[d+1] (scattered first when d+1 is gathered)
  void restrictInto(int d);  // r[d+1] = R(r[d] - L e[d]) (gathered when d+1 is gathered)
  double residualF(LevelData &phi, const LevelData &rhs, LevelData *resid64, int normType);
};

}  // namespace mgic
