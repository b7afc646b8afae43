// amr.hpp -- AMR levels > 0: coarse-fine interpolation,
// the AMRLevelOp multi-level operators, and a multi-level AMR V-cycle.
//
// The reference's operator inherits these from [Chombo] AMRPoissonOp (not in
// the tree): QuadCFInterp / homogeneousCFInterp (called by the reference at
// VariableCoeffPoissonOperator.cpp:156,296), AMROperator / AMRResidual (reflux
// is a no-op in the reference, .cpp:264-271), AMRRestrict (CoarseAverage of
// the fine residual of the correction onto the covered coarse cells),
// AMRProlong (piecewise constant), AMRUpdateResidual, and AMRMultiGrid's
// multi-level cycle, for the refinement ratio 2 the factory's AMRnewOp sets
// up (VariableCoeffPoissonOperatorFactory.cpp:236-295).  All restated, so
// parity unpinned; the GPU is bit-identical to the numpy restatement in
// oracle/amr.py.
#pragma once

#include "op.hpp"

namespace mgic {

// One AMR level's interface with the next coarser level (ratio 2).
struct CFLevel {
  std::shared_ptr<Grid> fine, coarse;
  std::shared_ptr<Grid> cfine;           // fine boxes coarsened by 2 (coarse index space)
  std::unique_ptr<CopyPlan> stage_plan;  // coarse valid -> cfine valid + 1-deep shell
  std::unique_ptr<CopyPlan> down_plan;   // cfine valid -> coarse valid (the covered cells)
  std::unique_ptr<LevelData> stage;      // on cfine
  int *d_cov = nullptr;                  // cfine boxes (device) for the covered test
  int ncov = 0;
  CFLevel(std::shared_ptr<Grid> fine, std::shared_ptr<Grid> coarse);
  ~CFLevel();
  CFLevel(const CFLevel &) = delete;
  CFLevel &operator=(const CFLevel &) = delete;
  // QuadCFInterp: the ghosts of every fine-box face that is not a domain face
  // from `coarse` (inhomogeneous) or from zero (coarse == nullptr); an
  // exchange afterwards overwrites the fine-fine parts
  void interp(LevelData &u, const LevelData *coarse, hipStream_t st);
  // coarse covered cells = CoarseAverage(fine) (sum of the 8 children / 8)
  void averageDown(LevelData &coarse, const LevelData &fine, hipStream_t st);
  // fine += piecewise-constant prolongation of coarse
  void prolongConstant(LevelData &fine, const LevelData &coarse, hipStream_t st);
  void zeroCovered(LevelData &coarse, hipStream_t st);
};

struct AMRLevelSpec {
  std::shared_ptr<Grid> grid;
  std::shared_ptr<LevelData> a, b;  // aCoef, bCoef on that level
};

class AMRSolver {
 public:
  // levels[0] is the coarsest (its boxes tile the domain); each finer
  // level's domain is the coarser one refined by 2 and its boxes are
  // properly nested (the coarsened boxes grown by one coarse cell lie in the
  // coarser level's boxes, or outside a non-periodic domain)
  void define(const std::vector<AMRLevelSpec> &levels, const OpParams &prm, const MGParams &base);
  int numLevels() const { return (int)L_.size(); }
  VariableCoeffPoissonOperator &op(int l) { return l == 0 ? base_.op(0) : *L_[l].op; }
  CFLevel &cf(int l) { return *L_[l].cf; }

  // AMRLevelOp pieces on level l (phiCoarse / corrCoarse == nullptr: none /
  // a zero coarse field)
  void AMROperator(int l, LevelData &Lphi, LevelData &phi, const LevelData *phiCoarse, bool hom);
  void AMRResidual(int l, LevelData &r, LevelData &phi, const LevelData *phiCoarse,
                   const LevelData &rhs, bool hom);
  void AMRRestrict(int l, LevelData &resCoarse, const LevelData &res, LevelData &corr,
                   const LevelData *corrCoarse);
  void AMRProlong(int l, LevelData &corr, const LevelData &corrCoarse);
  void AMRUpdateResidual(int l, LevelData &res, LevelData &corr, const LevelData *corrCoarse);

  // AMRMultiGrid on the whole hierarchy: the composite residual (covered
  // coarse cells zeroed) -> its norm (max over levels, if normType >= 0);
  // an iteration = one AMR V-cycle on the residuals, phi += e on every
  // level, average phi down, new residuals
  double initResidual(std::vector<LevelData *> &phi, const std::vector<LevelData *> &rhs,
                      int normType);
  double iteration(std::vector<LevelData *> &phi, const std::vector<LevelData *> &rhs,
                   int normType);
  LevelData &residual(int l) { return *L_[l].res; }

  // ---- MultilevelLinearOp<FArrayBox> over the hierarchy (Main_PoissonSolver.
  // cpp:103-117,169-184 with max_level > 0).  Vectors are one LevelData per
  // level.  [Chombo] semantics restated (MultilevelLinearOp is not in the
  // tree; parity unpinned, pinned to oracle/amr.py): the operator is
  // AMROperator on every level (CF ghosts from the next coarser level of the
  // same vector, reflux a no-op) with the covered coarse cells of the result
  // zeroed, as the composite residual is; dot products and norms therefore
  // see only uncovered cells wherever one operand is an operator result or a
  // residual.  dotProduct = sum over levels of dx_l^3 * levelDot; norm 0 =
  // max over levels; norm 1 / 2 = the dx_l^3-weighted sum / root of sums.
  void applyOp(std::vector<LevelData *> &lhs, std::vector<LevelData *> &x, bool hom);
  void residual(std::vector<LevelData *> &r, std::vector<LevelData *> &phi,
                const std::vector<LevelData *> &rhs, bool hom);
  double dotProduct(const std::vector<LevelData *> &x, const std::vector<LevelData *> &y);
  double norm(const std::vector<LevelData *> &x, int ord);
  // computeNorm / computeSum (the reference's NL-loop diagnostics,
  // Main_PoissonSolver.cpp:144-145,208-209): covered coarse cells masked,
  // each level weighted by dx_l^3; ord 0 = max norm, 1 / 2 = L1 / L2
  double compositeNorm(const std::vector<LevelData *> &x, int ord);
  double compositeSum(const std::vector<LevelData *> &x);
  // the dot product with x's covered coarse cells masked (the public entry
  // point: its operands need not have zero covered cells); the solver's own
  // dotProduct skips the mask where an operand's covered cells are zero
  double compositeDot(const std::vector<LevelData *> &x, const std::vector<LevelData *> &y);
  // MultilevelLinearOp::preCond: e = 0 on every level, then `iters` AMR
  // V-cycle iterations on (e, r) with homogeneous physical BCs (r's covered
  // coarse cells are zero; e's are the average of the finer level after
  // every iteration)
  void precondition(std::vector<LevelData *> &e, const std::vector<LevelData *> &r, int iters);
  // BiCGStabSolver<Vector<LevelData*>>::solve (the control flow of the
  // single-level BiCGStabSolver::solve) over applyOp / precondition;
  // returns the iterations, *final_norm = norm(rhs - L(phi), norm_type)
  int solve(std::vector<LevelData *> &phi, const std::vector<LevelData *> &rhs,
            const SolveParams &p, double *final_norm);

 private:
  struct Level {
    std::shared_ptr<Grid> grid;
    std::unique_ptr<VariableCoeffPoissonOperator> op;  // levels > 0
    std::shared_ptr<CFLevel> cf;                       // levels > 0
    std::unique_ptr<LevelData> corr, res, dcorr, tmp;
  };
  std::vector<Level> L_;
  VariableCoeffPoissonOperatorFactory fac0_;
  MultiGrid base_;  // level 0's MG hierarchy (the l_base solve)
  MGParams mgp_;
  void cycle(int l);
  // multi-level temporaries of solve() (9 vectors) and the masked copies of
  // compositeNorm / compositeSum
  std::vector<std::vector<std::unique_ptr<LevelData>>> bicg_;
  std::vector<std::unique_ptr<LevelData>> mask_;
  double weight(int l) const;  // dx_l^3
  std::vector<LevelData *> bicgVec(int i);
  void zeroCovered(std::vector<LevelData *> &x);
  std::vector<LevelData *> masked(const std::vector<LevelData *> &x);
};

}  // namespace mgic
