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
};

}  // namespace mgic
