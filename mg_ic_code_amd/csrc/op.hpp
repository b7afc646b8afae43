// op.hpp -- the reference's operator-plugin API, MI355X-native.
//
// VariableCoeffPoissonOperator mirrors Source/VariableCoeffPoissonOperator.H
// (method names, argument meaning, lazy lambda), VariableCoeffPoisson
// OperatorFactory mirrors Source/VariableCoeffPoissonOperatorFactory.H, and
// MultiGrid / BiCGStabSolver / AMRMultiGrid re-host the [Chombo] drivers
// that call them (MultiGrid::oneCycle, BiCGStabSolver::solve,
// AMRMultiGrid::solve on one AMR level).  Everything runs on the Comm's HIP
// stream; host code only sequences kernels (and reads back the scalars the
// Krylov bottom solver branches on).
#pragma once

#include <functional>

#include "level.hpp"

namespace mgic {

struct CFLevel;  // amr.hpp: the coarse-fine interface of an AMR level > 0
// homogeneousCFInterp: the CF ghosts of u from a zero coarse field
void cf_homogeneous(CFLevel &cf, LevelData &u, hipStream_t st);

// ParseBC state (SetBCs.cpp GlobalBCRS + ParmParse bc_value) and the
// operator constants/options of params.txt.
struct OpParams {
  double alpha = 0.0, beta = -1.0;  // factory defaults (Factory.cpp:317-322)
  int bc_lo[3] = {0, 0, 0};
  int bc_hi[3] = {0, 0, 0};
  double bc_value = 0.0;
  int coefficient_average_type = 0;  // 0 arithmetic (default), 1 harmonic
  int prolong_type = 1;              // 0 piecewise constant, 1 linear
  int relax_mode = 1;                // [Chombo] s_relaxMode: 1 GSRB, 4 Jacobi
  int fused_smoother = 1;            // fused red+black sweep: 0 off (per-colour passes),
                                     // 1 by box size, 2 z-streaming kernel, 3 3D-block kernel
  int deep_halo = 0;                 // fused sweeps on exchanged layouts: 4-deep ghost
                                     // shells, two sweeps per exchange (the first on the
                                     // box grown by 2 across exchanged faces); 0 off,
                                     // 1 every level, 2 levels of boxes <= 128^3
};

// relax flags (MultiGrid::cycle): the caller exchanged rhs's ghost layer
// already / wants the result's face ghosts exchanged on return
enum RelaxFlags { kRhsHaloReady = 1, kHaloOut = 2 };

class VariableCoeffPoissonOperator {
 public:
  static int s_maxCoarse;  // [Chombo] AMRPoissonOp::s_maxCoarse

  // AMRPoissonOp::define(grids, dx, domain, bc, exchangeCopier, cfregion)
  void define(std::shared_ptr<Grid> grid, const OpParams &prm);
  hipStream_t stream() const { return grid->comm->stream(); }

  // --- AMRLevelOp / MGLevelOp overrides (VariableCoeffPoissonOperator.H:39-90)
  void residualI(LevelData &lhs, LevelData &dpsi, const LevelData &rhs, bool homogeneous);
  // residual + norm(lhs, normType) (normType < 0: no norm, returns -1); the
  // max norm (0) is taken inside the residual launch
  double residualNorm(LevelData &lhs, LevelData &dpsi, const LevelData &rhs, bool homogeneous,
                      int normType);
  // the same, queued: returns a ticket for residualNormTake, or 0 with the
  // value in *now when it was computed synchronously (normType 1 / 2, no
  // fused residual) or not at all (normType < 0: -1).  The value travels in
  // its own result slot (kNormSlot), so reductions queued after it (a
  // BiCGStab bottom's) do not overwrite it before it is taken.
  unsigned long long residualNormQueue(LevelData &lhs, LevelData &dpsi, const LevelData &rhs,
                                       bool homogeneous, int normType, double *now);
  double residualNormTake(unsigned long long ticket);
  static constexpr int kNormSlot = 3;
  void residual(LevelData &lhs, LevelData &dpsi, const LevelData &rhs, bool homogeneous) {
    residualI(lhs, dpsi, rhs, homogeneous);
  }
  void preCond(LevelData &correction, const LevelData &residual);
  void applyOpI(LevelData &lhs, LevelData &dpsi, bool homogeneous);
  void applyOp(LevelData &lhs, LevelData &dpsi, bool homogeneous) { applyOpI(lhs, dpsi, homogeneous); }
  void applyOpNoBoundary(LevelData &lhs, LevelData &dpsi);
  void restrictResidual(LevelData &resCoarse, LevelData &dpsiFine, const LevelData &rhsFine,
                        bool exchange = true);
  // [Chombo] AMRPoissonOp::prolongIncrement (inherited)
  void prolongIncrement(LevelData &phiThisLevel, LevelData &correctCoarse);
  // same, with the coarse ghost layer already filled by the caller
  void prolongIncrementFilled(LevelData &phiThisLevel, const LevelData &correctCoarse);
  void setAlphaAndBeta(double alpha, double beta);
  void setCoefs(std::shared_ptr<LevelData> aCoef, std::shared_ptr<LevelData> bCoef, double alpha,
                double beta);
  void resetLambda();
  void computeLambda();
  void reflux() {}   // not implemented in the reference either (.cpp:264-271)
  void getFlux() {}  // (.cpp:389-397)
  void setTime(double t);
  void relax(LevelData &e, const LevelData &r, int iterations);  // [Chombo] AMRPoissonOp::relax
  void levelGSRB(LevelData &dpsi, const LevelData &rhs);
  void levelJacobi(LevelData &dpsi, const LevelData &rhs);
  [[noreturn]] void levelMultiColor(LevelData &, const LevelData &);
  [[noreturn]] void looseGSRB(LevelData &, const LevelData &);
  [[noreturn]] void overlapGSRB(LevelData &, const LevelData &);
  [[noreturn]] void levelGSRBLazy(LevelData &, const LevelData &);
  // ParseBC on every box (m_bc): writes the domain-face ghost layers
  void fillBC(LevelData &u, bool homogeneous);

  // --- LinearOp<LevelData> vector interface ([Chombo] AMRPoissonOp)
  std::unique_ptr<LevelData> create() const { return std::make_unique<LevelData>(grid); }
  void setToZero(LevelData &x);
  void assignLocal(LevelData &lhs, const LevelData &rhs);
  void assign(LevelData &lhs, const LevelData &rhs) { assignLocal(lhs, rhs); }
  void incr(LevelData &lhs, const LevelData &x, double scale);
  void axby(LevelData &lhs, const LevelData &x, const LevelData &y, double a, double b);
  void scale(LevelData &lhs, double s);
  void mult(LevelData &lhs, const LevelData &x);  // lhs *= x (FArrayBox::mult)
  void setVal(LevelData &lhs, double v);
  double dotProduct(const LevelData &x, const LevelData &y);
  double norm(const LevelData &x, int ord);
  // BiCGStab's fused updates (bit-identical to the separate passes):
  // s = r + ca v; e += cb pt; returns norm(s, ord)
  double axpy2Norm(LevelData &s, const LevelData &r, const LevelData &v, double ca, LevelData &e,
                   const LevelData &pt, double cb, int ord);
  // p = p beta + c v + r (scale(P, beta); incr(P, V, c); incr(P, R, 1))
  void bicgP(LevelData &p, const LevelData &v, const LevelData &r, double beta, double c);
  // dot(t, s) and dot(t, t) in one pass
  void dot2(const LevelData &t, const LevelData &s, double &ts, double &tt);
  // the same reductions queued: each publishes into result slot `slot` (dot2:
  // slots 0 and 1) and returns the ticket of its readback; result(slot) reads
  // it once Comm::wait_results has seen that ticket (the BiCGStab loop waits
  // once for several queued reductions)
  unsigned long long dotProductQueue(const LevelData &x, const LevelData &y, int slot);
  unsigned long long axpy2NormQueue(LevelData &s, const LevelData &r, const LevelData &v, double ca,
                                    LevelData &e, const LevelData &pt, double cb, int ord, int slot);
  unsigned long long dot2Queue(const LevelData &t, const LevelData &s);
  double result(int slot) const;

  // state (public as in the reference: m_aCoef, m_bCoef, m_lambda)
  std::shared_ptr<Grid> grid;
  OpParams prm;
  double m_alpha = 0.0, m_beta = -1.0, m_dx = 1.0, m_dxCrse = -1.0, m_time = 0.0;
  std::shared_ptr<LevelData> m_aCoef, m_bCoef;
  std::unique_ptr<LevelData> m_lambda;
  bool m_lambdaNeedsResetting = true;
  bool coef_ghosts_ = false;  // aCoef/bCoef face ghosts exchanged (fused sweep)
  // AMR level > 0 (AMRnewOp with a coarser level): levelGSRB and
  // restrictResidual fill the CF ghosts by homogeneousCFInterp first
  // (.cpp:156, :296); the per-colour kernels are used on such levels
  std::shared_ptr<CFLevel> cf;
  bool b_const_ = false;      // bCoef holds one value everywhere (all ranks)
  double b_val_ = 1.0;
  bool rcp_fast_ = false;     // StencilCoefs::rcp_fast (lambda's range, all ranks)
  bool rcp_fast32_ = false;   // StencilCoefs::rcp_fast32
  // a gathered MG depth (every box on one rank): its reductions are that
  // rank's alone -- no allreduce, no other rank involved -- and any other rank
  // that asks for one gets an error (MultiGrid never does); -1: collective
  int owner_local = -1;


 private:
  StencilCoefs coefs();  // refreshes lambda / coefficient state first
  const BoxArgs &args(int n, bool homogeneous);
  void build_args();
  double reduce(int kind, const LevelData &x, const LevelData *y);
  // partials (count `total`, per-box blocks) -> final -> allreduce -> host
  void finish_reduce(int kind, double *parts, int total, int slot, bool last = true);
  std::vector<BoxArgs> args_hom_, args_inhom_, args_plain_;
  // AMR level > 0 with isolated patches: args_hom_ with the coarse-fine
  // faces marked kBcCFHom, for the 3D-block fused sweep (cfFusedApplies)
  std::vector<BoxArgs> args_cf_;
  int cf_fused_ = -1;  // -1 undecided, 0 / 1
  bool cfFusedApplies();
  std::unique_ptr<LevelData> jac_tmp_;
  std::unique_ptr<LevelData> sweep_tmp_;  // out-of-place buffer of the fused sweep

 public:
  bool fusedSmootherApplies();
  // kernel arguments for other drivers (the mixed-precision V-cycle, the
  // device-side BiCGStab)
  const BoxArgs &boxArgs(int n, bool homogeneous) { return args(n, homogeneous); }
  const BoxArgs &boxArgsPlain(int n) const { return args_plain_[n]; }
  // preCond(cor, res) as ONE two-sweep launch from w = res * lambda, which
  // the caller has written (the device-side BiCGStab fuses that product into
  // its vector updates): whether it applies (one box, domain faces only, the
  // fused GSRB taking the two-sweep kernel for relax(cor, res, 2)), and the
  // launch (skip: as gsrb_sweep_tb2's).  Bit-identical to preCond.
  bool preCondFromScaledApplies();
  void preCondFromScaled(LevelData &cor, const LevelData &w, const LevelData &res,
                         const int *skip);
  StencilCoefs stencil() { return coefs(); }
  // `n` levelGSRB sweeps with the fused out-of-place kernel (alternating
  // dpsi and the scratch buffer; the result always ends in dpsi).
  // zero_in: dpsi is taken as identically zero and not read (its memory
  // need not be zeroed).
  // rst != nullptr: the last sweep also writes restrictResidual(rst, result,
  // rhs) when the fused kernel can (returns whether it did)
  // before_acc: called on the host right before the first launch that writes
  // acc (nothing queued before it changes acc)
  bool fusedRelax(LevelData &dpsi, const LevelData &rhs, int n, bool zero_in = false,
                  LevelData *acc = nullptr, int flags = 0, LevelData *rst = nullptr,
                  const std::function<void()> *before_acc = nullptr);
  bool deepApplies() const;
  // r's ghosts for the fused sweeps' rings (once per MultiGrid level visit):
  // face layer 1, or the 4-deep shell in deep-halo mode
  void rhsHalo(LevelData &r, hipStream_t st) const;
  // relax(e, r, n); phi += e -- the increment folded into the last fused
  // sweep (e is left as scratch in that case)
  // (before_acc: as fusedRelax's, called before phi is first written)
  void relaxAccumulate(LevelData &e, const LevelData &r, int n, LevelData &phi, int flags = 0,
                       const std::function<void()> *before_acc = nullptr);
  // e = 0; relax(e, r, n) -- without zeroing e in memory when the fused
  // smoother applies (the first sweep does not read its input)
  void relaxFromZero(LevelData &e, const LevelData &r, int n, int flags = 0);
  // relax(e, r, n) with RelaxFlags
  void relaxFlags(LevelData &e, const LevelData &r, int n, int flags);
  // (e = 0 when zero_in;) relax(e, r, n); and, when the fused sweep can
  // fold it into its last pass, restrictResidual(resC, e, r) -- returns
  // whether the restriction was done (else the caller restricts)
  bool relaxRestrict(LevelData &e, const LevelData &r, int n, bool zero_in, int flags,
                     LevelData &resC);
};

// throws kBadArg unless x lives on g's boxes with g's fab geometry
void check_same_layout(const Grid &g, const LevelData &x, const char *what);

// CoarseAverage (arithmetic / harmonic) of a fine LevelData onto the layout
// coarsened by `ratio` (same box order and owners).
std::shared_ptr<LevelData> average_coef(const LevelData &fine, std::shared_ptr<Grid> cgrid,
                                        int ratio, int harmonic);

// Smoother instrumentation: when enabled, every smoother launch on a box of
// at least min_cells cells is bracketed by hipEvents on its stream.
void prof_enable(bool on, long min_cells, int mode = 1);  // mode 1 per launch, 2 per relax
void prof_flush();
int prof_read(double *total_ms, long *passes);  // returns launches timed, total ms
// bracket one smoother launch (no-op unless enabled and ncells >= min_cells)
void prof_mark(hipStream_t st, long ncells, bool begin, int passes);

// VariableCoeffPoissonOperatorFactory (single AMR level; the configs have one)
class VariableCoeffPoissonOperatorFactory {
 public:
  // define(coarseDomain, grids, refRatios, coarsedx, bc, alpha, aCoef, beta, bCoef)
  void define(std::shared_ptr<Grid> grid, const OpParams &prm, std::shared_ptr<LevelData> aCoef,
              std::shared_ptr<LevelData> bCoef);
  // MGnewOp: nullptr once !coarsenable(2^depth * s_maxCoarse) (Factory.cpp:168-172)
  std::unique_ptr<VariableCoeffPoissonOperator> MGnewOp(int depth, bool homoOnly = true);
  std::unique_ptr<VariableCoeffPoissonOperator> AMRnewOp();
  int refToFiner() const { return 2; }  // refRatio forced to 2 (PoissonParameters.cpp:75-79)
  int m_coefficient_average_type = 0;

  std::shared_ptr<Grid> grid;
  OpParams prm;
  std::shared_ptr<LevelData> m_aCoef, m_bCoef;
};

struct BiCGStabParams {
  int imax = 80;
  double eps = 1.0e-6, reps = 1.0e-12, small = 1.0e-30;
  int numRestarts = 5;
  int normType = 2;
};

// [Chombo] BiCGStabSolver<LevelData<FArrayBox>>::solve restated (the same
// control flow as oracle/mgic_oracle.c orc_mg_bicgstab)
class BiCGStabSolver {
 public:
  BiCGStabParams prm;
  int last_iters = 0;
  double last_init_norm = 0.0;  // norm of the residual the last solve started from
  bool last_device = false;     // the last solve ran on the device (solveDevice)
  // preconditioner; empty = op.preCond (the bottom-solver use)
  std::function<void(LevelData &, const LevelData &)> precond;
  int solve(VariableCoeffPoissonOperator &op, LevelData &phi, const LevelData &rhs,
            bool homogeneous);
  // the same loop with its scalars and stop tests on the device (one box,
  // one rank's reductions, preCond as one two-sweep launch): batches of
  // iterations queued without a readback, one published state per batch
  // (MGIC_BICG_DEVICE=0: always the host loop; MGIC_BICG_BATCH: iterations
  // per batch, default 4).  Bit-identical to the host loop.
  bool deviceApplies(VariableCoeffPoissonOperator &op) const;
  int solveDevice(VariableCoeffPoissonOperator &op, LevelData &phi, const LevelData &rhs,
                  bool homogeneous);
  BiCGStabSolver() = default;
  BiCGStabSolver(const BiCGStabSolver &) = delete;
  BiCGStabSolver &operator=(const BiCGStabSolver &) = delete;
  ~BiCGStabSolver();

 private:
  std::map<const Grid *, std::vector<std::unique_ptr<LevelData>>> temps_;
  struct DevWork {
    kern::BicgState *d_st = nullptr;   // the loop's state (device)
    kern::BicgState *h_pub = nullptr;  // published copy (pinned, host-coherent)
    kern::BicgState *h_up = nullptr;   // upload staging (pinned)
    unsigned long long *h_seq = nullptr;
    unsigned long long seq = 0;
    double *d_parts = nullptr;         // two partial arrays
    unsigned int *d_cnt = nullptr;     // the reductions' last-block counters
  };
  std::map<const Grid *, std::unique_ptr<DevWork>> dev_;
  DevWork &devWork(VariableCoeffPoissonOperator &op);
};

struct MGParams {
  int max_depth = -1;  // deepest MG depth (-1: as deep as coarsenable)
  int n_pre = 4, n_post = 4, n_bottom = 4;
  int bottom_solver = 1;       // 0: relax(n_bottom), 1: BiCGStab
  int cycles = 1;              // 1 = V-cycle
  int agglomerate_below = 0;   // gather to rank 0 when a box side < this (0 off)
  BiCGStabParams bicg;
};

// [Chombo] MultiGrid hierarchy built from the factory's MGnewOp; oneCycle is
// MultiGrid::oneCycle (pre-relax, restrictResidual, recurse, prolongIncrement,
// post-relax; bottom solver at the coarsest depth).
class MultiGrid {
 public:
  void define(VariableCoeffPoissonOperatorFactory &factory, const MGParams &prm);
  void oneCycle(LevelData &e, const LevelData &r) {
    cycle(0, e, const_cast<LevelData &>(r), false, nullptr);
  }
  // e = 0; oneCycle(e, r)
  void oneCycleFromZero(LevelData &e, const LevelData &r) {
    cycle(0, e, const_cast<LevelData &>(r), true, nullptr);
  }
  // e = 0; oneCycle(e, r); phi += e (e is scratch afterwards); before_phi:
  // called on the host before the first launch that writes phi
  void oneCycleFromZeroInto(LevelData &e, const LevelData &r, LevelData &phi,
                            const std::function<void()> *before_phi = nullptr) {
    cycle(0, e, const_cast<LevelData &>(r), true, &phi, false, before_phi);
  }
  // full multigrid from the residual r at depth 0: r_{d+1} = R(r_d) at every
  // depth, the bottom solve from zero, then per finer depth e_d = P e_{d+1}
  // and `ncycles` V-cycles on it; phi += e_0 (folded into the last sweep)
  void fmg(LevelData &e, LevelData &r, LevelData &phi, int ncycles);
  int depths() const { return (int)levels_.size(); }
  VariableCoeffPoissonOperator &op(int d) { return *levels_[d].op; }
  LevelData *corr(int d) { return levels_[d].e.get(); }
  LevelData *resid(int d) { return levels_[d].r.get(); }
  // depth d is the first gathered depth (the restriction is gathered into it,
  // the correction scattered out of it)
  bool agglomerated(int d) const { return levels_[d].agg; }
  // the rank that holds every box of depth d when it is gathered (the first
  // gathered depth and every depth below it), else -1 (distributed)
  int owner(int d) const { return levels_[d].owner; }
  // this rank runs depth d (distributed, or gathered onto this rank)
  bool runs(int d) const {
    return levels_[d].owner < 0 || levels_[d].owner == levels_[d].op->grid->comm->rank();
  }
  // the first gathered depth's plans: the previous layout coarsened (the
  // restriction's target before the gather, the prolongation's source after
  // the scatter) -> the gathered box, and back
  std::shared_ptr<Grid> stage_grid(int d) const { return levels_[d].r_stage->grid; }
  CopyPlan &gather_plan(int d) { return *levels_[d].restrict_plan; }
  CopyPlan &scatter_plan(int d) { return *levels_[d].prolong_plan; }
  MGParams prm;
  BiCGStabSolver bottom;
  // HIP events around every BiCGStab bottom solve this rank runs (on: reset
  // and start recording); bottom_ms: their total time and count (waits for
  // the last one)
  void bottom_timer(bool on);
  double bottom_ms(int *calls);
  // BiCGStab iterations summed over the timed solves, and the smallest /
  // largest norm of the coarse residual they started from
  long bottom_iters(double *r0_min, double *r0_max) const;
  // the last bottom solve again, `n` times, each from e = 0 on the same
  // coarse residual (a fixed amount of work per solve): total ms between HIP
  // events, iterations per solve, the residual's norm.  Returns the solves
  // run (0 on a rank that does not own the coarsest depth, or before any
  // V-cycle has filled it).
  int bottom_replay(int n, double *ms, int *iters, double *r0);
  ~MultiGrid();

 private:
  struct Level {
    std::unique_ptr<VariableCoeffPoissonOperator> op;
    std::unique_ptr<LevelData> e, r;
    bool agg = false;  // the first gathered depth (plans below)
    int owner = -1;    // gathered: the rank holding its box
    std::unique_ptr<LevelData> r_stage, e_stage;  // previous layout coarsened
    std::unique_ptr<CopyPlan> restrict_plan, prolong_plan;
  };
  // e_zero: treat e as zero on entry (it is zeroed or never read);
  // phi_acc: phi += e at the end (at depth 0 folded into the last sweep)
  void cycle(int d, LevelData &e, LevelData &r, bool e_zero, LevelData *phi_acc,
             bool halo_out = false, const std::function<void()> *before_phi = nullptr);
  std::vector<Level> levels_;
  bool bt_on_ = false;
  bool bt_filled_ = false;  // a bottom solve has run (bottom_replay's input exists)
  size_t bt_used_ = 0;
  long bt_iters_ = 0, bt_solves_ = 0;
  double bt_r0_min_ = 0.0, bt_r0_max_ = 0.0;
  std::vector<hipEvent_t> bt_ev_;
  void bottom_solve(VariableCoeffPoissonOperator &op, LevelData &e, LevelData &r);
};

// [Chombo] AMRMultiGrid on a single AMR level: iterations of
//   e = 0; oneCycle(e, r); phi += e; r = rhs - L(phi)
struct SolveParams {  // Main_PoissonSolver.cpp:106-126 defaults (params.txt overrides)
  int num_mg_iterations = 1;  // numMGIterations (:107-109)
  int max_iterations = 10;    // max_iterations (:122-123) -> m_imax (:178)
  double tolerance = 1.0e-7;  // tolerance (:119-120) -> m_eps (:177)
  int norm_type = 0;          // m_normType (:176)
};

class AMRMultiGrid {
 public:
  void define(VariableCoeffPoissonOperatorFactory &factory, const MGParams &prm);
  // MultilevelLinearOp::preCond on this AMR level: e = 0, then `iters`
  // iterations on (e, r) with homogeneous BC
  void precondition(LevelData &e, const LevelData &r, int iters);
  // solver.solve(dpsi, rhs) (Main_PoissonSolver.cpp:174-184): BiCGStab
  // over the level operator, preconditioned by precondition(); returns
  // iterations, *final_norm = norm(rhs - L(phi), norm_type)
  int solve(LevelData &phi, const LevelData &rhs, const SolveParams &p, double *final_norm);
  // one iteration; returns norm(r, normType) if normType >= 0 (host sync),
  // else -1 without synchronising
  double iteration(LevelData &phi, const LevelData &rhs, LevelData &resid, int normType,
                   bool homogeneous);
  // `count` iterations from the state iteration() / initResidual() leave
  // (resid = rhs - L(phi)); norms[i] = what the i-th iteration() call would
  // return, bit for bit (the same launches in the same order).  The host
  // reads iteration i's norm while the GPU runs iteration i+1's V-cycle up
  // to its first phi-writing launch, which is queued only after the read --
  // the place a stop test on that norm would decide -- so the GPU does not
  // idle between iterations.
  void iterations(LevelData &phi, const LevelData &rhs, LevelData &resid, int count,
                  int normType, bool homogeneous, double *norms);
  double initResidual(LevelData &phi, const LevelData &rhs, LevelData &resid, int normType,
                      bool homogeneous);
  // an FMG cycle on the current residual (resid as left by initResidual /
  // iteration), phi += its correction, then resid = rhs - L(phi)
  double fmg(LevelData &phi, const LevelData &rhs, LevelData &resid, int normType,
             bool homogeneous, int ncycles);
  MultiGrid mg;

 private:
  std::unique_ptr<LevelData> corr_, pre_resid_;
  BiCGStabSolver outer_;
};

}  // namespace mgic
