/*
 * mgic_oracle.h -- CPU restatement of the reference VariableCoeffPoissonOperator
 * multigrid path.  TEST INFRASTRUCTURE ONLY: imported by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg, as the checker.
 * It is never linked into, loaded by, or called from the product library.
 *
 * PARITY STATUS: "parity unpinned" against the reference binary.  The
 * reference kernels are ChomboFortran (.ChF) that need Chombo's chfpp
 * preprocessor and Chombo 3.2 libraries, neither of which exists in this
 * image, and the reference ships no tests, fixtures or golden vectors
 * (SURVEY.md §4.1, §8(c)).  This file restates the arithmetic from the
 * reference text, statement by statement, citing file:line.  Behaviour that
 * lives in Chombo (BC fill, exchange, prolongation, V-cycle, BiCGStab) is
 * restated from Chombo 3.2's published algorithm and marked [Chombo].
 *
 * Layout: a "fab" is one component over an inclusive cell box [lo,hi]
 * (ghost cells included), column-major with i fastest -- the same layout as
 * a Chombo FArrayBox with one component.
 */
#ifndef MGIC_ORACLE_H
#define MGIC_ORACLE_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  double *p;
  int lo[3];
  int hi[3];
} orc_fab;

/* ---- the four 3-D ChF kernels (VariableCoeffPoissonOperatorF.ChF) ---- */
void orc_gsrbhelmholtzvc3d(orc_fab *dpsi, const orc_fab *rhs, const int *rlo,
                           const int *rhi, double dx, double alpha,
                           const orc_fab *aCoef, double beta,
                           const orc_fab *bCoef, const orc_fab *lambda,
                           int redBlack);
void orc_vccomputeop3d(orc_fab *lofdpsi, const orc_fab *dpsi, double alpha,
                       const orc_fab *aCoef, double beta, const orc_fab *bCoef,
                       const int *rlo, const int *rhi, double dx);
void orc_vccomputeres3d(orc_fab *res, const orc_fab *dpsi, const orc_fab *rhs,
                        double alpha, const orc_fab *aCoef, double beta,
                        const orc_fab *bCoef, const int *rlo, const int *rhi,
                        double dx);
/* restrictResidual for one box, including the res.setVal(0) and the
 * CHF_FRA_SHIFT index shift of VariableCoeffPoissonOperator.cpp:165-192 */
void orc_restrictresvc3d(orc_fab *res, const orc_fab *dpsi, const orc_fab *rhs,
                         double alpha, const orc_fab *aCoef, double beta,
                         const orc_fab *bCoef, const int *rlo, const int *rhi,
                         double dx);

/* ---- operator helpers ---- */
void orc_lambda(orc_fab *lam, const orc_fab *aCoef, const int *rlo,
                const int *rhi, double alpha, double beta, double dx);
/* CoarseAverage arithmetic (harmonic=0) / harmonic (harmonic=1) with
 * refinement ratio `ratio`, over the coarse region [crlo,crhi] */
void orc_average(orc_fab *coarse, const orc_fab *fine, const int *crlo,
                 const int *crhi, int ratio, int harmonic);
/* prolongIncrement for one box: fine[region] += P(coarse).  type 0 =
 * piecewise constant, 1 = linear.  avail_lo/avail_hi give, per direction,
 * whether the coarse face-ghost layer below/above the coarse valid box
 * [cvlo,cvhi] holds usable (exchanged) data. */
void orc_prolong(orc_fab *fine, const orc_fab *coarse, const int *frlo,
                 const int *frhi, const int *cvlo, const int *cvhi,
                 const int *avail_lo, const int *avail_hi, int type);

/* ---- multi-box level / multigrid hierarchy ---- */
typedef struct orc_mg orc_mg;

enum {
  ORC_PHI = 0,  /* level-0 solution (dpsi)            */
  ORC_RHS = 1,  /* level-0 right-hand side            */
  ORC_ACOEF = 2,
  ORC_BCOEF = 3,
  ORC_LAMBDA = 4,
  ORC_RESID = 5, /* residual (level 0) / restricted residual (level>0) */
  ORC_CORR = 6,  /* correction e                      */
  ORC_TMP = 7,
  ORC_NFIELD = 8
};

typedef struct {
  int nbox;
  const int *boxes;   /* nbox * 6 ints: lo0 lo1 lo2 hi0 hi1 hi2 (level 0) */
  int domain[6];      /* level-0 domain box */
  int periodic[3];
  int bc_lo[3];       /* 0 Dirichlet, 1 Neumann, 2 periodic flag (no-op) */
  int bc_hi[3];
  double bc_value;
  double dx;          /* level-0 cell spacing */
  double alpha, beta;
  int nlevels;        /* <=0: as deep as coarsenable(2^d * max_coarse) allows */
  int max_coarse;     /* AMRPoissonOp::s_maxCoarse [Chombo] (2) */
  int avg_type;       /* 0 arithmetic, 1 harmonic */
  int prolong_type;   /* 0 constant, 1 linear */
  int relax_mode;     /* 1 GSRB, 4 Jacobi */
  int n_pre, n_post, n_bottom;
  int bottom_solver;  /* 0 relax(n_bottom), 1 BiCGStab */
  int bicg_imax;
  double bicg_eps, bicg_reps, bicg_small;
  int bicg_restarts;
  int bicg_norm_type;
} orc_mg_params;

orc_mg *orc_mg_create(const orc_mg_params *prm);
void orc_mg_destroy(orc_mg *mg);
int orc_mg_nlevels(const orc_mg *mg);
/* box geometry of (level, box): writes lo[3],hi[3] of the valid box */
void orc_mg_box(const orc_mg *mg, int level, int box, int *lohi);
double orc_mg_dx(const orc_mg *mg, int level);
/* valid-region data, contiguous i-fastest over the box */
void orc_mg_set(orc_mg *mg, int level, int field, int box, const double *src);
void orc_mg_get(const orc_mg *mg, int level, int field, int box, double *dst);
/* full fab (ghosts included), contiguous over valid grown by 1 */
void orc_mg_set_full(orc_mg *mg, int level, int field, int box,
                     const double *src);
void orc_mg_get_full(const orc_mg *mg, int level, int field, int box,
                     double *dst);
/* coefficient coarsening (MGnewOp) + lambda (computeLambda) on all levels */
void orc_mg_setup(orc_mg *mg);

/* level operations (fields by ORC_* index) */
void orc_mg_exchange(orc_mg *mg, int level, int field);
void orc_mg_fill_bc(orc_mg *mg, int level, int field, int homogeneous);
void orc_mg_level_gsrb(orc_mg *mg, int level, int fu, int frhs);
void orc_mg_level_jacobi(orc_mg *mg, int level, int fu, int frhs);
void orc_mg_relax(orc_mg *mg, int level, int fu, int frhs, int n);
void orc_mg_residual(orc_mg *mg, int level, int fr, int fu, int frhs,
                     int homogeneous);
void orc_mg_apply_op(orc_mg *mg, int level, int flu, int fu, int homogeneous);
void orc_mg_restrict_residual(orc_mg *mg, int level, int fu, int frhs);
void orc_mg_prolong_increment(orc_mg *mg, int level, int fu);
void orc_mg_precond(orc_mg *mg, int level, int fe, int fr);
/* MultiGrid::oneCycle on (CORR, RESID) of `level` */
void orc_mg_one_cycle(orc_mg *mg, int level);
/* one AMRMultiGrid iteration at level 0: CORR=0, oneCycle, PHI+=CORR,
 * RESID = RHS - L(PHI); returns norm(RESID, norm_type) */
double orc_mg_iteration(orc_mg *mg, int norm_type);
/* full multigrid from RESID at level 0: PHI += FMG correction (see .c) */
double orc_mg_fmg(orc_mg *mg, int ncycles, int norm_type);
/* RESID = RHS - L(PHI) on level 0, returns its norm */
double orc_mg_init_residual(orc_mg *mg, int norm_type);
/* BiCGStab (homogeneous) on a level: solves L e = r for fields fe, fr */
int orc_mg_bicgstab(orc_mg *mg, int level, int fe, int fr, int homogeneous);
/* MultilevelLinearOp::preCond on level 0: fe = 0, then `iters`
 * AMRMultiGrid iterations on (fe, fr), homogeneous BC */
void orc_mg_amr_precond(orc_mg *mg, int fe, int fr, int iters);
/* the outer solve (Main_PoissonSolver.cpp:174-184): MG-preconditioned
 * BiCGStab on level-0 PHI / RHS; returns iterations, final residual norm */
int orc_mg_solve(orc_mg *mg, int mg_iters, int imax, double eps, int norm_type,
                 double *final_norm);
double orc_mg_norm(orc_mg *mg, int level, int field, int norm_type);
double orc_mg_dot(orc_mg *mg, int level, int fx, int fy);
int orc_mg_last_bicg_iters(const orc_mg *mg);

/* ---- input generator (SetLevelData.cpp / SetBinaryBH.H / MyPhiFunction.H) */
typedef struct {
  double L;          /* domain length (params.txt:16) */
  double G_Newton;
  double phi_amplitude, phi_wavelength;
  double bh1_bare_mass, bh2_bare_mass;
  double bh1_spin, bh2_spin;
  double bh1_offset, bh2_offset;
  double bh1_momentum, bh2_momentum;
  double constant_K;
} orc_bh_params;
/* aCoef and rhs at psi = 1 (NL iteration 0) over the cell box [lo,hi],
 * contiguous i fastest; dx is the cell spacing of that level */
void orc_binary_bh_coefs(const orc_bh_params *p, const int *lo, const int *hi,
                         double dx, double *acoef, double *rhs);
/* set_a_coef + set_rhs (SetLevelData.cpp:73-127, :281-325) at a general
 * psi given over the box grown by one (i fastest), constant_K from p */
void orc_nl_coefs(const orc_bh_params *p, const int *lo, const int *hi, double dx,
                  const double *psi, double *acoef, double *rhs);
/* set_constant_K_integrand (SetLevelData.cpp:131-180) at psi */
void orc_nl_integrand(const orc_bh_params *p, const int *lo, const int *hi, double dx,
                      const double *psi, double *out);

/* GETLAPLACIANPSIF (laplacian = 1) / GETRHOGRADPHIF (laplacian = 0) over
 * [lo, hi]; `in` over the box grown by one */
void orc_getlaplacianpsif(double *out, const double *in, const int *lo, const int *hi, double dx,
                          int laplacian);

/* WriteOutput.H's components over the cell box [lo, hi] (component-major,
 * i fastest).  kind 0: set_output_data (SetLevelData.cpp:343-396), the 31
 * GRChombo variables from psi (constant_K from p); kind 1: output_solver_data's
 * tempData (WriteOutput.H:84-100): dpsi, rhs, psi, A11_0, A12_0, A13_0, A22_0,
 * A23_0, A33_0, phi_0 (set_initial_conditions, SetLevelData.cpp:31-72).
 * psi / dpsi / rhs over the box (i fastest); dpsi, rhs unused for kind 0. */
void orc_output_vars(int kind, const orc_bh_params *p, const int *lo, const int *hi, double dx,
                     const double *psi, const double *dpsi, const double *rhs, double *out);

void orc_set_threads(int n);
int orc_get_threads(void);
int orc_pin_threads(const int *cpus, int n, int pin);

#ifdef __cplusplus
}
#endif
#endif
