/*
 * mgic_oracle.c -- CPU restatement of the reference multigrid hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see mgic_oracle.h): the checker for tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Parity status:
 * "parity unpinned" (the ChomboFortran reference cannot be built here and
 * ships no golden vectors); every formula below cites the reference line it
 * restates, and [Chombo] marks semantics restated from Chombo 3.2.
 *
 * Floating point: compiled with -ffp-contract=off; every expression keeps
 * the reference's evaluation order (Fortran/C++ left-to-right, parentheses
 * as written) so the HIP kernels can be compared bit for bit.
 */
#include "mgic_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#include <sched.h>
#endif

/* ------------------------------------------------------------------ */
/* fab indexing                                                        */
/* ------------------------------------------------------------------ */
static inline size_t fab_nx(const orc_fab *f) { return (size_t)(f->hi[0] - f->lo[0] + 1); }
static inline size_t fab_ny(const orc_fab *f) { return (size_t)(f->hi[1] - f->lo[1] + 1); }
static inline size_t fab_nz(const orc_fab *f) { return (size_t)(f->hi[2] - f->lo[2] + 1); }
static inline size_t IX(const orc_fab *f, int i, int j, int k) {
  return (size_t)(i - f->lo[0]) +
         fab_nx(f) * ((size_t)(j - f->lo[1]) + fab_ny(f) * (size_t)(k - f->lo[2]));
}
#define AT(f, i, j, k) ((f)->p[IX((f), (i), (j), (k))])

static inline int floordiv(int i, int r) { return (i >= 0) ? (i / r) : -((-i + r - 1) / r); }
static inline int floordiv2(int i) { return floordiv(i, 2); }

/* 7-point Laplacian, VariableCoeffPoissonOperatorF.ChF:111-120 (also
 * :216-225, :320-329, :416-425): CHF_DTERM expands to
 *   (u(i+1)+u(i-1)-two*u) + (u(j+1)+u(j-1)-two*u) + (u(k+1)+u(k-1)-two*u)
 * evaluated left to right. */
static inline double lap7(const orc_fab *u, int i, int j, int k) {
  const double c = AT(u, i, j, k);
  const double tx = (AT(u, i + 1, j, k) + AT(u, i - 1, j, k)) - 2.0 * c;
  const double ty = (AT(u, i, j + 1, k) + AT(u, i, j - 1, k)) - 2.0 * c;
  const double tz = (AT(u, i, j, k + 1) + AT(u, i, j, k - 1)) - 2.0 * c;
  return (tx + ty) + tz;
}

/* ------------------------------------------------------------------ */
/* The four 3-D kernels                                                */
/* ------------------------------------------------------------------ */

/* GSRBHELMHOLTZVC3D, VariableCoeffPoissonOperatorF.ChF:56-139 */
void orc_gsrbhelmholtzvc3d(orc_fab *dpsi, const orc_fab *rhs, const int *rlo,
                           const int *rhi, double dx, double alpha,
                           const orc_fab *aCoef, double beta,
                           const orc_fab *bCoef, const orc_fab *lambda,
                           int redBlack) {
  const double dxinv = 1.0 / (dx * dx); /* :89 */
#pragma omp parallel for schedule(static)
  for (int k = rlo[2]; k <= rhi[2]; ++k) {          /* :93 */
    for (int j = rlo[1]; j <= rhi[1]; ++j) {        /* :96 */
      int imin = rlo[0];                            /* :98 */
      const int indtot = imin + j + k;              /* :99 */
      imin = imin + abs((indtot + redBlack) % 2);   /* :104 */
      for (int i = imin; i <= rhi[0]; i += 2) {     /* :106 */
        double lofdpsi = alpha * AT(aCoef, i, j, k) * AT(dpsi, i, j, k); /* :107-108 */
        double ldpsi = lap7(dpsi, i, j, k);                              /* :111-120 */
        ldpsi = ldpsi * dxinv * AT(bCoef, i, j, k);                      /* :122 */
        lofdpsi = lofdpsi - beta * ldpsi;                                /* :124 */
        AT(dpsi, i, j, k) = AT(dpsi, i, j, k) -
                            AT(lambda, i, j, k) * (lofdpsi - AT(rhs, i, j, k)); /* :127-128 */
      }
    }
  }
}

/* VCCOMPUTEOP3D, VariableCoeffPoissonOperatorF.ChF:181-237 */
void orc_vccomputeop3d(orc_fab *lofdpsi, const orc_fab *dpsi, double alpha,
                       const orc_fab *aCoef, double beta, const orc_fab *bCoef,
                       const int *rlo, const int *rhi, double dx) {
  const double dxinv = 1.0 / (dx * dx); /* :208 */
#pragma omp parallel for schedule(static)
  for (int k = rlo[2]; k <= rhi[2]; ++k)
    for (int j = rlo[1]; j <= rhi[1]; ++j)
      for (int i = rlo[0]; i <= rhi[0]; ++i) {
        double lof = alpha * AT(aCoef, i, j, k) * AT(dpsi, i, j, k);  /* :211-212 */
        double ldpsi = lap7(dpsi, i, j, k);                           /* :216-225 */
        ldpsi = ldpsi * dxinv * beta * AT(bCoef, i, j, k);            /* :227 */
        AT(lofdpsi, i, j, k) = lof - ldpsi;                           /* :229 */
      }
}

/* VCCOMPUTERES3D, VariableCoeffPoissonOperatorF.ChF:283-339 */
void orc_vccomputeres3d(orc_fab *res, const orc_fab *dpsi, const orc_fab *rhs,
                        double alpha, const orc_fab *aCoef, double beta,
                        const orc_fab *bCoef, const int *rlo, const int *rhi,
                        double dx) {
  const double dxinv = 1.0 / (dx * dx); /* :311 */
#pragma omp parallel for schedule(static)
  for (int k = rlo[2]; k <= rhi[2]; ++k)
    for (int j = rlo[1]; j <= rhi[1]; ++j)
      for (int i = rlo[0]; i <= rhi[0]; ++i) {
        double r = AT(rhs, i, j, k) - alpha * AT(aCoef, i, j, k) * AT(dpsi, i, j, k); /* :314-316 */
        double ldpsi = lap7(dpsi, i, j, k);                                         /* :320-329 */
        ldpsi = ldpsi * dxinv * beta * AT(bCoef, i, j, k);                          /* :331 */
        AT(res, i, j, k) = r + ldpsi;                                               /* :333 */
      }
}

/* restrictResidual for one box: res.setVal(0) (VariableCoeffPoissonOperator
 * .cpp:177), boxes shifted so the fine region starts at iv and the coarse
 * one at coarsen(iv,2) (:173-192), then RESTRICTRESVC3D
 * (VariableCoeffPoissonOperatorF.ChF:379-437).  The Fortran walks the fine
 * region k,j,i and accumulates into res(i/2,j/2,k/2); we walk coarse
 * k-planes in parallel and, inside each, the fine cells in the same k,j,i
 * order, so every coarse cell receives its 8 terms in the reference order. */
void orc_restrictresvc3d(orc_fab *res, const orc_fab *dpsi, const orc_fab *rhs,
                         double alpha, const orc_fab *aCoef, double beta,
                         const orc_fab *bCoef, const int *rlo, const int *rhi,
                         double dx) {
  const double dxinv = 1.0 / (dx * dx); /* :401 */
  const double denom = 2 * 2 * 2;       /* :402 D_TERM(2, *2, *2) */
  const size_t ntot = fab_nx(res) * fab_ny(res) * fab_nz(res);
  for (size_t n = 0; n < ntot; ++n) res->p[n] = 0.0; /* res.setVal(0.0) */
  int civ[3];
  for (int d = 0; d < 3; ++d) civ[d] = floordiv2(rlo[d]); /* coarsen(iv, 2) */
  const int kc_lo = civ[2], kc_hi = civ[2] + (rhi[2] - rlo[2]) / 2;
#pragma omp parallel for schedule(static)
  for (int kc = kc_lo; kc <= kc_hi; ++kc) {
    for (int k = rlo[2]; k <= rhi[2]; ++k) {
      const int kk = civ[2] + (k - rlo[2]) / 2; /* :409 on shifted indices */
      if (kk != kc) continue;
      for (int j = rlo[1]; j <= rhi[1]; ++j) {
        const int jj = civ[1] + (j - rlo[1]) / 2; /* :408 */
        for (int i = rlo[0]; i <= rhi[0]; ++i) {
          const int ii = civ[0] + (i - rlo[0]) / 2; /* :407 */
          double lofdpsi = alpha * AT(aCoef, i, j, k) * AT(dpsi, i, j, k); /* :411-412 */
          double ldpsi = lap7(dpsi, i, j, k);                              /* :416-425 */
          ldpsi = ldpsi * dxinv * beta * AT(bCoef, i, j, k);               /* :427 */
          lofdpsi = lofdpsi - ldpsi;                                       /* :429 */
          AT(res, ii, jj, kk) = AT(res, ii, jj, kk) +
                                (AT(rhs, i, j, k) - lofdpsi) / denom;      /* :431-432 */
        }
      }
    }
  }
}

/* resetLambda, VariableCoeffPoissonOperator.cpp:220-249:
 *   lambda = a; lambda *= alpha; lambda += 2*SpaceDim*beta/(dx*dx);
 *   lambda = 1/lambda */
void orc_lambda(orc_fab *lam, const orc_fab *aCoef, const int *rlo,
                const int *rhi, double alpha, double beta, double dx) {
  const double shift = 2.0 * 3 * beta / (dx * dx); /* :240 */
#pragma omp parallel for schedule(static)
  for (int k = rlo[2]; k <= rhi[2]; ++k)
    for (int j = rlo[1]; j <= rhi[1]; ++j)
      for (int i = rlo[0]; i <= rhi[0]; ++i) {
        double v = AT(aCoef, i, j, k); /* :234 copy */
        v = v * alpha;                 /* :235 mult  */
        v = v + shift;                 /* :240 plus  */
        AT(lam, i, j, k) = 1.0 / v;    /* :243 invert(1.0) */
      }
}

/* [Chombo] CoarseAverage::averageToCoarse / averageToCoarseHarmonic
 * (AverageF.ChF AVERAGE / AVERAGEHARMONIC) with refinement ratio `ratio`:
 * the ratio^3 children summed in the k,j,i order of the refinement box,
 * scaled by refScale = 1/ratio^3; harmonic sums reciprocals and inverts.
 * MGnewOp averages straight from the AMR-level coefficients with ratio
 * 2^depth (VariableCoeffPoissonOperatorFactory.cpp:161-166, :208-223). */
void orc_average(orc_fab *coarse, const orc_fab *fine, const int *crlo,
                 const int *crhi, int ratio, int harmonic) {
  const double refScale = 1.0 / (ratio * ratio * ratio);
#pragma omp parallel for schedule(static)
  for (int K = crlo[2]; K <= crhi[2]; ++K)
    for (int J = crlo[1]; J <= crhi[1]; ++J)
      for (int I = crlo[0]; I <= crhi[0]; ++I) {
        double sum = 0.0;
        for (int kk = 0; kk < ratio; ++kk)
          for (int jj = 0; jj < ratio; ++jj)
            for (int ii = 0; ii < ratio; ++ii) {
              const double f = AT(fine, ratio * I + ii, ratio * J + jj, ratio * K + kk);
              sum = sum + (harmonic ? 1.0 / f : f);
            }
        AT(coarse, I, J, K) = harmonic ? 1.0 / (sum * refScale) : sum * refScale;
      }
}

/* [Chombo] AMRPoissonOp::prolongIncrement (inherited, not overridden in
 * VariableCoeffPoissonOperator.H): fine += P(coarse), ratio 2.  type 0:
 * piecewise constant (FORT_PROLONG).  type 1: linear (FORT_PROLONGLINEAR
 * restated): per direction, a fine cell in the upper half of its coarse
 * parent adds 0.25*(c[ic+1]-c[ic]), one in the lower half adds
 * -0.25*(c[ic]-c[ic-1]); where that neighbour lies beyond a non-periodic
 * domain face the opposite one-sided slope is used.  Coarse neighbours at
 * internal box faces come from the exchanged coarse ghost layer, which makes
 * the result independent of the box decomposition (stated deviation from a
 * box-local slope; parity unpinned). */
void orc_prolong(orc_fab *fine, const orc_fab *coarse, const int *frlo,
                 const int *frhi, const int *cvlo, const int *cvhi,
                 const int *avail_lo, const int *avail_hi, int type) {
#pragma omp parallel for schedule(static)
  for (int k = frlo[2]; k <= frhi[2]; ++k)
    for (int j = frlo[1]; j <= frhi[1]; ++j)
      for (int i = frlo[0]; i <= frhi[0]; ++i) {
        const int f[3] = {i, j, k};
        const int ic[3] = {floordiv2(i), floordiv2(j), floordiv2(k)};
        const double c0 = AT(coarse, ic[0], ic[1], ic[2]);
        double e = c0;
        if (type == 1) {
          for (int d = 0; d < 3; ++d) {
            int lo_n[3] = {ic[0], ic[1], ic[2]};
            int hi_n[3] = {ic[0], ic[1], ic[2]};
            lo_n[d] -= 1;
            hi_n[d] += 1;
            const int has_lo = (ic[d] > cvlo[d]) || avail_lo[d];
            const int has_hi = (ic[d] < cvhi[d]) || avail_hi[d];
            const int upper = f[d] - 2 * ic[d];
            const double fac = upper ? 0.25 : -0.25;
            double delta;
            int ok = 1;
            if (upper) {
              if (has_hi)
                delta = AT(coarse, hi_n[0], hi_n[1], hi_n[2]) - c0;
              else if (has_lo)
                delta = c0 - AT(coarse, lo_n[0], lo_n[1], lo_n[2]);
              else
                ok = 0, delta = 0.0;
            } else {
              if (has_lo)
                delta = c0 - AT(coarse, lo_n[0], lo_n[1], lo_n[2]);
              else if (has_hi)
                delta = AT(coarse, hi_n[0], hi_n[1], hi_n[2]) - c0;
              else
                ok = 0, delta = 0.0;
            }
            if (ok) e = e + delta * fac;
          }
        }
        AT(fine, i, j, k) = AT(fine, i, j, k) + e;
      }
}

/* ------------------------------------------------------------------ */
/* Multi-box levels and the multigrid hierarchy                        */
/* ------------------------------------------------------------------ */
#define ORC_NWORK 9
#define ORC_NF_ALL (ORC_NFIELD + ORC_NWORK)
enum { W_R = ORC_NFIELD, W_RT, W_E, W_P, W_PT, W_S, W_ST, W_T, W_V };

typedef struct {
  int nbox;
  int *vbox; /* nbox*6 */
  int dom[6];
  double dx;
  orc_fab *f[ORC_NF_ALL]; /* each: nbox fabs over valid grown by 1 */
} orc_level;

struct orc_mg {
  orc_mg_params prm;
  int nlev;
  orc_level *lev;
  int last_iters;
};

static const int *vb(const orc_level *L, int b) { return L->vbox + 6 * b; }

static int box_coarsenable(const int *b, int r) {
  for (int d = 0; d < 3; ++d) {
    if (((b[d] % r) + r) % r != 0) return 0;
    if ((((b[3 + d] + 1) % r) + r) % r != 0) return 0;
  }
  return 1;
}

static orc_fab *fab_of(orc_mg *mg, int l, int field, int b) {
  orc_level *L = &mg->lev[l];
  if (!L->f[field]) {
    L->f[field] = (orc_fab *)calloc((size_t)L->nbox, sizeof(orc_fab));
    for (int bb = 0; bb < L->nbox; ++bb) {
      orc_fab *fb = &L->f[field][bb];
      for (int d = 0; d < 3; ++d) {
        fb->lo[d] = vb(L, bb)[d] - 1;
        fb->hi[d] = vb(L, bb)[3 + d] + 1;
      }
      fb->p = (double *)calloc(fab_nx(fb) * fab_ny(fb) * fab_nz(fb), sizeof(double));
    }
  }
  return &L->f[field][b];
}

orc_mg *orc_mg_create(const orc_mg_params *prm) {
  orc_mg *mg = (orc_mg *)calloc(1, sizeof(orc_mg));
  mg->prm = *prm;
  if (mg->prm.max_coarse <= 0) mg->prm.max_coarse = 2;
  int nlev = prm->nlevels;
  if (nlev <= 0) {
    /* VariableCoeffPoissonOperatorFactory.cpp:163-172: depth d exists while
     * every box is coarsenable(2^d * s_maxCoarse) */
    nlev = 1;
    for (int d = 1; d < 30; ++d) {
      int ok = 1;
      for (int b = 0; b < prm->nbox && ok; ++b)
        ok = box_coarsenable(prm->boxes + 6 * b, (1 << d) * mg->prm.max_coarse);
      if (!ok) break;
      nlev = d + 1;
    }
  }
  for (int b = 0; b < prm->nbox; ++b)
    if (nlev > 1 && !box_coarsenable(prm->boxes + 6 * b, 1 << (nlev - 1))) {
      fprintf(stderr, "orc_mg_create: box %d not coarsenable to %d levels\n", b, nlev);
      free(mg);
      return NULL;
    }
  mg->nlev = nlev;
  mg->lev = (orc_level *)calloc((size_t)nlev, sizeof(orc_level));
  for (int l = 0; l < nlev; ++l) {
    orc_level *L = &mg->lev[l];
    L->nbox = prm->nbox;
    L->vbox = (int *)malloc(sizeof(int) * 6 * (size_t)prm->nbox);
    const int r = 1 << l;
    for (int b = 0; b < prm->nbox; ++b)
      for (int d = 0; d < 3; ++d) {
        L->vbox[6 * b + d] = floordiv(prm->boxes[6 * b + d], r);
        L->vbox[6 * b + 3 + d] = floordiv(prm->boxes[6 * b + 3 + d], r);
      }
    for (int d = 0; d < 3; ++d) {
      L->dom[d] = floordiv(prm->domain[d], r);
      L->dom[3 + d] = floordiv(prm->domain[3 + d], r);
    }
    L->dx = prm->dx * (double)r; /* MGnewOp: dx *= coarsening (:174) */
  }
  return mg;
}

void orc_mg_destroy(orc_mg *mg) {
  if (!mg) return;
  for (int l = 0; l < mg->nlev; ++l) {
    orc_level *L = &mg->lev[l];
    for (int f = 0; f < ORC_NF_ALL; ++f)
      if (L->f[f]) {
        for (int b = 0; b < L->nbox; ++b) free(L->f[f][b].p);
        free(L->f[f]);
      }
    free(L->vbox);
  }
  free(mg->lev);
  free(mg);
}

int orc_mg_nlevels(const orc_mg *mg) { return mg->nlev; }
int orc_mg_last_bicg_iters(const orc_mg *mg) { return mg->last_iters; }
double orc_mg_dx(const orc_mg *mg, int level) { return mg->lev[level].dx; }
void orc_mg_box(const orc_mg *mg, int level, int box, int *lohi) {
  memcpy(lohi, mg->lev[level].vbox + 6 * box, 6 * sizeof(int));
}

static void copy_valid(orc_mg *mg, int l, int field, int b, const double *src, double *dst) {
  orc_fab *f = fab_of(mg, l, field, b);
  const int *v = vb(&mg->lev[l], b);
  size_t n = 0;
  for (int k = v[2]; k <= v[5]; ++k)
    for (int j = v[1]; j <= v[4]; ++j)
      for (int i = v[0]; i <= v[3]; ++i, ++n) {
        if (src) AT(f, i, j, k) = src[n];
        else dst[n] = AT(f, i, j, k);
      }
}
void orc_mg_set(orc_mg *mg, int level, int field, int box, const double *src) {
  copy_valid(mg, level, field, box, src, NULL);
}
void orc_mg_get(const orc_mg *mg, int level, int field, int box, double *dst) {
  copy_valid((orc_mg *)mg, level, field, box, NULL, dst);
}
void orc_mg_set_full(orc_mg *mg, int level, int field, int box, const double *src) {
  orc_fab *f = fab_of(mg, level, field, box);
  memcpy(f->p, src, sizeof(double) * fab_nx(f) * fab_ny(f) * fab_nz(f));
}
void orc_mg_get_full(const orc_mg *mg, int level, int field, int box, double *dst) {
  orc_fab *f = fab_of((orc_mg *)mg, level, field, box);
  memcpy(dst, f->p, sizeof(double) * fab_nx(f) * fab_ny(f) * fab_nz(f));
}

/* -------- level vector ops (Chombo LevelDataOps semantics, valid cells) */
typedef void (*cellfn)(double *x, const double *y, double s);
static void lv_zero_all(orc_mg *mg, int l, int f) {
  for (int b = 0; b < mg->lev[l].nbox; ++b) {
    orc_fab *x = fab_of(mg, l, f, b);
    memset(x->p, 0, sizeof(double) * fab_nx(x) * fab_ny(x) * fab_nz(x));
  }
}
/* kind: 0 copy x=y, 1 incr x = x + s*y, 2 scale x = x*s, 3 mult x = x*y */
static void lv_op(orc_mg *mg, int l, int fx, int fy, double s, int kind) {
  orc_level *L = &mg->lev[l];
  for (int b = 0; b < L->nbox; ++b) {
    orc_fab *x = fab_of(mg, l, fx, b);
    orc_fab *y = (fy >= 0) ? fab_of(mg, l, fy, b) : NULL;
    const int *v = vb(L, b);
#pragma omp parallel for schedule(static)
    for (int k = v[2]; k <= v[5]; ++k)
      for (int j = v[1]; j <= v[4]; ++j)
        for (int i = v[0]; i <= v[3]; ++i) {
          double *px = &AT(x, i, j, k);
          switch (kind) {
            case 0: *px = AT(y, i, j, k); break;
            case 1: *px = *px + s * AT(y, i, j, k); break;
            case 2: *px = *px * s; break;
            default: *px = *px * AT(y, i, j, k); break;
          }
        }
  }
}
double orc_mg_dot(orc_mg *mg, int l, int fx, int fy) {
  orc_level *L = &mg->lev[l];
  double s = 0.0;
  for (int b = 0; b < L->nbox; ++b) {
    orc_fab *x = fab_of(mg, l, fx, b), *y = fab_of(mg, l, fy, b);
    const int *v = vb(L, b);
    for (int k = v[2]; k <= v[5]; ++k)
      for (int j = v[1]; j <= v[4]; ++j)
        for (int i = v[0]; i <= v[3]; ++i) s = s + AT(x, i, j, k) * AT(y, i, j, k);
  }
  return s;
}
double orc_mg_norm(orc_mg *mg, int l, int f, int norm_type) {
  orc_level *L = &mg->lev[l];
  double s = 0.0;
  for (int b = 0; b < L->nbox; ++b) {
    orc_fab *x = fab_of(mg, l, f, b);
    const int *v = vb(L, b);
    for (int k = v[2]; k <= v[5]; ++k)
      for (int j = v[1]; j <= v[4]; ++j)
        for (int i = v[0]; i <= v[3]; ++i) {
          const double a = fabs(AT(x, i, j, k));
          if (norm_type == 0) s = (a > s) ? a : s;
          else if (norm_type == 1) s = s + a;
          else s = s + a * a;
        }
  }
  return (norm_type == 2) ? sqrt(s) : s;
}

/* [Chombo] LevelData::exchange with m_exchangeCopier =
 * exchangeDefine(grids, Unit) + trimEdges (VariableCoeffPoissonOperator
 * Factory.cpp:82-99): every box's six 1-deep face slabs (edges/corners
 * trimmed) are filled from the valid cells of whichever box -- or periodic
 * image of a box -- covers them. */
void orc_mg_exchange(orc_mg *mg, int l, int field) {
  orc_level *L = &mg->lev[l];
  int len[3];
  for (int d = 0; d < 3; ++d) len[d] = L->dom[3 + d] - L->dom[d] + 1;
  for (int db = 0; db < L->nbox; ++db) {
    orc_fab *dst = fab_of(mg, l, field, db);
    const int *dv = vb(L, db);
    for (int dir = 0; dir < 3; ++dir)
      for (int side = 0; side < 2; ++side) {
        int R[6];
        memcpy(R, dv, sizeof(R));
        if (side == 0) R[dir] = R[3 + dir] = dv[dir] - 1;
        else R[dir] = R[3 + dir] = dv[3 + dir] + 1;
        for (int sb = 0; sb < L->nbox; ++sb) {
          const int *sv = vb(L, sb);
          orc_fab *src = fab_of(mg, l, field, sb);
          for (int sz = -1; sz <= 1; ++sz)
            for (int sy = -1; sy <= 1; ++sy)
              for (int sx = -1; sx <= 1; ++sx) {
                const int sh[3] = {sx * len[0], sy * len[1], sz * len[2]};
                if ((sx && !mg->prm.periodic[0]) || (sy && !mg->prm.periodic[1]) ||
                    (sz && !mg->prm.periodic[2]))
                  continue;
                int X[6], empty = 0;
                for (int d = 0; d < 3; ++d) {
                  X[d] = R[d] > sv[d] + sh[d] ? R[d] : sv[d] + sh[d];
                  X[3 + d] = R[3 + d] < sv[3 + d] + sh[d] ? R[3 + d] : sv[3 + d] + sh[d];
                  if (X[d] > X[3 + d]) empty = 1;
                }
                if (empty) continue;
                for (int k = X[2]; k <= X[5]; ++k)
                  for (int j = X[1]; j <= X[4]; ++j)
                    for (int i = X[0]; i <= X[3]; ++i)
                      AT(dst, i, j, k) = AT(src, i - sh[0], j - sh[1], k - sh[2]);
              }
        }
      }
  }
}

/* ParseBC, Source/SetBCs.cpp:49-131, with [Chombo] DiriBC (order 1:
 * ghost = 2*value - near) and NeumBC (ghost = near + isign*dx*value). */
void orc_mg_fill_bc(orc_mg *mg, int l, int field, int homogeneous) {
  orc_level *L = &mg->lev[l];
  const orc_mg_params *p = &mg->prm;
  for (int b = 0; b < L->nbox; ++b) {
    orc_fab *u = fab_of(mg, l, field, b);
    const int *v = vb(L, b);
    int contained = 1;
    for (int d = 0; d < 3; ++d)
      if (u->lo[d] < L->dom[d] || u->hi[d] > L->dom[3 + d]) contained = 0;
    if (contained) continue; /* :51 */
    for (int dir = 0; dir < 3; ++dir) {
      if (p->periodic[dir]) continue; /* :65 */
      for (int side = 0; side < 2; ++side) {
        const int at_dom = side == 0 ? (v[dir] == L->dom[dir]) : (v[3 + dir] == L->dom[3 + dir]);
        if (!at_dom) continue; /* :68, :98 */
        const int flag = side == 0 ? p->bc_lo[dir] : p->bc_hi[dir];
        if (flag == 2) continue; /* periodic flag: no-op (:86-92, :116-121) */
        if (flag != 0 && flag != 1) {
          fprintf(stderr, "bogus bc flag\n"); /* MayDay::Error (:94, :123) */
          abort();
        }
        const int isign = side == 0 ? -1 : 1;
        int R[6];
        memcpy(R, v, sizeof(R));
        if (side == 0) R[dir] = R[3 + dir] = v[dir] - 1;
        else R[dir] = R[3 + dir] = v[3 + dir] + 1;
        const double val = homogeneous ? 0.0 : p->bc_value; /* ParseValue :42-47 */
        for (int k = R[2]; k <= R[5]; ++k)
          for (int j = R[1]; j <= R[4]; ++j)
            for (int i = R[0]; i <= R[3]; ++i) {
              int n[3] = {i, j, k};
              n[dir] -= isign; /* ivClose = ivTo - isign*BASISV(dir) */
              const double near = AT(u, n[0], n[1], n[2]);
              if (flag == 0) {
                AT(u, i, j, k) = 2.0 * val - near;
              } else {
                AT(u, i, j, k) = near;
                if (!homogeneous) AT(u, i, j, k) = near + (double)isign * L->dx * val;
              }
            }
      }
    }
  }
}

/* MGnewOp coefficient coarsening + computeLambda
 * (VariableCoeffPoissonOperatorFactory.cpp:194-229) */
void orc_mg_setup(orc_mg *mg) {
  for (int l = 1; l < mg->nlev; ++l) {
    orc_level *L = &mg->lev[l];
    for (int b = 0; b < L->nbox; ++b) {
      const int *v = vb(L, b);
      const int lo[3] = {v[0], v[1], v[2]}, hi[3] = {v[3], v[4], v[5]};
      orc_average(fab_of(mg, l, ORC_ACOEF, b), fab_of(mg, 0, ORC_ACOEF, b), lo, hi, 1 << l,
                  mg->prm.avg_type);
      orc_average(fab_of(mg, l, ORC_BCOEF, b), fab_of(mg, 0, ORC_BCOEF, b), lo, hi, 1 << l,
                  mg->prm.avg_type);
    }
  }
  for (int l = 0; l < mg->nlev; ++l) {
    orc_level *L = &mg->lev[l];
    for (int b = 0; b < L->nbox; ++b) {
      const int *v = vb(L, b);
      const int lo[3] = {v[0], v[1], v[2]}, hi[3] = {v[3], v[4], v[5]};
      orc_lambda(fab_of(mg, l, ORC_LAMBDA, b), fab_of(mg, l, ORC_ACOEF, b), lo, hi,
                 mg->prm.alpha, mg->prm.beta, L->dx);
    }
  }
}

/* levelGSRB, VariableCoeffPoissonOperator.cpp:273-332 */
void orc_mg_level_gsrb(orc_mg *mg, int l, int fu, int frhs) {
  orc_level *L = &mg->lev[l];
  for (int pass = 0; pass <= 1; ++pass) { /* :290 */
    orc_mg_exchange(mg, l, fu);           /* :301 */
    orc_mg_fill_bc(mg, l, fu, 1);         /* :307-310 */
    for (int b = 0; b < L->nbox; ++b) {   /* :313-330 */
      const int *v = vb(L, b);
      const int lo[3] = {v[0], v[1], v[2]}, hi[3] = {v[3], v[4], v[5]};
      orc_gsrbhelmholtzvc3d(fab_of(mg, l, fu, b), fab_of(mg, l, frhs, b), lo, hi, L->dx,
                            mg->prm.alpha, fab_of(mg, l, ORC_ACOEF, b), mg->prm.beta,
                            fab_of(mg, l, ORC_BCOEF, b), fab_of(mg, l, ORC_LAMBDA, b), pass);
    }
  }
}

/* residualI, VariableCoeffPoissonOperator.cpp:30-67 */
void orc_mg_residual(orc_mg *mg, int l, int fr, int fu, int frhs, int homogeneous) {
  orc_level *L = &mg->lev[l];
  orc_mg_fill_bc(mg, l, fu, homogeneous); /* :43-45 */
  orc_mg_exchange(mg, l, fu);             /* :48 */
  for (int b = 0; b < L->nbox; ++b) {
    const int *v = vb(L, b);
    const int lo[3] = {v[0], v[1], v[2]}, hi[3] = {v[3], v[4], v[5]};
    orc_vccomputeres3d(fab_of(mg, l, fr, b), fab_of(mg, l, fu, b), fab_of(mg, l, frhs, b),
                       mg->prm.alpha, fab_of(mg, l, ORC_ACOEF, b), mg->prm.beta,
                       fab_of(mg, l, ORC_BCOEF, b), lo, hi, L->dx);
  }
}

/* applyOpI + applyOpNoBoundary, VariableCoeffPoissonOperator.cpp:106-149 */
void orc_mg_apply_op(orc_mg *mg, int l, int flu, int fu, int homogeneous) {
  orc_level *L = &mg->lev[l];
  orc_mg_fill_bc(mg, l, fu, homogeneous); /* :115-117 */
  orc_mg_exchange(mg, l, fu);             /* :131 */
  for (int b = 0; b < L->nbox; ++b) {
    const int *v = vb(L, b);
    const int lo[3] = {v[0], v[1], v[2]}, hi[3] = {v[3], v[4], v[5]};
    orc_vccomputeop3d(fab_of(mg, l, flu, b), fab_of(mg, l, fu, b), mg->prm.alpha,
                      fab_of(mg, l, ORC_ACOEF, b), mg->prm.beta, fab_of(mg, l, ORC_BCOEF, b),
                      lo, hi, L->dx);
  }
}

/* levelJacobi, VariableCoeffPoissonOperator.cpp:360-385 */
void orc_mg_level_jacobi(orc_mg *mg, int l, int fu, int frhs) {
  orc_mg_residual(mg, l, ORC_TMP, fu, frhs, 1); /* :372 */
  lv_op(mg, l, ORC_TMP, ORC_LAMBDA, 0.0, 3);    /* :377 resid *= lambda */
  lv_op(mg, l, fu, ORC_TMP, 0.5, 1);            /* :381 incr(dpsi, resid, 0.5) */
  orc_mg_exchange(mg, l, fu);                   /* :384 */
}

/* [Chombo] AMRPoissonOp::relax: s_relaxMode 1 -> levelGSRB, 4 -> levelJacobi */
void orc_mg_relax(orc_mg *mg, int l, int fu, int frhs, int n) {
  for (int it = 0; it < n; ++it) {
    if (mg->prm.relax_mode == 4) orc_mg_level_jacobi(mg, l, fu, frhs);
    else orc_mg_level_gsrb(mg, l, fu, frhs);
  }
}

/* restrictResidual, VariableCoeffPoissonOperator.cpp:151-194: writes the
 * coarse residual into RESID of level l+1 */
void orc_mg_restrict_residual(orc_mg *mg, int l, int fu, int frhs) {
  orc_level *L = &mg->lev[l];
  orc_mg_fill_bc(mg, l, fu, 1); /* :158-161 */
  orc_mg_exchange(mg, l, fu);   /* :163 */
  for (int b = 0; b < L->nbox; ++b) {
    const int *v = vb(L, b);
    const int lo[3] = {v[0], v[1], v[2]}, hi[3] = {v[3], v[4], v[5]};
    orc_restrictresvc3d(fab_of(mg, l + 1, ORC_RESID, b), fab_of(mg, l, fu, b),
                        fab_of(mg, l, frhs, b), mg->prm.alpha, fab_of(mg, l, ORC_ACOEF, b),
                        mg->prm.beta, fab_of(mg, l, ORC_BCOEF, b), lo, hi, L->dx);
  }
}

/* [Chombo] prolongIncrement: fu(level l) += P(CORR(level l+1)) */
void orc_mg_prolong_increment(orc_mg *mg, int l, int fu) {
  orc_level *L = &mg->lev[l], *C = &mg->lev[l + 1];
  if (mg->prm.prolong_type == 1) orc_mg_exchange(mg, l + 1, ORC_CORR);
  for (int b = 0; b < L->nbox; ++b) {
    const int *v = vb(L, b), *cv = vb(C, b);
    const int lo[3] = {v[0], v[1], v[2]}, hi[3] = {v[3], v[4], v[5]};
    const int clo[3] = {cv[0], cv[1], cv[2]}, chi[3] = {cv[3], cv[4], cv[5]};
    int alo[3], ahi[3];
    for (int d = 0; d < 3; ++d) {
      alo[d] = mg->prm.periodic[d] || cv[d] > C->dom[d];
      ahi[d] = mg->prm.periodic[d] || cv[3 + d] < C->dom[3 + d];
    }
    orc_prolong(fab_of(mg, l, fu, b), fab_of(mg, l + 1, ORC_CORR, b), lo, hi, clo, chi, alo, ahi,
                mg->prm.prolong_type);
  }
}

/* preCond, VariableCoeffPoissonOperator.cpp:72-104 */
void orc_mg_precond(orc_mg *mg, int l, int fe, int fr) {
  lv_op(mg, l, fe, fr, 0.0, 0);         /* :99 copy */
  lv_op(mg, l, fe, ORC_LAMBDA, 0.0, 3); /* :100 mult by lambda */
  orc_mg_relax(mg, l, fe, fr, 2);       /* :103 */
}

void orc_mg_one_cycle(orc_mg *mg, int l);

typedef struct {
  int imax;
  double eps, reps, small;
  int restarts, norm_type;
  int mg_iters; /* 0: op->preCond (bottom solver); > 0: MultilevelLinearOp::preCond */
} bicg_cfg;

static void bicg_precond(orc_mg *mg, int l, int fe, int fr, const bicg_cfg *c) {
  if (c->mg_iters > 0)
    orc_mg_amr_precond(mg, fe, fr, c->mg_iters);
  else
    orc_mg_precond(mg, l, fe, fr);
}

/* MultilevelLinearOp::preCond on one AMR level (Main_PoissonSolver.cpp:
 * 107-117 sets m_num_mg_iterations / m_num_mg_smooth), restated
 * (unpinned): e = 0, then `iters` AMRMultiGrid iterations on (e, r) with
 * homogeneous BC: CORR = 0; oneCycle(CORR, RESID); e += CORR;
 * RESID = r - L(e).  Level-0 CORR / RESID are the MG's own fields. */
void orc_mg_amr_precond(orc_mg *mg, int fe, int fr, int iters) {
  lv_zero_all(mg, 0, fe);
  orc_mg_residual(mg, 0, ORC_RESID, fe, fr, 1);
  for (int i = 0; i < iters; ++i) {
    lv_zero_all(mg, 0, ORC_CORR);
    orc_mg_one_cycle(mg, 0);
    lv_op(mg, 0, fe, ORC_CORR, 1.0, 1);
    orc_mg_residual(mg, 0, ORC_RESID, fe, fr, 1);
  }
}

/* [Chombo] BiCGStabSolver<T>::solve, restated (unpinned): van der Vorst
 * BiCGStab with a right preconditioner, m_eps relative tolerance on
 * norm(r, m_normType), |m| <= m_small*|rho| restarts. */
static int bicgstab_core(orc_mg *mg, int l, int fe, int fr, int hom, const bicg_cfg *c) {
  const bicg_cfg *p = c;
  const int nt = c->norm_type;
  orc_mg_residual(mg, l, W_R, fe, fr, hom);
  lv_op(mg, l, W_RT, W_R, 0.0, 0);
  lv_zero_all(mg, l, W_E);
  lv_zero_all(mg, l, W_PT);
  lv_zero_all(mg, l, W_ST);
  lv_zero_all(mg, l, W_P);
  lv_zero_all(mg, l, W_V);
  double rho1 = 0.0, rho2 = 0.0, alpha = 0.0, beta = 0.0, omega = 0.0;
  const double init_norm = orc_mg_norm(mg, l, W_R, nt);
  double nrm = init_norm;
  int it = 0, init = 1, restarts = 0;
  while (it < p->imax && nrm > p->eps * init_norm && nrm > p->reps) {
    ++it;
    rho2 = rho1;
    rho1 = orc_mg_dot(mg, l, W_RT, W_R);
    if (rho1 == 0.0) break;
    if (init) {
      lv_op(mg, l, W_P, W_R, 0.0, 0);
      init = 0;
    } else {
      beta = (rho1 / rho2) * (alpha / omega);
      lv_op(mg, l, W_P, -1, beta, 2);
      lv_op(mg, l, W_P, W_V, -beta * omega, 1);
      lv_op(mg, l, W_P, W_R, 1.0, 1);
    }
    bicg_precond(mg, l, W_PT, W_P, c);
    lv_zero_all(mg, l, W_V);
    orc_mg_apply_op(mg, l, W_V, W_PT, 1);
    const double m = orc_mg_dot(mg, l, W_RT, W_V);
    if (fabs(m) > p->small * fabs(rho1)) {
      alpha = rho1 / m;
      lv_op(mg, l, W_S, W_R, 0.0, 0);
      lv_op(mg, l, W_S, W_V, -alpha, 1);
      lv_op(mg, l, W_E, W_PT, alpha, 1);
      nrm = orc_mg_norm(mg, l, W_S, nt);
      if (nrm <= p->eps * init_norm || nrm <= p->reps) break;
      bicg_precond(mg, l, W_ST, W_S, c);
      lv_zero_all(mg, l, W_T);
      orc_mg_apply_op(mg, l, W_T, W_ST, 1);
      const double ts = orc_mg_dot(mg, l, W_T, W_S);
      const double tt = orc_mg_dot(mg, l, W_T, W_T);
      if (tt == 0.0) break;
      omega = ts / tt;
      lv_op(mg, l, W_R, W_S, 0.0, 0);
      lv_op(mg, l, W_R, W_T, -omega, 1);
      lv_op(mg, l, W_E, W_ST, omega, 1);
      nrm = orc_mg_norm(mg, l, W_R, nt);
      if (omega == 0.0) break;
    } else {
      if (restarts >= p->restarts) break;
      ++restarts;
      lv_op(mg, l, fe, W_E, 1.0, 1);
      orc_mg_residual(mg, l, W_R, fe, fr, hom);
      lv_op(mg, l, W_RT, W_R, 0.0, 0);
      lv_zero_all(mg, l, W_E);
      nrm = orc_mg_norm(mg, l, W_R, nt);
      init = 1;
    }
  }
  lv_op(mg, l, fe, W_E, 1.0, 1);
  mg->last_iters = it;
  return it;
}

int orc_mg_bicgstab(orc_mg *mg, int l, int fe, int fr, int hom) {
  const orc_mg_params *p = &mg->prm;
  const bicg_cfg c = {p->bicg_imax, p->bicg_eps, p->bicg_reps, p->bicg_small, p->bicg_restarts,
                      p->bicg_norm_type, 0};
  return bicgstab_core(mg, l, fe, fr, hom, &c);
}

/* solver.solve(dpsi, rhs) of Main_PoissonSolver.cpp:174-184 on one AMR
 * level: BiCGStab (m_normType = 0, m_eps = tolerance, m_imax =
 * max_iterations, inhomogeneous BC) on PHI / RHS, preconditioned by
 * MultilevelLinearOp::preCond.  Returns the iteration count; *final_norm =
 * norm(RHS - L(PHI), norm_type) afterwards (RESID holds it). */
int orc_mg_solve(orc_mg *mg, int mg_iters, int imax, double eps, int norm_type,
                 double *final_norm) {
  const orc_mg_params *p = &mg->prm;
  const bicg_cfg c = {imax, eps, p->bicg_reps, p->bicg_small, p->bicg_restarts, norm_type,
                      mg_iters > 0 ? mg_iters : 1};
  const int it = bicgstab_core(mg, 0, ORC_PHI, ORC_RHS, 0, &c);
  orc_mg_residual(mg, 0, ORC_RESID, ORC_PHI, ORC_RHS, 0);
  if (final_norm) *final_norm = orc_mg_norm(mg, 0, ORC_RESID, norm_type);
  return it;
}

/* [Chombo] MultiGrid::oneCycle(e, res) on (CORR, RESID) of level l */
void orc_mg_one_cycle(orc_mg *mg, int l) {
  const orc_mg_params *p = &mg->prm;
  if (l == mg->nlev - 1) {
    if (p->bottom_solver == 1) orc_mg_bicgstab(mg, l, ORC_CORR, ORC_RESID, 1);
    else orc_mg_relax(mg, l, ORC_CORR, ORC_RESID, p->n_bottom);
    return;
  }
  orc_mg_relax(mg, l, ORC_CORR, ORC_RESID, p->n_pre);
  orc_mg_restrict_residual(mg, l, ORC_CORR, ORC_RESID);
  lv_zero_all(mg, l + 1, ORC_CORR);
  orc_mg_one_cycle(mg, l + 1);
  orc_mg_prolong_increment(mg, l, ORC_CORR);
  orc_mg_relax(mg, l, ORC_CORR, ORC_RESID, p->n_post);
}

double orc_mg_init_residual(orc_mg *mg, int norm_type) {
  orc_mg_residual(mg, 0, ORC_RESID, ORC_PHI, ORC_RHS, 0);
  return orc_mg_norm(mg, 0, ORC_RESID, norm_type);
}

/* one [Chombo] AMRMultiGrid iteration on a single AMR level */
double orc_mg_iteration(orc_mg *mg, int norm_type) {
  lv_zero_all(mg, 0, ORC_CORR);
  orc_mg_one_cycle(mg, 0);
  lv_op(mg, 0, ORC_PHI, ORC_CORR, 1.0, 1);
  orc_mg_residual(mg, 0, ORC_RESID, ORC_PHI, ORC_RHS, 0);
  return orc_mg_norm(mg, 0, ORC_RESID, norm_type);
}

/* Full multigrid (FMG) from RESID at level 0 (as left by init_residual /
 * iteration), the schedule of mg_ic_code_amd/csrc/op.cpp MultiGrid::fmg:
 * RESID(l+1) = restrictResidual of a zero CORR(l) at every depth, the bottom
 * solve from zero, then per finer depth CORR = P CORR(l+1) and `ncycles`
 * oneCycle(CORR, RESID); PHI += CORR(0); RESID = RHS - L(PHI).  Not a
 * reference algorithm (BASELINE config C5 names FMG; Chombo's AMRMultiGrid
 * has no FMG driver), so parity unpinned. */
double orc_mg_fmg(orc_mg *mg, int ncycles, int norm_type) {
  const orc_mg_params *p = &mg->prm;
  const int D = mg->nlev;
  if (D == 1) {
    lv_zero_all(mg, 0, ORC_CORR);
    orc_mg_one_cycle(mg, 0);
  } else {
    for (int l = 0; l + 1 < D; ++l) {
      lv_zero_all(mg, l, ORC_CORR);
      orc_mg_restrict_residual(mg, l, ORC_CORR, ORC_RESID);
    }
    lv_zero_all(mg, D - 1, ORC_CORR);
    if (p->bottom_solver == 1) orc_mg_bicgstab(mg, D - 1, ORC_CORR, ORC_RESID, 1);
    else orc_mg_relax(mg, D - 1, ORC_CORR, ORC_RESID, p->n_bottom);
    for (int l = D - 2; l >= 0; --l) {
      lv_zero_all(mg, l, ORC_CORR);
      orc_mg_prolong_increment(mg, l, ORC_CORR);
      for (int c = 0; c < ncycles; ++c) orc_mg_one_cycle(mg, l);
    }
  }
  lv_op(mg, 0, ORC_PHI, ORC_CORR, 1.0, 1);
  orc_mg_residual(mg, 0, ORC_RESID, ORC_PHI, ORC_RHS, 0);
  return orc_mg_norm(mg, 0, ORC_RESID, norm_type);
}

/* ------------------------------------------------------------------ */
/* Input generator at psi = 1                                          */
/* ------------------------------------------------------------------ */
static double phi_fn(const orc_bh_params *p, const double loc[3]) {
  /* MyPhiFunction.H:11-16 */
  const double r2 = loc[0] * loc[0] + loc[1] * loc[1] + loc[2] * loc[2];
  return p->phi_amplitude * exp(-r2 / p->phi_wavelength);
}
static void cell_loc(const int iv[3], double dx, const double domlen[3], double loc[3]) {
  /* SetLevelData.cpp:101-103 */
  for (int d = 0; d < 3; ++d) loc[d] = ((double)iv[d] + 0.5) * dx - domlen[d] / 2.0;
}
static double bh_radius(double loc_bh[3], double off) { /* SetBinaryBH.H:15-20 */
  loc_bh[0] -= off;
  return sqrt(loc_bh[0] * loc_bh[0] + loc_bh[1] * loc_bh[1] + loc_bh[2] * loc_bh[2]);
}
static double get_Aij(int i, int j, double r1, double r2, const double *n1, const double *n2,
                      const double *J1, const double *J2, const double *P1, const double *P2) {
  /* SetBinaryBH.H:24-53 */
  double eps[3][3][3] = {{{0}}};
  eps[0][1][2] = 1.0;
  eps[1][2][0] = 1.0;
  eps[2][0][1] = 1.0;
  eps[0][2][1] = -1.0;
  eps[2][1][0] = -1.0;
  eps[1][0][2] = -1.0;
  double Aij = 1.5 / r1 / r1 * (n1[i] * P1[j] + n1[j] * P1[i]) +
               1.5 / r2 / r2 * (n2[i] * P2[j] + n2[j] * P2[i]);
  for (int k = 0; k < 3; k++) {
    Aij += 1.5 / r1 / r1 * (n1[i] * n1[j] - (double)(i == j)) * P1[k] * n1[k] +
           1.5 / r2 / r2 * (n2[i] * n2[j] - (double)(i == j)) * P2[k] * n2[k];
    for (int l = 0; l < 3; l++) {
      Aij += -3.0 / r1 / r1 / r1 * (eps[i][l][k] * n1[j] + eps[j][l][k] * n1[i]) * n1[l] * J1[k] -
             3.0 / r2 / r2 / r2 * (eps[i][l][k] * n2[j] + eps[j][l][k] * n2[i]) * n2[l] * J2[k];
    }
  }
  return Aij;
}

static void nl_core(const orc_bh_params *p, const int *lo, const int *hi, double dx,
                    const double *psi, double *acoef, double *rhs, int integrand) {
  const double domlen[3] = {p->L, p->L, p->L};
  const size_t nx = (size_t)(hi[0] - lo[0] + 1), ny = (size_t)(hi[1] - lo[1] + 1);
#pragma omp parallel for schedule(static)
  for (int k = lo[2]; k <= hi[2]; ++k)
    for (int j = lo[1]; j <= hi[1]; ++j)
      for (int i = lo[0]; i <= hi[0]; ++i) {
        const int iv[3] = {i, j, k};
        double loc[3];
        cell_loc(iv, dx, domlen, loc);
        /* GETRHOGRADPHIF, SetLevelDataF.ChF:65-103 */
        double rho_grad = 0.0;
        for (int d0 = 0; d0 < 3; ++d0) {
          int ip[3] = {i, j, k}, im[3] = {i, j, k};
          ip[d0] += 1;
          im[d0] -= 1;
          double lp[3], lm[3];
          cell_loc(ip, dx, domlen, lp);
          cell_loc(im, dx, domlen, lm);
          const double dphidx = 0.5 / dx * (+phi_fn(p, lp) - phi_fn(p, lm));
          rho_grad = rho_grad + 0.5 * dphidx * dphidx;
        }
        /* set_binary_bh_Aij, SetBinaryBH.H:55-83 */
        double l1[3] = {loc[0], loc[1], loc[2]}, l2[3] = {loc[0], loc[1], loc[2]};
        const double r1 = bh_radius(l1, p->bh1_offset);
        const double r2 = bh_radius(l2, p->bh2_offset);
        const double n1[3] = {l1[0] / r1, l1[1] / r1, l1[2] / r1};
        const double n2[3] = {l2[0] / r2, l2[1] / r2, l2[2] / r2};
        const double J1[3] = {0.0, 0.0, p->bh1_spin}, J2[3] = {0.0, 0.0, p->bh2_spin};
        const double P1[3] = {0.0, p->bh1_momentum, 0.0}, P2[3] = {0.0, p->bh2_momentum, 0.0};
        const double A11 = get_Aij(0, 0, r1, r2, n1, n2, J1, J2, P1, P2);
        const double A22 = get_Aij(1, 1, r1, r2, n1, n2, J1, J2, P1, P2);
        const double A33 = get_Aij(2, 2, r1, r2, n1, n2, J1, J2, P1, P2);
        const double A12 = get_Aij(0, 1, r1, r2, n1, n2, J1, J2, P1, P2);
        const double A13 = get_Aij(0, 2, r1, r2, n1, n2, J1, J2, P1, P2);
        const double A23 = get_Aij(1, 2, r1, r2, n1, n2, J1, J2, P1, P2);
        /* SetLevelData.cpp:312-317 */
        const double A2 = pow(A11, 2.0) + pow(A22, 2.0) + pow(A33, 2.0) + 2 * pow(A12, 2.0) +
                          2 * pow(A13, 2.0) + 2 * pow(A23, 2.0);
        /* set_m_value, :266-278 (Pi = V = 0) */
        const double rho = 0.5 * 0.0 * 0.0 + 0.0;
        const double K = integrand ? 0.0 : p->constant_K; /* :161 set_m_value(.., 0.0) */
        const double m = (2.0 / 3.0) * (K * K) - 16.0 * M_PI * p->G_Newton * rho;
        /* set_binary_bh_psi, SetBinaryBH.H:85-99; psi = 1 (:54) */
        double b1[3] = {loc[0], loc[1], loc[2]}, b2[3] = {loc[0], loc[1], loc[2]};
        const double rb1 = bh_radius(b1, p->bh1_offset), rb2 = bh_radius(b2, p->bh2_offset);
        const double psi_bh = p->bh1_bare_mass / rb1 + p->bh2_bare_mass / rb2;
        /* psi over the box grown by one (NULL: psi == 1, set_initial_conditions :54) */
        const size_t gx = nx + 2, gy = ny + 2;
        const size_t gc = (size_t)(i - lo[0] + 1) + gx * ((size_t)(j - lo[1] + 1) +
                                                          gy * (size_t)(k - lo[2] + 1));
        const size_t gs[3] = {1, gx, gx * gy};
        const double psi_c = psi ? psi[gc] : 1.0;
        const double psi_0 = psi_c + psi_bh; /* SetLevelData.cpp:319-320 */
        /* GETLAPLACIANPSIF (SetLevelDataF.ChF:15-58), 2nd order */
        double lap = 0.0;
        for (int d0 = 0; d0 < 3; ++d0) {
          const double pm = psi ? psi[gc - gs[d0]] : 1.0, pp = psi ? psi[gc + gs[d0]] : 1.0;
          lap = lap + 1.0 / dx / dx * (+1.0 * pm - 2.0 * psi_c + 1.0 * pp);
        }
        const size_t n = (size_t)(i - lo[0]) + nx * ((size_t)(j - lo[1]) + ny * (size_t)(k - lo[2]));
        if (integrand) { /* set_constant_K_integrand, SetLevelData.cpp:174-177 */
          acoef[n] = -1.5 * m + 1.5 * A2 * pow(psi_0, -12.0) +
                     24.0 * M_PI * p->G_Newton * rho_grad * pow(psi_0, -4.0) +
                     12.0 * lap * pow(psi_0, -5.0);
          continue;
        }
        /* set_a_coef, SetLevelData.cpp:321-322 */
        acoef[n] = -0.625 * m * pow(psi_0, 4.0) - A2 * pow(psi_0, -8.0) +
                   2.0 * M_PI * p->G_Newton * rho_grad;
        /* set_rhs, SetLevelData.cpp:121-124 */
        rhs[n] = 0.125 * m * pow(psi_0, 5.0) - 0.125 * A2 * pow(psi_0, -7.0) -
                 2.0 * M_PI * p->G_Newton * rho_grad * psi_0 - lap;
      }
}

/* GETLAPLACIANPSIF / GETRHOGRADPHIF (SetLevelDataF.ChF:15-58, :65-103) on
 * [lo, hi]; `in` over the box grown by one, `out` over the box, i fastest */
void orc_getlaplacianpsif(double *out, const double *in, const int *lo, const int *hi, double dx,
                          int laplacian) {
  const size_t nx = (size_t)(hi[0] - lo[0] + 1), ny = (size_t)(hi[1] - lo[1] + 1);
  const size_t gx = nx + 2, gy = ny + 2, gs[3] = {1, gx, gx * gy};
  for (int k = lo[2]; k <= hi[2]; ++k)
    for (int j = lo[1]; j <= hi[1]; ++j)
      for (int i = lo[0]; i <= hi[0]; ++i) {
        const size_t c = (size_t)(i - lo[0] + 1) + gx * ((size_t)(j - lo[1] + 1) +
                                                          gy * (size_t)(k - lo[2] + 1));
        double acc = 0.0;
        for (int d0 = 0; d0 < 3; ++d0) {
          if (laplacian) {
            const double d2 =
                1.0 / dx / dx * (+1.0 * in[c - gs[d0]] - 2.0 * in[c] + 1.0 * in[c + gs[d0]]);
            acc = acc + d2;
          } else {
            const double dphidx = 0.5 / dx * (+in[c + gs[d0]] - in[c - gs[d0]]);
            acc = acc + 0.5 * dphidx * dphidx;
          }
        }
        out[(size_t)(i - lo[0]) + nx * ((size_t)(j - lo[1]) + ny * (size_t)(k - lo[2]))] = acc;
      }
}

void orc_nl_coefs(const orc_bh_params *p, const int *lo, const int *hi, double dx,
                  const double *psi, double *acoef, double *rhs) {
  nl_core(p, lo, hi, dx, psi, acoef, rhs, 0);
}

void orc_nl_integrand(const orc_bh_params *p, const int *lo, const int *hi, double dx,
                      const double *psi, double *out) {
  nl_core(p, lo, hi, dx, psi, out, NULL, 1);
}

/* aCoef / rhs at psi = 1 (NL iteration 0) */
void orc_binary_bh_coefs(const orc_bh_params *p, const int *lo, const int *hi, double dx,
                         double *acoef, double *rhs) {
  orc_nl_coefs(p, lo, hi, dx, NULL, acoef, rhs);
}

void orc_output_vars(int kind, const orc_bh_params *p, const int *lo, const int *hi, double dx,
                     const double *psi, const double *dpsi, const double *rhs, double *out) {
  const double domlen[3] = {p->L, p->L, p->L};
  const size_t nx = (size_t)(hi[0] - lo[0] + 1), ny = (size_t)(hi[1] - lo[1] + 1),
               nz = (size_t)(hi[2] - lo[2] + 1);
  const size_t V = nx * ny * nz;
  for (int k = lo[2]; k <= hi[2]; ++k)
    for (int j = lo[1]; j <= hi[1]; ++j)
      for (int i = lo[0]; i <= hi[0]; ++i) {
        const int iv[3] = {i, j, k};
        const size_t n = (size_t)(i - lo[0]) + nx * ((size_t)(j - lo[1]) + ny * (size_t)(k - lo[2]));
        double loc[3];
        cell_loc(iv, dx, domlen, loc); /* SetLevelData.cpp:375-378 */
        /* multigrid_vars A_ij_0, phi_0 as set_initial_conditions left them
         * (SetLevelData.cpp:60-69, SetBinaryBH.H:55-83) */
        double l1[3] = {loc[0], loc[1], loc[2]}, l2[3] = {loc[0], loc[1], loc[2]};
        const double r1 = bh_radius(l1, p->bh1_offset);
        const double r2 = bh_radius(l2, p->bh2_offset);
        const double n1[3] = {l1[0] / r1, l1[1] / r1, l1[2] / r1};
        const double n2[3] = {l2[0] / r2, l2[1] / r2, l2[2] / r2};
        const double J1[3] = {0.0, 0.0, p->bh1_spin}, J2[3] = {0.0, 0.0, p->bh2_spin};
        const double P1[3] = {0.0, p->bh1_momentum, 0.0}, P2[3] = {0.0, p->bh2_momentum, 0.0};
        const double A11 = get_Aij(0, 0, r1, r2, n1, n2, J1, J2, P1, P2);
        const double A22 = get_Aij(1, 1, r1, r2, n1, n2, J1, J2, P1, P2);
        const double A33 = get_Aij(2, 2, r1, r2, n1, n2, J1, J2, P1, P2);
        const double A12 = get_Aij(0, 1, r1, r2, n1, n2, J1, J2, P1, P2);
        const double A13 = get_Aij(0, 2, r1, r2, n1, n2, J1, J2, P1, P2);
        const double A23 = get_Aij(1, 2, r1, r2, n1, n2, J1, J2, P1, P2);
        const double phi0 = phi_fn(p, loc);
        if (kind == 1) { /* WriteOutput.H:74-100: dpsi, rhs, then multigrid_vars */
          const double v[10] = {dpsi[n], rhs[n], psi[n], A11, A12, A13, A22, A23, A33, phi0};
          for (int c = 0; c < 10; ++c) out[c * V + n] = v[c];
          continue;
        }
        /* set_output_data, SetLevelData.cpp:357-394 */
        double v[31];
        for (int c = 0; c < 31; ++c) v[c] = 0.0;
        v[1] = v[4] = v[6] = 1.0; /* h11, h22, h33 */
        v[18] = 1.0;              /* lapse */
        v[7] = p->constant_K;     /* K */
        double b1[3] = {loc[0], loc[1], loc[2]}, b2[3] = {loc[0], loc[1], loc[2]};
        const double psi_bh = p->bh1_bare_mass / bh_radius(b1, p->bh1_offset) +
                              p->bh2_bare_mass / bh_radius(b2, p->bh2_offset);
        const double chi = pow(psi[n] + psi_bh, -4.0);
        const double factor = pow(chi, 1.5);
        v[0] = chi;
        v[25] = phi0; /* phi */
        v[8] = A11 * factor;
        v[9] = A12 * factor;
        v[10] = A13 * factor;
        v[11] = A22 * factor;
        v[12] = A23 * factor;
        v[13] = A33 * factor;
        for (int c = 0; c < 31; ++c) out[c * V + n] = v[c];
      }
}

void orc_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}
int orc_get_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* Pin OpenMP thread t of the next parallel regions to cpus[t % n] (n > 0),
 * or release every thread to the process's CPU set cpus[0 .. n) (pin = 0):
 * the CPU baseline's "all host cores, pinned" (SURVEY 8(d)).  Returns the
 * number of threads whose affinity was set. */
int orc_pin_threads(const int *cpus, int n, int pin) {
#ifdef _OPENMP
  if (n <= 0) return 0;
  int done = 0;
#pragma omp parallel reduction(+ : done)
  {
    cpu_set_t set;
    CPU_ZERO(&set);
    if (pin) {
      CPU_SET(cpus[omp_get_thread_num() % n], &set);
    } else {
      for (int i = 0; i < n; ++i) CPU_SET(cpus[i], &set);
    }
    done += sched_setaffinity(0, sizeof(set), &set) == 0;
  }
  return done;
#else
  (void)cpus;
  (void)n;
  (void)pin;
  return 0;
#endif
}
