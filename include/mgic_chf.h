/*
 * mgic_chf.h -- host drop-ins for the reference's ChomboFortran C ABI.
 *
 * These are the exact symbols and argument lists that Chombo's chfpp
 * generates for Source/VariableCoeffPoissonOperatorF.ChF and
 * Source/SetLevelDataF.ChF and that the reference binds in
 * Source/VariableCoeffPoissonOperatorF_F.H / SetLevelDataF_F.H
 * (FORTRAN_NAME(GSRBHELMHOLTZVC3D, gsrbhelmholtzvc3d) -> gsrbhelmholtzvc3d_):
 *   CHF_FRA[x]        -> double *x, const int *xlo0..xlo2, const int *xhi0..xhi2,
 *                        const int *xnComp
 *   CHF_FRA1[x]       -> the same without xnComp (one component)
 *   CHF_BOX[b]        -> const int *blo0..blo2, const int *bhi0..bhi2
 *   CHF_CONST_REAL[r] -> const double *r
 *   CHF_CONST_INT[i]  -> const int *i
 * Arrays are host FArrayBox data (column-major, i fastest, component
 * slowest).  Each call stages the operands to the GPU, runs the gfx950
 * kernel and copies the written region back -- a literal drop-in for the
 * object file built from the .ChF (linking libmgic.so in its place), meant
 * for parity checks.  The device-resident path (mgic.h) is the fast path.
 * Invalid arguments abort with a message, as MAYDAYERROR does in the
 * reference (.ChF:77-87).
 */
#ifndef MGIC_CHF_H
#define MGIC_CHF_H

#ifdef __cplusplus
extern "C" {
#endif

#define MGIC_CHF_FRA(x)                                                                    \
  double *x, const int *x##lo0, const int *x##lo1, const int *x##lo2, const int *x##hi0,   \
      const int *x##hi1, const int *x##hi2, const int *x##nComp
#define MGIC_CHF_CONST_FRA(x)                                                              \
  const double *x, const int *x##lo0, const int *x##lo1, const int *x##lo2,                \
      const int *x##hi0, const int *x##hi1, const int *x##hi2, const int *x##nComp
#define MGIC_CHF_FRA1(x)                                                                   \
  double *x, const int *x##lo0, const int *x##lo1, const int *x##lo2, const int *x##hi0,   \
      const int *x##hi1, const int *x##hi2
#define MGIC_CHF_CONST_FRA1(x)                                                             \
  const double *x, const int *x##lo0, const int *x##lo1, const int *x##lo2,                \
      const int *x##hi0, const int *x##hi1, const int *x##hi2
#define MGIC_CHF_BOX(b)                                                                    \
  const int *b##lo0, const int *b##lo1, const int *b##lo2, const int *b##hi0,              \
      const int *b##hi1, const int *b##hi2

/* VariableCoeffPoissonOperatorF_F.H:107-146 (GSRBHELMHOLTZVC3D) */
__attribute__((visibility("default"))) void gsrbhelmholtzvc3d_(
    MGIC_CHF_FRA(dpsi), MGIC_CHF_CONST_FRA(rhs), MGIC_CHF_BOX(region), const double *dx,
    const double *alpha, MGIC_CHF_CONST_FRA(aCoef), const double *beta,
    MGIC_CHF_CONST_FRA(bCoef), MGIC_CHF_CONST_FRA(lambda), const int *redBlack);

/* VariableCoeffPoissonOperatorF_F.H:233-266 (VCCOMPUTEOP3D) */
__attribute__((visibility("default"))) void vccomputeop3d_(
    MGIC_CHF_FRA(lofdpsi), MGIC_CHF_CONST_FRA(dpsi), const double *alpha,
    MGIC_CHF_CONST_FRA(aCoef), const double *beta, MGIC_CHF_CONST_FRA(bCoef),
    MGIC_CHF_BOX(region), const double *dx);

/* VariableCoeffPoissonOperatorF_F.H:359-395 (VCCOMPUTERES3D) */
__attribute__((visibility("default"))) void vccomputeres3d_(
    MGIC_CHF_FRA(res), MGIC_CHF_CONST_FRA(dpsi), MGIC_CHF_CONST_FRA(rhs), const double *alpha,
    MGIC_CHF_CONST_FRA(aCoef), const double *beta, MGIC_CHF_CONST_FRA(bCoef),
    MGIC_CHF_BOX(region), const double *dx);

/* VariableCoeffPoissonOperatorF_F.H:488-524 (RESTRICTRESVC3D); like the
 * Fortran it ACCUMULATES into res (the caller zeroes it first, .cpp:177) */
__attribute__((visibility("default"))) void restrictresvc3d_(
    MGIC_CHF_FRA(res), MGIC_CHF_CONST_FRA(dpsi), MGIC_CHF_CONST_FRA(rhs), const double *alpha,
    MGIC_CHF_CONST_FRA(aCoef), const double *beta, MGIC_CHF_CONST_FRA(bCoef),
    MGIC_CHF_BOX(region), const double *dx);

/* SetLevelDataF_F.H:15-19 (GETLAPLACIANPSIF): l = sum_d d2psi/dx_d^2 over box */
__attribute__((visibility("default"))) void getlaplacianpsif_(MGIC_CHF_FRA1(l_of_psi),
                                                              MGIC_CHF_CONST_FRA1(psi),
                                                              const double *dx, MGIC_CHF_BOX(box));

/* SetLevelDataF_F.H:43-47 (GETRHOGRADPHIF): rho = sum_d 0.5 (dphi/dx_d)^2 over box */
__attribute__((visibility("default"))) void getrhogradphif_(MGIC_CHF_FRA1(rho_grad_phi),
                                                            MGIC_CHF_CONST_FRA1(phi),
                                                            const double *dx, MGIC_CHF_BOX(box));

#ifdef __cplusplus
}
#endif
#endif /* MGIC_CHF_H */
