// chf_dropin.cpp -- the reference's ChomboFortran C ABI (include/mgic_chf.h)
// served by the gfx950 kernels.  Host FArrayBox operands are staged into
// the library's device geometry, the kernel runs, the written region is
// copied back.  Parity utility; the device-resident API is the fast path.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/mgic_chf.h"
#include "kernels.hpp"

using namespace mgic;

namespace {

struct HostFab {
  double *p;
  Box box;
  int nc;
  long idx(int i, int j, int k, int n) const {
    const long nx = box.size(0), ny = box.size(1), nz = box.size(2);
    return (long)(i - box.lo[0]) + nx * ((long)(j - box.lo[1]) + ny * ((long)(k - box.lo[2]) + nz * n));
  }
};

HostFab fab(const double *p, const int *l0, const int *l1, const int *l2, const int *h0,
            const int *h1, const int *h2, const int *nc) {
  HostFab f;
  f.p = const_cast<double *>(p);
  f.box.lo[0] = *l0;
  f.box.lo[1] = *l1;
  f.box.lo[2] = *l2;
  f.box.hi[0] = *h0;
  f.box.hi[1] = *h1;
  f.box.hi[2] = *h2;
  f.nc = *nc;
  return f;
}

[[noreturn]] void mayday(const char *msg) {
  std::fprintf(stderr, "MayDay: %s\n", msg);
  std::abort();
}

// one operand staged on the device in the common geometry of `region`
struct Stage {
  FabGeom g;
  double *base = nullptr;
  double *p = nullptr;
  double **tab = nullptr;
  explicit Stage(const Box &region) : g(FabGeom::make(region)) {
    MGIC_HIP(hipMalloc(&base, sizeof(double) * (size_t)g.total));
    MGIC_HIP(hipMemset(base, 0, sizeof(double) * (size_t)g.total));
    p = base + g.origin;
    MGIC_HIP(hipMalloc(&tab, sizeof(double *)));
    MGIC_HIP(hipMemcpy(tab, &p, sizeof(double *), hipMemcpyHostToDevice));
  }
  ~Stage() {
    (void)hipFree(base);
    (void)hipFree(tab);
  }
  BoxArgs args() const {
    BoxArgs a{};
    a.nx = g.nx;
    a.ny = g.ny;
    a.nz = g.nz;
    a.sy = g.sy;
    a.sz = g.sz;
    for (int d = 0; d < 3; ++d) a.glo[d] = g.valid.lo[d];
    return a;  // all faces kBcMemory: ghosts come from the caller's FAB
  }
};

// host fab component -> stage over box X (or stage -> host fab)
void transfer(Stage &s, const HostFab &f, int comp, Box X, bool to_device) {
  X = X.intersect(f.box);
  if (X.empty()) return;
  const long n = X.ncells();
  std::vector<double> buf((size_t)n);
  if (to_device) {
    long t = 0;
    for (int k = X.lo[2]; k <= X.hi[2]; ++k)
      for (int j = X.lo[1]; j <= X.hi[1]; ++j)
        for (int i = X.lo[0]; i <= X.hi[0]; ++i) buf[(size_t)t++] = f.p[f.idx(i, j, k, comp)];
  }
  double *dbuf = nullptr;
  CopyItem *ditem = nullptr;
  MGIC_HIP(hipMalloc(&dbuf, sizeof(double) * (size_t)n));
  MGIC_HIP(hipMalloc(&ditem, sizeof(CopyItem)));
  CopyItem it{};
  it.nx = X.size(0);
  it.ny = X.size(1);
  it.nz = X.size(2);
  const long off = s.g.offset(X.lo[0], X.lo[1], X.lo[2]);
  if (to_device) {
    it.src = -1;
    it.ssy = it.nx;
    it.ssz = (long)it.nx * it.ny;
    it.dst = 0;
    it.doff = off;
    it.dsy = s.g.sy;
    it.dsz = s.g.sz;
    MGIC_HIP(hipMemcpy(dbuf, buf.data(), sizeof(double) * (size_t)n, hipMemcpyHostToDevice));
    MGIC_HIP(hipMemcpy(ditem, &it, sizeof(it), hipMemcpyHostToDevice));
    kern::copy_items(ditem, 1, n, nullptr, dbuf, s.tab, nullptr, 0);
  } else {
    it.dst = -1;
    it.dsy = it.nx;
    it.dsz = (long)it.nx * it.ny;
    it.src = 0;
    it.soff = off;
    it.ssy = s.g.sy;
    it.ssz = s.g.sz;
    MGIC_HIP(hipMemcpy(ditem, &it, sizeof(it), hipMemcpyHostToDevice));
    kern::copy_items(ditem, 1, n, s.tab, nullptr, nullptr, dbuf, 0);
  }
  MGIC_HIP(hipDeviceSynchronize());
  if (!to_device) {
    MGIC_HIP(hipMemcpy(buf.data(), dbuf, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost));
    long t = 0;
    for (int k = X.lo[2]; k <= X.hi[2]; ++k)
      for (int j = X.lo[1]; j <= X.hi[1]; ++j)
        for (int i = X.lo[0]; i <= X.hi[0]; ++i) f.p[f.idx(i, j, k, comp)] = buf[(size_t)t++];
  }
  MGIC_HIP(hipFree(dbuf));
  MGIC_HIP(hipFree(ditem));
}

Box grow1(const Box &b) {
  Box g = b;
  for (int d = 0; d < 3; ++d) {
    g.lo[d] -= 1;
    g.hi[d] += 1;
  }
  return g;
}

StencilCoefs coefs(double dx, double alpha, double beta) {
  StencilCoefs s;
  s.alpha = alpha;
  s.beta = beta;
  s.dx = dx;
  s.dxinv = 1.0 / (dx * dx);
  s.lamshift = 2.0 * 3 * beta / (dx * dx);
  return s;
}

template <class F>
void run(const char *name, F &&f) {
  try {
    f();
  } catch (const std::exception &e) {
    std::fprintf(stderr, "%s: %s\n", name, e.what());
    std::abort();
  }
}

}  // namespace

#define UNPACK(x) x, x##lo0, x##lo1, x##lo2, x##hi0, x##hi1, x##hi2, x##nComp
#define REGION(b) \
  Box::make(std::vector<int>{*b##lo0, *b##lo1, *b##lo2, *b##hi0, *b##hi1, *b##hi2}.data())

extern "C" {

void gsrbhelmholtzvc3d_(MGIC_CHF_FRA(dpsi), MGIC_CHF_CONST_FRA(rhs), MGIC_CHF_BOX(region),
                        const double *dx, const double *alpha, MGIC_CHF_CONST_FRA(aCoef),
                        const double *beta, MGIC_CHF_CONST_FRA(bCoef),
                        MGIC_CHF_CONST_FRA(lambda), const int *redBlack) {
  run("gsrbhelmholtzvc3d_", [&] {
    HostFab u = fab(UNPACK(dpsi)), r = fab(UNPACK(rhs)), a = fab(UNPACK(aCoef)),
            b = fab(UNPACK(bCoef)), l = fab(UNPACK(lambda));
    const int ncomp = u.nc;  // .ChF:75-87
    if (ncomp != r.nc || ncomp != b.nc) mayday("GSRBHELMHOLTZVC3D: ncomp mismatch");
    const Box R = REGION(region);
    if (R.empty()) return;
    for (int n = 0; n < ncomp; ++n) {
      Stage su(R), sr(R), sa(R), sb(R), sl(R);
      transfer(su, u, n, grow1(R), true);
      transfer(sr, r, n, R, true);
      transfer(sa, a, n, R, true);
      transfer(sb, b, n, R, true);
      transfer(sl, l, n, R, true);
      kern::gsrb_pass(su.p, sr.p, sa.p, sb.p, sl.p, su.args(), coefs(*dx, *alpha, *beta), *redBlack, 0);
      MGIC_HIP(hipDeviceSynchronize());
      transfer(su, u, n, R, false);
    }
  });
}

void vccomputeop3d_(MGIC_CHF_FRA(lofdpsi), MGIC_CHF_CONST_FRA(dpsi), const double *alpha,
                    MGIC_CHF_CONST_FRA(aCoef), const double *beta, MGIC_CHF_CONST_FRA(bCoef),
                    MGIC_CHF_BOX(region), const double *dx) {
  run("vccomputeop3d_", [&] {
    HostFab lo = fab(UNPACK(lofdpsi)), u = fab(UNPACK(dpsi)), a = fab(UNPACK(aCoef)),
            b = fab(UNPACK(bCoef));
    const int ncomp = u.nc;  // .ChF:199-206
    if (ncomp != lo.nc || ncomp != b.nc) mayday("VCCOMPUTEOP3D: ncomp mismatch");
    const Box R = REGION(region);
    if (R.empty()) return;
    for (int n = 0; n < ncomp; ++n) {
      Stage so(R), su(R), sa(R), sb(R);
      transfer(su, u, n, grow1(R), true);
      transfer(sa, a, n, R, true);
      transfer(sb, b, n, R, true);
      kern::apply_op(so.p, su.p, sa.p, sb.p, su.args(), coefs(*dx, *alpha, *beta), 0);
      MGIC_HIP(hipDeviceSynchronize());
      transfer(so, lo, n, R, false);
    }
  });
}

void vccomputeres3d_(MGIC_CHF_FRA(res), MGIC_CHF_CONST_FRA(dpsi), MGIC_CHF_CONST_FRA(rhs),
                     const double *alpha, MGIC_CHF_CONST_FRA(aCoef), const double *beta,
                     MGIC_CHF_CONST_FRA(bCoef), MGIC_CHF_BOX(region), const double *dx) {
  run("vccomputeres3d_", [&] {
    HostFab rs = fab(UNPACK(res)), u = fab(UNPACK(dpsi)), r = fab(UNPACK(rhs)),
            a = fab(UNPACK(aCoef)), b = fab(UNPACK(bCoef));
    const int ncomp = u.nc;  // .ChF:302-309
    if (ncomp != rs.nc || ncomp != b.nc) mayday("VCCOMPUTERES3D: ncomp mismatch");
    const Box R = REGION(region);
    if (R.empty()) return;
    for (int n = 0; n < ncomp; ++n) {
      Stage so(R), su(R), sr(R), sa(R), sb(R);
      transfer(su, u, n, grow1(R), true);
      transfer(sr, r, n, R, true);
      transfer(sa, a, n, R, true);
      transfer(sb, b, n, R, true);
      kern::residual(so.p, su.p, sr.p, sa.p, sb.p, su.args(), coefs(*dx, *alpha, *beta), 0);
      MGIC_HIP(hipDeviceSynchronize());
      transfer(so, rs, n, R, false);
    }
  });
}

void restrictresvc3d_(MGIC_CHF_FRA(res), MGIC_CHF_CONST_FRA(dpsi), MGIC_CHF_CONST_FRA(rhs),
                      const double *alpha, MGIC_CHF_CONST_FRA(aCoef), const double *beta,
                      MGIC_CHF_CONST_FRA(bCoef), MGIC_CHF_BOX(region), const double *dx) {
  run("restrictresvc3d_", [&] {
    HostFab rc = fab(UNPACK(res)), u = fab(UNPACK(dpsi)), r = fab(UNPACK(rhs)),
            a = fab(UNPACK(aCoef)), b = fab(UNPACK(bCoef));
    const Box R = REGION(region);
    if (R.empty()) return;
    for (int d = 0; d < 3; ++d)
      if (R.lo[d] < 0 || (R.lo[d] & 1) || (R.size(d) & 1))
        mayday("RESTRICTRESVC3D: region must be a shifted box (lo >= 0, even lo and extent)");
    Box C;  // ii = i/2 (.ChF:407-409)
    for (int d = 0; d < 3; ++d) {
      C.lo[d] = R.lo[d] / 2;
      C.hi[d] = R.hi[d] / 2;
    }
    const int ncomp = u.nc;
    for (int n = 0; n < ncomp; ++n) {
      Stage sc(C), su(R), sr(R), sa(R), sb(R);
      transfer(sc, rc, n, C, true);
      transfer(su, u, n, grow1(R), true);
      transfer(sr, r, n, R, true);
      transfer(sa, a, n, R, true);
      transfer(sb, b, n, R, true);
      kern::restrict_residual(sc.p, sc.args(), su.p, sr.p, sa.p, sb.p, su.args(),
                              coefs(*dx, *alpha, *beta), 0, /*accumulate=*/true);
      MGIC_HIP(hipDeviceSynchronize());
      transfer(sc, rc, n, C, false);
    }
  });
}

static void fra1_unary(const char *name, double *out, const int *ol0, const int *ol1,
                       const int *ol2, const int *oh0, const int *oh1, const int *oh2,
                       const double *in, const int *il0, const int *il1, const int *il2,
                       const int *ih0, const int *ih1, const int *ih2, const double *dx,
                       const int *b0, const int *b1, const int *b2, const int *e0, const int *e1,
                       const int *e2, bool laplacian) {
  run(name, [&] {
    const int one = 1;
    HostFab fo = fab(out, ol0, ol1, ol2, oh0, oh1, oh2, &one);
    HostFab fi = fab(in, il0, il1, il2, ih0, ih1, ih2, &one);
    const int lohi[6] = {*b0, *b1, *b2, *e0, *e1, *e2};
    const Box R = Box::make(lohi);
    if (R.empty()) return;
    if (!fi.box.contains(grow1(R))) mayday("operand must cover the box grown by one");
    Stage so(R), si(R);
    transfer(si, fi, 0, grow1(R), true);
    if (laplacian) kern::lap_psi(so.p, si.p, si.args(), *dx, 0);
    else kern::rho_grad_phi(so.p, si.p, si.args(), *dx, 0);
    MGIC_HIP(hipDeviceSynchronize());
    transfer(so, fo, 0, R, false);
  });
}

void getlaplacianpsif_(MGIC_CHF_FRA1(l_of_psi), MGIC_CHF_CONST_FRA1(psi), const double *dx,
                       MGIC_CHF_BOX(box)) {
  fra1_unary("getlaplacianpsif_", l_of_psi, l_of_psilo0, l_of_psilo1, l_of_psilo2, l_of_psihi0,
             l_of_psihi1, l_of_psihi2, psi, psilo0, psilo1, psilo2, psihi0, psihi1, psihi2, dx,
             boxlo0, boxlo1, boxlo2, boxhi0, boxhi1, boxhi2, true);
}

void getrhogradphif_(MGIC_CHF_FRA1(rho_grad_phi), MGIC_CHF_CONST_FRA1(phi), const double *dx,
                     MGIC_CHF_BOX(box)) {
  fra1_unary("getrhogradphif_", rho_grad_phi, rho_grad_philo0, rho_grad_philo1, rho_grad_philo2,
             rho_grad_phihi0, rho_grad_phihi1, rho_grad_phihi2, phi, philo0, philo1, philo2,
             phihi0, phihi1, phihi2, dx, boxlo0, boxlo1, boxlo2, boxhi0, boxhi1, boxhi2, false);
}

}  // extern "C"
