// kernels.hpp -- host-side launchers for the gfx950 kernels in kernels.hip.
//
// Every stencil launcher works on ONE box: all arrays share the box's
// FabGeom (strides sy, sz; pointers point at the valid-lo cell) and the
// domain boundary is folded in through BoxArgs::bcm/bcc (see mgic_core.hpp).
#pragma once

#include "mgic_core.hpp"

namespace mgic {
namespace kern {

// GSRBHELMHOLTZVC3D (.ChF:56-139): one colour pass over the valid region.
// lam == nullptr: lambda = 1/(alpha*a + 2*3*beta/dx^2) is recomputed in
// registers (bit-identical to resetLambda, .cpp:234-243) instead of read.
void gsrb_pass(double *u, const double *rhs, const double *a, const double *b,
               const double *lam, const BoxArgs &g, const StencilCoefs &s, int colour,
               hipStream_t st);
// Fused red+black sweep (both passes of one levelGSRB, .cpp:290-331) in one
// launch, staged through LDS, OUT OF PLACE: u_out = sweep(u_in); bit-
// identical to two in-place gsrb_pass calls with an exchange before each.
// Domain faces (bcm != 0): the BC images are applied to the kernel's LDS
// copy of u_in (u_in itself is never written).  Exchanged faces (bcm == 0): u_in must hold the 2-deep ghost
// shell and rhs/a/b ghost layer 1.  zero_in: u_in is identically +0 and is
// not read (first sweep on a freshly zeroed correction).  acc != nullptr:
// acc += sweep(u_in) instead of writing u_out (phi += e of the last sweep).
// kind: 1 = by size (one-shot 3D blocks for boxes <= 128^3, z-streaming
// above), 2 = always z-streaming, 3 = always 3D blocks.
void gsrb_sweep_fused(double *u_out, double *u_in, const double *rhs, const double *a,
                      const double *b, const BoxArgs &g, const StencilCoefs &s, bool zero_in,
                      double *acc, int kind, hipStream_t st);
// The same sweep on fp32 fields (the mixed-precision V-cycle); the stencil
// constants are rounded to fp32 once; acc (phi += e) stays fp64.
void gsrb_sweep_fused_f(float *u_out, float *u_in, const float *rhs, const float *a,
                        const float *b, const BoxArgs &g, const StencilCoefs &s, bool zero_in,
                        double *acc, int kind, hipStream_t st);
// The last pre-smoothing sweep fused with restrictResidual: u_out = sweep(
// u_in) as gsrb_sweep_fused, and rc (the coarse box, coarsen(box, 2)) = the
// restricted residual rhs - L(u_out) with the homogeneous BC of g (exactly
// restrict_residual(rc, cg, u_out, rhs, a, b, g, s) with rc zeroed first).
// Applies to boxes whose six faces are domain faces, even extents, taking
// the z-streaming kernel (see _applies); the caller falls back otherwise.
bool gsrb_sweep_fused_restrict_applies(const BoxArgs &g, const BoxArgs &cg, int kind);
void gsrb_sweep_fused_restrict(double *u_out, double *u_in, const double *rhs, const double *a,
                               const double *b, const BoxArgs &g, const StencilCoefs &s,
                               double *rc, const BoxArgs &cg, hipStream_t st);
// Two consecutive red+black sweeps u_in -> u_out in one z-streaming launch
// (temporal blocking, smoother_tb.hip): bit-identical to two
// gsrb_sweep_fused calls; zero_in / acc as there.  Constant bCoef; domain
// faces, or exchanged faces whose 4-deep ghost shell of u and rhs / aCoef is
// filled.  _applies also keeps boxes the 3D-block kernel takes (kind 3, or
// kind 1 at most gsrb_block_max_cells() cells) on that kernel.
bool gsrb_sweep_tb2_applies(const BoxArgs &g, const StencilCoefs &s, int kind);
// skip (device, or null): the launch returns at once when *skip != 0 (a
// device-side solve that has stopped, BicgState::done)
void gsrb_sweep_tb2(double *u_out, const double *u_in, const double *rhs, const double *a,
                    const BoxArgs &g, const StencilCoefs &s, bool zero_in, double *acc,
                    hipStream_t st, const int *skip = nullptr);
// the same two-sweep launch on fp32 fields; acc (the fp64 phi, or null):
// the second sweep's values are added to it as (double)e instead of stored
void gsrb_sweep_tb2_f(float *u_out, const float *u_in, const float *rhs, const float *a,
                      const BoxArgs &g, const StencilCoefs &s, bool zero_in, double *acc,
                      hipStream_t st);
long gsrb_block_max_cells();
// VCCOMPUTEOP3D (.ChF:181-237)
void apply_op(double *lu, const double *u, const double *a, const double *b,
              const BoxArgs &g, const StencilCoefs &s, hipStream_t st);
// VCCOMPUTERES3D (.ChF:283-339)
void residual(double *r, const double *u, const double *rhs, const double *a,
              const double *b, const BoxArgs &g, const StencilCoefs &s, hipStream_t st);
// the same residual plus one max |r| partial per block into partials[0, n)
// (n = residual_norm_blocks(g); 0 when the streaming residual does not apply:
// then call residual + reduce_partial instead)
long residual_norm_blocks(const BoxArgs &g);
void residual_norm(double *r, const double *u, const double *rhs, const double *a, const double *b,
                   const BoxArgs &g, const StencilCoefs &s, double *partials, hipStream_t st);
// RESTRICTRESVC3D (.ChF:379-437) incl. setVal(0) on the coarse valid box
// accumulate=true adds into rc like the bare Fortran kernel (whose caller
// zeroes rc first); false writes 0 + sum, i.e. setVal(0) + kernel.
void restrict_residual(double *rc, const BoxArgs &cg, const double *u, const double *rhs,
                       const double *a, const double *b, const BoxArgs &fg,
                       const StencilCoefs &s, hipStream_t st, bool accumulate = false);
// prolongIncrement: uf += P(ec); type 0 constant, 1 linear
void prolong(double *uf, const BoxArgs &fg, const double *ec, const BoxArgs &cg,
             const int avail_lo[3], const int avail_hi[3], int type, hipStream_t st);
// resetLambda (.cpp:220-249)
void lambda(double *lam, const double *a, const BoxArgs &g, const StencilCoefs &s,
            hipStream_t st);
// CoarseAverage arithmetic / harmonic with refinement ratio `ratio`
void average(double *c, const BoxArgs &cg, const double *f, const BoxArgs &fg, int ratio,
             int harmonic, hipStream_t st);
// ParseBC: write the domain-face ghost layers (modes from g.bcm)
void fill_bc(double *u, const BoxArgs &g, hipStream_t st);

// BLAS-1 over the valid region: kind 0 x=y, 1 x=x+s*y, 2 x=x*s, 3 x=x*y,
// 4 x = s*y + t*z, 5 x = s (setVal), 6 x = y*z (copy, then mult)
void blas(int kind, double *x, const double *y, const double *z, double s, double t,
          const BoxArgs &g, hipStream_t st);
// Deterministic reductions: kind 0 dot(x,y), 1 sum|x|, 2 sum x^2, 3 max|x|,
// 4 max x, 5 max(-x).
// Writes nparts partials at partials[0..nparts); returns nparts.
int reduce_partial(int kind, const double *x, const double *y, const BoxArgs &g,
                   double *partials, hipStream_t st);
constexpr int kMaxPartsPerBox = 2048;
// A reduction's result published by its last kernel straight into pinned,
// host-coherent memory (Comm::host_pub): the value and, for the last result
// of a readback, the peer-mapped transport's error word and then the sequence
// number the host spins on (Comm::wait_results) -- no copy operation and no
// stream synchronisation per readback.  val == nullptr: nothing is published.
struct HostPub {
  double *val = nullptr;
  unsigned long long *seq = nullptr;
  unsigned long long seqv = 0;
  const unsigned long long *err_src = nullptr;  // device error word
  unsigned long long *err_dst = nullptr;
};
__device__ __forceinline__ void publish(const HostPub &p, double v) {
  if (!p.val) return;
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p.val),
                     (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
  if (!p.seq) return;
  if (p.err_dst)
    __hip_atomic_store(p.err_dst,
                       __hip_atomic_load(p.err_src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __hip_atomic_store(p.seq, p.seqv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
void reduce_final(int kind, const double *partials, int n, double *out, hipStream_t st,
                  const HostPub &pub = HostPub());
// publish *d_val (after a collective on it)
void publish_result(const double *d_val, const HostPub &pub, hipStream_t st);

// BiCGStab's fused vector updates (bit-identical to the separate passes):
// s = r + ca*v, e = e + cb*pt and the partials of reduction `kind` (1 sum|s|,
// 2 sum s^2, 3 max|s|) of s; the partials of dot(t,s) and dot(t,t); and
// p = ((p*beta) + c*v) + r.  Return the number of partials written.
int axpy2_reduce(int kind, double *s, const double *r, const double *v, double ca, double *e,
                 const double *pt, double cb, const BoxArgs &g, double *partials, hipStream_t st);
int dot2_partial(const double *t, const double *s, const BoxArgs &g, double *pts, double *ptt,
                 hipStream_t st);
void bicg_p(double *p, const double *v, const double *r, double beta, double c, const BoxArgs &g,
            hipStream_t st);

// ---- BiCGStab on the device (op.cpp BiCGStabSolver::solve_device): the
// host loop's scalars, its stop tests and their outcome, in device memory.
// Each launch below returns at once when done != 0; the last block of each
// reduction writes the next scalars (or stops the solve).
enum BicgReason {
  kBicgRun = 0,
  kBicgStop = 1,          // the loop's test (iterations, eps, reps)
  kBicgRho0 = 2,          // rho1 == 0
  kBicgHalf = 3,          // |S| met the tolerance (E += alpha PT pending)
  kBicgTt0 = 4,           // <T, T> == 0 (E += alpha PT pending)
  kBicgOmega0 = 5,        // omega == 0
  kBicgRestart = 6,       // |m| <= small |rho1|: the host restarts the solve
  kBicgRestartLimit = 7,  // the same with no restarts left
};
struct BicgState {
  double rho1, rho2, alpha, beta, omega, nrm, init_norm, rho_next, m, ts, tt;
  double eps, reps, small;
  int it, imax, done, reason, epend, init, restarts, num_restarts, nt;
  int xr;  // bicg_lblock: the XCD-contiguous row deal (host-set)
};
// the reductions' last-block counters (device, zeroed once; each launch
// leaves its own at zero): this many words
constexpr int kBicgCounterWords = 4 * 9 * 32;
// P = R (init) or ((P*beta) + ((-beta)*omega)*V) + 1.0*R; W = P * lambda
void bicg_dev_p(BicgState *st, double *p, double *w, const double *v, const double *r,
                const double *lam, const BoxArgs &g, hipStream_t st_);
// V = L(PT) (homogeneous BC of g); alpha = rho1 / <RT, V>
void bicg_dev_apply_dot(BicgState *st, double *v, const double *pt, const double *rt,
                        const double *a, const double *b, const BoxArgs &g, const StencilCoefs &s,
                        double *parts, unsigned int *cnt, hipStream_t st_);
// S = R + (-alpha)V; W = S * lambda; nrm = |S|
void bicg_dev_s(BicgState *st, double *s, double *w, const double *r, const double *v,
                const double *lam, const BoxArgs &g, int norm_kind, double *parts,
                unsigned int *cnt, hipStream_t st_);
// omega = <T, S> / <T, T>, T = L(ST) (not stored)
void bicg_dev_apply_dot2(BicgState *st, const double *stv, const double *s, const double *a,
                         const double *b, const BoxArgs &g, const StencilCoefs &sc,
                         double *parts_ts, double *parts_tt, unsigned int *cnt, hipStream_t st_);
// R = S + (-omega)L(ST); E = (E + alpha PT) + omega ST; nrm = |R|; the loop head
void bicg_dev_r(BicgState *st, double *r, double *e, const double *s, const double *a,
                const double *b, const StencilCoefs &sc, const double *pt, const double *stv,
                const double *rt, const BoxArgs &g, int norm_kind, double *parts_n,
                double *parts_d, unsigned int *cnt, hipStream_t st_);
// copy *st into pinned host memory, then store seqv into *seq (host-coherent)
void bicg_dev_publish(const BicgState *st, BicgState *host, unsigned long long *seq,
                      unsigned long long seqv, hipStream_t st_);
// partials written by the reductions above for box g
int bicg_dev_parts(const BoxArgs &g);

// batched rectangular copies (exchange / copyTo / pack / unpack)
void copy_items(const CopyItem *d_items, int nitems, long max_cells, double *const *src_tab,
                const double *src_buf, double *const *dst_tab, double *dst_buf,
                hipStream_t st);

// SetLevelData.cpp set_a_coef/set_rhs at psi = 1 (input generator)
struct BhParams {
  double domlen[3];
  double G_Newton, phi_amplitude, phi_wavelength;
  double m1, m2, spin1, spin2, off1, off2, mom1, mom2, constant_K;
};
// psi: nullptr = psi 1 everywhere, else read with its ghost layer
void binary_bh_coefs(double *acoef, double *rhs, const double *psi, const BoxArgs &g, double dx,
                     const BhParams &p, hipStream_t st);
// set_constant_K_integrand (SetLevelData.cpp:131-180) at psi (nullptr: 1)
void constant_k_integrand(double *out, const double *psi, const BoxArgs &g, double dx,
                          const BhParams &p, hipStream_t st);
// GETLAPLACIANPSIF / GETRHOGRADPHIF (SetLevelDataF.ChF), operand ghosts as is
void lap_psi(double *l, const double *psi, const BoxArgs &g, double dx, hipStream_t st);
void rho_grad_phi(double *r, const double *phi, const BoxArgs &g, double dx, hipStream_t st);
// WriteOutput.H's components for planes [k0, k0+nk) of a valid box,
// component-major, i fastest.  kind 0: the 31 GRChombo variables of
// set_output_data (psi); kind 1: output_solver_data's dpsi, rhs, psi, A_ij_0,
// phi_0
constexpr int kNumGRChomboVars = 31, kNumSolverVars = 10;
void output_vars(int kind, double *out, const double *psi, const double *dpsi, const double *rhs,
                 const BoxArgs &g, int k0, int nk, double dx, const BhParams &p, hipStream_t st);
// x += y over the valid box grown by `grow` (<= kGhost) cells
void incr_grown(double *x, const double *y, const BoxArgs &g, int grow, hipStream_t st);


// ---- fp32 variants for the mixed-precision V-cycle (fp32 smoother / fp64
// residual): the same expressions evaluated in float, constants rounded once
void residual_to_f(float *r, const double *u, const double *rhs, const double *a, const double *b,
                   const BoxArgs &g, const StencilCoefs &s, hipStream_t st);
void restrict_residual_f(float *rc, const BoxArgs &cg, const float *u, const float *rhs,
                         const float *a, const float *b, const BoxArgs &fg, const StencilCoefs &s,
                         hipStream_t st);
void prolong_f(float *uf, const BoxArgs &fg, const float *ec, const BoxArgs &cg,
               const int avail_lo[3], const int avail_hi[3], int type, hipStream_t st);
void copy_items_f(const CopyItem *d_items, int nitems, long max_cells, float *const *src_tab,
                  const float *src_buf, float *const *dst_tab, float *dst_buf, hipStream_t st);
void to_float(float *d, const double *s, const BoxArgs &g, int grow, hipStream_t st);
void copy_f(float *d, const float *s, const BoxArgs &g, hipStream_t st);
void incr_f(double *x, const float *y, const BoxArgs &g, hipStream_t st);  // x += (double)y

// ---- coarse-fine interpolation on one face of one fine box (AMR levels)
struct CFArgs {
  int face;                      // 0..5 (dir * 2 + side)
  int flo[3];                    // fine box valid lo (global fine index)
  int clo[3];                    // staged coarse box valid lo (global coarse index)
  long csy, csz;                 // its strides (valid-lo based pointer)
  int cdom_lo[3], cdom_hi[3];    // coarse problem domain
  int periodic[3];
  int ncov;                      // coarsened fine boxes of the level (covered test)
  const int *cov;                // device, 6 ints each (global coarse index)
};
void cf_interp(double *u, const double *coarse_stage, const BoxArgs &g, const CFArgs &c,
               bool homogeneous, hipStream_t st);

}  // namespace kern
}  // namespace mgic
