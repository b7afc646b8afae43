/*
 * mgic.h -- C ABI of the MI355X-native multigrid library (libmgic.so).
 *
 * The drop-in boundary for the reference's hot path: eugenealim/MG_IC_code
 * hands its V-cycle to Chombo through the operator-plugin API
 *   defineOperatorFactory / VariableCoeffPoissonOperatorFactory
 *     (Source/VariableCoeffPoissonOperatorFactory.H:22-117)
 *   VariableCoeffPoissonOperator  (Source/VariableCoeffPoissonOperator.H:25-170)
 * and the operator reaches its arithmetic through the ChomboFortran C ABI
 * (Source/VariableCoeffPoissonOperatorF_F.H; those host drop-ins are declared
 * in mgic_chf.h).  This header exposes the same surface with plain pointers
 * and integers: every handle-level entry point below names the reference
 * method it replaces.
 *
 * Conventions
 *   - Boxes are 6 ints {lo0, lo1, lo2, hi0, hi1, hi2}, inclusive cell
 *     indices in the level's global index space (Chombo Box).
 *   - Every function returns 0 on success and a negative MGIC_E* code on
 *     failure (the reference aborts through MayDay; this library never
 *     aborts); mgic_last_error() describes the last failure of the thread.
 *   - All device work is enqueued on the communicator's HIP stream; the
 *     functions that return host scalars (dot, norm, iteration norms,
 *     BiCGStab) synchronise that stream.
 *   - Fields are fp64, one component, one ghost layer, device resident.
 */
#ifndef MGIC_H
#define MGIC_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGIC_API __attribute__((visibility("default")))

#define MGIC_OK 0
#define MGIC_EBADARG (-1)
#define MGIC_EHIP (-2)
#define MGIC_ERCCL (-3)
#define MGIC_ESTATE (-4)
#define MGIC_EUNKNOWN (-5)
#define MGIC_UNIQUE_ID_BYTES 128

typedef struct mgic_comm_s *mgic_comm;       /* one rank: RCCL comm + HIP stream */
typedef struct mgic_grid_s *mgic_grid;       /* DisjointBoxLayout + ProblemDomain + dx */
typedef struct mgic_field_s *mgic_field;     /* LevelData<FArrayBox> (1 comp, 1 ghost) */
typedef struct mgic_factory_s *mgic_factory; /* VariableCoeffPoissonOperatorFactory */
typedef struct mgic_op_s *mgic_op;           /* VariableCoeffPoissonOperator */
typedef struct mgic_mg_s *mgic_mg;           /* AMRMultiGrid on one AMR level */
typedef struct mgic_plan_s *mgic_plan;       /* host-side view of a Copier plan */
typedef struct mgic_mixed_s *mgic_mixed;     /* fp32-smoother / fp64-residual V-cycle */
typedef struct mgic_amr_s *mgic_amr;         /* AMR hierarchy (levels > 0, ratio 2) */

/* Operator constants and ParseBC state (params.txt keys alpha, beta, bc_lo,
 * bc_hi, bc_value, coefficient_average_type; [Chombo] statics). */
typedef struct {
  double alpha, beta;          /* default 0, -1 (Factory.cpp:317-322) */
  int bc_lo[3], bc_hi[3];      /* 0 Dirichlet, 1 Neumann, 2 periodic flag */
  double bc_value;
  int coefficient_average_type; /* 0 arithmetic (default), 1 harmonic */
  int prolong_type;             /* 0 piecewise constant, 1 linear (default) */
  int relax_mode;               /* 1 GSRB (default), 4 Jacobi */
  int fused_smoother;           /* fused red+black sweep: 0 off (one launch per colour
                                   pass), 1 kernel by box size, 2 z-streaming, 3 3D blocks */
  int deep_halo;                /* fused sweeps on exchanged layouts: 4-deep ghost shells,
                                   two sweeps per exchange (the first on the box grown by
                                   2 across exchanged faces).  0 off (default), 1 every
                                   level, 2 levels of boxes <= 128^3 cells */
} mgic_op_params;

/* MultiGrid / bottom-solver configuration (MultilevelLinearOp knobs:
 * numMGsmooth, numMGIterations, preCondSolverDepth; BiCGStab defaults). */
typedef struct {
  int max_depth;         /* deepest MG depth, -1: as deep as coarsenable */
  int n_pre, n_post, n_bottom;
  int bottom_solver;     /* 0: relax(n_bottom), 1: BiCGStab */
  int cycles;            /* 1 = V-cycle */
  int agglomerate_below; /* gather to rank 0 once a box side < this; 0 off.  A
                            gathered depth (and every depth below it) runs on
                            rank 0 alone, its BiCGStab reductions included; the
                            other ranks go from the gather to the scatter */
  int bicg_imax;
  double bicg_eps, bicg_reps, bicg_small;
  int bicg_restarts, bicg_norm_type;
} mgic_mg_params;

/* The layout of the parameter structs above and the entry points' argument
 * lists: bumped whenever either changes (round 4 removed fields from the
 * middle of mgic_op_params / mgic_mg_params).  An integrator compiled against
 * this header checks mgic_abi_version() == MGIC_ABI_VERSION once at start-up. */
#define MGIC_ABI_VERSION 2
MGIC_API int mgic_abi_version(void);
MGIC_API const char *mgic_version(void);
MGIC_API const char *mgic_last_error(void);
MGIC_API int mgic_set_device(int device);
MGIC_API int mgic_get_device_count(int *count);
MGIC_API int mgic_device_synchronize(void);
MGIC_API void mgic_op_params_default(mgic_op_params *p);
MGIC_API void mgic_mg_params_default(mgic_mg_params *p);

/* ---- communicator (MPI_Init / process group, Main_PoissonSolver.cpp:261) */
MGIC_API int mgic_comm_unique_id(unsigned char id[MGIC_UNIQUE_ID_BYTES]);
MGIC_API int mgic_comm_create(int rank, int size, const unsigned char *id, int force_rccl,
                              mgic_comm *out);
/* The peer-mapped transport instead of RCCL (no RCCL communicator): every
 * rank maps every other rank's signal page and receive arena through
 * hipIpcOpenMemHandle, and an exchange is two kernels with device-side flags
 * (ranks may share one device).  `allgather` is the host's own collective
 * (MPI_Allgather in a Chombo build), called once inside this function:
 * gather `nbytes` from every rank into out[size * nbytes], rank order, 0 on
 * success; it may be NULL when size == 1.  arena_bytes: one message buffer
 * (0: MGIC_IPC_ARENA_MB, default 64 MB); every rank passes the same value.
 * Replaces the MPI transport of Chombo's Copier (exchange(),
 * VariableCoeffPoissonOperator.cpp:48,131,301) and of its norms. */
typedef int (*mgic_allgather_fn)(const void *in, size_t nbytes, void *out, void *user);
MGIC_API int mgic_comm_create_ipc(int rank, int size, mgic_allgather_fn allgather, void *user,
                                  size_t arena_bytes, mgic_comm *out);
/* transport of a communicator: 0 none (one rank), 1 RCCL, 2 peer-mapped */
MGIC_API int mgic_comm_transport(mgic_comm c, int *transport);
MGIC_API int mgic_comm_destroy(mgic_comm c);
MGIC_API int mgic_comm_set_stream(mgic_comm c, void *hip_stream); /* NULL: own stream */
MGIC_API int mgic_comm_get_stream(mgic_comm c, void **hip_stream);
MGIC_API int mgic_comm_set_self_messages(mgic_comm c, int on);
/* exchanges with messages (peer-mapped or RCCL) issued on this communicator so far:
   a measurement counter (tools/rank_proxy.py charges per-exchange latency with it) */
MGIC_API int mgic_comm_exchanges(mgic_comm c, unsigned long long *count);
MGIC_API int mgic_comm_synchronize(mgic_comm c); /* + raises a transport timeout */
MGIC_API int mgic_comm_rank(mgic_comm c, int *rank, int *size, int *uses_rccl);

/* ---- grids (DisjointBoxLayout(boxes, procs, domain); set_grids,
 *      Source/SetGrids.cpp:54-58) */
MGIC_API int mgic_grid_create(mgic_comm c, const int domain[6], const int periodic[3], double dx,
                              int nbox, const int *boxes, const int *owners, mgic_grid *out);
MGIC_API int mgic_grid_destroy(mgic_grid g);
MGIC_API int mgic_grid_num_local(mgic_grid g, int *n);
MGIC_API int mgic_grid_local_box(mgic_grid g, int n, int lohi[6], int *global_index);
MGIC_API int mgic_grid_coarsen(mgic_grid g, int ratio, mgic_grid *out);

/* ---- copy plans, host side (Copier / exchangeDefine + trimEdges,
 *      Source/VariableCoeffPoissonOperatorFactory.cpp:82-99,179-185).
 *      The exact plan rank `rank` of `size` executes for a layout pair
 *      (exchange: src = dst layout, with_faces = 1; gather/scatter for the
 *      coarse levels: with_valid = 1), computed WITHOUT a GPU so the
 *      multi-rank path can be checked on CPU.  Items are 12 int64 each:
 *      {src, dst, soff, doff, ssy, ssz, dsy, dsz, nx, ny, nz, peer}; src/dst
 *      are local box indices or -1 for the per-peer message buffer, offsets
 *      are in doubles from the box's valid-lo cell (or from the buffer
 *      start), strides in doubles.  which: 0 local copies, 1 pack (send),
 *      2 unpack (receive). */
MGIC_API int mgic_plan_create(int rank, int size, const int domain[6], const int periodic[3],
                              int nsrc, const int *src_boxes, const int *src_owners, int ndst,
                              const int *dst_boxes, const int *dst_owners, int with_valid,
                              int with_faces, mgic_plan *out);
/* the ghost-shell exchange (faces, edges and corners, `depth` deep) of one
 * layout: what the fused sweeps exchange (depth 2; 4 in deep-halo mode) */
MGIC_API int mgic_plan_create_shell(int rank, int size, const int domain[6],
                                    const int periodic[3], int nboxes, const int *boxes,
                                    const int *owners, int depth, mgic_plan *out);
/* the host-side tables transport `transport` (1 RCCL, 2 peer-mapped; the
 * numbering of mgic_comm_transport) builds for this plan before executing
 * it: 0, or an error when that transport cannot execute it (the peer-mapped
 * transport takes at most 32 peers per plan; RCCL has no such limit) */
MGIC_API int mgic_plan_check_transport(mgic_plan p, int transport);
/* the peer-mapped transport's block table of this plan (built as by
 * mgic_plan_check_transport(p, 2)): *n put and get blocks; with rows != NULL,
 * five values per block: side (0 put, 1 get), peer rank, flag, first element
 * in the message, element count.  Both sides of a message must list the same
 * (flag, first, count) rows: a get block waits for the put block of its flag */
MGIC_API int mgic_plan_ipc_blocks(mgic_plan p, int *n, long long *rows);
/* the same table for a block size other than the default: block_elems as
 * MGIC_IPC_BLOCK_ELEMS sets it (a multiple of 512 in [512, 2^20]); a plan's
 * table is built once, so one block size per plan handle */
MGIC_API int mgic_plan_ipc_blocks_per(mgic_plan p, long long block_elems, int *n,
                                      long long *rows);
MGIC_API int mgic_plan_destroy(mgic_plan p);
MGIC_API int mgic_plan_sizes(mgic_plan p, int *n_local, int *n_pack, int *n_unpack, int *n_peers);
MGIC_API int mgic_plan_items(mgic_plan p, int which, long long *items);
/* per peer (ascending rank): send/recv counts and buffer offsets, doubles */
MGIC_API int mgic_plan_peers(mgic_plan p, int *peers, long long *send_cnt, long long *send_off,
                             long long *recv_cnt, long long *recv_off);
/* FabGeom of local box n of the src (layout = 0) or dst (layout = 1)
 * layout: {sy, sz, origin, total} in doubles */
MGIC_API int mgic_plan_geom(mgic_plan p, int layout, int n, long long geom[4]);

/* ---- fields (LevelData<FArrayBox>) */
MGIC_API int mgic_field_create(mgic_grid g, mgic_field *out);
MGIC_API int mgic_field_destroy(mgic_field f);
/* device pointer of the valid-lo cell of local box n and its strides
 * {1, sy, sz} in doubles */
MGIC_API int mgic_field_device_ptr(mgic_field f, int n, double **valid_lo, long strides[3]);
/* host <-> device, contiguous i-fastest over the valid box (with_ghosts=0)
 * or over the valid box grown by one (with_ghosts=1); synchronous */
MGIC_API int mgic_field_upload(mgic_field f, int n, const double *host, int with_ghosts);
MGIC_API int mgic_field_download(mgic_field f, int n, double *host, int with_ghosts);
MGIC_API int mgic_field_set_val(mgic_field f, double v);  /* valid cells */
MGIC_API int mgic_field_set_zero(mgic_field f);           /* valid + ghosts */
MGIC_API int mgic_field_exchange(mgic_field f);           /* LevelData::exchange */
/* LevelData::copyTo: valid -> valid (+ dst face ghosts if with_faces) */
MGIC_API int mgic_field_copy_to(mgic_field src, mgic_field dst, int with_faces);
/* set_a_coef / set_rhs at psi = 1 (SetLevelData.cpp:73-127, :281-325);
 * bh[13] = {domain_length, G_Newton, phi_amplitude, phi_wavelength,
 *           bh1_bare_mass, bh2_bare_mass, bh1_spin, bh2_spin, bh1_offset,
 *           bh2_offset, bh1_momentum, bh2_momentum, constant_K} */
MGIC_API int mgic_field_binary_bh(mgic_field acoef, mgic_field rhs, const double bh[13]);
/* the same at a general conformal factor psi (read with its ghost layer);
 * psi = NULL is psi = 1 (NL iteration 0) */
MGIC_API int mgic_field_nl_coefs(mgic_field psi, mgic_field acoef, mgic_field rhs,
                                 const double bh[13]);
/* set_constant_K_integrand (SetLevelData.cpp:131-180) at psi (NULL: 1):
 * the integrand of the periodic integrability condition for K */
MGIC_API int mgic_field_nl_integrand(mgic_field psi, mgic_field out, const double bh[13]);
/* every cell of the allocation, ghosts included (set_initial_conditions
 * sets psi over the whole FAB, SetLevelData.cpp:31-72) */
MGIC_API int mgic_field_set_val_all(mgic_field f, double v);

/* ---- operator factory (defineOperatorFactory, Factory.cpp:29-49) */
MGIC_API int mgic_factory_define(mgic_grid g, const mgic_op_params *p, mgic_field aCoef,
                                 mgic_field bCoef, mgic_factory *out);
MGIC_API int mgic_factory_destroy(mgic_factory f);
/* MGnewOp (Factory.cpp:139-234): returns 1 with *out = NULL when the layout
 * is not coarsenable(2^depth * s_maxCoarse) */
MGIC_API int mgic_factory_mg_new_op(mgic_factory f, int depth, mgic_op *out);
MGIC_API int mgic_factory_amr_new_op(mgic_factory f, mgic_op *out); /* :236-295 */
MGIC_API int mgic_factory_ref_to_finer(mgic_factory f, int *ratio); /* :297-314 */

/* ---- operator (VariableCoeffPoissonOperator) */
MGIC_API int mgic_op_destroy(mgic_op op);
MGIC_API int mgic_op_grid(mgic_op op, mgic_grid *out);
MGIC_API int mgic_op_coef(mgic_op op, int which /* 0 aCoef, 1 bCoef, 2 lambda */,
                          mgic_field *out);
MGIC_API int mgic_op_residual(mgic_op op, mgic_field lhs, mgic_field dpsi, mgic_field rhs,
                              int homogeneous);                                  /* residualI */
MGIC_API int mgic_op_apply_op(mgic_op op, mgic_field lhs, mgic_field dpsi, int homogeneous);
MGIC_API int mgic_op_apply_op_no_boundary(mgic_op op, mgic_field lhs, mgic_field dpsi);
MGIC_API int mgic_op_precond(mgic_op op, mgic_field cor, mgic_field res);        /* preCond */
MGIC_API int mgic_op_relax(mgic_op op, mgic_field e, mgic_field r, int iterations);
MGIC_API int mgic_op_level_gsrb(mgic_op op, mgic_field dpsi, mgic_field rhs);
MGIC_API int mgic_op_level_jacobi(mgic_op op, mgic_field dpsi, mgic_field rhs);
MGIC_API int mgic_op_restrict_residual(mgic_op fine, mgic_field resCoarse, mgic_field dpsiFine,
                                       mgic_field rhsFine);
MGIC_API int mgic_op_prolong_increment(mgic_op fine, mgic_field phiFine, mgic_field corCoarse);
MGIC_API int mgic_op_set_alpha_beta(mgic_op op, double alpha, double beta);
MGIC_API int mgic_op_set_coefs(mgic_op op, mgic_field aCoef, mgic_field bCoef, double alpha,
                               double beta);
MGIC_API int mgic_op_reset_lambda(mgic_op op);
MGIC_API int mgic_op_set_time(mgic_op op, double t);
/* set_update_psi0 (SetLevelData.cpp:236-256): exchange dpsi, its domain
 * ghosts = the inhomogeneous BC image, psi += dpsi over the valid cells and
 * ghost layer 1 */
MGIC_API int mgic_op_update_psi(mgic_op op, mgic_field psi, mgic_field dpsi);
MGIC_API int mgic_op_fill_bc(mgic_op op, mgic_field u, int homogeneous);         /* m_bc */
MGIC_API int mgic_op_set_to_zero(mgic_op op, mgic_field x);
MGIC_API int mgic_op_assign(mgic_op op, mgic_field lhs, mgic_field rhs);
MGIC_API int mgic_op_incr(mgic_op op, mgic_field lhs, mgic_field x, double scale);
MGIC_API int mgic_op_axby(mgic_op op, mgic_field lhs, mgic_field x, mgic_field y, double a,
                          double b);
MGIC_API int mgic_op_scale(mgic_op op, mgic_field lhs, double s);
MGIC_API int mgic_op_dot(mgic_op op, mgic_field x, mgic_field y, double *out);
MGIC_API int mgic_op_norm(mgic_op op, mgic_field x, int ord, double *out);
/* BiCGStabSolver<LevelData>::solve with this op (bottom solver) */
MGIC_API int mgic_op_bicgstab(mgic_op op, mgic_field phi, mgic_field rhs, int homogeneous,
                              const mgic_mg_params *p, int *iterations);

/* ---- multigrid (AMRMultiGrid on one AMR level + MultiGrid hierarchy) */
MGIC_API int mgic_mg_create(mgic_factory f, const mgic_mg_params *p, mgic_mg *out);
MGIC_API int mgic_mg_destroy(mgic_mg mg);
MGIC_API int mgic_mg_num_depths(mgic_mg mg, int *n);
MGIC_API int mgic_mg_op(mgic_mg mg, int depth, mgic_op *out);
/* internal fields of depth >= 1: which 0 = correction e, 1 = residual r */
MGIC_API int mgic_mg_level_field(mgic_mg mg, int depth, int which, mgic_field *out);
MGIC_API int mgic_mg_one_cycle(mgic_mg mg, mgic_field e, mgic_field r); /* MultiGrid::oneCycle */
/* e = 0; oneCycle(e, resid); phi += e; resid = rhs - L(phi); *norm (if
 * norm_type >= 0, else not computed and nothing synchronised) */
MGIC_API int mgic_mg_iteration(mgic_mg mg, mgic_field phi, mgic_field rhs, mgic_field resid,
                               int norm_type, int homogeneous, double *norm);
/* `count` iterations (AMRMultiGrid::solve's loop body) from the state
 * mgic_mg_iteration / mgic_mg_init_residual leave; norms[i] (count values,
 * may be NULL) = what the i-th mgic_mg_iteration call would return, bit for
 * bit (the same launches in the same order).  Iteration i's norm is read on
 * the host after iteration i+1's V-cycle has been queued up to its first
 * launch that writes phi and before that launch is queued -- where a stop
 * test on the norm would decide -- so the device does not idle while the
 * host reads it. */
MGIC_API int mgic_mg_iterations(mgic_mg mg, mgic_field phi, mgic_field rhs, mgic_field resid,
                                int count, int norm_type, int homogeneous, double *norms);
MGIC_API int mgic_mg_init_residual(mgic_mg mg, mgic_field phi, mgic_field rhs,
                                   mgic_field resid, int norm_type, int homogeneous,
                                   double *norm);
/* full multigrid on the current resid (as left by init_residual /
 * iteration): resid restricted to every depth, bottom solve, then per finer
 * depth e = P e_coarse and `ncycles` V-cycles; phi += e; resid = rhs - L(phi) */
MGIC_API int mgic_mg_fmg(mgic_mg mg, mgic_field phi, mgic_field rhs, mgic_field resid,
                         int norm_type, int homogeneous, int ncycles, double *norm);
/* HIP events around every BiCGStab bottom solve this rank runs (bottom_solver
 * 1; with a gathered coarsest depth only its owner runs them): on != 0 resets
 * and starts recording; bottom_ms returns their total time and count */
MGIC_API int mgic_mg_bottom_timer(mgic_mg mg, int on);
MGIC_API int mgic_mg_bottom_ms(mgic_mg mg, double *ms, int *calls);
/* BiCGStab iterations summed over the solves timed since mgic_mg_bottom_timer
 * (1), and the smallest / largest norm of the coarse residual they started
 * from (the bench's proof that each timed solve did work) */
MGIC_API int mgic_mg_bottom_iters(mgic_mg mg, long long *iters, double *r0_min, double *r0_max);
/* the last BiCGStab bottom solve this rank ran: on the device (1) or by the
 * host loop (0), its iterations and the norm of the residual it started from */
MGIC_API int mgic_mg_bottom_info(mgic_mg mg, int *device, int *iters, double *r0);
/* the last bottom solve again, n times, each from e = 0 on the same coarse
 * residual: total ms (HIP events), iterations per solve, the residual's norm;
 * *solves = n, or 0 on a rank that does not run the coarsest depth or before
 * a V-cycle has run a bottom solve */
MGIC_API int mgic_mg_bottom_replay(mgic_mg mg, int n, double *ms, int *iters, double *r0,
                                   int *solves);

/* Mixed precision (BASELINE config C5): the same V-cycle schedule with the
 * correction equation in fp32 (GSRB / restrictResidual / prolongIncrement in
 * float, coefficients rounded from the fp64 hierarchy), the fine residual
 * rhs - L(phi) in fp64 rounded once, phi += e in fp64.  Bottom: relax
 * (n_bottom).  agglomerate_below and deep_halo as for the fp64 cycle (fp32
 * gathers / scatters and 4-deep fp32 shells).  resid (fp64) may be NULL
 * unless a norm is requested (norm_type >= 0).  Inhomogeneous BC for the fine
 * residual. */
MGIC_API int mgic_mixed_create(mgic_factory f, const mgic_mg_params *p, mgic_mixed *out);
MGIC_API int mgic_mixed_destroy(mgic_mixed m);
MGIC_API int mgic_mixed_num_depths(mgic_mixed m, int *n);
MGIC_API int mgic_mixed_init_residual(mgic_mixed m, mgic_field phi, mgic_field rhs,
                                      mgic_field resid, int norm_type, double *norm);
MGIC_API int mgic_mixed_iteration(mgic_mixed m, mgic_field phi, mgic_field rhs, mgic_field resid,
                                  int norm_type, double *norm);
MGIC_API int mgic_mixed_fmg(mgic_mixed m, mgic_field phi, mgic_field rhs, mgic_field resid,
                            int norm_type, int ncycles, double *norm);

/* ---- AMR levels > 0 ([Chombo] AMRPoissonOp multi-level
 * operators restated: QuadCFInterp, AMROperator / AMRResidual (reflux a
 * no-op as in the reference), AMRRestrict, AMRProlong, AMRUpdateResidual,
 * AMRMultiGrid's multi-level V-cycle).  grids[0] tiles its domain; level
 * l+1's domain is level l's refined by 2 and its boxes are properly nested
 * (mgic_grid_create_patches).  Level 0 is solved by its MultiGrid (base). */
MGIC_API int mgic_grid_create_patches(mgic_comm c, const int domain[6], const int periodic[3],
                                      double dx, int nbox, const int *boxes, const int *owners,
                                      mgic_grid *out); /* disjoint boxes inside the domain */
MGIC_API int mgic_amr_create(int nlevels, const mgic_grid *grids, const mgic_field *acoef,
                             const mgic_field *bcoef, const mgic_op_params *op,
                             const mgic_mg_params *base, mgic_amr *out);
MGIC_API int mgic_amr_destroy(mgic_amr a);
MGIC_API int mgic_amr_num_levels(mgic_amr a, int *n);
MGIC_API int mgic_amr_level_op(mgic_amr a, int level, mgic_op *out); /* borrowed */
/* coarse == NULL: homogeneousCFInterp (zero coarse field) */
MGIC_API int mgic_amr_cf_interp(mgic_amr a, int level, mgic_field u, mgic_field coarse);
MGIC_API int mgic_amr_average_down(mgic_amr a, int level, mgic_field coarse, mgic_field fine);
MGIC_API int mgic_amr_operator(mgic_amr a, int level, mgic_field lphi, mgic_field phi,
                               mgic_field phi_coarse, int homogeneous);
MGIC_API int mgic_amr_residual(mgic_amr a, int level, mgic_field r, mgic_field phi,
                               mgic_field phi_coarse, mgic_field rhs, int homogeneous);
MGIC_API int mgic_amr_restrict(mgic_amr a, int level, mgic_field res_coarse, mgic_field res,
                               mgic_field corr, mgic_field corr_coarse);
MGIC_API int mgic_amr_prolong(mgic_amr a, int level, mgic_field corr, mgic_field corr_coarse);
MGIC_API int mgic_amr_update_residual(mgic_amr a, int level, mgic_field res, mgic_field corr,
                                      mgic_field corr_coarse);
/* composite residuals rhs - L(phi) on every level (covered coarse cells
 * zeroed); *norm = max over levels (norm_type >= 0) */
MGIC_API int mgic_amr_init_residual(mgic_amr a, const mgic_field *phi, const mgic_field *rhs,
                                    int norm_type, double *norm);
/* one AMR V-cycle, phi += e on every level, average down, new residuals */
MGIC_API int mgic_amr_iteration(mgic_amr a, const mgic_field *phi, const mgic_field *rhs,
                                int norm_type, double *norm);
MGIC_API int mgic_amr_residual_field(mgic_amr a, int level, mgic_field *out); /* borrowed */
/* MultilevelLinearOp over the hierarchy (Main_PoissonSolver.cpp:103-117,
 * 169-170 with max_level > 0; [Chombo] semantics restated, see amr.hpp):
 * lhs = AMROperator on every level, covered coarse cells zeroed; dot =
 * sum_l dx_l^3 levelDot; norm 0 = max over levels, 1 / 2 = dx_l^3-weighted;
 * dot and norm mask the covered coarse cells of x (MultilevelLinearOp's
 * dotProduct / norm count each physical cell once, on its finest level) */
MGIC_API int mgic_amr_apply_op(mgic_amr a, const mgic_field *lhs, const mgic_field *x,
                               int homogeneous);
MGIC_API int mgic_amr_dot(mgic_amr a, const mgic_field *x, const mgic_field *y, double *out);
MGIC_API int mgic_amr_norm(mgic_amr a, const mgic_field *x, int ord, double *out);
/* computeNorm / computeSum (Main_PoissonSolver.cpp:144-145,208-209): covered
 * coarse cells masked, dx_l^3 weights (x is not modified) */
MGIC_API int mgic_amr_composite_norm(mgic_amr a, const mgic_field *x, int ord, double *out);
MGIC_API int mgic_amr_composite_sum(mgic_amr a, const mgic_field *x, double *out);
/* MultilevelLinearOp::preCond: e = 0, `iters` AMR V-cycle iterations on
 * (e, r) with homogeneous physical BCs */
MGIC_API int mgic_amr_precondition(mgic_amr a, const mgic_field *e, const mgic_field *r, int iters);

/* ---- output (WriteOutput.H).  For local box n, planes
 * [k0, k0+nk) of its valid box: the components the reference writes,
 * component-major and i fastest (the FArrayBox order of that box's chunk of
 * "data:datatype=0"), into out (host memory, or device memory if
 * out_on_device).
 * grchombo_vars: set_output_data (SetLevelData.cpp:343-396), the 31
 *   GRChombo variables (GRChomboUserVariables.hpp order) from psi, with
 *   constant_K = bh[12];
 * solver_vars: output_solver_data's 10 components (WriteOutput.H:74-100):
 *   dpsi, rhs, psi, A11_0, A12_0, A13_0, A22_0, A23_0, A33_0, phi_0. */
MGIC_API int mgic_field_grchombo_vars(mgic_field psi, int n, int k0, int nk, const double bh[13],
                                      double *out, int out_on_device);
MGIC_API int mgic_field_solver_vars(mgic_field dpsi, mgic_field rhs, mgic_field psi, int n, int k0,
                                    int nk, const double bh[13], double *out, int out_on_device);
/* the field's layout: domain, periodicity, dx, number of boxes (all ranks),
 * this rank and the job size; box i's extent, owner rank and local index
 * (-1 if not local); a barrier over the field's communicator */
MGIC_API int mgic_field_layout(mgic_field f, int domain[6], int periodic[3], double *dx, int *nbox,
                               int *rank, int *size);
MGIC_API int mgic_field_box(mgic_field f, int i, int lohi[6], int *owner, int *local_index);
MGIC_API int mgic_field_barrier(mgic_field f);
/* page-locked host memory (hipHostMalloc) for staging device output: the
 * D2H copies of mgic_field_*_vars run at full PCIe rate into it */
MGIC_API int mgic_host_alloc(size_t bytes, void **out);
MGIC_API int mgic_host_free(void *p);

/* MultilevelLinearOp::preCond: e = 0, then `iters` AMRMultiGrid iterations
 * on (e, r), homogeneous BC (Main_PoissonSolver.cpp:107-117) */
MGIC_API int mgic_mg_precondition(mgic_mg mg, mgic_field e, mgic_field r, int iters);

/* ---- the linear solve solver.solve(dpsi, rhs) (Main_PoissonSolver.cpp:
 *      103-126, 169-184): BiCGStab over the level operator, preconditioned
 *      by mgic_mg_precondition */
typedef struct {
  int num_mg_iterations; /* numMGIterations (default 1) */
  int max_iterations;    /* max_iterations -> BiCGStab m_imax (default 10) */
  double tolerance;      /* tolerance -> m_eps (default 1e-7) */
  int norm_type;         /* m_normType (0 = max norm) */
} mgic_solve_params;
MGIC_API void mgic_solve_params_default(mgic_solve_params *p);
MGIC_API int mgic_mg_solve(mgic_mg mg, mgic_field phi, mgic_field rhs, const mgic_solve_params *p,
                           int *iterations, double *final_norm);
/* the same solve over an AMR hierarchy (max_level > 0): BiCGStab over
 * mgic_amr_apply_op, preconditioned by mgic_amr_precondition */
MGIC_API int mgic_amr_solve(mgic_amr a, const mgic_field *phi, const mgic_field *rhs,
                            const mgic_solve_params *p, int *iterations, double *final_norm);

/* ---- instrumentation: hipEvents around the smoother launches on boxes of
 * at least min_cells cells (enable 1: a pair per launch; 2: a pair per run of
 * consecutive launches within one relax call -- fewer records in the timed
 * stream); launches / passes = launches timed and the colour passes they
 * performed (1 per-colour launch, 2 one fused sweep, 4 two fused sweeps) */
MGIC_API int mgic_prof_smoother(int enable, long min_cells);
MGIC_API int mgic_prof_smoother_read(int *launches, long *passes, double *total_ms);

#ifdef __cplusplus
}
#endif
#endif /* MGIC_H */
