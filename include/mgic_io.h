/* mgic_io.h -- HDF5 output in the reference's layouts.
 *
 * libmgic_io.so: a host library over libmgic (device fields) and libhdf5
 * (serial, /opt/conda).  It replaces the two writers in Source/WriteOutput.H:
 *
 *   output_final_data  (WriteOutput.H:127-227): the GRChombo checkpoint,
 *     31 components of set_output_data (SetLevelData.cpp:343-396) per level;
 *   output_solver_data (WriteOutput.H:52-123): the per-NL-iteration file of
 *     WriteAMRHierarchyHDF5 with dpsi, rhs and the 8 multigrid_vars.
 *
 * Both write Chombo's AMR HDF5 layout, restated (Chombo's CH_HDF5 / AMRIO
 * are not in the reference tree, so the layout is parity unpinned):
 *   /Chombo_global           attrs SpaceDim, testReal
 *   /                        header attrs (num_levels, num_components,
 *                            component_<c>, ...)
 *   /level_<l>               attrs ref_ratio, dx, dt, time, prob_domain, ...
 *   /level_<l>/boxes         compound {lo_i,lo_j,lo_k,hi_i,hi_j,hi_k}, layout order
 *   /level_<l>/Processors    owner rank per box
 *   /level_<l>/data:offsets=0   long long, nbox + 1 (cumulative doubles)
 *   /level_<l>/data:datatype=0  double, per box: components in order, each
 *                               over the valid box, i fastest (outputGhost 0)
 *   /level_<l>/data_attributes  attrs comps, objectType, ghost, outputGhost
 *
 * Every rank calls the device entry points (collective over the fields'
 * communicator): rank 0 creates the file and the datasets, then each rank in
 * turn writes its own boxes' hyperslabs.  Status codes as libmgic.
 */
#ifndef MGIC_IO_H
#define MGIC_IO_H

#include "mgic.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MGIC_IO_API __attribute__((visibility("default")))

MGIC_IO_API const char *mgic_io_last_error(void);

/* output_final_data (WriteOutput.H:127-227).  psi[l] is level l's
 * multigrid_vars psi (the level's grid, dx and domain come from it);
 * bh[13] as mgic_field_binary_bh with bh[12] = constant_K; max_level and
 * ref_ratio[l] as PoissonParameters.  filename NULL: "vcPoissonFinal.3d.hdf5". */
MGIC_IO_API int mgic_io_write_final_data(const char *filename, int nlevels, const mgic_field *psi,
                                         const double bh[13], int max_level,
                                         const int *ref_ratio);

/* output_solver_data (WriteOutput.H:52-123) for NL iteration iter (time =
 * iter, dt = 1).  filename NULL: "vcPoissonOut.3d_<iter>.hdf5". */
MGIC_IO_API int mgic_io_write_solver_data(const char *filename, int nlevels,
                                          const mgic_field *dpsi, const mgic_field *rhs,
                                          const mgic_field *psi, const double bh[13],
                                          const int *ref_ratio, int iter);

/* The same two layouts from host arrays (tests, and callers whose data is
 * already on the host).  kind 0: final data (31 components), 1: solver data
 * (10).  Level l has nbox[l] boxes (6 ints each, all levels concatenated in
 * `boxes`), domain domains[6 l..], cell size dx[l]; `data` holds every box of
 * every level in that order, each box component-major, i fastest.  iter and
 * max_level as above (iter ignored for kind 0, max_level for kind 1). */
MGIC_IO_API int mgic_io_write_host(const char *filename, int kind, int nlevels, const int *nbox,
                                   const int *boxes, const int *domains, const double *dx,
                                   const int *ref_ratio, const double *data, int max_level,
                                   int iter);

#ifdef __cplusplus
}
#endif
#endif /* MGIC_IO_H */
