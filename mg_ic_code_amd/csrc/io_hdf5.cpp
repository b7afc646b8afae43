// io_hdf5.cpp -- libmgic_io: the reference's two HDF5 writers
// (Source/WriteOutput.H) over libmgic device fields, in Chombo's AMR HDF5
// layout (see include/mgic_io.h).  Host code only: the per-box components are
// computed on the GPU by mgic_field_grchombo_vars / mgic_field_solver_vars
// (k_output_vars) in z-slabs and streamed into hyperslabs of
// "data:datatype=0".
#include "mgic_io.h"

#include <hdf5.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <exception>
#include <vector>

namespace {

thread_local std::string g_err;

struct IoError : std::runtime_error {
  int code;
  IoError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define H5OK(x)                                                             \
  ([&]() {                                                                     \
    auto r_ = (x);                                                             \
    if (r_ < 0) throw IoError(MGIC_EUNKNOWN, std::string("HDF5 call failed: ") + #x); \
    return r_;                                                                 \
  }())

void mg(int rc) {  // a libmgic call
  if (rc != MGIC_OK) throw IoError(rc, std::string("libmgic: ") + mgic_last_error());
}

// GRChomboUserVariables.hpp:58-75 and MultigridUserVariables.hpp:29-33
const char *const kGRChomboNames[31] = {
    "chi",    "h11",    "h12",    "h13",    "h22",    "h23", "h33", "K",   "A11",  "A12",  "A13",
    "A22",    "A23",    "A33",    "Theta",  "Gamma1", "Gamma2", "Gamma3", "lapse", "shift1",
    "shift2", "shift3", "B1",     "B2",     "B3",     "phi", "Pi",  "Ham", "Mom1", "Mom2", "Mom3"};
const char *const kSolverNames[10] = {"dpsi",  "rhs",   "psi",   "A11_0", "A12_0",
                                      "A13_0", "A22_0", "A23_0", "A33_0", "phi_0"};

// Chombo's HDF5Handle compound types
hid_t box_type() {
  hid_t t = H5OK(H5Tcreate(H5T_COMPOUND, 6 * sizeof(int)));
  const char *n[6] = {"lo_i", "lo_j", "lo_k", "hi_i", "hi_j", "hi_k"};
  for (int d = 0; d < 6; ++d) H5OK(H5Tinsert(t, n[d], d * sizeof(int), H5T_NATIVE_INT));
  return t;
}
hid_t intvect_type() {
  hid_t t = H5OK(H5Tcreate(H5T_COMPOUND, 3 * sizeof(int)));
  const char *n[3] = {"intvecti", "intvectj", "intvectk"};
  for (int d = 0; d < 3; ++d) H5OK(H5Tinsert(t, n[d], d * sizeof(int), H5T_NATIVE_INT));
  return t;
}

// HDF5HeaderData: named scalar attributes on a group
struct Header {
  std::map<std::string, double> reals;
  std::map<std::string, int> ints;
  std::map<std::string, std::string> strings;
  std::map<std::string, std::array<int, 3>> intvects;
  std::map<std::string, std::array<int, 6>> boxes;

  static void attr(hid_t loc, const std::string &name, hid_t type, const void *v) {
    hid_t sp = H5OK(H5Screate(H5S_SCALAR));
    hid_t a = H5OK(H5Acreate2(loc, name.c_str(), type, sp, H5P_DEFAULT, H5P_DEFAULT));
    H5OK(H5Awrite(a, type, v));
    H5Aclose(a);
    H5Sclose(sp);
  }
  void write(hid_t loc) const {
    for (auto &kv : reals) attr(loc, kv.first, H5T_NATIVE_DOUBLE, &kv.second);
    for (auto &kv : ints) attr(loc, kv.first, H5T_NATIVE_INT, &kv.second);
    for (auto &kv : strings) {
      hid_t t = H5OK(H5Tcopy(H5T_C_S1));
      H5OK(H5Tset_size(t, kv.second.empty() ? 1 : kv.second.size()));
      attr(loc, kv.first, t, kv.second.c_str());
      H5Tclose(t);
    }
    if (!intvects.empty()) {
      hid_t t = intvect_type();
      for (auto &kv : intvects) attr(loc, kv.first, t, kv.second.data());
      H5Tclose(t);
    }
    if (!boxes.empty()) {
      hid_t t = box_type();
      for (auto &kv : boxes) attr(loc, kv.first, t, kv.second.data());
      H5Tclose(t);
    }
  }
};

// One level's layout as the writer sees it.
struct LevelLayout {
  std::array<int, 6> domain{};
  double dx = 0.0;
  std::vector<std::array<int, 6>> boxes;
  std::vector<int> owners;
  long long ncells(size_t b) const {
    long long n = 1;
    for (int d = 0; d < 3; ++d) n *= boxes[b][3 + d] - boxes[b][d] + 1;
    return n;
  }
};

struct Job {
  int kind = 0;  // 0 final data, 1 solver data
  int ncomp = 31;
  std::vector<LevelLayout> levels;
  std::vector<int> ref_ratio;
  int max_level = 0, iter = 0;
};

// the file skeleton: global group, headers, boxes, offsets, an empty data
// dataset of the full size (rank 0 only)
void create_file(const std::string &fname, const Job &J) {
  hid_t f = H5OK(H5Fcreate(fname.c_str(), H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT));
  {  // HDF5Handle::open(CREATE): /Chombo_global {SpaceDim, testReal}
    hid_t g = H5OK(H5Gcreate2(f, "Chombo_global", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT));
    Header h;
    h.ints["SpaceDim"] = 3;
    h.reals["testReal"] = 0.0;
    h.write(g);
    H5Gclose(g);
  }
  const int nlev = (int)J.levels.size();
  const char *const *names = J.kind == 0 ? kGRChomboNames : kSolverNames;
  {
    Header h;
    hid_t root = H5OK(H5Gopen2(f, "/", H5P_DEFAULT));
    if (J.kind == 0) {  // output_final_data, WriteOutput.H:145-173
      h.ints["max_level"] = J.max_level;
      h.ints["num_levels"] = J.max_level + 1;
      h.ints["iteration"] = 0;
      h.reals["time"] = 0.0;
      for (int l = 0; l < nlev; ++l) {
        h.ints["regrid_interval_" + std::to_string(l)] = 1;
        h.ints["steps_since_regrid_" + std::to_string(l)] = 0;
      }
    } else {  // [Chombo] WriteAMRHierarchyHDF5 (AMRIO)
      h.strings["filetype"] = "VanillaAMRFileType";
      h.ints["num_levels"] = nlev;
    }
    h.ints["num_components"] = J.ncomp;
    for (int c = 0; c < J.ncomp; ++c) h.strings["component_" + std::to_string(c)] = names[c];
    h.write(root);
    H5Gclose(root);
  }
  double dt = 1.0;  // output_solver_data's fakeDt, refined with the levels
  for (int l = 0; l < nlev; ++l) {
    const LevelLayout &L = J.levels[l];
    hid_t g = H5OK(H5Gcreate2(f, ("level_" + std::to_string(l)).c_str(), H5P_DEFAULT,
                                 H5P_DEFAULT, H5P_DEFAULT));
    Header h;
    if (J.kind == 0) {  // WriteOutput.H:196-216
      h.ints["ref_ratio"] = J.ref_ratio[l];
      h.ints["tag_buffer_size"] = 3;
      h.reals["dx"] = L.dx;
      h.reals["dt"] = 0.25 * L.dx;
      h.reals["time"] = 0.0;
      for (int d = 0; d < 3; ++d) h.ints["is_periodic_" + std::to_string(d)] = 1;
    } else {  // writeLevel
      if (l > 0) dt /= J.ref_ratio[l - 1];
      h.ints["ref_ratio"] = l == nlev - 1 ? 1 : J.ref_ratio[l];
      h.reals["dx"] = L.dx;
      h.reals["dt"] = dt;
      h.reals["time"] = (double)J.iter;
    }
    h.boxes["prob_domain"] = L.domain;
    h.write(g);
    const hsize_t nb = L.boxes.size();
    {  // write(handle, BoxLayout): "boxes" (+ "Processors")
      hid_t bt = box_type();
      hid_t sp = H5OK(H5Screate_simple(1, &nb, nullptr));
      hid_t ds = H5OK(H5Dcreate2(g, "boxes", bt, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT));
      if (nb) H5OK(H5Dwrite(ds, bt, H5S_ALL, H5S_ALL, H5P_DEFAULT, L.boxes.data()));
      H5Dclose(ds);
      H5Tclose(bt);
      hid_t dp = H5OK(H5Dcreate2(g, "Processors", H5T_NATIVE_INT, sp, H5P_DEFAULT, H5P_DEFAULT,
                                    H5P_DEFAULT));
      if (nb) H5OK(H5Dwrite(dp, H5T_NATIVE_INT, H5S_ALL, H5S_ALL, H5P_DEFAULT, L.owners.data()));
      H5Dclose(dp);
      H5Sclose(sp);
    }
    {  // write(handle, LevelData, "data"): data_attributes, offsets, data
      hid_t ga = H5OK(H5Gcreate2(g, "data_attributes", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT));
      Header a;
      a.ints["comps"] = J.ncomp;
      a.strings["objectType"] = "FArrayBox";
      const int gh = J.kind == 0 ? 3 : 0;  // the LevelData's ghosts (WriteOutput.H:189 / :90)
      a.intvects["ghost"] = {gh, gh, gh};
      a.intvects["outputGhost"] = {0, 0, 0};
      a.write(ga);
      H5Gclose(ga);
      std::vector<long long> off(nb + 1, 0);
      for (size_t b = 0; b < nb; ++b) off[b + 1] = off[b] + L.ncells(b) * J.ncomp;
      const hsize_t no = nb + 1;
      hid_t so = H5OK(H5Screate_simple(1, &no, nullptr));
      hid_t dso = H5OK(H5Dcreate2(g, "data:offsets=0", H5T_NATIVE_LLONG, so, H5P_DEFAULT,
                                     H5P_DEFAULT, H5P_DEFAULT));
      H5OK(H5Dwrite(dso, H5T_NATIVE_LLONG, H5S_ALL, H5S_ALL, H5P_DEFAULT, off.data()));
      H5Dclose(dso);
      H5Sclose(so);
      const hsize_t nd = (hsize_t)off[nb];
      hid_t sd = H5OK(H5Screate_simple(1, &nd, nullptr));
      hid_t dsd = H5OK(H5Dcreate2(g, "data:datatype=0", H5T_NATIVE_DOUBLE, sd, H5P_DEFAULT,
                                     H5P_DEFAULT, H5P_DEFAULT));
      H5Dclose(dsd);
      H5Sclose(sd);
    }
    H5Gclose(g);
  }
  H5OK(H5Fclose(f));
}

// write `n` doubles at element `offset` of level l's data:datatype=0
struct DataWriter {
  hid_t f = -1;
  std::vector<hid_t> ds;
  DataWriter(const std::string &fname, int nlev) {
    f = H5OK(H5Fopen(fname.c_str(), H5F_ACC_RDWR, H5P_DEFAULT));
    for (int l = 0; l < nlev; ++l)
      ds.push_back(H5OK(
          H5Dopen2(f, ("level_" + std::to_string(l) + "/data:datatype=0").c_str(), H5P_DEFAULT)));
  }
  void write(int l, hsize_t offset, hsize_t n, const double *v) {
    if (!n) return;
    hid_t fs = H5OK(H5Dget_space(ds[l]));
    H5OK(H5Sselect_hyperslab(fs, H5S_SELECT_SET, &offset, nullptr, &n, nullptr));
    hid_t ms = H5OK(H5Screate_simple(1, &n, nullptr));
    H5OK(H5Dwrite(ds[l], H5T_NATIVE_DOUBLE, ms, fs, H5P_DEFAULT, v));
    H5Sclose(ms);
    H5Sclose(fs);
  }
  ~DataWriter() {
    for (hid_t d : ds) H5Dclose(d);
    if (f >= 0) H5Fclose(f);
  }
};

// the device path: layouts from the fields, rank 0 creates, ranks write
// their boxes in turn
void write_fields(const std::string &fname, Job &J, const std::vector<mgic_field> &lead,
                  const std::function<void(int l, int n, int k0, int nk, double *)> &produce) {
  const int nlev = (int)lead.size();
  int rank = 0, size = 1;
  J.levels.resize(nlev);
  for (int l = 0; l < nlev; ++l) {
    LevelLayout &L = J.levels[l];
    int dom[6], per[3], nbox = 0;
    mg(mgic_field_layout(lead[l], dom, per, &L.dx, &nbox, &rank, &size));
    for (int d = 0; d < 6; ++d) L.domain[d] = dom[d];
    L.boxes.resize(nbox);
    L.owners.resize(nbox);
    for (int b = 0; b < nbox; ++b) mg(mgic_field_box(lead[l], b, L.boxes[b].data(), &L.owners[b], nullptr));
  }
  if (rank == 0) create_file(fname, J);
  mg(mgic_field_barrier(lead[0]));
  const long long kSlabBytes = 256ll << 20;  // host staging per slab
  // two page-locked slabs: slab i+1 is computed and copied D2H while a
  // writer thread puts slab i into the file (only that thread calls HDF5
  // meanwhile; the main thread only calls libmgic)
  struct Pinned {
    double *p = nullptr;
    size_t n = 0;
    void reserve(size_t m) {
      if (m <= n) return;
      if (p) mgic_host_free(p);
      p = nullptr;
      n = 0;
      void *q = nullptr;
      mg(mgic_host_alloc(sizeof(double) * m, &q));
      p = static_cast<double *>(q);
      n = m;
    }
    ~Pinned() {
      if (p) mgic_host_free(p);
    }
  } host[2];
  std::thread writer;
  std::exception_ptr werr;
  auto join = [&] {
    if (writer.joinable()) writer.join();
    if (werr) std::rethrow_exception(werr);
  };
  for (int r = 0; r < size; ++r) {
    if (r == rank) {
      DataWriter W(fname, nlev);
      struct Joiner {  // an exception leaves no writer thread on W or the slabs
        std::thread &t;
        ~Joiner() {
          if (t.joinable()) t.join();
        }
      } joiner{writer};
      for (int l = 0; l < nlev; ++l) {
        const LevelLayout &L = J.levels[l];
        long long off = 0;
        for (size_t b = 0; b < L.boxes.size(); ++b) {
          const long long nc = L.ncells(b);
          int loc = -1, lohi[6], owner = 0;
          mg(mgic_field_box(lead[l], (int)b, lohi, &owner, &loc));
          if (loc >= 0) {
            const int nx = lohi[3] - lohi[0] + 1, ny = lohi[4] - lohi[1] + 1,
                      nz = lohi[5] - lohi[2] + 1;
            const long long plane = (long long)nx * ny;
            int nk = (int)std::max<long long>(1, kSlabBytes / (8ll * J.ncomp * plane));
            if (nk > nz) nk = nz;
            int cur = 0;
            for (int k0 = 0; k0 < nz; k0 += nk) {
              const int kk = std::min(nk, nz - k0);
              if (host[cur].n < (size_t)J.ncomp * plane * nk) {
                join();  // the writer may still read the other slab, not this one
                host[cur].reserve((size_t)J.ncomp * plane * nk);
              }
              double *buf = host[cur].p;
              produce(l, loc, k0, kk, buf);
              join();
              const int ncomp = J.ncomp;
              writer = std::thread([&W, &werr, l, off, nc, k0, kk, plane, ncomp, buf] {
                try {
                  for (int c = 0; c < ncomp; ++c)
                    W.write(l, (hsize_t)(off + c * nc + k0 * plane), (hsize_t)(kk * plane),
                            buf + (size_t)c * kk * plane);
                } catch (...) {
                  werr = std::current_exception();
                }
              });
              cur ^= 1;
            }
            join();
          }
          off += nc * J.ncomp;
        }
      }
    }
    mg(mgic_field_barrier(lead[0]));
  }
}

template <class F>
int guard(F &&f) {
  H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr);  // errors come back as status codes
  try {
    f();
    return MGIC_OK;
  } catch (const IoError &e) {
    g_err = e.what();
    return e.code;
  } catch (const std::exception &e) {
    g_err = e.what();
    return MGIC_EUNKNOWN;
  }
}

void need(const void *p, const char *what) {
  if (!p) throw IoError(MGIC_EBADARG, std::string("null argument: ") + what);
}

}  // namespace

extern "C" {

MGIC_IO_API const char *mgic_io_last_error(void) { return g_err.c_str(); }

MGIC_IO_API int mgic_io_write_final_data(const char *filename, int nlevels, const mgic_field *psi,
                                         const double bh[13], int max_level,
                                         const int *ref_ratio) {
  return guard([&] {
    need(psi, "psi");
    need(bh, "bh");
    need(ref_ratio, "ref_ratio");
    if (nlevels < 1) throw IoError(MGIC_EBADARG, "nlevels < 1");
    Job J;
    J.kind = 0;
    J.ncomp = 31;
    J.max_level = max_level;
    J.ref_ratio.assign(ref_ratio, ref_ratio + nlevels);
    std::vector<mgic_field> lead(psi, psi + nlevels);
    for (auto f : lead) need(f, "psi[l]");
    write_fields(filename ? filename : "vcPoissonFinal.3d.hdf5", J, lead,
                 [&](int l, int n, int k0, int nk, double *out) {
                   mg(mgic_field_grchombo_vars(psi[l], n, k0, nk, bh, out, 0));
                 });
  });
}

MGIC_IO_API int mgic_io_write_solver_data(const char *filename, int nlevels,
                                          const mgic_field *dpsi, const mgic_field *rhs,
                                          const mgic_field *psi, const double bh[13],
                                          const int *ref_ratio, int iter) {
  return guard([&] {
    need(dpsi, "dpsi");
    need(rhs, "rhs");
    need(psi, "psi");
    need(bh, "bh");
    need(ref_ratio, "ref_ratio");
    if (nlevels < 1) throw IoError(MGIC_EBADARG, "nlevels < 1");
    Job J;
    J.kind = 1;
    J.ncomp = 10;
    J.iter = iter;
    J.ref_ratio.assign(ref_ratio, ref_ratio + nlevels);
    std::vector<mgic_field> lead(psi, psi + nlevels);
    for (int l = 0; l < nlevels; ++l) {
      need(psi[l], "psi[l]");
      need(dpsi[l], "dpsi[l]");
      need(rhs[l], "rhs[l]");
    }
    char name[64];
    std::snprintf(name, sizeof name, "vcPoissonOut.3d_%d.hdf5", iter);  // WriteOutput.H:63-70
    write_fields(filename ? filename : name, J, lead, [&](int l, int n, int k0, int nk, double *out) {
      mg(mgic_field_solver_vars(dpsi[l], rhs[l], psi[l], n, k0, nk, bh, out, 0));
    });
  });
}

MGIC_IO_API int mgic_io_write_host(const char *filename, int kind, int nlevels, const int *nbox,
                                   const int *boxes, const int *domains, const double *dx,
                                   const int *ref_ratio, const double *data, int max_level,
                                   int iter) {
  return guard([&] {
    need(filename, "filename");
    need(nbox, "nbox");
    need(boxes, "boxes");
    need(domains, "domains");
    need(dx, "dx");
    need(ref_ratio, "ref_ratio");
    need(data, "data");
    if (nlevels < 1 || (kind != 0 && kind != 1)) throw IoError(MGIC_EBADARG, "bad nlevels/kind");
    Job J;
    J.kind = kind;
    J.ncomp = kind == 0 ? 31 : 10;
    J.max_level = max_level;
    J.iter = iter;
    J.ref_ratio.assign(ref_ratio, ref_ratio + nlevels);
    J.levels.resize(nlevels);
    const int *bp = boxes;
    for (int l = 0; l < nlevels; ++l) {
      LevelLayout &L = J.levels[l];
      for (int d = 0; d < 6; ++d) L.domain[d] = domains[6 * l + d];
      L.dx = dx[l];
      if (nbox[l] < 0) throw IoError(MGIC_EBADARG, "nbox < 0");
      for (int b = 0; b < nbox[l]; ++b, bp += 6) {
        std::array<int, 6> x;
        for (int d = 0; d < 6; ++d) x[d] = bp[d];
        for (int d = 0; d < 3; ++d)
          if (x[3 + d] < x[d]) throw IoError(MGIC_EBADARG, "empty box");
        L.boxes.push_back(x);
        L.owners.push_back(0);
      }
    }
    create_file(filename, J);
    DataWriter W(filename, nlevels);
    const double *p = data;
    for (int l = 0; l < nlevels; ++l) {
      long long tot = 0;
      for (size_t b = 0; b < J.levels[l].boxes.size(); ++b) tot += J.levels[l].ncells(b) * J.ncomp;
      W.write(l, 0, (hsize_t)tot, p);
      p += tot;
    }
  });
}

}  // extern "C"
