// MPI front end (libspfft_amd_mpi): MPI_Comm-taking constructors and getters
// of the C++ and C APIs, the Fortran communicator shims, and the MPI
// implementation of spfft::Communicator (reference: src/mpi_util/*, the MPI
// constructors in src/spfft/grid.cpp:40-45 and the *_fortran shims at
// grid.cpp:119-133, 278-290, transform.cpp:386-397).
//
// MPI is the control plane and the host data plane (MPI_Alltoallv on host
// buffers); GPU grids bootstrap RCCL through allgather() and move data over
// xGMI, never through MPI.
#include <mpi.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <memory>
#include <mutex>
#include <numeric>
#include <vector>

#include "spfft/communicator.hpp"
#include "spfft/exceptions.hpp"
#include "spfft/grid.h"
#include "spfft/grid.hpp"
#include "spfft/grid_float.h"
#include "spfft/grid_float.hpp"
#include "spfft/transform.h"
#include "spfft/transform.hpp"
#include "spfft/transform_float.h"
#include "spfft/transform_float.hpp"

namespace spfft {
namespace {

inline void mpi_check(int status) {
  if (status != MPI_SUCCESS) throw MPIError();
}

bool mpi_finalized() {
  int f = 0;
  MPI_Finalized(&f);
  return f != 0;
}

// Ordering domain of a user communicator (Communicator::channel_domain): a
// process-unique id cached on the communicator as an MPI attribute, so every
// grid built from the same communicator gets the same id, and a communicator
// created after another was freed (even under a recycled handle) a new one.
// Guarded: grids may be built concurrently by threads (MPI_THREAD_MULTIPLE).
unsigned long long domain_of(MPI_Comm comm) {
  static std::mutex m;
  static int keyval = MPI_KEYVAL_INVALID;
  static unsigned long long next = 0;
  std::lock_guard<std::mutex> lock(m);
  if (keyval == MPI_KEYVAL_INVALID)
    mpi_check(MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, MPI_COMM_NULL_DELETE_FN, &keyval, nullptr));
  void* v = nullptr;
  int found = 0;
  mpi_check(MPI_Comm_get_attr(comm, keyval, &v, &found));
  if (found) return static_cast<unsigned long long>(reinterpret_cast<std::uintptr_t>(v));
  const unsigned long long id = ++next;
  mpi_check(MPI_Comm_set_attr(comm, keyval, reinterpret_cast<void*>(static_cast<std::uintptr_t>(id))));
  return id;
}

}  // namespace

class MpiCommunicator : public Communicator {
public:
  // Duplicates `comm` (private message space per grid, reference
  // mpi_communicator_handle.hpp:48-66).
  explicit MpiCommunicator(MPI_Comm comm) : MpiCommunicator(comm, 0) {}
  // `domain` 0: the ordering domain of the user communicator `comm`
  MpiCommunicator(MPI_Comm comm, unsigned long long domain) {
    int init = 0;
    MPI_Initialized(&init);
    if (!init) throw MPISupportError();
    domain_ = domain ? domain : domain_of(comm);
    mpi_check(MPI_Comm_dup(comm, &comm_));
    mpi_check(MPI_Comm_rank(comm_, &rank_));
    mpi_check(MPI_Comm_size(comm_, &size_));
  }
  ~MpiCommunicator() override {
    if (comm_ != MPI_COMM_NULL && !mpi_finalized()) MPI_Comm_free(&comm_);
  }

  int rank() const override { return rank_; }
  int size() const override { return size_; }
  MPI_Comm get() const { return comm_; }

  void allgather(const void* send, void* recv, std::size_t bytes) override {
    if (bytes > static_cast<std::size_t>(INT_MAX)) throw OverflowError();
    mpi_check(MPI_Allgather(send, static_cast<int>(bytes), MPI_BYTE, recv, static_cast<int>(bytes),
                            MPI_BYTE, comm_));
  }

  // Byte counts/displacements in the largest element unit that divides all of
  // them (16, 8, 4 or 1 bytes), so that int counts reach far beyond 2 GiB.
  struct Counts {
    MPI_Datatype type = MPI_DATATYPE_NULL;
    std::vector<int> sc, sd, rc, rd;
    ~Counts() {
      if (type != MPI_DATATYPE_NULL && !mpi_finalized()) MPI_Type_free(&type);
    }
  };
  void make_counts(Counts& c, const std::size_t* sc, const std::size_t* sd, const std::size_t* rc,
                   const std::size_t* rd) const {
    std::size_t g = 0;
    for (int r = 0; r < size_; ++r) g = std::gcd(g, std::gcd(std::gcd(sc[r], sd[r]), std::gcd(rc[r], rd[r])));
    std::size_t unit = 1;
    for (std::size_t u : {std::size_t(16), std::size_t(8), std::size_t(4)}) {
      if (g % u == 0) {
        unit = u;
        break;
      }
    }
    c.sc.resize(size_);
    c.sd.resize(size_);
    c.rc.resize(size_);
    c.rd.resize(size_);
    for (int r = 0; r < size_; ++r) {
      const std::size_t v[4] = {sc[r] / unit, sd[r] / unit, rc[r] / unit, rd[r] / unit};
      for (std::size_t x : v)
        if (x > static_cast<std::size_t>(INT_MAX)) throw OverflowError();
      c.sc[r] = static_cast<int>(v[0]);
      c.sd[r] = static_cast<int>(v[1]);
      c.rc[r] = static_cast<int>(v[2]);
      c.rd[r] = static_cast<int>(v[3]);
    }
    mpi_check(MPI_Type_contiguous(static_cast<int>(unit), MPI_BYTE, &c.type));
    mpi_check(MPI_Type_commit(&c.type));
  }

  void alltoallv(const void* send, const std::size_t* sc, const std::size_t* sd, void* recv,
                 const std::size_t* rc, const std::size_t* rd) override {
    Counts c;
    make_counts(c, sc, sd, rc, rd);
    mpi_check(MPI_Alltoallv(send, c.sc.data(), c.sd.data(), c.type, recv, c.rc.data(), c.rd.data(),
                            c.type, comm_));
  }

  // MPI_Ialltoallv: the counts and the datatype live in the request until the
  // exchange completed (the MPI standard requires them until completion)
  struct Request : ExchangeRequest {
    Counts counts;
    MPI_Request req = MPI_REQUEST_NULL;
    ~Request() override {
      if (req != MPI_REQUEST_NULL && !mpi_finalized()) MPI_Wait(&req, MPI_STATUS_IGNORE);
    }
    void wait() override {
      if (req != MPI_REQUEST_NULL) mpi_check(MPI_Wait(&req, MPI_STATUS_IGNORE));
    }
  };
  std::unique_ptr<ExchangeRequest> ialltoallv(const void* send, const std::size_t* sc,
                                              const std::size_t* sd, void* recv,
                                              const std::size_t* rc,
                                              const std::size_t* rd) override {
    std::unique_ptr<Request> r(new Request());
    make_counts(r->counts, sc, sd, rc, rd);
    Counts& c = r->counts;
    mpi_check(MPI_Ialltoallv(send, c.sc.data(), c.sd.data(), c.type, recv, c.rc.data(),
                             c.rd.data(), c.type, comm_, &r->req));
    return std::unique_ptr<ExchangeRequest>(r.release());
  }

  // MPI_Alltoallw with one hvector datatype per peer (count blocks of a
  // contiguous unit type, byte strides): MPI gathers and scatters the strided
  // blocks itself, no pack buffer (reference UNBUFFERED,
  // src/transpose/transpose_mpi_unbuffered_host.cpp:66-181).
  struct WTypes {
    std::vector<MPI_Datatype> st, rt;
    std::vector<int> sc, sd, rc, rd;
    ~WTypes() {
      if (mpi_finalized()) return;
      for (auto* v : {&st, &rt})
        for (MPI_Datatype& t : *v)
          if (t != MPI_DATATYPE_NULL && t != MPI_BYTE) MPI_Type_free(&t);
    }
  };
  // The layout's byte offset is part of the datatype (an MPI_Aint struct
  // displacement), so alltoallw's int displacements stay 0 and offsets beyond
  // 2 GiB work (a slab side of more than 2 GiB per rank).
  static MPI_Datatype strided_type(const StridedLayout& l) {
    std::size_t unit = 1;
    for (std::size_t u : {std::size_t(16), std::size_t(8), std::size_t(4)})
      if (l.blockBytes % u == 0) {
        unit = u;
        break;
      }
    if (l.count > static_cast<std::size_t>(INT_MAX) || l.blockBytes / unit > static_cast<std::size_t>(INT_MAX))
      throw OverflowError();
    MPI_Datatype base = MPI_DATATYPE_NULL, vec = MPI_DATATYPE_NULL, t = MPI_DATATYPE_NULL;
    mpi_check(MPI_Type_contiguous(static_cast<int>(unit), MPI_BYTE, &base));
    mpi_check(MPI_Type_create_hvector(static_cast<int>(l.count), static_cast<int>(l.blockBytes / unit),
                                      static_cast<MPI_Aint>(l.strideBytes), base, &vec));
    int one = 1;
    MPI_Aint displ = static_cast<MPI_Aint>(l.offset);
    mpi_check(MPI_Type_create_struct(1, &one, &displ, &vec, &t));
    mpi_check(MPI_Type_free(&base));
    mpi_check(MPI_Type_free(&vec));
    mpi_check(MPI_Type_commit(&t));
    return t;
  }
  void make_wtypes(WTypes& w, const StridedLayout* sl, const StridedLayout* rl) const {
    w.st.assign(size_, MPI_BYTE);
    w.rt.assign(size_, MPI_BYTE);
    w.sc.assign(size_, 0);
    w.sd.assign(size_, 0);
    w.rc.assign(size_, 0);
    w.rd.assign(size_, 0);
    for (int r = 0; r < size_; ++r) {
      if (sl[r].count > 0 && sl[r].blockBytes > 0) {
        w.st[r] = strided_type(sl[r]);
        w.sc[r] = 1;
      }
      if (rl[r].count > 0 && rl[r].blockBytes > 0) {
        w.rt[r] = strided_type(rl[r]);
        w.rc[r] = 1;
      }
    }
  }
  void alltoallw(const void* send, const StridedLayout* sl, void* recv,
                 const StridedLayout* rl) override {
    WTypes w;
    make_wtypes(w, sl, rl);
    mpi_check(MPI_Alltoallw(send, w.sc.data(), w.sd.data(), w.st.data(), recv, w.rc.data(), w.rd.data(),
                            w.rt.data(), comm_));
  }
  struct WRequest : ExchangeRequest {
    WTypes types;
    MPI_Request req = MPI_REQUEST_NULL;
    ~WRequest() override {
      if (req != MPI_REQUEST_NULL && !mpi_finalized()) MPI_Wait(&req, MPI_STATUS_IGNORE);
    }
    void wait() override {
      if (req != MPI_REQUEST_NULL) mpi_check(MPI_Wait(&req, MPI_STATUS_IGNORE));
    }
  };
  std::unique_ptr<ExchangeRequest> ialltoallw(const void* send, const StridedLayout* sl, void* recv,
                                              const StridedLayout* rl) override {
    std::unique_ptr<WRequest> r(new WRequest());
    make_wtypes(r->types, sl, rl);
    WTypes& w = r->types;
    mpi_check(MPI_Ialltoallw(send, w.sc.data(), w.sd.data(), w.st.data(), recv, w.rc.data(), w.rd.data(),
                             w.rt.data(), comm_, &r->req));
    return std::unique_ptr<ExchangeRequest>(r.release());
  }

  void barrier() override { mpi_check(MPI_Barrier(comm_)); }

  std::shared_ptr<Communicator> duplicate() const override {
    return std::make_shared<MpiCommunicator>(comm_, domain_);
  }
  unsigned long long channel_domain() const override { return domain_; }

private:
  MPI_Comm comm_ = MPI_COMM_NULL;
  unsigned long long domain_ = 0;
  int rank_ = 0, size_ = 1;
};

namespace {
MPI_Comm comm_of(const std::shared_ptr<Communicator>& c) {
  auto* m = dynamic_cast<MpiCommunicator*>(c.get());
  if (m) return m->get();
  if (!c) return MPI_COMM_SELF;  // local grid
  throw InvalidParameterError();  // distributed over a non-MPI communicator
}
}  // namespace

// ---------------------------------------------------------------- C++ API
Grid::Grid(int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns, int maxLocalZLength,
           SpfftProcessingUnitType processingUnit, int maxNumThreads, MPI_Comm comm,
           SpfftExchangeType exchangeType)
    : Grid(maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, maxLocalZLength, processingUnit,
           maxNumThreads, std::make_shared<MpiCommunicator>(comm), exchangeType) {}

GridFloat::GridFloat(int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns,
                     int maxLocalZLength, SpfftProcessingUnitType processingUnit,
                     int maxNumThreads, MPI_Comm comm, SpfftExchangeType exchangeType)
    : GridFloat(maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, maxLocalZLength, processingUnit,
                maxNumThreads, std::make_shared<MpiCommunicator>(comm), exchangeType) {}

MPI_Comm Grid::communicator() const { return comm_of(spfft_communicator()); }
MPI_Comm GridFloat::communicator() const { return comm_of(spfft_communicator()); }
MPI_Comm Transform::communicator() const { return comm_of(spfft_communicator()); }
MPI_Comm TransformFloat::communicator() const { return comm_of(spfft_communicator()); }

}  // namespace spfft

// ------------------------------------------------------------------ C API
using namespace spfft;

namespace {
template <class F>
SpfftError guarded(F&& f) {
  try {
    f();
    return SPFFT_SUCCESS;
  } catch (const GenericError& e) {
    return e.error_code();
  } catch (...) {
    return SPFFT_UNKNOWN_ERROR;
  }
}
}  // namespace

extern "C" {

SpfftError spfft_grid_create_distributed(SpfftGrid* grid, int maxDimX, int maxDimY, int maxDimZ,
                                         int maxNumLocalZColumns, int maxLocalZLength,
                                         SpfftProcessingUnitType processingUnit, int maxNumThreads,
                                         MPI_Comm comm, SpfftExchangeType exchangeType) {
  if (!grid) return SPFFT_INVALID_PARAMETER_ERROR;
  return guarded([&] {
    *grid = new Grid(maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, maxLocalZLength,
                     processingUnit, maxNumThreads, comm, exchangeType);
  });
}

SpfftError spfft_float_grid_create_distributed(SpfftFloatGrid* grid, int maxDimX, int maxDimY,
                                               int maxDimZ, int maxNumLocalZColumns,
                                               int maxLocalZLength,
                                               SpfftProcessingUnitType processingUnit,
                                               int maxNumThreads, MPI_Comm comm,
                                               SpfftExchangeType exchangeType) {
  if (!grid) return SPFFT_INVALID_PARAMETER_ERROR;
  return guarded([&] {
    *grid = new GridFloat(maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, maxLocalZLength,
                          processingUnit, maxNumThreads, comm, exchangeType);
  });
}

SpfftError spfft_grid_communicator(SpfftGrid grid, MPI_Comm* comm) {
  if (!grid) return SPFFT_INVALID_HANDLE_ERROR;
  return guarded([&] { *comm = static_cast<Grid*>(grid)->communicator(); });
}
SpfftError spfft_float_grid_communicator(SpfftFloatGrid grid, MPI_Comm* comm) {
  if (!grid) return SPFFT_INVALID_HANDLE_ERROR;
  return guarded([&] { *comm = static_cast<GridFloat*>(grid)->communicator(); });
}
SpfftError spfft_transform_communicator(SpfftTransform t, MPI_Comm* comm) {
  if (!t) return SPFFT_INVALID_HANDLE_ERROR;
  return guarded([&] { *comm = static_cast<Transform*>(t)->communicator(); });
}
SpfftError spfft_float_transform_communicator(SpfftFloatTransform t, MPI_Comm* comm) {
  if (!t) return SPFFT_INVALID_HANDLE_ERROR;
  return guarded([&] { *comm = static_cast<TransformFloat*>(t)->communicator(); });
}

// Fortran shims: communicators as Fortran integers (MPI_Comm_f2c / c2f)
SPFFT_EXPORT SpfftError spfft_grid_create_distributed_fortran(
    SpfftGrid* grid, int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns,
    int maxLocalZLength, SpfftProcessingUnitType processingUnit, int maxNumThreads, int commFortran,
    SpfftExchangeType exchangeType) {
  return spfft_grid_create_distributed(grid, maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns,
                                       maxLocalZLength, processingUnit, maxNumThreads,
                                       MPI_Comm_f2c(commFortran), exchangeType);
}
SPFFT_EXPORT SpfftError spfft_float_grid_create_distributed_fortran(
    SpfftFloatGrid* grid, int maxDimX, int maxDimY, int maxDimZ, int maxNumLocalZColumns,
    int maxLocalZLength, SpfftProcessingUnitType processingUnit, int maxNumThreads, int commFortran,
    SpfftExchangeType exchangeType) {
  return spfft_float_grid_create_distributed(grid, maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns,
                                             maxLocalZLength, processingUnit, maxNumThreads,
                                             MPI_Comm_f2c(commFortran), exchangeType);
}
SPFFT_EXPORT SpfftError spfft_grid_communicator_fortran(SpfftGrid grid, int* commFortran) {
  MPI_Comm c;
  const SpfftError e = spfft_grid_communicator(grid, &c);
  if (e == SPFFT_SUCCESS) *commFortran = MPI_Comm_c2f(c);
  return e;
}
SPFFT_EXPORT SpfftError spfft_float_grid_communicator_fortran(SpfftFloatGrid grid,
                                                              int* commFortran) {
  MPI_Comm c;
  const SpfftError e = spfft_float_grid_communicator(grid, &c);
  if (e == SPFFT_SUCCESS) *commFortran = MPI_Comm_c2f(c);
  return e;
}
// (reference quirk fixed: the transform shim takes a transform handle)
SPFFT_EXPORT SpfftError spfft_transform_communicator_fortran(SpfftTransform t, int* commFortran) {
  MPI_Comm c;
  const SpfftError e = spfft_transform_communicator(t, &c);
  if (e == SPFFT_SUCCESS) *commFortran = MPI_Comm_c2f(c);
  return e;
}
SPFFT_EXPORT SpfftError spfft_float_transform_communicator_fortran(SpfftFloatTransform t,
                                                                   int* commFortran) {
  MPI_Comm c;
  const SpfftError e = spfft_float_transform_communicator(t, &c);
  if (e == SPFFT_SUCCESS) *commFortran = MPI_Comm_c2f(c);
  return e;
}

}  // extern "C"
