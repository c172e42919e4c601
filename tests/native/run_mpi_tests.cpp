// MPI tests (run with mpiexec -n P): distributed transforms over MPI_COMM_WORLD
// for every exchange type and several stick/plane distributions against a dense
// DFT (reference: tests/mpi_tests/test_transform.cpp, test_multi_transform.cpp).
#include <hip/hip_runtime_api.h>
#include <mpi.h>

#include <algorithm>
#include <cstdio>
#include <stdexcept>
#include <memory>
#include <numeric>

#include "spfft/spfft.h"
#include "spfft/spfft.hpp"
#include "test_util.hpp"

using namespace spfft_test;

namespace {
int g_rank = 0, g_size = 1;

// every rank generates the same global sticks and keeps those selected for it
struct Setup {
  std::vector<int> allIdx;     // global triplets, stick-major
  std::vector<int> stickOwner; // per global value: owning rank
};

// A grid and its transform, kept alive past run_case by the churn test.
struct Held {
  std::unique_ptr<spfft::Grid> grid;
  std::unique_ptr<spfft::Transform> t;
};

Held run_case(SpfftExchangeType ex, SpfftTransformType type, const std::vector<double>& stickW,
              const std::vector<double>& planeW, int nx, int ny, int nz, bool centered,
              SpfftProcessingUnitType pu) {
  std::mt19937 rng(123);
  std::uniform_real_distribution<double> u(0, 1);
  std::discrete_distribution<int> pick(stickW.begin(), stickW.end());
  const bool r2c = type == SPFFT_TRANS_R2C;
  const int nxf = r2c ? nx / 2 + 1 : nx;
  std::vector<int> idx, owner;
  for (int x = 0; x < nxf; ++x)
    for (int y = 0; y < ny; ++y) {
      const int r = pick(rng);
      if (!r2c && u(rng) > 0.8) continue;
      for (int z = 0; z < nz; ++z) {
        int t[3] = {x, y, z};
        if (centered) {
          if (!r2c && t[0] >= nx / 2 + 1) t[0] -= nx;
          if (t[1] >= ny / 2 + 1) t[1] -= ny;
          if (t[2] >= nz / 2 + 1) t[2] -= nz;
        }
        idx.insert(idx.end(), t, t + 3);
        owner.push_back(r);
      }
    }
  const int n = static_cast<int>(owner.size());
  // global values: random for C2C, spectrum of a real field for R2C
  std::vector<cd> vals(n);
  std::vector<cd> space;
  std::normal_distribution<double> g;
  if (!r2c) {
    for (auto& v : vals) v = cd(g(rng), g(rng));
    space = dense_backward(idx, vals, nx, ny, nz);
  } else {
    std::vector<cd> F(static_cast<size_t>(nx) * ny * nz);  // [x][y][z] of a real field
    for (auto& v : F) v = cd(g(rng), 0.0);
    space.resize(F.size());
    for (int x = 0; x < nx; ++x)
      for (int y = 0; y < ny; ++y)
        for (int z = 0; z < nz; ++z)
          space[(static_cast<size_t>(z) * ny + y) * nx + x] = F[(static_cast<size_t>(x) * ny + y) * nz + z];
    for (int ax = 0; ax < 3; ++ax) dft_axis(F, nx, ny, nz, ax, -1);
    for (int i = 0; i < n; ++i)
      vals[i] = F[(static_cast<size_t>(storage(nx, idx[3 * i])) * ny + storage(ny, idx[3 * i + 1])) * nz +
                  storage(nz, idx[3 * i + 2])];
    for (auto& v : space) v *= double(nx) * ny * nz;
  }
  // local part
  std::vector<int> myIdx;
  std::vector<cd> myVals;
  for (int i = 0; i < n; ++i)
    if (owner[i] == g_rank) {
      myIdx.insert(myIdx.end(), idx.begin() + 3 * i, idx.begin() + 3 * i + 3);
      myVals.push_back(vals[i]);
    }
  // planes by weight (remainder to the first rank with weight)
  std::vector<int> planes(g_size, 0);
  const double wsum = std::accumulate(planeW.begin(), planeW.end(), 0.0);
  for (int r = 0; r < g_size; ++r) planes[r] = static_cast<int>(planeW[r] / wsum * nz);
  int rest = nz - std::accumulate(planes.begin(), planes.end(), 0);
  for (int r = 0; r < g_size && rest; ++r)
    if (planeW[r] > 0) planes[r] += rest, rest = 0;
  const int myPlanes = planes[g_rank];
  int mySticks = 0;
  for (int i = 0; i < static_cast<int>(myVals.size()); ++i)
    if (i == 0 || myIdx[3 * i] != myIdx[3 * i - 3] || myIdx[3 * i + 1] != myIdx[3 * i - 2]) ++mySticks;

  Held held;
  held.grid.reset(new spfft::Grid(nx, ny, nz, std::max(1, mySticks), myPlanes, pu, 1, MPI_COMM_WORLD, ex));
  held.t.reset(new spfft::Transform(held.grid->create_transform(
      pu, type, nx, ny, nz, myPlanes, static_cast<int>(myVals.size()), SPFFT_INDEX_TRIPLETS, myIdx.data())));
  spfft::Transform& t = *held.t;
  EXPECT_EQ(t.local_z_length(), myPlanes);
  EXPECT_EQ(t.num_global_elements(), static_cast<long long>(n));
  const double tol = (ex == SPFFT_EXCH_BUFFERED_FLOAT || ex == SPFFT_EXCH_COMPACT_BUFFERED_FLOAT) ? 2e-6 : 1e-11;
  const size_t slice = static_cast<size_t>(myPlanes) * nx * ny;
  const size_t off = static_cast<size_t>(t.local_z_offset()) * nx * ny;
  for (int rep = 0; rep < 2; ++rep) {
    t.backward(reinterpret_cast<const double*>(myVals.data()), SPFFT_PU_HOST);
    const double* sd = t.space_domain_data(SPFFT_PU_HOST);
    double err = 0, ref = 1e-300;
    for (size_t i = 0; i < slice; ++i) {
      const cd got = r2c ? cd(sd[i], 0) : reinterpret_cast<const cd*>(sd)[i];
      const cd want = r2c ? cd(space[off + i].real(), 0) : space[off + i];
      err = std::max(err, std::abs(got - want));
    }
    for (const auto& v : space) ref = std::max(ref, std::abs(v));
    EXPECT_TRUE(err / ref < tol);
  }
  std::vector<cd> back(myVals.size());
  t.forward(SPFFT_PU_HOST, reinterpret_cast<double*>(back.data()), SPFFT_FULL_SCALING);
  if (!myVals.empty()) EXPECT_TRUE(max_rel(back.data(), myVals.data(), myVals.size()) < tol * 10);
  MPI_Comm c = t.communicator();
  int cs = 0;
  MPI_Comm_size(c, &cs);
  EXPECT_EQ(cs, g_size);
  return held;
}

const SpfftExchangeType kExchanges[] = {SPFFT_EXCH_DEFAULT,         SPFFT_EXCH_BUFFERED,
                                        SPFFT_EXCH_BUFFERED_FLOAT,  SPFFT_EXCH_COMPACT_BUFFERED,
                                        SPFFT_EXCH_COMPACT_BUFFERED_FLOAT, SPFFT_EXCH_UNBUFFERED};

std::vector<double> uniform() { return std::vector<double>(g_size, 1.0); }
std::vector<double> only(int r) {
  std::vector<double> w(g_size, 0.0);
  w[r] = 1.0;
  return w;
}
}  // namespace

SPFFT_TEST(mpi_c2c_uniform) {
  for (auto ex : kExchanges)
    for (bool c : {false, true}) run_case(ex, SPFFT_TRANS_C2C, uniform(), uniform(), 11, 12, 13, c, SPFFT_PU_HOST);
}
SPFFT_TEST(mpi_c2c_all_on_rank0) {
  for (auto ex : kExchanges) run_case(ex, SPFFT_TRANS_C2C, only(0), only(0), 12, 11, 10, false, SPFFT_PU_HOST);
}
SPFFT_TEST(mpi_c2c_sticks_rank0_planes_last) {
  for (auto ex : kExchanges)
    run_case(ex, SPFFT_TRANS_C2C, only(0), only(g_size - 1), 12, 13, 11, true, SPFFT_PU_HOST);
}
SPFFT_TEST(mpi_r2c_uniform) {
  for (auto ex : kExchanges) run_case(ex, SPFFT_TRANS_R2C, uniform(), uniform(), 12, 11, 13, false, SPFFT_PU_HOST);
}
SPFFT_TEST(mpi_r2c_planes_on_one_rank) {
  for (auto ex : kExchanges) run_case(ex, SPFFT_TRANS_R2C, uniform(), only(0), 11, 12, 10, true, SPFFT_PU_HOST);
}
SPFFT_TEST(mpi_gpu_c2c) {
  // rank r on device r % devices: one GPU per rank uses RCCL; ranks sharing a
  // device (the one-GPU test box) use the IPC peer-write plane
  int nd = spfft_amd_device_count();
  int ok = nd >= 1 ? 1 : 0, all = 0;
  MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
  if (!all) {
    if (g_rank == 0) std::printf("SKIP mpi_gpu_c2c: no GPU on some rank\n");
    return;
  }
  if (hipSetDevice(g_rank % nd) != hipSuccess) throw std::runtime_error("hipSetDevice");
  for (auto ex : kExchanges) {
    run_case(ex, SPFFT_TRANS_C2C, uniform(), uniform(), 16, 12, 32, true, SPFFT_PU_GPU);
    run_case(ex, SPFFT_TRANS_C2C, only(0), only(g_size - 1), 12, 13, 11, false, SPFFT_PU_GPU);
  }
  run_case(SPFFT_EXCH_DEFAULT, SPFFT_TRANS_R2C, uniform(), uniform(), 12, 11, 13, false, SPFFT_PU_GPU);
}
SPFFT_TEST(mpi_gpu_churn) {
  // every exchange type and both transform types with grids re-created per
  // case and destroyed by the ranks at different times: rank (case % P) drops
  // its grid at once, the others keep theirs until two more grids exist.
  // Destroying a grid needs no peer (reference: src/memory/gpu_array.hpp:88).
  int nd = spfft_amd_device_count();
  int ok = nd >= 1 ? 1 : 0, all = 0;
  MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
  if (!all) {
    if (g_rank == 0) std::printf("SKIP mpi_gpu_churn: no GPU on some rank\n");
    return;
  }
  if (hipSetDevice(g_rank % nd) != hipSuccess) throw std::runtime_error("hipSetDevice");
  std::vector<Held> kept;
  int c = 0;
  for (auto ex : kExchanges)
    for (auto type : {SPFFT_TRANS_C2C, SPFFT_TRANS_R2C}) {
      const std::vector<double> sticks = c % 3 == 0 ? only(c % g_size) : uniform();
      const std::vector<double> planes = c % 2 == 0 ? uniform() : only(g_size - 1);
      Held h = run_case(ex, type, sticks, planes, 12 + c % 5, 10 + c % 3, 14 + c % 4, c % 2 == 1,
                        SPFFT_PU_GPU);
      if (g_rank == c % g_size) {
        kept.clear();
      } else {
        kept.push_back(std::move(h));
        if (kept.size() > 2) kept.erase(kept.begin());
      }
      ++c;
    }
}
SPFFT_TEST(mpi_alltoallw_offset_beyond_int_max) {
  // UNBUFFERED host exchange with a layout offset past 2 GiB (a slab side of
  // more than 2 GiB per rank): the offset travels in the datatype (MPI_Aint),
  // not in alltoallw's int displacements. The buffers are reserved, not
  // touched, except for the blocks moved.
  spfft::Grid grid(4, 4, 4, 16, 4, SPFFT_PU_HOST, 1, MPI_COMM_WORLD, SPFFT_EXCH_UNBUFFERED);
  auto comm = grid.spfft_communicator();
  const std::size_t base = (std::size_t(1) << 31) + 4096;  // > INT_MAX
  const std::size_t block = 64, count = 3, stride = 256;
  const std::size_t span = base + static_cast<std::size_t>(g_size) * count * stride + stride;
  std::unique_ptr<unsigned char[]> send(new unsigned char[span]), recv(new unsigned char[span]);
  std::vector<spfft::StridedLayout> sl(g_size), rl(g_size);
  for (int r = 0; r < g_size; ++r) {
    const std::size_t off = base + static_cast<std::size_t>(r) * count * stride;
    sl[r] = {off, count, block, stride};
    rl[r] = {off, count, block, stride};
    for (std::size_t c = 0; c < count; ++c)
      for (std::size_t b = 0; b < block; ++b) {
        send[off + c * stride + b] = static_cast<unsigned char>((g_rank * 31 + r * 7 + c * 3 + b) & 0xFF);
        recv[off + c * stride + b] = 0;
      }
  }
  comm->alltoallw(send.get(), sl.data(), recv.get(), rl.data());
  bool ok = true;
  for (int r = 0; r < g_size; ++r) {
    const std::size_t off = base + static_cast<std::size_t>(r) * count * stride;
    for (std::size_t c = 0; c < count; ++c)
      for (std::size_t b = 0; b < block; ++b)
        ok = ok && recv[off + c * stride + b] == static_cast<unsigned char>((r * 31 + g_rank * 7 + c * 3 + b) & 0xFF);
  }
  EXPECT_TRUE(ok);
}
SPFFT_TEST(mpi_parameter_mismatch) {
  // ranks disagree on the exchange type -> every rank gets MPIParameterMismatchError
  if (g_size < 2) return;
  expect_throw<spfft::MPIParameterMismatchError>([&] {
    spfft::Grid grid(4, 4, 4, 16, 4, SPFFT_PU_HOST, 1, MPI_COMM_WORLD,
                     g_rank == 0 ? SPFFT_EXCH_BUFFERED : SPFFT_EXCH_COMPACT_BUFFERED);
  }, "mismatch");
  // duplicate sticks across ranks
  spfft::Grid grid(4, 4, 4, 16, g_rank == 0 ? 4 : 0, SPFFT_PU_HOST, 1, MPI_COMM_WORLD,
                   SPFFT_EXCH_DEFAULT);
  int idx[3] = {1, 1, g_rank % 4};
  expect_throw<spfft::DuplicateIndicesError>([&] {
    grid.create_transform(SPFFT_PU_HOST, SPFFT_TRANS_C2C, 4, 4, 4, g_rank == 0 ? 4 : 0, 1,
                          SPFFT_INDEX_TRIPLETS, idx);
  }, "duplicate");
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  MPI_Comm_rank(MPI_COMM_WORLD, &g_rank);
  MPI_Comm_size(MPI_COMM_WORLD, &g_size);
  const int failed = spfft_test::run_all(g_rank);
  int total = 0;
  MPI_Allreduce(&failed, &total, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
  MPI_Finalize();
  return total ? 1 : 0;
}
