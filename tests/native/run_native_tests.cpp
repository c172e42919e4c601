// Native (C++ and C API) tests of SpFFT-AMD: host engine sweep against a dense
// DFT, C API error contract, multi-transform, clone, local-group distribution,
// and GPU transforms when a device is present.
#include <hip/hip_runtime_api.h>

#include <cstring>
#include <thread>

#include "spfft/spfft.h"
#include "spfft/spfft.hpp"
#include "test_util.hpp"

using namespace spfft_test;

namespace {
bool have_gpu() { return spfft_amd_device_count() > 0; }

void check_c2c(SpfftProcessingUnitType pu, int nx, int ny, int nz, bool centered, unsigned seed) {
  std::mt19937 rng(seed);
  auto idx = random_indices(rng, nx, ny, nz, 0.7, 0.7, centered);
  const int n = static_cast<int>(idx.size() / 3);
  std::normal_distribution<double> g;
  std::vector<cd> vals(n);
  for (auto& v : vals) v = cd(g(rng), g(rng));
  spfft::Grid grid(nx, ny, nz, nx * ny, pu, 2);
  auto t = grid.create_transform(pu, SPFFT_TRANS_C2C, nx, ny, nz, nz, n, SPFFT_INDEX_TRIPLETS,
                                 idx.data());
  const auto ref = dense_backward(idx, vals, nx, ny, nz);
  for (int rep = 0; rep < 2; ++rep) {  // twice: zero-fill bugs
    t.backward(reinterpret_cast<double*>(vals.data()), SPFFT_PU_HOST);
    const cd* space = reinterpret_cast<const cd*>(t.space_domain_data(SPFFT_PU_HOST));
    EXPECT_TRUE(max_rel(space, ref.data(), ref.size()) < 1e-12);
  }
  std::vector<cd> back(n);
  t.forward(SPFFT_PU_HOST, reinterpret_cast<double*>(back.data()), SPFFT_FULL_SCALING);
  EXPECT_TRUE(max_rel(back.data(), vals.data(), n) < 1e-12);
}
}  // namespace

SPFFT_TEST(host_c2c_sweep) {
  const int sizes[] = {1, 2, 11, 12, 13};
  unsigned seed = 1;
  for (int a : sizes)
    for (int b : sizes)
      for (int c : sizes)
        if ((a + 2 * b + 3 * c) % 4 == 0) {
          check_c2c(SPFFT_PU_HOST, a, b, c, false, seed++);
          check_c2c(SPFFT_PU_HOST, a, b, c, true, seed++);
        }
}

// lengths whose plans use the prime-factor composite codelets 6, 10, 12, 15, 20
SPFFT_TEST(host_composite_lengths) {
  const int dims[][3] = {{6, 10, 15}, {20, 30, 12}, {45, 60, 2}, {90, 4, 120}, {240, 3, 5},
                         {180, 7, 36}, {360, 2, 1}};
  unsigned seed = 100;
  for (const auto& d : dims) {
    const bool centred = (seed & 1) != 0;
    check_c2c(SPFFT_PU_HOST, d[0], d[1], d[2], centred, seed);
    ++seed;
  }
}

SPFFT_TEST(gpu_c2c_sweep) {
  if (!have_gpu()) return;
  const int sizes[] = {1, 2, 11, 16, 32, 100};
  unsigned seed = 7;
  for (int a : sizes)
    for (int b : sizes)
      for (int c : sizes)
        if ((a + b + c) % 3 == 0) {
          check_c2c(SPFFT_PU_GPU, a, b, c, (seed & 1) != 0, seed);
          ++seed;
        }
}

SPFFT_TEST(readme_example_c_api) {
  // 2x2x2 C2C, SPFFT_PU_HOST, through the C API (reference README example)
  const int n = 8;
  int idx[3 * n];
  double vals[2 * n];
  for (int i = 0, x = 0; x < 2; ++x)
    for (int y = 0; y < 2; ++y)
      for (int z = 0; z < 2; ++z, ++i) {
        idx[3 * i] = x, idx[3 * i + 1] = y, idx[3 * i + 2] = z;
        vals[2 * i] = i, vals[2 * i + 1] = -i;
      }
  SpfftGrid grid = nullptr;
  EXPECT_EQ(spfft_grid_create(&grid, 2, 2, 2, 4, SPFFT_PU_HOST, -1), SPFFT_SUCCESS);
  SpfftTransform t = nullptr;
  EXPECT_EQ(spfft_transform_create(&t, grid, SPFFT_PU_HOST, SPFFT_TRANS_C2C, 2, 2, 2, 2, n,
                                   SPFFT_INDEX_TRIPLETS, idx),
            SPFFT_SUCCESS);
  EXPECT_EQ(spfft_grid_destroy(grid), SPFFT_SUCCESS);  // transform keeps the grid alive
  EXPECT_EQ(spfft_transform_backward(t, vals, SPFFT_PU_HOST), SPFFT_SUCCESS);
  double* space = nullptr;
  EXPECT_EQ(spfft_transform_get_space_domain(t, SPFFT_PU_HOST, &space), SPFFT_SUCCESS);
  double out[2 * n];
  EXPECT_EQ(spfft_transform_forward(t, SPFFT_PU_HOST, out, SPFFT_FULL_SCALING), SPFFT_SUCCESS);
  for (int i = 0; i < 2 * n; ++i) EXPECT_TRUE(std::abs(out[i] - vals[i]) < 1e-13);
  int v = 0;
  long long ll = 0;
  EXPECT_EQ(spfft_transform_dim_x(t, &v), SPFFT_SUCCESS);
  EXPECT_EQ(v, 2);
  EXPECT_EQ(spfft_transform_global_size(t, &ll), SPFFT_SUCCESS);
  EXPECT_EQ(ll, 8);
  EXPECT_EQ(spfft_transform_local_slice_size(t, &v), SPFFT_SUCCESS);
  EXPECT_EQ(v, 8);
  EXPECT_EQ(spfft_transform_destroy(t), SPFFT_SUCCESS);
}

SPFFT_TEST(c_api_error_codes) {
  EXPECT_EQ(spfft_grid_destroy(nullptr), SPFFT_INVALID_HANDLE_ERROR);
  int v;
  EXPECT_EQ(spfft_transform_dim_x(nullptr, &v), SPFFT_INVALID_HANDLE_ERROR);
  SpfftGrid grid = nullptr;
  EXPECT_EQ(spfft_grid_create(&grid, 0, 2, 2, 4, SPFFT_PU_HOST, 1), SPFFT_INVALID_PARAMETER_ERROR);
  EXPECT_EQ(spfft_grid_create(&grid, 4, 4, 4, 16, SPFFT_PU_HOST, 1), SPFFT_SUCCESS);
  SpfftTransform t = nullptr;
  int bad[3] = {4, 0, 0};  // x out of range for a non-centred 4-grid
  EXPECT_EQ(spfft_transform_create(&t, grid, SPFFT_PU_HOST, SPFFT_TRANS_C2C, 4, 4, 4, 4, 1,
                                   SPFFT_INDEX_TRIPLETS, bad),
            SPFFT_INVALID_INDICES_ERROR);
  int r2cBad[3] = {3, 0, 0};  // R2C: x <= 2 for dimX 4
  EXPECT_EQ(spfft_transform_create(&t, grid, SPFFT_PU_HOST, SPFFT_TRANS_R2C, 4, 4, 4, 4, 1,
                                   SPFFT_INDEX_TRIPLETS, r2cBad),
            SPFFT_INVALID_INDICES_ERROR);
  int ok[3] = {1, 1, 1};
  EXPECT_EQ(spfft_transform_create(&t, grid, SPFFT_PU_HOST, SPFFT_TRANS_C2C, 8, 4, 4, 4, 1,
                                   SPFFT_INDEX_TRIPLETS, ok),
            SPFFT_INVALID_PARAMETER_ERROR);  // larger than the grid
  EXPECT_EQ(spfft_transform_create(&t, grid, SPFFT_PU_GPU, SPFFT_TRANS_C2C, 4, 4, 4, 4, 1,
                                   SPFFT_INDEX_TRIPLETS, ok),
            SPFFT_INVALID_PARAMETER_ERROR);  // PU not supported by the grid
  EXPECT_EQ(spfft_transform_create(&t, grid, SPFFT_PU_HOST, SPFFT_TRANS_C2C, 4, 4, 4, 3, 1,
                                   SPFFT_INDEX_TRIPLETS, ok),
            SPFFT_INVALID_PARAMETER_ERROR);  // local grid needs localZ == dimZ
  EXPECT_EQ(spfft_transform_create(&t, grid, SPFFT_PU_HOST, SPFFT_TRANS_C2C, 4, 4, 4, 4, 1,
                                   static_cast<SpfftIndexFormatType>(7), ok),
            SPFFT_INTERNAL_ERROR);
  EXPECT_EQ(spfft_transform_create(&t, grid, SPFFT_PU_HOST, SPFFT_TRANS_C2C, 4, 4, 4, 4, 1,
                                   SPFFT_INDEX_TRIPLETS, ok),
            SPFFT_SUCCESS);
  double out[2];
  EXPECT_EQ(spfft_transform_forward(t, SPFFT_PU_GPU, out, SPFFT_NO_SCALING),
            SPFFT_INVALID_PARAMETER_ERROR);  // host transform, device location
  EXPECT_EQ(spfft_transform_destroy(t), SPFFT_SUCCESS);
  EXPECT_EQ(spfft_grid_destroy(grid), SPFFT_SUCCESS);
  // exception -> code mapping (InternalError fixed, reference exceptions.hpp:174)
  EXPECT_EQ(spfft::InternalError().error_code(), SPFFT_INTERNAL_ERROR);
  EXPECT_EQ(spfft::GPUFFTError().error_code(), SPFFT_GPU_FFT_ERROR);
}

SPFFT_TEST(multi_transform_c_api_and_shared_grid) {
  // constant values (i, i); backward then unscaled forward gives (i*N, i*N)
  // (reference tests/mpi_tests/test_multi_transform.cpp)
  const int nx = 6, ny = 5, nz = 4, n = nx * ny * nz;
  std::vector<int> idx;
  for (int x = 0; x < nx; ++x)
    for (int y = 0; y < ny; ++y)
      for (int z = 0; z < nz; ++z) idx.insert(idx.end(), {x, y, z});
  spfft::Grid grid(nx, ny, nz, nx * ny, SPFFT_PU_HOST, 2);
  auto t0 = grid.create_transform(SPFFT_PU_HOST, SPFFT_TRANS_C2C, nx, ny, nz, nz, n,
                                  SPFFT_INDEX_TRIPLETS, idx.data());
  spfft::Transform ts[3] = {t0, t0.clone(), t0.clone()};
  std::vector<std::vector<cd>> data(3, std::vector<cd>(n));
  for (int i = 0; i < 3; ++i)
    for (auto& v : data[i]) v = cd(i + 1, i + 1);
  double* ptrs[3] = {reinterpret_cast<double*>(data[0].data()),
                     reinterpret_cast<double*>(data[1].data()),
                     reinterpret_cast<double*>(data[2].data())};
  SpfftProcessingUnitType locs[3] = {SPFFT_PU_HOST, SPFFT_PU_HOST, SPFFT_PU_HOST};
  SpfftScalingType sc[3] = {SPFFT_NO_SCALING, SPFFT_NO_SCALING, SPFFT_NO_SCALING};
  spfft::multi_transform_backward(3, ts, ptrs, locs);
  spfft::multi_transform_forward(3, ts, locs, ptrs, sc);
  for (int i = 0; i < 3; ++i)
    for (auto& v : data[i]) EXPECT_TRUE(std::abs(v - cd(double(i + 1) * n, double(i + 1) * n)) < 1e-8);
  // C API takes an array of handles (reference quirk at multi_transform.cpp:57 fixed)
  SpfftTransform h[2] = {new spfft::Transform(ts[0]), new spfft::Transform(ts[1])};
  EXPECT_EQ(spfft_multi_transform_backward(2, h, ptrs, locs), SPFFT_SUCCESS);
  SpfftTransform same[2] = {h[0], h[0]};
  EXPECT_EQ(spfft_multi_transform_backward(2, same, ptrs, locs), SPFFT_INVALID_PARAMETER_ERROR);
  spfft_transform_destroy(h[0]);
  spfft_transform_destroy(h[1]);
}

SPFFT_TEST(local_group_distributed_host) {
  // three in-process ranks over the local-group communicator, every exchange type
  const int nx = 12, ny = 11, nz = 10, P = 3;
  std::mt19937 rng(3);
  auto idx = random_indices(rng, nx, ny, nz, 0.8, 1.0, true);
  const int n = static_cast<int>(idx.size() / 3);
  std::normal_distribution<double> g;
  std::vector<cd> vals(n);
  for (auto& v : vals) v = cd(g(rng), g(rng));
  const auto ref = dense_backward(idx, vals, nx, ny, nz);
  // whole sticks per rank: split by stick order (indices are stick-major)
  std::vector<int> bounds = {0};
  {
    std::vector<int> starts = {0};
    for (int i = 1; i < n; ++i)
      if (idx[3 * i] != idx[3 * i - 3] || idx[3 * i + 1] != idx[3 * i - 2]) starts.push_back(i);
    for (int r = 1; r < P; ++r) bounds.push_back(starts[starts.size() * r / P]);
    bounds.push_back(n);
  }
  const int planes[P] = {4, 0, 6};  // uneven, one rank without planes
  for (SpfftExchangeType ex : {SPFFT_EXCH_DEFAULT, SPFFT_EXCH_BUFFERED, SPFFT_EXCH_BUFFERED_FLOAT,
                               SPFFT_EXCH_COMPACT_BUFFERED, SPFFT_EXCH_COMPACT_BUFFERED_FLOAT,
                               SPFFT_EXCH_UNBUFFERED}) {
    auto comms = spfft::create_local_communicators(P);
    std::vector<double> err(P, 1.0);
    std::vector<std::thread> th;
    for (int r = 0; r < P; ++r)
      th.emplace_back([&, r] {
        const int b = bounds[r], e = bounds[r + 1];
        spfft::Grid grid(nx, ny, nz, nx * ny, planes[r], SPFFT_PU_HOST, 1, comms[r], ex);
        auto t = grid.create_transform(SPFFT_PU_HOST, SPFFT_TRANS_C2C, nx, ny, nz, planes[r], e - b,
                                       SPFFT_INDEX_TRIPLETS, idx.data() + 3 * b);
        t.backward(reinterpret_cast<const double*>(vals.data() + b), SPFFT_PU_HOST);
        const cd* s = reinterpret_cast<const cd*>(t.space_domain_data(SPFFT_PU_HOST));
        const size_t off = static_cast<size_t>(t.local_z_offset()) * nx * ny;
        err[r] = planes[r] ? max_rel(s, ref.data() + off, static_cast<size_t>(planes[r]) * nx * ny)
                           : 0.0;
      });
    for (auto& x : th) x.join();
    const double tol = (ex == SPFFT_EXCH_BUFFERED_FLOAT || ex == SPFFT_EXCH_COMPACT_BUFFERED_FLOAT) ? 1e-6 : 1e-12;
    for (double e : err) EXPECT_TRUE(e < tol);
  }
}

int main() { return spfft_test::run_all() ? 1 : 0; }
