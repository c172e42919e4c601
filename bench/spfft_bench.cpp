// spfft_bench: command-line benchmark of SpFFT-AMD (C++ API).
//
// Flags are a superset of the reference benchmark program
// (reference: tests/programs/benchmark.cpp:130-156, protocol :63-96):
//   -d X Y Z        grid size (required)
//   -r R            repeats; each repeat = one backward + one forward (required)
//   -o FILE         JSON output file ("" = none)
//   -m M            number of independent transforms run together (multi-transform)
//   -s S            sparsity: sticks with x < dimXFreq*S (reference data set)
//   -t c2c|r2c      transform type
//   -e all|compact|compactFloat|buffered|bufferedFloat|unbuffered
//   -p cpu|gpu|gpu-gpu   processing unit; gpu-gpu keeps input/output on the device
// Extensions:
//   --cutoff C      spherical cutoff |k/N| <= C instead of the slab sparsity
//   --precision double|single
//   --warmup W      untimed repeats before timing (default 1, as the reference)
//   --async         GPU: every transform runs stream-ordered on a stream of its own
//                   (no host wait per call; one device synchronisation after the
//                   timed repeats) instead of the reference's synchronous calls
//   --stage-times   also time every GPU stage (a hipEvent per stage boundary;
//                   the default timer tree holds host scopes only, like the
//                   reference's rt_graph timer)
//
// With MPI (libspfft_amd_mpi present) the ranks of MPI_COMM_WORLD share the
// grid: sticks and planes are split evenly, one GPU per rank (rank % devices).
// Metric: transforms/s = 2 * repeats * M / elapsed (elapsed = max over ranks).
#include <hip/hip_runtime.h>
#ifdef SPFFT_BENCH_MPI
#include <mpi.h>
#endif

#include <algorithm>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <memory>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "spfft/amd.h"
#include "spfft/spfft.hpp"

namespace {

struct Options {
  int dims[3] = {0, 0, 0};
  int repeats = -1;
  int warmup = 1;
  bool stageTimes = false;
  bool async = false;
  int numTransforms = 1;
  double sparsity = 1.0;
  double cutoff = -1.0;
  bool outputSet = false;
  std::string output;
  std::string type = "c2c";
  std::string exchange;
  std::string proc;
  bool single = false;
};

[[noreturn]] void usage(const char* msg) {
  std::fprintf(stderr,
               "error: %s\nusage: spfft_bench -d X Y Z -r R -o FILE -e EXCH -p cpu|gpu|gpu-gpu "
               "[-m M] [-s S] [-t c2c|r2c] [--cutoff C] [--precision double|single] [--warmup W] [--stage-times] [--async]\n",
               msg);
  std::exit(2);
}

Options parse(int argc, char** argv) {
  Options o;
  auto need = [&](int& i, int n) {
    if (i + n >= argc) usage((std::string("missing value for ") + argv[i]).c_str());
  };
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "-d") {
      need(i, 3);
      for (int k = 0; k < 3; ++k) o.dims[k] = std::atoi(argv[++i]);
    } else if (a == "-r") {
      need(i, 1);
      o.repeats = std::atoi(argv[++i]);
    } else if (a == "-o") {
      need(i, 1);
      o.output = argv[++i];
      o.outputSet = true;
    } else if (a == "-m") {
      need(i, 1);
      o.numTransforms = std::atoi(argv[++i]);
    } else if (a == "-s") {
      need(i, 1);
      o.sparsity = std::atof(argv[++i]);
    } else if (a == "-t") {
      need(i, 1);
      o.type = argv[++i];
    } else if (a == "-e") {
      need(i, 1);
      o.exchange = argv[++i];
    } else if (a == "-p") {
      need(i, 1);
      o.proc = argv[++i];
    } else if (a == "--cutoff") {
      need(i, 1);
      o.cutoff = std::atof(argv[++i]);
    } else if (a == "--precision") {
      need(i, 1);
      const std::string p = argv[++i];
      if (p != "double" && p != "single") usage("precision must be double or single");
      o.single = p == "single";
    } else if (a == "--warmup") {
      need(i, 1);
      o.warmup = std::atoi(argv[++i]);
    } else if (a == "--stage-times") {
      o.stageTimes = true;
    } else if (a == "--async") {
      o.async = true;
    } else if (a == "-h" || a == "--help") {
      usage("help");
    } else {
      usage(("unknown argument " + a).c_str());
    }
  }
  if (o.dims[0] <= 0 || o.dims[1] <= 0 || o.dims[2] <= 0) usage("-d X Y Z is required");
  if (o.repeats < 0) usage("-r is required");
  if (!o.outputSet) usage("-o is required");
  if (o.exchange.empty()) usage("-e is required");
  if (o.proc != "cpu" && o.proc != "gpu" && o.proc != "gpu-gpu") usage("-p cpu|gpu|gpu-gpu");
  if (o.type != "c2c" && o.type != "r2c") usage("-t c2c|r2c");
  if (o.numTransforms < 1) usage("-m must be >= 1");
  return o;
}

int centered(int i, int n) { return i <= n / 2 ? i : i - n; }

// Global stick list (centred x, y) in storage-key order and the z values of each stick.
struct Stick {
  int x, y;
  std::vector<int> z;
};

std::vector<Stick> make_sticks(const Options& o, bool r2c) {
  const int X = o.dims[0], Y = o.dims[1], Z = o.dims[2];
  std::vector<Stick> sticks;
  if (o.cutoff > 0) {
    // spherical cutoff, same set as spfft_amd.utils.indices.sphere_indices
    const double c2 = o.cutoff * o.cutoff + 1e-12;
    for (int xs = 0; xs < (r2c ? X / 2 + 1 : X); ++xs) {
      const int x = r2c ? xs : centered(xs, X);
      for (int ys = 0; ys < Y; ++ys) {
        const int y = centered(ys, Y);
        const double rr = double(x) * x / (double(X) * X) + double(y) * y / (double(Y) * Y);
        if (rr > c2) continue;
        Stick s{x, y, {}};
        for (int zs = 0; zs < Z; ++zs) {
          const int z = centered(zs, Z);
          if (double(z) * z / (double(Z) * Z) <= c2 - rr) s.z.push_back(z);
        }
        sticks.push_back(std::move(s));
      }
    }
  } else {
    // reference data set: full sticks for x < dimXFreq * sparsity (benchmark.cpp:172-205)
    const int xFreq = r2c ? X / 2 + 1 : X;
    const int yFreq = r2c ? Y / 2 + 1 : Y;
    for (int x = 0; x < xFreq * o.sparsity; ++x) {
      for (int y = 0; y < (x == 0 ? yFreq : Y); ++y) {
        Stick s{x, y, {}};
        for (int z = 0; z < Z; ++z) s.z.push_back(z);
        sticks.push_back(std::move(s));
      }
    }
  }
  auto key = [&](const Stick& s) {
    return static_cast<long long>(s.x < 0 ? s.x + X : s.x) * Y + (s.y < 0 ? s.y + Y : s.y);
  };
  std::stable_sort(sticks.begin(), sticks.end(),
                   [&](const Stick& a, const Stick& b) { return key(a) < key(b); });
  return sticks;
}

SpfftExchangeType exchange_of(const std::string& e) {
  if (e == "compact") return SPFFT_EXCH_COMPACT_BUFFERED;
  if (e == "compactFloat") return SPFFT_EXCH_COMPACT_BUFFERED_FLOAT;
  if (e == "buffered") return SPFFT_EXCH_BUFFERED;
  if (e == "bufferedFloat") return SPFFT_EXCH_BUFFERED_FLOAT;
  if (e == "unbuffered") return SPFFT_EXCH_UNBUFFERED;
  usage(("unknown exchange type " + e).c_str());
}

struct Env {
  int rank = 0, size = 1;
  double max_over_ranks(double v) const {
#ifdef SPFFT_BENCH_MPI
    double r = v;
    MPI_Allreduce(&v, &r, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    return r;
#else
    return v;
#endif
  }
  void barrier() const {
#ifdef SPFFT_BENCH_MPI
    MPI_Barrier(MPI_COMM_WORLD);
#endif
  }
};

template <typename GridT>
GridT make_grid(const Env& env, const Options& o, int maxSticks, int localZ,
                SpfftProcessingUnitType pu, SpfftExchangeType exch) {
#ifdef SPFFT_BENCH_MPI
  if (env.size > 1)
    return GridT(o.dims[0], o.dims[1], o.dims[2], maxSticks, localZ, pu, -1, MPI_COMM_WORLD, exch);
#endif
  (void)env;
  (void)localZ;
  (void)exch;
  return GridT(o.dims[0], o.dims[1], o.dims[2], maxSticks, pu, -1);
}

struct Result {
  std::string exchange;
  double seconds = 0;
  double transformsPerSecond = 0;
};

template <typename T, typename GridT, typename TransformT, typename MultiF, typename MultiB>
Result run(const Env& env, const Options& o, const std::vector<int>& triplets, int numLocalSticks,
           int localZ, SpfftExchangeType exch, const std::string& exchName, MultiF multiForward,
           MultiB multiBackward) {
  const bool r2c = o.type == "r2c";
  const SpfftProcessingUnitType pu = o.proc == "cpu" ? SPFFT_PU_HOST : SPFFT_PU_GPU;
  const SpfftProcessingUnitType loc = o.proc == "gpu-gpu" ? SPFFT_PU_GPU : SPFFT_PU_HOST;
  const int n = static_cast<int>(triplets.size() / 3);
  const int M = o.numTransforms;

  std::vector<TransformT> transforms;
  for (int m = 0; m < M; ++m) {
    GridT grid = make_grid<GridT>(env, o, std::max(numLocalSticks, 1), localZ, pu, exch);
    transforms.push_back(grid.create_transform(pu, r2c ? SPFFT_TRANS_R2C : SPFFT_TRANS_C2C,
                                               o.dims[0], o.dims[1], o.dims[2], localZ, n,
                                               SPFFT_INDEX_TRIPLETS, triplets.data()));
  }
  // random frequency values (host, and on the device for gpu-gpu)
  std::mt19937 gen(1234 + env.rank);
  std::uniform_real_distribution<T> dist(-1, 1);
  std::vector<std::vector<T>> host(M, std::vector<T>(2 * static_cast<std::size_t>(n)));
  for (auto& h : host)
    for (auto& v : h) v = dist(gen);
  std::vector<T*> ptr(M);
  std::vector<void*> devBufs;
  for (int m = 0; m < M; ++m) {
    if (loc == SPFFT_PU_GPU) {
      void* d = nullptr;
      if (hipMalloc(&d, sizeof(T) * std::max<std::size_t>(1, host[m].size())) != hipSuccess)
        throw std::runtime_error("hipMalloc failed");
      if (n) (void)hipMemcpy(d, host[m].data(), sizeof(T) * host[m].size(), hipMemcpyHostToDevice);
      devBufs.push_back(d);
      ptr[m] = static_cast<T*>(d);
    } else {
      ptr[m] = host[m].data();
    }
  }
  std::vector<hipStream_t> streams;
  if (o.async && pu == SPFFT_PU_GPU) {
    for (int m = 0; m < M; ++m) {
      hipStream_t st = nullptr;
      if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess)
        throw std::runtime_error("hipStreamCreate failed");
      streams.push_back(st);
      transforms[m].set_execution_stream(st, false);
    }
  }
  std::vector<SpfftProcessingUnitType> locs(M, loc);
  std::vector<SpfftScalingType> scal(M, SPFFT_NO_SCALING);
  auto once = [&]() {
    if (M == 1) {
      transforms[0].backward(ptr[0], loc);
      transforms[0].forward(loc, ptr[0], SPFFT_NO_SCALING);
    } else {
      multiBackward(M, transforms.data(), ptr.data(), locs.data());
      multiForward(M, transforms.data(), locs.data(), ptr.data(), scal.data());
    }
  };
  for (int w = 0; w < o.warmup; ++w) once();
  if (pu == SPFFT_PU_GPU) (void)hipDeviceSynchronize();
  env.barrier();
  (void)spfft_amd_timing_reset();
  const auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < o.repeats; ++r) once();
  if (pu == SPFFT_PU_GPU) (void)hipDeviceSynchronize();
  const auto t1 = std::chrono::steady_clock::now();
  env.barrier();
  for (void* d : devBufs) (void)hipFree(d);
  for (auto& t : transforms) t.synchronize();
  transforms.clear();
  for (hipStream_t st : streams) (void)hipStreamDestroy(st);
  Result res;
  res.exchange = exchName;
  res.seconds = env.max_over_ranks(std::chrono::duration<double>(t1 - t0).count());
  res.transformsPerSecond = res.seconds > 0 ? 2.0 * o.repeats * M / res.seconds : 0.0;
  return res;
}

std::string timing_json() {
  std::size_t need = 0;
  (void)spfft_amd_timing_json(nullptr, 0, &need);
  std::string s(need + 1, '\0');
  (void)spfft_amd_timing_json(&s[0], s.size(), &need);
  s.resize(std::strlen(s.c_str()));
  return s.empty() ? "null" : s;
}

}  // namespace

int main(int argc, char** argv) {
  Env env;
#ifdef SPFFT_BENCH_MPI
  int provided = 0;
  MPI_Init_thread(&argc, &argv, MPI_THREAD_FUNNELED, &provided);
  MPI_Comm_rank(MPI_COMM_WORLD, &env.rank);
  MPI_Comm_size(MPI_COMM_WORLD, &env.size);
#endif
  int rc = 0;
  try {
    const Options o = parse(argc, argv);
    const bool r2c = o.type == "r2c";
    if (o.proc != "cpu") {
      int ndev = 0;
      if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        throw std::runtime_error("no GPU visible for -p " + o.proc);
      (void)hipSetDevice(env.rank % ndev);
    }
    (void)spfft_amd_timing_enable(o.stageTimes ? 2 : 1);
    // even stick / plane split over ranks (reference: benchmark.cpp:166-198)
    const std::vector<Stick> sticks = make_sticks(o, r2c);
    const int S = static_cast<int>(sticks.size());
    const int mySticks = S / env.size + (env.rank < S % env.size ? 1 : 0);
    const int first = (S / env.size) * env.rank + std::min(env.rank, S % env.size);
    const int Z = o.dims[2];
    const int localZ = Z / env.size + (env.rank < Z % env.size ? 1 : 0);
    std::vector<int> triplets;
    long long globalValues = 0;
    for (const Stick& s : sticks) globalValues += static_cast<long long>(s.z.size());
    for (int i = first; i < first + mySticks; ++i)
      for (int z : sticks[i].z) {
        triplets.push_back(sticks[i].x);
        triplets.push_back(sticks[i].y);
        triplets.push_back(z);
      }
    std::vector<std::pair<SpfftExchangeType, std::string>> exchanges;
    if (o.exchange == "all") {
      exchanges = {{SPFFT_EXCH_BUFFERED, "buffered"},
                   {SPFFT_EXCH_COMPACT_BUFFERED, "compact"},
                   {SPFFT_EXCH_UNBUFFERED, "unbuffered"}};
    } else {
      exchanges = {{exchange_of(o.exchange), o.exchange}};
    }
    if (env.rank == 0) {
      std::printf("ranks: %d  grid: %d x %d x %d  type: %s  precision: %s  proc: %s\n", env.size,
                  o.dims[0], o.dims[1], o.dims[2], o.type.c_str(), o.single ? "single" : "double",
                  o.proc.c_str());
      std::printf("sticks: %d  values: %lld  data set: %s\n", S, globalValues,
                  o.cutoff > 0 ? ("spherical cutoff " + std::to_string(o.cutoff)).c_str()
                               : ("sparsity " + std::to_string(o.sparsity)).c_str());
    }
    std::vector<Result> results;
    for (const auto& e : exchanges) {
      Result r;
      if (o.single)
        r = run<float, spfft::GridFloat, spfft::TransformFloat>(
            env, o, triplets, mySticks, localZ, e.first, e.second,
            [](int k, spfft::TransformFloat* t, SpfftProcessingUnitType* l, float** out,
               SpfftScalingType* s) { spfft::multi_transform_forward(k, t, l, out, s); },
            [](int k, spfft::TransformFloat* t, float** in, SpfftProcessingUnitType* l) {
              spfft::multi_transform_backward(k, t, in, l);
            });
      else
        r = run<double, spfft::Grid, spfft::Transform>(
            env, o, triplets, mySticks, localZ, e.first, e.second,
            [](int k, spfft::Transform* t, SpfftProcessingUnitType* l, double** out,
               SpfftScalingType* s) { spfft::multi_transform_forward(k, t, l, out, s); },
            [](int k, spfft::Transform* t, double** in, SpfftProcessingUnitType* l) {
              spfft::multi_transform_backward(k, t, in, l);
            });
      results.push_back(r);
      if (env.rank == 0)
        std::printf("%-14s %10.3f ms/repeat  %12.1f transforms/s\n", r.exchange.c_str(),
                    1e3 * r.seconds / std::max(o.repeats, 1), r.transformsPerSecond);
    }
    if (env.rank == 0 && !o.output.empty()) {
      std::ostringstream j;
      const std::time_t now = std::time(nullptr);
      std::string when = std::ctime(&now);
      if (!when.empty()) when.pop_back();
      j << "{\n  \"parameters\": {\"proc\": \"" << o.proc << "\", \"data_on_gpu\": "
        << (o.proc == "gpu-gpu" ? "true" : "false") << ", \"gpu_direct\": true, \"num_ranks\": "
        << env.size << ", \"dim_x\": " << o.dims[0] << ", \"dim_y\": " << o.dims[1]
        << ", \"dim_z\": " << o.dims[2] << ", \"exchange_type\": \"" << o.exchange
        << "\", \"num_repeats\": " << o.repeats << ", \"num_transforms\": " << o.numTransforms
        << ", \"transform_type\": \"" << o.type << "\", \"precision\": \""
        << (o.single ? "single" : "double") << "\", \"sparsity\": " << o.sparsity
        << ", \"cutoff\": " << o.cutoff << ", \"num_values\": " << globalValues
        << ", \"calls\": \"" << (o.async ? "async" : "synchronous") << "\""
        << ", \"time\": \"" << when << "\"},\n  \"results\": [";
      for (std::size_t i = 0; i < results.size(); ++i)
        j << (i ? ", " : "") << "{\"exchange\": \"" << results[i].exchange
          << "\", \"seconds\": " << results[i].seconds
          << ", \"transforms_per_second\": " << results[i].transformsPerSecond << "}";
      j << "],\n  \"timings\": " << timing_json() << "\n}\n";
      std::ofstream f(o.output);
      f << j.str();
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "spfft_bench: %s (%s)\n", e.what(), spfft_amd_last_error_message());
    rc = 1;
  }
#ifdef SPFFT_BENCH_MPI
  MPI_Finalize();
#endif
  return rc;
}
