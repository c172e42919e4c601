// Fused single-GPU path (P = 1, C2C): two kernels per direction instead of three.
//
//   backward:  z_backward_pm   values -> plane-major sticks [z][stick]
//              yx_backward     sticks -> y-FFT -> L2 scratch -> x-FFT -> space
//   forward:   xy_forward      space -> x-FFT -> L2 scratch -> y-FFT -> sticks
//              z_forward_pm    sticks -> values
//
// The [z][column][y] intermediate of the three-kernel path (2 x 262 MB of HBM
// traffic per direction at 256^3) is replaced by a per-XCD ring of plane
// buffers that stays in that XCD's 4 MB L2. yx/xy are persistent kernels: every
// workgroup reads its XCD id (HW_REG_XCC_ID), the workgroups of one XCD own a
// static share of the planes and split each plane into column tasks (y-FFT)
// and row tasks (x-FFT), ordered Y(0) Y(1) X(0) Y(2) X(1) ... and dealt round-
// robin, so every dependency points to a task handed out earlier (no deadlock
// while the grid is resident; grid = CUs x workgroups-per-CU). Hand-off inside
// one XCD: producer stores (non-temporal: the line stays in the XCD's L2),
// every wave drains with s_waitcnt vmcnt(0), workgroup barrier, one counter add;
// the consumer polls the counter and reads with non-temporal loads, which are
// served by L2 (they bypass the CU's L1). Every spin is bounded: on timeout a
// host-visible error word is set and the kernel runs to completion.
#include "kernels/stage_kernels.hpp"
#include "kernels/fused_stage.hpp"

namespace spfft {
namespace dev {
namespace {

constexpr int kCtrlReg = 0;       // [8] workgroups registered per XCD
constexpr int kCtrlArrived = 8;   // grid registration barrier
constexpr int kCtrlCounters = 16; // [8][2][kMaxRing] per-XCD ring counters (y done, x done)

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7u;
}

__device__ __forceinline__ unsigned poll(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// thread 0 waits until *p >= target (bounded); the whole workgroup then proceeds
__device__ __forceinline__ void wait_counter(const unsigned* p, unsigned target, unsigned* failure,
                                             long long timeout, int debug = 0) {
  if (threadIdx.x == 0 && !(debug & 1)) {
    if (poll(p) < target) {
      const long long t0 = wall_clock64();
      while (poll(p) < target) {
        if (wall_clock64() - t0 > timeout) {
          __hip_atomic_fetch_or(failure, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
  __syncthreads();
}

// every wave's stores have reached L2, then one add publishes the task
__device__ __forceinline__ void signal_counter(unsigned* p) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Registration: XCD id, slot within the XCD, and (after a grid-wide barrier)
// the number of workgroups on every XCD. Planes go round-robin over the XCDs
// that have workgroups. Results in LDS-broadcast ints.
struct Team {
  int xcc, slot, members, xi, numXcd;
};

__device__ Team register_team(unsigned* ctrl, unsigned* failure, long long timeout, int* sh) {
  if (threadIdx.x == 0) {
    const unsigned x = xcc_id();
    const unsigned slot = __hip_atomic_fetch_add(&ctrl[kCtrlReg + x], 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&ctrl[kCtrlArrived], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const long long t0 = wall_clock64();
    while (poll(&ctrl[kCtrlArrived]) < gridDim.x) {
      if (wall_clock64() - t0 > timeout) {
        __hip_atomic_fetch_or(failure, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    int xi = 0, m = 0;
    for (int q = 0; q < 8; ++q) {
      const unsigned c = poll(&ctrl[kCtrlReg + q]);
      if (c > 0) {
        if (q == static_cast<int>(x)) xi = m;
        ++m;
      }
    }
    sh[0] = static_cast<int>(x);
    sh[1] = static_cast<int>(slot);
    sh[2] = static_cast<int>(poll(&ctrl[kCtrlReg + x]));
    sh[3] = xi;
    sh[4] = m;
  }
  __syncthreads();
  Team t{sh[0], sh[1], sh[2], sh[3], sh[4]};
  __syncthreads();
  return t;
}

// Task tau of one XCD's sequence with lag L: steps s = 0 .. Pn+L-1, step s holds
// the first-phase tasks of plane s (if s < Pn) followed by the second-phase
// tasks of plane s-L (if s >= L). A second-phase task of plane i is handed out
// L steps after plane i's first phase; a first-phase task of plane i reuses the
// ring buffer of plane i-R, whose second phase was handed out at step i-R+L < i
// (R > L), so every dependency points to an earlier task.
struct Task {
  bool first;
  int plane;  // local plane index i (global plane = xi + numXcd * i)
  int part;   // column group / row group
};
__device__ __forceinline__ Task decode(long long tau, int Pn, int L, int nFirst, int nSecond) {
  const int lead = min(L, Pn);
  const long long A = static_cast<long long>(lead) * nFirst;
  if (tau < A) return Task{true, static_cast<int>(tau / nFirst), static_cast<int>(tau % nFirst)};
  tau -= A;
  const int per = nFirst + nSecond;
  const long long Bn = static_cast<long long>(max(0, Pn - L)) * per;
  if (tau < Bn) {
    const int s = L + static_cast<int>(tau / per);
    const int k = static_cast<int>(tau % per);
    if (k < nFirst) return Task{true, s, k};
    return Task{false, s - L, k - nFirst};
  }
  tau -= Bn;
  const int s = max(L, Pn) + static_cast<int>(tau / nSecond);
  return Task{false, s - L, static_cast<int>(tau % nSecond)};
}

}  // namespace

// ------------------------------------------------------------ z stage (plane-major)
// Per-block value prefix of up to B simple sticks (desc), staged in LDS.
__device__ __forceinline__ int block_prefix(const StickDesc* d, int nl, int* pre) {
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int b = 0; b < nl; ++b) {
      pre[b] = acc;
      acc += d[b].count;
    }
    pre[nl] = acc;
  }
  __syncthreads();
  return pre[nl];
}

__device__ __forceinline__ int find_line(const int* pre, int nl, int idx) {
  int b = 0;
  while (b + 1 < nl && pre[b + 1] <= idx) ++b;
  return b;
}

__device__ __forceinline__ int desc_z(const StickDesc& q, int j) {
  return j < q.len0 ? q.z0 + j : q.z1 + (j - q.len0);
}

template <class Eng, typename T>
__global__ void __launch_bounds__(kMaxThreads)
    z_backward_pm_kernel(Eng eng, FusedArgs a, const cx<T>* __restrict__ values,
                         cx<T>* __restrict__ sticks, const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  const int B = eng.lines();
  const int n = eng.n();
  const int s0 = blockIdx.x * B;
  const int nl = min(B, a.S - s0);
  StickDesc* d = reinterpret_cast<StickDesc*>(reinterpret_cast<char*>(lds) + eng.lds_bytes());
  int* pre = reinterpret_cast<int*>(d + B);
  for (int b = threadIdx.x; b < nl; b += blockDim.x) d[b] = a.desc[s0 + b];
  zero_lds(lds, eng.input_elems());
  __syncthreads();
  const int total = block_prefix(d, nl, pre);
  // dense, coalesced value loads (lanes over the block's values), scattered into the lines
  gather_to_lds(lds, total, [&](int idx) {
    const int b = find_line(pre, nl, idx);
    return ld_values(&values[d[b].valueStart + idx - pre[b]]);
  }, [&](int idx) {
    const int b = find_line(pre, nl, idx);
    return eng.in_at(b, desc_z(d[b], idx - pre[b]));
  });
  __syncthreads();
  // line-fast lanes: consecutive lanes store consecutive sticks of one plane
  eng.lds_to_global(lds, tw, [&](int b, int pos, cx<T> v) {
    if (b < nl) st_stream(&sticks[static_cast<long long>(pos) * a.Sp + s0 + b], v);
  });
}

template <class Eng, typename T>
__global__ void __launch_bounds__(kMaxThreads)
    z_forward_pm_kernel(Eng eng, FusedArgs a, const cx<T>* __restrict__ sticks,
                        cx<T>* __restrict__ values, T scale, const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  const int B = eng.lines();
  const int s0 = blockIdx.x * B;
  const int nl = min(B, a.S - s0);
  StickDesc* d = reinterpret_cast<StickDesc*>(reinterpret_cast<char*>(lds) + eng.lds_bytes());
  int* pre = reinterpret_cast<int*>(d + B);
  for (int b = threadIdx.x; b < nl; b += blockDim.x) d[b] = a.desc[s0 + b];
  eng.global_to_lds(lds, tw, [&](int b, int pos) -> cx<T> {
    return b < nl ? ld_stream(&sticks[static_cast<long long>(pos) * a.Sp + s0 + b]) : czero<T>();
  });
  const int total = block_prefix(d, nl, pre);
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int b = find_line(pre, nl, idx);
    const int j = idx - pre[b];
    st_values(&values[d[b].valueStart + j], spfft::scale(lds[eng.out_at(b, desc_z(d[b], j))], scale));
  }
}

// --------------------------------------------------------------- fused y/x
// EY: engine of length Y (columns), EX: engine of length X (rows); both read
// their lines from LDS and (EX backward) store rows directly.
template <class EY, class EX, typename T>
__global__ void __launch_bounds__(kMaxThreads)
    yx_backward_kernel(EY ey, EX ex, FusedArgs a, const cx<T>* __restrict__ sticks,
                       cx<T>* __restrict__ space, cx<T>* __restrict__ scratch,
                       const cx<T>* __restrict__ twy, const cx<T>* __restrict__ twx) {
  SPFFT_LDS_DECL(T);
  const int ldsLines = max(ey.lds_bytes(), ex.lds_bytes());
  int* sh = reinterpret_cast<int*>(reinterpret_cast<char*>(lds) + ldsLines);
  int* xPos = sh + 8;  // column -> x position
  const Team team = register_team(a.ctrl, a.failure, a.timeout, sh);
  for (int c = threadIdx.x; c < a.ncols; c += blockDim.x) xPos[c] = a.colX[c];
  const int BY = ey.lines(), BX = ex.lines();
  const int nY = (a.ncols + BY - 1) / BY, nX = (a.Y + BX - 1) / BX;
  const int Pn = team.xi < a.Z ? (a.Z - team.xi + team.numXcd - 1) / team.numXcd : 0;
  unsigned* yDone = a.ctrl + kCtrlCounters + team.xcc * 2 * kMaxRing;
  unsigned* xDone = yDone + kMaxRing;
  const long long totalTasks = static_cast<long long>(Pn) * (nY + nX);
  cx<T>* scr0 = scratch + static_cast<long long>(team.xcc) * a.ring * a.scratchPlane;
  __syncthreads();
  for (long long tau = team.slot; tau < totalTasks; tau += team.members) {
    const Task tk = decode(tau, Pn, a.lag, nY, nX);
    const int buf = tk.plane % a.ring, use = tk.plane / a.ring;
    const int z = team.xi + team.numXcd * tk.plane;
    cx<T>* scr = scr0 + static_cast<long long>(buf) * a.scratchPlane;
    if (tk.first) {
      // columns [c0, c1) of plane z: sticks -> y-FFT -> scratch[y][c]
      if (use > 0) wait_counter(&xDone[buf], static_cast<unsigned>(nX * use), a.failure, a.timeout, a.debug);
      const int c0 = tk.part * BY, c1 = min(a.ncols, c0 + BY), nc = c1 - c0;
      zero_lds(lds, ey.input_elems());
      __syncthreads();
      const int e0 = a.colOffsets[c0], e1 = a.colOffsets[c1];
      const cx<T>* src = sticks + static_cast<long long>(z) * a.Sp;
      gather_to_lds(lds, e1 - e0, [&](int i) { return ld_stream(&src[e0 + i]); },
                    [&](int i) { return ey.in_at(a.entryCol[e0 + i] - c0, a.colY[e0 + i]); });
      __syncthreads();
      ey.lds_to_lds(lds, twy);
      for (int idx = threadIdx.x; idx < nc * a.Y; idx += blockDim.x) {
        const int y = idx / nc, c = idx - y * nc;
        st_stream(&scr[static_cast<long long>(y) * a.scratchStride + c0 + c], lds[ey.out_at(c, y)]);
      }
      signal_counter(&yDone[buf]);
    } else {
      // rows [y0, y1) of plane z: scratch -> x-FFT -> space rows
      wait_counter(&yDone[buf], static_cast<unsigned>(nY * (use + 1)), a.failure, a.timeout, a.debug);
      const int y0 = tk.part * BX, y1 = min(a.Y, y0 + BX), ny = y1 - y0;
      zero_lds(lds, ex.input_elems());
      __syncthreads();
      gather_to_lds(lds, ny * a.ncols, [&](int i) {
        const int r = i / a.ncols, c = i - r * a.ncols;
        return ld_stream(&scr[static_cast<long long>(y0 + r) * a.scratchStride + c]);
      }, [&](int i) {
        const int r = i / a.ncols, c = i - r * a.ncols;
        return ex.in_at(r, xPos[c]);
      });
      __syncthreads();
      cx<T>* dst = space + (static_cast<long long>(z) * a.Y + y0) * a.X;
      ex.lds_to_global(lds, twx, [&](int b, int pos, cx<T> v) {
        if (b < ny) st_stream(&dst[static_cast<long long>(b) * a.X + pos], v);
      });
      signal_counter(&xDone[buf]);
    }
  }
}

template <class EY, class EX, typename T>
__global__ void __launch_bounds__(kMaxThreads)
    xy_forward_kernel(EY ey, EX ex, FusedArgs a, const cx<T>* __restrict__ space,
                      cx<T>* __restrict__ sticks, cx<T>* __restrict__ scratch,
                      const cx<T>* __restrict__ twy, const cx<T>* __restrict__ twx) {
  SPFFT_LDS_DECL(T);
  const int ldsLines = max(ey.lds_bytes(), ex.lds_bytes());
  int* sh = reinterpret_cast<int*>(reinterpret_cast<char*>(lds) + ldsLines);
  int* xPos = sh + 8;
  const Team team = register_team(a.ctrl, a.failure, a.timeout, sh);
  for (int c = threadIdx.x; c < a.ncols; c += blockDim.x) xPos[c] = a.colX[c];
  const int BY = ey.lines(), BX = ex.lines();
  const int nY = (a.ncols + BY - 1) / BY, nX = (a.Y + BX - 1) / BX;
  const int Pn = team.xi < a.Z ? (a.Z - team.xi + team.numXcd - 1) / team.numXcd : 0;
  unsigned* xDone = a.ctrl + kCtrlCounters + team.xcc * 2 * kMaxRing;
  unsigned* yDone = xDone + kMaxRing;
  const long long totalTasks = static_cast<long long>(Pn) * (nY + nX);
  cx<T>* scr0 = scratch + static_cast<long long>(team.xcc) * a.ring * a.scratchPlane;
  __syncthreads();
  for (long long tau = team.slot; tau < totalTasks; tau += team.members) {
    // order X(0) X(1) Y(0) X(2) Y(1) ...: "first" phase = rows here
    const Task tk = decode(tau, Pn, a.lag, nX, nY);
    const bool isX = tk.first;
    const int buf = tk.plane % a.ring, use = tk.plane / a.ring;
    const int z = team.xi + team.numXcd * tk.plane;
    cx<T>* scr = scr0 + static_cast<long long>(buf) * a.scratchPlane;
    if (isX) {
      // rows [y0, y1): space -> x-FFT -> scratch[y][c] at the columns holding sticks
      if (use > 0) wait_counter(&yDone[buf], static_cast<unsigned>(nY * use), a.failure, a.timeout, a.debug);
      const int y0 = tk.part * BX, y1 = min(a.Y, y0 + BX), ny = y1 - y0;
      const cx<T>* rows = space + (static_cast<long long>(z) * a.Y + y0) * a.X;
      stage_rows(ex, lds, ny, a.X, [&](int b, int pos) {
        return ld_stream(&rows[static_cast<long long>(b) * a.X + pos]);
      });
      ex.lds_to_lds(lds, twx);
      for (int idx = threadIdx.x; idx < ny * a.ncols; idx += blockDim.x) {
        const int r = idx / a.ncols, c = idx - r * a.ncols;
        st_stream(&scr[static_cast<long long>(y0 + r) * a.scratchStride + c], lds[ex.out_at(r, xPos[c])]);
      }
      signal_counter(&xDone[buf]);
    } else {
      // columns [c0, c1): scratch -> y-FFT -> plane-major sticks
      wait_counter(&xDone[buf], static_cast<unsigned>(nX * (use + 1)), a.failure, a.timeout, a.debug);
      const int c0 = tk.part * BY, c1 = min(a.ncols, c0 + BY), nc = c1 - c0;
      gather_to_lds(lds, nc * a.Y, [&](int i) {
        const int y = i / nc, c = i - y * nc;
        return ld_stream(&scr[static_cast<long long>(y) * a.scratchStride + c0 + c]);
      }, [&](int i) {
        const int y = i / nc, c = i - y * nc;
        return ey.in_at(c, y);
      });
      __syncthreads();
      ey.lds_to_lds(lds, twy);
      const int e0 = a.colOffsets[c0], e1 = a.colOffsets[c1];
      cx<T>* dst = sticks + static_cast<long long>(z) * a.Sp;
      for (int i = threadIdx.x; i < e1 - e0; i += blockDim.x)
        st_stream(&dst[e0 + i], lds[ey.out_at(a.entryCol[e0 + i] - c0, a.colY[e0 + i])]);
      signal_counter(&yDone[buf]);
    }
  }
}

// ------------------------------------------------------------------ launchers
namespace {
template <typename T, int S, class F>
bool with_ct(int n, F&& f) {
  switch (n) {
#define SPFFT_FUSED_CASE(NN)              \
  case NN:                                \
    f(CtEng<T, NN, S, false>{});          \
    return true;
    SPFFT_FUSED_CASE(64)
    SPFFT_FUSED_CASE(128)
    SPFFT_FUSED_CASE(256)
    SPFFT_FUSED_CASE(512)
#undef SPFFT_FUSED_CASE
    default: return false;
  }
}
template <typename T, int S, class F>
bool with_ct_lf(int n, F&& f) {
  switch (n) {
#define SPFFT_FUSED_CASE(NN)             \
  case NN:                               \
    f(CtEng<T, NN, S, true>{});          \
    return true;
    SPFFT_FUSED_CASE(64)
    SPFFT_FUSED_CASE(128)
    SPFFT_FUSED_CASE(256)
    SPFFT_FUSED_CASE(512)
#undef SPFFT_FUSED_CASE
    default: return false;
  }
}
}  // namespace

bool fused_supported(int x, int y, int z) {
  // (the fused kernels are built for workgroups of at most kMaxThreads; the
  // wide 512-thread shapes of N = 512 are excluded)
  auto ok = [](int n) {
    return n == 64 || n == 128 || n == 256 ||
           (n == 512 && !SPFFT_WIDE_F512 && !SPFFT_WIDE_D512);
  };
  return ok(x) && ok(y) && ok(z);
}

template <typename T>
std::size_t fused_lds_bytes(int x, int y) {
  std::size_t l = 0;
  with_ct<T, +1>(y, [&](auto ey) {
    with_ct<T, +1>(x, [&](auto ex) {
      l = std::max(decltype(ey)::h_lds(), decltype(ex)::h_lds());
    });
  });
  return l;
}

template <typename T>
int fused_threads(int x, int y) {
  int t = 0;
  with_ct<T, +1>(y, [&](auto ey) {
    with_ct<T, +1>(x, [&](auto ex) {
      t = std::max(decltype(ey)::h_threads(), decltype(ex)::h_threads());
    });
  });
  return t;
}

template <typename T>
void launch_z_backward_pm(const FusedArgs& a, const cx<T>* values, cx<T>* sticks, const cx<T>* tw,
                          hipStream_t stream) {
  if (a.S <= 0) return;
  with_ct_lf<T, +1>(a.Z, [&](auto eng) {
    using E = decltype(eng);
    auto k = z_backward_pm_kernel<E, T>;
    const std::size_t lds = E::h_lds() + E::h_lines() * (sizeof(StickDesc) + sizeof(int)) + 16;
    prepare_kernel(k, lds);
    hipLaunchKernelGGL(k, dim3(ceil_div(a.S, E::h_lines())), dim3(E::h_threads()), lds, stream, eng,
                       a, values, sticks, tw);
    gpu_check_launch("z_backward_pm", stream);
  });
}

template <typename T>
void launch_z_forward_pm(const FusedArgs& a, const cx<T>* sticks, cx<T>* values, T scale,
                         const cx<T>* tw, hipStream_t stream) {
  if (a.S <= 0) return;
  with_ct_lf<T, -1>(a.Z, [&](auto eng) {
    using E = decltype(eng);
    auto k = z_forward_pm_kernel<E, T>;
    const std::size_t lds = E::h_lds() + E::h_lines() * (sizeof(StickDesc) + sizeof(int)) + 16;
    prepare_kernel(k, lds);
    hipLaunchKernelGGL(k, dim3(ceil_div(a.S, E::h_lines())), dim3(E::h_threads()), lds, stream, eng,
                       a, sticks, values, scale, tw);
    gpu_check_launch("z_forward_pm", stream);
  });
}

template <typename T>
void launch_yx_backward(const FusedArgs& a, int grid, const cx<T>* sticks, cx<T>* space,
                        cx<T>* scratch, const cx<T>* twy, const cx<T>* twx, hipStream_t stream) {
  with_ct<T, +1>(a.Y, [&](auto ey) {
    with_ct<T, +1>(a.X, [&](auto ex) {
      using EYt = decltype(ey);
      using EXt = decltype(ex);
      auto k = yx_backward_kernel<EYt, EXt, T>;
      const std::size_t lds = std::max(EYt::h_lds(), EXt::h_lds()) + (8 + a.ncols) * sizeof(int) + 16;
      prepare_kernel(k, lds);
      const int threads = std::max(EYt::h_threads(), EXt::h_threads());
      hipLaunchKernelGGL(k, dim3(grid), dim3(threads), lds, stream, ey, ex, a, sticks, space,
                         scratch, twy, twx);
      gpu_check_launch("yx_backward", stream);
    });
  });
}

template <typename T>
void launch_xy_forward(const FusedArgs& a, int grid, const cx<T>* space, cx<T>* sticks,
                       cx<T>* scratch, const cx<T>* twy, const cx<T>* twx, hipStream_t stream) {
  with_ct<T, -1>(a.Y, [&](auto ey) {
    with_ct<T, -1>(a.X, [&](auto ex) {
      using EYt = decltype(ey);
      using EXt = decltype(ex);
      auto k = xy_forward_kernel<EYt, EXt, T>;
      const std::size_t lds = std::max(EYt::h_lds(), EXt::h_lds()) + (8 + a.ncols) * sizeof(int) + 16;
      prepare_kernel(k, lds);
      const int threads = std::max(EYt::h_threads(), EXt::h_threads());
      hipLaunchKernelGGL(k, dim3(grid), dim3(threads), lds, stream, ey, ex, a, space, sticks,
                         scratch, twy, twx);
      gpu_check_launch("xy_forward", stream);
    });
  });
}

template <typename T>
int fused_blocks_per_cu(int x, int y) {
  int best = 0;
  with_ct<T, +1>(y, [&](auto ey) {
    with_ct<T, +1>(x, [&](auto ex) {
      using EYt = decltype(ey);
      using EXt = decltype(ex);
      auto k = yx_backward_kernel<EYt, EXt, T>;
      const std::size_t lds = std::max(EYt::h_lds(), EXt::h_lds()) + (8 + 1024) * sizeof(int) + 16;
      prepare_kernel(k, lds);
      int n = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
              &n, reinterpret_cast<const void*>(k), std::max(EYt::h_threads(), EXt::h_threads()),
              lds) != hipSuccess)
        n = 0;
      best = n;
    });
  });
  return best;
}

#define SPFFT_FUSED_INST(T)                                                                        \
  template std::size_t fused_lds_bytes<T>(int, int);                                              \
  template int fused_threads<T>(int, int);                                                        \
  template int fused_blocks_per_cu<T>(int, int);                                                  \
  template void launch_z_backward_pm<T>(const FusedArgs&, const cx<T>*, cx<T>*, const cx<T>*,     \
                                        hipStream_t);                                             \
  template void launch_z_forward_pm<T>(const FusedArgs&, const cx<T>*, cx<T>*, T, const cx<T>*,   \
                                       hipStream_t);                                              \
  template void launch_yx_backward<T>(const FusedArgs&, int, const cx<T>*, cx<T>*, cx<T>*,        \
                                      const cx<T>*, const cx<T>*, hipStream_t);                   \
  template void launch_xy_forward<T>(const FusedArgs&, int, const cx<T>*, cx<T>*, cx<T>*,         \
                                     const cx<T>*, const cx<T>*, hipStream_t);
SPFFT_FUSED_INST(double)
SPFFT_FUSED_INST(float)
#undef SPFFT_FUSED_INST

}  // namespace dev
}  // namespace spfft
