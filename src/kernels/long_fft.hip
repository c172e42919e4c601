// Long line FFTs (four-step in global memory, Bluestein on top) and the stage
// glue around them; see long_fft.hpp.
#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "kernels/long_fft.hpp"
#include "kernels/stage_kernels.hpp"

// after the HIP headers (codelets use __forceinline__ under hipcc)
#include "fft/host_fft.hpp"

namespace spfft {
namespace dev {

// ------------------------------------------------------------ glue helpers
// f(i) for i in [0, n), grid-stride
template <class F>
__global__ void __launch_bounds__(256) for_each_kernel(long long n, F f) {
  const long long stride = static_cast<long long>(gridDim.x) * blockDim.x;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < n; i += stride)
    f(i);
}

template <class F>
void for_each(long long n, hipStream_t s, F f) {
  if (n <= 0) return;
  const long long blocks = std::min<long long>((n + 255) / 256, 1 << 16);
  hipLaunchKernelGGL(for_each_kernel<F>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, n, f);
  gpu_check_launch("long_glue", s);
}

// hermitian completion (where the source is non-zero) of `count` lines of
// length n at base + l * stride, one workgroup per line, the reference's two
// half passes separated by a barrier
template <typename T>
__global__ void __launch_bounds__(256) herm_lines_kernel(cx<T>* base, long long stride, int n) {
  cx<T>* v = base + blockIdx.x * stride;
  const int h1 = n / 2;
  for (int k = 1 + threadIdx.x; k <= h1; k += blockDim.x) {
    const cx<T> x = v[k];
    if (nonzero(x)) v[n - k] = conj(x);
  }
  __syncthreads();
  for (int k = h1 + 1 + threadIdx.x; k < n; k += blockDim.x) {
    const cx<T> x = v[k];
    if (nonzero(x)) v[n - k] = conj(x);
  }
}

// ------------------------------------------------------------ four-step
// A pass workgroup runs its engine's B lines on a tile of lt lines x (B / lt)
// columns (cols pass: j2, rows pass: k1) of the [n1][n2] views; the B engine
// lines run lines fastest. lt = 1 (one line) where the stage side is a row of
// the line (sticks, rows of the intermediate or of the space domain); the x
// stage's intermediate side ([z][column][y]: consecutive x are a column apart)
// takes lt > 1, so its accesses cover lt consecutive y instead of one element.
struct PassArgs {
  int n1, n2;
  long long stride;  // work buffer line stride
  int blocksPerLine;  // tiles per line tile: ceil(n2 / (B / lt)) (cols), ceil(n1 / (B / lt)) (rows)
  int lt;     // lines per tile (a power of two dividing B)
  long long lines;
};

// Value at position z of a line after the reference's two-pass hermitian
// completion (src/symmetry/symmetry_host.hpp:68-94: only zero entries are
// filled), computed pointwise from the original entries: the (0,0) stick and
// the x = 0 column of R2C transforms, inside the fused loads.
template <typename T, class Get>
__device__ __forceinline__ cx<T> hermitian_at(Get get, int z, int n) {
  if (z == 0) return get(0);
  const cx<T> v = get(z);
  if (2 * z <= n) return nonzero(v) ? v : conj(get(n - z));
  const cx<T> u = get(n - z);
  return nonzero(u) ? conj(u) : v;
}

// Sources and sinks of the four-step passes. The columns pass reads its
// elements through io.load(line, pos), the rows pass delivers its results to
// io.store(line, pos, v): the stage launchers configure value gathers, the
// exchange layouts, hermitian fills and the x -> column tables there, so no
// glue kernel runs before the columns pass or after the rows pass. The variant
// is a run-time field (a workgroup-uniform branch per element): one kernel per
// engine, precision and exchange type, not one per call site.
template <typename T, typename BT>
struct LongIO {
  enum Kind : int {
    kPlain,      // src[line * srcStride + pos] / dst[line * dstStride + pos]
    kFilter,     // store: dst[...] = v * filt[pos] (Bluestein convolution)
    kZValues,    // load / store: the sparse values of stick s0 + line (simple sticks)
    kZSeg,       // load / store: the exchange layout (seg_index)
    kYCols,      // load / store: the stick entries of column c through its run descriptor
    kXCols,      // load: X[x] of row `line` from the intermediate's columns (x -> column table)
    kXPacked,    // load: packed-real C2R pre-pass of X[k], X[h-k]
    kXOdd,       // load: hermitian-extended complex row (odd length C2R)
    kXReal,      // load: real row as complex
    kXPut,       // store: the columns that hold sticks
    kReal,       // store: real part
  };
  int lk = kPlain, sk = kPlain;
  int n = 0;  // line length
  const cx<T>* src = nullptr;
  long long srcStride = 0;
  cx<T>* dst = nullptr;
  long long dstStride = 0;
  // Bluestein: chirp on the load (pos < chirpN: x d_pos, else 0) or on the store
  // (pos < chirpN: d_pos v * outScale, else dropped); d = conj(chirp) when chirpConj
  const cx<T>* chirpIn = nullptr;
  const cx<T>* chirpOut = nullptr;
  int chirpN = 0, chirpConj = 0;
  T outScale = T(1);
  const cx<T>* filt = nullptr;
  // z stage: exchange-side addressing of ZArgs (single, stickStride, zTab)
  int zSingle = 1;
  long long zStride = 0;
  const long long* zTab = nullptr;
  const StickDesc* desc = nullptr;
  const cx<T>* values = nullptr;
  cx<T>* valuesOut = nullptr;
  const BT* xin = nullptr;
  BT* xout = nullptr;
  int s0 = 0, zeroStick = -1;
  T vscale = T(1);
  // y stage
  const ColDesc* colDesc = nullptr;
  long long colStride = 0;
  int zb = 0, C = 1, x0 = -1;
  // x stage
  const cx<T>* inter = nullptr;
  cx<T>* interOut = nullptr;
  long long iz = 0, is = 0;
  int Y = 1, nf = 0, X = 0, h = 0;
  const int* xToCol = nullptr;
  const cx<T>* twFull = nullptr;
  const T* realSrc = nullptr;
  T* realDst = nullptr;

  __device__ __forceinline__ long long seg(long long line, int pos) const {
    const long long s = s0 + line;
    if (zSingle == 1) return s * zStride + pos;
    using V = long long __attribute__((ext_vector_type(2)));
    const V t = *reinterpret_cast<const V*>(zTab + 2 * pos);
    return t.x + s * t.y;
  }
  __device__ __forceinline__ cx<T> zvalue(long long s, int z) const {
    const StickDesc& q = desc[s0 + s];
    auto get = [&](int zz) -> cx<T> {
      const int j = desc_offset(q, zz);
      return j < 0 ? czero<T>() : values[q.valueStart + j];
    };
    return s0 + s == zeroStick ? hermitian_at<T>(get, z, n) : get(z);
  }
  __device__ __forceinline__ cx<T> ycol(long long l, int y) const {
    const int zz = static_cast<int>(l / C), c = static_cast<int>(l - static_cast<long long>(zz) * C);
    const ColDesc& d = colDesc[c];
    auto get = [&](int yy) -> cx<T> {
      long long base;
      return col_desc_find(d, colStride, yy, base) ? cvt<T>(xin[base + zb + zz]) : czero<T>();
    };
    return c == x0 ? hermitian_at<T>(get, y, n) : get(y);
  }
  __device__ __forceinline__ cx<T> xcol(long long l, int x) const {
    const long long zz = l / Y, y = l - zz * Y;
    const int c = x < nf ? xToCol[x] : -1;
    return c < 0 ? czero<T>() : inter[zz * iz + c * is + y];
  }
  __device__ __forceinline__ cx<T> base_load(long long line, int pos) const {
    switch (lk) {
      case kZValues:
        return zvalue(line, pos);
      case kZSeg:
        return cvt<T>(xin[seg(line, pos)]);
      case kYCols:
        return ycol(line, pos);
      case kXCols:
        return xcol(line, pos);
      case kXPacked: {
        cx<T> xk = xcol(line, pos), xm = xcol(line, h - pos);
        if (pos == 0) {
          xk.y = T(0);
          xm.y = T(0);
        }
        const cx<T> xmc = conj(xm);
        return (xk + xmc) + rot<+1>(twm<+1>(xk - xmc, twFull[pos]));
      }
      case kXOdd:
        return pos < nf ? xcol(line, pos) : conj(xcol(line, X - pos));
      case kXReal:
        return mk<T>(realSrc[line * X + pos], T(0));
      default:
        return src[line * srcStride + pos];
    }
  }
  __device__ __forceinline__ cx<T> load(long long line, int pos) const {
    if (chirpIn) {
      if (pos >= chirpN) return czero<T>();
      const cx<T> d = chirpConj ? conj(chirpIn[pos]) : chirpIn[pos];
      return cmul(base_load(line, pos), d);
    }
    return base_load(line, pos);
  }
  __device__ __forceinline__ void store(long long line, int pos, cx<T> v) const {
    if (chirpOut) {
      if (pos >= chirpN) return;
      const cx<T> d = chirpConj ? conj(chirpOut[pos]) : chirpOut[pos];
      v = scale(cmul(v, d), outScale);
    }
    switch (sk) {
      case kFilter:
        dst[line * dstStride + pos] = cmul(v, filt[pos]);
        return;
      case kZSeg:
        xout[seg(line, pos)] = cvt<typename BT::value_type>(v);
        return;
      case kZValues: {
        const StickDesc& q = desc[s0 + line];
        const int j = desc_offset(q, pos);
        if (j >= 0) valuesOut[q.valueStart + j] = scale(v, vscale);
        return;
      }
      case kYCols: {
        const int zz = static_cast<int>(line / C), c = static_cast<int>(line - static_cast<long long>(zz) * C);
        long long base;
        if (col_desc_find(colDesc[c], colStride, pos, base)) xout[base + zb + zz] = cvt<typename BT::value_type>(v);
        return;
      }
      case kXPut: {
        const int c = pos < nf ? xToCol[pos] : -1;
        if (c < 0) return;
        const long long zz = line / Y, y = line - zz * Y;
        interOut[zz * iz + c * is + y] = v;
        return;
      }
      case kReal:
        realDst[line * X + pos] = v.x;
        return;
      default:
        dst[line * dstStride + pos] = v;
    }
  }
};

// columns pass: for every column j2 of a line viewed as [n1][n2]: FFT_n1 over
// j1 -> k1, times exp(S 2 pi i j2 k1 / (n1 n2)), into work (same positions).
// The line comes from io.load(line, j1 n2 + j2) (fused) or from work itself
// (plain: the run-time engines, whose pass switch leaves no registers for the
// IO variants, read a line a glue pass staged). Lanes walk consecutive columns
// (coalesced rows of the [n1][n2] view).
template <class Eng, typename T, class Src>
__device__ __forceinline__ void long_cols_body(const Eng& eng, const PassArgs& a, Src src, cx<T>* work,
                                               const cx<T>* __restrict__ tw1, const cx<T>* __restrict__ twM,
                                               int S) {
  SPFFT_LDS_DECL(T);
  const int B = eng.lines();
  const int lt = a.lt, ltShift = __builtin_ctz(static_cast<unsigned>(lt));
  const long long l0 = static_cast<long long>(blockIdx.x / a.blocksPerLine) << ltShift;
  const int j20 = static_cast<int>(blockIdx.x % a.blocksPerLine) * (B >> ltShift);
  const int total = B * a.n1;
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int b = idx % B, j1 = idx / B, j2 = j20 + (b >> ltShift);
    const long long line = l0 + (b & (lt - 1));
    lds[eng.in_at(b, j1)] = (j2 < a.n2 && line < a.lines) ? src(line, j1 * a.n2 + j2) : czero<T>();
  }
  __syncthreads();
  eng.lds_to_lds(lds, tw1);
  // compile-time engines: a lane keeps its column j2 and walks k1 = k1f + m *
  // step (m < kIt), so its twiddles w^(j2 k1) are one table entry per group of
  // kG times the powers of w^(j2 step) formed in registers (twiddle_powers:
  // a few ulp), instead of one table load per element from the n1 n2-entry
  // table: those loads cost 305 -> 211 us of the 8192 x 64 x 64 fp64 forward
  // columns pass (all loads removed, profiles/r5/long)
  constexpr int kIt = [] {
    if constexpr (Eng::kBatchedCopy) {
      return 0;
    } else {
      constexpr int work = Eng::F::B * Eng::kN;
      return work % Eng::F::NT == 0 ? work / Eng::F::NT : 0;
    }
  }();
  auto generic = [&] {
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
      const int b = idx % B, k1 = idx / B, j2 = j20 + (b >> ltShift);
      const long long line = l0 + (b & (lt - 1));
      if (j2 < a.n2 && line < a.lines) {
        const cx<T> w = twM[static_cast<long long>(j2) * k1];
        const cx<T> v = lds[eng.out_at(b, k1)];
        work[line * a.stride + static_cast<long long>(k1) * a.n2 + j2] = S > 0 ? twm<+1>(v, w) : twm<-1>(v, w);
      }
    }
  };
  if constexpr (kIt >= 1) {
    // (launched with the engine's own thread count, four_step)
    if (blockDim.x != static_cast<unsigned>(Eng::F::NT)) {
      generic();
      return;
    }
    constexpr int kG = kIt < 8 ? kIt : 8;
    const int b = static_cast<int>(threadIdx.x) % B, j2 = j20 + (b >> ltShift);
    const long long line = l0 + (b & (lt - 1));
    const int step = static_cast<int>(blockDim.x) / B, k1f = static_cast<int>(threadIdx.x) / B;
    if (j2 < a.n2 && line < a.lines) {
      cx<T> pw[kG > 1 ? kG - 1 : 1];
      if constexpr (kG > 1) twiddle_powers<kG>(twM[static_cast<long long>(j2) * step], pw);
      cx<T>* dstLine = work + line * a.stride + j2;
#pragma unroll
      for (int g = 0; g < kIt / kG; ++g) {
        const int kg = k1f + g * kG * step;
        const cx<T> wb = twM[static_cast<long long>(j2) * kg];
#pragma unroll
        for (int r = 0; r < kG; ++r) {
          const int k1 = kg + r * step;
          const cx<T> w = r == 0 ? wb : cmul(wb, pw[r > 0 ? r - 1 : 0]);
          const cx<T> v = lds[eng.out_at(b, k1)];
          dstLine[static_cast<long long>(k1) * a.n2] = S > 0 ? twm<+1>(v, w) : twm<-1>(v, w);
        }
      }
    }
  } else {
    generic();
  }
}
template <class Eng, typename T, typename BT, int S>
__global__ void __launch_bounds__(Eng::kBlock)
    long_cols_kernel(Eng eng, PassArgs a, LongIO<T, BT> io, cx<T>* work, const cx<T>* __restrict__ tw1,
                     const cx<T>* __restrict__ twM) {
  long_cols_body<Eng, T>(eng, a, [&](long long l, int p) { return io.load(l, p); }, work, tw1, twM, S);
}
template <class Eng, typename T, int S>
__global__ void __launch_bounds__(Eng::kBlock)
    long_cols_plain_kernel(Eng eng, PassArgs a, cx<T>* work, const cx<T>* __restrict__ tw1,
                           const cx<T>* __restrict__ twM) {
  long_cols_body<Eng, T>(eng, a, [&](long long l, int p) { return work[l * a.stride + p]; }, work, tw1,
                         twM, S);
}

// rows pass: for every row k1 of work: FFT_n2 over j2 -> k2, delivered to
// position k1 + n1 k2 of io.store (fused) or of out (plain, natural order,
// stride n1 n2, for a glue pass); loads walk rows, stores walk k1 fastest
template <class Eng, typename T, class Dst>
__device__ __forceinline__ void long_rows_body(const Eng& eng, const PassArgs& a, const cx<T>* work,
                                               Dst dst, const cx<T>* __restrict__ tw2) {
  SPFFT_LDS_DECL(T);
  const int B = eng.lines();
  const int lt = a.lt, ltShift = __builtin_ctz(static_cast<unsigned>(lt));
  const long long l0 = static_cast<long long>(blockIdx.x / a.blocksPerLine) << ltShift;
  const int k10 = static_cast<int>(blockIdx.x % a.blocksPerLine) * (B >> ltShift);
  const int total = B * a.n2;
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int b = idx / a.n2, j2 = idx - b * a.n2, k1 = k10 + (b >> ltShift);
    const long long line = l0 + (b & (lt - 1));
    lds[eng.in_at(b, j2)] = (k1 < a.n1 && line < a.lines)
                                ? work[line * a.stride + static_cast<long long>(k1) * a.n2 + j2]
                                : czero<T>();
  }
  __syncthreads();
  eng.lds_to_lds(lds, tw2);
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int b = idx % B, k2 = idx / B, k1 = k10 + (b >> ltShift);
    const long long line = l0 + (b & (lt - 1));
    if (k1 < a.n1 && line < a.lines) dst(line, k1 + a.n1 * k2, lds[eng.out_at(b, k2)]);
  }
}
template <class Eng, typename T, typename BT, int S>
__global__ void __launch_bounds__(Eng::kBlock)
    long_rows_kernel(Eng eng, PassArgs a, const cx<T>* work, LongIO<T, BT> io,
                     const cx<T>* __restrict__ tw2) {
  long_rows_body<Eng, T>(eng, a, work, [&](long long l, int p, cx<T> v) { io.store(l, p, v); }, tw2);
}
template <class Eng, typename T, int S>
__global__ void __launch_bounds__(Eng::kBlock)
    long_rows_plain_kernel(Eng eng, PassArgs a, const cx<T>* work, cx<T>* out,
                           const cx<T>* __restrict__ tw2) {
  long_rows_body<Eng, T>(eng, a, work, [&](long long l, int p, cx<T> v) { out[l * a.stride + p] = v; },
                         tw2);
}

// Engines of the four-step passes: the power-of-two compile-time engines and
// the run-time engine (the factors are short with radices <= 13, long_plan).
// The mixed-radix compile-time engines are left out: with every IO variant in
// each pass kernel, 25 more engine instantiations tripled the compile time.
inline bool long_ct_factor(int n) { return n >= 16 && n <= 1024 && (n & (n - 1)) == 0; }
template <typename T, int S, class F>
inline void with_long_engine(int n, F&& f) {
  switch (n) {
#define SPFFT_LONG_CASE(NN)                                     \
  case NN: {                                                     \
    using E = CtEng<T, NN, S, true, true>;                       \
    f(E{}, E::h_threads(), E::h_lines(), E::h_lds());            \
    return;                                                      \
  }
    SPFFT_LONG_CASE(16)
    SPFFT_LONG_CASE(32)
    SPFFT_LONG_CASE(64)
    SPFFT_LONG_CASE(128)
    SPFFT_LONG_CASE(256)
    SPFFT_LONG_CASE(512)
    SPFFT_LONG_CASE(1024)
#undef SPFFT_LONG_CASE
    default: {
      RtEng<T, S, true> e{make_rt_plan(n, sizeof(cx<T>))};
      f(e, kRtThreads, e.p.lines, std::size_t(e.p.inplace ? 1 : 2) * e.p.lines * e.p.ls * sizeof(cx<T>));
    }
  }
}

// length n1 * n2 lines: io.load -> io.store, through `work` (lines * n1 * n2
// elements; may be the load's own buffer: a columns workgroup stages all of its
// elements before it writes them back). Run-time engine passes take a glue pass
// instead of the fused IO; `scratch` (lines * n1 * n2) holds the rows pass
// output for it.
template <typename T, typename BT, int S>
void four_step(const LongPlan& lp, long long lines, const LongIO<T, BT>& io, cx<T>* work,
               cx<T>* scratch, hipStream_t stream) {
  if (lines <= 0) return;
  const long long stride = static_cast<long long>(lp.n1) * lp.n2;
  const bool ct1 = long_ct_factor(lp.n1), ct2 = long_ct_factor(lp.n2);
  if (!ct1) {
    const LongIO<T, BT> l = io;
    for_each(lines * stride, stream, [=] __device__(long long i) {
      const long long line = i / stride;
      work[i] = l.load(line, static_cast<int>(i - line * stride));
    });
  }
  // the x stage's intermediate side: tiles of several lines (consecutive y)
  const auto tile = [](int B, bool xSide) { return xSide && B >= 8 ? B / 4 : 1; };
  const bool xLoad = io.lk == LongIO<T, BT>::kXCols || io.lk == LongIO<T, BT>::kXPacked ||
                     io.lk == LongIO<T, BT>::kXOdd;
  const bool xStore = io.sk == LongIO<T, BT>::kXPut;
  with_long_engine<T, S>(lp.n1, [&](auto eng, int threads, int B, std::size_t lds) {
    const int lt = decltype(eng)::kBatchedCopy ? 1 : tile(B, xLoad);
    PassArgs a{lp.n1, lp.n2, stride, static_cast<int>(ceil_div(lp.n2, B / lt)), lt, lines};
    const dim3 grid(static_cast<unsigned>(ceil_div(lines, lt) * a.blocksPerLine));
    const auto* tw1 = static_cast<const cx<T>*>(lp.tw1);
    const auto* twM = static_cast<const cx<T>*>(lp.twM);
    if constexpr (decltype(eng)::kBatchedCopy) {
      auto k = long_cols_plain_kernel<decltype(eng), T, S>;
      prepare_kernel(k, lds);
      hipLaunchKernelGGL(k, grid, dim3(threads), lds, stream, eng, a, work, tw1, twM);
    } else {
      auto k = long_cols_kernel<decltype(eng), T, BT, S>;
      prepare_kernel(k, lds);
      hipLaunchKernelGGL(k, grid, dim3(threads), lds, stream, eng, a, io, work, tw1, twM);
    }
    gpu_check_launch("long_cols", stream);
  });
  with_long_engine<T, S>(lp.n2, [&](auto eng, int threads, int B, std::size_t lds) {
    const int lt = decltype(eng)::kBatchedCopy ? 1 : tile(B, xStore);
    PassArgs a{lp.n1, lp.n2, stride, static_cast<int>(ceil_div(lp.n1, B / lt)), lt, lines};
    const dim3 grid(static_cast<unsigned>(ceil_div(lines, lt) * a.blocksPerLine));
    const auto* tw2 = static_cast<const cx<T>*>(lp.tw2);
    if constexpr (decltype(eng)::kBatchedCopy) {
      auto k = long_rows_plain_kernel<decltype(eng), T, S>;
      prepare_kernel(k, lds);
      hipLaunchKernelGGL(k, grid, dim3(threads), lds, stream, eng, a, work, scratch, tw2);
    } else {
      auto k = long_rows_kernel<decltype(eng), T, BT, S>;
      prepare_kernel(k, lds);
      hipLaunchKernelGGL(k, grid, dim3(threads), lds, stream, eng, a, work, io, tw2);
    }
    gpu_check_launch("long_rows", stream);
  });
  if (!ct2) {
    const LongIO<T, BT> l = io;
    const cx<T>* res = scratch;
    for_each(lines * stride, stream, [=] __device__(long long i) {
      const long long line = i / stride;
      l.store(line, static_cast<int>(i - line * stride), res[i]);
    });
  }
}

// One long FFT of sign S over `lines` lines of length lp.n: io.load -> io.store.
// Bluestein (X_k = d_k sum_j (x_j d_j) conj(d_{k-j}), d_j = exp(S i pi j^2 / n))
// runs as two four-steps of length m: the chirp folds into the first columns
// pass's loads, the filter into its rows pass's stores, the final chirp and
// 1/m into the second rows pass's stores: four kernels, no glue.
template <typename T, typename BT, int S>
void long_fft(const LongPlan& lp, long long lines, const LongIO<T, BT>& io, const LongBufs<T>& w,
              hipStream_t stream) {
  if (!lp.bluestein) {
    four_step<T, BT, S>(lp, lines, io, w.in, w.out, stream);
    return;
  }
  const int m = lp.m;
  const cx<T>* chirp = static_cast<const cx<T>*>(lp.chirp);
  LongIO<T, BT> first = io;  // the stage's load with the chirp; store: the filter product
  first.chirpIn = chirp;
  first.chirpN = lp.n;
  first.chirpConj = S < 0 ? 0 : 1;
  first.sk = LongIO<T, BT>::kFilter;
  first.chirpOut = nullptr;
  first.dst = w.w2;
  first.dstStride = m;
  first.filt = static_cast<const cx<T>*>(lp.filt) + (S < 0 ? 0 : m);
  four_step<T, BT, -1>(lp, lines, first, w.w1, w.out, stream);
  LongIO<T, BT> second = io;  // load: the convolution; the stage's store with the chirp
  second.lk = LongIO<T, BT>::kPlain;
  second.chirpIn = nullptr;
  second.src = w.w2;
  second.srcStride = m;
  second.chirpOut = chirp;
  second.chirpN = lp.n;
  second.chirpConj = S < 0 ? 0 : 1;
  second.outScale = T(1) / static_cast<T>(m);
  four_step<T, BT, +1>(lp, lines, second, w.w2, w.out, stream);
}

// ------------------------------------------------------------ plans
namespace {
int largest_prime(int n) {
  const std::vector<int> r = factorize_radices(n);
  int p = 1;
  for (int f : r) {
    // factorize_radices emits composite codelet radices (16, 8, 4, 9): reduce
    int q = f;
    for (int d = 2; d * d <= q; ++d)
      while (q % d == 0) {
        p = std::max(p, d);
        q /= d;
      }
    if (q > 1) p = std::max(p, q);
  }
  return p;
}
// a factor the one-workgroup engines run well (compile-time, or run-time with
// codelet radices only)
bool short_ok(int f) { return long_ct_factor(f) || (f >= 2 && f <= 4096 && largest_prime(f) <= 13); }

template <typename T>
void bluestein_host_tables(int n, int m, std::vector<cx<T>>& chirp, std::vector<cx<T>>& filt) {
  const long double pi = 3.141592653589793238462643383279502884L;
  chirp.resize(n);
  for (int j = 0; j < n; ++j) {
    const long long q = (static_cast<long long>(j) * j) % (2LL * n);  // exact phase reduction
    const long double a = pi * static_cast<long double>(q) / static_cast<long double>(n);
    chirp[j] = mk<T>(static_cast<T>(std::cos(a)), static_cast<T>(-std::sin(a)));
  }
  HostFft<double> fft(m);
  std::vector<cx<double>> work(fft.scratch_size()), b(m);
  filt.resize(2 * static_cast<std::size_t>(m));
  for (int s = 0; s < 2; ++s) {
    for (auto& v : b) v = mk<double>(0.0, 0.0);
    for (int j = 0; j < n; ++j) {
      const long long q = (static_cast<long long>(j) * j) % (2LL * n);
      const long double a = pi * static_cast<long double>(q) / static_cast<long double>(n);
      // conj(d_j): S = -1 -> exp(+i a), S = +1 -> exp(-i a)
      const cx<double> c = mk<double>(static_cast<double>(std::cos(a)),
                                      static_cast<double>(s == 0 ? std::sin(a) : -std::sin(a)));
      b[j] = c;
      if (j > 0) b[m - j] = c;
    }
    fft.execute(b.data(), 1, b.data(), 1, -1, work.data());
    for (int j = 0; j < m; ++j)
      filt[static_cast<std::size_t>(s) * m + j] = mk<T>(static_cast<T>(b[j].x), static_cast<T>(b[j].y));
  }
}
}  // namespace

bool needs_long_path(int n, bool dbl, LongAxis axis) {
  if (n <= 1 || has_ct_kernel(n)) return false;
  if (n > max_device_fft_length(dbl)) return true;
  const std::size_t eb = dbl ? sizeof(cx<double>) : sizeof(cx<float>);
  if (largest_prime(n) > kBluesteinPrime && !use_bluestein(n, eb)) return true;
  int lines = 0;
  std::size_t lds = 0;
  try {
    lds = in_lds_engine_bytes(n, eb, lines);
  } catch (const GPUFFTError&) {
    return true;
  }
  std::size_t extra = 0;
  if (axis == kLongAxisY) extra = static_cast<std::size_t>(n) * (sizeof(long long) + 2 * sizeof(int)) + 16;
  if (axis == kLongAxisX) extra = static_cast<std::size_t>(n + 1) * sizeof(int) + 16 + lines * eb;
  if (lds + extra > kLdsPerWorkgroup) return true;
  if (axis != kLongAxisZ && static_cast<std::size_t>(lines) * eb < 64) {
    for (int d = 16; d <= n / 16; d *= 2)
      if (n % d == 0 && long_ct_factor(d) && long_ct_factor(n / d)) return true;
  }
  return false;
}

LongPlan long_plan(int n, bool dbl) {
  static std::mutex mutex;
  static std::map<std::tuple<int, int, bool>, LongPlan> cache;
  int device = 0;
  gpu_check(hipGetDevice(&device), "hipGetDevice");
  std::lock_guard<std::mutex> lock(mutex);
  auto it = cache.find(std::make_tuple(device, n, dbl));
  if (it != cache.end()) return it->second;
  LongPlan p;
  p.n = n;
  // four-step factors: both short, compile-time engines first, then balanced
  int best = -1, bestScore = 1 << 30;
  for (int d = 2; d <= n / 2; ++d) {
    if (n % d || !short_ok(d) || !short_ok(n / d)) continue;
    const int score = ((long_ct_factor(d) ? 0 : 1) + (long_ct_factor(n / d) ? 0 : 1)) * (1 << 20) +
                      std::abs(d - n / d);
    if (score < bestScore) {
      bestScore = score;
      best = d;
    }
  }
  if (best > 0) {
    p.m = n;
    p.n1 = best;
    p.n2 = n / best;
  } else {
    p.bluestein = true;
    int m = 1, k = 0;
    while (m < 2 * n - 1) {
      m *= 2;
      ++k;
    }
    if (k > 20) throw GPUFFTError();
    p.m = m;
    p.n1 = 1 << (k / 2);
    p.n2 = m / p.n1;
  }
  const std::size_t eb = dbl ? sizeof(cx<double>) : sizeof(cx<float>);
  const std::size_t nc = p.bluestein ? static_cast<std::size_t>(n) : 0;
  const std::size_t nf = p.bluestein ? 2 * static_cast<std::size_t>(p.m) : 0;
  const std::size_t total = p.n1 + p.n2 + static_cast<std::size_t>(p.m) + nc + nf;
  auto* buf = new DeviceBuffer(total * eb);  // lives for the process (cached plan)
  char* base = buf->data<char>();
  auto put = [&](const void* host, std::size_t elems, std::size_t& off) -> const void* {
    char* dst = base + off * eb;
    gpu_check(hipMemcpy(dst, host, elems * eb, hipMemcpyHostToDevice), "hipMemcpy");
    off += elems;
    return dst;
  };
  std::size_t off = 0;
  auto fill = [&](auto tag) {
    using T = decltype(tag);
    const auto t1 = make_twiddles<T>(p.n1), t2 = make_twiddles<T>(p.n2), tm = make_twiddles<T>(p.m);
    p.tw1 = put(t1.data(), p.n1, off);
    p.tw2 = put(t2.data(), p.n2, off);
    p.twM = put(tm.data(), p.m, off);
    if (p.bluestein) {
      std::vector<cx<T>> chirp, filt;
      bluestein_host_tables<T>(n, p.m, chirp, filt);
      p.chirp = put(chirp.data(), n, off);
      p.filt = put(filt.data(), 2 * static_cast<std::size_t>(p.m), off);
    }
  };
  if (dbl)
    fill(double{});
  else
    fill(float{});
  cache.emplace(std::make_tuple(device, n, dbl), p);
  return p;
}

// ------------------------------------------------------------ z stage
// Fused when every stick is simple (StickDesc: at most two z-runs of contiguous
// values): the columns pass gathers the sparse values itself (with the (0,0)
// stick's hermitian fill) and the rows pass stores into the exchange layout.
// Other index sets stage the decompressed sticks in natural order first.
template <typename T, typename BT>
void launch_long_z_backward(const LongPlan& lp, const ZArgs& a, const cx<T>* values, BT* out,
                            const LongBufs<T>& w, hipStream_t stream) {
  const long long S = a.numSticks - a.stickBegin;
  if (S <= 0) return;
  const int n = a.n;
  const int s0 = a.stickBegin;
  LongIO<T, BT> io;
  io.n = n;
  io.zSingle = a.single;
  io.zStride = a.stickStride;
  io.zTab = a.zTab;
  io.s0 = s0;
  io.sk = LongIO<T, BT>::kZSeg;
  io.xout = out;
  if (a.desc) {
    io.lk = LongIO<T, BT>::kZValues;
    io.desc = a.desc;
    io.values = values;
    io.zeroStick = a.zeroStick;
    long_fft<T, BT, +1>(lp, S, io, w, stream);
    return;
  }
  cx<T>* in = w.out;
  gpu_check(hipMemsetAsync(in, 0, static_cast<std::size_t>(S) * n * sizeof(cx<T>), stream),
            "hipMemsetAsync");
  const StickRun* runs = a.runs;
  const int* ro = a.runOffsets;
  for_each(S, stream, [=] __device__(long long s) {
    const int st = s0 + static_cast<int>(s);
    for (int q = ro[st]; q < ro[st + 1]; ++q) {
      const StickRun r = runs[q];
      cx<T>* line = in + (r.stick - s0) * static_cast<long long>(n) + r.zStart;
      for (int j = 0; j < r.length; ++j) line[j] = values[r.valueStart + j];
    }
  });
  if (a.zeroStick >= s0 && a.zeroStick < a.numSticks) {
    hipLaunchKernelGGL(herm_lines_kernel<T>, dim3(1), dim3(256), 0, stream,
                       in + static_cast<long long>(a.zeroStick - s0) * n, static_cast<long long>(n), n);
    gpu_check_launch("long_herm", stream);
  }
  io.lk = LongIO<T, BT>::kPlain;
  io.src = in;
  io.srcStride = n;
  long_fft<T, BT, +1>(lp, S, io, w, stream);
}

template <typename T, typename BT>
void launch_long_z_forward(const LongPlan& lp, const ZArgs& a, const BT* in, cx<T>* values, T scl,
                           const LongBufs<T>& w, hipStream_t stream) {
  const long long S = a.numSticks - a.stickBegin;
  if (S <= 0) return;
  const int n = a.n;
  const int s0 = a.stickBegin;
  LongIO<T, BT> io;
  io.n = n;
  io.zSingle = a.single;
  io.zStride = a.stickStride;
  io.zTab = a.zTab;
  io.s0 = s0;
  io.lk = LongIO<T, BT>::kZSeg;
  io.xin = in;
  if (a.desc) {
    io.sk = LongIO<T, BT>::kZValues;
    io.desc = a.desc;
    io.valuesOut = values;
    io.vscale = scl;
    long_fft<T, BT, -1>(lp, S, io, w, stream);
    return;
  }
  cx<T>* res = w.out;
  io.sk = LongIO<T, BT>::kPlain;
  io.dst = res;
  io.dstStride = n;
  long_fft<T, BT, -1>(lp, S, io, w, stream);
  const StickRun* runs = a.runs;
  const int* ro = a.runOffsets;
  for_each(S, stream, [=] __device__(long long s) {
    const int st = s0 + static_cast<int>(s);
    for (int q = ro[st]; q < ro[st + 1]; ++q) {
      const StickRun r = runs[q];
      const cx<T>* line = res + (r.stick - s0) * static_cast<long long>(n) + r.zStart;
      for (int j = 0; j < r.length; ++j) values[r.valueStart + j] = scale(line[j], scl);
    }
  });
}

// ------------------------------------------------------------ y stage
// Fused when the plan has column run descriptors (YArgs::colDesc): the columns
// pass gathers the stick entries of a column (with the x = 0 column's
// hermitian fill), the forward rows pass stores into them.
template <typename T, typename BT>
void launch_long_y_backward(const LongPlan& lp, const YArgs& a, const BT* in, cx<T>* inter,
                            const LongBufs<T>& w, hipStream_t stream) {
  const int nz = a.L - a.zBegin;
  const int C = a.ncols, n = a.n, zb = a.zBegin;
  if (nz <= 0 || C <= 0) return;
  const long long lines = static_cast<long long>(nz) * C;
  LongIO<T, BT> io;
  io.n = n;
  // line l = (plane zz, column c) -> row (zb + zz, c) of [z][column][y]
  io.sk = LongIO<T, BT>::kPlain;
  io.dst = inter + zb * a.interZStride;
  io.dstStride = a.interStride;
  if (a.colDesc) {
    io.lk = LongIO<T, BT>::kYCols;
    io.colDesc = a.colDesc;
    io.colStride = a.colStride;
    io.xin = in;
    io.zb = zb;
    io.C = C;
    io.x0 = a.colOfX0;
    long_fft<T, BT, +1>(lp, lines, io, w, stream);
    return;
  }
  cx<T>* lin = w.out;
  gpu_check(hipMemsetAsync(lin, 0, static_cast<std::size_t>(lines) * n * sizeof(cx<T>), stream),
            "hipMemsetAsync");
  const int* co = a.colOffsets;
  const int* cy = a.colY;
  const long long* cb = a.colBase;
  for_each(lines, stream, [=] __device__(long long l) {
    const int zz = static_cast<int>(l / C), c = static_cast<int>(l - static_cast<long long>(zz) * C);
    cx<T>* line = lin + l * n;
    for (int k = co[c]; k < co[c + 1]; ++k) line[cy[k]] = cvt<T>(in[cb[k] + zb + zz]);
  });
  if (a.colOfX0 >= 0) {
    hipLaunchKernelGGL(herm_lines_kernel<T>, dim3(nz), dim3(256), 0, stream,
                       lin + static_cast<long long>(a.colOfX0) * n, static_cast<long long>(C) * n, n);
    gpu_check_launch("long_herm", stream);
  }
  io.lk = LongIO<T, BT>::kPlain;
  io.src = lin;
  io.srcStride = n;
  long_fft<T, BT, +1>(lp, lines, io, w, stream);
}

template <typename T, typename BT>
void launch_long_y_forward(const LongPlan& lp, const YArgs& a, cx<T>* inter, BT* out,
                           const LongBufs<T>& w, hipStream_t stream) {
  const int nz = a.L - a.zBegin;
  const int C = a.ncols, n = a.n, zb = a.zBegin;
  if (nz <= 0 || C <= 0) return;
  const long long lines = static_cast<long long>(nz) * C;
  LongIO<T, BT> io;
  io.n = n;
  io.lk = LongIO<T, BT>::kPlain;
  io.src = inter + zb * a.interZStride;
  io.srcStride = a.interStride;
  if (a.colDesc) {
    io.sk = LongIO<T, BT>::kYCols;
    io.colDesc = a.colDesc;
    io.colStride = a.colStride;
    io.xout = out;
    io.zb = zb;
    io.C = C;
    long_fft<T, BT, -1>(lp, lines, io, w, stream);
    return;
  }
  cx<T>* res = w.out;
  io.sk = LongIO<T, BT>::kPlain;
  io.dst = res;
  io.dstStride = n;
  long_fft<T, BT, -1>(lp, lines, io, w, stream);
  const int* co = a.colOffsets;
  const int* cy = a.colY;
  const long long* cb = a.colBase;
  for_each(lines, stream, [=] __device__(long long l) {
    const int zz = static_cast<int>(l / C), c = static_cast<int>(l - static_cast<long long>(zz) * C);
    const cx<T>* line = res + l * n;
    for (int k = co[c]; k < co[c + 1]; ++k)
      out[cb[k] + zb + zz] = cvt<typename BT::value_type>(line[cy[k]]);
  });
}

// ------------------------------------------------------------ x stage
// Fused: the columns pass reads the intermediate's columns through the x ->
// column table (XArgs::xToCol; the packed-real C2R pre-pass and the odd-length
// C2R mirror folded into the load), the rows pass writes the space rows; the
// forward rows pass stores the columns that hold sticks (C2C and odd R2C; the
// packed R2C post-pass pairs outputs k and h - k of one line and keeps its glue).
template <typename T>
void launch_long_x_backward(const LongPlan& lp, const XArgs& a, bool r2c, const cx<T>* inter,
                            void* space, const cx<T>* twFull, const LongBufs<T>& w,
                            hipStream_t stream) {
  const int nz = a.L - a.zBegin;
  const int Y = a.Y, X = a.n, zb = a.zBegin;
  if (nz <= 0 || Y <= 0) return;
  const long long lines = static_cast<long long>(nz) * Y;
  LongIO<T, cx<T>> io;
  io.inter = inter + zb * a.interZStride;
  io.iz = a.interZStride;
  io.is = a.interStride;
  io.Y = Y;
  io.X = X;
  io.nf = a.nFreq;
  io.xToCol = a.xToCol;
  io.twFull = twFull;
  if (!r2c) {
    io.n = X;
    io.lk = LongIO<T, cx<T>>::kXCols;
    io.dst = static_cast<cx<T>*>(space) + static_cast<long long>(zb) * Y * X;
    io.dstStride = X;
  } else if (X % 2 == 0) {
    // packed real rows: Z[k] = (X[k] + conj X[h-k]) + i (X[k] - conj X[h-k]) w^k,
    // w = exp(+2 pi i / X), imaginary parts of X[0], X[h] ignored; IDFT_h(Z)
    // interleaves the real row
    io.h = X / 2;
    io.n = io.h;
    io.lk = LongIO<T, cx<T>>::kXPacked;
    io.dst = reinterpret_cast<cx<T>*>(static_cast<T*>(space) + static_cast<long long>(zb) * Y * X);
    io.dstStride = io.h;
  } else {
    io.n = X;
    io.lk = LongIO<T, cx<T>>::kXOdd;
    io.sk = LongIO<T, cx<T>>::kReal;
    io.realDst = static_cast<T*>(space) + static_cast<long long>(zb) * Y * X;
  }
  long_fft<T, cx<T>, +1>(lp, lines, io, w, stream);
}

template <typename T>
void launch_long_x_forward(const LongPlan& lp, const XArgs& a, bool r2c, const void* space,
                           cx<T>* inter, const cx<T>* twFull, const LongBufs<T>& w,
                           hipStream_t stream) {
  const int nz = a.L - a.zBegin;
  const int Y = a.Y, X = a.n, C = a.ncols, zb = a.zBegin;
  if (nz <= 0 || Y <= 0) return;
  const long long lines = static_cast<long long>(nz) * Y;
  const long long iz = a.interZStride, is = a.interStride;
  cx<T>* dst = inter + zb * iz;
  LongIO<T, cx<T>> io;
  io.interOut = dst;
  io.iz = iz;
  io.is = is;
  io.Y = Y;
  io.X = X;
  io.nf = a.nFreq;
  io.xToCol = a.xToCol;
  io.sk = LongIO<T, cx<T>>::kXPut;
  if (!r2c) {
    // (the four-step works in its own buffer: the space domain stays intact)
    io.n = X;
    io.lk = LongIO<T, cx<T>>::kPlain;
    io.src = static_cast<const cx<T>*>(space) + static_cast<long long>(zb) * Y * X;
    io.srcStride = X;
    long_fft<T, cx<T>, -1>(lp, lines, io, w, stream);
  } else if (X % 2 == 0) {
    // packed real rows y[m] = x[2m] + i x[2m+1]: X[k] = (Y[k] + conj Y[h-k]) / 2
    // + w^k (Y[k] - conj Y[h-k]) / (2i), w = exp(-2 pi i / X), Y[h] = Y[0]
    const int h = X / 2;
    io.n = h;
    io.lk = LongIO<T, cx<T>>::kPlain;
    io.src = reinterpret_cast<const cx<T>*>(static_cast<const T*>(space) + static_cast<long long>(zb) * Y * X);
    io.srcStride = h;
    cx<T>* res = w.out;
    io.sk = LongIO<T, cx<T>>::kPlain;
    io.dst = res;
    io.dstStride = h;
    long_fft<T, cx<T>, -1>(lp, lines, io, w, stream);
    const int* colX = a.colX;
    for_each(lines * C, stream, [=] __device__(long long i) {
      const long long l = i / C;
      const int c = static_cast<int>(i - l * C);
      const long long zz = l / Y, y = l - zz * Y;
      const int k = colX[c];
      const cx<T> yk = res[l * h + (k == h ? 0 : k)];
      const cx<T> ym = conj(res[l * h + (k == 0 ? 0 : h - k)]);
      const cx<T> e = scale(yk + ym, T(0.5));
      const cx<T> o = scale(rot<-1>(yk - ym), T(0.5));
      dst[zz * iz + c * is + y] = e + twm<-1>(o, twFull[k]);
    });
  } else {
    io.n = X;
    io.lk = LongIO<T, cx<T>>::kXReal;
    io.realSrc = static_cast<const T*>(space) + static_cast<long long>(zb) * Y * X;
    long_fft<T, cx<T>, -1>(lp, lines, io, w, stream);
  }
}

#define SPFFT_LONG_INST(T, BT)                                                                   \
  template void launch_long_z_backward<T, BT>(const LongPlan&, const ZArgs&, const cx<T>*, BT*,   \
                                              const LongBufs<T>&, hipStream_t);                   \
  template void launch_long_z_forward<T, BT>(const LongPlan&, const ZArgs&, const BT*, cx<T>*, T, \
                                             const LongBufs<T>&, hipStream_t);                    \
  template void launch_long_y_backward<T, BT>(const LongPlan&, const YArgs&, const BT*, cx<T>*,   \
                                              const LongBufs<T>&, hipStream_t);                   \
  template void launch_long_y_forward<T, BT>(const LongPlan&, const YArgs&, cx<T>*, BT*,          \
                                             const LongBufs<T>&, hipStream_t);
SPFFT_LONG_INST(double, cx<double>)
SPFFT_LONG_INST(double, cx<float>)
SPFFT_LONG_INST(float, cx<float>)
#undef SPFFT_LONG_INST
template void launch_long_x_backward<double>(const LongPlan&, const XArgs&, bool, const cx<double>*,
                                             void*, const cx<double>*, const LongBufs<double>&,
                                             hipStream_t);
template void launch_long_x_backward<float>(const LongPlan&, const XArgs&, bool, const cx<float>*,
                                            void*, const cx<float>*, const LongBufs<float>&,
                                            hipStream_t);
template void launch_long_x_forward<double>(const LongPlan&, const XArgs&, bool, const void*,
                                            cx<double>*, const cx<double>*, const LongBufs<double>&,
                                            hipStream_t);
template void launch_long_x_forward<float>(const LongPlan&, const XArgs&, bool, const void*,
                                           cx<float>*, const cx<float>*, const LongBufs<float>&,
                                           hipStream_t);

}  // namespace dev
}  // namespace spfft
