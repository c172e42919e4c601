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
// f(i) for i in [0, n), grid-stride; fence: release this thread's stores
// system-wide at the end (peer-write exchange)
template <class F>
__global__ void __launch_bounds__(256) for_each_kernel(long long n, int fence, F f) {
  const long long stride = static_cast<long long>(gridDim.x) * blockDim.x;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < n; i += stride)
    f(i);
  release_remote(fence);
}

template <class F>
void for_each(long long n, hipStream_t s, F f, int fence = 0) {
  if (n <= 0) return;
  const long long blocks = std::min<long long>((n + 255) / 256, 1 << 16);
  hipLaunchKernelGGL(for_each_kernel<F>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, n,
                     fence, f);
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
struct PassArgs {
  int n1, n2;
  long long srcStride, dstStride;
  int blocksPerLine;
};

// columns pass, in place: for every column j2 of a line viewed as [n1][n2]:
// FFT_n1 over j1 -> k1, times exp(S 2 pi i j2 k1 / (n1 n2)). Lanes walk
// consecutive columns (coalesced rows of the [n1][n2] view).
template <class Eng, typename T, int S>
__global__ void __launch_bounds__(Eng::kBlock)
    long_cols_kernel(Eng eng, PassArgs a, cx<T>* data, const cx<T>* __restrict__ tw1,
                     const cx<T>* __restrict__ twM) {
  SPFFT_LDS_DECL(T);
  const int B = eng.lines();
  const long long line = blockIdx.x / a.blocksPerLine;
  const int j20 = static_cast<int>(blockIdx.x % a.blocksPerLine) * B;
  cx<T>* base = data + line * a.srcStride;
  const int total = B * a.n1;
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int b = idx % B, j1 = idx / B, j2 = j20 + b;
    lds[eng.in_at(b, j1)] = j2 < a.n2 ? base[static_cast<long long>(j1) * a.n2 + j2] : czero<T>();
  }
  __syncthreads();
  eng.lds_to_lds(lds, tw1);
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int b = idx % B, k1 = idx / B, j2 = j20 + b;
    if (j2 < a.n2)
      base[static_cast<long long>(k1) * a.n2 + j2] =
          twm<S>(lds[eng.out_at(b, k1)], twM[static_cast<long long>(j2) * k1]);
  }
}

// rows pass, out of place: for every row k1: FFT_n2 over j2 -> k2, stored at
// the natural position k1 + n1 k2 (loads walk rows, stores walk rows fastest)
template <class Eng, typename T, int S>
__global__ void __launch_bounds__(Eng::kBlock)
    long_rows_kernel(Eng eng, PassArgs a, const cx<T>* src, cx<T>* dst,
                     const cx<T>* __restrict__ tw2) {
  SPFFT_LDS_DECL(T);
  const int B = eng.lines();
  const long long line = blockIdx.x / a.blocksPerLine;
  const int k10 = static_cast<int>(blockIdx.x % a.blocksPerLine) * B;
  const cx<T>* s = src + line * a.srcStride;
  cx<T>* d = dst + line * a.dstStride;
  const int total = B * a.n2;
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int b = idx / a.n2, j2 = idx - b * a.n2, k1 = k10 + b;
    lds[eng.in_at(b, j2)] = k1 < a.n1 ? s[static_cast<long long>(k1) * a.n2 + j2] : czero<T>();
  }
  __syncthreads();
  eng.lds_to_lds(lds, tw2);
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int b = idx % B, k2 = idx / B, k1 = k10 + b;
    if (k1 < a.n1) d[k1 + static_cast<long long>(a.n1) * k2] = lds[eng.out_at(b, k2)];
  }
}

// length n1 * n2 lines: src (destroyed) -> dst, natural order both sides
template <typename T, int S>
void four_step(const LongPlan& lp, cx<T>* src, long long srcStride, cx<T>* dst, long long dstStride,
               long long lines, hipStream_t stream) {
  if (lines <= 0) return;
  with_engine<T, S, true>(lp.n1, [&](auto eng, int threads, int B, std::size_t lds) {
    PassArgs a{lp.n1, lp.n2, srcStride, srcStride, static_cast<int>(ceil_div(lp.n2, B))};
    auto k = long_cols_kernel<decltype(eng), T, S>;
    prepare_kernel(k, lds);
    hipLaunchKernelGGL(k, dim3(static_cast<unsigned>(lines * a.blocksPerLine)), dim3(threads), lds,
                       stream, eng, a, src, static_cast<const cx<T>*>(lp.tw1),
                       static_cast<const cx<T>*>(lp.twM));
    gpu_check_launch("long_cols", stream);
  });
  with_engine<T, S, true>(lp.n2, [&](auto eng, int threads, int B, std::size_t lds) {
    PassArgs a{lp.n1, lp.n2, srcStride, dstStride, static_cast<int>(ceil_div(lp.n1, B))};
    auto k = long_rows_kernel<decltype(eng), T, S>;
    prepare_kernel(k, lds);
    hipLaunchKernelGGL(k, dim3(static_cast<unsigned>(lines * a.blocksPerLine)), dim3(threads), lds,
                       stream, eng, a, src, dst, static_cast<const cx<T>*>(lp.tw2));
    gpu_check_launch("long_rows", stream);
  });
}

// one long FFT of sign S over `lines` lines: src (destroyed) -> dst
template <typename T, int S>
void long_fft(const LongPlan& lp, cx<T>* src, long long srcStride, cx<T>* dst, long long dstStride,
              long long lines, const LongBufs<T>& w, hipStream_t stream) {
  if (!lp.bluestein) {
    four_step<T, S>(lp, src, srcStride, dst, dstStride, lines, stream);
    return;
  }
  // X_k = d_k sum_j (x_j d_j) conj(d_{k-j}) (d_j = exp(S i pi j^2 / n)): one
  // cyclic convolution of length m through FFT_m(-1), the filter, FFT_m(+1)
  const int n = lp.n, m = lp.m;
  const cx<T>* chirp = static_cast<const cx<T>*>(lp.chirp);
  const cx<T>* filt = static_cast<const cx<T>*>(lp.filt) + (S < 0 ? 0 : m);
  cx<T>* w1 = w.w1;
  cx<T>* w2 = w.w2;
  for_each(lines * m, stream, [=] __device__(long long i) {
    const long long l = i / m;
    const int j = static_cast<int>(i - l * m);
    cx<T> v = czero<T>();
    if (j < n) {
      const cx<T> d = S < 0 ? chirp[j] : conj(chirp[j]);
      v = cmul(src[l * srcStride + j], d);
    }
    w1[i] = v;
  });
  four_step<T, -1>(lp, w1, m, w2, m, lines, stream);
  for_each(lines * m, stream, [=] __device__(long long i) {
    const int j = static_cast<int>(i % m);
    w2[i] = cmul(w2[i], filt[j]);
  });
  four_step<T, +1>(lp, w2, m, w1, m, lines, stream);
  const T inv = T(1) / static_cast<T>(m);
  for_each(lines * n, stream, [=] __device__(long long i) {
    const long long l = i / n;
    const int k = static_cast<int>(i - l * n);
    const cx<T> d = S < 0 ? chirp[k] : conj(chirp[k]);
    dst[l * dstStride + k] = scale(cmul(w1[l * m + k], d), inv);
  });
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
bool short_ok(int f) { return has_ct_kernel(f) || (f >= 2 && f <= 4096 && largest_prime(f) <= 13); }

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

bool needs_long_path(int n, bool dbl) {
  if (n <= 1 || has_ct_kernel(n)) return false;
  if (n > max_device_fft_length(dbl)) return true;
  if (largest_prime(n) <= kBluesteinPrime) return false;
  return !use_bluestein(n, dbl ? sizeof(cx<double>) : sizeof(cx<float>));
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
    const int score = ((has_ct_kernel(d) ? 0 : 1) + (has_ct_kernel(n / d) ? 0 : 1)) * (1 << 20) +
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
template <typename T, typename BT>
void launch_long_z_backward(const LongPlan& lp, const ZArgs& a, const cx<T>* values, BT* out,
                            const LongBufs<T>& w, hipStream_t stream) {
  const long long S = a.numSticks - a.stickBegin;
  if (S <= 0) return;
  const int n = a.n;
  const int s0 = a.stickBegin;
  cx<T>* in = w.in;
  gpu_check(hipMemsetAsync(in, 0, static_cast<std::size_t>(S) * n * sizeof(cx<T>), stream),
            "hipMemsetAsync");
  // decompress: one thread per run
  const StickRun* runs = a.runs;
  const int q0 = 0;
  (void)q0;
  const int* ro = a.runOffsets;
  // the run range of the sticks [s0, numSticks) is read on the device
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
  long_fft<T, +1>(lp, in, n, w.out, n, S, w, stream);
  const cx<T>* res = w.out;
  const ZArgs za = a;
  for_each(S * n, stream, [=] __device__(long long i) {
    const long long s = i / n;
    const int z = static_cast<int>(i - s * n);
    out[seg_index(za, s0 + static_cast<int>(s), z)] = cvt<typename BT::value_type>(res[i]);
  }, a.remote);
}

template <typename T, typename BT>
void launch_long_z_forward(const LongPlan& lp, const ZArgs& a, const BT* in, cx<T>* values, T scl,
                           const LongBufs<T>& w, hipStream_t stream) {
  const long long S = a.numSticks - a.stickBegin;
  if (S <= 0) return;
  const int n = a.n;
  const int s0 = a.stickBegin;
  cx<T>* lines = w.in;
  const ZArgs za = a;
  for_each(S * n, stream, [=] __device__(long long i) {
    const long long s = i / n;
    const int z = static_cast<int>(i - s * n);
    lines[i] = cvt<T>(in[seg_index(za, s0 + static_cast<int>(s), z)]);
  });
  long_fft<T, -1>(lp, lines, n, w.out, n, S, w, stream);
  const cx<T>* res = w.out;
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
template <typename T, typename BT>
void launch_long_y_backward(const LongPlan& lp, const YArgs& a, const BT* in, cx<T>* inter,
                            const LongBufs<T>& w, hipStream_t stream) {
  const int nz = a.L - a.zBegin;
  const int C = a.ncols, n = a.n, zb = a.zBegin;
  if (nz <= 0 || C <= 0) return;
  const long long lines = static_cast<long long>(nz) * C;
  cx<T>* lin = w.in;
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
  long_fft<T, +1>(lp, lin, n, inter + zb * a.interZStride, a.interStride, lines, w, stream);
}

template <typename T, typename BT>
void launch_long_y_forward(const LongPlan& lp, const YArgs& a, cx<T>* inter, BT* out,
                           const LongBufs<T>& w, hipStream_t stream) {
  const int nz = a.L - a.zBegin;
  const int C = a.ncols, n = a.n, zb = a.zBegin;
  if (nz <= 0 || C <= 0) return;
  const long long lines = static_cast<long long>(nz) * C;
  long_fft<T, -1>(lp, inter + zb * a.interZStride, a.interStride, w.out, n, lines, w, stream);
  const cx<T>* res = w.out;
  const int* co = a.colOffsets;
  const int* cy = a.colY;
  const long long* cb = a.colBase;
  for_each(lines, stream, [=] __device__(long long l) {
    const int zz = static_cast<int>(l / C), c = static_cast<int>(l - static_cast<long long>(zz) * C);
    const cx<T>* line = res + l * n;
    for (int k = co[c]; k < co[c + 1]; ++k)
      out[cb[k] + zb + zz] = cvt<typename BT::value_type>(line[cy[k]]);
  }, a.remote);
}

// ------------------------------------------------------------ x stage
template <typename T>
void launch_long_x_backward(const LongPlan& lp, const XArgs& a, bool r2c, const cx<T>* inter,
                            void* space, const cx<T>* twFull, const LongBufs<T>& w,
                            hipStream_t stream) {
  const int nz = a.L - a.zBegin;
  const int Y = a.Y, X = a.n, C = a.ncols, zb = a.zBegin;
  if (nz <= 0 || Y <= 0) return;
  const long long lines = static_cast<long long>(nz) * Y;
  const long long iz = a.interZStride, is = a.interStride;
  const int* colX = a.colX;
  const cx<T>* src = inter + zb * iz;
  auto scatter_cols = [&](cx<T>* dst, int rowLen) {
    gpu_check(hipMemsetAsync(dst, 0, static_cast<std::size_t>(lines) * rowLen * sizeof(cx<T>), stream),
              "hipMemsetAsync");
    for_each(lines * C, stream, [=] __device__(long long i) {
      const long long l = i / C;
      const int c = static_cast<int>(i - l * C);
      const long long zz = l / Y, y = l - zz * Y;
      dst[l * rowLen + colX[c]] = src[zz * iz + c * is + y];
    });
  };
  if (!r2c) {
    scatter_cols(w.in, X);
    long_fft<T, +1>(lp, w.in, X, static_cast<cx<T>*>(space) + static_cast<long long>(zb) * Y * X, X,
                    lines, w, stream);
  } else if (X % 2 == 0) {
    // packed real rows: Z[k] = (X[k] + conj X[h-k]) + i (X[k] - conj X[h-k]) w^k,
    // w = exp(+2 pi i / X), imaginary parts of X[0], X[h] ignored; IDFT_h(Z)
    // interleaves the real row
    const int h = X / 2;
    cx<T>* half = w.out;  // X[0..h] per line (stride h + 1)
    scatter_cols(half, h + 1);
    cx<T>* z = w.in;
    for_each(lines * h, stream, [=] __device__(long long i) {
      const long long l = i / h;
      const int k = static_cast<int>(i - l * h);
      cx<T> xk = half[l * (h + 1) + k], xm = half[l * (h + 1) + (h - k)];
      if (k == 0) {
        xk.y = T(0);
        xm.y = T(0);
      }
      const cx<T> xmc = conj(xm);
      z[i] = (xk + xmc) + rot<+1>(twm<+1>(xk - xmc, twFull[k]));
    });
    long_fft<T, +1>(lp, z, h, reinterpret_cast<cx<T>*>(static_cast<T*>(space) + static_cast<long long>(zb) * Y * X), h,
                    lines, w, stream);
  } else {
    const int nf = a.nFreq;
    cx<T>* full = w.in;
    scatter_cols(full, X);
    for_each(lines * X, stream, [=] __device__(long long i) {
      const long long l = i / X;
      const int x = static_cast<int>(i - l * X);
      if (x >= nf) full[i] = conj(full[l * X + (X - x)]);
    });
    long_fft<T, +1>(lp, full, X, w.out, X, lines, w, stream);
    const cx<T>* res = w.out;
    T* dst = static_cast<T*>(space) + static_cast<long long>(zb) * Y * X;
    for_each(lines * X, stream, [=] __device__(long long i) { dst[i] = res[i].x; });
  }
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
  const int* colX = a.colX;
  cx<T>* dst = inter + zb * iz;
  auto gather_cols = [&](const cx<T>* res, int rowLen) {
    for_each(lines * C, stream, [=] __device__(long long i) {
      const long long l = i / C;
      const int c = static_cast<int>(i - l * C);
      const long long zz = l / Y, y = l - zz * Y;
      dst[zz * iz + c * is + y] = res[l * rowLen + colX[c]];
    });
  };
  if (!r2c) {
    // the space domain stays intact: the four-step destroys its input
    gpu_check(hipMemcpyAsync(w.in, static_cast<const cx<T>*>(space) + static_cast<long long>(zb) * Y * X,
                             static_cast<std::size_t>(lines) * X * sizeof(cx<T>),
                             hipMemcpyDeviceToDevice, stream),
              "hipMemcpyAsync");
    long_fft<T, -1>(lp, w.in, X, w.out, X, lines, w, stream);
    gather_cols(w.out, X);
  } else if (X % 2 == 0) {
    // packed real rows y[m] = x[2m] + i x[2m+1]: X[k] = (Y[k] + conj Y[h-k]) / 2
    // + w^k (Y[k] - conj Y[h-k]) / (2i), w = exp(-2 pi i / X), Y[h] = Y[0]
    const int h = X / 2;
    gpu_check(hipMemcpyAsync(w.in, static_cast<const T*>(space) + static_cast<long long>(zb) * Y * X,
                             static_cast<std::size_t>(lines) * X * sizeof(T), hipMemcpyDeviceToDevice,
                             stream),
              "hipMemcpyAsync");
    long_fft<T, -1>(lp, w.in, h, w.out, h, lines, w, stream);
    const cx<T>* res = w.out;
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
    const T* sp = static_cast<const T*>(space) + static_cast<long long>(zb) * Y * X;
    cx<T>* lin = w.in;
    for_each(lines * X, stream, [=] __device__(long long i) { lin[i] = mk<T>(sp[i], T(0)); });
    long_fft<T, -1>(lp, lin, X, w.out, X, lines, w, stream);
    gather_cols(w.out, X);
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
