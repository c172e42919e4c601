// Device code of the fused stage kernels (included by z/y/x_stage.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "gpu/gpu_runtime.hpp"
#include "kernels/fft_device.hpp"
#include "kernels/stage_args.hpp"
#include "fft/fft_plan.hpp"

namespace spfft {
namespace dev {

// ------------------------------------------------------------ engine adapters
template <typename T, int N, int S>
struct CtEng {
  using F = FftCT<T, N, S>;
  __device__ int lines() const { return F::B; }
  __device__ int n() const { return N; }
  __device__ int in_at(int b, int pos) const { return F::in_at(b, pos); }
  __device__ int out_at(int b, int pos) const { return F::out_at(b, pos); }
  __device__ int input_elems() const { return F::B * F::LS; }
  template <class St>
  __device__ void lds_to_global(cx<T>* lds, const cx<T>* __restrict__ tw, St st) const {
    F::run(lds, tw, NoLoad{}, st);
  }
  template <class Ld>
  __device__ void global_to_lds(cx<T>* lds, const cx<T>* __restrict__ tw, Ld ld) const {
    F::run_to_lds(lds, tw, ld);
  }
  // host side
  static int h_lines() { return F::B; }
  static int h_threads() { return F::NT; }
  static std::size_t h_lds() { return F::lds_bytes(); }
};

template <typename T, int S>
struct RtEng {
  RtPlan p;
  __device__ int lines() const { return p.lines; }
  __device__ int n() const { return p.n; }
  __device__ int in_at(int b, int pos) const { return b * p.ls + pos; }
  __device__ int out_at(int b, int pos) const {
    return ((p.np & 1) ? p.lines * p.ls : 0) + b * p.ls + pos;
  }
  __device__ int input_elems() const { return p.lines * p.ls; }
  template <class St>
  __device__ void lds_to_global(cx<T>* lds, const cx<T>* __restrict__ tw, St st) const {
    const cx<T>* res = FftRT<T, S>::run_in_lds(p, lds, tw);
    const int total = p.lines * p.n;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
      const int b = idx / p.n, pos = idx - b * p.n;
      st(b, pos, res[b * p.ls + pos]);
    }
  }
  template <class Ld>
  __device__ void global_to_lds(cx<T>* lds, const cx<T>* __restrict__ tw, Ld ld) const {
    const int total = p.lines * p.n;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
      const int b = idx / p.n, pos = idx - b * p.n;
      lds[b * p.ls + pos] = ld(b, pos);
    }
    __syncthreads();
    FftRT<T, S>::run_in_lds(p, lds, tw);
  }
};

template <typename To, typename From>
__device__ __forceinline__ cx<To> cvt(const cx<From>& v) {
  return mk<To>(static_cast<To>(v.x), static_cast<To>(v.y));
}
template <typename T>
__device__ __forceinline__ bool nonzero(const cx<T>& v) {
  return v.x != T(0) || v.y != T(0);
}
template <typename T>
__device__ __forceinline__ cx<T> czero() {
  return mk<T>(T(0), T(0));
}

// Hermitian completion (only where the source is non-zero) of `count` LDS lines
// starting at line b0, with the two half passes of the reference
// (src/symmetry/gpu_kernels/symmetry_kernels.cu:56-78, 119-141) as two
// barrier-separated phases of one workgroup.
template <class Eng, typename T>
__device__ void hermitian_lines(const Eng& eng, cx<T>* lds, int b0, int count, int n) {
  const int h1 = n / 2;          // k in [1, n/2]
  const int h2 = n - 1 - h1;     // k in [n/2+1, n-1]
  for (int idx = threadIdx.x; idx < count * h1; idx += blockDim.x) {
    const int b = b0 + idx / h1, k = 1 + idx % h1;
    const cx<T> v = lds[eng.in_at(b, k)];
    if (nonzero(v)) lds[eng.in_at(b, n - k)] = conj(v);
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < count * h2; idx += blockDim.x) {
    const int b = b0 + idx / h2, k = h1 + 1 + idx % h2;
    const cx<T> v = lds[eng.in_at(b, k)];
    if (nonzero(v)) lds[eng.in_at(b, n - k)] = conj(v);
  }
  __syncthreads();
}

template <typename T>
__device__ __forceinline__ void zero_lds(cx<T>* lds, int count) {
  for (int i = threadIdx.x; i < count; i += blockDim.x) lds[i] = czero<T>();
}

__device__ __forceinline__ long long seg_index(const ZArgs& a, int s, int pos) {
  if (a.single) return static_cast<long long>(s) * a.n + pos;
  const int r = a.zRank[pos];
  return a.segDispl[r] + static_cast<long long>(s) * a.segStride[r] + (pos - a.segZOff[r]);
}

#define SPFFT_LDS_DECL(T)                                         \
  extern __shared__ __attribute__((aligned(16))) char spfftSmem[]; \
  cx<T>* lds = reinterpret_cast<cx<T>*>(spfftSmem)

// ---------------------------------------------------------------- z stage
template <class Eng, typename T, typename BT>
__global__ void __launch_bounds__(kMaxThreads)
    z_backward_kernel(Eng eng, ZArgs a, const cx<T>* __restrict__ values, BT* __restrict__ out,
                      const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  const int B = eng.lines();
  const int s0 = blockIdx.x * B;
  zero_lds(lds, eng.input_elems());
  __syncthreads();
  // decompress: one wave per stick, lanes stride the runs (coalesced value reads)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  for (int b = wave; b < B; b += nw) {
    const int s = s0 + b;
    if (s >= a.numSticks) break;
    const int q1 = a.runOffsets[s + 1];
    for (int q = a.runOffsets[s]; q < q1; ++q) {
      const StickRun r = a.runs[q];
      for (int j = lane; j < r.length; j += 64)
        lds[eng.in_at(b, r.zStart + j)] = values[r.valueStart + j];
    }
  }
  __syncthreads();
  if (a.zeroStick >= s0 && a.zeroStick < s0 + B) hermitian_lines(eng, lds, a.zeroStick - s0, 1, a.n);
  eng.lds_to_global(lds, tw, [&](int b, int pos, cx<T> v) {
    const int s = s0 + b;
    if (s < a.numSticks) out[seg_index(a, s, pos)] = cvt<typename BT::value_type>(v);
  });
}

template <class Eng, typename T, typename BT>
__global__ void __launch_bounds__(kMaxThreads)
    z_forward_kernel(Eng eng, ZArgs a, const BT* __restrict__ in, cx<T>* __restrict__ values,
                     T scale, const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  const int B = eng.lines();
  const int s0 = blockIdx.x * B;
  eng.global_to_lds(lds, tw, [&](int b, int pos) -> cx<T> {
    const int s = s0 + b;
    if (s >= a.numSticks) return czero<T>();
    return cvt<T>(in[seg_index(a, s, pos)]);
  });
  // compress (+ scaling): one wave per stick
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  for (int b = wave; b < B; b += nw) {
    const int s = s0 + b;
    if (s >= a.numSticks) break;
    const int q1 = a.runOffsets[s + 1];
    for (int q = a.runOffsets[s]; q < q1; ++q) {
      const StickRun r = a.runs[q];
      for (int j = lane; j < r.length; j += 64)
        values[r.valueStart + j] = spfft::scale(lds[eng.out_at(b, r.zStart + j)], scale);
    }
  }
}

// ---------------------------------------------------------------- y stage
template <class Eng, typename T, typename BT>
__global__ void __launch_bounds__(kMaxThreads)
    y_backward_kernel(Eng eng, YArgs a, const BT* __restrict__ in, cx<T>* __restrict__ inter,
                      const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  const int B = eng.lines();
  const int c = blockIdx.x;
  const int z0 = blockIdx.y * B;
  zero_lds(lds, eng.input_elems());
  __syncthreads();
  const int k0 = a.colOffsets[c];
  const int ne = a.colOffsets[c + 1] - k0;
  for (int idx = threadIdx.x; idx < ne * B; idx += blockDim.x) {
    const int e = idx / B, zz = idx - e * B;
    if (z0 + zz < a.L) lds[eng.in_at(zz, a.colY[k0 + e])] = cvt<T>(in[a.colBase[k0 + e] + z0 + zz]);
  }
  __syncthreads();
  if (c == a.colOfX0) hermitian_lines(eng, lds, 0, B, a.n);
  eng.lds_to_global(lds, tw, [&](int b, int pos, cx<T> v) {
    const int z = z0 + b;
    if (z < a.L) inter[(static_cast<long long>(z) * a.ncols + c) * a.n + pos] = v;
  });
}

template <class Eng, typename T, typename BT>
__global__ void __launch_bounds__(kMaxThreads)
    y_forward_kernel(Eng eng, YArgs a, const cx<T>* __restrict__ inter, BT* __restrict__ out,
                     const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  const int B = eng.lines();
  const int c = blockIdx.x;
  const int z0 = blockIdx.y * B;
  eng.global_to_lds(lds, tw, [&](int b, int pos) -> cx<T> {
    const int z = z0 + b;
    if (z >= a.L) return czero<T>();
    return inter[(static_cast<long long>(z) * a.ncols + c) * a.n + pos];
  });
  const int k0 = a.colOffsets[c];
  const int ne = a.colOffsets[c + 1] - k0;
  for (int idx = threadIdx.x; idx < ne * B; idx += blockDim.x) {
    const int e = idx / B, zz = idx - e * B;
    if (z0 + zz < a.L)
      out[a.colBase[k0 + e] + z0 + zz] = cvt<typename BT::value_type>(lds[eng.out_at(zz, a.colY[k0 + e])]);
  }
}

// ---------------------------------------------------------------- x stage
template <class Eng, typename T, bool R2C>
__global__ void __launch_bounds__(kMaxThreads)
    x_backward_kernel(Eng eng, XArgs a, const cx<T>* __restrict__ inter, void* __restrict__ space,
                      const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  const int B = eng.lines();
  const int zl = blockIdx.y;
  const int y0 = blockIdx.x * B;
  zero_lds(lds, eng.input_elems());
  __syncthreads();
  const cx<T>* src = inter + static_cast<long long>(zl) * a.ncols * a.Y;
  for (int idx = threadIdx.x; idx < a.ncols * B; idx += blockDim.x) {
    const int c = idx / B, yy = idx - c * B;
    if (y0 + yy < a.Y) lds[eng.in_at(yy, a.colX[c])] = src[static_cast<long long>(c) * a.Y + y0 + yy];
  }
  __syncthreads();
  if (R2C) {
    const int ext = a.n - a.nFreq;
    for (int idx = threadIdx.x; idx < B * ext; idx += blockDim.x) {
      const int yy = idx / ext, x = a.nFreq + idx % ext;
      lds[eng.in_at(yy, x)] = conj(lds[eng.in_at(yy, a.n - x)]);
    }
    __syncthreads();
  }
  eng.lds_to_global(lds, tw, [&](int b, int pos, cx<T> v) {
    const int y = y0 + b;
    if (y < a.Y) {
      const long long row = (static_cast<long long>(zl) * a.Y + y) * a.n;
      if (R2C)
        static_cast<T*>(space)[row + pos] = v.x;
      else
        static_cast<cx<T>*>(space)[row + pos] = v;
    }
  });
}

template <class Eng, typename T, bool R2C>
__global__ void __launch_bounds__(kMaxThreads)
    x_forward_kernel(Eng eng, XArgs a, const void* __restrict__ space, cx<T>* __restrict__ inter,
                     const cx<T>* __restrict__ tw) {
  SPFFT_LDS_DECL(T);
  const int B = eng.lines();
  const int zl = blockIdx.y;
  const int y0 = blockIdx.x * B;
  eng.global_to_lds(lds, tw, [&](int b, int pos) -> cx<T> {
    const int y = y0 + b;
    if (y >= a.Y) return czero<T>();
    const long long row = (static_cast<long long>(zl) * a.Y + y) * a.n;
    if (R2C) return mk<T>(static_cast<const T*>(space)[row + pos], T(0));
    return static_cast<const cx<T>*>(space)[row + pos];
  });
  cx<T>* dst = inter + static_cast<long long>(zl) * a.ncols * a.Y;
  for (int idx = threadIdx.x; idx < a.ncols * B; idx += blockDim.x) {
    const int c = idx / B, yy = idx - c * B;
    if (y0 + yy < a.Y) dst[static_cast<long long>(c) * a.Y + y0 + yy] = lds[eng.out_at(yy, a.colX[c])];
  }
}

// ------------------------------------------------------------ host helpers
RtPlan make_rt_plan(int n, std::size_t elemBytes);

template <class K>
inline void prepare_kernel(K kernel, std::size_t ldsBytes) {
  if (ldsBytes > 64 * 1024) {
    gpu_check(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(ldsBytes)),
              "hipFuncSetAttribute");
  }
}

// Calls f(engine, threads, lines, ldsBytes) with the CT engine of length n if
// there is one, else with the RT engine.
template <typename T, int S, class F>
inline void with_engine(int n, F&& f) {
  switch (n) {
#define SPFFT_CT_CASE(NN)                                                         \
  case NN: {                                                                      \
    using E = CtEng<T, NN, S>;                                                    \
    f(E{}, E::h_threads(), E::h_lines(), E::h_lds());                             \
    return;                                                                       \
  }
    SPFFT_CT_CASE(16)
    SPFFT_CT_CASE(32)
    SPFFT_CT_CASE(64)
    SPFFT_CT_CASE(128)
    SPFFT_CT_CASE(256)
    SPFFT_CT_CASE(512)
    SPFFT_CT_CASE(1024)
#undef SPFFT_CT_CASE
    default: {
      RtEng<T, S> e{make_rt_plan(n, sizeof(cx<T>))};
      f(e, kMaxThreads, e.p.lines, std::size_t(2) * e.p.lines * e.p.ls * sizeof(cx<T>));
      return;
    }
  }
}

inline unsigned ceil_div(long long a, long long b) { return static_cast<unsigned>((a + b - 1) / b); }

}  // namespace dev
}  // namespace spfft
