// MFMA vs VALU for the radix-16 DFT tiles of the stage kernels (SURVEY.md §7.5.1:
// "small DFT tiles as MFMA matmuls is an experiment; prove any gain with counters").
//
// A DFT-16 over 16 lines is the complex matrix product Y = W X (W 16x16, X 16 points
// x 16 lines): 4 real products, each 4 K-steps of a 16x16x4 MFMA -> 16 MFMAs per wave
// and 16 lines. The VALU form is the radix-16 codelet the FFT engines use (one line
// per lane, 64 lines per wave). Both iterate on register-resident data, so the
// numbers are pure compute throughput (the scaling by 1/4 keeps the iteration
// unitary). A layout self-test checks the MFMA operand/result lane mapping first.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I src tools/probes/mfma_dft.hip -o mfma_dft
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fft/codelets.hpp"

using namespace spfft;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <typename T>
struct Mfma;
template <>
struct Mfma<double> {
  using V = d4;
  __device__ static V run(double a, double b, V c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
};
template <>
struct Mfma<float> {
  using V = f4;
  __device__ static V run(float a, float b, V c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
};

// D = A B for 16x16 A, B (row-major in global), K = 16 in 4 steps. Lane l supplies
// A[l%16][4s + l/16] and B[4s + l/16][l%16]; writes its 4 result values raw.
template <typename T>
__global__ void layout_test(const T* A, const T* B, T* out) {
  const int l = threadIdx.x, i = l & 15, q = l >> 4;
  typename Mfma<T>::V c = {0, 0, 0, 0};
  for (int s = 0; s < 4; ++s) c = Mfma<T>::run(A[i * 16 + 4 * s + q], B[(4 * s + q) * 16 + i], c);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

// One wave = 16 lines. Lane (q = l/16, j = l%16) holds points 4s+q (s = 0..3) of
// line j; after a step it holds points 4q+r (r = 0..3), fed back as the next input
// (a fixed permutation of each line: the iteration stays unitary).
template <typename T, int S>
__global__ void __launch_bounds__(256) dft16_mfma(const cx<T>* in, cx<T>* out, int iters, int layout) {
  using V = typename Mfma<T>::V;
  const int lane = threadIdx.x & 63, q = lane >> 4, j = lane & 15;
  const long long wave = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
  T wr[4], wi[4], wn[4];
  for (int s = 0; s < 4; ++s) {
    const int e = (j * (4 * s + q)) & 15;
    const double a = S * 2.0 * 3.14159265358979323846 * e / 16.0;
    wr[s] = static_cast<T>(std::cos(a) * 0.25);
    wi[s] = static_cast<T>(std::sin(a) * 0.25);
    wn[s] = -wi[s];
  }
  T xr[4], xi[4];
  for (int s = 0; s < 4; ++s) {
    const cx<T> v = in[wave * 256 + j * 16 + 4 * s + q];
    xr[s] = v.x;
    xi[s] = v.y;
  }
  for (int it = 0; it < iters; ++it) {
    V yr = {0, 0, 0, 0}, yi = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      yr = Mfma<T>::run(wr[s], xr[s], yr);
      yr = Mfma<T>::run(wn[s], xi[s], yr);
      yi = Mfma<T>::run(wr[s], xi[s], yi);
      yi = Mfma<T>::run(wi[s], xr[s], yi);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      xr[r] = yr[r];
      xi[r] = yi[r];
    }
  }
  // result: lane holds points 4q+r (layout 0) or q+4r (layout 1) of line j
  for (int r = 0; r < 4; ++r)
    out[wave * 256 + j * 16 + (layout == 1 ? q + 4 * r : 4 * q + r)] = mk<T>(xr[r], xi[r]);
}

// One lane = one line of 16 points (the engines' radix-16 codelet).
template <typename T, int S>
__global__ void __launch_bounds__(256) dft16_valu(const cx<T>* in, cx<T>* out, int iters) {
  const long long line = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  cx<T> v[16];
  for (int k = 0; k < 16; ++k) v[k] = in[line * 16 + k];
  for (int it = 0; it < iters; ++it) {
    Dft<16, S, T>::run(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = scale(v[k], static_cast<T>(0.25));
  }
  for (int k = 0; k < 16; ++k) out[line * 16 + k] = v[k];
}

template <typename T>
static void host_dft16(const cx<T>* x, cx<double>* y, int S) {
  for (int k = 0; k < 16; ++k) {
    double re = 0, im = 0;
    for (int n = 0; n < 16; ++n) {
      const double a = S * 2.0 * M_PI * ((n * k) % 16) / 16.0;
      re += x[n].x * std::cos(a) - x[n].y * std::sin(a);
      im += x[n].x * std::sin(a) + x[n].y * std::cos(a);
    }
    y[k] = mk<double>(re * 0.25, im * 0.25);
  }
}

template <typename T>
static int run(const char* name, double tol) {
  int layout = 0;
  // ---- layout self-test
  {
    std::vector<T> A(256), B(256), out(256);
    for (int i = 0; i < 256; ++i) {
      A[i] = static_cast<T>((i * 37 % 101) / 101.0 - 0.5);
      B[i] = static_cast<T>((i * 53 % 97) / 97.0 - 0.5);
    }
    T *dA, *dB, *dO;
    CK(hipMalloc(&dA, 256 * sizeof(T)));
    CK(hipMalloc(&dB, 256 * sizeof(T)));
    CK(hipMalloc(&dO, 256 * sizeof(T)));
    CK(hipMemcpy(dA, A.data(), 256 * sizeof(T), hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), 256 * sizeof(T), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(layout_test<T>, dim3(1), dim3(64), 0, 0, dA, dB, dO);
    CK(hipMemcpy(out.data(), dO, 256 * sizeof(T), hipMemcpyDeviceToHost));
    // candidate result mappings: lane l, value r -> D[row][col] (j = l % 16, q = l / 16)
    const char* names[4] = {"D[4q+r][j]", "D[q+4r][j]", "D[j][4q+r]", "D[j][q+4r]"};
    double errs[4] = {0, 0, 0, 0};
    for (int m = 0; m < 4; ++m)
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
          const int q = l >> 4, jj = l & 15;
          int row = 0, col = 0;
          if (m == 0) { row = 4 * q + r; col = jj; }
          if (m == 1) { row = q + 4 * r; col = jj; }
          if (m == 2) { row = jj; col = 4 * q + r; }
          if (m == 3) { row = jj; col = q + 4 * r; }
          double d = 0;
          for (int k = 0; k < 16; ++k) d += static_cast<double>(A[row * 16 + k]) * B[k * 16 + col];
          errs[m] = std::fmax(errs[m], std::fabs(d - out[l * 4 + r]));
        }
    layout = -1;
    for (int m = 0; m < 4; ++m) {
      std::printf("[%s] mfma 16x16x4 result layout %-11s max err %.3e\n", name, names[m], errs[m]);
      if (layout < 0 && errs[m] < tol * 16) layout = m;
    }
    const double err = layout < 0 ? 1.0 : errs[layout];
    std::printf("[%s] layout: %s\n", name, layout < 0 ? "NONE MATCHES" : names[layout]);
    CK(hipFree(dA));
    CK(hipFree(dB));
    CK(hipFree(dO));
    if (err >= tol * 16) return 1;
  }
  // ---- correctness (1 iteration) and throughput
  const int blocks = 256 * 8, threads = 256;  // 8 waves per SIMD
  const long long lanes = static_cast<long long>(blocks) * threads;
  const long long valuLines = lanes, mfmaLines = lanes / 64 * 16;
  const long long elems = valuLines * 16;
  std::vector<cx<T>> h(elems);
  for (long long i = 0; i < elems; ++i)
    h[i] = mk<T>(static_cast<T>(std::sin(0.37 * i)), static_cast<T>(std::cos(0.11 * i)));
  cx<T> *din, *dout;
  CK(hipMalloc(&din, elems * sizeof(cx<T>)));
  CK(hipMalloc(&dout, elems * sizeof(cx<T>)));
  CK(hipMemcpy(din, h.data(), elems * sizeof(cx<T>), hipMemcpyHostToDevice));
  std::vector<cx<T>> o(elems);
  std::vector<cx<double>> ref(16);
  // VALU check
  hipLaunchKernelGGL((dft16_valu<T, -1>), dim3(blocks), dim3(threads), 0, 0, din, dout, 1);
  CK(hipMemcpy(o.data(), dout, elems * sizeof(cx<T>), hipMemcpyDeviceToHost));
  double ev = 0, em = 0;
  for (int line = 0; line < 64; ++line) {
    host_dft16(&h[line * 16], ref.data(), -1);
    for (int k = 0; k < 16; ++k)
      ev = std::fmax(ev, std::hypot(o[line * 16 + k].x - ref[k].x, o[line * 16 + k].y - ref[k].y));
  }
  // MFMA check: wave w, line j holds in[w*256 + j*16 + n]; output same indexing
  if (layout > 1) return 1;  // the DFT kernel assumes row = point index
  hipLaunchKernelGGL((dft16_mfma<T, -1>), dim3(blocks), dim3(threads), 0, 0, din, dout, 1, layout);
  CK(hipMemcpy(o.data(), dout, elems * sizeof(cx<T>), hipMemcpyDeviceToHost));
  for (int line = 0; line < 64; ++line) {
    host_dft16(&h[line * 16], ref.data(), -1);
    for (int k = 0; k < 16; ++k)
      em = std::fmax(em, std::hypot(o[line * 16 + k].x - ref[k].x, o[line * 16 + k].y - ref[k].y));
  }
  std::printf("[%s] DFT-16 check: valu err %.3e, mfma err %.3e %s\n", name, ev, em,
              (ev < tol && em < tol) ? "OK" : "FAIL");
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 2000;
  auto timeit = [&](auto kernel, auto... extra) {
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(threads), 0, 0, din, dout, 10, extra...);
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(threads), 0, 0, din, dout, iters, extra...);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e-3;
  };
  const double tv = timeit(dft16_valu<T, -1>);
  const double tm = timeit(dft16_mfma<T, -1>, layout);
  const double rv = valuLines * static_cast<double>(iters) / tv;
  const double rm = mfmaLines * static_cast<double>(iters) / tm;
  // 256^3 sphere z stage: 51431 sticks x 2 radix-16 passes x 16 DFT-16 per pass
  const double zDfts = 51431.0 * 32.0;
  std::printf("[%s] VALU: %.3e DFT-16/s (%.1f TFLOP/s at 5N log2 N) -> 256^3 z-stage DFTs in %.1f us\n",
              name, rv, rv * 320e-12, zDfts / rv * 1e6);
  std::printf("[%s] MFMA: %.3e DFT-16/s (%.1f TFLOP/s matrix rate) -> 256^3 z-stage DFTs in %.1f us\n",
              name, rm, rm * 2048e-12, zDfts / rm * 1e6);
  std::printf("[%s] MFMA / VALU DFT-16 throughput: %.3f\n", name, rm / rv);
  CK(hipFree(din));
  CK(hipFree(dout));
  return (ev < tol && em < tol) ? 0 : 1;
}

int main() {
  int rc = run<double>("fp64", 1e-12);
  rc |= run<float>("fp32", 1e-5);
  return rc;
}
