// Host cost of the HIP runtime calls on the multi-transform path (us per call).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
__global__ void empty_kernel(int* p) { if (p && threadIdx.x == 1000) p[0] = 1; }
template <class F> double us(F f, int n = 2000) {
  for (int i = 0; i < 50; ++i) f();
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) f();
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}
int main() {
  void* d = nullptr;
  (void)hipMalloc(&d, 1 << 20);
  hipStream_t s[4];
  for (auto& x : s) (void)hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
  hipEvent_t e;
  (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  hipPointerAttribute_t a;
  printf("hipPointerGetAttributes %.2f us\n", us([&] { (void)hipPointerGetAttributes(&a, d); }));
  printf("hipGetLastError         %.2f us\n", us([&] { (void)hipGetLastError(); }));
  printf("hipEventRecord          %.2f us\n", us([&] { (void)hipEventRecord(e, s[1]); }));
  printf("hipStreamWaitEvent      %.2f us\n", us([&] { (void)hipStreamWaitEvent(s[0], e, 0); }));
  printf("launch (1 stream)       %.2f us\n", us([&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s[0], (int*)nullptr); }));
  int k = 0;
  printf("launch (4 streams)      %.2f us\n", us([&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s[(k++) & 3], (int*)nullptr); }));
  (void)hipDeviceSynchronize();
  return 0;
}
