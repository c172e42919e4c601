// Probe: how ROCm implements hipStreamWaitValue64 / hipStreamWriteValue64 on
// ordinary device memory (VERDICT r4 item 2 proposed them for the peer
// barrier). Run under `rocprofv3 --kernel-trace --stats`: a wait that the CP
// executes leaves no kernel in the trace; a blit kernel shows up by name.
// Also measures the write -> wait release latency over 200 rounds.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));                      \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

__global__ void marker(int* out, int v) {
  if (threadIdx.x == 0) out[0] = v;
}

int main() {
  unsigned long long* flag = nullptr;
  int* out = nullptr;
  CHECK(hipMalloc(&flag, 64));
  CHECK(hipMemset(flag, 0, 64));
  CHECK(hipMalloc(&out, 64));
  hipStream_t a, b;
  CHECK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  // 1. a waits, the host sleeps, b writes: is a still blocked before the write?
  CHECK(hipStreamWaitValue64(a, flag, 1, hipStreamWaitValueGte, ~0ull));
  hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, a, out, 1);
  usleep(200000);
  const hipError_t q = hipStreamQuery(a);
  std::printf("stream blocked on the wait before the write: %s\n", q == hipErrorNotReady ? "yes" : "no");
  CHECK(hipStreamWriteValue64(b, flag, 1, 0));
  CHECK(hipStreamSynchronize(a));
  // 2. release latency: round i waits for i on a, b writes i
  const int rounds = 200;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 2; i < rounds + 2; ++i) {
    CHECK(hipStreamWaitValue64(a, flag, i, hipStreamWaitValueGte, ~0ull));
    hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, a, out, i);
    CHECK(hipStreamWriteValue64(b, flag, i, 0));
    CHECK(hipStreamSynchronize(a));
  }
  auto t1 = std::chrono::steady_clock::now();
  std::printf("write -> wait -> kernel -> host, per round: %.1f us\n",
              std::chrono::duration<double, std::micro>(t1 - t0).count() / rounds);
  return 0;
}
