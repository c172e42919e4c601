// Minimal fork-join thread pool for the host engine (replaces the OpenMP
// parallel regions of the reference, src/execution/execution_host.cpp:249-352;
// avoids mixing OpenMP runtimes with PyTorch inside one process).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace spfft {

class ThreadPool {
public:
  explicit ThreadPool(int numThreads);
  ~ThreadPool();
  ThreadPool(const ThreadPool&) = delete;
  ThreadPool& operator=(const ThreadPool&) = delete;

  int num_threads() const { return numThreads_; }

  // Calls fn(begin, end, threadIndex) on disjoint chunks covering [0, n).
  // Chunks have at most `grain` items. Blocks until all chunks completed.
  void parallel_for(std::int64_t n, std::int64_t grain,
                    const std::function<void(std::int64_t, std::int64_t, int)>& fn);

private:
  void worker(int index);
  void run_chunks(int index);

  int numThreads_;
  std::vector<std::thread> threads_;
  std::mutex mutex_;
  std::condition_variable startCv_, doneCv_;
  const std::function<void(std::int64_t, std::int64_t, int)>* job_ = nullptr;
  std::int64_t jobN_ = 0, jobGrain_ = 1;
  std::atomic<std::int64_t> next_{0};
  std::atomic<std::uint64_t> generation_{0};
  int running_ = 0;
  bool stop_ = false;
  std::exception_ptr error_;
};

}  // namespace spfft
