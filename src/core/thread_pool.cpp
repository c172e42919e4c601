#include "core/thread_pool.hpp"

#include <algorithm>
#include <exception>

namespace spfft {

ThreadPool::ThreadPool(int numThreads) : numThreads_(std::max(1, numThreads)) {
  for (int i = 1; i < numThreads_; ++i) threads_.emplace_back([this, i] { worker(i); });
}

ThreadPool::~ThreadPool() {
  {
    std::lock_guard<std::mutex> lock(mutex_);
    stop_ = true;
  }
  startCv_.notify_all();
  for (auto& t : threads_) t.join();
}

void ThreadPool::run_chunks(int index) {
  for (;;) {
    const std::int64_t b = next_.fetch_add(jobGrain_);
    if (b >= jobN_) break;
    const std::int64_t e = std::min(jobN_, b + jobGrain_);
    try {
      (*job_)(b, e, index);
    } catch (...) {
      std::lock_guard<std::mutex> lock(mutex_);
      if (!error_) error_ = std::current_exception();
      next_.store(jobN_);
    }
  }
}

void ThreadPool::worker(int index) {
  std::uint64_t seen = 0;
  for (;;) {
    {
      std::unique_lock<std::mutex> lock(mutex_);
      startCv_.wait(lock, [&] { return stop_ || generation_ != seen; });
      if (stop_) return;
      seen = generation_;
    }
    run_chunks(index);
    {
      std::lock_guard<std::mutex> lock(mutex_);
      if (--running_ == 0) doneCv_.notify_all();
    }
  }
}

void ThreadPool::parallel_for(std::int64_t n, std::int64_t grain,
                              const std::function<void(std::int64_t, std::int64_t, int)>& fn) {
  if (n <= 0) return;
  grain = std::max<std::int64_t>(1, grain);
  if (numThreads_ == 1 || n <= grain) {
    for (std::int64_t b = 0; b < n; b += grain) fn(b, std::min(n, b + grain), 0);
    return;
  }
  {
    std::lock_guard<std::mutex> lock(mutex_);
    job_ = &fn;
    jobN_ = n;
    jobGrain_ = grain;
    next_.store(0);
    error_ = nullptr;
    running_ = numThreads_ - 1;
    ++generation_;
  }
  startCv_.notify_all();
  run_chunks(0);
  std::exception_ptr err;
  {
    std::unique_lock<std::mutex> lock(mutex_);
    doneCv_.wait(lock, [&] { return running_ == 0; });
    job_ = nullptr;
    err = error_;
    error_ = nullptr;
  }
  if (err) std::rethrow_exception(err);
}

}  // namespace spfft
