#include "core/thread_pool.hpp"

#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <exception>
#include <vector>

namespace spfft {

namespace {
// Spreads a new worker over the allowed CPUs. Threads created in quick
// succession start on the creating thread's CPU, and short fork-join bursts
// never look busy long enough for the load balancer to move them: measured
// from a Python process, all eight threads of a pool ran on one CPU (no
// speed-up over one thread). Each worker moves itself to a distinct allowed
// CPU and then restores the full mask, so the kernel may still move it
// later; SPFFT_HOST_PIN=1 keeps the single-CPU binding.
void spread_worker(int index) {
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return;
  std::vector<int> cpus;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &allowed)) cpus.push_back(c);
  if (cpus.size() < 2) return;
  const int base = sched_getcpu();
  const std::size_t pos = std::find(cpus.begin(), cpus.end(), base) - cpus.begin();
  const int cpu = cpus[(pos + static_cast<std::size_t>(index)) % cpus.size()];
  cpu_set_t one;
  CPU_ZERO(&one);
  CPU_SET(cpu, &one);
  if (sched_setaffinity(0, sizeof(one), &one) != 0) return;
  sched_yield();  // migrate now
  const char* pin = std::getenv("SPFFT_HOST_PIN");
  if (!(pin && pin[0] == '1')) (void)sched_setaffinity(0, sizeof(allowed), &allowed);
}
}  // namespace

ThreadPool::ThreadPool(int numThreads) : numThreads_(std::max(1, numThreads)) {
  for (int i = 1; i < numThreads_; ++i)
    threads_.emplace_back([this, i] {
      spread_worker(i);
      worker(i);
    });
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
    // The stages of a transform are back-to-back parallel_for calls: poll for
    // the next job for a short while before sleeping, so the workers stay on
    // their cores and pick it up at once (woken from the condition variable
    // they arrive late and the calling thread ends up doing most chunks).
    const auto spinUntil = std::chrono::steady_clock::now() + std::chrono::microseconds(200);
    while (generation_.load(std::memory_order_acquire) == seen &&
           std::chrono::steady_clock::now() < spinUntil)
      std::this_thread::yield();
    {
      std::unique_lock<std::mutex> lock(mutex_);
      startCv_.wait(lock, [&] { return stop_ || generation_.load() != seen; });
      if (stop_) return;
      seen = generation_.load();
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
