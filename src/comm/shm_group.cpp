#include "comm/shm_group.hpp"

#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "core/common.hpp"
#include "core/fault.hpp"
#include "spfft/exceptions.hpp"

namespace spfft {

namespace {
constexpr std::size_t kHeader = 64;

std::size_t round_up(std::size_t v, std::size_t a) { return (v + a - 1) / a * a; }

bool process_alive(long long pid) { return pid <= 0 || ::kill(static_cast<pid_t>(pid), 0) == 0 || errno != ESRCH; }

// Identity of this process's pid namespace (the /proc/self/ns/pid link,
// e.g. "pid:[4026531836]"), hashed; 0 if unreadable.
unsigned long long pid_namespace_id() {
  char buf[128] = {0};
  const ssize_t n = ::readlink("/proc/self/ns/pid", buf, sizeof(buf) - 1);
  if (n <= 0) return 0;
  unsigned long long h = 1469598103934665603ull;
  for (ssize_t i = 0; i < n; ++i) h = (h ^ static_cast<unsigned char>(buf[i])) * 1099511628211ull;
  return h;
}
}  // namespace

ShmGroup::Slot* ShmGroup::slot(int q) const {
  return reinterpret_cast<Slot*>(static_cast<char*>(base_) + kHeader + static_cast<std::size_t>(q) * sizeof(Slot));
}

char* ShmGroup::payload(int parity, int q) const {
  const std::size_t slots = kHeader + static_cast<std::size_t>(P_) * sizeof(Slot);
  return static_cast<char*>(base_) + slots + (static_cast<std::size_t>(parity) * P_ + q) * stride_;
}

std::unique_ptr<ShmGroup> ShmGroup::create(Communicator& comm, std::size_t maxPayload, double timeoutSeconds) {
  const char* env = std::getenv("SPFFT_SHM_COLLECTIVES");
  if (env && *env == '0') return nullptr;
  std::unique_ptr<ShmGroup> g(new ShmGroup());
  g->me_ = comm.rank();
  g->P_ = comm.size();
  g->timeout_ = timeoutSeconds;
  g->stride_ = round_up(std::max<std::size_t>(maxPayload, 8), 64);
  g->bytes_ = kHeader + static_cast<std::size_t>(g->P_) * sizeof(Slot) + 2 * static_cast<std::size_t>(g->P_) * g->stride_;
  // rank 0 creates the segment under a fresh name and tells the others
  struct Name {
    char s[64];
  };
  Name mine{};
  int ok = 1;
  if (g->me_ == 0) {
    static std::atomic<unsigned> serial{0};
    std::random_device rd;
    std::snprintf(mine.s, sizeof(mine.s), "/spfft-%ld-%u-%08x", static_cast<long>(getpid()), serial++, rd());
    const int fd = ::shm_open(mine.s, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0 || ::ftruncate(fd, static_cast<off_t>(g->bytes_)) != 0) ok = 0;
    if (ok) {
      void* p = ::mmap(nullptr, g->bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      if (p == MAP_FAILED) ok = 0;
      else g->base_ = p;  // ftruncate zero-filled it: every epoch starts at 0
    }
    if (fd >= 0) ::close(fd);
    if (!ok) mine.s[0] = 0;
  }
  std::vector<Name> names(g->P_);
  comm.allgather(&mine, names.data(), sizeof(Name));
  const Name& name = names[0];
  if (g->me_ != 0) {
    ok = name.s[0] != 0;
    int fd = ok ? ::shm_open(name.s, O_RDWR, 0600) : -1;
    struct stat st {};
    if (fd < 0 || ::fstat(fd, &st) != 0 || static_cast<std::size_t>(st.st_size) != g->bytes_) ok = 0;
    if (ok) {
      void* p = ::mmap(nullptr, g->bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      if (p == MAP_FAILED) ok = 0;
      else g->base_ = p;
    }
    if (fd >= 0) ::close(fd);
  }
  std::vector<int> oks(g->P_);
  comm.allgather(&ok, oks.data(), sizeof(int));
  // every rank has opened (or failed to open) the name: it can go
  if (g->me_ == 0 && name.s[0]) ::shm_unlink(name.s);
  bool all = true;
  for (int v : oks) all = all && v != 0;
  if (!all) return nullptr;  // the destructor unmaps
  g->slot(g->me_)->pid.store(static_cast<long long>(getpid()), std::memory_order_relaxed);
  comm.barrier();  // every pid is published before the first wait
  // The waits detect a peer's exit by its pid, which only means something if
  // every rank sees every other rank's pid: ranks that share /dev/shm from
  // different pid namespaces (containers with a shared IPC namespace) would
  // see a peer's pid as absent, or as an unrelated process. Every rank checks
  // the namespaces and the published pids; if any check fails anywhere, the
  // group is not used (the caller falls back to the communicator).
  struct Check {
    unsigned long long ns;
    int pidsOk;
  };
  Check c{pid_namespace_id(), 1};
  // fault injection SHM_PIDNS (testing library): the last rank reports another namespace
  if (SPFFT_FAULT(SHM_PIDNS) == 1 && g->me_ == g->P_ - 1) c.ns ^= 1;
  for (int q = 0; q < g->P_; ++q) {
    const long long pid = g->slot(q)->pid.load(std::memory_order_relaxed);
    if (pid <= 0 || !process_alive(pid)) c.pidsOk = 0;
  }
  std::vector<Check> checks(g->P_);
  comm.allgather(&c, checks.data(), sizeof(Check));
  for (const Check& k : checks)
    if (!k.pidsOk || k.ns != checks[0].ns) return nullptr;
  return g;
}

ShmGroup::~ShmGroup() {
  if (base_) ::munmap(base_, bytes_);
}

void ShmGroup::barrier() {
  ++epoch_;
  slot(me_)->epoch.store(epoch_, std::memory_order_release);
  const auto t0 = std::chrono::steady_clock::now();
  auto lastCheck = t0;
  for (int q = 0; q < P_; ++q) {
    Slot* s = slot(q);
    unsigned spins = 0;
    while (s->epoch.load(std::memory_order_acquire) < epoch_) {
      if (++spins < 2048) continue;
      std::this_thread::yield();
      if ((spins & 1023) != 0) continue;
      const auto now = std::chrono::steady_clock::now();
      if (now - lastCheck < std::chrono::milliseconds(20)) continue;
      lastCheck = now;
      if (!process_alive(s->pid.load(std::memory_order_relaxed))) {
        set_error_detail("node-local barrier: rank " + std::to_string(q) + " (pid " +
                         std::to_string(s->pid.load()) + ") has exited");
        throw MPIError();
      }
      if (timeout_ > 0 && std::chrono::duration<double>(now - t0).count() > timeout_) {
        set_error_detail("node-local barrier: rank " + std::to_string(q) + " did not arrive within " +
                         std::to_string(timeout_) + " s (SPFFT_COMM_TIMEOUT)");
        throw MPIError();
      }
    }
  }
}

void ShmGroup::allgather(const void* send, void* recv, std::size_t bytes) {
  if (bytes > stride_) throw InternalError();
  // two payload areas by parity: allgather k + 2 reuses the area of k only after
  // every rank has passed the barrier of k + 1, i.e. has read k's data
  const int parity = static_cast<int>(gathers_++ & 1);
  if (bytes) std::memcpy(payload(parity, me_), send, bytes);
  barrier();
  for (int q = 0; q < P_; ++q)
    if (bytes) std::memcpy(static_cast<char*>(recv) + static_cast<std::size_t>(q) * bytes, payload(parity, q), bytes);
}

}  // namespace spfft
