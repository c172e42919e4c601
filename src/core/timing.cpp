#include "core/timing.hpp"

#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <vector>

namespace spfft {
namespace timing {
namespace {

struct Node {
  std::string name;
  Node* parent = nullptr;
  std::map<std::string, std::unique_ptr<Node>> children;
  std::vector<double> samples;  // seconds
};

struct Registry {
  std::mutex mutex;
  Node root;
  std::atomic<int> level{0};
  Registry() {
    // SPFFT_TIMING=1 (or any value but 0 / host): host scopes and GPU stage
    // events; SPFFT_TIMING=host: host scopes only
    const char* env = std::getenv("SPFFT_TIMING");
    const std::string v = env ? env : "";
    level = v.empty() || v == "0" ? 0 : (v == "host" ? 1 : 2);
    root.name = "root";
  }
};

Registry& registry() {
  static Registry r;
  return r;
}

thread_local std::vector<Node*> tlsStack;

// roctx is resolved lazily so the library has no hard dependency on it.
using PushFn = int (*)(const char*);
using PopFn = int (*)();
struct Roctx {
  PushFn push = nullptr;
  PopFn pop = nullptr;
  Roctx() {
    const char* off = std::getenv("SPFFT_NO_ROCTX");
    if (off && off[0] == '1') return;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
    pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
    if (!push || !pop) push = nullptr, pop = nullptr;
  }
};
Roctx& roctx() {
  static Roctx r;
  return r;
}

long long now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Stats {
  std::size_t count = 0;
  double total = 0, mean = 0, median = 0, min = 0, max = 0;
};

Stats stats_of(std::vector<double> s) {
  Stats st;
  st.count = s.size();
  if (s.empty()) return st;
  std::sort(s.begin(), s.end());
  for (double v : s) st.total += v;
  st.mean = st.total / s.size();
  st.median = s.size() % 2 ? s[s.size() / 2] : 0.5 * (s[s.size() / 2 - 1] + s[s.size() / 2]);
  st.min = s.front();
  st.max = s.back();
  return st;
}

double node_total(const Node& n) {
  double t = 0;
  for (double v : n.samples) t += v;
  if (n.samples.empty())
    for (const auto& c : n.children) t += node_total(*c.second);
  return t;
}

void json_node(const Node& n, std::ostringstream& os) {
  const Stats st = stats_of(n.samples);
  os << "{\"identifier\":\"" << n.name << "\",\"count\":" << st.count
     << ",\"total\":" << st.total << ",\"mean\":" << st.mean << ",\"median\":" << st.median
     << ",\"min\":" << st.min << ",\"max\":" << st.max << ",\"sub-timings\":[";
  bool first = true;
  for (const auto& c : n.children) {
    if (!first) os << ",";
    first = false;
    json_node(*c.second, os);
  }
  os << "]}";
}

void text_node(const Node& n, int depth, double parentTotal, double rootTotal,
               std::ostringstream& os) {
  const Stats st = stats_of(n.samples);
  const double total = n.samples.empty() ? node_total(n) : st.total;
  os << std::left << std::setw(40) << (std::string(2 * depth, ' ') + "- " + n.name) << std::right
     << std::setw(8) << st.count << std::setw(12) << std::setprecision(4) << total
     << std::setw(9) << std::setprecision(3)
     << (rootTotal > 0 ? 100.0 * total / rootTotal : 0.0) << std::setw(9)
     << (parentTotal > 0 ? 100.0 * total / parentTotal : 0.0) << std::setw(12)
     << std::setprecision(4) << st.median << std::setw(12) << st.min << std::setw(12) << st.max
     << "\n";
  for (const auto& c : n.children) text_node(*c.second, depth + 1, total, rootTotal, os);
}

}  // namespace

bool enabled() { return registry().level.load(std::memory_order_relaxed) > 0; }
bool gpu_stages() { return registry().level.load(std::memory_order_relaxed) > 1; }
void set_level(int level) { registry().level = level < 0 ? 0 : (level > 2 ? 2 : level); }

void reset() {
  auto& r = registry();
  std::lock_guard<std::mutex> lock(r.mutex);
  r.root.children.clear();
  r.root.samples.clear();
}

std::string report_json() {
  auto& r = registry();
  std::lock_guard<std::mutex> lock(r.mutex);
  std::ostringstream os;
  os << std::setprecision(9);
  os << "{\"timings\":[";
  bool first = true;
  for (const auto& c : r.root.children) {
    if (!first) os << ",";
    first = false;
    json_node(*c.second, os);
  }
  os << "]}";
  return os.str();
}

std::string report_text() {
  auto& r = registry();
  std::lock_guard<std::mutex> lock(r.mutex);
  std::ostringstream os;
  os << std::left << std::setw(40) << "identifier" << std::right << std::setw(8) << "count"
     << std::setw(12) << "total[s]" << std::setw(9) << "%" << std::setw(9) << "parent%"
     << std::setw(12) << "median[s]" << std::setw(12) << "min[s]" << std::setw(12) << "max[s]"
     << "\n";
  double rootTotal = 0;
  for (const auto& c : r.root.children) rootTotal += node_total(*c.second);
  for (const auto& c : r.root.children) text_node(*c.second, 0, rootTotal, rootTotal, os);
  return os.str();
}

void add_sample(std::initializer_list<const char*> path, double seconds) {
  if (!enabled()) return;
  auto& r = registry();
  std::lock_guard<std::mutex> lock(r.mutex);
  Node* n = &r.root;
  for (const char* name : path) {
    auto& slot = n->children[name];
    if (!slot) {
      slot.reset(new Node());
      slot->name = name;
      slot->parent = n;
    }
    n = slot.get();
  }
  n->samples.push_back(seconds);
}

Scope::Scope(const char* name) {
  auto& rx = roctx();
  if (rx.push) {
    rx.push(name);
    marker_ = true;
  }
  if (!enabled()) return;
  auto& r = registry();
  std::lock_guard<std::mutex> lock(r.mutex);
  Node* parent = tlsStack.empty() ? &r.root : tlsStack.back();
  auto& slot = parent->children[name];
  if (!slot) {
    slot.reset(new Node());
    slot->name = name;
    slot->parent = parent;
  }
  node_ = slot.get();
  tlsStack.push_back(slot.get());
  startNs_ = now_ns();
}

Scope::~Scope() {
  if (node_) {
    const double dt = 1e-9 * static_cast<double>(now_ns() - startNs_);
    auto& r = registry();
    std::lock_guard<std::mutex> lock(r.mutex);
    static_cast<Node*>(node_)->samples.push_back(dt);
    if (!tlsStack.empty()) tlsStack.pop_back();
  }
  if (marker_) roctx().pop();
}

}  // namespace timing
}  // namespace spfft
