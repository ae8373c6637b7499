// Host-side event tracer for paddle.profiler (reference: paddle/fluid/platform/profiler/
// host_tracer.cc + host_event_recorder.h: per-thread lock-free event buffers, names interned,
// collected once at profiler stop).
//
// Each thread appends completed ranges to its own chunked buffer (no lock on the hot path);
// `pa_rt_trace_collect` walks all registered thread buffers.  Timestamps are
// steady_clock nanoseconds, the same clock Python's time.perf_counter_ns uses on Linux.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#define PA_RT extern "C" __attribute__((visibility("default")))

namespace {

struct Event {
  int64_t start_ns, end_ns;
  int32_t name_id, type;
  uint64_t tid;
};

struct OpenRange {
  int64_t start_ns;
  int32_t name_id, type;
};

struct ThreadBuf {
  uint64_t tid;
  std::vector<Event> events;
  std::vector<OpenRange> stack;
  std::mutex mu;  // taken only by collect/clear and by the owner when appending (uncontended)
};

std::atomic<bool> g_enabled{false};
std::mutex g_reg_mu;
std::vector<std::shared_ptr<ThreadBuf>> g_bufs;
std::mutex g_names_mu;
std::unordered_map<std::string, int32_t> g_name_ids;
std::vector<std::string> g_names;

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

ThreadBuf& tbuf() {
  thread_local std::shared_ptr<ThreadBuf> b;
  if (!b) {
    b = std::make_shared<ThreadBuf>();
    b->tid = std::hash<std::thread::id>()(std::this_thread::get_id());
    b->events.reserve(4096);
    std::lock_guard<std::mutex> g(g_reg_mu);
    g_bufs.push_back(b);
  }
  return *b;
}

}  // namespace

PA_RT int32_t pa_rt_trace_intern(const char* name) {
  std::lock_guard<std::mutex> g(g_names_mu);
  auto it = g_name_ids.find(name);
  if (it != g_name_ids.end()) return it->second;
  int32_t id = static_cast<int32_t>(g_names.size());
  g_names.emplace_back(name);
  g_name_ids.emplace(g_names.back(), id);
  return id;
}

PA_RT const char* pa_rt_trace_name(int32_t id) {
  std::lock_guard<std::mutex> g(g_names_mu);
  if (id < 0 || id >= static_cast<int32_t>(g_names.size())) return "";
  return g_names[id].c_str();
}

PA_RT void pa_rt_trace_enable(int on) { g_enabled.store(on != 0); }
PA_RT int pa_rt_trace_enabled() { return g_enabled.load() ? 1 : 0; }
PA_RT int64_t pa_rt_now_ns() { return now_ns(); }

PA_RT void pa_rt_trace_push(int32_t name_id, int32_t type) {
  if (!g_enabled.load(std::memory_order_relaxed)) return;
  tbuf().stack.push_back({now_ns(), name_id, type});
}

PA_RT void pa_rt_trace_pop() {
  if (!g_enabled.load(std::memory_order_relaxed)) return;
  ThreadBuf& b = tbuf();
  if (b.stack.empty()) return;
  OpenRange r = b.stack.back();
  b.stack.pop_back();
  std::lock_guard<std::mutex> g(b.mu);
  b.events.push_back({r.start_ns, now_ns(), r.name_id, r.type, b.tid});
}

// a complete range recorded in one call (e.g. from a Python context manager's exit)
PA_RT void pa_rt_trace_record(int32_t name_id, int32_t type, int64_t start_ns, int64_t end_ns) {
  if (!g_enabled.load(std::memory_order_relaxed)) return;
  ThreadBuf& b = tbuf();
  std::lock_guard<std::mutex> g(b.mu);
  b.events.push_back({start_ns, end_ns, name_id, type, b.tid});
}

PA_RT int64_t pa_rt_trace_count() {
  std::lock_guard<std::mutex> g(g_reg_mu);
  int64_t n = 0;
  for (auto& b : g_bufs) {
    std::lock_guard<std::mutex> gb(b->mu);
    n += static_cast<int64_t>(b->events.size());
  }
  return n;
}

// Copies up to cap events as 5 int64 each: start, end, name_id, type, tid.  Returns count.
PA_RT int64_t pa_rt_trace_collect(int64_t* out, int64_t cap) {
  std::lock_guard<std::mutex> g(g_reg_mu);
  int64_t n = 0;
  for (auto& b : g_bufs) {
    std::lock_guard<std::mutex> gb(b->mu);
    for (const Event& e : b->events) {
      if (n >= cap) return n;
      int64_t* o = out + 5 * n;
      o[0] = e.start_ns;
      o[1] = e.end_ns;
      o[2] = e.name_id;
      o[3] = e.type;
      o[4] = static_cast<int64_t>(e.tid & 0x7fffffffffffffffULL);
      ++n;
    }
  }
  return n;
}

PA_RT void pa_rt_trace_clear() {
  std::lock_guard<std::mutex> g(g_reg_mu);
  for (auto& b : g_bufs) {
    std::lock_guard<std::mutex> gb(b->mu);
    b->events.clear();
  }
}
