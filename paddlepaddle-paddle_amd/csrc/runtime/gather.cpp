// Host data-path runtime: a persistent worker pool that gathers sample rows of in-memory
// arrays into (pinned) batch buffers, and a bounded blocking queue used as the loader's
// prefetch ring.  Called through ctypes, which drops the GIL for the duration of the call,
// so batch assembly runs truly parallel to the Python training loop.
//
// Reference behaviour: python/paddle/io/dataloader/dataloader_iter.py (prefetch of
// `prefetch_factor` batches per worker) and paddle/fluid/operators/reader/
// blocking_queue.h + buffered_reader.cc (double-buffered host->device staging).
#include <algorithm>
#include <cmath>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#define PA_RT extern "C" __attribute__((visibility("default")))

namespace {

class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < n; ++i) threads_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  int size() const { return static_cast<int>(threads_.size()); }

  // Run fn(0..parts-1) on the pool and the calling thread; returns when all parts finished.
  void parallel_for(int parts, const std::function<void(int)>& fn) {
    if (parts <= 1 || threads_.empty()) {
      for (int i = 0; i < parts; ++i) fn(i);
      return;
    }
    std::atomic<int> next{0};
    std::atomic<int> done{0};
    auto body = [&] {
      for (int i = next++; i < parts; i = next++) {
        fn(i);
        done++;
      }
    };
    int helpers = std::min(parts - 1, size());
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int i = 0; i < helpers; ++i) jobs_.push_back(body);
    }
    cv_.notify_all();
    body();
    // the caller drained the counter; wait for helpers still inside fn()
    while (done.load() < parts) std::this_thread::yield();
    // helpers that never started a part must not touch `next` after we return
    std::unique_lock<std::mutex> g(mu_);
    idle_cv_.wait(g, [&] { return running_ == 0 && jobs_.empty(); });
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || !jobs_.empty(); });
        if (stop_ && jobs_.empty()) return;
        job = std::move(jobs_.front());
        jobs_.pop_front();
        ++running_;
      }
      job();
      {
        std::lock_guard<std::mutex> g(mu_);
        --running_;
      }
      idle_cv_.notify_all();
    }
  }
  std::vector<std::thread> threads_;
  std::deque<std::function<void()>> jobs_;
  std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  int running_ = 0;
  bool stop_ = false;
};

Pool* g_pool = nullptr;
std::mutex g_pool_mu;

Pool& pool() {
  std::lock_guard<std::mutex> g(g_pool_mu);
  if (!g_pool) {
    unsigned hw = std::thread::hardware_concurrency();
    int n = static_cast<int>(std::min(16u, std::max(1u, hw / 2)));
    g_pool = new Pool(n - 1);
  }
  return *g_pool;
}

}  // namespace

PA_RT int pa_rt_num_threads() { return pool().size() + 1; }

PA_RT void pa_rt_set_num_threads(int n) {
  std::lock_guard<std::mutex> g(g_pool_mu);
  delete g_pool;
  g_pool = new Pool(std::max(0, n - 1));
}

// dst[i, :] = src[idx[i], :] for row_bytes-wide rows; idx < 0 or >= nrows is an error (-1 + no copy)
PA_RT int pa_rt_gather_rows(const void* src, int64_t nrows, int64_t row_bytes, const int64_t* idx, int64_t n,
                            void* dst) {
  for (int64_t i = 0; i < n; ++i)
    if (idx[i] < 0 || idx[i] >= nrows) return -1;
  const char* s = static_cast<const char*>(src);
  char* d = static_cast<char*>(dst);
  int64_t total = n * row_bytes;
  // ~256 KiB per part keeps every thread streaming while small batches stay single-threaded
  int parts = static_cast<int>(std::min<int64_t>(pa_rt_num_threads() * 4, std::max<int64_t>(1, total >> 18)));
  parts = static_cast<int>(std::min<int64_t>(parts, n));
  pool().parallel_for(parts, [&](int p) {
    int64_t lo = n * p / parts, hi = n * (p + 1) / parts;
    for (int64_t i = lo; i < hi; ++i) std::memcpy(d + i * row_bytes, s + idx[i] * row_bytes, row_bytes);
  });
  return 0;
}

// Parallel memcpy for large contiguous staging copies (e.g. pageable -> pinned)
PA_RT void pa_rt_memcpy(void* dst, const void* src, int64_t bytes) {
  int parts = static_cast<int>(std::min<int64_t>(pa_rt_num_threads(), std::max<int64_t>(1, bytes >> 20)));
  pool().parallel_for(parts, [&](int p) {
    int64_t lo = bytes * p / parts, hi = bytes * (p + 1) / parts;
    std::memcpy(static_cast<char*>(dst) + lo, static_cast<const char*>(src) + lo, hi - lo);
  });
}

// ---- bounded blocking queue of 64-bit handles ------------------------------------------
namespace {
struct Queue {
  explicit Queue(int cap) : cap(cap) {}
  int cap;
  std::deque<int64_t> q;
  std::mutex mu;
  std::condition_variable not_full, not_empty;
  bool closed = false;
};
}  // namespace

PA_RT void* pa_rt_queue_new(int cap) { return new Queue(std::max(1, cap)); }
PA_RT void pa_rt_queue_free(void* h) { delete static_cast<Queue*>(h); }

// 0 ok, 1 timeout, 2 closed
PA_RT int pa_rt_queue_push(void* h, int64_t v, int timeout_ms) {
  auto* q = static_cast<Queue*>(h);
  std::unique_lock<std::mutex> g(q->mu);
  auto ok = [&] { return q->closed || static_cast<int>(q->q.size()) < q->cap; };
  if (timeout_ms < 0)
    q->not_full.wait(g, ok);
  else if (!q->not_full.wait_for(g, std::chrono::milliseconds(timeout_ms), ok))
    return 1;
  if (q->closed) return 2;
  q->q.push_back(v);
  q->not_empty.notify_one();
  return 0;
}

PA_RT int pa_rt_queue_pop(void* h, int64_t* out, int timeout_ms) {
  auto* q = static_cast<Queue*>(h);
  std::unique_lock<std::mutex> g(q->mu);
  auto ok = [&] { return q->closed || !q->q.empty(); };
  if (timeout_ms < 0)
    q->not_empty.wait(g, ok);
  else if (!q->not_empty.wait_for(g, std::chrono::milliseconds(timeout_ms), ok))
    return 1;
  if (q->q.empty()) return 2;
  *out = q->q.front();
  q->q.pop_front();
  q->not_full.notify_one();
  return 0;
}

PA_RT void pa_rt_queue_close(void* h) {
  auto* q = static_cast<Queue*>(h);
  std::lock_guard<std::mutex> g(q->mu);
  q->closed = true;
  q->not_full.notify_all();
  q->not_empty.notify_all();
}

PA_RT int pa_rt_queue_size(void* h) {
  auto* q = static_cast<Queue*>(h);
  std::lock_guard<std::mutex> g(q->mu);
  return static_cast<int>(q->q.size());
}

// ---------------------------------------------------------------------------------------------
// Offloaded optimizer update (group-sharded training with offload=True; reference
// python/paddle/distributed/fleet/meta_parallel/sharding/group_sharded_stage3.py:98-127 and the
// CPU adam kernel it runs): the fp32 master / moments of this rank's shard live in host memory,
// the reduce-scattered gradient shard arrives by an async D2H copy into a pinned buffer, and the
// update runs here on the worker pool (one contiguous slice per thread, vectorised loop), writing
// the new master in place and the 16-bit parameter image (bf16 / fp16, round to nearest even)
// for the H2D copy back.  gdt / odt: 0 fp32, 1 bf16, 2 fp16 (grad / low-precision out, odt -1 = none).
namespace {
inline float bf16_to_f(uint16_t h) {
  uint32_t u = static_cast<uint32_t>(h) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return static_cast<uint16_t>((u >> 16) | 0x40);  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}
inline float f16_to_f(uint16_t h) {
  const uint32_t s = (h & 0x8000u) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff;
  uint32_t u;
  if (e == 0) {
    if (m == 0) {
      u = s;
    } else {  // subnormal
      int ee = -1;
      uint32_t mm = m;
      do {
        ++ee;
        mm <<= 1;
      } while (!(mm & 0x400));
      u = s | ((127 - 15 - ee) << 23) | ((mm & 0x3ff) << 13);
    }
  } else if (e == 31) {
    u = s | 0x7f800000u | (m << 13);
  } else {
    u = s | ((e + 127 - 15) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f_to_f16(float f) {  // round to nearest even, overflow to inf, NaN kept
  uint32_t u;
  std::memcpy(&u, &f, 4);
  const uint32_t s = (u >> 16) & 0x8000u;
  const uint32_t a = u & 0x7fffffffu;
  if (a >= 0x7f800000u) return static_cast<uint16_t>(s | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0u));
  if (a >= 0x477ff000u) return static_cast<uint16_t>(s | 0x7c00u);  // rounds past 65504
  if (a < 0x38800000u) {  // subnormal half (or zero)
    if (a < 0x33000000u) return static_cast<uint16_t>(s);
    const uint32_t e = a >> 23, mant = (a & 0x7fffffu) | 0x800000u;
    const uint32_t sh = 126 - e;  // 14 - (e - 127) + 13 - 1 ... shift to the 10-bit field
    uint32_t r = mant >> (sh);
    const uint32_t rem = mant & ((1u << sh) - 1), half = 1u << (sh - 1);
    if (rem > half || (rem == half && (r & 1u))) ++r;
    return static_cast<uint16_t>(s | r);
  }
  uint32_t r = a - 0x38000000u;  // rebias exponent 127 -> 15
  r += 0xfffu + ((r >> 13) & 1u);
  return static_cast<uint16_t>(s | (r >> 13));
}
}  // namespace

PA_RT int pa_rt_adamw(float* master, const void* grad, int gdt, float* m, float* v, void* out, int odt, int64_t n,
                      float lr, float b1, float b2, float eps, float wd, float b1p, float b2p, float grad_scale) {
  if (n <= 0) return 0;
  if (gdt < 0 || gdt > 2 || odt < -1 || odt > 2) return 1;
  const float bc2 = std::sqrt(1.f - b2p);
  const float step = lr * bc2 / (1.f - b1p);
  const float epsc = eps * bc2;
  const float decay = 1.f - lr * wd;
  const int64_t chunk = 1 << 16;
  const int parts = static_cast<int>((n + chunk - 1) / chunk);
  pool().parallel_for(parts, [&](int part) {
    const int64_t lo = part * chunk, hi = std::min(n, lo + chunk);
    for (int64_t i = lo; i < hi; ++i) {
      float g;
      if (gdt == 0) g = static_cast<const float*>(grad)[i];
      else if (gdt == 1) g = bf16_to_f(static_cast<const uint16_t*>(grad)[i]);
      else g = f16_to_f(static_cast<const uint16_t*>(grad)[i]);
      g *= grad_scale;
      float p = master[i] * decay;
      const float mi = m[i] * b1 + (1.f - b1) * g;
      const float vi = v[i] * b2 + (1.f - b2) * g * g;
      p -= step * mi / (std::sqrt(vi) + epsc);
      m[i] = mi;
      v[i] = vi;
      master[i] = p;
      if (odt == 1) static_cast<uint16_t*>(out)[i] = f_to_bf16(p);
      else if (odt == 2) static_cast<uint16_t*>(out)[i] = f_to_f16(p);
      else if (odt == 0) static_cast<float*>(out)[i] = p;
    }
  });
  return 0;
}
