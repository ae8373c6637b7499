// Native device memory allocator: auto-growth best-fit over large HBM chunks, per (device, stream)
// pools, coalescing free, chunk release on demand — installed as torch's device allocator through
// the pluggable-allocator hook (pa_torch_alloc / pa_torch_free), so every tensor of the process
// lives in it.
//
// Reference semantics: paddle/fluid/memory/allocation/auto_growth_best_fit_allocator.cc (chunks
// grown on demand, best-fit split of free blocks, neighbour merge on free, FreeIdleChunks),
// stream_safe_cuda_allocator.cc (a block freed on a stream is reused only by that stream),
// FLAGS_fraction_of_gpu_memory_to_use / FLAGS_auto_growth_chunk_size_in_mb.
//
// MI355X sizing: 288 GB HBM3E per GPU and one process per GPU, so chunks are large (default 1 GiB,
// or the request when larger): a 1.3B-parameter training step touches a few hundred blocks and
// hipMalloc (which synchronises the device) runs only while the working set is still growing.
// Blocks are 512-B aligned (every kernel's 16-B vector / LDS-DMA alignment holds, and split
// remainders stay aligned).
//
// The raw backend is hipMalloc/hipFree, or host malloc/free (backend 1) so the block logic is
// unit-tested on machines without a GPU.
#include <hip/hip_runtime.h>

#include <sys/types.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <list>
#include <map>
#include <mutex>
#include <set>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

constexpr size_t kAlign = 512;

struct Chunk;

struct Block {
  char* ptr;
  size_t size;
  bool free;
  Chunk* chunk;
};

struct Chunk {
  char* base;
  size_t size;
  std::list<Block> blocks;  // address order
  int device;
  void* stream;
};

using BlockIt = std::list<Block>::iterator;

struct Pool {
  std::set<std::pair<size_t, char*>> free_set;  // (size, ptr): best fit = lower_bound(size)
  std::unordered_map<char*, BlockIt> free_blocks;
};

struct Stats {
  long long allocated = 0, reserved = 0, peak_allocated = 0, peak_reserved = 0;
  long long num_allocs = 0, num_frees = 0, num_chunks = 0, num_raw_allocs = 0, num_ooms = 0;
};

struct State {
  std::mutex mu;
  int backend = 0;                                         // 0 = HIP, 1 = host
  size_t chunk_bytes = 1ull << 30;
  long long limit_bytes = -1;                              // per-device reserved cap (-1 = none)
  std::map<std::pair<int, void*>, Pool> pools;             // (device, stream) -> free blocks
  std::unordered_map<char*, std::pair<Chunk*, BlockIt>> live;  // allocated block start -> block
  std::list<Chunk*> chunks;
  std::map<int, Stats> stats;
};

State& S() {
  static State* s = new State();  // never destroyed: torch may free tensors during interpreter exit
  return *s;
}

size_t align_up(size_t n) { return (n + kAlign - 1) / kAlign * kAlign; }

void* raw_alloc(State& s, size_t n, int device) {
  if (s.backend == 1) return std::aligned_alloc(kAlign, n);
  void* p = nullptr;
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return nullptr;
  if (cur != device) (void)hipSetDevice(device);
  const hipError_t e = hipMalloc(&p, n);
  if (cur != device) (void)hipSetDevice(cur);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky OOM so the caller can retry after a release
    return nullptr;
  }
  return p;
}

void raw_free(State& s, void* p, int device) {
  if (s.backend == 1) {
    std::free(p);
    return;
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != device) (void)hipSetDevice(device);
  (void)hipFree(p);
  if (cur != device) (void)hipSetDevice(cur);
}

void pool_insert(Pool& pool, BlockIt b) {
  pool.free_set.emplace(b->size, b->ptr);
  pool.free_blocks[b->ptr] = b;
}

void pool_erase(Pool& pool, BlockIt b) {
  pool.free_set.erase({b->size, b->ptr});
  pool.free_blocks.erase(b->ptr);
}

// release every chunk of (device) that is one free block; returns bytes released
size_t release_idle(State& s, int device) {
  size_t freed = 0;
  for (auto it = s.chunks.begin(); it != s.chunks.end();) {
    Chunk* c = *it;
    if (c->device == device && c->blocks.size() == 1 && c->blocks.front().free) {
      Pool& pool = s.pools[{c->device, c->stream}];
      pool_erase(pool, c->blocks.begin());
      raw_free(s, c->base, c->device);
      Stats& st = s.stats[device];
      st.reserved -= (long long)c->size;
      st.num_chunks -= 1;
      freed += c->size;
      delete c;
      it = s.chunks.erase(it);
    } else {
      ++it;
    }
  }
  return freed;
}

void* alloc_locked(State& s, size_t req, int device, void* stream) {
  const size_t n = align_up(req == 0 ? 1 : req);
  Pool& pool = s.pools[{device, stream}];
  Stats& st = s.stats[device];
  auto fit = pool.free_set.lower_bound({n, nullptr});
  BlockIt b;
  Chunk* chunk = nullptr;
  if (fit != pool.free_set.end()) {
    b = pool.free_blocks.at(fit->second);
    chunk = b->chunk;
    pool_erase(pool, b);
  } else {
    size_t csz = n > s.chunk_bytes ? n : s.chunk_bytes;
    if (s.limit_bytes >= 0 && st.reserved + (long long)csz > s.limit_bytes) {
      release_idle(s, device);
      if (st.reserved + (long long)csz > s.limit_bytes) csz = n;  // exact-size chunk under the cap
      if (st.reserved + (long long)csz > s.limit_bytes) {
        st.num_ooms += 1;
        return nullptr;
      }
    }
    void* p = raw_alloc(s, csz, device);
    if (p == nullptr) {  // give idle chunks back and retry, then an exact-size chunk
      release_idle(s, device);
      p = raw_alloc(s, csz, device);
      if (p == nullptr && csz > n) {
        csz = n;
        p = raw_alloc(s, csz, device);
      }
      if (p == nullptr) {
        st.num_ooms += 1;
        return nullptr;
      }
    }
    chunk = new Chunk{static_cast<char*>(p), csz, {}, device, stream};
    chunk->blocks.push_back(Block{chunk->base, csz, true, chunk});
    b = chunk->blocks.begin();
    s.chunks.push_back(chunk);
    st.reserved += (long long)csz;
    st.num_chunks += 1;
    st.num_raw_allocs += 1;
    if (st.reserved > st.peak_reserved) st.peak_reserved = st.reserved;
  }
  if (b->size - n >= kAlign) {  // split: the tail stays free in this pool
    Block tail{b->ptr + n, b->size - n, true, chunk};
    b->size = n;
    BlockIt t = chunk->blocks.insert(std::next(b), tail);
    pool_insert(pool, t);
  }
  b->free = false;
  s.live[b->ptr] = {chunk, b};
  st.allocated += (long long)b->size;
  st.num_allocs += 1;
  if (st.allocated > st.peak_allocated) st.peak_allocated = st.allocated;
  return b->ptr;
}

void free_locked(State& s, void* ptr) {
  auto it = s.live.find(static_cast<char*>(ptr));
  if (it == s.live.end()) return;  // not ours (or a double free): ignore
  Chunk* chunk = it->second.first;
  BlockIt b = it->second.second;
  s.live.erase(it);
  Pool& pool = s.pools[{chunk->device, chunk->stream}];
  Stats& st = s.stats[chunk->device];
  st.allocated -= (long long)b->size;
  st.num_frees += 1;
  b->free = true;
  if (b != chunk->blocks.begin()) {  // merge with a free predecessor
    BlockIt p = std::prev(b);
    if (p->free) {
      pool_erase(pool, p);
      p->size += b->size;
      chunk->blocks.erase(b);
      b = p;
    }
  }
  BlockIt n = std::next(b);
  if (n != chunk->blocks.end() && n->free) {  // and a free successor
    pool_erase(pool, n);
    b->size += n->size;
    chunk->blocks.erase(n);
  }
  pool_insert(pool, b);
}

}  // namespace

#define PA_ALLOC_API extern "C" __attribute__((visibility("default")))

// backend: 0 = hipMalloc/hipFree, 1 = host malloc (tests).  chunk_mb: growth granularity.
// limit_mb: per-device reserved cap (<= 0: none; FLAGS_fraction_of_gpu_memory_to_use analogue).
PA_ALLOC_API int pa_alloc_config(int backend, long long chunk_mb, long long limit_mb) {
  State& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  if (!s.live.empty() && backend != s.backend) return -1;  // cannot switch with live blocks
  s.backend = backend;
  if (chunk_mb > 0) s.chunk_bytes = (size_t)chunk_mb << 20;
  s.limit_bytes = limit_mb > 0 ? (limit_mb << 20) : -1;
  return 0;
}

PA_ALLOC_API void* pa_alloc_malloc(long long size, int device, void* stream) {
  State& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  return alloc_locked(s, size < 0 ? 0 : (size_t)size, device, stream);
}

PA_ALLOC_API void pa_alloc_free(void* ptr) {
  State& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  free_locked(s, ptr);
}

// torch pluggable-allocator entry points (c10 CUDAPluggableAllocator signatures)
PA_ALLOC_API void* pa_torch_alloc(ssize_t size, int device, hipStream_t stream) {
  return pa_alloc_malloc((long long)size, device, (void*)stream);
}

PA_ALLOC_API void pa_torch_free(void* ptr, ssize_t size, int device, hipStream_t stream) {
  (void)size;
  (void)device;
  (void)stream;
  pa_alloc_free(ptr);
}

// out[0..8]: allocated, reserved, peak allocated, peak reserved, allocs, frees, chunks, raw allocs, ooms
PA_ALLOC_API void pa_alloc_stats(int device, long long* out) {
  State& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  const Stats& st = s.stats[device];
  const long long v[9] = {st.allocated, st.reserved, st.peak_allocated, st.peak_reserved, st.num_allocs,
                          st.num_frees, st.num_chunks, st.num_raw_allocs, st.num_ooms};
  std::memcpy(out, v, sizeof(v));
}

PA_ALLOC_API void pa_alloc_reset_peak(int device) {
  State& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  Stats& st = s.stats[device];
  st.peak_allocated = st.allocated;
  st.peak_reserved = st.reserved;
}

// Releases every fully idle chunk of the device (the caller synchronises the device first so no
// queued kernel still uses the memory).  Returns the bytes given back.
PA_ALLOC_API long long pa_alloc_empty_cache(int device) {
  State& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  return (long long)release_idle(s, device);
}

// Largest free block of the device's pools (fragmentation diagnostics).
PA_ALLOC_API long long pa_alloc_largest_free(int device) {
  State& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  size_t best = 0;
  for (auto& kv : s.pools)
    if (kv.first.first == device && !kv.second.free_set.empty())
      best = std::max(best, std::prev(kv.second.free_set.end())->first);
  return (long long)best;
}

PA_ALLOC_API long long pa_alloc_live_blocks() {
  State& s = S();
  std::lock_guard<std::mutex> g(s.mu);
  return (long long)s.live.size();
}
