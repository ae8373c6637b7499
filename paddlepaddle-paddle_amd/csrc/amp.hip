// Loss-scaling kernels of mixed-precision training, device-resident state (no host sync):
//
//  * pa_amp_check_unscale: multi-tensor  g *= 1 / scale  with a non-finite check, ONE launch for up
//    to 48 gradient tensors of any dtype mix (fp32 / bf16 / fp16), the inverse scale read from
//    device memory; any inf / nan sets *found = 1 (a plain store of the same value from every
//    offending lane: no atomics, no ordering needed).
//  * pa_amp_update_scale: the dynamic loss-scale rule on device scalars (scale, good / bad step
//    counters), one lane.
//
// Reference: paddle/phi/kernels/gpu/amp_kernel.cu (CheckFiniteAndUnscaleKernel,
// UpdateLossScalingKernel), python/paddle/static/amp/decorator.py:548,589 (where the static AMP
// decorator inserts them).
#include "common.h"

namespace pa {
namespace amp {

constexpr int kMaxT = 48;
constexpr int kChunk = 256 * 8 * 4;  // elements per block: 256 lanes x 8 x 4 iterations

struct Table {
  void* ptr[kMaxT];
  long long n[kMaxT];
  int first_block[kMaxT + 1];  // block prefix: tensor t owns blocks [first_block[t], first_block[t + 1])
  int dt[kMaxT];
  int count;
};

template <typename T>
__device__ __forceinline__ bool unscale_chunk(T* __restrict__ p, long long n, long long c0, float inv) {
  bool bad = false;
  const long long end = min(n, c0 + kChunk);
  constexpr int E = 16 / sizeof(T);
  const bool vec = (((uintptr_t)p) & 15) == 0;
  long long i = c0 + (long long)threadIdx.x * E;
  if (vec) {
    for (; i + E <= end; i += 256LL * E) {
      float v[E];
      load_f<T, E>(p + i, v);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        bad |= !isfinite(v[e]);
        v[e] *= inv;
      }
      store_f<T, E>(p + i, v);
    }
    // tail (< E elements at the end of the tensor)
    if (i < end) {
      for (long long k = i; k < end; ++k) {
        const float v = to_f(p[k]);
        bad |= !isfinite(v);
        p[k] = from_f<T>(v * inv);
      }
    }
  } else {
    for (long long k = c0 + threadIdx.x; k < end; k += 256) {
      const float v = to_f(p[k]);
      bad |= !isfinite(v);
      p[k] = from_f<T>(v * inv);
    }
  }
  return bad;
}

__global__ __launch_bounds__(256) void check_unscale_kernel(Table tab, const float* __restrict__ scale,
                                                            float* __restrict__ found) {
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < tab.count && b >= tab.first_block[t + 1]) ++t;
  const long long c0 = (long long)(b - tab.first_block[t]) * kChunk;
  const float s = scale[0];
  const float inv = s != 0.f ? 1.f / s : 0.f;
  bool bad;
  if (tab.dt[t] == 1) bad = unscale_chunk(reinterpret_cast<bf16_t*>(tab.ptr[t]), tab.n[t], c0, inv);
  else if (tab.dt[t] == 2) bad = unscale_chunk(reinterpret_cast<f16_t*>(tab.ptr[t]), tab.n[t], c0, inv);
  else bad = unscale_chunk(reinterpret_cast<float*>(tab.ptr[t]), tab.n[t], c0, inv);
  if (bad) found[0] = 1.f;
}

// state: scale, good (float-valued counter), bad; found read from the check kernel.
__global__ void update_scale_kernel(float* __restrict__ scale, float* __restrict__ good, float* __restrict__ bad,
                                    const float* __restrict__ found, int incr_every, int decr_every, float incr_ratio,
                                    float decr_ratio, float min_scale) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const bool f = found[0] != 0.f;
  float s = scale[0], g = good[0], bd = bad[0];
  if (f) {
    g = 0.f;
    bd += 1.f;
    if (bd >= (float)decr_every) {
      s = fmaxf(s * decr_ratio, min_scale);
      bd = 0.f;
    }
  } else {
    bd = 0.f;
    g += 1.f;
    if (g >= (float)incr_every) {
      const float ns = s * incr_ratio;
      if (isfinite(ns)) s = ns;
      g = 0.f;
    }
  }
  scale[0] = s;
  good[0] = g;
  bad[0] = bd;
}

}  // namespace amp
}  // namespace pa

// ptrs / numels / dtypes: host arrays of `count` (<= 48) gradient tensors.  found must be zeroed by
// the caller before the first call of a step (calls accumulate into it).
PA_API int pa_amp_check_unscale(void* const* ptrs, const long long* numels, const int* dtypes, int count,
                                const float* scale, float* found, hipStream_t st) {
  using namespace pa::amp;
  if (count < 1 || count > kMaxT || !scale || !found) return (int)hipErrorInvalidValue;
  Table tab;
  int blocks = 0;
  for (int t = 0; t < count; ++t) {
    if (dtypes[t] < 0 || dtypes[t] > 2 || numels[t] < 0) return (int)hipErrorInvalidValue;
    tab.ptr[t] = ptrs[t];
    tab.n[t] = numels[t];
    tab.dt[t] = dtypes[t];
    tab.first_block[t] = blocks;
    blocks += (int)((numels[t] + kChunk - 1) / kChunk);
  }
  tab.first_block[count] = blocks;
  tab.count = count;
  if (blocks == 0) return (int)hipSuccess;
  check_unscale_kernel<<<blocks, 256, 0, st>>>(tab, scale, found);
  return (int)hipGetLastError();
}

PA_API int pa_amp_update_scale(float* scale, float* good, float* bad, const float* found, int incr_every,
                               int decr_every, float incr_ratio, float decr_ratio, float min_scale, hipStream_t st) {
  using namespace pa::amp;
  update_scale_kernel<<<1, 64, 0, st>>>(scale, good, bad, found, incr_every, decr_every, incr_ratio, decr_ratio,
                                        min_scale);
  return (int)hipGetLastError();
}
