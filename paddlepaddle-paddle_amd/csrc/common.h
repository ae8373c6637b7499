// Shared device helpers for the paddle_amd HIP kernel library (gfx950 / CDNA4 only).
//
// Conventions
//  * dtype codes passed from Python: 0 = fp32, 1 = bf16, 2 = fp16.
//  * All launchers are extern "C", take raw device pointers and the caller's hipStream_t,
//    never allocate or synchronise (so they can be captured into hipGraphs), and return
//    hipError_t of the launch.
//  * Wave = 64 lanes. Block sizes are multiples of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PA_API extern "C" __attribute__((visibility("default")))

namespace pa {

constexpr int kWave = 64;

using bf16_t = __bf16;
using f16_t = _Float16;

template <typename T> struct Vec8;  // 16-byte vector of 8 x 16-bit or 4 x fp32 (handled separately)

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(bf16_t v) { return (float)v; }
__device__ __forceinline__ float to_f(f16_t v) { return (float)v; }

template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float v) { return (bf16_t)v; }
template <> __device__ __forceinline__ f16_t from_f<f16_t>(float v) { return (f16_t)v; }

// Load/store N contiguous elements (N*sizeof(T) must be 4, 8 or 16 bytes) as one vector access.
template <typename T, int N> struct alignas(sizeof(T) * N) Pack { T v[N]; };

template <typename T, int N>
__device__ __forceinline__ void load_f(const T* __restrict__ p, float (&out)[N]) {
  Pack<T, N> pk = *reinterpret_cast<const Pack<T, N>*>(p);
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = to_f(pk.v[i]);
}

template <typename T, int N>
__device__ __forceinline__ void store_f(T* __restrict__ p, const float (&in)[N]) {
  Pack<T, N> pk;
#pragma unroll
  for (int i = 0; i < N; ++i) pk.v[i] = from_f<T>(in[i]);
  *reinterpret_cast<Pack<T, N>*>(p) = pk;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += red[i];
  __syncthreads();
  return r;
}

template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, red[i]);
  __syncthreads();
  return r;
}

// Sum over the 16 lanes of a DPP row (lanes 16k .. 16k+15), result in every lane of the row: DPP
// quad_perm xor 1 / xor 2, then row_half_mirror and row_mirror (once a quad / half-row holds one
// value in every lane, mirroring adds the other quad / half): VALU only, no LDS crossbar traffic.
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, true));
  return v;
}

// Per-column batch-norm statistics of one wave's output slab, computed in the producing GEMM /
// convolution epilogue (fused_bn statistics: the standalone column pass over the activation is
// skipped).  Swapped-MFMA layout: the lane holds rows 16 i + (lane & 15) (i < FM) of columns
// 16 j + 4 (lane >> 4) + e (j < FN, e < 4) in acc[i][j][e]; rows at or past `nvalid` are excluded.
// Two-pass in registers (sum -> mean -> sum of squared deviations: no E[x^2] - E[x]^2
// cancellation), each pass reduced over the 16 lanes of a column group by DPP (row16_sum).  The
// slab's (mean, M2) over its nvalid rows go to pmean[col], pm2[col] (lanes with lane & 15 == 0;
// cols >= ncols skipped, ncols % 4 == 0).  `add` (nullable, 4 FN values per lane, e.g. the bias)
// is added to every value first.
template <int FM, int FN, typename V>
__device__ __forceinline__ void wave_col_stats(const V (&acc)[FM][FN], const float (*add)[4], int nvalid, int col0,
                                               int ncols, float* __restrict__ pmean, float* __restrict__ pm2) {
  if (nvalid <= 0) return;
  const int lane = threadIdx.x & 63, r16 = lane & 15;
  const float inv_n = 1.f / (float)nvalid;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const bool ok = 16 * i + r16 < nvalid;
#pragma unroll
      for (int e = 0; e < 4; ++e) s[e] += ok ? acc[i][j][e] + (add ? add[j][e] : 0.f) : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s[e] = row16_sum(s[e]) * inv_n;  // the slab mean, in every lane of the group
    }
    float q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const bool ok = 16 * i + r16 < nvalid;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = acc[i][j][e] + (add ? add[j][e] : 0.f) - s[e];
        q[e] += ok ? d * d : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) q[e] = row16_sum(q[e]);
    const int c = col0 + 16 * j + 4 * (lane >> 4);
    if (r16 == 0 && c < ncols) {
      *reinterpret_cast<float4*>(pmean + c) = make_float4(s[0], s[1], s[2], s[3]);
      *reinterpret_cast<float4*>(pm2 + c) = make_float4(q[0], q[1], q[2], q[3]);
    }
  }
}

// tanh(u) = 1 - 2 / (1 + e^{2u}) on the v_exp_f32 path (libm tanhf is a long polynomial
// branch ladder: it made the GeLU kernels VALU-bound instead of HBM-bound).  Saturates
// correctly at both ends (e^{2u} -> inf gives 1, -> 0 gives -1); |error| ~ 1e-7.
__device__ __forceinline__ float fast_tanh(float u) { return 1.f - __fdividef(2.f, 1.f + __expf(2.f * u)); }

// gelu_tanh(x) and its derivative from one tanh evaluation (the GEMM epilogue of the fused MLP
// stores the derivative for the backward instead of the pre-activation)
__device__ __forceinline__ void gelu_tanh_fdf(float x, float& f, float& df) {
  const float x2 = x * x;
  const float u = 0.79788456080286536f * x * (1.f + 0.044715f * x2);
  const float t = fast_tanh(u);
  const float hx = 0.5f * x;
  f = hx * (1.f + t);
  df = 0.5f * (1.f + t) + hx * (1.f - t * t) * 0.79788456080286536f * (1.f + 3.f * 0.044715f * x2);
}

// gelu_tanh and its derivative for a PAIR of values in the sigmoid form (packed-f32 VALU, one
// v_exp_f32 + one v_rcp_f32 per value): gelu_tanh(x) = x s, s = sigmoid(2u) = 1 / (1 + 2^z),
// z = -2 log2(e) u, u = c (x + a x^3);  gelu_tanh'(x) = s + x s (1 - s) 2c (1 + 3 a x^2)
// (= 0.5 (1 + t) + 0.5 x (1 - t^2) u' with t = 2s - 1).  Saturates cleanly: 2^z = inf -> s = 0.
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void gelu_tanh_fdf2(f32x2_t x, f32x2_t& f, f32x2_t& df) {
  constexpr float c = 0.79788456080286536f, a = 0.044715f, l2e = 1.4426950408889634f;
  constexpr float k1 = -2.f * l2e * c, k2 = -2.f * l2e * c * a, m1 = 2.f * c, m2 = 6.f * a * c;
  const f32x2_t x2 = x * x;
  const f32x2_t z = x * __builtin_elementwise_fma(x2, f32x2_t{k2, k2}, f32x2_t{k1, k1});
  f32x2_t d = f32x2_t{__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)} + 1.f;
  const f32x2_t sg = f32x2_t{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f = x * sg;
  const f32x2_t w = x * __builtin_elementwise_fma(x2, f32x2_t{m2, m2}, f32x2_t{m1, m1});
  const f32x2_t k = __builtin_elementwise_fma(-sg, sg, sg);  // s (1 - s)
  df = __builtin_elementwise_fma(w, k, sg);
}

// Exact-form GELU and its derivative for GEMM epilogues: erf by Abramowitz-Stegun 7.1.26 (|error|
// <= 1.5e-7, far below bf16 output rounding) sharing ONE exp with the derivative's normal density:
// z = |x|/sqrt2, t = 1/(1 + p z), erf(z) = 1 - t*poly(t)*exp(-z^2), exp(-z^2) = exp(-x^2/2).
__device__ __forceinline__ void gelu_erf_fdf(float x, float& f, float& df) {
  constexpr float p = 0.3275911f, a1 = 0.254829592f, a2 = -0.284496736f, a3 = 1.421413741f, a4 = -1.453152027f,
                  a5 = 1.061405429f, l2e = 1.4426950408889634f;
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(p, z, 1.f));
  const float e = __builtin_amdgcn_exp2f(-0.5f * l2e * x * x);
  const float poly = t * __builtin_fmaf(t, __builtin_fmaf(t, __builtin_fmaf(t, __builtin_fmaf(t, a5, a4), a3), a2), a1);
  const float erfz = __builtin_fmaf(-poly, e, 1.f);
  const float cdf = 0.5f + copysignf(0.5f * erfz, x);
  f = x * cdf;
  df = __builtin_fmaf(x * 0.39894228040143268f, e, cdf);
}

struct GeluTanh {
  static __device__ __forceinline__ float f(float x) {
    const float u = 0.79788456080286536f * (x + 0.044715f * x * x * x);
    return 0.5f * x * (1.f + fast_tanh(u));
  }
  static __device__ __forceinline__ float df(float x) {
    const float u = 0.79788456080286536f * (x + 0.044715f * x * x * x);
    const float t = fast_tanh(u);
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * 0.79788456080286536f * (1.f + 3.f * 0.044715f * x * x);
  }
};

// Graph-safe dropout streams: an optional device-resident generation counter mixed into every
// dropout seed once at kernel entry.  Eager steps leave it unset (the seed as drawn on the host);
// a captured training step (device/cuda/graphs.py TrainStepGraph) advances the counter as the
// first node of every replay, so the host seeds frozen into the graph still give a fresh keep-mask
// per step, and a step's backward regenerates its forward's masks (same counter value).  One
// pointer per translation unit (static), set by that file's pa_*_set_rng_gen.
static __constant__ const uint32_t* g_rng_gen = nullptr;
__device__ __forceinline__ uint32_t rng_mix(uint32_t seed) {
  const uint32_t* p = g_rng_gen;
  return p ? seed ^ (*p * 0x9E3779B1u) : seed;
}

// Counter-based RNG (for dropout): a cheap stateless hash of (seed, offset, index) → uniform [0,1).
__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  // murmur3-style finaliser chain
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u);
  h ^= c * 0x85EBCA77u;
  h ^= h >> 16; h *= 0x7FEB352Du;
  h ^= h >> 15; h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ float uniform01(uint32_t h) { return (h >> 8) * (1.0f / 16777216.0f); }

// Grid size for memory-bound grid-stride kernels: enough waves to fill 256 CUs.
inline int grid_for(long long work_items, int per_block, int cap = 256 * 16) {
  long long g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}


// out[c] (+)= sum_p part[p, c] over a [P, cols] fp32 partial-sum matrix (the second pass of every
// column reduction here: bias / gamma / beta gradients).  Block = 16 waves x 64 columns; wave w
// sums rows w, w+16, ... with 4 independent loads in flight per lane (each wave-row read is
// 256 contiguous bytes), then a 16-way LDS combine.  Deterministic (fixed order, no atomics).
template <typename OT>
__global__ __launch_bounds__(1024) void colsum_finish(const float* __restrict__ part, OT* __restrict__ out, int P,
                                                      int cols, int accum) {
  __shared__ float red[16][65];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < cols) {
    int p = w;
    for (; p + 48 < P; p += 64) {
      s0 += part[(size_t)p * cols + c];
      s1 += part[(size_t)(p + 16) * cols + c];
      s2 += part[(size_t)(p + 32) * cols + c];
      s3 += part[(size_t)(p + 48) * cols + c];
    }
    for (; p < P; p += 16) s0 += part[(size_t)p * cols + c];
  }
  red[w][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (w == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][lane];
    out[c] = from_f<OT>(accum ? to_f(out[c]) + t : t);
  }
}

template <typename OT>
inline hipError_t launch_colsum_finish(const float* part, void* out, int P, int cols, int accum, hipStream_t st) {
  colsum_finish<OT><<<(cols + 63) / 64, 1024, 0, st>>>(part, (OT*)out, P, cols, accum);
  return hipGetLastError();
}

// Up to three column-sum finishes over partial matrices of one shape [P, cols] in ONE launch
// (blockIdx.y = job): the gamma / beta / bias gradients of a fused norm backward, each with its own
// output dtype (0 fp32, 1 bf16, 2 fp16) and accumulate flag.  Same summation order as colsum_finish.
struct FinishJob {
  const float* part;
  void* out;
  int odt;
  int accum;
};
struct FinishJobs {
  FinishJob j[3];
};

template <typename OT>
__device__ __forceinline__ void finish_store(void* out, int c, float t, int accum) {
  OT* o = reinterpret_cast<OT*>(out);
  o[c] = from_f<OT>(accum ? to_f(o[c]) + t : t);
}

static __global__ __launch_bounds__(1024) void colsum_finish_multi(FinishJobs jobs, int P, int cols) {
  __shared__ float red[16][65];
  const int y = blockIdx.y;
  const FinishJob jb = y == 0 ? jobs.j[0] : (y == 1 ? jobs.j[1] : jobs.j[2]);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const float* __restrict__ part = jb.part;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < cols) {
    int p = w;
    for (; p + 48 < P; p += 64) {
      s0 += part[(size_t)p * cols + c];
      s1 += part[(size_t)(p + 16) * cols + c];
      s2 += part[(size_t)(p + 32) * cols + c];
      s3 += part[(size_t)(p + 48) * cols + c];
    }
    for (; p < P; p += 16) s0 += part[(size_t)p * cols + c];
  }
  red[w][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (w == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][lane];
    if (jb.odt == 0) finish_store<float>(jb.out, c, t, jb.accum);
    else if (jb.odt == 1) finish_store<bf16_t>(jb.out, c, t, jb.accum);
    else finish_store<f16_t>(jb.out, c, t, jb.accum);
  }
}

inline hipError_t launch_colsum_finish_multi(const FinishJobs& jobs, int njobs, int P, int cols, hipStream_t st) {
  if (njobs <= 0) return hipSuccess;
  colsum_finish_multi<<<dim3((cols + 63) / 64, njobs), 1024, 0, st>>>(jobs, P, cols);
  return hipGetLastError();
}

template <typename T> constexpr int dtcode_of();
template <> constexpr int dtcode_of<float>() { return 0; }
template <> constexpr int dtcode_of<bf16_t>() { return 1; }
template <> constexpr int dtcode_of<f16_t>() { return 2; }

// dtype-coded output (0 fp32, 1 bf16, 2 fp16)
inline hipError_t launch_colsum_finish_dt(const float* part, void* out, int odt, int P, int cols, int accum,
                                          hipStream_t st) {
  switch (odt) {
    case 0: return launch_colsum_finish<float>(part, out, P, cols, accum, st);
    case 1: return launch_colsum_finish<bf16_t>(part, out, P, cols, accum, st);
    case 2: return launch_colsum_finish<f16_t>(part, out, P, cols, accum, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pa

#define PA_DISPATCH_DTYPE(code, T, ...)                         \
  switch (code) {                                               \
    case 0: { using T = float; __VA_ARGS__; break; }            \
    case 1: { using T = pa::bf16_t; __VA_ARGS__; break; }       \
    case 2: { using T = pa::f16_t; __VA_ARGS__; break; }        \
    default: return hipErrorInvalidValue;                       \
  }
