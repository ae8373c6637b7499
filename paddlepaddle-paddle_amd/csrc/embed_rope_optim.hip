// Embedding gather/scatter-add, fused rotary position embedding, and the fused AdamW update
// over flat parameter buffers.
//
// Reference semantics: paddle/phi/kernels/gpu/embedding_kernel.cu / embedding_grad_kernel.cu,
// paddle/phi/kernels/fusion/gpu/fused_rope_kernel.cu (+ fused_rope_grad), paddle/phi/kernels/
// gpu/adamw_kernel.cu (paddle's AdamW: decoupled decay p *= 1 - lr*coeff, epsilon scaled by
// sqrt(1 - beta2^t)), multi_precision master weights.
#include "common.h"

namespace pa {

// out[i, :] = w[ids[i], :]   — one wave per row, 16-byte vectors
template <typename T>
__global__ __launch_bounds__(256) void embedding_fwd(const int64_t* __restrict__ ids, const T* __restrict__ w,
                                                     T* __restrict__ out, int n, int dim, int64_t vocab) {
  constexpr int E = 16 / sizeof(T);
  const int row = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  int64_t id = ids[row];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const T* src = w + id * dim;
  T* dst = out + (size_t)row * dim;
  for (int j = lane * E; j < dim; j += 64 * E)
    *reinterpret_cast<Pack<T, E>*>(dst + j) = *reinterpret_cast<const Pack<T, E>*>(src + j);
}

// dw32[ids[i], :] += dy[i, :]  (fp32 accumulation; 256-byte contiguous atomics per wave instruction)
template <typename T>
__global__ __launch_bounds__(256) void embedding_bwd(const int64_t* __restrict__ ids, const T* __restrict__ dy,
                                                     float* __restrict__ dw32, int n, int dim, int64_t vocab,
                                                     int64_t pad) {
  const int row = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  int64_t id = ids[row];
  if (id < 0 || id >= vocab || id == pad) return;
  const T* src = dy + (size_t)row * dim;
  float* dst = dw32 + id * dim;
  for (int j = lane; j < dim; j += 64) atomicAdd(dst + j, to_f(src[j]));
}

// Tiny tables (vocab <= 8: token-type / segment embeddings, where every row of the batch hits one
// of a few table rows): a thread owns two columns and sums its chunk of rows into per-vocab-row
// registers (the row's id is wave-uniform), then adds the V partial sums to dw32 — one atomic per
// (block, table element) instead of one per (batch row, element) on a few hot addresses.
template <typename T>
__global__ __launch_bounds__(256) void embedding_bwd_tiny(const int64_t* __restrict__ ids, const T* __restrict__ dy,
                                                          float* __restrict__ dw32, int n, int dim, int vocab,
                                                          int64_t pad, int rows_per_block) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 2;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(n, r0 + rows_per_block);
  float acc[8][2];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k][0] = acc[k][1] = 0.f;
  if (c < dim) {
#pragma unroll 8
    for (int row = r0; row < r1; ++row) {
      const int64_t id = ids[row];
      const T* src = dy + (size_t)row * dim + c;
      const float v0 = to_f(src[0]), v1 = to_f(src[1]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool hit = id == k && id != pad;
        acc[k][0] += hit ? v0 : 0.f;
        acc[k][1] += hit ? v1 : 0.f;
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < vocab && (acc[k][0] != 0.f || acc[k][1] != 0.f)) {
        atomicAdd(dw32 + (size_t)k * dim + c, acc[k][0]);
        atomicAdd(dw32 + (size_t)k * dim + c + 1, acc[k][1]);
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void cast_f32(const float* __restrict__ in, T* __restrict__ out, long long n,
                                                int accumulate) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    out[i] = from_f<T>(in[i] + (accumulate ? to_f(out[i]) : 0.f));
}

// Rotary embedding over x[B, S, H, D] (row stride = H*D, contiguous D).
//   half style (neox=0): pairs (i, i + D/2);  interleaved (neox=1): pairs (2i, 2i+1)
//   cos/sin: [S, D/2] fp32 tables;  sign = +1 forward, -1 backward (rotation by -theta)
template <typename T>
__global__ __launch_bounds__(256) void rope_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                   const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                   const int64_t* __restrict__ pos, int B, int S, int H, int D,
                                                   int interleaved, float sign) {
  const long long npairs = (long long)B * S * H * (D / 2);
  const int half = D / 2;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < npairs; i += (long long)gridDim.x * 256) {
    const int p = (int)(i % half);
    const long long bsh = i / half;
    const int s = (int)((bsh / H) % S);
    const int b = (int)(bsh / ((long long)H * S));
    const int ps = pos != nullptr ? (int)pos[(long long)b * S + s] : s;
    const float c = cosb[(size_t)ps * half + p];
    const float sn = sign * sinb[(size_t)ps * half + p];
    const long long base = bsh * D;
    const int i0 = interleaved ? 2 * p : p;
    const int i1 = interleaved ? 2 * p + 1 : p + half;
    const float a = to_f(x[base + i0]), bb = to_f(x[base + i1]);
    y[base + i0] = from_f<T>(a * c - bb * sn);
    y[base + i1] = from_f<T>(bb * c + a * sn);
  }
}

// Rotary embedding over strided rows: x / y [B, S, H, D] with D and H contiguous (head stride D)
// and row strides ldx / ldy (elements between consecutive (b, s) rows; batch stride S * ld) — the q /
// k slices of a fused QKV projection are read and their gradients written in place, no copies.
// One work item = 8 rotation pairs: 16-B loads of both pair halves and of the cos / sin rows.
// y may alias x (each item reads its pairs before writing them).
template <typename T>
__global__ __launch_bounds__(256) void rope_rows_kernel(const T* x, long long ldx, T* y, long long ldy,
                                                        const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                        const int64_t* __restrict__ pos, int B, int S, int H, int D,
                                                        int interleaved, float sign) {
  const int half = D / 2;
  const int g8 = half / 8;  // items per head
  const long long n = (long long)B * S * H * g8;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int g = (int)(i % g8);
    const long long bsh = i / g8;
    const int h = (int)(bsh % H);
    const long long bs = bsh / H;
    const int s = (int)(bs % S);
    const int b = (int)(bs / S);
    const int ps = pos != nullptr ? (int)pos[(long long)b * S + s] : s;
    const T* xr = x + bs * ldx + (long long)h * D;
    T* yr = y + bs * ldy + (long long)h * D;
    float c[8], sn[8];
    load_f<float, 4>(cosb + (size_t)ps * half + 8 * g, *reinterpret_cast<float(*)[4]>(&c[0]));
    load_f<float, 4>(cosb + (size_t)ps * half + 8 * g + 4, *reinterpret_cast<float(*)[4]>(&c[4]));
    load_f<float, 4>(sinb + (size_t)ps * half + 8 * g, *reinterpret_cast<float(*)[4]>(&sn[0]));
    load_f<float, 4>(sinb + (size_t)ps * half + 8 * g + 4, *reinterpret_cast<float(*)[4]>(&sn[4]));
    if (!interleaved) {  // pairs (p, p + D/2), p = 8 g .. 8 g + 7
      float a[8], bb[8], o0[8], o1[8];
      load_f<T, 8>(xr + 8 * g, a);
      load_f<T, 8>(xr + half + 8 * g, bb);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float se = sign * sn[e];
        o0[e] = a[e] * c[e] - bb[e] * se;
        o1[e] = bb[e] * c[e] + a[e] * se;
      }
      store_f<T, 8>(yr + 8 * g, o0);
      store_f<T, 8>(yr + half + 8 * g, o1);
    } else {  // pairs (2p, 2p + 1), p = 8 g .. 8 g + 7: elements 16 g .. 16 g + 15
      float v[16], o[16];
      load_f<T, 8>(xr + 16 * g, *reinterpret_cast<float(*)[8]>(&v[0]));
      load_f<T, 8>(xr + 16 * g + 8, *reinterpret_cast<float(*)[8]>(&v[8]));
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float se = sign * sn[e];
        o[2 * e] = v[2 * e] * c[e] - v[2 * e + 1] * se;
        o[2 * e + 1] = v[2 * e + 1] * c[e] + v[2 * e] * se;
      }
      store_f<T, 8>(yr + 16 * g, *reinterpret_cast<float(*)[8]>(&o[0]));
      store_f<T, 8>(yr + 16 * g + 8, *reinterpret_cast<float(*)[8]>(&o[8]));
    }
  }
}

// Paddle AdamW on a flat fp32 master buffer:
//   p *= (1 - lr * wd);  m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2
//   p -= lr * sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps * sqrt(1-b2^t))
// grad may be bf16/fp16/fp32; `lowp` (optional) receives the updated param in the model dtype.
// lr and (b1pow, b2pow) may be read from device scalars (lr_ptr, pows) so a captured hipGraph
// replays with fresh values.
typedef int nt_i4 __attribute__((ext_vector_type(4)));

// 16-byte streaming (nontemporal: no reuse, keep the caches for the rest) load / store of N
// elements of T (N * sizeof(T) == 16), converted to / from fp32
template <typename T, int N>
__device__ __forceinline__ void ld16(const T* __restrict__ ptr, float (&out)[N], bool nt) {
  static_assert(N * sizeof(T) == 16, "16-byte access");
  nt_i4 raw = nt ? __builtin_nontemporal_load(reinterpret_cast<const nt_i4*>(ptr)) : *reinterpret_cast<const nt_i4*>(ptr);
  const Pack<T, N> pk = __builtin_bit_cast(Pack<T, N>, raw);
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = to_f(pk.v[i]);
}

template <typename T, int N>
__device__ __forceinline__ void st16(T* __restrict__ ptr, const float* in, bool nt) {
  static_assert(N * sizeof(T) == 16, "16-byte access");
  Pack<T, N> pk;
#pragma unroll
  for (int i = 0; i < N; ++i) pk.v[i] = from_f<T>(in[i]);
  const nt_i4 raw = __builtin_bit_cast(nt_i4, pk);
  if (nt) __builtin_nontemporal_store(raw, reinterpret_cast<nt_i4*>(ptr));
  else *reinterpret_cast<nt_i4*>(ptr) = raw;
}

template <typename G, typename P, bool NTS = true>
__device__ __forceinline__ void adamw_vec8(float* __restrict__ p, const G* __restrict__ g, float* __restrict__ m,
                                           float* __restrict__ v, P* __restrict__ lowp, long long i, float gs,
                                           float decay, float b1, float b2, float step, float eps_hat) {
  constexpr int E = 8;
  float pv[E], gv[E], mv[E], vv[E];
  ld16<float, 4>(p + i, *reinterpret_cast<float(*)[4]>(pv), NTS);
  ld16<float, 4>(p + i + 4, *reinterpret_cast<float(*)[4]>(pv + 4), NTS);
  if constexpr (sizeof(G) == 2) {
    ld16<G, 8>(g + i, gv, NTS);
  } else {
    ld16<G, 4>(g + i, *reinterpret_cast<float(*)[4]>(gv), NTS);
    ld16<G, 4>(g + i + 4, *reinterpret_cast<float(*)[4]>(gv + 4), NTS);
  }
  ld16<float, 4>(m + i, *reinterpret_cast<float(*)[4]>(mv), NTS);
  ld16<float, 4>(m + i + 4, *reinterpret_cast<float(*)[4]>(mv + 4), NTS);
  ld16<float, 4>(v + i, *reinterpret_cast<float(*)[4]>(vv), NTS);
  ld16<float, 4>(v + i + 4, *reinterpret_cast<float(*)[4]>(vv + 4), NTS);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const float gg = gv[e] * gs;
    mv[e] = b1 * mv[e] + (1.f - b1) * gg;
    vv[e] = b2 * vv[e] + (1.f - b2) * gg * gg;
    // fast reciprocal: the update's relative error (~1 ulp) is far below bf16 resolution
    pv[e] = pv[e] * decay - step * mv[e] * __frcp_rn(__fsqrt_rn(vv[e]) + eps_hat);
  }
  st16<float, 4>(p + i, pv, NTS);
  st16<float, 4>(p + i + 4, pv + 4, NTS);
  st16<float, 4>(m + i, mv, NTS);
  st16<float, 4>(m + i + 4, mv + 4, NTS);
  st16<float, 4>(v + i, vv, NTS);
  st16<float, 4>(v + i + 4, vv + 4, NTS);
  if (lowp != nullptr) {
    if constexpr (sizeof(P) == 2) {
      st16<P, 8>(lowp + i, pv, NTS);
    } else {
      st16<P, 4>(lowp + i, pv, NTS);
      st16<P, 4>(lowp + i + 4, pv + 4, NTS);
    }
  }
}

// Unaligned fallback (views that do not start on a 16-byte boundary): one element per lane.
template <typename G, typename P>
__global__ __launch_bounds__(256) void adamw_scalar_kernel(float* __restrict__ p, const G* __restrict__ g,
                                                           float* __restrict__ m, float* __restrict__ v,
                                                           P* __restrict__ lowp, long long n,
                                                           const float* __restrict__ lr_ptr, float lr_host, float b1,
                                                           float b2, float eps, float wd, float b1pow, float b2pow,
                                                           const float* __restrict__ grad_scale,
    const float* __restrict__ pows) {
  if (pows != nullptr) {  // device-resident beta powers (graph-captured steps advance them)
    b1pow = pows[0];
    b2pow = pows[1];
  }
  const float lr = lr_ptr != nullptr ? *lr_ptr : lr_host;
  const float gs = grad_scale != nullptr ? *grad_scale : 1.f;
  const float bc2 = sqrtf(1.f - b2pow);
  const float step = lr * bc2 / (1.f - b1pow);
  const float decay = 1.f - lr * wd;
  const float eps_hat = eps * bc2;
  for (long long k = (long long)blockIdx.x * 256 + threadIdx.x; k < n; k += (long long)gridDim.x * 256) {
    const float gg = to_f(g[k]) * gs;
    float pv = p[k] * decay;
    const float mv = b1 * m[k] + (1.f - b1) * gg;
    const float vv = b2 * v[k] + (1.f - b2) * gg * gg;
    pv -= step * mv / (sqrtf(vv) + eps_hat);
    p[k] = pv;
    m[k] = mv;
    v[k] = vv;
    if (lowp != nullptr) lowp[k] = from_f<P>(pv);
  }
}

// Memory-bound (28 B/param read+write for bf16 grads/params with fp32 master/m/v): 8 params
// per lane (every access a full 16-byte vector, the bf16 gradient included).  ONE: one vector per
// lane over a grid that covers the buffer (no loop): 6.0 TB/s on a 1.3B-parameter buffer vs 5.7
// for a grid-stride loop with two vectors in flight per lane, and 4.8 with nontemporal loads
// (tools/adamw_variants.hip, profiles/r6o_adamw_variants.log) — plain loads and stores.
template <typename G, typename P, bool NTS, bool ONE = false>
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const G* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, P* __restrict__ lowp,
                                                    long long n, const float* __restrict__ lr_ptr, float lr_host,
                                                    float b1, float b2, float eps, float wd, float b1pow, float b2pow,
                                                    const float* __restrict__ grad_scale,
    const float* __restrict__ pows) {
  if (pows != nullptr) {  // device-resident beta powers (graph-captured steps advance them)
    b1pow = pows[0];
    b2pow = pows[1];
  }
  const float lr = lr_ptr != nullptr ? *lr_ptr : lr_host;
  const float gs = grad_scale != nullptr ? *grad_scale : 1.f;
  const float bc2 = sqrtf(1.f - b2pow);
  const float step = lr * bc2 / (1.f - b1pow);
  const float decay = 1.f - lr * wd;
  const float eps_hat = eps * bc2;
  constexpr int E = 8;
  const long long nv = n / E;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if constexpr (ONE) {
    if (i < nv) adamw_vec8<G, P, NTS>(p, g, m, v, lowp, i * E, gs, decay, b1, b2, step, eps_hat);
  } else {
    const long long stride = (long long)gridDim.x * 256;
    for (; i + stride < nv; i += 2 * stride) {
      adamw_vec8<G, P, NTS>(p, g, m, v, lowp, i * E, gs, decay, b1, b2, step, eps_hat);
      adamw_vec8<G, P, NTS>(p, g, m, v, lowp, (i + stride) * E, gs, decay, b1, b2, step, eps_hat);
    }
    if (i < nv) adamw_vec8<G, P, NTS>(p, g, m, v, lowp, i * E, gs, decay, b1, b2, step, eps_hat);
  }
  if (blockIdx.x == 0) {
    for (long long k = nv * E + threadIdx.x; k < n; k += 256) {
      const float gg = to_f(g[k]) * gs;
      float pv = p[k] * decay;
      const float mv = b1 * m[k] + (1.f - b1) * gg;
      const float vv = b2 * v[k] + (1.f - b2) * gg * gg;
      pv -= step * mv / (sqrtf(vv) + eps_hat);
      p[k] = pv;
      m[k] = mv;
      v[k] = vv;
      if (lowp != nullptr) lowp[k] = from_f<P>(pv);
    }
  }
}

// Fused (Nesterov) momentum over a flat buffer, paddle semantics (phi momentum_kernel, multi_precision):
//   g' = rescale * g + l2 * p ;  v = mu * v + g' ;  p -= lr * (nesterov ? g' + mu * v : v)
// fp32 master p / velocity v, gradient in the model dtype, optional low-precision param copy.
template <typename G, typename P>
__global__ __launch_bounds__(256) void momentum_kernel(float* __restrict__ p, const G* __restrict__ g,
                                                       float* __restrict__ v, P* __restrict__ lowp, long long n,
                                                       const float* __restrict__ lr_ptr, float lr_host, float mu,
                                                       float l2, float rescale, int nesterov,
                                                       const float* __restrict__ grad_scale) {
  const float lr = lr_ptr != nullptr ? *lr_ptr : lr_host;
  const float gs = (grad_scale != nullptr ? *grad_scale : 1.f) * rescale;
  constexpr int E = 4;
  const long long nv = n / E;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nv; i += (long long)gridDim.x * 256) {
    float pv[E], gv[E], vv[E];
    load_f<float, E>(p + i * E, pv);
    load_f<G, E>(g + i * E, gv);
    load_f<float, E>(v + i * E, vv);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float gg = gv[e] * gs + l2 * pv[e];
      vv[e] = mu * vv[e] + gg;
      pv[e] -= lr * (nesterov ? gg + mu * vv[e] : vv[e]);
    }
    store_f<float, E>(p + i * E, pv);
    store_f<float, E>(v + i * E, vv);
    if (lowp != nullptr) store_f<P, E>(lowp + i * E, pv);
  }
  if (blockIdx.x == 0) {
    for (long long k = nv * E + threadIdx.x; k < n; k += 256) {
      const float gg = to_f(g[k]) * gs + l2 * p[k];
      const float vk = mu * v[k] + gg;
      v[k] = vk;
      p[k] -= lr * (nesterov ? gg + mu * vk : vk);
      if (lowp != nullptr) lowp[k] = from_f<P>(p[k]);
    }
  }
}

// sum of squares of a flat buffer into out[blockIdx] (for global-norm clipping / found-inf check).
// 16-byte vector loads (8 x 16-bit or 4 x f32 per lane), 4 in flight per lane; scalar head/tail
// for a misaligned start or a ragged end.
template <typename T>
__global__ __launch_bounds__(256) void sumsq_kernel(const T* __restrict__ x, long long n, float* __restrict__ part) {
  constexpr int V = 16 / sizeof(T);
  __shared__ float red[4];
  float s = 0.f;
  const long long head = min(n, (long long)((16 - ((uintptr_t)x & 15)) & 15) / (long long)sizeof(T));
  const long long tid = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long nthr = (long long)gridDim.x * 256;
  if (tid < head) {
    const float v = to_f(x[tid]);
    s += v * v;
  }
  const T* xa = x + head;
  const long long nv = (n - head) / V;
  long long i = tid;
  for (; i + 3 * nthr < nv; i += 4 * nthr) {
    float a[4][V];
#pragma unroll
    for (int u = 0; u < 4; ++u) load_f<T, V>(xa + (i + u * nthr) * V, a[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < V; ++e) s += a[u][e] * a[u][e];
  }
  for (; i < nv; i += nthr) {
    float a[V];
    load_f<T, V>(xa + i * V, a);
#pragma unroll
    for (int e = 0; e < V; ++e) s += a[e] * a[e];
  }
  const long long t0 = head + nv * V;
  if (t0 + tid < n) {
    const float v = to_f(x[t0 + tid]);
    s += v * v;
  }
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

}  // namespace pa

using namespace pa;

PA_API hipError_t pa_embedding_fwd(const int64_t* ids, const void* w, void* out, int n, int dim, long long vocab,
                                   int dt, hipStream_t st) {
  if ((dim * (dt == 0 ? 4 : 2)) % 16 != 0) return hipErrorInvalidValue;
  PA_DISPATCH_DTYPE(dt, T, embedding_fwd<T><<<(n + 3) / 4, 256, 0, st>>>(ids, (const T*)w, (T*)out, n, dim, vocab));
  return hipGetLastError();
}

PA_API hipError_t pa_embedding_bwd_pad(const int64_t* ids, const void* dy, float* dw32, void* out, int n, int dim,
                                       long long vocab, int accumulate, long long pad, int dt, hipStream_t st);

// dw32 must be zeroed by the caller (hipMemsetAsync); out (param dtype) = dw32 (+ out if accumulate)
PA_API hipError_t pa_embedding_bwd(const int64_t* ids, const void* dy, float* dw32, void* out, int n, int dim,
                                   long long vocab, int accumulate, int dt, hipStream_t st) {
  return pa_embedding_bwd_pad(ids, dy, dw32, out, n, dim, vocab, accumulate, -1, dt, st);
}

// embedding gradient with a padding row (its gradient stays zero, torch / paddle padding_idx)
PA_API hipError_t pa_embedding_bwd_pad(const int64_t* ids, const void* dy, float* dw32, void* out, int n, int dim,
                                       long long vocab, int accumulate, long long pad, int dt, hipStream_t st) {
  PA_DISPATCH_DTYPE(dt, T, {
    if (vocab <= 8 && dim % 2 == 0) {
      const int rpb = 128;
      dim3 grid((dim / 2 + 255) / 256, (n + rpb - 1) / rpb);
      embedding_bwd_tiny<T><<<grid, 256, 0, st>>>(ids, (const T*)dy, dw32, n, dim, (int)vocab, pad, rpb);
    } else {
      embedding_bwd<T><<<(n + 3) / 4, 256, 0, st>>>(ids, (const T*)dy, dw32, n, dim, vocab, pad);
    }
    if (out != nullptr && (void*)out != (void*)dw32) {
      const long long tot = vocab * dim;
      cast_f32<T><<<grid_for(tot, 256, 256 * 8), 256, 0, st>>>(dw32, (T*)out, tot, accumulate);
    }
  });
  return hipGetLastError();
}

PA_API hipError_t pa_rope(const void* x, void* y, const float* cosb, const float* sinb, const int64_t* pos, int B,
                          int S, int H, int D, int interleaved, float sign, int dt, hipStream_t st) {
  const long long npairs = (long long)B * S * H * (D / 2);
  PA_DISPATCH_DTYPE(dt, T, rope_kernel<T><<<grid_for(npairs, 256, 256 * 8), 256, 0, st>>>(
                               (const T*)x, (T*)y, cosb, sinb, pos, B, S, H, D, interleaved, sign));
  return hipGetLastError();
}

// x, y: [B, S, H, D] rows of ldx / ldy elements (D % 16 == 0, 16-B aligned rows); y may be x.
PA_API hipError_t pa_rope_rows(const void* x, long long ldx, void* y, long long ldy, const float* cosb,
                               const float* sinb, const int64_t* pos, int B, int S, int H, int D, int interleaved,
                               float sign, int dt, hipStream_t st) {
  if (D % 16 || ldx % 8 || ldy % 8 || B <= 0 || S <= 0 || H <= 0) return hipErrorInvalidValue;
  const long long n = (long long)B * S * H * (D / 16);
  PA_DISPATCH_DTYPE(dt, T, rope_rows_kernel<T><<<grid_for(n, 256, 256 * 8), 256, 0, st>>>(
                               (const T*)x, ldx, (T*)y, ldy, cosb, sinb, pos, B, S, H, D, interleaved, sign));
  return hipGetLastError();
}

// A/B knobs for the streaming update: nontemporal 16-byte accesses (off: they cost 15-20 % on
// MI355X), and blocks per CU of the grid-stride form (0 = one vector per lane, the default)
static int g_adamw_nt = 0, g_adamw_bpc = 0;
PA_API void pa_adamw_tune(int nt, int blocks_per_cu) {
  g_adamw_nt = nt;
  g_adamw_bpc = blocks_per_cu > 0 ? blocks_per_cu : 0;
}

// gd = grad dtype, pd = low-precision param copy dtype (-1 = none)
PA_API hipError_t pa_adamw(float* p, const void* g, float* m, float* v, void* lowp, long long n, const float* lr_ptr,
                           float lr, float b1, float b2, float eps, float wd, float b1pow, float b2pow,
                           const float* grad_scale, const float* pows, int gd, int pd, hipStream_t st) {
  const long long nvec = n / 8;
  const bool one = g_adamw_bpc == 0 && nvec > 0 && (nvec + 255) / 256 < (1LL << 31);
  const int grid = one ? (int)((nvec + 255) / 256) : grid_for(n / 16 + 1, 256, 256 * g_adamw_bpc);
  // every 8-element access is a 16-byte vector (or two): all five streams must be 16-byte aligned
  const bool aligned = ((((uintptr_t)p | (uintptr_t)m | (uintptr_t)v | (uintptr_t)g | (uintptr_t)lowp) & 15) == 0);
#define PA_ADAM(G, P)                                                                                          \
  do {                                                                                                         \
    if (aligned && one && !g_adamw_nt)                                                                         \
      adamw_kernel<G, P, false, true><<<grid, 256, 0, st>>>(p, (const G*)g, m, v, (P*)lowp, n, lr_ptr, lr, b1, \
                                                            b2, eps, wd, b1pow, b2pow, grad_scale, pows);      \
    else if (aligned && one)                                                                                   \
      adamw_kernel<G, P, true, true><<<grid, 256, 0, st>>>(p, (const G*)g, m, v, (P*)lowp, n, lr_ptr, lr, b1,  \
                                                           b2, eps, wd, b1pow, b2pow, grad_scale, pows);       \
    else if (aligned && g_adamw_nt)                                                                            \
      adamw_kernel<G, P, true><<<grid, 256, 0, st>>>(p, (const G*)g, m, v, (P*)lowp, n, lr_ptr, lr, b1, b2, eps, \
                                                     wd, b1pow, b2pow, grad_scale, pows);                      \
    else if (aligned)                                                                                          \
      adamw_kernel<G, P, false><<<grid, 256, 0, st>>>(p, (const G*)g, m, v, (P*)lowp, n, lr_ptr, lr, b1, b2,   \
                                                      eps, wd, b1pow, b2pow, grad_scale, pows);                \
    else                                                                                                       \
      adamw_scalar_kernel<G, P><<<grid_for(n, 256, 256 * 8), 256, 0, st>>>(                                    \
          p, (const G*)g, m, v, (P*)lowp, n, lr_ptr, lr, b1, b2, eps, wd, b1pow, b2pow, grad_scale, pows);    \
  } while (0)
  if (pd < 0) lowp = nullptr;
  const int pp = pd < 0 ? 0 : pd;
  if (gd == 0 && pp == 0) PA_ADAM(float, float);
  else if (gd == 1 && pp == 1) PA_ADAM(bf16_t, bf16_t);
  else if (gd == 1 && pp == 0) PA_ADAM(bf16_t, float);
  else if (gd == 0 && pp == 1) PA_ADAM(float, bf16_t);
  else if (gd == 2 && pp == 2) PA_ADAM(f16_t, f16_t);
  else if (gd == 0 && pp == 2) PA_ADAM(float, f16_t);
  else return hipErrorInvalidValue;
#undef PA_ADAM
  return hipGetLastError();
}

PA_API int pa_sumsq_parts() { return 2048; }

PA_API hipError_t pa_sumsq(const void* x, long long n, float* part, int dt, hipStream_t st) {
  PA_DISPATCH_DTYPE(dt, T, sumsq_kernel<T><<<2048, 256, 0, st>>>((const T*)x, n, part));
  return hipGetLastError();
}

PA_API hipError_t pa_momentum(float* p, const void* g, float* v, void* lowp, long long n, const float* lr_ptr, float lr,
                              float mu, float l2, float rescale, int nesterov, const float* grad_scale, int gd,
                              int pd, hipStream_t st) {
  if ((((uintptr_t)p | (uintptr_t)v | (uintptr_t)g | (uintptr_t)lowp) & 7) != 0) return hipErrorInvalidValue;
  const int grid = grid_for(n / 4 + 1, 256, 256 * 8);
  if (pd < 0) lowp = nullptr;
#define PA_MOM(G, P)                                                                                         \
  momentum_kernel<G, P><<<grid, 256, 0, st>>>(p, (const G*)g, v, (P*)lowp, n, lr_ptr, lr, mu, l2, rescale, \
                                              nesterov, grad_scale)
  const int pp = pd < 0 ? 0 : pd;
  if (gd == 0 && pp == 0) PA_MOM(float, float);
  else if (gd == 1 && pp == 1) PA_MOM(bf16_t, bf16_t);
  else if (gd == 1 && pp == 0) PA_MOM(bf16_t, float);
  else if (gd == 2 && pp == 2) PA_MOM(f16_t, f16_t);
  else if (gd == 0 && pp == 1) PA_MOM(float, bf16_t);
  else return hipErrorInvalidValue;
#undef PA_MOM
  return hipGetLastError();
}
