// Row softmax (fwd/bwd, optional causal upper-triangle mask) and fused softmax-cross-entropy.
//
// Reference semantics: paddle/phi/kernels/gpudnn/softmax_gpudnn.h,
// paddle/phi/kernels/fusion/gpu/fused_softmax_mask_upper_triangle_kernel.cu,
// paddle/phi/kernels/gpu/cross_entropy_kernel.cu (softmax_with_cross_entropy, hard labels).
//
// Softmax: one wave per row when the row fits in registers (cols <= 64*E*MAXC), online
// (max, sum) in one pass otherwise. Cross-entropy: one 256-thread block per row streams
// the vocab row ONCE with an online max/sum (16-byte loads), writes loss and the row
// logsumexp; the backward streams it once more and writes softmax − onehot scaled by
// dloss — the [rows, vocab] probability tensor never exists in HBM.
#include "common.h"

namespace pa {

template <typename T, int MAXC, bool CAUSAL>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int rows,
                                                          int cols, int causal_cols_per_row_offset) {
  constexpr int E = 16 / sizeof(T);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * cols;
  // CAUSAL: row r of a [.., S, S] score matrix keeps columns <= (r % S) + offset
  const int limit = CAUSAL ? (row % causal_cols_per_row_offset) : cols - 1;
  float v[MAXC][E];
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int j = (c * 64 + lane) * E;
    if (j < cols) {
      load_f<T, E>(x + base + j, v[c]);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (CAUSAL && j + e > limit) v[c][e] = -INFINITY;
        m = fmaxf(m, v[c][e]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) v[c][e] = -INFINITY;
    }
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
#pragma unroll
    for (int e = 0; e < E; ++e) {
      v[c][e] = __expf(v[c][e] - m);
      s += v[c][e];
    }
  const float inv = 1.0f / wave_sum(s);
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int j = (c * 64 + lane) * E;
    if (j < cols) {
      float o[E];
#pragma unroll
      for (int e = 0; e < E; ++e) o[e] = v[c][e] * inv;
      store_f<T, E>(y + base + j, o);
    }
  }
}

template <typename T, bool CAUSAL>
__global__ __launch_bounds__(256) void softmax_fwd_generic(const T* __restrict__ x, T* __restrict__ y, int rows,
                                                           int cols, int S) {
  __shared__ float red[4];
  const int row = blockIdx.x;
  const size_t base = (size_t)row * cols;
  const int limit = CAUSAL ? (row % S) : cols - 1;
  float m = -INFINITY, s = 0.f;
  for (int j = threadIdx.x; j <= limit && j < cols; j += 256) {
    const float v = to_f(x[base + j]);
    const float nm = fmaxf(m, v);
    s = s * __expf(m - nm) + __expf(v - nm);
    m = nm;
  }
  const float M = block_max<256>(m, red);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - M);
  const float inv = 1.0f / block_sum<256>(s, red);
  for (int j = threadIdx.x; j < cols; j += 256) {
    const float v = (j <= limit) ? __expf(to_f(x[base + j]) - M) * inv : 0.f;
    y[base + j] = from_f<T>(v);
  }
}

// dx = y * (dy - sum(dy * y))
template <typename T, int MAXC>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const T* __restrict__ y, const T* __restrict__ dy,
                                                          T* __restrict__ dx, int rows, int cols) {
  constexpr int E = 16 / sizeof(T);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * cols;
  float yv[MAXC][E], gv[MAXC][E];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int j = (c * 64 + lane) * E;
    if (j < cols) {
      load_f<T, E>(y + base + j, yv[c]);
      load_f<T, E>(dy + base + j, gv[c]);
#pragma unroll
      for (int e = 0; e < E; ++e) s += yv[c][e] * gv[c][e];
    }
  }
  s = wave_sum(s);
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int j = (c * 64 + lane) * E;
    if (j < cols) {
      float o[E];
#pragma unroll
      for (int e = 0; e < E; ++e) o[e] = yv[c][e] * (gv[c][e] - s);
      store_f<T, E>(dx + base + j, o);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void softmax_bwd_generic(const T* __restrict__ y, const T* __restrict__ dy,
                                                           T* __restrict__ dx, int rows, int cols) {
  __shared__ float red[4];
  const size_t base = (size_t)blockIdx.x * cols;
  float s = 0.f;
  for (int j = threadIdx.x; j < cols; j += 256) s += to_f(y[base + j]) * to_f(dy[base + j]);
  s = block_sum<256>(s, red);
  for (int j = threadIdx.x; j < cols; j += 256)
    dx[base + j] = from_f<T>(to_f(y[base + j]) * (to_f(dy[base + j]) - s));
}

// ---------------------------------------------------------------- cross entropy
// loss[r] = lse[r] - x[r, label[r]]  (0 where label == ignore_index)
template <typename T>
__global__ __launch_bounds__(256) void xent_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       float* __restrict__ loss, float* __restrict__ lse, int rows,
                                                       int vocab, int64_t ignore_index) {
  constexpr int E = 16 / sizeof(T);
  __shared__ float red[8];
  const int row = blockIdx.x;
  const T* xr = logits + (size_t)row * vocab;
  float m = -INFINITY, s = 0.f;
  const bool vec = (vocab % E) == 0;
  if (vec) {
    for (int j = threadIdx.x * E; j < vocab; j += 256 * E) {
      float v[E];
      load_f<T, E>(xr + j, v);
      float lm = v[0];
#pragma unroll
      for (int e = 1; e < E; ++e) lm = fmaxf(lm, v[e]);
      const float nm = fmaxf(m, lm);
      float acc = s * __expf(m - nm);
#pragma unroll
      for (int e = 0; e < E; ++e) acc += __expf(v[e] - nm);
      s = acc;
      m = nm;
    }
  } else {
    for (int j = threadIdx.x; j < vocab; j += 256) {
      const float v = to_f(xr[j]);
      const float nm = fmaxf(m, v);
      s = s * __expf(m - nm) + __expf(v - nm);
      m = nm;
    }
  }
  const float M = block_max<256>(m, red);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - M);
  const float S = block_sum<256>(s, red);
  if (threadIdx.x == 0) {
    const float l = M + __logf(S);
    lse[row] = l;
    const int64_t lab = labels[row];
    loss[row] = (lab == ignore_index || lab < 0 || lab >= vocab) ? 0.f : l - to_f(xr[lab]);
  }
}

// dlogits[r, j] = dloss[r] * (exp(x - lse) - [j == label])
template <typename T>
__global__ __launch_bounds__(256) void xent_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse, const float* __restrict__ dloss,
                                                       int dloss_stride, T* __restrict__ dlogits, int rows, int vocab,
                                                       int64_t ignore_index) {
  constexpr int E = 16 / sizeof(T);
  const int row = blockIdx.x;
  const int64_t lab = labels[row];
  const bool ign = (lab == ignore_index || lab < 0 || lab >= vocab);
  const float g = ign ? 0.f : dloss[(size_t)row * dloss_stride];
  const float l = lse[row];
  const T* xr = logits + (size_t)row * vocab;
  T* dr = dlogits + (size_t)row * vocab;
  if ((vocab % E) == 0) {
    for (int j = threadIdx.x * E; j < vocab; j += 256 * E) {
      float v[E];
      load_f<T, E>(xr + j, v);
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] = g * (__expf(v[e] - l) - ((j + e) == lab ? 1.f : 0.f));
      store_f<T, E>(dr + j, v);
    }
  } else {
    for (int j = threadIdx.x; j < vocab; j += 256)
      dr[j] = from_f<T>(g * (__expf(to_f(xr[j]) - l) - (j == lab ? 1.f : 0.f)));
  }
}

template <typename T>
hipError_t launch_softmax_fwd(const void* x, void* y, int rows, int cols, int causal_S, hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  const int chunks = (cols + 64 * E - 1) / (64 * E);
  const bool vec = (cols % E) == 0;
  dim3 g((rows + 3) / 4);
  const bool causal = causal_S > 0;
#define PA_SM(C)                                                                                           \
  if (causal) softmax_fwd_kernel<T, C, true><<<g, 256, 0, st>>>((const T*)x, (T*)y, rows, cols, causal_S); \
  else softmax_fwd_kernel<T, C, false><<<g, 256, 0, st>>>((const T*)x, (T*)y, rows, cols, 1)
  if (vec && chunks <= 1) { PA_SM(1); }
  else if (vec && chunks <= 2) { PA_SM(2); }
  else if (vec && chunks <= 4) { PA_SM(4); }
  else if (vec && chunks <= 8) { PA_SM(8); }
  else if (causal) softmax_fwd_generic<T, true><<<rows, 256, 0, st>>>((const T*)x, (T*)y, rows, cols, causal_S);
  else softmax_fwd_generic<T, false><<<rows, 256, 0, st>>>((const T*)x, (T*)y, rows, cols, 1);
#undef PA_SM
  return hipGetLastError();
}

template <typename T>
hipError_t launch_softmax_bwd(const void* y, const void* dy, void* dx, int rows, int cols, hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  const int chunks = (cols + 64 * E - 1) / (64 * E);
  const bool vec = (cols % E) == 0;
  dim3 g((rows + 3) / 4);
  if (vec && chunks <= 1) softmax_bwd_kernel<T, 1><<<g, 256, 0, st>>>((const T*)y, (const T*)dy, (T*)dx, rows, cols);
  else if (vec && chunks <= 2) softmax_bwd_kernel<T, 2><<<g, 256, 0, st>>>((const T*)y, (const T*)dy, (T*)dx, rows, cols);
  else if (vec && chunks <= 4) softmax_bwd_kernel<T, 4><<<g, 256, 0, st>>>((const T*)y, (const T*)dy, (T*)dx, rows, cols);
  else softmax_bwd_generic<T><<<rows, 256, 0, st>>>((const T*)y, (const T*)dy, (T*)dx, rows, cols);
  return hipGetLastError();
}

}  // namespace pa

using namespace pa;

PA_API hipError_t pa_softmax_fwd(const void* x, void* y, int rows, int cols, int causal_S, int dt, hipStream_t st) {
  PA_DISPATCH_DTYPE(dt, T, return launch_softmax_fwd<T>(x, y, rows, cols, causal_S, st));
  return hipSuccess;
}

PA_API hipError_t pa_softmax_bwd(const void* y, const void* dy, void* dx, int rows, int cols, int dt, hipStream_t st) {
  PA_DISPATCH_DTYPE(dt, T, return launch_softmax_bwd<T>(y, dy, dx, rows, cols, st));
  return hipSuccess;
}

PA_API hipError_t pa_xent_fwd(const void* logits, const int64_t* labels, float* loss, float* lse, int rows, int vocab,
                              int64_t ignore_index, int dt, hipStream_t st) {
  PA_DISPATCH_DTYPE(dt, T, xent_fwd_kernel<T><<<rows, 256, 0, st>>>((const T*)logits, labels, loss, lse, rows, vocab,
                                                                    ignore_index));
  return hipGetLastError();
}

PA_API hipError_t pa_xent_bwd(const void* logits, const int64_t* labels, const float* lse, const float* dloss,
                              int dloss_stride, void* dlogits, int rows, int vocab, int64_t ignore_index, int dt,
                              hipStream_t st) {
  PA_DISPATCH_DTYPE(dt, T, xent_bwd_kernel<T><<<rows, 256, 0, st>>>((const T*)logits, labels, lse, dloss,
                                                                    dloss_stride, (T*)dlogits, rows, vocab,
                                                                    ignore_index));
  return hipGetLastError();
}
