// LayerNorm / RMSNorm forward + backward for gfx950.
//
// Reference semantics: paddle/phi/kernels/gpu/layer_norm_kernel.cu, layer_norm_grad_kernel.cu,
// paddle/phi/kernels/fusion/gpu/fused_layernorm_kernel.cu (rms_norm), with the optional fused
// residual add of fused_bias_dropout_residual_layer_norm.
//
// Design (memory-bound; HBM is the roof):
//  * forward: ONE wave per row, 16-byte vector loads (8 x bf16 per lane), the row cached in
//    registers (cols <= MAXC*64*E), exact two-pass mean/variance in fp32, mean/rstd saved
//    for backward. 4 rows per 256-thread block → rows/4 blocks (≫256 CUs for LLM shapes).
//  * backward: ONE block (4 waves) per row iteration, grid-stride over rows so each block's
//    per-column dgamma/dbeta partials stay in registers across its rows; partials are
//    written once per block and summed by a column-parallel finisher kernel (no atomics,
//    bitwise deterministic).
#include "common.h"

namespace pa {

template <typename T, typename WT, int MAXC, bool RMS>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                       const WT* __restrict__ w, const WT* __restrict__ b,
                                                       T* __restrict__ y, T* __restrict__ sum_out,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int rows, int cols, float eps) {
  constexpr int E = 16 / sizeof(T);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * cols;
  float v[MAXC][E];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int j = (c * 64 + lane) * E;
    if (j < cols) {
      load_f<T, E>(x + base + j, v[c]);
      if (res != nullptr) {
        float r[E];
        load_f<T, E>(res + base + j, r);
#pragma unroll
        for (int e = 0; e < E; ++e) v[c][e] += r[e];
        // the pre-norm residual stream is the rounded sum, exactly as an unfused add would store it
#pragma unroll
        for (int e = 0; e < E; ++e) v[c][e] = to_f(from_f<T>(v[c][e]));
        store_f<T, E>(sum_out + base + j, v[c]);
      }
#pragma unroll
      for (int e = 0; e < E; ++e) s += v[c][e];
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) v[c][e] = 0.f;
    }
  }
  const float inv_n = 1.0f / cols;
  float mean = 0.f;
  if (!RMS) mean = wave_sum(s) * inv_n;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int j = (c * 64 + lane) * E;
    if (j < cols) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float d = v[c][e] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) * inv_n + eps);
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int j = (c * 64 + lane) * E;
    if (j < cols) {
      float wv[E], o[E];
      load_f<WT, E>(w + j, wv);
      if (!RMS && b != nullptr) {
        float bv[E];
        load_f<WT, E>(b + j, bv);
#pragma unroll
        for (int e = 0; e < E; ++e) o[e] = (v[c][e] - mean) * rstd * wv[e] + bv[e];
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) o[e] = (v[c][e] - mean) * rstd * wv[e];
      }
      store_f<T, E>(y + base + j, o);
    }
  }
  if (lane == 0) {
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Generic scalar fallback (cols not a multiple of the vector width, or very wide rows).
template <typename T, typename WT, bool RMS>
__global__ __launch_bounds__(256) void norm_fwd_generic(const T* __restrict__ x, const T* __restrict__ res,
                                                        const WT* __restrict__ w, const WT* __restrict__ b,
                                                        T* __restrict__ y, T* __restrict__ sum_out,
                                                        float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                        int rows, int cols, float eps) {
  __shared__ float red[4];
  const int row = blockIdx.x;
  const size_t base = (size_t)row * cols;
  float s = 0.f;
  for (int j = threadIdx.x; j < cols; j += 256) {
    float v = to_f(x[base + j]);
    if (res != nullptr) {
      v = to_f(from_f<T>(v + to_f(res[base + j])));
      sum_out[base + j] = from_f<T>(v);
    }
    s += v;
  }
  const float mean = RMS ? 0.f : block_sum<256>(s, red) / cols;
  float q = 0.f;
  for (int j = threadIdx.x; j < cols; j += 256) {
    const float v = (res != nullptr ? to_f(sum_out[base + j]) : to_f(x[base + j])) - mean;
    q += v * v;
  }
  const float rstd = rsqrtf(block_sum<256>(q, red) / cols + eps);
  for (int j = threadIdx.x; j < cols; j += 256) {
    const float v = (res != nullptr ? to_f(sum_out[base + j]) : to_f(x[base + j])) - mean;
    float o = v * rstd * to_f(w[j]);
    if (!RMS && b != nullptr) o += to_f(b[j]);
    y[base + j] = from_f<T>(o);
  }
  if (threadIdx.x == 0) {
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Backward: block (256 threads) per row, grid-stride over rows.
// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * w        (LayerNorm)
// dx = rstd * (g - xhat * mean(g * xhat))                               (RMSNorm)
// dw_part[blockIdx] += dy * xhat ; db_part[blockIdx] += dy
template <typename T, typename WT, int MAXC, bool RMS>
__global__ __launch_bounds__(256) void norm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                       const WT* __restrict__ w, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, const T* __restrict__ dsum,
                                                       T* __restrict__ dx, float* __restrict__ dw_part,
                                                       float* __restrict__ db_part, int rows, int cols) {
  constexpr int E = 16 / sizeof(T);
  __shared__ float red[8];
  const int tid = threadIdx.x;
  float aw[MAXC][E], ab[MAXC][E], wv[MAXC][E];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int j = (c * 256 + tid) * E;
#pragma unroll
    for (int e = 0; e < E; ++e) { aw[c][e] = 0.f; ab[c][e] = 0.f; wv[c][e] = 0.f; }
    if (j < cols) load_f<WT, E>(w + j, wv[c]);
  }
  const float inv_n = 1.0f / cols;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const size_t base = (size_t)row * cols;
    const float mu = RMS ? 0.f : mean[row];
    const float rs = rstd[row];
    float xh[MAXC][E], g[MAXC][E];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int j = (c * 256 + tid) * E;
      if (j < cols) {
        float xv[E], dv[E];
        load_f<T, E>(x + base + j, xv);
        load_f<T, E>(dy + base + j, dv);
#pragma unroll
        for (int e = 0; e < E; ++e) {
          xh[c][e] = (xv[e] - mu) * rs;
          g[c][e] = dv[e] * wv[c][e];
          s1 += g[c][e];
          s2 += g[c][e] * xh[c][e];
          aw[c][e] += dv[e] * xh[c][e];
          ab[c][e] += dv[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) { xh[c][e] = 0.f; g[c][e] = 0.f; }
      }
    }
    // two block reductions fused into one barrier pair
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if ((tid & 63) == 0) { red[tid >> 6] = s1; red[4 + (tid >> 6)] = s2; }
    __syncthreads();
    const float m1 = RMS ? 0.f : (red[0] + red[1] + red[2] + red[3]) * inv_n;
    const float m2 = (red[4] + red[5] + red[6] + red[7]) * inv_n;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int j = (c * 256 + tid) * E;
      if (j < cols) {
        float o[E];
#pragma unroll
        for (int e = 0; e < E; ++e) o[e] = rs * (g[c][e] - m1 - xh[c][e] * m2);
        if (dsum != nullptr) {  // gradient flowing into the residual stream from later layers
          float ds[E];
          load_f<T, E>(dsum + base + j, ds);
#pragma unroll
          for (int e = 0; e < E; ++e) o[e] += ds[e];
        }
        store_f<T, E>(dx + base + j, o);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int j = (c * 256 + tid) * E;
    if (j < cols) {
      float* pw = dw_part + (size_t)blockIdx.x * cols + j;
#pragma unroll
      for (int e = 0; e < E; ++e) pw[e] = aw[c][e];
      if (!RMS) {
        float* pb = db_part + (size_t)blockIdx.x * cols + j;
#pragma unroll
        for (int e = 0; e < E; ++e) pb[e] = ab[c][e];
      }
    }
  }
}

template <typename T, typename WT, bool RMS>
__global__ __launch_bounds__(256) void norm_bwd_generic(const T* __restrict__ dy, const T* __restrict__ x,
                                                        const WT* __restrict__ w, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, const T* __restrict__ dsum,
                                                        T* __restrict__ dx, float* __restrict__ dw_part,
                                                        float* __restrict__ db_part, int rows, int cols) {
  __shared__ float red[8];
  for (int j = threadIdx.x; j < cols; j += 256) {
    dw_part[(size_t)blockIdx.x * cols + j] = 0.f;
    if (!RMS) db_part[(size_t)blockIdx.x * cols + j] = 0.f;
  }
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const size_t base = (size_t)row * cols;
    const float mu = RMS ? 0.f : mean[row];
    const float rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
    for (int j = threadIdx.x; j < cols; j += 256) {
      const float xh = (to_f(x[base + j]) - mu) * rs;
      const float d = to_f(dy[base + j]);
      const float g = d * to_f(w[j]);
      s1 += g;
      s2 += g * xh;
      dw_part[(size_t)blockIdx.x * cols + j] += d * xh;
      if (!RMS) db_part[(size_t)blockIdx.x * cols + j] += d;
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = s1; red[4 + (threadIdx.x >> 6)] = s2; }
    __syncthreads();
    const float m1 = RMS ? 0.f : (red[0] + red[1] + red[2] + red[3]) / cols;
    const float m2 = (red[4] + red[5] + red[6] + red[7]) / cols;
    __syncthreads();
    for (int j = threadIdx.x; j < cols; j += 256) {
      const float xh = (to_f(x[base + j]) - mu) * rs;
      const float g = to_f(dy[base + j]) * to_f(w[j]);
      float o = rs * (g - m1 - xh * m2);
      if (dsum != nullptr) o += to_f(dsum[base + j]);
      dx[base + j] = from_f<T>(o);
    }
  }
}

// out[c] = sum_p part[p, c]: block = 4 waves x 64 columns; the waves split the P partial rows
// (each wave-row read is 256 contiguous bytes), then a 4-way LDS reduce.  Deterministic.
template <typename WT>
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part, WT* __restrict__ out, int P,
                                                     int cols) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < cols) {
    int p = w;
    for (; p + 12 < P; p += 16) {  // 4 independent loads in flight per lane
      s += part[(size_t)p * cols + c] + part[(size_t)(p + 4) * cols + c] + part[(size_t)(p + 8) * cols + c] +
           part[(size_t)(p + 12) * cols + c];
    }
    for (; p < P; p += 4) s += part[(size_t)p * cols + c];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < cols) out[c] = from_f<WT>(red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]);
}

template <typename T, typename WT, bool RMS>
hipError_t launch_fwd(const void* x, const void* res, const void* w, const void* b, void* y, void* sum_out,
                      float* mean, float* rstd, int rows, int cols, float eps, hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  const T* xp = (const T*)x;
  const int chunks = (cols + 64 * E - 1) / (64 * E);
  const bool vec_ok = (cols % E) == 0;
  dim3 grid((rows + 3) / 4), block(256);
#define PA_NF(C) \
  norm_fwd_kernel<T, WT, C, RMS><<<grid, block, 0, st>>>(xp, (const T*)res, (const WT*)w, (const WT*)b, (T*)y, \
                                                         (T*)sum_out, mean, rstd, rows, cols, eps)
  if (vec_ok && chunks <= 1) PA_NF(1);
  else if (vec_ok && chunks <= 2) PA_NF(2);
  else if (vec_ok && chunks <= 4) PA_NF(4);
  else if (vec_ok && chunks <= 8) PA_NF(8);
  else if (vec_ok && chunks <= 16 && sizeof(T) == 2) PA_NF(16);
  else
    norm_fwd_generic<T, WT, RMS><<<rows, 256, 0, st>>>(xp, (const T*)res, (const WT*)w, (const WT*)b, (T*)y,
                                                        (T*)sum_out, mean, rstd, rows, cols, eps);
#undef PA_NF
  return hipGetLastError();
}

template <typename T, typename WT, bool RMS>
hipError_t launch_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                      const void* dsum, void* dx, float* part, void* dw, void* db, int rows, int cols, int nparts,
                      hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  const int chunks = (cols + 256 * E - 1) / (256 * E);
  const bool vec_ok = (cols % E) == 0;
  float* dw_part = part;
  float* db_part = part + (size_t)nparts * cols;
#define PA_NB(C)                                                                                              \
  norm_bwd_kernel<T, WT, C, RMS><<<nparts, 256, 0, st>>>((const T*)dy, (const T*)x, (const WT*)w, mean, rstd, \
                                                         (const T*)dsum, (T*)dx, dw_part, db_part, rows, cols)
  if (vec_ok && chunks <= 1) PA_NB(1);
  else if (vec_ok && chunks <= 2) PA_NB(2);
  else if (vec_ok && chunks <= 4) PA_NB(4);
  else if (vec_ok && chunks <= 8 && sizeof(T) == 2) PA_NB(8);
  else
    norm_bwd_generic<T, WT, RMS><<<nparts, 256, 0, st>>>((const T*)dy, (const T*)x, (const WT*)w, mean, rstd,
                                                         (const T*)dsum, (T*)dx, dw_part, db_part, rows, cols);
#undef PA_NB
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int g = (cols + 63) / 64;
  colsum_kernel<WT><<<g, 256, 0, st>>>(dw_part, (WT*)dw, nparts, cols);
  if (!RMS && db != nullptr) colsum_kernel<WT><<<g, 256, 0, st>>>(db_part, (WT*)db, nparts, cols);
  return hipGetLastError();
}

}  // namespace pa

using namespace pa;

#define PA_NORM_DISPATCH(xd, wd, RMS, CALL)                                        \
  if (xd == 0 && wd == 0) { using T = float; using WT = float; return CALL; }      \
  if (xd == 1 && wd == 1) { using T = bf16_t; using WT = bf16_t; return CALL; }    \
  if (xd == 1 && wd == 0) { using T = bf16_t; using WT = float; return CALL; }     \
  if (xd == 2 && wd == 2) { using T = f16_t; using WT = f16_t; return CALL; }      \
  if (xd == 2 && wd == 0) { using T = f16_t; using WT = float; return CALL; }      \
  return hipErrorInvalidValue;

// Number of partial rows the backward writes (callers size `part` as 2 * nparts * cols floats).
PA_API int pa_norm_bwd_nparts(int rows) { return rows < 512 ? (rows < 1 ? 1 : rows) : 512; }

PA_API hipError_t pa_layernorm_fwd(const void* x, const void* res, const void* w, const void* b, void* y,
                                   void* sum_out, float* mean, float* rstd, int rows, int cols, float eps, int xd,
                                   int wd, hipStream_t st) {
  PA_NORM_DISPATCH(xd, wd, false,
                   (launch_fwd<T, WT, false>(x, res, w, b, y, sum_out, mean, rstd, rows, cols, eps, st)))
}

PA_API hipError_t pa_rmsnorm_fwd(const void* x, const void* res, const void* w, void* y, void* sum_out, float* rstd,
                                 int rows, int cols, float eps, int xd, int wd, hipStream_t st) {
  PA_NORM_DISPATCH(xd, wd, true,
                   (launch_fwd<T, WT, true>(x, res, w, nullptr, y, sum_out, nullptr, rstd, rows, cols, eps, st)))
}

PA_API hipError_t pa_layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                                   const void* dsum, void* dx, float* part, void* dw, void* db, int rows, int cols,
                                   int xd, int wd, hipStream_t st) {
  const int np = pa_norm_bwd_nparts(rows);
  PA_NORM_DISPATCH(xd, wd, false,
                   (launch_bwd<T, WT, false>(dy, x, w, mean, rstd, dsum, dx, part, dw, db, rows, cols, np, st)))
}

PA_API hipError_t pa_rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd, const void* dsum,
                                 void* dx, float* part, void* dw, int rows, int cols, int xd, int wd,
                                 hipStream_t st) {
  const int np = pa_norm_bwd_nparts(rows);
  PA_NORM_DISPATCH(xd, wd, true,
                   (launch_bwd<T, WT, true>(dy, x, w, nullptr, rstd, dsum, dx, part, dw, nullptr, rows, cols, np, st)))
}
