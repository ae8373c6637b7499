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

// Dropout keep-mask of the fused (bias +) dropout + residual + norm path: a stateless hash of
// (seed, offset, 16-byte vector index of the element in the [rows, cols] matrix, lane in the
// vector), so the backward regenerates it bit-exactly without a stored mask.
struct DropSpec {
  float p;       // drop probability (0 < p < 1 when DROP)
  uint32_t seed, offset;
};

// Each 32-bit hash gives two 16-bit uniforms (one hash per PAIR of elements: the per-element hash
// made this VALU the larger half of the fused norm kernels' issue); p is applied at 1/65536
// resolution and the keep scale matches the quantised rate exactly.
template <int E>
__device__ __forceinline__ void drop_mask(const DropSpec& d, size_t vec_index, float (&m)[E]) {
  const uint32_t thr = (uint32_t)(d.p * 65536.f + 0.5f);
  const float scale = 65536.f / (float)(65536u - min(thr, 65535u));
  const uint32_t h0 = hash3(d.seed, d.offset, (uint32_t)vec_index);
#pragma unroll
  for (int e = 0; e < E; e += 2) {
    const uint32_t h = (e == 0) ? h0 : hash3(h0, (uint32_t)e, 0x2545F491u);
    m[e] = (h & 0xFFFFu) >= thr ? scale : 0.f;
    if (e + 1 < E) m[e + 1] = (h >> 16) >= thr ? scale : 0.f;
  }
}

// DROP: v = dropout(x + xbias) + res   (xbias optional, same dtype as x; res required)
template <typename T, typename WT, int MAXC, bool RMS, bool DROP>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                       const WT* __restrict__ w, const WT* __restrict__ b,
                                                       T* __restrict__ y, T* __restrict__ sum_out,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int rows, int cols, float eps, const T* __restrict__ xbias,
                                                       DropSpec dsp) {
  dsp.seed = rng_mix(dsp.seed);  // graph-captured steps: per-replay stream
  constexpr int E = 16 / sizeof(T);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * cols;
  float v[MAXC][E];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int j = (c * 64 + lane) * E;
    if (j < cols) {
      load_f<T, E>(x + base + j, v[c]);
      if constexpr (DROP) {
        if (xbias != nullptr) {
          float xb[E];
          load_f<T, E>(xbias + j, xb);
#pragma unroll
          for (int e = 0; e < E; ++e) v[c][e] += xb[e];
        }
        float m[E];
        drop_mask<E>(dsp, (base + j) / E, m);
#pragma unroll
        for (int e = 0; e < E; ++e) v[c][e] *= m[e];
      }
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
// DROP (fused bias + dropout + residual forward): dx is the residual-stream gradient,
// dxd = dx * keep / (1 - p) the gradient of the pre-dropout input, and
// xb_part[blockIdx] += dxd (the partial bias gradient, when xb_part != nullptr).
template <typename T, typename WT, int MAXC, bool RMS, bool DROP>
__global__ __launch_bounds__(256) void norm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                       const WT* __restrict__ w, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, const T* __restrict__ dsum,
                                                       T* __restrict__ dx, float* __restrict__ dw_part,
                                                       float* __restrict__ db_part, int rows, int cols,
                                                       T* __restrict__ dxd, float* __restrict__ xb_part,
                                                       DropSpec dsp) {
  dsp.seed = rng_mix(dsp.seed);  // graph-captured steps: per-replay stream
  constexpr int E = 16 / sizeof(T);
  __shared__ float red[8];
  const int tid = threadIdx.x;
  float aw[MAXC][E], ab[MAXC][E], wv[MAXC][E], axb[DROP ? MAXC : 1][E];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int j = (c * 256 + tid) * E;
#pragma unroll
    for (int e = 0; e < E; ++e) { aw[c][e] = 0.f; ab[c][e] = 0.f; wv[c][e] = 0.f; }
    if constexpr (DROP) {
#pragma unroll
      for (int e = 0; e < E; ++e) axb[c][e] = 0.f;
    }
    if (j < cols) load_f<WT, E>(w + j, wv[c]);
  }
  const float inv_n = 1.0f / cols;
  // Rows are software-pipelined: the next row's x / dy / dsum are loaded into registers before
  // this row's block reductions, so the HBM latency overlaps the barriers (the kernel was
  // latency-bound at one row in flight per block).
  Pack<T, E> px[MAXC], pd[MAXC], ps[MAXC];
  auto prefetch = [&](int r) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int j = (c * 256 + tid) * E;
      if (r < rows && j < cols) {
        const size_t b = (size_t)r * cols + j;
        px[c] = *reinterpret_cast<const Pack<T, E>*>(x + b);
        pd[c] = *reinterpret_cast<const Pack<T, E>*>(dy + b);
        if (dsum != nullptr) ps[c] = *reinterpret_cast<const Pack<T, E>*>(dsum + b);
      }
    }
  };
  prefetch(blockIdx.x);
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const size_t base = (size_t)row * cols;
    const float mu = RMS ? 0.f : mean[row];
    const float rs = rstd[row];
    float xh[MAXC][E], g[MAXC][E], dsv[MAXC][E];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int j = (c * 256 + tid) * E;
      if (j < cols) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float xv = to_f(px[c].v[e]), dv = to_f(pd[c].v[e]);
          xh[c][e] = (xv - mu) * rs;
          g[c][e] = dv * wv[c][e];
          s1 += g[c][e];
          s2 += g[c][e] * xh[c][e];
          aw[c][e] += dv * xh[c][e];
          ab[c][e] += dv;
          dsv[c][e] = dsum != nullptr ? to_f(ps[c].v[e]) : 0.f;
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) { xh[c][e] = 0.f; g[c][e] = 0.f; dsv[c][e] = 0.f; }
      }
    }
    prefetch(row + gridDim.x);
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
        for (int e = 0; e < E; ++e) o[e] = rs * (g[c][e] - m1 - xh[c][e] * m2) + dsv[c][e];
        store_f<T, E>(dx + base + j, o);
        if constexpr (DROP) {
          float m[E];
          drop_mask<E>(dsp, (base + j) / E, m);
#pragma unroll
          for (int e = 0; e < E; ++e) {
            o[e] *= m[e];
            axb[c][e] += o[e];
          }
          store_f<T, E>(dxd + base + j, o);
        }
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
      if constexpr (DROP) {
        if (xb_part != nullptr) {
          float* px = xb_part + (size_t)blockIdx.x * cols + j;
#pragma unroll
          for (int e = 0; e < E; ++e) px[e] = axb[c][e];
        }
      }
    }
  }
}

// Narrow rows (cols <= 64 * E * NCH: ERNIE / BERT-base hidden 768): ONE WAVE PER ROW, four rows in
// flight per block plus the next row's loads prefetched per wave, reductions by DPP / shuffles only
// (no barriers in the row loop).  The block-per-row kernel above leaves 160 of 256 threads idle at
// 768 columns with one row in flight per block (≈ 3 TB/s on [32768, 768]).  The four waves'
// gamma / beta / input-bias partial sums are combined through LDS at the end, so the partial
// layout ([nparts][cols] rows, one per block) and the finishing kernel stay the same.
template <typename T, typename WT, int NCH, bool RMS, bool DROP>
__global__ __launch_bounds__(256) void norm_bwd_wave_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                            const WT* __restrict__ w, const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const T* __restrict__ dsum, T* __restrict__ dx,
                                                            float* __restrict__ dw_part, float* __restrict__ db_part,
                                                            int rows, int cols, T* __restrict__ dxd,
                                                            float* __restrict__ xb_part, DropSpec dsp) {
  dsp.seed = rng_mix(dsp.seed);  // graph-captured steps: per-replay stream
  constexpr int E = 16 / sizeof(T);
  constexpr int W = 64 * E * NCH;  // widest row this instantiation handles
  __shared__ float red[4][W];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float aw[NCH][E], ab[NCH][E], wv[NCH][E], axb[DROP ? NCH : 1][E];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int j = (c * 64 + lane) * E;
#pragma unroll
    for (int e = 0; e < E; ++e) { aw[c][e] = 0.f; ab[c][e] = 0.f; wv[c][e] = 0.f; }
    if constexpr (DROP) {
#pragma unroll
      for (int e = 0; e < E; ++e) axb[c][e] = 0.f;
    }
    if (j < cols) load_f<WT, E>(w + j, wv[c]);
  }
  const float inv_n = 1.0f / cols;
  Pack<T, E> px[NCH], pd[NCH], ps[NCH];
  auto prefetch = [&](int r) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int j = (c * 64 + lane) * E;
      if (r < rows && j < cols) {
        const size_t b = (size_t)r * cols + j;
        px[c] = *reinterpret_cast<const Pack<T, E>*>(x + b);
        pd[c] = *reinterpret_cast<const Pack<T, E>*>(dy + b);
        if (dsum != nullptr) ps[c] = *reinterpret_cast<const Pack<T, E>*>(dsum + b);
      }
    }
  };
  const int row0 = blockIdx.x * 4 + wave, stride = gridDim.x * 4;
  prefetch(row0);
  for (int row = row0; row < rows; row += stride) {
    const size_t base = (size_t)row * cols;
    const float mu = RMS ? 0.f : mean[row];
    const float rs = rstd[row];
    float xh[NCH][E], g[NCH][E], dsv[NCH][E];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int j = (c * 64 + lane) * E;
      if (j < cols) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float xv = to_f(px[c].v[e]), dv = to_f(pd[c].v[e]);
          xh[c][e] = (xv - mu) * rs;
          g[c][e] = dv * wv[c][e];
          s1 += g[c][e];
          s2 += g[c][e] * xh[c][e];
          aw[c][e] += dv * xh[c][e];
          ab[c][e] += dv;
          dsv[c][e] = dsum != nullptr ? to_f(ps[c].v[e]) : 0.f;
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) { xh[c][e] = 0.f; g[c][e] = 0.f; dsv[c][e] = 0.f; }
      }
    }
    prefetch(row + stride);
    const float m1 = RMS ? 0.f : wave_sum(s1) * inv_n;
    const float m2 = wave_sum(s2) * inv_n;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int j = (c * 64 + lane) * E;
      if (j < cols) {
        float o[E];
#pragma unroll
        for (int e = 0; e < E; ++e) o[e] = rs * (g[c][e] - m1 - xh[c][e] * m2) + dsv[c][e];
        store_f<T, E>(dx + base + j, o);
        if constexpr (DROP) {
          float m[E];
          drop_mask<E>(dsp, (base + j) / E, m);
#pragma unroll
          for (int e = 0; e < E; ++e) {
            o[e] *= m[e];
            axb[c][e] += o[e];
          }
          store_f<T, E>(dxd + base + j, o);
        }
      }
    }
  }
  // the block's partial row of each column sum: the four waves' values added through LDS
  auto combine = [&](float (&acc)[NCH][E], float* __restrict__ part) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int e = 0; e < E; ++e) red[wave][(c * 64 + lane) * E + e] = acc[c][e];
    }
    __syncthreads();
    for (int j = tid; j < cols; j += 256) part[(size_t)blockIdx.x * cols + j] = red[0][j] + red[1][j] + red[2][j] + red[3][j];
    __syncthreads();
  };
  combine(aw, dw_part);
  if (!RMS) combine(ab, db_part);
  if constexpr (DROP) {
    if (xb_part != nullptr) combine(axb, xb_part);
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

struct FusedArgs {  // the fused (bias +) dropout + residual path; drop == false: plain (add +) norm
  bool drop;
  const void* xbias;  // forward: bias added to x before dropout (nullable)
  void* dxd;          // backward: gradient of the pre-dropout input
  void* xbgrad;       // backward: bias gradient (nullable), dtype code xbgd, accumulated if xbaccum
  int xbgd, xbaccum;
  DropSpec dsp;
  int wacc = 0;       // backward: dw / db accumulated (+=) into the parameters' gradient slots
};

template <typename T, typename WT, bool RMS>
hipError_t launch_fwd(const void* x, const void* res, const void* w, const void* b, void* y, void* sum_out,
                      float* mean, float* rstd, int rows, int cols, float eps, hipStream_t st,
                      const FusedArgs* fa = nullptr) {
  constexpr int E = 16 / sizeof(T);
  const T* xp = (const T*)x;
  const int chunks = (cols + 64 * E - 1) / (64 * E);
  const bool vec_ok = (cols % E) == 0;
  const bool drop = fa != nullptr && fa->drop;
  dim3 grid((rows + 3) / 4), block(256);
  const T* xb = drop ? (const T*)fa->xbias : nullptr;
  const DropSpec dsp = drop ? fa->dsp : DropSpec{0.f, 0u, 0u};
#define PA_NF(C)                                                                                                   \
  do {                                                                                                             \
    if (drop)                                                                                                      \
      norm_fwd_kernel<T, WT, C, RMS, true><<<grid, block, 0, st>>>(xp, (const T*)res, (const WT*)w, (const WT*)b,  \
                                                                   (T*)y, (T*)sum_out, mean, rstd, rows, cols,     \
                                                                   eps, xb, dsp);                                  \
    else                                                                                                           \
      norm_fwd_kernel<T, WT, C, RMS, false><<<grid, block, 0, st>>>(xp, (const T*)res, (const WT*)w, (const WT*)b, \
                                                                    (T*)y, (T*)sum_out, mean, rstd, rows, cols,    \
                                                                    eps, nullptr, dsp);                            \
  } while (0)
  if (drop && (!vec_ok || chunks > 16 || res == nullptr)) return hipErrorInvalidValue;
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

// A/B switch (pa_norm_set_bwd_wave): the one-wave-per-row backward for rows of <= 128 vectors
static int g_norm_bwd_wave = 1;

template <typename T, typename WT, bool RMS>
hipError_t launch_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                      const void* dsum, void* dx, float* part, void* dw, void* db, int rows, int cols, int nparts,
                      hipStream_t st, const FusedArgs* fa = nullptr) {
  constexpr int E = 16 / sizeof(T);
  const int chunks = (cols + 256 * E - 1) / (256 * E);
  const bool vec_ok = (cols % E) == 0;
  const bool drop = fa != nullptr && fa->drop;
  float* dw_part = part;
  float* db_part = part + (size_t)nparts * cols;
  float* xb_part = (drop && fa->xbgrad != nullptr) ? part + (size_t)2 * nparts * cols : nullptr;
  T* dxd = drop ? (T*)fa->dxd : nullptr;
  const DropSpec dsp = drop ? fa->dsp : DropSpec{0.f, 0u, 0u};
#define PA_NB(C)                                                                                                 \
  do {                                                                                                           \
    if (drop)                                                                                                    \
      norm_bwd_kernel<T, WT, C, RMS, true><<<nparts, 256, 0, st>>>((const T*)dy, (const T*)x, (const WT*)w,      \
                                                                   mean, rstd, (const T*)dsum, (T*)dx, dw_part,  \
                                                                   db_part, rows, cols, dxd, xb_part, dsp);      \
    else                                                                                                         \
      norm_bwd_kernel<T, WT, C, RMS, false><<<nparts, 256, 0, st>>>((const T*)dy, (const T*)x, (const WT*)w,     \
                                                                    mean, rstd, (const T*)dsum, (T*)dx, dw_part, \
                                                                    db_part, rows, cols, nullptr, nullptr, dsp); \
  } while (0)
#define PA_NBW(C)                                                                                                \
  do {                                                                                                           \
    if (drop)                                                                                                    \
      norm_bwd_wave_kernel<T, WT, C, RMS, true><<<nparts, 256, 0, st>>>((const T*)dy, (const T*)x, (const WT*)w, \
                                                                   mean, rstd, (const T*)dsum, (T*)dx, dw_part,  \
                                                                   db_part, rows, cols, dxd, xb_part, dsp);      \
    else                                                                                                         \
      norm_bwd_wave_kernel<T, WT, C, RMS, false><<<nparts, 256, 0, st>>>((const T*)dy, (const T*)x,              \
                                                                    (const WT*)w, mean, rstd, (const T*)dsum,    \
                                                                    (T*)dx, dw_part, db_part, rows, cols,        \
                                                                    nullptr, nullptr, dsp);                      \
  } while (0)
  if (drop && (!vec_ok || chunks > 4)) return hipErrorInvalidValue;
  if (vec_ok && cols <= 64 * E && g_norm_bwd_wave) PA_NBW(1);
  else if (vec_ok && cols <= 128 * E && g_norm_bwd_wave) PA_NBW(2);
  else if (vec_ok && chunks <= 1) PA_NB(1);
  else if (vec_ok && chunks <= 2) PA_NB(2);
  else if (vec_ok && chunks <= 4) PA_NB(4);
  else if (vec_ok && chunks <= 8 && sizeof(T) == 2) PA_NB(8);
  else
    norm_bwd_generic<T, WT, RMS><<<nparts, 256, 0, st>>>((const T*)dy, (const T*)x, (const WT*)w, mean, rstd,
                                                         (const T*)dsum, (T*)dx, dw_part, db_part, rows, cols);
#undef PA_NB
#undef PA_NBW
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // gamma / beta / input-bias gradient finishes: one launch
  const int wacc = fa != nullptr ? fa->wacc : 0;
  FinishJobs jobs{};
  int nj = 0;
  jobs.j[nj++] = FinishJob{dw_part, dw, dtcode_of<WT>(), wacc};
  if (!RMS && db != nullptr) jobs.j[nj++] = FinishJob{db_part, db, dtcode_of<WT>(), wacc};
  if (xb_part != nullptr) jobs.j[nj++] = FinishJob{xb_part, fa->xbgrad, fa->xbgd, fa->xbaccum};
  return launch_colsum_finish_multi(jobs, nj, nparts, cols, st);
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

// Number of partial rows the backward writes (callers size `part` as 2 * nparts * cols floats,
// 3 * nparts * cols for the fused-dropout backward with a bias gradient).
PA_API int pa_norm_set_bwd_wave(int v) {
  const int old = g_norm_bwd_wave;
  g_norm_bwd_wave = v;
  return old;
}

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

// Fused  s = dropout(x + xbias) + res ;  y = norm(s)   (reference:
// paddle/phi/kernels/fusion/gpu/fused_bias_dropout_residual_layer_norm_kernel.cu).  rms selects
// RMSNorm (b, mean unused).  Returns hipErrorInvalidValue when the shape has no fused kernel
// (cols % 8 != 0 or cols > 8192 for 16-bit data): the caller then runs the unfused ops.
PA_API hipError_t pa_dropout_add_norm_fwd(const void* x, const void* xbias, const void* res, const void* w,
                                          const void* b, void* y, void* sum_out, float* mean, float* rstd, int rows,
                                          int cols, float eps, int rms, float p, uint32_t seed, uint32_t offset,
                                          int xd, int wd, hipStream_t st) {
  FusedArgs fa{true, xbias, nullptr, nullptr, 0, 0, DropSpec{p, seed, offset}};
  if (rms) {
    PA_NORM_DISPATCH(xd, wd, true,
                     (launch_fwd<T, WT, true>(x, res, w, nullptr, y, sum_out, nullptr, rstd, rows, cols, eps, st, &fa)))
  }
  PA_NORM_DISPATCH(xd, wd, false,
                   (launch_fwd<T, WT, false>(x, res, w, b, y, sum_out, mean, rstd, rows, cols, eps, st, &fa)))
}

// Backward of the above: dres = norm_bwd(dy) + dsum, dx = dres * keep / (1 - p), xbgrad (+)= colsum(dx).
// `part` holds 3 * pa_norm_bwd_nparts(rows) * cols floats.
PA_API hipError_t pa_dropout_add_norm_bwd(const void* dy, const void* s, const void* w, const float* mean,
                                          const float* rstd, const void* dsum, void* dres, void* dx, float* part,
                                          void* dw, void* db, void* xbgrad, int xbgd, int xbaccum, int wacc, int rows,
                                          int cols, int rms, float p, uint32_t seed, uint32_t offset, int xd, int wd,
                                          hipStream_t st) {
  const int np = pa_norm_bwd_nparts(rows);
  FusedArgs fa{true, nullptr, dx, xbgrad, xbgd, xbaccum, DropSpec{p, seed, offset}, wacc};
  if (rms) {
    PA_NORM_DISPATCH(xd, wd, true,
                     (launch_bwd<T, WT, true>(dy, s, w, nullptr, rstd, dsum, dres, part, dw, nullptr, rows, cols, np,
                                              st, &fa)))
  }
  PA_NORM_DISPATCH(xd, wd, false,
                   (launch_bwd<T, WT, false>(dy, s, w, mean, rstd, dsum, dres, part, dw, db, rows, cols, np, st, &fa)))
}

// graph-safe dropout streams (common.h rng_mix): generation counter of this module's kernels
PA_API int pa_norm_set_rng_gen(const void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(pa::g_rng_gen), &p, sizeof(p));
}
