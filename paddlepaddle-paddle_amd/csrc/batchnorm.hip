// Channels-last (NHWC) batch normalisation with fused residual add + ReLU, training and inference.
//
// Reference semantics: paddle/phi/kernels/gpu/batch_norm_kernel.cu / batch_norm_grad_kernel.cu
// (NHWC path), paddle/phi/kernels/fusion/gpu/fused_bn_add_activation_kernel.cu and
// fused_bn_activation_kernel.cu:  y = act(gamma * (x - mean) * rstd + beta [+ z]),
// running = momentum * running + (1 - momentum) * batch (unbiased variance for the running var).
//
// MI355X design: an NHWC activation is a [R = N*H*W, C] row-major matrix, so every per-channel
// statistic is a COLUMN reduction.  All kernels are column-blocked: a lane owns 8 consecutive
// channels (one 16-byte bf16 vector), keeps their per-channel values (scale/shift, partial sums)
// in registers and walks a chunk of rows with 4 rows of loads in flight; a wave touches 1 KiB
// contiguous per row.  Partial statistics go to a [P, C] scratch and a 16-wave finisher combines
// them (Chan's parallel mean/M2 merge for the forward — no E[x^2]-E[x]^2 cancellation).
//   forward  : stats pass (read x) + apply pass (read x [+ z], write y)
//   backward : reduce pass (read dy, x [, y]) + apply pass (read dy, x [, y], write dx [, dz])
// ReLU's derivative is taken from the saved output y (y > 0), so no mask is stored.
#include "common.h"

namespace pa {
namespace bn {

constexpr int U = 4;           // rows in flight per lane
// block target of the partial-sum (reduction) passes (host-side knob pa_bn_tune; the workspace
// query pa_bn_ws_floats sizes for the current value)
static int kRedBlocks = 512;

// Lane -> (channel chunk, row phase) map.  Wide rows (>= 256 chunks of E channels): one row per
// pass, blockIdx.x selects the chunk range.  Narrow rows (C = 64 ... 1024 in ResNet): the block
// covers RPI = 256 / chunks rows per pass so all 256 lanes stay busy.
struct Map {
  int c0, sub, rpi, cpt;
  bool active;
};

template <int E>
__device__ __forceinline__ Map lane_map(int cols) {
  const int cpt = cols / E;
  Map m;
  m.cpt = cpt;
  if (cpt >= 256) {
    m.rpi = 1;
    m.sub = 0;
    m.c0 = (blockIdx.x * 256 + threadIdx.x) * E;
    m.active = m.c0 < cols;
  } else {
    m.rpi = 256 / cpt;
    m.sub = threadIdx.x / cpt;
    m.c0 = (threadIdx.x % cpt) * E;
    m.active = m.sub < m.rpi;
  }
  return m;
}

inline int col_blocks(int cols, int E) {
  const int cpt = cols / E;
  return cpt >= 256 ? (cpt + 255) / 256 : 1;
}

// target: ~2048 blocks for the streaming apply passes; the reduction passes use ~512 so the
// finisher merges few partial rows (it is latency-bound in its serial per-lane loop).
int rows_per_block(int rows, int colblocks, int target = 2048) {
  long long rpb = ((long long)rows * colblocks + target - 1) / target;
  if (rpb < 64) rpb = 64;
  if (rpb > rows) rpb = rows < 1 ? 1 : rows;
  return (int)rpb;
}

// Row order of the streaming passes (host knob pa_bn_set_interleave): 1 = row groups of
// U x (rows per pass) dealt round-robin over the blocks (so the blocks in flight at any moment
// stream one contiguous window of the tensor), 0 = one contiguous chunk of rows per block.  The
// round-robin order streams faster on MI355X (fused AdamW: 5.7 TB/s grid-stride vs 4.8-5.0 with
// contiguous per-block chunks, profiles/r6o_adamw_variants.log; ResNet50 step 29.53 vs 30.00 ms,
// profiles/r6t_bn_row_order_ab.log).  The mean/M2 statistics pass keeps contiguous slabs (its
// merge needs each partial's row range).
static int kInterleave = 1;
inline dim3 apply_grid(int rows, int cols, int E, dim3 chunk_grid) {
  if (!kInterleave) return chunk_grid;
  const int cpt = cols / E;
  const int rpi = cpt >= 256 ? 1 : 256 / cpt;
  const long long groups = ((long long)rows + (long long)U * rpi - 1) / ((long long)U * rpi);
  // as many blocks as the chunk form (a covering grid of one row group per block measured 34.8
  // vs 30.0 ms on the ResNet50 step: the per-block channel setup then dominates)
  const long long cap = chunk_grid.y;
  return dim3(chunk_grid.x, (unsigned)(groups < cap ? (groups < 1 ? 1 : groups) : cap));
}

// Sum E-wide per-lane vectors over the lanes that share a channel chunk (narrow rows), result
// valid in the sub == 0 lanes.  red: 256 * E floats of LDS.
template <int E>
__device__ __forceinline__ void block_colsum(float (&v)[E], const Map& m, float* red) {
  if (m.rpi == 1) return;
  __syncthreads();
  if (m.active)
#pragma unroll
    for (int e = 0; e < E; ++e) red[threadIdx.x * E + e] = v[e];
  __syncthreads();
  if (m.active && m.sub == 0) {
    for (int s = 1; s < m.rpi; ++s)
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] += red[(threadIdx.x + s * m.cpt) * E + e];
  }
}

// ---- forward statistics: per block chunk, sums shifted by the chunk's first row -> (mean, M2)
template <typename T>
__global__ __launch_bounds__(256) void stats_partial(const T* __restrict__ x, int rows, int cols, int rpb,
                                                     float* __restrict__ pmean, float* __restrict__ pm2) {
  constexpr int E = 16 / sizeof(T);
  __shared__ float red[256 * E];
  const Map m = lane_map<E>(cols);
  const int r0 = blockIdx.y * rpb;
  const int r1 = min(rows, r0 + rpb);
  float k[E], s[E], q[E];
#pragma unroll
  for (int e = 0; e < E; ++e) { k[e] = 0.f; s[e] = 0.f; q[e] = 0.f; }
  if (m.active) {
    load_f<T, E>(x + (size_t)r0 * cols + m.c0, k);
    int r = r0 + m.sub;
    for (; r + (U - 1) * m.rpi < r1; r += U * m.rpi) {
      float v[U][E];
#pragma unroll
      for (int u = 0; u < U; ++u) load_f<T, E>(x + (size_t)(r + u * m.rpi) * cols + m.c0, v[u]);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float d = v[u][e] - k[e];
          s[e] += d;
          q[e] += d * d;
        }
    }
    for (; r < r1; r += m.rpi) {
      float v[E];
      load_f<T, E>(x + (size_t)r * cols + m.c0, v);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float d = v[e] - k[e];
        s[e] += d;
        q[e] += d * d;
      }
    }
  }
  block_colsum<E>(s, m, red);
  block_colsum<E>(q, m, red);
  if (!m.active || m.sub != 0) return;
  const float n = (float)(r1 - r0);
  float mo[E], m2[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const float ds = s[e] / n;
    mo[e] = k[e] + ds;
    m2[e] = fmaxf(q[e] - s[e] * ds, 0.f);
  }
  float* pm = pmean + (size_t)blockIdx.y * cols + m.c0;
  float* pq = pm2 + (size_t)blockIdx.y * cols + m.c0;
#pragma unroll
  for (int e = 0; e < E; e += 4) {
    *reinterpret_cast<float4*>(pm + e) = make_float4(mo[e], mo[e + 1], mo[e + 2], mo[e + 3]);
    *reinterpret_cast<float4*>(pq + e) = make_float4(m2[e], m2[e + 1], m2[e + 2], m2[e + 3]);
  }
}

// Merge of the P chunk statistics (every chunk has rpb rows but the last) -> mean, rstd; running
// update.  Two parallel passes instead of a serial Chan chain: mean = sum n_p mean_p / N, then
// M2 = sum (M2_p + n_p (mean_p - mean)^2) — the same value, no per-step division, 4 loads in flight.
__global__ __launch_bounds__(1024) void stats_finish(const float* __restrict__ pmean, const float* __restrict__ pm2,
                                                     int P, int rows, int rpb, int cols, float eps, float momentum,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     float* __restrict__ run_mean, float* __restrict__ run_var) {
  __shared__ float red[16][65];
  __shared__ float mshare[64];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = blockIdx.x * 64 + lane;
  const float nlast = (float)(rows - (P - 1) * rpb), nfull = (float)rpb;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < cols) {
    int p = w;
    for (; p + 48 < P - 1; p += 64) {  // the (short) last chunk is left to the tail loop
      a0 += pmean[(size_t)p * cols + c];
      a1 += pmean[(size_t)(p + 16) * cols + c];
      a2 += pmean[(size_t)(p + 32) * cols + c];
      a3 += pmean[(size_t)(p + 48) * cols + c];
    }
    for (; p < P; p += 16) {
      const float v = pmean[(size_t)p * cols + c];
      if (p == P - 1) a1 += v * (nlast / nfull); else a0 += v;
    }
  }
  red[w][lane] = ((a0 + a1) + (a2 + a3)) * nfull;
  __syncthreads();
  if (w == 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][lane];
    mshare[lane] = t / (float)rows;
  }
  __syncthreads();
  const float mu = mshare[lane];
  a0 = a1 = a2 = a3 = 0.f;
  if (c < cols) {
    int p = w;
    for (; p + 48 < P - 1; p += 64) {
      float d;
      d = pmean[(size_t)p * cols + c] - mu;
      a0 += pm2[(size_t)p * cols + c] + nfull * d * d;
      d = pmean[(size_t)(p + 16) * cols + c] - mu;
      a1 += pm2[(size_t)(p + 16) * cols + c] + nfull * d * d;
      d = pmean[(size_t)(p + 32) * cols + c] - mu;
      a2 += pm2[(size_t)(p + 32) * cols + c] + nfull * d * d;
      d = pmean[(size_t)(p + 48) * cols + c] - mu;
      a3 += pm2[(size_t)(p + 48) * cols + c] + nfull * d * d;
    }
    for (; p < P; p += 16) {
      const float d = pmean[(size_t)p * cols + c] - mu;
      a0 += pm2[(size_t)p * cols + c] + (p == P - 1 ? nlast : nfull) * d * d;
    }
  }
  __syncthreads();
  red[w][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (w == 0 && c < cols) {
    float m2 = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) m2 += red[i][lane];
    const float n = (float)rows;
    const float var = m2 / n;
    mean_out[c] = mu;
    rstd_out[c] = rsqrtf(var + eps);
    if (run_mean != nullptr) {
      run_mean[c] = momentum * run_mean[c] + (1.f - momentum) * mu;
      run_var[c] = momentum * run_var[c] + (1.f - momentum) * (n > 1.f ? m2 / (n - 1.f) : var);
    }
  }
}

// ---- Chan merge of G consecutive slab statistics (mean, M2 over rpb rows each, the last slab of
// all P possibly short) into one (mean, M2) per group of G slabs: the epilogue-produced statistics
// of a convolution / GEMM (thousands of 64-128-row slabs) brought down to a few hundred chunks
// of G * rpb rows for stats_finish.  grid (ceil(cols / blockDim), ceil(P / G)), one column per thread.
__global__ __launch_bounds__(256) void stats_merge(const float* __restrict__ pmean, const float* __restrict__ pm2,
                                                   int P, int rows, int rpb, int cols, int G,
                                                   float* __restrict__ omean, float* __restrict__ om2, int P2) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  const int p0 = blockIdx.y * G, p1 = min(P, p0 + G);
  const float nfull = (float)rpb, nlast = (float)(rows - (P - 1) * rpb);
  float n = 0.f, s = 0.f;
#pragma unroll 8
  for (int p = p0; p < p1; ++p) {
    const float np = p == P - 1 ? nlast : nfull;
    s += np * pmean[(size_t)p * cols + c];
    n += np;
  }
  const float mu = s / n;
  float m2 = 0.f;
#pragma unroll 8
  for (int p = p0; p < p1; ++p) {
    const float np = p == P - 1 ? nlast : nfull;
    const float d = pmean[(size_t)p * cols + c] - mu;
    m2 += pm2[(size_t)p * cols + c] + np * d * d;
  }
  omean[(size_t)blockIdx.y * cols + c] = mu;
  om2[(size_t)blockIdx.y * cols + c] = m2;
}

// ---- y = act(x * a + b [+ z]),  a = gamma * rstd, b = beta - mean * a  (per channel)
template <typename T, typename WT, bool RELU, bool RES>
__global__ __launch_bounds__(256) void apply_fwd(const T* __restrict__ x, const T* __restrict__ z,
                                                 const float* __restrict__ mean, const float* __restrict__ rstd,
                                                 const WT* __restrict__ gamma, const WT* __restrict__ beta,
                                                 T* __restrict__ y, int rows, int cols, int rpb, int inter) {
  constexpr int E = 16 / sizeof(T);
  const Map m = lane_map<E>(cols);
  if (!m.active) return;
  const int c0 = m.c0, st = m.rpi;
  float a[E], b[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const float g = gamma != nullptr ? to_f(gamma[c0 + e]) : 1.f;
    const float bt = beta != nullptr ? to_f(beta[c0 + e]) : 0.f;
    a[e] = g * rstd[c0 + e];
    b[e] = bt - mean[c0 + e] * a[e];
  }
  auto rows_u = [&](int r) {  // rows r, r + st, ... r + (U - 1) st
    float v[U][E], zz[U][E];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      load_f<T, E>(x + (size_t)(r + u * st) * cols + c0, v[u]);
      if constexpr (RES) load_f<T, E>(z + (size_t)(r + u * st) * cols + c0, zz[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        float o = v[u][e] * a[e] + b[e];
        if constexpr (RES) o += zz[u][e];
        if constexpr (RELU) o = fmaxf(o, 0.f);
        v[u][e] = o;
      }
      store_f<T, E>(y + (size_t)(r + u * st) * cols + c0, v[u]);
    }
  };
  auto row_1 = [&](int r) {
    float v[E], zz[E];
    load_f<T, E>(x + (size_t)r * cols + c0, v);
    if constexpr (RES) load_f<T, E>(z + (size_t)r * cols + c0, zz);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float o = v[e] * a[e] + b[e];
      if constexpr (RES) o += zz[e];
      if constexpr (RELU) o = fmaxf(o, 0.f);
      v[e] = o;
    }
    store_f<T, E>(y + (size_t)r * cols + c0, v);
  };
  if (inter) {  // row groups of U * st rows dealt round-robin over the blocks (see kInterleave)
    const long long RG = (long long)U * st;
    for (long long g = blockIdx.y; g * RG < rows; g += gridDim.y) {
      const int rb = (int)(g * RG) + m.sub;
      if ((g + 1) * RG <= rows) {
        rows_u(rb);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (rb + u * st < rows) row_1(rb + u * st);
      }
    }
    return;
  }
  const int r0 = blockIdx.y * rpb;
  const int r1 = min(rows, r0 + rpb);
  int r = r0 + m.sub;
  for (; r + (U - 1) * st < r1; r += U * st) rows_u(r);
  for (; r < r1; r += st) row_1(r);
}

// ---- backward reduce: per channel  s1 = sum g,  s2 = sum g * (x - mean),  g = dy [* (y > 0)]
// XM (ReLU without a residual input): the ReLU mask is recomputed from x with the forward's own
// affine (a = gamma * rstd, b = beta - mean * a; y > 0 <=> x * a + b > 0, the same fp32 expression
// as apply_fwd), so y is never read: one activation-sized read less per pass.
template <typename WT>
__device__ __forceinline__ void affine_of(const WT* gamma, const WT* beta, const float* mean, const float* rstd, int c,
                                          float& a, float& b) {
  const float g = gamma != nullptr ? to_f(gamma[c]) : 1.f;
  const float bt = beta != nullptr ? to_f(beta[c]) : 0.f;
  a = g * rstd[c];
  b = bt - mean[c] * a;
}

template <typename T, bool RELU, typename WT = float, bool XM = false>
__global__ __launch_bounds__(256) void bwd_partial(const T* __restrict__ dy, const T* __restrict__ x,
                                                   const T* __restrict__ y, const float* __restrict__ mean, int rows,
                                                   int cols, int rpb, float* __restrict__ p1, float* __restrict__ p2,
                                                   const WT* __restrict__ gamma = nullptr,
                                                   const WT* __restrict__ beta = nullptr,
                                                   const float* __restrict__ rstd = nullptr, int inter = 0) {
  constexpr int E = 16 / sizeof(T);
  __shared__ float red[256 * E];
  const Map m = lane_map<E>(cols);
  float mu[E], s1[E], s2[E], fa[E], fb[E];
#pragma unroll
  for (int e = 0; e < E; ++e) { mu[e] = 0.f; s1[e] = 0.f; s2[e] = 0.f; fa[e] = 0.f; fb[e] = 0.f; }
  if (m.active) {
    const int c0 = m.c0, st = m.rpi;
#pragma unroll
    for (int e = 0; e < E; ++e) mu[e] = mean[c0 + e];
    if constexpr (XM) {
#pragma unroll
      for (int e = 0; e < E; ++e) affine_of<WT>(gamma, beta, mean, rstd, c0 + e, fa[e], fb[e]);
    }
    auto rows_u = [&](int r) {
      float g[U][E], v[U][E], o[U][E];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        load_f<T, E>(dy + (size_t)(r + u * st) * cols + c0, g[u]);
        load_f<T, E>(x + (size_t)(r + u * st) * cols + c0, v[u]);
        if constexpr (RELU && !XM) load_f<T, E>(y + (size_t)(r + u * st) * cols + c0, o[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < E; ++e) {
          float gg = g[u][e];
          if constexpr (XM) gg = (v[u][e] * fa[e] + fb[e]) > 0.f ? gg : 0.f;
          else if constexpr (RELU) gg = o[u][e] > 0.f ? gg : 0.f;
          s1[e] += gg;
          s2[e] += gg * (v[u][e] - mu[e]);
        }
    };
    auto row_1 = [&](int r) {
      float g[E], v[E], o[E];
      load_f<T, E>(dy + (size_t)r * cols + c0, g);
      load_f<T, E>(x + (size_t)r * cols + c0, v);
      if constexpr (RELU && !XM) load_f<T, E>(y + (size_t)r * cols + c0, o);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        float gg = g[e];
        if constexpr (XM) gg = (v[e] * fa[e] + fb[e]) > 0.f ? gg : 0.f;
        else if constexpr (RELU) gg = o[e] > 0.f ? gg : 0.f;
        s1[e] += gg;
        s2[e] += gg * (v[e] - mu[e]);
      }
    };
    if (inter) {
      const long long RG = (long long)U * st;
      for (long long gi = blockIdx.y; gi * RG < rows; gi += gridDim.y) {
        const int rb = (int)(gi * RG) + m.sub;
        if ((gi + 1) * RG <= rows) {
          rows_u(rb);
        } else {
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (rb + u * st < rows) row_1(rb + u * st);
        }
      }
    } else {
      const int r0 = blockIdx.y * rpb;
      const int r1 = min(rows, r0 + rpb);
      int r = r0 + m.sub;
      for (; r + (U - 1) * st < r1; r += U * st) rows_u(r);
      for (; r < r1; r += st) row_1(r);
    }
  }
  block_colsum<E>(s1, m, red);
  block_colsum<E>(s2, m, red);
  if (!m.active || m.sub != 0) return;
  float* q1 = p1 + (size_t)blockIdx.y * cols + m.c0;
  float* q2 = p2 + (size_t)blockIdx.y * cols + m.c0;
#pragma unroll
  for (int e = 0; e < E; e += 4) {
    *reinterpret_cast<float4*>(q1 + e) = make_float4(s1[e], s1[e + 1], s1[e + 2], s1[e + 3]);
    *reinterpret_cast<float4*>(q2 + e) = make_float4(s2[e], s2[e + 1], s2[e + 2], s2[e + 3]);
  }
}

// sums -> dbeta = s1, dgamma = s2 * rstd (param dtype), and fp32 copies for the apply pass
template <typename WT>
__global__ __launch_bounds__(1024) void bwd_finish(const float* __restrict__ p1, const float* __restrict__ p2, int P,
                                                   int cols, const float* __restrict__ rstd, WT* __restrict__ dgamma,
                                                   WT* __restrict__ dbeta, float* __restrict__ s_out, int accumulate) {
  __shared__ float r1[16][65], r2[16][65];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = blockIdx.x * 64 + lane;
  float a = 0.f, b = 0.f, a2 = 0.f, b2 = 0.f, a3 = 0.f, b3 = 0.f, a4 = 0.f, b4 = 0.f;
  if (c < cols) {
    int p = w;
    for (; p + 48 < P; p += 64) {
      a += p1[(size_t)p * cols + c];
      b += p2[(size_t)p * cols + c];
      a2 += p1[(size_t)(p + 16) * cols + c];
      b2 += p2[(size_t)(p + 16) * cols + c];
      a3 += p1[(size_t)(p + 32) * cols + c];
      b3 += p2[(size_t)(p + 32) * cols + c];
      a4 += p1[(size_t)(p + 48) * cols + c];
      b4 += p2[(size_t)(p + 48) * cols + c];
    }
    for (; p < P; p += 16) {
      a += p1[(size_t)p * cols + c];
      b += p2[(size_t)p * cols + c];
    }
  }
  r1[w][lane] = (a + a2) + (a3 + a4);
  r2[w][lane] = (b + b2) + (b3 + b4);
  __syncthreads();
  if (w == 0 && c < cols) {
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) { s1 += r1[i][lane]; s2 += r2[i][lane]; }
    s_out[c] = s1;
    s_out[cols + c] = s2;
    // accumulate: += into the parameters' flat gradient slots (no separate AccumulateGrad add)
    if (dbeta != nullptr) dbeta[c] = from_f<WT>(s1 + (accumulate ? to_f(dbeta[c]) : 0.f));
    if (dgamma != nullptr) dgamma[c] = from_f<WT>(s2 * rstd[c] + (accumulate ? to_f(dgamma[c]) : 0.f));
  }
}

// dx = gamma * rstd * (g - s1/R - (x - mean) * rstd^2 * s2/R);  dz = g (residual branch)
template <typename T, typename WT, bool RELU, bool RES, bool XM = false>
__global__ __launch_bounds__(256) void bwd_apply(const T* __restrict__ dy, const T* __restrict__ x,
                                                 const T* __restrict__ y, const float* __restrict__ mean,
                                                 const float* __restrict__ rstd, const WT* __restrict__ gamma,
                                                 const float* __restrict__ sums, T* __restrict__ dx,
                                                 T* __restrict__ dz, int rows, int cols, int rpb, int inter,
                                                 const WT* __restrict__ beta = nullptr) {
  constexpr int E = 16 / sizeof(T);
  const Map m = lane_map<E>(cols);
  if (!m.active) return;
  const int c0 = m.c0, st = m.rpi;
  const float invR = 1.f / (float)rows;
  float k1[E], k2[E], k3[E], mu[E], fa[E], fb[E];  // dx = k1 * g + k2 * (x - mu) + k3
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if constexpr (XM) affine_of<WT>(gamma, beta, mean, rstd, c0 + e, fa[e], fb[e]);
    const float rs = rstd[c0 + e];
    const float gr = (gamma != nullptr ? to_f(gamma[c0 + e]) : 1.f) * rs;
    mu[e] = mean[c0 + e];
    k1[e] = gr;
    k2[e] = -gr * rs * rs * sums[cols + c0 + e] * invR;
    k3[e] = -gr * sums[c0 + e] * invR;
  }
  auto rows_u = [&](int r) {
    float g[U][E], v[U][E], o[U][E];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      load_f<T, E>(dy + (size_t)(r + u * st) * cols + c0, g[u]);
      load_f<T, E>(x + (size_t)(r + u * st) * cols + c0, v[u]);
      if constexpr (RELU && !XM) load_f<T, E>(y + (size_t)(r + u * st) * cols + c0, o[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if constexpr (XM) g[u][e] = (v[u][e] * fa[e] + fb[e]) > 0.f ? g[u][e] : 0.f;
        else if constexpr (RELU) g[u][e] = o[u][e] > 0.f ? g[u][e] : 0.f;
        v[u][e] = k1[e] * g[u][e] + k2[e] * (v[u][e] - mu[e]) + k3[e];
      }
      store_f<T, E>(dx + (size_t)(r + u * st) * cols + c0, v[u]);
      if constexpr (RES) store_f<T, E>(dz + (size_t)(r + u * st) * cols + c0, g[u]);
    }
  };
  auto row_1 = [&](int r) {
    float g[E], v[E], o[E];
    load_f<T, E>(dy + (size_t)r * cols + c0, g);
    load_f<T, E>(x + (size_t)r * cols + c0, v);
    if constexpr (RELU && !XM) load_f<T, E>(y + (size_t)r * cols + c0, o);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if constexpr (XM) g[e] = (v[e] * fa[e] + fb[e]) > 0.f ? g[e] : 0.f;
      else if constexpr (RELU) g[e] = o[e] > 0.f ? g[e] : 0.f;
      v[e] = k1[e] * g[e] + k2[e] * (v[e] - mu[e]) + k3[e];
    }
    store_f<T, E>(dx + (size_t)r * cols + c0, v);
    if constexpr (RES) store_f<T, E>(dz + (size_t)r * cols + c0, g);
  };
  if (inter) {
    const long long RG = (long long)U * st;
    for (long long gi = blockIdx.y; gi * RG < rows; gi += gridDim.y) {
      const int rb = (int)(gi * RG) + m.sub;
      if ((gi + 1) * RG <= rows) {
        rows_u(rb);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (rb + u * st < rows) row_1(rb + u * st);
      }
    }
    return;
  }
  const int r0 = blockIdx.y * rpb;
  const int r1 = min(rows, r0 + rpb);
  int r = r0 + m.sub;
  for (; r + (U - 1) * st < r1; r += U * st) rows_u(r);
  for (; r < r1; r += st) row_1(r);
}

template <typename T, typename WT>
hipError_t fwd(const void* x, const void* z, const void* gamma, const void* beta, void* y, float* mean, float* rstd,
               float* run_mean, float* run_var, float* ws, int rows, int cols, float eps, float momentum, int training,
               int relu, hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  const int cb = col_blocks(cols, E);
  const int rpb = rows_per_block(rows, cb);
  const dim3 grid(cb, (rows + rpb - 1) / rpb);
  const dim3 agrid = apply_grid(rows, cols, E, grid);
  if (training) {
    const int rrb = rows_per_block(rows, cb, kRedBlocks);
    const int P = (rows + rrb - 1) / rrb;
    stats_partial<T><<<dim3(cb, P), 256, 0, st>>>((const T*)x, rows, cols, rrb, ws, ws + (size_t)P * cols);
    stats_finish<<<(cols + 63) / 64, 1024, 0, st>>>(ws, ws + (size_t)P * cols, P, rows, rrb, cols, eps, momentum,
                                                    mean, rstd, run_mean, run_var);
  }
#define PA_BNF(R, Z) apply_fwd<T, WT, R, Z><<<agrid, 256, 0, st>>>((const T*)x, (const T*)z, mean, rstd, \
                                                                  (const WT*)gamma, (const WT*)beta, (T*)y, rows, cols, \
                                                                  rpb, kInterleave)
  if (relu && z) PA_BNF(true, true);
  else if (relu) PA_BNF(true, false);
  else if (z) PA_BNF(false, true);
  else PA_BNF(false, false);
#undef PA_BNF
  return hipGetLastError();
}

// forward from slab statistics produced by the producer's epilogue (parts: fp32 [2][P][cols],
// slabs of rpb rows, the last possibly short); ws: 2 * min(P, 512) * cols floats
template <typename T, typename WT>
hipError_t fwd_parts(const void* x, const void* z, const void* gamma, const void* beta, void* y, float* mean,
                     float* rstd, float* run_mean, float* run_var, const float* parts, int P, int prpb, float* ws,
                     int rows, int cols, float eps, float momentum, int relu, hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  const int cb = col_blocks(cols, E);
  const int rpb = rows_per_block(rows, cb);
  const dim3 grid(cb, (rows + rpb - 1) / rpb);
  const dim3 agrid = apply_grid(rows, cols, E, grid);
  const float* pm = parts;
  const float* pq = parts + (size_t)P * cols;
  int Pf = P, rf = prpb;
  if (P > 512) {  // merge groups of G slabs first (the finisher's per-lane loop is serial)
    const int G = (P + 511) / 512;
    const int P2 = (P + G - 1) / G;
    const int bt = cols >= 256 ? 256 : (cols + 63) / 64 * 64;  // narrow rows: one wave per block
    stats_merge<<<dim3((cols + bt - 1) / bt, P2), bt, 0, st>>>(pm, pq, P, rows, prpb, cols, G, ws,
                                                               ws + (size_t)P2 * cols, P2);
    pm = ws;
    pq = ws + (size_t)P2 * cols;
    Pf = P2;
    rf = prpb * G;
  }
  stats_finish<<<(cols + 63) / 64, 1024, 0, st>>>(pm, pq, Pf, rows, rf, cols, eps, momentum, mean, rstd, run_mean,
                                                  run_var);
#define PA_BNF(R, Z) apply_fwd<T, WT, R, Z><<<agrid, 256, 0, st>>>((const T*)x, (const T*)z, mean, rstd, \
                                                                  (const WT*)gamma, (const WT*)beta, (T*)y, rows, cols, \
                                                                  rpb, kInterleave)
  if (relu && z) PA_BNF(true, true);
  else if (relu) PA_BNF(true, false);
  else if (z) PA_BNF(false, true);
  else PA_BNF(false, false);
#undef PA_BNF
  return hipGetLastError();
}

template <typename T, typename WT>
hipError_t bwd(const void* dy, const void* x, const void* y, const float* mean, const float* rstd, const void* gamma,
               const void* beta, void* dx, void* dz, void* dgamma, void* dbeta, float* ws, int rows, int cols, int relu,
               int accumulate, hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  const int cb = col_blocks(cols, E);
  const int rpb = rows_per_block(rows, cb);
  const dim3 grid(cb, (rows + rpb - 1) / rpb);
  const int rrb = rows_per_block(rows, cb, kRedBlocks);
  const int P = (rows + rrb - 1) / rrb;
  float* p1 = ws;
  float* p2 = ws + (size_t)P * cols;
  float* sums = ws + (size_t)2 * P * cols;
  const dim3 rgrid(cb, P);
  const dim3 agrid = apply_grid(rows, cols, E, grid);
  const bool xm = relu && dz == nullptr;  // ReLU mask from x: y is not read
  if (xm)
    bwd_partial<T, true, WT, true><<<rgrid, 256, 0, st>>>((const T*)dy, (const T*)x, nullptr, mean, rows, cols, rrb, p1,
                                                          p2, (const WT*)gamma, (const WT*)beta, rstd, kInterleave);
  else if (relu)
    bwd_partial<T, true, WT><<<rgrid, 256, 0, st>>>((const T*)dy, (const T*)x, (const T*)y, mean, rows, cols, rrb, p1, p2,
                                                (const WT*)nullptr, (const WT*)nullptr, nullptr, kInterleave);
  else
    bwd_partial<T, false, WT><<<rgrid, 256, 0, st>>>((const T*)dy, (const T*)x, nullptr, mean, rows, cols, rrb, p1, p2,
                                                 (const WT*)nullptr, (const WT*)nullptr, nullptr, kInterleave);
  bwd_finish<WT><<<(cols + 63) / 64, 1024, 0, st>>>(p1, p2, P, cols, rstd, (WT*)dgamma, (WT*)dbeta, sums,
                                                    accumulate);
#define PA_BNB(R, Z) bwd_apply<T, WT, R, Z><<<agrid, 256, 0, st>>>((const T*)dy, (const T*)x, (const T*)y, mean, \
                                                                  rstd, (const WT*)gamma, sums, (T*)dx, (T*)dz, rows, \
                                                                  cols, rpb, kInterleave)
  if (relu && dz) PA_BNB(true, true);
  else if (xm)
    bwd_apply<T, WT, true, false, true><<<agrid, 256, 0, st>>>((const T*)dy, (const T*)x, nullptr, mean, rstd,
                                                               (const WT*)gamma, sums, (T*)dx, nullptr, rows, cols, rpb,
                                                               kInterleave, (const WT*)beta);
  else if (dz) PA_BNB(false, true);
  else PA_BNB(false, false);
#undef PA_BNB
  return hipGetLastError();
}

}  // namespace bn
}  // namespace pa

using namespace pa;

// scratch floats the kernels need (callers allocate ws of this many fp32)
PA_API long long pa_bn_ws_floats(int rows, int cols, int dt) {
  const int E = dt == 0 ? 4 : 8;
  const int cb = bn::col_blocks(cols, E);
  const int rpb = bn::rows_per_block(rows, cb, bn::kRedBlocks);
  const long long P = (rows + rpb - 1) / rpb;
  return 2 * P * cols + 2LL * cols;
}

#define PA_BN_DISPATCH(xd, wd, CALL)                                             \
  if (xd == 1 && wd == 0) { using T = bf16_t; using WT = float; return CALL; }   \
  if (xd == 1 && wd == 1) { using T = bf16_t; using WT = bf16_t; return CALL; }  \
  if (xd == 2 && wd == 0) { using T = f16_t; using WT = float; return CALL; }    \
  if (xd == 2 && wd == 2) { using T = f16_t; using WT = f16_t; return CALL; }    \
  if (xd == 0 && wd == 0) { using T = float; using WT = float; return CALL; }    \
  return hipErrorInvalidValue;

// x, z (residual, nullable), y: [rows, cols] NHWC; mean/rstd: [cols] fp32 (computed when training,
// read otherwise: pass mean = running mean, rstd = 1/sqrt(running var + eps) for inference).
PA_API hipError_t pa_bn_fwd(const void* x, const void* z, const void* gamma, const void* beta, void* y, float* mean,
                            float* rstd, float* run_mean, float* run_var, float* ws, int rows, int cols, float eps,
                            float momentum, int training, int relu, int xd, int wd, hipStream_t st) {
  if (cols % (xd == 0 ? 4 : 8) != 0 || rows < 1) return hipErrorInvalidValue;
  PA_BN_DISPATCH(xd, wd, (bn::fwd<T, WT>(x, z, gamma, beta, y, mean, rstd, run_mean, run_var, ws, rows, cols, eps,
                                          momentum, training, relu, st)))
}

// Training forward whose batch statistics come from the producing kernel's epilogue (parts: fp32
// [2][P][cols] slab means then M2s, slabs of rpb rows, only the last one short — csrc/conv.hip
// pa_conv2d_fwd_stats, csrc/gemm8.hip epi 5); ws: >= 2 * 512 * cols floats.
PA_API hipError_t pa_bn_fwd_parts(const void* x, const void* z, const void* gamma, const void* beta, void* y,
                                  float* mean, float* rstd, float* run_mean, float* run_var, const float* parts, int P,
                                  int rpb, float* ws, int rows, int cols, float eps, float momentum, int relu, int xd,
                                  int wd, hipStream_t st) {
  if (cols % (xd == 0 ? 4 : 8) != 0 || rows < 1 || P < 1 || rpb < 1 || (long long)(P - 1) * rpb >= rows ||
      (long long)P * rpb < rows)
    return hipErrorInvalidValue;
  PA_BN_DISPATCH(xd, wd, (bn::fwd_parts<T, WT>(x, z, gamma, beta, y, mean, rstd, run_mean, run_var, parts, P, rpb, ws,
                                                rows, cols, eps, momentum, relu, st)))
}

// dz (nullable): gradient of the residual input z (= dy masked by ReLU).  y is the saved output
// (needed only when relu with a residual; ReLU without one recomputes the mask from x, gamma, beta).
// dgamma/dbeta in the parameter dtype (nullable; accumulate != 0: +=).
PA_API hipError_t pa_bn_bwd(const void* dy, const void* x, const void* y, const float* mean, const float* rstd,
                            const void* gamma, const void* beta, void* dx, void* dz, void* dgamma, void* dbeta,
                            float* ws, int rows, int cols, int relu, int accumulate, int xd, int wd, hipStream_t st) {
  if (cols % (xd == 0 ? 4 : 8) != 0 || rows < 1) return hipErrorInvalidValue;
  PA_BN_DISPATCH(xd, wd, (bn::bwd<T, WT>(dy, x, y, mean, rstd, gamma, beta, dx, dz, dgamma, dbeta, ws, rows, cols,
                                          relu, accumulate, st)))
}

// A/B knob: block target of the BN reduction passes (returns the previous value).
PA_API int pa_bn_set_interleave(int v) {
  const int old = bn::kInterleave;
  bn::kInterleave = v;
  return old;
}

PA_API int pa_bn_tune(int red_blocks) {
  const int old = bn::kRedBlocks;
  if (red_blocks >= 64 && red_blocks <= 8192) bn::kRedBlocks = red_blocks;
  return old;
}
