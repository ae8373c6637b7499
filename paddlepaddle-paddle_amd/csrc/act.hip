// Fused activation / dropout kernels (vectorised 16-byte, grid-stride, fp32 math).
//
// Reference semantics: paddle/phi/kernels/gpu/gelu_kernel.cu / gelu_grad_kernel.cu,
// paddle/phi/kernels/fusion/gpu/fused_bias_act_kernel.cu (bias + act in one pass),
// paddle/phi/kernels/fusion/gpu/fused_dropout_add_kernel.cu, swiglu (incubate).
//
// Dropout masks are never stored: the keep-decision is a stateless hash of
// (seed, offset, element index), so backward regenerates it bit-exactly.
#include "common.h"

namespace pa {

struct GeluErf {
  static __device__ __forceinline__ float f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
  static __device__ __forceinline__ float df(float x) {
    return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
  }
};
// fast_tanh / GeluTanh live in common.h (shared with the GEMM epilogues of gemm8.hip)
struct Silu {
  static __device__ __forceinline__ float f(float x) { return x / (1.f + __expf(-x)); }
  static __device__ __forceinline__ float df(float x) {
    const float s = 1.f / (1.f + __expf(-x));
    return s * (1.f + x * (1.f - s));
  }
};
struct Relu {
  static __device__ __forceinline__ float f(float x) { return x > 0.f ? x : 0.f; }
  static __device__ __forceinline__ float df(float x) { return x > 0.f ? 1.f : 0.f; }
};
struct Ident {
  static __device__ __forceinline__ float f(float x) { return x; }
  static __device__ __forceinline__ float df(float) { return 1.f; }
};

// y = act(x + bias[col])   (bias may be null);   cols = size of the bias (last dim)
template <typename T, typename Act>
__global__ __launch_bounds__(256) void bias_act_fwd(const T* __restrict__ x, const T* __restrict__ bias,
                                                    T* __restrict__ y, long long n, int cols) {
  constexpr int E = 16 / sizeof(T);
  const long long nv = n / E;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nv; i += (long long)gridDim.x * 256) {
    float v[E];
    load_f<T, E>(x + i * E, v);
    if (bias != nullptr) {
      float b[E];
      load_f<T, E>(bias + (int)((i * E) % cols), b);
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] += b[e];
    }
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = Act::f(v[e]);
    store_f<T, E>(y + i * E, v);
  }
  // tail (n % E elements) handled by the first block
  if (blockIdx.x == 0) {
    for (long long i = nv * E + threadIdx.x; i < n; i += 256) {
      float v = to_f(x[i]) + (bias != nullptr ? to_f(bias[i % cols]) : 0.f);
      y[i] = from_f<T>(Act::f(v));
    }
  }
}

// dx = dy * act'(x + bias);  dbias is reduced by the caller from dx (bias grad = colsum(dx))
template <typename T, typename Act>
__global__ __launch_bounds__(256) void bias_act_bwd(const T* __restrict__ dy, const T* __restrict__ x,
                                                    const T* __restrict__ bias, T* __restrict__ dx, long long n,
                                                    int cols) {
  constexpr int E = 16 / sizeof(T);
  const long long nv = n / E;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nv; i += (long long)gridDim.x * 256) {
    float v[E], g[E];
    load_f<T, E>(x + i * E, v);
    load_f<T, E>(dy + i * E, g);
    if (bias != nullptr) {
      float b[E];
      load_f<T, E>(bias + (int)((i * E) % cols), b);
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] += b[e];
    }
#pragma unroll
    for (int e = 0; e < E; ++e) g[e] *= Act::df(v[e]);
    store_f<T, E>(dx + i * E, g);
  }
  if (blockIdx.x == 0) {
    for (long long i = nv * E + threadIdx.x; i < n; i += 256) {
      float v = to_f(x[i]) + (bias != nullptr ? to_f(bias[i % cols]) : 0.f);
      dx[i] = from_f<T>(to_f(dy[i]) * Act::df(v));
    }
  }
}

// Column-blocked backward with the bias gradient fused: block (bx, by) owns columns
// [bx*256*E, +256*E) and rows [by*rpb, +rpb); each lane keeps E per-column fp32 sums of dx in
// registers across its rows (16-byte loads, a wave reads 1 KiB contiguous per row) and writes
// them once to part[by, :].  colsum_finish adds the partial rows into the bias gradient.
// ACT == nullptr-like Ident with no x: plain column sum of dy (dx, x unused).
template <typename T, typename Act, bool HAS_X>
__global__ __launch_bounds__(256) void bias_act_bwd_cs(const T* __restrict__ dy, const T* __restrict__ x,
                                                       const T* __restrict__ bias, T* __restrict__ dx,
                                                       float* __restrict__ part, int rows, int cols, int rpb,
                                                       int inter) {
  constexpr int E = 16 / sizeof(T);
  constexpr int U = 4;  // rows in flight per lane
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * E;
  if (c0 >= cols) return;  // no barriers below
  float b[E], acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) { b[e] = 0.f; acc[e] = 0.f; }
  if (HAS_X && bias != nullptr) load_f<T, E>(bias + c0, b);
  auto rows_u = [&](int r) {
    float g[U][E], v[U][E];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      load_f<T, E>(dy + (size_t)(r + u) * cols + c0, g[u]);
      if constexpr (HAS_X) load_f<T, E>(x + (size_t)(r + u) * cols + c0, v[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (HAS_X) {
#pragma unroll
        for (int e = 0; e < E; ++e) g[u][e] *= Act::df(v[u][e] + b[e]);
        store_f<T, E>(dx + (size_t)(r + u) * cols + c0, g[u]);
      }
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] += g[u][e];
    }
  };
  auto row_1 = [&](int r) {
    const size_t o0 = (size_t)r * cols + c0;
    float g0[E];
    load_f<T, E>(dy + o0, g0);
    if constexpr (HAS_X) {
      float v0[E];
      load_f<T, E>(x + o0, v0);
#pragma unroll
      for (int e = 0; e < E; ++e) g0[e] *= Act::df(v0[e] + b[e]);
      store_f<T, E>(dx + o0, g0);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] += g0[e];
  };
  if (inter) {  // groups of U rows dealt round-robin over the row blocks (see g_cs_inter)
    for (long long gi = blockIdx.y; gi * U < rows; gi += gridDim.y) {
      const int rb = (int)(gi * U);
      if (rb + U <= rows) rows_u(rb);
      else
        for (int r = rb; r < rows; ++r) row_1(r);
    }
  } else {
    const int r0 = blockIdx.y * rpb;
    const int r1 = min(rows, r0 + rpb);
    int r = r0;
    for (; r + U <= r1; r += U) rows_u(r);
    for (; r < r1; ++r) row_1(r);
  }
  float* pp = part + (size_t)blockIdx.y * cols + c0;
#pragma unroll
  for (int e = 0; e < E; e += 4) *reinterpret_cast<float4*>(pp + e) = make_float4(acc[e], acc[e + 1], acc[e + 2], acc[e + 3]);
}

// Column-blocked forward y = act(x + bias): the lane's E bias values stay in registers across
// its rows (no per-element column index math), 4 rows in flight.
template <typename T, typename Act, int U>
__global__ __launch_bounds__(256) void bias_act_fwd_2d(const T* __restrict__ x, const T* __restrict__ bias,
                                                       T* __restrict__ y, int rows, int cols, int rpb) {
  constexpr int E = 16 / sizeof(T);
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * E;
  if (c0 >= cols) return;
  const int r0 = blockIdx.y * rpb;
  const int r1 = min(rows, r0 + rpb);
  float b[E];
  load_f<T, E>(bias + c0, b);
  int r = r0;
  for (; r + U <= r1; r += U) {
    float v[U][E];
#pragma unroll
    for (int u = 0; u < U; ++u) load_f<T, E>(x + (size_t)(r + u) * cols + c0, v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int e = 0; e < E; ++e) v[u][e] = Act::f(v[u][e] + b[e]);
      store_f<T, E>(y + (size_t)(r + u) * cols + c0, v[u]);
    }
  }
  for (; r < r1; ++r) {
    float v[E];
    load_f<T, E>(x + (size_t)r * cols + c0, v);
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = Act::f(v[e] + b[e]);
    store_f<T, E>(y + (size_t)r * cols + c0, v);
  }
}

// rows per block for the column-blocked kernels: aim at g_cs_blocks workgroups (A/B knob
// pa_act_cs_tune), >= 16 rows each so the per-block column partials stay small
static int g_cs_blocks = 1024;
// row order of the column-sum kernels (pa_act_cs_set_interleave): 1 = groups of 4 rows dealt
// round-robin over the row blocks, 0 = a contiguous chunk per block (the batch-norm passes gained
// 2.6 % of the ResNet50 step from the round-robin order, profiles/r6t_bn_row_order_ab.log)
static int g_cs_inter = 1;
int cs_rows_per_block(int rows, int colblocks) {
  long long rpb = ((long long)rows * colblocks + g_cs_blocks - 1) / g_cs_blocks;
  if (rpb < 16) rpb = 16;
  if (rpb > rows) rpb = rows < 1 ? 1 : rows;
  return (int)rpb;
}

template <typename T, typename Act>
void launch_cs(dim3 grid, const void* dy, const void* x, const void* bias, void* dx, float* part, int rows, int cols,
               int rpb, hipStream_t st) {
  bias_act_bwd_cs<T, Act, true><<<grid, 256, 0, st>>>((const T*)dy, (const T*)x, (const T*)bias, (T*)dx, part, rows,
                                                       cols, rpb, g_cs_inter);
}

// swiglu: y = silu(a) * b   (a, b: separate tensors of n elements, both contiguous)
template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ y,
                                                  long long n, int a_stride_rows, int cols) {
  constexpr int E = 16 / sizeof(T);
  const long long nv = n / E;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nv; i += (long long)gridDim.x * 256) {
    const long long e0 = i * E;
    const long long r = e0 / cols, c = e0 % cols;
    const long long src = r * a_stride_rows + c;
    float va[E], vb[E], o[E];
    load_f<T, E>(a + src, va);
    load_f<T, E>(b + src, vb);
#pragma unroll
    for (int e = 0; e < E; ++e) o[e] = Silu::f(va[e]) * vb[e];
    store_f<T, E>(y + e0, o);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd(const T* __restrict__ a, const T* __restrict__ b,
                                                  const T* __restrict__ dy, T* __restrict__ da, T* __restrict__ db,
                                                  long long n, int a_stride_rows, int cols) {
  constexpr int E = 16 / sizeof(T);
  const long long nv = n / E;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nv; i += (long long)gridDim.x * 256) {
    const long long e0 = i * E;
    const long long r = e0 / cols, c = e0 % cols;
    const long long src = r * a_stride_rows + c;
    float va[E], vb[E], g[E], oa[E], ob[E];
    load_f<T, E>(a + src, va);
    load_f<T, E>(b + src, vb);
    load_f<T, E>(dy + e0, g);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      oa[e] = g[e] * vb[e] * Silu::df(va[e]);
      ob[e] = g[e] * Silu::f(va[e]);
    }
    store_f<T, E>(da + src, oa);
    store_f<T, E>(db + src, ob);
  }
}

// out = (residual ? residual : 0) + x * keep / (1 - p)
template <typename T>
__global__ __launch_bounds__(256) void dropout_add_fwd(const T* __restrict__ x, const T* __restrict__ residual,
                                                       T* __restrict__ y, long long n, float p, uint32_t seed,
                                                       uint32_t offset) {
  seed = rng_mix(seed);  // graph-captured steps: per-replay stream
  constexpr int E = 16 / sizeof(T);
  const float scale = 1.f / (1.f - p);
  const long long nv = n / E;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nv; i += (long long)gridDim.x * 256) {
    float v[E];
    load_f<T, E>(x + i * E, v);
    const uint32_t h0 = hash3(seed, offset, (uint32_t)(i));
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint32_t h = (e == 0) ? h0 : hash3(h0, (uint32_t)e, 0x2545F491u);
      v[e] = uniform01(h) >= p ? v[e] * scale : 0.f;
    }
    if (residual != nullptr) {
      float r[E];
      load_f<T, E>(residual + i * E, r);
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] += r[e];
    }
    store_f<T, E>(y + i * E, v);
  }
  if (blockIdx.x == 0) {
    for (long long i = nv * E + threadIdx.x; i < n; i += 256) {
      const uint32_t h = hash3(seed ^ 0x5bd1e995u, offset, (uint32_t)i);
      float v = uniform01(h) >= p ? to_f(x[i]) * scale : 0.f;
      if (residual != nullptr) v += to_f(residual[i]);
      y[i] = from_f<T>(v);
    }
  }
}

// dx = dy * keep / (1 - p)   (same hash stream as the forward)
template <typename T>
__global__ __launch_bounds__(256) void dropout_bwd(const T* __restrict__ dy, T* __restrict__ dx, long long n, float p,
                                                   uint32_t seed, uint32_t offset) {
  seed = rng_mix(seed);  // graph-captured steps: per-replay stream
  constexpr int E = 16 / sizeof(T);
  const float scale = 1.f / (1.f - p);
  const long long nv = n / E;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nv; i += (long long)gridDim.x * 256) {
    float v[E];
    load_f<T, E>(dy + i * E, v);
    const uint32_t h0 = hash3(seed, offset, (uint32_t)(i));
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint32_t h = (e == 0) ? h0 : hash3(h0, (uint32_t)e, 0x2545F491u);
      v[e] = uniform01(h) >= p ? v[e] * scale : 0.f;
    }
    store_f<T, E>(dx + i * E, v);
  }
  if (blockIdx.x == 0) {
    for (long long i = nv * E + threadIdx.x; i < n; i += 256) {
      const uint32_t h = hash3(seed ^ 0x5bd1e995u, offset, (uint32_t)i);
      dx[i] = from_f<T>(uniform01(h) >= p ? to_f(dy[i]) * scale : 0.f);
    }
  }
}

// y[c, r] = x[r, c] for 2-byte dtypes, [rows, cols] with both dims multiples of 64.
// One 64x64 tile per block through LDS: 16-byte global loads along x's rows, 16-byte global
// stores along y's rows; the LDS row pitch of 66 elements (33 banks) spreads the column reads.
// Used to hand hipBLASLt a K-major copy of paddle's [in, out] Linear weight for the forward GEMM.
__global__ __launch_bounds__(256) void transpose2d_b16(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                       int rows, int cols) {
  __shared__ uint16_t tile[64][66];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int lr = tid >> 3, lc = (tid & 7) * 8;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = lr + p * 32;
    const uint4 v = *reinterpret_cast<const uint4*>(x + (long long)(r0 + r) * cols + c0 + lc);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tile[r][lc + 2 * j] = (uint16_t)(w[j] & 0xffffu);
      tile[r][lc + 2 * j + 1] = (uint16_t)(w[j] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int c = lr + p * 32;  // output row (input column)
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = (uint32_t)tile[lc + 2 * j][c] | ((uint32_t)tile[lc + 2 * j + 1][c] << 16);
    *reinterpret_cast<uint4*>(y + (long long)(c0 + c) * rows + r0 + lc) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Wide form for cols % 128 == 0: a block transposes two side-by-side 64x64 tiles (four 16-byte
// loads in flight per thread instead of two), element pairs go to LDS as one dword (the even
// 66-element pitch keeps (2j, 2j + 1) in one dword), and each thread builds the 16-byte chunks of
// two adjacent output rows from eight dword reads (low halves -> row c, high halves -> row c + 1),
// a quarter of the LDS instructions of the 16-bit form.
__global__ __launch_bounds__(256) void transpose2d_b16_w(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                         int rows, int cols) {
  __shared__ uint32_t tile[2][64][33];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 128;
  const int lr = tid >> 3, ch = tid & 7;
  uint4 v[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int p = 0; p < 2; ++p)
      v[t][p] = *reinterpret_cast<const uint4*>(x + (long long)(r0 + lr + 32 * p) * cols + c0 + 64 * t + 8 * ch);
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      uint32_t* row = &tile[t][lr + 32 * p][4 * ch];
      row[0] = v[t][p].x;
      row[1] = v[t][p].y;
      row[2] = v[t][p].z;
      row[3] = v[t][p].w;
    }
  __syncthreads();
  const int c = 2 * (tid >> 3);  // output rows c, c + 1 of each tile (input columns)
  const int e0 = 8 * ch;         // output elements e0 .. e0 + 7 (input rows)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    uint32_t d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = tile[t][e0 + i][c >> 1];
    uint32_t a[4], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] = (d[2 * j] & 0xffffu) | (d[2 * j + 1] << 16);
      b[j] = (d[2 * j] >> 16) | (d[2 * j + 1] & 0xffff0000u);
    }
    const long long yc = c0 + 64 * t + c;
    *reinterpret_cast<uint4*>(y + yc * rows + r0 + e0) = make_uint4(a[0], a[1], a[2], a[3]);
    *reinterpret_cast<uint4*>(y + (yc + 1) * rows + r0 + e0) = make_uint4(b[0], b[1], b[2], b[3]);
  }
}

int cs_rows_per_block(int rows, int colblocks);

// forward bias+activation launch shape (A/B knob: pa_act_fwd_tune)
static int g_act_fwd_blocks = 8192;  // measured: 142 -> 105 us on [16384, 8192] bf16 GELU (copy: 100 us)
static int g_act_fwd_unroll = 2;

template <typename T, typename Act>
hipError_t launch_act(int dir, const void* dy, const void* x, const void* bias, void* out, long long n, int cols,
                      hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  if (dir == 0 && bias != nullptr && cols % E == 0 && n % cols == 0 && n / cols < (1LL << 31)) {
    const int rows = (int)(n / cols);
    const int cb = (cols + 256 * E - 1) / (256 * E);
    // rows per block: aim at g_act_fwd_blocks workgroups (>= 8 rows each); U rows of 16-byte loads in flight
    long long rpb = ((long long)rows * cb + g_act_fwd_blocks - 1) / g_act_fwd_blocks;
    rpb = rpb < 8 ? 8 : (rpb > rows ? rows : rpb);
    const dim3 grid(cb, (unsigned)((rows + rpb - 1) / rpb));
    if (g_act_fwd_unroll >= 8)
      bias_act_fwd_2d<T, Act, 8><<<grid, 256, 0, st>>>((const T*)x, (const T*)bias, (T*)out, rows, cols, (int)rpb);
    else if (g_act_fwd_unroll >= 4)
      bias_act_fwd_2d<T, Act, 4><<<grid, 256, 0, st>>>((const T*)x, (const T*)bias, (T*)out, rows, cols, (int)rpb);
    else
      bias_act_fwd_2d<T, Act, 2><<<grid, 256, 0, st>>>((const T*)x, (const T*)bias, (T*)out, rows, cols, (int)rpb);
    return hipGetLastError();
  }
  const int g = grid_for(n / E + 1, 256, 256 * 8);
  if (dir == 0) bias_act_fwd<T, Act><<<g, 256, 0, st>>>((const T*)x, (const T*)bias, (T*)out, n, cols);
  else bias_act_bwd<T, Act><<<g, 256, 0, st>>>((const T*)dy, (const T*)x, (const T*)bias, (T*)out, n, cols);
  return hipGetLastError();
}

}  // namespace pa

using namespace pa;

// act: 0 = gelu(erf), 1 = gelu(tanh), 2 = silu, 3 = relu, 4 = identity (bias add only)
// dir: 0 = forward (out = act(x + bias)), 1 = backward (out = dy * act'(x + bias))
PA_API hipError_t pa_bias_act(int act, int dir, const void* dy, const void* x, const void* bias, void* out,
                              long long n, int cols, int dt, hipStream_t st) {
  PA_DISPATCH_DTYPE(dt, T, {
    switch (act) {
      case 0: return launch_act<T, GeluErf>(dir, dy, x, bias, out, n, cols, st);
      case 1: return launch_act<T, GeluTanh>(dir, dy, x, bias, out, n, cols, st);
      case 2: return launch_act<T, Silu>(dir, dy, x, bias, out, n, cols, st);
      case 3: return launch_act<T, Relu>(dir, dy, x, bias, out, n, cols, st);
      case 4: return launch_act<T, Ident>(dir, dy, x, bias, out, n, cols, st);
      default: return hipErrorInvalidValue;
    }
  });
  return hipSuccess;
}

PA_API void pa_act_cs_tune(int target_blocks) {
  if (target_blocks > 0) g_cs_blocks = target_blocks;
}

PA_API int pa_act_cs_set_interleave(int v) {
  const int old = g_cs_inter;
  g_cs_inter = v;
  return old;
}

PA_API void pa_act_fwd_tune(int target_blocks, int unroll) {
  if (target_blocks > 0) g_act_fwd_blocks = target_blocks;
  if (unroll > 0) g_act_fwd_unroll = unroll;
}

// y = x^T for a contiguous 2-byte [rows, cols] matrix (rows, cols multiples of 64).
PA_API hipError_t pa_transpose2d(const void* x, void* y, int rows, int cols, int elem_bytes, hipStream_t st) {
  if (elem_bytes != 2 || rows % 64 != 0 || cols % 64 != 0 || rows <= 0 || cols <= 0 || rows / 64 > 65535)
    return hipErrorInvalidValue;
  if (cols % 128 == 0)
    transpose2d_b16_w<<<dim3(cols / 128, rows / 64), 256, 0, st>>>((const uint16_t*)x, (uint16_t*)y, rows, cols);
  else
    transpose2d_b16<<<dim3(cols / 64, rows / 64), 256, 0, st>>>((const uint16_t*)x, (uint16_t*)y, rows, cols);
  return hipGetLastError();
}

// a, b: [rows, cols] views with row stride a_stride (elements); y / da / db dense [rows, cols]
// (da/db written with the same strided layout as a/b, so a fused [rows, 2*cols] gate buffer works).
PA_API hipError_t pa_swiglu_fwd(const void* a, const void* b, void* y, long long n, int a_stride, int cols, int dt,
                                hipStream_t st) {
  if (cols % 8 != 0 && dt != 0) return hipErrorInvalidValue;
  PA_DISPATCH_DTYPE(dt, T, {
    const int g = grid_for(n / (16 / sizeof(T)) + 1, 256, 256 * 8);
    swiglu_fwd<T><<<g, 256, 0, st>>>((const T*)a, (const T*)b, (T*)y, n, a_stride, cols);
  });
  return hipGetLastError();
}

PA_API hipError_t pa_swiglu_bwd(const void* a, const void* b, const void* dy, void* da, void* db, long long n,
                                int a_stride, int cols, int dt, hipStream_t st) {
  if (cols % 8 != 0 && dt != 0) return hipErrorInvalidValue;
  PA_DISPATCH_DTYPE(dt, T, {
    const int g = grid_for(n / (16 / sizeof(T)) + 1, 256, 256 * 8);
    swiglu_bwd<T><<<g, 256, 0, st>>>((const T*)a, (const T*)b, (const T*)dy, (T*)da, (T*)db, n, a_stride, cols);
  });
  return hipGetLastError();
}

PA_API hipError_t pa_dropout_add_fwd(const void* x, const void* residual, void* y, long long n, float p, uint32_t seed,
                                     uint32_t offset, int dt, hipStream_t st) {
  PA_DISPATCH_DTYPE(dt, T, {
    const int g = grid_for(n / (16 / sizeof(T)) + 1, 256, 256 * 8);
    dropout_add_fwd<T><<<g, 256, 0, st>>>((const T*)x, (const T*)residual, (T*)y, n, p, seed, offset);
  });
  return hipGetLastError();
}

PA_API hipError_t pa_dropout_bwd(const void* dy, void* dx, long long n, float p, uint32_t seed, uint32_t offset, int dt,
                                 hipStream_t st) {
  PA_DISPATCH_DTYPE(dt, T, {
    const int g = grid_for(n / (16 / sizeof(T)) + 1, 256, 256 * 8);
    dropout_bwd<T><<<g, 256, 0, st>>>((const T*)dy, (T*)dx, n, p, seed, offset);
  });
  return hipGetLastError();
}

// Partial-row count the column-blocked kernels use (callers size `part` as nparts * cols floats).
PA_API int pa_colsum_nparts(int rows, int cols, int dt) {
  const int E = dt == 0 ? 4 : 8;
  const int cb = (cols + 256 * E - 1) / (256 * E);
  const int rpb = cs_rows_per_block(rows, cb);
  return (rows + rpb - 1) / rpb;
}

// dx = dy * act'(x + bias) over [rows, cols] AND dbias (+)= colsum(dx) (out dtype odt, accumulated
// in place when accum) — the bias gradient never takes a separate pass over dx.
PA_API hipError_t pa_bias_act_bwd_dbias(int act, const void* dy, const void* x, const void* bias, void* dx,
                                        float* part, void* dbias, int odt, int accum, int rows, int cols, int dt,
                                        hipStream_t st) {
  const int E = dt == 0 ? 4 : 8;
  if (cols % E != 0) return hipErrorInvalidValue;
  const int cb = (cols + 256 * E - 1) / (256 * E);
  const int rpb = cs_rows_per_block(rows, cb);
  const dim3 grid(cb, (rows + rpb - 1) / rpb);
  PA_DISPATCH_DTYPE(dt, T, {
    switch (act) {
      case 0: launch_cs<T, GeluErf>(grid, dy, x, bias, dx, part, rows, cols, rpb, st); break;
      case 1: launch_cs<T, GeluTanh>(grid, dy, x, bias, dx, part, rows, cols, rpb, st); break;
      case 2: launch_cs<T, Silu>(grid, dy, x, bias, dx, part, rows, cols, rpb, st); break;
      case 3: launch_cs<T, Relu>(grid, dy, x, bias, dx, part, rows, cols, rpb, st); break;
      case 4: launch_cs<T, Ident>(grid, dy, x, bias, dx, part, rows, cols, rpb, st); break;
      default: return hipErrorInvalidValue;
    }
  });
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_colsum_finish_dt(part, dbias, odt, (int)grid.y, cols, accum, st);
}

// out (+)= sum of the nrows fp32 partial rows part[nrows][cols] (partials produced elsewhere, e.g. the
// fused fc2-dgrad GEMM epilogue's column sums).
PA_API hipError_t pa_colsum_finish_parts(const float* part, void* out, int odt, int accum, int nrows, int cols,
                                         hipStream_t st) {
  return launch_colsum_finish_dt(part, out, odt, nrows, cols, accum, st);
}

// out (+)= colsum(dy) for dy [rows, cols] with row stride ld == cols (the bias gradient of a Linear).
PA_API hipError_t pa_colsum(const void* dy, float* part, void* out, int odt, int accum, int rows, int cols, int dt,
                            hipStream_t st) {
  const int E = dt == 0 ? 4 : 8;
  if (cols % E != 0) return hipErrorInvalidValue;
  const int cb = (cols + 256 * E - 1) / (256 * E);
  const int rpb = cs_rows_per_block(rows, cb);
  const dim3 grid(cb, (rows + rpb - 1) / rpb);
  PA_DISPATCH_DTYPE(dt, T, {
    bias_act_bwd_cs<T, Ident, false><<<grid, 256, 0, st>>>((const T*)dy, nullptr, nullptr, nullptr, part, rows, cols,
                                                            rpb, g_cs_inter);
  });
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_colsum_finish_dt(part, out, odt, (int)grid.y, cols, accum, st);
}

// graph-safe dropout streams (common.h rng_mix): generation counter of this module's kernels
PA_API int pa_act_set_rng_gen(const void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(pa::g_rng_gen), &p, sizeof(p));
}
