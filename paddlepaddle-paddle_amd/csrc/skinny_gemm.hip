// Skinny (decode) GEMM for gfx950: Y[M, N] = X[M, K] @ W + bias, M <= 64 new tokens, weight-
// streaming bound (every weight byte is read once; the activations are tiny).
//
// Reference semantics: the matmul / fused_linear calls of the decode step of
// paddle/phi/kernels/fusion/gpu/fused_multi_transformer_kernel.cu (and any Linear at small batch),
// where cuBLAS / hipBLASLt pick GEMV-like kernels.  The library ran the Llama-2-13B layer shapes at
// 2.3-2.6x the weight-streaming bound (tools/decode_gemm_bench.py).
//
// CDNA4 design:
//  * W [K][N] n-contiguous (paddle's Linear weight): a lane owns an 8 x 8 block of W (8 k rows x 8
//    columns; the 16 lanes of a row group read 16 contiguous 16-B chunks = 256 B of one weight
//    row) and transposes it in registers with v_perm_b32, giving one MFMA B fragment (8 k values of
//    one column) per column.  v_mfma_f32_16x16x32_bf16 number c (c = 0..7) then multiplies the
//    activation fragment (A: 16 rows x 32 k) by "column c of every lane's block": the 16 MFMA
//    columns are the 16 column blocks, so a wave covers 128 columns with 8 MFMAs per 32-deep k
//    step and no LDS at all.
//  * W [N][K] k-contiguous (transposed weights, e.g. trans_qkvw): a lane's 16-B load already is a
//    B fragment; 8 MFMAs cover 8 groups of 16 columns.
//  * Up to 4 row tiles of 16 (M <= 64) reuse every B fragment.  Weight loads of the next 3 steps
//    (M <= 32; 1 step at M <= 64) are in flight while a step multiplies (register stages).
//  * Parallelism: blocks = 128-column tiles x K splits (~2 per CU); the 4 waves of a block split
//    its K range and are summed through LDS; the K splits go to an fp32 partial buffer that a
//    second kernel sums (+ bias) into the bf16 output.
#include "common.h"

namespace pa {
namespace sk {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// One 32-deep k step's weight registers of a lane: W n-major -> 8 rows of a 16-B chunk; k-major
// -> 8 chunks of 8 k (one per 16-column group).
struct WRegs {
  uint4 v[8];
};

template <bool KMAJ>
__device__ __forceinline__ void load_w(WRegs& r, const uint16_t* __restrict__ W, long long ldw, int k0, int n0,
                                       int lane, int N) {
  const int g = lane >> 4, i = lane & 15;
  if constexpr (!KMAJ) {
    const int col = min(n0 + 8 * i, N - 8);  // clamped columns are never stored
#pragma unroll
    for (int q = 0; q < 8; ++q) r.v[q] = *reinterpret_cast<const uint4*>(W + (long long)(k0 + 8 * g + q) * ldw + col);
  } else {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int col = min(n0 + 16 * c + i, N - 1);
      r.v[c] = *reinterpret_cast<const uint4*>(W + (long long)col * ldw + k0 + 8 * g);
    }
  }
}

// B fragment c: n-major -> column c of the lane's 8 x 8 block (k = 8g .. 8g+7), by byte selects.
template <bool KMAJ>
__device__ __forceinline__ s16x8 bfrag(const WRegs& r, int c) {
  if constexpr (KMAJ) {
    return __builtin_bit_cast(s16x8, r.v[c]);
  } else {
    const unsigned sel = (c & 1) ? 0x07060302u : 0x05040100u;
    unsigned d[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 a = r.v[2 * q], b = r.v[2 * q + 1];
      const unsigned wa = (c >> 1) == 0 ? a.x : (c >> 1) == 1 ? a.y : (c >> 1) == 2 ? a.z : a.w;
      const unsigned wb = (c >> 1) == 0 ? b.x : (c >> 1) == 1 ? b.y : (c >> 1) == 2 ? b.z : b.w;
      d[q] = __builtin_amdgcn_perm(wb, wa, sel);
    }
    return __builtin_bit_cast(s16x8, make_uint4(d[0], d[1], d[2], d[3]));
  }
}

// grid (ceil(N / 128), KS), 256 threads.  part: fp32 [KS][M][N].
// NST register stages: a stage holds one 32-deep step's weights AND activation fragments, so the
// wait for a step's operands never waits on a later step's weight loads (vmcnt retires in order);
// NST - 1 steps of weight loads stay in flight while a step multiplies.
template <int MT, bool KMAJ, int NST>
__global__ __launch_bounds__(256) void skinny_kernel(const uint16_t* __restrict__ X, long long ldx,
                                                     const uint16_t* __restrict__ W, long long ldw,
                                                     float* __restrict__ part, int M, int N, int K, int kchunk) {
  __shared__ float red[3][MT * 8 * 4][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n0 = blockIdx.x * 128;
  const int kw = kchunk / 4;  // per wave, multiple of 32
  const int kbeg = blockIdx.y * kchunk + w * kw;
  const int kend = min(K, kbeg + kw);
  const int g = lane >> 4, i = lane & 15;
  f32x4 acc[MT][8];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  WRegs rw[NST];
  s16x8 rx[NST][MT];
  auto load_stage = [&](int st, int k0) {
    load_w<KMAJ>(rw[st], W, ldw, k0, n0, lane, N);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = 16 * t + i;
      rx[st][t] = m < M ? *reinterpret_cast<const s16x8*>(X + (long long)m * ldx + k0 + 8 * g)
                        : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
#pragma unroll
  for (int st = 0; st < NST; ++st)
    if (kbeg + 32 * st < kend) load_stage(st, kbeg + 32 * st);
  for (int base = kbeg; base < kend; base += 32 * NST) {
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      const int k0 = base + 32 * st;
      if (k0 >= kend) break;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const s16x8 bf = bfrag<KMAJ>(rw[st], c);
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[t][c] = mfma(rx[st][t], bf, acc[t][c]);
      }
      if (k0 + 32 * NST < kend) load_stage(st, k0 + 32 * NST);
    }
  }
  // sum the 4 waves' K slices through LDS (waves 1-3 park, wave 0 adds and stores)
  if (w > 0) {
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[w - 1][(t * 8 + c) * 4 + r][lane] = acc[t][c][r];
  }
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[t][c][r] += red[0][(t * 8 + c) * 4 + r][lane] + red[1][(t * 8 + c) * 4 + r][lane] +
                        red[2][(t * 8 + c) * 4 + r][lane];
  // lane holds C[m = 16t + 4g + r][j = i] of MFMA c; j -> column n0 + 8i + c (n-major) or
  // n0 + 16c + i (k-major)
  float* out = part + (long long)blockIdx.y * M * N;
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 16 * t + 4 * g + r;
      if (m >= M) continue;
      if constexpr (!KMAJ) {
        const int col = n0 + 8 * i;
        if (col < N) {
          float* o = out + (long long)m * N + col;
          *reinterpret_cast<float4*>(o) = make_float4(acc[t][0][r], acc[t][1][r], acc[t][2][r], acc[t][3][r]);
          *reinterpret_cast<float4*>(o + 4) = make_float4(acc[t][4][r], acc[t][5][r], acc[t][6][r], acc[t][7][r]);
        }
      } else {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const int col = n0 + 16 * c + i;
          if (col < N) out[(long long)m * N + col] = acc[t][c][r];
        }
      }
    }
}

// Y[m, n] = sum_s part[s][m][n] (+ bias[n]), 8 columns per thread
__global__ __launch_bounds__(256) void skinny_finish(const float* __restrict__ part, int KS, int M, int N,
                                                     const uint16_t* __restrict__ bias, uint16_t* __restrict__ Y,
                                                     long long ldy) {
  const long long e = ((long long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (e >= (long long)M * N) return;
  const int m = (int)(e / N), n = (int)(e - (long long)m * N);
  float v[8];
  {
    const float4 a = *reinterpret_cast<const float4*>(part + e), b = *reinterpret_cast<const float4*>(part + e + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  for (int s = 1; s < KS; ++s) {
    const float* p = part + (long long)s * M * N + e;
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
  }
  if (bias != nullptr) {
    float bb[8];
    load_f<bf16_t, 8>(reinterpret_cast<const bf16_t*>(bias + n), bb);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] += bb[q];
  }
  store_f<bf16_t, 8>(reinterpret_cast<bf16_t*>(Y + (long long)m * ldy + n), v);
}

// K splits: ~2 blocks per CU over the 128-column tiles; each split a multiple of 128 rows
static void plan(int N, int K, int& KS, int& kchunk) {
  const int tiles = (N + 127) / 128;
  int ks = (512 + tiles - 1) / tiles;
  const int kmax = (K + 127) / 128;
  ks = ks < 1 ? 1 : (ks > kmax ? kmax : ks);
  kchunk = ((K + ks - 1) / ks + 127) / 128 * 128;
  KS = (K + kchunk - 1) / kchunk;
}

}  // namespace sk
}  // namespace pa

// Contract: 1 <= M <= 64, K % 32 == 0, N % 8 == 0, X rows k-contiguous (ldx % 8 == 0), W either
// [K][N] row-major (wkmajor = 0, ldw % 8 == 0) or [N][K] row-major (wkmajor = 1), 16-B aligned.
PA_API int pa_skinny_ok(int M, int N, int K, long long ldx, long long ldw) {
  return M >= 1 && M <= 64 && K >= 32 && K % 32 == 0 && N >= 8 && N % 8 == 0 && ldx % 8 == 0 && ldw % 8 == 0;
}

// fp32 scratch floats pa_skinny_gemm needs
PA_API long long pa_skinny_ws_floats(int M, int N, int K) {
  int KS, kc;
  pa::sk::plan(N, K, KS, kc);
  return (long long)KS * M * N;
}

PA_API int pa_skinny_gemm(const void* X, const void* W, const void* bias, void* Y, float* ws, int M, int N, int K,
                          long long ldx, long long ldw, long long ldy, int wkmajor, hipStream_t st) {
  using namespace pa::sk;
  if (!pa_skinny_ok(M, N, K, ldx, ldw) || ws == nullptr || ldy % 8) return (int)hipErrorInvalidValue;
  int KS, kchunk;
  plan(N, K, KS, kchunk);
  const dim3 grid((N + 127) / 128, KS);
  const uint16_t* x = (const uint16_t*)X;
  const uint16_t* w = (const uint16_t*)W;
#define SK_LAUNCH(MT, NST)                                                                                \
  do {                                                                                                    \
    if (wkmajor) skinny_kernel<MT, true, NST><<<grid, 256, 0, st>>>(x, ldx, w, ldw, ws, M, N, K, kchunk); \
    else skinny_kernel<MT, false, NST><<<grid, 256, 0, st>>>(x, ldx, w, ldw, ws, M, N, K, kchunk);        \
  } while (0)
  if (M <= 16) SK_LAUNCH(1, 4);
  else if (M <= 32) SK_LAUNCH(2, 4);
  else SK_LAUNCH(4, 2);
#undef SK_LAUNCH
  const long long groups = ((long long)M * N + 7) / 8;
  skinny_finish<<<(unsigned)((groups + 255) / 256), 256, 0, st>>>(ws, KS, M, N, (const uint16_t*)bias, (uint16_t*)Y,
                                                                  ldy);
  return (int)hipGetLastError();
}
