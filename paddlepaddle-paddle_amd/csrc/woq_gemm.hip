// Weight-only int8 / int4 decode GEMM for gfx950 (W8A16 / W4A16): Y[M, N] = X[M, K] @ dequant(Wq)^T
// (+ bias), M <= 32 new tokens.  The weight is streamed from HBM once in its quantised form (1 or
// 0.5 byte per element instead of 2) and dequantised in registers, straight into MFMA B fragments.
//
// Reference semantics: paddle/phi/kernels/gpu/weight_only_linear_kernel.cu (CUTLASS fpA_intB GEMV /
// GEMM), python/paddle/nn/quant/quantized_linear.py:151 weight_only_linear, with this framework's
// weight layout (nn/quant/quantized_linear.py weight_quantize): int8 [N][K] (k contiguous), int4
// packed two signed nibbles per byte along k ([N][K/2]; per 8 k: byte b = k b low nibble, k 4 + b high
// nibble), symmetric scales per
// output channel ([N]) or per k-group of 64 / 128 ([K/G][N]).
//
// CDNA4 design (the k-major path of skinny_gemm.hip, widened per byte):
//  * A wave owns 128 output columns: lane (g = lane>>4, i = lane&15) handles columns n0 + 16c + i
//    (c = 0..7).  Per k chunk it loads ONE 16-B piece per column: int8 -> 16 k values (chunk 64),
//    int4 -> 32 k values (chunk 128), so a chunk is 8 x 16 B per lane like the bf16 kernel's 32-k
//    step, but covers 2x / 4x the k.
//  * k order inside a chunk is permuted identically for both operands: lane group g takes k values
//    [16g, 16g+16) (int8) or [32g, 32g+32) (int4) and splits them into 2 / 4 MFMA steps of 8; the
//    activation fragment of step s is X[m][k0 + 16g + 8s .. +8] (int8) / X[m][k0 + 32g + 8s ..]
//    (int4) — 16-B loads of contiguous bf16, no shuffles.  Every k appears exactly once, so the
//    dot products are exact sums in a different order.
//  * Dequant, group scales: a byte u (int8 xor 0x80, int4 nibble xor 0x8) becomes the fp32 2^23 + u
//    with one v_perm_b32 (exponent byte 0x4B, two zero bytes, u), minus (2^23 + 128 / 8) gives the
//    signed integer exactly; the group scale multiplies in fp32 before the 16-bit pack.  Per-channel
//    scales: the MFMA runs on unsigned codes held exactly in 16 bits (frag_u8 / frag_u4, the
//    constant offset removed in the epilogue with per-row sums of X) and the scale is applied to
//    the fp32 accumulator at the end.
//  * Up to 2 row tiles of 16 (M <= 32) share each dequantised fragment; NST register stages keep the
//    next chunks' weight loads in flight (all loads unconditional, so the waits are counted); the 4 waves of a block split its K range and are summed
//    through LDS; K splits across blocks go to an fp32 partial buffer summed by the finish kernel
//    (+ per-channel scale, + bias).
#include "common.h"

namespace pa {
namespace woq {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <typename T>
__device__ __forceinline__ f32x4 mfma(s16x8 a, s16x8 b, f32x4 c) {
  if constexpr (__is_same(T, f16_t))
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
}

// byte b (0..3) of d as the fp32 2^23 + byte
__device__ __forceinline__ float magic(unsigned d, int b) {
  return __builtin_bit_cast(float, __builtin_amdgcn_perm(0x4B000000u, d, 0x07040400u | (unsigned)b));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// two floats -> one packed 16-bit pair in ONE v_cvt_pk_{bf16,f16}_f32 (element-wise conversions
// compiled to two converts plus a pack)
template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  const f32x2 v = {a, b};
  if constexpr (__is_same(T, f16_t))
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, f16x2));
  else
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}

// acc + the sum of the 8 16-bit values of a fragment: 4 v_dot2c_f32_{bf16,f16} against (1, 1)
template <typename T>
__device__ __forceinline__ float rowsum8(s16x8 f, float acc) {
  const uint4 u = __builtin_bit_cast(uint4, f);
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if constexpr (__is_same(T, f16_t)) {
      const f16x2 one = {(_Float16)1.f, (_Float16)1.f};
      acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, w[j]), one, acc, false);
    } else {
      const bf16x2 one = {(__bf16)1.f, (__bf16)1.f};
      acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, w[j]), one, acc, false);
    }
  }
  return acc;
}

// 8 signed values (exact integers, or * s when SCALE) of one MFMA fragment.
// int8: bytes q[0..7] of the two dwords lo, hi (k order = byte order).
template <typename T, bool SCALE>
__device__ __forceinline__ s16x8 frag_i8(unsigned lo, unsigned hi, float s) {
  lo ^= 0x80808080u;
  hi ^= 0x80808080u;
  constexpr float off = 8388608.0f + 128.0f;
  float v[8];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    v[b] = magic(lo, b) - off;
    v[4 + b] = magic(hi, b) - off;
  }
  if constexpr (SCALE) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= s;
  }
  return __builtin_bit_cast(s16x8, make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]),
                                              pack2<T>(v[6], v[7])));
}

// int4: one dword = 8 nibbles, k = b (low nibble of byte b), 4 + b (high nibble)
template <typename T, bool SCALE>
__device__ __forceinline__ s16x8 frag_i4(unsigned d, float s) {
  const unsigned lo = (d & 0x0F0F0F0Fu) ^ 0x08080808u;         // k = 0, 1, 2, 3
  const unsigned hi = ((d >> 4) & 0x0F0F0F0Fu) ^ 0x08080808u;  // k = 4, 5, 6, 7
  constexpr float off = 8388608.0f + 8.0f;
  float v[8];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    v[b] = magic(lo, b) - off;
    v[4 + b] = magic(hi, b) - off;
  }
  if constexpr (SCALE) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= s;
  }
  return __builtin_bit_cast(s16x8, make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]),
                                              pack2<T>(v[6], v[7])));
}

// Per-channel-scale path (no group scales): the MFMA runs on the UNSIGNED codes u = q + 128
// (int8) / q + 8 (int4), exact in bf16 / fp16 (integers <= 256), converted with one
// v_cvt_f32_ubyte per element (the backend's byte -> float instruction) and one pack per pair: 12
// VALU per 8 int8 elements instead of 22 with the magic-number form (the kernel was VALU-issue
// bound: SQ_WAIT_INST_ANY 50 %, profiles/r4j_woq_pmc.txt).  The offset comes back out exactly in
// the finish kernel: y = s * (sum_k x_k u_k - off * sum_k x_k), from per-row sums of X.
template <typename T>
__device__ __forceinline__ s16x8 frag_u8(unsigned lo, unsigned hi) {
  lo ^= 0x80808080u;  // two's-complement byte q -> unsigned code q + 128
  hi ^= 0x80808080u;
  if constexpr (__is_same(T, f16_t)) {
    // fp16 holds 1024 + u exactly (10 mantissa bits): one byte permute per pair, as frag_u4
    constexpr unsigned E = 0x64646464u;
    return __builtin_bit_cast(s16x8, make_uint4(__builtin_amdgcn_perm(E, lo, 0x04010400u),
                                                __builtin_amdgcn_perm(E, lo, 0x04030402u),
                                                __builtin_amdgcn_perm(E, hi, 0x04010400u),
                                                __builtin_amdgcn_perm(E, hi, 0x04030402u)));
  }
  float v[8];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    v[b] = (float)((lo >> (8 * b)) & 0xFFu);
    v[4 + b] = (float)((hi >> (8 * b)) & 0xFFu);
  }
  return __builtin_bit_cast(s16x8, make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]),
                                              pack2<T>(v[6], v[7])));
}

// int4, per-channel scale: the byte codes u = q + 8 (0..15) of a dword's low nibbles (k 0..3) and
// high nibbles (k 4..7) become 16-bit operands with ONE v_perm_b32 per pair: each code is placed
// under a constant exponent byte — bf16 0x43:u = 128 + u (exact, 7 mantissa bits), fp16 0x64:u =
// 1024 + u — so 8 values cost 4 extract + 4 permute VALU (was 16 with byte -> float -> pack).  The
// constant comes back out in the epilogue with the row sums: y = s * (sum x v - off * sum x),
// off = 136 (bf16) / 1032 (fp16).
template <typename T>
__device__ __forceinline__ s16x8 frag_u4(unsigned d) {
  const unsigned t = d ^ 0x88888888u;                 // two's-complement nibble q -> code q + 8
  const unsigned lo = t & 0x0F0F0F0Fu;                // k = 0, 1, 2, 3
  const unsigned hi = (t >> 4) & 0x0F0F0F0Fu;         // k = 4, 5, 6, 7
  constexpr unsigned E = __is_same(T, f16_t) ? 0x64646464u : 0x43434343u;
  // v_perm_b32(src0 = E, src1 = x, sel): selector 0..3 = byte of x, 4 = the exponent byte
  return __builtin_bit_cast(s16x8, make_uint4(__builtin_amdgcn_perm(E, lo, 0x04010400u),
                                              __builtin_amdgcn_perm(E, lo, 0x04030402u),
                                              __builtin_amdgcn_perm(E, hi, 0x04010400u),
                                              __builtin_amdgcn_perm(E, hi, 0x04030402u)));
}

// grid (ceil(N / 128), KS), 256 threads.  part: fp32 [KS][M][N].  BITS 8 / 4; G = group size (0 =
// per channel: the scale is applied by the finish kernel).
template <typename T, int BITS, int MT, int NST, bool GRP, int CT = 8>
__global__ __launch_bounds__(256) void woq_kernel(const uint16_t* __restrict__ X, long long ldx,
                                                  const uint8_t* __restrict__ Wq, long long ldw_bytes,
                                                  const float* __restrict__ gscale, int group,
                                                  float* __restrict__ part, int M, int N, int K, int kchunk,
                                                  float* __restrict__ xsum, uint16_t* __restrict__ Y, long long ldy,
                                                  const uint16_t* __restrict__ bias, float off) {
  constexpr int KC = BITS == 8 ? 64 : 128;  // k per chunk
  constexpr int NS = KC / 32;                // MFMA steps per chunk
  __shared__ float red[3][MT * CT * 4][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n0 = blockIdx.x * 16 * CT;
  const int kw = kchunk / 4;  // per wave, a multiple of KC
  const int kbeg = blockIdx.y * kchunk + w * kw;
  const int kend = min(K, kbeg + kw);
  const int g = lane >> 4, i = lane & 15;
  f32x4 acc[MT][CT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  int cols[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) cols[c] = min(n0 + 16 * c + i, N - 1);  // clamped columns are never stored
  uint4 rw[NST][CT];
  s16x8 rx[NST][MT][NS];
  float rs[NST][GRP ? CT : 1];  // group scales of the stage's k range (GRP)
  // every load below is unconditional: chunk indices past the wave's range are clamped to its last
  // chunk (re-read, never used), so the compiler's counted waits retire exactly one stage (guarded
  // loads made it wait for vmcnt(0) and the register stages never overlapped)
  const int nch = (kend - kbeg) / KC;  // kbeg..kend is a whole number of chunks
  auto load_stage = [&](int st, int j) {
    const int k0 = kbeg + KC * min(j, max(nch - 1, 0));
    const long long kb = BITS == 8 ? (long long)(k0 + 16 * g) : (long long)(k0 / 2 + 16 * g);
#pragma unroll
    for (int c = 0; c < CT; ++c) rw[st][c] = *reinterpret_cast<const uint4*>(Wq + (long long)cols[c] * ldw_bytes + kb);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = min(16 * t + i, M - 1);  // rows past M are never stored
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int kk = k0 + (BITS == 8 ? 16 : 32) * g + 8 * s;
        rx[st][t][s] = *reinterpret_cast<const s16x8*>(X + (long long)m * ldx + kk);
      }
    }
    if constexpr (GRP) {
      // this lane's k range [k0 + 16g, +16) / [k0 + 32g, +32) lies inside one group (group >= 64)
      const int gi = (k0 + (BITS == 8 ? 16 : 32) * g) / group;
#pragma unroll
      for (int c = 0; c < CT; ++c) rs[st][c] = gscale[(long long)gi * N + cols[c]];
    }
  };
  // !GRP: per-row sums of the X fragments this wave multiplies (column tile 0 only), for the
  // finish kernel's offset correction
  float xs[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) xs[t] = 0.f;
  // fused epilogue (Y != null, the K range is not split across blocks): every block needs its rows'
  // sums for the offset correction
  const bool want_xs = !GRP && (Y != nullptr || blockIdx.x == 0);
  auto compute = [&](int st) {
    if (!GRP && want_xs) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int s = 0; s < NS; ++s) xs[t] = rowsum8<T>(rx[st][t][s], xs[t]);
    }
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const uint4 q = rw[st][c];
      const float sc = GRP ? rs[st][GRP ? c : 0] : 1.f;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        s16x8 bf;
        if constexpr (BITS == 8 && GRP) {
          bf = s == 0 ? frag_i8<T, GRP>(q.x, q.y, sc) : frag_i8<T, GRP>(q.z, q.w, sc);
        } else if constexpr (BITS == 8) {
          bf = s == 0 ? frag_u8<T>(q.x, q.y) : frag_u8<T>(q.z, q.w);
        } else if constexpr (GRP) {
          const unsigned d = s == 0 ? q.x : s == 1 ? q.y : s == 2 ? q.z : q.w;
          bf = frag_i4<T, GRP>(d, sc);
        } else {
          const unsigned d = s == 0 ? q.x : s == 1 ? q.y : s == 2 ? q.z : q.w;
          bf = frag_u4<T>(d);
        }
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[t][c] = mfma<T>(rx[st][t][s], bf, acc[t][c]);
      }
    }
  };
  if (nch > 0) {
#pragma unroll
    for (int st = 0; st < NST; ++st) load_stage(st, st);
  }
  for (int j = 0; j < nch; j += NST) {
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      if (j + st < nch) compute(st);  // wave-uniform; no loads inside
      load_stage(st, j + st + NST);
    }
  }
  __shared__ float xred[4][MT * 16];
  if (want_xs) {
    // lanes (g, i) of row 16t + i: sum over the 4 k-slice groups, then over the 4 waves
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      float v = xs[t];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g == 0) xred[w][t * 16 + i] = v;
    }
  }
  if (w > 0) {
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[w - 1][(t * CT + c) * 4 + r][lane] = acc[t][c][r];
  }
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[t][c][r] += red[0][(t * CT + c) * 4 + r][lane] + red[1][(t * CT + c) * 4 + r][lane] +
                        red[2][(t * CT + c) * 4 + r][lane];
  if (Y != nullptr) {
    // fused finish (one K split): y = (acc - off * rowsum) * cscale + bias, straight to Y; the lane
    // holds C[m = 16t + 4g + r][column n0 + 16c + i]
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * t + 4 * g + r;
        if (m >= M) continue;
        const float xr = GRP ? 0.f : xred[0][m] + xred[1][m] + xred[2][m] + xred[3][m];
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          const int col = n0 + 16 * c + i;
          if (col >= N) continue;
          float v = acc[t][c][r];
          if constexpr (!GRP) v = (v - off * xr) * gscale[col];
          if (bias != nullptr) v += to_f(__builtin_bit_cast(T, bias[col]));
          Y[(long long)m * ldy + col] = __builtin_bit_cast(uint16_t, from_f<T>(v));
        }
      }
    return;
  }
  if (want_xs && lane < MT * 16 && lane < M) {
    xsum[(long long)blockIdx.y * M + lane] = xred[0][lane] + xred[1][lane] + xred[2][lane] + xred[3][lane];
  }
  // lane holds C[m = 16t + 4g + r][column n0 + 16c + i]
  float* out = part + (long long)blockIdx.y * M * N;
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 16 * t + 4 * g + r;
      if (m >= M) continue;
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        const int col = n0 + 16 * c + i;
        if (col < N) out[(long long)m * N + col] = acc[t][c][r];
      }
    }
}

// Y[m, n] = (sum_s part[s][m][n]) * (cscale ? cscale[n] : 1) (+ bias[n]), 8 columns per thread
// (xsum != null: the partials are of the unsigned codes; subtract off * sum_s xsum[s][m] first)
template <typename T>
__global__ __launch_bounds__(256) void woq_finish(const float* __restrict__ part, int KS, int M, int N,
                                                  const float* __restrict__ cscale, const uint16_t* __restrict__ bias,
                                                  uint16_t* __restrict__ Y, long long ldy,
                                                  const float* __restrict__ xsum, float off) {
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
  if (xsum != nullptr) {
    float xs = 0.f;
    for (int s = 0; s < KS; ++s) xs += xsum[(long long)s * M + m];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] -= off * xs;
  }
  if (cscale != nullptr) {
    const float4 a = *reinterpret_cast<const float4*>(cscale + n), b = *reinterpret_cast<const float4*>(cscale + n + 4);
    v[0] *= a.x; v[1] *= a.y; v[2] *= a.z; v[3] *= a.w; v[4] *= b.x; v[5] *= b.y; v[6] *= b.z; v[7] *= b.w;
  }
  if (bias != nullptr) {
    float bb[8];
    load_f<T, 8>(reinterpret_cast<const T*>(bias + n), bb);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] += bb[q];
  }
  store_f<T, 8>(reinterpret_cast<T*>(Y + (long long)m * ldy + n), v);
}

// tuning knobs (pa_woq_tune): target blocks of the K-split plan, register stages of the M <= 16 kernel
// (graph-timed sweeps, profiles/r4n_woq_sweep.log / r4p_woq_sweep.log: 2 register stages and ~256
// blocks at M <= 16; for the M <= 32 kernel ~256 blocks on wide outputs (>= 100 column tiles), ~512 on
// narrow ones; g_target_blocks > 0 overrides)
static int g_target_blocks = 0, g_nst = 2;
// A/B switch (pa_woq_set_fused_finish): single-split launches finish in the main kernel (default on)
static int g_fused_finish = 1;

// K splits: ~g_target_blocks blocks over the 128-column tiles; each split a multiple of 4 waves x chunk
// 16-column tiles per wave of the M <= 16 kernel (8 = 128 columns per block, 4 = 64, 2 = 32): narrower
// tiles mean fewer registers per wave, more waves and more independent dequant chains in flight.
// Automatic (g_ct = 0): 2 at M <= 4, 4 at M <= 16 — graph-timed on the Llama-2-13B shapes, M = 1
// int8 1.38-1.60x / int4 1.50-2.07x the bf16 skinny GEMM (profiles/r4q_woq_sweep.log).
// Since the single-split launches finish in the main kernel (no finish pass), the sweep after the
// byte-permute int4 dequant (profiles/r5v_woq_sweep.log) favours one K split with 32-column waves
// wherever that still gives >= 128 blocks: M <= 4 always (ffn2 K = 13824: int8 21.5 -> 18.5 us, int4
// 15.0 -> 12.4); 5 <= M <= 16 unless the output is wide (N >= 16384) or deep (K > 2N), where 64-column
// waves split over ~256 blocks stay ahead (ffn1 25.9 vs 33.3 us int4).
static int g_ct = 0;
static bool wide_or_deep(int N, int K) { return N >= 16384 || K > 2 * N; }
static int eff_ct(int M, int N, int K) {
  return M > 16 ? 8 : (g_ct ? g_ct : (M <= 4 || !wide_or_deep(N, K) ? 2 : 4));
}

static void plan(int N, int K, int bits, int M, int& KS, int& kchunk) {
  const int unit = 4 * (bits == 8 ? 64 : 128);
  const int ct = eff_ct(M, N, K);
  const int tiles = (N + 16 * ct - 1) / (16 * ct);
  const int target = g_target_blocks > 0
                         ? g_target_blocks
                         : (M <= 4 || (M <= 16 && !wide_or_deep(N, K)) ? 128 : (M <= 16 || tiles >= 100 ? 256 : 512));
  int ks = (target + tiles - 1) / tiles;
  const int kmax = (K + unit - 1) / unit;
  ks = ks < 1 ? 1 : (ks > kmax ? kmax : ks);
  kchunk = ((K + ks - 1) / ks + unit - 1) / unit * unit;
  KS = (K + kchunk - 1) / kchunk;
}

template <typename T, int BITS, bool GRP>
static void launch(const void* X, long long ldx, const void* Wq, long long ldwb, const float* gscale, int group,
                   float* ws, int M, int N, int K, int KS, int kchunk, float* xsum, uint16_t* Y, long long ldy,
                   const uint16_t* bias, float off, hipStream_t st) {
  const dim3 grid((N + 16 * eff_ct(M, N, K) - 1) / (16 * eff_ct(M, N, K)), KS);
  const uint16_t* x = (const uint16_t*)X;
  const uint8_t* w = (const uint8_t*)Wq;
  // (a 4-row-tile variant for M <= 64 spills at 256 VGPRs: M > 32 takes the dequantise + GEMM path)
  const int ct = eff_ct(M, N, K);
  if (M <= 16 && ct == 2)
    woq_kernel<T, BITS, 1, 2, GRP, 2><<<grid, 256, 0, st>>>(x, ldx, w, ldwb, gscale, group, ws, M, N, K, kchunk, xsum, Y, ldy, bias, off);
  else if (M <= 16 && ct == 4 && g_nst == 4)
    woq_kernel<T, BITS, 1, 4, GRP, 4><<<grid, 256, 0, st>>>(x, ldx, w, ldwb, gscale, group, ws, M, N, K, kchunk, xsum, Y, ldy, bias, off);
  else if (M <= 16 && ct == 4 && g_nst == 3)
    woq_kernel<T, BITS, 1, 3, GRP, 4><<<grid, 256, 0, st>>>(x, ldx, w, ldwb, gscale, group, ws, M, N, K, kchunk, xsum, Y, ldy, bias, off);
  else if (M <= 16 && ct == 4)
    woq_kernel<T, BITS, 1, 2, GRP, 4><<<grid, 256, 0, st>>>(x, ldx, w, ldwb, gscale, group, ws, M, N, K, kchunk, xsum, Y, ldy, bias, off);
  else if (M <= 16 && g_nst == 2)
    woq_kernel<T, BITS, 1, 2, GRP><<<grid, 256, 0, st>>>(x, ldx, w, ldwb, gscale, group, ws, M, N, K, kchunk, xsum, Y, ldy, bias, off);
  else if (M <= 16 && g_nst == 4)
    woq_kernel<T, BITS, 1, 4, GRP><<<grid, 256, 0, st>>>(x, ldx, w, ldwb, gscale, group, ws, M, N, K, kchunk, xsum, Y, ldy, bias, off);
  else if (M <= 16)
    woq_kernel<T, BITS, 1, 3, GRP><<<grid, 256, 0, st>>>(x, ldx, w, ldwb, gscale, group, ws, M, N, K, kchunk, xsum, Y, ldy, bias, off);
  else
    woq_kernel<T, BITS, 2, 2, GRP><<<grid, 256, 0, st>>>(x, ldx, w, ldwb, gscale, group, ws, M, N, K, kchunk, xsum, Y, ldy, bias, off);
}

}  // namespace woq
}  // namespace pa

// Contract: 1 <= M <= 32; bits 8: K % 64 == 0, bits 4: K % 128 == 0; N % 8 == 0; X rows k-contiguous
// (ldx % 8 == 0, 16-B aligned); Wq [N][ldw_bytes] with ldw_bytes % 16 == 0; group 0 (per-channel
// scale [N]) or 64 / 128 (scale [K / group][N]); dt 1 = bf16, 2 = fp16 activations / output.
PA_API int pa_woq_ok(int M, int N, int K, long long ldx, long long ldw_bytes, int bits, int group, int dt) {
  if (M < 1 || M > 32 || N < 8 || N % 8 || ldx % 8 || ldw_bytes % 16 || (dt != 1 && dt != 2)) return 0;
  if (bits == 8 && K % 64) return 0;
  if (bits == 4 && K % 128) return 0;
  if (bits != 8 && bits != 4) return 0;
  if (group != 0 && group != 64 && group != 128) return 0;
  if (group && K % group) return 0;
  return 1;
}

// A/B knobs: target block count of the K-split plan (default 0 = by output width), register stages
// (2 / 3 / 4) of the M <= 16 kernel (default 2); target < 0 restores the width rule, 0 keeps the
// value, nst <= 0 keeps it.  Returns the previous target.
PA_API int pa_woq_tune(int target_blocks, int nst) {
  const int old = pa::woq::g_target_blocks;
  if (target_blocks > 0) pa::woq::g_target_blocks = target_blocks;
  else if (target_blocks < 0) pa::woq::g_target_blocks = 0;
  if (nst > 0) pa::woq::g_nst = nst;
  return old;
}

// A/B knob: 16-column tiles per wave of the M <= 16 kernel (2 / 4 / 8; 0 = automatic by M); returns
// the previous value
PA_API int pa_woq_set_ct(int ct) {
  const int old = pa::woq::g_ct;
  if (ct == 0 || ct == 2 || ct == 4 || ct == 8) pa::woq::g_ct = ct;
  return old;
}

PA_API int pa_woq_set_fused_finish(int on) {
  const int old = pa::woq::g_fused_finish;
  if (on >= 0) pa::woq::g_fused_finish = on ? 1 : 0;
  return old;
}

PA_API long long pa_woq_ws_floats(int M, int N, int K, int bits) {
  int KS, kc;
  pa::woq::plan(N, K, bits, M, KS, kc);
  return (long long)KS * M * N + (long long)KS * M;  // partials + per-split row sums of X
}

PA_API int pa_woq_gemm(const void* X, const void* Wq, const float* scale, const void* bias, void* Y, float* ws, int M,
                       int N, int K, long long ldx, long long ldw_bytes, long long ldy, int bits, int group, int dt,
                       hipStream_t st) {
  using namespace pa::woq;
  if (!pa_woq_ok(M, N, K, ldx, ldw_bytes, bits, group, dt) || ws == nullptr || scale == nullptr || ldy % 8)
    return (int)hipErrorInvalidValue;
  int KS, kchunk;
  plan(N, K, bits, M, KS, kchunk);
  const bool grp = group != 0;
  float* xsum = ws + (long long)KS * M * N;
  // one K split: the main kernel finishes the tile itself (scale, offset, bias, 16-bit store)
  const bool fused = KS == 1 && g_fused_finish;
  uint16_t* Yf = fused ? (uint16_t*)Y : nullptr;
  const uint16_t* bf = fused ? (const uint16_t*)bias : nullptr;
  // unsigned-code offsets of the per-channel paths (frag_u8: u = q + 128; frag_u4: 128 + q + 8 /
  // 1024 + q + 8)
  const float off = bits == 8 ? (dt == 1 ? 128.f : 1152.f) : (dt == 1 ? 136.f : 1032.f);
#define WOQ_DISPATCH(T)                                                                                        \
  do {                                                                                                         \
    if (bits == 8 && grp) launch<T, 8, true>(X, ldx, Wq, ldw_bytes, scale, group, ws, M, N, K, KS, kchunk, xsum, Yf, ldy, bf, off, st); \
    else if (bits == 8) launch<T, 8, false>(X, ldx, Wq, ldw_bytes, scale, 0, ws, M, N, K, KS, kchunk, xsum, Yf, ldy, bf, off, st);      \
    else if (grp) launch<T, 4, true>(X, ldx, Wq, ldw_bytes, scale, group, ws, M, N, K, KS, kchunk, xsum, Yf, ldy, bf, off, st);         \
    else launch<T, 4, false>(X, ldx, Wq, ldw_bytes, scale, 0, ws, M, N, K, KS, kchunk, xsum, Yf, ldy, bf, off, st);                     \
    if (fused) break;                                                                                          \
    const long long groups = ((long long)M * N + 7) / 8;                                                       \
    woq_finish<T><<<(unsigned)((groups + 255) / 256), 256, 0, st>>>(ws, KS, M, N, grp ? nullptr : scale,       \
                                                                     (const uint16_t*)bias, (uint16_t*)Y, ldy,  \
                                                                     grp ? nullptr : xsum,                      \
                                                                     off);                                      \
  } while (0)
  if (dt == 1) WOQ_DISPATCH(pa::bf16_t);
  else WOQ_DISPATCH(pa::f16_t);
#undef WOQ_DISPATCH
  return (int)hipGetLastError();
}
