// Device code of the hand-written 8-phase MFMA GEMM (included by gemm8.hip — the bf16 training
// GEMMs — and gemm8x.hip — fp16 / batched / fp8 instantiations in their own translation unit so
// they do not perturb the register allocation of the tuned bf16 kernels).
#pragma once
// Hand-written bf16 MFMA GEMM for gfx950, 8-phase ping-pong schedule (the main GEMM of the
// training step: Linear forward, dgrad and weight gradient, the tied LM head).
//
// Reference semantics: paddle/phi/kernels/funcs/blas/blaslt_impl.cu.h (matmul),
// fusion/gpu/fused_gemm_epilogue_kernel.cu (bias epilogue) and
// fusion/gpu/fused_linear_param_grad_add_kernel.cu (W.grad += X^T dY, beta = 1 epilogue).
//
//   C[M,N] = alpha * op(A) @ op(B) (+ beta * C) (+ bias[N])
//   AK: A stored [M][K] (k contiguous) else [K][M];  BK: B stored [N][K] else [K][N].
//
// CDNA4 structure (why it is shaped like this):
//  * 256x256 block tile, K consumed 64 deep, 512 threads = 8 waves as 2 (M) x 4 (N); each wave
//    owns 128x64 of C = 8x4 accumulators of v_mfma_f32_16x16x32_bf16 (128 acc VGPRs).
//  * The two waves that share a SIMD (wave w and w+4) PING-PONG: waves 4-7 start one barrier
//    late, so in every barrier interval one wave of each SIMD runs a 16-MFMA quadrant (256
//    cycles of matrix pipe) while its partner issues the LDS reads / LDS-DMA for its next
//    quadrant.  A K-tile is 8 intervals per wave: L0 M0 L1 M1 L2 M2 L3 M3 (L = load segment,
//    M = 16 MFMAs on one 64x32 quadrant of the wave's 128x64).
//  * Operands are staged HBM -> LDS by global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip),
//    two K-tiles resident (2 x 64 KB).  Each wave group g stages the 128-row A half and the
//    128-col B half with index g; tile t+2 is issued into tile t's buffer as soon as every
//    reader of that half has retired its reads (B after L0 of both groups, A after L2), and
//    retired with a COUNTED vmcnt(8) one K-tile later, so 8-12 barrier intervals of HBM/L2
//    latency hide behind the matrix work.  The DMA is issued from inline asm (hipcc would
//    otherwise drain it with vmcnt(0) at every ds_read).
//  * Every layout is read as it sits in HBM: k-contiguous operands become [128][64] images
//    read with ds_read_b128; m/n-contiguous operands become [64][128] images read with
//    ds_read_b64_tr_b16 (hardware transpose).  Both images are XOR-swizzled on 16-B chunks
//    (the swizzle is folded into the per-lane DMA SOURCE address, the DMA destination being
//    lane-linear) and both read kinds are bank-conflict free (analysis at koff / moff).
//  * Products are computed swapped (mfma(B, A) = C^T fragment) so each lane owns 4
//    consecutive output columns (8-byte stores, 4-wide bias reads).
//  * XCD-aware grouped tile order (blocks b and b+8 share an XCD L2).
#include "common.h"
#include "fp8_util.h"

namespace pa {
namespace g8 {

// Split-K slice (in k) for ``splitk`` slices of K: ceil(K / 64 / splitk) * 64.  Uneven splits are
// allowed when every slice is non-empty and the last one holds >= 2 k-blocks (splitk_uneven_ok);
// the kernels shorten the last slice (nt = min(ksplit, K - kbeg) / BK).
__host__ __device__ inline int ksplit_of(int K, int splitk) {
  const int kb = K / 64;
  return ((kb + splitk - 1) / splitk) * 64;
}
inline bool splitk_uneven_ok(int K, int splitk) {
  if (K % 64 || splitk < 1) return false;
  if (K % (64 * splitk) == 0) return true;  // even slices (any K % 64 == 0 unsplit)
  const int kb = K / 64, q = (kb + splitk - 1) / splitk;
  const int last = kb - (splitk - 1) * q;
  return last >= 2;
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BM = 256, BN = 256, BK = 64;
// A/B switch for the 16-B-wide epilogue of schedule 11 (pa_gemm8_set_wide_epi); read by every
// block, set only between launches.
#ifndef PA_G8_EXTRA_TU
__constant__ int g_wide_epi = 1;
// A/B switch (pa_gemm8_set_nt_store): the wave-staged epilogue's row stores non-temporal
__constant__ int g_nt_store = 0;
#else
static __constant__ int g_wide_epi = 1;  // gemm8x.hip: a private copy (its kernels do not read it)
static __constant__ int g_nt_store = 0;
#endif

constexpr int HALF = 128 * BK * 2;  // one 128-row (or 128-col) half of an operand tile: 16 KB
constexpr int OPB = 2 * HALF;       // 32 KB
constexpr int BUF = 2 * OPB;        // A + B of one K-tile: 64 KB
constexpr int LDS_BYTES = 2 * BUF;  // two K-tiles resident: 128 KB

__device__ __forceinline__ f32x4 mfma(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// Operand-type tags of the kernel templates: bf16_t (default), f16_t (fp16 in, fp16 out) and
// F8<FA, FB> (OCP fp8 operands, 0 = e4m3, 1 = e5m2; bf16 out).  fp8 reuses the bf16 byte images
// unchanged: a 64-element bf16 k-tile row is 128 bytes = 128 fp8 k values, and the two 16-B
// fragments a lane reads for k-halves 0 and 1 (chunks g and g + 4 of the row) concatenate into the
// 32-byte operand of ONE v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales) in place of the two
// bf16 MFMAs — same LDS bytes, same matrix-pipe cycles per tile, twice the FLOPs.  The k order
// inside an MFMA is a permutation applied identically to A and B, so the dot products are exact.
template <int FA, int FB>
struct F8 {
  static constexpr int fa = FA, fb = FB;
};
// int8 operands (signed), int32 accumulation, bf16 out with per-row x per-column dequant scales:
// like fp8, the bf16 byte images are reused unchanged — a 64-element bf16 k-half (64 bytes) is 64
// int8 k values, exactly one v_mfma_i32_16x16x64_i8 per fragment pair (the lane -> byte mapping of
// the 16x16x64 i8 operand equals the 16x16x32 bf16 one; a k permutation shared by A and B leaves
// the dot products exact).  The int32 sums live in the f32x4 accumulator registers as raw bits.
struct I8T {};
template <typename T>
struct is_f8 { static constexpr bool value = false; };
template <int FA, int FB>
struct is_f8<F8<FA, FB>> { static constexpr bool value = true; };
template <typename T>
struct OutT { using type = bf16_t; };
template <>
struct OutT<f16_t> { using type = f16_t; };

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

typedef int i32x4 __attribute__((ext_vector_type(4)));

// accumulator register type per operand tag: int32 sums for int8 (kept as i32x4 through the whole
// loop — carrying them in f32x4 registers through bit casts miscompiles on ROCm 7.2: only element
// 0 of a bit-cast MFMA result survives, tools/probe/i8_mfma_probe.hip)
template <typename T>
struct AccOf { using type = f32x4; };
template <>
struct AccOf<I8T> { using type = i32x4; };

template <typename T, typename A>
__device__ __forceinline__ A mfmaT(s16x8 a, s16x8 b, A c) {
  if constexpr (__is_same(T, I8T))
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, a), __builtin_bit_cast(i32x4, b), c, 0, 0,
                                                 0);
  else if constexpr (__is_same(T, f16_t))
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
  else
    return mfma(a, b, c);
}

// fp8: the two k-half fragments of a lane as one 32-byte scaled-MFMA operand
template <int FA, int FB>
__device__ __forceinline__ f32x4 mfma_f8(s16x8 a0, s16x8 a1, s16x8 b0, s16x8 b1, f32x4 c) {
  const i32x8 a = __builtin_bit_cast(i32x8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12,
                                                                    13, 14, 15));
  const i32x8 b = __builtin_bit_cast(i32x8, __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12,
                                                                    13, 14, 15));
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, FA, FB, 0, 127, 0, 127);
}

// one fp8 step of the swapped product (B fragment first, as mfma(fb, fa) in the bf16 loops)
template <typename T>
__device__ __forceinline__ f32x4 f8_step(s16x8 b0, s16x8 b1, s16x8 a0, s16x8 a1, f32x4 c);
template <int FA, int FB>
struct F8Step {
  static __device__ __forceinline__ f32x4 run(s16x8 b0, s16x8 b1, s16x8 a0, s16x8 a1, f32x4 c) {
    return mfma_f8<FB, FA>(b0, b1, a0, a1, c);
  }
};
template <typename T>
__device__ __forceinline__ f32x4 f8_step(s16x8 b0, s16x8 b1, s16x8 a0, s16x8 a1, f32x4 c) {
  if constexpr (is_f8<T>::value) return F8Step<T::fa, T::fb>::run(b0, b1, a0, a1, c);
  else return c;
}

// K-major half image [128 rows][64 k], 128-B rows: chunk c (0..7) of row r at c ^ ((r >> 1) & 7).
// A ds_read_b128 lane group ({0-3,12-15,20-27} etc.) holds rows {0-3,12-15} of one chunk and rows
// {4-11} of the next (or the mirror); with this XOR the 16 (row, chunk) pairs cover the 16
// distinct 16-B slots of the 256-B bank row: conflict free.
__device__ __forceinline__ int koff(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
// MN-major half image [64 k][128 cols], 256-B rows: chunk c (0..15) of k-row r at c ^ hsw(r).
// A tr-read 32-lane half touches k-rows {8g + q} (g in a pair, q = 0..3, + 4 for the second
// read) at one aligned chunk pair; hsw maps those 8 rows to 8 distinct chunk pairs: conflict free.
__device__ __forceinline__ int hsw(int r) { return ((r & 3) | (((r >> 3) & 1) << 2)) << 1; }
__device__ __forceinline__ int moff(int r, int c) { return r * 256 + ((c ^ hsw(r)) << 4); }

// Fragment of 16 rows (m or n) x 32 k (k-half kh of the 64-deep tile) for lane (g = lane>>4,
// i = lane&15): element j = operand[row0 + i][32 kh + 8 g + j].
template <bool KMAJ>
__device__ __forceinline__ s16x8 frag(const char* img, int row0, int kh, int lane) {
  const int g = lane >> 4;
  if constexpr (KMAJ) {
    return *reinterpret_cast<const s16x8*>(img + koff(row0 + (lane & 15), kh * 4 + g));
  } else {
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int kr = kh * 32 + 8 * g + q;
    const int ch = (row0 >> 3) + (p >> 1);
    const int bi = (p & 1) * 8;
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + moff(kr, ch) + bi));
    const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + moff(kr + 4, ch) + bi));
    return s16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  }
}

// Byte offset (from the operand base, K-tile 0 of this split) of the 16-B source chunk that
// lane `lane` of wave-slot idx (0..15, 1 KB of the half image each) DMAs.  rc0 = first row
// (K-major) / column (MN-major) of the half; rows / columns past lim are clamped (their
// products land in C rows / columns that are never stored).
template <bool KMAJ>
__device__ __forceinline__ unsigned src_off(int idx, int lane, int rc0, int lim, long long ld, int k0) {
  if constexpr (KMAJ) {
    const int row = idx * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const long long r = min(rc0 + row, lim - 1);
    return (unsigned)((r * ld + k0 + c * 8) * 2);
  } else {
    const int row = idx * 4 + (lane >> 4);
    const int c = (lane & 15) ^ hsw(row);
    const long long col = min(rc0 + c * 8, lim - 8);  // lim % 8 == 0 (host check)
    return (unsigned)(((long long)(k0 + row) * ld + col) * 2);
  }
}

// One 16-B-per-lane LDS-DMA: global (saddr base + 32-bit lane offset) -> LDS (M0 base + lane*16).
// Inline asm so hipcc does not count it (it would wait vmcnt(0) before every ds_read); the
// queue is retired by hand with counted vmcnt (wait_vm).
__device__ __forceinline__ void glds(const char* base, unsigned off, unsigned lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(off), "s"(base), "s"(lds_dst)
      : "memory");
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Bijective XCD remap + grouped (GROUP_M tile rows per column sweep) tile order.
__device__ __forceinline__ void tile_coords(int bid, int nwg, int tm, int tn, int& mt, int& nt) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  const int w = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  constexpr int GROUP_M = 8;
  const int per_group = GROUP_M * tn;
  const int gidx = w / per_group;
  const int first_m = gidx * GROUP_M;
  const int gm = min(tm - first_m, GROUP_M);
  const int in = w - gidx * per_group;
  mt = first_m + in % gm;
  nt = in / gm;
}

// Epilogue: lane owns C[mb + 16i + (lane&15)][nb + 16j + 4(lane>>4) + 0..3] (swapped products).
template <int EPI>
__device__ __forceinline__ void epilogue(const f32x4 (&acc)[8][4], uint16_t* __restrict__ C, float* __restrict__ ws,
                                         const uint16_t* __restrict__ bias, int M, int N, long long ldc, float alpha,
                                         float beta, int mb, int nb, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mb + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nb + j * 16 + 4 * g;
      if (n >= N) continue;  // N % 8 == 0: a 4-wide group is all in or all out
      if constexpr (EPI == 1) {
        *reinterpret_cast<f32x4*>(ws + (long long)blockIdx.z * M * N + (long long)m * N + n) = acc[i][j];
      } else if constexpr (EPI == 2) {  // h = alpha*acc + bias: C = gelu_tanh(h), aux = gelu_tanh'(h)
        float h[4] = {acc[i][j][0] * alpha, acc[i][j][1] * alpha, acc[i][j][2] * alpha, acc[i][j][3] * alpha};
        if (bias) {
          float bb[4];
          load_f<bf16_t, 4>(reinterpret_cast<const bf16_t*>(bias + n), bb);
#pragma unroll
          for (int r = 0; r < 4; ++r) h[r] += bb[r];
        }
        const long long o = (long long)m * ldc + n;
        float g[4], d[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) gelu_tanh_fdf(h[r], g[r], d[r]);
        store_f<bf16_t, 4>(reinterpret_cast<bf16_t*>(ws) + o, d);
        store_f<bf16_t, 4>(reinterpret_cast<bf16_t*>(C + o), g);
      } else if constexpr (EPI == 3 || EPI == 4) {  // C = alpha*acc * aux  (aux = the saved gelu_tanh'(h))
        const long long o = (long long)m * ldc + n;
        float d[4];
        load_f<bf16_t, 4>(reinterpret_cast<const bf16_t*>(ws) + o, d);
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * alpha * d[r];
        store_f<bf16_t, 4>(reinterpret_cast<bf16_t*>(C + o), v);
      } else {
        float v[4] = {acc[i][j][0] * alpha, acc[i][j][1] * alpha, acc[i][j][2] * alpha, acc[i][j][3] * alpha};
        uint16_t* dst = C + (long long)m * ldc + n;
        if (beta != 0.f) {
          float o[4];
          load_f<bf16_t, 4>(reinterpret_cast<const bf16_t*>(dst), o);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += beta * o[r];
        }
        if (bias) {
          float bb[4];
          load_f<bf16_t, 4>(reinterpret_cast<const bf16_t*>(bias + n), bb);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += bb[r];
        }
        store_f<bf16_t, 4>(reinterpret_cast<bf16_t*>(dst), v);
      }
    }
  }
  if constexpr (EPI == 5)  // + batch-norm column statistics of the 128-row slab (ws: [2][ceil(M/128)][N])
    wave_col_stats<8, 4>(acc, nullptr, min(128, M - mb), nb, N, ws + (long long)(mb / 128) * N,
                         ws + ((long long)((M + 127) / 128) + mb / 128) * N);
}

// 16-B-wide epilogue (CDNA4 v_permlane16_swap): lanes of 16-lane rows g and g^1 hold adjacent
// 4-column groups of the same output row, so swapping the group-2p data of the upper row with
// the group-(2p+1) data of the lower row gives every lane 8 consecutive columns: 16 stores of
// 16 B per lane (each instruction: 16 rows x 64 contiguous bytes) instead of 32 stores of 8 B
// (16 rows x 32 B) — the K = 2048 GEMMs of the step are epilogue-store-issue bound at the tail
// (cdna_hip_programming T21).  Bias / beta / aux reads become 16-B loads too.
// Diagnostic variants (pa_gemm8_diag only): EPI 10 + e runs epilogue e's arithmetic but skips its
// global stores (a data-dependent never-true guard keeps the math alive) — the epilogue's store
// cost is the time difference to EPI e; EPI 20 stores the same bytes with every store instruction
// covering 1 KiB of consecutive addresses (a block's tile as one 128 KiB run; wrong layout, timing
// only) — what full-line stores would buy over the tile's 16 rows x 64 B per instruction.
template <int EPI_>
__device__ __forceinline__ void epilogue_wide(const f32x4 (&acc)[8][4], uint16_t* __restrict__ C,
                                              float* __restrict__ ws, const uint16_t* __restrict__ bias, int M, int N,
                                              long long ldc, float alpha, float beta, int mb, int nb, int lane) {
  constexpr int EPI = EPI_ % 10;
  constexpr bool NOSTORE = EPI_ >= 10 && EPI_ < 20;
  constexpr bool LINEAR = EPI_ >= 20;  // diagnostic: same bytes, each store 1 KiB contiguous
  const int g = lane >> 4;
  const bool upper = (g & 1) != 0;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int n = nb + (upper ? 16 * (2 * p + 1) + 4 * (g - 1) : 16 * (2 * p) + 4 * g);
    float bb[8];
    if (EPI != 3 && EPI != 4 && bias != nullptr && n < N)
      load_f<bf16_t, 8>(reinterpret_cast<const bf16_t*>(bias + n), bb);
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // EPI 4: column sums of this lane's rows
    // EPI 3: issue all eight 16-B loads of the saved derivative before any use (one memory round
    // trip per p instead of eight serialised ones)
    Pack<bf16_t, 8> hv[8];
    if constexpr (EPI == 3 || EPI == 4) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = mb + i * 16 + (lane & 15);
        if (m < M && n < N)
          hv[i] = *reinterpret_cast<const Pack<bf16_t, 8>*>(reinterpret_cast<const bf16_t*>(ws) + (long long)m * ldc + n);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // inline asm: hipcc (ROCm 7.2) CSEs the four __builtin_amdgcn_permlane16_swap calls of this
        // loop into one (every v[e] came out as v[0]); s_nop 1 = the VALU-write -> permlane hazard
        float lo = acc[i][2 * p][e], hi = acc[i][2 * p + 1][e];
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(lo), "+v"(hi));
        v[e] = lo * alpha;
        v[4 + e] = hi * alpha;
      }
      const int m = mb + i * 16 + (lane & 15);
      if (m >= M || n >= N) continue;
      const long long o = (long long)m * ldc + n;
      if constexpr (EPI == 3 || EPI == 4) {
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] *= (float)hv[i].v[r];
        store_f<bf16_t, 8>(reinterpret_cast<bf16_t*>(C + o), v);
        if constexpr (EPI == 4) {
#pragma unroll
          for (int r = 0; r < 8; ++r) cs[r] += (float)(bf16_t)v[r];  // the value as stored
        }
      } else {
        if (bias != nullptr) {
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] += bb[r];
        }
        if constexpr (EPI == 2) {
          float d[8];
#pragma unroll
          for (int r = 0; r < 8; r += 2) {
            f32x2_t fv, dv;
            gelu_tanh_fdf2(f32x2_t{v[r], v[r + 1]}, fv, dv);
            v[r] = fv.x;
            v[r + 1] = fv.y;
            d[r] = dv.x;
            d[r + 1] = dv.y;
          }
          if (!NOSTORE || d[0] == 1234567.f) store_f<bf16_t, 8>(reinterpret_cast<bf16_t*>(ws) + o, d);
        } else if (beta != 0.f) {
          float old[8];
          load_f<bf16_t, 8>(reinterpret_cast<const bf16_t*>(C + o), old);
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] += beta * old[r];
        }
        if constexpr (LINEAR) {
          const long long lo = (long long)blockIdx.x * 65536 + (threadIdx.x >> 6) * 8192 + p * 4096 + i * 512 + lane * 8;
          store_f<bf16_t, 8>(reinterpret_cast<bf16_t*>(C + lo), v);
        } else if (!NOSTORE || v[0] == 1234567.f) {
          store_f<bf16_t, 8>(reinterpret_cast<bf16_t*>(C + o), v);
        }
      }
    }
    if constexpr (EPI == 4) {
      // bias-gradient fusion: rows of the wave's 128-row slab live in lanes (lane & 15) x i; sum
      // the 16 lanes of this column group and write one partial row per slab (finished by
      // pa_colsum_finish_parts into the bias gradient)
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        cs[r] += __shfl_xor(cs[r], 1);
        cs[r] += __shfl_xor(cs[r], 2);
        cs[r] += __shfl_xor(cs[r], 4);
        cs[r] += __shfl_xor(cs[r], 8);
      }
      if ((lane & 15) == 0 && n < N && mb < M) {
        float* dst = reinterpret_cast<float*>(const_cast<uint16_t*>(bias)) + (long long)(mb / 128) * N + n;
        *reinterpret_cast<float4*>(dst) = make_float4(cs[0], cs[1], cs[2], cs[3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
      }
    }
  }
}

// LDS-staged epilogue (schedule 11): the block's 256 x 256 bf16 output tile is assembled in the
// (then idle) 128 KiB of LDS and written back in whole rows — every store instruction covers two
// rows x 512 contiguous bytes (full 128-B lines) instead of 16 rows x 64 B.  Measured on the
// GPT-3 1.3B shapes: the register-fragment stores cost 8-13 % of a K = 2048 GEMM, the same bytes
// as 1 KiB runs almost nothing (tools/gemm_epi_cost.py EPI 20, profiles/r3s2_gemm_epilogue_cost*).
// Inputs of the epilogue (the saved GELU derivative of EPI 3/4, the old C of beta != 0) come in
// the same way: row-contiguous loads into the LDS tile, fragment reads out of it.
// Tile layout: row r (0..255) at r * 512 B, 16-B chunk c (0..31) at slot c ^ (r & 31): the
// fragment writes / reads (16 rows x one chunk per 16 lanes) and the row reads / writes (one
// row's 32 chunks per 32 lanes) are both bank-conflict free.
__device__ __forceinline__ int stile(int r, int c) { return r * 512 + ((c ^ (r & 31)) << 4); }

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x2 lds_u32x2;

// global [rows of the tile] -> LDS tile.  Wave w moves rows 32w .. 32w + 31, two per instruction.
__device__ __forceinline__ void tile_in(const uint16_t* __restrict__ src, long long ld, int m0, int n0, int M, int N,
                                        lds_char* lds, int wave, int lane) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = wave * 32 + 2 * (8 * h + j) + (lane >> 5), c = lane & 31;
      // clamped, branch-free (rows / chunks past the edge load an in-bounds neighbour that is
      // never stored back; a per-load branch here makes the register allocator spill the
      // accumulators inside the main loop)
      const int m = min(m0 + r, M - 1), n = min(n0 + c * 8, N - 8);
      v[j] = *reinterpret_cast<const u32x4*>(src + (long long)m * ld + n);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = wave * 32 + 2 * (8 * h + j) + (lane >> 5), c = lane & 31;
      *(lds_u32x4*)(lds + stile(r, c)) = v[j];
    }
  }
}

// LDS tile -> global rows (bounds-checked per 16-B chunk: N % 8 == 0).
__device__ __forceinline__ void tile_out(uint16_t* __restrict__ dst, long long ld, int m0, int n0, int M, int N,
                                         const lds_char* lds, int wave, int lane) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = wave * 32 + 2 * (8 * h + j) + (lane >> 5), c = lane & 31;
      v[j] = *(const lds_u32x4*)(lds + stile(r, c));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = wave * 32 + 2 * (8 * h + j) + (lane >> 5), c = lane & 31;
      const int m = m0 + r, n = n0 + c * 8;
      if (m < M && n < N) *reinterpret_cast<u32x4*>(dst + (long long)m * ld + n) = v[j];
    }
  }
}

template <typename OT>
__device__ __forceinline__ u32x4 pack8(const float (&v)[8]) {
  Pack<OT, 8> pk;
#pragma unroll
  for (int r = 0; r < 8; ++r) pk.v[r] = (OT)v[r];
  return __builtin_bit_cast(u32x4, pk);
}

__device__ __forceinline__ u32x4 pack_bf16x8(const float (&v)[8]) {
  Pack<bf16_t, 8> pk;
#pragma unroll
  for (int r = 0; r < 8; ++r) pk.v[r] = (bf16_t)v[r];
  return __builtin_bit_cast(u32x4, pk);
}

template <int EPI>
__device__ __forceinline__ void epilogue_staged(const f32x4 (&acc)[8][4], uint16_t* __restrict__ C,
                                                float* __restrict__ ws, const uint16_t* __restrict__ bias, int M,
                                                int N, long long ldc, float alpha, float beta, int m0, int n0,
                                                int wr, int wc, int lane, lds_char* lds) {
  static_assert(EPI == 0 || EPI == 2 || EPI == 3 || EPI == 4, "staged epilogue: EPI 0/2/3/4");
  // opaque lane id: every address below depends on it, so none of them is hoisted above the main
  // loop (the compiler otherwise precomputes ~80 registers of epilogue addresses there and spills)
  asm volatile("" : "+v"(lane));
  const int wave = wr * 4 + wc;
  const int g = lane >> 4;
  const bool upper = (g & 1) != 0;
  const int mb = m0 + wr * 128, nb = n0 + wc * 64;
  constexpr bool AUX_IN = EPI == 3 || EPI == 4;
  const bool old_in = EPI == 0 && beta != 0.f;
  // (no barrier first: the main loop's closing barriers already order every wave's last fragment
  // reads before this point)
  if (AUX_IN) tile_in(reinterpret_cast<const uint16_t*>(ws), ldc, m0, n0, M, N, lds, wave, lane);
  else if (old_in) tile_in(C, ldc, m0, n0, M, N, lds, wave, lane);
  if (AUX_IN || old_in) __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int n = nb + (upper ? 16 * (2 * p + 1) + 4 * (g - 1) : 16 * (2 * p) + 4 * g);
    const int ch = (n - n0) >> 3;
    float bb[8];
    if (!AUX_IN && bias != nullptr && n < N) load_f<bf16_t, 8>(reinterpret_cast<const bf16_t*>(bias + n), bb);
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float lo = acc[i][2 * p][e], hi = acc[i][2 * p + 1][e];
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(lo), "+v"(hi));
        v[e] = lo * alpha;
        v[4 + e] = hi * alpha;
      }
      const int r = wr * 128 + i * 16 + (lane & 15);
      lds_char* slot = lds + stile(r, ch);
      const bool valid = m0 + r < M && n < N;
      if constexpr (AUX_IN) {
        const Pack<bf16_t, 8> hv = __builtin_bit_cast(Pack<bf16_t, 8>, *(const lds_u32x4*)slot);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= (float)hv.v[e];
        if constexpr (EPI == 4) {
          if (valid) {
#pragma unroll
            for (int e = 0; e < 8; ++e) cs[e] += (float)(bf16_t)v[e];  // the value as stored
          }
        }
      } else {
        if (bias != nullptr) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += bb[e];
        }
        if constexpr (EPI == 2) {
          float d[8];
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            f32x2_t fv, dv;
            gelu_tanh_fdf2(f32x2_t{v[e], v[e + 1]}, fv, dv);
            v[e] = fv.x;
            v[e + 1] = fv.y;
            d[e] = dv.x;
            d[e + 1] = dv.y;
          }
          (void)d;  // gelu'(h) is recomputed from the accumulators after C has left the tile
        } else if (old_in) {
          float old[8];
          const Pack<bf16_t, 8> ov = __builtin_bit_cast(Pack<bf16_t, 8>, *(const lds_u32x4*)slot);
#pragma unroll
          for (int e = 0; e < 8; ++e) old[e] = (float)ov.v[e];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += beta * old[e];
        }
      }
      // in place: this lane is the only reader / writer of its (row, chunk) slots
      *(lds_u32x4*)slot = pack_bf16x8(v);
    }
    if constexpr (EPI == 4) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        cs[e] += __shfl_xor(cs[e], 1);
        cs[e] += __shfl_xor(cs[e], 2);
        cs[e] += __shfl_xor(cs[e], 4);
        cs[e] += __shfl_xor(cs[e], 8);
      }
      if ((lane & 15) == 0 && n < N && mb < M) {
        float* dst = reinterpret_cast<float*>(const_cast<uint16_t*>(bias)) + (long long)(mb / 128) * N + n;
        *reinterpret_cast<float4*>(dst) = make_float4(cs[0], cs[1], cs[2], cs[3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
      }
    }
  }
  __syncthreads();
  tile_out(C, ldc, m0, n0, M, N, lds, wave, lane);
  if constexpr (EPI == 2) {
    // second tile: gelu'(h), recomputed from the accumulators (holding it packed through the C
    // pass would cost 64 registers and spill the main loop)
    __syncthreads();  // every wave has read its C rows out of the tile
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int n = nb + (upper ? 16 * (2 * p + 1) + 4 * (g - 1) : 16 * (2 * p) + 4 * g);
      const int ch = (n - n0) >> 3;
      float bb[8];
      if (bias != nullptr && n < N) load_f<bf16_t, 8>(reinterpret_cast<const bf16_t*>(bias + n), bb);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float lo = acc[i][2 * p][e], hi = acc[i][2 * p + 1][e];
          asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(lo), "+v"(hi));
          v[e] = lo * alpha;
          v[4 + e] = hi * alpha;
        }
        if (bias != nullptr) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += bb[e];
        }
        float d[8];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          f32x2_t fv, dv;
          gelu_tanh_fdf2(f32x2_t{v[e], v[e + 1]}, fv, dv);
          d[e] = dv.x;
          d[e + 1] = dv.y;
        }
        *(lds_u32x4*)(lds + stile(wr * 128 + i * 16 + (lane & 15), ch)) = pack_bf16x8(d);
      }
    }
    __syncthreads();
    tile_out(reinterpret_cast<uint16_t*>(ws), ldc, m0, n0, M, N, lds, wave, lane);
  }
}

// Wave-local staged epilogue (schedule 11): no block barrier.  Each wave owns 16 KiB of the (then
// idle) LDS and its 128 x 64 output slice goes out in two 64-row halves: the fragments of a half
// are written to the wave's region ([64 rows][128 B], 16-B chunk c of row r at c ^ ((r >> 1) & 7):
// conflict-free both ways), read back row-wise and stored as whole 128-B lines (8 rows x 128 B
// per store instruction instead of 16 rows x 64 B).  EPI 2 keeps both outputs of a half in the
// region (C in the first 8 KiB, gelu' in the second); EPI 3/4 and beta != 0 bring their input tile
// in row-wise the same way.  LDS accesses of one wave complete in order, so no waits are needed
// between the writes and the reads of other lanes' rows; wave_barrier keeps the compiler from
// reordering them.
__device__ __forceinline__ int wtile(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int EPI, typename OT = bf16_t>
__device__ __forceinline__ void epilogue_wstaged(const f32x4 (&acc)[8][4], uint16_t* __restrict__ C,
                                                 float* __restrict__ ws, const uint16_t* __restrict__ bias, int M,
                                                 int N, long long ldc, float alpha, float beta, int mb, int nb,
                                                 int lane, lds_char* region) {
  // EPI 6 / 7 / 8: inference activations after the bias (relu / gelu erf / gelu tanh), no aux
  // output — the fc_fuse_pass epilogue of imported programs (static/ir_passes.py fused_linear).
  // EPI 9: EPI 2 with the exact (erf) GELU: C = gelu(h), aux = gelu'(h) = Phi(h) + h phi(h) — the
  // training fc1 of static programs (static/ir_passes.py fused_ffn)
  static_assert(EPI == 0 || EPI == 2 || EPI == 3 || EPI == 4 || EPI == 5 || EPI == 6 || EPI == 7 || EPI == 8 ||
                    EPI == 9,
                "staged epilogue: EPI 0/2/3/4/5/6/7/8/9");
  constexpr bool TWO_OUT = EPI == 2 || EPI == 9;
  const int g = lane >> 4;
  const bool upper = (g & 1) != 0;
  constexpr bool AUX_IN = EPI == 3 || EPI == 4;
  const bool old_in = EPI == 0 && beta != 0.f;
  lds_char* reg_c = region;          // [64][128 B] output half (EPI 2: C)
  lds_char* reg_a = region + 8192;   // EPI 2: gelu' half
  const uint16_t* src_in = AUX_IN ? reinterpret_cast<const uint16_t*>(ws) : C;
  float cs[2][8];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[p][e] = 0.f;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int rb = mb + half * 64;  // first row of this half
    if (AUX_IN || old_in) {
      // input half, row-wise: 8 rows x 128 B per load (clamped at the edges: never stored back)
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = 8 * j + (lane >> 3), c = lane & 7;
        const int m = min(rb + r, M - 1), n = min(nb + c * 8, N - 8);
        v[j] = *reinterpret_cast<const u32x4*>(src_in + (long long)m * ldc + n);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) *(lds_u32x4*)(reg_c + wtile(8 * j + (lane >> 3), lane & 7)) = v[j];
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int n = nb + (upper ? 16 * (2 * p + 1) + 4 * (g - 1) : 16 * (2 * p) + 4 * g);
      const int ch = (n - nb) >> 3;
      float bb[8];
      if (!AUX_IN && bias != nullptr && n < N) load_f<OT, 8>(reinterpret_cast<const OT*>(bias + n), bb);
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = half * 4 + ii;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float lo = acc[i][2 * p][e], hi = acc[i][2 * p + 1][e];
          asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(lo), "+v"(hi));
          v[e] = lo * alpha;
          v[4 + e] = hi * alpha;
        }
        const int r = ii * 16 + (lane & 15);  // row within the half
        lds_char* slot = reg_c + wtile(r, ch);
        if constexpr (AUX_IN) {
          const Pack<bf16_t, 8> hv = __builtin_bit_cast(Pack<bf16_t, 8>, *(const lds_u32x4*)slot);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= (float)hv.v[e];
          if constexpr (EPI == 4) {
            if (rb + r < M && n < N) {
#pragma unroll
              for (int e = 0; e < 8; ++e) cs[p][e] += (float)(bf16_t)v[e];  // the value as stored
            }
          }
        } else {
          if (bias != nullptr) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += bb[e];
          }
          if constexpr (EPI == 2) {
            float d[8];
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              f32x2_t fv, dv;
              gelu_tanh_fdf2(f32x2_t{v[e], v[e + 1]}, fv, dv);
              v[e] = fv.x;
              v[e + 1] = fv.y;
              d[e] = dv.x;
              d[e + 1] = dv.y;
            }
            *(lds_u32x4*)(reg_a + wtile(r, ch)) = pack_bf16x8(d);
          } else if constexpr (EPI == 9) {
            float d[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) gelu_erf_fdf(v[e], v[e], d[e]);
            *(lds_u32x4*)(reg_a + wtile(r, ch)) = pack_bf16x8(d);
          } else if constexpr (EPI == 6) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
          } else if constexpr (EPI == 7) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              float dd;
              gelu_erf_fdf(v[e], v[e], dd);
              (void)dd;
            }
          } else if constexpr (EPI == 8) {
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              f32x2_t fv, dv;
              gelu_tanh_fdf2(f32x2_t{v[e], v[e + 1]}, fv, dv);
              v[e] = fv.x;
              v[e + 1] = fv.y;
            }
          } else if (old_in) {
            const Pack<OT, 8> ov = __builtin_bit_cast(Pack<OT, 8>, *(const lds_u32x4*)slot);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += beta * (float)ov.v[e];
          }
        }
        *(lds_u32x4*)slot = pack8<OT>(v);  // in place: only this lane touches this slot
      }
    }
    __builtin_amdgcn_wave_barrier();
    // the half, row-wise: 8 rows x 128 B per store
#pragma unroll
    for (int o = 0; o < (TWO_OUT ? 2 : 1); ++o) {
      const lds_char* rg = o == 0 ? reg_c : reg_a;
      uint16_t* dst = o == 0 ? C : reinterpret_cast<uint16_t*>(ws);
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = *(const lds_u32x4*)(rg + wtile(8 * j + (lane >> 3), lane & 7));
      const bool nt = g_nt_store != 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = rb + 8 * j + (lane >> 3), n = nb + (lane & 7) * 8;
        if (m < M && n < N) {
          u32x4* ptr = reinterpret_cast<u32x4*>(dst + (long long)m * ldc + n);
          if (nt)
            __builtin_nontemporal_store(v[j], ptr);
          else
            *ptr = v[j];
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next half overwrites the region after these reads
  }
  if constexpr (EPI == 5)  // EPI 0 + batch-norm column statistics of the slab (ws: [2][ceil(M/128)][N])
    wave_col_stats<8, 4>(acc, nullptr, min(128, M - mb), nb, N, ws + (long long)(mb / 128) * N,
                         ws + ((long long)((M + 127) / 128) + mb / 128) * N);
  if constexpr (EPI == 4) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int n = nb + (upper ? 16 * (2 * p + 1) + 4 * (g - 1) : 16 * (2 * p) + 4 * g);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        cs[p][e] += __shfl_xor(cs[p][e], 1);
        cs[p][e] += __shfl_xor(cs[p][e], 2);
        cs[p][e] += __shfl_xor(cs[p][e], 4);
        cs[p][e] += __shfl_xor(cs[p][e], 8);
      }
      if ((lane & 15) == 0 && n < N && mb < M) {
        float* dst = reinterpret_cast<float*>(const_cast<uint16_t*>(bias)) + (long long)(mb / 128) * N + n;
        *reinterpret_cast<float4*>(dst) = make_float4(cs[p][0], cs[p][1], cs[p][2], cs[p][3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(cs[p][4], cs[p][5], cs[p][6], cs[p][7]);
      }
    }
  }
}

// Quarter-tile wave-staged epilogue of the persistent schedule 12 (EPI 0): the operand LDS is busy
// with the next work item's first K-tiles, so each wave stages its 128 x 64 slice through its own
// 4 KiB of the spare LDS above them (32 rows per round, four rounds) and stores whole 128-B lines
// as epilogue_wstaged does — the store tail overlaps the next item's staging DMA instead of a
// block exit + prologue.
template <typename OT = bf16_t>
__device__ __forceinline__ void epilogue_wq(const f32x4 (&acc)[8][4], uint16_t* __restrict__ C,
                                            const uint16_t* __restrict__ bias, int M, int N, long long ldc,
                                            float alpha, float beta, int mb, int nb, int lane, lds_char* region) {
  const int g = lane >> 4;
  const bool upper = (g & 1) != 0;
  const bool old_in = beta != 0.f;
#pragma unroll
  for (int qr = 0; qr < 4; ++qr) {
    const int rb = mb + qr * 32;  // first row of this quarter
    if (old_in) {
      u32x4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 8 * j + (lane >> 3), c = lane & 7;
        const int m = min(rb + r, M - 1), n = min(nb + c * 8, N - 8);
        v[j] = *reinterpret_cast<const u32x4*>(C + (long long)m * ldc + n);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) *(lds_u32x4*)(region + wtile(8 * j + (lane >> 3), lane & 7)) = v[j];
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int n = nb + (upper ? 16 * (2 * p + 1) + 4 * (g - 1) : 16 * (2 * p) + 4 * g);
      const int ch = (n - nb) >> 3;
      float bb[8];
      if (bias != nullptr && n < N) load_f<OT, 8>(reinterpret_cast<const OT*>(bias + n), bb);
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = qr * 2 + ii;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float lo = acc[i][2 * p][e], hi = acc[i][2 * p + 1][e];
          asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(lo), "+v"(hi));
          v[e] = lo * alpha;
          v[4 + e] = hi * alpha;
        }
        const int r = ii * 16 + (lane & 15);
        lds_char* slot = region + wtile(r, ch);
        if (bias != nullptr) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += bb[e];
        }
        if (old_in) {
          const Pack<OT, 8> ov = __builtin_bit_cast(Pack<OT, 8>, *(const lds_u32x4*)slot);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += beta * (float)ov.v[e];
        }
        *(lds_u32x4*)slot = pack8<OT>(v);
      }
    }
    __builtin_amdgcn_wave_barrier();
    u32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = *(const lds_u32x4*)(region + wtile(8 * j + (lane >> 3), lane & 7));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = rb + 8 * j + (lane >> 3), n = nb + (lane & 7) * 8;
      if (m < M && n < N) *reinterpret_cast<u32x4*>(C + (long long)m * ldc + n) = v[j];
    }
    __builtin_amdgcn_wave_barrier();  // the next quarter overwrites the region after these reads
  }
}

// same, with an explicit split-K slab index (persistent kernels: blockIdx.z is not the slice)
template <int EPI>
__device__ __forceinline__ void epilogue_z(const f32x4 (&acc)[8][4], uint16_t* __restrict__ C,
                                           float* __restrict__ ws, const uint16_t* __restrict__ bias, int M, int N,
                                           long long ldc, float alpha, float beta, int mb, int nb, int lane, int z) {
  if constexpr (EPI == 1) {
    const int g = lane >> 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mb + i * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nb + j * 16 + 4 * g;
        if (n >= N) continue;
        *reinterpret_cast<f32x4*>(ws + (long long)z * M * N + (long long)m * N + n) = acc[i][j];
      }
    }
  } else {
    epilogue<EPI>(acc, C, ws, bias, M, N, ldc, alpha, beta, mb, nb, lane);
  }
}

// EPI 0: bf16 C = alpha*acc (+ beta*C) (+ bias);  EPI 1: raw fp32 split-K slab (ws[z][M][N]);
// EPI 2: fc1 forward, h = alpha*acc + bias, C = gelu_tanh(h) and aux (= ws, bf16, ldc) = gelu_tanh'(h);
// EPI 3: fc2 dgrad, C = alpha*acc * aux (the saved derivative: the epilogue of a 1-block-per-CU
// GEMM is exposed time, so the tanh work is done once, in the forward): the bias_act kernels of
// the MLP (reference fusion/gpu/fused_gemm_epilogue_kernel.cu, fused_gemm_epilogue_grad) vanish.
template <bool AK, bool BKM, int EPI>
__global__ __launch_bounds__(512, 1) void gemm8_kernel(const char* __restrict__ A, const char* __restrict__ B,
                                                       uint16_t* __restrict__ C, float* __restrict__ ws,
                                                       const uint16_t* __restrict__ bias, int M, int N, int K,
                                                       long long lda, long long ldb, long long ldc, float alpha,
                                                       float beta, int ksplit) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int wr = wave >> 2, wc = wave & 3, wq = wave & 3;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  int mt, ntile;
  tile_coords(blockIdx.x, tm * tn, tm, tn, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int kbeg = blockIdx.z * ksplit;
  const int nt = min(ksplit, K - kbeg) / BK;  // uneven split-K: the last slice is shorter

  // this wave's DMA slots: 4 KB of A half `wr` and 4 KB of B half `wr` per K-tile
  unsigned offA[4], offB[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    offA[u] = src_off<AK>(wq * 4 + u, lane, m0 + wr * 128, M, lda, kbeg);
    offB[u] = src_off<BKM>(wq * 4 + u, lane, n0 + wr * 128, N, ldb, kbeg);
  }
  const long long kstepA = AK ? BK * 2 : (long long)BK * lda * 2;
  const long long kstepB = BKM ? BK * 2 : (long long)BK * ldb * 2;
  const unsigned lds0 = (unsigned)(size_t)(lds_void*)smem;
  const unsigned dstA = lds0 + wr * HALF + wq * 4096;
  const unsigned dstB = lds0 + OPB + wr * HALF + wq * 4096;

  auto stageA = [&](int t) {
    const char* base = A + (long long)t * kstepA;
    const unsigned d = dstA + (t & 1) * BUF;
#pragma unroll
    for (int u = 0; u < 4; ++u) glds(base, offA[u], d + u * 1024);
  };
  auto stageB = [&](int t) {
    const char* base = B + (long long)t * kstepB;
    const unsigned d = dstB + (t & 1) * BUF;
#pragma unroll
    for (int u = 0; u < 4; ++u) glds(base, offB[u], d + u * 1024);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: K-tiles 0 and 1 in flight; retire tile 0 (all waves) before the first reads
  stageB(0);
  stageA(0);
  if (nt > 1) {
    stageB(1);
    stageA(1);
    wait_vm<8>();
  } else {
    wait_vm<0>();
  }
  bar();
  if (wr == 1) bar();  // stagger: waves 4-7 run one interval behind waves 0-3

  const int bcol = (wc & 1) * 64;  // this wave's columns inside its B half
  s16x8 fa[4][2], fb0[2][2], fb1[2][2];
  for (int t = 0; t < nt; ++t) {
    const char* ia = smem + (t & 1) * BUF + wr * HALF;
    const char* ib = smem + (t & 1) * BUF + OPB + (wc >> 1) * HALF;
    const bool more = t + 2 < nt;
    // L0: A rows 0-63 of the wave, all 64 B columns
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        fb0[j][kh] = frag<BKM>(ib, bcol + j * 16, kh, lane);
        fb1[j][kh] = frag<BKM>(ib, bcol + 32 + j * 16, kh, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i][kh] = frag<AK>(ia, i * 16, kh, lane);
    }
    bar();
    // M0: quadrant (A 0-63, B 0-31)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(fb0[j][kh], fa[i][kh], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // L1: group 1 restages B half 1 (every reader retired its L0 reads two barriers ago)
    if (wr == 1 && more) stageB(t + 2);
    bar();
    // M1: quadrant (A 0-63, B 32-63)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][2 + j] = mfma(fb1[j][kh], fa[i][kh], acc[i][2 + j]);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // L2: A rows 64-127; group 0 restages B half 0
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i][kh] = frag<AK>(ia, 64 + i * 16, kh, lane);
    if (wr == 0 && more) stageB(t + 2);
    bar();
    // M2: quadrant (A 64-127, B 32-63)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[4 + i][2 + j] = mfma(fb1[j][kh], fa[i][kh], acc[4 + i][2 + j]);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // L3: restage this group's A half; group 1 retires K-tile t+1 before group 0 reads it
    if (more) stageA(t + 2);
    if (wr == 1) {
      if (more) wait_vm<8>();
      else wait_vm<0>();
    }
    bar();
    // M3: quadrant (A 64-127, B 0-31); group 0 retires K-tile t+1
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[4 + i][j] = mfma(fb0[j][kh], fa[i][kh], acc[4 + i][j]);
    __builtin_amdgcn_s_setprio(0);
    if (wr == 0) {
      if (more) wait_vm<8>();
      else wait_vm<0>();
    }
    bar();
  }
  if (wr == 0) bar();  // match group 1's barrier count

  epilogue<EPI>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0 + wr * 128, n0 + wc * 64, lane);
}


// ---------------------------------------------------------------------------------------------
// Schedule 9: the same ping-pong, but every K-tile image is split by K HALF (k 0-31 / 32-63)
// instead of by row half, and a phase is (A 64-row sub-tile) x (all 64 B columns) x (one k half):
//   L0: A sub0 k0 (4 frags) + B k0 (4 frags)   M0: acc[0..3][*]
//   L1: A sub1 k0                              M1: acc[4..7][*]
//   L2: A sub0 k1 + B k1                       M2: acc[0..3][*]
//   L3: A sub1 k1                              M3: acc[4..7][*]
// so every load segment carries either 8 fragment reads or 4 reads + 4 LDS-DMA (schedule 8's
// first segment carried 16 reads: 64 KB per CU in one 256-cycle interval = the LDS peak), only
// 32 fragment VGPRs are live, and a k-half image is free for re-staging as soon as its last
// readers retire (B k0 after L0, A k0 after L1, ...).  Waves 0-3 stage A (k0 in L3, k1 in L1 of
// the next tile), waves 4-7 stage B (k0 in L1, k1 in L3); every stage is retired with a counted
// vmcnt 9-12 barrier intervals after issue.  Images: K-major [256][32] (64-B rows),
// MN-major [32][256] (512-B rows), both swizzled conflict free for their read kind.
constexpr int KH = 256 * 32 * 2;  // one k-half image: 16 KB
// K-major [256 rows][32 k]: chunk ch (0..3) of row r at ch ^ (((r >> 3) & 1) << 1)
__device__ __forceinline__ int k9off(int r, int ch) { return r * 64 + ((ch ^ (((r >> 3) & 1) << 1)) << 4); }
// MN-major [32 k][256 cols]: chunk ch (0..31) of k-row r at ch ^ hsw(r)
__device__ __forceinline__ int m9off(int r, int ch) { return r * 512 + ((ch ^ hsw(r)) << 4); }

template <bool KMAJ>
__device__ __forceinline__ s16x8 frag9(const char* img, int row0, int lane) {
  const int g = lane >> 4;
  if constexpr (KMAJ) {
    return *reinterpret_cast<const s16x8*>(img + k9off(row0 + (lane & 15), g));
  } else {
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int kr = 8 * g + q;
    const int ch = (row0 >> 3) + (p >> 1);
    const int bi = (p & 1) * 8;
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + m9off(kr, ch) + bi));
    const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + m9off(kr + 4, ch) + bi));
    return s16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  }
}

// source byte offset (k-half 0 of K-tile 0 of this split) for lane `lane` of wave-slot idx (0..15)
template <bool KMAJ>
__device__ __forceinline__ unsigned src9(int idx, int lane, int rc0, int lim, long long ld, int k0) {
  if constexpr (KMAJ) {
    const int row = idx * 16 + (lane >> 2);
    const int ch = (lane & 3) ^ (((row >> 3) & 1) << 1);
    const long long r = min(rc0 + row, lim - 1);
    return (unsigned)((r * ld + k0 + ch * 8) * 2);
  } else {
    const int row = idx * 2 + (lane >> 5);
    const int ch = (lane & 31) ^ hsw(row);
    const long long col = min(rc0 + ch * 8, lim - 8);
    return (unsigned)(((long long)(k0 + row) * ld + col) * 2);
  }
}

__device__ __forceinline__ void wait_vm_n(int n) {  // n in {0, 4, 8, 12}, wave-uniform
  if (n >= 12) wait_vm<12>();
  else if (n >= 8) wait_vm<8>();
  else if (n >= 4) wait_vm<4>();
  else wait_vm<0>();
}

// Second problem of a grouped launch (GRP): blocks [tiles of problem 0, +tiles of problem 1) take
// it.  Same K, layout, alpha / beta and epilogue as problem 0.  Used to run two weight gradients
// whose tile counts add up to one full round of the chip (the GPT QKV and out-projection weight
// gradients: 192 + 64 = 256 tiles) as one launch instead of a partly idle round plus a split-K.
struct Prob {
  const char* A;
  const char* B;
  uint16_t* C;
  int M, N;
  long long lda, ldb, ldc;
};

// T: operand type tag (bf16_t / f16_t); BAT: blockIdx.y indexes a batch of problems at byte
// strides sA / sB and element stride sC (stride 0 = a broadcast operand).
template <bool AK, bool BKM, int EPI, bool GRP = false, typename T = bf16_t, bool BAT = false>
__global__ __launch_bounds__(512, 1) void gemm9_kernel(const char* __restrict__ A, const char* __restrict__ B,
                                                       uint16_t* __restrict__ C, float* __restrict__ ws,
                                                       const uint16_t* __restrict__ bias, int M, int N, int K,
                                                       long long lda, long long ldb, long long ldc, float alpha,
                                                       float beta, int ksplit, Prob p1 = Prob{}, long long sA = 0,
                                                       long long sB = 0, long long sC = 0) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3, wq = wave & 3;
  int bid = blockIdx.x;
  if constexpr (GRP) {
    const int t0 = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (bid >= t0) {  // block-uniform: this block computes a tile of problem 1
      A = p1.A, B = p1.B, C = p1.C, M = p1.M, N = p1.N, lda = p1.lda, ldb = p1.ldb, ldc = p1.ldc;
      bid -= t0;
    }
  }
  if constexpr (BAT) {
    A += (long long)blockIdx.y * sA;
    B += (long long)blockIdx.y * sB;
    C += (long long)blockIdx.y * sC;
  }
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  int mt, ntile;
  tile_coords(bid, tm * tn, tm, tn, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int kbeg = blockIdx.z * ksplit;
  const int nt = min(ksplit, K - kbeg) / BK;  // uneven split-K: the last slice is shorter

  // waves 0-3 stage A, waves 4-7 stage B: 4 x 1 KB of a k-half image each per stage
  const bool isA = wr == 0;
  const bool km = isA ? AK : BKM;
  const long long ld = isA ? lda : ldb;
  const char* opnd = isA ? A : B;
  unsigned off[4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
    off[u] = isA ? src9<AK>(wq * 4 + u, lane, m0, M, lda, kbeg) : src9<BKM>(wq * 4 + u, lane, n0, N, ldb, kbeg);
  const long long kstep = km ? BK * 2 : (long long)BK * ld * 2;    // bytes per K-tile
  const long long khstep = km ? 32 * 2 : (long long)32 * ld * 2;   // bytes to k-half 1
  const unsigned lds0 = (unsigned)(size_t)(lds_void*)smem;
  // buffer layout: [A k0][A k1][B k0][B k1]
  const unsigned dst0 = lds0 + (isA ? 0 : 2 * KH) + wq * 4096;
  auto stage = [&](int t, int kh) {
    const char* base = opnd + (long long)t * kstep + kh * khstep;
    const unsigned d = dst0 + (t & 1) * BUF + kh * KH;
#pragma unroll
    for (int u = 0; u < 4; ++u) glds(base, off[u], d + u * 1024);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue, in the steady-state issue order (A: k0(t+2) in L3(t), k1(t+1) in L1(t);
  // B: k0(t+2) in L1(t), k1(t+2) in L3(t))
  const int more1 = nt > 1;
  if (isA) {
    stage(0, 0);
    stage(0, 1);
    if (more1) stage(1, 0);
    wait_vm_n(4 + 4 * more1);  // A k0(0) landed
  } else {
    stage(0, 0);
    stage(0, 1);
    if (more1) {
      stage(1, 0);
      stage(1, 1);
    }
    wait_vm_n(4 + 8 * more1);  // B k0(0) landed
  }
  bar();
  if (wr == 1) bar();  // stagger: waves 4-7 run one interval behind waves 0-3

  s16x8 fa[4], fb[4];
  const int arow = wr * 128, bcol = wc * 64;
  for (int t = 0; t < nt; ++t) {
    const char* buf = smem + (t & 1) * BUF;
    const int m1 = t + 1 < nt, m2 = t + 2 < nt;
    // L0: A sub0 k0, B k0
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = frag9<BKM>(buf + 2 * KH, bcol + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag9<AK>(buf, arow + i * 16, lane);
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfmaT<T>(fb[j], fa[i], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // L1: A sub1 k0; A waves stage A k1(t+1), B waves stage B k0(t+2); B waves retire B k1(t)
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag9<AK>(buf, arow + 64 + i * 16, lane);
    if (isA) {
      if (m1) stage(t + 1, 1);
    } else {
      if (m2) stage(t + 2, 0);
      wait_vm_n(8 * m1 + 4 * m2);
    }
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[4 + i][j] = mfmaT<T>(fb[j], fa[i], acc[4 + i][j]);
    __builtin_amdgcn_s_setprio(0);
    if (isA) wait_vm_n(8 * m1);  // A k1(t) landed
    bar();
    // L2: A sub0 k1, B k1
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = frag9<BKM>(buf + 3 * KH, bcol + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag9<AK>(buf + KH, arow + i * 16, lane);
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfmaT<T>(fb[j], fa[i], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // L3: A sub1 k1; A waves stage A k0(t+2), B waves stage B k1(t+2); B waves retire B k0(t+1)
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag9<AK>(buf + KH, arow + 64 + i * 16, lane);
    if (m2) stage(t + 2, isA ? 0 : 1);
    if (!isA) wait_vm_n(4 * m1 + 8 * m2);
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[4 + i][j] = mfmaT<T>(fb[j], fa[i], acc[4 + i][j]);
    __builtin_amdgcn_s_setprio(0);
    if (isA) wait_vm_n(4 * m1 + 4 * m2);  // A k0(t+1) landed
    bar();
  }
  if (wr == 0) bar();  // match waves 4-7's barrier count

  // (the 16-B epilogue measured neutral here: weight gradients, K = 16384, beta = 1)
  if constexpr (EPI >= 200)  // wave-local staged epilogue (its own instantiation)
    epilogue_wstaged<EPI - 200, typename OutT<T>::type>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0 + wr * 128, n0 + wc * 64, lane,
                                (lds_char*)smem + (wr * 4 + wc) * 16384);
  else
    epilogue<EPI>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0 + wr * 128, n0 + wc * 64, lane);
}


// fp8-output form of the wave-staged epilogue (fp8 feed-forward blocks, ops/fp8.py _FP8FFN):
//   EPI 9 (fc1: h = s*acc + bias, out = gelu(h), aux = gelu'(h)) with out quantised to e4m3;
//   EPI 4 (fc2 data gradient: out = s*acc * aux, column partial sums of out into ``bias``) with
//   out quantised to e5m2.
// The bf16 ``out`` is never written: the tile goes out as fp8 q [M][ldq] AND its transpose
// qt [N][M] (the two images an fp8 Linear needs), quantised with the delayed scale *scale_p
// (pa_fp8_scale_prep ran the cast's bookkeeping), and the tile's amax is folded into *amax_p —
// the separate cast + transpose pass over the bf16 tensor disappears.  Per half (64 rows x 64
// columns) the fp8 bytes are staged as a [64][64 B] LDS tile, stored row-wise (16 B per lane)
// and gathered column-wise for qt (16 B per lane).  Contract: M % 16 == 0, N % 16 == 0.
template <int EPI, int FMT>
__device__ __forceinline__ void epilogue_wstaged_q(const f32x4 (&acc)[8][4], uint8_t* __restrict__ q,
                                                   float* __restrict__ ws, const uint16_t* __restrict__ bias, int M,
                                                   int N, long long ldq, float alpha, uint8_t* __restrict__ qt,
                                                   const float* __restrict__ scale_p, float* __restrict__ amax_p,
                                                   int mb, int nb, int lane, lds_char* region) {
  static_assert(EPI == 9 || EPI == 4, "fp8-output staged epilogue: EPI 9 / 4");
  constexpr bool AUX_IN = EPI == 4;
  const int g = lane >> 4;
  const bool upper = (g & 1) != 0;
  lds_char* reg_c = region;         // EPI 4: aux input half;  EPI 9: the fp8 tile
  lds_char* reg_a = region + 8192;  // EPI 9: gelu' half;        EPI 4: the fp8 tile
  lds_char* tq = AUX_IN ? reg_a : reg_c;
  const float sc = scale_p[0];
  float am = 0.f;
  float cs[2][8];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[p][e] = 0.f;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int rb = mb + half * 64;
    if (AUX_IN) {
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = 8 * j + (lane >> 3), c = lane & 7;
        const int m = min(rb + r, M - 1), n = min(nb + c * 8, N - 8);
        v[j] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint16_t*>(ws) + (long long)m * ldq + n);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) *(lds_u32x4*)(reg_c + wtile(8 * j + (lane >> 3), lane & 7)) = v[j];
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int n = nb + (upper ? 16 * (2 * p + 1) + 4 * (g - 1) : 16 * (2 * p) + 4 * g);
      const int ch = (n - nb) >> 3;
      float bb[8];
      if (!AUX_IN && bias != nullptr && n < N) load_f<bf16_t, 8>(reinterpret_cast<const bf16_t*>(bias + n), bb);
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = half * 4 + ii;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float lo = acc[i][2 * p][e], hi = acc[i][2 * p + 1][e];
          asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(lo), "+v"(hi));
          v[e] = lo * alpha;
          v[4 + e] = hi * alpha;
        }
        const int r = ii * 16 + (lane & 15);
        const bool ok = rb + r < M && n < N;
        if constexpr (AUX_IN) {
          const Pack<bf16_t, 8> hv = __builtin_bit_cast(Pack<bf16_t, 8>, *(const lds_u32x4*)(reg_c + wtile(r, ch)));
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= (float)hv.v[e];
          if (ok) {
#pragma unroll
            for (int e = 0; e < 8; ++e) cs[p][e] += v[e];
          }
        } else {
          if (bias != nullptr) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += bb[e];
          }
          float d[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) gelu_erf_fdf(v[e], v[e], d[e]);
          *(lds_u32x4*)(reg_a + wtile(r, ch)) = pack_bf16x8(d);
        }
        if (ok) {
#pragma unroll
          for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(v[e]));
        }
        const uint32_t w0 = f8::cvt2<FMT>(v[0] * sc, v[1] * sc) | (f8::cvt2<FMT>(v[2] * sc, v[3] * sc) << 16);
        const uint32_t w1 = f8::cvt2<FMT>(v[4] * sc, v[5] * sc) | (f8::cvt2<FMT>(v[6] * sc, v[7] * sc) << 16);
        *(lds_u32x2*)(tq + r * 64 + ch * 8) = u32x2{w0, w1};
      }
    }
    __builtin_amdgcn_wave_barrier();
    if constexpr (!AUX_IN) {  // the gelu' half, row-wise (as the bf16 epilogue stores it)
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = *(const lds_u32x4*)(reg_a + wtile(8 * j + (lane >> 3), lane & 7));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = rb + 8 * j + (lane >> 3), n = nb + (lane & 7) * 8;
        if (m < M && n < N) *reinterpret_cast<u32x4*>(reinterpret_cast<uint16_t*>(ws) + (long long)m * ldq + n) = v[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // q rows: 64 rows x 64 B, 16 B per lane
      const int idx = lane + 64 * j, r = idx >> 2, c16 = idx & 3;
      const u32x4 v = *(const lds_u32x4*)(tq + r * 64 + c16 * 16);
      const int m = rb + r, n = nb + c16 * 16;
      if (m < M && n < N) *reinterpret_cast<u32x4*>(q + (long long)m * ldq + n) = v;
    }
    {  // qt rows: lane = (column group of 4, 16-row group): 16 dword reads, a 16x4 byte transpose,
       // 4 x 16-B stores of the columns' row segments
      const int cg = lane >> 2, m16 = lane & 3;
      uint32_t rw[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        rw[i] = *(const __attribute__((address_space(3))) uint32_t*)(tq + (m16 * 16 + i) * 64 + 4 * cg);
      const int m = rb + m16 * 16;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t o[4];
#pragma unroll
        for (int kq = 0; kq < 4; ++kq)
          o[kq] = ((rw[4 * kq] >> (8 * j)) & 0xFFu) | (((rw[4 * kq + 1] >> (8 * j)) & 0xFFu) << 8) |
                  (((rw[4 * kq + 2] >> (8 * j)) & 0xFFu) << 16) | (((rw[4 * kq + 3] >> (8 * j)) & 0xFFu) << 24);
        const int n = nb + 4 * cg + j;
        if (n < N && m < M) *reinterpret_cast<u32x4*>(qt + (long long)n * M + m) = u32x4{o[0], o[1], o[2], o[3]};
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next half overwrites the LDS tiles after these reads
  }
  am = wave_max(am);
  if (lane == 0) f8::atomic_max_pos(amax_p, am);
  if constexpr (AUX_IN) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int n = nb + (upper ? 16 * (2 * p + 1) + 4 * (g - 1) : 16 * (2 * p) + 4 * g);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        cs[p][e] += __shfl_xor(cs[p][e], 1);
        cs[p][e] += __shfl_xor(cs[p][e], 2);
        cs[p][e] += __shfl_xor(cs[p][e], 4);
        cs[p][e] += __shfl_xor(cs[p][e], 8);
      }
      if ((lane & 15) == 0 && n < N && mb < M) {
        float* dst = reinterpret_cast<float*>(const_cast<uint16_t*>(bias)) + (long long)(mb / 128) * N + n;
        *reinterpret_cast<float4*>(dst) = make_float4(cs[p][0], cs[p][1], cs[p][2], cs[p][3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(cs[p][4], cs[p][5], cs[p][6], cs[p][7]);
      }
    }
  }
}


// epilogue dispatch of schedule 11 (shared by the float and the int8 accumulator forms)
template <int EPI, typename T>
__device__ __forceinline__ void gemm11_epilogue(const f32x4 (&acc)[8][4], uint16_t* __restrict__ C,
                                                float* __restrict__ ws, const uint16_t* __restrict__ bias, int M, int N,
                                                long long ldc, float alpha, float beta, int m0, int n0, int wr, int wc,
                                                int lane, char* smem, long long x0 = 0, long long x1 = 0,
                                                long long x2 = 0) {
  if constexpr (EPI == 210 || EPI == 211)  // fp8-output epilogues: x0 = qt, x1 = scale, x2 = amax slot
    epilogue_wstaged_q<EPI == 210 ? 9 : 4, EPI == 210 ? 0 : 1>(
        acc, reinterpret_cast<uint8_t*>(C), ws, bias, M, N, ldc, alpha, reinterpret_cast<uint8_t*>(x0),
        reinterpret_cast<const float*>(x1), reinterpret_cast<float*>(x2), m0 + wr * 128, n0 + wc * 64, lane,
        (lds_char*)smem + (wr * 4 + wc) * 16384);
  else if constexpr (EPI == 1)
    epilogue<EPI>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0 + wr * 128, n0 + wc * 64, lane);
  else if constexpr (EPI >= 200)  // wave-local staged epilogue of EPI - 200 (its own instantiation)
    epilogue_wstaged<EPI - 200, typename OutT<T>::type>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0 + wr * 128,
                                                        n0 + wc * 64, lane, (lds_char*)smem + (wr * 4 + wc) * 16384);
  else if constexpr (EPI >= 100)  // block-staged epilogue of EPI - 100 (its own instantiation)
    epilogue_staged<EPI - 100>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0, n0, wr, wc, lane, (lds_char*)smem);
  else if constexpr (EPI == 5)  // batch-norm statistics: the register epilogue carries them
    epilogue<EPI>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0 + wr * 128, n0 + wc * 64, lane);
  else if constexpr (EPI == 4)
    epilogue_wide<EPI>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0 + wr * 128, n0 + wc * 64, lane);
  else if (g_wide_epi)
    epilogue_wide<EPI>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0 + wr * 128, n0 + wc * 64, lane);
  else
    epilogue<EPI>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0 + wr * 128, n0 + wc * 64, lane);
}


// ---------------------------------------------------------------------------------------------
// Schedule 11: schedule 8's images (row halves, full 128-B lines for k-contiguous operands) with
// 32 MFMAs per segment instead of 16, halving the barriers per K-tile (4 per wave):
//   L0: A sub0 (4 frags x 2 k halves) + B (4 frags x 2 k halves)   M0: acc[0..3][*]  (32 MFMA)
//   L1: A sub1                                                      M1: acc[4..7][*]  (32 MFMA)
// Staging (tile t in buffer t&1): waves 0-3 issue A half 0 + B half 0 of tile t+1 in L0(t) and
// retire them (vmcnt) at the end of M1(t); waves 4-7 issue A half 1 of tile t+1 in L0(t) and
// B half 1 of tile t+2 in L1(t), retiring B half 1 of t+1 before the barrier that opens L0(t+1)
// of waves 0-3 and A half 1 of t+1 at the end of their M1(t).
// T: operand type tag (bf16_t / f16_t / F8<FA, FB>: fp8 takes K, lda, ldb in units of 2 bytes,
// i.e. the byte counts / 2, and the device dequant scales sa, sb); BAT: blockIdx.y indexes a batch
// of problems (byte strides sA / sB, element stride sC).
template <bool AK, bool BKM, int EPI, typename T = bf16_t, bool BAT = false>
__global__ __launch_bounds__(512, 1) void gemm11_kernel(const char* __restrict__ A, const char* __restrict__ B,
                                                        uint16_t* __restrict__ C, float* __restrict__ ws,
                                                        const uint16_t* __restrict__ bias, int M, int N, int K,
                                                        long long lda, long long ldb, long long ldc, float alpha,
                                                        float beta, int ksplit, long long sA = 0, long long sB = 0,
                                                        long long sC = 0, const float* __restrict__ sa = nullptr,
                                                        const float* __restrict__ sb = nullptr) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3, wq = wave & 3;
  if constexpr (BAT) {
    A += (long long)blockIdx.y * sA;
    B += (long long)blockIdx.y * sB;
    C += (long long)blockIdx.y * sC;
  }
  if constexpr (is_f8<T>::value) {  // device-resident per-tensor dequant scales (no host sync)
    if (sa) alpha *= sa[0];
    if (sb) alpha *= sb[0];
  }
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  int mt, ntile;
  tile_coords(blockIdx.x, tm * tn, tm, tn, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int kbeg = blockIdx.z * ksplit;
  const int nt = min(ksplit, K - kbeg) / BK;  // uneven split-K: the last slice is shorter

  unsigned offA[4], offB[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    offA[u] = src_off<AK>(wq * 4 + u, lane, m0 + wr * 128, M, lda, kbeg);
    offB[u] = src_off<BKM>(wq * 4 + u, lane, n0 + wr * 128, N, ldb, kbeg);
  }
  const long long kstepA = AK ? BK * 2 : (long long)BK * lda * 2;
  const long long kstepB = BKM ? BK * 2 : (long long)BK * ldb * 2;
  const unsigned lds0 = (unsigned)(size_t)(lds_void*)smem;
  const unsigned dstA = lds0 + wr * HALF + wq * 4096;
  const unsigned dstB = lds0 + OPB + wr * HALF + wq * 4096;
  auto stageA = [&](int t) {
    const char* base = A + (long long)t * kstepA;
    const unsigned d = dstA + (t & 1) * BUF;
#pragma unroll
    for (int u = 0; u < 4; ++u) glds(base, offA[u], d + u * 1024);
  };
  auto stageB = [&](int t) {
    const char* base = B + (long long)t * kstepB;
    const unsigned d = dstB + (t & 1) * BUF;
#pragma unroll
    for (int u = 0; u < 4; ++u) glds(base, offB[u], d + u * 1024);
  };

  typename AccOf<T>::type acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = typename AccOf<T>::type{0, 0, 0, 0};

  // prologue in the steady-state issue order
  if (wr == 0) {
    stageA(0);
    stageB(0);
    wait_vm<0>();
  } else {
    stageB(0);
    stageA(0);
    if (nt > 1) {
      stageB(1);
      wait_vm<4>();
    } else {
      wait_vm<0>();
    }
  }
  bar();
  if (wr == 1) bar();  // stagger: waves 4-7 run one interval behind waves 0-3

  const int bcol = (wc & 1) * 64;
  s16x8 fa[4][2], fb[4][2];
  for (int t = 0; t < nt; ++t) {
    const char* ia = smem + (t & 1) * BUF + wr * HALF;
    const char* ib = smem + (t & 1) * BUF + OPB + (wc >> 1) * HALF;
    const int m1 = t + 1 < nt, m2 = t + 2 < nt;
    // L0
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j][kh] = frag<BKM>(ib, bcol + j * 16, kh, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i][kh] = frag<AK>(ia, i * 16, kh, lane);
    }
    if (m1) {
      stageA(t + 1);
      if (wr == 0) stageB(t + 1);
    }
    bar();
    // M0
    __builtin_amdgcn_s_setprio(1);
    if constexpr (is_f8<T>::value) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f8_step<T>(fb[j][0], fb[j][1], fa[i][0], fa[i][1], acc[i][j]);
    } else {
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfmaT<T>(fb[j][kh], fa[i][kh], acc[i][j]);
    }
    __builtin_amdgcn_s_setprio(0);
    bar();
    // L1
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i][kh] = frag<AK>(ia, 64 + i * 16, kh, lane);
    if (wr == 1) {
      if (m2) stageB(t + 2);
      // B half 1 of tile t+1 (issued in L1(t-1)) must land before L0(t+1) of waves 0-3
      if (m2) wait_vm<8>();
      else if (m1) wait_vm<4>();
      else wait_vm<0>();
    }
    bar();
    // M1
    __builtin_amdgcn_s_setprio(1);
    if constexpr (is_f8<T>::value) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[4 + i][j] = f8_step<T>(fb[j][0], fb[j][1], fa[i][0], fa[i][1], acc[4 + i][j]);
    } else {
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[4 + i][j] = mfmaT<T>(fb[j][kh], fa[i][kh], acc[4 + i][j]);
    }
    __builtin_amdgcn_s_setprio(0);
    if (wr == 0) wait_vm<0>();  // A half 0 + B half 0 of tile t+1
    else if (m2) wait_vm<4>();  // A half 1 of tile t+1 (B half 1 of t+2 stays in flight)
    else wait_vm<0>();
    bar();
  }
  if (wr == 0) bar();

  if constexpr (__is_same(T, I8T)) {
    // int32 sums -> fp32 with the dequant scales: sa = per-row (token) scales [M], sb = per-column
    // (output channel) scales [N]; lane owns C[mb + 16i + (lane & 15)][nb + 16j + 4(lane >> 4) + r]
    const int mb = m0 + wr * 128, nb = n0 + wc * 64;
    float cs[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[j][r] = sb ? sb[min(nb + 16 * j + 4 * (lane >> 4) + r, N - 1)] : 1.f;
    f32x4 accf[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float rs = sa ? sa[min(mb + 16 * i + (lane & 15), M - 1)] : 1.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) accf[i][j][r] = (float)acc[i][j][r] * rs * cs[j][r];
    }
    gemm11_epilogue<EPI, T>(accf, C, ws, bias, M, N, ldc, alpha, beta, m0, n0, wr, wc, lane, smem, sA, sB, sC);
  } else {
    gemm11_epilogue<EPI, T>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0, n0, wr, wc, lane, smem, sA, sB, sC);
  }
}



// ---------------------------------------------------------------------------------------------
// Schedule 12: schedule 11 made PERSISTENT.  A grid of at most 256 blocks (one per CU) walks its
// work items (tile x split-K slice) as ONE continuous stream of K-tiles: the staging of item j+1's
// first K-tiles is issued during item j's last K-tiles exactly as within an item, so the pipeline
// never drains between tiles and the epilogue of item j (after its last M1) runs while the next
// item's operands are already in flight — no per-tile prologue latency, no block launch.
// Items are dealt per XCD (blocks b = x mod 8 share an XCD): each XCD owns a contiguous chunk of
// the grouped tile order and its 32 blocks walk it 32 tiles at a time, so concurrently running
// tiles share A row-panels / B column-panels in that XCD's L2.
__device__ __forceinline__ void item_coords(int item, int splitk, int tm, int tn, int ksplit, int& m0, int& n0,
                                            int& kb, int& z) {
  z = item % splitk;
  const int tile = item / splitk;
  constexpr int GROUP_M = 8;
  const int per_group = GROUP_M * tn;
  const int gidx = tile / per_group;
  const int first_m = gidx * GROUP_M;
  const int gm = min(tm - first_m, GROUP_M);
  const int in = tile - gidx * per_group;
  m0 = (first_m + in % gm) * BM;
  n0 = (in / gm) * BN;
  kb = z * ksplit;
}

// EPI 300: EPI 0 with the quarter-tile wave-staged epilogue (epilogue_wq) in the 32 KiB of LDS above
// the operand buffers (its own instantiation: 160 KiB of LDS)
template <bool AK, bool BKM, int EPI>
__global__ __launch_bounds__(512, 1) void gemm12_kernel(const char* __restrict__ A, const char* __restrict__ B,
                                                        uint16_t* __restrict__ C, float* __restrict__ ws,
                                                        const uint16_t* __restrict__ bias, int M, int N, int K,
                                                        long long lda, long long ldb, long long ldc, float alpha,
                                                        float beta, int ksplit, int splitk) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES + (EPI == 300 ? 32768 : 0)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3, wq = wave & 3;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  const int nt = ksplit / BK;
  // this block's items: XCD x = b & 7 owns a contiguous chunk, its blocks stride through it
  const int nitems = tm * tn * splitk;
  const int G = gridDim.x, bpx = G >> 3, x = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int q = nitems >> 3, r = nitems & 7;
  const int cstart = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  const int clen = q + (x < r ? 1 : 0);
  const int nmine = clen > slot ? (clen - slot + bpx - 1) / bpx : 0;
  const int E = nmine * nt;  // K-tiles in this block's stream
  if (E == 0) return;
  auto item_of = [&](int j) { return cstart + slot + j * bpx; };

  const long long kstepA = AK ? BK * 2 : (long long)BK * lda * 2;
  const long long kstepB = BKM ? BK * 2 : (long long)BK * ldb * 2;
  const unsigned lds0 = (unsigned)(size_t)(lds_void*)smem;
  const unsigned dstA = lds0 + wr * HALF + wq * 4096;
  const unsigned dstB = lds0 + OPB + wr * HALF + wq * 4096;

  // staging streams (wave-uniform cursors): which item / K-tile the next stage of each operand
  // targets, and the per-lane source offsets of that item (recomputed when the item changes)
  int ja = 0, ka = 0, jb = 0, kbt = 0, ea = 0, eb = 0;
  int jaoff = -1, jboff = -1;
  unsigned offA[4], offB[4];
  auto stageA = [&]() {
    if (ja != jaoff) {
      int m0, n0, kb, z;
      item_coords(item_of(ja), splitk, tm, tn, ksplit, m0, n0, kb, z);
#pragma unroll
      for (int u = 0; u < 4; ++u) offA[u] = src_off<AK>(wq * 4 + u, lane, m0 + wr * 128, M, lda, kb);
      jaoff = ja;
    }
    const char* base = A + (long long)ka * kstepA;
    const unsigned d = dstA + (ea & 1) * BUF;
#pragma unroll
    for (int u = 0; u < 4; ++u) glds(base, offA[u], d + u * 1024);
    ++ea;
    if (++ka == nt) { ka = 0; ++ja; }
  };
  auto stageB = [&]() {
    if (jb != jboff) {
      int m0, n0, kb, z;
      item_coords(item_of(jb), splitk, tm, tn, ksplit, m0, n0, kb, z);
#pragma unroll
      for (int u = 0; u < 4; ++u) offB[u] = src_off<BKM>(wq * 4 + u, lane, n0 + wr * 128, N, ldb, kb);
      jboff = jb;
    }
    const char* base = B + (long long)kbt * kstepB;
    const unsigned d = dstB + (eb & 1) * BUF;
#pragma unroll
    for (int u = 0; u < 4; ++u) glds(base, offB[u], d + u * 1024);
    ++eb;
    if (++kbt == nt) { kbt = 0; ++jb; }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (wr == 0) {
    stageA();
    stageB();
    wait_vm<0>();
  } else {
    stageB();
    stageA();
    if (E > 1) {
      stageB();
      wait_vm<4>();
    } else {
      wait_vm<0>();
    }
  }
  bar();
  if (wr == 1) bar();

  const int bcol = (wc & 1) * 64;
  s16x8 fa[4][2], fb[4][2];
  int j = 0, kt = 0;
  for (int e = 0; e < E; ++e) {
    const char* ia = smem + (e & 1) * BUF + wr * HALF;
    const char* ib = smem + (e & 1) * BUF + OPB + (wc >> 1) * HALF;
    const int m1 = e + 1 < E, m2 = e + 2 < E;
    // L0
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) fb[jj][kh] = frag<BKM>(ib, bcol + jj * 16, kh, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i][kh] = frag<AK>(ia, i * 16, kh, lane);
    }
    if (m1) {
      stageA();
      if (wr == 0) stageB();
    }
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[i][jj] = mfma(fb[jj][kh], fa[i][kh], acc[i][jj]);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // L1
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i][kh] = frag<AK>(ia, 64 + i * 16, kh, lane);
    if (wr == 1) {
      if (m2) stageB();
      // B half 1 of era e+1 must land before L0(e+1) of waves 0-3 (after an epilogue its stores
      // are older than that DMA and are waited for as well: correct, they had two intervals)
      if (m2) wait_vm<8>();
      else if (m1) wait_vm<4>();
      else wait_vm<0>();
    }
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[4 + i][jj] = mfma(fb[jj][kh], fa[i][kh], acc[4 + i][jj]);
    __builtin_amdgcn_s_setprio(0);
    if (wr == 0) wait_vm<0>();
    else if (m2) wait_vm<4>();
    else wait_vm<0>();
    bar();
    if (++kt == nt) {  // item j complete: epilogue from registers, then a fresh accumulator
      int m0, n0, kb, z;
      item_coords(item_of(j), splitk, tm, tn, ksplit, m0, n0, kb, z);
      if constexpr (EPI == 300)
        epilogue_wq(acc, C, bias, M, N, ldc, alpha, beta, m0 + wr * 128, n0 + wc * 64, lane,
                    (lds_char*)smem + LDS_BYTES + wave * 4096);
      else if constexpr (EPI == 1)
        epilogue_z<EPI>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0 + wr * 128, n0 + wc * 64, lane, z);
      else if (g_wide_epi)
        epilogue_wide<EPI>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0 + wr * 128, n0 + wc * 64, lane);
      else
        epilogue<EPI>(acc, C, ws, bias, M, N, ldc, alpha, beta, m0 + wr * 128, n0 + wc * 64, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
      kt = 0;
      ++j;
    }
  }
  if (wr == 0) bar();
}


}  // namespace g8
}  // namespace pa
