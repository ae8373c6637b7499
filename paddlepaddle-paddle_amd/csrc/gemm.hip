// Hand-written bf16 MFMA GEMM for gfx950 (CDNA4) with fused epilogues and split-K.
//
// Reference semantics: paddle/phi/kernels/funcs/blas/blas_impl.cu.h (GEMM), fusion/gpu/
// fused_gemm_epilogue_kernel.cu (bias epilogue), fused_linear_param_grad_add_kernel.cu (weight
// gradient accumulated in place: C += A^T B).
//
//   C[M,N] = alpha * op(A) @ op(B)  (+ beta * C)  (+ bias[N])
//   op(A): transA = 0 → A stored [M][K] (k contiguous); 1 → A stored [K][M] (m contiguous)
//   op(B): transB = 0 → B stored [K][N] (n contiguous); 1 → B stored [N][K] (k contiguous)
//
// CDNA4 design (not a translation of a CUDA tiling):
//  * 256x256x64 block tile, 512 threads = 8 waves laid out 2(M) x 4(N); each wave owns a
//    128x64 output tile = 8x4 v_mfma_f32_16x16x32_bf16 accumulators (128 acc registers).
//  * Staging is global_load_lds (16 B per lane, LDS-DMA, no VGPR round trip) into a ring of
//    4 LDS slots (32-deep K sub-tiles, 4 x (16 KB A + 16 KB B) = 128 KB of the 160 KB LDS);
//    the DMA runs 3 sub-tiles ahead and stays in flight across the per-step barrier (counted
//    vmcnt + raw s_barrier), so HBM/L2 latency hides behind matrix work.
//  * Every operand layout is staged exactly as it sits in HBM (no transposes in memory):
//    k-contiguous operands become [256 rows][64 k] images read with ds_read_b128;
//    m/n-contiguous operands become [64 k][256 cols] images read with ds_read_b64_tr_b16
//    (the hardware transposed LDS read), so the weight-gradient GEMM (A^T B, both operands
//    k-strided) runs at the same rate as the forward.
//  * LDS images are XOR-swizzled on 16-byte chunks; because the LDS-DMA destination is
//    lane-linear the swizzle is applied to the per-lane SOURCE address and undone on the read.
//    Both read kinds are bank-conflict free (see swz_* below).
//  * Products are computed swapped (mfma(B, A) = C^T fragment) so each lane owns 4
//    consecutive output COLUMNS: the epilogue writes 8-byte vectors and reads bias 4-wide.
//  * XCD-aware tile order: the 8 XCDs each get a contiguous chunk of the (grouped) tile order,
//    so blocks that share A row-panels / B column-panels share an L2.
//  * Split-K (gridDim.z slices) writes fp32 slabs; pa_gemm_splitk_reduce folds them with the
//    beta/bias epilogue (used when the output has too few 256x256 tiles to fill 256 CUs, e.g.
//    the 2048x2048 weight gradient with K = 16k tokens).
#include "common.h"

namespace pa {
namespace gemm {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BM = 256, BN = 256, BK = 32;
// K is consumed in 32-deep sub-tiles through a ring of NSLOT LDS slots; the DMA for sub-tile
// s + NSLOT is issued while sub-tile s is multiplied, and each step retires only the sub-tile
// the NEXT step reads with a counted vmcnt, so up to two sub-tiles stay in flight across every
// barrier (a plain __syncthreads() would drain them all: vmcnt(0)).
constexpr int NSLOT = 4;
constexpr int OP_BYTES = 256 * BK * 2;                // one operand image per slot: 16 KB
constexpr int SLOT_BYTES = 2 * OP_BYTES;              // A + B
constexpr int LDS_BYTES = NSLOT * SLOT_BYTES;         // 128 KB

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ f32x4 mfma(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// ---- LDS image addressing ------------------------------------------------------------------
// K-major image ([256 rows][32 k], 64-B rows): chunk ch (0..3) of row r lives at chunk
// ch ^ (((r >> 3) & 1) << 1).  ds_read_b128 services a wave in four 16-lane groups
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32): each group mixes rows of two k-chunks, and
// with this XOR every group's 16 (row, chunk) pairs land on 16 distinct 16-B bank slots.
__device__ __forceinline__ int kimg_off(int row, int ch) { return row * 64 + ((ch ^ (((row >> 3) & 1) << 1)) << 4); }
// MN-major image ([32 k][256 cols], 512-B rows): chunk ch (0..31) of k-row r lives at chunk
// ch ^ f(r), f(r) = 2 * ((r & 3) | ((r >> 3) & 1) << 2).  A tr-read 32-lane half touches k-rows
// {8g + q} for g in a pair, q = 0..3 — eight distinct even f values, each row reading an aligned
// chunk pair → 16 distinct slots: conflict free.
__device__ __forceinline__ int swz_mn(int r) { return ((r & 3) | (((r >> 3) & 1) << 2)) << 1; }
__device__ __forceinline__ int mimg_off(int row, int ch) { return row * 512 + ((ch ^ swz_mn(row)) << 4); }

// Fragment of 16 rows/cols x 32 k for lane (g = lane>>4, i = lane&15):
// element j = operand[row0 + i][8g + j].
template <bool KMAJOR>
__device__ __forceinline__ s16x8 ld_frag(const char* img, int row0, int lane) {
  const int g = lane >> 4;
  if constexpr (KMAJOR) {
    const int r = row0 + (lane & 15);
    return *reinterpret_cast<const s16x8*>(img + kimg_off(r, g));
  } else {
    // lane 4q+p of each 16-lane group addresses k-row (8g + q) [+4], columns row0+4p..+3
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int kr = 8 * g + q;
    const int ch = (row0 >> 3) + (p >> 1);
    const int bi = (p & 1) * 8;
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + mimg_off(kr, ch) + bi));
    const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + mimg_off(kr + 4, ch) + bi));
    s16x8 v;
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
    return v;
  }
}

// Per-thread staging source for one operand: OP_BYTES / (NT * 16) x 16-B LDS-DMA per sub-tile.
// Chunk c = i*NT + tid.  K-major: row = c >> 2, chunk c & 3.  MN-major: k-row = c >> 5,
// chunk c & 31.  The source chunk is pre-swizzled so the lane-linear DMA image is the XOR image.
template <int NT>
struct Src {
  static constexpr int N = OP_BYTES / (NT * 16);
  const uint16_t* p[N];
  long long kstep;  // elements to advance per sub-tile
};

template <bool KMAJOR, int NT>
__device__ __forceinline__ Src<NT> make_src(const uint16_t* base, long long ld, int rc0, int rc_lim, int k0, int tid) {
  Src<NT> s;
#pragma unroll
  for (int i = 0; i < Src<NT>::N; ++i) {
    const int c = i * NT + tid;
    if constexpr (KMAJOR) {
      const int row = c >> 2;
      const int lch = (c & 3) ^ (((row >> 3) & 1) << 1);
      const int grow = min(rc0 + row, rc_lim - 1);  // clamp ragged rows (their results are never stored)
      s.p[i] = base + (long long)grow * ld + k0 + lch * 8;
    } else {
      const int row = c >> 5;
      const int lch = (c & 31) ^ swz_mn(row);
      const int gcol = min(rc0 + lch * 8, rc_lim - 8);  // rc_lim % 8 == 0 (checked on the host)
      s.p[i] = base + (long long)(k0 + row) * ld + gcol;
    }
  }
  s.kstep = KMAJOR ? BK : (long long)BK * ld;
  return s;
}

// LDS-DMA issued from inline asm: hipcc treats a __builtin_amdgcn_global_load_lds as a pending
// write to the one LDS array and would put vmcnt(0) before every ds_read (draining the ring);
// here the DMA queue is counted by hand (wait_barrier), so the compiler must not see it.
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

template <int NT>
__device__ __forceinline__ void stage(const Src<NT>& s, char* img, int t, int wave) {
  const unsigned base = (unsigned)(size_t)(lds_void*)img;
#pragma unroll
  for (int i = 0; i < Src<NT>::N; ++i) {
    // wave-uniform LDS destination: lanes land at base + lane*16 (lane-linear DMA)
    const unsigned dst = __builtin_amdgcn_readfirstlane(base + (i * NT + wave * 64) * 16);
    glds16(s.p[i] + t * s.kstep, dst);
  }
}

// retire all but the youngest n sub-tiles of LDS-DMA, then a raw barrier (no vmcnt(0) fence).
// The DMA count is inline asm (hipcc does not see the DMA); the LDS-read drain is the builtin
// so hipcc's own scoreboard knows every ds_read has retired and adds no lgkmcnt(0) later.
template <int PER_SLOT>
__device__ __forceinline__ void wait_barrier(int n_inflight) {
  if (n_inflight >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER_SLOT) : "memory");
  else if (n_inflight == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_SLOT) : "memory");
  else if (n_inflight == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_SLOT) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt/expcnt unconstrained
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Bijective XCD remap (blocks b ≡ x mod 8 share an XCD) followed by a grouped tile order
// (GROUP_M tile-rows per column sweep) so consecutive work on one XCD shares panels in its L2.
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

// Waves: 2 (M) x WN (N).  WN = 4: 8 waves, 128x64 per wave (2 waves per SIMD, 32 accumulator
// tiles).  WN = 2: 4 waves, 128x128 per wave (one wave per SIMD, 64 accumulator tiles that live
// in the AGPR half of the 512-entry register file, half the LDS bytes per MFMA).
// EPI: 0 = bf16 out (alpha, beta*C, bias);  1 = fp32 split-K slab out (raw acc)
template <bool AK, bool BK_, int EPI, int WN, int NS = NSLOT>
__global__ __launch_bounds__(128 * WN, 1) void gemm_kernel(const uint16_t* __restrict__ A,
                                                           const uint16_t* __restrict__ B, uint16_t* __restrict__ C,
                                                           float* __restrict__ ws, const uint16_t* __restrict__ bias,
                                                           int M, int N, int K, long long lda, long long ldb,
                                                           long long ldc, float alpha, float beta, int ksplit) {
  constexpr int NT = 128 * WN;
  constexpr int FM = 8, FN = 16 / WN;  // 16x16 fragments per wave along M / N
  constexpr int PER_SLOT = 2 * Src<NT>::N;
  __shared__ __attribute__((aligned(1024))) char smem[NS * SLOT_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  int mt, ntile;
  tile_coords(blockIdx.x, tm * tn, tm, tn, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int kbeg = blockIdx.z * ksplit;
  const int ns = ksplit / BK;  // even: K % 64 == 0

  const Src<NT> sa = make_src<AK, NT>(A, lda, m0, M, kbeg, tid);
  const Src<NT> sb = make_src<BK_, NT>(B, ldb, n0, N, kbeg, tid);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Register double-buffered fragments: step s multiplies sub-tile s from registers while its
  // ds_reads fetch sub-tile s+1, so no step starts on an LDS-latency bubble.  The DMA runs
  // NSLOT sub-tiles ahead into the slot of sub-tile s (read during step s-1, before the last
  // barrier); each step retires sub-tile s+2 (read during step s+1).
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (s < ns) {
      stage<NT>(sa, smem + s * SLOT_BYTES, s, wave);
      stage<NT>(sb, smem + s * SLOT_BYTES + OP_BYTES, s, wave);
    }
  }
  wait_barrier<PER_SLOT>(max(min(ns, NS) - 2, 0));  // sub-tiles 0 and 1 landed
  s16x8 fa[2][FM], fb[2][FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) fb[0][j] = ld_frag<BK_>(smem + OP_BYTES, wc * (16 * FN) + j * 16, lane);
#pragma unroll
  for (int i = 0; i < FM; ++i) fa[0][i] = ld_frag<AK>(smem, wr * 128 + i * 16, lane);
  // Two sub-steps per trip, fragment sets alternate without copies.  The prefetch reads are
  // unconditional (past the last sub-tile they read a stale slot, unused) so hipcc sees no merge
  // point that would force lgkmcnt(0) before the MFMAs.
  int slot = 0;  // ring slot of sub-tile ss (wave-uniform, wrapped incrementally)
  for (int s = 0; s < ns; s += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int ss = s + u;
      const int nslot = slot + 1 == NS ? 0 : slot + 1;
      if (ss + NS < ns) {
        stage<NT>(sa, smem + slot * SLOT_BYTES, ss + NS, wave);
        stage<NT>(sb, smem + slot * SLOT_BYTES + OP_BYTES, ss + NS, wave);
      }
      const char* ia = smem + nslot * SLOT_BYTES;
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[u ^ 1][j] = ld_frag<BK_>(ia + OP_BYTES, wc * (16 * FN) + j * 16, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[u ^ 1][i] = ld_frag<AK>(ia, wr * 128 + i * 16, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma(fb[u][j], fa[u][i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      wait_barrier<PER_SLOT>(max(min(ns - 1, ss + NS) - (ss + 2), 0));
      slot = nslot;
    }
  }

  // epilogue: swapped product → lane owns C[m = m0 + wr*128 + 16i + (lane&15)][n = n0 + wc*16FN + 16j + 4(lane>>4) + r]
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wr * 128 + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wc * (16 * FN) + j * 16 + 4 * g;
      if (n >= N) continue;  // N % 4 == 0 (host check) → a 4-wide group is all in or all out
      if constexpr (EPI == 1) {
        float* dst = ws + (long long)blockIdx.z * M * N + (long long)m * N + n;
        *reinterpret_cast<f32x4*>(dst) = acc[i][j];
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
}

// ============================================================================ FP8 (OCP)
// C[M,N] (bf16) = alpha * A[M,K] @ B[N,K]^T (+ beta*C) (+ bias), A/B in OCP e4m3 / e5m2 with
// per-tensor dequant scales (device scalars) folded into alpha.  Both operands k-contiguous
// (the "TN" layout of an fp8 Linear: activations [tokens][in], weight [out][in]).
// v_mfma_scale_f32_16x16x128_f8f6f4 with unit E8M0 block scales (127 = 2^0) runs fp8 at twice
// the bf16 MFMA rate.  Tile 256x256 x 128 k-bytes per sub-tile, 8 waves 2(M)x4(N), two LDS
// slots (2 x (32 KB + 32 KB)), the next sub-tile's DMA in flight during the current MFMAs.
// Fragment: lane (g = lane>>4, i = lane&15) holds 32 k-bytes of row i — 16-byte chunks g and
// g+4 of the 128-byte row (the same k bijection for A and B, so the sum is unchanged); the image
// is swizzled chunk ^ ((row >> 1) & 7), conflict free for both ds_read_b128 of a fragment.
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int F8_BKB = 128;                       // k-bytes per sub-tile
constexpr int F8_OP = 256 * F8_BKB;               // 32 KB
constexpr int F8_SLOT = 2 * F8_OP;
constexpr int F8_DMA = F8_OP / (512 * 16);        // 4 per operand per thread

__device__ __forceinline__ int f8_off(int row, int ch) { return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4); }

__device__ __forceinline__ i32x8 f8_frag(const char* img, int row0, int lane) {
  const int r = row0 + (lane & 15), g = lane >> 4;
  const i32x4 lo = *reinterpret_cast<const i32x4*>(img + f8_off(r, g));
  const i32x4 hi = *reinterpret_cast<const i32x4*>(img + f8_off(r, g + 4));
  return i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int FA, int FB>
__device__ __forceinline__ f32x4 mfma_f8(i32x8 a, i32x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, FA, FB, 0, 127, 0, 127);
}

struct F8Src {
  const uint8_t* p[F8_DMA];
};

__device__ __forceinline__ F8Src f8_src(const uint8_t* base, long long ld, int r0, int lim, int tid) {
  F8Src s;
#pragma unroll
  for (int i = 0; i < F8_DMA; ++i) {
    const int c = i * 512 + tid;
    const int row = c >> 3;
    const int lch = (c & 7) ^ ((row >> 1) & 7);
    s.p[i] = base + (long long)min(r0 + row, lim - 1) * ld + lch * 16;
  }
  return s;
}

__device__ __forceinline__ void f8_stage(const F8Src& s, char* img, int t, int wave) {
  const unsigned base = (unsigned)(size_t)(lds_void*)img;
#pragma unroll
  for (int i = 0; i < F8_DMA; ++i) {
    const unsigned dst = __builtin_amdgcn_readfirstlane(base + (i * 512 + wave * 64) * 16);
    glds16(s.p[i] + (long long)t * F8_BKB, dst);
  }
}

template <int FA, int FB>
__global__ __launch_bounds__(512, 1) void gemm_fp8_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                          uint16_t* __restrict__ C, const uint16_t* __restrict__ bias,
                                                          int M, int N, int K, long long lda, long long ldb,
                                                          long long ldc, float alpha, float beta,
                                                          const float* __restrict__ scale_a,
                                                          const float* __restrict__ scale_b) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * F8_SLOT];
  // device-resident per-tensor dequant scales (no host sync to read them)
  if (scale_a) alpha *= scale_a[0];
  if (scale_b) alpha *= scale_b[0];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  int mt, ntile;
  tile_coords(blockIdx.x, tm * tn, tm, tn, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int ns = K / F8_BKB;
  const F8Src sa = f8_src(A, lda, m0, M, tid);
  const F8Src sb = f8_src(B, ldb, n0, N, tid);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  f8_stage(sa, smem, 0, wave);
  f8_stage(sb, smem + F8_OP, 0, wave);
  wait_barrier<2 * F8_DMA>(0);
  if (ns > 1) {
    f8_stage(sa, smem + F8_SLOT, 1, wave);
    f8_stage(sb, smem + F8_SLOT + F8_OP, 1, wave);
  }
  for (int s = 0; s < ns; ++s) {
    const char* ia = smem + (s & 1) * F8_SLOT;
    const char* ib = ia + F8_OP;
    i32x8 bf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = f8_frag(ib, wc * 64 + j * 16, lane);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      i32x8 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = f8_frag(ia, wr * 128 + (h * 4 + i) * 16, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h * 4 + i][j] = mfma_f8<FB, FA>(bf[j], af[i], acc[h * 4 + i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    // sub-tile s+1 landed (nothing else in flight) and every wave is done with slot s&1 ...
    wait_barrier<2 * F8_DMA>(0);
    // ... so sub-tile s+2 can be staged into it
    if (s + 2 < ns) {
      f8_stage(sa, smem + (s & 1) * F8_SLOT, s + 2, wave);
      f8_stage(sb, smem + (s & 1) * F8_SLOT + F8_OP, s + 2, wave);
    }
  }

  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wc * 64 + j * 16 + 4 * g;
      if (n >= N) continue;
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

// C = alpha * sum_s ws[s] + beta * C + bias, 4 columns per thread
__global__ void splitk_reduce(const float* __restrict__ ws, uint16_t* __restrict__ C, const uint16_t* __restrict__ bias,
                              int M, int N, long long ldc, int S, float alpha, float beta) {
  const long long idx = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long long MN = (long long)M * N;
  if (idx >= MN) return;
  const int m = (int)(idx / N), n = (int)(idx - (long long)m * N);
  f32x4 s = *reinterpret_cast<const f32x4*>(ws + idx);
  for (int k = 1; k < S; ++k) s += *reinterpret_cast<const f32x4*>(ws + k * MN + idx);
  float v[4] = {s[0] * alpha, s[1] * alpha, s[2] * alpha, s[3] * alpha};
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

static int g_variant = 0;  // 0 = auto: the 8-phase kernel, schedule picked per operand layout

template <bool AK, bool BKM, int EPI>
static hipError_t launch(const void* A, const void* B, void* C, float* ws, const void* bias, int M, int N, int K,
                         long long lda, long long ldb, long long ldc, float alpha, float beta, int splitk,
                         hipStream_t st) {
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  dim3 grid(tm * tn, 1, splitk);
  if (g_variant == 3)
    gemm_kernel<AK, BKM, EPI, 4, 5><<<grid, 512, 0, st>>>((const uint16_t*)A, (const uint16_t*)B, (uint16_t*)C, ws,
                                                          (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, beta,
                                                          K / splitk);
  else if (g_variant == 2)
    gemm_kernel<AK, BKM, EPI, 2><<<grid, 256, 0, st>>>((const uint16_t*)A, (const uint16_t*)B, (uint16_t*)C, ws,
                                                       (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, beta,
                                                       K / splitk);
  else
    gemm_kernel<AK, BKM, EPI, 4><<<grid, 512, 0, st>>>((const uint16_t*)A, (const uint16_t*)B, (uint16_t*)C, ws,
                                                       (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, beta,
                                                       K / splitk);
  return hipGetLastError();
}

template <int EPI>
static hipError_t dispatch(int transA, int transB, const void* A, const void* B, void* C, float* ws, const void* bias,
                           int M, int N, int K, long long lda, long long ldb, long long ldc, float alpha, float beta,
                           int splitk, hipStream_t st) {
  const bool ak = transA == 0, bk = transB != 0;
  if (ak && bk) return launch<true, true, EPI>(A, B, C, ws, bias, M, N, K, lda, ldb, ldc, alpha, beta, splitk, st);
  if (ak && !bk) return launch<true, false, EPI>(A, B, C, ws, bias, M, N, K, lda, ldb, ldc, alpha, beta, splitk, st);
  if (!ak && bk) return launch<false, true, EPI>(A, B, C, ws, bias, M, N, K, lda, ldb, ldc, alpha, beta, splitk, st);
  return launch<false, false, EPI>(A, B, C, ws, bias, M, N, K, lda, ldb, ldc, alpha, beta, splitk, st);
}

}  // namespace gemm
}  // namespace pa

using namespace pa::gemm;

// the 8-phase ping-pong kernel (csrc/gemm8.hip, its own translation unit so its register
// allocation is not perturbed by this file's template instances)
extern "C" int pa_gemm8_ok(int M, int N, int K, long long lda, long long ldb, long long ldc, int transA, int transB,
                           int splitk);
extern "C" int pa_gemm8_set_sched(int v);
extern "C" int pa_gemm8_bf16(const void* A, const void* B, void* C, const void* bias, void* ws, int M, int N, int K,
                             long long lda, long long ldb, long long ldc, int transA, int transB, float alpha,
                             float beta, int splitk, hipStream_t st);

// Shape contract (checked here; Python falls back to hipBLASLt when it does not hold):
// K % (64 * splitk) == 0, N % 8 == 0, M % 8 == 0, leading dims % 8 == 0, 16-B aligned pointers.
// splitk > 1 needs ws of splitk * M * N floats.
PA_API int pa_gemm_ok(int M, int N, int K, long long lda, long long ldb, long long ldc, int splitk) {
  if (M <= 0 || N <= 0 || K <= 0 || splitk < 1) return 0;
  if (K % 64 != 0 || M % 8 || N % 8 || lda % 8 || ldb % 8 || ldc % 8) return 0;
  // uneven slices (the last one shorter) only on the 8-phase kernels (pa_gemm8_ok checks them)
  if (K % (64 * splitk) != 0) {
    const int kb = K / 64, q = (kb + splitk - 1) / splitk;
    if (kb - (splitk - 1) * q < 2) return 0;
  }
  return 1;
}

// block layout (A/B benchmarking): 1 = 8 waves of 128x64, 2 = 4 waves of 128x128,
// 3 = 8 waves with a 5-slot ring (160 KB LDS: three sub-tiles of DMA in flight;
// +2-9 % over 1 on the GPT-3 shapes, profiles/hip_gemm_r1_v3.log), 8 = the 8-phase ping-pong
// kernel of csrc/gemm8.hip (row-half
// staging), 9 = the same with k-half staging (balanced load segments)
PA_API int pa_gemm_set_variant(int v) {
  const int old = g_variant;
  g_variant = v;
  if (v >= 8) pa_gemm8_set_sched(v);
  return old;
}

PA_API int pa_gemm_bf16(const void* A, const void* B, void* C, const void* bias, void* ws, int M, int N, int K,
                        long long lda, long long ldb, long long ldc, int transA, int transB, float alpha, float beta,
                        int splitk, hipStream_t st) {
  if (!pa_gemm_ok(M, N, K, lda, ldb, ldc, splitk)) return (int)hipErrorInvalidValue;
  // auto: k-contiguous A -> schedule 11 (row-half staging keeps its DMA on full 128-B lines; the
  // persistent form 12 is within noise in isolation and 3 % slower inside the training step);
  // m-contiguous A (weight gradients) -> schedule 9 (k-half staging, balanced load segments).
  // Measured per layout on the GPT-3 1.3B shapes: profiles/r2_gemm_sched*.log.  (A one-wave-
  // per-SIMD 128x128-per-wave schedule was tried and dropped: hipcc rotates its 256 AGPR
  // accumulators through copies, 0.87-1.0 PF.)
  if (g_variant == 0) pa_gemm8_set_sched(transA == 0 ? 11 : 9);
  const bool v8 = (g_variant == 0 || g_variant >= 8) && pa_gemm8_ok(M, N, K, lda, ldb, ldc, transA, transB, splitk);
  if (!v8 && K % (64 * splitk) != 0) return (int)hipErrorInvalidValue;  // the older kernels split evenly
  if (splitk == 1) {
    if (v8) return pa_gemm8_bf16(A, B, C, bias, nullptr, M, N, K, lda, ldb, ldc, transA, transB, alpha, beta, 1, st);
    return (int)dispatch<0>(transA, transB, A, B, C, nullptr, bias, M, N, K, lda, ldb, ldc, alpha, beta, 1, st);
  }
  if (!ws) return (int)hipErrorInvalidValue;
  hipError_t e = v8 ? (hipError_t)pa_gemm8_bf16(A, B, C, nullptr, ws, M, N, K, lda, ldb, ldc, transA, transB, 1.f, 0.f,
                                                splitk, st)
                    : dispatch<1>(transA, transB, A, B, C, (float*)ws, nullptr, M, N, K, lda, ldb, ldc, 1.f, 0.f,
                                  splitk, st);
  if (e != hipSuccess) return (int)e;
  const long long MN = (long long)M * N;
  splitk_reduce<<<(unsigned)((MN / 4 + 255) / 256), 256, 0, st>>>((const float*)ws, (uint16_t*)C,
                                                                   (const uint16_t*)bias, M, N, ldc, splitk, alpha,
                                                                   beta);
  return (int)hipGetLastError();
}

// fp8 GEMM contract: K % 128 == 0, M % 8 == 0, N % 8 == 0, lda/ldb % 16 == 0 (bytes = elements),
// ldc % 8 == 0.  fmt: 0 = e4m3 (OCP e4m3fn), 1 = e5m2.
PA_API int pa_gemm_fp8_ok(int M, int N, int K, long long lda, long long ldb, long long ldc) {
  return M > 0 && N > 0 && K > 0 && K % 128 == 0 && M % 8 == 0 && N % 8 == 0 && lda % 16 == 0 && ldb % 16 == 0 &&
         ldc % 8 == 0;
}

PA_API int pa_gemm_fp8(const void* A, const void* B, void* C, const void* bias, const void* scale_a,
                       const void* scale_b, int M, int N, int K, long long lda, long long ldb, long long ldc,
                       float alpha, float beta, int fmtA, int fmtB, hipStream_t st) {
  if (!pa_gemm_fp8_ok(M, N, K, lda, ldb, ldc) || fmtA < 0 || fmtA > 1 || fmtB < 0 || fmtB > 1)
    return (int)hipErrorInvalidValue;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  dim3 grid(tm * tn);
  auto args = [&](auto kern) {
    kern<<<grid, 512, 0, st>>>((const uint8_t*)A, (const uint8_t*)B, (uint16_t*)C, (const uint16_t*)bias, M, N, K,
                               lda, ldb, ldc, alpha, beta, (const float*)scale_a, (const float*)scale_b);
  };
  if (fmtA == 0 && fmtB == 0) args(gemm_fp8_kernel<0, 0>);
  else if (fmtA == 0) args(gemm_fp8_kernel<0, 1>);
  else if (fmtB == 0) args(gemm_fp8_kernel<1, 0>);
  else args(gemm_fp8_kernel<1, 1>);
  return (int)hipGetLastError();
}
