// NHWC 2-D convolution forward as an implicit GEMM on MFMA (gfx950), bf16 in / fp32 accumulate.
//
// Reference semantics: paddle/phi/kernels/gpudnn/conv_kernel.cu (conv2d, NHWC data_format,
// stride / padding / dilation, groups = 1), fusion/gpu/fused_conv2d_add_act (bias epilogue).
//
//   Y[n, ho, wo, co] = sum_{r, s, c} X[n, ho*sh - ph + r*dh, wo*sw - pw + s*dw, c] * W[co, r, s, c] (+ bias[co])
//
// GEMM view: M = N*Ho*Wo output pixels, N = Cout, K = R*S*C with k = (r, s, c), c fastest.
// CDNA4 design (shares the staging/pipeline of csrc/gemm.hip, not a translation of a CUDA conv):
//  * Block tile 256 pixels x BN output channels (BN = 256 / 128 / 64 chosen from Cout), 8 waves
//    2(M) x 4(N), K consumed in 32-deep sub-tiles through a 4-slot LDS ring.
//  * The im2col matrix is never materialised: every 32-deep K sub-tile lies inside one filter tap
//    (C % 32 == 0), so each 16-byte LDS-DMA of the A tile is 8 contiguous channels of one input
//    pixel; the per-lane SOURCE address is computed per sub-tile from the tap (wave-uniform) and the
//    lane's output pixel, and taps that fall into the zero padding point at a 64-byte zero block —
//    padding costs no branch and no extra pass.
//  * Weights are pre-packed [Cout][R][S][C] (k-contiguous) and staged like a GEMM B^T operand.
//  * Same counted-vmcnt ring (DMA in flight across barriers), XOR-swizzled images (conflict-free
//    ds_read_b128) and register double-buffered fragments as the GEMM; swapped products give each
//    lane 4 consecutive output channels for 8-byte stores with the bias fused.
#include "common.h"

namespace pa {
namespace conv {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BM = 256, BK = 32, NT = 512;

// DMA source for taps in the zero padding (and clamped-away rows never stored)
__device__ uint4 g_zero16[4];

struct Geom {
  int N, H, W, C, Ho, Wo, Cout, R, S, sh, sw, ph, pw, dh, dw;
};

__device__ __forceinline__ f32x4 mfma(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// K-major [rows][32 k] image, 64-B rows, chunk ^ (((row >> 3) & 1) << 1): conflict free for the
// ds_read_b128 lane groups (see csrc/gemm.hip)
__device__ __forceinline__ int img_off(int row, int ch) { return row * 64 + ((ch ^ (((row >> 3) & 1) << 1)) << 4); }

__device__ __forceinline__ s16x8 ld_frag(const char* img, int row0, int lane) {
  return *reinterpret_cast<const s16x8*>(img + img_off(row0 + (lane & 15), lane >> 4));
}

__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

template <int PER_SLOT, int N = 6>
__device__ __forceinline__ void wait_vm(int n_inflight) {
  if constexpr (N == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (n_inflight >= N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N * PER_SLOT) : "memory");
    else wait_vm<PER_SLOT, N - 1>(n_inflight);
  }
}

template <int PER_SLOT>
__device__ __forceinline__ void wait_barrier(int n_inflight) {
  wait_vm<PER_SLOT>(n_inflight);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

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

template <int BN>
__global__ __launch_bounds__(NT, 1) void conv_fwd_kernel(const uint16_t* __restrict__ X,
                                                         const uint16_t* __restrict__ Wt, uint16_t* __restrict__ Y,
                                                         const uint16_t* __restrict__ bias, Geom g, int M, int K) {
  constexpr int FN = BN / 64;                 // 16-wide fragments per wave along N
  constexpr int OPA = BM * BK * 2;            // 16 KB
  constexpr int OPB = BN * BK * 2;
  constexpr int SLOT = OPA + OPB;
  constexpr int NBC = BN * 4;                 // 16-B chunks of one B sub-tile
  constexpr int DMA_B = NBC >= NT ? NBC / NT : 1;  // BN = 64: waves 4-7 repeat waves 0-3 (same bytes, same place)
  constexpr int PER_SLOT = 2 + DMA_B;
  // ring depth 4: filling all 160 KB (5-8 slots) measured slower on the ResNet shapes (short K
  // loops pay the longer prologue, and BN = 64/128 blocks lose their second block per CU)
  constexpr int NSLOT = 4;
  __shared__ __attribute__((aligned(1024))) char smem[NSLOT * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int tm = (M + BM - 1) / BM, tn = (g.Cout + BN - 1) / BN;
  int mt, ntile;
  tile_coords(blockIdx.x, tm * tn, tm, tn, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int ns = K / BK;

  // A (im2col) source state per DMA: output pixel of row i*128 + tid/4, 8-channel chunk tid%4
  long long xb[2];
  int hb[2], wb[2], lch[2];
  bool mv[2];
  const int HoWo = g.Ho * g.Wo;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = i * 128 + (tid >> 2);
    const int m = m0 + row;
    mv[i] = m < M;
    const int mm = mv[i] ? m : 0;
    const int n = mm / HoWo, rem = mm - n * HoWo;
    const int ho = rem / g.Wo, wo = rem - ho * g.Wo;
    xb[i] = (long long)n * g.H * g.W * g.C;
    hb[i] = ho * g.sh - g.ph;
    wb[i] = wo * g.sw - g.pw;
    lch[i] = (tid & 3) ^ (((row >> 3) & 1) << 1);
  }
  // B (packed weights [Cout][K]) source per DMA
  const uint16_t* bsrc[DMA_B];
#pragma unroll
  for (int j = 0; j < DMA_B; ++j) {
    const int c = (j * NT + tid) % NBC;
    const int row = c >> 2;
    const int l = (c & 3) ^ (((row >> 3) & 1) << 1);
    bsrc[j] = Wt + (long long)min(n0 + row, g.Cout - 1) * K + l * 8;
  }

  auto stage = [&](int s, int slot) {
    char* ia = smem + slot * SLOT;
    const unsigned abase = (unsigned)(size_t)(lds_void*)ia;
    const unsigned bbase = abase + OPA;
    const int kk = s * BK;
    const int tap = kk / g.C;
    const int c0 = kk - tap * g.C;
    const int r = tap / g.S, q = tap - r * g.S;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int hi = hb[i] + r * g.dh, wi = wb[i] + q * g.dw;
      const bool ok = mv[i] && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
      const void* src = ok ? (const void*)(X + xb[i] + ((long long)hi * g.W + wi) * g.C + c0 + lch[i] * 8)
                           : (const void*)g_zero16;
      glds16(src, __builtin_amdgcn_readfirstlane(abase + (i * NT + wave * 64) * 16));
    }
#pragma unroll
    for (int j = 0; j < DMA_B; ++j)
      glds16(bsrc[j] + kk, __builtin_amdgcn_readfirstlane(bbase + ((j * NT + wave * 64) % NBC) * 16));
  };

  f32x4 acc[8][FN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NSLOT; ++s)
    if (s < ns) stage(s, s);
  wait_barrier<PER_SLOT>(max(min(ns, NSLOT) - 2, 0));
  s16x8 fa[2][8], fb[2][FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) fb[0][j] = ld_frag(smem + OPA, wc * (16 * FN) + j * 16, lane);
#pragma unroll
  for (int i = 0; i < 8; ++i) fa[0][i] = ld_frag(smem, wr * 128 + i * 16, lane);
  int slot = 0;
  for (int s = 0; s < ns; s += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int ss = s + u;
      const int nslot = slot + 1 == NSLOT ? 0 : slot + 1;
      if (ss + NSLOT < ns) stage(ss + NSLOT, slot);
      const char* ia = smem + nslot * SLOT;
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[u ^ 1][j] = ld_frag(ia + OPA, wc * (16 * FN) + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[u ^ 1][i] = ld_frag(ia, wr * 128 + i * 16, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma(fb[u][j], fa[u][i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      wait_barrier<PER_SLOT>(max(min(ns - 1, ss + NSLOT) - (ss + 2), 0));
      slot = nslot;
    }
  }

  const int gq = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wc * (16 * FN) + j * 16 + 4 * gq;
      if (n >= g.Cout) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (bias) {
        float bb[4];
        load_f<bf16_t, 4>(reinterpret_cast<const bf16_t*>(bias + n), bb);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bb[r];
      }
      store_f<bf16_t, 4>(reinterpret_cast<bf16_t*>(Y + (long long)m * g.Cout + n), v);
    }
  }
}

}  // namespace conv
}  // namespace pa

using namespace pa::conv;

// Contract: bf16 NHWC input [N,H,W,C], packed weight [Cout][R][S][C], output [N,Ho,Wo,Cout];
// C % 32 == 0, (R*S*C) % 64 == 0, Cout % 8 == 0 (checked; Python falls back to MIOpen otherwise).
PA_API int pa_conv2d_fwd_ok(int C, int Cout, int R, int S) {
  return C > 0 && C % 32 == 0 && (R * S * C) % 64 == 0 && Cout > 0 && Cout % 8 == 0;
}

PA_API int pa_conv2d_fwd(const void* x, const void* wpk, void* y, const void* bias, int N, int H, int W, int C,
                         int Cout, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int Ho, int Wo,
                         hipStream_t st) {
  if (!pa_conv2d_fwd_ok(C, Cout, R, S) || N <= 0 || Ho <= 0 || Wo <= 0) return (int)hipErrorInvalidValue;
  Geom g{N, H, W, C, Ho, Wo, Cout, R, S, sh, sw, ph, pw, dh, dw};
  const long long Mll = (long long)N * Ho * Wo;
  if (Mll > (1LL << 30)) return (int)hipErrorInvalidValue;
  const int M = (int)Mll, K = R * S * C;
  const int BN = Cout >= 256 ? 256 : (Cout > 64 ? 128 : 64);
  const int tm = (M + BM - 1) / BM, tn = (Cout + BN - 1) / BN;
  const dim3 grid(tm * tn);
  if (BN == 256)
    conv_fwd_kernel<256><<<grid, NT, 0, st>>>((const uint16_t*)x, (const uint16_t*)wpk, (uint16_t*)y,
                                              (const uint16_t*)bias, g, M, K);
  else if (BN == 128)
    conv_fwd_kernel<128><<<grid, NT, 0, st>>>((const uint16_t*)x, (const uint16_t*)wpk, (uint16_t*)y,
                                              (const uint16_t*)bias, g, M, K);
  else
    conv_fwd_kernel<64><<<grid, NT, 0, st>>>((const uint16_t*)x, (const uint16_t*)wpk, (uint16_t*)y,
                                             (const uint16_t*)bias, g, M, K);
  return (int)hipGetLastError();
}
