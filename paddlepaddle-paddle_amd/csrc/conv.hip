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
  long long total;  // input elements (im2col bounds; 0 elsewhere)
  // forward only: channels as STORED in X when the K decomposition uses C padded to a multiple of
  // 32 (C % 32 != 0, C % 8 == 0: the padded 8-channel chunks read the zero block); 0 = C
  int Cs;
};

// Filter taps of the implicit GEMM (k = (tap, c)): input row/col offsets of each tap, so a kernel
// can run a SUBSET of the filter (a stride class of the data gradient), and the output pixel
// mapping y = (oy0 + osy*ho, ox0 + osx*wo) in a [HY, WY] map (a stride class writes every s-th
// pixel of dX).  Forward: all R*S taps at (r*dh - ph, s*dw - pw), identity mapping.
constexpr int MAX_TAPS = 64, MAX_CLS = 9;
struct Taps {
  short th[MAX_TAPS], tw[MAX_TAPS];
  int oy0, ox0, osy, osx, HY, WY;
  long long ldw;  // row stride (elements) of the packed filter [Cout_y][taps][C]
  // ncls > 0: a multi-class data-gradient launch (class c owns blocks [cls_end[c-1], cls_end[c]))
  int ncls;
  int cls_end[MAX_CLS], cls_tap0[MAX_CLS], cls_T[MAX_CLS], cls_a[MAX_CLS], cls_b[MAX_CLS], cls_Hc[MAX_CLS],
      cls_Wc[MAX_CLS];
  long long cls_woff[MAX_CLS];
  // forward launches only (nullable): batch-norm column statistics of every 16*FM-row wave slab,
  // fp32 [2][ceil(M / (16 FM))][Cout] (slab means, then M2s) — fused_bn statistics in the epilogue
  float* stats;
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

typedef __attribute__((address_space(3))) char lds_char;
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x2 lds_u32x2;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

// Staged store of one wave's (16 FM) x (16 FN) output tile: the 8-B fragments go to the wave's
// own LDS region ([rows][32 FN bytes], 16-B chunk c of row r at c ^ ((r / rows-per-256-B) % chunks))
// and come back row-wise, 16 B per lane, so every store instruction writes whole 64-256-B row
// segments instead of 16 rows x 8 B (each lane's 4 columns) — the same measure as the GEMM's
// wave-local staged epilogue (csrc/gemm8.hip epilogue_wstaged).  No block barrier: a wave's LDS
// accesses complete in order; wave_barrier only stops the compiler from reordering them.
template <int FM, int FN>
__device__ __forceinline__ int cstage_off(int r, int c) {
  constexpr int RB = 32 * FN, CPR = RB / 16, RPL = RB >= 256 ? 1 : 256 / RB;
  return r * RB + ((c ^ ((r / RPL) & (CPR - 1))) << 4);
}

template <int BN, int WM, bool STG = true, bool PADC = false>
__global__ __launch_bounds__(NT, 1) void conv_fwd_kernel(const uint16_t* __restrict__ X,
                                                         const uint16_t* __restrict__ Wt, uint16_t* __restrict__ Y,
                                                         const uint16_t* __restrict__ bias, Geom g, Taps tp, int M,
                                                         int K) {
  constexpr int WNW = 8 / WM;                 // waves: WM along pixels x WNW along channels
  constexpr int FM = 16 / WM, FN = BN / (16 * WNW);  // 16x16 fragments per wave
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
  const int wr = wave / WNW, wc = wave % WNW;
  const int Cs = PADC ? g.Cs : g.C;  // channels per stored input pixel
  // stride classes of a data gradient share one launch: the block finds its class (tile ranges
  // are prefix sums) and takes the class's pixel grid, tap range, packed weights and output offset
  int Ho = g.Ho, Wo = g.Wo, tap0 = 0, oy0 = tp.oy0, ox0 = tp.ox0, bid = blockIdx.x;
  const uint16_t* Wp = Wt;
  if (tp.ncls > 0) {
    int c = 0;
    while (c + 1 < tp.ncls && bid >= tp.cls_end[c]) ++c;
    bid -= c ? tp.cls_end[c - 1] : 0;
    Ho = tp.cls_Hc[c];
    Wo = tp.cls_Wc[c];
    tap0 = tp.cls_tap0[c];
    oy0 = tp.cls_a[c];
    ox0 = tp.cls_b[c];
    M = g.N * Ho * Wo;
    K = tp.cls_T[c] * g.C;
    Wp = Wt + tp.cls_woff[c];
  }
  const int tm = (M + BM - 1) / BM, tn = (g.Cout + BN - 1) / BN;
  int mt, ntile;
  tile_coords(bid, tm * tn, tm, tn, mt, ntile);
  const int m0 = mt * BM, n0 = ntile * BN;
  const int ns = K / BK;

  // A (im2col) source state per DMA: output pixel of row i*128 + tid/4, 8-channel chunk tid%4
  long long xb[2];
  int hb[2], wb[2], lch[2];
  bool mv[2];
  const int HoWo = Ho * Wo;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = i * 128 + (tid >> 2);
    const int m = m0 + row;
    mv[i] = m < M;
    const int mm = mv[i] ? m : 0;
    const int n = mm / HoWo, rem = mm - n * HoWo;
    const int ho = rem / Wo, wo = rem - ho * Wo;
    xb[i] = (long long)n * g.H * g.W * Cs;
    hb[i] = ho * g.sh;
    wb[i] = wo * g.sw;
    lch[i] = (tid & 3) ^ (((row >> 3) & 1) << 1);
  }
  // B (packed weights [Cout][K]) source per DMA
  const uint16_t* bsrc[DMA_B];
#pragma unroll
  for (int j = 0; j < DMA_B; ++j) {
    const int c = (j * NT + tid) % NBC;
    const int row = c >> 2;
    const int l = (c & 3) ^ (((row >> 3) & 1) << 1);
    bsrc[j] = Wp + (long long)min(n0 + row, g.Cout - 1) * tp.ldw + l * 8;
  }

  auto stage = [&](int s, int slot) {
    char* ia = smem + slot * SLOT;
    const unsigned abase = (unsigned)(size_t)(lds_void*)ia;
    const unsigned bbase = abase + OPA;
    const int kk = s * BK;
    const int tap = kk / g.C;
    const int c0 = kk - tap * g.C;  // g.C: the (padded) channels of the K decomposition
    const int th = tp.th[tap0 + tap], tw = tp.tw[tap0 + tap];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int hi = hb[i] + th, wi = wb[i] + tw;
      const bool ok = mv[i] && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W &&
                      (PADC == false || c0 + lch[i] * 8 < Cs);
      const void* src = ok ? (const void*)(X + xb[i] + ((long long)hi * g.W + wi) * Cs + c0 + lch[i] * 8)
                           : (const void*)g_zero16;
      glds16(src, __builtin_amdgcn_readfirstlane(abase + (i * NT + wave * 64) * 16));
    }
#pragma unroll
    for (int j = 0; j < DMA_B; ++j)
      glds16(bsrc[j] + kk, __builtin_amdgcn_readfirstlane(bbase + ((j * NT + wave * 64) % NBC) * 16));
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NSLOT; ++s)
    if (s < ns) stage(s, s);
  wait_barrier<PER_SLOT>(max(min(ns, NSLOT) - 2, 0));
  s16x8 fa[2][FM], fb[2][FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) fb[0][j] = ld_frag(smem + OPA, wc * (16 * FN) + j * 16, lane);
#pragma unroll
  for (int i = 0; i < FM; ++i) fa[0][i] = ld_frag(smem, wr * (16 * FM) + i * 16, lane);
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
      for (int i = 0; i < FM; ++i) fa[u ^ 1][i] = ld_frag(ia, wr * (16 * FM) + i * 16, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma(fb[u][j], fa[u][i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      wait_barrier<PER_SLOT>(max(min(ns - 1, ss + NSLOT) - (ss + 2), 0));
      slot = nslot;
    }
  }

  const int gq = lane >> 4;
  const bool ident = tp.osy == 1 && tp.osx == 1 && oy0 == 0 && ox0 == 0;
  if (tp.stats != nullptr) {  // wave-uniform: forward launches without bias (host contract)
    constexpr int RW = 16 * FM;
    const int mw = m0 + wr * RW;
    const long long P = (M + RW - 1) / RW;
    wave_col_stats<FM, FN>(acc, nullptr, min(RW, M - mw), n0 + wc * (16 * FN), g.Cout,
                           tp.stats + (long long)(mw / RW) * g.Cout, tp.stats + (P + mw / RW) * g.Cout);
  }
  if constexpr (STG) {
    constexpr int RB = 32 * FN, CPR = RB / 16, RPI = 64 / CPR;  // row bytes, 16-B chunks per row, rows per read
    lds_char* reg = (lds_char*)smem + wave * (16 * FM * RB);
    float bb[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wc * (16 * FN) + j * 16 + 4 * gq;
#pragma unroll
      for (int r = 0; r < 4; ++r) bb[j][r] = 0.f;
      if (bias && n < g.Cout) load_f<bf16_t, 4>(reinterpret_cast<const bf16_t*>(bias + n), bb[j]);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int r = i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        Pack<bf16_t, 4> pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk.v[e] = (bf16_t)(acc[i][j][e] + bb[j][e]);
        const int cb = j * 32 + gq * 8;  // byte column within the wave's row
        *(lds_u32x2*)(reg + cstage_off<FM, FN>(r, cb >> 4) + (cb & 15)) = __builtin_bit_cast(u32x2, pk);
      }
    }
    __builtin_amdgcn_wave_barrier();
    constexpr int NRD = 16 * FM / RPI;  // row-read instructions per wave
#pragma unroll
    for (int q = 0; q < NRD; q += 8) {
      u32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (q + u < NRD) v[u] = *(const lds_u32x4*)(reg + cstage_off<FM, FN>((q + u) * RPI + lane / CPR, lane % CPR));
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (q + u >= NRD) continue;
        const int r = (q + u) * RPI + lane / CPR;
        const int m = m0 + wr * (16 * FM) + r;
        const int n = n0 + wc * (16 * FN) + (lane % CPR) * 8;
        if (m >= M || n >= g.Cout) continue;
        long long ym = m;
        if (!ident) {
          const int nn = m / HoWo, rem = m - nn * HoWo;
          const int ho = rem / Wo, wo = rem - ho * Wo;
          ym = ((long long)nn * tp.HY + oy0 + tp.osy * ho) * tp.WY + ox0 + tp.osx * wo;
        }
        *reinterpret_cast<u32x4*>(Y + ym * g.Cout + n) = v[u];
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wr * (16 * FM) + i * 16 + (lane & 15);
    if (m >= M) continue;
    long long ym = m;
    if (!ident) {
      const int nn = m / HoWo, rem = m - nn * HoWo;
      const int ho = rem / Wo, wo = rem - ho * Wo;
      ym = ((long long)nn * tp.HY + oy0 + tp.osy * ho) * tp.WY + ox0 + tp.osx * wo;
    }
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
      store_f<bf16_t, 4>(reinterpret_cast<bf16_t*>(Y + ym * g.Cout + n), v);
    }
  }
}


// ============================================================================ filter gradient
// dW[co, r, s, c] = sum_{n, ho, wo} dY[n, ho, wo, co] * X[n, ho*sh - ph + r*dh, wo*sw - pw + s*dw, c]
//
// Implicit GEMM with the PIXELS as the reduction axis: C'[m = (r, s, c)][co] = sum_p A[m][p] B[p][co],
// A[m][p] = X at pixel p shifted by tap (r, s) (the im2col matrix, never stored), B = dY viewed
// [P][Cout].  Both operands are m/n-contiguous along their rows (channels are the fastest axis of
// NHWC), so both are staged as [32 pixels][cols] images and read with ds_read_b64_tr_b16, the
// hardware transposed LDS read (the layout of the Linear weight-gradient GEMM in csrc/gemm.hip).
//  * The tap/channel of every 16-B A chunk is fixed per thread (a 256-wide m tile covers whole
//    8-channel groups of one tap, C % 8 == 0); the pixel advances by 32 per sub-tile, tracked
//    incrementally as (n, ho, wo) — no division in the loop; taps in the zero padding and pixels
//    past the split's end DMA a zero block.
//  * B chunks stride by 32*Cout elements per sub-tile; rows past P are clamped (A is zero there).
//  * Cout sits on the narrow tile side (BN = 64/128/256 from Cout) so the 64-channel layers do
//    not waste MFMA work; the many-pixel reduction is split over gridDim.z (fp32 slabs [z][M][Cout]
//    summed by the caller) to fill the 256 CUs — a 56x56 batch-256 layer has 800k pixels.
//  * B images narrower than 256 columns use 64-/128-/256-B-row swizzles chosen so the 8 k-rows a
//    32-lane half of a transposed read touches land on 8 distinct 32-B bank slots.
template <int WCH>
__device__ __forceinline__ int swz_w(int r) {
  if constexpr (WCH >= 16) return ((r & 3) | (((r >> 3) & 1) << 2)) << 1;
  else return (((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1;
}
template <int WCH>
__device__ __forceinline__ int mn_off(int row, int ch) { return row * (WCH * 16) + ((ch ^ swz_w<WCH>(row)) << 4); }

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// fragment element j of lane (g = lane>>4, i = lane&15) = operand[col0 + i][k = 8g + j]
template <int WCH>
__device__ __forceinline__ s16x8 ld_frag_mn(const char* img, int col0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int kr = 8 * g + q;
  const int ch = (col0 >> 3) + (p >> 1);
  const int bi = (p & 1) * 8;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + mn_off<WCH>(kr, ch) + bi));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + mn_off<WCH>(kr + 4, ch) + bi));
  s16x8 v;
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  return v;
}

template <int BN, int WM, bool STG = true>
__global__ __launch_bounds__(NT, 1) void conv_wgrad_kernel(const uint16_t* __restrict__ X,
                                                           const uint16_t* __restrict__ dY, float* __restrict__ ws,
                                                           Geom g, int M, int P, int kchunk) {
  constexpr int WNW = 8 / WM;                 // waves along Cout
  constexpr int FM = 16 / WM, FN = BN / (16 * WNW);  // 16x16 fragments per wave
  constexpr int WB = BN / 8;                  // 16-B chunks per B image row
  constexpr int OPA = 256 * BK * 2;           // 16 KB: [32 pixels][256 (tap, c)]
  constexpr int OPB = BN * BK * 2;
  constexpr int SLOT = OPA + OPB;
  constexpr int NBC = BK * WB;                // chunks of one B sub-tile
  constexpr int DMA_B = NBC >= NT ? NBC / NT : 1;
  constexpr int PER_SLOT = 2 + DMA_B;
  constexpr int NSLOT = 4;
  __shared__ __attribute__((aligned(1024))) char smem[NSLOT * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WNW, wc = wave % WNW;
  const int tm = (M + 255) / 256, tn = (g.Cout + BN - 1) / BN;
  int mt, ntile;
  tile_coords(blockIdx.x, tm * tn, tm, tn, mt, ntile);
  const int m0 = mt * 256, n0 = ntile * BN;
  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(P, kbeg + kchunk);
  const int ns = (kend - kbeg + BK - 1) / BK;

  // A chunk i: k-row kr = 16 i + tid / 32, logical column chunk (tid % 32) ^ swz(kr)
  const int HoWo = g.Ho * g.Wo;
  const int dq = BK / g.Wo, dr = BK - dq * g.Wo;
  long long xoff[2];
  int offh[2], offw[2], n_[2], oh_[2], ow_[2], pp[2];
  bool mv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int kr = 16 * i + (tid >> 5);
    const int lch = (tid & 31) ^ swz_w<32>(kr);
    const int m = m0 + lch * 8;
    mv[i] = m < M;
    const int mm = mv[i] ? m : 0;
    const int tap = mm / g.C, c = mm - tap * g.C;
    const int r = tap / g.S, q = tap - r * g.S;
    offh[i] = r * g.dh - g.ph;
    offw[i] = q * g.dw - g.pw;
    xoff[i] = c;
    const int p = kbeg + kr;
    pp[i] = p;
    const int pc = min(p, P - 1);
    n_[i] = pc / HoWo;
    const int rem = pc - n_[i] * HoWo;
    oh_[i] = rem / g.Wo;
    ow_[i] = rem - oh_[i] * g.Wo;
  }
  // B chunk j: k-row c / WB, logical chunk (c % WB) ^ swz(row)
  const uint16_t* bsrc[DMA_B];
  int brow[DMA_B];
#pragma unroll
  for (int j = 0; j < DMA_B; ++j) {
    const int c = (j * NT + tid) % NBC;
    const int row = c / WB;
    const int l = (c % WB) ^ swz_w<WB>(row);
    brow[j] = kbeg + row;
    bsrc[j] = dY + min(n0 + l * 8, g.Cout - 8);
  }

  auto stage = [&](int s, int slot) {
    char* ia = smem + slot * SLOT;
    const unsigned abase = (unsigned)(size_t)(lds_void*)ia;
    const unsigned bbase = abase + OPA;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int hi = oh_[i] * g.sh + offh[i], wi = ow_[i] * g.sw + offw[i];
      const bool ok = mv[i] && pp[i] < kend && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
      const void* src = ok ? (const void*)(X + (((long long)n_[i] * g.H + hi) * g.W + wi) * g.C + xoff[i])
                           : (const void*)g_zero16;
      glds16(src, __builtin_amdgcn_readfirstlane(abase + (i * NT + wave * 64) * 16));
      // advance this chunk's pixel by 32 (sub-tile s+1 of this thread)
      pp[i] += BK;
      ow_[i] += dr;
      oh_[i] += dq;
      if (ow_[i] >= g.Wo) { ow_[i] -= g.Wo; ++oh_[i]; }
      while (oh_[i] >= g.Ho) { oh_[i] -= g.Ho; ++n_[i]; }
    }
#pragma unroll
    for (int j = 0; j < DMA_B; ++j) {
      const int p = min(brow[j] + s * BK, P - 1);
      glds16(bsrc[j] + (long long)p * g.Cout, __builtin_amdgcn_readfirstlane(bbase + ((j * NT + wave * 64) % NBC) * 16));
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NSLOT; ++s)
    if (s < ns) stage(s, s);
  wait_barrier<PER_SLOT>(max(min(ns, NSLOT) - 2, 0));
  s16x8 fa[2][FM], fb[2][FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) fb[0][j] = ld_frag_mn<WB>(smem + OPA, wc * (16 * FN) + j * 16, lane);
#pragma unroll
  for (int i = 0; i < FM; ++i) fa[0][i] = ld_frag_mn<32>(smem, wr * (16 * FM) + i * 16, lane);
  int slot = 0;
  for (int s = 0; s < ns; s += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int ss = s + u;
      const int nslot = slot + 1 == NSLOT ? 0 : slot + 1;
      if (ss + NSLOT < ns) stage(ss + NSLOT, slot);
      const char* ia = smem + nslot * SLOT;
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[u ^ 1][j] = ld_frag_mn<WB>(ia + OPA, wc * (16 * FN) + j * 16, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[u ^ 1][i] = ld_frag_mn<32>(ia, wr * (16 * FM) + i * 16, lane);
      if (ss < ns) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mfma(fb[u][j], fa[u][i], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
      wait_barrier<PER_SLOT>(max(min(ns - 1, ss + NSLOT) - (ss + 2), 0));
      slot = nslot;
    }
  }

  const int gq = lane >> 4;
  float* slab = ws + (long long)blockIdx.z * M * g.Cout;
  if constexpr (STG) {
    // fp32 slab rows leave whole: per 16-row fragment band, the wave's 16 x (16 FN) fp32 go to its
    // own 16 x 64 FN-byte LDS region and come back row-wise (16 B per lane, 64 FN-byte row
    // segments per store) instead of 16 rows x 64 B per store instruction
    constexpr int RB = 64 * FN, CPR = RB / 16, RPI = 64 / CPR, RPL = RB >= 256 ? 1 : 256 / RB;
    lds_char* reg = (lds_char*)smem + wave * (16 * RB);
    auto off = [&](int r, int c) { return r * RB + ((c ^ ((r / RPL) & (CPR - 1))) << 4); };
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
        *(lds_u32x4*)(reg + off(lane & 15, j * 4 + gq)) = __builtin_bit_cast(u32x4, acc[i][j]);
      __builtin_amdgcn_wave_barrier();
      u32x4 v[16 / RPI];
#pragma unroll
      for (int u = 0; u < 16 / RPI; ++u) v[u] = *(const lds_u32x4*)(reg + off(u * RPI + lane / CPR, lane % CPR));
#pragma unroll
      for (int u = 0; u < 16 / RPI; ++u) {
        const int m = m0 + wr * (16 * FM) + i * 16 + u * RPI + lane / CPR;
        const int n = n0 + wc * (16 * FN) + (lane % CPR) * 4;
        if (m < M && n < g.Cout) *reinterpret_cast<u32x4*>(slab + (long long)m * g.Cout + n) = v[u];
      }
      __builtin_amdgcn_wave_barrier();  // the next band overwrites the region after these reads
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wr * (16 * FM) + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wc * (16 * FN) + j * 16 + 4 * gq;
      if (n >= g.Cout) continue;
      *reinterpret_cast<f32x4*>(slab + (long long)m * g.Cout + n) = acc[i][j];
    }
  }
}

// fp32 slabs [splits][R*S*C][Cout] -> bf16 OIHW filter gradient [Cout][C][R][S], in two passes:
// (1) groups of WZ slabs summed with float4 loads over the whole grid (a 56x56 layer has hundreds
//     of slabs: one thread walking all of them per element would be latency bound),
// (2) the per-group partials summed and written transposed into the OIHW image.
constexpr int WZ = 16;
__global__ __launch_bounds__(256) void wgrad_zsum_kernel(const float* __restrict__ ws, float* __restrict__ part,
                                                         int splits, long long total4) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= total4) return;
  const int z0 = blockIdx.y * WZ, z1 = min(splits, z0 + WZ);
  const float4* src = reinterpret_cast<const float4*>(ws) + e;
  float4 a = src[(long long)z0 * total4];
  for (int z = z0 + 1; z < z1; ++z) {
    const float4 b = src[(long long)z * total4];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  reinterpret_cast<float4*>(part)[(long long)blockIdx.y * total4 + e] = a;
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, uint16_t* __restrict__ dw,
                                                           int ngroups, int RS, int C, int Cout, int accumulate) {
  const long long total = (long long)RS * C * Cout;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    // e enumerates the slab order (co fastest): coalesced partial reads
    const int co = (int)(e % Cout);
    const long long mc = e / Cout;
    const int c = (int)(mc % C), rs = (int)(mc / C);
    float v = 0.f;
    for (int z = 0; z < ngroups; ++z) v += part[(long long)z * total + e];
    bf16_t* o = reinterpret_cast<bf16_t*>(dw) + ((long long)co * C + c) * RS + rs;
    if (accumulate) v += (float)*o;  // in place into the flat gradient slot
    *o = (bf16_t)v;
  }
}

}  // namespace conv
}  // namespace pa

using namespace pa::conv;

// staged (row-segment) output stores of the forward / data-gradient and filter-gradient kernels (A/B knob pa_conv2d_set_staged; default on)
static int g_conv_staged = 1;
PA_API int pa_conv2d_set_staged(int v) {
  const int old = g_conv_staged;
  g_conv_staged = v ? 1 : 0;
  return old;
}

// Contract: bf16 NHWC input [N,H,W,C], packed weight [Cout][R][S][C], output [N,Ho,Wo,Cout];
// C % 32 == 0, (R*S*C) % 64 == 0, Cout % 8 == 0 (checked; Python falls back to MIOpen otherwise).
// Zero taps appended to the filter so that K = taps * C is a multiple of the 64-deep main loop
// (C % 64 == 32 with an odd tap count, e.g. a 3x3 conv over 32 channels): the extra tap reads the
// zero block (offset far outside the image) against zero filter columns.  The packed filter of
// pa_conv2d_fwd / _stats is [Cout][R*S + pa_conv2d_fwd_pad_taps(C, R, S)][C].
PA_API int pa_conv2d_fwd_pad_taps(int C, int R, int S) { return ((long long)R * S * C) % 64 != 0 ? 1 : 0; }

// Channels of the K decomposition for C stored input channels: C itself when C % 32 == 0, else C
// rounded up to 32 (C % 8 == 0): the padded 8-channel chunks of every tap read the zero block and
// meet zero filter columns (packed filter [Cout][taps][pa_conv2d_fwd_cpad(C)]).
PA_API int pa_conv2d_fwd_cpad(int C) { return (C + 31) / 32 * 32; }

PA_API int pa_conv2d_fwd_ok(int C, int Cout, int R, int S) {
  if (C <= 0 || C % 8 != 0) return 0;
  const int Cp = pa_conv2d_fwd_cpad(C);
  return R > 0 && S > 0 && R * S + pa_conv2d_fwd_pad_taps(Cp, R, S) <= MAX_TAPS && Cout > 0 && Cout % 8 == 0;
}

// waves along the pixel side per Cout tile width (A/B knob; index 0/1/2 = BN 64/128/256)
static int g_fwd_wm[3] = {4, 4, 2};  // measured: BN 64 and 128 tiles are LDS-read bound at 2(M)x4(N)
PA_API int pa_conv2d_set_wm(int bn, int wm) {
  const int k = bn >= 256 ? 2 : (bn >= 128 ? 1 : 0);
  const int old = g_fwd_wm[k];
  if (wm == 2 || wm == 4 || wm == 8) g_fwd_wm[k] = wm;
  return old;
}


template <bool STG, bool PADC = false>
static void launch_fwd_kernel_t(int BN, dim3 grid, const uint16_t* xp, const uint16_t* wp, uint16_t* yp,
                                const uint16_t* bp, const Geom& g, const Taps& tp, int M, int K, hipStream_t st) {
  if (BN == 256) {
    if (g_fwd_wm[2] == 4) conv_fwd_kernel<256, 4, STG, PADC><<<grid, NT, 0, st>>>(xp, wp, yp, bp, g, tp, M, K);
    else conv_fwd_kernel<256, 2, STG, PADC><<<grid, NT, 0, st>>>(xp, wp, yp, bp, g, tp, M, K);
  } else if (BN == 128) {
    if (g_fwd_wm[1] == 4) conv_fwd_kernel<128, 4, STG, PADC><<<grid, NT, 0, st>>>(xp, wp, yp, bp, g, tp, M, K);
    else conv_fwd_kernel<128, 2, STG, PADC><<<grid, NT, 0, st>>>(xp, wp, yp, bp, g, tp, M, K);
  } else {
    if (g_fwd_wm[0] == 4) conv_fwd_kernel<64, 4, STG, PADC><<<grid, NT, 0, st>>>(xp, wp, yp, bp, g, tp, M, K);
    else if (g_fwd_wm[0] == 8) conv_fwd_kernel<64, 8, STG, PADC><<<grid, NT, 0, st>>>(xp, wp, yp, bp, g, tp, M, K);
    else conv_fwd_kernel<64, 2, STG, PADC><<<grid, NT, 0, st>>>(xp, wp, yp, bp, g, tp, M, K);
  }
}

static void launch_fwd_kernel(int BN, dim3 grid, const uint16_t* xp, const uint16_t* wp, uint16_t* yp,
                              const uint16_t* bp, const Geom& g, const Taps& tp, int M, int K, hipStream_t st) {
  if (g.Cs > 0 && g.Cs != g.C) launch_fwd_kernel_t<true, true>(BN, grid, xp, wp, yp, bp, g, tp, M, K, st);
  else if (g_conv_staged) launch_fwd_kernel_t<true>(BN, grid, xp, wp, yp, bp, g, tp, M, K, st);
  else launch_fwd_kernel_t<false>(BN, grid, xp, wp, yp, bp, g, tp, M, K, st);
}

static int launch_fwd(const void* x, const void* wpk, void* y, const void* bias, const Geom& g, const Taps& tp,
                      int ntaps, hipStream_t st) {
  const long long Mll = (long long)g.N * g.Ho * g.Wo;
  if (Mll > (1LL << 30) || Mll <= 0) return (int)hipErrorInvalidValue;
  const int M = (int)Mll, K = ntaps * g.C;
  const int BN = g.Cout >= 256 ? 256 : (g.Cout > 64 ? 128 : 64);
  const int tm = (M + BM - 1) / BM, tn = (g.Cout + BN - 1) / BN;
  const dim3 grid(tm * tn);
  const uint16_t *xp = (const uint16_t*)x, *wp = (const uint16_t*)wpk, *bp = (const uint16_t*)bias;
  uint16_t* yp = (uint16_t*)y;
  launch_fwd_kernel(BN, grid, xp, wp, yp, bp, g, tp, M, K, st);
  return (int)hipGetLastError();
}

// rows per batch-norm statistics slab of a forward launch with Cout output channels (16 x the
// fragments per wave along the pixels: 256 / WM of the tile width the launcher picks)
PA_API int pa_conv2d_fwd_stat_rows(int Cout) {
  const int BN = Cout >= 256 ? 256 : (Cout > 64 ? 128 : 64);
  return 256 / g_fwd_wm[BN >= 256 ? 2 : (BN >= 128 ? 1 : 0)];
}

static int conv2d_fwd_impl(const void* x, const void* wpk, void* y, const void* bias, float* stats, int N, int H,
                           int W, int C, int Cout, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw,
                           int Ho, int Wo, hipStream_t st);

PA_API int pa_conv2d_fwd(const void* x, const void* wpk, void* y, const void* bias, int N, int H, int W, int C,
                         int Cout, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int Ho, int Wo,
                         hipStream_t st) {
  return conv2d_fwd_impl(x, wpk, y, bias, nullptr, N, H, W, C, Cout, R, S, sh, sw, ph, pw, dh, dw, Ho, Wo, st);
}

// forward + batch-norm column statistics (stats: fp32 [2][ceil(N*Ho*Wo / rows)][Cout], rows =
// pa_conv2d_fwd_stat_rows(Cout)); no bias
PA_API int pa_conv2d_fwd_stats(const void* x, const void* wpk, void* y, float* stats, int N, int H, int W, int C,
                               int Cout, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int Ho, int Wo,
                               hipStream_t st) {
  if (stats == nullptr) return (int)hipErrorInvalidValue;
  return conv2d_fwd_impl(x, wpk, y, nullptr, stats, N, H, W, C, Cout, R, S, sh, sw, ph, pw, dh, dw, Ho, Wo, st);
}

static int conv2d_fwd_impl(const void* x, const void* wpk, void* y, const void* bias, float* stats, int N, int H,
                           int W, int C, int Cout, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw,
                           int Ho, int Wo, hipStream_t st) {
  if (!pa_conv2d_fwd_ok(C, Cout, R, S) || N <= 0 || Ho <= 0 || Wo <= 0 || H >= 16384 || W >= 16384)
    return (int)hipErrorInvalidValue;
  const int Cs = C;
  C = pa_conv2d_fwd_cpad(Cs);  // K decomposition channels (filter packed with this many)
  Geom g{N, H, W, C, Ho, Wo, Cout, R, S, sh, sw, ph, pw, dh, dw, 0, Cs};
  Taps tp{};
  for (int r = 0; r < R; ++r)
    for (int q = 0; q < S; ++q) {
      tp.th[r * S + q] = (short)(r * dh - ph);
      tp.tw[r * S + q] = (short)(q * dw - pw);
    }
  const int ntaps = R * S + pa_conv2d_fwd_pad_taps(C, R, S);
  for (int t = R * S; t < ntaps; ++t) tp.th[t] = tp.tw[t] = (short)-30000;  // always outside: zero block
  tp.oy0 = tp.ox0 = 0;
  tp.osy = tp.osx = 1;
  tp.HY = Ho;
  tp.WY = Wo;
  tp.ldw = (long long)ntaps * C;
  tp.stats = stats;
  return launch_fwd(x, wpk, y, bias, g, tp, ntaps, st);
}

// Data gradient of a strided conv, all stride classes in ONE launch.  Class c = (a, b) covers
// dX[n, a + s_h*i, b + s_w*j, :] and sees T_c filter taps at dY offsets (th, tw):
//   dX[n, a + s_h*i, b + s_w*j, c] = sum_t sum_co dY[n, i + th[t], j + tw[t], co] * Wd_c[c][t][co].
// dy: [N, Hd, Wd, Cout] bf16; wd: packed filter [C][sum_c T_c][Cout] (class c's taps at tap0_c);
// cls: ncls x {a, b, T}; th/tw: the taps of all classes in class order; dx: [N, H, W, C] (pixels of
// classes without taps are not written — the caller zero-fills when there are any).
PA_API int pa_conv2d_dgrad_classes(const void* dy, const void* wd, void* dx, int N, int Hd, int Wd, int Cout, int C,
                                   int H, int W, int s_h, int s_w, int ncls, const int* cls, const int* th,
                                   const int* tw, hipStream_t st) {
  if (ncls <= 0 || ncls > MAX_CLS || s_h <= 0 || s_w <= 0 || Cout % 32 || C % 8 || C <= 0)
    return (int)hipErrorInvalidValue;
  Geom g{N, Hd, Wd, Cout, 0, 0, C, 1, 1, 1, 1, 0, 0, 1, 1};
  Taps tp{};
  tp.osy = s_h;
  tp.osx = s_w;
  tp.HY = H;
  tp.WY = W;
  const int BN = C >= 256 ? 256 : (C > 64 ? 128 : 64);
  const int tn = (C + BN - 1) / BN;
  int tap = 0, blocks = 0, k = 0;
  long long woff = 0;
  for (int c = 0; c < ncls; ++c) {
    const int a = cls[3 * c], b = cls[3 * c + 1], T = cls[3 * c + 2];
    const int Hc = (H - a + s_h - 1) / s_h, Wc = (W - b + s_w - 1) / s_w;
    if (T <= 0 || tap + T > MAX_TAPS || Hc <= 0 || Wc <= 0 || (T * Cout) % 64) return (int)hipErrorInvalidValue;
    for (int t = 0; t < T; ++t) {
      tp.th[tap + t] = (short)th[tap + t];
      tp.tw[tap + t] = (short)tw[tap + t];
    }
    const long long Mc = (long long)N * Hc * Wc;
    if (Mc > (1LL << 30)) return (int)hipErrorInvalidValue;
    blocks += (int)((Mc + BM - 1) / BM) * tn;
    tp.cls_end[k] = blocks;
    tp.cls_tap0[k] = tap;
    tp.cls_T[k] = T;
    tp.cls_a[k] = a;
    tp.cls_b[k] = b;
    tp.cls_Hc[k] = Hc;
    tp.cls_Wc[k] = Wc;
    tp.cls_woff[k] = woff;
    tap += T;
    woff += (long long)T * Cout;
    ++k;
  }
  tp.ncls = k;
  tp.ldw = (long long)tap * Cout;
  const dim3 grid(blocks);
  const uint16_t *xp = (const uint16_t*)dy, *wp = (const uint16_t*)wd;
  uint16_t* yp = (uint16_t*)dx;
  launch_fwd_kernel(BN, grid, xp, wp, yp, nullptr, g, tp, 0, 0, st);
  return (int)hipGetLastError();
}

static int g_wgrad_bn_cap = 128;  // widest Cout tile (A/B knob)
static int g_wgrad_wm = 4;        // waves along the (tap, c) side: 2 / 4 (/ 8 for BN = 64)
PA_API int pa_conv2d_wgrad_set_wm(int v) {
  const int old = g_wgrad_wm;
  if (v == 2 || v == 4 || v == 8) g_wgrad_wm = v;
  return old;
}
PA_API int pa_conv2d_wgrad_set_bncap(int v) {
  const int old = g_wgrad_bn_cap;
  if (v > 0) g_wgrad_bn_cap = v;
  return old;
}

template <bool STG>
static void launch_wgrad_kernel(int BN, dim3 grid, const uint16_t* xp, const uint16_t* dp, float* wsp, const Geom& g,
                                int M, int P, int kchunk, hipStream_t st) {
  if (BN == 256) {
    if (g_wgrad_wm == 2) conv_wgrad_kernel<256, 2, STG><<<grid, NT, 0, st>>>(xp, dp, wsp, g, M, P, kchunk);
    else conv_wgrad_kernel<256, 4, STG><<<grid, NT, 0, st>>>(xp, dp, wsp, g, M, P, kchunk);
  } else if (BN == 128) {
    if (g_wgrad_wm == 2) conv_wgrad_kernel<128, 2, STG><<<grid, NT, 0, st>>>(xp, dp, wsp, g, M, P, kchunk);
    else conv_wgrad_kernel<128, 4, STG><<<grid, NT, 0, st>>>(xp, dp, wsp, g, M, P, kchunk);
  } else {
    if (g_wgrad_wm == 2) conv_wgrad_kernel<64, 2, STG><<<grid, NT, 0, st>>>(xp, dp, wsp, g, M, P, kchunk);
    else if (g_wgrad_wm == 8) conv_wgrad_kernel<64, 8, STG><<<grid, NT, 0, st>>>(xp, dp, wsp, g, M, P, kchunk);
    else conv_wgrad_kernel<64, 4, STG><<<grid, NT, 0, st>>>(xp, dp, wsp, g, M, P, kchunk);
  }
}

// Filter gradient.  x: bf16 NHWC [N,H,W,C], dy: bf16 NHWC [N,Ho,Wo,Cout], ws: fp32 scratch of
// (splits + ceil(splits / 16)) * R*S*C * Cout floats (splits = pa_conv2d_wgrad_splits), dw: bf16 [Cout][C][R][S]
// (accumulate != 0: dw += the gradient, in place).  C % 8 == 0, Cout % 8 == 0, kchunk % 32 == 0.
// im2col of an NHWC input for convolutions whose channel count the implicit-GEMM kernel does not
// take (the 3-channel RGB stem).  Row-segment layout: k = r * RK + s * C + c with RK = S*C rounded
// up to 8, so each filter row's S*C taps are one contiguous run of the input (channels fastest,
// then w) and one 16-B-aligned run of the output row; out [M = N*Ho*Wo][Kp] bf16, zeros for taps
// in the padding, for the RK - S*C slots of each filter row and for k >= R*RK (Kp % 8 == 0).  One
// thread per 16-B output chunk, consecutive lanes on consecutive chunks (whole-row stores), 8
// 2-byte gathers each with constant-divisor tap math (a thread per pixel writing 24 chunks at a
// 384-B lane stride measured 0.81 ms on the ResNet50 stem; per-element runtime divisions 1.24 ms).
// The convolution is then a 1 x 1 convolution of this matrix on conv_fwd_kernel with the filter
// packed in the same k order.
template <int S, int C>
__global__ __launch_bounds__(256) void im2col_rows_kernel(const uint16_t* __restrict__ X, uint16_t* __restrict__ out,
                                                          Geom g, int M, int Kp) {
  constexpr int SC = S * C, RK = (SC + 7) / 8 * 8, CPR = RK / 8;  // 16-B chunks per filter row
  const int cpo = Kp >> 3;                                         // 16-B chunks per output row
  // 32-bit index math (host: M * Kp / 8 < 2^31): 64-bit divisions are software sequences of ~150
  // instructions, which made this gather kernel VALU-bound
  const unsigned t = blockIdx.x * 256u + threadIdx.x;  // consecutive lanes: consecutive chunks
  const unsigned m = t / (unsigned)cpo;
  if (m >= (unsigned)M) return;
  const int q = (int)(t - m * (unsigned)cpo);
  const int r = q / CPR, t0 = (q - r * CPR) * 8;
  uint16_t v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = 0;
  if (r < g.R) {
    const unsigned HoWo = (unsigned)(g.Ho * g.Wo);
    const unsigned n = m / HoWo, rem = m - n * HoWo;
    const int ho = (int)(rem / (unsigned)g.Wo), wo = (int)rem - ho * g.Wo;
    const int hi = ho * g.sh - g.ph + r * g.dh;
    if ((unsigned)hi < (unsigned)g.H) {
      const long long row0 = ((long long)n * g.H + hi) * g.W * C;  // element index of the input row
      const int wi0 = wo * g.sw - g.pw;
      // with unit dilation the S*C taps of a filter row are ONE contiguous run of the input row, so
      // a chunk's 8 values are 8 consecutive elements: two aligned 16-B loads + a 2-byte-granular
      // funnel shift instead of 8 scattered 2-byte gathers (which were TA-bound)
      const long long b0 = row0 + (long long)wi0 * C + t0;
      const long long a0 = b0 >= 0 ? (b0 & ~7LL) : -1;
      if (g.dw == 1 && a0 >= 0 && a0 + 16 <= g.total) {
        const uint4 lo = *reinterpret_cast<const uint4*>(X + a0);
        const uint4 hi4 = *reinterpret_cast<const uint4*>(X + a0 + 8);
        const unsigned w[8] = {lo.x, lo.y, lo.z, lo.w, hi4.x, hi4.y, hi4.z, hi4.w};
        const int sh2 = (int)(b0 - a0) * 2;  // byte shift 0..14
        const int wq = sh2 >> 2, bq = sh2 & 3;
        unsigned o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // words wq + j and wq + j + 1 of the window (wq <= 3): 4-way selects, no dynamic indexing
          const unsigned x0 = wq == 0 ? w[j] : wq == 1 ? w[j + 1] : wq == 2 ? w[j + 2] : w[j + 3];
          const unsigned x1 = wq == 0 ? w[j + 1] : wq == 1 ? w[j + 2] : wq == 2 ? w[j + 3] : w[j + 4];
          o[j] = __builtin_amdgcn_alignbyte(x1, x0, bq);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int tt = t0 + e;
          const int wi = wi0 + tt / C;
          const uint16_t val = (uint16_t)(o[e >> 1] >> ((e & 1) * 16));
          v[e] = (tt < SC && (unsigned)wi < (unsigned)g.W) ? val : 0;
        }
      } else {
        const uint16_t* xr = X + row0;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int tt = t0 + e;  // (s, c) = (tt / C, tt % C): constant divisors
          const int sidx = tt / C, c = tt - sidx * C;
          const int wi = wi0 + sidx * g.dw;
          if (tt < SC && (unsigned)wi < (unsigned)g.W) v[e] = xr[(long long)wi * C + c];
        }
      }
    }
  }
  uint4 pk;
  pk.x = v[0] | ((unsigned)v[1] << 16);
  pk.y = v[2] | ((unsigned)v[3] << 16);
  pk.z = v[4] | ((unsigned)v[5] << 16);
  pk.w = v[6] | ((unsigned)v[7] << 16);
  *reinterpret_cast<uint4*>(out + (long long)m * Kp + q * 8) = pk;
}

// returns hipErrorInvalidValue for (S, C) pairs without an instantiation (the caller falls back)
PA_API int pa_im2col_rows_ok(int S, int C) { return (S == 7 && C == 3) || (S == 3 && C == 3) || (S == 3 && C == 5); }

PA_API int pa_im2col_nhwc(const void* x, void* out, int N, int H, int W, int C, int R, int S, int sh, int sw, int ph,
                          int pw, int dh, int dw, int Ho, int Wo, int Kp, hipStream_t st) {
  const long long M = (long long)N * Ho * Wo;
  const int RK = (S * C + 7) / 8 * 8;
  if (M <= 0 || M * (Kp / 8) >= (1LL << 31) || Kp % 8 || Kp < R * RK || C <= 0 || !pa_im2col_rows_ok(S, C))
    return (int)hipErrorInvalidValue;
  Geom g{N, H, W, C, Ho, Wo, 0, R, S, sh, sw, ph, pw, dh, dw, (long long)N * H * W * C};
  const unsigned blocks = (unsigned)((M * (Kp / 8) + 255) / 256);
  const uint16_t* xp = (const uint16_t*)x;
  uint16_t* op = (uint16_t*)out;
  if (S == 7 && C == 3) im2col_rows_kernel<7, 3><<<blocks, 256, 0, st>>>(xp, op, g, (int)M, Kp);
  else if (S == 3 && C == 3) im2col_rows_kernel<3, 3><<<blocks, 256, 0, st>>>(xp, op, g, (int)M, Kp);
  else im2col_rows_kernel<3, 5><<<blocks, 256, 0, st>>>(xp, op, g, (int)M, Kp);
  return (int)hipGetLastError();
}

// A/B (pa_conv_set_wgrad_direct): <= 16 pixel splits summed by the finishing pass itself
static int g_wgrad_direct = 1;
PA_API int pa_conv_set_wgrad_direct(int v) {
  const int old = g_wgrad_direct;
  g_wgrad_direct = v;
  return old;
}

PA_API int pa_conv2d_wgrad_ok(int C, int Cout) { return C > 0 && C % 8 == 0 && Cout > 0 && Cout % 8 == 0; }

PA_API int pa_conv2d_wgrad(const void* x, const void* dy, void* ws, void* dw, int N, int H, int W, int C, int Cout,
                           int R, int S, int sh, int sw, int ph, int pw, int dh, int dw_, int Ho, int Wo, int splits,
                           int accumulate, hipStream_t st) {
  if (!pa_conv2d_wgrad_ok(C, Cout) || N <= 0 || Ho <= 0 || Wo <= 0 || splits <= 0) return (int)hipErrorInvalidValue;
  const long long Pll = (long long)N * Ho * Wo;
  if (Pll > (1LL << 30) || (long long)N * H * W * C > (1LL << 40)) return (int)hipErrorInvalidValue;
  Geom g{N, H, W, C, Ho, Wo, Cout, R, S, sh, sw, ph, pw, dh, dw_};
  const int P = (int)Pll, M = R * S * C;
  int kchunk = (int)(((Pll + splits - 1) / splits + 31) / 32 * 32);
  splits = (P + kchunk - 1) / kchunk;  // no empty split
  const int BN = (Cout >= 256 && g_wgrad_bn_cap >= 256) ? 256 : (Cout > 64 && g_wgrad_bn_cap >= 128 ? 128 : 64);
  const int tm = (M + 255) / 256, tn = (Cout + BN - 1) / BN;
  const dim3 grid(tm * tn, 1, splits);
  const uint16_t *xp = (const uint16_t*)x, *dp = (const uint16_t*)dy;
  float* wsp = (float*)ws;
  if (g_conv_staged) launch_wgrad_kernel<true>(BN, grid, xp, dp, wsp, g, M, P, kchunk, st);
  else launch_wgrad_kernel<false>(BN, grid, xp, dp, wsp, g, M, P, kchunk, st);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const long long total = (long long)M * Cout;  // Cout % 8 == 0: float4 groups never straddle a row
  const long long nb = (total + 255) / 256;
  const int blocks = (int)(nb < 2048 ? nb : 2048);
  if (splits <= WZ && g_wgrad_direct) {
    // few slices: the finishing pass sums them straight from the split workspace ([splits][total],
    // coalesced per slice) — one launch and no partial round trip (the pre-sum pass was a second
    // ~11 us launch per convolution: ~0.5 ms of the ResNet50 step)
    wgrad_reduce_kernel<<<blocks, 256, 0, st>>>((const float*)ws, (uint16_t*)dw, splits, R * S, C, Cout, accumulate);
    return (int)hipGetLastError();
  }
  const int ngroups = (splits + WZ - 1) / WZ;
  float* part = (float*)ws + (long long)splits * total;  // scratch tail: ngroups x total
  const dim3 zgrid((unsigned)((total / 4 + 255) / 256), ngroups);
  wgrad_zsum_kernel<<<zgrid, 256, 0, st>>>((const float*)ws, part, splits, total / 4);
  wgrad_reduce_kernel<<<blocks, 256, 0, st>>>(part, (uint16_t*)dw, ngroups, R * S, C, Cout, accumulate);
  return (int)hipGetLastError();
}

// the split count pa_conv2d_wgrad will actually use (scratch sizing)
PA_API int pa_conv2d_wgrad_splits(int N, int Ho, int Wo, int splits) {
  const long long P = (long long)N * Ho * Wo;
  const long long kchunk = ((P + splits - 1) / splits + 31) / 32 * 32;
  return (int)((P + kchunk - 1) / kchunk);
}
