// Few-channel NHWC convolution forward (the RGB stem: C = 3, 7x7 / stride 2) on MFMA, gfx950.
//
// Reference: paddle/phi/kernels/gpudnn/conv_kernel.cu (the cuDNN / MIOpen forward the reference
// runs for every convolution, the 3-channel stem included).
//
// Why a separate kernel: the implicit-GEMM forward (conv.hip) stages 32-channel slices of a pixel
// with LDS-DMA, so a 3-channel input would be 90 % zero padding, and an explicit im2col writes and
// re-reads a [pixels, 192] matrix (1.2 GB for ResNet50's stem at batch 256).  Here the GEMM
// K axis is (filter row r, s*C + c): for one output pixel the S*C values of filter row r are ONE
// contiguous run of the NHWC input row (pixel stride C), so a block stages the R input-row
// segments its output-row segment needs once in LDS (zero filled outside the image: the padding
// costs nothing afterwards) and every MFMA operand fragment is 8 consecutive elements of a staged
// row — no index arithmetic per tap, no im2col buffer.
//  * k = r * RK + j, RK = S*C rounded up to 8 (an 8-element fragment never straddles two filter
//    rows), K padded to a multiple of 32 with zero filter columns; the filter comes in as the
//    [Cout][Kp] k-contiguous image (host-packed, tiny).
//  * Block = 256 threads = 4 waves, RB consecutive output rows (same image) of one output-row
//    segment of up to 128 pixels x 64 output channels; a wave owns 32 pixels (two 16-pixel MFMA
//    tiles) x 64 channels.  The (RB - 1) * sh + R input rows the RB output rows need are staged
//    once (16-byte aligned chunk copies: the segment start is rounded down to 8 elements), and
//    each wave keeps its whole filter slice (KSTEPS x 4 fragments) in registers for all RB rows.
//  * Input fragments: an 8-element run starting at any (2-byte) element is 5 ds_read_b32 and 4
//    v_alignbit (shift 0 or 16): no per-element LDS reads for odd channel counts.
//  * Products are D = W * X^T (v_mfma_f32_16x16x32) with the filter rows PERMUTED so that a lane
//    ends with 16 CONSECUTIVE output channels of one pixel (tile t row r is channel
//    16 (r >> 2) + 4 t + (r & 3)): two 16-byte NHWC stores per pixel tile.
//  * Optional batch-norm statistics epilogue (fused_bn statistics, like the implicit-GEMM
//    forward): per output-row segment (one slab of min(Wo, 128) pixels) the column (mean, M2),
//    reduced over a wave's pixels by DPP and over the 4 waves by a Chan merge in LDS.
#include "common.h"

namespace pa {
namespace stem {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int PT = 128;  // output pixels per block row
constexpr int CT = 64;   // output channels per block
constexpr int RBMAX = 8; // output rows per block (fewer when the staged rows would not fit)

template <typename T> __device__ __forceinline__ f32x4 mfma(s16x8 a, s16x8 b, f32x4 c);
template <> __device__ __forceinline__ f32x4 mfma<bf16_t>(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <> __device__ __forceinline__ f32x4 mfma<f16_t>(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

struct Geo {
  int H, W, C, Ho, Wo, Cout, R, S, sh, sw, ph, pw, RK, Kp;
  int SEGP;  // staged row pitch (elements, multiple of 8)
  int RB;    // output rows per block
  int NR;    // staged input rows = (RB - 1) * sh + R
  int HB;    // row blocks per image = ceil(Ho / RB)
  int vec;   // 16-byte chunk loads allowed (row length % 8 == 0, 16-byte aligned input)
  long long P;  // statistics slabs = N * Ho * ceil(Wo / PT)
};

// grid (ceil(Wo / PT), N * HB, Cout / CT); dynamic LDS = NR * SEGP * 2 (+ RB * 2 KB with STATS)
template <typename T, int KSTEPS, bool STATS>
__global__ __launch_bounds__(256) void fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ wimg,
                                                  const T* __restrict__ bias, uint16_t* __restrict__ y,
                                                  float* __restrict__ stats, Geo g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t rows[];  // [NR][SEGP]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ow0 = blockIdx.x * PT;
  const int n = blockIdx.y / g.HB;
  const int oh0 = (blockIdx.y - n * g.HB) * g.RB;
  const int co0 = blockIdx.z * CT;
  // staged row i = input row oh0*sh - ph + i; staged element e = input element ea + e of that row
  const int e0 = (ow0 * g.sw - g.pw) * g.C;
  const int ea = e0 & ~7;  // floor to a multiple of 8 (also for negative e0)
  const int off = e0 - ea;
  const int rowlen = g.W * g.C;
  const int nch = g.SEGP >> 3;
  for (int idx = tid; idx < g.NR * nch; idx += 256) {
    const int i = idx / nch, ch = idx - i * nch;
    const int ih = oh0 * g.sh - g.ph + i;
    const int ge = ea + 8 * ch;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (ih >= 0 && ih < g.H) {
      const uint16_t* src = x + ((long long)n * g.H + ih) * rowlen;
      if (g.vec && ge >= 0 && ge + 8 <= rowlen) {
        v = *reinterpret_cast<const uint4*>(src + ge);
      } else {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int a = ge + 2 * k;
          const uint32_t lo = (a >= 0 && a < rowlen) ? src[a] : 0u;
          const uint32_t hi = (a + 1 >= 0 && a + 1 < rowlen) ? src[a + 1] : 0u;
          w[k] = lo | (hi << 16);
        }
        v = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
    *reinterpret_cast<uint4*>(rows + i * g.SEGP + 8 * ch) = v;
  }

  const int g4 = lane >> 4, l16 = lane & 15;
  const int SC = g.S * g.C;
  // the wave's filter slice for all K steps, rows permuted (see the header).  Up to 8 K steps it
  // stays in registers for all RB rows; the deep filters (AlexNet's 11x11: Kp = 448, 14 steps,
  // instantiated as KSTEPS 16 with the live count g.Kp / 32) re-read it per step from L1/L2
  // (64 x Kp x 2 bytes, shared by every block of the launch) instead of holding 224 VGPRs.
  constexpr bool WREG = KSTEPS <= 8;
  const uint16_t* wb = wimg + (long long)(co0 + 16 * (l16 >> 2) + (l16 & 3)) * g.Kp + 8 * g4;
  s16x8 wf[WREG ? KSTEPS : 1][4];
  if constexpr (WREG) {
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
      for (int t = 0; t < 4; ++t) wf[ks][t] = *reinterpret_cast<const s16x8*>(wb + (long long)4 * t * g.Kp + ks * 32);
  }
  const int nks = WREG ? KSTEPS : g.Kp / 32;
  // this lane's (filter row, run offset) per K step
  int kr[KSTEPS], kj[KSTEPS];
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
    const int kk = ks * 32 + 8 * g4;
    kr[ks] = kk / g.RK;
    kj[ks] = kk - kr[ks] * g.RK;
  }
  int pq[2];  // staged element of this lane's pixel (m-tile m), before the tap offset
#pragma unroll
  for (int m = 0; m < 2; ++m) pq[m] = off + (32 * wave + 16 * m + l16) * g.sw * g.C;
  const int nvw = max(0, min(32, g.Wo - ow0 - 32 * wave));  // valid pixels of this wave
  // Cout % 16 == 0: a lane's 16 channels co0 + 16 g4 .. + 15 are all valid or none (not stored)
  const bool cvalid = co0 + 16 * g4 < g.Cout;
  const int cbase = min(co0 + 16 * g4, g.Cout - 16);  // in-bounds bias reads either way
  float* wst = reinterpret_cast<float*>(rows + g.NR * g.SEGP);  // STATS: [RB][4 waves][2][64]
  __syncthreads();

  for (int rb = 0; rb < g.RB; ++rb) {
    const int oh = oh0 + rb;
    if (oh >= g.Ho) break;  // block-uniform
    f32x4 acc[2][4];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      if (!WREG && ks >= nks) break;  // block-uniform
      s16x8 wk[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        wk[t] = WREG ? wf[WREG ? ks : 0][t] : *reinterpret_cast<const s16x8*>(wb + (long long)4 * t * g.Kp + ks * 32);
      const int r = kr[ks], j0 = kj[ks];
      const bool live = r < g.R;
      const uint16_t* rowp = rows + (rb * g.sh + (live ? r : 0)) * g.SEGP;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int q = pq[m] + j0;
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(rowp) + (q >> 1);
        uint32_t w[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) w[k] = wp[k];
        const uint32_t shf = (q & 1) * 16;
        s16x8 xf;
        uint32_t d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d[k] = __builtin_amdgcn_alignbit(w[k + 1], w[k], shf);
          const int j = j0 + 2 * k;
          d[k] = (!live || j >= SC) ? 0u : (j + 1 >= SC ? (d[k] & 0xFFFFu) : d[k]);
        }
        xf = __builtin_bit_cast(s16x8, d);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[m][t] = mfma<T>(wk[t], xf, acc[m][t]);
      }
    }
    // lane: channels co0 + 16 g4 + 4 t + e (acc[m][t][e]) of pixel ow0 + 32 wave + 16 m + l16
    const long long nh = (long long)n * g.Ho + oh;
    float bv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) bv[i] = 0.f;
    if (bias != nullptr) {
#pragma unroll
      for (int i = 0; i < 16; ++i) bv[i] = to_f(bias[cbase + i]);
    }
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int ow = ow0 + 32 * wave + 16 * m + l16;
      if (ow >= g.Wo || !cvalid) continue;
      uint16_t* dst = y + (nh * g.Wo + ow) * g.Cout + co0 + 16 * g4;
      float v0[8], v1[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v0[i] = acc[m][i >> 2][i & 3] + bv[i];
        v1[i] = acc[m][2 + (i >> 2)][i & 3] + bv[8 + i];
      }
      store_f<T, 8>(reinterpret_cast<T*>(dst), v0);
      store_f<T, 8>(reinterpret_cast<T*>(dst + 8), v1);
    }
    if constexpr (STATS) {
      // wave slab (mean, M2) over its nvw pixels, two-pass in registers, DPP over the 16 pixels of a group
      float* ws = wst + (rb * 4 + wave) * 128;
      if (nvw > 0) {
        const float inv = 1.f / (float)nvw;
        float mu[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float s = 0.f;
#pragma unroll
          for (int m = 0; m < 2; ++m) s += (16 * m + l16 < nvw) ? acc[m][i >> 2][i & 3] : 0.f;
          mu[i] = row16_sum(s) * inv;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float q = 0.f;
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            const float dd = acc[m][i >> 2][i & 3] - mu[i];
            q += (16 * m + l16 < nvw) ? dd * dd : 0.f;
          }
          q = row16_sum(q);
          if (l16 == i) {  // spread the 16 channel writes over the group's lanes
            ws[16 * g4 + i] = mu[i];
            ws[64 + 16 * g4 + i] = q;
          }
        }
      }
    }
  }
  if constexpr (STATS) {
    __syncthreads();
    const long long P = g.P;
    for (int idx = tid; idx < g.RB * CT; idx += 256) {
      const int rb = idx >> 6, c = idx & 63;
      const int oh = oh0 + rb;
      if (oh >= g.Ho || co0 + c >= g.Cout) continue;
      float cnt = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {  // Chan merge of the wave slabs
        const int nw = max(0, min(32, g.Wo - ow0 - 32 * w));
        if (nw == 0) continue;
        const float* ws = wst + (rb * 4 + w) * 128;
        const float nb = (float)nw, tot = cnt + nb;
        const float dlt = ws[c] - mean;
        mean += dlt * (nb / tot);
        m2 += ws[64 + c] + dlt * dlt * (cnt * nb / tot);
        cnt = tot;
      }
      const long long slab = ((long long)n * g.Ho + oh) * gridDim.x + blockIdx.x;
      stats[slab * g.Cout + co0 + c] = mean;
      stats[(P + slab) * g.Cout + co0 + c] = m2;
    }
  }
}

}  // namespace stem
}  // namespace pa

using namespace pa;

static bool stem_geo(int N, int H, int W, int C, int Ho, int Wo, int Cout, int R, int S, int sh, int sw, int ph,
                     int pw, bool stats, pa::stem::Geo& g) {
  using namespace pa::stem;
  // Cout % 16: the last block's missing channels have zero filter rows (the host pads the image to
  // a multiple of 64 rows) and are not stored
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C > 8 || Ho <= 0 || Wo <= 0 || Cout <= 0 || Cout % 16 != 0) return false;
  if (R <= 0 || S <= 0 || R > 11 || S > 11 || sh <= 0 || sw <= 0 || sh > 4 || sw > 4 || ph < 0 || pw < 0) return false;
  if ((long long)W * C >= (1LL << 30)) return false;
  const int RK = (S * C + 7) / 8 * 8;
  const int Kp = (R * RK + 31) / 32 * 32;
  if (Kp > 512) return false;  // > 256: the streamed-filter instantiation
  // staged segment: columns (ow0*sw - pw) .. ((ow0+PT-1)*sw - pw + S - 1), plus up to 7 elements
  // of round-down slack in front and the last fragment's read-ahead (RK - S*C + the 5th dword)
  const int SEGP = ((((PT - 1) * sw + S) * C + RK + 16) + 7) / 8 * 8;
  int RB = RBMAX;
  auto lds = [&](int rb) { return (long long)((rb - 1) * sh + R) * SEGP * 2 + (stats ? rb * 4 * 128 * 4 : 0); };
  while (RB > 1 && lds(RB) > 64 * 1024) --RB;
  if (lds(RB) > 64 * 1024) return false;
  const long long gx = (Wo + PT - 1) / PT;
  g = Geo{H, W, C, Ho, Wo, Cout, R, S, sh, sw, ph, pw, RK, Kp, SEGP, RB, (RB - 1) * sh + R, (Ho + RB - 1) / RB, 0,
          (long long)N * Ho * gx};
  return true;
}

static size_t stem_lds(const pa::stem::Geo& g, bool stats) {
  return (size_t)g.NR * g.SEGP * 2 + (stats ? (size_t)g.RB * 4 * 128 * 4 : 0);
}

PA_API int pa_conv_stem_ok(int C, int Cout, int R, int S, int sh, int sw) {
  pa::stem::Geo g;
  return stem_geo(1, 16, 16, C, 1, 1, Cout, R, S, sh, sw, 0, 0, true, g) ? 1 : 0;
}

// K extent of the packed filter image ([Cout][Kp], k = r * RK + s * C + c, zeros elsewhere)
PA_API int pa_conv_stem_kp(int C, int R, int S) { return (R * ((S * C + 7) / 8 * 8) + 31) / 32 * 32; }
PA_API int pa_conv_stem_rk(int C, int S) { return (S * C + 7) / 8 * 8; }

// rows per batch-norm statistics slab of a stem forward with Wo output columns (one output-row
// segment per slab; all slabs equal only when Wo <= 128 or Wo % 128 == 0), 0 = no statistics
PA_API int pa_conv_stem_stat_rows(int Wo) {
  const int PT = pa::stem::PT;
  return Wo > 0 && (Wo <= PT || Wo % PT == 0) ? (Wo < PT ? Wo : PT) : 0;
}

// x [N,H,W,C] (16-bit), wimg [ceil(Cout / 64) * 64][Kp] (rows past Cout zero), bias [Cout] or null ->
// y [N,Ho,Wo,Cout]; Cout % 16 == 0; dilation 1.
// stats (nullable, no bias): fp32 [2][N*Ho*ceil(Wo/128)][Cout] slab means then M2s.
PA_API hipError_t pa_conv_stem_fwd(const void* x, const void* wimg, const void* bias, void* y, float* stats, int N,
                                   int H, int W, int C, int Cout, int R, int S, int sh, int sw, int ph, int pw, int Ho,
                                   int Wo, int dt, hipStream_t st) {
  pa::stem::Geo g;
  const bool wst = stats != nullptr;
  if (!stem_geo(N, H, W, C, Ho, Wo, Cout, R, S, sh, sw, ph, pw, wst, g)) return hipErrorInvalidValue;
  if (wst && (bias != nullptr || pa_conv_stem_stat_rows(Wo) == 0)) return hipErrorInvalidValue;
  const long long gy = (long long)N * g.HB;
  if (gy > 2147483647LL || (long long)N * H * W * C >= (1LL << 46)) return hipErrorInvalidValue;
  g.vec = ((W * C) % 8 == 0 && ((uintptr_t)x & 15) == 0) ? 1 : 0;
  const dim3 grid((Wo + pa::stem::PT - 1) / pa::stem::PT, (unsigned)gy, (Cout + pa::stem::CT - 1) / pa::stem::CT);
  const size_t lds = stem_lds(g, wst);
  const int ks = g.Kp / 32;
#define PA_STEM_LAUNCH(T, K)                                                                               \
  do {                                                                                                     \
    if (wst)                                                                                               \
      pa::stem::fwd_kernel<T, K, true><<<grid, 256, lds, st>>>((const uint16_t*)x, (const uint16_t*)wimg, \
                                                               (const T*)bias, (uint16_t*)y, stats, g);    \
    else                                                                                                   \
      pa::stem::fwd_kernel<T, K, false><<<grid, 256, lds, st>>>((const uint16_t*)x, (const uint16_t*)wimg, \
                                                                (const T*)bias, (uint16_t*)y, nullptr, g); \
  } while (0)
#define PA_STEM_KS(T)                           \
  switch (ks) {                                 \
    case 1: PA_STEM_LAUNCH(T, 1); break;        \
    case 2: PA_STEM_LAUNCH(T, 2); break;        \
    case 3: PA_STEM_LAUNCH(T, 3); break;        \
    case 4: PA_STEM_LAUNCH(T, 4); break;        \
    case 5: PA_STEM_LAUNCH(T, 5); break;        \
    case 6: PA_STEM_LAUNCH(T, 6); break;        \
    case 7: PA_STEM_LAUNCH(T, 7); break;        \
    case 8: PA_STEM_LAUNCH(T, 8); break;        \
    default: PA_STEM_LAUNCH(T, 16); break;      \
  }
  if (dt == 1) {
    PA_STEM_KS(bf16_t)
  } else if (dt == 2) {
    PA_STEM_KS(f16_t)
  } else {
    return hipErrorInvalidValue;
  }
#undef PA_STEM_KS
#undef PA_STEM_LAUNCH
  return hipGetLastError();
}
