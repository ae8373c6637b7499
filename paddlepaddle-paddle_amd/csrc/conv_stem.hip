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
//  * Block = 256 threads = 4 waves, one output-row segment of up to 128 pixels x 64 output
//    channels; a wave owns 32 pixels (two 16-pixel MFMA tiles) x 64 channels.
//  * Products are D = W * X^T (v_mfma_f32_16x16x32), so a lane ends with 4 consecutive output
//    channels of one pixel: 8-byte NHWC stores.
//  * The input fragments are 8 x ds_read_u16 (a fragment's start is only 2-byte aligned when C
//    is odd); the stem is bound by its 411 MB output write, not by these reads.
#include "common.h"

namespace pa {
namespace stem {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int PT = 128;  // output pixels per block
constexpr int CT = 64;   // output channels per block

template <typename T> __device__ __forceinline__ f32x4 mfma(s16x8 a, s16x8 b, f32x4 c);
template <> __device__ __forceinline__ f32x4 mfma<bf16_t>(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <> __device__ __forceinline__ f32x4 mfma<f16_t>(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

struct Geo {
  int H, W, C, Ho, Wo, Cout, R, S, sh, sw, ph, pw, RK, Kp, SEG;
};

// grid (ceil(Wo / PT), N * Ho, Cout / CT); dynamic LDS = R * SEG * 2 bytes
template <typename T, int KSTEPS>
__global__ __launch_bounds__(256) void fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ wimg,
                                                  const T* __restrict__ bias, uint16_t* __restrict__ y, Geo g) {
  extern __shared__ uint16_t rows[];  // [R][SEG]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ow0 = blockIdx.x * PT;
  const int nh = blockIdx.y;
  const int oh = nh % g.Ho;
  const long long n = nh / g.Ho;
  const int co0 = blockIdx.z * CT;
  // stage the R input-row segments: element e of row r is input element (iw0 * C + e) of input
  // row ih = oh*sh - ph + r, zero outside the image
  const int e0 = (ow0 * g.sw - g.pw) * g.C;
  const int rowlen = g.W * g.C;
  for (int r = 0; r < g.R; ++r) {
    const int ih = oh * g.sh - g.ph + r;
    const bool hin = ih >= 0 && ih < g.H;
    const uint16_t* src = x + (n * g.H + (hin ? ih : 0)) * (long long)rowlen;
    for (int e = tid; e < g.SEG; e += 256) {
      const int ie = e0 + e;
      rows[r * g.SEG + e] = (hin && ie >= 0 && ie < rowlen) ? src[ie] : (uint16_t)0;
    }
  }
  __syncthreads();

  const int g4 = lane >> 4, l16 = lane & 15;
  const int SC = g.S * g.C;
  f32x4 acc[2][4];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this lane's pixel of m-tile m: local column (32 * wave + 16 * m + l16) of the segment
  int pbase[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) pbase[m] = (32 * wave + 16 * m + l16) * g.sw * g.C;
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
    const int kk = ks * 32 + 8 * g4;
    const int r = kk / g.RK, j0 = kk - r * g.RK;
    // filter fragments: W[co0 + 16t + l16][kk .. kk+8)
    s16x8 wf[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      wf[t] = *reinterpret_cast<const s16x8*>(wimg + (long long)(co0 + 16 * t + l16) * g.Kp + kk);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      s16x8 xf;
      if (r < g.R) {
        const uint16_t* src = rows + r * g.SEG + pbase[m] + j0;
#pragma unroll
        for (int i = 0; i < 8; ++i) xf[i] = (j0 + i < SC) ? (short)src[i] : (short)0;
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) xf[i] = 0;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[m][t] = mfma<T>(wf[t], xf, acc[m][t]);
    }
  }
  // lane holds output channels co0 + 16t + 4*g4 + (0..3) of pixel ow0 + 32*wave + 16*m + l16
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int ow = ow0 + 32 * wave + 16 * m + l16;
    if (ow >= g.Wo) continue;
    uint16_t* dst = y + ((long long)nh * g.Wo + ow) * g.Cout + co0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = 16 * t + 4 * g4;
      float v[4] = {acc[m][t][0], acc[m][t][1], acc[m][t][2], acc[m][t][3]};
      if (bias != nullptr) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] += to_f(bias[co0 + c + i]);
      }
      store_f<T, 4>(reinterpret_cast<T*>(dst + c), v);
    }
  }
}

}  // namespace stem
}  // namespace pa

using namespace pa;

static bool stem_geo(int H, int W, int C, int Ho, int Wo, int Cout, int R, int S, int sh, int sw, int ph, int pw,
                     pa::stem::Geo& g) {
  if (H <= 0 || W <= 0 || C <= 0 || C > 8 || Ho <= 0 || Wo <= 0 || Cout <= 0 || Cout % pa::stem::CT != 0) return false;
  if (R <= 0 || S <= 0 || R > 11 || S > 11 || sh <= 0 || sw <= 0 || sh > 4 || sw > 4 || ph < 0 || pw < 0) return false;
  const int RK = (S * C + 7) / 8 * 8;
  const int Kp = (R * RK + 31) / 32 * 32;
  if (Kp > 256) return false;
  // the segment a block stages: columns (ow0*sw - pw) .. ((ow0+PT-1)*sw - pw + S - 1), plus the
  // slack of the last fragment (j0 + 7 < RK) which reads at most RK - S*C elements past the run
  const int SEG = ((pa::stem::PT - 1) * sw + S) * C + RK;
  if ((long long)R * SEG * 2 > 64 * 1024) return false;
  g = pa::stem::Geo{H, W, C, Ho, Wo, Cout, R, S, sh, sw, ph, pw, RK, Kp, SEG};
  return true;
}

PA_API int pa_conv_stem_ok(int C, int Cout, int R, int S, int sh, int sw) {
  pa::stem::Geo g;
  return stem_geo(16, 16, C, 1, 1, Cout, R, S, sh, sw, 0, 0, g) ? 1 : 0;
}

// K extent of the packed filter image ([Cout][Kp], k = r * RK + s * C + c, zeros elsewhere)
PA_API int pa_conv_stem_kp(int C, int R, int S) { return (R * ((S * C + 7) / 8 * 8) + 31) / 32 * 32; }
PA_API int pa_conv_stem_rk(int C, int S) { return (S * C + 7) / 8 * 8; }

// x [N,H,W,C] (16-bit), wimg [Cout][Kp], bias [Cout] or null -> y [N,Ho,Wo,Cout]; dilation 1
PA_API hipError_t pa_conv_stem_fwd(const void* x, const void* wimg, const void* bias, void* y, int N, int H, int W,
                                   int C, int Cout, int R, int S, int sh, int sw, int ph, int pw, int Ho, int Wo,
                                   int dt, hipStream_t st) {
  pa::stem::Geo g;
  if (N <= 0 || !stem_geo(H, W, C, Ho, Wo, Cout, R, S, sh, sw, ph, pw, g)) return hipErrorInvalidValue;
  if ((long long)N * Ho > 2147483647LL) return hipErrorInvalidValue;
  const dim3 grid((Wo + pa::stem::PT - 1) / pa::stem::PT, N * Ho, Cout / pa::stem::CT);
  const size_t lds = (size_t)R * g.SEG * 2;
  const int ks = g.Kp / 32;
#define PA_STEM_LAUNCH(T, K)                                                                                     \
  pa::stem::fwd_kernel<T, K><<<grid, 256, lds, st>>>((const uint16_t*)x, (const uint16_t*)wimg, (const T*)bias, \
                                                     (uint16_t*)y, g)
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
    default: return hipErrorInvalidValue;       \
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
