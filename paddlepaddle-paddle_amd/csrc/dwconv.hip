// Channels-last (NHWC) depthwise 2-D convolution for gfx950: forward, data gradient, filter
// gradient (channel multiplier 1: groups == C_in == C_out, the MobileNet / EfficientNet /
// ShuffleNet form).
//
// Reference: paddle/phi/kernels/gpu/depthwise_conv.h (KernelDepthwiseConvSp / ...InputGradSp /
// ...FilterGradSp, NCHW-first with per-element atomics in the filter gradient).
//
// MI355X design: a depthwise convolution has no reduction over channels, so there is nothing for
// the MFMA units; all three passes are HBM streams with R*S-fold reuse that the caches serve.
//  * Every thread owns one 16-byte channel vector (8 bf16 / f16 channels) of one pixel, so every
//    load and store is a full 16-byte access and a wave touches 1 KiB of contiguous channels.
//  * Forward and data gradient are both GATHERS (the data gradient visits the output pixels whose
//    windows cover its input pixel): no atomics, no zero fill, deterministic.
//  * Filter gradient: each block reduces a contiguous range of output pixels for up to 9 taps of
//    its channel slice in registers, folds its pixel lanes through LDS, and writes one fp32 partial
//    row per (split, tap); a second kernel sums the splits in a fixed order (deterministic) into
//    the [C][1][R][S] filter gradient, optionally accumulating into an existing gradient.
#include "common.h"

namespace pa {
namespace dw {

constexpr int TAPS = 9;  // filter-gradient taps per block (3x3 in one pass; 5x5 / 7x7 in chunks)

struct Geo {
  int N, H, W, C, Ho, Wo, R, S, sh, sw, ph, pw, dh, dw;
};

// y[n, oh, ow, c] = sum_{r,s} x[n, oh*sh - ph + r*dh, ow*sw - pw + s*dw, c] * w[r*S + s][c] (+ b[c])
template <typename T>
__global__ __launch_bounds__(256) void fwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                  const T* __restrict__ bias, T* __restrict__ y, Geo g,
                                                  long long total) {
  constexpr int E = 16 / sizeof(T);
  const int CV = g.C / E;
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int cv = (int)(t % CV);
    const long long pix = t / CV;
    const int ow = (int)(pix % g.Wo);
    const long long nh = pix / g.Wo;
    const int oh = (int)(nh % g.Ho);
    const long long n = nh / g.Ho;
    float acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.f;
    if (bias != nullptr) load_f<T, E>(bias + cv * E, acc);
    const int h0 = oh * g.sh - g.ph, w0 = ow * g.sw - g.pw;
    for (int r = 0; r < g.R; ++r) {
      const int h = h0 + r * g.dh;
      if (h < 0 || h >= g.H) continue;
      const T* xrow = x + ((n * g.H + h) * g.W) * g.C + cv * E;
      for (int s = 0; s < g.S; ++s) {
        const int ww = w0 + s * g.dw;
        if (ww < 0 || ww >= g.W) continue;
        float xv[E], wv[E];
        load_f<T, E>(xrow + (long long)ww * g.C, xv);
        load_f<T, E>(w + (long long)(r * g.S + s) * g.C + cv * E, wv);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = __builtin_fmaf(xv[e], wv[e], acc[e]);
      }
    }
    store_f<T, E>(y + t * E, acc);
  }
}

// dx[n, ih, iw, c] = sum over (r, s) with oh = (ih + ph - r*dh) / sh integral and in range (same
// for ow) of dy[n, oh, ow, c] * w[r*S + s][c]
template <typename T>
__global__ __launch_bounds__(256) void dgrad_kernel(const T* __restrict__ dy, const T* __restrict__ w,
                                                    T* __restrict__ dx, Geo g, long long total) {
  constexpr int E = 16 / sizeof(T);
  const int CV = g.C / E;
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int cv = (int)(t % CV);
    const long long pix = t / CV;
    const int iw = (int)(pix % g.W);
    const long long nh = pix / g.W;
    const int ih = (int)(nh % g.H);
    const long long n = nh / g.H;
    float acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.f;
    for (int r = 0; r < g.R; ++r) {
      const int hh = ih + g.ph - r * g.dh;
      if (hh < 0 || hh % g.sh != 0) continue;
      const int oh = hh / g.sh;
      if (oh >= g.Ho) continue;
      const T* dyrow = dy + ((n * g.Ho + oh) * g.Wo) * g.C + cv * E;
      for (int s = 0; s < g.S; ++s) {
        const int ww = iw + g.pw - s * g.dw;
        if (ww < 0 || ww % g.sw != 0) continue;
        const int ow = ww / g.sw;
        if (ow >= g.Wo) continue;
        float gv[E], wv[E];
        load_f<T, E>(dyrow + (long long)ow * g.C, gv);
        load_f<T, E>(w + (long long)(r * g.S + s) * g.C + cv * E, wv);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = __builtin_fmaf(gv[e], wv[e], acc[e]);
      }
    }
    store_f<T, E>(dx + t * E, acc);
  }
}

// Filter-gradient partials.  grid (splits, tap chunks, channel-vector chunks); block = PL pixel
// lanes x CVB channel vectors.  ws[split][tap][c] (fp32).
template <typename T>
__global__ __launch_bounds__(256) void wgrad_part_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                         float* __restrict__ ws, Geo g, int CVB, long long per) {
  constexpr int E = 16 / sizeof(T);
  __shared__ float red[256 * E];
  const int PL = 256 / CVB;
  const int lanev = threadIdx.x % CVB, pl = threadIdx.x / CVB;
  const int cv = blockIdx.z * CVB + lanev;
  const int CV = g.C / E;
  const int RS = g.R * g.S;
  const int t0 = blockIdx.y * TAPS;
  const int nt = min(TAPS, RS - t0);
  const long long P = (long long)g.N * g.Ho * g.Wo;
  const long long p0 = (long long)blockIdx.x * per, p1 = min(P, p0 + per);
  const bool live = pl < PL && cv < CV;
  float acc[TAPS][E];
#pragma unroll
  for (int k = 0; k < TAPS; ++k)
#pragma unroll
    for (int e = 0; e < E; ++e) acc[k][e] = 0.f;
  if (live) {
    for (long long p = p0 + pl; p < p1; p += PL) {
      const int ow = (int)(p % g.Wo);
      const long long nh = p / g.Wo;
      const int oh = (int)(nh % g.Ho);
      const long long n = nh / g.Ho;
      float gv[E];
      load_f<T, E>(dy + p * g.C + cv * E, gv);
      const int h0 = oh * g.sh - g.ph, w0 = ow * g.sw - g.pw;
#pragma unroll
      for (int k = 0; k < TAPS; ++k) {
        if (k < nt) {
          const int tap = t0 + k;
          const int r = tap / g.S, s = tap - r * g.S;
          const int h = h0 + r * g.dh, ww = w0 + s * g.dw;
          if (h >= 0 && h < g.H && ww >= 0 && ww < g.W) {
            float xv[E];
            load_f<T, E>(x + ((n * g.H + h) * g.W + ww) * g.C + cv * E, xv);
#pragma unroll
            for (int e = 0; e < E; ++e) acc[k][e] = __builtin_fmaf(gv[e], xv[e], acc[k][e]);
          }
        }
      }
    }
  }
  // fold the pixel lanes: one tap at a time through LDS
  const long long split = blockIdx.x;
#pragma unroll
  for (int k = 0; k < TAPS; ++k) {
    if (k >= nt) continue;  // block-uniform
#pragma unroll
    for (int e = 0; e < E; ++e) red[threadIdx.x * E + e] = acc[k][e];
    __syncthreads();
    if (pl == 0 && cv < CV) {
      float sum[E];
#pragma unroll
      for (int e = 0; e < E; ++e) sum[e] = red[lanev * E + e];
      for (int q = 1; q < PL; ++q)
#pragma unroll
        for (int e = 0; e < E; ++e) sum[e] += red[(q * CVB + lanev) * E + e];
      float* dst = ws + (split * RS + t0 + k) * g.C + cv * E;
#pragma unroll
      for (int e = 0; e < E; ++e) dst[e] = sum[e];
    }
    __syncthreads();
  }
}

// dw[c][0][r][s] (+)= sum_split ws[split][r*S + s][c]  (fixed split order: deterministic)
template <typename T>
__global__ __launch_bounds__(256) void wgrad_finish_kernel(const float* __restrict__ ws, T* __restrict__ dw, int C,
                                                           int RS, int splits, int accum) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // i = tap * C + c (coalesced partial reads)
  if (i >= RS * C) return;
  const int tap = i / C, c = i - tap * C;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += ws[(long long)k * RS * C + i];
  T* o = dw + (long long)c * RS + tap;
  if (accum) s += to_f(*o);
  *o = from_f<T>(s);
}

}  // namespace dw
}  // namespace pa

using namespace pa;
using pa::dw::Geo;

static bool dw_geo_ok(const Geo& g, int dt) {
  if (dt != 1 && dt != 2) return false;  // 16-bit activations (8 channels per 16-byte vector)
  if (g.N <= 0 || g.H <= 0 || g.W <= 0 || g.C <= 0 || g.C % 8 != 0 || g.Ho <= 0 || g.Wo <= 0) return false;
  if (g.R <= 0 || g.S <= 0 || g.R * g.S > 64 || g.sh <= 0 || g.sw <= 0 || g.dh <= 0 || g.dw <= 0) return false;
  if (g.ph < 0 || g.pw < 0) return false;  // every tap access is bounds-checked in the kernels
  return (long long)g.N * g.H * g.W * g.C < (1LL << 40);
}

static Geo mkgeo(int N, int H, int W, int C, int Ho, int Wo, int R, int S, int sh, int sw, int ph, int pw, int dh,
                 int dwd) {
  return Geo{N, H, W, C, Ho, Wo, R, S, sh, sw, ph, pw, dh, dwd};
}

static int grid_for(long long total) {
  long long b = (total + 255) / 256;
  return (int)(b < 65536 ? b : 65536);
}

PA_API int pa_dwconv_ok(int N, int H, int W, int C, int Ho, int Wo, int R, int S, int sh, int sw, int ph, int pw,
                        int dh, int dwd, int dt) {
  return dw_geo_ok(mkgeo(N, H, W, C, Ho, Wo, R, S, sh, sw, ph, pw, dh, dwd), dt) ? 1 : 0;
}

// x [N,H,W,C], w [R*S][C] (tap-major), bias [C] or null -> y [N,Ho,Wo,C]
PA_API hipError_t pa_dwconv_fwd(const void* x, const void* w, const void* bias, void* y, int N, int H, int W, int C,
                                int Ho, int Wo, int R, int S, int sh, int sw, int ph, int pw, int dh, int dwd, int dt,
                                hipStream_t st) {
  const Geo g = mkgeo(N, H, W, C, Ho, Wo, R, S, sh, sw, ph, pw, dh, dwd);
  if (!dw_geo_ok(g, dt)) return hipErrorInvalidValue;
  const long long total = (long long)N * Ho * Wo * (C / 8);
  PA_DISPATCH_DTYPE(dt, T, {
    dw::fwd_kernel<T><<<grid_for(total), 256, 0, st>>>((const T*)x, (const T*)w, (const T*)bias, (T*)y, g, total);
  });
  return hipGetLastError();
}

// dy [N,Ho,Wo,C], w [R*S][C] -> dx [N,H,W,C] (every element written)
PA_API hipError_t pa_dwconv_dgrad(const void* dy, const void* w, void* dx, int N, int H, int W, int C, int Ho, int Wo,
                                  int R, int S, int sh, int sw, int ph, int pw, int dh, int dwd, int dt,
                                  hipStream_t st) {
  const Geo g = mkgeo(N, H, W, C, Ho, Wo, R, S, sh, sw, ph, pw, dh, dwd);
  if (!dw_geo_ok(g, dt)) return hipErrorInvalidValue;
  const long long total = (long long)N * H * W * (C / 8);
  PA_DISPATCH_DTYPE(dt, T, {
    dw::dgrad_kernel<T><<<grid_for(total), 256, 0, st>>>((const T*)dy, (const T*)w, (T*)dx, g, total);
  });
  return hipGetLastError();
}

// splits of the filter-gradient pixel reduction (workspace: splits * R*S * C floats)
PA_API int pa_dwconv_wgrad_splits(int N, int Ho, int Wo, int C, int R, int S) {
  const long long P = (long long)N * Ho * Wo;
  const int CV = C / 8, CVB = CV < 64 ? CV : 64;
  const int zc = (CV + CVB - 1) / CVB, tc = (R * S + dw::TAPS - 1) / dw::TAPS;
  const int PL = 256 / CVB;
  long long want = 1024 / ((long long)zc * tc);  // ~4 blocks per CU
  const long long maxs = (P + 4LL * PL - 1) / (4LL * PL);  // at least 4 pixels per lane
  if (want > maxs) want = maxs;
  if (want < 1) want = 1;
  return (int)want;
}

// x [N,H,W,C], dy [N,Ho,Wo,C] -> dw [C][1][R][S] (accum: added to its contents); ws >= splits*R*S*C floats
PA_API hipError_t pa_dwconv_wgrad(const void* x, const void* dy, float* ws, void* dwout, int N, int H, int W, int C,
                                  int Ho, int Wo, int R, int S, int sh, int sw, int ph, int pw, int dh, int dwd,
                                  int splits, int accum, int dt, hipStream_t st) {
  const Geo g = mkgeo(N, H, W, C, Ho, Wo, R, S, sh, sw, ph, pw, dh, dwd);
  if (!dw_geo_ok(g, dt) || splits <= 0) return hipErrorInvalidValue;
  const long long P = (long long)N * Ho * Wo;
  const int CV = C / 8, CVB = CV < 64 ? CV : 64;
  const long long per = (P + splits - 1) / splits;
  const dim3 grid(splits, (R * S + dw::TAPS - 1) / dw::TAPS, (CV + CVB - 1) / CVB);
  PA_DISPATCH_DTYPE(dt, T, {
    dw::wgrad_part_kernel<T><<<grid, 256, 0, st>>>((const T*)x, (const T*)dy, ws, g, CVB, per);
    dw::wgrad_finish_kernel<T><<<(R * S * C + 255) / 256, 256, 0, st>>>(ws, (T*)dwout, C, R * S, splits, accum);
  });
  return hipGetLastError();
}
