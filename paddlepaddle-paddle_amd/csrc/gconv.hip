// Channels-last (NHWC) GROUPED 2-D convolution for gfx950 (1 < groups < C_in, the ResNeXt /
// ShuffleNet-v1 form): forward, data gradient, filter gradient.  Depthwise (groups == C_in) has its
// own kernels in dwconv.hip; groups == 1 runs on the implicit-GEMM MFMA kernels of conv.hip.
//
// Reference: paddle/phi/kernels/gpudnn/conv_kernel.cu / conv_grad_kernel.cu (cuDNN / MIOpen with
// groups) — the reference has no hand-written grouped kernel.
//
// MI355X design: a group reduces over only Cg = C_in / groups input channels (4..32 in ResNeXt:
// 32 groups x 4..32 channels), far below the 32-deep K slices the MFMA conv needs, so these are
// VALU kernels that stream HBM with the tap reuse served by L1/L2:
//  * forward: a thread owns 8 (4 when C_out / groups = 4) consecutive output channels of one pixel; per tap
//    it reads the group's Cg input channels as 16- (or 8-) byte vectors and the [tap][ci][co]
//    filter image rows (16-byte loads of 8 output channels), fp32 FMAs;
//  * data gradient: a GATHER (no atomics): a thread owns EO input channels of one input pixel and
//    visits the output pixels whose windows cover it, reading the [tap][co][ci] filter image;
//  * filter gradient: blocks reduce a contiguous pixel range for up to 9 taps of (8 output
//    channels, 1 input channel) roles in registers, fold their pixel lanes through LDS and write
//    fp32 partials per split; a finish kernel sums the splits in a fixed order (deterministic).
#include "common.h"

namespace pa {
namespace gc {

constexpr int TAPS = 9;

struct Geo {
  int N, H, W, C, Ho, Wo, Cout, R, S, sh, sw, ph, pw, dh, dw;
  int Cg, Cog;  // input / output channels per group
};

// y[n,oh,ow,co] = sum_{r,s,ci} x[n, oh*sh-ph+r*dh, ow*sw-pw+s*dw, grp*Cg + ci] * wf[r*S+s][ci][co]
template <typename T, int EI, int EV>
__global__ __launch_bounds__(256) void fwd_kernel(const T* __restrict__ x, const T* __restrict__ wf,
                                                  const T* __restrict__ bias, T* __restrict__ y, Geo g,
                                                  long long total) {
  const int CV = g.Cout / EV;
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int cv = (int)(t % CV);
    const long long pix = t / CV;
    const int ow = (int)(pix % g.Wo);
    const long long nh = pix / g.Wo;
    const int oh = (int)(nh % g.Ho);
    const long long n = nh / g.Ho;
    const int co0 = cv * EV;
    const int ci0 = (co0 / g.Cog) * g.Cg;
    float acc[EV];
#pragma unroll
    for (int e = 0; e < EV; ++e) acc[e] = 0.f;
    if (bias != nullptr) load_f<T, EV>(bias + co0, acc);
    const int h0 = oh * g.sh - g.ph, w0 = ow * g.sw - g.pw;
    for (int r = 0; r < g.R; ++r) {
      const int h = h0 + r * g.dh;
      if (h < 0 || h >= g.H) continue;
      for (int s = 0; s < g.S; ++s) {
        const int ww = w0 + s * g.dw;
        if (ww < 0 || ww >= g.W) continue;
        const T* xp = x + ((n * g.H + h) * g.W + ww) * g.C + ci0;
        const T* wp = wf + (long long)(r * g.S + s) * g.Cg * g.Cout + co0;
        for (int ci = 0; ci < g.Cg; ci += EI) {
          float xv[EI];
          load_f<T, EI>(xp + ci, xv);
#pragma unroll
          for (int k = 0; k < EI; ++k) {
            float wv[EV];
            load_f<T, EV>(wp + (long long)(ci + k) * g.Cout, wv);
#pragma unroll
            for (int e = 0; e < EV; ++e) acc[e] = __builtin_fmaf(xv[k], wv[e], acc[e]);
          }
        }
      }
    }
    store_f<T, EV>(y + t * EV, acc);
  }
}

// dx[n,ih,iw,ci] = sum over covering (r, s) and the group's output channels co of
// dy[n,oh,ow,co] * wd[r*S+s][co][ci - grp*Cg]
template <typename T, int EO, int EV>
__global__ __launch_bounds__(256) void dgrad_kernel(const T* __restrict__ dy, const T* __restrict__ wd,
                                                    T* __restrict__ dx, Geo g, long long total) {
  const int CV = g.C / EO;
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int cv = (int)(t % CV);
    const long long pix = t / CV;
    const int iw = (int)(pix % g.W);
    const long long nh = pix / g.W;
    const int ih = (int)(nh % g.H);
    const long long n = nh / g.H;
    const int c0 = cv * EO;
    const int grp = c0 / g.Cg, cil = c0 - grp * g.Cg;
    const int co0 = grp * g.Cog;
    float acc[EO];
#pragma unroll
    for (int e = 0; e < EO; ++e) acc[e] = 0.f;
    for (int r = 0; r < g.R; ++r) {
      const int hh = ih + g.ph - r * g.dh;
      if (hh < 0 || hh % g.sh != 0) continue;
      const int oh = hh / g.sh;
      if (oh >= g.Ho) continue;
      for (int s = 0; s < g.S; ++s) {
        const int ww = iw + g.pw - s * g.dw;
        if (ww < 0 || ww % g.sw != 0) continue;
        const int ow = ww / g.sw;
        if (ow >= g.Wo) continue;
        const T* dp = dy + ((n * g.Ho + oh) * g.Wo + ow) * g.Cout + co0;
        const T* wp = wd + ((long long)(r * g.S + s) * g.Cout + co0) * g.Cg + cil;
        for (int co = 0; co < g.Cog; co += EV) {
          float gv[EV];
          load_f<T, EV>(dp + co, gv);
#pragma unroll
          for (int k = 0; k < EV; ++k) {
            float wv[EO];
            load_f<T, EO>(wp + (long long)(co + k) * g.Cg, wv);
#pragma unroll
            for (int e = 0; e < EO; ++e) acc[e] = __builtin_fmaf(gv[k], wv[e], acc[e]);
          }
        }
      }
    }
    store_f<T, EO>(dx + t * EO, acc);
  }
}

// Filter-gradient partials.  Role rl = ci + Cg * cv (8 output channels cv*8.., input channel ci of
// their group); grid (splits, tap chunks, role chunks); block = PL pixel lanes x RB roles.
// ws[split][tap][rl][8] (fp32).
template <typename T, int EV>
__global__ __launch_bounds__(256) void wgrad_part_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                         float* __restrict__ ws, Geo g, int RB, long long per) {
  __shared__ float red[256 * EV];
  const int NR = (g.Cout / EV) * g.Cg;
  const int PL = 256 / RB;
  const int lr = threadIdx.x % RB, pl = threadIdx.x / RB;
  const int rl = blockIdx.z * RB + lr;
  const int RS = g.R * g.S;
  const int t0 = blockIdx.y * TAPS;
  const int nt = min(TAPS, RS - t0);
  const long long P = (long long)g.N * g.Ho * g.Wo;
  const long long p0 = (long long)blockIdx.x * per, p1 = min(P, p0 + per);
  const bool live = pl < PL && rl < NR;
  const int cv = live ? rl / g.Cg : 0, ci = live ? rl - cv * g.Cg : 0;
  const int cx = (cv * EV / g.Cog) * g.Cg + ci;  // input channel
  float acc[TAPS][EV];
#pragma unroll
  for (int k = 0; k < TAPS; ++k)
#pragma unroll
    for (int e = 0; e < EV; ++e) acc[k][e] = 0.f;
  if (live) {
    for (long long p = p0 + pl; p < p1; p += PL) {
      const int ow = (int)(p % g.Wo);
      const long long nh = p / g.Wo;
      const int oh = (int)(nh % g.Ho);
      const long long n = nh / g.Ho;
      float gv[EV];
      load_f<T, EV>(dy + p * g.Cout + cv * EV, gv);
      const int h0 = oh * g.sh - g.ph, w0 = ow * g.sw - g.pw;
#pragma unroll
      for (int k = 0; k < TAPS; ++k) {
        if (k < nt) {
          const int tap = t0 + k;
          const int r = tap / g.S, s = tap - r * g.S;
          const int h = h0 + r * g.dh, ww = w0 + s * g.dw;
          if (h >= 0 && h < g.H && ww >= 0 && ww < g.W) {
            const float xv = to_f(x[((n * g.H + h) * g.W + ww) * g.C + cx]);
#pragma unroll
            for (int e = 0; e < EV; ++e) acc[k][e] = __builtin_fmaf(gv[e], xv, acc[k][e]);
          }
        }
      }
    }
  }
  const long long split = blockIdx.x;
#pragma unroll
  for (int k = 0; k < TAPS; ++k) {
    if (k >= nt) continue;  // block-uniform
#pragma unroll
    for (int e = 0; e < EV; ++e) red[threadIdx.x * EV + e] = acc[k][e];
    __syncthreads();
    if (pl == 0 && rl < NR) {
      float sum[EV];
#pragma unroll
      for (int e = 0; e < EV; ++e) sum[e] = red[lr * EV + e];
      for (int q = 1; q < PL; ++q)
#pragma unroll
        for (int e = 0; e < EV; ++e) sum[e] += red[(q * RB + lr) * EV + e];
      float* dst = ws + ((split * RS + t0 + k) * NR + rl) * EV;
#pragma unroll
      for (int e = 0; e < EV; ++e) dst[e] = sum[e];
    }
    __syncthreads();
  }
}

// dw[co][ci][r][s] (+)= sum_split ws[split][tap][rl][e], co = EV cv + e, rl = ci + Cg cv
template <typename T, int EV>
__global__ __launch_bounds__(256) void wgrad_finish_kernel(const float* __restrict__ ws, T* __restrict__ dw, int Cout,
                                                           int Cg, int RS, int splits, int accum) {
  const long long NR8 = (long long)(Cout / EV) * Cg * EV;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;  // i = tap * NR8 + rl * EV + e
  if (i >= RS * NR8) return;
  const int tap = (int)(i / NR8);
  const int rem = (int)(i - tap * NR8);
  const int rl = rem / EV, e = rem - rl * EV;
  const int cv = rl / Cg, ci = rl - cv * Cg;
  const int co = cv * EV + e;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += ws[(long long)k * RS * NR8 + i];
  T* o = dw + ((long long)co * Cg + ci) * RS + tap;
  if (accum) s += to_f(*o);
  *o = from_f<T>(s);
}

}  // namespace gc
}  // namespace pa

using namespace pa;
using pa::gc::Geo;

static bool gc_geo_ok(const Geo& g, int dt) {
  if (dt != 1 && dt != 2) return false;
  if (g.N <= 0 || g.H <= 0 || g.W <= 0 || g.C <= 0 || g.Cout <= 0 || g.Ho <= 0 || g.Wo <= 0) return false;
  if (g.Cg <= 0 || g.Cog <= 0 || g.C % g.Cg || g.Cout % g.Cog || g.C / g.Cg != g.Cout / g.Cog) return false;
  if (g.Cg % 4 != 0 || g.Cog % 4 != 0) return false;  // vector widths of the three kernels (8 or 4)
  if (g.R <= 0 || g.S <= 0 || g.R * g.S > 64 || g.sh <= 0 || g.sw <= 0 || g.dh <= 0 || g.dw <= 0) return false;
  if (g.ph < 0 || g.pw < 0) return false;
  return (long long)g.N * g.H * g.W * g.C < (1LL << 40) && (long long)g.N * g.Ho * g.Wo * g.Cout < (1LL << 40);
}

static Geo mkgeo(int N, int H, int W, int C, int Ho, int Wo, int Cout, int G, int R, int S, int sh, int sw, int ph,
                 int pw, int dh, int dwd) {
  return Geo{N, H, W, C, Ho, Wo, Cout, R, S, sh, sw, ph, pw, dh, dwd, G > 0 ? C / G : 0, G > 0 ? Cout / G : 0};
}

static int gc_grid(long long total) {
  long long b = (total + 255) / 256;
  return (int)(b < 65536 ? b : 65536);
}

PA_API int pa_gconv_ok(int N, int H, int W, int C, int Ho, int Wo, int Cout, int G, int R, int S, int sh, int sw,
                       int ph, int pw, int dh, int dwd, int dt) {
  if (G <= 1 || C % G || Cout % G) return 0;
  return gc_geo_ok(mkgeo(N, H, W, C, Ho, Wo, Cout, G, R, S, sh, sw, ph, pw, dh, dwd), dt) ? 1 : 0;
}

// x [N,H,W,C], wf [R*S][Cg][Cout], bias [Cout] or null -> y [N,Ho,Wo,Cout]
PA_API hipError_t pa_gconv_fwd(const void* x, const void* wf, const void* bias, void* y, int N, int H, int W, int C,
                               int Ho, int Wo, int Cout, int G, int R, int S, int sh, int sw, int ph, int pw, int dh,
                               int dwd, int dt, hipStream_t st) {
  if (!pa_gconv_ok(N, H, W, C, Ho, Wo, Cout, G, R, S, sh, sw, ph, pw, dh, dwd, dt)) return hipErrorInvalidValue;
  const Geo g = mkgeo(N, H, W, C, Ho, Wo, Cout, G, R, S, sh, sw, ph, pw, dh, dwd);
  const int ev = g.Cog % 8 == 0 ? 8 : 4;
  const long long total = (long long)N * Ho * Wo * (Cout / ev);
#define PA_GC_FWD(EI, EV) \
  gc::fwd_kernel<T, EI, EV><<<gc_grid(total), 256, 0, st>>>((const T*)x, (const T*)wf, (const T*)bias, (T*)y, g, total)
  PA_DISPATCH_DTYPE(dt, T, {
    if (g.Cg % 8 == 0) {
      if (ev == 8) PA_GC_FWD(8, 8); else PA_GC_FWD(8, 4);
    } else {
      if (ev == 8) PA_GC_FWD(4, 8); else PA_GC_FWD(4, 4);
    }
  });
#undef PA_GC_FWD
  return hipGetLastError();
}

// dy [N,Ho,Wo,Cout], wd [R*S][Cout][Cg] -> dx [N,H,W,C] (every element written)
PA_API hipError_t pa_gconv_dgrad(const void* dy, const void* wd, void* dx, int N, int H, int W, int C, int Ho, int Wo,
                                 int Cout, int G, int R, int S, int sh, int sw, int ph, int pw, int dh, int dwd, int dt,
                                 hipStream_t st) {
  if (!pa_gconv_ok(N, H, W, C, Ho, Wo, Cout, G, R, S, sh, sw, ph, pw, dh, dwd, dt)) return hipErrorInvalidValue;
  const Geo g = mkgeo(N, H, W, C, Ho, Wo, Cout, G, R, S, sh, sw, ph, pw, dh, dwd);
  const int eo = g.Cg % 8 == 0 ? 8 : 4, ev = g.Cog % 8 == 0 ? 8 : 4;
  const long long total = (long long)N * H * W * (C / eo);
#define PA_GC_DG(EO, EV) \
  gc::dgrad_kernel<T, EO, EV><<<gc_grid(total), 256, 0, st>>>((const T*)dy, (const T*)wd, (T*)dx, g, total)
  PA_DISPATCH_DTYPE(dt, T, {
    if (eo == 8) {
      if (ev == 8) PA_GC_DG(8, 8); else PA_GC_DG(8, 4);
    } else {
      if (ev == 8) PA_GC_DG(4, 8); else PA_GC_DG(4, 4);
    }
  });
#undef PA_GC_DG
  return hipGetLastError();
}

static void wgrad_shape(int Cout, int Cg, int Cog, int RS, int& NR, int& RB, int& zc, int& tc) {
  NR = (Cout / (Cog % 8 == 0 ? 8 : 4)) * Cg;
  RB = NR < 256 ? NR : 256;
  zc = (NR + RB - 1) / RB;
  tc = (RS + gc::TAPS - 1) / gc::TAPS;
}

// splits of the filter-gradient pixel reduction (workspace: splits * R*S * Cout * Cg floats)
PA_API int pa_gconv_wgrad_splits(int N, int Ho, int Wo, int Cout, int G, int R, int S, int C) {
  if (G <= 0 || C % G || Cout % G) return 1;
  int NR, RB, zc, tc;
  wgrad_shape(Cout, C / G, Cout / G, R * S, NR, RB, zc, tc);
  const long long P = (long long)N * Ho * Wo;
  const int PL = 256 / RB;
  long long want = 1024 / ((long long)zc * tc);
  const long long maxs = (P + 8LL * PL - 1) / (8LL * PL);  // at least 8 pixels per lane
  if (want > maxs) want = maxs;
  // partial workspace bounded to 64 Mi floats
  const long long per_split = (long long)R * S * Cout * (C / G);
  if (per_split > 0 && want * per_split > (64LL << 20)) want = (64LL << 20) / per_split;
  if (want < 1) want = 1;
  return (int)want;
}

// x [N,H,W,C], dy [N,Ho,Wo,Cout] -> dw [Cout][Cg][R][S] (accum: added); ws >= splits*R*S*Cout*Cg floats
PA_API hipError_t pa_gconv_wgrad(const void* x, const void* dy, float* ws, void* dwout, int N, int H, int W, int C,
                                 int Ho, int Wo, int Cout, int G, int R, int S, int sh, int sw, int ph, int pw, int dh,
                                 int dwd, int splits, int accum, int dt, hipStream_t st) {
  if (!pa_gconv_ok(N, H, W, C, Ho, Wo, Cout, G, R, S, sh, sw, ph, pw, dh, dwd, dt) || splits <= 0)
    return hipErrorInvalidValue;
  const Geo g = mkgeo(N, H, W, C, Ho, Wo, Cout, G, R, S, sh, sw, ph, pw, dh, dwd);
  int NR, RB, zc, tc;
  wgrad_shape(Cout, g.Cg, g.Cog, R * S, NR, RB, zc, tc);
  const int ev = g.Cog % 8 == 0 ? 8 : 4;
  const long long P = (long long)N * Ho * Wo;
  const long long per = (P + splits - 1) / splits;
  const dim3 grid(splits, tc, zc);
  const long long nout = (long long)R * S * NR * ev;
  const unsigned fb = (unsigned)((nout + 255) / 256);
  PA_DISPATCH_DTYPE(dt, T, {
    if (ev == 8) {
      gc::wgrad_part_kernel<T, 8><<<grid, 256, 0, st>>>((const T*)x, (const T*)dy, ws, g, RB, per);
      gc::wgrad_finish_kernel<T, 8><<<fb, 256, 0, st>>>(ws, (T*)dwout, Cout, g.Cg, R * S, splits, accum);
    } else {
      gc::wgrad_part_kernel<T, 4><<<grid, 256, 0, st>>>((const T*)x, (const T*)dy, ws, g, RB, per);
      gc::wgrad_finish_kernel<T, 4><<<fb, 256, 0, st>>>(ws, (T*)dwout, Cout, g.Cg, R * S, splits, accum);
    }
  });
  return hipGetLastError();
}
