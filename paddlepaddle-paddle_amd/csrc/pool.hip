// Channels-last (NHWC) 2-D max pooling for gfx950.
//
// Reference: paddle/phi/kernels/funcs/pooling.cu (MaxPool2dWithIndex / KernelMaxPool2DGrad,
// NCHW-first, atomics-free backward through stored indices).
//
// MI355X design: both directions are pure HBM streams, so every thread owns one 16-byte
// channel vector (8 bf16) of one output (forward) or one input (backward) pixel:
//  * forward reads the window, writes the max and a one-byte window offset per element
//    (argmax; 1/2 the bytes of the output instead of torch's int64 indices),
//  * backward is a GATHER: each input pixel visits the <= ceil(k/s)^2 output windows that
//    cover it and adds dy where the stored offset points back at it — no atomics, no zero-fill
//    pass, deterministic, one 16-byte store per thread.
// ResNet50's 3x3/s2 stem pool (256x112x112x64 bf16): forward 0.29 -> 0.19-0.20 ms, forward +
// backward 1.15 -> 0.64 ms vs the library kernels (tools/pool_bench.py, profiles/pool_r1.log).
#include "common.h"

namespace pa {

template <typename T, int E> struct IdxPack;
template <> struct IdxPack<float, 4> { using V = uint32_t; };
template <> struct IdxPack<bf16_t, 8> { using V = uint2; };
template <> struct IdxPack<f16_t, 8> { using V = uint2; };

template <typename T>
__global__ __launch_bounds__(256) void maxpool_fwd_nhwc(const T* __restrict__ x, T* __restrict__ y,
                                                        uint8_t* __restrict__ idx, int H, int W, int C, int OH,
                                                        int OW, int kh, int kw, int sh, int sw, int ph, int pw,
                                                        int rows) {
  constexpr int E = 16 / sizeof(T);
  const int CV = C / E;
  const int q = blockIdx.x * 256 + threadIdx.x;  // (ow, channel vector) within one output row
  if (q >= OW * CV) return;
  const int cv = q % CV, ow = q / CV;
  for (int row = blockIdx.y; row < rows; row += gridDim.y) {  // row = n * OH + oh
    const int oh = row % OH;
    const long long n = row / OH;
    const long long t = (long long)row * OW * CV + q;
    float m[E];
    uint8_t a[E];
#pragma unroll
    for (int e = 0; e < E; ++e) { m[e] = -__builtin_inff(); a[e] = 0; }
    const int h0 = oh * sh - ph, w0 = ow * sw - pw;
    for (int i = 0; i < kh; ++i) {
      const int h = h0 + i;
      if (h < 0 || h >= H) continue;
      for (int j = 0; j < kw; ++j) {
        const int w = w0 + j;
        if (w < 0 || w >= W) continue;
        float v[E];
        load_f<T, E>(x + ((n * H + h) * W + w) * C + (long long)cv * E, v);
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if (v[e] > m[e] || (v[e] != v[e] && m[e] == m[e])) {  // first max wins; NaN propagates
            m[e] = v[e];
            a[e] = (uint8_t)(i * kw + j);
          }
        }
      }
    }
    store_f<T, E>(y + t * E, m);
    typename IdxPack<T, E>::V pk;
    __builtin_memcpy(&pk, a, E);
    *reinterpret_cast<typename IdxPack<T, E>::V*>(idx + t * E) = pk;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_nhwc(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                        T* __restrict__ dx, int H, int W, int C, int OH, int OW,
                                                        int kh, int kw, int sh, int sw, int ph, int pw,
                                                        int rows) {
  constexpr int E = 16 / sizeof(T);
  const int CV = C / E;
  const int q = blockIdx.x * 256 + threadIdx.x;  // (w, channel vector) within one input row
  if (q >= W * CV) return;
  const int cv = q % CV, w = q / CV;
  for (int row = blockIdx.y; row < rows; row += gridDim.y) {  // row = n * H + h
    const int h = row % H;
    const long long n = row / H;
    const long long t = (long long)row * W * CV + q;
    float acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.f;
    const int hl = h + ph - kh + 1, wl = w + pw - kw + 1;
    const int ohs = hl <= 0 ? 0 : (hl + sh - 1) / sh, ohe = min(OH - 1, (h + ph) / sh);
    const int ows = wl <= 0 ? 0 : (wl + sw - 1) / sw, owe = min(OW - 1, (w + pw) / sw);
    for (int oh = ohs; oh <= ohe; ++oh) {
      for (int ow = ows; ow <= owe; ++ow) {
        const long long o = ((n * OH + oh) * OW + ow) * C + (long long)cv * E;
        const typename IdxPack<T, E>::V pk = *reinterpret_cast<const typename IdxPack<T, E>::V*>(idx + o);
        uint8_t a[E];
        __builtin_memcpy(a, &pk, E);
        const int pos = (h - (oh * sh - ph)) * kw + (w - (ow * sw - pw));
        float g[E];
        load_f<T, E>(dy + o, g);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] += (a[e] == pos) ? g[e] : 0.f;
      }
    }
    store_f<T, E>(dx + t * E, acc);
  }
}

}  // namespace pa

using namespace pa;

static bool pool_args_ok(int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh, int sw, int ph, int pw,
                         int dt) {
  const int E = dt == 0 ? 4 : 8;
  if ((long long)N * (H > OH ? H : OH) >= (1LL << 31) || (long long)W * C >= (1LL << 31)) return false;
  return N > 0 && H > 0 && W > 0 && C > 0 && C % E == 0 && OH > 0 && OW > 0 && kh > 0 && kw > 0 && kh * kw <= 256 &&
         sh > 0 && sw > 0 && ph >= 0 && pw >= 0 && ph < kh && pw < kw && (OH - 1) * sh - ph < H &&
         (OW - 1) * sw - pw < W;
}

// x [N,H,W,C] -> y [N,OH,OW,C] + idx [N,OH,OW,C] (uint8 window offset of the max).
PA_API hipError_t pa_maxpool2d_nhwc_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, int OH, int OW,
                                        int kh, int kw, int sh, int sw, int ph, int pw, int dt, hipStream_t st) {
  if (!pool_args_ok(N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw, dt)) return hipErrorInvalidValue;
  PA_DISPATCH_DTYPE(dt, T, {
    const int q = OW * (C / (16 / (int)sizeof(T)));
    const dim3 grid((q + 255) / 256, min(N * OH, 65535));
    maxpool_fwd_nhwc<T><<<grid, 256, 0, st>>>((const T*)x, (T*)y, (uint8_t*)idx, H, W, C, OH, OW, kh, kw, sh, sw,
                                              ph, pw, N * OH);
  });
  return hipGetLastError();
}

// dy [N,OH,OW,C] + idx -> dx [N,H,W,C] (every element written).
PA_API hipError_t pa_maxpool2d_nhwc_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W, int C, int OH,
                                        int OW, int kh, int kw, int sh, int sw, int ph, int pw, int dt, hipStream_t st) {
  if (!pool_args_ok(N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw, dt)) return hipErrorInvalidValue;
  PA_DISPATCH_DTYPE(dt, T, {
    const int q = W * (C / (16 / (int)sizeof(T)));
    const dim3 grid((q + 255) / 256, min(N * H, 65535));
    maxpool_bwd_nhwc<T><<<grid, 256, 0, st>>>((const T*)dy, (const uint8_t*)idx, (T*)dx, H, W, C, OH, OW, kh, kw,
                                              sh, sw, ph, pw, N * H);
  });
  return hipGetLastError();
}
