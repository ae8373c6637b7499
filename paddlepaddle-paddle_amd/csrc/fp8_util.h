// fp8 (OCP e4m3fn / e5m2) conversion and delayed-scaling helpers shared by the cast kernels
// (fp8_cast.hip) and the GEMM epilogues that quantise their output (gemm8_impl.h EPI 210 / 211).
#pragma once
#include "common.h"

namespace pa {
namespace f8 {

template <int FMT>
__device__ __forceinline__ float fmax_of() { return FMT == 0 ? 448.f : 57344.f; }

// two floats -> two fp8 bytes (low 16 bits of the result), saturating (clamped before the cvt)
template <int FMT>
__device__ __forceinline__ uint32_t cvt2(float a, float b) {
  const float m = fmax_of<FMT>();
  a = fminf(fmaxf(a, -m), m);
  b = fminf(fmaxf(b, -m), m);
  if constexpr (FMT == 0)
    return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false) & 0xFFFFu;
  else
    return (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false) & 0xFFFFu;
}

__device__ __forceinline__ float scale_from_hist(const float* __restrict__ hist, int L, int cur, float fmax,
                                                 float margin_mul) {
  float am = 0.f;
  const int nxt = (cur + 1) % L;
  for (int j = 0; j < L; ++j)
    if (j != cur && j != nxt) am = fmaxf(am, hist[j]);
  if (!(am > 0.f) || !isfinite(am)) return 1.f;
  const float s = fmax / am * margin_mul;
  return isfinite(s) ? s : 1.f;
}

__device__ __forceinline__ void atomic_max_pos(float* addr, float v) {
  atomicMax(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

}  // namespace f8
}  // namespace pa
