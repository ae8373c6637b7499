// Flash attention for head_dim 96 and 256 (reference: python/paddle/nn/functional/flash_attention.py
// accepts head dims up to 256; paddle/phi/kernels/gpu/flash_attn_kernel.cu).  Same kernels as
// flash_attn.hip (flash_attn_kernels.h), instantiated in their own module so the head_dim 64/128
// code objects are not perturbed (cdna_hip_programming rule 19):
//  * D = 96: 3 k-steps / 6 d-blocks of MFMA work (no zero padding to 128); the LDS tiles keep
//    the 256-byte D = 128 row pitch so the XOR swizzles stay within a row (fa_pitch).
//  * D = 256: 8 k-steps / 16 d-blocks; the O / dK / dV accumulators (64-128 VGPRs per wave) need
//    the whole register file, so these kernels run one wave per SIMD (launch bounds min 1) with
//    4-wave blocks in every direction.
// Entry points are reached through pa_flash_fwd / pa_flash_bwd / *_ex (flash_attn.hip) when
// D is 96 or 256.
#define PA_FA_PAIR_GROUP_DECL static __constant__
#include "flash_attn_kernels.h"

using namespace pa;
using namespace pa::fa;

#define FAW_DISPATCH(dt, D, causal, ...)                                                                           \
  if (dt == 1 && D == 256 && causal) { using T = bf16_t; constexpr int DD = 256; constexpr bool CC = true; __VA_ARGS__; }        \
  else if (dt == 1 && D == 256 && !causal) { using T = bf16_t; constexpr int DD = 256; constexpr bool CC = false; __VA_ARGS__; } \
  else if (dt == 1 && D == 96 && causal) { using T = bf16_t; constexpr int DD = 96; constexpr bool CC = true; __VA_ARGS__; }     \
  else if (dt == 1 && D == 96 && !causal) { using T = bf16_t; constexpr int DD = 96; constexpr bool CC = false; __VA_ARGS__; }   \
  else if (dt == 2 && D == 256 && causal) { using T = f16_t; constexpr int DD = 256; constexpr bool CC = true; __VA_ARGS__; }    \
  else if (dt == 2 && D == 256 && !causal) { using T = f16_t; constexpr int DD = 256; constexpr bool CC = false; __VA_ARGS__; }  \
  else if (dt == 2 && D == 96 && causal) { using T = f16_t; constexpr int DD = 96; constexpr bool CC = true; __VA_ARGS__; }      \
  else if (dt == 2 && D == 96 && !causal) { using T = f16_t; constexpr int DD = 96; constexpr bool CC = false; __VA_ARGS__; }    \
  else return hipErrorInvalidValue;

namespace pa {
namespace fa {

int wide_set_pair_group(int v) {
  int old = 0;
  (void)hipMemcpyFromSymbol(&old, HIP_SYMBOL(g_pair_group), sizeof(int));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pair_group), &v, sizeof(int));
  return old;
}

int wide_set_rng_gen(const void* p) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(pa::g_rng_gen), &p, sizeof(p)); }

hipError_t wide_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int Sq, int Sk, int Hq,
                    int Hk, int D, Strides qs, Strides ks, Strides vs, Strides os, float scale, int causal, int dt,
                    const Extra* ex, hipStream_t st) {
  const int feat = ex ? (1 | (ex->mask ? 2 : 0) | (ex->p_drop > 0.f ? 4 : 0) | (ex->rows ? 8 : 0)) : 0;
  // query rows per block: 128 (2 tiles per wave), 64 at D = 256 (fwd_kernel QT)
#define FAW_FWD(F)                                                                                                \
  fwd_kernel<T, DD, CC, F><<<grid, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v,      \
                                                 (uint16_t*)o, lse, Sq, Sk, Hq, Hk, qs, ks, vs, os, scale * kLog2e, \
                                                 ex ? *ex : Extra{})
  FAW_DISPATCH(dt, D, causal, {
    const dim3 grid(Hq, B, DD > 128 ? (Sq + 63) / 64 : (Sq + 127) / 128);
    switch (feat) {
      case 0: FAW_FWD(0); break;
      case 1: FAW_FWD(1); break;
      case 3: FAW_FWD(3); break;
      case 5: FAW_FWD(5); break;
      case 7: FAW_FWD(7); break;
      case 9: FAW_FWD(9); break;
      default: FAW_FWD(13); break;
    }
  });
#undef FAW_FWD
  return hipGetLastError();
}

// dQ (which also writes the delta rows when o != null) then dK/dV, 4-wave blocks of 16-row tiles
hipError_t wide_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                    float* delta, void* dq, void* dk, void* dv, int B, int Sq, int Sk, int Hq, int Hk, int D,
                    Strides qs, Strides ks, Strides vs, Strides os, Strides dos, Strides dqs, Strides dks,
                    Strides dvs, float scale, int causal, int dt, const Extra* ex, hipStream_t st) {
  const dim3 g1(Hq, B, (Sk + 63) / 64), g2(Hq, B, (Sq + 63) / 64);
  const int feat = ex ? (1 | (ex->mask ? 2 : 0) | (ex->p_drop > 0.f ? 4 : 0) | (ex->rows ? 8 : 0)) : 0;
#define FAW_BWD(F)                                                                                                  \
  do {                                                                                                              \
    const Extra e_ = ex ? *ex : Extra{};                                                                            \
    bwd_dq_kernel<T, DD, CC, 1, 4, F><<<g2, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)k,                   \
                                                          (const uint16_t*)v, (const uint16_t*)dout, lse, delta,    \
                                                          (uint16_t*)dq, Sq, Sk, Hq, Hk, qs, ks, vs, dos, dqs,      \
                                                          scale, e_, (const uint16_t*)o, os);                       \
    bwd_dkdv_kernel<T, DD, CC, 1, 4, F><<<g1, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)k,                 \
                                                            (const uint16_t*)v, (const uint16_t*)dout, lse, delta,  \
                                                            (uint16_t*)dk, (uint16_t*)dv, Sq, Sk, Hq, Hk, qs, ks,   \
                                                            vs, dos, dks, dvs, scale, e_);                          \
  } while (0)
  FAW_DISPATCH(dt, D, causal, {
    switch (feat) {
      case 0: FAW_BWD(0); break;
      case 1: FAW_BWD(1); break;
      case 3: FAW_BWD(3); break;
      case 5: FAW_BWD(5); break;
      case 7: FAW_BWD(7); break;
      case 9: FAW_BWD(9); break;
      default: FAW_BWD(13); break;
    }
  });
#undef FAW_BWD
  return hipGetLastError();
}

}  // namespace fa
}  // namespace pa
