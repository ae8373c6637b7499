// Per-row (per-token) symmetric int8 quantisation of activations for the int8 MFMA GEMM
// (pa_gemm8_i8): scale[m] = max_k |x[m,k]| / 127 over the columns NOT excluded by colmask (the
// LLM.int8 outlier columns, which run in 16-bit), q[m,k] = round(x[m,k] / scale[m]) (0 on excluded
// columns).  One 256-lane block per row, 16-B vector accesses; the second pass re-reads the row
// from L2.  Reference: the activation quantisation of paddle/phi/kernels/gpu/llm_int8_linear_kernel.cu.
#include "common.h"

namespace pa {
namespace i8q {

template <typename T>
__global__ __launch_bounds__(256) void quant_rows_kernel(const T* __restrict__ x, int K, long long ldx,
                                                         const uint8_t* __restrict__ excl, int8_t* __restrict__ q,
                                                         long long ldq, float* __restrict__ scale) {
  __shared__ float red[4];
  const long long m = blockIdx.x;
  const T* row = x + m * ldx;
  constexpr int E = 8;
  float amax = 0.f;
  for (int k = threadIdx.x * E; k < K; k += 256 * E) {
    float v[E];
    load_f<T, E>(row + k, v);
    if (excl) {
      const uint2 ex = *reinterpret_cast<const uint2*>(excl + k);
      const uint8_t* eb = reinterpret_cast<const uint8_t*>(&ex);
#pragma unroll
      for (int e = 0; e < E; ++e) amax = eb[e] ? amax : fmaxf(amax, fabsf(v[e]));
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) amax = fmaxf(amax, fabsf(v[e]));
    }
  }
  amax = block_max<256>(amax, red);
  const float s = amax > 0.f ? amax / 127.f : 1.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) scale[m] = s;
  for (int k = threadIdx.x * E; k < K; k += 256 * E) {
    float v[E];
    load_f<T, E>(row + k, v);
    uint8_t eb[E] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (excl) {
      const uint2 ex = *reinterpret_cast<const uint2*>(excl + k);
      const uint8_t* p = reinterpret_cast<const uint8_t*>(&ex);
#pragma unroll
      for (int e = 0; e < E; ++e) eb[e] = p[e];
    }
    union {
      int8_t b[E];
      uint2 u;
    } o;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float r = rintf(fminf(fmaxf(v[e] * inv, -127.f), 127.f));
      o.b[e] = eb[e] ? (int8_t)0 : (int8_t)r;
    }
    *reinterpret_cast<uint2*>(q + m * ldq + k) = o.u;
  }
}

// Static (calibrated, per-tensor) quantisation of the int8 fused_multi_transformer Linears:
// q = clip(round(x * mul), lo, hi) with mul = max_bound * in_scale (round_type 1: half away from zero,
// 0: half to even).  Rows M..R-1 (the GEMM's row padding) are written as zeros.  OutT int8 feeds the
// int8 MFMA GEMM; OutT bf16 holds the same integers (exact) for the decode-shaped W8A16 kernel.
template <typename T, typename OutT>
__global__ __launch_bounds__(256) void quant_static_kernel(const T* __restrict__ x, int M, int R, int K,
                                                           long long ldx, OutT* __restrict__ q, long long ldq,
                                                           float mul, float lo, float hi, int round_type) {
  constexpr int E = 8;
  const int kv = K / E;
  const long long total = (long long)R * kv;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long m = i / kv;
    const int k = (int)(i - m * kv) * E;
    float v[E];
    if (m < M) {
      load_f<T, E>(x + m * ldx + k, v);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float t = v[e] * mul;
        const float r = round_type == 0 ? rintf(t) : roundf(t);
        v[e] = fminf(fmaxf(r, lo), hi);
      }
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] = 0.f;
    }
    if constexpr (sizeof(OutT) == 1) {
      union {
        int8_t b[E];
        uint2 u;
      } o;
#pragma unroll
      for (int e = 0; e < E; ++e) o.b[e] = (int8_t)v[e];
      *reinterpret_cast<uint2*>(q + m * ldq + k) = o.u;
    } else {
      store_f<OutT, E>(q + m * ldq + k, v);
    }
  }
}

}  // namespace i8q
}  // namespace pa

// x: [M][ldx] (dt 1 bf16, 2 fp16, 0 fp32), K % 8 == 0, 16-B aligned rows; q: [R][ldq] (R >= M) of
// int8 (odt 0) or bf16 (odt 1).
PA_API int pa_i8_quant_static(const void* x, int M, int R, int K, long long ldx, void* q, long long ldq, float mul,
                              float lo, float hi, int round_type, int dt, int odt, hipStream_t st) {
  using namespace pa::i8q;
  if (M <= 0 || R < M || K <= 0 || K % 8 || ldx % 8 || ldq % 8 || !q || (odt != 0 && odt != 1))
    return (int)hipErrorInvalidValue;
  const long long total = (long long)R * (K / 8);
  const long long nb = (total + 255) / 256;
  const int grid = (int)(nb < 4096 ? nb : 4096);
#define PA_QS(T)                                                                                                  \
  if (odt == 0)                                                                                                   \
    quant_static_kernel<T, int8_t><<<grid, 256, 0, st>>>((const T*)x, M, R, K, ldx, (int8_t*)q, ldq, mul, lo, hi, \
                                                         round_type);                                             \
  else                                                                                                            \
    quant_static_kernel<T, pa::bf16_t><<<grid, 256, 0, st>>>((const T*)x, M, R, K, ldx, (pa::bf16_t*)q, ldq, mul, \
                                                             lo, hi, round_type);
  if (dt == 1) {
    PA_QS(pa::bf16_t)
  } else if (dt == 2) {
    PA_QS(pa::f16_t)
  } else if (dt == 0) {
    PA_QS(float)
  } else {
    return (int)hipErrorInvalidValue;
  }
#undef PA_QS
  return (int)hipGetLastError();
}

// x: [M][ldx] of dtype dt (1 bf16, 2 fp16, 0 fp32), K % 8 == 0, 16-B aligned rows; excl: uint8 [K]
// (nonzero = excluded column) or null; q: int8 [M][ldq] (ldq % 8 == 0); scale: fp32 [M].
PA_API int pa_i8_quant_rows(const void* x, int M, int K, long long ldx, const void* excl, void* q, long long ldq,
                            float* scale, int dt, hipStream_t st) {
  using namespace pa::i8q;
  if (M <= 0 || K <= 0 || K % 8 || ldx % 8 || ldq % 8 || !q || !scale) return (int)hipErrorInvalidValue;
  if (dt == 1)
    quant_rows_kernel<pa::bf16_t><<<M, 256, 0, st>>>((const pa::bf16_t*)x, K, ldx, (const uint8_t*)excl,
                                                     (int8_t*)q, ldq, scale);
  else if (dt == 2)
    quant_rows_kernel<pa::f16_t><<<M, 256, 0, st>>>((const pa::f16_t*)x, K, ldx, (const uint8_t*)excl, (int8_t*)q,
                                                    ldq, scale);
  else if (dt == 0)
    quant_rows_kernel<float><<<M, 256, 0, st>>>((const float*)x, K, ldx, (const uint8_t*)excl, (int8_t*)q, ldq,
                                                scale);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
