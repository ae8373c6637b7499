// Extra instantiations of the 8-phase MFMA GEMM (gemm8_impl.h) in their own translation unit, so
// the tuned bf16 training-step kernels of gemm8.hip keep their register allocation (co-compiled
// template variants perturb each other's codegen):
//
//  * pa_gemmx: general bf16 / fp16 GEMM, optionally BATCHED (blockIdx.y = batch index, per-operand
//    element strides, stride 0 = broadcast) — the hand-written path behind paddle.matmul / mm / bmm /
//    einsum contractions and Linear outside the training engines (eval, no_grad, inference).
//    Reference semantics: paddle/phi/kernels/impl/matmul_kernel_impl.h (MatMulFunction, batched
//    broadcast) over funcs/blas/blaslt_impl.cu.h.
//  * pa_gemm8_fp8: OCP fp8 (e4m3 / e5m2) x fp8 -> bf16 on the same schedule (schedule 11, both
//    operands k-contiguous), one v_mfma_scale_f32_16x16x128_f8f6f4 per 16x16 fragment and 128-byte
//    k-tile: the bf16 kernel's LDS images, DMA pipeline and epilogue unchanged, twice the FLOPs per
//    matrix-pipe cycle.  Per-tensor dequant scales are device scalars (delayed scaling, no host
//    sync).  Reference: paddle/phi/kernels/fusion/fp8_gemm, python/paddle/static/amp/decorator.py:755.
#define PA_G8_EXTRA_TU 1
#include "gemm8_impl.h"

namespace pa {
namespace g8 {

template <typename T, bool BAT>
static hipError_t launchx(int transA, int transB, const void* A, const void* B, void* C, const void* bias, int M,
                          int N, int K, long long lda, long long ldb, long long ldc, int batch, long long sA,
                          long long sB, long long sC, float alpha, float beta, hipStream_t st) {
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  dim3 grid(tm * tn, batch, 1);
  const long long bA = sA * 2, bB = sB * 2;  // byte strides
  const char* a = (const char*)A;
  const char* b = (const char*)B;
  uint16_t* c = (uint16_t*)C;
  const uint16_t* bi = (const uint16_t*)bias;
  // k-contiguous A: schedule 11 (row-half staging, full 128-B DMA lines); m-contiguous A: schedule 9
  // (k-half staging) — the same per-layout choice as the bf16 training GEMMs (pa_gemm_bf16)
  if (transA == 0) {
    if (transB)
      gemm11_kernel<true, true, 200, T, BAT><<<grid, 512, 0, st>>>(a, b, c, nullptr, bi, M, N, K, lda, ldb, ldc,
                                                                   alpha, beta, K, bA, bB, sC);
    else
      gemm11_kernel<true, false, 200, T, BAT><<<grid, 512, 0, st>>>(a, b, c, nullptr, bi, M, N, K, lda, ldb, ldc,
                                                                    alpha, beta, K, bA, bB, sC);
  } else {
    if (transB)
      gemm9_kernel<false, true, 200, false, T, BAT><<<grid, 512, 0, st>>>(a, b, c, nullptr, bi, M, N, K, lda, ldb,
                                                                          ldc, alpha, beta, K, Prob{}, bA, bB, sC);
    else
      gemm9_kernel<false, false, 200, false, T, BAT><<<grid, 512, 0, st>>>(a, b, c, nullptr, bi, M, N, K, lda, ldb,
                                                                           ldc, alpha, beta, K, Prob{}, bA, bB, sC);
  }
  return hipGetLastError();
}

}  // namespace g8
}  // namespace pa

static bool spanx_ok(int transX, int rows, int K, long long ld) {
  const long long span = transX == 0 ? ((long long)rows * ld) * 2 : ((long long)K * ld) * 2;
  return span < (1LL << 32);
}

// Contract (else the caller falls back to the library): K % 64 == 0, M, N, lda, ldb, ldc % 8 == 0,
// 16-B aligned operands (and batch strides % 8 == 0), each operand matrix spanning < 4 GiB (32-bit
// DMA offsets; the batch offset is added to the 64-bit base).  dt: 1 = bf16, 2 = fp16.
PA_API int pa_gemmx_ok(int M, int N, int K, long long lda, long long ldb, long long ldc, int transA, int transB,
                       int dt) {
  if (M <= 0 || N <= 0 || K <= 0 || (dt != 1 && dt != 2)) return 0;
  if (K % 64 || M % 8 || N % 8 || lda % 8 || ldb % 8 || ldc % 8) return 0;
  return spanx_ok(transA, M, K, lda) && spanx_ok(transB != 0 ? 0 : 1, N, K, ldb);
}

// C[b] = alpha * op(A[b]) @ op(B[b]) (+ beta * C[b]) (+ bias), b < batch.  transA == 0: A[b] is
// [M][lda] (k contiguous), else [K][lda]; transB != 0: B[b] is [N][ldb], else [K][ldb].  Strides in
// elements between consecutive batch matrices (0 = the same matrix for every b).
PA_API int pa_gemmx(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, long long lda,
                    long long ldb, long long ldc, int transA, int transB, int batch, long long sA, long long sB,
                    long long sC, int dt, float alpha, float beta, hipStream_t st) {
  using namespace pa::g8;
  if (!pa_gemmx_ok(M, N, K, lda, ldb, ldc, transA, transB, dt) || batch < 1 || batch > 65535 || sA % 8 ||
      sB % 8 || sC % 8)
    return (int)hipErrorInvalidValue;
  if (dt == 1) {
    if (batch == 1)
      return (int)launchx<pa::bf16_t, false>(transA, transB, A, B, C, bias, M, N, K, lda, ldb, ldc, 1, 0, 0, 0, alpha,
                                             beta, st);
    return (int)launchx<pa::bf16_t, true>(transA, transB, A, B, C, bias, M, N, K, lda, ldb, ldc, batch, sA, sB, sC,
                                          alpha, beta, st);
  }
  if (batch == 1)
    return (int)launchx<pa::f16_t, false>(transA, transB, A, B, C, bias, M, N, K, lda, ldb, ldc, 1, 0, 0, 0, alpha,
                                          beta, st);
  return (int)launchx<pa::f16_t, true>(transA, transB, A, B, C, bias, M, N, K, lda, ldb, ldc, batch, sA, sB, sC, alpha,
                                       beta, st);
}

// fp8 contract: K % 128 == 0, M % 8 == 0, N % 8 == 0, lda / ldw % 16 (bytes), ldc % 8, both operands
// k-contiguous (A [M][lda], W [N][ldw], the fp8 Linear layout), spans < 4 GiB.
PA_API int pa_gemm8_fp8_ok(int M, int N, int K, long long lda, long long ldw, long long ldc) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 128 || M % 8 || N % 8 || lda % 16 || ldw % 16 || ldc % 8) return 0;
  return (long long)M * lda < (1LL << 32) && (long long)N * ldw < (1LL << 32);
}

// C[M,N] (bf16) = alpha * scale_a * scale_b * A @ W^T (+ beta * C) (+ bias); fmt 0 = e4m3, 1 = e5m2.
PA_API int pa_gemm8_fp8(const void* A, const void* W, void* C, const void* bias, const void* scale_a,
                        const void* scale_b, int M, int N, int K, long long lda, long long ldw, long long ldc,
                        float alpha, float beta, int fmtA, int fmtB, hipStream_t st) {
  using namespace pa::g8;
  if (!pa_gemm8_fp8_ok(M, N, K, lda, ldw, ldc) || fmtA < 0 || fmtA > 1 || fmtB < 0 || fmtB > 1)
    return (int)hipErrorInvalidValue;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  dim3 grid(tm * tn, 1, 1);
  // the kernel counts k and leading dims in 2-byte units: fp8 bytes / 2
  const int K2 = K / 2;
  const long long la = lda / 2, lw = ldw / 2;
  auto go = [&](auto kern) {
    kern<<<grid, 512, 0, st>>>((const char*)A, (const char*)W, (uint16_t*)C, nullptr, (const uint16_t*)bias, M, N, K2,
                               la, lw, ldc, alpha, beta, K2, 0LL, 0LL, 0LL, (const float*)scale_a,
                               (const float*)scale_b);
  };
  if (fmtA == 0 && fmtB == 0) go(gemm11_kernel<true, true, 200, F8<0, 0>, false>);
  else if (fmtA == 0) go(gemm11_kernel<true, true, 200, F8<0, 1>, false>);
  else if (fmtB == 0) go(gemm11_kernel<true, true, 200, F8<1, 0>, false>);
  else go(gemm11_kernel<true, true, 200, F8<1, 1>, false>);
  return (int)hipGetLastError();
}

// fp8 GEMMs of a fused GELU feed-forward block (ops/fp8.py _FP8FFN, static training programs'
// fuse_gemm_epilogue_pass) with the wave-staged epilogues of the bf16 MLP GEMMs: epi 9 / 2 (fc1
// forward: h = s*A@W^T + bias, C = gelu(h), aux = gelu'(h); exact / tanh GELU), epi 4 (fc2 data
// gradient: C = s*A@W^T * aux, per-128-row-slab column sums of C into ``bias`` as fp32
// [ceil(M/128)][N]).  aux: bf16 [M][ldc].  Same contract and formats as pa_gemm8_fp8.
PA_API int pa_gemm8_fp8_epi(const void* A, const void* W, void* C, const void* bias, void* aux, const void* scale_a,
                            const void* scale_b, int M, int N, int K, long long lda, long long ldw, long long ldc,
                            float alpha, int fmtA, int fmtB, int epi, hipStream_t st) {
  using namespace pa::g8;
  if (!pa_gemm8_fp8_ok(M, N, K, lda, ldw, ldc) || fmtA < 0 || fmtA > 1 || fmtB != 0 || aux == nullptr)
    return (int)hipErrorInvalidValue;
  if (epi == 4 && bias == nullptr) return (int)hipErrorInvalidValue;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  dim3 grid(tm * tn, 1, 1);
  const int K2 = K / 2;
  const long long la = lda / 2, lw = ldw / 2;
  auto go = [&](auto kern) {
    kern<<<grid, 512, 0, st>>>((const char*)A, (const char*)W, (uint16_t*)C, (float*)aux, (const uint16_t*)bias, M, N,
                               K2, la, lw, ldc, alpha, 0.f, K2, 0LL, 0LL, 0LL, (const float*)scale_a,
                               (const float*)scale_b);
  };
  if (epi == 9 && fmtA == 0) go(gemm11_kernel<true, true, 209, F8<0, 0>, false>);
  else if (epi == 2 && fmtA == 0) go(gemm11_kernel<true, true, 202, F8<0, 0>, false>);
  else if (epi == 4 && fmtA == 1) go(gemm11_kernel<true, true, 204, F8<1, 0>, false>);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// The same fp8 FFN GEMMs with the OUTPUT quantised in the epilogue (gemm8_impl.h
// epilogue_wstaged_q): epi 10 = epi 9 whose gelu(h) leaves as e4m3 q [M][N] + q^T [N][M]; epi 11 =
// epi 4 whose product leaves as e5m2 q + q^T.  scale: the device quantisation scale
// (pa_fp8_scale_prep), amax: the history slot receiving this tensor's amax.  No bf16 output.
// Contract: pa_gemm8_fp8_ok, M % 16 == 0, N % 16 == 0.
PA_API int pa_gemm8_fp8_epi_q(const void* A, const void* W, void* q, void* qt, const void* bias, void* aux,
                              const void* scale_a, const void* scale_b, const void* scale, void* amax, int M, int N,
                              int K, long long lda, long long ldw, float alpha, int fmtA, int epi, hipStream_t st) {
  using namespace pa::g8;
  if (!pa_gemm8_fp8_ok(M, N, K, lda, ldw, N) || M % 16 || N % 16 || !q || !qt || !aux || !scale || !amax)
    return (int)hipErrorInvalidValue;
  if ((epi == 11 && bias == nullptr) || (epi == 10 && fmtA != 0) || (epi == 11 && fmtA != 1))
    return (int)hipErrorInvalidValue;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  dim3 grid(tm * tn, 1, 1);
  const int K2 = K / 2;
  const long long la = lda / 2, lw = ldw / 2;
  const long long x0 = (long long)(size_t)qt, x1 = (long long)(size_t)scale, x2 = (long long)(size_t)amax;
  auto go = [&](auto kern) {
    kern<<<grid, 512, 0, st>>>((const char*)A, (const char*)W, (uint16_t*)q, (float*)aux, (const uint16_t*)bias, M, N,
                               K2, la, lw, (long long)N, alpha, 0.f, K2, x0, x1, x2, (const float*)scale_a,
                               (const float*)scale_b);
  };
  if (epi == 10) go(gemm11_kernel<true, true, 210, F8<0, 0>, false>);
  else if (epi == 11) go(gemm11_kernel<true, true, 211, F8<1, 0>, false>);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// Split-K fp8 GEMM (the fp8 Linear weight gradient X^T dY: M x N = in x out features, K = tokens —
// e.g. 768 x 2304 x 32768 is 27 output tiles for 256 CUs, so the K range is split over gridDim.z
// slices writing fp32 slabs ws[z][M][N], folded by fp8_splitk_reduce with the dequant scales).
// Contract: pa_gemm8_fp8_ok and K % (128 * splitk) == 0; ws holds splitk * M * N floats.
namespace pa {
namespace g8 {
__global__ __launch_bounds__(256) void fp8_splitk_reduce(const float* __restrict__ ws, uint16_t* __restrict__ C,
                                                         const uint16_t* __restrict__ bias, int M, int N,
                                                         long long ldc, int S, float alpha, float beta,
                                                         const float* __restrict__ sa, const float* __restrict__ sb) {
  const long long idx = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long long MN = (long long)M * N;
  if (idx >= MN) return;
  float a = alpha;
  if (sa) a *= sa[0];
  if (sb) a *= sb[0];
  const int m = (int)(idx / N), n = (int)(idx - (long long)m * N);
  f32x4 s = *reinterpret_cast<const f32x4*>(ws + idx);
  for (int k = 1; k < S; ++k) s += *reinterpret_cast<const f32x4*>(ws + k * MN + idx);
  float v[4] = {s[0] * a, s[1] * a, s[2] * a, s[3] * a};
  uint16_t* dst = C + (long long)m * ldc + n;
  if (beta != 0.f) {
    float o[4];
    load_f<bf16_t, 4>(reinterpret_cast<const bf16_t*>(dst), o);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += beta * o[r];
  }
  if (bias) {
    float bb[4];
    load_f<bf16_t, 4>(reinterpret_cast<const bf16_t*>(bias + n), bb);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += bb[r];
  }
  store_f<bf16_t, 4>(reinterpret_cast<bf16_t*>(dst), v);
}
}  // namespace g8
}  // namespace pa

PA_API int pa_gemm8_fp8_splitk(const void* A, const void* W, void* C, const void* bias, const void* scale_a,
                               const void* scale_b, void* ws, int M, int N, int K, long long lda, long long ldw,
                               long long ldc, float alpha, float beta, int fmtA, int fmtB, int splitk,
                               hipStream_t st) {
  using namespace pa::g8;
  // uneven slices allowed (the last one shorter, >= 2 k-tiles of 128 fp8 values): ksplit_of in 2-byte units
  if (splitk < 2 || !ws || K % 128 || !splitk_uneven_ok(K / 2, splitk) || !pa_gemm8_fp8_ok(M, N, K, lda, ldw, ldc) ||
      fmtA < 0 || fmtA > 1 ||
      fmtB < 0 || fmtB > 1)
    return (int)hipErrorInvalidValue;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  dim3 grid(tm * tn, 1, splitk);
  const int K2 = K / 2;
  const long long la = lda / 2, lw = ldw / 2;
  auto go = [&](auto kern) {
    kern<<<grid, 512, 0, st>>>((const char*)A, (const char*)W, nullptr, (float*)ws, nullptr, M, N, K2, la, lw, N,
                               1.f, 0.f, ksplit_of(K2, splitk), 0LL, 0LL, 0LL, nullptr, nullptr);
  };
  if (fmtA == 0 && fmtB == 0) go(gemm11_kernel<true, true, 1, F8<0, 0>, false>);
  else if (fmtA == 0) go(gemm11_kernel<true, true, 1, F8<0, 1>, false>);
  else if (fmtB == 0) go(gemm11_kernel<true, true, 1, F8<1, 0>, false>);
  else go(gemm11_kernel<true, true, 1, F8<1, 1>, false>);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const long long MN = (long long)M * N;
  fp8_splitk_reduce<<<(unsigned)((MN / 4 + 255) / 256), 256, 0, st>>>((const float*)ws, (uint16_t*)C,
                                                                       (const uint16_t*)bias, M, N, ldc, splitk,
                                                                       alpha, beta, (const float*)scale_a,
                                                                       (const float*)scale_b);
  return (int)hipGetLastError();
}

// int8 GEMM (LLM.int8 / W8A8): C[M,N] (bf16) = (A @ W^T) * row_scale[m] * col_scale[n] (+ beta * C)
// (+ bias), A int8 [M][lda], W int8 [N][ldw] (both k-contiguous), int32 accumulation in
// v_mfma_i32_16x16x64_i8 (2x the bf16 MFMA rate).  Reference: paddle/phi/kernels/gpu/
// llm_int8_linear_kernel.cu (python/paddle/nn/quant/quantized_linear.py:239).
// Contract: K % 128 == 0, M, N % 8 == 0, lda / ldw % 16, ldc % 8, spans < 4 GiB.
PA_API int pa_gemm8_i8_ok(int M, int N, int K, long long lda, long long ldw, long long ldc) {
  return pa_gemm8_fp8_ok(M, N, K, lda, ldw, ldc);
}

PA_API int pa_gemm8_i8(const void* A, const void* W, void* C, const void* bias, const float* row_scale,
                       const float* col_scale, int M, int N, int K, long long lda, long long ldw, long long ldc,
                       float beta, hipStream_t st) {
  using namespace pa::g8;
  if (!pa_gemm8_i8_ok(M, N, K, lda, ldw, ldc)) return (int)hipErrorInvalidValue;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  dim3 grid(tm * tn, 1, 1);
  const int K2 = K / 2;  // the kernel counts k and leading dims in 2-byte units
  gemm11_kernel<true, true, 200, I8T, false><<<grid, 512, 0, st>>>(
      (const char*)A, (const char*)W, (uint16_t*)C, nullptr, (const uint16_t*)bias, M, N, K2, lda / 2, ldw / 2, ldc,
      1.f, beta, K2, 0LL, 0LL, 0LL, row_scale, col_scale);
  return (int)hipGetLastError();
}
