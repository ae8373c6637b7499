// Hand-written bf16 MFMA GEMM for gfx950, 8-phase ping-pong schedule (the main GEMM of the
// training step: Linear forward, dgrad and weight gradient, the tied LM head).
//
// Reference semantics: paddle/phi/kernels/funcs/blas/blaslt_impl.cu.h (matmul),
// fusion/gpu/fused_gemm_epilogue_kernel.cu (bias epilogue) and
// fusion/gpu/fused_linear_param_grad_add_kernel.cu (W.grad += X^T dY, beta = 1 epilogue).
//
//   C[M,N] = alpha * op(A) @ op(B) (+ beta * C) (+ bias[N])
//   AK: A stored [M][K] (k contiguous) else [K][M];  BK: B stored [N][K] else [K][N].
//
// CDNA4 structure (why it is shaped like this):
//  * 256x256 block tile, K consumed 64 deep, 512 threads = 8 waves as 2 (M) x 4 (N); each wave
//    owns 128x64 of C = 8x4 accumulators of v_mfma_f32_16x16x32_bf16 (128 acc VGPRs).
//  * The two waves that share a SIMD (wave w and w+4) PING-PONG: waves 4-7 start one barrier
//    late, so in every barrier interval one wave of each SIMD runs a 16-MFMA quadrant (256
//    cycles of matrix pipe) while its partner issues the LDS reads / LDS-DMA for its next
//    quadrant.  A K-tile is 8 intervals per wave: L0 M0 L1 M1 L2 M2 L3 M3 (L = load segment,
//    M = 16 MFMAs on one 64x32 quadrant of the wave's 128x64).
//  * Operands are staged HBM -> LDS by global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip),
//    two K-tiles resident (2 x 64 KB).  Each wave group g stages the 128-row A half and the
//    128-col B half with index g; tile t+2 is issued into tile t's buffer as soon as every
//    reader of that half has retired its reads (B after L0 of both groups, A after L2), and
//    retired with a COUNTED vmcnt(8) one K-tile later, so 8-12 barrier intervals of HBM/L2
//    latency hide behind the matrix work.  The DMA is issued from inline asm (hipcc would
//    otherwise drain it with vmcnt(0) at every ds_read).
//  * Every layout is read as it sits in HBM: k-contiguous operands become [128][64] images
//    read with ds_read_b128; m/n-contiguous operands become [64][128] images read with
//    ds_read_b64_tr_b16 (hardware transpose).  Both images are XOR-swizzled on 16-B chunks
//    (the swizzle is folded into the per-lane DMA SOURCE address, the DMA destination being
//    lane-linear) and both read kinds are bank-conflict free (analysis at koff / moff).
//  * Products are computed swapped (mfma(B, A) = C^T fragment) so each lane owns 4
//    consecutive output columns (8-byte stores, 4-wide bias reads).
//  * XCD-aware grouped tile order (blocks b and b+8 share an XCD L2).
#include "gemm8_impl.h"

namespace pa {
namespace g8 {


static int g_sched = 9;
// LDS-staged epilogue of schedule 11 (pa_gemm8_set_staged_epi).  4 (default): the wave-local
// staged epilogue (EPI + 200 instantiation, no block barrier, whole 128-B lines) for EPI 0/2/3/4 —
// faster than the register-fragment stores on every GPT-3 1.3B shape (fc1 + GELU 525 -> 486 us,
// fc2 dgrad x gelu' 550 -> 482, qkv 319 -> 309: profiles/r3s2_gemm_epilogue_cost_wstaged.log).
// The block-staged form (EPI + 100, one block barrier, 512-B rows): 1: the GELU-derivative GEMMs (EPI 3/4: the staged aux-tile READ is
// what pays, fc2 dgrad 543 -> 496 us); 2: also EPI 0/2 (measured 0-1.5 % faster on the K = 2048
// shapes, 4 % slower at K = 8192 / two tile rounds, and EPI 2 loses to its derivative recompute:
// profiles/r3s2_gemm_epilogue_cost_staged.log); 3: the wave-local staged epilogue (EPI + 200,
// no block barrier) for EPI 3/4; 4: wave-local for EPI 0/2/3/4; 0: off.
static int g_staged = 4;
// wave-local staged epilogue in schedule 9 (the weight-gradient GEMM, beta = 1 accumulate)
static int g_staged9 = 1;
static int g_epi_sched = 11;  // schedule of the fused-epilogue MLP GEMMs (11 or 12)

template <bool AK, bool BKM, int EPI>
static hipError_t launch(const void* A, const void* B, void* C, float* ws, const void* bias, int M, int N, int K,
                         long long lda, long long ldb, long long ldc, float alpha, float beta, int splitk,
                         hipStream_t st) {
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  dim3 grid(tm * tn, 1, splitk);
  if (g_sched == 12) {
    if (K % (64 * splitk) != 0) return hipErrorInvalidValue;  // the persistent schedule splits evenly
    const int items = tm * tn * splitk;
    const int g = items >= 256 ? 256 : (items + 7) / 8 * 8;  // one block per CU, a multiple of 8 (XCDs)
    if constexpr (EPI == 0) {
      if (g_staged == 4 && splitk == 1) {  // the quarter-tile wave-staged epilogue (EPI 300)
        gemm12_kernel<AK, BKM, 300><<<g, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, ws,
                                                       (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, beta,
                                                       K, 1);
        return hipGetLastError();
      }
    }
    gemm12_kernel<AK, BKM, EPI><<<g, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, ws,
                                                   (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, beta,
                                                   ksplit_of(K, splitk), splitk);
  } else if (g_sched == 11) {
    if constexpr (EPI == 0) {
      if (g_staged == 2) {
        gemm11_kernel<AK, BKM, 100><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, ws,
                                                          (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, beta,
                                                          ksplit_of(K, splitk));
        return hipGetLastError();
      }
      if (g_staged == 4) {
        gemm11_kernel<AK, BKM, 200><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, ws,
                                                          (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, beta,
                                                          ksplit_of(K, splitk));
        return hipGetLastError();
      }
    }
    gemm11_kernel<AK, BKM, EPI><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, ws,
                                                      (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, beta,
                                                      ksplit_of(K, splitk));
  }
  else if (g_sched == 9) {
    if constexpr (EPI == 0) {
      if (g_staged9) {
        gemm9_kernel<AK, BKM, 200><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, ws,
                                                         (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, beta,
                                                         ksplit_of(K, splitk));
        return hipGetLastError();
      }
    }
    gemm9_kernel<AK, BKM, EPI><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, ws,
                                                     (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, beta,
                                                     ksplit_of(K, splitk));
  }
  else
    gemm8_kernel<AK, BKM, EPI><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, ws,
                                                     (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, beta,
                                                     ksplit_of(K, splitk));
  return hipGetLastError();
}

template <int EPI>
static hipError_t dispatch(int transA, int transB, const void* A, const void* B, void* C, float* ws, const void* bias,
                           int M, int N, int K, long long lda, long long ldb, long long ldc, float alpha, float beta,
                           int splitk, hipStream_t st) {
  const bool ak = transA == 0, bk = transB != 0;
  if (ak && bk) return launch<true, true, EPI>(A, B, C, ws, bias, M, N, K, lda, ldb, ldc, alpha, beta, splitk, st);
  if (ak && !bk) return launch<true, false, EPI>(A, B, C, ws, bias, M, N, K, lda, ldb, ldc, alpha, beta, splitk, st);
  if (!ak && bk) return launch<false, true, EPI>(A, B, C, ws, bias, M, N, K, lda, ldb, ldc, alpha, beta, splitk, st);
  return launch<false, false, EPI>(A, B, C, ws, bias, M, N, K, lda, ldb, ldc, alpha, beta, splitk, st);
}

template <int EPI>
static hipError_t launch_epi(int transB, const void* A, const void* B, void* C, void* aux, const void* bias, int M,
                             int N, int K, long long lda, long long ldb, long long ldc, float alpha, hipStream_t st) {
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  dim3 grid(tm * tn, 1, 1);
  if (g_epi_sched == 12 && EPI != 4 && EPI != 5) {  // persistent: the epilogue overlaps the next tile's staging
    const int items = tm * tn;
    const int g = items >= 256 ? 256 : (items + 7) / 8 * 8;
    if (transB)
      gemm12_kernel<true, true, EPI><<<g, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, (float*)aux,
                                                        (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, 0.f, K, 1);
    else
      gemm12_kernel<true, false, EPI><<<g, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, (float*)aux,
                                                         (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, 0.f, K, 1);
    return hipGetLastError();
  }
  if (g_staged == 4 || (g_staged == 3 && EPI != 2)) {
    if (transB)
      gemm11_kernel<true, true, EPI + 200><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C,
                                                                 (float*)aux, (const uint16_t*)bias, M, N, K, lda, ldb,
                                                                 ldc, alpha, 0.f, K);
    else
      gemm11_kernel<true, false, EPI + 200><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C,
                                                                  (float*)aux, (const uint16_t*)bias, M, N, K, lda,
                                                                  ldb, ldc, alpha, 0.f, K);
    return hipGetLastError();
  }
  if (EPI != 5 && (g_staged == 2 || (g_staged == 1 && EPI != 2))) {
    if (transB)
      gemm11_kernel<true, true, EPI == 5 ? 100 : EPI + 100><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C,
                                                                 (float*)aux, (const uint16_t*)bias, M, N, K, lda, ldb,
                                                                 ldc, alpha, 0.f, K);
    else
      gemm11_kernel<true, false, EPI == 5 ? 100 : EPI + 100><<<grid, 512, 0, st>>>(
          (const char*)A, (const char*)B, (uint16_t*)C, (float*)aux, (const uint16_t*)bias, M, N, K, lda, ldb, ldc,
          alpha, 0.f, K);
    return hipGetLastError();
  }
  if (transB)
    gemm11_kernel<true, true, EPI><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, (float*)aux,
                                                         (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, 0.f, K);
  else
    gemm11_kernel<true, false, EPI><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, (float*)aux,
                                                          (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, 0.f, K);
  return hipGetLastError();
}

}  // namespace g8
}  // namespace pa

// Operand byte span as addressed by the kernel's 32-bit DMA offsets must stay below 4 GiB.
static bool span_ok(int transX, int rows, int K, long long ld) {
  const long long span = transX == 0 ? ((long long)rows * ld) * 2 : ((long long)K * ld) * 2;
  return span < (1LL << 32);
}

// Contract: K % (64 * splitk) == 0, M, N, lda, ldb, ldc % 8 == 0, 16-B aligned operands, operand
// spans < 4 GiB.  Returns hipErrorInvalidValue when the shape is outside it (caller falls back).
PA_API int pa_gemm8_ok(int M, int N, int K, long long lda, long long ldb, long long ldc, int transA, int transB,
                       int splitk) {
  if (M <= 0 || N <= 0 || K <= 0 || splitk < 1) return 0;
  if (!pa::g8::splitk_uneven_ok(K, splitk) || M % 8 || N % 8 || lda % 8 || ldb % 8 || ldc % 8) return 0;
  // A: transA==0 -> [M][lda]; else [K][lda].  B: transB!=0 -> [N][ldb]; else [K][ldb]
  if (!span_ok(transA, M, K, lda)) return 0;
  if (!span_ok(transB != 0 ? 0 : 1, N, K, ldb)) return 0;
  return 1;
}

PA_API int pa_gemm8_bf16(const void* A, const void* B, void* C, const void* bias, void* ws, int M, int N, int K,
                         long long lda, long long ldb, long long ldc, int transA, int transB, float alpha, float beta,
                         int splitk, hipStream_t st) {
  using namespace pa::g8;
  if (!pa_gemm8_ok(M, N, K, lda, ldb, ldc, transA, transB, splitk)) return (int)hipErrorInvalidValue;
  if (splitk == 1)
    return (int)dispatch<0>(transA, transB, A, B, C, nullptr, bias, M, N, K, lda, ldb, ldc, alpha, beta, 1, st);
  if (!ws) return (int)hipErrorInvalidValue;
  return (int)dispatch<1>(transA, transB, A, B, C, (float*)ws, nullptr, M, N, K, lda, ldb, ldc, 1.f, 0.f, splitk, st);
}

// Fused-epilogue GEMMs of the GPT MLP (A k-contiguous [M][lda], schedule 11).  epi 2: h = alpha*A@B +
// bias, C = gelu(h), aux = gelu'(h);  epi 3: C = alpha*A@B * aux.  aux: bf16 [M][ldc].
PA_API int pa_gemm8_bf16_epi(const void* A, const void* B, void* C, const void* bias, void* aux, int M, int N, int K,
                             long long lda, long long ldb, long long ldc, int transB, float alpha, int epi,
                             hipStream_t st) {
  using namespace pa::g8;
  if (!pa_gemm8_ok(M, N, K, lda, ldb, ldc, 0, transB, 1) || !aux) return (int)hipErrorInvalidValue;
  if (epi == 2) return (int)launch_epi<2>(transB, A, B, C, aux, bias, M, N, K, lda, ldb, ldc, alpha, st);
  if (epi == 3) return (int)launch_epi<3>(transB, A, B, C, aux, nullptr, M, N, K, lda, ldb, ldc, alpha, st);
  // epi 9: epi 2 with the exact (erf) GELU, wave-staged epilogue only
  if (epi == 9) {
    dim3 grid(((M + BM - 1) / BM) * ((N + BN - 1) / BN), 1, 1);
    if (transB)
      gemm11_kernel<true, true, 209><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, (float*)aux,
                                                          (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, 0.f, K);
    else
      gemm11_kernel<true, false, 209><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, (float*)aux,
                                                           (const uint16_t*)bias, M, N, K, lda, ldb, ldc, alpha, 0.f, K);
    return (int)hipGetLastError();
  }
  // epi 4: epi 3 + column partial sums of C, one fp32 row per 128-row slab, into bias ([ceil(M/128)][N])
  if (epi == 4 && bias != nullptr) return (int)launch_epi<4>(transB, A, B, C, aux, bias, M, N, K, lda, ldb, ldc, alpha, st);
  // epi 5: plain C = alpha*A@B + batch-norm column statistics (mean, M2) of every 128-row slab into
  // aux (fp32 [2][ceil(M/128)][N]: means, then M2s), finished by pa_bn_fwd_parts; no bias
  if (epi == 5 && bias == nullptr) return (int)launch_epi<5>(transB, A, B, C, aux, nullptr, M, N, K, lda, ldb, ldc, alpha, st);
  return (int)hipErrorInvalidValue;
}

// Inference epilogues: C = act(alpha * A @ B + bias) with act 6 relu, 7 gelu (erf), 8 gelu (tanh) in
// the wave-staged epilogue of schedule 11; no aux output (imported programs' fc_fuse_pass).
PA_API int pa_gemm8_bf16_act(const void* A, const void* B, void* C, const void* bias, int M, int N, int K,
                             long long lda, long long ldb, long long ldc, int transB, float alpha, int act,
                             hipStream_t st) {
  using namespace pa::g8;
  if (!pa_gemm8_ok(M, N, K, lda, ldb, ldc, 0, transB, 1) || act < 6 || act > 8) return (int)hipErrorInvalidValue;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  dim3 grid(tm * tn, 1, 1);
#define PA_G8_ACT(E)                                                                                                \
  do {                                                                                                             \
    if (transB)                                                                                                    \
      gemm11_kernel<true, true, E + 200><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C,        \
                                                               nullptr, (const uint16_t*)bias, M, N, K, lda, ldb,  \
                                                               ldc, alpha, 0.f, K);                                \
    else                                                                                                           \
      gemm11_kernel<true, false, E + 200><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C,       \
                                                                nullptr, (const uint16_t*)bias, M, N, K, lda, ldb, \
                                                                ldc, alpha, 0.f, K);                               \
  } while (0)
  if (act == 6) PA_G8_ACT(6);
  else if (act == 7) PA_G8_ACT(7);
  else PA_G8_ACT(8);
#undef PA_G8_ACT
  return (int)hipGetLastError();
}

// Two weight gradients in one launch (schedule 9, both operands m/n-contiguous as the Linear
// weight gradient reads them: A = X^T [K][M], B = dY [K][N]), C_i = alpha * A_i @ B_i + beta * C_i,
// shared K.  Returns hipErrorInvalidValue outside the kernel contract.
PA_API int pa_gemm8_wgrad_grouped2(const void* A0, const void* B0, void* C0, int M0, int N0, long long lda0,
                                   long long ldb0, long long ldc0, const void* A1, const void* B1, void* C1, int M1,
                                   int N1, long long lda1, long long ldb1, long long ldc1, int K, float alpha,
                                   float beta, hipStream_t st) {
  using namespace pa::g8;
  if (!pa_gemm8_ok(M0, N0, K, lda0, ldb0, ldc0, 1, 0, 1) || !pa_gemm8_ok(M1, N1, K, lda1, ldb1, ldc1, 1, 0, 1))
    return (int)hipErrorInvalidValue;
  const int t0 = ((M0 + BM - 1) / BM) * ((N0 + BN - 1) / BN), t1 = ((M1 + BM - 1) / BM) * ((N1 + BN - 1) / BN);
  Prob p1{(const char*)A1, (const char*)B1, (uint16_t*)C1, M1, N1, lda1, ldb1, ldc1};
  if (g_staged9) {
    gemm9_kernel<false, false, 200, true><<<t0 + t1, 512, 0, st>>>((const char*)A0, (const char*)B0, (uint16_t*)C0,
                                                                   nullptr, nullptr, M0, N0, K, lda0, ldb0, ldc0,
                                                                   alpha, beta, K, p1);
    return (int)hipGetLastError();
  }
  gemm9_kernel<false, false, 0, true><<<t0 + t1, 512, 0, st>>>((const char*)A0, (const char*)B0, (uint16_t*)C0,
                                                               nullptr, nullptr, M0, N0, K, lda0, ldb0, ldc0, alpha,
                                                               beta, K, p1);
  return (int)hipGetLastError();
}

PA_API int pa_gemm8_set_staged_epi(int v) {
  const int old = pa::g8::g_staged;
  pa::g8::g_staged = v < 0 ? 0 : (v > 4 ? 4 : v);
  return old;
}

PA_API int pa_gemm8_set_staged9(int v) {
  const int old = pa::g8::g_staged9;
  pa::g8::g_staged9 = v ? 1 : 0;
  return old;
}

PA_API int pa_gemm8_set_nt_store(int v) {
  int old = 0;
  (void)hipMemcpyFromSymbol(&old, HIP_SYMBOL(pa::g8::g_nt_store), sizeof(int));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(pa::g8::g_nt_store), &v, sizeof(int));
  return old;
}

PA_API int pa_gemm8_set_wide_epi(int v) {
  int old = 1;
  (void)hipMemcpyFromSymbol(&old, HIP_SYMBOL(pa::g8::g_wide_epi), sizeof(int));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(pa::g8::g_wide_epi), &v, sizeof(int));
  return old;
}

// schedule select (A/B benchmarking): 8 = row-half staging, 9 = k-half staging (default),
// 11 = row-half staging with 32-MFMA segments, 12 = schedule 11 persistent
PA_API int pa_gemm8_set_sched(int v) {
  const int old = pa::g8::g_sched;
  pa::g8::g_sched = v;
  return old;
}

// schedule of the fused-epilogue GEMMs (pa_gemm8_bf16_epi): 11 (default) or 12 (persistent)
PA_API int pa_gemm8_set_epi_sched(int v) {
  const int old = pa::g8::g_epi_sched;
  pa::g8::g_epi_sched = v == 12 ? 12 : 11;
  return old;
}

// Diagnostic: schedule-11 GEMM (A, B k-contiguous) with epilogue variant epi (0, 2, 10, 12; see
// epilogue_wide).  aux: bf16 [M][ldc] for the GELU forms.
PA_API int pa_gemm8_diag(const void* A, const void* B, void* C, const void* bias, void* aux, int M, int N, int K,
                         int epi, hipStream_t st) {
  using namespace pa::g8;
  if (!pa_gemm8_ok(M, N, K, K, K, N, 0, 1, 1)) return (int)hipErrorInvalidValue;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  dim3 grid(tm * tn, 1, 1);
#define PA_DIAG(E)                                                                                              \
  gemm11_kernel<true, true, E><<<grid, 512, 0, st>>>((const char*)A, (const char*)B, (uint16_t*)C, (float*)aux, \
                                                     (const uint16_t*)bias, M, N, K, K, K, N, 1.f, 0.f, K)
  if (epi == 0) PA_DIAG(0);
  else if (epi == 2) PA_DIAG(2);
  else if (epi == 10) PA_DIAG(10);
  else if (epi == 12) PA_DIAG(12);
  else if (epi == 20) PA_DIAG(20);
  else if (epi == 100) PA_DIAG(100);
  else if (epi == 102) PA_DIAG(102);
  else if (epi == 200) PA_DIAG(200);
  else if (epi == 202) PA_DIAG(202);
  else return (int)hipErrorInvalidValue;
#undef PA_DIAG
  return (int)hipGetLastError();
}
