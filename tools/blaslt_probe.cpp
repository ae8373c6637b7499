// Feasibility probe: hipBLASLt fused epilogues (GELU_AUX_BIAS, DGELU_BGRAD, BGRADA) on gfx950 for
// the GPT-3 1.3B MLP shapes vs the plain GEMM of the same shape.  Prints algo count and the best
// of the heuristic's top candidates (timed), in TFLOP/s.  Build:
//   hipcc -O2 --offload-arch=gfx950 tools/blaslt_probe.cpp -lhipblaslt -o tools/blaslt_probe
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { auto _e = (x); if (_e != 0) { printf("ERR %s:%d %d\n", __FILE__, __LINE__, (int)_e); exit(1); } } while (0)

static hipblasLtHandle_t H;
static void* WS;
static const size_t WSB = 64ull << 20;

struct Res { int nalgo; float best_ms; };

// column-major D[m x n] = op(A) op(B) (+ beta C), all bf16, fp32 compute
static Res run(int m, int n, int k, bool ta, bool tb, const void* A, int lda, const void* B, int ldb, void* D, int ldd,
               float beta, hipblasLtEpilogue_t epi, void* bias, void* aux, int ldaux) {
  hipblasLtMatmulDesc_t op;
  CK(hipblasLtMatmulDescCreate(&op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t oa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, ob = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa)));
  CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob)));
  CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  if (bias) {
    CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
    hipDataType bt = HIP_R_16BF;
    CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  if (aux) {
    CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)));
    int64_t l = ldaux;
    CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &l, sizeof(l)));
  }
  hipblasLtMatrixLayout_t la, lb, lc;
  CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, ta ? k : m, ta ? m : k, lda));
  CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, tb ? n : k, tb ? k : n, ldb));
  CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_16BF, m, n, ldd));
  hipblasLtMatmulPreference_t pref;
  CK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t wsb = WSB;
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  hipblasLtMatmulHeuristicResult_t res[16];
  int nres = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(H, op, la, lb, lc, lc, pref, 16, res, &nres);
  Res out{st == HIPBLAS_STATUS_SUCCESS ? nres : -1, 1e9f};
  float alpha = 1.f;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < nres && st == HIPBLAS_STATUS_SUCCESS; ++i) {
    bool ok = true;
    for (int w = 0; w < 2 && ok; ++w)
      ok = hipblasLtMatmul(H, op, &alpha, A, la, B, lb, &beta, D, lc, D, lc, &res[i].algo, WS, WSB, 0) == 0;
    if (!ok) continue;
    hipEventRecord(e0, 0);
    for (int it = 0; it < 10; ++it) hipblasLtMatmul(H, op, &alpha, A, la, B, lb, &beta, D, lc, D, lc, &res[i].algo, WS, WSB, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    if (ms < out.best_ms) out.best_ms = ms;
  }
  hipblasLtMatmulPreferenceDestroy(pref);
  hipblasLtMatrixLayoutDestroy(la);
  hipblasLtMatrixLayoutDestroy(lb);
  hipblasLtMatrixLayoutDestroy(lc);
  hipblasLtMatmulDescDestroy(op);
  return out;
}

static void* rnd(size_t n) {
  std::vector<uint16_t> h(n);
  for (size_t i = 0; i < n; ++i) {
    float f = (rand() / (float)RAND_MAX) * 2.f - 1.f;
    uint32_t u;
    memcpy(&u, &f, 4);
    h[i] = (uint16_t)(u >> 16);
  }
  void* d;
  CK(hipMalloc(&d, n * 2));
  CK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
  return d;
}

static void report(const char* name, Res r, double flops) {
  printf("%-34s algos=%2d best %8.1f us  %6.0f TF\n", name, r.nalgo, r.best_ms * 1e3, flops / (r.best_ms * 1e-3) / 1e12);
}

int main() {
  CK(hipblasLtCreate(&H));
  CK(hipMalloc(&WS, WSB));
  const int M = 16384, Hd = 2048, F = 8192;
  void* x = rnd((size_t)M * Hd);      // [M, 2048] row-major
  void* w1 = rnd((size_t)Hd * F);     // [2048, 8192] row-major (paddle [in, out])
  void* b1 = rnd(F);
  void* z = rnd((size_t)M * F);       // aux [M, 8192]
  void* g = rnd((size_t)M * F);       // out [M, 8192]
  void* w2 = rnd((size_t)F * Hd);     // [8192, 2048]
  void* dy = rnd((size_t)M * Hd);     // [M, 2048]
  void* dw = rnd((size_t)F * Hd);
  void* db = rnd(F);
  double fl = 2.0 * M * Hd * F;
  // fc1 fwd: col-major g^T[F x M] = W1^T? (row-major W1 [Hd,F] == col-major [F x Hd], ld F) x (col-major x^T [Hd x M], ld Hd)
  report("fc1 fwd plain", run(F, M, Hd, false, false, w1, F, x, Hd, g, F, 0.f, HIPBLASLT_EPILOGUE_DEFAULT, nullptr, nullptr, 0), fl);
  report("fc1 fwd bias", run(F, M, Hd, false, false, w1, F, x, Hd, g, F, 0.f, HIPBLASLT_EPILOGUE_BIAS, b1, nullptr, 0), fl);
  report("fc1 fwd gelu_bias", run(F, M, Hd, false, false, w1, F, x, Hd, g, F, 0.f, HIPBLASLT_EPILOGUE_GELU_BIAS, b1, nullptr, 0), fl);
  report("fc1 fwd gelu_aux_bias", run(F, M, Hd, false, false, w1, F, x, Hd, g, F, 0.f, HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, b1, z, F), fl);
  // fc2 dgrad: dg row-major [M, F] = dy [M,Hd] @ W2^T ; col-major D [F x M] = (W2 col-major [Hd x F], ld Hd)^T x dy^T [Hd x M]
  report("fc2 dgrad plain", run(F, M, Hd, true, false, w2, Hd, dy, Hd, g, F, 0.f, HIPBLASLT_EPILOGUE_DEFAULT, nullptr, nullptr, 0), fl);
  report("fc2 dgrad dgelu", run(F, M, Hd, true, false, w2, Hd, dy, Hd, g, F, 0.f, HIPBLASLT_EPILOGUE_DGELU, nullptr, z, F), fl);
  report("fc2 dgrad dgelu_bgrad", run(F, M, Hd, true, false, w2, Hd, dy, Hd, g, F, 0.f, HIPBLASLT_EPILOGUE_DGELU_BGRAD, db, z, F), fl);
  // fc2 wgrad: dW2 row-major [F, Hd] = g^T [F, M] @ dy [M, Hd]; col-major D [Hd x F] = dy^T [Hd x M] (A = dy, ld Hd) x g (col-major [F x M] ld F, T)
  report("fc2 wgrad plain (beta 1)", run(Hd, F, M, false, true, dy, Hd, g, F, dw, Hd, 1.f, HIPBLASLT_EPILOGUE_DEFAULT, nullptr, nullptr, 0), fl);
  report("fc2 wgrad bgrada (beta 1)", run(Hd, F, M, false, true, dy, Hd, g, F, dw, Hd, 1.f, HIPBLASLT_EPILOGUE_BGRADA, db, nullptr, 0), fl);
  report("fc2 wgrad bgradb (beta 1)", run(Hd, F, M, false, true, dy, Hd, g, F, dw, Hd, 1.f, HIPBLASLT_EPILOGUE_BGRADB, db, nullptr, 0), fl);
  return 0;
}
