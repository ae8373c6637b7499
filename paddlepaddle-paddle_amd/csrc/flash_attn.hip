// Flash attention host entry points (head_dim 64 / 128 instantiations); the kernels and their
// design notes are in flash_attn_kernels.h, head_dim 96 / 256 in flash_attn_wide.hip.
#include "flash_attn_kernels.h"

namespace pa {
namespace fa {
// head_dim 96 / 256 (flash_attn_wide.hip)
hipError_t wide_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int Sq, int Sk, int Hq,
                    int Hk, int D, Strides qs, Strides ks, Strides vs, Strides os, float scale, int causal, int dt,
                    const Extra* ex, hipStream_t st);
hipError_t wide_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                    float* delta, void* dq, void* dk, void* dv, int B, int Sq, int Sk, int Hq, int Hk, int D,
                    Strides qs, Strides ks, Strides vs, Strides os, Strides dos, Strides dqs, Strides dks,
                    Strides dvs, float scale, int causal, int dt, const Extra* ex, hipStream_t st);
int wide_set_pair_group(int v);
int wide_set_rng_gen(const void* p);
}  // namespace fa
}  // namespace pa

static inline bool wide_d(int D) { return D == 96 || D == 256; }

using namespace pa;
using namespace pa::fa;

#define FA_DISPATCH(dt, D, causal, ...)                                                            \
  if (dt == 1 && D == 128 && causal) { using T = bf16_t; constexpr int DD = 128; constexpr bool CC = true; __VA_ARGS__; } \
  else if (dt == 1 && D == 128 && !causal) { using T = bf16_t; constexpr int DD = 128; constexpr bool CC = false; __VA_ARGS__; } \
  else if (dt == 1 && D == 64 && causal) { using T = bf16_t; constexpr int DD = 64; constexpr bool CC = true; __VA_ARGS__; } \
  else if (dt == 1 && D == 64 && !causal) { using T = bf16_t; constexpr int DD = 64; constexpr bool CC = false; __VA_ARGS__; } \
  else if (dt == 2 && D == 128 && causal) { using T = f16_t; constexpr int DD = 128; constexpr bool CC = true; __VA_ARGS__; } \
  else if (dt == 2 && D == 128 && !causal) { using T = f16_t; constexpr int DD = 128; constexpr bool CC = false; __VA_ARGS__; } \
  else if (dt == 2 && D == 64 && causal) { using T = f16_t; constexpr int DD = 64; constexpr bool CC = true; __VA_ARGS__; } \
  else if (dt == 2 && D == 64 && !causal) { using T = f16_t; constexpr int DD = 64; constexpr bool CC = false; __VA_ARGS__; } \
  else return hipErrorInvalidValue;

// forward K/V double buffering (fwd_kernel PIPE): -2 = not read yet (env PA_FA_FWD_PIPE), else 0/1
static int g_fwd_pipe = -2;
static bool fwd_pipe() {
  if (g_fwd_pipe == -2) {
    const char* e = getenv("PA_FA_FWD_PIPE");
    g_fwd_pipe = e ? atoi(e) : 0;
  }
  return g_fwd_pipe > 0;
}
PA_API int pa_flash_set_fwd_pipe(int v) {
  fwd_pipe();
  const int old = g_fwd_pipe;
  g_fwd_pipe = v;
  return old;
}

// software-pipelined forward (fwd_sp_kernel): -2 = not read yet (env PA_FA_FWD_SP), else 0/1
static int g_fwd_sp = -2;
static bool fwd_sp() {
  if (g_fwd_sp == -2) {
    const char* e = getenv("PA_FA_FWD_SP");
    g_fwd_sp = e ? atoi(e) : 0;
  }
  return g_fwd_sp > 0;
}
PA_API int pa_flash_set_fwd_sp(int v) {
  fwd_sp();
  const int old = g_fwd_sp;
  g_fwd_sp = v;
  return old;
}

// strides: [b, s, h] element strides for each tensor (head_dim stride must be 1)
PA_API hipError_t pa_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int Sq, int Sk,
                               int Hq, int Hk, int D, const long long* qst, const long long* kst, const long long* vst,
                               const long long* ost, float scale, int causal, int dt, hipStream_t st) {
  if (Hk <= 0 || Hq % Hk != 0) return hipErrorInvalidValue;
  Strides qs{qst[0], qst[1], qst[2]}, ks{kst[0], kst[1], kst[2]}, vs{vst[0], vst[1], vst[2]}, os{ost[0], ost[1], ost[2]};
  if (wide_d(D)) return wide_fwd(q, k, v, o, lse, B, Sq, Sk, Hq, Hk, D, qs, ks, vs, os, scale, causal, dt, nullptr, st);
  dim3 grid(Hq, B, (Sq + 127) / 128);
  if (fwd_sp() && D == 64) {
    FA_DISPATCH(dt, D, causal, if constexpr (DD == 64) {
      fwd_sp_kernel<T, DD, CC><<<grid, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v,
                                                     (uint16_t*)o, lse, Sq, Sk, Hq, Hk, qs, ks, vs, os, scale * kLog2e);
    });
  } else if (fwd_pipe()) {
    FA_DISPATCH(dt, D, causal,
                fwd_kernel<T, DD, CC, 0, true><<<grid, 256, 0, st>>>(
                    (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o, lse, Sq, Sk, Hq, Hk, qs,
                    ks, vs, os, scale * kLog2e));
  } else {
    FA_DISPATCH(dt, D, causal,
                fwd_kernel<T, DD, CC><<<grid, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)k,
                                                            (const uint16_t*)v, (uint16_t*)o, lse, Sq, Sk, Hq, Hk, qs,
                                                            ks, vs, os, scale * kLog2e));
  }
  return hipGetLastError();
}

// backward tiling: 1 = 16 rows per wave (2 waves/SIMD), 2 = 32 rows per wave (1 wave/SIMD),
// 3 = 16 rows per wave in 8-wave blocks (128 rows share each staged tile; default at D = 128);
// PA_FA_BWD_VARIANT selects (A/B), default 1 (measured on MI355X, B16 S1024 H16 D128 causal:
// fwd+bwd 1.04 ms with 1 vs 1.30 ms with 2 — the 32-row tiles lose occupancy to VGPR pressure).
static int g_bwd_variant = -2;  // -2: not read yet, -1: automatic (by head dim)
static int bwd_variant(int D) {
  if (g_bwd_variant == -2) {
    const char* e = getenv("PA_FA_BWD_VARIANT");
    g_bwd_variant = e ? atoi(e) : -1;
  }
  if (g_bwd_variant > 0) return g_bwd_variant;
  // measured (tools/attn_bench.py, longest-first grids): 8-wave blocks win at D = 128
  // (B16 S1024 H16 causal fwd+bwd 0.695 vs 0.755 ms), 4-wave blocks at D = 64
  return D == 128 ? 3 : 1;
}

// v <= 0: automatic; returns the previous setting (-1 = automatic)
// attention block order (g_pair_group above); returns the previous setting
PA_API int pa_flash_set_pair_group(int v) {
  int old = 0;
  (void)hipMemcpyFromSymbol(&old, HIP_SYMBOL(pa::fa::g_pair_group), sizeof(int));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(pa::fa::g_pair_group), &v, sizeof(int));
  wide_set_pair_group(v);
  return old;
}

PA_API int pa_flash_set_bwd_variant(int v) {
  bwd_variant(128);
  const int old = g_bwd_variant;
  g_bwd_variant = v > 0 ? v : -1;
  return old;
}


// dk/dv are per-q-head buffers (caller reduces over GQA groups when Hq != Hk).
PA_API hipError_t pa_flash_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                               const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int Sq, int Sk,
                               int Hq, int Hk, int D, const long long* qst, const long long* kst, const long long* vst,
                               const long long* ost, const long long* dost, const long long* dqst,
                               const long long* dkst, const long long* dvst, float scale, int causal, int dt,
                               hipStream_t st) {
  if (Hk <= 0 || Hq % Hk != 0) return hipErrorInvalidValue;
  Strides qs{qst[0], qst[1], qst[2]}, ks{kst[0], kst[1], kst[2]}, vs{vst[0], vst[1], vst[2]},
      os{ost[0], ost[1], ost[2]}, dos{dost[0], dost[1], dost[2]}, dqs{dqst[0], dqst[1], dqst[2]},
      dks{dkst[0], dkst[1], dkst[2]}, dvs{dvst[0], dvst[1], dvst[2]};
  if (wide_d(D))
    return wide_bwd(q, k, v, o, dout, lse, delta, dq, dk, dv, B, Sq, Sk, Hq, Hk, D, qs, ks, vs, os, dos, dqs, dks, dvs,
                    scale, causal, dt, nullptr, st);
  // dQ runs first in every variant: it computes the delta rows (rowsum dO * O) from its own dO
  // fragments and stores them for the dK/dV kernel that follows on the same stream
  FA_DISPATCH(dt, D, causal, {
    if (bwd_variant(D) == 4) {
      dim3 g2(Hq, B, (Sq + 127) / 128);
      bwd_dq_kernel<T, DD, CC, 1, 8, 0, true><<<g2, 512, 0, st>>>(
          (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta,
          (uint16_t*)dq, Sq, Sk, Hq, Hk, qs, ks, vs, dos, dqs, scale, Extra{}, (const uint16_t*)o, os);
      dim3 g1(Hq, B, (Sk + 127) / 128);
      bwd_dkdv_kernel<T, DD, CC, 1, 8, 0, true><<<g1, 512, 0, st>>>(
          (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta,
          (uint16_t*)dk, (uint16_t*)dv, Sq, Sk, Hq, Hk, qs, ks, vs, dos, dks, dvs, scale);
    } else if (bwd_variant(D) == 3) {
      dim3 g2(Hq, B, (Sq + 127) / 128);
      bwd_dq_kernel<T, DD, CC, 1, 8><<<g2, 512, 0, st>>>((const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v,
                                                         (const uint16_t*)dout, lse, delta, (uint16_t*)dq, Sq, Sk,
                                                         Hq, Hk, qs, ks, vs, dos, dqs, scale, Extra{}, (const uint16_t*)o, os);
      dim3 g1(Hq, B, (Sk + 127) / 128);
      bwd_dkdv_kernel<T, DD, CC, 1, 8><<<g1, 512, 0, st>>>((const uint16_t*)q, (const uint16_t*)k,
                                                           (const uint16_t*)v, (const uint16_t*)dout, lse, delta,
                                                           (uint16_t*)dk, (uint16_t*)dv, Sq, Sk, Hq, Hk, qs, ks, vs,
                                                           dos, dks, dvs, scale);
    } else if (bwd_variant(D) == 2) {
      dim3 g2(Hq, B, (Sq + 127) / 128);
      bwd_dq_kernel<T, DD, CC, 2><<<g2, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v,
                                                      (const uint16_t*)dout, lse, delta, (uint16_t*)dq, Sq, Sk, Hq,
                                                      Hk, qs, ks, vs, dos, dqs, scale, Extra{}, (const uint16_t*)o, os);
      dim3 g1(Hq, B, (Sk + 127) / 128);
      bwd_dkdv_kernel<T, DD, CC, 2><<<g1, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v,
                                                        (const uint16_t*)dout, lse, delta, (uint16_t*)dk,
                                                        (uint16_t*)dv, Sq, Sk, Hq, Hk, qs, ks, vs, dos, dks, dvs,
                                                        scale);
    } else {
      dim3 g2(Hq, B, (Sq + 63) / 64);
      bwd_dq_kernel<T, DD, CC, 1><<<g2, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v,
                                                      (const uint16_t*)dout, lse, delta, (uint16_t*)dq, Sq, Sk, Hq,
                                                      Hk, qs, ks, vs, dos, dqs, scale, Extra{}, (const uint16_t*)o, os);
      dim3 g1(Hq, B, (Sk + 63) / 64);
      bwd_dkdv_kernel<T, DD, CC, 1><<<g1, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v,
                                                        (const uint16_t*)dout, lse, delta, (uint16_t*)dk,
                                                        (uint16_t*)dv, Sq, Sk, Hq, Hk, qs, ks, vs, dos, dks, dvs,
                                                        scale);
    }
  });
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- extended entry points
// Varlen (cu_q / cu_k != null: q/k/v/o packed [total, H, D], B = number of sequences, Sq/Sk =
// max lengths, LSE / delta [Hq, total_q]), additive masks (fp32 or the activation dtype, element
// strides mb/mh/mq, unit key stride) and in-kernel dropout (p_drop > 0, counter-hash keep mask
// regenerated in backward).
static Extra make_extra(const int* cu_q, const int* cu_k, int total_q, const void* mask, long long mb, long long mh,
                        long long mq, int mask_f32, float p_drop, unsigned seed, unsigned offset,
                        const int* rows, long long rb, long long rh) {
  Extra e;
  e.rows = rows;
  e.rb = rb;
  e.rh = rh;
  e.cu_q = cu_q;
  e.cu_k = cu_k;
  e.total_q = total_q;
  e.mask = mask;
  e.mb = mb;
  e.mh = mh;
  e.mq = mq;
  e.mask_f32 = mask_f32;
  e.p_drop = p_drop;
  e.seed = seed;
  e.offset = offset;
  const int th = (int)((double)p_drop * 256.0 + 0.5);
  e.drop_thresh = (uint32_t)(th > 256 ? 256 : th);
  e.keep_scale = e.drop_thresh < 256 ? 256.f / (256.f - (float)e.drop_thresh) : 0.f;
  return e;
}

PA_API hipError_t pa_flash_fwd_ex(const void* q, const void* k, const void* v, void* o, float* lse, int B, int Sq,
                                  int Sk, int Hq, int Hk, int D, const long long* qst, const long long* kst,
                                  const long long* vst, const long long* ost, float scale, int causal, int dt,
                                  const int* cu_q, const int* cu_k, int total_q, const void* mask, long long mb,
                                  long long mh, long long mq, int mask_f32, float p_drop, unsigned seed,
                                  unsigned offset, const int* rows, long long rb, long long rh, const int* mask_all,
                                  hipStream_t st) {
  if (Hk <= 0 || Hq % Hk != 0 || (cu_q == nullptr) != (cu_k == nullptr)) return hipErrorInvalidValue;
  Strides qs{qst[0], qst[1], qst[2]}, ks{kst[0], kst[1], kst[2]}, vs{vst[0], vst[1], vst[2]}, os{ost[0], ost[1], ost[2]};
  if (mask && rows) return hipErrorInvalidValue;  // one mask form per call
  Extra ex = make_extra(cu_q, cu_k, total_q, mask, mb, mh, mq, mask_f32, p_drop, seed, offset, rows, rb, rh);
  ex.mask_all = mask ? mask_all : nullptr;
  if (wide_d(D)) return wide_fwd(q, k, v, o, lse, B, Sq, Sk, Hq, Hk, D, qs, ks, vs, os, scale, causal, dt, &ex, st);
  dim3 grid(Hq, B, (Sq + 127) / 128);
  const int feat = 1 | (mask ? 2 : 0) | (p_drop > 0.f ? 4 : 0) | (rows ? 8 : 0);
#define FA_FWD_EX(F)                                                                                            \
  if constexpr (DD == 64) {                                                                                     \
    if (fwd_sp()) {                                                                                             \
      fwd_sp_kernel<T, DD, CC, F><<<grid, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)k,                 \
                                                        (const uint16_t*)v, (uint16_t*)o, lse, Sq, Sk, Hq, Hk,  \
                                                        qs, ks, vs, os, scale * kLog2e, ex);                    \
      break;                                                                                                    \
    }                                                                                                           \
  }                                                                                                             \
  if (fwd_pipe())                                                                                               \
    fwd_kernel<T, DD, CC, F, true><<<grid, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)k,                \
                                                         (const uint16_t*)v, (uint16_t*)o, lse, Sq, Sk, Hq, Hk, \
                                                         qs, ks, vs, os, scale * kLog2e, ex);                   \
  else                                                                                                          \
    fwd_kernel<T, DD, CC, F><<<grid, 256, 0, st>>>((const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v,  \
                                                   (uint16_t*)o, lse, Sq, Sk, Hq, Hk, qs, ks, vs, os,           \
                                                   scale * kLog2e, ex)
  FA_DISPATCH(dt, D, causal, {
    switch (feat) {
      case 1: FA_FWD_EX(1); break;
      case 3: FA_FWD_EX(3); break;
      case 5: FA_FWD_EX(5); break;
      case 7: FA_FWD_EX(7); break;
      case 9: FA_FWD_EX(9); break;
      default: FA_FWD_EX(13); break;
    }
  });
#undef FA_FWD_EX
  return hipGetLastError();
}

// dK/dV + dQ launches of one feature set (D = 128: 8-wave blocks, D = 64: 4-wave blocks)
template <typename T, int DD, bool CC, int F>
static void bwd_ex(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                   float* delta, void* dq, void* dk, void* dv, int B, int Sq, int Sk, int Hq, int Hk, Strides qs,
                   Strides ks, Strides vs, Strides os, Strides dos, Strides dqs, Strides dks, Strides dvs, float scale,
                   const Extra& ex, hipStream_t st) {
  // dQ first: it computes the delta rows from its own dO fragments (o != null) and stores them
  // for the dK/dV kernel that follows on the same stream
  constexpr int NW = DD == 128 ? 8 : 4;
  dim3 g1(Hq, B, (Sk + 16 * NW - 1) / (16 * NW));
  dim3 g2(Hq, B, (Sq + 16 * NW - 1) / (16 * NW));
  if (bwd_variant(DD) == 4) {  // double-buffered tiles
    bwd_dq_kernel<T, DD, CC, 1, NW, F, true><<<g2, 64 * NW, 0, st>>>(
        (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta, (uint16_t*)dq,
        Sq, Sk, Hq, Hk, qs, ks, vs, dos, dqs, scale, ex, (const uint16_t*)o, os);
    bwd_dkdv_kernel<T, DD, CC, 1, NW, F, true><<<g1, 64 * NW, 0, st>>>(
        (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta, (uint16_t*)dk,
        (uint16_t*)dv, Sq, Sk, Hq, Hk, qs, ks, vs, dos, dks, dvs, scale, ex);
    return;
  }
  bwd_dq_kernel<T, DD, CC, 1, NW, F><<<g2, 64 * NW, 0, st>>>(
      (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta, (uint16_t*)dq,
      Sq, Sk, Hq, Hk, qs, ks, vs, dos, dqs, scale, ex, (const uint16_t*)o, os);
  bwd_dkdv_kernel<T, DD, CC, 1, NW, F><<<g1, 64 * NW, 0, st>>>(
      (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta, (uint16_t*)dk,
      (uint16_t*)dv, Sq, Sk, Hq, Hk, qs, ks, vs, dos, dks, dvs, scale, ex);
}

PA_API hipError_t pa_flash_bwd_ex(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                  const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int Sq, int Sk,
                                  int Hq, int Hk, int D, const long long* qst, const long long* kst,
                                  const long long* vst, const long long* ost, const long long* dost,
                                  const long long* dqst, const long long* dkst, const long long* dvst, float scale,
                                  int causal, int dt, const int* cu_q, const int* cu_k, int total_q, const void* mask,
                                  long long mb, long long mh, long long mq, int mask_f32, float p_drop, unsigned seed,
                                  unsigned offset, const int* rows, long long rb, long long rh, const int* mask_all,
                                  hipStream_t st) {
  if (Hk <= 0 || Hq % Hk != 0 || (cu_q == nullptr) != (cu_k == nullptr)) return hipErrorInvalidValue;
  Strides qs{qst[0], qst[1], qst[2]}, ks{kst[0], kst[1], kst[2]}, vs{vst[0], vst[1], vst[2]},
      os{ost[0], ost[1], ost[2]}, dos{dost[0], dost[1], dost[2]}, dqs{dqst[0], dqst[1], dqst[2]},
      dks{dkst[0], dkst[1], dkst[2]}, dvs{dvst[0], dvst[1], dvst[2]};
  if (mask && rows) return hipErrorInvalidValue;  // one mask form per call
  Extra ex = make_extra(cu_q, cu_k, total_q, mask, mb, mh, mq, mask_f32, p_drop, seed, offset, rows, rb, rh);
  ex.mask_all = mask ? mask_all : nullptr;
  // delta rows: [B, Hq, Sq] or, varlen, [Hq, total_q] (one "batch" of total_q packed rows)
  // (written by the dQ kernel, which runs first)
  if (wide_d(D))
    return wide_bwd(q, k, v, o, dout, lse, delta, dq, dk, dv, B, Sq, Sk, Hq, Hk, D, qs, ks, vs, os, dos, dqs, dks, dvs,
                    scale, causal, dt, &ex, st);
  FA_DISPATCH(dt, D, causal, {
    const int feat = 1 | (mask ? 2 : 0) | (p_drop > 0.f ? 4 : 0) | (rows ? 8 : 0);
    switch (feat) {
      case 1: bwd_ex<T, DD, CC, 1>(q, k, v, o, dout, lse, delta, dq, dk, dv, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
      case 3: bwd_ex<T, DD, CC, 3>(q, k, v, o, dout, lse, delta, dq, dk, dv, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
      case 5: bwd_ex<T, DD, CC, 5>(q, k, v, o, dout, lse, delta, dq, dk, dv, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
      case 7: bwd_ex<T, DD, CC, 7>(q, k, v, o, dout, lse, delta, dq, dk, dv, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
      case 9: bwd_ex<T, DD, CC, 9>(q, k, v, o, dout, lse, delta, dq, dk, dv, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
      default: bwd_ex<T, DD, CC, 13>(q, k, v, o, dout, lse, delta, dq, dk, dv, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
    }
  });
  return hipGetLastError();
}

// graph-safe dropout streams (common.h rng_mix): generation counter of this module's kernels
PA_API int pa_flash_set_rng_gen(const void* p) {
  const int e = (int)hipMemcpyToSymbol(HIP_SYMBOL(pa::g_rng_gen), &p, sizeof(p));
  const int e2 = wide_set_rng_gen(p);
  return e ? e : e2;
}
