// Flash-attention backward with a materialised dS (head_dim 64 / 128, every feature: causal,
// varlen, additive mask, dropout, flashmask rows).
//
// Reference: paddle/phi/kernels/gpu/flash_attn_grad_kernel.cu (flash-attn 2: one kernel per key
// block accumulating dQ with float atomics).  The default backward here (flash_attn.hip) runs a
// dQ kernel and a dK/dV kernel that BOTH recompute S = QK^T and dP = dO V^T: 7 GEMM-sized MFMA
// passes against the forward's 2.  With 288 GB of HBM a bf16 dS (0.5 GB for GPT-3 1.3B's
// 16 x 16 heads x 1024^2, half of it causal) costs less than recomputing it:
//  1. delta kernel: delta = rowsum(dO * O) (fp32, [B, Hq, Sq] or [Hq, total_q] for varlen);
//  2. dK/dV kernel (bwd_dkdv_kernel<..., WDS = true>): unchanged math, and it stores the dS tile
//     it already holds in registers as dS^T rows ([key][query], 8-byte stores that complete
//     128-byte lines over the four query sub-blocks);
//  3. dQ kernel from dS: dQ = dS K per query block — only the dS^T tiles (staged in LDS with the
//     D = 128 swizzled image, read with ds_read_b64_tr_b16: exactly the permuted k order the
//     recompute kernel uses for its register dS) and the K tiles are read; no exp, no S/dP MFMAs.
// No float atomics, deterministic.  Tiles the dK/dV kernel skips (entirely above the causal
// diagonal) are never written: the dQ kernel masks keys > query + (Sk - Sq) and keys >= Sk with
// selects on the loaded fragments (stale bytes may be any bit pattern).
#define PA_FA_PAIR_GROUP_DECL static __constant__
#include "flash_attn_kernels.h"

namespace pa {
namespace fa {

// delta[lrow + q] = sum_d dO[q, h, d] * O[q, h, d]; grid (Hq, B, ceil(Sq / 64)), 256 threads.
template <typename T, int D, int EXT>
__global__ __launch_bounds__(256) void delta_kernel(const uint16_t* __restrict__ O, const uint16_t* __restrict__ dO,
                                                    float* __restrict__ Delta, int Sq_, int Sk_, int Hq, Strides os,
                                                    Strides dos, Extra ex) {
  constexpr int LPR = D / 8;          // lanes per row (16-B chunks)
  constexpr int RPP = 256 / LPR;      // rows per pass
  const int h = blockIdx.x, b = blockIdx.y;
  const Seq sq_ = seq_of<EXT != 0>(ex, b, h, Hq, Sq_, Sk_);
  const int q0 = blockIdx.z * 64;
  if (q0 >= sq_.sq) return;
  const bool vl = EXT && ex.cu_q;
  const uint16_t* ob = O + (vl ? 0 : (long long)b * os.b) + sq_.qo * os.s + (long long)h * os.h;
  const uint16_t* db = dO + (vl ? 0 : (long long)b * dos.b) + sq_.qo * dos.s + (long long)h * dos.h;
  const int ch = threadIdx.x % LPR, rr = threadIdx.x / LPR;
#pragma unroll
  for (int p = 0; p < 64 / RPP; ++p) {
    const int q = q0 + p * RPP + rr;
    float s = 0.f;
    if (q < sq_.sq) {
      float a[8], c[8];
      load_f<T, 8>(reinterpret_cast<const T*>(ob + (long long)q * os.s + 8 * ch), a);
      load_f<T, 8>(reinterpret_cast<const T*>(db + (long long)q * dos.s + 8 * ch), c);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += a[e] * c[e];
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (ch == 0 && q < sq_.sq) Delta[sq_.lrow + q] = s;
  }
}

// dQ[q, d] = scale * sum_k dS[q, k] K[k, d]: grid (Hq, B, ceil(Sq / 128)), 4 waves x 2 query
// tiles of 16; loop over 64-key blocks.  dS^T rows at dsT + b * dsb + h * dsh + key * dsld.
template <typename T, int D, bool CAUSAL, int EXT>
__global__ __launch_bounds__(256, 2) void dq_from_ds_kernel(const uint16_t* __restrict__ K,
                                                            const uint16_t* __restrict__ dsT, uint16_t* __restrict__ dQ,
                                                            int Sq_, int Sk_, int Hq, int Hk, Strides ks_, Strides dqs,
                                                            long long dsb, long long dsh, int dsld, float scale,
                                                            Extra ex) {
  constexpr int NT = 2, NW = 4, QB = 16 * NT * NW;  // 128 queries per block
  constexpr int DB = D / 16;
  constexpr bool BT = (fa_pitch<D>() >= 128);
  constexpr int KT = 64 * fa_pitch<D>() * 2;  // K tile bytes
  __shared__ __attribute__((aligned(16))) char smem[KT + 64 * QB * 2];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int nqb = (Sq_ + QB - 1) / QB;
  int h, b, zi;
  pair_order(Hq, (int)gridDim.y, nqb, h, b, zi);
  const int qb = nqb - 1 - zi;
  const int hk = h / (Hq / Hk);
  const Seq sq_ = seq_of<EXT != 0>(ex, b, h, Hq, Sq_, Sk_);
  const int Sq = sq_.sq, Sk = sq_.sk;
  const int q0 = qb * QB;
  if (q0 >= Sq) return;
  const int qw = q0 + wave * 16 * NT;
  const int off = Sk - Sq;
  const bool vl = EXT && ex.cu_q;
  const uint16_t* kbase = K + (vl ? 0 : (long long)b * ks_.b) + sq_.ko * ks_.s + (long long)hk * ks_.h;
  // dS^T tiles [64 keys][128 queries] of this query block: tile kb at dshead + kb * tstride
  const uint16_t* dshead = dsT + (long long)b * dsb + (long long)h * dsh + (long long)qb * 8192;
  const long long tstride = (long long)(dsld >> 7) * 8192;
  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + QB + off);
  const int nkb = kend > 0 ? (kend + 63) / 64 : 0;
  f32x4 acc[NT][DB];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int d = 0; d < DB; ++d) acc[t][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  Tile<D, 256> kt;
  Tile<128, 256> st;  // the dS^T tile: 64 key rows x 128 queries (D = 128 image)
  kt.init(kbase, ks_.s);
  st.init(dshead, 128);
  if (nkb > 0) {
    kt.load(0, Sk);
    st.load(0, Sk);
  }
  char* k_lds = smem;
  char* s_lds = smem + KT;
  for (int kb = 0; kb < nkb; ++kb) {
    const int k0 = kb * 64;
    __syncthreads();
    kt.template store<BT>(k_lds);
    st.template store<true>(s_lds);
    __syncthreads();
    if (kb + 1 < nkb) {
      kt.load(k0 + 64, Sk);
      st.init(dshead + (kb + 1) * tstride, 128);
      st.load(0, Sk - (k0 + 64));
    }
    if (CAUSAL && k0 > qw + 16 * NT - 1 + off) continue;  // whole key block above this wave's rows
    // dS^T fragments: lane (g, i) of tile t, step s: keys k0 + 32s + 4g + (0..3) / + 16, query qw + 16t + i
    s16x8 dsf[NT][2];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) dsf[t][s] = ld_tr8<128, true>(s_lds, 32 * s, (qw - q0) / 16 + t, lane);
    const bool need_mask = (k0 + 64 > Sk) || (CAUSAL && k0 + 63 > qw + off);
    if (need_mask) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int q = qw + 16 * t + (lane & 15);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int key = k0 + 32 * s + 4 * g + (e & 3) + (e >= 4 ? 16 : 0);
            const bool masked = (key >= Sk) || (CAUSAL && key > q + off);
            dsf[t][s][e] = masked ? (short)0 : dsf[t][s][e];
          }
      }
    }
    // dQ^T += K^T dS^T
#pragma unroll
    for (int d = 0; d < DB; ++d) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const s16x8 ka = ld_tr8<D, BT>(k_lds, 32 * s, d, lane);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t][d] = Mfma<T>::run(ka, dsf[t][s], acc[t][d]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int myq = qw + 16 * t + (lane & 15);
    if (myq < Sq) {
      uint16_t* row = dQ + (vl ? 0 : (long long)b * dqs.b) + (long long)h * dqs.h + (sq_.qo + myq) * dqs.s;
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        s16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2s<T>(acc[t][d][r] * scale);
        *reinterpret_cast<s16x4*>(row + 16 * d + 4 * g) = o;
      }
    }
  }
}

// dQ from dS, head_dim 128, as a stream: the kernel above is HBM-latency bound (~2.5 TB/s of dS^T:
// one tile staged ahead in registers, two barriers per key block).  Here the dS^T and K tiles of
// NS key blocks live in an LDS ring filled by LDS-DMA (global_load_lds_dwordx4, no register
// round trip): NS - 1 key blocks are in flight while one is multiplied, retired by a counted
// vmcnt, one barrier per key block.  Same grid, fragments, masking and numerics as
// dq_from_ds_kernel (the LDS images are the same swizzled [64][128] tiles).
template <typename T, bool CAUSAL, int EXT, int NS>
__global__ __launch_bounds__(256, NS == 2 ? 2 : 1) void dq_from_ds_dma_kernel(const uint16_t* __restrict__ K,
                                                                const uint16_t* __restrict__ dsT,
                                                                uint16_t* __restrict__ dQ, int Sq_, int Sk_, int Hq,
                                                                int Hk, Strides ks_, Strides dqs, long long dsb,
                                                                long long dsh, int dsld, float scale, Extra ex) {
  static_assert(NS >= 2 && NS <= 4, "ring depth 2..4 (counted waits below)");
  constexpr int D = 128, NT = 2, NW = 4, QB = 16 * NT * NW;  // 128 queries per block
  constexpr int DB = D / 16;
  constexpr int TILE = 64 * D * 2;  // one [64][128] 16-bit tile: 16 KB
  constexpr int VM = 2 * DmaTile<D, true>::NI;  // LDS-DMA instructions per wave per key block
  __shared__ __attribute__((aligned(16))) char smem[NS * 2 * TILE];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int nqb = (Sq_ + QB - 1) / QB;
  int h, b, zi;
  pair_order(Hq, (int)gridDim.y, nqb, h, b, zi);
  const int qb = nqb - 1 - zi;
  const int hk = h / (Hq / Hk);
  const Seq sq_ = seq_of<EXT != 0>(ex, b, h, Hq, Sq_, Sk_);
  const int Sq = sq_.sq, Sk = sq_.sk;
  const int q0 = qb * QB;
  if (q0 >= Sq) return;  // block-uniform: no barrier below is skipped by part of the block
  const int qw = q0 + wave * 16 * NT;
  const int off = Sk - Sq;
  const bool vl = EXT && ex.cu_q;
  const uint16_t* kbase = K + (vl ? 0 : (long long)b * ks_.b) + sq_.ko * ks_.s + (long long)hk * ks_.h;
  const uint16_t* dshead = dsT + (long long)b * dsb + (long long)h * dsh + (long long)qb * 8192;
  const long long tstride = (long long)(dsld >> 7) * 8192;
  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + QB + off);
  const int nkb = kend > 0 ? (kend + 63) / 64 : 0;
  f32x4 acc[NT][DB];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int d = 0; d < DB; ++d) acc[t][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  DmaTile<D, true> kd, sd;
  kd.init(wave, lane);
  sd.init(wave, lane);
  auto issue = [&](int kb) {
    char* slot = smem + (kb % NS) * 2 * TILE;
    kd.issue(kbase, ks_.s, kb * 64, Sk, slot, wave);
    sd.issue(dshead + kb * tstride, 128, 0, 64, slot + TILE, wave);  // every tile row exists
  };
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < nkb) issue(i);
  for (int kb = 0; kb < nkb; ++kb) {
    const int k0 = kb * 64;
    // key blocks issued beyond kb: min(NS - 2, nkb - 1 - kb); retire kb's pieces only
    const int ahead = min(NS - 2, nkb - 1 - kb);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * VM) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // raw barrier: __syncthreads() would drain every DMA in flight (its fence waits for vmcnt(0));
    // the "memory" clobbers keep the compiler from moving LDS reads across it
    __builtin_amdgcn_s_barrier();  // kb resident for every wave; every wave is done with kb - 1's slot
    asm volatile("" ::: "memory");
    if (kb + NS - 1 < nkb) issue(kb + NS - 1);
    if (CAUSAL && k0 > qw + 16 * NT - 1 + off) continue;  // whole key block above this wave's rows
    const char* k_lds = smem + (kb % NS) * 2 * TILE;
    const char* s_lds = k_lds + TILE;
    s16x8 dsf[NT][2];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) dsf[t][s] = ld_tr8<128, true>(s_lds, 32 * s, (qw - q0) / 16 + t, lane);
    const bool need_mask = (k0 + 64 > Sk) || (CAUSAL && k0 + 63 > qw + off);
    if (need_mask) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int q = qw + 16 * t + (lane & 15);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int key = k0 + 32 * s + 4 * g + (e & 3) + (e >= 4 ? 16 : 0);
            const bool masked = (key >= Sk) || (CAUSAL && key > q + off);
            dsf[t][s][e] = masked ? (short)0 : dsf[t][s][e];
          }
      }
    }
#pragma unroll
    for (int d = 0; d < DB; ++d) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const s16x8 ka = ld_tr8<D, true>(k_lds, 32 * s, d, lane);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t][d] = Mfma<T>::run(ka, dsf[t][s], acc[t][d]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int myq = qw + 16 * t + (lane & 15);
    if (myq < Sq) {
      uint16_t* row = dQ + (vl ? 0 : (long long)b * dqs.b) + (long long)h * dqs.h + (sq_.qo + myq) * dqs.s;
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        s16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2s<T>(acc[t][d][r] * scale);
        *reinterpret_cast<s16x4*>(row + 16 * d + 4 * g) = o;
      }
    }
  }
}

}  // namespace fa
}  // namespace pa

using namespace pa;
using namespace pa::fa;

// A/B switch (pa_flash_ds_set_dq_dma): the LDS-DMA ring dQ kernel at head_dim 128 (0 = the
// register-staged kernel); host-side, read at launch.  The kernel is bound by its LDS operand
// reads (each K fragment feeds two MFMAs), not by the prefetch depth: see the measurements below.
static int g_dq_dma = 2;

#define FAD_DISPATCH(dt, D, causal, ...)                                                                          \
  if (dt == 1 && D == 128 && causal) { using T = bf16_t; constexpr int DD = 128; constexpr bool CC = true; __VA_ARGS__; }        \
  else if (dt == 1 && D == 128 && !causal) { using T = bf16_t; constexpr int DD = 128; constexpr bool CC = false; __VA_ARGS__; } \
  else if (dt == 1 && D == 64 && causal) { using T = bf16_t; constexpr int DD = 64; constexpr bool CC = true; __VA_ARGS__; }     \
  else if (dt == 1 && D == 64 && !causal) { using T = bf16_t; constexpr int DD = 64; constexpr bool CC = false; __VA_ARGS__; }   \
  else if (dt == 2 && D == 128 && causal) { using T = f16_t; constexpr int DD = 128; constexpr bool CC = true; __VA_ARGS__; }    \
  else if (dt == 2 && D == 128 && !causal) { using T = f16_t; constexpr int DD = 128; constexpr bool CC = false; __VA_ARGS__; }  \
  else if (dt == 2 && D == 64 && causal) { using T = f16_t; constexpr int DD = 64; constexpr bool CC = true; __VA_ARGS__; }      \
  else if (dt == 2 && D == 64 && !causal) { using T = f16_t; constexpr int DD = 64; constexpr bool CC = false; __VA_ARGS__; }    \
  else return hipErrorInvalidValue;

// block order of this module's kernels (pair_order's G; the module has its own copy of the
// constant): returns the previous value
PA_API int pa_flash_ds_set_pair_group(int v) {
  int old = 0;
  (void)hipMemcpyFromSymbol(&old, HIP_SYMBOL(pa::fa::g_pair_group), sizeof(int));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(pa::fa::g_pair_group), &v, sizeof(int));
  return old;
}

// dS^T workspace geometry: per (b, h) ceil(Sk / 64) x ceil(Sq / 128) tiles of [64][128] elements
// (dsld = ceil(Sq / 128) * 128 elements per 64-key tile row)
PA_API int pa_flash_ds_ld(int Sq) { return (Sq + 127) / 128 * 128; }
PA_API long long pa_flash_ds_ws_elems(int B, int Hq, int Sq, int Sk) {
  return (long long)B * Hq * ((Sk + 63) / 64 * 64) * pa_flash_ds_ld(Sq);
}

template <typename T, int DD, bool CC, int F>
static void bwd_ds(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                   float* delta, void* dq, void* dk, void* dv, void* dsT, int B, int Sq, int Sk, int Hq, int Hk,
                   Strides qs, Strides ks, Strides vs, Strides os, Strides dos, Strides dqs, Strides dks, Strides dvs,
                   float scale, const Extra& ex, hipStream_t st) {
  constexpr int NW = DD == 128 ? 8 : 4;
  const int dsld = pa_flash_ds_ld(Sq);
  const long long dsh = (long long)((Sk + 63) / 64 * 64) * dsld, dsb = (long long)Hq * dsh;
  delta_kernel<T, DD, F><<<dim3(Hq, B, (Sq + 63) / 64), 256, 0, st>>>((const uint16_t*)o, (const uint16_t*)dout,
                                                                      delta, Sq, Sk, Hq, os, dos, ex);
  bwd_dkdv_kernel<T, DD, CC, 1, NW, F, false, true><<<dim3(Hq, B, (Sk + 16 * NW - 1) / (16 * NW)), 64 * NW, 0, st>>>(
      (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta, (uint16_t*)dk,
      (uint16_t*)dv, Sq, Sk, Hq, Hk, qs, ks, vs, dos, dks, dvs, scale, ex, (uint16_t*)dsT, dsb, dsh, dsld);
  const dim3 qgrid(Hq, B, (Sq + 127) / 128);
  if constexpr (DD == 128) {
    if (g_dq_dma == 2) {
      dq_from_ds_dma_kernel<T, CC, F, 2><<<qgrid, 256, 0, st>>>((const uint16_t*)k, (const uint16_t*)dsT, (uint16_t*)dq,
                                                                Sq, Sk, Hq, Hk, ks, dqs, dsb, dsh, dsld, scale, ex);
      return;
    }
  }
  dq_from_ds_kernel<T, DD, CC, F><<<qgrid, 256, 0, st>>>((const uint16_t*)k, (const uint16_t*)dsT, (uint16_t*)dq, Sq,
                                                           Sk, Hq, Hk, ks, dqs, dsb, dsh, dsld, scale, ex);
}

// A/B: 0 = register-staged dQ kernel, 2 = the LDS-DMA ring (GPT-3 1.3B shape: 109.6 vs 111.5 us;
// ring depths 3 / 4 at one block per CU were 143 / 153 us, profiles/r6q_dq_from_ds_ring_ab.log)
PA_API int pa_flash_ds_set_dq_dma(int v) {
  const int old = g_dq_dma;
  g_dq_dma = v;
  return old;
}

// Same contract as pa_flash_bwd_ex (cu_q == null: dense; mask / dropout / flashmask rows optional)
// plus the dS^T workspace: pa_flash_ds_ws_elems(B, Hq, Sq, Sk) elements of the activation dtype
// (varlen: B sequences, Sq / Sk the maximum lengths).
PA_API hipError_t pa_flash_bwd_ds(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                  const float* lse, float* delta, void* dq, void* dk, void* dv, void* dsT, int B,
                                  int Sq, int Sk, int Hq, int Hk, int D, const long long* qst, const long long* kst,
                                  const long long* vst, const long long* ost, const long long* dost,
                                  const long long* dqst, const long long* dkst, const long long* dvst, float scale,
                                  int causal, int dt, const int* cu_q, const int* cu_k, int total_q, const void* mask,
                                  long long mb, long long mh, long long mq, int mask_f32, float p_drop, unsigned seed,
                                  unsigned offset, const int* rows, long long rb, long long rh, const int* mask_all,
                                  hipStream_t st) {
  if (Hk <= 0 || Hq % Hk != 0 || (cu_q == nullptr) != (cu_k == nullptr) || dsT == nullptr) return hipErrorInvalidValue;
  if (mask && rows) return hipErrorInvalidValue;
  Strides qs{qst[0], qst[1], qst[2]}, ks{kst[0], kst[1], kst[2]}, vs{vst[0], vst[1], vst[2]},
      os{ost[0], ost[1], ost[2]}, dos{dost[0], dost[1], dost[2]}, dqs{dqst[0], dqst[1], dqst[2]},
      dks{dkst[0], dkst[1], dkst[2]}, dvs{dvst[0], dvst[1], dvst[2]};
  Extra ex;
  ex.rows = rows;
  ex.rb = rb;
  ex.rh = rh;
  ex.cu_q = cu_q;
  ex.cu_k = cu_k;
  ex.total_q = total_q;
  ex.mask = mask;
  ex.mb = mb;
  ex.mh = mh;
  ex.mq = mq;
  ex.mask_f32 = mask_f32;
  ex.mask_all = mask ? mask_all : nullptr;
  ex.p_drop = p_drop;
  ex.seed = seed;
  ex.offset = offset;
  const int th = (int)((double)p_drop * 256.0 + 0.5);
  ex.drop_thresh = (uint32_t)(th > 256 ? 256 : th);
  ex.keep_scale = ex.drop_thresh < 256 ? 256.f / (256.f - (float)ex.drop_thresh) : 0.f;
  const bool any = cu_q || mask || rows || p_drop > 0.f;
  const int feat = any ? (1 | (mask ? 2 : 0) | (p_drop > 0.f ? 4 : 0) | (rows ? 8 : 0)) : 0;
  FAD_DISPATCH(dt, D, causal, {
    switch (feat) {
      case 0: bwd_ds<T, DD, CC, 0>(q, k, v, o, dout, lse, delta, dq, dk, dv, dsT, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
      case 1: bwd_ds<T, DD, CC, 1>(q, k, v, o, dout, lse, delta, dq, dk, dv, dsT, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
      case 3: bwd_ds<T, DD, CC, 3>(q, k, v, o, dout, lse, delta, dq, dk, dv, dsT, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
      case 5: bwd_ds<T, DD, CC, 5>(q, k, v, o, dout, lse, delta, dq, dk, dv, dsT, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
      case 7: bwd_ds<T, DD, CC, 7>(q, k, v, o, dout, lse, delta, dq, dk, dv, dsT, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
      case 9: bwd_ds<T, DD, CC, 9>(q, k, v, o, dout, lse, delta, dq, dk, dv, dsT, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
      default: bwd_ds<T, DD, CC, 13>(q, k, v, o, dout, lse, delta, dq, dk, dv, dsT, B, Sq, Sk, Hq, Hk, qs, ks, vs, os, dos, dqs, dks, dvs, scale, ex, st); break;
    }
  });
  return hipGetLastError();
}

// graph-safe dropout streams for this module's kernels (see pa_flash_set_rng_gen)
PA_API int pa_flash_ds_set_rng_gen(const void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(pa::g_rng_gen), &p, sizeof(p));
}
