// Decode-phase attention for generation: one new query token per sequence attending over a KV
// cache, contiguous ([2, B, Hkv, max_len, D], the fused_multi_transformer / masked_multihead_attention
// layout) or paged ([num_blocks, Hkv, block_size, D] + block_tables, block_multihead_attention).
//
// Reference semantics: paddle/phi/kernels/fusion/gpu/masked_multihead_attention_kernel.cu:660,
// block_multi_head_attention_kernel.cu:886 (decoder branch), python/paddle/incubate/nn/functional/
// masked_multihead_attention.py, block_multihead_attention.py.
//
// MI355X design.  Decode attention is a pure HBM stream over the cache (every K/V byte is read
// once per step), so the kernel is shaped for bytes in flight, not for MFMA:
//  * split-K over the sequence (flash-decoding): grid (splits, Hkv, B), each block streams a
//    contiguous chunk of positions of one KV head for ALL query heads of its GQA group (the K/V
//    bytes are read once per group, not once per query head); partial (max, sum, acc[D]) are
//    combined by a second tiny kernel (or written directly when there is one split);
//  * 16 lanes per position: a wave reads 4 positions (4 x D x 2 B, fully coalesced 16-B loads)
//    per K (and V) load instruction; 4 waves x 4 unrolled steps keep 64 positions = 32 KB per
//    block (D=128) in flight, several blocks per CU;
//  * q . k reduced across the 16 lanes with 4 xor-shuffles; online softmax per lane group in
//    fp32 (exp2 domain, scale folded); the 16 lane groups of a block are merged through LDS.
//  * new K/V of the step are written into the cache by pa_kv_cache_write (bias fused) before the
//    attention launch, so the attention blocks only ever read the cache.
#include "common.h"

namespace pa {
namespace dec {

constexpr float kLog2e = 1.4426950408889634f;

template <typename T, int N>
__device__ __forceinline__ void ld16(const T* p, float (&o)[N]) {
  if constexpr (N == 16) {
    float a[8], b[8];
    load_f<T, 8>(p, a);
    load_f<T, 8>(p + 8, b);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      o[i] = a[i];
      o[8 + i] = b[i];
    }
  } else {
    load_f<T, N>(p, o);
  }
}

struct Cache {
  const void* k;
  const void* v;
  const int* block_tables;  // paged: [B, max_blocks]
  int max_blocks, block_size;
  long long max_len;        // contiguous: positions per (b, head)
};

template <bool PAGED>
__device__ __forceinline__ long long pos_off(const Cache& c, int b, int hk, int Hkv, int p, int D) {
  if constexpr (PAGED) {
    const int blk = c.block_tables[(long long)b * c.max_blocks + p / c.block_size];
    return (((long long)blk * Hkv + hk) * c.block_size + (p % c.block_size)) * D;
  } else {
    return (((long long)b * Hkv + hk) * c.max_len + p) * D;
  }
}

// Sum over the 16 lanes of a DPP row (all 16 lanes get the total): xor-1 and xor-2 quad
// permutes, then half-row and row mirrors.  VALU-only (no LDS crossbar, unlike __shfl_xor).
__device__ __forceinline__ float row_sum16(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

// cache element -> float: bf16 / fp16 as is; int8 caches store round(x * quant_scale), uint8 ones
// the same offset by 128 (the reference's layout); the dequant scale is folded in elsewhere
__device__ __forceinline__ float cvt(bf16_t v) { return (float)v; }
__device__ __forceinline__ float cvt(f16_t v) { return (float)v; }
__device__ __forceinline__ float cvt(int8_t v) { return (float)v; }
__device__ __forceinline__ float cvt(uint8_t v) { return (float)v - 128.f; }

template <typename T, int N>
__device__ __forceinline__ void unpack(const Pack<T, N>& p, float (&o)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) o[i] = cvt(p.v[i]);
}

// Dequantisation of an 8-bit KV cache: per KV head (static, sb = 0) or per (sequence, KV head)
// (dynamic, sb = Hkv) scales.  The K scale is folded into the query (q . (s k) = s (q . k)); the V
// scale multiplies the merged accumulator (constant over the positions of a (sequence, head)).
struct Deq {
  const float* ks = nullptr;
  const float* vs = nullptr;
  long long sb = 0;
};

// grid (nsplit, Hkv, B), 256 threads.  G = query heads per KV head (GQA group size), D head dim.
// q: [B, Hq*D] rows of stride q_stride (elements) (+ optional q bias [Hq*D]).
// lens[b]: number of cache positions to attend (the new token included).
// mask: optional additive fp32 [B, mask_stride] over positions.
// out: [B, Hq, D] (stride out_stride per row) when nsplit == 1, else partials to ws:
//   ws[((b*Hq + h)*nsplit + s)*(D+2)] = {m, l, acc[0..D)}.
// A block iteration covers 16*U consecutive positions: lane group (wave, grp) owns positions
// base + 16u + 4*wave + grp.  Raw K/V stay packed in registers until used; the softmax of a lane
// group is updated once per iteration (one max / rescale per head for its U positions).
// Paged caches with block_size % (16*U) == 0 and an aligned chunk look the block id up once per
// iteration (a wave-uniform scalar load) instead of once per position.  8-bit caches issue the
// loads of iteration i+1 before the math of iteration i (two register sets of raw K/V).
template <typename T, int D, int G, bool PAGED, typename CT = T>
__global__ __launch_bounds__(256) void attn_split_kernel(const T* __restrict__ q, long long q_stride,
                                                         const T* __restrict__ q_bias, Cache cache,
                                                         const int* __restrict__ lens, const float* __restrict__ mask,
                                                         long long mask_stride, T* __restrict__ out,
                                                         long long out_stride, float* __restrict__ ws, int Hq, int Hkv,
                                                         int nsplit, int chunk, float scale, Deq dq = Deq{}) {
  constexpr int EPL = D / 16;  // elements per lane
  constexpr int U = 4;         // positions per lane group per iteration
  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = lane >> 4, sub = lane & 15;
  const int len = lens[b];
  const int p0 = split * chunk, p1 = min(len, p0 + chunk);
  const float sl2 = scale * kLog2e;

  float qf[G][EPL];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int h = hk * G + g;
    ld16<T, EPL>(q + (long long)b * q_stride + (long long)h * D + sub * EPL, qf[g]);
    if (q_bias) {
      float bb[EPL];
      ld16<T, EPL>(q_bias + (long long)h * D + sub * EPL, bb);
#pragma unroll
      for (int e = 0; e < EPL; ++e) qf[g][e] += bb[e];
    }
    const float ksc = dq.ks != nullptr ? dq.ks[(long long)b * dq.sb + hk] : 1.f;  // 8-bit cache: K dequant
#pragma unroll
    for (int e = 0; e < EPL; ++e) qf[g][e] *= sl2 * ksc;  // scores come out in log2 units
  }
  const float vsc = dq.vs != nullptr ? dq.vs[(long long)b * dq.sb + hk] : 1.f;  // 8-bit cache: V dequant
  float m[G], l[G], acc[G][EPL];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) acc[g][e] = 0.f;
  }
  const CT* kc = reinterpret_cast<const CT*>(cache.k);
  const CT* vc = reinterpret_cast<const CT*>(cache.v);
  typedef Pack<CT, EPL> PK;
  const bool blk_aligned = PAGED && (cache.block_size % (16 * U) == 0) && (chunk % (16 * U) == 0);
  // K/V of iteration `base` -> registers (lanes past p1 load nothing)
  auto load = [&](int base, PK (&kr)[U], PK (&vr)[U], bool (&ok)[U]) {
    long long o0 = 0;
    if (PAGED && blk_aligned && base < p1) {
      const int blk = cache.block_tables[(long long)b * cache.max_blocks + base / cache.block_size];
      o0 = (((long long)blk * Hkv + hk) * cache.block_size + (base % cache.block_size)) * D;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rel = 16 * u + 4 * wave + grp;
      ok[u] = base + rel < p1;
      if (ok[u]) {
        const long long o = (PAGED && blk_aligned) ? o0 + (long long)rel * D + sub * EPL
                                                   : pos_off<PAGED>(cache, b, hk, Hkv, base + rel, D) + sub * EPL;
        kr[u] = *reinterpret_cast<const PK*>(kc + o);
        vr[u] = *reinterpret_cast<const PK*>(vc + o);
      }
    }
  };
  // one iteration's math on raw K/V registers (positions base + 16u + 4*wave + grp)
  auto step = [&](int base, const PK (&kr)[U], const PK (&vr)[U], const bool (&ok)[U]) {
    float sc[G][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float kf[EPL];
      unpack<CT, EPL>(kr[u], kf);
      const float mk = (mask && ok[u]) ? mask[(long long)b * mask_stride + base + 16 * u + 4 * wave + grp] * kLog2e
                                       : 0.f;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float sdot = 0.f;
#pragma unroll
        for (int e = 0; e < EPL; ++e) sdot += qf[g][e] * kf[e];
        sc[g][u] = ok[u] ? row_sum16(sdot) + mk : -INFINITY;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float mx = sc[g][0];
#pragma unroll
      for (int u = 1; u < U; ++u) mx = fmaxf(mx, sc[g][u]);
      const float mn = fmaxf(m[g], mx);
      if (mn == -INFINITY) continue;  // nothing valid yet for this group (uniform over the row)
      const float a = __builtin_amdgcn_exp2f(m[g] - mn);
      m[g] = mn;
      l[g] *= a;
#pragma unroll
      for (int e = 0; e < EPL; ++e) acc[g][e] *= a;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float pr = __builtin_amdgcn_exp2f(sc[g][u] - mn);
        l[g] += pr;
        if (ok[u]) {
          float vf[EPL];
          unpack<CT, EPL>(vr[u], vf);
#pragma unroll
          for (int e = 0; e < EPL; ++e) acc[g][e] += pr * vf[e];
        }
      }
    }
  };
  PK kr[U], vr[U];
  bool ok[U];
  if constexpr (sizeof(CT) == 1) {
    // 8-bit caches: software pipeline, the next iteration's K/V in flight while this one computes
    // (half-size raw registers; measured 1.1-1.2x on the int8 path, a loss for 16-bit caches,
    // whose larger register sets cost occupancy)
    load(p0, kr, vr, ok);
    for (int base = p0; base < p1; base += 16 * U) {
      PK kn[U], vn[U];
      bool okn[U];
      load(base + 16 * U, kn, vn, okn);
      step(base, kr, vr, ok);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        kr[u] = kn[u];
        vr[u] = vn[u];
        ok[u] = okn[u];
      }
    }
  } else {
    for (int base = p0; base < p1; base += 16 * U) {
      load(base, kr, vr, ok);
      step(base, kr, vr, ok);
    }
  }

  // merge the 16 lane groups of the block: LDS [16 groups][G][D + 2]
  __shared__ float red[16][G][D + 2];
  const int gid = wave * 4 + grp;
#pragma unroll
  for (int g = 0; g < G; ++g) {
#pragma unroll
    for (int e = 0; e < EPL; ++e) red[gid][g][sub * EPL + e] = acc[g][e];
    if (sub == 0) {
      red[gid][g][D] = m[g];
      red[gid][g][D + 1] = l[g];
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < G * D; t += 256) {
    const int g = t / D, d = t % D;
    float M = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) M = fmaxf(M, red[i][g][D]);
    float L = 0.f, A = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float w = __builtin_amdgcn_exp2f(red[i][g][D] - M);
        L += red[i][g][D + 1] * w;
        A += red[i][g][d] * w;
      }
    }
    A *= vsc;
    const int h = hk * G + g;
    if (nsplit == 1) {
      out[(long long)b * out_stride + (long long)h * D + d] = from_f<T>(L > 0.f ? A / L : 0.f);
    } else {
      float* w = ws + (((long long)b * Hq + h) * nsplit + split) * (D + 2);
      w[d] = A;
      if (d == 0) {
        w[D] = M;
        w[D + 1] = L;
      }
    }
  }
}

// combine split partials: one block of D threads per (b, h)
template <typename T, int D>
__global__ void combine_kernel(const float* __restrict__ ws, T* __restrict__ out, long long out_stride, int Hq,
                               int nsplit) {
  const int bh = blockIdx.x, d = threadIdx.x;
  const int b = bh / Hq, h = bh % Hq;
  const float* w = ws + (long long)bh * nsplit * (D + 2);
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, w[s * (D + 2) + D]);
  float L = 0.f, A = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < nsplit; ++s) {
      const float x = __builtin_amdgcn_exp2f(w[s * (D + 2) + D] - M);
      L += w[s * (D + 2) + D + 1] * x;
      A += w[s * (D + 2) + d] * x;
    }
  }
  out[(long long)b * out_stride + (long long)h * D + d] = from_f<T>(L > 0.f ? A / L : 0.f);
}

// Write K and V rows (+ bias) into the cache (paged or contiguous): row r of knew/vnew (stride
// kv_stride, head h at h*D) goes to sequence seq_of[r] (r itself when seq_of is null) at position
// pos[r] (< 0 skips the row).  grid (rows, Hkv).  Decode: one row per sequence; prefill (block
// attention): one row per prompt token.
template <typename T, bool PAGED>
__global__ void kv_write_kernel(const T* __restrict__ knew, const T* __restrict__ vnew, long long kv_stride,
                                const T* __restrict__ kbias, const T* __restrict__ vbias, Cache cache,
                                const int* __restrict__ seq_of, const int* __restrict__ pos, int Hkv, int D) {
  const int r = blockIdx.x, hk = blockIdx.y;
  const int b = seq_of ? seq_of[r] : r;
  const int p = pos[r];
  if (p < 0) return;
  const long long o = pos_off<PAGED>(cache, b, hk, Hkv, p, D);
  T* kc = reinterpret_cast<T*>(const_cast<void*>(cache.k));
  T* vc = reinterpret_cast<T*>(const_cast<void*>(cache.v));
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float kk = to_f(knew[(long long)r * kv_stride + (long long)hk * D + d]);
    float vv = to_f(vnew[(long long)r * kv_stride + (long long)hk * D + d]);
    if (kbias) kk += to_f(kbias[(long long)hk * D + d]);
    if (vbias) vv += to_f(vbias[(long long)hk * D + d]);
    kc[o + d] = from_f<T>(kk);
    vc[o + d] = from_f<T>(vv);
  }
}

// Quantising variant for 8-bit caches: q = clip(round(x * quant_scale), qmin, qmax) (+128 for
// uint8), quant scales per KV head (sb = 0) or per (sequence, head) (sb = Hkv).  round_type 0:
// half to even (rint), 1: half away from zero.
template <typename T, bool PAGED, typename CT>
__global__ void kv_write_q8_kernel(const T* __restrict__ knew, const T* __restrict__ vnew, long long kv_stride,
                                   Cache cache, const int* __restrict__ seq_of, const int* __restrict__ pos, int Hkv,
                                   int D, const float* __restrict__ kqs, const float* __restrict__ vqs, long long sb,
                                   int round_type, float qmax, float qmin) {
  const int r = blockIdx.x, hk = blockIdx.y;
  const int b = seq_of ? seq_of[r] : r;
  const int p = pos[r];
  if (p < 0) return;
  const long long o = pos_off<PAGED>(cache, b, hk, Hkv, p, D);
  CT* kc = reinterpret_cast<CT*>(const_cast<void*>(cache.k));
  CT* vc = reinterpret_cast<CT*>(const_cast<void*>(cache.v));
  const float ks = kqs[(long long)b * sb + hk], vs = vqs[(long long)b * sb + hk];
  const float zp = sizeof(CT) == 1 && CT(-1) > CT(0) ? 128.f : 0.f;  // unsigned cache: offset by 128
  auto qz = [&](float x) {
    const float y = round_type == 0 ? rintf(x) : roundf(x);
    return CT(fminf(fmaxf(y, qmin), qmax) + zp);
  };
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    kc[o + d] = qz(to_f(knew[(long long)r * kv_stride + (long long)hk * D + d]) * ks);
    vc[o + d] = qz(to_f(vnew[(long long)r * kv_stride + (long long)hk * D + d]) * vs);
  }
}

template <typename T, int D, int G, bool PAGED, typename CT = T>
static hipError_t launch_attn(const void* q, long long q_stride, const void* q_bias, const Cache& c, const int* lens,
                              const float* mask, long long mask_stride, void* out, long long out_stride, float* ws,
                              int B, int Hq, int Hkv, int max_len, int nsplit, float scale, hipStream_t st,
                              const Deq& dq = Deq{}) {
  if constexpr (D * G > 1024) {
    return hipErrorInvalidValue;  // outside pa_decode_ok (not instantiated)
  } else {
  int chunk = (max_len + nsplit - 1) / nsplit;
  chunk = (chunk + 63) / 64 * 64;  // whole 64-position iterations (aligned paged lookups)
  dim3 grid(nsplit, Hkv, B);
  attn_split_kernel<T, D, G, PAGED, CT><<<grid, 256, 0, st>>>((const T*)q, q_stride, (const T*)q_bias, c, lens, mask,
                                                              mask_stride, (T*)out, out_stride, ws, Hq, Hkv, nsplit,
                                                              chunk, scale, dq);
  if (nsplit > 1) combine_kernel<T, D><<<B * Hq, D, 0, st>>>(ws, (T*)out, out_stride, Hq, nsplit);
  return hipGetLastError();
  }
}

template <typename T, int D, bool PAGED, typename CT = T>
static hipError_t dispatch_g(int G, const void* q, long long q_stride, const void* q_bias, const Cache& c,
                             const int* lens, const float* mask, long long mask_stride, void* out, long long out_stride,
                             float* ws, int B, int Hq, int Hkv, int max_len, int nsplit, float scale, hipStream_t st,
                             const Deq& dq = Deq{}) {
#define PA_DEC_G(GG)                                                                                                 \
  case GG:                                                                                                           \
    return launch_attn<T, D, GG, PAGED, CT>(q, q_stride, q_bias, c, lens, mask, mask_stride, out, out_stride, ws, B, \
                                            Hq, Hkv, max_len, nsplit, scale, st, dq);
  switch (G) {
    PA_DEC_G(1)
    PA_DEC_G(2)
    PA_DEC_G(4)
    PA_DEC_G(5)
    PA_DEC_G(8)
    default: return hipErrorInvalidValue;
  }
#undef PA_DEC_G
}

}  // namespace dec
}  // namespace pa

using namespace pa::dec;

// Number of sequence splits for a decode launch (>= ~8 blocks per CU, >= 256 positions each).
PA_API int pa_decode_nsplit(int B, int Hkv, int max_len) {
  int s = 1;
  while ((long long)B * Hkv * s < 2048 && (max_len + 2 * s - 1) / (2 * s) >= 256 && s < 64) s *= 2;
  return s;
}

// Supported: dtype 1 (bf16) / 2 (fp16); D in {64, 128, 256}; G = Hq/Hkv in {1, 2, 4, 5, 8}.
PA_API int pa_decode_ok(int dtype, int D, int G) {
  return (dtype == 1 || dtype == 2) && (D == 64 || D == 128 || D == 256) &&
         (G == 1 || G == 2 || G == 4 || G == 5 || G == 8) && (D * G <= 1024);
}

// q: [B, >= Hq*D] rows (stride q_stride); cache k/v base pointers; paged when block_tables != null
// (then max_blocks/block_size describe it), else contiguous with max_len positions per (b, head).
// lens: int32 [B]; mask: optional fp32 [B, mask_stride]; ws: B*Hq*nsplit*(D+2) floats when nsplit>1.
PA_API int pa_decode_attn(int dtype, const void* q, long long q_stride, const void* q_bias, const void* kc,
                          const void* vc, const int* block_tables, int max_blocks, int block_size, long long max_len,
                          const int* lens, const float* mask, long long mask_stride, void* out, long long out_stride,
                          float* ws, int B, int Hq, int Hkv, int D, int nsplit, float scale, hipStream_t st) {
  if (Hkv <= 0 || Hq % Hkv) return (int)hipErrorInvalidValue;
  const int G = Hq / Hkv;
  if (!pa_decode_ok(dtype, D, G) || (nsplit > 1 && !ws)) return (int)hipErrorInvalidValue;
  Cache c{kc, vc, block_tables, max_blocks, block_size, max_len};
  const int span = block_tables ? max_blocks * block_size : (int)max_len;
  const bool paged = block_tables != nullptr;
#define PA_DEC_D(TT, DD)                                                                                           \
  if (D == DD) {                                                                                                   \
    if (paged)                                                                                                     \
      return (int)dispatch_g<TT, DD, true>(G, q, q_stride, q_bias, c, lens, mask, mask_stride, out, out_stride, ws, \
                                           B, Hq, Hkv, span, nsplit, scale, st);                                   \
    return (int)dispatch_g<TT, DD, false>(G, q, q_stride, q_bias, c, lens, mask, mask_stride, out, out_stride, ws,  \
                                          B, Hq, Hkv, span, nsplit, scale, st);                                    \
  }
  if (dtype == 1) {
    PA_DEC_D(pa::bf16_t, 64)
    PA_DEC_D(pa::bf16_t, 128)
    PA_DEC_D(pa::bf16_t, 256)
  } else {
    PA_DEC_D(pa::f16_t, 64)
    PA_DEC_D(pa::f16_t, 128)
    PA_DEC_D(pa::f16_t, 256)
  }
#undef PA_DEC_D
  return (int)hipErrorInvalidValue;
}

// Quantising cache write into an 8-bit cache (cdt 3: int8, 4: uint8 with zero point 128): rows of
// knew / vnew (dtype 1 bf16 / 2 fp16, stride kv_stride) at pos[r] of sequence seq_of[r];
// quant scales kqs / vqs [Hkv] (scale_b_stride 0) or [B, Hkv] (scale_b_stride Hkv).
PA_API int pa_kv_cache_write_q8(int dtype, int cdt, const void* knew, const void* vnew, long long kv_stride, void* kc,
                                void* vc, const int* block_tables, int max_blocks, int block_size, long long max_len,
                                const int* seq_of, const int* pos, int R, int Hkv, int D, const float* kqs,
                                const float* vqs, long long scale_b_stride, int round_type, float qmax, float qmin,
                                hipStream_t st) {
  if (R <= 0) return 0;
  if ((dtype != 1 && dtype != 2) || (cdt != 3 && cdt != 4) || !kqs || !vqs || Hkv <= 0 || D <= 0)
    return (int)hipErrorInvalidValue;
  Cache c{kc, vc, block_tables, max_blocks, block_size, max_len};
  dim3 grid(R, Hkv);
  const int th = D >= 256 ? 256 : (D + 63) / 64 * 64;
#define PA_KVQ(TT, CT, PG)                                                                                      \
  kv_write_q8_kernel<TT, PG, CT><<<grid, th, 0, st>>>((const TT*)knew, (const TT*)vnew, kv_stride, c, seq_of, pos, \
                                                       Hkv, D, kqs, vqs, scale_b_stride, round_type, qmax, qmin)
#define PA_KVQ_T(TT)                                                           \
  if (cdt == 3) {                                                              \
    if (block_tables) PA_KVQ(TT, int8_t, true); else PA_KVQ(TT, int8_t, false);  \
  } else {                                                                     \
    if (block_tables) PA_KVQ(TT, uint8_t, true); else PA_KVQ(TT, uint8_t, false); \
  }
  if (dtype == 1) {
    PA_KVQ_T(pa::bf16_t)
  } else {
    PA_KVQ_T(pa::f16_t)
  }
#undef PA_KVQ_T
#undef PA_KVQ
  return (int)hipGetLastError();
}

// Decode over an 8-bit KV cache (cdt 3: int8 q = round(x * quant_scale); 4: uint8 = that + 128),
// dequantised in the kernel: kscale / vscale [Hkv] (static) or [B, Hkv] (dynamic: scale_b_stride
// = Hkv).  bf16 queries / outputs, D in {64, 128}; otherwise as pa_decode_attn.
PA_API int pa_decode_attn_q8(int cdt, const void* q, long long q_stride, const void* q_bias, const void* kc,
                             const void* vc, const int* block_tables, int max_blocks, int block_size,
                             long long max_len, const int* lens, const float* mask, long long mask_stride, void* out,
                             long long out_stride, float* ws, int B, int Hq, int Hkv, int D, int nsplit, float scale,
                             const float* kscale, const float* vscale, long long scale_b_stride, hipStream_t st) {
  if (Hkv <= 0 || Hq % Hkv || (cdt != 3 && cdt != 4) || !kscale || !vscale) return (int)hipErrorInvalidValue;
  const int G = Hq / Hkv;
  if (!pa_decode_ok(1, D, G) || D == 256 || (nsplit > 1 && !ws)) return (int)hipErrorInvalidValue;
  Cache c{kc, vc, block_tables, max_blocks, block_size, max_len};
  Deq dq;
  dq.ks = kscale;
  dq.vs = vscale;
  dq.sb = scale_b_stride;
  const int span = block_tables ? max_blocks * block_size : (int)max_len;
  const bool paged = block_tables != nullptr;
#define PA_DEC_Q(CT, DD)                                                                                             \
  if (D == DD) {                                                                                                    \
    if (paged)                                                                                                      \
      return (int)dispatch_g<pa::bf16_t, DD, true, CT>(G, q, q_stride, q_bias, c, lens, mask, mask_stride, out,      \
                                                       out_stride, ws, B, Hq, Hkv, span, nsplit, scale, st, dq);     \
    return (int)dispatch_g<pa::bf16_t, DD, false, CT>(G, q, q_stride, q_bias, c, lens, mask, mask_stride, out,       \
                                                      out_stride, ws, B, Hq, Hkv, span, nsplit, scale, st, dq);      \
  }
  if (cdt == 3) {
    PA_DEC_Q(int8_t, 64)
    PA_DEC_Q(int8_t, 128)
  } else {
    PA_DEC_Q(uint8_t, 64)
    PA_DEC_Q(uint8_t, 128)
  }
#undef PA_DEC_Q
  return (int)hipErrorInvalidValue;
}

// Cache update: rows of knew/vnew (stride kv_stride) with optional biases [Hkv*D] written for
// sequence seq_of[r] (null: r) at pos[r] (int32; < 0 skips the row).
PA_API int pa_kv_cache_write(int dtype, const void* knew, const void* vnew, long long kv_stride, const void* kbias,
                             const void* vbias, const void* kc, const void* vc, const int* block_tables,
                             int max_blocks, int block_size, long long max_len, const int* seq_of, const int* pos,
                             int rows, int Hkv, int D, hipStream_t st) {
  Cache c{kc, vc, block_tables, max_blocks, block_size, max_len};
  dim3 grid(rows, Hkv);
  const int thr = D < 256 ? D : 256;
  if (dtype == 1) {
    if (block_tables)
      kv_write_kernel<pa::bf16_t, true><<<grid, thr, 0, st>>>((const pa::bf16_t*)knew, (const pa::bf16_t*)vnew,
                                                              kv_stride, (const pa::bf16_t*)kbias,
                                                              (const pa::bf16_t*)vbias, c, seq_of, pos, Hkv, D);
    else
      kv_write_kernel<pa::bf16_t, false><<<grid, thr, 0, st>>>((const pa::bf16_t*)knew, (const pa::bf16_t*)vnew,
                                                               kv_stride, (const pa::bf16_t*)kbias,
                                                               (const pa::bf16_t*)vbias, c, seq_of, pos, Hkv, D);
  } else if (dtype == 2) {
    if (block_tables)
      kv_write_kernel<pa::f16_t, true><<<grid, thr, 0, st>>>((const pa::f16_t*)knew, (const pa::f16_t*)vnew, kv_stride,
                                                             (const pa::f16_t*)kbias, (const pa::f16_t*)vbias, c, seq_of,
                                                             pos, Hkv, D);
    else
      kv_write_kernel<pa::f16_t, false><<<grid, thr, 0, st>>>((const pa::f16_t*)knew, (const pa::f16_t*)vnew,
                                                              kv_stride, (const pa::f16_t*)kbias,
                                                              (const pa::f16_t*)vbias, c, seq_of, pos, Hkv, D);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
