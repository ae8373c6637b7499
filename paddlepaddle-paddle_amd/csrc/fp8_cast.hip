// FP8 training casts for gfx950: bf16 -> OCP e4m3fn / e5m2 with delayed (amax-history) scaling,
// writing the row-major image and/or its transpose in ONE pass over the bf16 tensor.
//
// An fp8 Linear needs every operand k-contiguous for the TN fp8 GEMM (csrc/gemm.hip):
//   forward  Y  = X  @ W        A = X  [M,K]     B = W^T  [N,K]   (weight transposed)
//   dgrad    dX = dY @ W^T      A = dY [M,N]     B = W    [K,N]   (weight as stored)
//   wgrad    dW = X^T @ dY      A = X^T [K,M]    B = dY^T [N,M]   (both transposed)
// so X, W and dY are each needed in both orientations: a cast that emits q and q^T together
// reads the bf16 tensor once (reference role: the cast + transpose of an fp8 training recipe;
// the reference framework itself has no fp8 path — see SURVEY §2 row "fp8 GEMM").
//
// Scaling (delayed, no host sync): hist[L] is the tensor's amax history on the device.  The
// quantisation scale is fmax / max(hist[j], j != cur, cur+1) / 2^margin (1 when the history is
// empty), every block folds its tile amax into hist[cur] (float atomicMax on the bit pattern —
// amax >= 0, so the unsigned order is the float order), and block 0 zeroes hist[cur+1], the
// slot the NEXT call records into (no reader of this call touches either slot).  Block 0 also
// writes the dequant scale 1/scale to scale_inv, which the fp8 GEMM reads on the device.
//
// Tiles: 128x128 per 256-thread block.  Row pass: thread t owns 64 contiguous columns of row
// t/2 (8 x 16-B bf16 loads), stores 64 fp8 bytes of q and the same bytes as 16-B LDS writes
// into a [128][144] byte tile.  Column pass: thread t gathers 64 rows of input column t/2 from
// the tile (byte reads: 4 lanes share a dword, conflict free) and stores them as 4 x 16-B
// chunks of the q^T row — every q / q^T row segment a wave writes is a whole 128-B line.
// Edge tiles take the guarded element path.
#include "fp8_util.h"

namespace pa {
namespace f8 {

constexpr int T = 128;

template <int FMT>
__global__ __launch_bounds__(256) void cast_transpose_kernel(const bf16_t* __restrict__ x, int R, int C, long long ldx,
                                                             uint8_t* __restrict__ q, uint8_t* __restrict__ qt,
                                                             float* __restrict__ hist, int L, int cur,
                                                             float* __restrict__ scale_inv, float margin_mul) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[T][T + 16];  // [row][col] fp8 bytes, 16-B padded rows
  __shared__ float red[4];
  const float fmax = fmax_of<FMT>();
  const float s = scale_from_hist(hist, L, cur, fmax, margin_mul);
  const int tid = threadIdx.x;
  const int r0 = blockIdx.y * T, c0 = blockIdx.x * T;
  const int lr = tid >> 1, lc = (tid & 1) * 64;  // row pass: 64 contiguous columns of one row
  const int r = r0 + lr, c = c0 + lc;
  const bool full = (r0 + T <= R) && (c0 + T <= C);
  float am = 0.f;
#pragma unroll
  for (int h = 0; h < 4; ++h) {  // 4 x 16 columns: two 16-B bf16 loads -> one 16-B fp8 chunk
    float v[16];
    const int cc = c + 16 * h;
    if (full) {
      load_f<bf16_t, 8>(x + (long long)r * ldx + cc, *reinterpret_cast<float(*)[8]>(&v[0]));
      load_f<bf16_t, 8>(x + (long long)r * ldx + cc + 8, *reinterpret_cast<float(*)[8]>(&v[8]));
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = (r < R && cc + i < C) ? (float)x[(long long)r * ldx + cc + i] : 0.f;
    }
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      am = fmaxf(am, fmaxf(fmaxf(fabsf(v[4 * i]), fabsf(v[4 * i + 1])), fmaxf(fabsf(v[4 * i + 2]), fabsf(v[4 * i + 3]))));
      w[i] = cvt2<FMT>(v[4 * i] * s, v[4 * i + 1] * s) | (cvt2<FMT>(v[4 * i + 2] * s, v[4 * i + 3] * s) << 16);
    }
    const uint4 pk = make_uint4(w[0], w[1], w[2], w[3]);
    if (q) {
      if (full) {
        *reinterpret_cast<uint4*>(q + (long long)r * C + cc) = pk;
      } else if (r < R) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (cc + i < C) q[(long long)r * C + cc + i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
      }
    }
    if (qt) *reinterpret_cast<uint4*>(&tile[lr][lc + 16 * h]) = pk;
  }
  if (qt) {
    __syncthreads();
    // column pass: q^T row (input column) c0 + oc, 64 bytes of input rows r0 + orr ..
    const int oc = tid >> 1, orr = (tid & 1) * 64;
    const int orow = c0 + oc;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      uint32_t w[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rr = orr + 16 * h + 4 * i;
        w[i] = (uint32_t)tile[rr][oc] | ((uint32_t)tile[rr + 1][oc] << 8) | ((uint32_t)tile[rr + 2][oc] << 16) |
               ((uint32_t)tile[rr + 3][oc] << 24);
      }
      const int ocol = r0 + orr + 16 * h;
      if (full) {
        *reinterpret_cast<uint4*>(qt + (long long)orow * R + ocol) = make_uint4(w[0], w[1], w[2], w[3]);
      } else if (orow < C) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (ocol + i < R) qt[(long long)orow * R + ocol + i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
      }
    }
  }
  am = wave_max(am);
  if ((tid & 63) == 0) red[tid >> 6] = am;
  __syncthreads();
  if (tid == 0) {
    const float b = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomic_max_pos(hist + cur, b);
    if (blockIdx.x == 0 && blockIdx.y == 0) {
      hist[(cur + 1) % L] = 0.f;
      scale_inv[0] = 1.f / s;
    }
  }
}

// Full-tile variant (R, C multiples of 128): every global access a wave makes is contiguous.
//  * row pass: chunk k = tid + 256 i (i < 8) of the tile = 16 B of bf16 at row k / 16, column
//    8 (k % 16): one load instruction covers 4 rows x 256 B; its 8 fp8 bytes go to q (4 rows x
//    128 B per store instruction) and, as two dwords, to the LDS tile (pitch 132 B: the 32 lanes
//    of a ds_write_b32 half touch 2 rows x 16 chunks on distinct banks);
//  * column pass: lane (rg = lane / 8, cg = lane % 8) of wave w reads 16 rows x 4 bytes
//    (ds_read_b32, rows 16 rg .. +15, columns 4 (8 w + cg) .. +3 — conflict free: bank =
//    16 rg + cg + const within each 32-lane half), transposes the 16 x 4 bytes in registers and
//    stores four 16-B q^T chunks; 8 lanes cover one 128-B q^T row segment per store instruction.
// The old kernel's 2-lanes-per-row mapping gave 64 scattered 16-B segments per load / store
// instruction (2.3 TB/s on [16384, 2048]).
constexpr int P2 = T + 4;

template <int FMT>
__device__ __forceinline__ void cast_tile_full(uint8_t* tile, float* red, const bf16_t* __restrict__ x, int R, int C,
                                               long long ldx, uint8_t* __restrict__ q, uint8_t* __restrict__ qt,
                                               float* __restrict__ hist, int L, int cur,
                                               float* __restrict__ scale_inv, float margin_mul, int bx, int by) {
  const float fmax = fmax_of<FMT>();
  const float s = scale_from_hist(hist, L, cur, fmax, margin_mul);
  const int tid = threadIdx.x;
  const int r0 = by * T, c0 = bx * T;
  float am = 0.f;
  float v[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // all eight 16-B loads in flight before any use
    const int k = tid + 256 * i, row = k >> 4, ch = k & 15;
    load_f<bf16_t, 8>(x + (long long)(r0 + row) * ldx + c0 + 8 * ch, v[i]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int k = tid + 256 * i, row = k >> 4, ch = k & 15;
    uint32_t w[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      am = fmaxf(am, fmaxf(fmaxf(fabsf(v[i][4 * j]), fabsf(v[i][4 * j + 1])),
                           fmaxf(fabsf(v[i][4 * j + 2]), fabsf(v[i][4 * j + 3]))));
      w[j] = cvt2<FMT>(v[i][4 * j] * s, v[i][4 * j + 1] * s) | (cvt2<FMT>(v[i][4 * j + 2] * s, v[i][4 * j + 3] * s) << 16);
    }
    if (q) *reinterpret_cast<uint2*>(q + (long long)(r0 + row) * C + c0 + 8 * ch) = make_uint2(w[0], w[1]);
    if (qt) {
      uint32_t* t32 = reinterpret_cast<uint32_t*>(tile + row * P2 + 8 * ch);
      t32[0] = w[0];
      t32[1] = w[1];
    }
  }
  if (qt) {
    __syncthreads();
    const int lane = tid & 63, wave = tid >> 6;
    const int rg = lane >> 3, cgl = lane & 7;
    {  // 4 waves x 8 column groups of 4 = the tile's 128 columns; 8 row groups of 16 = its 128 rows
      const int cg = wave * 8 + cgl;  // column group: input columns 4 cg .. 4 cg + 3
      uint32_t rw[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) rw[i] = *reinterpret_cast<const uint32_t*>(tile + (16 * rg + i) * P2 + 4 * cg);
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // q^T row (input column) c0 + 4 cg + j, bytes of rows 16 rg ..
        uint32_t o[4];
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) {
          const uint32_t a = (rw[4 * kq] >> (8 * j)) & 0xFFu, b = (rw[4 * kq + 1] >> (8 * j)) & 0xFFu;
          const uint32_t c = (rw[4 * kq + 2] >> (8 * j)) & 0xFFu, d = (rw[4 * kq + 3] >> (8 * j)) & 0xFFu;
          o[kq] = a | (b << 8) | (c << 16) | (d << 24);
        }
        *reinterpret_cast<uint4*>(qt + (long long)(c0 + 4 * cg + j) * R + r0 + 16 * rg) =
            make_uint4(o[0], o[1], o[2], o[3]);
      }
    }
  }
  am = wave_max(am);
  if ((tid & 63) == 0) red[tid >> 6] = am;
  __syncthreads();
  if (tid == 0) {
    const float b = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomic_max_pos(hist + cur, b);
    if (bx == 0 && by == 0) {
      hist[(cur + 1) % L] = 0.f;
      scale_inv[0] = 1.f / s;
    }
  }
}

template <int FMT>
__global__ __launch_bounds__(256) void cast_transpose_full_kernel(const bf16_t* __restrict__ x, int R, int C,
                                                                  long long ldx, uint8_t* __restrict__ q,
                                                                  uint8_t* __restrict__ qt, float* __restrict__ hist,
                                                                  int L, int cur, float* __restrict__ scale_inv,
                                                                  float margin_mul) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[T * P2];
  __shared__ float red[4];
  cast_tile_full<FMT>(tile, red, x, R, C, ldx, q, qt, hist, L, cur, scale_inv, margin_mul, blockIdx.x, blockIdx.y);
}

// Persistent form of the full-tile cast: a grid of a few blocks per CU walks the tiles, and the
// NEXT tile's eight 16-B loads per thread are issued before the current tile is converted and
// stored, so HBM reads stay in flight under the stores and the LDS transpose (the one-tile-per-block
// kernel runs every block's loads, then every block's stores: 3.4 TB/s on [32768, 768]).
__device__ __forceinline__ void bf16x8_to_f(const uint4 u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
  }
}

// cs != null: also the per-tile column sums of x (fp32 [R / 128][C], row-tile major) — the bias
// gradient partials of an fp8 Linear's dY, taken from the values this pass reads anyway (the
// separate column-sum pass re-read dY: ~20 us per Linear backward at ERNIE-base shapes).
template <int FMT>
__global__ __launch_bounds__(256) void cast_transpose_persist_kernel(const bf16_t* __restrict__ x, int R, int C,
                                                                     long long ldx, uint8_t* __restrict__ q,
                                                                     uint8_t* __restrict__ qt,
                                                                     float* __restrict__ hist, int L, int cur,
                                                                     float* __restrict__ scale_inv, float margin_mul,
                                                                     float* __restrict__ cs = nullptr) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[T * P2];
  __shared__ float red[4];
  __shared__ float csr[4][T];  // cs: the four waves' column sums of a tile
  const float s = scale_from_hist(hist, L, cur, fmax_of<FMT>(), margin_mul);
  const int tid = threadIdx.x;
  const int tx = C / T, ntiles = tx * (R / T);
  float am = 0.f;
  int t = blockIdx.x;
  uint4 raw[8];
  if (t < ntiles) {
    const int r0 = (t / tx) * T, c0 = (t % tx) * T;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = tid + 256 * i, row = k >> 4, ch = k & 15;
      raw[i] = *reinterpret_cast<const uint4*>(x + (long long)(r0 + row) * ldx + c0 + 8 * ch);
    }
  }
  for (; t < ntiles; t += gridDim.x) {
    const int r0 = (t / tx) * T, c0 = (t % tx) * T;
    const int tn = t + gridDim.x;
    uint4 nxt[8];
    if (tn < ntiles) {  // the next tile's reads go out before this tile's writes
      const int nr0 = (tn / tx) * T, nc0 = (tn % tx) * T;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int k = tid + 256 * i, row = k >> 4, ch = k & 15;
        nxt[i] = *reinterpret_cast<const uint4*>(x + (long long)(nr0 + row) * ldx + nc0 + 8 * ch);
      }
    }
    float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // cs: this thread's 8 columns (ch = tid & 15)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = tid + 256 * i, row = k >> 4, ch = k & 15;
      float v[8];
      bf16x8_to_f(raw[i], v);
      if (cs) {
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[e] += v[e];
      }
      uint32_t w[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        am = fmaxf(am, fmaxf(fmaxf(fabsf(v[4 * j]), fabsf(v[4 * j + 1])), fmaxf(fabsf(v[4 * j + 2]), fabsf(v[4 * j + 3]))));
        w[j] = cvt2<FMT>(v[4 * j] * s, v[4 * j + 1] * s) | (cvt2<FMT>(v[4 * j + 2] * s, v[4 * j + 3] * s) << 16);
      }
      if (q) *reinterpret_cast<uint2*>(q + (long long)(r0 + row) * C + c0 + 8 * ch) = make_uint2(w[0], w[1]);
      if (qt) {
        uint32_t* t32 = reinterpret_cast<uint32_t*>(tile + row * P2 + 8 * ch);
        t32[0] = w[0];
        t32[1] = w[1];
      }
    }
    if (qt) {
      __syncthreads();
      const int lane = tid & 63, wave = tid >> 6;
      const int rg = lane >> 3, cg = wave * 8 + (lane & 7);
      uint32_t rw[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) rw[i] = *reinterpret_cast<const uint32_t*>(tile + (16 * rg + i) * P2 + 4 * cg);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t o[4];
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) {
          const uint32_t a = (rw[4 * kq] >> (8 * j)) & 0xFFu, b = (rw[4 * kq + 1] >> (8 * j)) & 0xFFu;
          const uint32_t c = (rw[4 * kq + 2] >> (8 * j)) & 0xFFu, d = (rw[4 * kq + 3] >> (8 * j)) & 0xFFu;
          o[kq] = a | (b << 8) | (c << 16) | (d << 24);
        }
        *reinterpret_cast<uint4*>(qt + (long long)(c0 + 4 * cg + j) * R + r0 + 16 * rg) = make_uint4(o[0], o[1], o[2], o[3]);
      }
      __syncthreads();  // the tile is rewritten by the next iteration
    }
    if (cs) {  // lanes l, l^16, l^32, l^48 of a wave hold the same 8 columns; then the 4 waves via LDS
      const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        csum[e] += __shfl_xor(csum[e], 16, 64);
        csum[e] += __shfl_xor(csum[e], 32, 64);
      }
      if (lane < 16) {
#pragma unroll
        for (int e = 0; e < 8; ++e) csr[wave][8 * lane + e] = csum[e];
      }
      __syncthreads();
      if (tid < T) cs[(long long)(r0 / T) * C + c0 + tid] = (csr[0][tid] + csr[1][tid]) + (csr[2][tid] + csr[3][tid]);
      __syncthreads();  // csr is rewritten by the next tile
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) raw[i] = nxt[i];
  }
  am = wave_max(am);
  if ((tid & 63) == 0) red[tid >> 6] = am;
  __syncthreads();
  if (tid == 0) {
    atomic_max_pos(hist + cur, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
    if (blockIdx.x == 0) {
      hist[(cur + 1) % L] = 0.f;
      scale_inv[0] = 1.f / s;
    }
  }
}

// Many casts in ONE launch (the weights of an fp8 static program, cast once at the start of each
// step instead of one small launch per Linear): the 1-D grid is the concatenation of every job's
// 128x128 tiles; a block finds its job by binary search over the jobs' first-tile indices.  Every
// job is a full-tile one (R, C multiples of 128) of the same fp8 format.
struct CastJob {
  const bf16_t* x;
  uint8_t* q;
  uint8_t* qt;
  float* hist;
  float* scale_inv;
  long long ldx;
  int R, C, L, cur, tiles_x, tile0;
  float margin_mul;
  int pad;
};
static_assert(sizeof(CastJob) == 80, "CastJob layout is packed by ops/fp8.py");

template <int FMT>
__global__ __launch_bounds__(256) void cast_transpose_multi_kernel(const CastJob* __restrict__ jobs, int njobs) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[T * P2];
  __shared__ float red[4];
  const int bid = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].tile0 <= bid) lo = mid; else hi = mid - 1;
  }
  const CastJob& j = jobs[lo];
  const int t = bid - j.tile0;
  cast_tile_full<FMT>(tile, red, j.x, j.R, j.C, j.ldx, j.q, j.qt, j.hist, j.L, j.cur, j.scale_inv, j.margin_mul,
                      t % j.tiles_x, t / j.tiles_x);
}

// amax of a bf16 [R, C] tensor folded into *out (first use of a tensor: seeds the history)
__global__ __launch_bounds__(256) void amax_kernel(const bf16_t* __restrict__ x, int R, int C, long long ldx,
                                                   float* __restrict__ out) {
  __shared__ float red[4];
  float am = 0.f;
  const long long n8 = (long long)R * (C / 8);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    const long long row = i / (C / 8), col = (i % (C / 8)) * 8;
    float v[8];
    load_f<bf16_t, 8>(x + row * ldx + col, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(v[j]));
  }
  am = wave_max(am);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
  __syncthreads();
  if (threadIdx.x == 0) atomic_max_pos(out, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

}  // namespace f8
}  // namespace pa

using namespace pa;

// A/B switch for 128-multiple shapes: 2 = persistent full-tile kernel, 1 = one full tile per
// block, 0 = the guarded kernel
static int g_cast_full = 2;
PA_API int pa_fp8_set_cast_full(int v) {
  const int old = g_cast_full;
  g_cast_full = v;
  return old;
}

// pa_fp8_cast_transpose plus the column sums of x per 128-row tile into cs (fp32 [R / 128][C]):
// full-tile shapes only (R, C multiples of 128), else hipErrorInvalidValue and nothing runs.
PA_API int pa_fp8_cast_transpose_cs(const void* x, int R, int C, long long ldx, void* q, void* qt, void* hist, int L,
                                    int cur, void* scale_inv, int fmt, float margin_mul, float* cs, hipStream_t st) {
  if (R <= 0 || C <= 0 || R % f8::T || C % f8::T || ldx % 8 || L < 3 || cur < 0 || cur >= L || !hist ||
      !scale_inv || !cs)
    return (int)hipErrorInvalidValue;
  const int ntiles = (R / f8::T) * (C / f8::T);
  const int per = (ntiles + 1023) / 1024;
  const int g = (ntiles + per - 1) / per;
  if (fmt == 0)
    f8::cast_transpose_persist_kernel<0><<<g, 256, 0, st>>>((const bf16_t*)x, R, C, ldx, (uint8_t*)q, (uint8_t*)qt,
                                                            (float*)hist, L, cur, (float*)scale_inv, margin_mul, cs);
  else
    f8::cast_transpose_persist_kernel<1><<<g, 256, 0, st>>>((const bf16_t*)x, R, C, ldx, (uint8_t*)q, (uint8_t*)qt,
                                                            (float*)hist, L, cur, (float*)scale_inv, margin_mul, cs);
  return (int)hipGetLastError();
}

// x: bf16 [R, C] (row stride ldx, 16-B aligned rows), q: [R, C] fp8 or null, qt: [C, R] fp8 or null.
// fmt 0 = e4m3fn, 1 = e5m2.  C % 8 == 0.
PA_API int pa_fp8_cast_transpose(const void* x, int R, int C, long long ldx, void* q, void* qt, void* hist, int L,
                                 int cur, void* scale_inv, int fmt, float margin_mul, hipStream_t st) {
  if (R <= 0 || C <= 0 || C % 8 || ldx % 8 || L < 3 || cur < 0 || cur >= L || !hist || !scale_inv)
    return (int)hipErrorInvalidValue;
  dim3 grid((C + f8::T - 1) / f8::T, (R + f8::T - 1) / f8::T);
  if (grid.y > 65535) return (int)hipErrorInvalidValue;
  if (R % f8::T == 0 && C % f8::T == 0 && ldx % 8 == 0 && g_cast_full == 2) {
    const int ntiles = (R / f8::T) * (C / f8::T);
    // at most 4 blocks per CU walk the tiles, every block the same number of them (no tail of
    // blocks with one tile more than the rest)
    const int per = (ntiles + 1023) / 1024;
    const int g = (ntiles + per - 1) / per;
    if (fmt == 0)
      f8::cast_transpose_persist_kernel<0><<<g, 256, 0, st>>>((const bf16_t*)x, R, C, ldx, (uint8_t*)q, (uint8_t*)qt,
                                                              (float*)hist, L, cur, (float*)scale_inv, margin_mul);
    else
      f8::cast_transpose_persist_kernel<1><<<g, 256, 0, st>>>((const bf16_t*)x, R, C, ldx, (uint8_t*)q, (uint8_t*)qt,
                                                              (float*)hist, L, cur, (float*)scale_inv, margin_mul);
    return (int)hipGetLastError();
  }
  if (R % f8::T == 0 && C % f8::T == 0 && ldx % 8 == 0 && g_cast_full) {
    if (fmt == 0)
      f8::cast_transpose_full_kernel<0><<<grid, 256, 0, st>>>((const bf16_t*)x, R, C, ldx, (uint8_t*)q, (uint8_t*)qt,
                                                                (float*)hist, L, cur, (float*)scale_inv, margin_mul);
    else
      f8::cast_transpose_full_kernel<1><<<grid, 256, 0, st>>>((const bf16_t*)x, R, C, ldx, (uint8_t*)q, (uint8_t*)qt,
                                                                (float*)hist, L, cur, (float*)scale_inv, margin_mul);
    return (int)hipGetLastError();
  }
  if (fmt == 0)
    f8::cast_transpose_kernel<0><<<grid, 256, 0, st>>>((const bf16_t*)x, R, C, ldx, (uint8_t*)q, (uint8_t*)qt,
                                                         (float*)hist, L, cur, (float*)scale_inv, margin_mul);
  else
    f8::cast_transpose_kernel<1><<<grid, 256, 0, st>>>((const bf16_t*)x, R, C, ldx, (uint8_t*)q, (uint8_t*)qt,
                                                         (float*)hist, L, cur, (float*)scale_inv, margin_mul);
  return (int)hipGetLastError();
}

// jobs: device array of f8::CastJob (80 B each, tile0 ascending, full 128x128 tiles), total_tiles
// = the grid; fmt 0 = e4m3fn, 1 = e5m2 for every job.
PA_API int pa_fp8_cast_transpose_multi(const void* jobs, int njobs, int total_tiles, int fmt, hipStream_t st) {
  if (!jobs || njobs <= 0 || total_tiles <= 0 || fmt < 0 || fmt > 1) return (int)hipErrorInvalidValue;
  if (fmt == 0)
    f8::cast_transpose_multi_kernel<0><<<total_tiles, 256, 0, st>>>((const f8::CastJob*)jobs, njobs);
  else
    f8::cast_transpose_multi_kernel<1><<<total_tiles, 256, 0, st>>>((const f8::CastJob*)jobs, njobs);
  return (int)hipGetLastError();
}

namespace pa {
namespace f8 {
// The delayed-scaling bookkeeping of one cast, for producers that quantise inside their own
// epilogue (gemm8x.hip pa_gemm8_fp8_epi_q): scale from the history (cur / cur+1 excluded, as in
// the cast kernels), its inverse for the consuming GEMM, and the next slot zeroed.
__global__ void scale_prep_kernel(float* __restrict__ hist, int L, int cur, float fmax, float margin_mul,
                                  float* __restrict__ scale, float* __restrict__ scale_inv) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const float s = scale_from_hist(hist, L, cur, fmax, margin_mul);
    scale[0] = s;
    scale_inv[0] = 1.f / s;
    hist[(cur + 1) % L] = 0.f;
  }
}
}  // namespace f8
}  // namespace pa

PA_API int pa_fp8_scale_prep(void* hist, int L, int cur, int fmt, float margin_mul, void* scale, void* scale_inv,
                             hipStream_t st) {
  if (L < 3 || cur < 0 || cur >= L || fmt < 0 || fmt > 1 || !hist || !scale || !scale_inv)
    return (int)hipErrorInvalidValue;
  pa::f8::scale_prep_kernel<<<1, 64, 0, st>>>((float*)hist, L, cur, fmt == 0 ? 448.f : 57344.f, margin_mul,
                                              (float*)scale, (float*)scale_inv);
  return (int)hipGetLastError();
}

PA_API int pa_fp8_amax(const void* x, int R, int C, long long ldx, void* out, hipStream_t st) {
  if (R <= 0 || C <= 0 || C % 8 || ldx % 8) return (int)hipErrorInvalidValue;
  const long long n8 = (long long)R * (C / 8);
  int g = (int)((n8 + 255) / 256);
  if (g > 2048) g = 2048;
  f8::amax_kernel<<<g, 256, 0, st>>>((const bf16_t*)x, R, C, ldx, (float*)out);
  return (int)hipGetLastError();
}
