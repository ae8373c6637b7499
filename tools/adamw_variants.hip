// Stand-alone A/B of fused-AdamW streaming structures on a GPT-3 1.3B-sized flat buffer
// (fp32 master / m / v, bf16 grad and bf16 model copy: 28 B per parameter).
//   v0: the same 5 read + 4 write streams with no math (the ceiling of this access mix)
//   v1: grid-stride, 8 params per lane, 2 iterations in flight (the library kernel's structure)
//   v2: grid-stride, 8 params per lane, 4 iterations in flight
//   v3: contiguous chunk per block (each block sweeps its own range), 8 params per lane, 2 in flight
//   v4: v1 with plain (temporal) accesses
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/adamw_variants tools/adamw_variants.hip
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int nt_i4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

template <bool NT>
__device__ __forceinline__ nt_i4 ld(const void* p) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<const nt_i4*>(p));
  return *reinterpret_cast<const nt_i4*>(p);
}
template <bool NT>
__device__ __forceinline__ void st(void* p, nt_i4 v) {
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<nt_i4*>(p));
  else *reinterpret_cast<nt_i4*>(p) = v;
}
__device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float((unsigned)h << 16); }
__device__ __forceinline__ u16 f2bf(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (u16)(u >> 16);
}

struct Args {
  float *p, *m, *v;
  const u16* g;
  u16* low;
  long long n;
  float b1, b2, step, decay, eps;
};

template <bool NT, bool MATH, bool NTS = NT>
__device__ __forceinline__ void vec8(const Args& a, long long i) {
  nt_i4 P0 = ld<NT>(a.p + i), P1 = ld<NT>(a.p + i + 4);
  nt_i4 G = ld<NT>(a.g + i);
  nt_i4 M0 = ld<NT>(a.m + i), M1 = ld<NT>(a.m + i + 4);
  nt_i4 V0 = ld<NT>(a.v + i), V1 = ld<NT>(a.v + i + 4);
  float pv[8], mv[8], vv[8], gv[8];
  *reinterpret_cast<nt_i4*>(pv) = P0;
  *reinterpret_cast<nt_i4*>(pv + 4) = P1;
  *reinterpret_cast<nt_i4*>(mv) = M0;
  *reinterpret_cast<nt_i4*>(mv + 4) = M1;
  *reinterpret_cast<nt_i4*>(vv) = V0;
  *reinterpret_cast<nt_i4*>(vv + 4) = V1;
  u16 gh[8];
  *reinterpret_cast<nt_i4*>(gh) = G;
#pragma unroll
  for (int e = 0; e < 8; ++e) gv[e] = bf2f(gh[e]);
  if (MATH) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gg = gv[e];
      mv[e] = a.b1 * mv[e] + (1.f - a.b1) * gg;
      vv[e] = a.b2 * vv[e] + (1.f - a.b2) * gg * gg;
      pv[e] = pv[e] * a.decay - a.step * mv[e] * __builtin_amdgcn_rcpf(__builtin_sqrtf(vv[e]) + a.eps);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      pv[e] += gv[e];
    }
  }
  st<NTS>(a.p + i, *reinterpret_cast<nt_i4*>(pv));
  st<NTS>(a.p + i + 4, *reinterpret_cast<nt_i4*>(pv + 4));
  st<NTS>(a.m + i, *reinterpret_cast<nt_i4*>(mv));
  st<NTS>(a.m + i + 4, *reinterpret_cast<nt_i4*>(mv + 4));
  st<NTS>(a.v + i, *reinterpret_cast<nt_i4*>(vv));
  st<NTS>(a.v + i + 4, *reinterpret_cast<nt_i4*>(vv + 4));
  u16 lo[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) lo[e] = f2bf(pv[e]);
  st<NTS>(a.low + i, *reinterpret_cast<nt_i4*>(lo));
}

template <bool NT, bool MATH, int U, bool NTS = NT>
__global__ __launch_bounds__(256) void k_stride(Args a) {
  const long long nv = a.n / 8;
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < nv; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) vec8<NT, MATH, NTS>(a, (i + u * stride) * 8);
  }
  for (; i < nv; i += stride) vec8<NT, MATH, NTS>(a, i * 8);
}

// each block sweeps a contiguous range of vectors; U vectors in flight per lane
template <bool NT, int U, bool NTS = NT>
__global__ __launch_bounds__(256) void k_chunk(Args a) {
  const long long nv = a.n / 8;
  const long long per = (nv + gridDim.x - 1) / gridDim.x;
  const long long beg = (long long)blockIdx.x * per;
  const long long end = beg + per < nv ? beg + per : nv;
  long long i = beg + threadIdx.x;
  for (; i + (U - 1) * 256 < end; i += U * 256) {
#pragma unroll
    for (int u = 0; u < U; ++u) vec8<NT, true, NTS>(a, (i + u * 256) * 8);
  }
  for (; i < end; i += 256) vec8<NT, true, NTS>(a, i * 8);
}

int main() {
  const long long n = 1316000000LL;
  Args a;
  CK(hipMalloc(&a.p, n * 4));
  CK(hipMalloc(&a.m, n * 4));
  CK(hipMalloc(&a.v, n * 4));
  CK(hipMalloc((void**)&a.g, n * 2));
  CK(hipMalloc(&a.low, n * 2));
  CK(hipMemset(a.p, 0, n * 4));
  CK(hipMemset(a.m, 0, n * 4));
  CK(hipMemset(a.v, 0, n * 4));
  CK(hipMemset((void*)a.g, 0, n * 2));
  a.n = n;
  a.b1 = 0.9f;
  a.b2 = 0.95f;
  a.step = 1e-4f;
  a.decay = 0.999f;
  a.eps = 1e-8f;
  int cus = 256;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    for (int w = 0; w < 2; ++w) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int R = 5;
    for (int r = 0; r < R; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double t = ms / 1e3 / R;
    printf("%-44s %8.1f us  %5.2f TB/s\n", name, t * 1e6, 28.0 * n / t / 1e12);
    fflush(stdout);
  };
  char nm[128];
  for (int bpc : {2, 4, 8}) {
    const int grid = cus * bpc;
    snprintf(nm, sizeof nm, "v0 copy-only stride U2 temporal bpc%d", bpc);
    timeit(nm, [&] { k_stride<false, false, 2><<<grid, 256>>>(a); });
    snprintf(nm, sizeof nm, "v1 stride U2 NT bpc%d", bpc);
    timeit(nm, [&] { k_stride<true, true, 2><<<grid, 256>>>(a); });
    snprintf(nm, sizeof nm, "v4 stride U2 temporal bpc%d", bpc);
    timeit(nm, [&] { k_stride<false, true, 2><<<grid, 256>>>(a); });
    snprintf(nm, sizeof nm, "v4b stride U1 temporal bpc%d", bpc);
    timeit(nm, [&] { k_stride<false, true, 1><<<grid, 256>>>(a); });
    snprintf(nm, sizeof nm, "v4c stride U4 temporal bpc%d", bpc);
    timeit(nm, [&] { k_stride<false, true, 4><<<grid, 256>>>(a); });
    snprintf(nm, sizeof nm, "v6 stride U2 NT-load temporal-store bpc%d", bpc);
    timeit(nm, [&] { k_stride<true, true, 2, false><<<grid, 256>>>(a); });
    snprintf(nm, sizeof nm, "v7 stride U2 temporal-load NT-store bpc%d", bpc);
    timeit(nm, [&] { k_stride<false, true, 2, true><<<grid, 256>>>(a); });
    snprintf(nm, sizeof nm, "v3 chunk U1 temporal bpc%d", bpc);
    timeit(nm, [&] { k_chunk<false, 1><<<grid, 256>>>(a); });
  }
  {
    const long long nv = n / 8;
    const int grid = (int)((nv + 255) / 256);
    timeit("v5 one-shot grid NT", [&] { k_stride<true, true, 1><<<grid, 256>>>(a); });
    timeit("v5b one-shot grid temporal", [&] { k_stride<false, true, 1><<<grid, 256>>>(a); });
    timeit("v5c one-shot grid NT-load temporal-store", [&] { k_stride<true, true, 1, false><<<grid, 256>>>(a); });
  }
  return 0;
}
