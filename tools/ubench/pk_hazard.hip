// Microbenchmark / hazard probe (round 5, DESIGN.md §5 "co-residency fault").
// The fault-era backward recurrence (commit 001db35) gave wrong gate
// gradients only in lanes 48-63 of its cell waves (the last quarter-wave)
// and only while other kernels' waves shared its SIMDs; the first wrong value
// was always the LOW half of a packed-FP32 multiply C that reads a VGPR pair
// written by another packed multiply B one VALU instruction earlier
// (B: v_pk_mul_f32 v[22:23], .., v[22:23]; one unrelated v_pk_mul_f32;
// C: v_pk_mul_f32 vD, vS, v[22:23]).
//
// This probe runs such dependent chains in inline assembly (no compiler
// hazard handling inside the asm block) on one wave per SIMD, with or without
// an MFMA + LDS "aggressor" kernel co-resident on the same CUs, and counts per
// lane and per half the results that differ from the same products computed
// in plain C++.
//
// usage: pk_hazard [iters_millions] ; prints one line per (pattern, aggressor)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));

// pattern 0: B; independent pk; C      (the fault-era sequence)
// pattern 1: B; C                      (back to back)
// pattern 2: B; v_mov; C
// pattern 3: B; two independent pk; C
// pattern 4: op_sel A; v_mov; B; independent pk; C (the whole chain)
// pattern 5: two f16 -> f32 converts of one packed input, then 1 - x on the
//            pair as v_pk_add_f32 with neg_lo / neg_hi (the fault-era
//            gate-complement instruction)
// pattern 6: as 5 with the x + 1 pk_add first (the fault-era pair)
// pattern 7: op_sel A; v_mov; B (B's result checked)
// pattern 8: op_sel A; B back to back
// pattern 9: op_sel A; two v_mov; B
// pattern 10: A without op_sel; v_mov; B; pk; C (pattern 4 minus the op_sel)
// pattern 11: op_sel A; v_mov; v_mov; v_mov; v_mov; B
// single instructions, result checked directly (c = f(b, y)):
// pattern 12: v_pk_mul_f32 c, b, y op_sel_hi:[0,1]  (b.lo broadcast to the high lane)
// pattern 13: v_pk_mul_f32 c, b, y op_sel:[1,0]     (b.hi into the low lane)
// pattern 14: v_pk_fma_f32 c, b, y, y op_sel:[1,0,0]
// pattern 15: v_pk_mul_f32 c, b, y op_sel:[0,1]     (not in place)
// pattern 16: v_pk_mul_f32 c, b, y op_sel_hi:[1,0]  (y.lo broadcast)
template <int P>
__device__ __forceinline__ f2 chain(f2 a1, f2 a2, f2 b, f2 x, f2 y, f2& xo, unsigned h = 0) {
  f2 c;
  if constexpr (P == 5) {
    asm volatile(
        "v_cvt_f32_f16_sdwa v201, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n\t"
        "v_cvt_f32_f16_e32 v200, %1\n\t"
        "v_pk_add_f32 %0, v[200:201], 1.0 op_sel_hi:[1,0] neg_lo:[1,0] neg_hi:[1,0]\n\t"
        : "=&v"(c)
        : "v"(h)
        : "v200", "v201");
    xo = x;
    return c;
  } else if constexpr (P == 6) {
    f2 d;
    asm volatile(
        "v_cvt_f32_f16_sdwa v201, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n\t"
        "v_cvt_f32_f16_e32 v200, %2\n\t"
        "v_pk_add_f32 %1, v[200:201], 1.0 op_sel_hi:[1,0]\n\t"
        "v_pk_add_f32 %0, v[200:201], 1.0 op_sel_hi:[1,0] neg_lo:[1,0] neg_hi:[1,0]\n\t"
        : "=&v"(c), "=&v"(d)
        : "v"(h)
        : "v200", "v201");
    xo = x + d;
    return c;
  } else if constexpr (P == 0) {
    asm volatile(
        "v_pk_mul_f32 %0, %3, %0\n\t"
        "v_pk_mul_f32 %1, %4, %1\n\t"
        "v_pk_mul_f32 %2, %5, %0\n\t"
        : "+v"(b), "+v"(x), "=&v"(c)
        : "v"(a1), "v"(y), "v"(a2));
  } else if constexpr (P == 1) {
    asm volatile(
        "v_pk_mul_f32 %0, %3, %0\n\t"
        "v_pk_mul_f32 %2, %5, %0\n\t"
        "v_pk_mul_f32 %1, %4, %1\n\t"
        : "+v"(b), "+v"(x), "=&v"(c)
        : "v"(a1), "v"(y), "v"(a2));
  } else if constexpr (P == 2) {
    float t;
    asm volatile(
        "v_pk_mul_f32 %0, %4, %0\n\t"
        "v_mov_b32 %3, %7\n\t"
        "v_pk_mul_f32 %2, %6, %0\n\t"
        "v_pk_mul_f32 %1, %5, %1\n\t"
        : "+v"(b), "+v"(x), "=&v"(c), "=&v"(t)
        : "v"(a1), "v"(y), "v"(a2), "v"(a1.x));
    (void)t;
  } else if constexpr (P == 3) {
    asm volatile(
        "v_pk_mul_f32 %0, %3, %0\n\t"
        "v_pk_mul_f32 %1, %4, %1\n\t"
        "v_pk_mul_f32 %1, %4, %1\n\t"
        "v_pk_mul_f32 %2, %5, %0\n\t"
        : "+v"(b), "+v"(x), "=&v"(c)
        : "v"(a1), "v"(y), "v"(a2));
  } else if constexpr (P == 7 || P == 8 || P == 9 || P == 11) {
    float t;
    if constexpr (P == 7)
      asm volatile(
          "v_pk_mul_f32 %0, %0, %3 op_sel:[0,1]\n\t"
          "v_mov_b32 %2, %4\n\t"
          "v_pk_mul_f32 %1, %5, %0\n\t"
          : "+v"(b), "=&v"(c), "=&v"(t)
          : "v"(y), "v"(a1.x), "v"(a1));
    else if constexpr (P == 8)
      asm volatile(
          "v_pk_mul_f32 %0, %0, %3 op_sel:[0,1]\n\t"
          "v_pk_mul_f32 %1, %5, %0\n\t"
          "v_mov_b32 %2, %4\n\t"
          : "+v"(b), "=&v"(c), "=&v"(t)
          : "v"(y), "v"(a1.x), "v"(a1));
    else if constexpr (P == 9)
      asm volatile(
          "v_pk_mul_f32 %0, %0, %3 op_sel:[0,1]\n\t"
          "v_mov_b32 %2, %4\n\t"
          "v_mov_b32 %2, %4\n\t"
          "v_pk_mul_f32 %1, %5, %0\n\t"
          : "+v"(b), "=&v"(c), "=&v"(t)
          : "v"(y), "v"(a1.x), "v"(a1));
    else
      asm volatile(
          "v_pk_mul_f32 %0, %0, %3 op_sel:[0,1]\n\t"
          "v_mov_b32 %2, %4\n\t"
          "v_mov_b32 %2, %4\n\t"
          "v_mov_b32 %2, %4\n\t"
          "v_mov_b32 %2, %4\n\t"
          "v_pk_mul_f32 %1, %5, %0\n\t"
          : "+v"(b), "=&v"(c), "=&v"(t)
          : "v"(y), "v"(a1.x), "v"(a1));
    (void)t;
  } else if constexpr (P >= 12) {
    if constexpr (P == 12)
      asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=&v"(c) : "v"(b), "v"(y));
    else if constexpr (P == 13)
      asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0]" : "=&v"(c) : "v"(b), "v"(y));
    else if constexpr (P == 14)
      asm volatile("v_pk_fma_f32 %0, %1, %2, %2 op_sel:[1,0,0]" : "=&v"(c) : "v"(b), "v"(y));
    else if constexpr (P == 15)
      asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1]" : "=&v"(c) : "v"(b), "v"(y));
    else
      asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=&v"(c) : "v"(b), "v"(y));
  } else if constexpr (P == 10) {
    float t;
    asm volatile(
        "v_pk_mul_f32 %0, %0, %5\n\t"
        "v_mov_b32 %3, %7\n\t"
        "v_pk_mul_f32 %0, %4, %0\n\t"
        "v_pk_mul_f32 %1, %5, %1\n\t"
        "v_pk_mul_f32 %2, %6, %0\n\t"
        : "+v"(b), "+v"(x), "=&v"(c), "=&v"(t)
        : "v"(a1), "v"(y), "v"(a2), "v"(a1.x));
    (void)t;
  } else {
    // A: b = (b.x * y.y, b.y * y.y) (op_sel:[0,1]); B: b = a1 * b; pk; C
    float t;
    asm volatile(
        "v_pk_mul_f32 %0, %0, %5 op_sel:[0,1]\n\t"
        "v_mov_b32 %3, %7\n\t"
        "v_pk_mul_f32 %0, %4, %0\n\t"
        "v_pk_mul_f32 %1, %5, %1\n\t"
        "v_pk_mul_f32 %2, %6, %0\n\t"
        : "+v"(b), "+v"(x), "=&v"(c), "=&v"(t)
        : "v"(a1), "v"(y), "v"(a2), "v"(a1.x));
    (void)t;
  }
  xo = x;
  return c;
}

__device__ __forceinline__ float h2f(unsigned h, int hi) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)(hi ? h >> 16 : h & 0xffff));
}
template <int P>
__device__ __forceinline__ f2 chain_ref(f2 a1, f2 a2, f2 b, f2 y, unsigned h = 0) {
  if constexpr (P == 5 || P == 6) return f2{1.f - h2f(h, 0), 1.f - h2f(h, 1)};
  if constexpr (P == 12) return f2{b.x * y.x, b.x * y.y};
  if constexpr (P == 13) return f2{b.y * y.x, b.y * y.y};
  if constexpr (P == 14) return f2{__builtin_fmaf(b.y, y.x, y.x), __builtin_fmaf(b.y, y.y, y.y)};
  if constexpr (P == 15) return f2{b.x * y.y, b.y * y.y};
  if constexpr (P == 16) return f2{b.x * y.x, b.y * y.x};
  if constexpr (P == 10) b = f2{b.x * y.x, b.y * y.y};
  else if constexpr (P == 4 || P >= 7) b = f2{b.x * y.y, b.y * y.y};
  b = f2{a1.x * b.x, a1.y * b.y};
  if constexpr (P >= 7 && P != 10) return b;
  return f2{a2.x * b.x, a2.y * b.y};
}

// one wave per SIMD (256 threads, one work-group per CU); cnt[2 * lane + half]
template <int P>
__global__ void __launch_bounds__(256) victim(long long iters, unsigned* cnt, f2* sink, float* dbg) {
  const int lane = threadIdx.x & 63;
  const float s = 1.f + 1e-3f * (float)(threadIdx.x + 7 * blockIdx.x);
  f2 a1 = {1.0001f * s, 0.9997f / s}, a2 = {1.0003f / s, 0.9999f * s};
  f2 x = {1.f, 1.f}, y = {0.99991f, 1.00007f};
  unsigned e_lo = 0, e_hi = 0;
  f2 acc = {0.f, 0.f};
  for (long long it = 0; it < iters; ++it) {
    // b changes every iteration, so a stale read of B's result differs
    const float v = 1.f + (float)(it & 1023) * (1.f / 1024.f);
    const f2 b = {v * s, 2.f - v};
    // packed fp16 pair for patterns 5 / 6 (changes every iteration)
    const unsigned h = (unsigned)__builtin_bit_cast(unsigned short, (_Float16)(0.25f * v * s)) |
                       ((unsigned)__builtin_bit_cast(unsigned short, (_Float16)(0.5f - 0.2f * v)) << 16);
    const f2 c = chain<P>(a1, a2, b, x, y, x, h);
    const f2 r = chain_ref<P>(a1, a2, b, y, h);
    if (__float_as_uint(c.x) != __float_as_uint(r.x) && atomicCAS((unsigned*)dbg, 0u, 1u) == 0u) {
      // first wrong low half: the value, the expected one and the operands
      dbg[1] = c.x; dbg[2] = r.x; dbg[3] = b.x; dbg[4] = y.x; dbg[5] = y.y; dbg[6] = a1.x;
      dbg[7] = a2.x; dbg[8] = (float)lane; dbg[9] = c.y; dbg[10] = r.y;
    }
    e_lo += __float_as_uint(c.x) != __float_as_uint(r.x);
    e_hi += __float_as_uint(c.y) != __float_as_uint(r.y);
    acc += c;
    if (x.x > 1e30f) x = f2{1.f, 1.f};
  }
  atomicAdd(&cnt[2 * lane], e_lo);
  atomicAdd(&cnt[2 * lane + 1], e_hi);
  sink[blockIdx.x * 256 + threadIdx.x] = acc + x;
}

// co-resident MFMA + LDS traffic (a GEMM's main-loop mix without global I/O)
__global__ void __launch_bounds__(256) aggressor(long long iters, float* sink, const float4* src,
                                                 long long nsrc) {
  __shared__ __attribute__((aligned(16))) short lds[256 * 64];
  typedef short s8 __attribute__((ext_vector_type(8)));
  typedef float f16v __attribute__((ext_vector_type(16)));
  for (int i = threadIdx.x; i < 256 * 64; i += 256) lds[i] = (short)(i * 7);
  __syncthreads();
  f16v acc0 = {}, acc1 = {}, acc2 = {}, acc3 = {};
  const int lane = threadIdx.x & 63;
  for (long long it = 0; it < iters; ++it) {
    const int o = ((int)(it & 31) * 64 + lane * 8) & (256 * 64 - 8);
    const s8 a = *reinterpret_cast<const s8*>(&lds[o]);
    const s8 b = *reinterpret_cast<const s8*>(&lds[(o + 512) & (256 * 64 - 8)]);
    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, b, acc3, 0, 0, 0);
    if (src) {   // + streaming global loads (GEMM operand traffic)
      const float4 g = src[((long long)it * 2048 + blockIdx.x * 256 + threadIdx.x) % nsrc];
      acc0[0] += g.x;
    }
  }
  float s = 0.f;
  for (int k = 0; k < 16; ++k) s += acc0[k] + acc1[k] + acc2[k] + acc3[k];
  sink[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int P>
int run(long long iters, int aggr, int ncu) {
  unsigned* cnt;
  f2* sink;
  float* asink;
  CK(hipMalloc(&cnt, 128 * sizeof(unsigned)));
  CK(hipMemset(cnt, 0, 128 * sizeof(unsigned)));
  float* dbg;
  CK(hipMalloc(&dbg, 16 * sizeof(float)));
  CK(hipMemset(dbg, 0, 16 * sizeof(float)));
  CK(hipMalloc(&sink, (size_t)ncu * 256 * sizeof(f2)));
  CK(hipMalloc(&asink, (size_t)ncu * 8 * 256 * sizeof(float)));
  const long long nsrc = 64ll << 20;   // 1 GiB of float4
  float4* src = nullptr;
  if (aggr == 2) {
    CK(hipMalloc(&src, nsrc * sizeof(float4)));
    CK(hipMemset(src, 0, nsrc * sizeof(float4)));
  }
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s1));
  hipLaunchKernelGGL(victim<P>, dim3(ncu), dim3(256), 0, s1, iters, cnt, sink, dbg);
  CK(hipGetLastError());
  CK(hipEventRecord(e1, s1));
  if (aggr) {
    // started after the victim: fills the wave slots the victim leaves
    hipLaunchKernelGGL(aggressor, dim3(ncu * 8), dim3(256), 0, s2, iters / 4, asink, src, nsrc);
    CK(hipGetLastError());
  }
  CK(hipDeviceSynchronize());
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned h[128];
  CK(hipMemcpy(h, cnt, sizeof(h), hipMemcpyDeviceToHost));
  unsigned long long lo = 0, hi = 0;
  char lanes[512] = {0};
  for (int l = 0; l < 64; ++l) {
    lo += h[2 * l];
    hi += h[2 * l + 1];
    if (h[2 * l] || h[2 * l + 1]) {
      char b[32];
      snprintf(b, sizeof(b), "%d:%u/%u ", l, h[2 * l], h[2 * l + 1]);
      if (strlen(lanes) + strlen(b) < sizeof(lanes)) strcat(lanes, b);
    }
  }
  float hd[16];
  CK(hipMemcpy(hd, dbg, sizeof(hd), hipMemcpyDeviceToHost));
  if (hd[0] != 0.f)
    printf("  first wrong low: got %.9g want %.9g (b.x %.9g y.x %.9g y.y %.9g a1.x %.9g a2.x %.9g "
           "lane %g; high got %.9g want %.9g)\n", hd[1], hd[2], hd[3], hd[4], hd[5], hd[6], hd[7],
           hd[8], hd[9], hd[10]);
  CK(hipFree(dbg));
  printf("pattern %d aggressor %d: victim %.1f ms, %lld x %d lanes; wrong low %llu high %llu; "
         "lanes %s\n", P, (int)aggr, ms, iters, ncu * 256, lo, hi, lanes[0] ? lanes : "-");
  fflush(stdout);
  CK(hipFree(cnt));
  CK(hipFree(sink));
  CK(hipFree(asink));
  if (src) CK(hipFree(src));
  CK(hipStreamDestroy(s1));
  CK(hipStreamDestroy(s2));
  return 0;
}

int main(int argc, char** argv) {
  const long long iters = (long long)((argc > 1 ? atof(argv[1]) : 2.0) * 1e6);
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  int rc = 0;
  const int ag0 = argc > 2 ? atoi(argv[2]) : 0;
  // one pattern per binary (-DPAT=n): many instantiations in one device
  // module crashed the ROCm 7.2 compiler
#ifndef PAT
#define PAT 4
#endif
  for (int ag = ag0; ag < 3 && !rc; ++ag) {
    rc |= run<0>(iters, ag, ncu);
    rc |= run<PAT>(iters, ag, ncu);
  }
  return rc;
}
