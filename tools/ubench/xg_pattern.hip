// Microbenchmark of the forward recurrence's hand-off pattern without compute:
// 256 work-groups (one per CU), groups of 32 per XCD (registered by XCC_ID),
// 4 sweeper waves + 2 publisher waves per work-group.  Each step every member
// publishes 64 8-B {value, tag} granules (8 rows x 8 granules of its 16
// units) into the step-parity buffer [R=8 rows][256 granules] of its group;
// sweepers poll the whole 16 KB (8 x 16-B loads per lane, 32 lanes per wave)
// until every tag matches; one __syncthreads per step plus one after publish.
// Variants: nload = loads per sweeper lane (8 = full payload); pubfull = 1
// makes each publisher wave write whole 128-B lines (same bytes, different
// lane->address map); extra = per-step HBM loads + stores by the publishers
// (the cell waves' input prefetch / output stores).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((address_space(1))) unsigned long long gu64;

__global__ void __launch_bounds__(384) pattern(unsigned long long* g, int* reg, int T, int nload,
                                               int extra, float* big, unsigned long long* out) {
  extern __shared__ char pin[];
  __shared__ int s_slot, s_x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) {
    const unsigned x = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
    s_x = x;
    s_slot = atomicAdd(&reg[x * 16], 1);
  }
  __syncthreads();
  const int grp = s_x, mem = s_slot;
  unsigned long long* base = g + (long long)grp * 2 * 8 * 256;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 2 * 8 * 256 * 8, 0x00020000);
  unsigned long long t0 = 0;
  float acc = 0.f;
  for (int s = 0; s < T; ++s) {
    if (s == 16) t0 = __builtin_amdgcn_s_memrealtime();
    if (wave < 4) {
      if (s > 0) {
        const int ln = lane & 15, kq = lane >> 4;
        const unsigned tag = (unsigned)s;
        const unsigned rowoff = (unsigned)((((s - 1) & 1) * 8 + (ln & 7)) * 256 * 8);
        for (unsigned spins = 0;; ++spins) {
          int ok = 1;
          if (ln < 8) {
            for (int i = 0; i < 4; ++i) {
              if (2 * i >= nload) break;
              const unsigned off = rowoff + (unsigned)((16 * (wave + 4 * i) + 4 * kq) * 8);
              u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16 | (1u << 31));
              u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 16 | (1u << 31));
              ok &= (int)(a[1] == tag) & (int)(a[3] == tag) & (int)(b[1] == tag) & (int)(b[3] == tag);
              acc += __uint_as_float(a[0] ^ b[2]);
            }
          }
          if (__all(ok)) break;
          if (spins > (1u << 20)) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      __syncthreads();
    } else {
      __syncthreads();
      const int ct = tid - 256, row = ct >> 4, unit = ct & 15;
      if ((unit & 1) == 0) {
        unsigned long long* p = base + ((s & 1) * 8 + row) * 256 + (mem * 16 + unit) / 2;
        __hip_atomic_store((gu64*)p, ((unsigned long long)(s + 1) << 32) | 7u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __syncthreads();
      if (extra) {
        const long long o = ((long long)blockIdx.x * 128 + ct) + (long long)(s % 512) * 256 * 128 * 8;
        for (int q = 0; q < 4; ++q) acc += big[o + q * 256 * 128];
        for (int q = 0; q < 6; ++q) big[o + (q + 4) * 256 * 128] = acc;
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) out[blockIdx.x] = (t1 - t0) * 1000 / (T - 16) + (acc == 1.2345f);
}

int main() {
  unsigned long long *g, *out;
  int* reg;
  float* big;
  hipMalloc(&g, 1 << 20);
  hipMalloc(&out, 256 * 8);
  hipMalloc(&reg, 4096);
  const size_t bigsz = (size_t)512 * 256 * 128 * 8 * 4 + (1 << 20);
  hipMalloc(&big, bigsz);
  hipMemset(big, 0, bigsz);
  const size_t pin = 96 * 1024;
  for (int extra = 0; extra < 2; ++extra)
    for (int nload : {8, 4, 2}) {
      hipMemset(g, 0, 1 << 20);
      hipMemset(reg, 0, 4096);
      hipLaunchKernelGGL(pattern, dim3(256), dim3(384), pin, 0, g, reg, 1016, nload, extra, big, out);
      hipDeviceSynchronize();
      std::vector<unsigned long long> h(256);
      hipMemcpy(h.data(), out, 256 * 8, hipMemcpyDeviceToHost);
      std::sort(h.begin(), h.end());
      printf("extra=%d loads/lane=%d: %.3f us per step (median), p90 %.3f\n", extra, nload,
             h[128] / 1000.0 / 100.0, h[230] / 1000.0 / 100.0);
    }
  return 0;
}
