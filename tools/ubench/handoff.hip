// Microbenchmark: same-XCD hand-off round trip on MI355X.
// Mode A (ping-pong): blocks 0 and 8 (same XCD under round-robin placement;
// checked with HW_REG_XCC_ID) bounce a step counter through one 8-B granule
// each; reports us per one-way hop.
// Mode B (allgather): 256 blocks; group = XCD (registered by XCC_ID); each
// member publishes an 8-B {value, tag} granule per step and polls all the
// group's granules (one lane per granule) before the next step.
// store_mode: 0 plain (workgroup-scope relaxed store), 1 sc1 (agent scope).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) int gint;

__device__ __forceinline__ unsigned xcc_id() {
  return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
}

__device__ __forceinline__ void put(unsigned long long* p, unsigned long long v, int mode) {
  if (mode) __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ unsigned long long get(unsigned long long* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void pingpong(unsigned long long* g, int iters, int mode, unsigned long long* out,
                         int* xcc) {
  extern __shared__ char pin[];
  if (threadIdx.x != 0) return;
  const int me = blockIdx.x == 0 ? 0 : 1;
  if (blockIdx.x != 0 && blockIdx.x != 8) return;
  xcc[me] = xcc_id();
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 1; i <= iters; ++i) {
    if (me == 0) {
      put(g, (unsigned long long)(2 * i - 1), mode);
      while (get(g + 16) != (unsigned long long)(2 * i)) {}
    } else {
      while (get(g) != (unsigned long long)(2 * i - 1)) {}
      put(g + 16, (unsigned long long)(2 * i), mode);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (me == 0) out[0] = t1 - t0;
}

// allgather within groups of 32 (one group per XCD; slot by atomic ticket)
__global__ void __launch_bounds__(64) allgather(unsigned long long* g, int* reg, int iters,
                                                int mode, unsigned long long* out) {
  extern __shared__ char pin[];
  __shared__ int s_slot, s_x;
  const int lane = threadIdx.x;
  if (lane == 0) {
    const unsigned x = xcc_id();
    s_x = x;
    s_slot = atomicAdd(&reg[x * 16], 1);
  }
  __syncthreads();
  const int x = s_x, slot = s_slot;
  unsigned long long* grp = g + (long long)x * 2 * 32 * 16;  // [2 parity][32 members] (128-B apart)
  unsigned long long t0 = 0;
  for (int s = 1; s <= iters; ++s) {
    if (s == 8) t0 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) put(grp + ((s & 1) * 32 + slot) * 16, ((unsigned long long)s << 32) | slot, mode);
    if (lane < 32) {
      unsigned long long* p = grp + ((s & 1) * 32 + lane) * 16;
      for (unsigned spins = 0;; ++spins) {
        if ((get(p) >> 32) == (unsigned long long)s) break;
        if (spins > (1u << 22)) break;
      }
    }
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) out[blockIdx.x] = (t1 - t0) * 1000 / (iters - 8);
}

int main() {
  unsigned long long *g, *out;
  int *xcc, *reg;
  hipMalloc(&g, 1 << 20);
  hipMalloc(&out, 256 * 8);
  hipMalloc(&xcc, 64);
  hipMalloc(&reg, 4096);
  const size_t pin = 96 * 1024;
  for (int mode = 0; mode < 2; ++mode) {
    hipMemset(g, 0, 1 << 20);
    hipLaunchKernelGGL(pingpong, dim3(16), dim3(64), pin, 0, g, 2000, mode, out, xcc);
    hipDeviceSynchronize();
    unsigned long long t;
    int hx[2];
    hipMemcpy(&t, out, 8, hipMemcpyDeviceToHost);
    hipMemcpy(hx, xcc, 8, hipMemcpyDeviceToHost);
    printf("pingpong store=%s xcc %d/%d: %.3f us per one-way hop\n", mode ? "sc1" : "plain",
           hx[0], hx[1], t / 100.0 / 4000.0);
  }
  for (int mode = 0; mode < 2; ++mode) {
    hipMemset(g, 0, 1 << 20);
    hipMemset(reg, 0, 4096);
    hipLaunchKernelGGL(allgather, dim3(256), dim3(64), pin, 0, g, reg, 1008, mode, out);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(256);
    hipMemcpy(h.data(), out, 256 * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    printf("allgather 32/XCD store=%s: %.3f us per step (median), p90 %.3f\n", mode ? "sc1" : "plain",
           h[128] / 1000.0 / 100.0, h[230] / 1000.0 / 100.0);
  }
  return 0;
}
