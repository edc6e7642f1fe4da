// Microbenchmark: latency of one "poll" (N x 16-B sc1 buffer loads per lane,
// 32 active lanes per wave, 4 waves per work-group, one work-group per CU)
// over an L2-resident 16 KB region, with all work-groups of an XCD reading the
// SAME region (like the recurrence's consumers) or each its own.
// Reports median cycles (s_memrealtime, 100 MHz) per poll iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

template <int N>
__global__ void __launch_bounds__(256) poll(const unsigned* buf, int iters, int shared,
                                            unsigned long long* out, int active_lanes) {
  extern __shared__ char pin[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned region = shared ? 0u : (unsigned)blockIdx.x * 16384u;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)buf, 0, 0x7fffffff, 0x00020000);
  unsigned acc = 0;
  unsigned long long t0 = 0;
  for (int it = 0; it < iters; ++it) {
    if (it == 8) t0 = __builtin_amdgcn_s_memrealtime();
    if (lane < active_lanes) {
      u32x4 v[N];
#pragma unroll
      for (int i = 0; i < N; ++i)
        v[i] = __builtin_amdgcn_raw_buffer_load_b128(
            rs, region + (unsigned)(wave * 4096 + i * 512 + (lane & 31) * 16), 0, 16 | (1u << 31));
#pragma unroll
      for (int i = 0; i < N; ++i) acc += v[i][0] ^ v[i][1];
    }
    acc = __builtin_amdgcn_readfirstlane(acc);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[blockIdx.x] = (t1 - t0) * 1000 / (iters - 8) + (acc == 12345 ? 1 : 0);
}

int main() {
  unsigned* buf;
  unsigned long long* out;
  hipMalloc(&buf, 256 * 16384 + 65536);
  hipMemset(buf, 1, 256 * 16384 + 65536);
  hipMalloc(&out, 256 * 8);
  std::vector<unsigned long long> h(256);
  const size_t pin = 96 * 1024;
  for (int shared = 0; shared < 2; ++shared)
    for (int lanes : {32, 64}) {
      for (int n : {1, 2, 8}) {
        auto k = n == 1 ? poll<1> : n == 2 ? poll<2> : poll<8>;
        for (int rep = 0; rep < 2; ++rep) {
          hipLaunchKernelGGL(k, dim3(256), dim3(256), pin, 0, buf, 208, shared, out, lanes);
          hipDeviceSynchronize();
        }
        hipMemcpy(h.data(), out, 256 * 8, hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        printf("shared=%d lanes=%d loads/lane=%d  poll = %.3f us (median over CUs; p90 %.3f)\n",
               shared, lanes, n, h[128] / 1000.0 / 100.0, h[230] / 1000.0 / 100.0);
      }
    }
  // single work-group (idle chip)
  hipLaunchKernelGGL(poll<8>, dim3(1), dim3(256), pin, 0, buf, 208, 1, out, 32);
  hipDeviceSynchronize();
  hipMemcpy(h.data(), out, 8, hipMemcpyDeviceToHost);
  printf("single WG, 8 loads/lane: %.3f us\n", h[0] / 1000.0 / 100.0);
  hipLaunchKernelGGL(poll<1>, dim3(1), dim3(256), pin, 0, buf, 208, 1, out, 32);
  hipDeviceSynchronize();
  hipMemcpy(h.data(), out, 8, hipMemcpyDeviceToHost);
  printf("single WG, 1 load/lane: %.3f us\n", h[0] / 1000.0 / 100.0);
  return 0;
}
