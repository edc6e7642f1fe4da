// Probe (round 5): which XCDs / CUs does a CU-masked stream's work run on?
// For a set of masks over the logical CU ids hipExtStreamCreateWithCUMask
// takes, launch 512 one-wave work-groups that record XCC_ID and HW_ID, and
// print per mask the XCDs used and the distinct (XCD, SE, CU) slots.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <set>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void where(unsigned* out) {
  if (threadIdx.x) return;
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  // busy a little so the work-groups spread instead of reusing one CU
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(4);
  out[2 * blockIdx.x] = xcc;
  out[2 * blockIdx.x + 1] = hw;
}

int main() {
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int NB = 512;
  unsigned* d;
  CK(hipMalloc(&d, NB * 2 * sizeof(unsigned)));
  struct M { const char* name; int kind; };
  const M ms[] = {{"all", 0}, {"ids 0-127", 1}, {"ids 128-255", 2}, {"ids 0-31", 3},
                  {"ids % 8 == 0", 4}, {"ids % 2 == 0", 5}, {"ids 0-63", 6}};
  for (const M& m : ms) {
    uint32_t mask[16] = {0};
    for (int c = 0; c < ncu; ++c) {
      bool on = m.kind == 0 || (m.kind == 1 && c < 128) || (m.kind == 2 && c >= 128) ||
                (m.kind == 3 && c < 32) || (m.kind == 4 && c % 8 == 0) ||
                (m.kind == 5 && c % 2 == 0) || (m.kind == 6 && c < 64);
      if (on) mask[c >> 5] |= 1u << (c & 31);
    }
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)((ncu + 31) / 32), mask));
    CK(hipMemset(d, 0xff, NB * 2 * sizeof(unsigned)));
    hipLaunchKernelGGL(where, dim3(NB), dim3(64), 0, s, d);
    CK(hipStreamSynchronize(s));
    std::vector<unsigned> h(NB * 2);
    CK(hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
    int per_xcc[16] = {0};
    std::set<unsigned> slots;
    for (int i = 0; i < NB; ++i) {
      per_xcc[h[2 * i] & 15]++;
      const unsigned hw = h[2 * i + 1];
      const unsigned cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      slots.insert((h[2 * i] << 16) | (se << 8) | (sh << 4) | cu);
    }
    printf("mask %-14s: work-groups per XCC", m.name);
    for (int x = 0; x < 8; ++x) printf(" %3d", per_xcc[x]);
    printf("   distinct (xcc,se,sh,cu) %zu\n", slots.size());
    CK(hipStreamDestroy(s));
  }
  CK(hipFree(d));
  return 0;
}
