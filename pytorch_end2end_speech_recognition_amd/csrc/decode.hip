// CTC best-path decoding on gfx950 (replaces the numpy GreedyDecoder,
// models/pytorch_v3/ctc/decoders/greedy_decoder.py:19-47), plus a row argmax
// used by scheduled sampling / greedy attention decoding.
//
// best path: one wave per utterance.  Per frame the 64 lanes reduce the
// argmax over V (first maximum wins ties, as np.argmax); frames are processed in
// chunks of 64 (one frame per lane after the reductions) so the collapse of
// repeats and the blank removal are a wave prefix-sum (ballot + popcount), and
// the surviving labels are written compactly.  Output: hyps [B][T] (first
// hyp_lens[b] entries valid), lengths [B].
#include "common.h"

namespace asr {
namespace {

__device__ __forceinline__ void argmax_pair(float& v, int& i, float ov, int oi) {
  if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
}

__global__ void __launch_bounds__(64) best_path_kernel(const float* __restrict__ logits,
                                                       long long st, long long sb, int T, int V,
                                                       const int32_t* __restrict__ lens, int blank,
                                                       int32_t* __restrict__ hyps,
                                                       int32_t* __restrict__ hyp_lens) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int Tb = min(lens[b], T);
  int prev = -1;      // label of the previous frame (for collapsing repeats)
  int count = 0;
  int32_t* out = hyps + (long long)b * T;
  for (int t0 = 0; t0 < Tb; t0 += 64) {
    int my_label = -1;
    const int nf = min(64, Tb - t0);
    for (int f = 0; f < nf; ++f) {
      const float* x = logits + (long long)(t0 + f) * st + (long long)b * sb;
      float bv = -__builtin_huge_valf();
      int bi = 0x7fffffff;
      for (int v = lane; v < V; v += 64) argmax_pair(bv, bi, x[v], v);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        argmax_pair(bv, bi, ov, oi);
      }
      if (lane == f) my_label = bi;
    }
    // lane f holds frame t0+f's argmax; previous frame's label via shuffle
    int left = __shfl_up(my_label, 1, 64);
    if (lane == 0) left = prev;
    const bool valid = lane < nf;
    const bool keep = valid && my_label != left && my_label != blank;
    const unsigned long long mask = __ballot(keep);
    const int pos = __popcll(mask & ((1ull << lane) - 1ull));
    if (keep) out[count + pos] = my_label;
    count += __popcll(mask);
    prev = __shfl(my_label, nf - 1, 64);
  }
  if (lane == 0) hyp_lens[b] = count;
}

__global__ void row_argmax_kernel(const float* __restrict__ x, int rows, int V,
                                  long long* __restrict__ out) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* p = x + (long long)r * V;
  float bv = -__builtin_huge_valf();
  int bi = 0x7fffffff;
  for (int v = lane; v < V; v += 64) argmax_pair(bv, bi, p[v], v);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    argmax_pair(bv, bi, ov, oi);
  }
  if (lane == 0) out[r] = bi;
}

}  // namespace
}  // namespace asr

using namespace asr;

extern "C" int asr_ctc_best_path(const float* logits, long long stride_t, long long stride_b,
                                 int T, int B, int V, const int32_t* lens, int blank,
                                 int32_t* hyps, int32_t* hyp_lens, void* stream) {
  ASR_REQUIRE(logits && lens && hyps && hyp_lens, ASR_ERR_ARG, "best_path: null pointer");
  ASR_REQUIRE(T > 0 && B > 0 && V > 0, ASR_ERR_ARG, "best_path: bad shape");
  hipLaunchKernelGGL(best_path_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, logits,
                     stride_t, stride_b, T, V, lens, blank, hyps, hyp_lens);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_row_argmax(const float* x, int rows, int V, long long* out, void* stream) {
  ASR_REQUIRE(x && out, ASR_ERR_ARG, "row_argmax: null pointer");
  if (rows <= 0) return ASR_OK;
  hipLaunchKernelGGL(row_argmax_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     x, rows, V, out);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}
