// Fused softmax cross-entropy + uniform label smoothing on gfx950.
// Replaces F.cross_entropy(sum, ignore_index=-1) of the attention decoder
// (attention_seq2seq.py:588-591) and cross_entropy_label_smoothing
// (criterion.py:51-80, used at attention_seq2seq.py:594-601 and ctc.py:329-337):
//
//   loss = ce_scale * sum_{rows, tgt>=0} (lse - x[tgt])
//        + ls_scale * sum_{rows in LS mask} -(1/V) sum_v (x[v] - lse)
//   dx[v] = g * ( ce_scale*(p[v] - [v==tgt])*[tgt>=0] + ls_scale*(p[v] - 1/V)*[LS row] )
//
// LS mask: t < lens[b] when lens is given (rows indexed b*T + t), else tgt >= 0.
// One wave per row; the row's lse is kept for backward; per-row losses are
// reduced in a fixed order (deterministic).  Also a plain row softmax.
#include "common.h"

namespace asr {
namespace {

__device__ __forceinline__ void row_stats(const float* x, int V, int lane, float& lse, float& sx) {
  float m = neg_inf();
  for (int v = lane; v < V; v += 64) m = fmaxf(m, x[v]);
  m = wave_max(m);
  float s = 0.f, a = 0.f;
  for (int v = lane; v < V; v += 64) {
    s += __expf(x[v] - m);
    a += x[v];
  }
  s = wave_sum(s);
  sx = wave_sum(a);
  lse = m + __logf(s);
}

__device__ __forceinline__ bool ls_row(int r, int T, const int32_t* lens, const long long* tgt) {
  if (lens) return (r % T) < lens[r / T];
  return tgt ? tgt[r] >= 0 : true;
}

__global__ void xent_fwd(const float* __restrict__ x, int R, int V, int T,
                         const long long* __restrict__ tgt, const int32_t* __restrict__ lens,
                         float ce_scale, float ls_scale, float* __restrict__ lse_out,
                         float* __restrict__ row_loss) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  const float* p = x + (long long)r * V;
  float lse, sx;
  row_stats(p, V, lane, lse, sx);
  if (lane == 0) {
    float l = 0.f;
    if (tgt && ce_scale != 0.f && tgt[r] >= 0) {
      long long c = tgt[r] < V ? tgt[r] : V - 1;
      l += ce_scale * (lse - p[c]);
    }
    if (ls_scale != 0.f && ls_row(r, T, lens, tgt)) l += ls_scale * (-(sx - V * lse) / V);
    lse_out[r] = lse;
    row_loss[r] = l;
  }
}

__global__ void sum_rows(const float* __restrict__ v, int n, float* __restrict__ out) {
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += v[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

__global__ void xent_bwd(const float* __restrict__ x, int R, int V, int T,
                         const long long* __restrict__ tgt, const int32_t* __restrict__ lens,
                         float ce_scale, float ls_scale, const float* __restrict__ lse,
                         const float* __restrict__ g, float gmul, float* __restrict__ dx) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  const float gs = (g ? g[0] : 1.f) * gmul;
  const float* p = x + (long long)r * V;
  float* d = dx + (long long)r * V;
  const bool ce = tgt && ce_scale != 0.f && tgt[r] >= 0;
  const long long c = ce ? (tgt[r] < V ? tgt[r] : V - 1) : -1;
  const bool ls = ls_scale != 0.f && ls_row(r, T, lens, tgt);
  const float z = lse[r];
  const float invV = 1.f / V;
  for (int v = lane; v < V; v += 64) {
    const float pv = __expf(p[v] - z);
    float o = 0.f;
    if (ce) o += ce_scale * (pv - (v == c ? 1.f : 0.f));
    if (ls) o += ls_scale * (pv - invV);
    d[v] = o * gs;
  }
}

__global__ void softmax_rows(const float* __restrict__ x, int R, int V, float* __restrict__ y) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  const float* p = x + (long long)r * V;
  float lse, sx;
  row_stats(p, V, lane, lse, sx);
  for (int v = lane; v < V; v += 64) y[(long long)r * V + v] = __expf(p[v] - lse);
}

}  // namespace
}  // namespace asr

using namespace asr;

extern "C" size_t asr_xent_workspace_bytes(int R) { return (size_t)2 * (R > 0 ? R : 1) * 4; }

extern "C" int asr_xent_forward(const float* logits, int R, int V, int T, const long long* targets,
                                const int32_t* lens, float ce_scale, float ls_scale,
                                float* loss_out, void* workspace, size_t ws_bytes, void* stream) {
  ASR_REQUIRE(logits && loss_out && workspace, ASR_ERR_ARG, "xent: null pointer");
  ASR_REQUIRE(ws_bytes >= asr_xent_workspace_bytes(R), ASR_ERR_WORKSPACE, "xent: workspace");
  ASR_REQUIRE(!lens || T > 0, ASR_ERR_ARG, "xent: T must be > 0 with lens");
  hipStream_t s = (hipStream_t)stream;
  float* lse = (float*)workspace;
  float* rl = lse + R;
  if (R > 0) {
    hipLaunchKernelGGL(xent_fwd, dim3((R + 3) / 4), dim3(256), 0, s, logits, R, V, T, targets,
                       lens, ce_scale, ls_scale, lse, rl);
    ASR_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(sum_rows, dim3(1), dim3(256), 0, s, rl, R, loss_out);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_xent_backward(const float* logits, int R, int V, int T,
                                 const long long* targets, const int32_t* lens, float ce_scale,
                                 float ls_scale, const float* grad_scale, float scale,
                                 float* dlogits, const void* workspace, size_t ws_bytes,
                                 void* stream) {
  ASR_REQUIRE(logits && dlogits && workspace, ASR_ERR_ARG, "xent_backward: null pointer");
  ASR_REQUIRE(ws_bytes >= asr_xent_workspace_bytes(R), ASR_ERR_WORKSPACE, "xent: workspace");
  if (R <= 0) return ASR_OK;
  hipLaunchKernelGGL(xent_bwd, dim3((R + 3) / 4), dim3(256), 0, (hipStream_t)stream, logits, R, V,
                     T, targets, lens, ce_scale, ls_scale, (const float*)workspace, grad_scale,
                     scale, dlogits);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_softmax(const float* x, int R, int V, float* y, void* stream) {
  ASR_REQUIRE(x && y, ASR_ERR_ARG, "softmax: null pointer");
  if (R <= 0) return ASR_OK;
  hipLaunchKernelGGL(softmax_rows, dim3((R + 3) / 4), dim3(256), 0, (hipStream_t)stream, x, R, V,
                     y);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}
