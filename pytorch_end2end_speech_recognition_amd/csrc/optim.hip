// Fused optimizer step over the model's flat parameter / gradient buffers
// (gfx950).  Replaces torch.nn.utils.clip_grad_norm(params, max_norm) +
// torch.optim.{Adam,SGD} (models/pytorch_v3/base.py:141-213,
// utils/training/training_loop.py:46-51).
//
//   asr_grad_sqnorm: deterministic two-pass sum of squares -> device scalar
//   asr_optim_step : clip coefficient computed ON DEVICE from that scalar
//                    (no host sync), then the update, one pass over HBM:
//                    reads p, g, m, v; writes p, m, v (+ optional bf16 copy of p).
// Semantics follow torch: clip_coef = max_norm / (||g|| + 1e-6) applied when
// < 1; L2 weight decay added to the gradient; Adam bias corrections from the
// host-side step count.
#include "common.h"

namespace asr {
namespace {

constexpr int NB_RED = 1024;  // partial-sum blocks (fixed -> deterministic)

__global__ void sqnorm_partial(const float* __restrict__ g, long long n,
                               float* __restrict__ partial) {
  __shared__ float red[256];
  float s = 0.f;
  const long long stride = (long long)gridDim.x * blockDim.x * 4;
  for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 4 <= n) {
      float4 v = *reinterpret_cast<const float4*>(g + i);
      s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    } else {
      for (long long j = i; j < n; ++j) s += g[j] * g[j];
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ void sqnorm_final(const float* __restrict__ partial, int np, float* __restrict__ out) {
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < np; i += 256) s += partial[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

struct StepArgs {
  float lr, beta1, beta2, eps, weight_decay, bc1, bc2_sqrt, momentum, dampening;
  float max_norm;
  int kind;      // 0 adam, 1 sgd, 2 momentum, 3 nesterov
  int first;     // first step for the momentum buffer
};

__device__ __forceinline__ float clip_coef(const float* sqnorm, float max_norm) {
  if (!sqnorm || max_norm <= 0.f) return 1.f;
  const float c = max_norm / (sqrtf(sqnorm[0]) + 1e-6f);
  return c < 1.f ? c : 1.f;
}

__global__ void optim_step_kernel(float* __restrict__ p, const float* __restrict__ g,
                                  float* __restrict__ m, float* __restrict__ v, long long n,
                                  StepArgs a, const float* __restrict__ sqnorm,
                                  uint16_t* __restrict__ shadow, const int* __restrict__ guard) {
  // guard: the step's recurrence status words (asr_lstm_status_gather); a
  // bounded spin that gave up invalidated the gradients -> no update at all
  // (the bf16 shadow is still rewritten from the unchanged parameters, so it
  // matches them after every step, skipped or not)
  const long long stride = (long long)gridDim.x * blockDim.x;
  if (guard && (guard[0] | guard[1])) {
    if (shadow)
      for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        shadow[i] = f2bf(p[i]);
    return;
  }
  const float coef = clip_coef(sqnorm, a.max_norm);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float w = p[i];
    float gr = g[i] * coef + a.weight_decay * w;
    if (a.kind == 0) {
      const float mi = a.beta1 * m[i] + (1.f - a.beta1) * gr;
      const float vi = a.beta2 * v[i] + (1.f - a.beta2) * gr * gr;
      m[i] = mi;
      v[i] = vi;
      const float denom = sqrtf(vi) / a.bc2_sqrt + a.eps;
      w -= (a.lr / a.bc1) * mi / denom;
    } else if (a.kind == 1) {
      w -= a.lr * gr;
    } else {
      float buf = a.first ? gr : a.momentum * m[i] + (1.f - a.dampening) * gr;
      m[i] = buf;
      const float d = a.kind == 3 ? gr + a.momentum * buf : buf;
      w -= a.lr * d;
    }
    p[i] = w;
    if (shadow) shadow[i] = f2bf(w);
  }
}

}  // namespace
}  // namespace asr

using namespace asr;

extern "C" size_t asr_grad_sqnorm_workspace_bytes(void) { return NB_RED * sizeof(float); }

extern "C" int asr_grad_sqnorm(const float* g, long long n, float* out, void* workspace,
                               size_t ws_bytes, void* stream) {
  ASR_REQUIRE(g && out && workspace, ASR_ERR_ARG, "grad_sqnorm: null pointer");
  ASR_REQUIRE(ws_bytes >= NB_RED * sizeof(float), ASR_ERR_WORKSPACE,
              "grad_sqnorm: workspace too small");
  ASR_REQUIRE(((uintptr_t)g & 15) == 0, ASR_ERR_ARG, "grad_sqnorm: g must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sqnorm_partial, dim3(NB_RED), dim3(256), 0, s, g, n, (float*)workspace);
  ASR_LAUNCH_CHECK();
  hipLaunchKernelGGL(sqnorm_final, dim3(1), dim3(256), 0, s, (const float*)workspace, NB_RED, out);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_optim_step_guarded(int kind, float* params, const float* grads, float* m,
                                      float* v, long long n, float lr, float beta1, float beta2,
                                      float eps, float weight_decay, long long step,
                                      float momentum, float dampening, const float* grad_sqnorm,
                                      float max_norm, uint16_t* bf16_shadow, const int* guard,
                                      void* stream) {
  ASR_REQUIRE(params && grads, ASR_ERR_ARG, "optim_step: null pointer");
  ASR_REQUIRE(kind >= 0 && kind <= 3, ASR_ERR_ARG, "optim_step: bad kind %d", kind);
  ASR_REQUIRE(kind == 1 || m, ASR_ERR_ARG, "optim_step: state buffer m is null");
  ASR_REQUIRE(kind != 0 || v, ASR_ERR_ARG, "optim_step: state buffer v is null");
  StepArgs a;
  a.lr = lr; a.beta1 = beta1; a.beta2 = beta2; a.eps = eps; a.weight_decay = weight_decay;
  a.bc1 = (float)(1.0 - pow((double)beta1, (double)step));
  a.bc2_sqrt = (float)sqrt(1.0 - pow((double)beta2, (double)step));
  a.momentum = momentum; a.dampening = dampening; a.max_norm = max_norm;
  a.kind = kind; a.first = step <= 1;
  if (n <= 0) return ASR_OK;
  const long long nb = (n + 255) / 256;
  const int blocks = (int)(nb < 8192 ? nb : 8192);
  hipLaunchKernelGGL(optim_step_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, params,
                     grads, m, v, n, a, grad_sqnorm, bf16_shadow, guard);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_optim_step(int kind, float* params, const float* grads, float* m, float* v,
                              long long n, float lr, float beta1, float beta2, float eps,
                              float weight_decay, long long step, float momentum,
                              float dampening, const float* grad_sqnorm, float max_norm,
                              uint16_t* bf16_shadow, void* stream) {
  return asr_optim_step_guarded(kind, params, grads, m, v, n, lr, beta1, beta2, eps,
                                weight_decay, step, momentum, dampening, grad_sqnorm, max_norm,
                                bf16_shadow, nullptr, stream);
}
