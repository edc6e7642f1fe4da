// Small memory-bound ops of the step (gfx950): dropout with a counter-based
// RNG (mask recomputed in backward, never stored), embedding lookup /
// gradient, tanh.  Vectorised 16 B per lane where the layout allows.
#include "mfma.h"

#include <algorithm>

namespace asr {
namespace {

__global__ void dropout_kernel(const float* __restrict__ x, float* __restrict__ y, long long n,
                               float p, unsigned long long seed) {
  const float scale = 1.f / (1.f - p);
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = u01(seed, i) >= p ? x[i] * scale : 0.f;
}

// out[r, :] = W[idx[r], :]   (W [V][E]) or W[:, idx[r]] (W^T stored [E][V])
__global__ void embedding_fwd(const long long* __restrict__ idx, const float* __restrict__ w,
                              int n, int V, int E, int trans, float* __restrict__ out) {
  const long long total = (long long)n * E;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / E), e = (int)(i % E);
    long long v = idx[r];
    v = v < 0 ? 0 : (v >= V ? V - 1 : v);
    out[i] = trans ? w[(long long)e * V + v] : w[v * E + e];
  }
}

// gw[v, e] += sum_{r: idx[r]==v} dout[r, e]  (skip v == padding_idx); fixed
// order over r -> deterministic.  One thread per (v, e).
__global__ void embedding_bwd(const long long* __restrict__ idx, const float* __restrict__ dout,
                              int n, int V, int E, int trans, int padding_idx,
                              float* __restrict__ gw) {
  const long long total = (long long)V * E;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int v = (int)(i / E), e = (int)(i % E);
    if (v == padding_idx) continue;
    float s = 0.f;
    for (int r = 0; r < n; ++r)
      if (idx[r] == v) s += dout[(long long)r * E + e];
    if (trans) gw[(long long)e * V + v] += s;
    else gw[i] += s;
  }
}

// Same sum with the rows grouped by token on the host (CSR: rows order[starts[v]
// .. starts[v+1]) hold token v, ascending): one work-group per token, O(n E)
// total.  EMB_SLOTS row slots of 64 columns each: slot r sums rows j0 + r,
// j0 + r + EMB_SLOTS, ... (four independent partial sums, combined in a fixed
// order), then the slots are added in slot order through LDS -- a fixed
// summation order (deterministic), with every slot's loads in flight at once
// (one 64-thread sequential loop per token took 257 us / step at att4x320).
constexpr int EMB_SLOTS = 16;
__global__ void __launch_bounds__(64 * EMB_SLOTS) embedding_bwd_csr(
    const int32_t* __restrict__ order, const int32_t* __restrict__ starts,
    const float* __restrict__ dout, int V, int E, int trans, int padding_idx,
    float* __restrict__ gw) {
  __shared__ float part[EMB_SLOTS][64];
  const int v = blockIdx.x;
  if (v == padding_idx) return;
  const int j0 = starts[v], j1 = starts[v + 1];
  if (j0 == j1) return;
  const int c = threadIdx.x & 63, r = threadIdx.x >> 6;
  for (int e0 = 0; e0 < E; e0 += 64) {
    const int e = e0 + c;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (e < E) {
      int j = j0 + r;
      for (; j + 3 * EMB_SLOTS < j1; j += 4 * EMB_SLOTS) {
        s0 += dout[(long long)order[j] * E + e];
        s1 += dout[(long long)order[j + EMB_SLOTS] * E + e];
        s2 += dout[(long long)order[j + 2 * EMB_SLOTS] * E + e];
        s3 += dout[(long long)order[j + 3 * EMB_SLOTS] * E + e];
      }
      for (; j < j1; j += EMB_SLOTS) s0 += dout[(long long)order[j] * E + e];
    }
    part[r][c] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (r == 0 && e < E) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < EMB_SLOTS; ++q) s += part[q][c];
      if (trans) gw[(long long)e * V + v] += s;
      else gw[(long long)v * E + e] += s;
    }
    __syncthreads();
  }
}

__global__ void tanh_fwd(const float* __restrict__ x, float* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    y[i] = tanhf(x[i]);
}

__global__ void tanh_bwd(const float* __restrict__ y, const float* __restrict__ dy,
                         float* __restrict__ dx, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    dx[i] = dy[i] * (1.f - y[i] * y[i]);
}

// dst[r][c] = bf16(src[row(r) + c]) for the rows of an asr_rowmap_t (zeros for
// rows mapping outside [0, t_limit)); 8 columns per thread, 16-B stores when
// ncols % 8 == 0.
// p > 0: the source is read through dropout (element at linear offset i of
// src kept iff u01(seed, i) >= p, scaled by 1/(1-p)) -- the mask asr_dropout
// would apply to the whole src tensor, fused into the bf16 staging.
template <bool DROP>
__global__ void convert_rows_kernel(const float* __restrict__ src, asr_rowmap_t m, int nrows,
                                    int ncols, int ld, uint16_t* __restrict__ dst, float p,
                                    unsigned long long seed) {
  const float scale = DROP ? 1.f / (1.f - p) : 1.f;
  auto val = [&](const float* q, float x) {
    if (!DROP) return x;
    return u01(seed, (unsigned long long)(q - src)) >= p ? x * scale : 0.f;
  };
  const int cpr = (ld + 7) >> 3;   // columns [ncols, ld) are written as zeros
  const long long nchunks = (long long)nrows * cpr;
  const int rpb = m.rows_per_b > 0 ? m.rows_per_b : 0x7fffffff;
  const int tmul = m.t_mul == 0 ? 1 : m.t_mul;
  const int tlim = m.t_limit > 0 ? m.t_limit : 0x7fffffff;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < nchunks;
       e += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(e / cpr), c0 = (int)(e - (long long)r * cpr) * 8;
    const int b = r / rpb, t = r - b * rpb;
    const int tp = t * tmul + m.t_add;
    const bool ok = tp >= 0 && tp < tlim;
    const float* s = ok ? src + (long long)(m.perm ? m.perm[b] : b) * m.stride_b +
                              (long long)tp * m.stride_t + c0
                        : nullptr;
    uint16_t* d = dst + (long long)r * ld + c0;
    if (ncols % 8 == 0 && ld % 8 == 0) {
      u16x8 v;
      if (ok && c0 < ncols) {
        const float4 x0 = *reinterpret_cast<const float4*>(s);
        const float4 x1 = *reinterpret_cast<const float4*>(s + 4);
        v = u16x8{f2bf(val(s, x0.x)), f2bf(val(s + 1, x0.y)), f2bf(val(s + 2, x0.z)),
                  f2bf(val(s + 3, x0.w)), f2bf(val(s + 4, x1.x)), f2bf(val(s + 5, x1.y)),
                  f2bf(val(s + 6, x1.z)), f2bf(val(s + 7, x1.w))};
      } else {
        v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
      *reinterpret_cast<u16x8*>(d) = v;
    } else {
      for (int j = 0; j < 8 && c0 + j < ld; ++j)
        d[j] = (ok && c0 + j < ncols) ? f2bf(val(s + j, s[j])) : (uint16_t)0;
    }
  }
}

// The same for rows whose width is not a multiple of 8 (e.g. the 10001-class
// output layer's gradient, whose f32 rows are only 4-B aligned): lane-
// consecutive columns, so every load and store instruction is coalesced (the
// 8-columns-per-thread form above issued eight 32-B-strided scalar loads and
// 2-B stores per thread: 300 us for an 8000 x 10001 gradient).  Block
// (x, y): columns [x * 1024, +1024) of rows y, y + gridDim.y, ...
template <bool DROP>
__global__ void convert_rows_cols(const float* __restrict__ src, asr_rowmap_t m, int nrows,
                                  int ncols, int ld, uint16_t* __restrict__ dst, float p,
                                  unsigned long long seed) {
  const float scale = DROP ? 1.f / (1.f - p) : 1.f;
  const int rpb = m.rows_per_b > 0 ? m.rows_per_b : 0x7fffffff;
  const int tmul = m.t_mul == 0 ? 1 : m.t_mul;
  const int tlim = m.t_limit > 0 ? m.t_limit : 0x7fffffff;
  for (int r = blockIdx.y; r < nrows; r += gridDim.y) {
    const int b = r / rpb, t = r - b * rpb;
    const int tp = t * tmul + m.t_add;
    const bool ok = tp >= 0 && tp < tlim;
    const long long so = ok ? (long long)(m.perm ? m.perm[b] : b) * m.stride_b +
                                  (long long)tp * m.stride_t
                            : 0;
    uint16_t* d = dst + (long long)r * ld;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = (blockIdx.x * 4 + k) * 256 + threadIdx.x;
      if (c >= ld) break;
      float x = 0.f;
      if (ok && c < ncols) {
        x = src[so + c];
        if (DROP && u01(seed, (unsigned long long)(so + c)) < p) x = 0.f;
        else if (DROP) x *= scale;
      }
      d[c] = f2bf(x);
    }
  }
}

// y = tanh(a + b): the attention bottleneck tanh(W_d(dec) + W_c(ctx)) when the
// two LinearND outputs carry their own dropout (attention_seq2seq.py:788-790)
__global__ void add_tanh_fwd(const float* __restrict__ a, const float* __restrict__ b,
                             float* __restrict__ y, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = tanhf(a[i] + b[i]);
}

// Residual connection sum (rnn.py:456-462), one read of each operand.
__global__ void add_fwd(const float* __restrict__ a, const float* __restrict__ b,
                        float* __restrict__ y, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = a[i] + b[i];
}

inline int grid_for(long long n) {
  long long b = (n + 255) / 256;
  return (int)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

// Up to four row-map conversions (the vector form of convert_rows_kernel<false>:
// ncols % 8 == 0, ld % 8 == 0, 16-B aligned rows) in one launch: job k owns
// blocks [blk0[k], blk0[k + 1]).  The GEMM's operand staging converted each
// f32 operand in a launch of its own, ~5 us apiece however small.
struct ConvJob {
  const float* src;
  asr_rowmap_t m;
  int nrows, ld;
  uint16_t* dst;
  int blk0;
};
struct ConvJobs {
  ConvJob j[4];
  int n;
};
__global__ void __launch_bounds__(256) convert_rows_multi(ConvJobs J) {
  int k = 0;
  while (k + 1 < J.n && (int)blockIdx.x >= J.j[k + 1].blk0) ++k;
  const ConvJob& jb = J.j[k];
  const int nb = (k + 1 < J.n ? J.j[k + 1].blk0 : (int)gridDim.x) - jb.blk0;
  const asr_rowmap_t& m = jb.m;
  const int cpr = jb.ld >> 3;
  const long long nchunks = (long long)jb.nrows * cpr;
  const int rpb = m.rows_per_b > 0 ? m.rows_per_b : 0x7fffffff;
  const int tmul = m.t_mul == 0 ? 1 : m.t_mul;
  const int tlim = m.t_limit > 0 ? m.t_limit : 0x7fffffff;
  for (long long e = (long long)(blockIdx.x - jb.blk0) * blockDim.x + threadIdx.x; e < nchunks;
       e += (long long)nb * blockDim.x) {
    const int r = (int)(e / cpr), c0 = (int)(e - (long long)r * cpr) * 8;
    const int b = r / rpb, t = r - b * rpb;
    const int tp = t * tmul + m.t_add;
    const bool ok = tp >= 0 && tp < tlim;
    u16x8 v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (ok) {
      const float* s = jb.src + (long long)(m.perm ? m.perm[b] : b) * m.stride_b +
                       (long long)tp * m.stride_t + c0;
      const float4 x0 = *reinterpret_cast<const float4*>(s);
      const float4 x1 = *reinterpret_cast<const float4*>(s + 4);
      v = u16x8{f2bf(x0.x), f2bf(x0.y), f2bf(x0.z), f2bf(x0.w),
                f2bf(x1.x), f2bf(x1.y), f2bf(x1.z), f2bf(x1.w)};
    }
    *reinterpret_cast<u16x8*>(jb.dst + (long long)r * jb.ld + c0) = v;
  }
}

}  // namespace

// n <= 4 conversions with ncols == ld (multiples of 8) and 16-B aligned rows,
// one launch (the GEMM operand staging); false when a job does not qualify
// (the caller converts one by one)
int convert_rows_bf16_multi(const float* const* src, const asr_rowmap_t* maps, const int* nrows,
                            const int* ncols, uint16_t* const* dst, int n, void* stream) {
  if (n < 1 || n > 4) return 0;
  ConvJobs J{};
  int blk = 0;
  for (int k = 0; k < n; ++k) {
    if (ncols[k] % 8 || nrows[k] <= 0 || ((uintptr_t)src[k] & 15) || ((uintptr_t)dst[k] & 15) ||
        maps[k].stride_t % 4 || maps[k].stride_b % 4)
      return 0;
    J.j[k] = ConvJob{src[k], maps[k], nrows[k], ncols[k], dst[k], blk};
    blk += grid_for((long long)nrows[k] * (ncols[k] / 8));
  }
  J.n = n;
  hipLaunchKernelGGL(convert_rows_multi, dim3(blk), dim3(256), 0, (hipStream_t)stream, J);
  return hipGetLastError() == hipSuccess ? 1 : -1;
}

}  // namespace asr

using namespace asr;

extern "C" int asr_dropout(const float* x, float* y, long long n, float p,
                           unsigned long long seed, void* stream) {
  ASR_REQUIRE(x && y, ASR_ERR_ARG, "dropout: null pointer");
  ASR_REQUIRE(p >= 0.f && p < 1.f, ASR_ERR_ARG, "dropout: p=%f", p);
  if (n <= 0) return ASR_OK;
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, y,
                     n, p, seed);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_embedding_forward(const long long* idx, const float* weight, int n, int V,
                                     int E, int trans, float* out, void* stream) {
  ASR_REQUIRE(idx && weight && out, ASR_ERR_ARG, "embedding: null pointer");
  if (n <= 0) return ASR_OK;
  hipLaunchKernelGGL(embedding_fwd, dim3(grid_for((long long)n * E)), dim3(256), 0,
                     (hipStream_t)stream, idx, weight, n, V, E, trans, out);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_embedding_backward(const long long* idx, const float* dout, int n, int V,
                                      int E, int trans, int padding_idx, float* grad_weight,
                                      void* stream) {
  ASR_REQUIRE(idx && dout && grad_weight, ASR_ERR_ARG, "embedding_backward: null pointer");
  if (n <= 0) return ASR_OK;
  hipLaunchKernelGGL(embedding_bwd, dim3(grid_for((long long)V * E)), dim3(256), 0,
                     (hipStream_t)stream, idx, dout, n, V, E, trans, padding_idx, grad_weight);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_embedding_backward_csr(const int32_t* order, const int32_t* starts,
                                          const float* dout, int V, int E, int trans,
                                          int padding_idx, float* grad_weight, void* stream) {
  ASR_REQUIRE(order && starts && dout && grad_weight, ASR_ERR_ARG,
              "embedding_backward_csr: null pointer");
  if (V <= 0 || E <= 0) return ASR_OK;
  hipLaunchKernelGGL(embedding_bwd_csr, dim3(V), dim3(64 * EMB_SLOTS), 0, (hipStream_t)stream, order, starts,
                     dout, V, E, trans, padding_idx, grad_weight);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_tanh_forward(const float* x, float* y, long long n, void* stream) {
  ASR_REQUIRE(x && y, ASR_ERR_ARG, "tanh: null pointer");
  if (n <= 0) return ASR_OK;
  hipLaunchKernelGGL(tanh_fwd, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, y, n);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_add_tanh_forward(const float* a, const float* b, float* y, long long n,
                                    void* stream) {
  ASR_REQUIRE(a && b && y, ASR_ERR_ARG, "add_tanh: null pointer");
  if (n <= 0) return ASR_OK;
  hipLaunchKernelGGL(add_tanh_fwd, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, a, b, y,
                     n);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_add_forward(const float* a, const float* b, float* y, long long n,
                               void* stream) {
  ASR_REQUIRE(a && b && y, ASR_ERR_ARG, "add: null pointer");
  if (n <= 0) return ASR_OK;
  hipLaunchKernelGGL(add_fwd, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, a, b, y, n);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_tanh_backward(const float* y, const float* dy, float* dx, long long n,
                                 void* stream) {
  ASR_REQUIRE(y && dy && dx, ASR_ERR_ARG, "tanh_backward: null pointer");
  if (n <= 0) return ASR_OK;
  hipLaunchKernelGGL(tanh_bwd, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, y, dy, dx, n);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_convert_rows_bf16_ld(const float* src, asr_rowmap_t map, int nrows,
                                        int ncols, int ld, uint16_t* dst, void* stream) {
  ASR_REQUIRE(src && dst && nrows >= 0 && ncols >= 0 && ld >= ncols, ASR_ERR_ARG,
              "convert_rows: bad args");
  if (ncols % 8 == 0 && ld % 8 == 0)
    ASR_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0 &&
                    map.stride_t % 4 == 0 && map.stride_b % 4 == 0,
                ASR_ERR_ARG, "convert_rows: vector path needs 16-B aligned rows");
  const long long n = (long long)nrows * ((ld + 7) / 8);
  if (n <= 0) return ASR_OK;
  if (!(ncols % 8 == 0 && ld % 8 == 0))
    hipLaunchKernelGGL(convert_rows_cols<false>, dim3((ld + 1023) / 1024, std::min(nrows, 8192)),
                       dim3(256), 0, (hipStream_t)stream, src, map, nrows, ncols, ld, dst, 0.f,
                       0ull);
  else
    hipLaunchKernelGGL(convert_rows_kernel<false>, dim3(grid_for(n)), dim3(256), 0,
                       (hipStream_t)stream, src, map, nrows, ncols, ld, dst, 0.f, 0ull);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_convert_rows_bf16_multi(int n, const float* const* src,
                                           const asr_rowmap_t* maps, const int* nrows,
                                           const int* ncols, uint16_t* const* dst, void* stream) {
  if (!src || !maps || !nrows || !ncols || !dst || n < 1 || n > 4) return 0;
  for (int k = 0; k < n; ++k)
    if (!src[k] || !dst[k]) return 0;
  return convert_rows_bf16_multi(src, maps, nrows, ncols, dst, n, stream);
}

extern "C" int asr_convert_rows_bf16_dropout(const float* src, asr_rowmap_t map, int nrows,
                                             int ncols, uint16_t* dst, float p,
                                             unsigned long long seed, void* stream) {
  ASR_REQUIRE(p >= 0.f && p < 1.f, ASR_ERR_ARG, "convert_rows_dropout: p=%f", (double)p);
  if (p == 0.f) return asr_convert_rows_bf16_ld(src, map, nrows, ncols, ncols, dst, stream);
  ASR_REQUIRE(src && dst && nrows >= 0 && ncols >= 0, ASR_ERR_ARG, "convert_rows: bad args");
  if (ncols % 8 == 0)
    ASR_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0 &&
                    map.stride_t % 4 == 0 && map.stride_b % 4 == 0,
                ASR_ERR_ARG, "convert_rows: vector path needs 16-B aligned rows");
  const long long n = (long long)nrows * ((ncols + 7) / 8);
  if (n <= 0) return ASR_OK;
  if (ncols % 8 != 0)
    hipLaunchKernelGGL(convert_rows_cols<true>, dim3((ncols + 1023) / 1024, std::min(nrows, 8192)),
                       dim3(256), 0, (hipStream_t)stream, src, map, nrows, ncols, ncols, dst, p,
                       seed);
  else
    hipLaunchKernelGGL(convert_rows_kernel<true>, dim3(grid_for(n)), dim3(256), 0,
                       (hipStream_t)stream, src, map, nrows, ncols, ncols, dst, p, seed);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_convert_rows_bf16(const float* src, asr_rowmap_t map, int nrows, int ncols,
                                     uint16_t* dst, void* stream) {
  return asr_convert_rows_bf16_ld(src, map, nrows, ncols, ncols, dst, stream);
}

// ---------------------------------------------------------------------------
// nn.LSTMCell nonlinearity (RNNDecoder.forward's cell, rnn_decoder.py:80-86;
// gate order i, f, g, o): pre [B][4D] = x W_ih^T + b_ih + h W_hh^T + b_hh (the
// caller's GEMM) -> c = sig(f) c_prev + sig(i) tanh(g), h = sig(o) tanh(c);
// act [B][4D] keeps the activated gates for the backward.
// ---------------------------------------------------------------------------
namespace {
__global__ void lstm_cell_fwd(const float* __restrict__ pre, const float* __restrict__ c_prev,
                              int B, int D, float* __restrict__ act, float* __restrict__ h,
                              float* __restrict__ c) {
  const long long n = (long long)B * D;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long b = i / D, j = i % D, g0 = b * 4 * D + j;
    const float ig = sigmoidf_(pre[g0]), fg = sigmoidf_(pre[g0 + D]);
    const float gg = tanhf_(pre[g0 + 2 * D]), og = sigmoidf_(pre[g0 + 3 * D]);
    const float cc = fg * (c_prev ? c_prev[i] : 0.f) + ig * gg;
    c[i] = cc;
    h[i] = og * tanhf_(cc);
    act[g0] = ig;
    act[g0 + D] = fg;
    act[g0 + 2 * D] = gg;
    act[g0 + 3 * D] = og;
  }
}

__global__ void lstm_cell_bwd(const float* __restrict__ act, const float* __restrict__ c_prev,
                              const float* __restrict__ c, const float* __restrict__ dh,
                              const float* __restrict__ dc, int B, int D,
                              float* __restrict__ dpre, float* __restrict__ dc_prev) {
  const long long n = (long long)B * D;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long b = i / D, j = i % D, g0 = b * 4 * D + j;
    const float ig = act[g0], fg = act[g0 + D], gg = act[g0 + 2 * D], og = act[g0 + 3 * D];
    const float tc = tanhf_(c[i]);
    const float dhv = dh ? dh[i] : 0.f;
    const float dct = (dc ? dc[i] : 0.f) + dhv * og * (1.f - tc * tc);
    const float cp = c_prev ? c_prev[i] : 0.f;
    dpre[g0] = dct * gg * ig * (1.f - ig);
    dpre[g0 + D] = dct * cp * fg * (1.f - fg);
    dpre[g0 + 2 * D] = dct * ig * (1.f - gg * gg);
    dpre[g0 + 3 * D] = dhv * tc * og * (1.f - og);
    if (dc_prev) dc_prev[i] = dct * fg;
  }
}
}  // namespace

extern "C" int asr_lstm_cell_forward(const float* pre, const float* c_prev, int B, int D,
                                     float* act, float* h, float* c, void* stream) {
  ASR_REQUIRE(pre && act && h && c && B > 0 && D > 0, ASR_ERR_ARG, "lstm_cell: bad arguments");
  const long long n = (long long)B * D;
  hipLaunchKernelGGL(lstm_cell_fwd, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, pre,
                     c_prev, B, D, act, h, c);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_lstm_cell_backward(const float* act, const float* c_prev, const float* c,
                                      const float* dh, const float* dc, int B, int D, float* dpre,
                                      float* dc_prev, void* stream) {
  ASR_REQUIRE(act && c && dpre && B > 0 && D > 0, ASR_ERR_ARG,
              "lstm_cell_backward: bad arguments");
  const long long n = (long long)B * D;
  hipLaunchKernelGGL(lstm_cell_bwd, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, act,
                     c_prev, c, dh, dc, B, D, dpre, dc_prev);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}
