// VGG front-end of the encoder (models/pytorch_v3/encoders/cnn.py:124-165) on
// gfx950: per layer Conv2d 3x3 (stride 1, padding 1) -> ReLU -> MaxPool
// (kernel = stride; the first pool floor mode, later ones ceil mode) ->
// BatchNorm2d (training: batch statistics over every (b, f, t), padding frames
// included, as the reference computes them) -> Dropout.
//
// Layout: the reference's NCHW view [B, C, F, T] (cnn.py:143-149) is kept
// channels-last and zero-haloed: a layer input is [B][T+2][F+2][C] ("padded
// pixels" x channels), so a 3x3 tap is a constant row shift of
// (dt)*(F+2) + df and the convolution is ONE implicit GEMM on the MFMA kernels
// of gemm.hip (asr_operand_t tap addressing): M = padded pixels, N = C_out,
// K = 9 C_in.  Rows of halo pixels are computed and ignored.  Layers whose
// channel counts the tap addressing cannot take (the first layer, C_in = 1)
// use direct kernels.  This file holds the bandwidth-bound
// pieces around the GEMMs:
//   vgg_pad_input   xs [B][T][F] -> [B][T+2][F+2] (zero halo)
//   conv_direct_*   3x3 conv without the GEMM (C_in = 1, small channel counts)
//   post_fwd        ReLU + max-pool -> P [B][T'][F'][C], argmax slot per output
//   bn stats        per-channel mean / inverse std over P (two passes, fixed order)
//   apply_fwd       BN affine + dropout -> next layer's padded input (f32 or
//                   bf16) or the encoder input [B][T'][F'*C] (cnn.py:155-157)
//   bwd             dropout, BN backward (sum dy, sum dy xhat), pool + ReLU
//                   routing into dZ [padded pixels][C] (halo zero)
#include "mfma.h"

namespace asr {
namespace {

constexpr int CT = 256;

__device__ __forceinline__ long long pad_row(int b, int t, int f, int T, int F) {
  return ((long long)b * (T + 2) + (t + 1)) * (F + 2) + (f + 1);
}

// out[b][t+1][f+1][c] = xs[b][t][f] for c = 0, 0 for c < Cp and on the halo
// (the input plane as a Cp-channel padded image, Cp = 1 or 16 for the GEMM path)
template <typename TO>
__global__ void vgg_pad_input(const float* __restrict__ xs, int B, int T, int F, int Cp,
                              TO* __restrict__ out) {
  const long long n = (long long)B * (T + 2) * (F + 2) * Cp;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const long long pix = i / Cp;
    const int fp = (int)(pix % (F + 2));
    const long long q = pix / (F + 2);
    const int tp = (int)(q % (T + 2));
    const int b = (int)(q / (T + 2));
    const int t = tp - 1, f = fp - 1;
    const float v = (c == 0 && t >= 0 && t < T && f >= 0 && f < F)
                        ? xs[((long long)b * T + t) * F + f] : 0.f;
    if constexpr (sizeof(TO) == 2) out[i] = f2bf(v);
    else out[i] = v;
  }
}

// Direct 3x3 convolution for layers whose channel counts do not suit the
// tap-addressed GEMM (C_in = 1 of the first layer, small test configs).
// x [padded pixels][Ci] f32, w the torch weight [Co][Ci][3(f)][3(t)].
// z[p][co] = sum_{ci,kh,kw} w[co][ci][kh][kw] x[p + (kw-1)(F+2) + kh-1][ci] (+ bias),
// valid pixels only.
__global__ void conv_direct_fwd(const float* __restrict__ x, int B, int T, int F, int Ci, int Co,
                                const float* __restrict__ w, const float* __restrict__ bias,
                                float* __restrict__ z) {
  const long long n = (long long)B * T * F * Co;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(i % Co);
    const long long pix = i / Co;
    const int f = (int)(pix % F);
    const int t = (int)((pix / F) % T);
    const int b = (int)(pix / ((long long)F * T));
    const long long p = pad_row(b, t, f, T, F);
    float s = bias ? bias[co] : 0.f;
    for (int ci = 0; ci < Ci; ++ci) {
      const float* wr = w + ((long long)co * Ci + ci) * 9;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
          s += wr[kh * 3 + kw] * x[(p + (long long)(kw - 1) * (F + 2) + (kh - 1)) * Ci + ci];
    }
    z[p * Co + co] = s;
  }
}

// First VGG layer (one input channel) forward as a direct stencil: one
// work-group per (utterance, frame); the three padded input rows it needs
// (channel 0 of the padded operand, pitch cstride elements) and the Co x 9
// weights go to LDS; each thread produces 4 channels of a pixel per
// iteration (16-B z stores, 16 threads = one pixel's 64 channels).  The
// tap-addressed GEMM did this with the channel padded to 16 (K = 144 of which
// 9 useful) in 837 us at vgg_hier; this is bound by z's f32 write.
template <typename TX>
__global__ void __launch_bounds__(CT) conv3x3_c1_fwd(const TX* __restrict__ x, int cstride, int T,
                                                     int F, int Co, const float* __restrict__ w,
                                                     const float* __restrict__ bias,
                                                     float* __restrict__ z) {
  extern __shared__ float sm[];
  float* xr = sm;                    // [3][F + 2]
  float* ws = sm + 3 * (F + 2);      // [9][Co]: tap-major, channel fastest
  const int bt = blockIdx.x;
  const int b = bt / T, t = bt - b * T;
  const long long row0 = ((long long)b * (T + 2) + t) * (F + 2);   // padded row t - 1
  for (int i = threadIdx.x; i < 3 * (F + 2); i += CT) {
    const TX v = x[(row0 + i) * cstride];
    if constexpr (sizeof(TX) == 2) xr[i] = bf2f((uint16_t)v);
    else xr[i] = (float)v;
  }
  for (int i = threadIdx.x; i < 9 * Co; i += CT) {
    const int co = i % Co, tap = i / Co;     // tap = kh * 3 + kw
    ws[i] = w[co * 9 + tap];
  }
  __syncthreads();
  const int ng = Co >> 2;
  for (int i = threadIdx.x; i < F * ng; i += CT) {
    const int f = i / ng, c4 = 4 * (i - (i / ng) * ng);
    float4 acc = bias ? *reinterpret_cast<const float4*>(bias + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        // z[p] += w[co][kh][kw] x[p + (kw - 1)(F + 2) + (kh - 1)]
        const float xv = xr[kw * (F + 2) + f + kh];
        const float4 wv = *reinterpret_cast<const float4*>(ws + (kh * 3 + kw) * Co + c4);
        acc.x += wv.x * xv;
        acc.y += wv.y * xv;
        acc.z += wv.z * xv;
        acc.w += wv.w * xv;
      }
    *reinterpret_cast<float4*>(z + (row0 + (F + 2) + f + 1) * Co + c4) = acc;
  }
}

// The same stencil from the raw features xs [B][T][F] (f32, contiguous rows)
// instead of channel 0 of the padded operand: a work-group takes C1_FT frames
// of one utterance, stages their C1_FT + 2 input rows with a zero halo (each
// value rounded to bf16 first when round_bf16, exactly as the bf16 operand the
// weight-gradient GEMM reads), and each thread keeps the 9 taps of its 4
// output channels in registers (its channel group is fixed: CT % (Co / 4) == 0).
// One wave writes 4 pixels x 64 channels = 1 KB of contiguous z per store.
constexpr int C1_FT = 4;

template <typename TZ>
__global__ void __launch_bounds__(CT) conv3x3_c1_fwd_xs(const float* __restrict__ xs, int T,
                                                        int F, int Co, int round_bf16,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ bias,
                                                        TZ* __restrict__ z) {
  extern __shared__ float sm[];
  float* xr = sm;                    // [C1_FT + 2][F + 2], zero halo
  const int ntile = (T + C1_FT - 1) / C1_FT;
  const int b = blockIdx.x / ntile, t0 = (blockIdx.x - b * ntile) * C1_FT;
  const int W = F + 2;
  for (int i = threadIdx.x; i < (C1_FT + 2) * W; i += CT) {
    const int r = i / W, fp = i - r * W;
    const int t = t0 - 1 + r, f = fp - 1;
    float v = 0.f;
    if (t >= 0 && t < T && f >= 0 && f < F) {
      v = xs[((long long)b * T + t) * F + f];
      if (round_bf16) v = bf2f(f2bf(v));
    }
    xr[i] = v;
  }
  const int ng = Co >> 2;
  const int c4 = 4 * (threadIdx.x % ng);
  float4 wr[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {   // torch weight [Co][1][3 (f)][3 (t)], tap = kh * 3 + kw
    wr[tap].x = w[(c4 + 0) * 9 + tap];
    wr[tap].y = w[(c4 + 1) * 9 + tap];
    wr[tap].z = w[(c4 + 2) * 9 + tap];
    wr[tap].w = w[(c4 + 3) * 9 + tap];
  }
  const float4 b4 = bias ? *reinterpret_cast<const float4*>(bias + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  const int nt = min(C1_FT, T - t0);
  const int ppi = CT / ng;           // pixels per iteration
  for (int q = threadIdx.x / ng; q < nt * F; q += ppi) {
    const int r = q / F, f = q - r * F;
    float4 acc = b4;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        // z[p] += w[co][kh][kw] x[p + (kw - 1)(F + 2) + (kh - 1)]
        const float xv = xr[(r + kw) * W + f + kh];
        const float4 wv = wr[kh * 3 + kw];
        acc.x += wv.x * xv;
        acc.y += wv.y * xv;
        acc.z += wv.z * xv;
        acc.w += wv.w * xv;
      }
    const long long p = ((long long)b * (T + 2) + t0 + r + 1) * W + f + 1;
    if constexpr (sizeof(TZ) == 2) {   // bf16 z: one 8-B store
      uint2 o;
      o.x = (unsigned)f2bf(acc.x) | ((unsigned)f2bf(acc.y) << 16);
      o.y = (unsigned)f2bf(acc.z) | ((unsigned)f2bf(acc.w) << 16);
      *reinterpret_cast<uint2*>(z + p * Co + c4) = o;
    } else {
      *reinterpret_cast<float4*>(z + p * Co + c4) = acc;
    }
  }
}

// The same stencil with the next element-wise pass folded in, for an unpooled
// layer followed by batch norm (vgg_hier's first layer): P = max(0, bf16(z))
// written bf16 to the flat [B][T][F][Co] layout -- the value post_fwd would
// store from the bf16 z -- and, with mpart / qpart, the batch-norm moment
// partials of P - shift per block ([block][Co], a lane's four channels summed
// in registers, the block's lanes combined in lane order).  z is never
// written or read back.  ft time rows per block (so the partial count stays
// near 1024).
__global__ void __launch_bounds__(CT) conv3x3_c1_fwd_relu_p(
    const float* __restrict__ xs, int T, int F, int Co, int round_bf16, int ft,
    const float* __restrict__ w, const float* __restrict__ bias, uint16_t* __restrict__ P,
    const float* __restrict__ shift, float* __restrict__ mpart, float* __restrict__ qpart) {
  extern __shared__ float sm[];
  __shared__ float red[CT * 4];
  float* xr = sm;                    // [ft + 2][F + 2], zero halo
  const int ntile = (T + ft - 1) / ft;
  const int b = blockIdx.x / ntile, t0 = (blockIdx.x - b * ntile) * ft;
  const int W = F + 2;
  for (int i = threadIdx.x; i < (ft + 2) * W; i += CT) {
    const int r = i / W, fp = i - r * W;
    const int t = t0 - 1 + r, f = fp - 1;
    float v = 0.f;
    if (t >= 0 && t < T && f >= 0 && f < F) {
      v = xs[((long long)b * T + t) * F + f];
      if (round_bf16) v = bf2f(f2bf(v));
    }
    xr[i] = v;
  }
  const int ng = Co >> 2;
  const int c4 = 4 * (threadIdx.x % ng);
  float4 wr[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    wr[tap].x = w[(c4 + 0) * 9 + tap];
    wr[tap].y = w[(c4 + 1) * 9 + tap];
    wr[tap].z = w[(c4 + 2) * 9 + tap];
    wr[tap].w = w[(c4 + 3) * 9 + tap];
  }
  const float4 b4 = bias ? *reinterpret_cast<const float4*>(bias + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
  float sh[4] = {0.f, 0.f, 0.f, 0.f}, macc[4] = {0.f, 0.f, 0.f, 0.f}, qacc[4] = {0.f, 0.f, 0.f, 0.f};
  if (mpart && shift) {
#pragma unroll
    for (int j = 0; j < 4; ++j) sh[j] = shift[c4 + j];
  }
  __syncthreads();
  const int nt = min(ft, T - t0);
  const int ppi = CT / ng;
  for (int q = threadIdx.x / ng; q < nt * F; q += ppi) {
    const int r = q / F, f = q - r * F;
    float4 acc = b4;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const float xv = xr[(r + kw) * W + f + kh];
        const float4 wv = wr[kh * 3 + kw];
        acc.x += wv.x * xv;
        acc.y += wv.y * xv;
        acc.z += wv.z * xv;
        acc.w += wv.w * xv;
      }
    const uint16_t h[4] = {f2bf(acc.x), f2bf(acc.y), f2bf(acc.z), f2bf(acc.w)};
    float pv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pv[j] = fmaxf(bf2f(h[j]), 0.f);   // exact: a bf16 value or 0
      const float d = pv[j] - sh[j];
      macc[j] += d;
      qacc[j] += d * d;
    }
    uint2 o;
    o.x = (unsigned)f2bf(pv[0]) | ((unsigned)f2bf(pv[1]) << 16);
    o.y = (unsigned)f2bf(pv[2]) | ((unsigned)f2bf(pv[3]) << 16);
    *reinterpret_cast<uint2*>(P + (((long long)b * T + t0 + r) * F + f) * Co + c4) = o;
  }
  if (mpart) {   // lanes tid, tid + ng, ... hold the same four channels
    auto reduce = [&](const float (&acc)[4], float* out) {
      const int tid = threadIdx.x;
#pragma unroll
      for (int j = 0; j < 4; ++j) red[tid * 4 + j] = acc[j];
      __syncthreads();
      for (int cc = tid; cc < Co; cc += CT) {
        const int g2 = cc >> 2, j = cc & 3;
        float t = 0.f;
        for (int k = g2; k < CT; k += ng) t += red[k * 4 + j];
        out[cc] = t;
      }
      __syncthreads();
    };
    reduce(macc, mpart + (long long)blockIdx.x * Co);
    if (qpart) reduce(qacc, qpart + (long long)blockIdx.x * Co);
  }
}

// dx[p][ci] = sum_{co,kh,kw} dz[p - shift][co] w[co][ci][kh][kw] (dz halo rows zero)
__global__ void conv_direct_dgrad(const float* __restrict__ dz, int B, int T, int F, int Ci,
                                  int Co, const float* __restrict__ w, float* __restrict__ dx) {
  const long long n = (long long)B * T * F * Ci;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % Ci);
    const long long pix = i / Ci;
    const int f = (int)(pix % F);
    const int t = (int)((pix / F) % T);
    const int b = (int)(pix / ((long long)F * T));
    const long long p = pad_row(b, t, f, T, F);
    float s = 0.f;
    for (int co = 0; co < Co; ++co) {
      const float* wr = w + ((long long)co * Ci + ci) * 9;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
          s += wr[kh * 3 + kw] * dz[(p - (long long)(kw - 1) * (F + 2) - (kh - 1)) * Co + co];
    }
    dx[p * Ci + ci] = s;
  }
}

// partial[chunk][(co*Ci + ci)*9 + kh*3 + kw] = sum over the chunk's valid pixels of
// dz[p][co] x[p + shift][ci]; partial[chunk][Co*Ci*9 + co] = sum dz (bias).
__global__ void conv_direct_wgrad(const float* __restrict__ x, const float* __restrict__ dz,
                                  int B, int T, int F, int Ci, int Co, int pix_per_chunk,
                                  float* __restrict__ partial) {
  const long long npix = (long long)B * T * F;
  const long long p0 = (long long)blockIdx.x * pix_per_chunk;
  const long long p1 = min(npix, p0 + pix_per_chunk);
  const int nw = Co * Ci * 9, nout = nw + Co;
  for (int o = threadIdx.x; o < nout; o += blockDim.x) {
    const bool isb = o >= nw;
    const int co = isb ? o - nw : o / (Ci * 9);
    const int ci = isb ? 0 : (o / 9) % Ci, tap = isb ? 0 : o % 9;
    const int kh = tap / 3, kw = tap % 3;
    float s = 0.f;
    for (long long q = p0; q < p1; ++q) {
      const int f = (int)(q % F);
      const int t = (int)((q / F) % T);
      const int b = (int)(q / ((long long)F * T));
      const long long p = pad_row(b, t, f, T, F);
      const float g = dz[p * Co + co];
      s += isb ? g : g * x[(p + (long long)(kw - 1) * (F + 2) + (kh - 1)) * Ci + ci];
    }
    partial[(long long)blockIdx.x * nout + o] = s;
  }
}

struct Pool {
  int pt, pf;     // pool size = stride along time / freq (0 = no pooling)
  int To, Fo;     // output extent
};

// Index math of the element-wise passes: 32-bit (the host checks every extent
// fits) and per V-channel group, not per element -- 64-bit division per
// element made these passes ALU-bound (post_bwd 544 us at the first vgg_hier
// layer against ~60 us of traffic).
struct PixIdx {
  int b, to, fo;
};
__device__ __forceinline__ PixIdx pix_of(unsigned q, int To, int Fo) {
  PixIdx p;
  const unsigned r = q / (unsigned)Fo;
  p.fo = (int)(q - r * (unsigned)Fo);
  p.b = (int)(r / (unsigned)To);
  p.to = (int)(r - (unsigned)p.b * (unsigned)To);
  return p;
}

template <int V>
struct VecF;
template <>
struct VecF<1> {
  float v[1];
  __device__ __forceinline__ void load(const float* p) { v[0] = *p; }
  __device__ __forceinline__ void load(const uint16_t* p) { v[0] = bf2f(*p); }
  __device__ __forceinline__ void store(float* p) const { *p = v[0]; }
  __device__ __forceinline__ void store(uint16_t* p) const { *p = f2bf(v[0]); }
};
template <>
struct VecF<4> {
  float v[4];
  __device__ __forceinline__ void load(const float* p) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  }
  __device__ __forceinline__ void load(const uint16_t* p) {   // four bf16 (8-B aligned)
    const uint2 x = *reinterpret_cast<const uint2*>(p);
    v[0] = bf2f((uint16_t)(x.x & 0xffffu)); v[1] = bf2f((uint16_t)(x.x >> 16));
    v[2] = bf2f((uint16_t)(x.y & 0xffffu)); v[3] = bf2f((uint16_t)(x.y >> 16));
  }
  __device__ __forceinline__ void store(float* p) const {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
  __device__ __forceinline__ void store(uint16_t* p) const {   // four bf16 (8-B aligned)
    *reinterpret_cast<uint2*>(p) =
        make_uint2(f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16), f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16));
  }
};
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const uint16_t* p) { return bf2f(*p); }

// P[b][t'][f'][c] = max over the window of relu(z); slot = argmax in torch's
// scan order (freq outer, time inner; first maximum wins).  V channels per
// thread (V = 4 when C % 4 == 0).
// TP = uint16_t (bf16 z only): P = max(0, max z) is a bf16 value, stored exactly.
template <int V, typename TZ = float, typename TP = float>
__global__ void __launch_bounds__(CT) post_fwd(const TZ* __restrict__ z, int B, int T, int F,
                                               int C, Pool pl, TP* __restrict__ P,
                                               uint8_t* __restrict__ slot,
                                               float* __restrict__ mpart,
                                               const float* __restrict__ shift,
                                               float* __restrict__ qpart) {
  // mpart (nullable): per-block column sums of the P values written (the batch
  // norm's mean pass folded in: threads tid, tid + CV, ... hold the same
  // channels; the block's phases are combined in a fixed order).  qpart
  // (nullable, with mpart): the variance pass folded in as well -- mpart then
  // sums P - shift[c] and qpart (P - shift[c])^2, shift being the running mean
  // (a centre close to the batch mean, so E[d^2] - E[d]^2 does not cancel)
  __shared__ float red[CT * V];
  const unsigned CV = (unsigned)(C / V);
  const unsigned n = (unsigned)B * pl.To * pl.Fo * CV;
  float macc[V], qacc[V], sh[V];
  {
    const int c0 = (int)((blockIdx.x * blockDim.x + threadIdx.x) % CV) * V;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      macc[j] = qacc[j] = 0.f;
      sh[j] = qpart ? shift[c0 + j] : 0.f;
    }
  }
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const unsigned q = e / CV;
    const int c = (int)(e - q * CV) * V;
    const PixIdx px = pix_of(q, pl.To, pl.Fo);
    const long long i = (long long)q * C + c;
    VecF<V> best;
    if (!pl.pt) {
      best.load(z + pad_row(px.b, px.to, px.fo, T, F) * C + c);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        best.v[j] = fmaxf(best.v[j], 0.f);
        const float d = best.v[j] - sh[j];
        macc[j] += d;
        qacc[j] += d * d;
      }
      best.store(P + i);
      continue;
    }
    int bs[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      best.v[j] = -__builtin_huge_valf();
      bs[j] = 0;
    }
    for (int df = 0; df < pl.pf; ++df) {
      const int f = px.fo * pl.pf + df;
      if (f >= F) break;
      for (int dt = 0; dt < pl.pt; ++dt) {
        const int t = px.to * pl.pt + dt;
        if (t >= T) break;
        VecF<V> x;
        x.load(z + pad_row(px.b, t, f, T, F) * C + c);
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float v = fmaxf(x.v[j], 0.f);
          if (v > best.v[j]) { best.v[j] = v; bs[j] = df * pl.pt + dt; }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float d = best.v[j] - sh[j];
      macc[j] += d;
      qacc[j] += d * d;
    }
    best.store(P + i);
#pragma unroll
    for (int j = 0; j < V; ++j) slot[i + j] = (uint8_t)bs[j];
  }
  if (mpart) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < V; ++j) red[tid * V + j] = macc[j];
    __syncthreads();
    for (int cc = tid; cc < C; cc += CT) {
      const int g2 = cc / V, j = cc % V;
      float t = 0.f;
      for (int k = g2; k < CT; k += (int)CV) t += red[k * V + j];
      mpart[(long long)blockIdx.x * C + cc] = t;
    }
    if (qpart) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < V; ++j) red[tid * V + j] = qacc[j];
      __syncthreads();
      for (int cc = tid; cc < C; cc += CT) {
        const int g2 = cc / V, j = cc % V;
        float t = 0.f;
        for (int k = g2; k < CT; k += (int)CV) t += red[k * V + j];
        qpart[(long long)blockIdx.x * C + cc] = t;
      }
    }
  }
}

// Column statistics of X [n][C] in fixed chunk order: partial[chunk][c] =
// sum over the chunk's rows of (x - shift[c]) (shift = nullptr: 0) or of its
// square.  The block's threads split the rows into CT / C interleaved phases
// (C divides CT), four accumulators each; phases combine in LDS in order.
template <typename TP = float>
__global__ void __launch_bounds__(CT) col_moment(const TP* __restrict__ X, long long n, int C,
                                                 long long rows_per,
                                                 const float* __restrict__ shift, int square,
                                                 float* __restrict__ partial) {
  __shared__ float red[CT];
  const long long r0 = (long long)blockIdx.x * rows_per;
  const long long r1 = min(n, r0 + rows_per);
  const int tid = threadIdx.x;
  const int ph = CT / C, c = tid % C, q = tid / C;
  float acc = 0.f;
  if (q < ph) {
    const float m = shift ? shift[c] : 0.f;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    long long r = r0 + q;
    for (; r + 3 * ph < r1; r += 4 * ph) {
      const float d0 = ld1(X + r * C + c) - m, d1 = ld1(X + (r + ph) * C + c) - m;
      const float d2 = ld1(X + (r + 2 * ph) * C + c) - m, d3 = ld1(X + (r + 3 * ph) * C + c) - m;
      s0 += square ? d0 * d0 : d0;
      s1 += square ? d1 * d1 : d1;
      s2 += square ? d2 * d2 : d2;
      s3 += square ? d3 * d3 : d3;
    }
    for (; r < r1; r += ph) {
      const float d = ld1(X + r * C + c) - m;
      s0 += square ? d * d : d;
    }
    acc = (s0 + s1) + (s2 + s3);
  }
  red[tid] = acc;
  __syncthreads();
  if (tid < C) {
    float t = 0.f;
    for (int j = 0; j < ph; ++j) t += red[j * C + tid];
    partial[(long long)blockIdx.x * C + tid] = t;
  }
}

// out[c] = scale * sum_q partial[q][c], fixed order: 16 columns per block, 16
// interleaved phases per column (each summing every 16th partial into four
// accumulators), phases combined in order through LDS.  (With 64 columns x 4
// phases per block a 128-channel layer ran 2-4 blocks of 256-long dependent
// chains: 35 us per call for a 0.5 MB read.)
constexpr int SP_COLS = 16;
__global__ void __launch_bounds__(CT) sum_partials(const float* __restrict__ partial, int nchunk,
                                                   int C, float scale, float* __restrict__ out) {
  __shared__ float red[CT];
  const int tid = threadIdx.x;
  const int cl = tid % SP_COLS, q0 = tid / SP_COLS;
  constexpr int NPH = CT / SP_COLS;
  const int c = blockIdx.x * SP_COLS + cl;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < C) {
    int q = q0;
    for (; q + 3 * NPH < nchunk; q += 4 * NPH) {
      s0 += partial[(long long)q * C + c];
      s1 += partial[(long long)(q + NPH) * C + c];
      s2 += partial[(long long)(q + 2 * NPH) * C + c];
      s3 += partial[(long long)(q + 3 * NPH) * C + c];
    }
    for (; q < nchunk; q += NPH) s0 += partial[(long long)q * C + c];
  }
  red[tid] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (q0 == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < NPH; ++j) t += red[j * SP_COLS + cl];
    out[c] = t * scale;
  }
}

// mean -> (mean, rstd) from the centred second moment; running stats update
// (momentum, unbiased variance) as nn.BatchNorm2d in training mode.
__global__ void bn_finalize(const float* __restrict__ mean, const float* __restrict__ m2,
                            int C, long long n, float eps, float momentum,
                            float* __restrict__ rstd, float* __restrict__ run_mean,
                            float* __restrict__ run_var) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float var = m2[c];   // biased (already / n)
  rstd[c] = rsqrtf(var + eps);
  if (run_mean) {
    const float unb = n > 1 ? var * ((float)n / (float)(n - 1)) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean[c];
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
  }
}

// the folded form: mean = shift + E[d], biased var = E[d^2] - E[d]^2 (d = x -
// shift, both moments already / n); mean is written in place of E[d]
__global__ void bn_finalize_shift(float* __restrict__ mean, const float* __restrict__ m2,
                                  const float* shift, int C, long long n, float eps,
                                  float momentum, float* __restrict__ rstd,
                                  float* run_mean, float* __restrict__ run_var) {
  // (shift is normally run_mean itself: each thread reads its entry first)
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float d = mean[c];
  const float var = fmaxf(m2[c] - d * d, 0.f);
  const float mu = shift[c] + d;
  mean[c] = mu;
  rstd[c] = rsqrtf(var + eps);
  if (run_mean) {
    const float unb = n > 1 ? var * ((float)n / (float)(n - 1)) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mu;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
  }
}

__global__ void bn_eval_stats(const float* __restrict__ run_mean, const float* __restrict__ run_var,
                              int C, float eps, float* __restrict__ mean, float* __restrict__ rstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = run_mean[c];
  rstd[c] = rsqrtf(run_var[c] + eps);
}

struct Affine {
  const float* mean;    // nullable: no BN
  const float* rstd;
  const float* gamma;
  const float* beta;
  float drop;
  unsigned long long seed;
};

// y = dropout(BN(P)); written to the next layer's padded input (bf16 / f32,
// halo untouched: the caller zeroes it) or, out_flat, to [B][T'][F'][C].
template <typename TO, int V, typename TP = float>
__global__ void apply_fwd(const TP* __restrict__ P, int B, int To, int Fo, int C, Affine af,
                          TO* __restrict__ out, int flat) {
  const unsigned CV = (unsigned)(C / V);
  const unsigned n = (unsigned)B * To * Fo * CV;
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const unsigned q = e / CV;
    const int c = (int)(e - q * CV) * V;
    const long long i = (long long)q * C + c;
    VecF<V> y;
    y.load(P + i);
    if (af.mean) {
      VecF<V> m, r, g, bt;
      m.load(af.mean + c);
      r.load(af.rstd + c);
      g.load(af.gamma + c);
      bt.load(af.beta + c);
#pragma unroll
      for (int j = 0; j < V; ++j) y.v[j] = (y.v[j] - m.v[j]) * r.v[j] * g.v[j] + bt.v[j];
    }
    if (af.drop > 0.f) {
#pragma unroll
      for (int j = 0; j < V; ++j) y.v[j] *= drop_scale(af.drop, af.seed, (unsigned long long)(i + j));
    }
    long long o = i;
    if (!flat) {
      const PixIdx px = pix_of(q, To, Fo);
      o = pad_row(px.b, px.to, px.fo, To, Fo) * C + c;
    }
    if constexpr (sizeof(TO) == 2 && V == 4) {   // one 8-B store of four bf16
      const unsigned lo = f2bf(y.v[0]) | ((unsigned)f2bf(y.v[1]) << 16);
      const unsigned hi = f2bf(y.v[2]) | ((unsigned)f2bf(y.v[3]) << 16);
      *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + o) = make_uint2(lo, hi);
    } else if constexpr (sizeof(TO) == 2) {
#pragma unroll
      for (int j = 0; j < V; ++j) out[o + j] = f2bf(y.v[j]);
    } else {
      y.store(reinterpret_cast<float*>(out) + o);
    }
  }
}

// dy (after the dropout mask) of the V elements at (pooled pixel q, channel c),
// from the next layer's dX (padded rows, flat = 0) or the encoder's gradient
// [B][T'][F'][C] (flat = 1).
template <int V, typename TD = float>
__device__ __forceinline__ VecF<V> dy_at(const TD* __restrict__ dnext, unsigned q, int c,
                                         int To, int Fo, int C, int flat, float drop,
                                         unsigned long long seed) {
  const long long i = (long long)q * C + c;
  long long o = i;
  if (!flat) {
    const PixIdx px = pix_of(q, To, Fo);
    o = pad_row(px.b, px.to, px.fo, To, Fo) * C + c;
  }
  VecF<V> g;
  g.load(dnext + o);
  if (drop > 0.f) {
#pragma unroll
    for (int j = 0; j < V; ++j) g.v[j] *= drop_scale(drop, seed, (unsigned long long)(i + j));
  }
  return g;
}

// partial[chunk][c] = sum dy, partial[chunk][C + c] = sum dy * xhat over the
// chunk's rows: thread (channel group, row phase), V channels per thread,
// row phases combined in LDS in order
template <int V, typename TD = float, typename TP = float>
__global__ void __launch_bounds__(CT) bn_bwd_moments(const TD* __restrict__ dnext,
                                                     const TP* __restrict__ P, int B, int To,
                                                     int Fo, int C, int flat, Affine af,
                                                     long long rows_per,
                                                     float* __restrict__ partial) {
  __shared__ float red[2 * CT * V];
  const long long n = (long long)B * To * Fo;
  const long long r0 = (long long)blockIdx.x * rows_per;
  const long long r1 = min(n, r0 + rows_per);
  const int tid = threadIdx.x;
  const int CV = C / V, ph = CT / CV, cg = tid % CV, q = tid / CV, c = cg * V;
  float s1[V], s2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) s1[j] = s2[j] = 0.f;
  if (q < ph) {
    float m[V], rs[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      m[j] = af.mean[c + j];
      rs[j] = af.rstd[c + j];
    }
    for (long long r = r0 + q; r < r1; r += ph) {
      const VecF<V> g = dy_at<V>(dnext, (unsigned)r, c, To, Fo, C, flat, af.drop, af.seed);
      VecF<V> x;
      x.load(P + r * C + c);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        s1[j] += g.v[j];
        s2[j] += g.v[j] * (x.v[j] - m[j]) * rs[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    red[(q * CV + cg) * V + j] = s1[j];          // == red[q * C + c + j]
    red[CT * V + (q * CV + cg) * V + j] = s2[j];
  }
  __syncthreads();
  for (int cc = tid; cc < C; cc += CT) {
    float t1 = 0.f, t2 = 0.f;
    for (int jq = 0; jq < ph; ++jq) {
      t1 += red[jq * C + cc];
      t2 += red[CT * V + jq * C + cc];
    }
    partial[((long long)blockIdx.x * 2) * C + cc] = t1;
    partial[((long long)blockIdx.x * 2 + 1) * C + cc] = t2;
  }
}

// sums [2C] (sum dy, sum dy xhat) -> dgamma += sum dy xhat, dbeta += sum dy
__global__ void bn_bwd_finalize(const float* __restrict__ sums, int C, float* __restrict__ dgamma,
                                float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (dgamma) dgamma[c] += sums[C + c];
  if (dbeta) dbeta[c] += sums[c];
}

// dP = BN backward (or dy without BN); routed to the pooled-from pixel if its
// conv output was positive (ReLU), written into dZ [padded pixels][C] (TO).
// bias_part (nullable): per-block column sums of the f32 dZ values, the conv
// bias gradient before its fixed-order sum over blocks -- so dZ itself can be
// a bf16 GEMM operand (C divides the block size: a thread's channels are the
// same in every grid-stride iteration).
template <typename TO, int V, typename TZ = float, typename TP = float>
__global__ void __launch_bounds__(CT) post_bwd(const float* __restrict__ dnext,
                                               const TP* __restrict__ P,
                                               const TZ* __restrict__ z,
                                               const uint8_t* __restrict__ slot, int B, int T,
                                               int F, int C, Pool pl, int flat, Affine af,
                                               const float* __restrict__ sums,
                                               TO* __restrict__ dz,
                                               float* __restrict__ bias_part) {
  __shared__ float red[CT * V];
  const unsigned nr = (unsigned)B * pl.To * pl.Fo;
  const unsigned CV = (unsigned)(C / V);
  const unsigned n = nr * CV;
  const float inv_n = 1.f / (float)nr;
  float bacc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) bacc[j] = 0.f;
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const unsigned q = e / CV;
    const int c = (int)(e - q * CV) * V;
    const long long i = (long long)q * C + c;
    VecF<V> g = dy_at<V>(dnext, q, c, pl.To, pl.Fo, C, flat, af.drop, af.seed);
    if (af.mean) {
      VecF<V> x, m, r, gm, s1, s2;
      x.load(P + i);
      m.load(af.mean + c);
      r.load(af.rstd + c);
      gm.load(af.gamma + c);
      s1.load(sums + c);
      s2.load(sums + C + c);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float xh = (x.v[j] - m.v[j]) * r.v[j];
        g.v[j] = gm.v[j] * r.v[j] * (g.v[j] - s1.v[j] * inv_n - xh * s2.v[j] * inv_n);
      }
    }
    const PixIdx px = pix_of(q, pl.To, pl.Fo);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      int t = px.to, f = px.fo;
      if (pl.pt) {
        const int sl = slot[i + j];
        t = px.to * pl.pt + sl % pl.pt;
        f = px.fo * pl.pf + sl / pl.pt;
      }
      const long long p = pad_row(px.b, t, f, T, F) * C + c + j;
      float zp;
      if constexpr (sizeof(TZ) == 2) zp = bf2f(z[p]);
      else zp = z[p];
      const float v = zp > 0.f ? g.v[j] : 0.f;
      bacc[j] += v;
      if constexpr (sizeof(TO) == 2) dz[p] = f2bf(v);
      else dz[p] = v;
    }
  }
  if (bias_part) {   // threads tid, tid + CV, ... hold the same channels
    const int tid = threadIdx.x, cg = tid % (int)CV;
#pragma unroll
    for (int j = 0; j < V; ++j) red[tid * V + j] = bacc[j];
    __syncthreads();
    for (int cc = tid; cc < C; cc += CT) {
      const int g2 = cc / V, j = cc % V;
      float t = 0.f;
      for (int k = g2; k < CT; k += (int)CV) t += red[k * V + j];
      bias_part[(long long)blockIdx.x * C + cc] = t;
    }
    (void)cg;
  }
}

// post_bwd over the full-resolution pixels: thread (pixel, 4 channels) finds
// its pool window, takes the window's gradient (BN backward applied) where
// the pixel was the window's argmax and z > 0, and writes dz for EVERY pixel
// as one 8-B (bf16) / 16-B store next to one 16-B z load.  post_bwd instead
// walked the pooled elements and gathered z / scattered dz one channel at a
// time (554 us at the first pooled vgg_hier layer).  The window's gradient is
// recomputed by each of its pixels (dnext / P / slot are a quarter of z's
// size and come from the cache).  Bias partials as in post_bwd.
template <typename TO, typename TZ = float, typename TD = float, typename TP = float>
__global__ void __launch_bounds__(CT) post_bwd_full(const TD* __restrict__ dnext,
                                                    const TP* __restrict__ P,
                                                    const TZ* __restrict__ z,
                                                    const uint8_t* __restrict__ slot, int B, int T,
                                                    int F, int C, Pool pl, int flat, Affine af,
                                                    const float* __restrict__ sums,
                                                    TO* __restrict__ dz,
                                                    float* __restrict__ bias_part) {
  constexpr int V = 4;
  __shared__ float red[CT * V];
  const unsigned nr = (unsigned)B * pl.To * pl.Fo;
  const unsigned CV = (unsigned)(C / V);
  const unsigned n = (unsigned)B * T * F * CV;
  const float inv_n = 1.f / (float)nr;
  float bacc[V] = {0.f, 0.f, 0.f, 0.f};
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const unsigned q = e / CV;
    const int c = (int)(e - q * CV) * V;
    const PixIdx px = pix_of(q, T, F);            // (b, t, f) at full resolution
    int to = px.to, fo = px.fo;
    bool in = true;
    if (pl.pt) {
      to = px.to / pl.pt;
      fo = px.fo / pl.pf;
      in = to < pl.To && fo < pl.Fo;
    }
    const long long p = pad_row(px.b, px.to, px.fo, T, F) * C + c;
    float v[V] = {0.f, 0.f, 0.f, 0.f};
    if (in) {
      const unsigned qp = ((unsigned)px.b * pl.To + to) * pl.Fo + fo;
      const long long ip = (long long)qp * C + c;
      VecF<V> g = dy_at<V>(dnext, qp, c, pl.To, pl.Fo, C, flat, af.drop, af.seed);
      VecF<V> x;   // the pooled pre-BN value (read when BN or the pool needs it)
      if (af.mean || pl.pt) x.load(P + ip);
      if (af.mean) {
        VecF<V> m, r, gm, s1, s2;
        m.load(af.mean + c);
        r.load(af.rstd + c);
        gm.load(af.gamma + c);
        s1.load(sums + c);
        s2.load(sums + C + c);
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float xh = (x.v[j] - m.v[j]) * r.v[j];
          g.v[j] = gm.v[j] * r.v[j] * (g.v[j] - s1.v[j] * inv_n - xh * s2.v[j] * inv_n);
        }
      }
      // ReLU mask: z > 0 at the window's argmax pixel <=> the pooled value
      // P = max(0, max z) > 0 there, so pooled layers read P (a quarter of the
      // bytes, already loaded for BN) instead of the full-resolution z; an
      // unpooled layer's P = max(0, z) is loaded for BN and gives the same mask
      VecF<V> zv;
      if (pl.pt || af.mean) zv = x;
      else zv.load(z + p);
      unsigned sl = 0u, me = 0u;
      if (pl.pt) {
        sl = *reinterpret_cast<const unsigned*>(slot + ip);   // four channels' argmax slots
        me = (unsigned)((px.fo - fo * pl.pf) * pl.pt + (px.to - to * pl.pt));
      }
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const bool hit = !pl.pt || ((sl >> (8 * j)) & 0xffu) == me;
        v[j] = (hit && zv.v[j] > 0.f) ? g.v[j] : 0.f;
        bacc[j] += v[j];
      }
    }
    if constexpr (sizeof(TO) == 2) {
      uint2 o;
      o.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
      o.y = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
      *reinterpret_cast<uint2*>(dz + p) = o;
    } else {
      *reinterpret_cast<float4*>(dz + p) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  if (bias_part) {   // threads tid, tid + CV, ... hold the same channels
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < V; ++j) red[tid * V + j] = bacc[j];
    __syncthreads();
    for (int cc = tid; cc < C; cc += CT) {
      const int g2 = cc / V, j = cc % V;
      float t = 0.f;
      for (int k = g2; k < CT; k += (int)CV) t += red[k * V + j];
      bias_part[(long long)blockIdx.x * C + cc] = t;
    }
  }
}

// ---------------------------------------------------------------------------
// Row-blocked forms of the bf16 element-wise passes (z / P / dz bf16, C % 8 ==
// 0 and C / 8 dividing 256, no pooling or 2 x 2 pooling).  A block owns
// consecutive image rows (b, t) of the pass's grid; within a row the pixels x C
// channels are contiguous in every operand -- flat rows and the interior of
// padded rows alike -- so lane l covers 8 channels (one 16-B access) of pixel
// g / (C / 8) for g = l, l + 256, ...: no per-element index division (the
// grid-stride forms above spent two to three 32-bit divisions per 8-B access
// and ran the 64-channel vgg_hier layer at 2.4-3.6 TB/s), and a lane's
// channels are the same in every row (256 is a multiple of C / 8), so the
// per-channel parameters and partial sums live in its registers.  Partial sums
// are combined per block in a fixed order (lanes of a channel group in lane
// order) and across blocks by sum_partials: run-to-run deterministic.
// ---------------------------------------------------------------------------
constexpr int RW_NT = 256;

struct Bf8 {
  float v[8];
  __device__ __forceinline__ void load(const uint16_t* p) {
    const uint4 x = *reinterpret_cast<const uint4*>(p);
    const unsigned w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = bf2f((uint16_t)(w[k] & 0xffffu));
      v[2 * k + 1] = bf2f((uint16_t)(w[k] >> 16));
    }
  }
  __device__ __forceinline__ void load(const float* p) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ void store(uint16_t* p) const {
    uint4 x;
    x.x = f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
    x.y = f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
    x.z = f2bf(v[4]) | ((unsigned)f2bf(v[5]) << 16);
    x.w = f2bf(v[6]) | ((unsigned)f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(p) = x;
  }
  __device__ __forceinline__ void store(float* p) const {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// element offset of pixel (b, t, 0) of a [B][T][F] grid: flat rows, or the
// first interior pixel of padded rows [B][T+2][F+2]
__device__ __forceinline__ long long row_base(int b, int t, int T, int F, int C, int flat) {
  return flat ? ((long long)b * T + t) * F * C
              : (((long long)b * (T + 2) + t + 1) * (F + 2) + 1) * C;
}

// A block's rows [r0, r1) of a grid with Tr rows per utterance, walked as one
// flat sequence of 8-channel groups: lane l takes group l, then every 256th --
// across row ends (rows of a 2 x 2-pooled 128-channel layer hold 320 groups:
// per-row loops left most lanes idle in each row's tail).  ng % (C / 8) == 0
// and 256 % (C / 8) == 0 keep a lane's channels fixed.
struct RowWalk {
  int r, b, t, g;
  __device__ __forceinline__ RowWalk() {}
  // goff: this walker's first group beyond the lane's (U walkers per lane keep
  // U 16-B loads in flight: with one, a lane's load -> use -> store chain left
  // the passes at ~3.3 TB/s)
  __device__ __forceinline__ RowWalk(int r0, int r1, int Tr, int ng, int goff = 0) {
    r = r0;
    b = r0 / Tr;
    t = r0 - b * Tr;
    g = threadIdx.x + goff;
    settle(r1, Tr, ng);
  }
  __device__ __forceinline__ void settle(int r1, int Tr, int ng) {
    while (g >= ng && r < r1) {
      g -= ng;
      ++r;
      if (++t == Tr) { t = 0; ++b; }
    }
  }
  __device__ __forceinline__ void next(int r1, int Tr, int ng, int stride = RW_NT) {
    g += stride;
    settle(r1, Tr, ng);
  }
};
// walkers per lane: 1.  Four (2 for the pooled forward and the backward)
// measured slower at vgg_hier (kernel trace, same build otherwise: rw_apply
// 116 -> 145 us, rw_bn_moments 116 -> 137, rw_post_bwd<0> 158 -> 185) and no
// faster elsewhere, so the walker arrays stay at one element.
constexpr int RW_U = 1;

// lanes with the same channel group (tid % cg8) hold partial sums of the same
// 8 channels: out[c] = their sum in lane order (c < C)
__device__ __forceinline__ void rw_reduce(const float (&acc)[8], int cg8, int C, float* red,
                                          float* __restrict__ out) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[tid * 8 + j] = acc[j];
  __syncthreads();
  for (int cc = tid; cc < C; cc += RW_NT) {
    const int g = cc >> 3, j = cc & 7;
    float t = 0.f;
    for (int k = g; k < RW_NT; k += cg8) t += red[k * 8 + j];
    out[cc] = t;
  }
  __syncthreads();
}

// y = dropout(BN(P)) row by row into the next layer's padded input (bf16) or
// the flat f32 encoder input; the same arithmetic as apply_fwd.
template <typename TO>
__global__ void __launch_bounds__(RW_NT) rw_apply(const uint16_t* __restrict__ P, int B, int To,
                                                  int Fo, int C, Affine af, TO* __restrict__ out,
                                                  int flat, int rpb) {
  const int tid = threadIdx.x, cg8 = C >> 3;
  const int c = (tid & (cg8 - 1)) * 8;
  float m[8], r[8], g[8], bt[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[j] = af.mean ? af.mean[c + j] : 0.f;
    r[j] = af.mean ? af.rstd[c + j] : 0.f;
    g[j] = af.mean ? af.gamma[c + j] : 0.f;
    bt[j] = af.mean ? af.beta[c + j] : 0.f;
  }
  const int rows = B * To, ng = Fo * cg8;
  const int r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  RowWalk it[RW_U];
#pragma unroll
  for (int u = 0; u < RW_U; ++u) it[u] = RowWalk(r0, r1, To, ng, u * RW_NT);
  while (it[0].r < r1) {   // walker 0 trails the others
    Bf8 y[RW_U];
    long long pe[RW_U];
#pragma unroll
    for (int u = 0; u < RW_U; ++u) {
      pe[u] = (long long)it[u].r * Fo * C + (long long)it[u].g * 8;
      if (it[u].r < r1) y[u].load(P + pe[u]);
    }
#pragma unroll
    for (int u = 0; u < RW_U; ++u) {
      if (it[u].r >= r1) continue;
      if (af.mean) {
#pragma unroll
        for (int j = 0; j < 8; ++j) y[u].v[j] = (y[u].v[j] - m[j]) * r[j] * g[j] + bt[j];
      }
      if (af.drop > 0.f) {
        drop_n_aligned<8>(y[u].v, af.drop, af.seed, (unsigned long long)pe[u]);
      }
      y[u].store(out + row_base(it[u].b, it[u].t, To, Fo, C, flat) + (long long)it[u].g * 8);
      it[u].next(r1, To, ng, RW_U * RW_NT);
    }
  }
}

// ReLU (+ 2 x 2 max pool, PL = 2) of bf16 z rows into bf16 P (+ slot), with the
// batch-norm moment partials of P - shift (mpart, qpart: [block][C]; qpart
// nullable).  The same window scan as post_fwd (freq outer, time inner, first
// maximum wins).
template <int PL>
__global__ void __launch_bounds__(RW_NT) __attribute__((amdgpu_waves_per_eu(8, 8))) rw_post_fwd(const uint16_t* __restrict__ z, int B, int T,
                                                     int F, int C, Pool pl,
                                                     uint16_t* __restrict__ P,
                                                     uint8_t* __restrict__ slot,
                                                     float* __restrict__ mpart,
                                                     const float* __restrict__ shift,
                                                     float* __restrict__ qpart, int rpb) {
  __shared__ float red[RW_NT * 8];
  const int tid = threadIdx.x, cg8 = C >> 3, sh3 = __builtin_ctz(cg8);
  const int c = (tid & (cg8 - 1)) * 8;
  float sh[8], macc[8], qacc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sh[j] = qpart ? shift[c + j] : 0.f;
    macc[j] = qacc[j] = 0.f;
  }
  const int rows = B * pl.To, ng = pl.Fo * cg8;
  const int r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  constexpr int U = RW_U;   // walkers per lane
  RowWalk it[U];
#pragma unroll
  for (int u = 0; u < U; ++u) it[u] = RowWalk(r0, r1, pl.To, ng, u * RW_NT);
  while (it[0].r < r1) {
    Bf8 best[U];
    unsigned bs[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (it[u].r >= r1) continue;
      const int b = it[u].b, to = it[u].t;
      const int fo = it[u].g >> sh3;
      if constexpr (PL == 0) {
        best[u].load(z + row_base(b, to, T, F, C, 0) + (long long)it[u].g * 8);
      } else {
        // the window's four pixels kept packed (16 B each) until compared:
        // unpacked on load they held 32 VGPRs and the pass ran at 5 waves / SIMD
        uint4 x[4];
#pragma unroll
        for (int df = 0; df < 2; ++df)
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const int f = fo * 2 + df, t = to * 2 + dt;
            x[df * 2 + dt] = uint4{0u, 0u, 0u, 0u};
            if (f < F && t < T)
              x[df * 2 + dt] = *reinterpret_cast<const uint4*>(z + row_base(b, t, T, F, C, 0) +
                                                               (long long)f * C + c);
          }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          best[u].v[j] = -__builtin_huge_valf();
          bs[u][j] = 0u;
        }
#pragma unroll
        for (int df = 0; df < 2; ++df)
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const int f = fo * 2 + df, t = to * 2 + dt;
            if (f < F && t < T) {
              const uint4 w4 = x[df * 2 + dt];
              const unsigned w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const uint16_t hb = (uint16_t)((j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xffffu));
                const float v = fmaxf(bf2f(hb), 0.f);
                if (v > best[u].v[j]) { best[u].v[j] = v; bs[u][j] = (unsigned)(df * 2 + dt); }
              }
            }
          }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {   // in walker order: the moment sums' order is fixed
      if (it[u].r >= r1) continue;
      const long long pe = (long long)it[u].r * pl.Fo * C + (long long)it[u].g * 8;
      if constexpr (PL == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) best[u].v[j] = fmaxf(best[u].v[j], 0.f);
      } else {
        uint2 sl;
        sl.x = bs[u][0] | (bs[u][1] << 8) | (bs[u][2] << 16) | (bs[u][3] << 24);
        sl.y = bs[u][4] | (bs[u][5] << 8) | (bs[u][6] << 16) | (bs[u][7] << 24);
        *reinterpret_cast<uint2*>(slot + pe) = sl;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = best[u].v[j] - sh[j];
        macc[j] += d;
        qacc[j] += d * d;
      }
      best[u].store(P + pe);
      it[u].next(r1, pl.To, ng, U * RW_NT);
    }
  }
  if (mpart) {
    rw_reduce(macc, cg8, C, red, mpart + (long long)blockIdx.x * C);
    if (qpart) rw_reduce(qacc, cg8, C, red, qpart + (long long)blockIdx.x * C);
  }
}

// partial[block][c] = sum dy, partial[block][C + c] = sum dy * xhat (as
// bn_bwd_moments) over the block's rows of the pooled grid
template <typename TD>
__global__ void __launch_bounds__(RW_NT) rw_bn_moments(const TD* __restrict__ dnext,
                                                       const uint16_t* __restrict__ P, int B,
                                                       int To, int Fo, int C, int flat,
                                                       Affine af, float* __restrict__ partial,
                                                       int rpb) {
  __shared__ float red[RW_NT * 8];
  const int tid = threadIdx.x, cg8 = C >> 3;
  const int c = (tid & (cg8 - 1)) * 8;
  float m[8], rs[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[j] = af.mean[c + j];
    rs[j] = af.rstd[c + j];
    s1[j] = s2[j] = 0.f;
  }
  const int rows = B * To, ng = Fo * cg8;
  const int r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  RowWalk it[RW_U];
#pragma unroll
  for (int u = 0; u < RW_U; ++u) it[u] = RowWalk(r0, r1, To, ng, u * RW_NT);
  while (it[0].r < r1) {
    Bf8 gv[RW_U], x[RW_U];
    long long pe[RW_U];
#pragma unroll
    for (int u = 0; u < RW_U; ++u) {
      const long long e = (long long)it[u].g * 8;
      pe[u] = (long long)it[u].r * Fo * C + e;
      if (it[u].r < r1) {
        gv[u].load(dnext + row_base(it[u].b, it[u].t, To, Fo, C, flat) + e);
        x[u].load(P + pe[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < RW_U; ++u) {   // in walker order: the sums' order is fixed
      if (it[u].r >= r1) continue;
      if (af.drop > 0.f) {
        drop_n_aligned<8>(gv[u].v, af.drop, af.seed, (unsigned long long)pe[u]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += gv[u].v[j];
        s2[j] += gv[u].v[j] * (x[u].v[j] - m[j]) * rs[j];
      }
      it[u].next(r1, To, ng, RW_U * RW_NT);
    }
  }
  rw_reduce(s1, cg8, C, red, partial + (long long)blockIdx.x * 2 * C);
  rw_reduce(s2, cg8, C, red, partial + ((long long)blockIdx.x * 2 + 1) * C);
}

// rw_bn_moments with NT threads per work-group and U rows-walkers per lane
// (U 16-B load pairs in flight per lane): the pass reads 1.1 GB per vgg_hier
// step at ~2 TB/s with NT = 256, U = 1 -- its grid is capped by the 1024
// partial rows, so the loads in flight per CU are what it can raise.  Sums in
// walker order, then lane order (deterministic; another association than
// U = 1).  ASR_VGG_BNM=<NT>x<U> selects it (A/B).
template <int NT>
__device__ __forceinline__ void rw_reduce_nt(const float (&acc)[8], int cg8, int C, float* red,
                                             float* __restrict__ out) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[tid * 8 + j] = acc[j];
  __syncthreads();
  for (int cc = tid; cc < C; cc += NT) {
    const int g = cc >> 3, j = cc & 7;
    float t = 0.f;
    for (int k = g; k < NT; k += cg8) t += red[k * 8 + j];
    out[cc] = t;
  }
  __syncthreads();
}
template <typename TD, int NT, int U>
__global__ void __launch_bounds__(NT) rw_bn_moments_nu(const TD* __restrict__ dnext,
                                                       const uint16_t* __restrict__ P, int B,
                                                       int To, int Fo, int C, int flat,
                                                       Affine af, float* __restrict__ partial,
                                                       int rpb) {
  extern __shared__ __attribute__((aligned(16))) float red_nu[];   // [NT * 8]
  const int tid = threadIdx.x, cg8 = C >> 3;
  const int c = (tid & (cg8 - 1)) * 8;
  float m[8], rs[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[j] = af.mean[c + j];
    rs[j] = af.rstd[c + j];
    s1[j] = s2[j] = 0.f;
  }
  const int rows = B * To, ng = Fo * cg8;
  const int r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  RowWalk it[U];
#pragma unroll
  for (int u = 0; u < U; ++u) it[u] = RowWalk(r0, r1, To, ng, u * NT);
  while (it[0].r < r1) {
    Bf8 gv[U], x[U];
    long long pe[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long e = (long long)it[u].g * 8;
      pe[u] = (long long)it[u].r * Fo * C + e;
      if (it[u].r < r1) {
        gv[u].load(dnext + row_base(it[u].b, it[u].t, To, Fo, C, flat) + e);
        x[u].load(P + pe[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (it[u].r >= r1) continue;
      if (af.drop > 0.f) {
        drop_n_aligned<8>(gv[u].v, af.drop, af.seed, (unsigned long long)pe[u]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += gv[u].v[j];
        s2[j] += gv[u].v[j] * (x[u].v[j] - m[j]) * rs[j];
      }
      it[u].next(r1, To, ng, U * NT);
    }
  }
  rw_reduce_nt<NT>(s1, cg8, C, red_nu, partial + (long long)blockIdx.x * 2 * C);
  rw_reduce_nt<NT>(s2, cg8, C, red_nu, partial + ((long long)blockIdx.x * 2 + 1) * C);
}

// dz over full-resolution rows (as post_bwd_full, BN present): each pixel takes
// its window's gradient where it was the argmax (PL = 2) and the pooled /
// unpooled value P > 0 (the ReLU mask); bf16 dz at every interior pixel, the
// conv-bias partials of the f32 values per block (bias_part nullable).
template <int PL, typename TD>
__global__ void __launch_bounds__(RW_NT) __attribute__((amdgpu_waves_per_eu(8, 8))) rw_post_bwd(const TD* __restrict__ dnext,
                                                     const uint16_t* __restrict__ P,
                                                     const uint8_t* __restrict__ slot, int B, int T,
                                                     int F, int C, Pool pl, int flat, Affine af,
                                                     const float* __restrict__ sums,
                                                     uint16_t* __restrict__ dz,
                                                     float* __restrict__ bias_part, int rpb) {
  __shared__ float red[RW_NT * 8];
  // the per-channel batch-norm parameters [5][C] (mean, rstd, gamma, the two
  // BN-backward sums) in LDS, read per group: held in registers they took the
  // kernel to 90 VGPRs, 5 waves per SIMD, for a pass bound by loads in flight
  extern __shared__ __attribute__((aligned(16))) float prm[];
  const int tid = threadIdx.x, cg8 = C >> 3, sh3 = __builtin_ctz(cg8);
  const int c = (tid & (cg8 - 1)) * 8;
  const float inv_n = 1.f / (float)((unsigned)B * pl.To * pl.Fo);
  for (int i = tid; i < C; i += RW_NT) {
    prm[i] = af.mean[i];
    prm[C + i] = af.rstd[i];
    prm[2 * C + i] = af.gamma[i];
    prm[3 * C + i] = sums[i];
    prm[4 * C + i] = sums[C + i];
  }
  float bacc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bacc[j] = 0.f;
  __syncthreads();
  auto ld4 = [&](int k, int h, float (&o)[4]) {
    const float4 a = *reinterpret_cast<const float4*>(&prm[k * C + c + h]);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  };
  const int rows = B * T, ng = F * cg8;
  const int r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  constexpr int U = RW_U;   // walkers per lane
  RowWalk it[U];
#pragma unroll
  for (int u = 0; u < U; ++u) it[u] = RowWalk(r0, r1, T, ng, u * RW_NT);
  while (it[0].r < r1) {
    Bf8 g[U], x[U];
    unsigned long long sl[U];
    bool in[U];
    long long pbi[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = it[u].t, to = PL ? t >> 1 : t;
      const int f = it[u].g >> sh3, fo = PL ? f >> 1 : f;
      in[u] = it[u].r < r1 && to < pl.To && fo < pl.Fo;
      const long long ip = (long long)fo * C + c;
      pbi[u] = ((long long)it[u].b * pl.To + to) * pl.Fo * C + ip;
      sl[u] = 0ull;
      if (in[u]) {
        g[u].load(dnext + row_base(it[u].b, to, pl.To, pl.Fo, C, flat) + ip);
        x[u].load(P + pbi[u]);
        if constexpr (PL != 0) sl[u] = *reinterpret_cast<const unsigned long long*>(slot + pbi[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {   // in walker order: the bias sums' order is fixed
      if (it[u].r >= r1) continue;
      const int t = it[u].t, to = PL ? t >> 1 : t;
      const int f = it[u].g >> sh3, fo = PL ? f >> 1 : f;
      Bf8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v.v[j] = 0.f;
      if (in[u]) {
        if (af.drop > 0.f) {
          drop_n_aligned<8>(g[u].v, af.drop, af.seed, (unsigned long long)pbi[u]);
        }
        const unsigned long long me =
            PL ? (unsigned long long)((f - fo * 2) * 2 + (t - to * 2)) : 0ull;
#pragma unroll
        for (int h = 0; h < 8; h += 4) {   // four channels' parameters live at a time
          float m[4], r[4], gm[4], a1[4], a2[4];
          ld4(0, h, m); ld4(1, h, r); ld4(2, h, gm); ld4(3, h, a1); ld4(4, h, a2);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int j = h + e;
            const float xh = (x[u].v[j] - m[e]) * r[e];
            const float gj = gm[e] * r[e] * (g[u].v[j] - a1[e] * inv_n - xh * a2[e] * inv_n);
            const bool hit = PL == 0 || ((sl[u] >> (8 * j)) & 0xffull) == me;
            v.v[j] = (hit && x[u].v[j] > 0.f) ? gj : 0.f;
            bacc[j] += v.v[j];
          }
        }
      }
      v.store(dz + row_base(it[u].b, t, T, F, C, 0) + (long long)it[u].g * 8);
      it[u].next(r1, T, ng, U * RW_NT);
    }
  }
  if (bias_part) rw_reduce(bacc, cg8, C, red, bias_part + (long long)blockIdx.x * C);
}

// The pooled layers' backward on the POOLED grid (every input pixel inside a
// window: ceil mode or even extents): each group's ReLU / batch-norm backward
// is computed once and scattered to its 2 x 2 window -- the argmax pixel gets
// it, the other three 0 -- where rw_post_bwd<2> walks the input pixels and
// recomputes it (and reloads dnext, P and the slots) for each of the four.
// Same arithmetic per element; the conv-bias sums add the same values in
// another fixed order.
template <typename TD>
__global__ void __launch_bounds__(RW_NT)
    rw_post_bwd_pool(const TD* __restrict__ dnext, const uint16_t* __restrict__ P,
                     const uint8_t* __restrict__ slot, int B, int T, int F, int C, Pool pl,
                     int flat, Affine af, const float* __restrict__ sums,
                     uint16_t* __restrict__ dz, float* __restrict__ bias_part, int rpb) {
  __shared__ float red[RW_NT * 8];
  extern __shared__ __attribute__((aligned(16))) float prm[];   // [5][C], as rw_post_bwd
  const int tid = threadIdx.x, cg8 = C >> 3, sh3 = __builtin_ctz(cg8);
  const int c = (tid & (cg8 - 1)) * 8;
  const float inv_n = 1.f / (float)((unsigned)B * pl.To * pl.Fo);
  for (int i = tid; i < C; i += RW_NT) {
    prm[i] = af.mean[i];
    prm[C + i] = af.rstd[i];
    prm[2 * C + i] = af.gamma[i];
    prm[3 * C + i] = sums[i];
    prm[4 * C + i] = sums[C + i];
  }
  float bacc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bacc[j] = 0.f;
  __syncthreads();
  auto ld4 = [&](int k, int h, float (&o)[4]) {
    const float4 a = *reinterpret_cast<const float4*>(&prm[k * C + c + h]);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  };
  const int rows = B * pl.To, ng = pl.Fo * cg8;
  const int r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  for (RowWalk it(r0, r1, pl.To, ng); it.r < r1; it.next(r1, pl.To, ng)) {
    const int b = it.b, to = it.t, fo = it.g >> sh3;
    const long long ip = (long long)fo * C + c;
    const long long pbi = ((long long)b * pl.To + to) * pl.Fo * C + ip;
    Bf8 g, x;
    g.load(dnext + row_base(b, to, pl.To, pl.Fo, C, flat) + ip);
    x.load(P + pbi);
    const unsigned long long sl = *reinterpret_cast<const unsigned long long*>(slot + pbi);
    if (af.drop > 0.f) drop_n_aligned<8>(g.v, af.drop, af.seed, (unsigned long long)pbi);
    float gj[8];
#pragma unroll
    for (int h = 0; h < 8; h += 4) {
      float m[4], r[4], gm[4], a1[4], a2[4];
      ld4(0, h, m); ld4(1, h, r); ld4(2, h, gm); ld4(3, h, a1); ld4(4, h, a2);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = h + e;
        const float xh = (x.v[j] - m[e]) * r[e];
        const float v = gm[e] * r[e] * (g.v[j] - a1[e] * inv_n - xh * a2[e] * inv_n);
        gj[j] = x.v[j] > 0.f ? v : 0.f;
      }
    }
    // one window pixel at a time (unrolled, the four pixels' values were all
    // live at once: 102 VGPRs, 4 waves per SIMD)
#pragma unroll 1
    for (int w = 0; w < 4; ++w) {
        const int df = w >> 1, dt = w & 1;
        const int f = fo * 2 + df, t = to * 2 + dt;
        if (f < F && t < T) {
          const unsigned long long me = (unsigned long long)w;
          Bf8 v;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            v.v[j] = ((sl >> (8 * j)) & 0xffull) == me ? gj[j] : 0.f;
            bacc[j] += v.v[j];
          }
          v.store(dz + row_base(b, t, T, F, C, 0) + (long long)f * C + c);
        }
      }
  }
  if (bias_part) rw_reduce(bacc, cg8, C, red, bias_part + (long long)blockIdx.x * C);
}

// GEMM weight images of a torch Conv2d weight W [Co][Ci][3(f)][3(t)], tap
// j = kw*3 + kh (the row shift (kw-1)(F+2) + (kh-1) of gemm.hip tap addressing):
//   mode 0 (forward):  out[co][j*Ci + ci] = W[co][ci][kh][kw]
//   mode 1 (d input):  out[ci][j*Co + co] = W[co][ci][kh][kw]
// (Cip >= Ci: the image's input-channel pitch; padded channels are left as the
// caller zeroed them)
template <typename TO>
__global__ void weight_pack(const float* __restrict__ w, int Co, int Ci, int Cip, int mode,
                            TO* __restrict__ out) {
  const long long n = (long long)Co * Ci * 9;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int kw = (int)(i % 3), kh = (int)((i / 3) % 3);
    const int ci = (int)((i / 9) % Ci), co = (int)(i / (9LL * Ci));
    const int j = kw * 3 + kh;
    const long long o = mode == 0 ? ((long long)co * 9 + j) * Cip + ci
                                  : ((long long)ci * 9 + j) * Co + co;
    if constexpr (sizeof(TO) == 2) out[o] = f2bf(w[i]);
    else out[o] = w[i];
  }
}

// dW [Co][Ci][3][3] += packed [Co][9 Ci] (mode-0 image layout)
__global__ void weight_unpack_acc(const float* __restrict__ pk, int Co, int Ci, int Cip,
                                  float* __restrict__ dw) {
  const long long n = (long long)Co * Ci * 9;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int kw = (int)(i % 3), kh = (int)((i / 3) % 3);
    const int ci = (int)((i / 9) % Ci), co = (int)(i / (9LL * Ci));
    dw[i] += pk[((long long)co * 9 + kw * 3 + kh) * Cip + ci];
  }
}

// dW [Co][Ci][3][3] += packed_t [9 Cip][Co] (the transposed mode-0 image)
__global__ void weight_unpack_acc_t(const float* __restrict__ pk, int Co, int Ci, int Cip,
                                    float* __restrict__ dw) {
  const long long n = (long long)Co * Ci * 9;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int kw = (int)(i % 3), kh = (int)((i / 3) % 3);
    const int ci = (int)((i / 9) % Ci), co = (int)(i / (9LL * Ci));
    dw[i] += pk[((long long)(kw * 3 + kh) * Cip + ci) * Co + co];
  }
}

inline int grid_for(long long n) {
  const long long b = (n + CT - 1) / CT;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

inline long long rows_per_chunk(long long n) {
  const long long nchunk = n < 1024 ? 1 : 1024;
  return (n + nchunk - 1) / nchunk;
}

Pool make_pool(int T, int F, int pt, int pf, int ceil_mode) {
  Pool pl{pt, pf, T, F};
  if (pt > 0) {
    auto out = [&](int n, int k) {
      if (!ceil_mode) return (n - k) / k + 1;
      int o = (n - k + k - 1) / k + 1;
      if ((o - 1) * k >= n) --o;   // the last window must start inside the input
      return o;
    };
    pl.To = out(T, pt);
    pl.Fo = out(F, pf);
  }
  return pl;
}

}  // namespace
}  // namespace asr

using namespace asr;

extern "C" int asr_vgg_pad_input_ch(const float* xs, int B, int T, int F, int Cp, int out_dtype,
                                    void* out, void* stream);

extern "C" int asr_vgg_pad_input(const float* xs, int B, int T, int F, float* out, void* stream) {
  return asr_vgg_pad_input_ch(xs, B, T, F, 1, ASR_DT_F32, out, stream);
}

extern "C" int asr_vgg_pad_input_ch(const float* xs, int B, int T, int F, int Cp, int out_dtype,
                                    void* out, void* stream) {
  ASR_REQUIRE(xs && out && B > 0 && T > 0 && F > 0 && Cp > 0, ASR_ERR_ARG,
              "vgg_pad_input: bad args");
  const long long n = (long long)B * (T + 2) * (F + 2) * Cp;
  if (out_dtype == ASR_DT_BF16)
    hipLaunchKernelGGL((vgg_pad_input<uint16_t>), dim3(grid_for(n)), dim3(CT), 0,
                       (hipStream_t)stream, xs, B, T, F, Cp, (uint16_t*)out);
  else
    hipLaunchKernelGGL((vgg_pad_input<float>), dim3(grid_for(n)), dim3(CT), 0,
                       (hipStream_t)stream, xs, B, T, F, Cp, (float*)out);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_conv_weight_pack_pad(const float* w, int Co, int Ci, int Cip, int mode,
                                        int out_dtype, void* out, void* stream);
extern "C" int asr_conv_weight_unpack_acc_pad(const float* packed, int Co, int Ci, int Cip,
                                              float* dw, void* stream);

extern "C" int asr_conv_weight_pack(const float* w, int Co, int Ci, int mode, int out_dtype,
                                    void* out, void* stream) {
  return asr_conv_weight_pack_pad(w, Co, Ci, Ci, mode, out_dtype, out, stream);
}

extern "C" int asr_conv_weight_pack_pad(const float* w, int Co, int Ci, int Cip, int mode,
                                        int out_dtype, void* out, void* stream) {
  ASR_REQUIRE(w && out && Co > 0 && Ci > 0 && (mode == 0 || mode == 1), ASR_ERR_ARG,
              "conv_weight_pack: bad args");
  ASR_REQUIRE(Cip >= Ci && (mode == 0 || Cip == Ci), ASR_ERR_ARG,
              "conv_weight_pack: channel pitch %d < %d (or padded mode 1)", Cip, Ci);
  const long long n = (long long)Co * Ci * 9;
  if (out_dtype == ASR_DT_BF16)
    hipLaunchKernelGGL((weight_pack<uint16_t>), dim3(grid_for(n)), dim3(CT), 0,
                       (hipStream_t)stream, w, Co, Ci, Cip, mode, (uint16_t*)out);
  else
    hipLaunchKernelGGL((weight_pack<float>), dim3(grid_for(n)), dim3(CT), 0, (hipStream_t)stream,
                       w, Co, Ci, Cip, mode, (float*)out);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_conv_weight_unpack_acc(const float* packed, int Co, int Ci, float* dw,
                                          void* stream) {
  return asr_conv_weight_unpack_acc_pad(packed, Co, Ci, Ci, dw, stream);
}

extern "C" int asr_conv_weight_unpack_acc_pad_t(const float* packed_t, int Co, int Ci, int Cip,
                                                float* dw, void* stream) {
  ASR_REQUIRE(packed_t && dw && Co > 0 && Ci > 0 && Cip >= Ci, ASR_ERR_ARG,
              "conv_weight_unpack_t: bad args");
  const long long n = (long long)Co * Ci * 9;
  hipLaunchKernelGGL(weight_unpack_acc_t, dim3(grid_for(n)), dim3(CT), 0, (hipStream_t)stream,
                     packed_t, Co, Ci, Cip, dw);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_conv_weight_unpack_acc_pad(const float* packed, int Co, int Ci, int Cip,
                                              float* dw, void* stream) {
  ASR_REQUIRE(packed && dw && Co > 0 && Ci > 0 && Cip >= Ci, ASR_ERR_ARG,
              "conv_weight_unpack_acc: bad args");
  hipLaunchKernelGGL(weight_unpack_acc, dim3(grid_for((long long)Co * Ci * 9)), dim3(CT), 0,
                     (hipStream_t)stream, packed, Co, Ci, Cip, dw);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_conv_direct_forward(const float* x, int B, int T, int F, int Ci, int Co,
                                       const float* w, const float* bias, float* z,
                                       void* stream) {
  ASR_REQUIRE(x && w && z && B > 0 && T > 0 && F > 0 && Ci > 0 && Co > 0, ASR_ERR_ARG,
              "conv_direct_forward: bad args");
  hipLaunchKernelGGL(conv_direct_fwd, dim3(grid_for((long long)B * T * F * Co)), dim3(CT), 0,
                     (hipStream_t)stream, x, B, T, F, Ci, Co, w, bias, z);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

// Single-input-channel 3x3 convolution forward from channel 0 of a padded
// operand x [B][T+2][F+2][cstride] (x_dtype F32 or BF16): z [B][T+2][F+2][Co]
// f32 at valid pixels, + bias.  Co % 4 == 0, Co <= 512.
extern "C" int asr_conv3x3_c1_forward(const void* x, int x_dtype, int cstride, int B, int T,
                                      int F, int Co, const float* w, const float* bias, float* z,
                                      void* stream) {
  ASR_REQUIRE(x && w && z && B > 0 && T > 0 && F > 0 && cstride > 0, ASR_ERR_ARG,
              "conv3x3_c1_forward: bad args");
  ASR_REQUIRE(Co > 0 && Co % 4 == 0 && Co <= 512, ASR_ERR_UNSUPPORTED,
              "conv3x3_c1_forward: Co must be a multiple of 4, <= 512");
  ASR_REQUIRE(((uintptr_t)z & 15) == 0 && (!bias || ((uintptr_t)bias & 15) == 0), ASR_ERR_ARG,
              "conv3x3_c1_forward: z / bias not 16-B aligned");
  const size_t lds = (size_t)(3 * (F + 2) + 9 * Co) * 4;
  ASR_REQUIRE(lds <= 64 * 1024, ASR_ERR_UNSUPPORTED, "conv3x3_c1_forward: F too large");
  hipStream_t s = (hipStream_t)stream;
  if (x_dtype == ASR_DT_BF16)
    hipLaunchKernelGGL(conv3x3_c1_fwd<uint16_t>, dim3(B * T), dim3(CT), lds, s,
                       (const uint16_t*)x, cstride, T, F, Co, w, bias, z);
  else
    hipLaunchKernelGGL(conv3x3_c1_fwd<float>, dim3(B * T), dim3(CT), lds, s, (const float*)x,
                       cstride, T, F, Co, w, bias, z);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

// asr_conv3x3_c1_forward from the raw features xs [B][T][F] f32 (rounded to
// bf16 first when round_bf16: the values of the bf16 padded operand).
// Co % 4 == 0 and 256 % (Co / 4) == 0.
extern "C" int asr_conv3x3_c1_forward_xs(const float* xs, int round_bf16, int B, int T, int F,
                                         int Co, const float* w, const float* bias, void* z,
                                         int z_dtype, void* stream) {
  ASR_REQUIRE(xs && w && z && B > 0 && T > 0 && F > 0, ASR_ERR_ARG,
              "conv3x3_c1_forward_xs: bad args");
  ASR_REQUIRE(Co > 0 && Co % 4 == 0 && CT % (Co / 4) == 0, ASR_ERR_UNSUPPORTED,
              "conv3x3_c1_forward_xs: Co / 4 must divide %d", CT);
  ASR_REQUIRE(((uintptr_t)z & 15) == 0 && (!bias || ((uintptr_t)bias & 15) == 0), ASR_ERR_ARG,
              "conv3x3_c1_forward_xs: z / bias not 16-B aligned");
  const size_t lds = (size_t)(C1_FT + 2) * (F + 2) * 4;
  ASR_REQUIRE(lds <= 64 * 1024, ASR_ERR_UNSUPPORTED, "conv3x3_c1_forward_xs: F too large");
  const long long nwg = (long long)B * ((T + C1_FT - 1) / C1_FT);
  ASR_REQUIRE(nwg < (1LL << 31), ASR_ERR_UNSUPPORTED, "conv3x3_c1_forward_xs: grid too large");
  if (z_dtype == ASR_DT_BF16)
    hipLaunchKernelGGL(conv3x3_c1_fwd_xs<uint16_t>, dim3((unsigned)nwg), dim3(CT), lds,
                       (hipStream_t)stream, xs, T, F, Co, round_bf16, w, bias, (uint16_t*)z);
  else
    hipLaunchKernelGGL(conv3x3_c1_fwd_xs<float>, dim3((unsigned)nwg), dim3(CT), lds,
                       (hipStream_t)stream, xs, T, F, Co, round_bf16, w, bias, (float*)z);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

// Rows per block of asr_vgg_c1_forward_relu_p (its partial count = the return
// value of asr_vgg_c1_relu_p_blocks).
static int c1p_rows(int B, int T) {
  const long long want = 1024;
  int ft = (int)(((long long)B * T + want - 1) / want);
  return std::max(4, std::min(ft, 64));
}
extern "C" int asr_vgg_c1_relu_p_blocks(int B, int T) {
  const int ft = c1p_rows(B, T);
  return B * ((T + ft - 1) / ft);
}

extern "C" int asr_vgg_c1_forward_relu_p(const float* xs, int round_bf16, int B, int T, int F,
                                         int Co, const float* w, const float* bias,
                                         uint16_t* P, const float* shift, float* mpart,
                                         float* qpart, void* stream) {
  ASR_REQUIRE(xs && w && P && B > 0 && T > 0 && F > 0, ASR_ERR_ARG, "c1_forward_relu_p: bad args");
  ASR_REQUIRE(Co > 0 && Co % 4 == 0 && CT % (Co / 4) == 0, ASR_ERR_UNSUPPORTED,
              "c1_forward_relu_p: Co / 4 must divide %d", CT);
  ASR_REQUIRE(((uintptr_t)P & 7) == 0 && (!bias || ((uintptr_t)bias & 15) == 0), ASR_ERR_ARG,
              "c1_forward_relu_p: P / bias alignment");
  ASR_REQUIRE(!qpart || (mpart && shift), ASR_ERR_ARG, "c1_forward_relu_p: qpart needs mpart, shift");
  const int ft = c1p_rows(B, T);
  const size_t lds = (size_t)(ft + 2) * (F + 2) * 4;
  ASR_REQUIRE(lds <= 48 * 1024, ASR_ERR_UNSUPPORTED, "c1_forward_relu_p: F too large");
  const int nwg = asr_vgg_c1_relu_p_blocks(B, T);
  hipLaunchKernelGGL(conv3x3_c1_fwd_relu_p, dim3((unsigned)nwg), dim3(CT), lds, (hipStream_t)stream,
                     xs, T, F, Co, round_bf16, ft, w, bias, P, shift, mpart, qpart);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_conv_direct_dgrad(const float* dz, int B, int T, int F, int Ci, int Co,
                                     const float* w, float* dx, void* stream) {
  ASR_REQUIRE(dz && w && dx && B > 0 && T > 0 && F > 0 && Ci > 0 && Co > 0, ASR_ERR_ARG,
              "conv_direct_dgrad: bad args");
  hipLaunchKernelGGL(conv_direct_dgrad, dim3(grid_for((long long)B * T * F * Ci)), dim3(CT), 0,
                     (hipStream_t)stream, dz, B, T, F, Ci, Co, w, dx);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

namespace asr {
namespace {
__global__ void acc_kernel(const float* __restrict__ a, float* __restrict__ d, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] += a[i];
}
}  // namespace
}  // namespace asr

extern "C" int asr_vgg_accumulate(const float* a, float* dst, int n, const float* a2, float* dst2,
                                  int n2, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n > 0) hipLaunchKernelGGL(acc_kernel, dim3((n + CT - 1) / CT), dim3(CT), 0, s, a, dst, n);
  if (a2 && dst2 && n2 > 0)
    hipLaunchKernelGGL(acc_kernel, dim3((n2 + CT - 1) / CT), dim3(CT), 0, s, a2, dst2, n2);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" size_t asr_conv_direct_wgrad_workspace_bytes(int B, int T, int F, int Ci, int Co) {
  const long long npix = (long long)B * T * F;
  const long long per = rows_per_chunk(npix);
  const long long nchunk = (npix + per - 1) / per;
  return (size_t)nchunk * (Co * Ci * 9 + Co) * sizeof(float);
}

extern "C" int asr_conv_direct_wgrad(const float* x, const float* dz, int B, int T, int F, int Ci,
                                     int Co, float* dw, float* dbias, void* workspace,
                                     size_t ws_bytes, void* stream) {
  ASR_REQUIRE(x && dz && dw && workspace, ASR_ERR_ARG, "conv_direct_wgrad: null pointer");
  ASR_REQUIRE(ws_bytes >= asr_conv_direct_wgrad_workspace_bytes(B, T, F, Ci, Co),
              ASR_ERR_WORKSPACE, "conv_direct_wgrad: workspace too small");
  const long long npix = (long long)B * T * F;
  const long long per = rows_per_chunk(npix);
  const int nchunk = (int)((npix + per - 1) / per);
  const int nout = Co * Ci * 9 + Co;
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  hipLaunchKernelGGL(conv_direct_wgrad, dim3(nchunk), dim3(CT), 0, s, x, dz, B, T, F, Ci, Co,
                     (int)per, part);
  ASR_LAUNCH_CHECK();
  // row 0 <- column totals (each column is read entirely before its thread writes it)
  hipLaunchKernelGGL(sum_partials, dim3((nout + SP_COLS - 1) / SP_COLS), dim3(CT), 0, s, part, nchunk, nout,
                     1.f, part);
  ASR_LAUNCH_CHECK();
  return asr_vgg_accumulate(part, dw, Co * Ci * 9, dbias ? part + Co * Ci * 9 : nullptr, dbias,
                            Co, stream);
}

extern "C" int asr_vgg_pool_dims(int T, int F, int pt, int pf, int ceil_mode, int* To, int* Fo) {
  ASR_REQUIRE(To && Fo, ASR_ERR_ARG, "vgg_pool_dims: null pointer");
  const Pool pl = make_pool(T, F, pt, pf, ceil_mode);
  *To = pl.To;
  *Fo = pl.Fo;
  return ASR_OK;
}

// post_bwd's grid (block count) for a layer of nr pooled pixels x C channels
inline int post_grid(long long nr, int C) {
  return grid_for(C % 4 == 0 ? nr * C / 4 : nr * C);
}

// the row-blocked passes apply: bf16 P, C % 8 == 0 with C / 8 dividing 256, no
// pooling or 2 x 2 pooling; ASR_VGG_ROWS=0 keeps the grid-stride passes (A/B)
template <typename TP>
bool rw_ok(int C, int pt, int pf) {
  const char* e = getenv("ASR_VGG_ROWS");
  if (e && e[0] == '0') return false;
  if (sizeof(TP) != 2 || C % 8 || 256 % (C / 8)) return false;
  return pt == 0 || (pt == 2 && pf == 2);
}

extern "C" size_t asr_vgg_block_workspace_bytes(int B, int To, int Fo, int C) {
  const long long n = (long long)B * To * Fo;
  const long long per = rows_per_chunk(n);
  const long long nchunk = (n + per - 1) / per;
  // BN partials + sums, then the conv-bias partials of post_bwd (+ their total)
  return (size_t)(nchunk * 2 + 4) * C * sizeof(float) +
         (size_t)(post_grid(n, C) + 1) * C * sizeof(float);
}

// ReLU + pool + BatchNorm (+ stats) + dropout of one VGG layer.
// z: conv output [padded pixels of (T, F)][C]; P / slot: saved for backward;
// bn_mean / bn_rstd: the statistics used ([C] each, written); gamma == NULL: no
// BN.  training: batch statistics and running-stat update, else running stats.
// out: next layer input, padded rows of (T', F') (out_dtype f32 / bf16; the
// caller zeroes it) or, flat, [B][T'][F'][C] f32.
extern "C" int asr_vgg_block_forward_z(const void* z, int z_dtype, int B, int T, int F, int C,
                                       int pt, int pf, int ceil_mode, float* P, uint8_t* slot,
                                       const float* gamma, const float* beta, float* run_mean,
                                       float* run_var, int training, float momentum, float eps,
                                       float* bn_mean, float* bn_rstd, float drop,
                                       unsigned long long seed, void* out, int out_dtype, int flat,
                                       void* workspace, size_t ws_bytes, void* stream);

extern "C" int asr_vgg_block_forward(const float* z, int B, int T, int F, int C, int pt, int pf,
                                     int ceil_mode, float* P, uint8_t* slot, const float* gamma,
                                     const float* beta, float* run_mean, float* run_var,
                                     int training, float momentum, float eps, float* bn_mean,
                                     float* bn_rstd, float drop, unsigned long long seed,
                                     void* out, int out_dtype, int flat, void* workspace,
                                     size_t ws_bytes, void* stream) {
  return asr_vgg_block_forward_z(z, ASR_DT_F32, B, T, F, C, pt, pf, ceil_mode, P, slot, gamma,
                                 beta, run_mean, run_var, training, momentum, eps, bn_mean,
                                 bn_rstd, drop, seed, out, out_dtype, flat, workspace, ws_bytes,
                                 stream);
}

// z_dtype ASR_DT_BF16: the conv output z is bf16 (P and the statistics stay f32)
// TP: the pooled-value store P (float, or bf16 when z is bf16 -- exact)
template <typename TP>
static int vgg_block_forward_impl(const void* z, int z_dtype, int B, int T, int F, int C, int pt,
                                  int pf, int ceil_mode, TP* P, uint8_t* slot, const float* gamma,
                                  const float* beta, float* run_mean, float* run_var, int training,
                                  float momentum, float eps, float* bn_mean, float* bn_rstd,
                                  float drop, unsigned long long seed, void* out, int out_dtype,
                                  int flat, void* workspace, size_t ws_bytes, void* stream) {
  ASR_REQUIRE(z && P && out && B > 0 && T > 0 && F > 0 && C > 0, ASR_ERR_ARG,
              "vgg_block_forward: bad args");
  ASR_REQUIRE(!pt || slot, ASR_ERR_ARG, "vgg_block_forward: pooling needs slot");
  const Pool pl = make_pool(T, F, pt, pf, ceil_mode);
  ASR_REQUIRE(pl.To > 0 && pl.Fo > 0, ASR_ERR_ARG, "vgg_block_forward: empty output");
  ASR_REQUIRE(C <= CT && CT % C == 0, ASR_ERR_UNSUPPORTED,
              "vgg_block_forward: channels %d must divide %d", C, CT);
  hipStream_t s = (hipStream_t)stream;
  const long long nr = (long long)B * pl.To * pl.Fo;
  ASR_REQUIRE((long long)B * (T + 2) * (F + 2) * C < (1LL << 31), ASR_ERR_UNSUPPORTED,
              "vgg_block_forward: layer too large for 32-bit element indices");
  const bool v4 = C % 4 == 0;
  // batch-norm mean folded into the pool pass: per-block sums into the
  // workspace's post_bwd partial region (unused in the forward)
  const char* fm = getenv("ASR_VGG_FUSED_MEAN");
  const bool fused_mean = gamma && training && v4 && workspace && !(fm && fm[0] == '0') &&
                          ws_bytes >= asr_vgg_block_workspace_bytes(B, pl.To, pl.Fo, C);
  float* mpart = nullptr;
  if (fused_mean) {
    const long long per = rows_per_chunk(nr);
    const long long nchunk = (nr + per - 1) / per;
    mpart = (float*)workspace + (size_t)(nchunk * 2 + 4) * C;
  }
  // fused: at most 1024 blocks, so the ordered partial sum (one thread per
  // column phase) stays short -- 8192 partials took 1 ms / step at vgg_hier
  const int fgrid = fused_mean ? std::min(post_grid(nr, C), 1024) : post_grid(nr, C);
  // ... and the variance pass with it, centred on the running mean: the
  // squared sums go to the BN partial region (fgrid <= its 1024 chunks)
  const char* fv = getenv("ASR_VGG_FUSED_VAR");
  const long long vchunks = (nr + rows_per_chunk(nr) - 1) / rows_per_chunk(nr);
  const bool fused_var = fused_mean && run_mean && run_var && !(fv && fv[0] == '0') &&
                         fgrid <= vchunks;
  float* qpart = fused_var ? (float*)workspace : nullptr;
  const float* vshift = fused_var ? run_mean : nullptr;
  const bool zb = z_dtype == ASR_DT_BF16;
  ASR_REQUIRE(!zb || (v4 && ((uintptr_t)z & 7) == 0), ASR_ERR_UNSUPPORTED,
              "vgg_block_forward: bf16 z needs C % 4 == 0 and 8-B alignment");
  // row-blocked passes (rw_*): bf16 z and P, 16-B aligned operands
  const bool rows_ok = rw_ok<TP>(C, pt, pf) && ((uintptr_t)z & 15) == 0 &&
                       ((uintptr_t)P & 15) == 0 && (!slot || ((uintptr_t)slot & 7) == 0) &&
                       (!gamma || !training || fused_mean);
  const int nrow = B * pl.To;
  int rgrid = fgrid, rrpb = 1;
  if (rows_ok) {   // blocks <= the partial regions' capacity (fgrid, the BN chunks)
    rrpb = (nrow + fgrid - 1) / fgrid;
    rgrid = (nrow + rrpb - 1) / rrpb;
  }
  if (rows_ok) {
    if (pt)
      hipLaunchKernelGGL((rw_post_fwd<2>), dim3(rgrid), dim3(RW_NT), 0, s, (const uint16_t*)z, B,
                         T, F, C, pl, (uint16_t*)P, slot, mpart, vshift, qpart, rrpb);
    else
      hipLaunchKernelGGL((rw_post_fwd<0>), dim3(rgrid), dim3(RW_NT), 0, s, (const uint16_t*)z, B,
                         T, F, C, pl, (uint16_t*)P, slot, mpart, vshift, qpart, rrpb);
  } else if (zb)
    hipLaunchKernelGGL((post_fwd<4, uint16_t, TP>), dim3(fgrid), dim3(CT), 0, s, (const uint16_t*)z, B,
                       T, F, C, pl, P, slot, mpart, vshift, qpart);
  else if (v4)
    hipLaunchKernelGGL((post_fwd<4, float, TP>), dim3(fgrid), dim3(CT), 0, s, (const float*)z, B, T, F, C, pl,
                       P, slot, mpart, vshift, qpart);
  else
    hipLaunchKernelGGL((post_fwd<1, float, TP>), dim3(post_grid(nr, C)), dim3(CT), 0, s, (const float*)z, B, T,
                       F, C, pl, P, slot, (float*)nullptr, (const float*)nullptr,
                       (float*)nullptr);
  ASR_LAUNCH_CHECK();
  Affine af{nullptr, nullptr, nullptr, nullptr, drop, seed};
  if (gamma) {
    ASR_REQUIRE(beta && bn_mean && bn_rstd && workspace, ASR_ERR_ARG,
                "vgg_block_forward: BN needs beta / mean / rstd / workspace");
    ASR_REQUIRE(ws_bytes >= asr_vgg_block_workspace_bytes(B, pl.To, pl.Fo, C), ASR_ERR_WORKSPACE,
                "vgg_block_forward: workspace too small");
    if (training) {
      const long long per = rows_per_chunk(nr);
      const int nchunk = (int)((nr + per - 1) / per);
      float* part = (float*)workspace;
      float* m2 = part + (size_t)nchunk * C;
      if (fused_var) {
        hipLaunchKernelGGL(sum_partials, dim3((C + SP_COLS - 1) / SP_COLS), dim3(CT), 0, s, mpart,
                           rgrid, C, 1.f / (float)nr, bn_mean);
        hipLaunchKernelGGL(sum_partials, dim3((C + SP_COLS - 1) / SP_COLS), dim3(CT), 0, s, qpart,
                           rgrid, C, 1.f / (float)nr, m2);
        hipLaunchKernelGGL(bn_finalize_shift, dim3((C + CT - 1) / CT), dim3(CT), 0, s, bn_mean, m2,
                           run_mean, C, nr, eps, momentum, bn_rstd, run_mean, run_var);
      } else if (fused_mean) {
        hipLaunchKernelGGL(sum_partials, dim3((C + SP_COLS - 1) / SP_COLS), dim3(CT), 0, s, mpart, rgrid, C,
                           1.f / (float)nr, bn_mean);
      } else {
        hipLaunchKernelGGL(col_moment<TP>, dim3(nchunk), dim3(CT), 0, s, P, nr, C, per, nullptr, 0,
                           part);
        hipLaunchKernelGGL(sum_partials, dim3((C + SP_COLS - 1) / SP_COLS), dim3(CT), 0, s, part, nchunk, C,
                           1.f / (float)nr, bn_mean);
      }
      if (!fused_var) {
        hipLaunchKernelGGL(col_moment<TP>, dim3(nchunk), dim3(CT), 0, s, P, nr, C, per, bn_mean, 1,
                           part);
        hipLaunchKernelGGL(sum_partials, dim3((C + SP_COLS - 1) / SP_COLS), dim3(CT), 0, s, part,
                           nchunk, C, 1.f / (float)nr, m2);
        hipLaunchKernelGGL(bn_finalize, dim3((C + CT - 1) / CT), dim3(CT), 0, s, bn_mean, m2, C,
                           nr, eps, momentum, bn_rstd, run_mean, run_var);
      }
    } else {
      ASR_REQUIRE(run_mean && run_var, ASR_ERR_ARG, "vgg_block_forward: eval needs running stats");
      hipLaunchKernelGGL(bn_eval_stats, dim3((C + CT - 1) / CT), dim3(CT), 0, s, run_mean,
                         run_var, C, eps, bn_mean, bn_rstd);
    }
    ASR_LAUNCH_CHECK();
    af.mean = bn_mean;
    af.rstd = bn_rstd;
    af.gamma = gamma;
    af.beta = beta;
  }
  const long long ng = v4 ? nr * C / 4 : nr * C;
  const bool out16 = ((uintptr_t)out & 15) == 0;
  if (rows_ok && out16 && (out_dtype == ASR_DT_F32 || !flat)) {
    const int agrid = std::min(nrow, 4096), arpb = (nrow + agrid - 1) / agrid;
    if (out_dtype == ASR_DT_BF16)
      hipLaunchKernelGGL((rw_apply<uint16_t>), dim3((nrow + arpb - 1) / arpb), dim3(RW_NT), 0, s,
                         (const uint16_t*)P, B, pl.To, pl.Fo, C, af, (uint16_t*)out, flat, arpb);
    else
      hipLaunchKernelGGL((rw_apply<float>), dim3((nrow + arpb - 1) / arpb), dim3(RW_NT), 0, s,
                         (const uint16_t*)P, B, pl.To, pl.Fo, C, af, (float*)out, flat, arpb);
  } else if (out_dtype == ASR_DT_BF16 && !flat) {
    if (v4)
      hipLaunchKernelGGL((apply_fwd<uint16_t, 4, TP>), dim3(grid_for(ng)), dim3(CT), 0, s, P, B,
                         pl.To, pl.Fo, C, af, (uint16_t*)out, 0);
    else
      hipLaunchKernelGGL((apply_fwd<uint16_t, 1, TP>), dim3(grid_for(ng)), dim3(CT), 0, s, P, B,
                         pl.To, pl.Fo, C, af, (uint16_t*)out, 0);
  } else {
    if (v4)
      hipLaunchKernelGGL((apply_fwd<float, 4, TP>), dim3(grid_for(ng)), dim3(CT), 0, s, P, B, pl.To,
                         pl.Fo, C, af, (float*)out, flat);
    else
      hipLaunchKernelGGL((apply_fwd<float, 1, TP>), dim3(grid_for(ng)), dim3(CT), 0, s, P, B, pl.To,
                         pl.Fo, C, af, (float*)out, flat);
  }
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_vgg_block_forward_zp(const void* z, int z_dtype, int B, int T, int F, int C,
                                        int pt, int pf, int ceil_mode, void* P, int p_dtype,
                                        uint8_t* slot, const float* gamma, const float* beta,
                                        float* run_mean, float* run_var, int training,
                                        float momentum, float eps, float* bn_mean, float* bn_rstd,
                                        float drop, unsigned long long seed, void* out,
                                        int out_dtype, int flat, void* workspace, size_t ws_bytes,
                                        void* stream) {
  if (p_dtype == ASR_DT_BF16) {
    ASR_REQUIRE(z_dtype == ASR_DT_BF16 && C % 4 == 0 && ((uintptr_t)P & 7) == 0,
                ASR_ERR_UNSUPPORTED, "vgg_block_forward: bf16 P needs bf16 z and C %% 4 == 0");
    return vgg_block_forward_impl(z, z_dtype, B, T, F, C, pt, pf, ceil_mode, (uint16_t*)P, slot,
                                  gamma, beta, run_mean, run_var, training, momentum, eps,
                                  bn_mean, bn_rstd, drop, seed, out, out_dtype, flat, workspace,
                                  ws_bytes, stream);
  }
  ASR_REQUIRE(p_dtype == ASR_DT_F32, ASR_ERR_ARG, "vgg_block_forward: P dtype %d", p_dtype);
  return vgg_block_forward_impl(z, z_dtype, B, T, F, C, pt, pf, ceil_mode, (float*)P, slot, gamma,
                                beta, run_mean, run_var, training, momentum, eps, bn_mean, bn_rstd,
                                drop, seed, out, out_dtype, flat, workspace, ws_bytes, stream);
}

extern "C" int asr_vgg_block_forward_z(const void* z, int z_dtype, int B, int T, int F, int C,
                                       int pt, int pf, int ceil_mode, float* P, uint8_t* slot,
                                       const float* gamma, const float* beta, float* run_mean,
                                       float* run_var, int training, float momentum, float eps,
                                       float* bn_mean, float* bn_rstd, float drop,
                                       unsigned long long seed, void* out, int out_dtype, int flat,
                                       void* workspace, size_t ws_bytes, void* stream) {
  return asr_vgg_block_forward_zp(z, z_dtype, B, T, F, C, pt, pf, ceil_mode, P, ASR_DT_F32, slot,
                                  gamma, beta, run_mean, run_var, training, momentum, eps, bn_mean,
                                  bn_rstd, drop, seed, out, out_dtype, flat, workspace, ws_bytes,
                                  stream);
}

// asr_vgg_block_forward_zp for an unpooled layer whose P (bf16, flat) and
// batch-norm moment partials were produced by its convolution
// (asr_vgg_c1_forward_relu_p; mpart / qpart [nblk][C] of P - run_mean and its
// square): the statistics, the running-stat update and the next layer's
// input, without the ReLU pass.  workspace >= C floats.
extern "C" int asr_vgg_block_forward_given_p(const uint16_t* P, int B, int T, int F, int C,
                                             const float* gamma, const float* beta,
                                             float* run_mean, float* run_var, int training,
                                             float momentum, float eps, float* bn_mean,
                                             float* bn_rstd, float drop, unsigned long long seed,
                                             void* out, int out_dtype, int flat,
                                             const float* mpart, const float* qpart, int nblk,
                                             void* workspace, size_t ws_bytes, void* stream) {
  ASR_REQUIRE(P && out && B > 0 && T > 0 && F > 0, ASR_ERR_ARG, "vgg_block_forward_given_p: bad args");
  ASR_REQUIRE(rw_ok<uint16_t>(C, 0, 0) && ((uintptr_t)P & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
              (out_dtype == ASR_DT_F32 || !flat), ASR_ERR_UNSUPPORTED,
              "vgg_block_forward_given_p: row-blocked apply only");
  hipStream_t s = (hipStream_t)stream;
  const long long nr = (long long)B * T * F;
  Affine af{nullptr, nullptr, nullptr, nullptr, drop, seed};
  if (gamma) {
    ASR_REQUIRE(beta && bn_mean && bn_rstd, ASR_ERR_ARG, "vgg_block_forward_given_p: BN args");
    if (training) {
      ASR_REQUIRE(mpart && qpart && nblk > 0 && run_mean && run_var && workspace &&
                  ws_bytes >= (size_t)C * sizeof(float), ASR_ERR_ARG,
                  "vgg_block_forward_given_p: training needs the partials and running stats");
      float* m2 = (float*)workspace;
      hipLaunchKernelGGL(sum_partials, dim3((C + SP_COLS - 1) / SP_COLS), dim3(CT), 0, s, mpart,
                         nblk, C, 1.f / (float)nr, bn_mean);
      hipLaunchKernelGGL(sum_partials, dim3((C + SP_COLS - 1) / SP_COLS), dim3(CT), 0, s, qpart,
                         nblk, C, 1.f / (float)nr, m2);
      hipLaunchKernelGGL(bn_finalize_shift, dim3((C + CT - 1) / CT), dim3(CT), 0, s, bn_mean, m2,
                         run_mean, C, nr, eps, momentum, bn_rstd, run_mean, run_var);
    } else {
      ASR_REQUIRE(run_mean && run_var, ASR_ERR_ARG, "vgg_block_forward_given_p: eval needs running stats");
      hipLaunchKernelGGL(bn_eval_stats, dim3((C + CT - 1) / CT), dim3(CT), 0, s, run_mean, run_var,
                         C, eps, bn_mean, bn_rstd);
    }
    ASR_LAUNCH_CHECK();
    af.mean = bn_mean;
    af.rstd = bn_rstd;
    af.gamma = gamma;
    af.beta = beta;
  }
  const int nrow = B * T;
  const int agrid = std::min(nrow, 4096), arpb = (nrow + agrid - 1) / agrid;
  if (out_dtype == ASR_DT_BF16)
    hipLaunchKernelGGL((rw_apply<uint16_t>), dim3((nrow + arpb - 1) / arpb), dim3(RW_NT), 0, s, P, B,
                       T, F, C, af, (uint16_t*)out, flat, arpb);
  else
    hipLaunchKernelGGL((rw_apply<float>), dim3((nrow + arpb - 1) / arpb), dim3(RW_NT), 0, s, P, B, T,
                       F, C, af, (float*)out, flat, arpb);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

// Backward of asr_vgg_block_forward (same geometry / saved tensors): dnext is
// the gradient of `out` (padded rows f32 or flat); dz [padded pixels][C] of
// dz_dtype receives d(conv output) (the caller zeroes it: halo and
// not-selected pixels stay 0); dgamma / dbeta accumulate (+=).
extern "C" int asr_vgg_block_backward_ex(const float* dnext, int flat, const float* z, int B,
                                         int T, int F, int C, int pt, int pf, int ceil_mode,
                                         const float* P, const uint8_t* slot, const float* gamma,
                                         const float* bn_mean, const float* bn_rstd,
                                         float* dgamma, float* dbeta, float drop,
                                         unsigned long long seed, void* dz, int dz_dtype,
                                         float* dbias, void* workspace, size_t ws_bytes,
                                         void* stream);

extern "C" int asr_vgg_block_backward(const float* dnext, int flat, const float* z, int B, int T,
                                      int F, int C, int pt, int pf, int ceil_mode,
                                      const float* P, const uint8_t* slot, const float* gamma,
                                      const float* bn_mean, const float* bn_rstd, float* dgamma,
                                      float* dbeta, float drop, unsigned long long seed,
                                      void* dz, int dz_dtype, void* workspace, size_t ws_bytes,
                                      void* stream) {
  return asr_vgg_block_backward_ex(dnext, flat, z, B, T, F, C, pt, pf, ceil_mode, P, slot, gamma,
                                   bn_mean, bn_rstd, dgamma, dbeta, drop, seed, dz, dz_dtype,
                                   nullptr, workspace, ws_bytes, stream);
}

// ... and dbias (nullable) += the conv bias gradient, sum of dZ per channel
// (formed from the f32 values before dZ is stored, in a fixed order).
extern "C" int asr_vgg_block_backward_z(const float* dnext, int flat, const void* z,
                                        int z_dtype, int B, int T, int F, int C, int pt, int pf,
                                        int ceil_mode, const float* P, const uint8_t* slot,
                                        const float* gamma, const float* bn_mean,
                                        const float* bn_rstd, float* dgamma, float* dbeta,
                                        float drop, unsigned long long seed, void* dz,
                                        int dz_dtype, float* dbias, void* workspace,
                                        size_t ws_bytes, void* stream);

extern "C" int asr_vgg_block_backward_ex(const float* dnext, int flat, const float* z, int B,
                                         int T, int F, int C, int pt, int pf, int ceil_mode,
                                         const float* P, const uint8_t* slot, const float* gamma,
                                         const float* bn_mean, const float* bn_rstd,
                                         float* dgamma, float* dbeta, float drop,
                                         unsigned long long seed, void* dz, int dz_dtype,
                                         float* dbias, void* workspace, size_t ws_bytes,
                                         void* stream) {
  return asr_vgg_block_backward_z(dnext, flat, z, ASR_DT_F32, B, T, F, C, pt, pf, ceil_mode, P,
                                  slot, gamma, bn_mean, bn_rstd, dgamma, dbeta, drop, seed, dz,
                                  dz_dtype, dbias, workspace, ws_bytes, stream);
}

// z_dtype ASR_DT_BF16: the saved conv output z is bf16 (the ReLU mask read back);
// dnext_dtype ASR_DT_BF16 (full-resolution pass with C % 4 == 0 only): the
// incoming gradient is bf16 (the input-gradient convolution writes it so)
template <typename TP>
static int vgg_block_backward_impl(const void* dnext_v, int dnext_dtype, int flat, const void* z,
                                   int z_dtype, int B, int T, int F, int C, int pt, int pf,
                                   int ceil_mode, const TP* P, const uint8_t* slot,
                                   const float* gamma, const float* bn_mean, const float* bn_rstd,
                                   float* dgamma, float* dbeta, float drop,
                                   unsigned long long seed, void* dz, int dz_dtype, float* dbias,
                                   void* workspace, size_t ws_bytes, void* stream) {
  const float* dnext = (const float*)dnext_v;
  const uint16_t* dnh = (const uint16_t*)dnext_v;
  const bool db16 = dnext_dtype == ASR_DT_BF16;
  ASR_REQUIRE(dnext && z && P && dz && B > 0 && T > 0 && F > 0 && C > 0, ASR_ERR_ARG,
              "vgg_block_backward: bad args");
  ASR_REQUIRE(!db16 || (C % 4 == 0 && z_dtype == ASR_DT_BF16 && dz_dtype == ASR_DT_BF16 &&
                        ((uintptr_t)dnh & 7) == 0),
              ASR_ERR_UNSUPPORTED, "vgg_block_backward: bf16 dnext needs the bf16 full pass");
  const Pool pl = make_pool(T, F, pt, pf, ceil_mode);
  hipStream_t s = (hipStream_t)stream;
  const long long nr = (long long)B * pl.To * pl.Fo;
  ASR_REQUIRE((long long)B * (T + 2) * (F + 2) * C < (1LL << 31), ASR_ERR_UNSUPPORTED,
              "vgg_block_backward: layer too large for 32-bit element indices");
  ASR_REQUIRE(C <= CT && CT % C == 0, ASR_ERR_UNSUPPORTED,
              "vgg_block_backward: channels %d must divide %d", C, CT);
  const bool v4 = C % 4 == 0;
  Affine af{nullptr, nullptr, nullptr, nullptr, drop, seed};
  float* sums = nullptr;
  float* bpart = nullptr;
  const int pgrid = post_grid(nr, C);
  // row-blocked passes (rw_*): bf16 z / P / dz with batch norm, 16-B aligned
  // z == P (the convolution wrote only P, asr_vgg_c1_forward_relu_p): the ReLU
  // mask must come from P -- the row-blocked pass or the full pass with BN
  const bool z_is_p = (const void*)z == (const void*)P;
  const bool rows_b = rw_ok<TP>(C, pt, pf) && gamma && z_dtype == ASR_DT_BF16 &&
                      dz_dtype == ASR_DT_BF16 && ((uintptr_t)P & 15) == 0 &&
                      ((uintptr_t)dz & 15) == 0 && ((uintptr_t)dnext_v & 15) == 0 &&
                      (!slot || ((uintptr_t)slot & 7) == 0);
  if (dbias) {
    ASR_REQUIRE(workspace && ws_bytes >= asr_vgg_block_workspace_bytes(B, pl.To, pl.Fo, C),
                ASR_ERR_WORKSPACE, "vgg_block_backward: bias needs the workspace");
    const long long per = rows_per_chunk(nr);
    const long long nchunk = (nr + per - 1) / per;
    bpart = (float*)workspace + (size_t)(nchunk * 2 + 4) * C;
  }
  if (gamma) {
    ASR_REQUIRE(bn_mean && bn_rstd && workspace, ASR_ERR_ARG, "vgg_block_backward: BN args");
    ASR_REQUIRE(ws_bytes >= asr_vgg_block_workspace_bytes(B, pl.To, pl.Fo, C), ASR_ERR_WORKSPACE,
                "vgg_block_backward: workspace too small");
    af.mean = bn_mean;
    af.rstd = bn_rstd;
    af.gamma = gamma;
    const long long per = rows_per_chunk(nr);
    const int nchunk = (int)((nr + per - 1) / per);
    float* part = (float*)workspace;
    sums = part + (size_t)nchunk * 2 * C;
    int mchunk = nchunk;
    if (rows_b) {   // row-blocked moments: at most nchunk blocks
      const int nrow = B * pl.To, rpb = (nrow + nchunk - 1) / nchunk;
      mchunk = (nrow + rpb - 1) / rpb;
      const char* bnm = getenv("ASR_VGG_BNM");   // "<NT>x<U>" (A/B; read per call)
      int bnt = 256, bu = 1;
      if (bnm) sscanf(bnm, "%dx%d", &bnt, &bu);
      const size_t lnu = (size_t)bnt * 8 * sizeof(float);
#define ASR_BNM(NT, U)                                                                           \
  hipLaunchKernelGGL((rw_bn_moments_nu<uint16_t, NT, U>), dim3(mchunk), dim3(NT), lnu, s, dnh,   \
                     (const uint16_t*)P, B, pl.To, pl.Fo, C, flat, af, part, rpb)
      if (db16 && bnt == 256 && bu == 2) ASR_BNM(256, 2);
      else if (db16 && bnt == 256 && bu == 4) ASR_BNM(256, 4);
      else if (db16 && bnt == 512 && bu == 1) ASR_BNM(512, 1);
      else if (db16 && bnt == 512 && bu == 2) ASR_BNM(512, 2);
      else if (db16 && bnt == 1024 && bu == 1) ASR_BNM(1024, 1);
      else if (db16 && bnt == 1024 && bu == 2) ASR_BNM(1024, 2);
#undef ASR_BNM
      else if (db16)
        hipLaunchKernelGGL((rw_bn_moments<uint16_t>), dim3(mchunk), dim3(RW_NT), 0, s, dnh,
                           (const uint16_t*)P, B, pl.To, pl.Fo, C, flat, af, part, rpb);
      else
        hipLaunchKernelGGL((rw_bn_moments<float>), dim3(mchunk), dim3(RW_NT), 0, s, dnext,
                           (const uint16_t*)P, B, pl.To, pl.Fo, C, flat, af, part, rpb);
    } else if (db16)
      hipLaunchKernelGGL((bn_bwd_moments<4, uint16_t, TP>), dim3(nchunk), dim3(CT), 0, s, dnh, P, B,
                         pl.To, pl.Fo, C, flat, af, per, part);
    else if (v4)
      hipLaunchKernelGGL((bn_bwd_moments<4, float, TP>), dim3(nchunk), dim3(CT), 0, s, dnext, P, B, pl.To,
                         pl.Fo, C, flat, af, per, part);
    else
      hipLaunchKernelGGL((bn_bwd_moments<1, float, TP>), dim3(nchunk), dim3(CT), 0, s, dnext, P, B, pl.To,
                         pl.Fo, C, flat, af, per, part);
    hipLaunchKernelGGL(sum_partials, dim3((2 * C + SP_COLS - 1) / SP_COLS), dim3(CT), 0, s, part, mchunk, 2 * C,
                       1.f, sums);
    hipLaunchKernelGGL(bn_bwd_finalize, dim3((C + CT - 1) / CT), dim3(CT), 0, s, sums, C, dgamma,
                       dbeta);
    ASR_LAUNCH_CHECK();
  }
  const char* pfe = getenv("ASR_VGG_POST_FULL");   // A/B: full-resolution dz pass
  const bool zb = z_dtype == ASR_DT_BF16;
  const bool full = v4 && !(pfe && pfe[0] == '0') && ((uintptr_t)dz & 15) == 0 &&
                    ((uintptr_t)z & (zb ? 7 : 15)) == 0;
  ASR_REQUIRE(!zb || v4, ASR_ERR_UNSUPPORTED, "vgg_block_backward: bf16 z needs C % 4 == 0");
  const float* zf = (const float*)z;
  const uint16_t* zh = (const uint16_t*)z;
  ASR_REQUIRE(!db16 || full, ASR_ERR_UNSUPPORTED, "vgg_block_backward: bf16 dnext needs the full pass");
  ASR_REQUIRE(!z_is_p || rows_b || (full && gamma && pt == 0), ASR_ERR_UNSUPPORTED,
              "vgg_block_backward: z aliased to P needs a pass that masks from P");
  int bgrid = pgrid;
  // pooled layers whose windows cover every input pixel: the pooled-grid walk
  // (ASR_VGG_POOL_WALK=0: the input-pixel walk)
  const char* pwe = getenv("ASR_VGG_POOL_WALK");
  const bool pool_walk = rows_b && pt && !(pwe && pwe[0] == '0') && 2 * pl.To >= T &&
                         2 * pl.Fo >= F;
  if (pool_walk) {
    const int nrow = B * pl.To, rpb = (nrow + pgrid - 1) / pgrid;
    bgrid = (nrow + rpb - 1) / rpb;
    if (db16)
      hipLaunchKernelGGL((rw_post_bwd_pool<uint16_t>), dim3(bgrid), dim3(RW_NT), 5 * C * sizeof(float),
                         s, dnh, (const uint16_t*)P, slot, B, T, F, C, pl, flat, af, sums,
                         (uint16_t*)dz, bpart, rpb);
    else
      hipLaunchKernelGGL((rw_post_bwd_pool<float>), dim3(bgrid), dim3(RW_NT), 5 * C * sizeof(float),
                         s, dnext, (const uint16_t*)P, slot, B, T, F, C, pl, flat, af, sums,
                         (uint16_t*)dz, bpart, rpb);
  } else if (rows_b) {   // at most pgrid blocks (the bias-partial region)
    const int nrow = B * T, rpb = (nrow + pgrid - 1) / pgrid;
    bgrid = (nrow + rpb - 1) / rpb;
    if (db16) {

      if (pt)
        hipLaunchKernelGGL((rw_post_bwd<2, uint16_t>), dim3(bgrid), dim3(RW_NT), 5 * C * sizeof(float), s, dnh,
                           (const uint16_t*)P, slot, B, T, F, C, pl, flat, af, sums, (uint16_t*)dz,
                           bpart, rpb);
      else
        hipLaunchKernelGGL((rw_post_bwd<0, uint16_t>), dim3(bgrid), dim3(RW_NT), 5 * C * sizeof(float), s, dnh,
                           (const uint16_t*)P, slot, B, T, F, C, pl, flat, af, sums, (uint16_t*)dz,
                           bpart, rpb);
    } else {
      if (pt)
        hipLaunchKernelGGL((rw_post_bwd<2, float>), dim3(bgrid), dim3(RW_NT), 5 * C * sizeof(float), s, dnext,
                           (const uint16_t*)P, slot, B, T, F, C, pl, flat, af, sums, (uint16_t*)dz,
                           bpart, rpb);
      else
        hipLaunchKernelGGL((rw_post_bwd<0, float>), dim3(bgrid), dim3(RW_NT), 5 * C * sizeof(float), s, dnext,
                           (const uint16_t*)P, slot, B, T, F, C, pl, flat, af, sums, (uint16_t*)dz,
                           bpart, rpb);
    }
  } else if (db16) {
    hipLaunchKernelGGL((post_bwd_full<uint16_t, uint16_t, uint16_t, TP>), dim3(pgrid), dim3(CT), 0, s,
                       dnh, P, zh, slot, B, T, F, C, pl, flat, af, sums, (uint16_t*)dz, bpart);
  } else if (zb) {
    if (full && dz_dtype == ASR_DT_BF16)
      hipLaunchKernelGGL((post_bwd_full<uint16_t, uint16_t, float, TP>), dim3(pgrid), dim3(CT), 0, s, dnext,
                         P, zh, slot, B, T, F, C, pl, flat, af, sums, (uint16_t*)dz, bpart);
    else if (full)
      hipLaunchKernelGGL((post_bwd_full<float, uint16_t, float, TP>), dim3(pgrid), dim3(CT), 0, s, dnext, P,
                         zh, slot, B, T, F, C, pl, flat, af, sums, (float*)dz, bpart);
    else if (dz_dtype == ASR_DT_BF16)
      hipLaunchKernelGGL((post_bwd<uint16_t, 4, uint16_t, TP>), dim3(pgrid), dim3(CT), 0, s, dnext, P,
                         zh, slot, B, T, F, C, pl, flat, af, sums, (uint16_t*)dz, bpart);
    else
      hipLaunchKernelGGL((post_bwd<float, 4, uint16_t, TP>), dim3(pgrid), dim3(CT), 0, s, dnext, P,
                         zh, slot, B, T, F, C, pl, flat, af, sums, (float*)dz, bpart);
  } else if (full && dz_dtype == ASR_DT_BF16) {
    hipLaunchKernelGGL((post_bwd_full<uint16_t, float, float, TP>), dim3(pgrid), dim3(CT), 0, s, dnext, P, zf, slot, B,
                       T, F, C, pl, flat, af, sums, (uint16_t*)dz, bpart);
  } else if (full) {
    hipLaunchKernelGGL((post_bwd_full<float, float, float, TP>), dim3(pgrid), dim3(CT), 0, s, dnext, P, zf, slot, B, T,
                       F, C, pl, flat, af, sums, (float*)dz, bpart);
  } else if (dz_dtype == ASR_DT_BF16) {
    if (v4)
      hipLaunchKernelGGL((post_bwd<uint16_t, 4, float, TP>), dim3(pgrid), dim3(CT), 0, s, dnext, P, zf, slot,
                         B, T, F, C, pl, flat, af, sums, (uint16_t*)dz, bpart);
    else
      hipLaunchKernelGGL((post_bwd<uint16_t, 1, float, TP>), dim3(pgrid), dim3(CT), 0, s, dnext, P, zf, slot,
                         B, T, F, C, pl, flat, af, sums, (uint16_t*)dz, bpart);
  } else {
    if (v4)
      hipLaunchKernelGGL((post_bwd<float, 4, float, TP>), dim3(pgrid), dim3(CT), 0, s, dnext, P, zf, slot, B,
                         T, F, C, pl, flat, af, sums, (float*)dz, bpart);
    else
      hipLaunchKernelGGL((post_bwd<float, 1, float, TP>), dim3(pgrid), dim3(CT), 0, s, dnext, P, zf, slot, B,
                         T, F, C, pl, flat, af, sums, (float*)dz, bpart);
  }
  ASR_LAUNCH_CHECK();
  if (dbias) {   // total over the blocks in order, then dbias += total
    float* tot = bpart + (size_t)pgrid * C;
    hipLaunchKernelGGL(sum_partials, dim3((C + SP_COLS - 1) / SP_COLS), dim3(CT), 0, s, bpart, bgrid, C, 1.f,
                       tot);
    ASR_LAUNCH_CHECK();
    return asr_vgg_accumulate(tot, dbias, C, nullptr, nullptr, 0, stream);
  }
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

// p_dtype ASR_DT_BF16: P was stored bf16 by asr_vgg_block_forward_zp
extern "C" int asr_vgg_block_backward_zdp(const void* dnext, int dnext_dtype, int flat,
                                          const void* z, int z_dtype, int B, int T, int F, int C,
                                          int pt, int pf, int ceil_mode, const void* P,
                                          int p_dtype, const uint8_t* slot, const float* gamma,
                                          const float* bn_mean, const float* bn_rstd,
                                          float* dgamma, float* dbeta, float drop,
                                          unsigned long long seed, void* dz, int dz_dtype,
                                          float* dbias, void* workspace, size_t ws_bytes,
                                          void* stream) {
  if (p_dtype == ASR_DT_BF16) {
    ASR_REQUIRE(z_dtype == ASR_DT_BF16 && C % 4 == 0 && ((uintptr_t)P & 7) == 0,
                ASR_ERR_UNSUPPORTED, "vgg_block_backward: bf16 P needs bf16 z and C %% 4 == 0");
    return vgg_block_backward_impl(dnext, dnext_dtype, flat, z, z_dtype, B, T, F, C, pt, pf,
                                   ceil_mode, (const uint16_t*)P, slot, gamma, bn_mean, bn_rstd,
                                   dgamma, dbeta, drop, seed, dz, dz_dtype, dbias, workspace,
                                   ws_bytes, stream);
  }
  ASR_REQUIRE(p_dtype == ASR_DT_F32, ASR_ERR_ARG, "vgg_block_backward: P dtype %d", p_dtype);
  return vgg_block_backward_impl(dnext, dnext_dtype, flat, z, z_dtype, B, T, F, C, pt, pf,
                                 ceil_mode, (const float*)P, slot, gamma, bn_mean, bn_rstd, dgamma,
                                 dbeta, drop, seed, dz, dz_dtype, dbias, workspace, ws_bytes,
                                 stream);
}

extern "C" int asr_vgg_block_backward_zd(const void* dnext_v, int dnext_dtype, int flat,
                                         const void* z, int z_dtype, int B, int T, int F, int C,
                                         int pt, int pf, int ceil_mode, const float* P,
                                         const uint8_t* slot, const float* gamma,
                                         const float* bn_mean, const float* bn_rstd,
                                         float* dgamma, float* dbeta, float drop,
                                         unsigned long long seed, void* dz, int dz_dtype,
                                         float* dbias, void* workspace, size_t ws_bytes,
                                         void* stream) {
  return asr_vgg_block_backward_zdp(dnext_v, dnext_dtype, flat, z, z_dtype, B, T, F, C, pt, pf,
                                    ceil_mode, P, ASR_DT_F32, slot, gamma, bn_mean, bn_rstd,
                                    dgamma, dbeta, drop, seed, dz, dz_dtype, dbias, workspace,
                                    ws_bytes, stream);
}

extern "C" int asr_vgg_block_backward_z(const float* dnext, int flat, const void* z,
                                        int z_dtype, int B, int T, int F, int C, int pt, int pf,
                                        int ceil_mode, const float* P, const uint8_t* slot,
                                        const float* gamma, const float* bn_mean,
                                        const float* bn_rstd, float* dgamma, float* dbeta,
                                        float drop, unsigned long long seed, void* dz,
                                        int dz_dtype, float* dbias, void* workspace,
                                        size_t ws_bytes, void* stream) {
  return asr_vgg_block_backward_zd(dnext, ASR_DT_F32, flat, z, z_dtype, B, T, F, C, pt, pf,
                                   ceil_mode, P, slot, gamma, bn_mean, bn_rstd, dgamma, dbeta,
                                   drop, seed, dz, dz_dtype, dbias, workspace, ws_bytes, stream);
}
