// Teacher-forced location-attention decoder loop on gfx950 -- the sequential
// part of AttentionSeq2seq._decode_train (attention_seq2seq.py:704-799) with
// the bahdanau order, one LSTMCell layer (rnn_decoder.py:63-113) and location
// attention (attention_layer.py:74-98, 155-251).
//
// Everything that does not depend on the recurrence is hoisted out of the
// loop by the host into large GEMMs (the embedding projection of all steps,
// W_enc, the bottleneck W_d / W_c, the output layer fc and their gradients),
// so the per-step sequential work is exactly two kernels forward:
//   cell_fwd : gates = pre_emb[t] + [ctx_{t-1}; h_{t-1}] @ Wcat^T, Wcat = [W_ih_ctx | W_hh]
//              (16 gate columns x 32 utterances per work-group, MFMA, 4 waves split K)
//   att_fwd  : one work-group per utterance: conv(aw_{t-1}) -> energy
//              V.tanh(enc_a + W_dec h + W_conv f) -> multiplicative mask, sharpen,
//              softmax -> context = sum_t aw enc (enc/enc_a stay L2/MALL resident)
// and three backward:
//   r        = dgates_{t+1} @ Wcat       (asr_gemm; d ctx_t and d h_t from step t+1)
//   att_bwd  : softmax / tanh / conv backward, per-step partial weight gradients
//   cell_bwd : LSTMCell backward, dgates written over the saved gates
// Bahdanau quirk (attention_seq2seq.py:750-759): at t = 0 there is no cell step;
// the first attention uses the initial state h0.
#include <string.h>

#include "mfma.h"
#include "prof.h"

namespace asr {
namespace {

struct Dims {
  int B, T, E, A, C, K, D, S;
  float sharpen;
  int sigmoid;
};

inline Dims to_dims(const asr_attdec_dims_t& d) {
  return Dims{d.B, d.T, d.E, d.A, d.C, d.K, d.D, d.S, d.sharpening, d.sigmoid_smoothing};
}

constexpr int MB = 32;   // utterances per cell work-group
constexpr int CU = 4;    // hidden units per cell work-group (16 gate columns)
constexpr int ATT_THREADS = 512;   // 8 waves: two per SIMD hide the per-frame latencies

template <typename T>
__device__ __forceinline__ float ldw(const T* p, long long i);
template <>
__device__ __forceinline__ float ldw<float>(const float* p, long long i) { return p[i]; }
template <>
__device__ __forceinline__ float ldw<uint16_t>(const uint16_t* p, long long i) { return bf2f(p[i]); }

template <typename T>
__device__ __forceinline__ bf16x8 frag8g(const T* row, int k, int klim, bool vec) {
  if (row == nullptr) return as_bf16x8(u16x8{0, 0, 0, 0, 0, 0, 0, 0});
  if (vec && k + 8 <= klim) {
    if constexpr (sizeof(T) == 2) return load_bf16x8((const uint16_t*)row + k);
    else return load_bf16x8_from_f32((const float*)row + k);
  }
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (k + j < klim) ? f2bf(ldw<T>(row, k + j)) : (uint16_t)0;
  return as_bf16x8(r);
}

// acc0/acc1 += rows xr0/xr1 (K floats) x row wr (K weights), this wave's k
// steps (wave * 32 + 128 j for bf16 MFMA, wave * 4 + 16 j for f32 MFMA) in the
// same order as a plain loop, but with the fragments of NB steps loaded before
// their MFMAs: one memory round trip per NB steps instead of one per step.
template <bool BF16, typename TW>
__device__ __forceinline__ void rows_mma(const float* xr0, const float* xr1, const TW* wr, int K,
                                         int wave, int lane, bool vec, f32x4& acc0, f32x4& acc1) {
  if constexpr (BF16) {
    constexpr int NB = 4;
    for (int kb = wave * 32; kb < K; kb += 128 * NB) {
      bf16x8 fw[NB], f0[NB], f1[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const bool live = kb + 128 * j < K;
        const int k = kb + 128 * j + 8 * (lane >> 4);
        fw[j] = frag8g<TW>(live ? wr : nullptr, k, K, vec);
        f0[j] = frag8g<float>(live ? xr0 : nullptr, k, K, vec);
        f1[j] = frag8g<float>(live ? xr1 : nullptr, k, K, vec);
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (kb + 128 * j < K) {   // wave-uniform
          acc0 = mfma_bf16(f0[j], fw[j], acc0);
          acc1 = mfma_bf16(f1[j], fw[j], acc1);
        }
      }
    }
  } else {
    constexpr int NB = 8;
    for (int kb = wave * 4; kb < K; kb += 16 * NB) {
      float w[NB], x0[NB], x1[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int k = kb + 16 * j + (lane >> 4);
        w[j] = (wr && k < K) ? ldw<TW>(wr, k) : 0.f;
        x0[j] = (xr0 && k < K) ? xr0[k] : 0.f;
        x1[j] = (xr1 && k < K) ? xr1[k] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (kb + 16 * j < K) {   // wave-uniform
          acc0 = mfma_f32(x0[j], w[j], acc0);
          acc1 = mfma_f32(x1[j], w[j], acc1);
        }
      }
    }
  }
}

// -------------------------------------------------------------- init kernel
// dec[b,0] = h0, x[b,1,E:] = h0, c[b,0] = 0, gates[b,0,:] = 0
__global__ void dec_init(Dims d, const float* __restrict__ h0, float* __restrict__ dec,
                         float* __restrict__ x, float* __restrict__ c, float* __restrict__ gates) {
  const int b = blockIdx.x;
  const int ED = d.E + d.D;
  for (int j = threadIdx.x; j < d.D; j += blockDim.x) {
    const float h = h0 ? h0[(long long)b * d.D + j] : 0.f;
    dec[((long long)b * d.S) * d.D + j] = h;
    c[((long long)b * d.S) * d.D + j] = 0.f;
    if (d.S > 1) x[((long long)b * d.S + 1) * ED + d.E + j] = h;
  }
  for (int j = threadIdx.x; j < 4 * d.D; j += blockDim.x) gates[((long long)b * d.S) * 4 * d.D + j] = 0.f;
  for (int j = threadIdx.x; j < ED; j += blockDim.x) x[((long long)b * d.S) * ED + j] = 0.f;
}

// Wcat[g][0:E] = w_ih[g][emb : emb+E] (row stride ld_ih), Wcat[g][E:] = w_hh[g][:]
template <typename TO>
__global__ void build_wcat(Dims d, const float* __restrict__ w_ih_ctx, long long ld_ih,
                           const float* __restrict__ w_hh, TO* __restrict__ out) {
  const int ED = d.E + d.D;
  const long long n = 4LL * d.D * ED;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long g = i / ED;
    const int k = (int)(i % ED);
    const float v = k < d.E ? w_ih_ctx[g * ld_ih + k] : w_hh[g * d.D + (k - d.E)];
    if constexpr (sizeof(TO) == 2) out[i] = f2bf(v);
    else out[i] = v;
  }
}

// Zcat[z][0:E] = W_c[z][:], Zcat[z][E:] = W_d[z][:] (z < Dz): the bottleneck rows
// of a sampled step's z = W_c ctx + W_d h, in Wcat's column layout
template <typename TO>
__global__ void build_zcat(Dims d, int Dz, const float* __restrict__ w_c,
                           const float* __restrict__ w_d, TO* __restrict__ out) {
  const int ED = d.E + d.D;
  const long long n = (long long)Dz * ED;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long z = i / ED;
    const int k = (int)(i % ED);
    const float v = k < d.E ? w_c[z * d.E + k] : w_d[z * d.D + (k - d.E)];
    if constexpr (sizeof(TO) == 2) out[i] = f2bf(v);
    else out[i] = v;
  }
}

// Wcat^T[n][g] (n < E + D): the backward's per-step r = dgates @ Wcat reads rows
template <typename TO>
__global__ void build_wcat_t(Dims d, const float* __restrict__ w_ih_ctx, long long ld_ih,
                             const float* __restrict__ w_hh, TO* __restrict__ out) {
  const int ED = d.E + d.D, G = 4 * d.D;
  const long long n = (long long)G * ED;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int col = (int)(i / G);
    const long long g = i % G;
    const float v = col < d.E ? w_ih_ctx[g * ld_ih + col] : w_hh[g * d.D + (col - d.E)];
    if constexpr (sizeof(TO) == 2) out[i] = f2bf(v);
    else out[i] = v;
  }
}

// -------------------------------------------------------------- cell forward
template <bool BF16, typename TW>
__global__ void __launch_bounds__(256) cell_fwd(int t, Dims d, const TW* __restrict__ wcat,
                                                const float* __restrict__ pre_emb,
                                                float* __restrict__ x, float* __restrict__ gates,
                                                float* __restrict__ c_all, float* __restrict__ dec,
                                                int vec, float drop_h, unsigned long long seed_h) {
  __shared__ float part[4][MB][16];
  const int ED = d.E + d.D, G = 4 * d.D;
  const int u0 = blockIdx.x * CU, b0 = blockIdx.y * MB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ra = b0 + (lane & 15), rb = b0 + 16 + (lane & 15);
  const float* xr0 = ra < d.B ? x + ((long long)ra * d.S + t) * ED : nullptr;
  const float* xr1 = rb < d.B ? x + ((long long)rb * d.S + t) * ED : nullptr;
  const int n = lane & 15, g = n >> 2, u = u0 + (n & 3);
  const TW* wr = u < d.D ? wcat + (long long)(g * d.D + u) * ED : nullptr;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  rows_mma<BF16, TW>(xr0, xr1, wr, ED, wave, lane, vec != 0, acc0, acc1);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    part[wave][4 * (lane >> 4) + r][lane & 15] = acc0[r];
    part[wave][16 + 4 * (lane >> 4) + r][lane & 15] = acc1[r];
  }
  __syncthreads();
  if (threadIdx.x >= MB * CU) return;
  const int row = threadIdx.x >> 2, uu = threadIdx.x & 3;
  const int b = b0 + row, j = u0 + uu;
  if (b >= d.B || j >= d.D) return;
  const long long gb = ((long long)b * d.S + t) * G + j;
  float pre[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    pre[q] = part[0][row][q * 4 + uu] + part[1][row][q * 4 + uu] + part[2][row][q * 4 + uu] +
             part[3][row][q * 4 + uu] + pre_emb[gb + (long long)q * d.D];
  const float cprev = c_all[((long long)b * d.S + t - 1) * d.D + j];
  const float ig = sigmoidf_(pre[0]), fg = sigmoidf_(pre[1]);
  const float gg = tanhf_(pre[2]), og = sigmoidf_(pre[3]);
  const float c = fg * cprev + ig * gg;
  float h = og * tanhf_(c);
  if (drop_h > 0.f) h *= drop_scale(drop_h, seed_h, ((unsigned long long)b * d.S + t) * d.D + j);
  c_all[((long long)b * d.S + t) * d.D + j] = c;
  dec[((long long)b * d.S + t) * d.D + j] = h;
  gates[gb] = ig;
  gates[gb + d.D] = fg;
  gates[gb + 2 * d.D] = gg;
  gates[gb + 3 * d.D] = og;
  if (t + 1 < d.S) x[((long long)b * d.S + t + 1) * ED + d.E + j] = h;
}

// -------------------------------------------------------- attention kernels
// The location-attention step is spread over (frame chunk, utterance) work
// groups -- TCH frames each -- instead of one work-group per utterance, so a
// B = 32 batch at T' = 250 fills 256 work-groups.  The only cross-chunk
// dependencies of a step are the softmax over T (recomputed per work-group
// from the [B][T] energies, which costs T flops) and the 201-tap convolution
// windows (read from the previous kernel's output).  Forward per step:
//   att_energy  (chunk, b): W_dec h, conv(aw_{t-1}) features, energies, mask, sharpen
//   att_context (E chunk, b): softmax (or sigmoid) over T, context slice
// Backward per step:
//   rgemm            : r = dgates_{t+1} @ Wcat (d [ctx_t; h_t] from step t+1)
//   att_bwd_daw      (chunk, b): d ctx total, d aw_t = carry + enc . d ctx
//   att_bwd_energy   (chunk, b): softmax / tanh backward, d enc_a, dF, weight partials
//   att_bwd_conv     (chunk, b): d aw_{t-1} (conv transpose), conv-kernel partials,
//                                (chunk 0) dW_dec input sum and d dec
constexpr int TCH = 32;   // frames per attention work-group
constexpr int ATT_WAVES = ATT_THREADS / 64;
constexpr int FPW = TCH / ATT_WAVES;   // frames per wave
constexpr int ECH = 64;   // context columns per work-group

inline int att_chunks(const Dims& d) { return (d.T + TCH - 1) / TCH; }
// rows per utterance of the backward's weight-gradient partials: the per-step
// kernels' frame chunks or the persistent pass's 8, whichever is more (rows a
// pass does not write are zero)
inline int part_rows(const Dims& d) { return att_chunks(d) > 8 ? att_chunks(d) : 8; }

struct EnLds {
  float* h;     // [D]      dec_out_t
  float* wd;    // [A]      W_dec h
  float* cw;    // [C*K]    conv kernel
  float* wc;    // [A*C]    W_conv
  float* v;     // [A]
  float* awin;  // [TCH+K-1] aw_{t-1}[tt0 - K/2 + i] (0 outside [0, T))
  float* f;     // [TCH*C]  conv features of the chunk
  float* e;     // [TCH]    d energy (backward)
  float* awt;   // [T]      aw_t (backward)
  float* red;   // [64]
  float* cmb;   // [2A + A*C] wave-combine of the backward partials
};

__host__ __device__ inline size_t conv_lds_floats(const Dims& d) {
  return (size_t)d.C * d.K + (size_t)(TCH + d.K - 1) * (d.C + 1) + d.A + (size_t)TCH * d.C +
         ATT_THREADS;
}

__host__ __device__ inline size_t en_lds_floats(const Dims& d) {
  return (size_t)d.D + 2 * d.A + (size_t)d.C * d.K + (size_t)d.A * d.C + (TCH + d.K - 1) +
         (size_t)TCH * d.C + TCH + d.T + 64 + 2 * d.A + (size_t)d.A * d.C;
}

__device__ inline EnLds carve_en(float* s, const Dims& d) {
  EnLds L;
  L.h = s; s += d.D;
  L.wd = s; s += d.A;
  L.cw = s; s += (size_t)d.C * d.K;
  L.wc = s; s += (size_t)d.A * d.C;
  L.v = s; s += d.A;
  L.awin = s; s += TCH + d.K - 1;
  L.f = s; s += (size_t)TCH * d.C;
  L.e = s; s += TCH;
  L.awt = s; s += d.T;
  L.red = s; s += 64;
  L.cmb = s;
  return L;
}

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = is_max ? wave_max(v) : wave_sum(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < nw; ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
  __syncthreads();
  return r;
}

// Diagnostics: phase stamps (s_memrealtime, 100 MHz) of work-group (0, 0) at
// decoder step ATT_TR_STEP, read by asr_att_trace_read.
__device__ unsigned long long g_att_tr[64];
constexpr int ATT_TR_STEP = 10;
#define ATT_TR(k)                                                                     \
  do {                                                                                \
    if (t == ATT_TR_STEP && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)   \
      g_att_tr[k] = __builtin_amdgcn_s_memrealtime();                                 \
  } while (0)

// sum_{i < n} x[i * sx] y[i * sy] over LDS with eight products in flight (four
// partial sums): the conv windows' serial dot products were LDS-latency-bound.
__device__ __forceinline__ float dot_lds(const float* x, int sx, const float* y, int sy, int n) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    float a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = x[(long long)(i + j) * sx];
      b[j] = y[(long long)(i + j) * sy];
    }
    s0 += a[0] * b[0] + a[4] * b[4];
    s1 += a[1] * b[1] + a[5] * b[5];
    s2 += a[2] * b[2] + a[6] * b[6];
    s3 += a[3] * b[3] + a[7] * b[7];
  }
  for (; i < n; ++i) s0 += x[(long long)i * sx] * y[(long long)i * sy];
  return (s0 + s1) + (s2 + s3);
}

// Global -> LDS copy of up to four arrays in which each thread issues all of
// its loads (16 per pass) before its first LDS store: one memory round trip for
// up to 16 * blockDim.x floats instead of one per loop iteration.  The per-step
// attention kernels are latency-bound (SQ_WAIT_ANY was 2/3 of their wave
// cycles): every global read is batched like this or prefetched whole.
struct LdsSeg {
  float* dst;
  const float* src;
  int n;
};
__device__ __forceinline__ void lds_fill(const LdsSeg& s0, const LdsSeg& s1, const LdsSeg& s2,
                                         const LdsSeg& s3) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const int c1 = s0.n, c2 = c1 + s1.n, c3 = c2 + s2.n, total = c3 + s3.n;
  for (int base = 0; base < total; base += 16 * nt) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int i = base + j * nt + tid;
      v[j] = i < c1 ? s0.src[i] : i < c2 ? s1.src[i - c1] : i < c3 ? s2.src[i - c2]
           : i < total ? s3.src[i - c3] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int i = base + j * nt + tid;
      if (i < c1) s0.dst[i] = v[j];
      else if (i < c2) s1.dst[i - c1] = v[j];
      else if (i < c3) s2.dst[i - c2] = v[j];
      else if (i < total) s3.dst[i - c3] = v[j];
    }
  }
}

// Weights, h_t (or the precomputed W_dec h_t rows), W_dec h_t, the aw_{t-1}
// window and the chunk's conv features.
__device__ void en_prologue(int t, const Dims& d, int b, int tt0, const EnLds& L,
                            const float* __restrict__ w_dec, const float* __restrict__ w_conv,
                            const float* __restrict__ conv_w, const float* __restrict__ vw,
                            const float* __restrict__ dec, const float* __restrict__ aw_all,
                            const float* __restrict__ wd_pre = nullptr, int trb = 0) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const int half = d.K / 2;
  ATT_TR(trb + 0);
  float awv[2];   // the window (TCH + K - 1 <= 2 * blockDim.x) rides with the batch
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = tid + j * nt, tt = tt0 - half + i;
    awv[j] = (i < TCH + d.K - 1 && t > 0 && tt >= 0 && tt < d.T)
                 ? aw_all[((long long)b * d.S + t - 1) * d.T + tt] : 0.f;
  }
  // backward: W_dec h_t of every step from one GEMM before the loop
  const LdsSeg last = wd_pre ? LdsSeg{L.wd, wd_pre + ((long long)b * d.S + t) * d.A, d.A}
                             : LdsSeg{L.h, dec + ((long long)b * d.S + t) * d.D, d.D};
  lds_fill(LdsSeg{L.wc, w_conv, d.A * d.C}, LdsSeg{L.cw, conv_w, d.C * d.K},
           LdsSeg{L.v, vw, d.A}, last);
#pragma unroll
  for (int j = 0; j < 2; ++j)
    if (tid + j * nt < TCH + d.K - 1) L.awin[tid + j * nt] = awv[j];
  __syncthreads();
  ATT_TR(trb + 1);
  if (!wd_pre) {
    // W_dec h_t: (row a, K slice qk) per thread, ten float4 of the row in flight
    // per round, slices summed through L.cmb (2A + A C floats: nq <= 2 + C)
    const int a = tid % d.A, qk = tid / d.A;
    const int nq = min(nt / d.A, 2 + d.C);                    // >= 1 (A <= 256)
    float s = 0.f;
    if (qk < nq && (d.D & 3) == 0) {
      const int kq = ((d.D / 4 + nq - 1) / nq) * 4;           // K per quarter (mult of 4)
      const int k0 = qk * kq, k1 = min(d.D, k0 + kq);
      const float* wr = w_dec + (long long)a * d.D;
      for (int kb = k0; kb < k1; kb += 40) {
        float4 u[10];
#pragma unroll
        for (int j = 0; j < 10; ++j)
          u[j] = kb + 4 * j < k1 ? *reinterpret_cast<const float4*>(wr + kb + 4 * j)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < 10; ++j) {
          const int k = kb + 4 * j;
          if (k < k1)
            s += u[j].x * L.h[k] + u[j].y * L.h[k + 1] + u[j].z * L.h[k + 2] +
                 u[j].w * L.h[k + 3];
        }
      }
    } else if (qk == 0) {
      const float* wr = w_dec + (long long)a * d.D;
      for (int k = 0; k < d.D; ++k) s += wr[k] * L.h[k];
    }
    if (qk < nq) L.cmb[qk * d.A + a] = s;
    __syncthreads();
    for (int r = tid; r < d.A; r += nt) {
      float v = L.cmb[r];
      for (int q = 1; q < nq && (d.D & 3) == 0; ++q) v += L.cmb[q * d.A + r];
      L.wd[r] = v;
    }
  }
  ATT_TR(trb + 2);
  for (int i = tid; i < TCH * d.C; i += nt) {
    const int fi = i / d.C, c = i % d.C;
    float s = 0.f;
    if (tt0 + fi < d.T) {
      const float* cwr = L.cw + c * d.K;
      const float* aw = L.awin + fi;        // aw_{t-1}[tt - half + k] = awin[fi + k]
      s = dot_lds(cwr, 1, aw, 1, d.K);
    }
    L.f[i] = s;
  }
  __syncthreads();
  ATT_TR(trb + 3);
}

template <int CC>
__global__ void __launch_bounds__(ATT_THREADS) att_energy(
    int t, Dims d, const float* __restrict__ enc_a, const int32_t* __restrict__ lens,
    const float* __restrict__ w_dec, const float* __restrict__ w_conv,
    const float* __restrict__ conv_w, const float* __restrict__ vw, const float* __restrict__ dec,
    const float* __restrict__ aw_all, float* __restrict__ ebuf) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Dims dd = d;
  EnLds L = carve_en(smem, dd);
  const int b = blockIdx.y, tt0 = blockIdx.x * TCH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // one wave per frame (frames w + FPW_STRIDE f), lanes over the attention dim
  // (a = lane + 64 q, A <= 256): every enc_a row this wave needs is loaded
  // before the prologue, so its latency overlaps the prologue's
  float ea[FPW][4];
#pragma unroll
  for (int f = 0; f < FPW; ++f) {
    const int tt = tt0 + w + ATT_WAVES * f;
    const float* er = enc_a + ((long long)b * d.T + tt) * d.A;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int a = lane + 64 * q;
      ea[f][q] = (tt < d.T && a < d.A) ? er[a] : 0.f;
    }
  }
  en_prologue(t, dd, b, tt0, L, w_dec, w_conv, conv_w, vw, dec, aw_all, nullptr, 0);
  const int len = lens[b];
#pragma unroll
  for (int f = 0; f < FPW; ++f) {
    const int i = w + ATT_WAVES * f;
    const int tt = tt0 + i;
    if (tt >= d.T) break;
    const float* eac = ea[f];
    constexpr int CM = CC ? CC : 16;
    const int C = CC ? CC : d.C;
    float frv[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c) frv[c] = (CC || c < C) ? L.f[i * C + c] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int a = lane + 64 * q;
      if (64 * q < d.A && a < d.A) {
        float p = eac[q] + L.wd[a];
#pragma unroll
        for (int c = 0; c < CM; ++c)
          if (CC || c < C) p += frv[c] * L.wc[a * C + c];
        s += L.v[a] * tanhf(p);
      }
    }
    s = wave_sum(s);
    // multiplicative mask (attention_layer.py:216-225), then sharpening
    if (lane == 0) ebuf[(long long)b * d.T + tt] = (tt < len ? s : 0.f) * d.sharpen;
  }
  ATT_TR(4);
}

__global__ void __launch_bounds__(ATT_THREADS) att_context(
    int t, Dims d, const float* __restrict__ enc, const float* __restrict__ ebuf,
    float* __restrict__ aw_all, float* __restrict__ ctx_all, float* __restrict__ x) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* aw = smem;             // [T]
  float* red = aw + d.T;        // [64]
  float* part = red + 64;       // [ATT_THREADS / ECH][ECH]
  const int b = blockIdx.y, e0 = blockIdx.x * ECH;
  const int tid = threadIdx.x;
  float mx = -__builtin_huge_valf();
  for (int i = tid; i < d.T; i += blockDim.x) {
    const float e = ebuf[(long long)b * d.T + i];
    aw[i] = e;
    mx = fmaxf(mx, e);
  }
  __syncthreads();
  if (d.sigmoid) {
    for (int i = tid; i < d.T; i += blockDim.x) aw[i] = sigmoidf_(aw[i]);
  } else {
    mx = block_reduce(mx, red, true);
    float sm = 0.f;
    for (int i = tid; i < d.T; i += blockDim.x) {
      const float p = __expf(aw[i] - mx);
      aw[i] = p;
      sm += p;
    }
    sm = block_reduce(sm, red, false);
    const float inv = 1.f / sm;
    for (int i = tid; i < d.T; i += blockDim.x) aw[i] *= inv;
  }
  __syncthreads();
  if (blockIdx.x == 0)
    for (int i = tid; i < d.T; i += blockDim.x) aw_all[((long long)b * d.S + t) * d.T + i] = aw[i];
  const int col = tid & (ECH - 1), r = tid / ECH, nr = blockDim.x / ECH;
  const int e = e0 + col;
  float s = 0.f;
  if (e < d.E) {   // sixteen frames' loads in flight per round
    const float* er = enc + (long long)b * d.T * d.E + e;
    for (int tb = r; tb < d.T; tb += 16 * nr) {
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int tt = tb + j * nr;
        v[j] = tt < d.T ? er[(long long)tt * d.E] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int tt = tb + j * nr;
        if (tt < d.T) s += aw[tt] * v[j];
      }
    }
  }
  part[r * ECH + col] = s;
  __syncthreads();
  if (r == 0 && e < d.E) {
    float c = part[col];
    for (int q = 1; q < nr; ++q) c += part[q * ECH + col];
    ctx_all[((long long)b * d.S + t) * d.E + e] = c;
    if (t + 1 < d.S) x[((long long)b * d.S + t + 1) * (d.E + d.D) + e] = c;
  }
}

// r[b][n] = sum_g dg[b, t+1, g] * WcatT[n][g]   (n < E + D; 16 columns x 32 rows
// per work-group, 4 waves split K = 4D; same fragment scheme as cell_fwd)
template <bool BF16, typename TW>
__global__ void __launch_bounds__(256) rgemm(int t1, Dims d, const TW* __restrict__ wT,
                                             const float* __restrict__ dg, float* __restrict__ r,
                                             int vec) {
  __shared__ float part[4][MB][16];
  const int ED = d.E + d.D, G = 4 * d.D;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * MB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ra = b0 + (lane & 15), rb = b0 + 16 + (lane & 15);
  const float* xr0 = ra < d.B ? dg + ((long long)ra * d.S + t1) * G : nullptr;
  const float* xr1 = rb < d.B ? dg + ((long long)rb * d.S + t1) * G : nullptr;
  const int n = n0 + (lane & 15);
  const TW* wr = n < ED ? wT + (long long)n * G : nullptr;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  rows_mma<BF16, TW>(xr0, xr1, wr, G, wave, lane, vec != 0, acc0, acc1);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    part[wave][4 * (lane >> 4) + q][lane & 15] = acc0[q];
    part[wave][16 + 4 * (lane >> 4) + q][lane & 15] = acc1[q];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < MB * 16; i += blockDim.x) {
    const int row = i >> 4, cc = i & 15;
    const int b = b0 + row, nn = n0 + cc;
    if (b < d.B && nn < ED)
      r[(long long)b * ED + nn] = part[0][row][cc] + part[1][row][cc] + part[2][row][cc] +
                                  part[3][row][cc];
  }
}

// d ctx total for step t = d_ctx_in[b,t] + r[b, 0:E] (stored into dctx_tot by chunk 0);
// d aw_t[tt] = carry[b,tt] (from step t+1) + enc[b,tt,:] . d ctx
__global__ void __launch_bounds__(ATT_THREADS) att_bwd_daw(
    int t, Dims d, const float* __restrict__ enc, const float* __restrict__ dctx_in,
    const float* __restrict__ r, const float* __restrict__ carry, float* __restrict__ dctx_tot,
    float* __restrict__ dawbuf) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* dct = smem;   // [E]
  const int b = blockIdx.y, tt0 = blockIdx.x * TCH;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  const int ED = d.E + d.D;
  (void)nw;
  // d ctx: every thread's elements loaded in one round (E <= 4 * blockDim.x
  // per pass)
  for (int e0 = 0; e0 < d.E; e0 += 4 * ATT_THREADS) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = e0 + j * ATT_THREADS + tid;
      v[j] = e < d.E ? dctx_in[((long long)b * d.S + t) * d.E + e] +
                           (r ? r[(long long)b * ED + e] : 0.f)
                     : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = e0 + j * ATT_THREADS + tid;
      if (e < d.E) {
        dct[e] = v[j];
        if (blockIdx.x == 0) dctx_tot[((long long)b * d.S + t) * d.E + e] = v[j];
      }
    }
  }
  __syncthreads();
  // this wave's frames (w + ATT_WAVES f): NE enc elements of every frame in
  // flight per round
  constexpr int NE = 4;
  float s[FPW];
#pragma unroll
  for (int f = 0; f < FPW; ++f) s[f] = 0.f;
  for (int eb = lane; eb < d.E; eb += 64 * NE) {
    float v[FPW][NE];
#pragma unroll
    for (int f = 0; f < FPW; ++f) {
      const int tt = tt0 + w + ATT_WAVES * f;
      const float* er = enc + ((long long)b * d.T + tt) * d.E;
#pragma unroll
      for (int j = 0; j < NE; ++j) {
        const int e = eb + 64 * j;
        v[f][j] = (tt < d.T && e < d.E) ? er[e] : 0.f;
      }
    }
#pragma unroll
    for (int f = 0; f < FPW; ++f)
#pragma unroll
      for (int j = 0; j < NE; ++j) {
        const int e = eb + 64 * j;
        if (e < d.E) s[f] += v[f][j] * dct[e];
      }
  }
#pragma unroll
  for (int f = 0; f < FPW; ++f) {
    const int tt = tt0 + w + ATT_WAVES * f;
    const float v = wave_sum(s[f]);
    if (lane == 0 && tt < d.T) dawbuf[(long long)b * d.T + tt] = carry[(long long)b * d.T + tt] + v;
  }
}

// softmax / sigmoid backward -> d energy; per (frame, a): tanh backward -> d enc_a
// (utterance-private RMW), dF [B][T][C], and chunk partials of dV, dW_dec-input,
// dW_conv (fixed-order sums: deterministic).
// CC: the conv channel count at compile time (0 = runtime d.C <= 16): with it
// the per-frame channel loops are straight-line code over registers.
template <int CC>
__global__ void __launch_bounds__(ATT_THREADS) att_bwd_energy(
    int t, Dims d, const float* __restrict__ enc_a, const int32_t* __restrict__ lens,
    const float* __restrict__ w_dec, const float* __restrict__ w_conv,
    const float* __restrict__ conv_w, const float* __restrict__ vw, const float* __restrict__ dec,
    const float* __restrict__ aw_all, const float* __restrict__ dawbuf,
    const float* __restrict__ wd_all, float* __restrict__ d_enc_a, float* __restrict__ dFbuf,
    float* __restrict__ dwd_chunk, float* __restrict__ dv_part, float* __restrict__ dwc_part) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Dims dd = d;
  EnLds L = carve_en(smem, dd);
  const int b = blockIdx.y, ch = blockIdx.x, tt0 = ch * TCH, NC = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  const float* awt = aw_all + ((long long)b * d.S + t) * d.T;
  const float* daw = dawbuf + (long long)b * d.T;
  ATT_TR(10);
  // every enc_a / d_enc_a row of this wave's frames (w + ATT_WAVES f) is loaded
  // first: its latency overlaps the softmax backward and the prologue
  float ea[FPW][4], dea_in[FPW][4];
#pragma unroll
  for (int f = 0; f < FPW; ++f) {
    const int tt = tt0 + w + ATT_WAVES * f;
    const long long ro = ((long long)b * d.T + tt) * d.A;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int a = lane + 64 * q;
      const bool ok = tt < d.T && a < d.A;
      ea[f][q] = ok ? enc_a[ro + a] : 0.f;
      dea_in[f][q] = ok ? d_enc_a[ro + a] : 0.f;
    }
  }
  float sdot = 0.f;
  for (int i = tid; i < d.T; i += blockDim.x) {
    const float a = awt[i];
    L.awt[i] = a;
    sdot += a * daw[i];
  }
  if (!d.sigmoid) sdot = block_reduce(sdot, L.red, false);
  __syncthreads();
  const int len = lens[b];
  for (int i = tid; i < TCH; i += blockDim.x) {
    const int tt = tt0 + i;
    float de = 0.f;
    if (tt < d.T && tt < len) {
      const float a = L.awt[tt], g = daw[tt];
      de = (d.sigmoid ? g * a * (1.f - a) : a * (g - sdot)) * d.sharpen;
    }
    L.e[i] = de;
  }
  ATT_TR(11);
  en_prologue(t, dd, b, tt0, L, w_dec, w_conv, conv_w, vw, dec, aw_all, wd_all, 12);
  constexpr int CM = CC ? CC : 16;
  const int C = CC ? CC : d.C;
  float accV[4] = {0.f, 0.f, 0.f, 0.f}, accWd[4] = {0.f, 0.f, 0.f, 0.f};
  float accWc[4][CM];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int c = 0; c < CM; ++c) accWc[q][c] = 0.f;
#pragma unroll
  for (int f = 0; f < FPW; ++f) {
    const int i = w + ATT_WAVES * f;
    const int tt = tt0 + i;
    if (tt >= d.T) break;
    const float de = L.e[i];
    const float* eac = ea[f];
    const float* deac = dea_in[f];
    float* dfo = dFbuf + ((long long)b * d.T + tt) * C;
    if (de == 0.f) {               // padded / masked frame: nothing flows
      if (lane < C) dfo[lane] = 0.f;
      continue;
    }
    float* dea = d_enc_a + ((long long)b * d.T + tt) * d.A;
    float frv[CM], dfc[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c) {
      frv[c] = (CC || c < C) ? L.f[i * C + c] : 0.f;
      dfc[c] = 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int a = lane + 64 * q;
      if (64 * q < d.A) {          // wave-uniform
        float wrv[CM];
#pragma unroll
        for (int c = 0; c < CM; ++c) wrv[c] = (a < d.A && (CC || c < C)) ? L.wc[a * C + c] : 0.f;
        float p = eac[q] + (a < d.A ? L.wd[a] : 0.f);
#pragma unroll
        for (int c = 0; c < CM; ++c) p += frv[c] * wrv[c];
        const float th = tanhf(p);
        const float dp = a < d.A ? de * L.v[a] * (1.f - th * th) : 0.f;
        accV[q] += a < d.A ? de * th : 0.f;
        accWd[q] += dp;
        if (a < d.A) dea[a] = deac[q] + dp;
#pragma unroll
        for (int c = 0; c < CM; ++c) {
          accWc[q][c] += dp * frv[c];
          dfc[c] += dp * wrv[c];
        }
      }
    }
#pragma unroll
    for (int c = 0; c < CM; ++c) {
      if (CC || c < C) {
        const float sv = wave_sum(dfc[c]);
        if (lane == 0) dfo[c] = sv;
      }
    }
  }
  ATT_TR(16);
  // combine the per-wave partials in LDS in a fixed wave order, then one store
  // of this chunk's slots
  // this chunk's row of the partials, summed over the steps in backward order
  // (the last step writes, earlier ones add: fixed order, deterministic)
  const long long slot = (long long)b * NC + ch;
  const bool first = t == d.S - 1;
  float* cV = L.cmb;                  // [A]
  float* cWd = cV + d.A;              // [A]
  float* cWc = cWd + d.A;             // [A*C]
  for (int pass = 0; pass < nw; ++pass) {
    if (w == pass) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int a = lane + 64 * q;
        if (a < d.A) {
          cV[a] = pass ? cV[a] + accV[q] : accV[q];
          cWd[a] = pass ? cWd[a] + accWd[q] : accWd[q];
#pragma unroll
          for (int c = 0; c < CM; ++c)
            if (CC || c < C) cWc[a * C + c] = pass ? cWc[a * C + c] + accWc[q][c] : accWc[q][c];
        }
      }
    }
    __syncthreads();
  }
  float* dvp = dv_part + slot * d.A;
  float* dwcp = dwc_part + slot * d.A * d.C;
  float* dwdp = dwd_chunk + ((long long)b * NC + ch) * d.A;
  for (int i = tid; i < d.A; i += blockDim.x) {
    dvp[i] = first ? cV[i] : dvp[i] + cV[i];
    dwdp[i] = cWd[i];
  }
  for (int i = tid; i < d.A * d.C; i += blockDim.x) dwcp[i] = first ? cWc[i] : dwcp[i] + cWc[i];
  ATT_TR(17);
}

// d aw_{t-1} (conv transpose of dF; written over carry for step t-1), this
// chunk's conv-kernel partial, and (chunk 0) the dW_dec input sum dwd_all[b,t]
// and d dec_t from the attention (ddec_att = W_dec^T dWd).
__global__ void __launch_bounds__(ATT_THREADS) att_bwd_conv(
    int t, Dims d, const float* __restrict__ conv_w, const float* __restrict__ aw_all,
    const float* __restrict__ dFbuf, const float* __restrict__ w_dec,
    const float* __restrict__ dwd_chunk, float* __restrict__ carry, float* __restrict__ dcw_part,
    float* __restrict__ dwd_all, float* __restrict__ ddec_att) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int W = TCH + d.K - 1;
  float* cw = smem;                        // [C*K]
  float* dFw = cw + d.C * d.K;             // [W][C] rows j0 - half ..
  float* awin = dFw + (size_t)W * d.C;     // [W]   aw_{t-1}[j0 - half + i]
  float* dWd = awin + W;                   // [A]
  float* cpart = dWd + d.A;                // [TCH][C]
  float* dred = cpart + TCH * d.C;         // [blockDim.x] d dec slice partials
  const int b = blockIdx.y, ch = blockIdx.x, j0 = ch * TCH, NC = gridDim.x;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int half = d.K / 2;
  ATT_TR(20);
  // conv kernel, the dF window and the aw_{t-1} window in batched rounds (16
  // loads in flight per thread), zero outside [0, T)
  {
    const int n1 = d.C * d.K, n2 = n1 + W * d.C, total = n2 + W;
    const long long dfb = ((long long)b * d.T + j0 - half) * d.C;   // dF row j0 - half, col 0
    const float* awp = aw_all + ((long long)b * d.S + t - 1) * d.T + (j0 - half);
    for (int base = 0; base < total; base += 16 * nt) {
      float v[16];
#pragma unroll
      for (int jx = 0; jx < 16; ++jx) {
        const int i = base + jx * nt + tid;
        float x = 0.f;
        if (i < n1) {
          x = conv_w[i];
        } else if (i < n2) {
          const int row = j0 - half + (i - n1) / d.C;
          if (row >= 0 && row < d.T) x = dFbuf[dfb + (i - n1)];
        } else if (i < total) {
          const int tt = j0 - half + (i - n2);
          if (t > 0 && tt >= 0 && tt < d.T) x = awp[i - n2];
        }
        v[jx] = x;
      }
#pragma unroll
      for (int jx = 0; jx < 16; ++jx) {
        const int i = base + jx * nt + tid;
        if (i < n1) cw[i] = v[jx];
        else if (i < n2) dFw[i - n1] = v[jx];
        else if (i < total) awin[i - n2] = v[jx];
      }
    }
  }
  __syncthreads();
  ATT_TR(21);
  // d aw_{t-1}[j] = sum_c sum_k dF[j - k + half, c] cw[c, k]; window row of j - k + half
  // is (j - j0) + (K - 1) - k
  for (int i = tid; i < TCH * d.C; i += nt) {   // one thread per (frame, channel)
    const int jj = i / d.C, c = i % d.C;
    float s = 0.f;
    if (j0 + jj < d.T) {
      const float* cwr = cw + c * d.K;
      const float* dfr = dFw + (size_t)(jj + d.K - 1) * d.C + c;
      s = dot_lds(dfr, -d.C, cwr, 1, d.K);
    }
    cpart[i] = s;
  }
  __syncthreads();
  ATT_TR(22);
  for (int jj = tid; jj < TCH; jj += nt) {
    const int j = j0 + jj;
    if (j >= d.T) break;
    float s = 0.f;
    for (int c = 0; c < d.C; ++c) s += cpart[jj * d.C + c];
    carry[(long long)b * d.T + j] = s;
  }
  // conv-kernel partial: dcw[c, k] = sum_{tt in chunk} dF[tt, c] aw_{t-1}[tt + k - half]
  // (row b * NC + ch, summed over the steps like att_bwd_energy's partials)
  float* dcwp = dcw_part + ((long long)b * NC + ch) * d.C * d.K;
  const bool first = t == d.S - 1;
  const int nrow = min(TCH, d.T - j0);
  for (int i = tid; i < d.C * d.K; i += nt) {
    const int c = i / d.K, k = i % d.K;
    float s = 0.f;
    s = dot_lds(dFw + (size_t)half * d.C + c, d.C, awin + k, 1, nrow);
    dcwp[i] = first ? s : dcwp[i] + s;
  }
  ATT_TR(24);
  // dW_dec input of step t (sum of the chunks' partials: every chunk forms it,
  // chunk 0 stores it) and d dec_t = W_dec^T dWd, its D outputs split over the
  // utterance's NC chunk work-groups: (output k, slice of A) per thread
  for (int a = tid; a < d.A; a += nt) {
    float s = 0.f;
    for (int q = 0; q < NC; ++q) s += dwd_chunk[((long long)b * NC + q) * d.A + a];
    dWd[a] = s;
    if (ch == 0) dwd_all[((long long)b * d.S + t) * d.A + a] = s;
  }
  __syncthreads();
  ATT_TR(23);
  const int KS = (d.D + NC - 1) / NC, k0 = ch * KS, nk = min(KS, d.D - k0);
  if (nk > 0 && KS > nt) {   // few chunks, wide decoder: whole-A sums per output
    for (int k = tid; k < nk; k += nt) {
      float v = 0.f;
      for (int a = 0; a < d.A; ++a) v += w_dec[(long long)a * d.D + k0 + k] * dWd[a];
      ddec_att[(long long)b * d.D + k0 + k] = v;
    }
  } else if (nk > 0) {
    const int ns = max(1, min(nt / KS, d.A));            // A slices
    const int kk = tid % KS, sl = tid / KS;
    const int AS = (d.A + ns - 1) / ns, a0 = sl * AS, a1 = min(d.A, a0 + AS);
    float sacc = 0.f;
    if (sl < ns && kk < nk) {
      for (int ab = a0; ab < a1; ab += 16) {   // sixteen W_dec rows in flight per round
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j)
          v[j] = ab + j < a1 ? w_dec[(long long)(ab + j) * d.D + k0 + kk] : 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (ab + j < a1) sacc += v[j] * dWd[ab + j];
      }
    }
    if (sl < ns) dred[sl * KS + kk] = sacc;
    __syncthreads();
    for (int k = tid; k < nk; k += nt) {
      float v = dred[k];
      for (int q = 1; q < ns; ++q) v += dred[q * KS + k];
      ddec_att[(long long)b * d.D + k0 + k] = v;
    }
  }
  ATT_TR(26);
}

// -------------------------------------------------------------- cell backward
// dh = d_dec_in[b,t] + r[b, E:] + ddec_att[b];  writes dgates over gates (t >= 1),
// or d_h0 (t == 0).
__global__ void cell_bwd(int t, Dims d, const float* __restrict__ d_dec_in,
                         const float* __restrict__ r, const float* __restrict__ ddec_att,
                         float* __restrict__ gates, const float* __restrict__ c_all,
                         float* __restrict__ dc, float* __restrict__ d_h0, float drop_h,
                         unsigned long long seed_h) {
  const int ED = d.E + d.D, G = 4 * d.D;
  const long long n = (long long)d.B * d.D;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / d.D), j = (int)(i % d.D);
    const float dh = d_dec_in[((long long)b * d.S + t) * d.D + j] +
                     (r ? r[(long long)b * ED + d.E + j] : 0.f) + ddec_att[i];
    if (t == 0) {
      if (d_h0) d_h0[i] = dh;
      continue;
    }
    // dh is w.r.t. the dropped h (dec_out and the recurrent state): back through the mask
    const float dhr =
        drop_h > 0.f ? dh * drop_scale(drop_h, seed_h, ((unsigned long long)b * d.S + t) * d.D + j)
                     : dh;
    const long long gb = ((long long)b * d.S + t) * G + j;
    const float ig = gates[gb], fg = gates[gb + d.D], gg = gates[gb + 2 * d.D],
                og = gates[gb + 3 * d.D];
    const float c = c_all[((long long)b * d.S + t) * d.D + j];
    const float cp = c_all[((long long)b * d.S + t - 1) * d.D + j];
    const float tc = tanhf(c);
    const float dcell = dc[i] + dhr * og * (1.f - tc * tc);
    gates[gb] = dcell * gg * ig * (1.f - ig);
    gates[gb + d.D] = dcell * cp * fg * (1.f - fg);
    gates[gb + 2 * d.D] = dcell * ig * (1.f - gg * gg);
    gates[gb + 3 * d.D] = dhr * tc * og * (1.f - og);
    dc[i] = dcell * fg;
  }
}

// ------------------------------------------------------ scheduled sampling
// One work-group per utterance, before the cell of a sampled step t >= 1:
// logits_{t-1} = fc(tanh(drop_d(W_d dec_{t-1} + b_d) + drop_c(W_c ctx_{t-1} + b_c))),
// tok = first argmax, e = drop_emb(emb(tok)), pre_ss[b,t] = W_ih[:, :Y] e + b_ih + b_hh.
constexpr int SS_THREADS = 256;

__global__ void __launch_bounds__(SS_THREADS) ss_step(int t, Dims d, asr_attdec_opts_t o,
                                                      const float* __restrict__ dec,
                                                      const float* __restrict__ ctx_all) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* h = sm;              // [D]
  float* cx = h + d.D;        // [E]
  float* z = cx + d.E;        // [Dz]
  float* e = z + o.Dz;        // [Y]
  float* rv = e + o.Y;        // [SS_THREADS / 64] best values
  int* ri = (int*)(rv + SS_THREADS / 64);
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = SS_THREADS / 64;
  const long long prev = (long long)b * d.S + (t - 1);
  for (int i = tid; i < d.D; i += SS_THREADS) h[i] = dec[prev * d.D + i];
  for (int i = tid; i < d.E; i += SS_THREADS) cx[i] = ctx_all[prev * d.E + i];
  __syncthreads();
  for (int k = w; k < o.Dz; k += nw) {   // one wave per bottleneck unit, lanes over K
    const float* wd = o.w_d + (long long)k * d.D;
    const float* wc = o.w_c + (long long)k * d.E;
    float sa = 0.f, sc = 0.f;
    for (int j = lane; j < d.D; j += 64) sa += wd[j] * h[j];
    for (int j = lane; j < d.E; j += 64) sc += wc[j] * cx[j];
    sa = wave_sum(sa);
    sc = wave_sum(sc);
    if (lane == 0) {
      float a = sa + (o.b_d ? o.b_d[k] : 0.f), c = sc + (o.b_c ? o.b_c[k] : 0.f);
      const unsigned long long idx = (unsigned long long)prev * o.Dz + k;
      if (o.drop_d > 0.f) a *= drop_scale(o.drop_d, o.seed_d, idx);
      if (o.drop_c > 0.f) c *= drop_scale(o.drop_c, o.seed_c, idx);
      z[k] = tanhf(a + c);
    }
  }
  __syncthreads();
  float best = -__builtin_huge_valf();
  int bi = 0x7fffffff;
  for (int v = w; v < o.V; v += nw) {    // one wave per class; classes ascending per wave
    const float* wr = o.w_fc + (long long)v * o.Dz;
    float s = 0.f;
    for (int k = lane; k < o.Dz; k += 64) s += wr[k] * z[k];
    s = wave_sum(s) + (o.b_fc ? o.b_fc[v] : 0.f);
    if (s > best) { best = s; bi = v; }   // strict: the first maximum wins
  }
  if (lane == 0) { rv[w] = best; ri[w] = bi; }
  __syncthreads();
  float bv = rv[0];
  int tok = ri[0];
  for (int i = 1; i < nw; ++i)
    if (rv[i] > bv || (rv[i] == bv && ri[i] < tok)) { bv = rv[i]; tok = ri[i]; }
  const long long cur = (long long)b * d.S + t;
  for (int y = tid; y < o.Y; y += SS_THREADS) {
    float ev = o.emb_trans ? o.emb_w[(long long)y * o.V + tok] : o.emb_w[(long long)tok * o.Y + y];
    if (o.drop_emb > 0.f) ev *= drop_scale(o.drop_emb, o.seed_emb, (unsigned long long)cur * o.Y + y);
    e[y] = ev;
    o.emb_ss[cur * o.Y + y] = ev;
  }
  if (tid == 0 && o.tok_ss) o.tok_ss[cur] = tok;
  __syncthreads();
  const int G = 4 * d.D;
  for (int g = tid; g < G; g += SS_THREADS) {
    const float* wr = o.w_ih_emb + (long long)g * o.ld_ih;
    float s = o.b_ih[g] + o.b_hh[g];
    for (int y = 0; y < o.Y; ++y) s += wr[y] * e[y];
    o.pre_ss[cur * G + g] = s;
  }
}

// d_pre = dG with sampled steps zeroed; dg_ss = dG at sampled steps only.
__global__ void ss_split(Dims d, const int32_t* __restrict__ flags, const float* __restrict__ dg,
                         float* __restrict__ d_pre, float* __restrict__ dg_ss) {
  const int G = 4 * d.D;
  const long long n = (long long)d.B * d.S * G;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int t = (int)((i / G) % d.S);
    const float v = dg[i];
    const bool smp = flags[t] != 0;
    d_pre[i] = smp ? 0.f : v;
    dg_ss[i] = smp ? v : 0.f;
  }
}

size_t wcat_bytes(const Dims& d, int cdt) {
  return ((size_t)4 * d.D * (d.E + d.D) * (cdt == ASR_DT_BF16 ? 2 : 4) + 255) & ~size_t(255);
}

int check_dims(const Dims& d) {
  ASR_REQUIRE(d.B > 0 && d.T > 0 && d.E > 0 && d.A > 0 && d.C > 0 && d.K > 0 && d.D > 0 &&
                  d.S > 0,
              ASR_ERR_ARG, "attdec: bad dims");
  ASR_REQUIRE(d.A <= 256 && d.C <= 16, ASR_ERR_UNSUPPORTED,
              "attdec: attention_dim <= 256 and conv channels <= 16 supported (A=%d C=%d)", d.A,
              d.C);
  ASR_REQUIRE(d.K % 2 == 1, ASR_ERR_ARG, "attdec: conv width must be odd");
  ASR_REQUIRE(en_lds_floats(d) * 4 <= 160 * 1024 && conv_lds_floats(d) * 4 <= 160 * 1024 &&
                  ((size_t)d.T + 64 + ATT_THREADS) * 4 <= 160 * 1024,
              ASR_ERR_UNSUPPORTED, "attdec: LDS need %zu B > 160 KiB", en_lds_floats(d) * 4);
  return ASR_OK;
}

size_t al256(size_t n) { return (n + 255) & ~size_t(255); }

// Workspace: [Wcat (fwd) or Wcat^T (bwd)][energies / d aw [B][T]] and, backward
// only, [r][carry][ddec_att][dc][flags][dF [B][T][C]][dWd chunk partials].
struct AttWs {
  size_t wcat, ebuf, r, carry, ddec, dc, flags, dF, dwdc, wd, pbuf, ctr, sbuf, lbuf, ssd, zcat,
      total;
};
AttWs att_ws(const Dims& d, int cdt, bool bwd) {
  AttWs w;
  size_t o = 0;
  w.wcat = o; o += wcat_bytes(d, cdt);
  w.ebuf = o; o += al256((size_t)d.B * d.T * 4);
  if (bwd) {
    w.r = o; o += al256((size_t)d.B * (d.E + d.D) * 4);
    w.carry = o; o += al256((size_t)d.B * d.T * 4);
    w.ddec = o; o += al256((size_t)d.B * d.D * 4);
    w.dc = o; o += al256((size_t)d.B * d.D * 4);
    w.flags = o; o += al256((size_t)d.S * 4);
    w.dF = o; o += al256((size_t)d.B * d.T * d.C * 4);
    w.dwdc = o; o += al256((size_t)d.B * part_rows(d) * d.A * 4);
    w.wd = o; o += al256((size_t)d.B * d.S * d.A * 4);
    w.sbuf = o; o += al256((size_t)d.B * 8 * 4);
    w.ctr = o; o += al256((size_t)(1 + 8) * 64 * 4);
  } else {   // the persistent forward's W_dec h partials and group counters
    w.pbuf = o; o += al256((size_t)8 * 32 * 4 * d.A * 4);
    // (1 + 8) counters of the three per-step hand-offs + 8 of the sampled-step
    // logits hand-off, then the partial logits of the sampled steps
    // [8 groups][32 members][4 slots][PD_VMAX = 128] and the step flags [S]
    w.ctr = o; o += al256((size_t)(1 + 2 * 8) * 64 * 4);
    w.lbuf = o; o += al256((size_t)8 * 32 * 4 * 128 * 4);
    w.flags = o; o += al256((size_t)d.S * 4);
    w.ssd = o; o += 512;   // the sampled steps' operand record (PdSs)
    // [W_c | W_d] rows of the sampled steps (Dz <= 512), f32 or bf16
    w.zcat = o; o += al256((size_t)512 * (d.E + d.D) * (cdt == ASR_DT_BF16 ? 2 : 4));
  }
  w.total = o;
  return w;
}

// ---------------------------------------------------------------------------
// Persistent forward pass (bf16 mode): all S steps of cell_fwd -> att_energy
// -> att_context in ONE launch of 256 work-groups (one per CU).
//
// The batch is split into 8 groups of up to 4 utterances (b = g + 8 slot, so
// the length-sorted batch spreads evenly); group g is the 32 work-groups
// blockIdx % 8 == g, which the dispatcher deals to one XCD, so every
// hand-off of a group stays in one L2.  Member m (= blockIdx / 8) of a group
// holds, for the whole pass:
//   cell role   : hidden units [m UPW, (m+1) UPW) of the group's 4 utterances;
//                 its 4 UPW rows of Wcat = [W_ih_ctx | W_hh] as MFMA B
//                 fragments in VGPRs (3 row tiles x 2 K halves on waves 0-5),
//                 the cell states in registers, W_dec's columns of its units;
//   frame role  : utterance slot m / 8, frames [ch FCH, (ch+1) FCH) and
//                 context columns [ch ECW, (ch+1) ECW), ch = m % 8: the conv
//                 kernel, W_conv, V in LDS, the frames' enc_a rows in VGPRs,
//                 the enc column slice [T][ECW] in LDS, and aw_{t-1} of the
//                 whole utterance (recomputed from the energies by each of its
//                 8 work-groups, so the 201-tap conv windows need no hand-off).
// Three group-wide hand-offs per step, each a monotonic per-group counter
// (MI355X_MICROARCH.md visibility, valid form row 1: sc1 payload stores, every
// storing wave's vmcnt(0), a workgroup barrier, one agent-scope add; one-lane
// sc1 poll, workgroup barrier, sc1 payload loads):
//   C (cell)   -> h_t into x[b][t+1][E:], W_dec[:, units] h_t partials
//   E (energy) -> masked, sharpened energies of the frame chunk
//   X (context)-> softmax, aw_t, ctx_t into x[b][t+1][:E]
// Same arithmetic as the per-step kernels (bf16 MFMA for the cell, f32 for
// the attention); only f32 summation orders differ.  Spins are bounded: a
// give-up sets the abort word and the recurrence status bit (step skipped).
// ---------------------------------------------------------------------------
constexpr int PD_GROUPS = 8;
constexpr int PD_MEMBERS = 32;
constexpr int PD_SLOTS = 4;
constexpr int PD_CHUNKS = PD_MEMBERS / PD_SLOTS;
constexpr int PD_THREADS = 512;
constexpr int PD_KMAX = 16;      // K blocks of 32 per wave: E + D <= 1024
constexpr int PD_UMAX = 12;      // hidden units per member: 4 UPW <= 48 rows (3 MFMA tiles)
constexpr int PD_FPW = 8;        // frames per wave: FCH <= 64
constexpr int PD_CTR = 64;       // ints per counter (own 256-B line)
constexpr int PD_CM = 4;         // conv channels of the generic instantiations (C <= 4)
constexpr unsigned PD_SPIN_LIMIT = 1u << 20;
constexpr int PD_VMAX = 128;     // sampled steps in the pass: classes <= PD_THREADS / PD_SLOTS
constexpr int PD_YMAX = 64;      // ... embedding dim
constexpr int PD_ZMAX = 16;      // ... bottleneck units per member (Dz <= 512: one MFMA tile)

// Scheduled sampling inside the persistent forward (attention_seq2seq.py:742-748,
// asr_attdec_opts_t): flags == nullptr when no step of the pass samples.
struct PdSs {
  const int32_t* flags;          // [S] (device), t >= 1
  const float *w_d, *b_d, *w_c, *b_c, *w_fc, *b_fc, *emb_w, *w_ih_emb, *b_ih, *b_hh;
  float drop_d, drop_c, drop_emb;
  unsigned long long seed_d, seed_c, seed_emb;
  int Y, Dz, V, emb_trans;
  long long ld_ih;
  float *pre_ss, *emb_ss;
  long long* tok_ss;
  float* lbuf;                   // [PD_GROUPS][PD_MEMBERS][PD_SLOTS][PD_VMAX] partial logits
  const void* zcat;              // [Dz][E + D] = [W_c | W_d] in the pass's Wcat dtype
};
static_assert(sizeof(PdSs) <= 512, "AttWs::ssd holds one PdSs");

// asr_attdec_set_conv_feat: the next persistent decoder pass from this host
// thread writes (forward) / reads (backward) the conv features of every step
// here ([B][S][8 chunks][FCH][FS] f32), NULL: recomputed in the backward.
thread_local float* g_pd_fsave = nullptr;

// Host staging of the PdSs records: a ring of pinned slots, each reused only
// after the copy that read it has completed (its event).
int pd_ss_upload(const PdSs& v, void* dst, hipStream_t s) {
  constexpr int NSLOT = 64;
  static PdSs* ring = nullptr;
  static hipEvent_t ev[NSLOT];
  static int next = 0;
  if (!ring) {
    if (hipHostMalloc((void**)&ring, NSLOT * sizeof(PdSs), hipHostMallocDefault) != hipSuccess) {
      ring = nullptr;
      return ASR_ERR_HIP;
    }
    for (int i = 0; i < NSLOT; ++i)
      if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return ASR_ERR_HIP;
  }
  const int k = next;
  next = (next + 1) % NSLOT;
  if (hipEventSynchronize(ev[k]) != hipSuccess) return ASR_ERR_HIP;   // never recorded: returns
  ring[k] = v;
  if (hipMemcpyAsync(dst, &ring[k], sizeof(PdSs), hipMemcpyHostToDevice, s) != hipSuccess)
    return ASR_ERR_HIP;
  if (hipEventRecord(ev[k], s) != hipSuccess) return ASR_ERR_HIP;
  return ASR_OK;
}

typedef __attribute__((address_space(1))) int pd_gint;
typedef __attribute__((ext_vector_type(4))) unsigned int pd_u32x4;

struct PdGeom {
  int UPW, FCH, ECW, ED, NKB, half, FS;
  int xs, wdl, cw, wc, v, awp, wd, wq, f, hs, part, red, cpart, mp, encs, total;   // LDS floats
};

__host__ __device__ inline PdGeom pd_geom(const Dims& d) {
  PdGeom g;
  g.UPW = (d.D + PD_MEMBERS - 1) / PD_MEMBERS;
  g.FCH = (d.T + PD_CHUNKS - 1) / PD_CHUNKS;
  g.ECW = (d.E + PD_CHUNKS - 1) / PD_CHUNKS;
  g.ED = d.E + d.D;
  g.NKB = (g.ED + 31) / 32;
  g.half = d.K / 2;
  int o = 0;
  g.xs = o; o += PD_SLOTS * g.ED;
  g.wdl = o; o += d.A * g.UPW;
  g.cw = o; o += d.C * d.K;
  g.wc = o; o += d.A * d.C;
  g.v = o; o += d.A;
  g.awp = o; o += d.T + 2 * g.half + 16;
  g.wd = o; o += d.A;
  g.wq = o; o += 4 * d.A;
  o = (o + 3) & ~3;
  g.FS = (d.C + 3) & ~3;
  g.f = o; o += g.FCH * g.FS;
  g.hs = o; o += PD_SLOTS * PD_UMAX;
  g.part = o; o += 6 * PD_SLOTS * 16;
  g.red = o; o += 64;
  g.cpart = o; o += PD_THREADS;
  g.mp = o; o += 2048;
  g.encs = o; o += d.T * g.ECW;
  g.total = (o + 3) & ~3;
  return g;
}

// LDS regions of the sampled steps (floats), after the base geometry (base =
// pd_geom(d).total): only a pass with sampled steps allocates them.
struct PdSsGeom {
  int zp, zz, lg, tk, ev, wie, bs, wfc, ssf, total;
};
__host__ __device__ inline PdSsGeom pd_ss_geom(const Dims& d, int base, int UPW, int Y, int ZPW) {
  PdSsGeom g;
  int o = base;
  g.ssf = o; o += (d.S + 3) & ~3;           // the step flags (int bits); first: at base
  g.zp = o; o += 2 * 2 * PD_SLOTS * 16;     // z MFMA partials [wave 6/7][ctx/h][slot][unit]
  g.zz = o; o += PD_SLOTS * 16;             // z = tanh(...) of this member's units
  g.lg = o; o += PD_SLOTS * PD_VMAX;        // the group's logits of the previous step
  g.tk = o; o += 8;                         // sampled token per slot (int bits)
  g.ev = o; o += PD_SLOTS * Y;              // the sampled embeddings (dropout applied)
  g.wie = o; o += 4 * UPW * Y;              // W_ih[:, :Y] rows of this member's gate rows
  g.bs = o; o += 4 * UPW;                   // their b_ih + b_hh
  g.wfc = o; o += ZPW * PD_VMAX;            // fc columns of this member's bottleneck units
  g.total = (o + 3) & ~3;
  return g;
}

// Conv features of a frame chunk on the f32 MFMA (16x16x4): f[i][c] =
// sum_k cw[c][k] win[i + k] for frames i < FCH <= 64, channels c < C <= 16
// (win[i + k] = aw_{t-1}[tt0 + i + k - K/2]).  All 8 waves: wave w takes row
// tile w % MT and K part w / MT (MT = ceil(FCH / 16)); the K parts' tiles are
// summed in order through part (LDS, 2048 floats).  A Toeplitz product: one
// window load and one kernel load per lane per 4 taps, against two LDS loads
// per tap of a dot-product loop.
__device__ __forceinline__ void pd_conv_feat(const float* cw, const float* win, int C, int K,
                                             int FCH, float* part, float* f, int fs, int ks,
                                             float* gout = nullptr) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int MT = FCH <= 16 ? 1 : FCH <= 32 ? 2 : 4;
  const int KP = 8 / MT;
  const int mt = wave % MT, kp = wave / MT;
  const int nks = (K + 3) / 4, per = (nks + KP - 1) / KP;
  const int s0 = kp * per, s1 = min(nks, s0 + per);
  const int row = mt * 16 + (lane & 15), kk = lane >> 4, col = lane & 15;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int st = s0; st < s1; st += 4) {
    float a[4], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = (st + j) * 4 + kk;
      const bool ok = st + j < s1 && k < K;
      // unconditional loads at clamped (in-range) indices, then selects: no branches
      const int kc = min(k, K - 1);
      const float av = win[min(row, FCH - 1) + kc], bv = cw[min(col, C - 1) * ks + kc];
      a[j] = (ok && row < FCH) ? av : 0.f;
      b[j] = (ok && col < C) ? bv : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = mfma_f32(a[j], b[j], acc);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) part[(wave * 16 + 4 * (lane >> 4) + r) * 16 + col] = acc[r];
  __syncthreads();
  for (int i = threadIdx.x; i < FCH * fs; i += blockDim.x) {   // rows padded to fs (zeros)
    const int fi = i / fs, c = i % fs, tl = fi >> 4, rr = fi & 15;
    float v = 0.f;
    if (c < C)
      for (int q = 0; q < KP; ++q) v += part[((q * MT + tl) * 16 + rr) * 16 + c];
    f[i] = v;
    if (gout) gout[i] = v;   // (the forward keeps them for the backward pass)
  }
}

// tanh through one exp and one reciprocal (the persistent passes' energy
// tanh; |error| ~1e-7, the per-step kernels use libm tanhf)
__device__ __forceinline__ float pd_tanh(float x) {
  const float e = __expf(2.f * fminf(fmaxf(x, -15.f), 15.f));
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pd_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float pd_ld(__amdgpu_buffer_rsrc_t r, long long i) {   // sc1
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (unsigned)(i * 4), 0, 16));
}
__device__ __forceinline__ void pd_st(__amdgpu_buffer_rsrc_t r, long long i, float v) {  // sc1
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (unsigned)(i * 4), 0, 16);
}

// One lane: wait until *ctr >= target.  false = gave up (abort word set / timeout).
__device__ __forceinline__ bool pd_wait(int* ctr, int target, int* abort_w, int* status) {
  pd_gint* c = (pd_gint*)ctr;
  pd_gint* a = (pd_gint*)abort_w;
  for (unsigned spins = 0;; ++spins) {
    if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    if (__hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
    if (spins >= PD_SPIN_LIMIT) {
      __hip_atomic_store(a, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (status) atomicOr(status, 1);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// every storing wave drains its sc1 stores, the work-group joins, one add
__device__ __forceinline__ void pd_publish(int* ctr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add((pd_gint*)ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// phase stamps of work-group 0 at decoder step ATT_TR_STEP (tools/att_trace.py)
#define PD_TR(k)                                                                 \
  do {                                                                           \
    if (t == ATT_TR_STEP && blockIdx.x == 0 && threadIdx.x == 0)                 \
      g_att_tr[k] = __builtin_amdgcn_s_memrealtime();                            \
  } while (0)

// NQ: 64-lane groups of the attention dim (A <= 64 NQ).  SA, SE, SD, SK: the
// attention / encoder / decoder dims and the conv width fixed at compile time
// (0 = from Dims): the production instantiation folds its whole geometry.
// F32 (fp32 mode): Wcat and x_t in f32, the cell product on
// v_mfma_f32_16x16x4_f32 (each of the six cell waves holds its tile's K half as
// 8 PD_KMAX f32 fragments: k-step s of the half is k = 4 (kh + 2 s) + lane / 16).
template <int CC, int NQ, int SA, int SE, int SD, int SK, bool F32 = false>
__global__ void __launch_bounds__(PD_THREADS) attdec_fwd_persist(
    Dims dd, const void* __restrict__ wcat_v, const float* __restrict__ pre_emb,
    const float* __restrict__ h0, const float* __restrict__ enc, const float* __restrict__ enc_a,
    const int32_t* __restrict__ lens, const float* __restrict__ w_dec,
    const float* __restrict__ w_conv, const float* __restrict__ conv_w,
    const float* __restrict__ vw, float* __restrict__ dec, float* __restrict__ c_all,
    float* __restrict__ gates, float* x, float* __restrict__ ctx_all,
    float* __restrict__ aw_all, float* pbuf, float* ebuf, int* ctr, int* status, float drop_h,
    unsigned long long seed_h, const PdSs* __restrict__ ssp, float* __restrict__ fsave) {
  extern __shared__ __attribute__((aligned(16))) float L[];
  Dims d = dd;
  if (CC) d.C = CC;
  if (SA) d.A = SA;
  if (SE) d.E = SE;
  if (SD) d.D = SD;
  if (SK) d.K = SK;
  __shared__ int s_ok;
  // sampled steps (ssp: the operands, in device memory -- read where used, so
  // they never hold scalar registers across the pass)
  const bool ss_on = ssp != nullptr;     // kernel-uniform
  const PdGeom G = pd_geom(d);
  const int UPW = G.UPW, FCH = G.FCH, ECW = G.ECW, ED = G.ED, NKB = G.NKB, half = G.half;
  const int grp = blockIdx.x % PD_GROUPS, m = blockIdx.x / PD_GROUPS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int u0 = m * UPW, nu = max(0, min(UPW, d.D - u0));
  const int G4 = 4 * d.D;
  int* my_ctr = ctr + (1 + grp) * PD_CTR;
  int* ss_ctr = ctr + (1 + PD_GROUPS + grp) * PD_CTR;   // sampled steps' logits hand-off
  const __amdgpu_buffer_rsrc_t rx = pd_rsrc(x, (unsigned)((size_t)d.B * d.S * ED * 4));
  const __amdgpu_buffer_rsrc_t rp =
      pd_rsrc(pbuf, (unsigned)((size_t)PD_GROUPS * PD_MEMBERS * PD_SLOTS * d.A * 4));
  const __amdgpu_buffer_rsrc_t re = pd_rsrc(ebuf, (unsigned)((size_t)d.B * d.T * 4));
  // frame role
  const int fsl = m / PD_CHUNKS, ch = m % PD_CHUNKS;
  const int be = grp + PD_GROUPS * fsl;
  const bool fact = be < d.B;                 // work-group uniform
  const int tt0 = ch * FCH, nfr = max(0, min(FCH, d.T - tt0));
  const int e0 = ch * ECW, ecn = max(0, min(ECW, d.E - e0));
  const int len = fact ? lens[be] : 0;
  constexpr int CM = CC ? CC : PD_CM;
  const int C = CC ? CC : d.C;

  // ---- once per pass: weights and the utterance's constant rows
  constexpr int KM32 = F32 ? 8 * PD_KMAX : 1;
  bf16x8 wf[F32 ? 1 : PD_KMAX];
  float wf32[KM32];
  // sampled steps: member m's bottleneck units [zu0, zu0 + nz) of Dz
  {
    const int tile = wave >> 1, kh = wave & 1;
    const int gr = tile * 16 + (lane & 15), q = gr / UPW, u = gr % UPW;
    const bool ok = wave < 6 && q < 4 && u < nu;
    // waves 6, 7 (idle in the cell product): row tile 3 = [W_c | W_d] rows of
    // this member's bottleneck units, so a sampled step's z = W_c ctx + W_d h
    // runs beside the gate product on the same x rows (ctx and h parts kept
    // apart: their dropout masks differ)
    const int zdz = ss_on ? ssp->Dz : 0, zpw = (zdz + PD_MEMBERS - 1) / PD_MEMBERS;
    const int zr = m * zpw + (lane & 15);
    const bool zok = ss_on && wave >= 6 && (lane & 15) < zpw && zr < zdz;
    const void* wsrc = zok ? ssp->zcat : wcat_v;
    const long long wrow = ok ? q * d.D + u0 + u : zok ? zr : 0;
    const bool wl = ok || zok;
    if constexpr (F32) {
      const float* wr = (const float*)wsrc + wrow * ED;
#pragma unroll
      for (int i = 0; i < KM32; ++i) {
        const int k = 4 * (kh + 2 * i) + (lane >> 4);
        wf32[i] = (wl && k < ED) ? wr[k] : 0.f;
      }
    } else {
      const uint16_t* wr = (const uint16_t*)wsrc + wrow * ED;
#pragma unroll
      for (int i = 0; i < PD_KMAX; ++i) {
        const int k = (kh + 2 * i) * 32 + 8 * (lane >> 4);
        wf[i] = (wl && kh + 2 * i < NKB && k < ED) ? load_bf16x8(wr + k)
                                                    : as_bf16x8(u16x8{0, 0, 0, 0, 0, 0, 0, 0});
      }
    }
  }
  float ea[PD_FPW][NQ];
#pragma unroll
  for (int f = 0; f < PD_FPW; ++f) {
    const int i = wave + 8 * f, tt = tt0 + i;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int a = lane + 64 * q;
      ea[f][q] = (fact && i < nfr && a < d.A) ? enc_a[((long long)be * d.T + tt) * d.A + a] : 0.f;
    }
  }
  constexpr int CM4 = (CM + 3) / 4;
  float wcr[NQ][CM], vr[NQ];   // this lane's attention units' W_conv rows and V
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int a = lane + 64 * q;
    vr[q] = a < d.A ? vw[a] : 0.f;
#pragma unroll
    for (int c = 0; c < CM; ++c) wcr[q][c] = (a < d.A && (CC || c < C)) ? w_conv[a * C + c] : 0.f;
  }
  for (int i = tid; i < d.A * UPW; i += PD_THREADS) {
    const int a = i / UPW, u = i % UPW;
    L[G.wdl + i] = u < nu ? w_dec[(long long)a * d.D + u0 + u] : 0.f;
  }
  for (int i = tid; i < d.C * d.K; i += PD_THREADS) L[G.cw + i] = conv_w[i];
  for (int i = tid; i < d.A * d.C; i += PD_THREADS) L[G.wc + i] = w_conv[i];
  for (int i = tid; i < d.A; i += PD_THREADS) L[G.v + i] = vw[i];
  for (int i = tid; i < d.T + 2 * half + 16; i += PD_THREADS) L[G.awp + i] = 0.f;
  for (int i = tid; i < d.T * ECW; i += PD_THREADS) {
    const int tt = i / ECW, cc = i % ECW;
    L[G.encs + i] = (fact && cc < ecn) ? enc[((long long)be * d.T + tt) * d.E + e0 + cc] : 0.f;
  }
  // cell role: thread (slot, unit) for tid < 4 UPW
  const int csl = tid / UPW, cu = tid % UPW;
  const int cb = grp + PD_GROUPS * csl, cj = u0 + cu;
  const bool cown = tid < PD_SLOTS * UPW && cu < nu && cb < d.B;
  float c_reg = 0.f;
  // sampled steps: the step flags, this member's W_ih[:, :Y] gate rows, the
  // cell threads' bias sums, the (slot, class) threads' fc columns of this
  // member's bottleneck units
  // (in LDS, not registers: the pass is at its VGPR budget)
  if (ss_on) {
    const PdSs& ss = *ssp;
    const int Y = ss.Y, ZPW = (ss.Dz + PD_MEMBERS - 1) / PD_MEMBERS, zu0 = m * ZPW;
    const int nz = max(0, min(ZPW, ss.Dz - zu0));
    const PdSsGeom Z = pd_ss_geom(d, G.total, UPW, Y, ZPW);
    int* fl = reinterpret_cast<int*>(&L[Z.ssf]);
    for (int i = tid; i < d.S; i += PD_THREADS) fl[i] = ss.flags[i];
    for (int i = tid; i < 4 * UPW * Y; i += PD_THREADS) {
      const int q = i / (UPW * Y), u = (i / Y) % UPW, y = i % Y;
      L[Z.wie + i] = u < nu ? ss.w_ih_emb[(long long)(q * d.D + u0 + u) * ss.ld_ih + y] : 0.f;
    }
    for (int i = tid; i < 4 * UPW; i += PD_THREADS) {
      const int q = i / UPW, u = i % UPW, r = q * d.D + u0 + u;
      L[Z.bs + i] = u < nu ? ss.b_ih[r] + ss.b_hh[r] : 0.f;
    }
    for (int i = tid; i < ZPW * PD_VMAX; i += PD_THREADS) {
      const int z = i / PD_VMAX, v = i % PD_VMAX;
      L[Z.wfc + i] = (z < nz && v < ss.V) ? ss.w_fc[(long long)v * ss.Dz + zu0 + z] : 0.f;
    }
  }
  int nss = 0;   // sampled steps so far (the logits hand-off's counter target)
  __syncthreads();

  for (int t = 0; t < d.S; ++t) {
    // ================= C: cell step t (t = 0: the initial state h0) =================
    PD_TR(32);
    // step t feeds embed(argmax logits_{t-1}) instead of the teacher token
    // (work-group and group uniform: every member reads the same flags)
    const int smp = (ss_on && t > 0) ? reinterpret_cast<const int*>(&L[G.total])[t] : 0;
    if (t > 0) {
      if (tid == 0) s_ok = pd_wait(my_ctr, PD_MEMBERS * 3 * t, ctr, status);
      __syncthreads();
      if (!s_ok) return;
      PD_TR(33);
      // x_t rows of the 4 utterances, rounded to bf16 once (the MFMA A operand;
      // f32 as they are with F32)
      uint16_t* xsb = reinterpret_cast<uint16_t*>(&L[G.xs]);
      const int nv = ED / 4;
      for (int i = tid; i < PD_SLOTS * nv; i += PD_THREADS) {
        const int sl = i / nv, k4 = i % nv, bb = grp + PD_GROUPS * sl;
        pd_u32x4 v = {0u, 0u, 0u, 0u};
        if (bb < d.B)
          v = __builtin_amdgcn_raw_buffer_load_b128(
              rx, (unsigned)((((long long)bb * d.S + t) * ED + 4 * k4) * 4), 0, 16);
        if constexpr (F32) {
          *reinterpret_cast<pd_u32x4*>(&L[G.xs + sl * ED + 4 * k4]) = v;
        } else {
          const unsigned lo = f2bf(__uint_as_float(v[0])) | ((unsigned)f2bf(__uint_as_float(v[1])) << 16);
          const unsigned hi = f2bf(__uint_as_float(v[2])) | ((unsigned)f2bf(__uint_as_float(v[3])) << 16);
          *reinterpret_cast<uint2*>(xsb + sl * ED + 4 * k4) = make_uint2(lo, hi);
        }
      }
      __syncthreads();
      PD_TR(34);
      if constexpr (F32) {
        if (wave < 6) {
          const int kh = wave & 1, mm = lane & 15;
          f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int i = 0; i < KM32; ++i) {
            if (4 * (kh + 2 * i) < ED) {   // wave-uniform
              const int k = 4 * (kh + 2 * i) + (lane >> 4);
              const float a = (mm < PD_SLOTS && k < ED) ? L[G.xs + mm * ED + k] : 0.f;
              if (i & 1) acc1 = mfma_f32(a, wf32[i], acc1);
              else acc0 = mfma_f32(a, wf32[i], acc0);
            }
          }
          if (lane < 16) {
#pragma unroll
            for (int r = 0; r < 4; ++r) L[G.part + (wave * PD_SLOTS + r) * 16 + lane] = acc0[r] + acc1[r];
          }
        } else if (smp) {   // waves 6, 7: z partials of a sampled step (ctx / h apart)
          const int kh = wave & 1, mm = lane & 15;
          f32x4 ac = {0.f, 0.f, 0.f, 0.f}, ad = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int i = 0; i < KM32; ++i) {
            if (4 * (kh + 2 * i) < ED) {   // wave-uniform
              const int k = 4 * (kh + 2 * i) + (lane >> 4);
              const float a = (mm < PD_SLOTS && k < ED) ? L[G.xs + mm * ED + k] : 0.f;
              // k-step kh + 2 i is a ctx column iff i < E / 8 (E % 8 == 0: pd_ss_ok)
              if (i < d.E / 8) ac = mfma_f32(a, wf32[i], ac);
              else ad = mfma_f32(a, wf32[i], ad);
            }
          }
          if (lane < 16) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int zp = G.total + ((d.S + 3) & ~3);   // pd_ss_geom's zp
              L[zp + (((wave - 6) * 2 + 0) * PD_SLOTS + r) * 16 + lane] = ac[r];
              L[zp + (((wave - 6) * 2 + 1) * PD_SLOTS + r) * 16 + lane] = ad[r];
            }
          }
        }
      } else if (wave >= 6) {
        if (smp) {   // waves 6, 7: z partials of a sampled step (ctx / h apart)
          const int kh = wave & 1, mm = lane & 15;
          f32x4 ac = {0.f, 0.f, 0.f, 0.f}, ad = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int i = 0; i < PD_KMAX; ++i) {
            const int kb = kh + 2 * i;
            if (kb < NKB) {   // wave-uniform
              const int k = kb * 32 + 8 * (lane >> 4);
              const bf16x8 a = (mm < PD_SLOTS && k < ED) ? load_bf16x8(xsb + mm * ED + k)
                                                        : as_bf16x8(u16x8{0, 0, 0, 0, 0, 0, 0, 0});
              // block kh + 2 i is a ctx block iff i < E / 64 (E % 64 == 0: pd_ss_ok)
              if (i < d.E / 64) ac = mfma_bf16(a, wf[i], ac);
              else ad = mfma_bf16(a, wf[i], ad);
            }
          }
          if (lane < 16) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int zp = G.total + ((d.S + 3) & ~3);   // pd_ss_geom's zp
              L[zp + (((wave - 6) * 2 + 0) * PD_SLOTS + r) * 16 + lane] = ac[r];
              L[zp + (((wave - 6) * 2 + 1) * PD_SLOTS + r) * 16 + lane] = ad[r];
            }
          }
        }
      } else {
        const int kh = wave & 1, mm = lane & 15;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < PD_KMAX; ++i) {
          const int kb = kh + 2 * i;
          if (kb < NKB) {   // wave-uniform
            const int k = kb * 32 + 8 * (lane >> 4);
            const bf16x8 a = (mm < PD_SLOTS && k < ED) ? load_bf16x8(xsb + mm * ED + k)
                                                      : as_bf16x8(u16x8{0, 0, 0, 0, 0, 0, 0, 0});
            acc = mfma_bf16(a, wf[i], acc);
          }
        }
        if (lane < 16) {
#pragma unroll
          for (int r = 0; r < 4; ++r) L[G.part + (wave * PD_SLOTS + r) * 16 + lane] = acc[r];
        }
      }
      __syncthreads();
      PD_TR(35);
      float pss[4] = {0.f, 0.f, 0.f, 0.f};
      if (smp) {
        // ---- sampled step (ss_step's arithmetic, split over the group):
        // z = tanh(drop_d(W_d h_{t-1} + b_d) + drop_c(W_c ctx_{t-1} + b_c)) of
        // this member's units -> partial logits over them -> one group hand-off
        // -> logits_{t-1} (fixed member order) -> first argmax -> the sampled
        // embedding (dropout) -> pre = W_ih[:, :Y] e + b_ih + b_hh
        ++nss;
        const PdSs& ss = *ssp;
        const int ZPW = (ss.Dz + PD_MEMBERS - 1) / PD_MEMBERS, zu0 = m * ZPW;
        const int nz = max(0, min(ZPW, ss.Dz - zu0));
        const PdSsGeom Z = pd_ss_geom(d, G.total, UPW, ss.Y, ZPW);
        if (tid < PD_SLOTS * 16) {
          const int sl = tid >> 4, zu = tid & 15, bb = grp + PD_GROUPS * sl;
          float zv = 0.f;
          if (zu < nz && bb < d.B) {
            const int zr = zu0 + zu;
            float a = L[Z.zp + ((0 * 2 + 1) * PD_SLOTS + sl) * 16 + zu] +
                      L[Z.zp + ((1 * 2 + 1) * PD_SLOTS + sl) * 16 + zu] + (ss.b_d ? ss.b_d[zr] : 0.f);
            float c = L[Z.zp + ((0 * 2 + 0) * PD_SLOTS + sl) * 16 + zu] +
                      L[Z.zp + ((1 * 2 + 0) * PD_SLOTS + sl) * 16 + zu] + (ss.b_c ? ss.b_c[zr] : 0.f);
            const unsigned idx = ((unsigned)bb * d.S + (t - 1)) * (unsigned)ss.Dz + zr;
            if (ss.drop_d > 0.f) a *= drop_scale(ss.drop_d, ss.seed_d, idx);
            if (ss.drop_c > 0.f) c *= drop_scale(ss.drop_c, ss.seed_c, idx);
            zv = tanhf(a + c);
          }
          L[Z.zz + tid] = zv;
        }
        __syncthreads();
        const int lsl = tid / ss.V, lv = tid % ss.V;
        const bool lown = tid < PD_SLOTS * ss.V;
        if (lown) {
          float pl = 0.f;
          for (int z = 0; z < nz; ++z) pl += L[Z.wfc + z * PD_VMAX + lv] * L[Z.zz + lsl * 16 + z];
          pd_st(pd_rsrc(ss.lbuf, (unsigned)((size_t)PD_GROUPS * PD_MEMBERS * PD_SLOTS * PD_VMAX * 4)),
                (((long long)grp * PD_MEMBERS + m) * PD_SLOTS + lsl) * PD_VMAX + lv, pl);
        }
        pd_publish(ss_ctr);
        if (tid == 0) s_ok = pd_wait(ss_ctr, PD_MEMBERS * nss, ctr, status);
        __syncthreads();
        if (!s_ok) return;
        if (lown) {
          const __amdgpu_buffer_rsrc_t rl =
              pd_rsrc(ss.lbuf, (unsigned)((size_t)PD_GROUPS * PD_MEMBERS * PD_SLOTS * PD_VMAX * 4));
          float lsum = 0.f;
          const int lb = (grp * PD_MEMBERS * PD_SLOTS + lsl) * PD_VMAX + lv;
#pragma unroll 1
          for (int j0 = 0; j0 < PD_MEMBERS; j0 += 4) {
            float pv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) pv[j] = pd_ld(rl, lb + (j0 + j) * PD_SLOTS * PD_VMAX);
#pragma unroll
            for (int j = 0; j < 4; ++j) lsum += pv[j];
          }
          L[Z.lg + lsl * PD_VMAX + lv] = lsum + (ss.b_fc ? ss.b_fc[lv] : 0.f);
        }
        __syncthreads();
        int* tk = reinterpret_cast<int*>(&L[Z.tk]);
        if (tid < PD_SLOTS) {   // strict: the first maximum wins (torch.max)
          float best = -__builtin_huge_valf();
          int bi = 0;
          for (int v = 0; v < ss.V; ++v) {
            const float l = L[Z.lg + tid * PD_VMAX + v];
            if (l > best) { best = l; bi = v; }
          }
          tk[tid] = bi;
          const int bb = grp + PD_GROUPS * tid;
          if (m == 0 && bb < d.B && ss.tok_ss) ss.tok_ss[(long long)bb * d.S + t] = bi;
        }
        __syncthreads();
        for (int i = tid; i < PD_SLOTS * ss.Y; i += PD_THREADS) {
          const int sl = i / ss.Y, y = i % ss.Y, bb = grp + PD_GROUPS * sl, tok = tk[sl];
          float ev = ss.emb_trans ? ss.emb_w[(long long)y * ss.V + tok]
                                  : ss.emb_w[(long long)tok * ss.Y + y];
          const unsigned ei = ((unsigned)bb * d.S + t) * (unsigned)ss.Y + y;
          if (ss.drop_emb > 0.f) ev *= drop_scale(ss.drop_emb, ss.seed_emb, ei);
          L[Z.ev + i] = ev;
          if (m == 0 && bb < d.B) ss.emb_ss[ei] = ev;
        }
        __syncthreads();
        if (cown) {
          const long long gb = ((long long)cb * d.S + t) * G4 + cj;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float sv = L[Z.bs + q * UPW + cu];
            const float* wr = &L[Z.wie + (q * UPW + cu) * ss.Y];
            const float* ev = &L[Z.ev + csl * ss.Y];
            for (int y = 0; y < ss.Y; ++y) sv += wr[y] * ev[y];
            pss[q] = sv;
            ss.pre_ss[gb + (long long)q * d.D] = sv;
          }
        }
      }
      if (cown) {
        const long long gb = ((long long)cb * d.S + t) * G4 + cj;
        float pre[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int gr = q * UPW + cu, tile = gr >> 4, col = gr & 15;
          pre[q] = L[G.part + ((2 * tile) * PD_SLOTS + csl) * 16 + col] +
                   L[G.part + ((2 * tile + 1) * PD_SLOTS + csl) * 16 + col] +
                   (smp ? pss[q] : pre_emb[gb + (long long)q * d.D]);
        }
        const float ig = sigmoidf_(pre[0]), fg = sigmoidf_(pre[1]);
        const float gg = tanhf_(pre[2]), og = sigmoidf_(pre[3]);
        const float c = fg * c_reg + ig * gg;
        float h = og * tanhf_(c);
        if (drop_h > 0.f)
          h *= drop_scale(drop_h, seed_h, ((unsigned long long)cb * d.S + t) * d.D + cj);
        c_reg = c;
        c_all[((long long)cb * d.S + t) * d.D + cj] = c;
        dec[((long long)cb * d.S + t) * d.D + cj] = h;
        gates[gb] = ig;
        gates[gb + d.D] = fg;
        gates[gb + 2 * d.D] = gg;
        gates[gb + 3 * d.D] = og;
        if (t + 1 < d.S) pd_st(rx, ((long long)cb * d.S + t + 1) * ED + d.E + cj, h);
        L[G.hs + csl * PD_UMAX + cu] = h;   // absent (slot, unit) entries stay 0 from t = 0
      }
    } else {
      for (int i = tid; i < FCH * G.FS; i += PD_THREADS) L[G.f + i] = 0.f;   // aw_{-1} = 0
      if (tid < PD_SLOTS * PD_UMAX) {
        const int sl = tid / PD_UMAX, u = tid % PD_UMAX, bb = grp + PD_GROUPS * sl;
        L[G.hs + tid] = (h0 && u < nu && bb < d.B) ? h0[(long long)bb * d.D + u0 + u] : 0.f;
      }
    }
    __syncthreads();
    PD_TR(36);
    // partial W_dec h_t over this member's units, one (slot, a) per thread
    for (int i = tid; i < PD_SLOTS * d.A; i += PD_THREADS) {
      const int sl = i / d.A, a = i % d.A;
      float s = 0.f;
      for (int u = 0; u < nu; ++u) s += L[G.wdl + a * UPW + u] * L[G.hs + sl * PD_UMAX + u];
      pd_st(rp, (((long long)grp * PD_MEMBERS + m) * PD_SLOTS + sl) * d.A + a, s);
    }
    pd_publish(my_ctr);
    PD_TR(37);
    // conv features of aw_{t-1} for this chunk (local data: before the wait)
    if (fact && t > 0)
      pd_conv_feat(&L[G.cw], &L[G.awp + tt0], C, d.K, FCH, &L[G.mp], &L[G.f], G.FS, d.K,
                   fsave ? fsave + (((long long)be * d.S + t) * PD_CHUNKS + ch) * FCH * G.FS
                         : nullptr);

    // ================= E: energies of this work-group's frame chunk =================
    if (tid == 0) s_ok = pd_wait(my_ctr, PD_MEMBERS * (3 * t + 1), ctr, status);
    __syncthreads();
    if (!s_ok) return;
    PD_TR(38);
    if (fact) {
      for (int i = tid; i < 4 * d.A; i += PD_THREADS) {   // W_dec h_t: 32 partials, fixed order
        const int a = i % d.A, qq = i / d.A;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = pd_ld(rp, (((long long)grp * PD_MEMBERS + qq * 8 + j) * PD_SLOTS + fsl) * d.A + a);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[j];
        L[G.wq + qq * d.A + a] = s;
      }
      __syncthreads();
      PD_TR(39);
      for (int a = tid; a < d.A; a += PD_THREADS)
        L[G.wd + a] = (L[G.wq + a] + L[G.wq + d.A + a]) + (L[G.wq + 2 * d.A + a] + L[G.wq + 3 * d.A + a]);
      __syncthreads();
      PD_TR(40);
      // every frame's lane partial first, then the wave sums together (independent
      // reduction chains in flight)
      float sf[PD_FPW];
#pragma unroll
      for (int f = 0; f < PD_FPW; ++f) {
        const int i = wave + 8 * f;
        sf[f] = 0.f;
        if (i < nfr) {   // wave-uniform
          float frv[CM4 * 4];
#pragma unroll
          for (int c4 = 0; c4 < CM4; ++c4) {
            const float4 v4 = 4 * c4 < G.FS ? *reinterpret_cast<const float4*>(&L[G.f + i * G.FS + 4 * c4])
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
            frv[4 * c4] = v4.x;
            frv[4 * c4 + 1] = v4.y;
            frv[4 * c4 + 2] = v4.z;
            frv[4 * c4 + 3] = v4.w;
          }
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const int a = lane + 64 * q;
            if (64 * q < d.A && a < d.A) {
              float p = ea[f][q] + L[G.wd + a];
#pragma unroll
              for (int c = 0; c < CM; ++c)
                if (CC || c < C) p += frv[c] * wcr[q][c];
              sf[f] += vr[q] * pd_tanh(p);
            }
          }
        }
      }
#pragma unroll
      for (int f = 0; f < PD_FPW; ++f) {
        const int i = wave + 8 * f;
        if (i < nfr) sf[f] = wave_sum(sf[f]);
      }
      if (lane == 0) {
#pragma unroll
        for (int f = 0; f < PD_FPW; ++f) {
          const int i = wave + 8 * f, tt = tt0 + i;
          if (i < nfr) pd_st(re, (long long)be * d.T + tt, (tt < len ? sf[f] : 0.f) * d.sharpen);
        }
      }
    }
    PD_TR(41);
    pd_publish(my_ctr);
    PD_TR(42);

    // ================= X: softmax over the utterance, context slice =================
    if (tid == 0) s_ok = pd_wait(my_ctr, PD_MEMBERS * (3 * t + 2), ctr, status);
    __syncthreads();
    if (!s_ok) return;
    PD_TR(43);
    if (fact) {
      float* aw = &L[G.awp + half];
      float* red = &L[G.red];
      float mx = -__builtin_huge_valf();
      for (int i = tid; i < d.T; i += PD_THREADS) {
        const float e = pd_ld(re, (long long)be * d.T + i);
        aw[i] = e;
        mx = fmaxf(mx, e);
      }
      if (d.sigmoid) {
        for (int i = tid; i < d.T; i += PD_THREADS) aw[i] = sigmoidf_(aw[i]);
      } else {   // (each thread re-reads only the elements it wrote: no barrier)
        mx = wave_max(mx);
        if (lane == 0) red[wave] = mx;
        __syncthreads();
        mx = red[0];
#pragma unroll
        for (int w = 1; w < 8; ++w) mx = fmaxf(mx, red[w]);
        float sm = 0.f;
        for (int i = tid; i < d.T; i += PD_THREADS) {
          const float p = __expf(aw[i] - mx);
          aw[i] = p;
          sm += p;
        }
        sm = wave_sum(sm);
        if (lane == 0) red[8 + wave] = sm;
        __syncthreads();
        sm = red[8];
#pragma unroll
        for (int w = 1; w < 8; ++w) sm += red[8 + w];
        const float inv = 1.f / sm;
        for (int i = tid; i < d.T; i += PD_THREADS) aw[i] *= inv;
      }
      __syncthreads();
      PD_TR(44);
      for (int i = tid; i < nfr; i += PD_THREADS)
        aw_all[((long long)be * d.S + t) * d.T + tt0 + i] = aw[tt0 + i];
      const int NR = PD_THREADS / ECW, col = tid % ECW, r = tid / ECW;
      float s = 0.f;
      if (r < NR && col < ecn && r < d.T)
        s = dot_lds(&aw[r], NR, &L[G.encs + r * ECW + col], NR * ECW, (d.T - r + NR - 1) / NR);
      if (r < NR) L[G.cpart + r * ECW + col] = s;
      __syncthreads();
      if (tid < ecn) {
        float cv = 0.f;
        for (int q = 0; q < NR; ++q) cv += L[G.cpart + q * ECW + tid];
        ctx_all[((long long)be * d.S + t) * d.E + e0 + tid] = cv;
        if (t + 1 < d.S) pd_st(rx, ((long long)be * d.S + t + 1) * ED + e0 + tid, cv);
      }
    }
    PD_TR(45);
    pd_publish(my_ctr);
    PD_TR(46);
  }
}


// ---------------------------------------------------------------------------
// Persistent backward pass (bf16): all S steps of rgemm -> att_bwd_daw ->
// att_bwd_energy -> att_bwd_conv -> cell_bwd in ONE launch, with the forward
// pass's group layout (8 per-XCD groups of 32 work-groups, 4 utterances per
// group, b = g + 8 slot; member m = blockIdx / 8).  Member roles:
//   r role     : columns [m NPW, (m+1) NPW) of r = dgates_{t+1} Wcat for the
//                group's 4 utterances; its Wcat^T rows as MFMA B fragments in
//                VGPRs (2 column tiles x 4 K quarters over the 8 waves);
//   frame role : utterance slot m / 8, frames [ch FCH, (ch+1) FCH), ch = m % 8:
//                the frames' enc rows and enc_a rows in LDS, their d enc_a and
//                the chunk's dV / dW_conv / conv-kernel partial sums in
//                registers for the whole pass, the d aw carry in LDS;
//   cell role  : hidden units [m UPW, (m+1) UPW), their d c carries in
//                registers, W_dec's columns of the units in LDS.
// Four group-wide hand-offs per step t (same protocol as the forward pass):
//   H (t+1 < S) r role     : r = dgates_{t+1} Wcat            -> r [B][E+D]
//   E           frame role : d ctx_t = d_ctx_in + r[:E]; d aw_t = carry + enc . d ctx;
//                            chunk sum of aw d aw (softmax)    -> sdot partials
//                            (and, no hand-off, the conv features of aw_{t-1})
//   F           frame role : softmax / tanh backward            -> dF rows, d W_dec-input
//                                                                 chunk sums
//   G           frame role : d aw_{t-1} = conv^T(dF window) (next step's carry),
//                            conv-kernel partials
//               cell role  : d dec_t = d_dec_in + r[E:] + W_dec^T dWd_t;
//                            LSTMCell backward                 -> dgates_t (over gates)
// Arithmetic as the per-step kernels (bf16 MFMA for r, f32 elsewhere); the
// weight-gradient partials are summed over the steps in registers instead of
// per-step rows, so their f32 summation order differs.
// ---------------------------------------------------------------------------
constexpr int PB_KQ = 12;         // K blocks of 32 per wave quarter: 4 D <= 1536
constexpr int PB_CM = PD_CM;

struct PbGeom {
  int UPW, FCH, ECW, ED, G4, NPW, NKB, KQ, half, W, FS, AP, KQ4, KP;
  int encr, ea, cw, wc, v, dct, awin, f, daw, awt, de, carry, wd, un, dgs, part, dwdl, wdl,
      cmb, cmbn, red, total;   // LDS floats
};

__host__ __device__ inline PbGeom pb_geom(const Dims& d, bool f32 = false) {
  PbGeom g;
  g.UPW = (d.D + PD_MEMBERS - 1) / PD_MEMBERS;
  g.FCH = (d.T + PD_CHUNKS - 1) / PD_CHUNKS;
  g.ECW = (d.E + PD_CHUNKS - 1) / PD_CHUNKS;
  g.ED = d.E + d.D;
  g.G4 = 4 * d.D;
  g.NPW = (g.ED + PD_MEMBERS - 1) / PD_MEMBERS;
  g.NKB = (g.G4 + 31) / 32;
  g.KQ = (g.NKB + 3) / 4;
  g.half = d.K / 2;
  g.W = g.FCH + d.K - 1;
  int o = 0;
  g.encr = o; o += g.FCH * d.E;
  g.ea = o; o += g.FCH * d.A;
  g.KQ4 = 4 * ((d.K + 15) / 16);   // taps per quarter of the conv transpose (multiple of 4)
  g.KP = 4 * g.KQ4;                 // conv kernel rows padded with zero taps to KP
  o = (o + 3) & ~3;
  g.cw = o; o += d.C * g.KP;
  g.wc = o; o += d.A * d.C;
  g.v = o; o += d.A;
  g.dct = o; o += d.E;
  g.awin = o; o += g.W;
  o = (o + 3) & ~3;
  g.FS = (d.C + 3) & ~3;
  g.f = o; o += g.FCH * g.FS;
  g.daw = o; o += g.FCH;
  g.awt = o; o += g.FCH;
  g.de = o; o += g.FCH;
  g.carry = o; o += g.FCH;
  g.wd = o; o += d.A;
  o = (o + 3) & ~3;
  {  // one region, used by phase H (bf16 dgates rows [4][G4], f32 with f32), F
     // (the chunk's d enc_a rows) and G (dF window [W][C] + the W_dec^T dWd partials)
    int un = f32 ? PD_SLOTS * g.G4 + 4 : PD_SLOTS * g.G4 / 2 + 4;
    g.AP = d.A + 1;   // the [frames][A] tiles' row stride (odd: no bank conflicts down a column)
    un = max(un, g.FCH * g.AP);
    un = max(un, (8 + g.W) * d.C + PD_SLOTS * g.UPW * 8);   // dF window after 8 zero rows
    un = max(un, 2048);   // E: the conv features' MFMA partial tiles
    g.un = o; o += un;
    g.dgs = g.un;
  }
  g.part = o; o += 8 * PD_SLOTS * 16;
  g.dwdl = o; o += PD_SLOTS * d.A;
  g.wdl = o; o += d.A * g.UPW;
  g.cmb = o;
  g.cmbn = max(max(8 * d.A, PD_THREADS), 4 * ((g.FCH + 3) / 4) * 4 * d.C);
  o += g.cmbn;
  g.red = o; o += 64;
  g.total = (o + 3) & ~3;
  return g;
}

// F32 (fp32 mode): Wcat^T and dgates in f32, r on v_mfma_f32_16x16x4_f32 (each
// wave holds its column tile's K quarter as f32 fragments: k-step s of the
// quarter is k = 4 (kq KQ32 + s) + lane / 16).
template <int CC, int NQ, int SA, int SE, int SD, int SK, bool F32 = false, bool FS = false>
__global__ void __launch_bounds__(PD_THREADS) attdec_bwd_persist(
    Dims dd, const void* __restrict__ wcatT_v, const float* __restrict__ enc,
    const float* __restrict__ enc_a, const int32_t* __restrict__ lens,
    const float* __restrict__ w_dec, const float* __restrict__ w_conv,
    const float* __restrict__ conv_w, const float* __restrict__ vw,
    const float* __restrict__ c_all, const float* __restrict__ aw_all,
    const float* __restrict__ wd_all, const float* __restrict__ d_dec_in,
    const float* __restrict__ d_ctx_in, float* gates, float* __restrict__ dctx_tot,
    float* __restrict__ d_enc_a, float* __restrict__ d_h0, float* __restrict__ dwd_all,
    float* __restrict__ dv_part, float* __restrict__ dwc_part, float* __restrict__ dcw_part,
    float* rbuf, float* sbuf, float* dwdc, float* dFbuf, int* ctr, int* status, float drop_h,
    unsigned long long seed_h, const float* __restrict__ fsave) {
  extern __shared__ __attribute__((aligned(16))) float L[];
  Dims d = dd;
  if (CC) d.C = CC;
  if (SA) d.A = SA;
  if (SE) d.E = SE;
  if (SD) d.D = SD;
  if (SK) d.K = SK;
  __shared__ int s_ok;
  __shared__ float s_sdot;
  const PbGeom G = pb_geom(d, F32);
  const int UPW = G.UPW, FCH = G.FCH, ECW = G.ECW, ED = G.ED, G4 = G.G4, NPW = G.NPW;
  const int half = G.half, KW = G.W;
  const int grp = blockIdx.x % PD_GROUPS, m = blockIdx.x / PD_GROUPS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int u0 = m * UPW, nu = max(0, min(UPW, d.D - u0));
  const int n0 = m * NPW, nn = max(0, min(NPW, ED - n0));
  int* my_ctr = ctr + (1 + grp) * PD_CTR;
  const __amdgpu_buffer_rsrc_t rg = pd_rsrc(gates, (unsigned)((size_t)d.B * d.S * G4 * 4));
  const __amdgpu_buffer_rsrc_t rr = pd_rsrc(rbuf, (unsigned)((size_t)d.B * ED * 4));
  const __amdgpu_buffer_rsrc_t rs = pd_rsrc(sbuf, (unsigned)((size_t)d.B * PD_CHUNKS * 4));
  const __amdgpu_buffer_rsrc_t rw = pd_rsrc(dwdc, (unsigned)((size_t)d.B * PD_CHUNKS * d.A * 4));
  const __amdgpu_buffer_rsrc_t rf = pd_rsrc(dFbuf, (unsigned)((size_t)d.B * d.T * d.C * 4));
  // frame role
  const int fsl = m / PD_CHUNKS, ch = m % PD_CHUNKS;
  const int be = grp + PD_GROUPS * fsl;
  const bool fact = be < d.B;
  const int tt0 = ch * FCH, nfr = max(0, min(FCH, d.T - tt0));
  const int e0 = ch * ECW, ecn = max(0, min(ECW, d.E - e0));
  const int len = fact ? lens[be] : 0;
  constexpr int CM = CC ? CC : PB_CM;
  const int C = CC ? CC : d.C;
  // cell role
  const int csl = tid / UPW, cu = tid % UPW;
  const int cb = grp + PD_GROUPS * csl, cj = u0 + cu;
  const bool cown = tid < PD_SLOTS * UPW && cu < nu && cb < d.B;
  float dc_reg = 0.f;

  // ---- once per pass
  constexpr int KB32 = F32 ? 8 * PB_KQ : 1;
  const int KQ32 = ((G4 + 3) / 4 + 3) / 4;   // f32 k-steps per K quarter
  bf16x8 wf[F32 ? 1 : PB_KQ];
  float wf32[KB32];
  {
    const int tile = wave & 1, kq = wave >> 1;
    const int c16 = tile * 16 + (lane & 15);
    const bool ok = c16 < nn;
    if constexpr (F32) {
      const float* wr = (const float*)wcatT_v + (long long)(ok ? n0 + c16 : 0) * G4;
#pragma unroll
      for (int i = 0; i < KB32; ++i) {
        const int k = 4 * (kq * KQ32 + i) + (lane >> 4);
        wf32[i] = (ok && i < KQ32 && k < G4) ? wr[k] : 0.f;
      }
    } else {
      const uint16_t* wr = (const uint16_t*)wcatT_v + (long long)(ok ? n0 + c16 : 0) * G4;
#pragma unroll
      for (int i = 0; i < PB_KQ; ++i) {
        const int kb = kq * G.KQ + i;
        const int k = kb * 32 + 8 * (lane >> 4);
        wf[i] = (ok && i < G.KQ && kb < G.NKB && k < G4)
                    ? load_bf16x8(wr + k) : as_bf16x8(u16x8{0, 0, 0, 0, 0, 0, 0, 0});
      }
    }
  }
  for (int i = tid; i < FCH * d.E; i += PD_THREADS) {
    const int fi = i / d.E, e = i % d.E;
    L[G.encr + i] = (fact && fi < nfr) ? enc[((long long)be * d.T + tt0 + fi) * d.E + e] : 0.f;
  }
  for (int i = tid; i < FCH * d.A; i += PD_THREADS) {
    const int fi = i / d.A, a = i % d.A;
    L[G.ea + i] = (fact && fi < nfr) ? enc_a[((long long)be * d.T + tt0 + fi) * d.A + a] : 0.f;
  }
  for (int i = tid; i < d.C * G.KP; i += PD_THREADS) {
    const int c = i / G.KP, k = i % G.KP;
    L[G.cw + i] = k < d.K ? conv_w[c * d.K + k] : 0.f;
  }
  for (int i = tid; i < d.A * d.C; i += PD_THREADS) L[G.wc + i] = w_conv[i];
  for (int i = tid; i < d.A; i += PD_THREADS) L[G.v + i] = vw[i];
  for (int i = tid; i < d.A * UPW; i += PD_THREADS) {
    const int a = i / UPW, u = i % UPW;
    L[G.wdl + i] = u < nu ? w_dec[(long long)a * d.D + u0 + u] : 0.f;
  }
  for (int i = tid; i < FCH; i += PD_THREADS) L[G.carry + i] = 0.f;
  // accumulators over the whole pass: the dV partial of this thread's (unit,
  // frame group) pairs; the chunk's dW_conv tiles (rows a = (wave + 8 j) 16 ..,
  // columns c) and conv-kernel tiles (rows c, columns k = (wave + 8 j) 16 ..)
  // as MFMA accumulators.  d enc_a: this work-group's rows of d_enc_a, zeroed
  // by the host, read-modify-written per step.
  const int NG = PD_THREADS / d.A, ta = tid % d.A, fg = tid / d.A;
  float accVr = 0.f;
  float accWc[CM];   // dW_conv row of this thread's attention unit (its frame group's part)
#pragma unroll
  for (int c = 0; c < CM; ++c) accWc[c] = 0.f;
  f32x4 dcwM[2];
  dcwM[0] = f32x4{0.f, 0.f, 0.f, 0.f};
  dcwM[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  int nph = 0;
  __syncthreads();

#define PB_WAIT()                                                              \
  do {                                                                         \
    if (nph > 0) {                                                             \
      if (tid == 0) s_ok = pd_wait(my_ctr, PD_MEMBERS * nph, ctr, status);     \
      __syncthreads();                                                         \
      if (!s_ok) return;                                                       \
    }                                                                          \
  } while (0)
#define PB_PUBLISH()     \
  do {                   \
    pd_publish(my_ctr);  \
    ++nph;               \
  } while (0)

  for (int t = d.S - 1; t >= 0; --t) {
    const bool has_r = t + 1 < d.S;
    PD_TR(48);
    // ================= H: r = dgates_{t+1} Wcat (this member's columns) =================
    // the dF window phase E reads (written by the previous step's F phase,
    // complete once H's wait has passed): loaded right after that wait, so
    // its latency passes behind H
    constexpr int PB_DFR = 5;   // registers per thread (8 + KW) C <= 5 x 512 (production 2400)
    // (the bf16 production geometry only: the f32 and runtime-geometry
    // instantiations have no registers to spare)
    constexpr bool PB_PREF = !F32 && SE != 0;
    const bool dfpre = PB_PREF && fact && has_r && (8 + KW) * C <= PB_DFR * PD_THREADS;
    float dfv[PB_DFR];
    if (has_r) {
      PB_WAIT();
      if (dfpre) {
#pragma unroll
        for (int j = 0; j < PB_DFR; ++j) {
          const int i = tid + j * PD_THREADS;
          const int row = i / C - 8, c = i % C, tt = tt0 - half + row;
          dfv[j] = (i < (8 + KW) * C && row >= 0 && tt >= 0 && tt < d.T)
                       ? pd_ld(rf, ((long long)be * d.T + tt) * d.C + c) : 0.f;
        }
      }
      PD_TR(49);
      uint16_t* dgs = reinterpret_cast<uint16_t*>(&L[G.dgs]);
      const int nv = G4 / 4;
      for (int i = tid; i < PD_SLOTS * nv; i += PD_THREADS) {
        const int sl = i / nv, k4 = i % nv, bb = grp + PD_GROUPS * sl;
        pd_u32x4 v = {0u, 0u, 0u, 0u};
        if (bb < d.B)
          v = __builtin_amdgcn_raw_buffer_load_b128(
              rg, (unsigned)((((long long)bb * d.S + t + 1) * G4 + 4 * k4) * 4), 0, 16);
        if constexpr (F32) {
          *reinterpret_cast<pd_u32x4*>(&L[G.dgs + sl * G4 + 4 * k4]) = v;
        } else {
          uint16_t* o = dgs + sl * G4 + 4 * k4;
          o[0] = f2bf(__uint_as_float(v[0]));
          o[1] = f2bf(__uint_as_float(v[1]));
          o[2] = f2bf(__uint_as_float(v[2]));
          o[3] = f2bf(__uint_as_float(v[3]));
        }
      }
      __syncthreads();
      if constexpr (F32) {
        const int kq = wave >> 1, mm = lane & 15;
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < KB32; ++i) {
          const int k = 4 * (kq * KQ32 + i) + (lane >> 4);
          if (i < KQ32 && 4 * (kq * KQ32 + i) < G4) {   // wave-uniform
            const float a = (mm < PD_SLOTS && k < G4) ? L[G.dgs + mm * G4 + k] : 0.f;
            if (i & 1) acc1 = mfma_f32(a, wf32[i], acc1);
            else acc0 = mfma_f32(a, wf32[i], acc0);
          }
        }
        if (lane < 16) {
#pragma unroll
          for (int rr4 = 0; rr4 < 4; ++rr4)
            L[G.part + (wave * PD_SLOTS + rr4) * 16 + lane] = acc0[rr4] + acc1[rr4];
        }
      } else {
        const int kq = wave >> 1, mm = lane & 15;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < PB_KQ; ++i) {
          const int kb = kq * G.KQ + i;
          if (i < G.KQ && kb < G.NKB) {   // wave-uniform
            const int k = kb * 32 + 8 * (lane >> 4);
            const bf16x8 a = (mm < PD_SLOTS && k < G4) ? load_bf16x8(dgs + mm * G4 + k)
                                                      : as_bf16x8(u16x8{0, 0, 0, 0, 0, 0, 0, 0});
            acc = mfma_bf16(a, wf[i], acc);
          }
        }
        if (lane < 16) {
#pragma unroll
          for (int rr4 = 0; rr4 < 4; ++rr4) L[G.part + (wave * PD_SLOTS + rr4) * 16 + lane] = acc[rr4];
        }
      }
      __syncthreads();
      if (tid < PD_SLOTS * 32) {
        const int sl = tid >> 5, c32 = tid & 31, tile = c32 >> 4, col = c32 & 15;
        const int bb = grp + PD_GROUPS * sl;
        if (c32 < nn && bb < d.B) {
          float s = 0.f;
#pragma unroll
          for (int kq = 0; kq < 4; ++kq) s += L[G.part + ((2 * kq + tile) * PD_SLOTS + sl) * 16 + col];
          pd_st(rr, (long long)bb * ED + n0 + c32, s);
        }
      }
      PD_TR(50);
      PB_PUBLISH();
    }
    PD_TR(51);

    // ================= E: d ctx_t, d aw_t, softmax chunk sums; conv features =================
    // this step's forward outputs (no hand-off: d_ctx_in, aw_t of the chunk, the
    // aw_{t-1} window, W_dec h_t) are loaded first, so their latency passes
    // behind the conv transpose below; they go to LDS after it (its aw window
    // of step t + 1 is still in use until then)
    const int pn1 = d.E, pn2 = pn1 + FCH, pn3 = pn2 + KW, ptotal = pn3 + d.A;
    const long long pst = (long long)be * d.S + t;
    auto pre_load = [&](int base, float (&v)[4]) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = base + j * PD_THREADS + tid;
        float x = 0.f;
        if (i < pn1) {
          x = d_ctx_in[pst * d.E + i];
        } else if (i < pn2) {
          if (i - pn1 < nfr) x = aw_all[pst * d.T + tt0 + (i - pn1)];
        } else if (i < pn3) {
          const int tt = tt0 - half + (i - pn2);
          if (t > 0 && tt >= 0 && tt < d.T) x = aw_all[(pst - 1) * d.T + tt];
        } else if (i < ptotal) {
          x = wd_all[pst * d.A + (i - pn3)];
        }
        v[j] = x;
      }
    };
    float pv0[4] = {0.f, 0.f, 0.f, 0.f};
    if (PB_PREF && fact) pre_load(0, pv0);
    // the conv features of aw_{t-1}: kept by the forward pass (fsave) instead
    // of recomputed (the same pd_conv_feat on the same aw values: bitwise)
    // (FS: a separate instantiation -- the load and the recompute paths in one
    // kernel cost the production bf16 kernel a 12-B spill, +4.6 ms / att step)
    const float* fsv = FS ? fsave + (((long long)be * d.S + t) * PD_CHUNKS + ch) * FCH * G.FS
                          : nullptr;
    const bool fpre = PB_PREF && FS && fact && t > 0 && FCH * G.FS <= PD_THREADS;
    const float fv0 = (fpre && tid < FCH * G.FS) ? fsv[tid] : 0.f;
    // the previous step's (t + 1) conv transpose -> d aw_t carry and conv-kernel
    // tiles, moved here from its G phase: they feed only this phase's d aw, so
    // they run beside this phase's wait instead of on the dgates hand-off
    // chain (G -> H).  The dF window goes to `un` after H is done with it; the
    // aw_t window of step t + 1 is still in `awin` (reloaded below).
    if (fact && has_r) {
      {   // dF window rows [tt0 - half, tt0 + FCH + half) after 8 zero rows
        if (dfpre) {
#pragma unroll
          for (int j = 0; j < PB_DFR; ++j) {
            const int i = tid + j * PD_THREADS;
            if (i < (8 + KW) * C) L[G.un + i] = dfv[j];
          }
        } else {
          for (int i = tid; i < (8 + KW) * C; i += PD_THREADS) {
            const int row = i / C - 8, c = i % C, tt = tt0 - half + row;
            L[G.un + i] = (row >= 0 && tt >= 0 && tt < d.T)
                              ? pd_ld(rf, ((long long)be * d.T + tt) * d.C + c) : 0.f;
          }
        }
      }
      __syncthreads();
      PD_TR(18);
      {
        // d aw_{t-1}[j] = sum_c sum_k dF[j - k + half, c] cw[c, k] (dF window row
        // j + K - 1 - k): (channel, 4 frames, K quarter) per item with a sliding
        // 4-row register window -- two LDS loads per 4 products
        const float* dFw = &L[G.un + 8 * C];   // row r of the window (rows -8..-1 are zero)
        float* cp = &L[G.cmb];   // [4 quarters][FCH4][C]
        const int NJG = (FCH + 3) / 4, FCH4 = NJG * 4, KQ4 = G.KQ4;
        for (int it = tid; it < C * NJG * 4; it += PD_THREADS) {
          const int kq = it & 3, rest = it >> 2, c = rest % C, jg = rest / C;
          const int j0 = jg * 4, k0 = kq * KQ4;
          float o0 = 0.f, o1 = 0.f, o2 = 0.f, o3 = 0.f;
          if (j0 < nfr) {   // taps past K are zero in the padded kernel rows
            int r = j0 + d.K - 1 - k0;
            float w0 = dFw[r * C + c], w1 = dFw[(r + 1) * C + c], w2 = dFw[(r + 2) * C + c],
                  w3 = dFw[(r + 3) * C + c];
            const float* cwr = &L[G.cw + c * G.KP + k0];
            for (int k = 0; k < KQ4; k += 4) {   // four taps' loads first, no branches
              const float4 cv = *reinterpret_cast<const float4*>(cwr + k);
              const float n0 = dFw[(r - 1) * C + c], n1 = dFw[(r - 2) * C + c],
                          n2 = dFw[(r - 3) * C + c], n3 = dFw[(r - 4) * C + c];
              o0 += w0 * cv.x; o1 += w1 * cv.x; o2 += w2 * cv.x; o3 += w3 * cv.x;
              o0 += n0 * cv.y; o1 += w0 * cv.y; o2 += w1 * cv.y; o3 += w2 * cv.y;
              o0 += n1 * cv.z; o1 += n0 * cv.z; o2 += w0 * cv.z; o3 += w1 * cv.z;
              o0 += n2 * cv.w; o1 += n1 * cv.w; o2 += n0 * cv.w; o3 += w0 * cv.w;
              w0 = n3;
              w1 = n2;
              w2 = n1;
              w3 = n0;
              r -= 4;
            }
          }
          float* o = cp + (kq * FCH4 + j0) * C + c;
          o[0] = o0;
          o[C] = o1;
          o[2 * C] = o2;
          o[3 * C] = o3;
        }
        PD_TR(10);
        // conv-kernel tiles: dcw[c][k] += sum_{own frames} dF[i][c] aw_{t-1}[i + k]
  #pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int nt = wave + 8 * jj;
          if (nt * 16 < d.K) {   // wave-uniform
            const int crow = lane & 15, kk = lane >> 4, kcol = nt * 16 + (lane & 15);
            const int nks = (FCH + 3) / 4;
            f32x4 acc = dcwM[jj];
            for (int st = 0; st < nks; st += 4) {
              float a4[4], b4[4];
  #pragma unroll
              for (int j = 0; j < 4; ++j) {
                const int i = (st + j) * 4 + kk;
                const bool ok = st + j < nks && i < nfr;
                const int ic = min(i, FCH - 1);
                const float av = dFw[(half + ic) * C + min(crow, C - 1)];
                const float bv = L[G.awin + ic + min(kcol, d.K - 1)];
                a4[j] = (ok && crow < C) ? av : 0.f;
                b4[j] = (ok && kcol < d.K) ? bv : 0.f;
              }
  #pragma unroll
              for (int j = 0; j < 4; ++j) acc = mfma_f32(a4[j], b4[j], acc);
            }
            dcwM[jj] = acc;
          }
        }
      }
      __syncthreads();
      PD_TR(19);
      {
        const int FCH4 = ((FCH + 3) / 4) * 4;
        for (int i = tid; i < FCH; i += PD_THREADS) {
          float s = 0.f;
          for (int kq = 0; kq < 4; ++kq)
            for (int c = 0; c < C; ++c) s += L[G.cmb + (kq * FCH4 + i) * C + c];
          L[G.carry + i] = s;
        }
      }
      __syncthreads();
      PD_TR(27);
    }
    // before the wait (forward outputs, no hand-off): d_ctx_in, aw_t of the
    // chunk, the aw_{t-1} window, W_dec h_t, in one batch of loads; the conv
    // features of aw_{t-1}
    if (fact) {
      for (int base = 0; base < ptotal; base += 4 * PD_THREADS) {
        float v[4];
        if (PB_PREF && base == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = pv0[j];
        } else {
          pre_load(base, v);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = base + j * PD_THREADS + tid;
          if (i < pn1) L[G.dct + i] = v[j];
          else if (i < pn2) L[G.awt + i - pn1] = v[j];
          else if (i < pn3) L[G.awin + i - pn2] = v[j];
          else if (i < ptotal) L[G.wd + i - pn3] = v[j];
        }
      }
      __syncthreads();
      PD_TR(28);
      if (t > 0 && fpre) {
        if (tid < FCH * G.FS) L[G.f + tid] = fv0;
      } else if (FS && t > 0) {
        for (int i = tid; i < FCH * G.FS; i += PD_THREADS) L[G.f + i] = fsv[i];
      } else if (!FS && t > 0) {
        pd_conv_feat(&L[G.cw], &L[G.awin], C, d.K, FCH, &L[G.un], &L[G.f], G.FS, G.KP);
      } else {
        for (int i = tid; i < FCH * G.FS; i += PD_THREADS) L[G.f + i] = 0.f;
      }
      PD_TR(29);
    }
    PB_WAIT();
    PD_TR(52);
    if (fact) {
      for (int e = tid; e < d.E; e += PD_THREADS) {
        float v = L[G.dct + e];
        if (has_r) v += pd_ld(rr, (long long)be * ED + e);
        L[G.dct + e] = v;
        if (e >= e0 && e < e0 + ecn) dctx_tot[((long long)be * d.S + t) * d.E + e] = v;
      }
      __syncthreads();
      // d aw over this wave's frames: lanes over e
#pragma unroll
      for (int f = 0; f < PD_FPW; ++f) {
        const int i = wave + 8 * f;
        if (i >= nfr) break;
        float s = lane < d.E ? dot_lds(&L[G.encr + i * d.E + lane], 64, &L[G.dct + lane], 64,
                                       (d.E - lane + 63) / 64) : 0.f;
        s = wave_sum(s);
        if (lane == 0) L[G.daw + i] = L[G.carry + i] + s;
      }
      __syncthreads();
      if (wave == 0) {
        float s = 0.f;
        for (int i = lane; i < nfr; i += 64) s += L[G.awt + i] * L[G.daw + i];
        s = wave_sum(s);
        if (lane == 0) pd_st(rs, (long long)be * PD_CHUNKS + ch, s);
      }
    }
    PD_TR(53);
    PB_PUBLISH();
    PD_TR(54);

    // ================= F: softmax / tanh backward of the chunk =================
    // before the wait: this work-group's d enc_a rows (its own earlier
    // read-modify-writes; sc1 loads: other waves of the work-group wrote them)
    if (fact) {
      const __amdgpu_buffer_rsrc_t ra =
          pd_rsrc(d_enc_a + (long long)be * d.T * d.A, (unsigned)((size_t)d.T * d.A * 4));
      for (int i = tid; i < nfr * d.A; i += PD_THREADS)
        L[G.un + (i / d.A) * G.AP + i % d.A] = pd_ld(ra, (long long)tt0 * d.A + i);
    }
    PB_WAIT();
    PD_TR(55);
    if (fact) {
      if (wave == 0) {
        float s = lane < PD_CHUNKS ? pd_ld(rs, (long long)be * PD_CHUNKS + lane) : 0.f;
        s = wave_sum(s);
        if (lane == 0) s_sdot = s;
      }
      __syncthreads();
      PD_TR(0);
      const float sdot = s_sdot;
      for (int i = tid; i < FCH; i += PD_THREADS) {
        const int tt = tt0 + i;
        float de = 0.f;
        if (i < nfr && tt < len) {
          const float a = L[G.awt + i], g = L[G.daw + i];
          de = (d.sigmoid ? g * a * (1.f - a) : a * (g - sdot)) * d.sharpen;
        }
        L[G.de + i] = de;
      }
      __syncthreads();
      PD_TR(1);
      // (frame, attention unit) pairs, thread (a = tid % A, frame group tid / A):
      // tanh backward -> dp, d enc_a; dp tile [FCH][A] over the d enc_a rows.
      // The thread also accumulates, for its (a, frames), the dW_conv row
      // dp f (the pass's accumulators, registers) and the chunk's dWd sum.
      if (fg < NG) {
        float wcr[CM];
#pragma unroll
        for (int c = 0; c < CM; ++c) wcr[c] = (CC || c < C) ? L[G.wc + ta * C + c] : 0.f;
        const float va = L[G.v + ta], wda = L[G.wd + ta];
        float sdp = 0.f;
        for (int i = fg; i < FCH; i += NG) {
          const float de = L[G.de + i];   // 0 beyond nfr
          float dp = 0.f;
          if (de != 0.f) {
            constexpr int CM4 = (CM + 3) / 4;
            float frv[CM4 * 4];
#pragma unroll
            for (int c4 = 0; c4 < CM4; ++c4) {
              const float4 v4 = 4 * c4 < G.FS ? *reinterpret_cast<const float4*>(&L[G.f + i * G.FS + 4 * c4])
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
              frv[4 * c4] = v4.x;
              frv[4 * c4 + 1] = v4.y;
              frv[4 * c4 + 2] = v4.z;
              frv[4 * c4 + 3] = v4.w;
            }
            float p = L[G.ea + i * d.A + ta] + wda;
#pragma unroll
            for (int c = 0; c < CM; ++c)
              if (CC || c < C) p += frv[c] * wcr[c];
            const float th = pd_tanh(p);
            dp = de * va * (1.f - th * th);
            accVr += de * th;
#pragma unroll
            for (int c = 0; c < CM; ++c) accWc[c] += dp * frv[c];
            sdp += dp;
            d_enc_a[((long long)be * d.T + tt0 + i) * d.A + ta] = L[G.un + i * G.AP + ta] + dp;
          }
          L[G.un + i * G.AP + ta] = dp;
        }
        L[G.part + fg * d.A + ta] = sdp;   // NG * A <= 512 = the part region
      }
      __syncthreads();
      PD_TR(2);
      // dF [frames][C] = dp . W_conv: row tile rt, K half kh per wave (the
      // halves summed below in order)
      const int MT = FCH <= 16 ? 1 : FCH <= 32 ? 2 : 4;
      const int nks = (d.A + 3) / 4;
      const int KH = (2 * MT * 256 <= G.cmbn && 2 * MT <= PD_THREADS / 64) ? 2 : 1;
      const int nh = KH == 2 ? ((nks + 7) / 8) * 4 : nks;
      if (wave < KH * MT) {
        const int rt = wave % MT, kh = wave / MT;
        const int row = rt * 16 + (lane & 15), kk = lane >> 4, col = lane & 15;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int st = kh * nh; st < (kh + 1 == KH ? nks : nh); st += 4) {
          float a4[4], b4[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int k = (st + j) * 4 + kk;
            const bool ok = st + j < nks && k < d.A;
            const int kc = min(k, d.A - 1);
            const float av = L[G.un + min(row, FCH - 1) * G.AP + kc];
            const float bv = L[G.wc + kc * C + min(col, C - 1)];
            a4[j] = (ok && row < FCH) ? av : 0.f;
            b4[j] = (ok && col < C) ? bv : 0.f;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) acc = mfma_f32(a4[j], b4[j], acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
          L[G.cmb + ((kh * MT + rt) * 16 + 4 * (lane >> 4) + r) * 16 + col] = acc[r];
      }
      __syncthreads();
      PD_TR(3);
      for (int idx = tid; idx < MT * 256; idx += PD_THREADS) {
        const int rt = idx >> 8, r16 = (idx >> 4) & 15, col = idx & 15;
        const int i = rt * 16 + r16;
        float v = L[G.cmb + idx];
        if (KH == 2) v += L[G.cmb + MT * 256 + idx];
        if (i < nfr && col < C) pd_st(rf, ((long long)be * d.T + tt0 + i) * d.C + col, v);
      }
      PD_TR(4);
      // the chunk's d W_dec-input sum over its frames (frame-group partials in order)
      for (int a = tid; a < d.A; a += PD_THREADS) {
        float sacc = 0.f;
        for (int q = 0; q < NG; ++q) sacc += L[G.part + q * d.A + a];
        pd_st(rw, ((long long)be * PD_CHUNKS + ch) * d.A + a, sacc);
      }
    }
    PD_TR(56);
    PB_PUBLISH();
    PD_TR(57);

    // ================= G: conv transpose (frames), LSTMCell backward (units) =================
    // before the wait: the cell's operands (forward outputs; r of step t+1 was
    // handed off before phase E)
    float g_ig = 0.f, g_fg = 0.f, g_gg = 0.f, g_og = 0.f, g_c = 0.f, g_cp = 0.f, g_dh = 0.f;
    if (cown) {
      g_dh = d_dec_in[((long long)cb * d.S + t) * d.D + cj] +
             (has_r ? pd_ld(rr, (long long)cb * ED + d.E + cj) : 0.f);
      if (t > 0) {
        const long long gb = ((long long)cb * d.S + t) * G4 + cj;
        g_ig = gates[gb];
        g_fg = gates[gb + d.D];
        g_gg = gates[gb + 2 * d.D];
        g_og = gates[gb + 3 * d.D];
        g_c = c_all[((long long)cb * d.S + t) * d.D + cj];
        g_cp = c_all[((long long)cb * d.S + t - 1) * d.D + cj];
      }
    }
    PB_WAIT();
    PD_TR(58);
    for (int i = tid; i < PD_SLOTS * d.A; i += PD_THREADS) {   // dWd_t of the 4 utterances
      const int sl = i / d.A, a = i % d.A, bb = grp + PD_GROUPS * sl;
      float s = 0.f;
      if (bb < d.B) {
        float v8[PD_CHUNKS];
#pragma unroll
        for (int j = 0; j < PD_CHUNKS; ++j)
          v8[j] = pd_ld(rw, ((long long)bb * PD_CHUNKS + j) * d.A + a);
#pragma unroll
        for (int j = 0; j < PD_CHUNKS; ++j) s += v8[j];
        if (m == 0) dwd_all[((long long)bb * d.S + t) * d.A + a] = s;
      }
      L[G.dwdl + i] = s;
    }
    __syncthreads();
    PD_TR(59);
    PD_TR(11);
    // d dec from the attention, W_dec^T dWd_t over this member's units:
    // (slot, unit, eighth of A) per thread, eighths summed in order
    float* ddp = &L[G.un + (8 + KW) * C];
    {
      const int np = PD_SLOTS * UPW * 8;
      const int a8 = (d.A + 7) / 8;
      for (int i = tid; i < np; i += PD_THREADS) {
        const int su = i >> 3, e8 = i & 7, sl = su / UPW, u = su % UPW;
        const int a0 = e8 * a8, a1 = min(d.A, a0 + a8);
        float s0 = 0.f, s1 = 0.f;
        int a = a0;
        for (; a + 1 < a1; a += 2) {
          s0 += L[G.wdl + a * UPW + u] * L[G.dwdl + sl * d.A + a];
          s1 += L[G.wdl + (a + 1) * UPW + u] * L[G.dwdl + sl * d.A + a + 1];
        }
        if (a < a1) s0 += L[G.wdl + a * UPW + u] * L[G.dwdl + sl * d.A + a];
        ddp[i] = s0 + s1;
      }
    }
    __syncthreads();
    PD_TR(12);
    if (cown) {
      float dd = 0.f;
#pragma unroll
      for (int e8 = 0; e8 < 8; ++e8) dd += ddp[tid * 8 + e8];
      const float dh = g_dh + dd;
      if (t == 0) {
        if (d_h0) d_h0[(long long)cb * d.D + cj] = dh;
      } else {
        const float dhr =
            drop_h > 0.f ? dh * drop_scale(drop_h, seed_h, ((unsigned long long)cb * d.S + t) * d.D + cj)
                         : dh;
        const long long gb = ((long long)cb * d.S + t) * G4 + cj;
        const float ig = g_ig, fg = g_fg, gg = g_gg, og = g_og, c = g_c, cprev = g_cp;
        const float tc = tanhf(c);
        const float dcell = dc_reg + dhr * og * (1.f - tc * tc);
        pd_st(rg, gb, dcell * gg * ig * (1.f - ig));
        pd_st(rg, gb + d.D, dcell * cprev * fg * (1.f - fg));
        pd_st(rg, gb + 2 * d.D, dcell * ig * (1.f - gg * gg));
        pd_st(rg, gb + 3 * d.D, dhr * tc * og * (1.f - og));
        dc_reg = dcell * fg;
      }
    }
    PD_TR(13);
    __syncthreads();
    PD_TR(14);
    PD_TR(60);
    PB_PUBLISH();
    PD_TR(61);
  }
#undef PB_WAIT
#undef PB_PUBLISH

  // ---- end of pass: the chunk's weight-gradient partial rows
  if (!fact) return;
  const long long row = (long long)be * PD_CHUNKS + ch;
  float* cV = &L[G.cmb];
  __syncthreads();
  if (fg < NG) cV[fg * d.A + ta] = accVr;
  __syncthreads();
  for (int a = tid; a < d.A; a += PD_THREADS) {
    float s = 0.f;
    for (int q = 0; q < NG; ++q) s += cV[q * d.A + a];
    dv_part[row * d.A + a] = s;
  }
  // dW_conv: the frame groups' rows summed in order, one channel at a time
  for (int c = 0; c < C; ++c) {
    __syncthreads();
    float v = 0.f;
#pragma unroll
    for (int cc = 0; cc < CM; ++cc)
      if (cc == c) v = accWc[cc];
    if (fg < NG) cV[fg * d.A + ta] = v;
    __syncthreads();
    for (int a = tid; a < d.A; a += PD_THREADS) {
      float sacc = 0.f;
      for (int q = 0; q < NG; ++q) sacc += cV[q * d.A + a];
      dwc_part[row * d.A * d.C + a * d.C + c] = sacc;
    }
  }
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int nt = wave + 8 * jj;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 4 * (lane >> 4) + r, k = nt * 16 + (lane & 15);
      if (c < C && k < d.K) dcw_part[row * d.C * d.K + c * d.K + k] = dcwM[jj][r];
    }
  }
}

}  // namespace

int* lstm_persist_status_word();   // lstm_persist.hip

namespace {
int device_cus() {
  static int n = -1;
  if (n < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 0;
  }
  return n;
}

// The persistent forward pass takes a shape when its work split fits (see the
// kernel's comment) and the 256-work-group grid is co-resident, one per CU.
// ASR_ATT_PERSIST=0 keeps the per-step kernels (A/B).
// the instantiations: 2 = the production shape folded at compile time (10
// channels x 201, A 128, E 640, D 320), 1 = 10 channels with A <= 128, 0 =
// generic (C <= 4)
int pd_kind(const Dims& d) {
  if (d.C == 10 && d.A == 128 && d.E == 640 && d.D == 320 && d.K == 201) return 2;
  return d.C == 10 && d.A <= 128 ? 1 : 0;
}
bool pd_ten(const Dims& d) { return pd_kind(d) > 0; }
#define PD_SEL(K, KIND, F)                                                                   \
  ((KIND) == 2 ? (const void*)K<10, 2, 128, 640, 320, 201, F>                                \
               : (KIND) == 1 ? (const void*)K<10, 2, 0, 0, 0, 0, F>                          \
                             : (const void*)K<0, 4, 0, 0, 0, 0, F>)

// f32: fp32 mode (the f32-MFMA cell / r products).  ASR_ATT_PERSIST32=0 keeps
// fp32 mode on the per-step kernels.
bool pd_eligible(const Dims& d, bool f32, int ssY = 0, int ssDz = 0) {
  const char* e = getenv("ASR_ATT_PERSIST");
  if (e && e[0] == '0') return false;
  const char* e32 = getenv("ASR_ATT_PERSIST32");
  if (f32 && e32 && e32[0] == '0') return false;
  if (f32 && (d.E + d.D) % 4 != 0) return false;   // 16-B x rows
  const PdGeom G = pd_geom(d);
  const size_t lds = (size_t)(ssY ? pd_ss_geom(d, G.total, G.UPW, ssY,
                                               (ssDz + PD_MEMBERS - 1) / PD_MEMBERS).total
                                  : G.total) * 4;
  if (d.B > PD_GROUPS * PD_SLOTS || G.UPW > PD_UMAX || G.ED % 8 != 0 || G.NKB > 2 * PD_KMAX ||
      G.FCH > 8 * PD_FPW || d.A > 256 || (!pd_ten(d) && d.C > PD_CM) || G.ECW > PD_THREADS ||
      lds > 160 * 1024 ||
      (size_t)d.B * d.S * G.ED * 4 >= (1ull << 31) || (size_t)d.B * d.T * 4 >= (1ull << 31))
    return false;
  if (device_cus() < PD_GROUPS * PD_MEMBERS) return false;
  const void* k = f32 ? PD_SEL(attdec_fwd_persist, pd_kind(d), true)
                      : PD_SEL(attdec_fwd_persist, pd_kind(d), false);
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return false;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, PD_THREADS, lds) != hipSuccess)
    return false;
  return per_cu >= 1;
}

// Scheduled sampling inside the persistent forward (the sampled steps' phase of
// attdec_fwd_persist): classes, embedding and bottleneck within the in-pass
// limits, the ctx / h boundary of x where each K half's interleaved blocks
// split by index alone (E % 64 == 0), every operand given.
// ASR_ATT_PERSIST_SS=0: a pass with sampled steps takes the per-step kernels.
bool pd_ss_ok(const Dims& d, const asr_attdec_opts_t& o) {
  const char* e = getenv("ASR_ATT_PERSIST_SS");
  if (e && e[0] == '0') return false;
  return o.V > 0 && o.V <= PD_VMAX && o.Y > 0 && o.Y <= PD_YMAX && o.Dz > 0 &&
         (o.Dz + PD_MEMBERS - 1) / PD_MEMBERS <= PD_ZMAX && d.E % 64 == 0 && o.w_d && o.w_c &&
         o.w_fc && o.emb_w && o.w_ih_emb && o.b_ih && o.b_hh && o.pre_ss && o.emb_ss;
}

bool pb_eligible(const Dims& d, bool f32) {
  const char* e = getenv("ASR_ATT_PERSIST");
  if (e && e[0] == '0') return false;
  const char* eb = getenv("ASR_ATT_PERSIST_BWD");
  if (eb && eb[0] == '0') return false;
  const char* e32 = getenv("ASR_ATT_PERSIST32");
  if (f32 && e32 && e32[0] == '0') return false;
  if (f32 && ((4 * d.D + 3) / 4 + 3) / 4 > 8 * PB_KQ) return false;
  const PbGeom G = pb_geom(d, f32);
  const size_t lds = (size_t)G.total * 4;
  if (d.B > PD_GROUPS * PD_SLOTS || G.UPW > PD_UMAX || G.NPW > 32 || G.G4 % 8 != 0 ||
      G.KQ > PB_KQ || G.FCH > 8 * PD_FPW || d.A > 256 || (!pd_ten(d) && d.C > PB_CM) ||
      d.K > 16 * 16 ||
      lds > 160 * 1024 || (size_t)d.B * d.S * G.G4 * 4 >= (1ull << 31) ||
      (size_t)d.B * d.T * d.C * 4 >= (1ull << 31))
    return false;
  if (device_cus() < PD_GROUPS * PD_MEMBERS) return false;
  const void* k = f32 ? PD_SEL(attdec_bwd_persist, pd_kind(d), true)
                      : PD_SEL(attdec_bwd_persist, pd_kind(d), false);
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return false;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, PD_THREADS, lds) != hipSuccess)
    return false;
  return per_cu >= 1;
}
}  // namespace
}  // namespace asr

using namespace asr;

extern "C" int asr_att_trace_read(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(asr::g_att_tr), sizeof(asr::g_att_tr)) ==
                 hipSuccess ? ASR_OK : ASR_ERR_HIP;
}

extern "C" size_t asr_attdec_workspace_bytes(const asr_attdec_dims_t* dims, int compute_dtype,
                                             int backward) {
  return att_ws(to_dims(*dims), compute_dtype, backward != 0).total;
}

// Rows per utterance of the backward partials dv_part, dwc_part and dcw_part
// (B * this many rows, each summed over the steps; rows a pass does not use
// are written zero).
extern "C" int asr_attdec_chunks(const asr_attdec_dims_t* dims) {
  return part_rows(to_dims(*dims));
}

namespace {
int check_opts(const Dims& d, const asr_attdec_opts_t* o, bool* ss) {
  *ss = false;
  if (!o) return ASR_OK;
  ASR_REQUIRE(o->dropout_hidden >= 0.f && o->dropout_hidden < 1.f, ASR_ERR_ARG,
              "attdec: dropout_hidden=%f", o->dropout_hidden);
  if (!o->ss_steps_host) return ASR_OK;
  for (int t = 1; t < d.S; ++t) *ss |= o->ss_steps_host[t] != 0;
  if (!*ss) return ASR_OK;
  ASR_REQUIRE(o->Y > 0 && o->Dz > 0 && o->V > 0 && o->w_d && o->w_c && o->w_fc && o->emb_w &&
                  o->w_ih_emb && o->b_ih && o->b_hh && o->pre_ss && o->emb_ss,
              ASR_ERR_ARG, "attdec: scheduled sampling needs Y/Dz/V and its weights");
  ASR_REQUIRE(o->drop_d >= 0.f && o->drop_d < 1.f && o->drop_c >= 0.f && o->drop_c < 1.f &&
                  o->drop_emb >= 0.f && o->drop_emb < 1.f,
              ASR_ERR_ARG, "attdec: bad dropout probability");
  return ASR_OK;
}
}  // namespace

extern "C" int asr_attdec_forward(const asr_attdec_dims_t* dims, int compute_dtype,
                                  const float* enc, const float* enc_a, const int32_t* lens,
                                  const float* w_ih_ctx, long long ld_ih, const float* w_hh,
                                  const float* w_dec, const float* w_conv, const float* conv_w,
                                  const float* v, const float* pre_emb, const float* h0,
                                  float* dec, float* c_all, float* gates, float* x,
                                  float* ctx_all, float* aw_all, void* workspace,
                                  size_t ws_bytes, void* stream) {
  return asr_attdec_forward_ex(dims, nullptr, compute_dtype, enc, enc_a, lens, w_ih_ctx, ld_ih,
                               w_hh, w_dec, w_conv, conv_w, v, pre_emb, h0, dec, c_all, gates, x,
                               ctx_all, aw_all, workspace, ws_bytes, stream);
}

// Algorithmic bytes of one decoder pass: per decoder step and
// utterance the attention reads enc_out_a (A), enc_out (E) and the previous
// weights / writes the new ones (2 values) over T' frames, 4 B each.
static double att_pass_bytes(const Dims& d) {
  return (double)d.B * d.S * (d.A + d.E + 2) * 4.0 * d.T;
}

// Which attention-step instantiations the last forward / backward launched:
// {forward channel template (10, 3 or 0 = generic), forward frame chunks,
//  backward channel template, backward frame chunks} (host-side record).
static int g_att_last[4];
static int g_att_persist_last[2];   // {forward pass persistent, backward pass persistent}

extern "C" int asr_attdec_forward_ex(const asr_attdec_dims_t* dims, const asr_attdec_opts_t* opts,
                                     int compute_dtype, const float* enc, const float* enc_a,
                                     const int32_t* lens, const float* w_ih_ctx, long long ld_ih,
                                     const float* w_hh, const float* w_dec, const float* w_conv,
                                     const float* conv_w, const float* v, const float* pre_emb,
                                     const float* h0, float* dec, float* c_all, float* gates,
                                     float* x, float* ctx_all, float* aw_all, void* workspace,
                                     size_t ws_bytes, void* stream) {
  ASR_REQUIRE(dims, ASR_ERR_ARG, "attdec: dims is null");
  const Dims d = to_dims(*dims);
  int rc = check_dims(d);
  if (rc) return rc;
  bool ss = false;
  rc = check_opts(d, opts, &ss);
  if (rc) return rc;
  const float drop_h = opts ? opts->dropout_hidden : 0.f;
  const unsigned long long seed_h = opts ? opts->seed_hidden : 0ull;
  ASR_REQUIRE(enc && enc_a && lens && w_ih_ctx && w_hh && w_dec && w_conv && conv_w && v &&
                  pre_emb && dec && c_all && gates && x && ctx_all && aw_all && workspace,
              ASR_ERR_ARG, "attdec_forward: null pointer");
  ASR_REQUIRE(ws_bytes >= asr_attdec_workspace_bytes(dims, compute_dtype, 0), ASR_ERR_WORKSPACE,
              "attdec_forward: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const bool bf = compute_dtype == ASR_DT_BF16;
  const long long nw = 4LL * d.D * (d.E + d.D);
  const int gb = (int)((nw + 255) / 256 < 4096 ? (nw + 255) / 256 : 4096);
  if (bf)
    hipLaunchKernelGGL((build_wcat<uint16_t>), dim3(gb), dim3(256), 0, s, d, w_ih_ctx, ld_ih, w_hh,
                       (uint16_t*)workspace);
  else
    hipLaunchKernelGGL((build_wcat<float>), dim3(gb), dim3(256), 0, s, d, w_ih_ctx, ld_ih, w_hh,
                       (float*)workspace);
  ASR_LAUNCH_CHECK();
  hipLaunchKernelGGL(dec_init, dim3(d.B), dim3(256), 0, s, d, h0, dec, x, c_all, gates);
  ASR_LAUNCH_CHECK();
  const AttWs W = att_ws(d, compute_dtype, false);
  float* ebuf = (float*)((char*)workspace + W.ebuf);
  const size_t en_lds = en_lds_floats(d) * 4;
  const size_t cx_lds = ((size_t)d.T + 64 + ATT_THREADS) * 4;
  const dim3 eg(att_chunks(d), d.B), xg(ceil_div(d.E, ECH), d.B);
  const int vec = ((d.E + d.D) % 8 == 0) ? 1 : 0;
  const dim3 cg(ceil_div(d.D, CU), ceil_div(d.B, MB));
  const size_t ss_lds = ss ? ((size_t)d.D + d.E + opts->Dz + opts->Y + 2 * (SS_THREADS / 64)) * 4
                          : 0;
  ASR_REQUIRE(ss_lds <= 160 * 1024, ASR_ERR_UNSUPPORTED, "attdec: sampling LDS %zu B", ss_lds);
  g_att_last[0] = (d.C == 10 || d.C == 3) ? d.C : 0;
  g_att_last[1] = (int)eg.x;
  g_att_persist_last[0] = 0;
  // sampled steps run inside the persistent pass when their operands fit its
  // limits (pd_ss_ok); otherwise such a pass takes the per-step kernels
  const bool ssin = ss && pd_ss_ok(d, *opts);
  const int ssY = ssin ? opts->Y : 0, ssDz = ssin ? opts->Dz : 0;
  if ((!ss || ssin) && pd_eligible(d, !bf, ssY, ssDz)) {
    const PdGeom G = pd_geom(d);
    int* ctr = (int*)((char*)workspace + W.ctr);
    float* pbuf = (float*)((char*)workspace + W.pbuf);
    ASR_CHECK_HIP(hipMemsetAsync(ctr, 0, (size_t)(1 + 2 * PD_GROUPS) * PD_CTR * 4, s));
    PdSs pss;
    memset(&pss, 0, sizeof(pss));
    PdSs* ssdev = nullptr;
    if (ssin) {
      int32_t* fl = (int32_t*)((char*)workspace + W.flags);
      ASR_CHECK_HIP(hipMemcpyAsync(fl, opts->ss_steps_host, (size_t)d.S * 4,
                                   hipMemcpyHostToDevice, s));
      pss.flags = fl;
      pss.w_d = opts->w_d; pss.b_d = opts->b_d; pss.w_c = opts->w_c; pss.b_c = opts->b_c;
      pss.w_fc = opts->w_fc; pss.b_fc = opts->b_fc; pss.emb_w = opts->emb_w;
      pss.w_ih_emb = opts->w_ih_emb; pss.b_ih = opts->b_ih; pss.b_hh = opts->b_hh;
      pss.drop_d = opts->drop_d; pss.drop_c = opts->drop_c; pss.drop_emb = opts->drop_emb;
      pss.seed_d = opts->seed_d; pss.seed_c = opts->seed_c; pss.seed_emb = opts->seed_emb;
      pss.Y = opts->Y; pss.Dz = opts->Dz; pss.V = opts->V; pss.emb_trans = opts->emb_trans;
      pss.ld_ih = opts->ld_ih;
      pss.pre_ss = opts->pre_ss; pss.emb_ss = opts->emb_ss; pss.tok_ss = opts->tok_ss;
      pss.lbuf = (float*)((char*)workspace + W.lbuf);
      void* zc = (char*)workspace + W.zcat;
      pss.zcat = zc;
      {
        const long long nz = (long long)opts->Dz * (d.E + d.D);
        const int gz = (int)((nz + 255) / 256 < 4096 ? (nz + 255) / 256 : 4096);
        if (bf)
          hipLaunchKernelGGL((build_zcat<uint16_t>), dim3(gz), dim3(256), 0, s, d, opts->Dz,
                             opts->w_c, opts->w_d, (uint16_t*)zc);
        else
          hipLaunchKernelGGL((build_zcat<float>), dim3(gz), dim3(256), 0, s, d, opts->Dz,
                             opts->w_c, opts->w_d, (float*)zc);
        ASR_LAUNCH_CHECK();
      }
      ssdev = (PdSs*)((char*)workspace + W.ssd);
      rc = pd_ss_upload(pss, ssdev, s);
      if (rc) return rc;
    }
    const size_t lds = (size_t)(ssin ? pd_ss_geom(d, G.total, G.UPW, ssY,
                                                  (ssDz + PD_MEMBERS - 1) / PD_MEMBERS).total
                                     : G.total) * 4;
    const dim3 grid(PD_GROUPS * PD_MEMBERS);
    // (A + E + 2) * 4 * T' algorithmic bytes per decoder step and utterance
    const int pslot = prof_begin_launch(ASR_PROF_ATT_FWD, s, att_pass_bytes(d));
#define ASR_PD2(CC, NQ, SA, SE, SD, SK, F)                                                         \
  hipLaunchKernelGGL((attdec_fwd_persist<CC, NQ, SA, SE, SD, SK, F>), grid, dim3(PD_THREADS), lds,  \
                     s, d, (const void*)workspace, pre_emb, h0, enc, enc_a, lens, w_dec, w_conv,  \
                     conv_w, v, dec, c_all, gates, x, ctx_all, aw_all, pbuf, ebuf, ctr,          \
                     lstm_persist_status_word(), drop_h, seed_h, ssdev, g_pd_fsave)
#define ASR_PD(CC, NQ, SA, SE, SD, SK)                  \
  do {                                                  \
    if (bf) ASR_PD2(CC, NQ, SA, SE, SD, SK, false);     \
    else ASR_PD2(CC, NQ, SA, SE, SD, SK, true);         \
  } while (0)
    if (pd_kind(d) == 2) ASR_PD(10, 2, 128, 640, 320, 201);
    else if (pd_kind(d) == 1) ASR_PD(10, 2, 0, 0, 0, 0);
    else ASR_PD(0, 4, 0, 0, 0, 0);
#undef ASR_PD
#undef ASR_PD2
    ASR_LAUNCH_CHECK();
    prof_end_launch(ASR_PROF_ATT_FWD, pslot, s);
    g_att_last[0] = pd_ten(d) ? 10 : 0;
    g_att_persist_last[0] = 1;
    return ASR_OK;
  }
  for (int t = 0; t < d.S; ++t) {
    if (t > 0) {
      const bool smp = ss && opts->ss_steps_host[t] != 0;
      if (smp) {
        hipLaunchKernelGGL(ss_step, dim3(d.B), dim3(SS_THREADS), ss_lds, s, t, d, *opts, dec,
                           ctx_all);
        ASR_LAUNCH_CHECK();
      }
      const float* pre = smp ? opts->pre_ss : pre_emb;
      if (bf)
        hipLaunchKernelGGL((cell_fwd<true, uint16_t>), cg, dim3(256), 0, s, t, d,
                           (const uint16_t*)workspace, pre, x, gates, c_all, dec, vec, drop_h,
                           seed_h);
      else
        hipLaunchKernelGGL((cell_fwd<false, float>), cg, dim3(256), 0, s, t, d,
                           (const float*)workspace, pre, x, gates, c_all, dec, vec, drop_h,
                           seed_h);
      ASR_LAUNCH_CHECK();
    }
    if (d.C == 10)
      hipLaunchKernelGGL(att_energy<10>, eg, dim3(ATT_THREADS), en_lds, s, t, d, enc_a, lens,
                         w_dec, w_conv, conv_w, v, dec, aw_all, ebuf);
    else if (d.C == 3)
      hipLaunchKernelGGL(att_energy<3>, eg, dim3(ATT_THREADS), en_lds, s, t, d, enc_a, lens,
                         w_dec, w_conv, conv_w, v, dec, aw_all, ebuf);
    else
      hipLaunchKernelGGL(att_energy<0>, eg, dim3(ATT_THREADS), en_lds, s, t, d, enc_a, lens,
                         w_dec, w_conv, conv_w, v, dec, aw_all, ebuf);
    ASR_LAUNCH_CHECK();
    hipLaunchKernelGGL(att_context, xg, dim3(ATT_THREADS), cx_lds, s, t, d, enc, ebuf, aw_all,
                       ctx_all, x);
    ASR_LAUNCH_CHECK();
  }
  return ASR_OK;
}

// {forward, backward}: 1 if the last decoder pass of that direction ran as
// one persistent launch (host-side record).
extern "C" int asr_attdec_persist_last(int* out2) {
  ASR_REQUIRE(out2, ASR_ERR_ARG, "attdec_persist_last: null pointer");
  out2[0] = g_att_persist_last[0];
  out2[1] = g_att_persist_last[1];
  return ASR_OK;
}

// The conv-feature buffer of the next persistent decoder pass from this host
// thread (NULL: none); asr_attdec_conv_feat_bytes: its size for dims.
extern "C" int asr_attdec_set_conv_feat(float* buf) {
  g_pd_fsave = buf;
  return ASR_OK;
}

extern "C" size_t asr_attdec_conv_feat_bytes(const asr_attdec_dims_t* dims) {
  if (!dims || dims->B <= 0 || dims->S <= 0 || dims->T <= 0) return 0;
  const size_t fch = (size_t)(dims->T + PD_CHUNKS - 1) / PD_CHUNKS;
  const size_t fs = (size_t)((dims->C + 3) & ~3);
  return (size_t)dims->B * dims->S * PD_CHUNKS * fch * fs * sizeof(float);
}

extern "C" int asr_attdec_last_launch(int* out4) {
  ASR_REQUIRE(out4, ASR_ERR_ARG, "attdec_last_launch: null pointer");
  for (int i = 0; i < 4; ++i) out4[i] = g_att_last[i];
  return ASR_OK;
}

extern "C" int asr_attdec_backward(const asr_attdec_dims_t* dims, int compute_dtype,
                                   const float* enc, const float* enc_a, const int32_t* lens,
                                   const float* w_ih_ctx, long long ld_ih, const float* w_hh,
                                   const float* w_dec, const float* w_conv, const float* conv_w,
                                   const float* v, const float* dec, const float* c_all,
                                   const float* aw_all, const float* d_dec_in,
                                   const float* d_ctx_in, float* gates_dg, float* dctx_tot,
                                   float* d_enc_a, float* d_h0, float* dwd_all, float* dv_part,
                                   float* dwc_part, float* dcw_part, void* workspace,
                                   size_t ws_bytes, void* stream) {
  return asr_attdec_backward_ex(dims, nullptr, compute_dtype, enc, enc_a, lens, w_ih_ctx, ld_ih,
                                w_hh, w_dec, w_conv, conv_w, v, dec, c_all, aw_all, d_dec_in,
                                d_ctx_in, gates_dg, dctx_tot, d_enc_a, d_h0, dwd_all, dv_part,
                                dwc_part, dcw_part, workspace, ws_bytes, stream);
}

extern "C" int asr_attdec_backward_ex(const asr_attdec_dims_t* dims, const asr_attdec_opts_t* opts,
                                      int compute_dtype, const float* enc, const float* enc_a,
                                      const int32_t* lens, const float* w_ih_ctx, long long ld_ih,
                                      const float* w_hh, const float* w_dec, const float* w_conv,
                                      const float* conv_w, const float* v, const float* dec,
                                      const float* c_all, const float* aw_all,
                                      const float* d_dec_in, const float* d_ctx_in,
                                      float* gates_dg, float* dctx_tot, float* d_enc_a,
                                      float* d_h0, float* dwd_all, float* dv_part,
                                      float* dwc_part, float* dcw_part, void* workspace,
                                      size_t ws_bytes, void* stream) {
  ASR_REQUIRE(dims, ASR_ERR_ARG, "attdec: dims is null");
  const Dims d = to_dims(*dims);
  int rc = check_dims(d);
  if (rc) return rc;
  bool ss = false;
  rc = check_opts(d, opts, &ss);
  if (rc) return rc;
  ASR_REQUIRE(!ss || (opts->d_pre && opts->dg_ss), ASR_ERR_ARG,
              "attdec_backward: scheduled sampling needs d_pre and dg_ss");
  const float drop_h = opts ? opts->dropout_hidden : 0.f;
  const unsigned long long seed_h = opts ? opts->seed_hidden : 0ull;
  ASR_REQUIRE(enc && enc_a && lens && w_ih_ctx && w_hh && w_dec && w_conv && conv_w && v &&
                  dec && c_all && aw_all && d_dec_in && d_ctx_in && gates_dg && dctx_tot &&
                  d_enc_a && dwd_all && dv_part && dwc_part && dcw_part && workspace,
              ASR_ERR_ARG, "attdec_backward: null pointer");
  ASR_REQUIRE(ws_bytes >= asr_attdec_workspace_bytes(dims, compute_dtype, 1), ASR_ERR_WORKSPACE,
              "attdec_backward: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const bool bf = compute_dtype == ASR_DT_BF16;
  const int ED = d.E + d.D, G = 4 * d.D;
  const AttWs W = att_ws(d, compute_dtype, true);
  char* p = (char*)workspace;
  void* wcatT = p + W.wcat;
  float* dawbuf = (float*)(p + W.ebuf);
  float* r = (float*)(p + W.r);
  float* carry = (float*)(p + W.carry);
  float* ddec_att = (float*)(p + W.ddec);
  float* dc = (float*)(p + W.dc);
  int32_t* flags = (int32_t*)(p + W.flags);
  float* dFbuf = (float*)(p + W.dF);
  float* dwd_chunk = (float*)(p + W.dwdc);
  float* wd_all = (float*)(p + W.wd);
  {  // W_dec dec_t for every step at once (exact-f32 MFMA, as the forward's f32 dot products)
    asr_gemm_t g;
    memset(&g, 0, sizeof(g));
    g.a.ptr = dec;
    g.a.dtype = ASR_DT_F32;
    g.a.map.stride_t = d.D;
    g.a.bytes = 4LL * d.B * d.S * d.D;   // the extents: the f32 fast kernel's buffer bounds
    g.b.ptr = w_dec;
    g.b.dtype = ASR_DT_F32;
    g.b.map.stride_t = d.D;
    g.b.bytes = 4LL * d.A * d.D;
    g.c = wd_all;
    g.c_map.stride_t = d.A;
    g.M = d.B * d.S; g.N = d.A; g.K = d.D;
    g.alpha = 1.f; g.beta = 0.f; g.batch = 1;
    rc = asr_gemm(&g, 1, ASR_DT_F32, stream);
    if (rc) return rc;
  }
  const long long nw = 4LL * d.D * ED;
  const int gb = (int)((nw + 255) / 256 < 4096 ? (nw + 255) / 256 : 4096);
  if (bf)
    hipLaunchKernelGGL((build_wcat_t<uint16_t>), dim3(gb), dim3(256), 0, s, d, w_ih_ctx, ld_ih,
                       w_hh, (uint16_t*)wcatT);
  else
    hipLaunchKernelGGL((build_wcat_t<float>), dim3(gb), dim3(256), 0, s, d, w_ih_ctx, ld_ih, w_hh,
                       (float*)wcatT);
  ASR_LAUNCH_CHECK();
  {  // rows of the partials a pass does not write stay zero
    const size_t prow = (size_t)d.B * part_rows(d);
    ASR_CHECK_HIP(hipMemsetAsync(dv_part, 0, prow * d.A * 4, s));
    ASR_CHECK_HIP(hipMemsetAsync(dwc_part, 0, prow * d.A * d.C * 4, s));
    ASR_CHECK_HIP(hipMemsetAsync(dcw_part, 0, prow * d.C * d.K * 4, s));
  }
  g_att_persist_last[1] = 0;
  if (pb_eligible(d, !bf)) {
    const PbGeom PG = pb_geom(d, !bf);
    int* ctr = (int*)(p + W.ctr);
    float* sbuf = (float*)(p + W.sbuf);
    ASR_CHECK_HIP(hipMemsetAsync(ctr, 0, (size_t)(1 + PD_GROUPS) * PD_CTR * 4, s));
    ASR_CHECK_HIP(hipMemsetAsync(d_enc_a, 0, (size_t)d.B * d.T * d.A * 4, s));
    const size_t lds = (size_t)PG.total * 4;
    const dim3 grid(PD_GROUPS * PD_MEMBERS);
    const int pslot = prof_begin_launch(ASR_PROF_ATT_BWD, s, att_pass_bytes(d));
#define ASR_PB3(CC, NQ, SA, SE, SD, SK, F, FS)                                                     \
  hipLaunchKernelGGL((attdec_bwd_persist<CC, NQ, SA, SE, SD, SK, F, FS>), grid, dim3(PD_THREADS),   \
                     lds,                                                                        \
                     s, d, (const void*)wcatT, enc, enc_a, lens, w_dec, w_conv, conv_w, v, c_all, \
                     aw_all, wd_all, d_dec_in, d_ctx_in, gates_dg, dctx_tot, d_enc_a, d_h0,      \
                     dwd_all, dv_part, dwc_part, dcw_part, r, sbuf, dwd_chunk, dFbuf, ctr,       \
                     lstm_persist_status_word(), drop_h, seed_h, (const float*)g_pd_fsave)
#define ASR_PB2(CC, NQ, SA, SE, SD, SK, F)                                       \
  do {                                                                          \
    if (g_pd_fsave) ASR_PB3(CC, NQ, SA, SE, SD, SK, F, true);                   \
    else ASR_PB3(CC, NQ, SA, SE, SD, SK, F, false);                             \
  } while (0)
#define ASR_PB(CC, NQ, SA, SE, SD, SK)                  \
  do {                                                  \
    if (bf) ASR_PB2(CC, NQ, SA, SE, SD, SK, false);     \
    else ASR_PB2(CC, NQ, SA, SE, SD, SK, true);         \
  } while (0)
    if (pd_kind(d) == 2) ASR_PB(10, 2, 128, 640, 320, 201);
    else if (pd_kind(d) == 1) ASR_PB(10, 2, 0, 0, 0, 0);
    else ASR_PB(0, 4, 0, 0, 0, 0);
#undef ASR_PB
#undef ASR_PB2
#undef ASR_PB3
    ASR_LAUNCH_CHECK();
    prof_end_launch(ASR_PROF_ATT_BWD, pslot, s);
    g_att_last[2] = pd_ten(d) ? 10 : 0;
    g_att_last[3] = att_chunks(d);   // (the frame split the per-step kernels would use)
    g_att_persist_last[1] = 1;
  } else {
  ASR_CHECK_HIP(hipMemsetAsync(carry, 0, (size_t)d.B * d.T * 4, s));
  ASR_CHECK_HIP(hipMemsetAsync(dc, 0, (size_t)d.B * d.D * 4, s));
  ASR_CHECK_HIP(hipMemsetAsync(d_enc_a, 0, (size_t)d.B * d.T * d.A * 4, s));
  const size_t en_lds = en_lds_floats(d) * 4;
  const size_t cv_lds = conv_lds_floats(d) * 4;
  const size_t dw_lds = (size_t)d.E * 4;
  const dim3 eg(att_chunks(d), d.B);
  const dim3 rg(ceil_div(ED, 16), ceil_div(d.B, MB));
  const int vec = (G % 8 == 0) ? 1 : 0;
  const long long nbd = (long long)d.B * d.D;
  const int cgrid = (int)((nbd + 255) / 256);
  g_att_last[2] = (d.C == 10 || d.C == 3) ? d.C : 0;
  g_att_last[3] = (int)eg.x;
  for (int t = d.S - 1; t >= 0; --t) {
    const float* rp = nullptr;
    if (t + 1 < d.S) {   // r = dgates_{t+1} @ Wcat: d [ctx_t; h_t] through step t+1's cell
      if (bf)
        hipLaunchKernelGGL((rgemm<true, uint16_t>), rg, dim3(256), 0, s, t + 1, d,
                           (const uint16_t*)wcatT, gates_dg, r, vec);
      else
        hipLaunchKernelGGL((rgemm<false, float>), rg, dim3(256), 0, s, t + 1, d,
                           (const float*)wcatT, gates_dg, r, vec);
      ASR_LAUNCH_CHECK();
      rp = r;
    }
    hipLaunchKernelGGL(att_bwd_daw, eg, dim3(ATT_THREADS), dw_lds, s, t, d, enc, d_ctx_in, rp,
                       carry, dctx_tot, dawbuf);
    ASR_LAUNCH_CHECK();
#define ASR_BWD_EN(CC)                                                                        \
  hipLaunchKernelGGL(att_bwd_energy<CC>, eg, dim3(ATT_THREADS), en_lds, s, t, d, enc_a, lens,    \
                     w_dec, w_conv, conv_w, v, dec, aw_all, dawbuf, wd_all, d_enc_a, dFbuf,      \
                     dwd_chunk, dv_part, dwc_part)
    if (d.C == 10) ASR_BWD_EN(10);
    else if (d.C == 3) ASR_BWD_EN(3);
    else ASR_BWD_EN(0);
#undef ASR_BWD_EN
    ASR_LAUNCH_CHECK();
    hipLaunchKernelGGL(att_bwd_conv, eg, dim3(ATT_THREADS), cv_lds, s, t, d, conv_w, aw_all, dFbuf,
                       w_dec, dwd_chunk, carry, dcw_part, dwd_all, ddec_att);
    ASR_LAUNCH_CHECK();
    hipLaunchKernelGGL(cell_bwd, dim3(cgrid), dim3(256), 0, s, t, d, d_dec_in, rp, ddec_att,
                       gates_dg, c_all, dc, d_h0, drop_h, seed_h);
    ASR_LAUNCH_CHECK();
  }
  }
  if (ss) {
    ASR_CHECK_HIP(hipMemcpyAsync(flags, opts->ss_steps_host, (size_t)d.S * 4,
                                 hipMemcpyHostToDevice, s));
    const long long n = (long long)d.B * d.S * G;
    const int gs = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
    hipLaunchKernelGGL(ss_split, dim3(gs), dim3(256), 0, s, d, flags, gates_dg, opts->d_pre,
                       opts->dg_ss);
    ASR_LAUNCH_CHECK();
  }
  return ASR_OK;
}

// ---------------------------------------------------------------------------
// One location-attention step as a standalone op: AttentionMechanism.forward
// (attention_layer.py:123-251) -- the layer-level boundary, for callers that
// drive the decoder themselves (decode loops, visualisation).  The training
// loop runs the same kernels inside asr_attdec_forward_ex / _backward_ex.
//
// The step is launched as step t = 1 of a two-step layout in the workspace:
// slot 0 holds aw_{t-1} (the caller's aw_step), slot 1 dec_out / the outputs,
// so the kernels run unchanged (their aw_{t-1} read, masks, chunked partials).
// ---------------------------------------------------------------------------
namespace {
struct StepWs {
  size_t dec2, aw2, ctx2, dctx2, dtot2, wd2, dwd2, ebuf, carry, ddec, dF, dwdc, total;
};
StepWs step_ws(const Dims& d) {   // d.S == 2
  StepWs w;
  size_t o = 0;
  w.dec2 = o; o += al256((size_t)d.B * 2 * d.D * 4);
  w.aw2 = o; o += al256((size_t)d.B * 2 * d.T * 4);
  w.ctx2 = o; o += al256((size_t)d.B * 2 * d.E * 4);
  w.dctx2 = o; o += al256((size_t)d.B * 2 * d.E * 4);
  w.dtot2 = o; o += al256((size_t)d.B * 2 * d.E * 4);
  w.wd2 = o; o += al256((size_t)d.B * 2 * d.A * 4);
  w.dwd2 = o; o += al256((size_t)d.B * 2 * d.A * 4);
  w.ebuf = o; o += al256((size_t)d.B * d.T * 4);
  w.carry = o; o += al256((size_t)d.B * d.T * 4);
  w.ddec = o; o += al256((size_t)d.B * d.D * 4);
  w.dF = o; o += al256((size_t)d.B * d.T * d.C * 4);
  w.dwdc = o; o += al256((size_t)d.B * att_chunks(d) * d.A * 4);
  w.total = o;
  return w;
}

Dims step_dims(const asr_attdec_dims_t* dims) {
  Dims d = to_dims(*dims);
  d.S = 2;
  return d;
}

// rows [B][n] <-> slot `slot` of a [B][2][n] layout
hipError_t to_slot(float* dst2, int slot, const float* src, int B, int n, hipStream_t s) {
  return hipMemcpy2DAsync(dst2 + (size_t)slot * n, 2 * n * 4, src, n * 4, n * 4, B,
                          hipMemcpyDeviceToDevice, s);
}
hipError_t from_slot(float* dst, const float* src2, int slot, int B, int n, hipStream_t s) {
  return hipMemcpy2DAsync(dst, n * 4, src2 + (size_t)slot * n, 2 * n * 4, n * 4, B,
                          hipMemcpyDeviceToDevice, s);
}
}  // namespace

extern "C" size_t asr_att_step_workspace_bytes(const asr_attdec_dims_t* dims) {
  return step_ws(step_dims(dims)).total;
}

extern "C" int asr_att_step_forward(const asr_attdec_dims_t* dims, const float* enc,
                                    const float* enc_a, const int32_t* lens, const float* w_dec,
                                    const float* w_conv, const float* conv_w, const float* v,
                                    const float* dec_out, const float* aw_prev, float* ctx_out,
                                    float* aw_out, void* workspace, size_t ws_bytes,
                                    void* stream) {
  ASR_REQUIRE(dims, ASR_ERR_ARG, "att_step: dims is null");
  const Dims d = step_dims(dims);
  int rc = check_dims(d);
  if (rc) return rc;
  ASR_REQUIRE(enc && enc_a && lens && w_dec && w_conv && conv_w && v && dec_out && aw_prev &&
                  ctx_out && aw_out && workspace,
              ASR_ERR_ARG, "att_step_forward: null pointer");
  const StepWs W = step_ws(d);
  ASR_REQUIRE(ws_bytes >= W.total, ASR_ERR_WORKSPACE, "att_step_forward: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  char* p = (char*)workspace;
  float* dec2 = (float*)(p + W.dec2);
  float* aw2 = (float*)(p + W.aw2);
  float* ctx2 = (float*)(p + W.ctx2);
  float* ebuf = (float*)(p + W.ebuf);
  ASR_CHECK_HIP(to_slot(dec2, 1, dec_out, d.B, d.D, s));
  ASR_CHECK_HIP(to_slot(aw2, 0, aw_prev, d.B, d.T, s));
  const size_t en_lds = en_lds_floats(d) * 4;
  const size_t cx_lds = ((size_t)d.T + 64 + ATT_THREADS) * 4;
  const dim3 eg(att_chunks(d), d.B), xg(ceil_div(d.E, ECH), d.B);
  const int t = 1;
  if (d.C == 10)
    hipLaunchKernelGGL(att_energy<10>, eg, dim3(ATT_THREADS), en_lds, s, t, d, enc_a, lens, w_dec,
                       w_conv, conv_w, v, dec2, aw2, ebuf);
  else if (d.C == 3)
    hipLaunchKernelGGL(att_energy<3>, eg, dim3(ATT_THREADS), en_lds, s, t, d, enc_a, lens, w_dec,
                       w_conv, conv_w, v, dec2, aw2, ebuf);
  else
    hipLaunchKernelGGL(att_energy<0>, eg, dim3(ATT_THREADS), en_lds, s, t, d, enc_a, lens, w_dec,
                       w_conv, conv_w, v, dec2, aw2, ebuf);
  ASR_LAUNCH_CHECK();
  hipLaunchKernelGGL(att_context, xg, dim3(ATT_THREADS), cx_lds, s, t, d, enc, ebuf, aw2, ctx2,
                     (float*)nullptr);
  ASR_LAUNCH_CHECK();
  ASR_CHECK_HIP(from_slot(aw_out, aw2, 1, d.B, d.T, s));
  ASR_CHECK_HIP(from_slot(ctx_out, ctx2, 1, d.B, d.E, s));
  return ASR_OK;
}

// Backward of asr_att_step_forward.  Inputs: the forward's operands, its aw_out,
// the cotangents d_ctx [B][E] and d_aw_out [B][T] (nullable).  Outputs (all
// written, none accumulated): d_enc_a [B][T][A], d_dec [B][D], d_aw_prev [B][T],
// dctx_tot [B][E] (= d_ctx: d enc = aw_out^T dctx_tot is the caller's GEMM),
// dwd [B][A] (d of W_dec dec_out: dW_dec = dwd^T dec_out), and per
// (utterance, frame chunk) partials dv_part [B*NC][A], dwc_part [B*NC][A*C],
// dcw_part [B*NC][C*K] (written: step t = 1 = S - 1) whose column sums are dV, dW_conv, d conv kernel
// (NC = asr_attdec_chunks).
extern "C" int asr_att_step_backward(const asr_attdec_dims_t* dims, const float* enc,
                                     const float* enc_a, const int32_t* lens, const float* w_dec,
                                     const float* w_conv, const float* conv_w, const float* v,
                                     const float* dec_out, const float* aw_prev,
                                     const float* aw_out, const float* d_ctx,
                                     const float* d_aw_out, float* d_enc_a, float* d_dec,
                                     float* d_aw_prev, float* dctx_tot, float* dwd,
                                     float* dv_part, float* dwc_part, float* dcw_part,
                                     void* workspace, size_t ws_bytes, void* stream) {
  ASR_REQUIRE(dims, ASR_ERR_ARG, "att_step: dims is null");
  const Dims d = step_dims(dims);
  int rc = check_dims(d);
  if (rc) return rc;
  ASR_REQUIRE(enc && enc_a && lens && w_dec && w_conv && conv_w && v && dec_out && aw_prev &&
                  aw_out && d_ctx && d_enc_a && d_dec && d_aw_prev && dctx_tot && dwd &&
                  dv_part && dwc_part && dcw_part && workspace,
              ASR_ERR_ARG, "att_step_backward: null pointer");
  const StepWs W = step_ws(d);
  ASR_REQUIRE(ws_bytes >= W.total, ASR_ERR_WORKSPACE, "att_step_backward: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  char* p = (char*)workspace;
  float* dec2 = (float*)(p + W.dec2);
  float* aw2 = (float*)(p + W.aw2);
  float* dctx2 = (float*)(p + W.dctx2);
  float* dtot2 = (float*)(p + W.dtot2);
  float* wd2 = (float*)(p + W.wd2);
  float* dwd2 = (float*)(p + W.dwd2);
  float* dawbuf = (float*)(p + W.ebuf);
  float* carry = (float*)(p + W.carry);
  float* dFbuf = (float*)(p + W.dF);
  float* dwd_chunk = (float*)(p + W.dwdc);
  const int NC = att_chunks(d);
  ASR_CHECK_HIP(hipMemsetAsync(dec2, 0, (size_t)d.B * 2 * d.D * 4, s));
  ASR_CHECK_HIP(to_slot(dec2, 1, dec_out, d.B, d.D, s));
  ASR_CHECK_HIP(to_slot(aw2, 0, aw_prev, d.B, d.T, s));
  ASR_CHECK_HIP(to_slot(aw2, 1, aw_out, d.B, d.T, s));
  ASR_CHECK_HIP(to_slot(dctx2, 1, d_ctx, d.B, d.E, s));
  if (d_aw_out)   // d aw_t enters where the loop's next step would have put its conv term
    ASR_CHECK_HIP(hipMemcpyAsync(carry, d_aw_out, (size_t)d.B * d.T * 4, hipMemcpyDeviceToDevice,
                                 s));
  else
    ASR_CHECK_HIP(hipMemsetAsync(carry, 0, (size_t)d.B * d.T * 4, s));
  ASR_CHECK_HIP(hipMemsetAsync(d_enc_a, 0, (size_t)d.B * d.T * d.A * 4, s));
  {  // rows the step's chunks do not write stay zero
    const size_t prow = (size_t)d.B * part_rows(d);
    ASR_CHECK_HIP(hipMemsetAsync(dv_part, 0, prow * d.A * 4, s));
    ASR_CHECK_HIP(hipMemsetAsync(dwc_part, 0, prow * d.A * d.C * 4, s));
    ASR_CHECK_HIP(hipMemsetAsync(dcw_part, 0, prow * d.C * d.K * 4, s));
  }
  {  // W_dec dec (exact-f32 MFMA, as the decoder backward)
    asr_gemm_t g;
    memset(&g, 0, sizeof(g));
    g.a.ptr = dec2;
    g.a.dtype = ASR_DT_F32;
    g.a.map.stride_t = d.D;
    g.a.bytes = 4LL * d.B * 2 * d.D;
    g.b.ptr = w_dec;
    g.b.dtype = ASR_DT_F32;
    g.b.map.stride_t = d.D;
    g.b.bytes = 4LL * d.A * d.D;
    g.c = wd2;
    g.c_map.stride_t = d.A;
    g.M = d.B * 2; g.N = d.A; g.K = d.D;
    g.alpha = 1.f; g.beta = 0.f; g.batch = 1;
    rc = asr_gemm(&g, 1, ASR_DT_F32, stream);
    if (rc) return rc;
  }
  const size_t en_lds = en_lds_floats(d) * 4;
  const size_t cv_lds = conv_lds_floats(d) * 4;
  const size_t dw_lds = (size_t)d.E * 4;
  const dim3 eg(NC, d.B);
  const int t = 1;
  hipLaunchKernelGGL(att_bwd_daw, eg, dim3(ATT_THREADS), dw_lds, s, t, d, enc, dctx2,
                     (const float*)nullptr, carry, dtot2, dawbuf);
  ASR_LAUNCH_CHECK();
#define ASR_STEP_BWD_EN(CC)                                                                    \
  hipLaunchKernelGGL(att_bwd_energy<CC>, eg, dim3(ATT_THREADS), en_lds, s, t, d, enc_a, lens,    \
                     w_dec, w_conv, conv_w, v, dec2, aw2, dawbuf, wd2, d_enc_a, dFbuf, dwd_chunk, \
                     dv_part, dwc_part)
  if (d.C == 10) ASR_STEP_BWD_EN(10);
  else if (d.C == 3) ASR_STEP_BWD_EN(3);
  else ASR_STEP_BWD_EN(0);
#undef ASR_STEP_BWD_EN
  ASR_LAUNCH_CHECK();
  hipLaunchKernelGGL(att_bwd_conv, eg, dim3(ATT_THREADS), cv_lds, s, t, d, conv_w, aw2, dFbuf,
                     w_dec, dwd_chunk, carry, dcw_part, dwd2, d_dec);
  ASR_LAUNCH_CHECK();
  ASR_CHECK_HIP(hipMemcpyAsync(d_aw_prev, carry, (size_t)d.B * d.T * 4, hipMemcpyDeviceToDevice,
                               s));
  ASR_CHECK_HIP(from_slot(dctx_tot, dtot2, 1, d.B, d.E, s));
  ASR_CHECK_HIP(from_slot(dwd, dwd2, 1, d.B, d.A, s));
  return ASR_OK;
}
