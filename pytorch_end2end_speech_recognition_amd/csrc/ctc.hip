// CTC forward-backward on gfx950 -- replaces warp-ctc's gpu_ctc as bound by
// models/pytorch_v3/ctc/ctc.py:30-66 (my_warpctc).  Algorithm restated from the
// reference's own numpy CTC text (models/chainer/ctc/ctc_loss_from_chainer.py):
// log-space alpha/beta over the blank-interleaved label lattice, gradient =
// softmax - label occupancy, masked beyond the input length.
//
// Kernels (all stream-ordered, no host sync):
//   ctc_prep    1 block: exclusive scan of label_lens -> label offsets; label
//               range check -> status word.
//   ctc_emit    one wave (V <= 1024) or one work-group (ctc_emit_wide) per
//               (b,t) row: online log-sum-exp over V (one HBM read of the row) and the S emissions e_t(s) = x[lab(s)] - lse, stored
//               lattice-contiguous so the sequential kernel streams them.
//   ctc_lattice two work-groups per utterance, run concurrently: the alpha
//               lattice (forward over t, then log P and the cost) and the beta
//               lattice (backward over t); lane l owns K consecutive lattice
//               states in registers, neighbours come through DPP wave shifts.
//               A loader wave streams the emission rows into an LDS ring so
//               the lattice wave never waits on a global load.  The sequential
//               depth is T steps, not the 2T of an alpha-then-beta pass.
//   ctc_grad    one row per block: occupancy exp(alpha+beta-e-logP) of the
//               row's S states, summed per class through LDS (repeated
//               labels), grad = (softmax - occupancy) * scale written once.
//   ctc_loss    1 block: loss = scale * sum_b cost_b (fixed-order tree).
#include "common.h"
#include "prof.h"

namespace asr {
namespace {

constexpr int kMaxK = 16;  // up to 64*16 = 1024 lattice states (labels <= 511)

struct CtcWs {
  float* lse;      // [B*T]
  float* emit;     // [B*T*Spad]
  float* alpha;    // [B*T*Spad]
  float* beta;     // [B*T*Spad]
  float* logp;     // [B]
  int32_t* offs;   // [B]
  int32_t* status; // [4]
};

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

inline int pick_k(int max_label_len) {
  int S = 2 * max_label_len + 1;
  int k = 1;
  while (64 * k < S) k <<= 1;
  return k;
}

inline size_t ws_layout(int T, int B, int max_label_len, CtcWs* ws, char* base) {
  const int Spad = 64 * pick_k(max_label_len);
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = align256(off + bytes); return base + o; };
  char* p;
  p = take(sizeof(float) * (size_t)B * T);                 if (ws) ws->lse = (float*)p;
  p = take(sizeof(float) * (size_t)B * T * Spad);          if (ws) ws->emit = (float*)p;
  p = take(sizeof(float) * (size_t)B * T * Spad);          if (ws) ws->alpha = (float*)p;
  p = take(sizeof(float) * (size_t)B * T * Spad);          if (ws) ws->beta = (float*)p;
  p = take(sizeof(float) * (size_t)B);                     if (ws) ws->logp = (float*)p;
  p = take(sizeof(int32_t) * (size_t)B);                   if (ws) ws->offs = (int32_t*)p;
  p = take(sizeof(int32_t) * 4);                           if (ws) ws->status = (int32_t*)p;
  return off;
}

__global__ void ctc_prep(const int32_t* __restrict__ label_lens, const int32_t* __restrict__ labels,
                         int B, int V, int blank, int max_label_len, int32_t* __restrict__ offs,
                         int32_t* __restrict__ status) {
  // single thread scan: B is the utterance count (<= a few thousand)
  if (threadIdx.x == 0) {
    int acc = 0, bad = 0;
    for (int b = 0; b < B; ++b) {
      offs[b] = acc;
      int L = label_lens[b];
      if (L < 0 || L > max_label_len) bad |= 1;
      acc += L < 0 ? 0 : L;
    }
    status[0] = bad;
    status[1] = acc;
  }
  __syncthreads();
  int total = status[1];
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    int v = labels[i];
    if (v < 0 || v >= V || v == blank) atomicOr(&status[0], 2);
  }
}

// A work-group barrier that orders LDS only, for the lattices' per-chunk
// barriers: __syncthreads also drains vmcnt, i.e. waits for the lattice rows'
// global stores and the loader's prefetch loads issued just before it -- one
// memory round trip per chunk on the sequential chain.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The lattice runs in base 2 (emissions scaled by log2 e in ctc_emit; alpha,
// beta and log P in log2 units; the cost converted back with ln 2), so every
// transcendental is a bare v_exp_f32 / v_log_f32.
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float lg2(float x) { return __builtin_amdgcn_logf(x); }

// Online log-sum-exp accumulator (running max m, sum s of exp(x - m)).
__device__ __forceinline__ void lse_acc4(float& m, float& s, float4 v) {
  const float mx = fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w));
  if (mx > m) { s *= __expf(m - mx); m = mx; }
  s += __expf(v.x - m) + __expf(v.y - m) + __expf(v.z - m) + __expf(v.w - m);
}
__device__ __forceinline__ void lse_acc1(float& m, float& s, float x) {
  if (x > m) { s *= __expf(m - x); m = x; }
  s += __expf(x - m);
}

// Elements of a row before its first 16-B boundary.
__device__ __forceinline__ int head_elems(const float* p) {
  return (int)((4 - (((size_t)p >> 2) & 3)) & 3);
}

// One wave per (b,t) row; the row is read ONCE (online max / sum, 16-B loads
// from the row's first aligned element, four in flight per lane).
__global__ void __launch_bounds__(256) ctc_emit(const float* __restrict__ acts, long long st,
                                                long long sb, int T, int B, int V,
                                                const int32_t* __restrict__ labels,
                                                const int32_t* __restrict__ label_lens,
                                                const int32_t* __restrict__ act_lens,
                                                const int32_t* __restrict__ offs, int blank,
                                                int Spad, float* __restrict__ lse_out,
                                                float* __restrict__ emit) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= (long long)B * T) return;
  const int b = (int)(row / T), t = (int)(row % T);
  if (t >= act_lens[b]) return;
  const float* x = acts + (long long)t * st + (long long)b * sb;
  float m = neg_inf(), s = 0.f;
  const int h = min(head_elems(x), V);
  if (lane < h) lse_acc1(m, s, x[lane]);
  const int n4 = (V - h) >> 2;
  const float4* x4 = reinterpret_cast<const float4*>(x + h);
  int i = lane;
  for (; i + 192 < n4; i += 256) {
    const float4 v0 = x4[i], v1 = x4[i + 64], v2 = x4[i + 128], v3 = x4[i + 192];
    lse_acc4(m, s, v0); lse_acc4(m, s, v1); lse_acc4(m, s, v2); lse_acc4(m, s, v3);
  }
  for (; i < n4; i += 64) lse_acc4(m, s, x4[i]);
  for (int v = h + 4 * n4 + lane; v < V; v += 64) lse_acc1(m, s, x[v]);
  const float M = wave_max(m);
  const float tot = wave_sum(m == neg_inf() ? 0.f : s * __expf(m - M));
  const float lse = M + __logf(tot);
  if (lane == 0) lse_out[row] = lse;
  const int L = min(label_lens[b], (Spad - 1) / 2);
  const int S = 2 * L + 1;
  const int32_t* lab = labels + offs[b];
  float* e = emit + row * Spad;
  for (int st_ = lane; st_ < Spad; st_ += 64) {
    float v = neg_inf();
    if (st_ < S) {
      int c = (st_ & 1) ? lab[st_ >> 1] : blank;
      c = c < 0 ? 0 : (c >= V ? V - 1 : c);
      v = (x[c] - lse) * kLog2e;
    }
    e[st_] = v;
  }
}

// Wide rows (V > 1024): one 256-thread work-group per (b,t) row, so four
// times the loads in flight per row; (max, sum) pairs combined through LDS.
__global__ void __launch_bounds__(256) ctc_emit_wide(const float* __restrict__ acts, long long st,
                                                     long long sb, int T, int V,
                                                     const int32_t* __restrict__ labels,
                                                     const int32_t* __restrict__ label_lens,
                                                     const int32_t* __restrict__ act_lens,
                                                     const int32_t* __restrict__ offs, int blank,
                                                     int Spad, float* __restrict__ lse_out,
                                                     float* __restrict__ emit, int rev) {
  __shared__ float red_m[4], red_s[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // rev: rows in descending order (see ctc_row_order)
  const long long row = rev ? (long long)gridDim.x - 1 - blockIdx.x : blockIdx.x;
  const int b = (int)(row / T), t = (int)(row % T);
  if (t >= act_lens[b]) return;
  const float* x = acts + (long long)t * st + (long long)b * sb;
  float m = neg_inf(), s = 0.f;
  const int h = min(head_elems(x), V);
  if (tid < h) lse_acc1(m, s, x[tid]);
  const int n4 = (V - h) >> 2;
  const float4* x4 = reinterpret_cast<const float4*>(x + h);
  int i = tid;
  for (; i + 768 < n4; i += 1024) {
    const float4 v0 = x4[i], v1 = x4[i + 256], v2 = x4[i + 512], v3 = x4[i + 768];
    // one rescale per 16 values
    const float mx = fmaxf(fmaxf(fmaxf(fmaxf(v0.x, v0.y), fmaxf(v0.z, v0.w)),
                                 fmaxf(fmaxf(v1.x, v1.y), fmaxf(v1.z, v1.w))),
                           fmaxf(fmaxf(fmaxf(v2.x, v2.y), fmaxf(v2.z, v2.w)),
                                 fmaxf(fmaxf(v3.x, v3.y), fmaxf(v3.z, v3.w))));
    const float mn = fmaxf(m, mx);
    s *= __expf(m - mn);  // m = -inf on the first chunk: 0 * 0
    m = mn;
    s += (__expf(v0.x - m) + __expf(v0.y - m) + __expf(v0.z - m) + __expf(v0.w - m)) +
         (__expf(v1.x - m) + __expf(v1.y - m) + __expf(v1.z - m) + __expf(v1.w - m)) +
         (__expf(v2.x - m) + __expf(v2.y - m) + __expf(v2.z - m) + __expf(v2.w - m)) +
         (__expf(v3.x - m) + __expf(v3.y - m) + __expf(v3.z - m) + __expf(v3.w - m));
  }
  for (; i < n4; i += 256) lse_acc4(m, s, x4[i]);
  for (int v = h + 4 * n4 + tid; v < V; v += 256) lse_acc1(m, s, x[v]);
  float M = wave_max(m);
  float tot = wave_sum(m == neg_inf() ? 0.f : s * __expf(m - M));
  if (lane == 0) { red_m[w] = M; red_s[w] = tot; }
  __syncthreads();
  M = fmaxf(fmaxf(red_m[0], red_m[1]), fmaxf(red_m[2], red_m[3]));
  tot = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) tot += red_m[q] == neg_inf() ? 0.f : red_s[q] * __expf(red_m[q] - M);
  const float lse = M + __logf(tot);
  if (tid == 0) lse_out[row] = lse;
  const int L = min(label_lens[b], (Spad - 1) / 2);
  const int S = 2 * L + 1;
  const int32_t* lab = labels + offs[b];
  float* e = emit + row * Spad;
  for (int st_ = tid; st_ < Spad; st_ += 256) {
    float v = neg_inf();
    if (st_ < S) {
      int c = (st_ & 1) ? lab[st_ >> 1] : blank;
      c = c < 0 ? 0 : (c >= V ? V - 1 : c);
      v = (x[c] - lse) * kLog2e;
    }
    e[st_] = v;
  }
}

// The head GEMM's epilogue already formed each row's log-sum-exp in 64-column
// slabs (asr_gemm_lse_ws: (max, sum exp) pairs, part[2 (q M + row)]): one
// thread per row folds its nslab pairs (consecutive rows: coalesced 8-B
// reads) -- the activations are not read for the normaliser at all.
__global__ void __launch_bounds__(256) ctc_lse_from_parts(const float* __restrict__ part,
                                                          int nslab, long long M, int T,
                                                          const int32_t* __restrict__ act_lens,
                                                          int rev, float* __restrict__ lse_out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= M) return;
  const long long row = rev ? M - 1 - i : i;
  const int b = (int)(row / T), t = (int)(row % T);
  if (t >= act_lens[b]) return;
  // 16 slabs' loads in flight per round, then their fold (a load-use chain
  // per slab ran the pass at one memory latency per slab)
  constexpr int QB = 16;
  float m = neg_inf(), sm = 0.f;
  for (int q0 = 0; q0 < nslab; q0 += QB) {
    float2 pq[QB];
#pragma unroll
    for (int k = 0; k < QB; ++k)
      pq[k] = q0 + k < nslab
                  ? *reinterpret_cast<const float2*>(part + 2 * ((long long)(q0 + k) * M + row))
                  : make_float2(neg_inf(), 0.f);
    float mq = m;
#pragma unroll
    for (int k = 0; k < QB; ++k) mq = fmaxf(mq, pq[k].x);
    // (with m still -inf, sm holds only empty slabs' sums: 0, or a NaN to keep)
    sm = m == neg_inf() ? sm : sm * __expf(m - mq);
#pragma unroll
    for (int k = 0; k < QB; ++k)   // an empty slab's sum is 0, or NaN from a NaN logit
      sm += pq[k].x != neg_inf() ? pq[k].y * __expf(pq[k].x - mq) : pq[k].y;
    m = mq;
  }
  lse_out[row] = m + __logf(sm);
}

// The S emissions of a row from its log-sum-exp (ctc_emit's tail): one wave
// per row, four rows per work-group.
__global__ void __launch_bounds__(256) ctc_emit_gather(const float* __restrict__ acts, long long st,
                                                       long long sb, int T, int B, int V,
                                                       const int32_t* __restrict__ labels,
                                                       const int32_t* __restrict__ label_lens,
                                                       const int32_t* __restrict__ act_lens,
                                                       const int32_t* __restrict__ offs, int blank,
                                                       int Spad, const float* __restrict__ lse_in,
                                                       float* __restrict__ emit) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= (long long)B * T) return;
  const int b = (int)(row / T), t = (int)(row % T);
  if (t >= act_lens[b]) return;
  const float* x = acts + (long long)t * st + (long long)b * sb;
  const float lse = lse_in[row];
  const int L = min(label_lens[b], (Spad - 1) / 2);
  const int S = 2 * L + 1;
  const int32_t* lab = labels + offs[b];
  float* e = emit + row * Spad;
  for (int st_ = lane; st_ < Spad; st_ += 64) {
    float v = neg_inf();
    if (st_ < S) {
      int c = (st_ & 1) ? lab[st_ >> 1] : blank;
      c = c < 0 ? 0 : (c >= V ? V - 1 : c);
      v = (x[c] - lse) * kLog2e;
    }
    e[st_] = v;
  }
}

template <int K>
__device__ __forceinline__ void load_k(float (&r)[K], const float* p) {
  if constexpr (K % 4 == 0) {
#pragma unroll
    for (int k = 0; k < K; k += 4) {
      float4 v = *reinterpret_cast<const float4*>(p + k);
      r[k] = v.x; r[k + 1] = v.y; r[k + 2] = v.z; r[k + 3] = v.w;
    }
  } else if constexpr (K == 2) {
    float2 v = *reinterpret_cast<const float2*>(p);
    r[0] = v.x; r[1] = v.y;
  } else {
    r[0] = p[0];
  }
}

template <int K>
__device__ __forceinline__ void store_k(float* p, const float (&r)[K]) {
  if constexpr (K % 4 == 0) {
#pragma unroll
    for (int k = 0; k < K; k += 4)
      *reinterpret_cast<float4*>(p + k) = make_float4(r[k], r[k + 1], r[k + 2], r[k + 3]);
  } else if constexpr (K == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(r[0], r[1]);
  } else {
    p[0] = r[0];
  }
}

typedef __attribute__((ext_vector_type(4))) float f32x4;

// DPP wave shifts (GFX9 wave_shr:1 / wave_shl:1): lane i receives lane i-1 /
// i+1; the lane without a source receives 0 (callers overwrite it).
__device__ __forceinline__ float from_lower_lane(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float from_upper_lane(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x130, 0xf, 0xf, false));
}

// log2(2^a + 2^b + 2^c): the largest term is 2^0 = 1 after the shift, so two
// exponentials and one logarithm (max3 / med3 / min3 order the triple).
__device__ __forceinline__ float lse3_b2(float a, float b, float c) {
  const float m = fmaxf(fmaxf(a, b), c);
  const float md = __builtin_amdgcn_fmed3f(a, b, c);
  const float lo = fminf(fminf(a, b), c);
  const float r = m + lg2(1.f + ex2(md - m) + ex2(lo - m));
  return (m == neg_inf()) ? m : r;
}
__device__ __forceinline__ float lse2_b2(float a, float b) {
  const float m = fmaxf(a, b), lo = fminf(a, b);
  const float r = m + lg2(1.f + ex2(lo - m));
  return (m == neg_inf()) ? m : r;
}

// One work-group of two waves per (utterance, direction) (blockIdx.y: 0 =
// alpha, 1 = beta).  Wave 0 runs the lattice: lane l owns states s = l*K + k,
// neighbours come through DPP wave shifts, and it issues no global load inside
// its loop (only the alpha / beta row stores), so it never waits on memory.
// Wave 1 is the loader: it streams the emission rows of the lattice's visit
// order into a two-chunk LDS ring (chunk c+1 written while the lattice
// consumes chunk c, chunk c+2 already in flight in its registers).  A single
// wave doing both stalled one memory latency per step (the waitcnt of a
// prefetched row also covers the row stores issued after it).
template <int K>
__global__ void __launch_bounds__(128) ctc_lattice(int T, const int32_t* __restrict__ labels,
                                                   const int32_t* __restrict__ label_lens,
                                                   const int32_t* __restrict__ act_lens,
                                                   const int32_t* __restrict__ offs, int blank,
                                                   int zero_infinity, const float* __restrict__ emit,
                                                   float* __restrict__ alpha,
                                                   float* __restrict__ beta,
                                                   float* __restrict__ logp_out,
                                                   float* __restrict__ costs) {
  constexpr int Spad = 64 * K;
  constexpr int C = K <= 4 ? 16 : (K == 8 ? 8 : 4);  // rows per chunk (LDS ring 2*C*Spad*4 B)
  __shared__ __attribute__((aligned(16))) float ring[2][C][Spad];
  const int b = blockIdx.x;
  const bool is_beta = blockIdx.y == 1;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int Tb = min(act_lens[b], T);
  const int L = min(label_lens[b], (Spad - 1) / 2);
  const int S = 2 * L + 1;
  const int32_t* lab = labels + offs[b];
  const float NEG = neg_inf();

  if (Tb <= 0) {
    if (threadIdx.x == 0 && !is_beta) {
      bool feas = (L == 0);
      logp_out[b] = feas ? 0.f : NEG;
      costs[b] = feas ? 0.f : (zero_infinity ? 0.f : __builtin_huge_valf());
    }
    return;
  }
  const int N = Tb - 1;               // lattice steps after the initial row
  const int nch = (N + C - 1) / C;
  // row of the n-th step in visit order (clamped: the loader's overrun rows are harmless)
  auto row_of = [&](int n) {
    n = min(n, N - 1);
    return is_beta ? Tb - 2 - n : 1 + n;
  };
  const float* E = emit + (size_t)b * T * Spad + lane * K;

  if (wave == 1) {
    // ---------------- loader ----------------
    float r[C][K];
    if (nch > 0) {
#pragma unroll
      for (int j = 0; j < C; ++j) load_k<K>(r[j], E + (size_t)row_of(j) * Spad);
#pragma unroll
      for (int j = 0; j < C; ++j) store_k<K>(&ring[0][j][lane * K], r[j]);
      if (nch > 1) {
#pragma unroll
        for (int j = 0; j < C; ++j) load_k<K>(r[j], E + (size_t)row_of(C + j) * Spad);
      }
    }
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      if (c + 1 < nch) {
#pragma unroll
        for (int j = 0; j < C; ++j) store_k<K>(&ring[(c + 1) & 1][j][lane * K], r[j]);
        if (c + 2 < nch) {
#pragma unroll
          for (int j = 0; j < C; ++j)
            load_k<K>(r[j], E + (size_t)row_of((c + 2) * C + j) * Spad);
        }
      }
      lds_barrier();
    }
    return;
  }

  bool valid[K];
#pragma unroll
  for (int k = 0; k < K; ++k) valid[k] = lane * K + k < S;

  if (!is_beta) {
    // ---------------- alpha ----------------
    // skip[k]: transition s-2 -> s allowed (s odd label state, label differs).
    bool skip[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int s = lane * K + k;
      skip[k] = (s & 1) && s >= 3 && s < S && lab[s >> 1] != lab[(s >> 1) - 1];
    }
    float* A = alpha + (size_t)b * T * Spad + lane * K;
    float a[K];
    {
      float e0[K];
      load_k<K>(e0, E);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int s = lane * K + k;
        a[k] = (s < 2 && valid[k]) ? e0[k] : NEG;
      }
      store_k<K>(A, a);
    }
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      // the chunk's emissions into registers first: one LDS wait per chunk
      // instead of one on every step's dependency chain
      float ec[C][K];
#pragma unroll
      for (int j = 0; j < C; ++j) load_k<K>(ec[j], &ring[c & 1][j][lane * K]);
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const int n = c * C + j;
        if (n < N) {
          const float (&e)[K] = ec[j];
          float p1 = from_lower_lane(a[K - 1]);
          float p2 = (K >= 2) ? from_lower_lane(a[K >= 2 ? K - 2 : 0]) : from_lower_lane(p1);
          if (lane == 0) { p1 = NEG; p2 = NEG; }
          if (K == 1 && lane == 1) p2 = NEG;
          float nx[K];
#pragma unroll
          for (int k = 0; k < K; ++k) {
            const float a1 = (k >= 1) ? a[k >= 1 ? k - 1 : 0] : p1;
            const float a2 = (k >= 2) ? a[k >= 2 ? k - 2 : 0] : ((k == 1) ? p1 : p2);
            // K even: state parity = k parity, and blank (even) states never skip
            const float v = ((K % 2 == 0) && (k % 2 == 0) ? lse2_b2(a[k], a1)
                                                          : lse3_b2(a[k], a1, skip[k] ? a2 : NEG)) +
                            e[k];
            nx[k] = valid[k] ? v : NEG;
          }
#pragma unroll
          for (int k = 0; k < K; ++k) a[k] = nx[k];
          store_k<K>(A + (size_t)(1 + n) * Spad, a);
        }
      }
      lds_barrier();
    }

    // log P from the last two states at t = Tb-1
    float part = NEG;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int s = lane * K + k;
      if (s == S - 1 || s == S - 2) part = lse2_b2(part, a[k]);
    }
    float mx = wave_max(part);
    float sm = (mx == NEG) ? 0.f : wave_sum(ex2(part - mx));
    const float logP = (mx == NEG) ? NEG : mx + lg2(sm);  // log2 units
    if (lane == 0) {
      logp_out[b] = logP;
      costs[b] = (logP == NEG) ? (zero_infinity ? 0.f : __builtin_huge_valf()) : -logP * kLn2;
    }
    return;
  }

  // ---------------- beta ----------------
  // skipf[k]: transition s -> s+2 allowed (== skip of state s+2).
  bool skipf[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int s = lane * K + k;
    skipf[k] = (s & 1) && s + 2 < S && lab[s >> 1] != lab[(s >> 1) + 1];
  }
  float* Bt = beta + (size_t)b * T * Spad + lane * K;
  float be[K];
  {
    float et[K];
    load_k<K>(et, E + (size_t)(Tb - 1) * Spad);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int s = lane * K + k;
      be[k] = (valid[k] && (s == S - 1 || s == S - 2)) ? et[k] : NEG;
    }
    store_k<K>(Bt + (size_t)(Tb - 1) * Spad, be);
  }
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    float ec[C][K];
#pragma unroll
    for (int j = 0; j < C; ++j) load_k<K>(ec[j], &ring[c & 1][j][lane * K]);
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const int n = c * C + j;
      if (n < N) {
        const float (&e)[K] = ec[j];
        float n1 = from_upper_lane(be[0]);
        float n2 = (K >= 2) ? from_upper_lane(be[K >= 2 ? 1 : 0]) : from_upper_lane(n1);
        if (lane == 63) { n1 = NEG; n2 = NEG; }
        if (K == 1 && lane == 62) n2 = NEG;
        float nx[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float b1 = (k < K - 1) ? be[k < K - 1 ? k + 1 : 0] : n1;
          const float b2 = (k < K - 2) ? be[k < K - 2 ? k + 2 : 0] : ((k == K - 2) ? n1 : n2);
          const float v = ((K % 2 == 0) && (k % 2 == 0) ? lse2_b2(be[k], b1)
                                                        : lse3_b2(be[k], b1, skipf[k] ? b2 : NEG)) +
                          e[k];
          nx[k] = valid[k] ? v : NEG;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) be[k] = nx[k];
        store_k<K>(Bt + (size_t)(Tb - 2 - n) * Spad, be);
      }
    }
    lds_barrier();
  }
}

// The lattice split over W waves (round 6): wave w owns states [w 64 KW,
// (w+1) 64 KW), KW = K / W per lane, so a step costs each wave a W-th of the
// transcendental and VALU work of the one-wave form -- which bounds it (one
// wave issuing ~10 v_exp / v_log per lane per step at K = 4).  The recursion
// only looks DOWN the state axis for alpha (s-1, s-2) and UP for beta (s+1,
// s+2), so the waves form a one-way pipeline: after each step a wave posts its
// two edge states (with the step number as a tag, one 16-B LDS record) and its
// neighbour on the dependent side spins on that record before the same step --
// no work-group barrier per step, the downstream waves simply run a step or two
// behind.  The records live in a ring of 2 C steps; the per-chunk barrier of
// the emission ring bounds any wave's lead to one chunk, so a record is never
// overwritten before it is read.  Every alpha / beta value is computed by
// the same arithmetic as in ctc_lattice (bitwise equal); log P sums the two
// final states across lanes / waves in another grouping (last-bit changes).
template <int K, int W>
__global__ void __launch_bounds__(64 * (W + 1)) ctc_lattice_w(
    int T, const int32_t* __restrict__ labels, const int32_t* __restrict__ label_lens,
    const int32_t* __restrict__ act_lens, const int32_t* __restrict__ offs, int blank,
    int zero_infinity, const float* __restrict__ emit, float* __restrict__ alpha,
    float* __restrict__ beta, float* __restrict__ logp_out, float* __restrict__ costs) {
  static_assert(K % W == 0, "states per lane split evenly over the waves");
  constexpr int KW = K / W;
  constexpr int Spad = 64 * K;
  constexpr int C = K <= 4 ? 32 : (K == 8 ? 16 : 8);   // rows per chunk (ring 2 C Spad 4 B <= 64 KB)
  constexpr int RB = 2 * C;                            // edge-record ring (steps)
  __shared__ __attribute__((aligned(16))) float ring[2][C][Spad];
  __shared__ __attribute__((aligned(16))) f32x4 edge[W][RB];   // {v1, v2, tag, -}
  __shared__ float lpart[W];
  const int b = blockIdx.x;
  const bool is_beta = blockIdx.y == 1;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int Tb = min(act_lens[b], T);
  const int L = min(label_lens[b], (Spad - 1) / 2);
  const int S = 2 * L + 1;
  const int32_t* lab = labels + offs[b];
  const float NEG = neg_inf();

  if (Tb <= 0) {
    if (threadIdx.x == 0 && !is_beta) {
      bool feas = (L == 0);
      logp_out[b] = feas ? 0.f : NEG;
      costs[b] = feas ? 0.f : (zero_infinity ? 0.f : __builtin_huge_valf());
    }
    return;
  }
  const int N = Tb - 1;
  const int nch = (N + C - 1) / C;
  auto row_of = [&](int n) {
    n = min(n, N - 1);
    return is_beta ? Tb - 2 - n : 1 + n;
  };
  for (int e = threadIdx.x; e < W * RB; e += blockDim.x)
    (&edge[0][0])[e] = f32x4{0.f, 0.f, __int_as_float(-1), 0.f};
  __syncthreads();   // no record is posted before every tag reads -1

  if (wave == W) {
    // ---------------- loader (whole rows, as ctc_lattice) ----------------
    const float* E = emit + (size_t)b * T * Spad + lane * K;
    float r[C][K];
    if (nch > 0) {
#pragma unroll
      for (int j = 0; j < C; ++j) load_k<K>(r[j], E + (size_t)row_of(j) * Spad);
#pragma unroll
      for (int j = 0; j < C; ++j) store_k<K>(&ring[0][j][lane * K], r[j]);
      if (nch > 1) {
#pragma unroll
        for (int j = 0; j < C; ++j) load_k<K>(r[j], E + (size_t)row_of(C + j) * Spad);
      }
    }
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      if (c + 1 < nch) {
#pragma unroll
        for (int j = 0; j < C; ++j) store_k<K>(&ring[(c + 1) & 1][j][lane * K], r[j]);
        if (c + 2 < nch) {
#pragma unroll
          for (int j = 0; j < C; ++j)
            load_k<K>(r[j], E + (size_t)row_of((c + 2) * C + j) * Spad);
        }
      }
      lds_barrier();
    }
    lds_barrier();   // the lattice waves' log P reduction
    return;
  }

  const int sb = wave * 64 * KW + lane * KW;   // this lane's first state
  const float* E = emit + (size_t)b * T * Spad + sb;
  bool valid[KW];
#pragma unroll
  for (int k = 0; k < KW; ++k) valid[k] = sb + k < S;
  // the edge record of step n posted by wave v: read once ahead (issued after
  // the previous step, so its LDS latency overlaps that step's row store),
  // then re-read until its tag says step n
  auto read_edge = [&](int v, int n) {
    return *reinterpret_cast<const volatile f32x4*>(&edge[v][n & (RB - 1)]);
  };
  auto wait_edge = [&](int v, int n, f32x4 rec) {
    for (unsigned spins = 0; __float_as_int(rec[2]) != n && spins <= (1u << 20); ++spins) {
      __builtin_amdgcn_s_sleep(0);   // (bounded: never hangs)
      rec = read_edge(v, n);
    }
    return rec;
  };
  auto post_edge = [&](int n, float v1, float v2, bool poster) {
    if (poster) edge[wave][n & (RB - 1)] = f32x4{v1, v2, __int_as_float(n), 0.f};
  };

  if (!is_beta) {
    // ---------------- alpha: wave w waits on wave w-1 ----------------
    bool skip[KW];
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      const int s = sb + k;
      skip[k] = (s & 1) && s >= 3 && s < S && lab[s >> 1] != lab[(s >> 1) - 1];
    }
    float* A = alpha + (size_t)b * T * Spad + sb;
    float a[KW];
    {
      float e0[KW];
      load_k<KW>(e0, E);
#pragma unroll
      for (int k = 0; k < KW; ++k) {
        const int s = sb + k;
        a[k] = (s < 2 && valid[k]) ? e0[k] : NEG;
      }
      store_k<KW>(A, a);
    }
    // edge: the two top states (lane 63; with KW = 1 the second from lane 62)
    auto post_top = [&](int n) {
      const float lo = KW >= 2 ? a[KW >= 2 ? KW - 2 : 0] : from_lower_lane(a[0]);
      if (wave + 1 < W) post_edge(n, a[KW - 1], lo, lane == 63);
    };
    post_top(0);
    __syncthreads();
    f32x4 ahead = read_edge(wave > 0 ? wave - 1 : 0, 0);
    for (int c = 0; c < nch; ++c) {
      float ec[C][KW];
#pragma unroll
      for (int j = 0; j < C; ++j) load_k<KW>(ec[j], &ring[c & 1][j][sb]);
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const int n = c * C + j;
        if (n < N) {
          const float (&e)[KW] = ec[j];
          float p1 = from_lower_lane(a[KW - 1]);
          float p2 = (KW >= 2) ? from_lower_lane(a[KW >= 2 ? KW - 2 : 0]) : from_lower_lane(p1);
          float e1 = NEG, e2 = NEG;   // states sb_wave - 1, - 2 at step n (row n)
          if (wave > 0) {
            const f32x4 r = wait_edge(wave - 1, n, ahead);
            e1 = r[0];
            e2 = r[1];
          }
          if (lane == 0) { p1 = e1; p2 = e2; }
          if (KW == 1 && lane == 1) p2 = e1;
          float nx[KW];
#pragma unroll
          for (int k = 0; k < KW; ++k) {
            const float a1 = (k >= 1) ? a[k >= 1 ? k - 1 : 0] : p1;
            const float a2 = (k >= 2) ? a[k >= 2 ? k - 2 : 0] : ((k == 1) ? p1 : p2);
            const float v = ((KW % 2 == 0) && (k % 2 == 0) ? lse2_b2(a[k], a1)
                                                            : lse3_b2(a[k], a1, skip[k] ? a2 : NEG)) +
                            e[k];
            nx[k] = valid[k] ? v : NEG;
          }
#pragma unroll
          for (int k = 0; k < KW; ++k) a[k] = nx[k];
          post_top(n + 1);
          if (wave > 0) ahead = read_edge(wave - 1, n + 1);
          store_k<KW>(A + (size_t)(1 + n) * Spad, a);
        }
      }
      lds_barrier();
    }
    float part = NEG;
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      const int s = sb + k;
      if (s == S - 1 || s == S - 2) part = lse2_b2(part, a[k]);
    }
    float mx = wave_max(part);
    float sm = (mx == NEG) ? 0.f : wave_sum(ex2(part - mx));
    if (lane == 0) lpart[wave] = (mx == NEG) ? NEG : mx + lg2(sm);
    lds_barrier();
    if (wave == 0 && lane == 0) {
      // the two final states lie in one wave or straddle two: combine in order
      float logP = NEG;
#pragma unroll
      for (int v = 0; v < W; ++v) logP = lse2_b2(logP, lpart[v]);
      logp_out[b] = logP;
      costs[b] = (logP == NEG) ? (zero_infinity ? 0.f : __builtin_huge_valf()) : -logP * kLn2;
    }
    return;
  }

  // ---------------- beta: wave w waits on wave w+1 ----------------
  bool skipf[KW];
#pragma unroll
  for (int k = 0; k < KW; ++k) {
    const int s = sb + k;
    skipf[k] = (s & 1) && s + 2 < S && lab[s >> 1] != lab[(s >> 1) + 1];
  }
  float* Bt = beta + (size_t)b * T * Spad + sb;
  float be[KW];
  {
    float et[KW];
    load_k<KW>(et, E + (size_t)(Tb - 1) * Spad);
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      const int s = sb + k;
      be[k] = (valid[k] && (s == S - 1 || s == S - 2)) ? et[k] : NEG;
    }
    store_k<KW>(Bt + (size_t)(Tb - 1) * Spad, be);
  }
  // edge: the two bottom states (lane 0; with KW = 1 the second from lane 1)
  auto post_bottom = [&](int n) {
    const float hi = KW >= 2 ? be[KW >= 2 ? 1 : 0] : from_upper_lane(be[0]);
    if (wave > 0) post_edge(n, be[0], hi, lane == 0);
  };
  post_bottom(0);
  __syncthreads();
  f32x4 ahead = read_edge(wave + 1 < W ? wave + 1 : 0, 0);
  for (int c = 0; c < nch; ++c) {
    float ec[C][KW];
#pragma unroll
    for (int j = 0; j < C; ++j) load_k<KW>(ec[j], &ring[c & 1][j][sb]);
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const int n = c * C + j;
      if (n < N) {
        const float (&e)[KW] = ec[j];
        float n1 = from_upper_lane(be[0]);
        float n2 = (KW >= 2) ? from_upper_lane(be[KW >= 2 ? 1 : 0]) : from_upper_lane(n1);
        float e1 = NEG, e2 = NEG;   // states sb_wave + 64 KW, + 1 at step n
        if (wave + 1 < W) {
          const f32x4 r = wait_edge(wave + 1, n, ahead);
          e1 = r[0];
          e2 = r[1];
        }
        if (lane == 63) { n1 = e1; n2 = e2; }
        if (KW == 1 && lane == 62) n2 = e1;
        float nx[KW];
#pragma unroll
        for (int k = 0; k < KW; ++k) {
          const float b1 = (k < KW - 1) ? be[k < KW - 1 ? k + 1 : 0] : n1;
          const float b2 = (k < KW - 2) ? be[k < KW - 2 ? k + 2 : 0] : ((k == KW - 2) ? n1 : n2);
          const float v = ((KW % 2 == 0) && (k % 2 == 0) ? lse2_b2(be[k], b1)
                                                          : lse3_b2(be[k], b1, skipf[k] ? b2 : NEG)) +
                          e[k];
          nx[k] = valid[k] ? v : NEG;
        }
#pragma unroll
        for (int k = 0; k < KW; ++k) be[k] = nx[k];
        post_bottom(n + 1);
        if (wave + 1 < W) ahead = read_edge(wave + 1, n + 1);
        store_k<KW>(Bt + (size_t)(Tb - 2 - n) * Spad, be);
      }
    }
    lds_barrier();
  }
  lds_barrier();   // (pairs with the alpha side's log P barrier; the loader's last)
}

// grad = (softmax - occupancy) * scale, one row (b,t) per block.
//   kTable (V <= 256): occupancies summed per class in a V-entry LDS table.
//   otherwise, no V-sized table: (1) the S state occupancies go to LDS; (2) the
//   first state of each distinct class sums, in state order, the occupancies
//   of every state of its class (repeated labels and all blanks fold
//   together); (3) the row is streamed once, softmax * scale written with 16-B
//   accesses; (4) after the barrier the class representatives overwrite their
//   own columns with (softmax - occupancy) * scale.
template <bool kTable>
__global__ void __launch_bounds__(256) ctc_grad(
    const float* __restrict__ acts, long long st, long long sb, int T, int V,
    const int32_t* __restrict__ labels, const int32_t* __restrict__ label_lens,
    const int32_t* __restrict__ act_lens, const int32_t* __restrict__ offs, int blank, int Spad,
    const float* __restrict__ lse, const float* __restrict__ emit,
    const float* __restrict__ alpha, const float* __restrict__ beta,
    const float* __restrict__ logp, const float* __restrict__ grad_scale, float scale_mul,
    float* __restrict__ grads, long long gst, long long gsb, int rev) {
  extern __shared__ __attribute__((aligned(16))) float occ[];  // [V] (kTable) or [Spad]
  const long long row = rev ? (long long)gridDim.x - 1 - blockIdx.x : blockIdx.x;
  const int b = (int)(row / T), t = (int)(row % T);
  float* g = grads + (long long)t * gst + (long long)b * gsb;
  const float* x = acts + (long long)t * st + (long long)b * sb;
  const int tid = threadIdx.x, nth = blockDim.x;
  const int Tb = act_lens[b];
  const float lp = logp[b];
  if (t >= Tb || lp == neg_inf()) {
    for (int v = tid; v < V; v += nth) g[v] = 0.f;
    return;
  }
  const float scale = (grad_scale ? grad_scale[0] : 1.0f) * scale_mul;
  const float z = lse[row];
  const int L = min(label_lens[b], (Spad - 1) / 2);
  const int S = 2 * L + 1;
  const int32_t* lab = labels + offs[b];
  auto cls = [&](int s_) {
    int c = (s_ & 1) ? lab[s_ >> 1] : blank;
    return c < 0 ? 0 : (c >= V ? V - 1 : c);
  };
  const float* al = alpha + row * Spad;
  const float* bt = beta + row * Spad;
  const float* em = emit + row * Spad;

  if constexpr (kTable) {
    for (int v = tid; v < V; v += nth) occ[v] = 0.f;
    __syncthreads();
    for (int s_ = tid; s_ < S; s_ += nth) atomicAdd(&occ[cls(s_)], ex2(al[s_] + bt[s_] - em[s_] - lp));
    __syncthreads();
    for (int v = tid; v < V; v += nth) g[v] = (__expf(x[v] - z) - occ[v]) * scale;
    return;
  } else {
    int* clsT = (int*)(occ + Spad);   // the row's state classes (LDS, see ctc_grad_bf16)
    for (int s_ = tid; s_ < S; s_ += nth) {
      occ[s_] = ex2(al[s_] + bt[s_] - em[s_] - lp);
      clsT[s_] = cls(s_);
    }
    __syncthreads();
    // representatives (at most 4 states per thread: the host keeps Spad <= 4 * nth)
    int rep_c[4];
    float rep_v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      rep_c[r] = -1;
      rep_v[r] = 0.f;
      const int s_ = tid + r * nth;
      if (s_ >= S) continue;
      const int c = clsT[s_];
      bool first;
      if ((s_ & 1) == 0) {
        first = s_ == 0;
      } else {
        first = c != blank;
        for (int q = 1; q < s_ && first; q += 2) first = clsT[q] != c;
      }
      if (!first) continue;
      float acc = 0.f;
      for (int q = 0; q < S; ++q)
        if (clsT[q] == c) acc += occ[q];
      rep_c[r] = c;
      rep_v[r] = acc;
    }
    // stream the row: g = softmax * scale
    if ((((size_t)x ^ (size_t)g) & 15) == 0) {
      const int h = min(head_elems(x), V);
      if (tid < h) g[tid] = __expf(x[tid] - z) * scale;
      const int n4 = (V - h) >> 2;
      const float4* x4 = reinterpret_cast<const float4*>(x + h);
      float4* g4 = reinterpret_cast<float4*>(g + h);
      int i = tid;
      for (; i + 3 * nth < n4; i += 4 * nth) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = x4[i + u * nth];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          g4[i + u * nth] = make_float4(__expf(v[u].x - z) * scale, __expf(v[u].y - z) * scale,
                                        __expf(v[u].z - z) * scale, __expf(v[u].w - z) * scale);
      }
      for (; i < n4; i += nth) {
        const float4 v = x4[i];
        g4[i] = make_float4(__expf(v.x - z) * scale, __expf(v.y - z) * scale,
                            __expf(v.z - z) * scale, __expf(v.w - z) * scale);
      }
      for (int v = h + 4 * n4 + tid; v < V; v += nth) g[v] = __expf(x[v] - z) * scale;
    } else {
      for (int v = tid; v < V; v += nth) g[v] = __expf(x[v] - z) * scale;
    }
    // the streamed stores are acknowledged (s_waitcnt vmcnt(0): __syncthreads
    // alone only waits for LDS) before any representative overwrites a column
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (rep_c[r] >= 0) g[rep_c[r]] = (__expf(x[rep_c[r]] - z) - rep_v[r]) * scale;
  }
}

template <int A>
__device__ __forceinline__ void take8(const float (&v)[12], float (&o)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = v[A + j];
}

// The same gradient written as the bf16 dY operand of the output layer's two
// GEMMs (ctc_grad_bf16): rows (b, t) of `gld` columns (gld >= V, gld % 8 == 0,
// 16-B aligned rows), columns [V, gld) zero -- the zero-padded pitch the
// staged LinearND product reads (native_ops.LinearCTCFn), so the f32 gradient
// is never written and never restaged.  Eight columns per thread, one 16-B
// store; the class representatives then overwrite their own column.
// NCH > 0: the block also sums its `rpb` consecutive rows' f32 gradient per
// column BEFORE the bf16 rounding (the output layer's bias gradient; column
// sums of the rounded operand lose the cancellation of softmax - occupancy),
// into colpart[block][gld]: thread-owned chunks k = tid + j * nth (j < NCH)
// accumulate in registers; the occupancy terms of the class representatives
// go to an LDS table [V] -- one representative per class and row, rows
// separated by barriers, so every sum has a fixed order (deterministic).
template <bool kTable, int NCH, bool AL = false>
__global__ void __launch_bounds__(256) ctc_grad_bf16(
    const float* __restrict__ acts, long long st, long long sb, int T, int V,
    const int32_t* __restrict__ labels, const int32_t* __restrict__ label_lens,
    const int32_t* __restrict__ act_lens, const int32_t* __restrict__ offs, int blank, int Spad,
    const float* __restrict__ lse, const float* __restrict__ emit,
    const float* __restrict__ alpha, const float* __restrict__ beta,
    const float* __restrict__ logp, const float* __restrict__ grad_scale, float scale_mul,
    uint16_t* __restrict__ grads, long long gst, long long gsb, int gld, int rev,
    int acts_bytes, float* __restrict__ colpart, int rpb, long long nrows) {
  // kTable: occ [V]; else occ [Spad] (+ the representatives' table [V] when NCH > 0)
  // + the row's state classes [Spad] (the representative search reads them
  // from LDS: from the label array it was a chain of dependent global loads,
  // ~S of them per row, on the critical path of every one of a block's rows)
  extern __shared__ __attribute__((aligned(16))) float occ[];
  float* rtab = occ + Spad;
  int* clsT = (int*)(occ + Spad + (NCH > 0 ? V : 0));
  const int tid = threadIdx.x, nth = blockDim.x;
  const int n8 = gld >> 3;
  const float scale = (grad_scale ? grad_scale[0] : 1.0f) * scale_mul;
  float acc[NCH > 0 ? NCH : 1][8];
  if constexpr (NCH > 0) {
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[j][e] = 0.f;
    if constexpr (!kTable) {
      for (int v = tid; v < V; v += nth) rtab[v] = 0.f;
    }
  }
  for (int r = 0; r < rpb; ++r) {
    const long long lin = (long long)blockIdx.x * rpb + r;
    if (lin >= nrows) break;                       // block-uniform
    const long long row = rev ? nrows - 1 - lin : lin;
    const int b = (int)(row / T), t = (int)(row % T);
    uint16_t* g = grads + (long long)t * gst + (long long)b * gsb;
    const float* x = acts + (long long)t * st + (long long)b * sb;
    const int Tb = act_lens[b];
    const float lp = logp[b];
    if (t >= Tb || lp == neg_inf()) {               // row-uniform
      for (int i = tid; i < n8; i += nth) reinterpret_cast<uint4*>(g)[i] = make_uint4(0u, 0u, 0u, 0u);
      continue;
    }
    const float z = lse[row];
    const int L = min(label_lens[b], (Spad - 1) / 2);
    const int S = 2 * L + 1;
    const int32_t* lab = labels + offs[b];
    auto cls = [&](int s_) {
      int c = (s_ & 1) ? lab[s_ >> 1] : blank;
      return c < 0 ? 0 : (c >= V ? V - 1 : c);
    };
    const float* al = alpha + row * Spad;
    const float* bt = beta + row * Spad;
    const float* em = emit + row * Spad;
    // 8 columns c0 .. c0 + 7 -> one 16-B store (+ their f32 values into a[])
    auto pack = [&](int c0, auto val, float* a) {
      unsigned w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + 2 * j;
        const float lo = c < V ? val(c) : 0.f;
        const float hi = c + 1 < V ? val(c + 1) : 0.f;
        if (a) { a[2 * j] += lo; a[2 * j + 1] += hi; }
        w[j] = (c < V ? (unsigned)f2bf(lo) : 0u) | ((c + 1 < V ? (unsigned)f2bf(hi) : 0u) << 16);
      }
      reinterpret_cast<uint4*>(g)[c0 >> 3] = make_uint4(w[0], w[1], w[2], w[3]);
    };
    if constexpr (kTable) {
      for (int v = tid; v < V; v += nth) occ[v] = 0.f;
      __syncthreads();
      for (int s_ = tid; s_ < S; s_ += nth) atomicAdd(&occ[cls(s_)], ex2(al[s_] + bt[s_] - em[s_] - lp));
      __syncthreads();
      auto val = [&](int c) { return (__expf(x[c] - z) - occ[c]) * scale; };
      if constexpr (NCH > 0) {
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
          const int k = tid + j * nth;
          if (k < n8) pack(8 * k, val, acc[j]);
        }
      } else {
        for (int i = tid; i < n8; i += nth) pack(8 * i, val, (float*)nullptr);
      }
      __syncthreads();   // occ is rewritten by the next row
    } else {
      for (int s_ = tid; s_ < S; s_ += nth) {
        occ[s_] = ex2(al[s_] + bt[s_] - em[s_] - lp);
        clsT[s_] = cls(s_);
      }
      __syncthreads();
      int rep_c[4];
      float rep_v[4];
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        rep_c[q4] = -1;
        rep_v[q4] = 0.f;
        const int s_ = tid + q4 * nth;
        if (s_ >= S) continue;
        const int c = clsT[s_];
        bool first;
        if ((s_ & 1) == 0) {
          first = s_ == 0;
        } else {
          first = c != blank;
          for (int q = 1; q < s_ && first; q += 2) first = clsT[q] != c;
        }
        if (!first) continue;
        float sum = 0.f;
        for (int q = 0; q < S; ++q)
          if (clsT[q] == c) sum += occ[q];
        rep_c[q4] = c;
        rep_v[q4] = sum;
      }
      // stream the row: g = softmax * scale.  The f32 row starts at any 4-B
      // alignment, a (row-uniform) elements past a 16-B boundary; each thread
      // takes 8 columns at a time with three aligned 16-B buffer loads (past the
      // activations' end they read zeros) and keeps elements a .. a + 7
      if (acts_bytes) {
        const long long xo = (long long)t * st + (long long)b * sb;   // row start (elements)
        const int a = AL ? 0 : (int)(xo & 3);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)acts, 0, acts_bytes, 0x00020000);
        const unsigned base = (unsigned)((xo - a) * 4);
        // AL (16-B aligned rows: the fused head's padded logits pitch): two 16-B
        // loads per 8 columns and no window shift -- the shift over a runtime a
        // is folded by the compiler into a dynamically indexed array, i.e.
        // scratch memory per lane (48 B per chunk in flight)
        auto load12 = [&](int k, float (&v)[12]) {
#pragma unroll
          for (int q = 0; q < (AL ? 2 : 3); ++q) {
            const f32x4 w = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + (unsigned)(32 * k + 16 * q), 0, 0));
            v[4 * q] = w[0]; v[4 * q + 1] = w[1]; v[4 * q + 2] = w[2]; v[4 * q + 3] = w[3];
          }
        };
        auto chunk_v = [&](int k, const float (&v)[12], float* ac) {
          float o[8];
          if constexpr (AL) {
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = v[j];
          } else {
            switch (a) {   // row-uniform
              case 0: take8<0>(v, o); break;
              case 1: take8<1>(v, o); break;
              case 2: take8<2>(v, o); break;
              default: take8<3>(v, o); break;
            }
          }
          const int c0 = 8 * k;
          unsigned w4[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float lo = c0 + 2 * j < V ? __expf(o[2 * j] - z) * scale : 0.f;
            const float hi = c0 + 2 * j + 1 < V ? __expf(o[2 * j + 1] - z) * scale : 0.f;
            if (ac) { ac[2 * j] += lo; ac[2 * j + 1] += hi; }
            w4[j] = (c0 + 2 * j < V ? (unsigned)f2bf(lo) : 0u) |
                    ((c0 + 2 * j + 1 < V ? (unsigned)f2bf(hi) : 0u) << 16);
          }
          reinterpret_cast<uint4*>(g)[k] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        };
        auto chunk = [&](int k, float* ac) {
          float v[12];
          load12(k, v);
          chunk_v(k, v, ac);
        };
        if constexpr (NCH > 0) {
          // every chunk's loads in flight before the first use (the buffer loads
          // may alias the gradient stores as far as the compiler knows)
          float vv[NCH][12];
#pragma unroll
          for (int j = 0; j < NCH; ++j) {
            const int k = tid + j * nth;
            if (k < n8) load12(k, vv[j]);
          }
#pragma unroll
          for (int j = 0; j < NCH; ++j) {
            const int k = tid + j * nth;
            if (k < n8) chunk_v(k, vv[j], acc[j]);
          }
        } else {
          int i = tid;
          for (; i + nth < n8; i += 2 * nth) {
            chunk(i, nullptr);
            chunk(i + nth, nullptr);
          }
          for (; i < n8; i += nth) chunk(i, nullptr);
        }
      } else {
        auto val = [&](int c) { return __expf(x[c] - z) * scale; };
        if constexpr (NCH > 0) {
#pragma unroll
          for (int j = 0; j < NCH; ++j) {
            const int k = tid + j * nth;
            if (k < n8) pack(8 * k, val, acc[j]);
          }
        } else {
          for (int i = tid; i < n8; i += nth) pack(8 * i, val, (float*)nullptr);
        }
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
        if (rep_c[q4] >= 0) {
          g[rep_c[q4]] = f2bf((__expf(x[rep_c[q4]] - z) - rep_v[q4]) * scale);
          if constexpr (NCH > 0) atomicAdd(&rtab[rep_c[q4]], rep_v[q4] * scale);
        }
    }
  }
  if constexpr (NCH > 0) {
    __syncthreads();   // the representatives' table is complete
    float* o = colpart + (long long)blockIdx.x * gld;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int k = tid + j * nth;
      if (k >= n8) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = 8 * k + e;
        v[e] = acc[j][e];
        if constexpr (!kTable) v[e] -= c < V ? rtab[c] : 0.f;
      }
      *reinterpret_cast<f32x4*>(o + 8 * k) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(o + 8 * k + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
  }
}

// The narrow head's gradient pass (V <= 256: the char / phone CTC heads):
// ctc_grad_bf16<true>'s per-row work with each of a work-group's four waves on
// rows of its own (a wave-private class table in LDS, no block barrier per
// row).  ctc_grad_bf16<true> ran one 64-thread work-group per row or a
// block's rows one after another: ~1000 single-wave work-groups, each a chain
// of 31 rows at 32000 rows (ctc5x512: 106 us for 3.7 MB).  Here the rows of a
// work-group are dealt to its waves round-robin (one row per wave by default,
// the row's activation loads issued before its occupancy work), so the rows
// run in parallel instead of as one wave's chain; the bias partials of the four
// waves are summed in wave order into the block's colpart row (deterministic).
// dY values: bitwise ctc_grad_bf16<true>'s (same per-row arithmetic and
// atomic order within a wave).
template <int NCH>
__global__ void __launch_bounds__(256) ctc_grad_bf16_narrow(
    const float* __restrict__ acts, long long st, long long sb, int T, int V,
    const int32_t* __restrict__ labels, const int32_t* __restrict__ label_lens,
    const int32_t* __restrict__ act_lens, const int32_t* __restrict__ offs, int blank, int Spad,
    const float* __restrict__ lse, const float* __restrict__ emit,
    const float* __restrict__ alpha, const float* __restrict__ beta,
    const float* __restrict__ logp, const float* __restrict__ grad_scale, float scale_mul,
    uint16_t* __restrict__ grads, long long gst, long long gsb, int gld, int rev,
    float* __restrict__ colpart, int rpb, long long nrows) {
  constexpr int NW = 4;
  // occ [NW][V] | wave partials [NW][gld] (colpart only)
  extern __shared__ __attribute__((aligned(16))) float lds_n[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* occ = lds_n + wave * V;
  const int n8 = gld >> 3;
  const float scale = (grad_scale ? grad_scale[0] : 1.0f) * scale_mul;
  float acc[NCH][8];
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[j][e] = 0.f;
  for (int r = wave; r < rpb; r += NW) {
    const long long lin = (long long)blockIdx.x * rpb + r;
    if (lin >= nrows) break;                       // wave-uniform
    const long long row = rev ? nrows - 1 - lin : lin;
    const int b = (int)(row / T), t = (int)(row % T);
    uint16_t* g = grads + (long long)t * gst + (long long)b * gsb;
    const float* x = acts + (long long)t * st + (long long)b * sb;
    const int Tb = act_lens[b];
    const float lp = logp[b];
    if (t >= Tb || lp == neg_inf()) {               // row-uniform
      for (int i = lane; i < n8; i += 64) reinterpret_cast<uint4*>(g)[i] = make_uint4(0u, 0u, 0u, 0u);
      continue;
    }
    // the row's activations first: their loads overlap the occupancy work
    float xv[NCH][8];
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = 8 * (lane + 64 * j) + e;
        xv[j][e] = c < V ? x[c] : 0.f;
      }
    const float z = lse[row];
    const int L = min(label_lens[b], (Spad - 1) / 2);
    const int S = 2 * L + 1;
    const int32_t* lab = labels + offs[b];
    const float* al = alpha + row * Spad;
    const float* bt = beta + row * Spad;
    const float* em = emit + row * Spad;
    for (int v = lane; v < V; v += 64) occ[v] = 0.f;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int s_ = lane; s_ < S; s_ += 64) {
      int c = (s_ & 1) ? lab[s_ >> 1] : blank;
      c = c < 0 ? 0 : (c >= V ? V - 1 : c);
      atomicAdd(&occ[c], ex2(al[s_] + bt[s_] - em[s_] - lp));
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int k = lane + 64 * j;
      if (k >= n8) continue;
      unsigned w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 8 * k + 2 * q;
        const float lo = c < V ? (__expf(xv[j][2 * q] - z) - occ[c]) * scale : 0.f;
        const float hi = c + 1 < V ? (__expf(xv[j][2 * q + 1] - z) - occ[c + 1]) * scale : 0.f;
        acc[j][2 * q] += lo;
        acc[j][2 * q + 1] += hi;
        w[q] = (c < V ? (unsigned)f2bf(lo) : 0u) | ((c + 1 < V ? (unsigned)f2bf(hi) : 0u) << 16);
      }
      reinterpret_cast<uint4*>(g)[k] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();   // occ is rewritten by this wave's next row
  }
  if (!colpart) return;
  float* wp = lds_n + NW * V;   // [NW][gld]
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int k = lane + 64 * j;
    if (k >= n8) continue;
#pragma unroll
    for (int e = 0; e < 8; ++e) wp[wave * gld + 8 * k + e] = acc[j][e];
  }
  __syncthreads();
  float* o = colpart + (long long)blockIdx.x * gld;
  for (int c = threadIdx.x; c < gld; c += 64 * NW) {
    float v = wp[c];
#pragma unroll
    for (int w = 1; w < NW; ++w) v += wp[w * gld + c];
    o[c] = v;
  }
}

// The wide fused head's gradient pass (V > 256, 16-B aligned rows; the
// class-table-free form of ctc_grad_bf16) with a block's rows software-
// pipelined.  A block streams rpb consecutive rows one after another (the
// bias sums stay in registers, in row order), so its time is rpb times a row's
// chain of memory round trips; here that chain is one: while row r streams,
// the next row's header (length, log P, log-sum-exp) and state values (alpha,
// beta, emission) are already in flight, its label classes are re-read only
// when the utterance changes, and the class representatives' occupancy sums
// go to an LDS correction table BEFORE the row is streamed -- every column is
// written once as (softmax - corr) * scale, with no store-completion wait,
// barrier and read-modify-write of the representatives' columns after it.
// Values: bitwise those of ctc_grad_bf16's dY; the bias sums differ only in
// f32 summation order (sum of differences instead of difference of sums).
template <int NCH>
__global__ void __launch_bounds__(256) ctc_grad_bf16_pipe(
    const float* __restrict__ acts, long long st, long long sb, int T, int V,
    const int32_t* __restrict__ labels, const int32_t* __restrict__ label_lens,
    const int32_t* __restrict__ act_lens, const int32_t* __restrict__ offs, int blank, int Spad,
    const float* __restrict__ lse, const float* __restrict__ emit,
    const float* __restrict__ alpha, const float* __restrict__ beta,
    const float* __restrict__ logp, const float* __restrict__ grad_scale, float scale_mul,
    uint16_t* __restrict__ grads, long long gst, long long gsb, int gld, int rev,
    int acts_bytes, float* __restrict__ colpart, int rpb, long long nrows) {
  // occ [Spad] | corr [V] | clsT [Spad]
  extern __shared__ __attribute__((aligned(16))) float occ[];
  float* corr = occ + Spad;
  int* clsT = (int*)(occ + Spad + V);
  __shared__ int s_b;   // utterance whose classes clsT holds
  const int tid = threadIdx.x, nth = blockDim.x;
  const int n8 = gld >> 3;
  const float scale = (grad_scale ? grad_scale[0] : 1.0f) * scale_mul;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)acts, 0, acts_bytes, 0x00020000);
  float acc[NCH > 0 ? NCH : 1][8];
#pragma unroll
  for (int j = 0; j < (NCH > 0 ? NCH : 1); ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[j][e] = 0.f;
  for (int v = tid; v < V; v += nth) corr[v] = 0.f;
  if (tid == 0) s_b = -1;
  // a row's header and this thread's four state values (s = tid + 256 q)
  struct Row { long long row; int b, t, Tb, L; float lp, z; float sv[4]; };
  auto fetch = [&](int r, Row& h) {
    const long long lin = (long long)blockIdx.x * rpb + r;
    h.row = rev ? nrows - 1 - lin : lin;
    h.b = (int)(h.row / T);
    h.t = (int)(h.row % T);
    h.Tb = act_lens[h.b];
    h.lp = logp[h.b];
    h.z = lse[h.row];
    h.L = label_lens[h.b];
    const long long so = h.row * Spad;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int s_ = tid + q * nth;   // < 4 nth = Spad bound (host: Spad <= 1024)
      h.sv[q] = s_ < Spad ? alpha[so + s_] + beta[so + s_] - emit[so + s_] : 0.f;
    }
  };
  const int nr = (int)min((long long)rpb, nrows - (long long)blockIdx.x * rpb);
  Row cur;
  if (nr > 0) fetch(0, cur);
  for (int r = 0; r < nr; ++r) {
    const int b = cur.b, t = cur.t;
    uint16_t* g = grads + (long long)t * gst + (long long)b * gsb;
    const bool live = t < cur.Tb && cur.lp != neg_inf();   // row-uniform
    const int L = min(cur.L, (Spad - 1) / 2);
    const int S = 2 * L + 1;
    // the utterance's state classes (consecutive rows share it)
    __syncthreads();   // previous row's reads of clsT / occ / corr done
    if (live && s_b != b) {
      const int32_t* lab = labels + offs[b];
      for (int s_ = tid; s_ < S; s_ += nth) {
        int c = (s_ & 1) ? lab[s_ >> 1] : blank;
        clsT[s_] = c < 0 ? 0 : (c >= V ? V - 1 : c);
      }
    }
    if (live) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int s_ = tid + q * nth;
        if (s_ < S) occ[s_] = ex2(cur.sv[q] - cur.lp);
      }
    }
    __syncthreads();   // occ, clsT
    if (tid == 0 && live) s_b = b;
    int rep_c[4] = {-1, -1, -1, -1};
    if (live) {
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const int s_ = tid + q4 * nth;
        if (s_ >= S) continue;
        const int c = clsT[s_];
        bool first;
        if ((s_ & 1) == 0) {
          first = s_ == 0;
        } else {
          first = c != blank;
          for (int q = 1; q < s_ && first; q += 2) first = clsT[q] != c;
        }
        if (!first) continue;
        float sum = 0.f;
        for (int q = 0; q < S; ++q)
          if (clsT[q] == c) sum += occ[q];
        rep_c[q4] = c;
        corr[c] = sum;
      }
    }
    __syncthreads();   // corr complete
    // this row's stream loads, then the next row's header / states
    const float z = cur.z;
    const long long xo = (long long)t * st + (long long)b * sb;
    const unsigned base = (unsigned)(xo * 4);
    float vv[NCH > 0 ? NCH : 1][8];
    if (live) {
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const int k = tid + j * nth;
        if (k < n8) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const f32x4 w = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + (unsigned)(32 * k + 16 * q), 0, 0));
            vv[j][4 * q] = w[0]; vv[j][4 * q + 1] = w[1]; vv[j][4 * q + 2] = w[2]; vv[j][4 * q + 3] = w[3];
          }
        }
      }
    }
    Row nxt;
    if (r + 1 < nr) fetch(r + 1, nxt);
    if (live) {
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const int k = tid + j * nth;
        if (k >= n8) continue;
        const int c0 = 8 * k;
        float cr[8];
        if (c0 + 8 <= V) {
          const f32x4 c_lo = *reinterpret_cast<const f32x4*>(corr + c0);
          const f32x4 c_hi = *reinterpret_cast<const f32x4*>(corr + c0 + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) { cr[e] = c_lo[e]; cr[4 + e] = c_hi[e]; }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) cr[e] = c0 + e < V ? corr[c0 + e] : 0.f;
        }
        unsigned w4[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int c = c0 + 2 * jj;
          const float lo = c < V ? (__expf(vv[j][2 * jj] - z) - cr[2 * jj]) * scale : 0.f;
          const float hi = c + 1 < V ? (__expf(vv[j][2 * jj + 1] - z) - cr[2 * jj + 1]) * scale : 0.f;
          if (NCH > 0) { acc[j][2 * jj] += lo; acc[j][2 * jj + 1] += hi; }
          w4[jj] = (c < V ? (unsigned)f2bf(lo) : 0u) | ((c + 1 < V ? (unsigned)f2bf(hi) : 0u) << 16);
        }
        reinterpret_cast<uint4*>(g)[k] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
    } else {
      for (int i = tid; i < n8; i += nth) reinterpret_cast<uint4*>(g)[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    __syncthreads();   // every read of corr for this row done
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4)
      if (rep_c[q4] >= 0) corr[rep_c[q4]] = 0.f;
    if (r + 1 < nr) cur = nxt;
  }
  if (NCH > 0 && colpart) {
    float* o = colpart + (long long)blockIdx.x * gld;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int k = tid + j * nth;
      if (k >= n8) continue;
      *reinterpret_cast<f32x4*>(o + 8 * k) = f32x4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
      *reinterpret_cast<f32x4*>(o + 8 * k + 4) = f32x4{acc[j][4], acc[j][5], acc[j][6], acc[j][7]};
    }
  }
}

// The wide fused head's gradient pass, streamed (V > 256, 16-B aligned
// activation rows of a padded pitch; ASR_CTC_GRAD_STREAM=0 selects
// ctc_grad_bf16_pipe).  512 threads, two work-groups per CU (grid = 2 x CUs,
// each a contiguous run of rows), and the rows software-pipelined two deep:
// while row r is turned into dY, row r+1's activations (3 x 32 B per thread at
// V = 10001) and row r+2's header / state sums are in flight, so the HBM
// stream never waits on a row's occupancy work.  The per-row class work is
// O(multiplicity), not O(S): per utterance (when the block's rows cross one)
// each label state learns whether it is its class's first occurrence and the
// next state of its class (nxt); per row a class representative sums its chain
// of occupancies, the blank class's sum is a block reduction, and the
// representative is pushed onto its 8-column chunk's list (head[k] ->
// link[]), so a chunk reads one LDS word and, in the rare chunk holding a
// label class, walks a one- or two-entry list -- no V-sized correction table
// (LDS per work-group ~20 KB, not 40 KB).  dY values: bitwise those of
// ctc_grad_bf16 (each column subtracts its single class sum); bias sums in f32
// over the block's rows in row order.
template <int NCH>
__global__ void __launch_bounds__(512, 4) ctc_grad_bf16_stream(
    const float* __restrict__ acts, long long st, long long sb, int T, int V,
    const int32_t* __restrict__ labels, const int32_t* __restrict__ label_lens,
    const int32_t* __restrict__ act_lens, const int32_t* __restrict__ offs, int blank, int Spad,
    const float* __restrict__ lse, const float* __restrict__ emit,
    const float* __restrict__ alpha, const float* __restrict__ beta,
    const float* __restrict__ logp, const float* __restrict__ grad_scale, float scale_mul,
    uint16_t* __restrict__ grads, long long gst, long long gsb, int gld, int rev,
    int acts_bytes, float* __restrict__ colpart, int rpb, long long nrows) {
  constexpr int NT = 512, NW = NT / 64;
  // occ [Spad] f32 | repv [Spad] f32 | clsT [Spad] | nxt [Spad] | link [Spad] | head [n8] | red [NW]
  extern __shared__ __attribute__((aligned(16))) float occ[];
  float* repv = occ + Spad;
  int* clsT = (int*)(repv + Spad);
  int* nxt = clsT + Spad;
  int* link = nxt + Spad;
  int* head = link + Spad;
  const int n8 = gld >> 3;
  float* red = (float*)(head + n8);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float scale = (grad_scale ? grad_scale[0] : 1.0f) * scale_mul;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)acts, 0, acts_bytes, 0x00020000);
  for (int k = tid; k < n8; k += NT) head[k] = 0;
  float acc[NCH][8];
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[j][e] = 0.f;

  struct Row { int b, t, Tb, L; float lp, z; float sv[2]; bool live; };
  const long long r0 = (long long)blockIdx.x * rpb;
  const int nr = (int)max(0LL, min((long long)rpb, nrows - r0));
  auto fetch = [&](int r, Row& h) {
    const long long lin = r0 + r;
    const long long row = rev ? nrows - 1 - lin : lin;
    h.b = (int)(row / T);
    h.t = (int)(row % T);
    h.Tb = act_lens[h.b];
    h.lp = logp[h.b];
    h.z = lse[row];
    h.L = min(label_lens[h.b], (Spad - 1) / 2);
    h.live = h.t < h.Tb && h.lp != neg_inf();
    const long long so = row * Spad;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int s_ = tid + q * NT;
      h.sv[q] = s_ < 2 * h.L + 1 ? alpha[so + s_] + beta[so + s_] - emit[so + s_] : 0.f;
    }
  };
  auto load_row = [&](const Row& h, float (&v)[NCH][8]) {
    if (!h.live) return;
    const unsigned base = (unsigned)(((long long)h.t * st + (long long)h.b * sb) * 4);
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int k = tid + j * NT;
      if (8 * k < V) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 w = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + (unsigned)(32 * k + 16 * q), 0, 0));
          v[j][4 * q] = w[0]; v[j][4 * q + 1] = w[1]; v[j][4 * q + 2] = w[2]; v[j][4 * q + 3] = w[3];
        }
      }
    }
  };
  // per-utterance state classes: rep[q] (first state of a label class), isb[q] (blank class)
  int ub = -1;
  bool rep[2] = {false, false}, isb[2] = {false, false};
  auto setup_utt = [&](const Row& h) {
    const int S = 2 * h.L + 1;
    const int32_t* lab = labels + offs[h.b];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int s_ = tid + q * NT;
      if (s_ < S) {
        int c = (s_ & 1) ? lab[s_ >> 1] : blank;
        clsT[s_] = c < 0 ? 0 : (c >= V ? V - 1 : c);
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int s_ = tid + q * NT;
      rep[q] = false;
      isb[q] = false;
      if (s_ >= S) continue;
      const int c = clsT[s_];
      isb[q] = c == blank;
      if (c == blank) continue;   // only odd states reach here
      bool first = true;
      for (int p = s_ - 2; p >= 1 && first; p -= 2) first = clsT[p] != c;
      int nx = -1;
      for (int p = s_ + 2; p < S && nx < 0; p += 2)
        if (clsT[p] == c) nx = p;
      rep[q] = first;
      nxt[s_] = nx;
    }
    // the blank class's representative: state 0
    if (tid == 0) rep[0] = true;
    ub = h.b;
  };
  auto step = [&](int r, const Row& cur, Row& n1, Row& n2, float (&vc)[NCH][8], float (&vn)[NCH][8]) {
    // in flight: row r+1's activations, row r+2's header
    if (r + 1 < nr) load_row(n1, vn);
    if (r + 2 < nr) fetch(r + 2, n2);
    const int S = 2 * cur.L + 1;
    if (cur.live && cur.b != ub) setup_utt(cur);   // block-uniform
    float bl = 0.f;
    if (cur.live) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int s_ = tid + q * NT;
        if (s_ < S) {
          const float o = ex2(cur.sv[q] - cur.lp);
          occ[s_] = o;
          if (isb[q]) bl += o;
        }
      }
      bl = wave_sum(bl);
      if (lane == 0) red[wave] = bl;
    }
    __syncthreads();   // occ, red
    if (cur.live) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int s_ = tid + q * NT;
        if (!rep[q] || s_ >= S) continue;
        float sum;
        int c;
        if (s_ == 0) {
          sum = 0.f;
#pragma unroll
          for (int w = 0; w < NW; ++w) sum += red[w];
          c = blank;
        } else {
          sum = occ[s_];
          for (int p = nxt[s_]; p >= 0; p = nxt[p]) sum += occ[p];
          c = clsT[s_];
        }
        repv[s_] = sum;
        link[s_] = atomicExch(&head[c >> 3], s_ + 1);
      }
    }
    __syncthreads();   // head / link / repv
    uint16_t* g = grads + (long long)cur.t * gst + (long long)cur.b * gsb;
    const float z = cur.z;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int k = tid + j * NT;
      if (k >= n8) continue;
      const int c0 = 8 * k;
      float e[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj)
        e[jj] = (cur.live && c0 + jj < V) ? __expf(vc[j][jj] - z) : 0.f;
      if (cur.live) {
        for (int h = head[k]; h != 0; h = link[h - 1]) {
          const int sr = h - 1;
          const int off = clsT[sr] - c0;   // clsT[0] = blank
          const float rv = repv[sr];
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) e[jj] -= off == jj ? rv : 0.f;
        }
      }
      unsigned w4[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float lo = e[2 * jj] * scale, hi = e[2 * jj + 1] * scale;
        acc[j][2 * jj] += lo;
        acc[j][2 * jj + 1] += hi;
        w4[jj] = (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
      }
      reinterpret_cast<uint4*>(g)[k] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
    __syncthreads();   // every read of head / link / repv / clsT for this row done
    if (cur.live) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int s_ = tid + q * NT;
        if (rep[q] && s_ < S) head[clsT[s_] >> 3] = 0;
      }
    }
  };
  Row ra, rb, rc;
  float va[NCH][8], vb[NCH][8];
  if (nr > 0) {
    fetch(0, ra);
    if (nr > 1) fetch(1, rb);
    load_row(ra, va);
  }
  __syncthreads();   // head cleared
  // three headers (rows r, r+1, r+2) and two activation buffers (rows r,
  // r+1) rotate with period 6: a six-way unroll keeps every one in registers
  // without a copy (copying a register with a load in flight waits for it)
  for (int r = 0; r < nr; r += 6) {
#define ASR_GS(I, C, N1, N2, VC, VN) \
  if (r + I >= nr) break;            \
  step(r + I, C, N1, N2, VC, VN);
    ASR_GS(0, ra, rb, rc, va, vb)
    ASR_GS(1, rb, rc, ra, vb, va)
    ASR_GS(2, rc, ra, rb, va, vb)
    ASR_GS(3, ra, rb, rc, vb, va)
    ASR_GS(4, rb, rc, ra, va, vb)
    ASR_GS(5, rc, ra, rb, vb, va)
#undef ASR_GS
  }
  if (colpart) {
    float* o = colpart + (long long)blockIdx.x * gld;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int k = tid + j * NT;
      if (k >= n8) continue;
      *reinterpret_cast<f32x4*>(o + 8 * k) = f32x4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
      *reinterpret_cast<f32x4*>(o + 8 * k + 4) = f32x4{acc[j][4], acc[j][5], acc[j][6], acc[j][7]};
    }
  }
}

__global__ void ctc_loss_reduce(const float* __restrict__ costs, int B, float scale,
                                float* __restrict__ out) {
  __shared__ float red[256];
  float s = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) s += costs[b];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0] * scale;
}

int check_common(const float* acts, int T, int B, int V, const int32_t* labels,
                 const int32_t* label_lens, const int32_t* act_lens, int max_label_len, int blank,
                 const void* ws, size_t ws_bytes) {
  ASR_REQUIRE(acts && label_lens && act_lens && ws, ASR_ERR_ARG, "ctc: null pointer argument");
  ASR_REQUIRE(T > 0 && B > 0 && V > 1, ASR_ERR_ARG, "ctc: bad shape T=%d B=%d V=%d", T, B, V);
  ASR_REQUIRE(blank >= 0 && blank < V, ASR_ERR_ARG, "ctc: blank %d out of range", blank);
  ASR_REQUIRE(max_label_len >= 0 && 2 * max_label_len + 1 <= 64 * kMaxK, ASR_ERR_UNSUPPORTED,
              "ctc: max_label_len %d exceeds %d", max_label_len, (64 * kMaxK - 1) / 2);
  ASR_REQUIRE(labels || max_label_len == 0, ASR_ERR_ARG, "ctc: labels is null");
  size_t need = asr_ctc_workspace_bytes(T, B, V, max_label_len);
  ASR_REQUIRE(ws_bytes >= need, ASR_ERR_WORKSPACE, "ctc: workspace %zu < %zu", ws_bytes, need);
  return ASR_OK;
}

}  // namespace
}  // namespace asr

using namespace asr;

extern "C" size_t asr_ctc_workspace_bytes(int T, int B, int V, int max_label_len) {
  (void)V;
  if (T <= 0 || B <= 0 || max_label_len < 0) return 0;
  return ws_layout(T, B, max_label_len, nullptr, nullptr);
}

// Row order of the two passes that stream the activations (ASR_CTC_ORDER: bit
// 0 the emission pass descending, bit 1 the gradient pass descending).  At
// V = 10001 the [B][T][V] activations (320 MB) exceed the 256 MB Infinity
// Cache by little: the gradient pass reading first the rows the emission pass
// read last finds part of them still cached.
static int ctc_row_order() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ASR_CTC_ORDER");
    v = e ? (atoi(e) & 3) : 2;
  }
  return v;
}

// Which kernels the last CTC forward / gradient ran (host-side record;
// asr_ctc_last_path): {normaliser: 0 the emission pass over the logits, 1 the
// head GEMM epilogue's (max, sum exp) partials; gradient: 0 f32 ctc_grad,
// 1 ctc_grad_bf16, 2 ctc_grad_bf16_narrow, 3 ctc_grad_bf16_pipe,
// 4 ctc_grad_bf16_stream}; [2] (round 6, asr_ctc_last_lattice_waves): the
// waves of the last forward's lattice (1: ctc_lattice, else ctc_lattice_w).
static int g_ctc_last_path[3];

extern "C" int asr_ctc_last_path(int* out2) {
  ASR_REQUIRE(out2, ASR_ERR_ARG, "ctc_last_path: null pointer");
  out2[0] = g_ctc_last_path[0];
  out2[1] = g_ctc_last_path[1];
  return ASR_OK;
}

extern "C" int asr_ctc_last_lattice_waves(void) { return g_ctc_last_path[2]; }

static int ctc_forward_impl(const float* acts, long long stride_t, long long stride_b, int T,
                            int B, int V, const float* lse_part, int nslab,
                            const int32_t* labels_flat, const int32_t* label_lens,
                            const int32_t* act_lens, int max_label_len, int blank,
                            int zero_infinity, float* costs, float* loss_out, float loss_scale,
                            void* workspace, size_t ws_bytes, void* stream) {
  int rc = check_common(acts, T, B, V, labels_flat, label_lens, act_lens, max_label_len, blank,
                        workspace, ws_bytes);
  if (rc) return rc;
  ASR_REQUIRE(costs, ASR_ERR_ARG, "ctc: costs is null");
  ASR_REQUIRE(!lse_part || nslab == (V + 63) / 64, ASR_ERR_ARG,
              "ctc: %d log-sum-exp slabs for V=%d (need %d)", nslab, V, (V + 63) / 64);
  hipStream_t s = (hipStream_t)stream;
  CtcWs ws;
  ws_layout(T, B, max_label_len, &ws, (char*)workspace);
  const int K = pick_k(max_label_len);
  const int Spad = 64 * K;
  hipLaunchKernelGGL(ctc_prep, dim3(1), dim3(256), 0, s, label_lens, labels_flat, B, V, blank,
                     max_label_len, ws.offs, ws.status);
  ASR_LAUNCH_CHECK();
  const long long rows = (long long)B * T;
  // algorithmic HBM bytes of the forward: the activations read once,
  // or with the GEMM's partials, those (8 B per slab per row)
  const int pslot = prof_begin_launch(
      ASR_PROF_CTC_FWD, s, (lse_part ? 8.0 * nslab : 4.0 * (double)V) * (double)rows, V);
  g_ctc_last_path[0] = lse_part ? 1 : 0;
  if (lse_part) {
    hipLaunchKernelGGL(ctc_lse_from_parts, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s,
                       lse_part, nslab, rows, T, act_lens, 0, ws.lse);
    ASR_LAUNCH_CHECK();
    hipLaunchKernelGGL(ctc_emit_gather, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, acts,
                       stride_t, stride_b, T, B, V, labels_flat, label_lens, act_lens, ws.offs,
                       blank, Spad, ws.lse, ws.emit);
  } else if (V > 1024)
    hipLaunchKernelGGL(ctc_emit_wide, dim3((unsigned)rows), dim3(256), 0, s, acts, stride_t,
                       stride_b, T, V, labels_flat, label_lens, act_lens, ws.offs, blank, Spad,
                       ws.lse, ws.emit, ctc_row_order() & 1);
  else
    hipLaunchKernelGGL(ctc_emit, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, acts, stride_t,
                       stride_b, T, B, V, labels_flat, label_lens, act_lens, ws.offs, blank, Spad,
                       ws.lse, ws.emit);
  ASR_LAUNCH_CHECK();
#define ASR_CTC_LAT(KK)                                                                        \
  hipLaunchKernelGGL(ctc_lattice<KK>, dim3(B, 2), dim3(128), 0, s, T, labels_flat, label_lens,  \
                     act_lens, ws.offs, blank, zero_infinity, ws.emit, ws.alpha, ws.beta,      \
                     ws.logp, costs)
#define ASR_CTC_LATW(KK, WW)                                                                   \
  hipLaunchKernelGGL((ctc_lattice_w<KK, WW>), dim3(B, 2), dim3(64 * (WW + 1)), 0, s, T,         \
                     labels_flat, label_lens, act_lens, ws.offs, blank, zero_infinity, ws.emit,  \
                     ws.alpha, ws.beta, ws.logp, costs)
  // the one-wave kernel by default; ASR_CTC_LATTICE_W=2 / 4: the lattice over
  // at most two / four waves (ctc_lattice_w) -- measured SLOWER at ctc5x512
  // (B 32 x T 1000, K 4: forward 195 us one wave, 265 two, 262 four;
  // tools/ctc_lattice_bench.py), kept as a tested alternative
  const char* lw = getenv("ASR_CTC_LATTICE_W");
  const int wmax = lw ? atoi(lw) : 1;
  const int W = K < 2 || wmax <= 1 ? 1 : (wmax == 2 || K == 2 ? 2 : 4);
  g_ctc_last_path[2] = W;
  switch (K) {
    case 1: ASR_CTC_LAT(1); break;
    case 2: if (W > 1) ASR_CTC_LATW(2, 2); else ASR_CTC_LAT(2); break;
    case 4: if (W == 4) ASR_CTC_LATW(4, 4); else if (W == 2) ASR_CTC_LATW(4, 2); else ASR_CTC_LAT(4); break;
    case 8: if (W == 4) ASR_CTC_LATW(8, 4); else if (W == 2) ASR_CTC_LATW(8, 2); else ASR_CTC_LAT(8); break;
    case 16: if (W == 4) ASR_CTC_LATW(16, 4); else if (W == 2) ASR_CTC_LATW(16, 2); else ASR_CTC_LAT(16); break;
    default: set_error("ctc: unsupported K=%d", K); return ASR_ERR_UNSUPPORTED;
  }
#undef ASR_CTC_LATW
#undef ASR_CTC_LAT
  ASR_LAUNCH_CHECK();
  prof_end_launch(ASR_PROF_CTC_FWD, pslot, s);
  if (loss_out) {
    hipLaunchKernelGGL(ctc_loss_reduce, dim3(1), dim3(256), 0, s, costs, B, loss_scale, loss_out);
    ASR_LAUNCH_CHECK();
  }
  return ASR_OK;
}

extern "C" int asr_ctc_forward(const float* acts, long long stride_t, long long stride_b, int T,
                               int B, int V, const int32_t* labels_flat,
                               const int32_t* label_lens, const int32_t* act_lens,
                               int max_label_len, int blank, int zero_infinity, float* costs,
                               float* loss_out, float loss_scale, void* workspace,
                               size_t ws_bytes, void* stream) {
  return ctc_forward_impl(acts, stride_t, stride_b, T, B, V, nullptr, 0, labels_flat, label_lens,
                          act_lens, max_label_len, blank, zero_infinity, costs, loss_out,
                          loss_scale, workspace, ws_bytes, stream);
}

extern "C" int asr_ctc_forward_lse(const float* acts, long long stride_t, long long stride_b,
                                   int T, int B, int V, const float* lse_part, int nslab,
                                   const int32_t* labels_flat, const int32_t* label_lens,
                                   const int32_t* act_lens, int max_label_len, int blank,
                                   int zero_infinity, float* costs, float* loss_out,
                                   float loss_scale, void* workspace, size_t ws_bytes,
                                   void* stream) {
  ASR_REQUIRE(lse_part, ASR_ERR_ARG, "ctc: lse_part is null");
  return ctc_forward_impl(acts, stride_t, stride_b, T, B, V, lse_part, nslab, labels_flat,
                          label_lens, act_lens, max_label_len, blank, zero_infinity, costs,
                          loss_out, loss_scale, workspace, ws_bytes, stream);
}

extern "C" int asr_ctc_backward(const float* acts, long long stride_t, long long stride_b, int T,
                                int B, int V, const int32_t* labels_flat,
                                const int32_t* label_lens, const int32_t* act_lens,
                                int max_label_len, int blank, const float* grad_scale,
                                float scale, float* grads, long long gstride_t,
                                long long gstride_b,
                                const void* workspace, size_t ws_bytes, void* stream) {
  int rc = check_common(acts, T, B, V, labels_flat, label_lens, act_lens, max_label_len, blank,
                        workspace, ws_bytes);
  if (rc) return rc;
  ASR_REQUIRE(grads, ASR_ERR_ARG, "ctc: grads is null");
  hipStream_t s = (hipStream_t)stream;
  CtcWs ws;
  ws_layout(T, B, max_label_len, &ws, (char*)workspace);
  const int Spad = 64 * pick_k(max_label_len);
  const bool table = V <= 256;
  const int threads = table ? 64 : 256;  // compact mode: Spad <= 1024 = 4 * threads
  // algorithmic HBM bytes: activations read + gradient written
  const int pslot = prof_begin_launch(ASR_PROF_CTC_GRAD, s, 8.0 * (double)V * B * T, V);
  g_ctc_last_path[1] = 0;
  if (table)
    hipLaunchKernelGGL(ctc_grad<true>, dim3((unsigned)((long long)B * T)), dim3(threads),
                       V * sizeof(float), s, acts, stride_t, stride_b, T, V, labels_flat,
                       label_lens, act_lens, ws.offs, blank, Spad, ws.lse, ws.emit, ws.alpha,
                       ws.beta, ws.logp, grad_scale, scale, grads, gstride_t, gstride_b,
                       (ctc_row_order() >> 1) & 1);
  else
    hipLaunchKernelGGL(ctc_grad<false>, dim3((unsigned)((long long)B * T)), dim3(threads),
                       2 * Spad * sizeof(float), s, acts, stride_t, stride_b, T, V, labels_flat,
                       label_lens, act_lens, ws.offs, blank, Spad, ws.lse, ws.emit, ws.alpha,
                       ws.beta, ws.logp, grad_scale, scale, grads, gstride_t, gstride_b,
                       (ctc_row_order() >> 1) & 1);
  ASR_LAUNCH_CHECK();
  prof_end_launch(ASR_PROF_CTC_GRAD, pslot, s);
  return ASR_OK;
}

// Output-layer bias gradient of the fused head (asr_ctc_backward_bf16_db):
// rows per block and blocks of the column-partial pass.
static void ctc_bias_grid(int T, int B, int V, int* rpb, int* nblk) {
  const long long rows = (long long)B * T;
  // partial rows: nblk x gld f32.  A block's rows run one after another, so
  // fewer rows per block hide more latency at the price of partial traffic:
  // at V = 10001, 534 / 1067 / 2134 blocks measured 265 + 13 / 202 + 20 /
  // 185 + 33 us (gradient + column sums).  ASR_CTC_BIAS_BLOCKS: the target (A/B)
  const char* bb_env = getenv("ASR_CTC_BIAS_BLOCKS");   // per call: the tests switch it
  const long long env_target = bb_env ? atoll(bb_env) : 0;
  // narrow heads (V <= 256, ctc_grad_bf16_narrow): 4 rows per work-group, one
  // per wave (the partials are gld <= 256 columns; a row is a chain of ~3
  // dependent memory round trips, so rows in parallel, not in sequence: 16
  // rows per work-group measured 54 us at 32000 rows)
  const long long target = env_target > 0 ? env_target : V <= 256 ? (rows + 3) / 4 : 1024;
  long long r = rows / target;
  if (r < 1) r = 1;
  if (r > 64) r = 64;
  *rpb = (int)r;
  *nblk = (int)((rows + r - 1) / r);
}

extern "C" size_t asr_ctc_bias_workspace_bytes(int T, int B, int V, int gld) {
  if (T <= 0 || B <= 0 || V <= 1 || gld < V) return 0;
  int rpb, nblk;
  ctc_bias_grid(T, B, V, &rpb, &nblk);
  const size_t part = ((size_t)nblk * gld * sizeof(float) + 255) & ~(size_t)255;
  return part + asr_colsum_workspace_bytes(nblk, V);
}

static int ctc_backward_bf16_impl(const float* acts, long long stride_t, long long stride_b, int T,
                                  int B, int V, const int32_t* labels_flat,
                                  const int32_t* label_lens, const int32_t* act_lens,
                                  int max_label_len, int blank, const float* grad_scale,
                                  float scale, uint16_t* grads, long long gstride_t,
                                  long long gstride_b, int gld, const void* workspace,
                                  size_t ws_bytes, float* dbias, void* bws, size_t bws_bytes,
                                  void* stream) {
  int rc = check_common(acts, T, B, V, labels_flat, label_lens, act_lens, max_label_len, blank,
                        workspace, ws_bytes);
  if (rc) return rc;
  ASR_REQUIRE(grads, ASR_ERR_ARG, "ctc_bf16: grads is null");
  ASR_REQUIRE(gld >= V && gld % 8 == 0 && gstride_t % 8 == 0 && gstride_b % 8 == 0 &&
                  ((uintptr_t)grads & 15) == 0,
              ASR_ERR_ARG, "ctc_bf16: gradient rows must be 16-B aligned with gld %d >= V %d", gld,
              V);
  hipStream_t s = (hipStream_t)stream;
  CtcWs ws;
  ws_layout(T, B, max_label_len, &ws, (char*)workspace);
  const int Spad = 64 * pick_k(max_label_len);
  const bool table = V <= 256;
  const int threads = table ? 64 : 256;
  // aligned 16-B buffer loads of the activation rows (compact form) when the
  // activations are one dense [B][T][V] or [T][B][V] block below 2 GiB
  // (or [B][T] rows of a padded pitch >= V: the fused heads' logits); the
  // buffer's extent ends with the last row.  al: every row 16-B aligned
  const long long nb =
      stride_t >= 0 && stride_b >= 0
          ? 4LL * ((long long)(B - 1) * stride_b + (long long)(T - 1) * stride_t + V)
          : 0;
  const bool dense = (stride_t == V && stride_b == (long long)T * V) ||
                     (stride_b == V && stride_t == (long long)B * V) ||
                     (stride_t >= V && stride_b == (long long)T * stride_t);
  const int abytes = (!table && dense && nb > 0 && nb < 0x7fffff00LL && ((uintptr_t)acts & 15) == 0)
                         ? (int)nb : 0;
  const bool al = abytes && stride_t % 4 == 0 && stride_b % 4 == 0;
  const long long rows = (long long)B * T;
  const int rev = (ctc_row_order() >> 1) & 1;
  int rpb = 1, nblk = (int)rows, nch = 0;
  float* colpart = nullptr;
  if (dbias) {
    ASR_REQUIRE(bws && bws_bytes >= asr_ctc_bias_workspace_bytes(T, B, V, gld), ASR_ERR_WORKSPACE,
                "ctc_bf16_db: bias workspace %zu < %zu", bws_bytes,
                asr_ctc_bias_workspace_bytes(T, B, V, gld));
    const int n8 = gld >> 3;
    nch = (n8 + threads - 1) / threads;
    nch = nch <= 1 ? 1 : nch <= 2 ? 2 : nch <= 4 ? 4 : nch <= 5 ? 5 : nch <= 8 ? 8 : 0;
    ASR_REQUIRE(nch > 0 && (table || (size_t)(2 * Spad + V) * 4 <= 64 * 1024), ASR_ERR_UNSUPPORTED,
                "ctc_bf16_db: V %d too wide for the in-kernel bias sums", V);
    ctc_bias_grid(T, B, V, &rpb, &nblk);
    colpart = (float*)bws;
  }
  // algorithmic HBM bytes: activations read (4 V) + bf16 gradient written (2 gld) per row
  const int pslot = prof_begin_launch(ASR_PROF_CTC_GRAD, s, (4.0 * V + 2.0 * gld) * B * T, V);
  const size_t lds = (table ? V : 2 * Spad + (dbias ? V : 0)) * sizeof(float);
#define ASR_CTC_G16A(TB, NC, A)                                                                  \
  hipLaunchKernelGGL((ctc_grad_bf16<TB, NC, A>), dim3((unsigned)nblk), dim3(threads), lds, s,     \
                     acts, stride_t, stride_b, T, V, labels_flat, label_lens, act_lens, ws.offs,  \
                     blank, Spad, ws.lse, ws.emit, ws.alpha, ws.beta, ws.logp, grad_scale, scale, \
                     grads, gstride_t, gstride_b, gld, rev, abytes, colpart, rpb, rows)
#define ASR_CTC_G16(TB, NC)                  \
  do {                                       \
    if (al) ASR_CTC_G16A(TB, NC, true);      \
    else ASR_CTC_G16A(TB, NC, false);        \
  } while (0)
  // narrow heads: four waves per work-group on rows of their own
  // (ASR_CTC_GRAD_NARROW=0: ctc_grad_bf16<true>, one wave per work-group)
  const char* en = getenv("ASR_CTC_GRAD_NARROW");
  if (table && !(en && en[0] == '0')) {
    if (!dbias) {
      rpb = 4;
      nblk = (int)((rows + 3) / 4);
    }
    const size_t ldsn = (size_t)(4 * V + (dbias ? 4 * gld : 0)) * sizeof(float);
    g_ctc_last_path[1] = 2;
    hipLaunchKernelGGL((ctc_grad_bf16_narrow<1>), dim3((unsigned)nblk), dim3(256), ldsn, s, acts,
                       stride_t, stride_b, T, V, labels_flat, label_lens, act_lens, ws.offs, blank,
                       Spad, ws.lse, ws.emit, ws.alpha, ws.beta, ws.logp, grad_scale, scale, grads,
                       gstride_t, gstride_b, gld, rev, colpart, rpb, rows);
    ASR_LAUNCH_CHECK();
    prof_end_launch(ASR_PROF_CTC_GRAD, pslot, s);
    if (dbias) {
      const size_t part = ((size_t)nblk * gld * sizeof(float) + 255) & ~(size_t)255;
      rc = asr_colsum_accumulate(colpart, gld, nblk, V, 1.0f, dbias, nullptr, (char*)bws + part,
                                 bws_bytes - part, stream);
      if (rc) return rc;
    }
    return ASR_OK;
  }
  const char* ep = getenv("ASR_CTC_GRAD_PIPE");   // 0: the unpipelined pass (A/B)
  const bool pipe = al && !table && nch > 0 && !(ep && ep[0] == '0');
  // the streamed pass (512 threads, 2 work-groups per CU): ASR_CTC_GRAD_STREAM=0 (A/B)
  const char* es = getenv("ASR_CTC_GRAD_STREAM");
  const int n8s = gld >> 3;
  const int nchs = (n8s + 511) / 512;
  if (al && !table && nchs <= 3 && !(es && es[0] == '0')) {   // NCH 4 spills at 128 VGPRs
    static int cus = 0;
    if (cus == 0) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          cus <= 0)
        cus = 256;
    }
    long long nb2 = std::min<long long>(rows, 2LL * cus);
    if (dbias) nb2 = std::min<long long>(nb2, nblk);   // the bias workspace holds nblk partials
    const long long rp2 = (rows + nb2 - 1) / nb2;
    rpb = (int)rp2;
    nblk = (int)((rows + rp2 - 1) / rp2);
    const size_t lds2 = (size_t)(5 * Spad + n8s + 8) * sizeof(float);
    g_ctc_last_path[1] = 4;
#define ASR_CTC_GS(NC)                                                                           \
  hipLaunchKernelGGL((ctc_grad_bf16_stream<NC>), dim3((unsigned)nblk), dim3(512), lds2, s, acts, \
                     stride_t, stride_b, T, V, labels_flat, label_lens, act_lens, ws.offs, blank, \
                     Spad, ws.lse, ws.emit, ws.alpha, ws.beta, ws.logp, grad_scale, scale, grads, \
                     gstride_t, gstride_b, gld, rev, abytes, colpart, rpb, rows)
    switch (nchs) {
      case 1: ASR_CTC_GS(1); break;
      case 2: ASR_CTC_GS(2); break;
      default: ASR_CTC_GS(3); break;
    }
#undef ASR_CTC_GS
  } else
#define ASR_CTC_GP(NC)                                                                           \
  hipLaunchKernelGGL((ctc_grad_bf16_pipe<NC>), dim3((unsigned)nblk), dim3(threads), lds, s, acts, \
                     stride_t, stride_b, T, V, labels_flat, label_lens, act_lens, ws.offs, blank, \
                     Spad, ws.lse, ws.emit, ws.alpha, ws.beta, ws.logp, grad_scale, scale, grads, \
                     gstride_t, gstride_b, gld, rev, abytes, colpart, rpb, rows)
  if (pipe) {
    g_ctc_last_path[1] = 3;
    switch (nch) {
      case 1: ASR_CTC_GP(1); break;
      case 2: ASR_CTC_GP(2); break;
      case 4: ASR_CTC_GP(4); break;
      case 5: ASR_CTC_GP(5); break;
      default: ASR_CTC_GP(8); break;
    }
  } else if (table) {
    g_ctc_last_path[1] = 1;
    if (nch) ASR_CTC_G16A(true, 1, false);
    else ASR_CTC_G16A(true, 0, false);
  } else {
    g_ctc_last_path[1] = 1;
    switch (nch) {
      case 0: ASR_CTC_G16(false, 0); break;
      case 1: ASR_CTC_G16(false, 1); break;
      case 2: ASR_CTC_G16(false, 2); break;
      case 4: ASR_CTC_G16(false, 4); break;
      case 5: ASR_CTC_G16(false, 5); break;
      default: ASR_CTC_G16(false, 8); break;
    }
  }
#undef ASR_CTC_G16A
#undef ASR_CTC_GP
#undef ASR_CTC_G16
  ASR_LAUNCH_CHECK();
  prof_end_launch(ASR_PROF_CTC_GRAD, pslot, s);
  if (dbias) {   // fixed-order column sums of the per-block partials, added into dbias
    const size_t part = ((size_t)nblk * gld * sizeof(float) + 255) & ~(size_t)255;
    rc = asr_colsum_accumulate(colpart, gld, nblk, V, 1.0f, dbias, nullptr, (char*)bws + part,
                               bws_bytes - part, stream);
    if (rc) return rc;
  }
  return ASR_OK;
}

extern "C" int asr_ctc_backward_bf16(const float* acts, long long stride_t, long long stride_b,
                                     int T, int B, int V, const int32_t* labels_flat,
                                     const int32_t* label_lens, const int32_t* act_lens,
                                     int max_label_len, int blank, const float* grad_scale,
                                     float scale, uint16_t* grads, long long gstride_t,
                                     long long gstride_b, int gld, const void* workspace,
                                     size_t ws_bytes, void* stream) {
  return ctc_backward_bf16_impl(acts, stride_t, stride_b, T, B, V, labels_flat, label_lens,
                                act_lens, max_label_len, blank, grad_scale, scale, grads,
                                gstride_t, gstride_b, gld, workspace, ws_bytes, nullptr, nullptr, 0,
                                stream);
}

extern "C" int asr_ctc_backward_bf16_db(const float* acts, long long stride_t, long long stride_b,
                                        int T, int B, int V, const int32_t* labels_flat,
                                        const int32_t* label_lens, const int32_t* act_lens,
                                        int max_label_len, int blank, const float* grad_scale,
                                        float scale, uint16_t* grads, long long gstride_t,
                                        long long gstride_b, int gld, const void* workspace,
                                        size_t ws_bytes, float* dbias, void* bias_ws,
                                        size_t bias_ws_bytes, void* stream) {
  ASR_REQUIRE(dbias, ASR_ERR_ARG, "ctc_bf16_db: dbias is null");
  return ctc_backward_bf16_impl(acts, stride_t, stride_b, T, B, V, labels_flat, label_lens,
                                act_lens, max_label_len, blank, grad_scale, scale, grads,
                                gstride_t, gstride_b, gld, workspace, ws_bytes, dbias, bias_ws,
                                bias_ws_bytes, stream);
}

extern "C" int asr_ctc_fwd_bwd(const float* acts, long long stride_t, long long stride_b, int T,
                               int B, int V, const int32_t* labels_flat,
                               const int32_t* label_lens, const int32_t* act_lens,
                               int max_label_len, int blank, int zero_infinity, float* costs,
                               float* grads, void* workspace, size_t ws_bytes, void* stream) {
  int rc = asr_ctc_forward(acts, stride_t, stride_b, T, B, V, labels_flat, label_lens, act_lens,
                           max_label_len, blank, zero_infinity, costs, nullptr, 1.f, workspace,
                           ws_bytes, stream);
  if (rc || !grads) return rc;
  return asr_ctc_backward(acts, stride_t, stride_b, T, B, V, labels_flat, label_lens, act_lens,
                          max_label_len, blank, nullptr, 1.f, grads, stride_t, stride_b, workspace,
                          ws_bytes, stream);
}
