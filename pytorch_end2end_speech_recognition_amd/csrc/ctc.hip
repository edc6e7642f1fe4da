// CTC forward-backward on gfx950 -- replaces warp-ctc's gpu_ctc as bound by
// models/pytorch_v3/ctc/ctc.py:30-66 (my_warpctc).  Algorithm restated from the
// reference's own numpy CTC text (models/chainer/ctc/ctc_loss_from_chainer.py):
// log-space alpha/beta over the blank-interleaved label lattice, gradient =
// softmax - label occupancy, masked beyond the input length.
//
// Kernels (all stream-ordered, no host sync):
//   ctc_prep    1 block: exclusive scan of label_lens -> label offsets; label
//               range check -> status word.
//   ctc_emit    one wave per (b,t) row: log-sum-exp over V (one HBM read of the
//               row) and the S emissions e_t(s) = x[lab(s)] - lse, stored
//               lattice-contiguous so the sequential kernel streams them.
//   ctc_lattice two waves per utterance, run concurrently: the alpha wave
//               (forward over t, then log P and the cost) and the beta wave
//               (backward over t); lane l owns K consecutive lattice states in
//               registers, neighbours come through DPP wave shifts (one
//               v_mov_dpp per step, no LDS, no barrier).  The sequential depth
//               is T steps, not the 2T of an alpha-then-beta pass.
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

// One wave per (b,t) row.
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
  float m = neg_inf();
  for (int v = lane; v < V; v += 64) m = fmaxf(m, x[v]);
  m = wave_max(m);
  float s = 0.f;
  for (int v = lane; v < V; v += 64) s += __expf(x[v] - m);
  s = wave_sum(s);
  const float lse = m + __logf(s);
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
      v = x[c] - lse;
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

// DPP wave shifts (GFX9 wave_shr:1 / wave_shl:1): lane i receives lane i-1 /
// i+1; the lane without a source receives 0 (callers overwrite it).
__device__ __forceinline__ float from_lower_lane(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float from_upper_lane(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x130, 0xf, 0xf, false));
}

// Two waves per utterance (blockIdx.y: 0 = alpha, 1 = beta).  Lane l owns
// lattice states s = l*K + k.
template <int K>
__global__ void __launch_bounds__(64) ctc_lattice(int T, const int32_t* __restrict__ labels,
                                                  const int32_t* __restrict__ label_lens,
                                                  const int32_t* __restrict__ act_lens,
                                                  const int32_t* __restrict__ offs, int blank,
                                                  int zero_infinity, const float* __restrict__ emit,
                                                  float* __restrict__ alpha,
                                                  float* __restrict__ beta,
                                                  float* __restrict__ logp_out,
                                                  float* __restrict__ costs) {
  constexpr int Spad = 64 * K;
  constexpr int D = 4;  // emission prefetch distance (steps)
  const int b = blockIdx.x;
  const bool is_beta = blockIdx.y == 1;
  const int lane = threadIdx.x;
  const int Tb = min(act_lens[b], T);
  const int L = min(label_lens[b], (Spad - 1) / 2);
  const int S = 2 * L + 1;
  const int32_t* lab = labels + offs[b];
  const float NEG = neg_inf();

  if (Tb <= 0) {
    if (lane == 0 && !is_beta) {
      bool feas = (L == 0);
      logp_out[b] = feas ? 0.f : NEG;
      costs[b] = feas ? 0.f : (zero_infinity ? 0.f : __builtin_huge_valf());
    }
    return;
  }

  bool valid[K];
#pragma unroll
  for (int k = 0; k < K; ++k) valid[k] = lane * K + k < S;
  const float* E = emit + (size_t)b * T * Spad + lane * K;
  float eb[D][K];

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
#pragma unroll
    for (int j = 0; j < D; ++j) load_k<K>(eb[j], E + (size_t)min(1 + j, T - 1) * Spad);

    for (int t0 = 1; t0 < Tb; t0 += D) {
#pragma unroll
      for (int j = 0; j < D; ++j) {
        const int t = t0 + j;
        if (t < Tb) {
          float p1 = from_lower_lane(a[K - 1]);
          float p2 = (K >= 2) ? from_lower_lane(a[K >= 2 ? K - 2 : 0]) : from_lower_lane(p1);
          if (lane == 0) { p1 = NEG; p2 = NEG; }
          if (K == 1 && lane == 1) p2 = NEG;
          float n[K];
#pragma unroll
          for (int k = 0; k < K; ++k) {
            const float a1 = (k >= 1) ? a[k >= 1 ? k - 1 : 0] : p1;
            const float a2 = (k >= 2) ? a[k >= 2 ? k - 2 : 0] : ((k == 1) ? p1 : p2);
            const float v = lse3(a[k], a1, skip[k] ? a2 : NEG) + eb[j][k];
            n[k] = valid[k] ? v : NEG;
          }
#pragma unroll
          for (int k = 0; k < K; ++k) a[k] = n[k];
          store_k<K>(A + (size_t)t * Spad, a);
          load_k<K>(eb[j], E + (size_t)min(t + D, T - 1) * Spad);
        }
      }
    }

    // log P from the last two states at t = Tb-1
    float part = NEG;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int s = lane * K + k;
      if (s == S - 1 || s == S - 2) part = lse2(part, a[k]);
    }
    float mx = wave_max(part);
    float sm = (mx == NEG) ? 0.f : wave_sum(__expf(part - mx));
    const float logP = (mx == NEG) ? NEG : mx + __logf(sm);
    if (lane == 0) {
      logp_out[b] = logP;
      costs[b] = (logP == NEG) ? (zero_infinity ? 0.f : __builtin_huge_valf()) : -logP;
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
#pragma unroll
  for (int j = 0; j < D; ++j) load_k<K>(eb[j], E + (size_t)max(Tb - 2 - j, 0) * Spad);
  for (int t0 = Tb - 2; t0 >= 0; t0 -= D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int t = t0 - j;
      if (t >= 0) {
        float n1 = from_upper_lane(be[0]);
        float n2 = (K >= 2) ? from_upper_lane(be[K >= 2 ? 1 : 0]) : from_upper_lane(n1);
        if (lane == 63) { n1 = NEG; n2 = NEG; }
        if (K == 1 && lane == 62) n2 = NEG;
        float n[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float b1 = (k < K - 1) ? be[k < K - 1 ? k + 1 : 0] : n1;
          const float b2 = (k < K - 2) ? be[k < K - 2 ? k + 2 : 0] : ((k == K - 2) ? n1 : n2);
          const float v = lse3(be[k], b1, skipf[k] ? b2 : NEG) + eb[j][k];
          n[k] = valid[k] ? v : NEG;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) be[k] = n[k];
        store_k<K>(Bt + (size_t)t * Spad, be);
        load_k<K>(eb[j], E + (size_t)max(t - D, 0) * Spad);
      }
    }
  }
}

// grad = (softmax - occupancy) * scale, one row (b,t) per block.
__global__ void ctc_grad(const float* __restrict__ acts, long long st, long long sb, int T, int V,
                         const int32_t* __restrict__ labels, const int32_t* __restrict__ label_lens,
                         const int32_t* __restrict__ act_lens, const int32_t* __restrict__ offs,
                         int blank, int Spad, const float* __restrict__ lse,
                         const float* __restrict__ emit, const float* __restrict__ alpha,
                         const float* __restrict__ beta, const float* __restrict__ logp,
                         const float* __restrict__ grad_scale, float scale_mul,
                         float* __restrict__ grads,
                         long long gst, long long gsb) {
  extern __shared__ __attribute__((aligned(16))) float acc[];
  const long long row = blockIdx.x;
  const int b = (int)(row / T), t = (int)(row % T);
  float* g = grads + (long long)t * gst + (long long)b * gsb;
  const int Tb = act_lens[b];
  const float lp = logp[b];
  if (t >= Tb || lp == neg_inf()) {
    for (int v = threadIdx.x; v < V; v += blockDim.x) g[v] = 0.f;
    return;
  }
  const float scale = (grad_scale ? grad_scale[0] : 1.0f) * scale_mul;
  for (int v = threadIdx.x; v < V; v += blockDim.x) acc[v] = 0.f;
  __syncthreads();
  const int L = min(label_lens[b], (Spad - 1) / 2);
  const int S = 2 * L + 1;
  const int32_t* lab = labels + offs[b];
  const float* al = alpha + row * Spad;
  const float* bt = beta + row * Spad;
  const float* em = emit + row * Spad;
  for (int s = threadIdx.x; s < S; s += blockDim.x) {
    int c = (s & 1) ? lab[s >> 1] : blank;
    c = c < 0 ? 0 : (c >= V ? V - 1 : c);
    atomicAdd(&acc[c], __expf(al[s] + bt[s] - em[s] - lp));
  }
  __syncthreads();
  const float* x = acts + (long long)t * st + (long long)b * sb;
  const float z = lse[row];
  for (int v = threadIdx.x; v < V; v += blockDim.x) g[v] = (__expf(x[v] - z) - acc[v]) * scale;
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

extern "C" int asr_ctc_forward(const float* acts, long long stride_t, long long stride_b, int T,
                               int B, int V, const int32_t* labels_flat,
                               const int32_t* label_lens, const int32_t* act_lens,
                               int max_label_len, int blank, int zero_infinity, float* costs,
                               float* loss_out, float loss_scale, void* workspace,
                               size_t ws_bytes, void* stream) {
  int rc = check_common(acts, T, B, V, labels_flat, label_lens, act_lens, max_label_len, blank,
                        workspace, ws_bytes);
  if (rc) return rc;
  ASR_REQUIRE(costs, ASR_ERR_ARG, "ctc: costs is null");
  hipStream_t s = (hipStream_t)stream;
  CtcWs ws;
  ws_layout(T, B, max_label_len, &ws, (char*)workspace);
  const int K = pick_k(max_label_len);
  const int Spad = 64 * K;
  hipLaunchKernelGGL(ctc_prep, dim3(1), dim3(256), 0, s, label_lens, labels_flat, B, V, blank,
                     max_label_len, ws.offs, ws.status);
  ASR_LAUNCH_CHECK();
  const long long rows = (long long)B * T;
  // algorithmic HBM bytes of the forward: the activations read once
  const int pslot = prof_begin_launch(ASR_PROF_CTC_FWD, s, 4.0 * (double)V * (double)rows);
  hipLaunchKernelGGL(ctc_emit, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, acts, stride_t,
                     stride_b, T, B, V, labels_flat, label_lens, act_lens, ws.offs, blank, Spad,
                     ws.lse, ws.emit);
  ASR_LAUNCH_CHECK();
#define ASR_CTC_LAT(KK)                                                                        \
  hipLaunchKernelGGL(ctc_lattice<KK>, dim3(B, 2), dim3(64), 0, s, T, labels_flat, label_lens,  \
                     act_lens, ws.offs, blank, zero_infinity, ws.emit, ws.alpha, ws.beta,      \
                     ws.logp, costs)
  switch (K) {
    case 1: ASR_CTC_LAT(1); break;
    case 2: ASR_CTC_LAT(2); break;
    case 4: ASR_CTC_LAT(4); break;
    case 8: ASR_CTC_LAT(8); break;
    case 16: ASR_CTC_LAT(16); break;
    default: set_error("ctc: unsupported K=%d", K); return ASR_ERR_UNSUPPORTED;
  }
#undef ASR_CTC_LAT
  ASR_LAUNCH_CHECK();
  prof_end_launch(ASR_PROF_CTC_FWD, pslot, s);
  if (loss_out) {
    hipLaunchKernelGGL(ctc_loss_reduce, dim3(1), dim3(256), 0, s, costs, B, loss_scale, loss_out);
    ASR_LAUNCH_CHECK();
  }
  return ASR_OK;
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
  ASR_REQUIRE((size_t)V * 4 <= 160 * 1024, ASR_ERR_UNSUPPORTED, "ctc: V=%d too large", V);
  hipStream_t s = (hipStream_t)stream;
  CtcWs ws;
  ws_layout(T, B, max_label_len, &ws, (char*)workspace);
  const int Spad = 64 * pick_k(max_label_len);
  const int threads = V <= 256 ? 64 : 256;
  // algorithmic HBM bytes: activations read + gradient written
  const int pslot = prof_begin_launch(ASR_PROF_CTC_GRAD, s, 8.0 * (double)V * B * T);
  hipLaunchKernelGGL(ctc_grad, dim3((unsigned)((long long)B * T)), dim3(threads), V * sizeof(float),
                     s, acts, stride_t, stride_b, T, V, labels_flat, label_lens, act_lens, ws.offs,
                     blank, Spad, ws.lse, ws.emit, ws.alpha, ws.beta, ws.logp, grad_scale, scale,
                     grads, gstride_t,
                     gstride_b);
  ASR_LAUNCH_CHECK();
  prof_end_launch(ASR_PROF_CTC_GRAD, pslot, s);
  return ASR_OK;
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
