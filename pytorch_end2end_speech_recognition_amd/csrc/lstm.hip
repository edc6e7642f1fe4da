// Bidirectional LSTM recurrence for the encoder (gfx950).  Replaces the cuDNN /
// MIOpen packed nn.LSTM(bidirectional=True) of models/pytorch_v3/encoders/rnn.py
// (:166-172 fast path, :218-224 per-layer path, packing :343-358, :377-390).
//
// Semantics (nn.LSTM, gate order i,f,g,o; h0 = c0 = 0, rnn.py:499-536):
//   pre  = gx[b,t] + h_prev @ W_hh^T          (gx = x @ W_ih^T + b_ih + b_hh, one GEMM)
//   c    = sig(f) * c_prev + sig(i) * tanh(g),  h = sig(o) * tanh(c)
// Packed-sequence behaviour is reproduced with per-utterance length masks: for
// t >= len[b] the state and the output are 0, so the reverse direction starts at
// each utterance's own last frame and padded outputs are zero (pad_packed).
//
// One launch per time step processes BOTH directions (forward at t = s, reverse
// at t = T-1-s).  Work-group = (4 hidden units x 4 gates = 16 gate columns) x 32
// utterances; its 4 waves split the K = H reduction and combine through LDS, so
// the 16x16 MFMA tile holds all four gates of its units and the cell update is
// fused into the same kernel.  h_{t-1} is read from a ping-pong buffer kept in
// the compute dtype (bf16 in performance mode: half the bytes per step).
//
// Backward: one launch per step in reverse processing order.  Work-group = 16
// units x 32 utterances, K = 4H over the previous step's gate gradients times
// W_hh (a transposed copy, so each lane's 8-element MFMA fragment is contiguous).
// The gate gradients are written over the saved activations and then feed the
// weight-gradient GEMMs (asr_gemm) outside the recurrence.
#include <algorithm>

#include "mfma.h"
#include "prof.h"

namespace asr {

// persistent recurrence (lstm_persist.hip)
size_t persist_ctr_bytes(int B);
int persist_rows(int B);
int lstm_fwd_persistent(int B, int T, int H, const int32_t* lens, const uint16_t* wbf,
                        float* gx_act, float* y, float* cst, uint16_t* hx, int* ctr,
                        uint16_t* ybf, hipStream_t s, bool dry);
int lstm_bwd_persistent(int B, int T, int H, const int32_t* lens, const uint16_t* wt,
                        const float* dy, float* act_dg, const float* cst, uint16_t* dgx, int* ctr,
                        uint16_t* dgbf, hipStream_t s, bool dry);
// tagged-granule persistent recurrence (lstm_xg.hip), preferred when eligible
size_t lstm_xg_fwd_bytes(int B, int H);
size_t lstm_xg_bwd_bytes(int B, int H);
int lstm_fwd_xg_launch(int B, int T, int H, const int32_t* lens, const float* whh_f,
                       const float* whh_r, float* gx_act, float* y, float* cst, void* ws,
                       uint16_t* ybf, hipStream_t s, bool dry);
int lstm_bwd_xg_launch(int B, int T, int H, const int32_t* lens, const float* whh_f,
                       const float* whh_r, const float* dy, float* act_dg, const float* cst,
                       void* ws, uint16_t* dgbf, float* dbpart, hipStream_t s, bool dry,
                       bool dg_f32, const uint16_t* acth = nullptr);
// the same hand-off at reference precision (f32 granules, f32 MFMA)
size_t lstm_xg32_fwd_bytes(int B, int H);
size_t lstm_xg32_bwd_bytes(int B, int H);
int lstm_fwd_xg32_launch(int B, int T, int H, const int32_t* lens, const float* whh_f,
                         const float* whh_r, float* gx_act, float* y, float* cst, void* ws,
                         hipStream_t s, bool dry);
int lstm_bwd_xg32_launch(int B, int T, int H, const int32_t* lens, const float* whh_f,
                         const float* whh_r, const float* dy, float* act_dg, const float* cst,
                         void* ws, float* dbpart, hipStream_t s, bool dry);

namespace {

// db_ih[n] += sum_b part[b][n]; db_hh[n] += the same (fixed order over b).
__global__ void bias_from_partials(const float* __restrict__ part, int B, int N,
                                   float* __restrict__ db_ih, float* __restrict__ db_hh) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  // four independent partial sums (every load in flight; combined in a fixed order)
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int b = 0;
  for (; b + 4 <= B; b += 4) {
    s0 += part[(long long)b * N + n];
    s1 += part[(long long)(b + 1) * N + n];
    s2 += part[(long long)(b + 2) * N + n];
    s3 += part[(long long)(b + 3) * N + n];
  }
  for (; b < B; ++b) s0 += part[(long long)b * N + n];
  const float s = (s0 + s1) + (s2 + s3);
  db_ih[n] += s;
  if (db_hh) db_hh[n] += s;
}


constexpr int FU = 4;   // forward: units per work-group (16 gate columns)
constexpr int BU = 16;   // backward: units per work-group
constexpr int MB = 32;   // utterances per work-group (two 16-row MFMA blocks)

// ---- operand fragment loads (guarded for arbitrary H / B) ----------------
template <typename T>
__device__ __forceinline__ float ldf(const T* p, long long i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, long long i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<uint16_t>(const uint16_t* p, long long i) { return bf2f(p[i]); }

// 8 consecutive elements [k, k+8) of row `row` (nullptr row -> zeros), k < klim.
template <typename T>
__device__ __forceinline__ bf16x8 frag8(const T* row, int k, int klim, bool vec) {
  if (row == nullptr) return as_bf16x8(u16x8{0, 0, 0, 0, 0, 0, 0, 0});
  if (vec && k + 8 <= klim) {
    if constexpr (sizeof(T) == 2) return load_bf16x8((const uint16_t*)row + k);
    else return load_bf16x8_from_f32((const float*)row + k);
  }
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (k + j < klim) ? f2bf(ldf<T>(row, k + j)) : (uint16_t)0;
  return as_bf16x8(r);
}

template <typename T>
__device__ __forceinline__ float frag1(const T* row, int k, int klim) {
  return (row != nullptr && k < klim) ? ldf<T>(row, k) : 0.f;
}

// Partial products of one wave: acc[mb] (+)= A[rows of block mb][k-range] * B[cols][k-range]
// A rows: a_row[mb] (per lane: row l&15 of block mb), B row: b_row (per lane: col l&15).
template <bool BF16, typename TA, typename TB>
__device__ __forceinline__ void wave_dot(const TA* a_row0, const TA* a_row1, const TB* b_row,
                                         int K, int wave, bool vec, f32x4& acc0, f32x4& acc1) {
  const int lane = threadIdx.x & 63;
  if (BF16) {
    for (int k0 = wave * 32; k0 < K; k0 += 4 * 32) {
      const int k = k0 + 8 * (lane >> 4);
      const bf16x8 b = frag8<TB>(b_row, k, K, vec);
      acc0 = mfma_bf16(frag8<TA>(a_row0, k, K, vec), b, acc0);
      acc1 = mfma_bf16(frag8<TA>(a_row1, k, K, vec), b, acc1);
    }
  } else {
    for (int k0 = wave * 4; k0 < K; k0 += 4 * 4) {
      const int k = k0 + (lane >> 4);
      const float b = frag1<TB>(b_row, k, K);
      acc0 = mfma_f32(frag1<TA>(a_row0, k, K), b, acc0);
      acc1 = mfma_f32(frag1<TA>(a_row1, k, K), b, acc1);
    }
  }
}

__device__ __forceinline__ void store_state(float* p, long long i, float v) { p[i] = v; }
__device__ __forceinline__ void store_state(uint16_t* p, long long i, float v) { p[i] = f2bf(v); }

// ---------------------------------------------------------------------------
// forward step.  grid = (ceil(H/FU), 2 directions, ceil(B/MB)), block = 256
// ---------------------------------------------------------------------------
template <bool BF16, typename TW, typename TS>
__global__ void __launch_bounds__(256) lstm_fwd_step(
    int s, int B, int T, int H, const int32_t* __restrict__ lens, const TW* __restrict__ whh_f,
    const TW* __restrict__ whh_r, float* __restrict__ gx_act, float* __restrict__ y,
    float* __restrict__ cst, TS* __restrict__ hbuf, int vec) {
  __shared__ float part[4][MB][16];
  const int dir = blockIdx.y;
  const int u0 = blockIdx.x * FU;
  const int b0 = blockIdx.z * MB;
  const int t = dir == 0 ? s : T - 1 - s;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const TW* W = dir == 0 ? whh_f : whh_r;
  const long long BH = (long long)B * H;
  // ping-pong h: hbuf[parity][dir][b][H]; step s reads parity (s+1)&1, writes s&1
  const TS* hprev = hbuf + ((long long)((s + 1) & 1) * 2 + dir) * BH;
  TS* hnext = hbuf + ((long long)(s & 1) * 2 + dir) * BH;

  // fragment rows for this lane
  const int ra = b0 + (lane & 15), rb = b0 + 16 + (lane & 15);
  const TS* a_row0 = ra < B ? hprev + (long long)ra * H : nullptr;
  const TS* a_row1 = rb < B ? hprev + (long long)rb * H : nullptr;
  const int n = lane & 15, g = n >> 2, u = u0 + (n & 3);
  const TW* b_row = u < H ? W + (long long)(g * H + u) * H : nullptr;

  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if (s > 0) wave_dot<BF16, TS, TW>(a_row0, a_row1, b_row, H, wave, vec != 0, acc0, acc1);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    part[wave][4 * (lane >> 4) + r][lane & 15] = acc0[r];
    part[wave][16 + 4 * (lane >> 4) + r][lane & 15] = acc1[r];
  }
  __syncthreads();
  if (threadIdx.x >= MB * FU) return;
  const int row = threadIdx.x >> 2, uu = threadIdx.x & 3;
  const int b = b0 + row, j = u0 + uu;
  if (b >= B || j >= H) return;
  const bool active = t < lens[b];
  const long long gbase = ((long long)b * T + t) * 8 * H + (long long)dir * 4 * H + j;
  const long long sidx = ((long long)b * T + t) * 2 * H + (long long)dir * H + j;
  float pre[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    pre[q] = part[0][row][q * 4 + uu] + part[1][row][q * 4 + uu] + part[2][row][q * 4 + uu] +
             part[3][row][q * 4 + uu] + gx_act[gbase + (long long)q * H];
  const int tp = dir == 0 ? t - 1 : t + 1;
  const float cprev = (tp >= 0 && tp < T) ? cst[sidx + (long long)(tp - t) * 2 * H] : 0.f;
  const float ig = sigmoidf_(pre[0]), fg = sigmoidf_(pre[1]);
  const float gg = tanhf_(pre[2]), og = sigmoidf_(pre[3]);
  float c = fg * cprev + ig * gg;
  float h = og * tanhf_(c);
  if (!active) { c = 0.f; h = 0.f; }
  y[sidx] = h;
  cst[sidx] = c;
  gx_act[gbase] = active ? ig : 0.f;
  gx_act[gbase + H] = active ? fg : 0.f;
  gx_act[gbase + 2 * H] = active ? gg : 0.f;
  gx_act[gbase + 3 * H] = active ? og : 0.f;
  store_state(hnext, (long long)b * H + j, h);
}

// ---------------------------------------------------------------------------
// Latency-optimised bf16 step kernels (H % 32 == 0).  A step is a short
// dependent chain, so everything a thread will need is put in flight at kernel
// entry: the epilogue operands (gates input, c_{t-1}, length) and ALL of the
// wave's MFMA fragments (no guards, clamped rows -> no branches between loads
// and one vmcnt wait), then the MFMAs, one LDS combine, the fused cell update.
// ---------------------------------------------------------------------------
template <int MAXKS>
__global__ void __launch_bounds__(256) lstm_fwd_step_fast(
    int s, int B, int T, int H, const int32_t* __restrict__ lens,
    const uint16_t* __restrict__ whh_f, const uint16_t* __restrict__ whh_r,
    float* __restrict__ gx_act, float* __restrict__ y, float* __restrict__ cst,
    uint16_t* __restrict__ hbuf) {
  __shared__ float part[4][MB][16];
  const int dir = blockIdx.y;
  const int u0 = blockIdx.x * FU;
  const int b0 = blockIdx.z * MB;
  const int t = dir == 0 ? s : T - 1 - s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long long BH = (long long)B * H;

  // epilogue prefetch (threads < 128: one (utterance, unit) each)
  const int row = tid >> 2, uu = tid & 3;
  const int b = b0 + row, j = u0 + uu;
  const bool own = tid < MB * FU && b < B && j < H;
  const int bc = own ? b : 0, jc = own ? j : 0;
  const long long gbase = ((long long)bc * T + t) * 8 * H + (long long)dir * 4 * H + jc;
  const long long sidx = ((long long)bc * T + t) * 2 * H + (long long)dir * H + jc;
  const int tp = dir == 0 ? t - 1 : t + 1;
  const bool has_prev = tp >= 0 && tp < T;
  float gxv[4], cprev = 0.f;
  int len = 0;
  if (own) {
#pragma unroll
    for (int q = 0; q < 4; ++q) gxv[q] = gx_act[gbase + (long long)q * H];
    cprev = has_prev ? cst[sidx + (long long)(tp - t) * 2 * H] : 0.f;
    len = lens[bc];
  }

  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if (s > 0) {
    const uint16_t* hprev = hbuf + ((long long)((s + 1) & 1) * 2 + dir) * BH;
    const uint16_t* W = dir == 0 ? whh_f : whh_r;
    const int ra = min(b0 + (lane & 15), B - 1), rb = min(b0 + 16 + (lane & 15), B - 1);
    const int n = lane & 15, g = n >> 2, u = min(u0 + (n & 3), H - 1);
    const uint16_t* pa0 = hprev + (long long)ra * H + 8 * (lane >> 4);
    const uint16_t* pa1 = hprev + (long long)rb * H + 8 * (lane >> 4);
    const uint16_t* pb = W + (long long)(g * H + u) * H + 8 * (lane >> 4);
    const int nks = H >> 5;
    bf16x8 fa0[MAXKS], fa1[MAXKS], fb[MAXKS];
#pragma unroll
    for (int i = 0; i < MAXKS; ++i) {   // unconditional (clamped) loads: no branch, one wait
      const int kc = min(wave + 4 * i, nks - 1) * 32;
      fb[i] = load_bf16x8(pb + kc);
      fa0[i] = load_bf16x8(pa0 + kc);
      fa1[i] = load_bf16x8(pa1 + kc);
    }
#pragma unroll
    for (int i = 0; i < MAXKS; ++i) {
      if (wave + 4 * i < nks) {
        acc0 = mfma_bf16(fa0[i], fb[i], acc0);
        acc1 = mfma_bf16(fa1[i], fb[i], acc1);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    part[tid >> 6][4 * (lane >> 4) + r][lane & 15] = acc0[r];
    part[tid >> 6][16 + 4 * (lane >> 4) + r][lane & 15] = acc1[r];
  }
  __syncthreads();
  if (!own) return;
  float pre[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    pre[q] = part[0][row][q * 4 + uu] + part[1][row][q * 4 + uu] + part[2][row][q * 4 + uu] +
             part[3][row][q * 4 + uu] + gxv[q];
  const bool active = t < len;
  const float ig = sigmoidf_(pre[0]), fg = sigmoidf_(pre[1]);
  const float gg = tanhf_(pre[2]), og = sigmoidf_(pre[3]);
  float c = fg * cprev + ig * gg;
  float h = og * tanhf_(c);
  if (!active) { c = 0.f; h = 0.f; }
  y[sidx] = h;
  cst[sidx] = c;
  gx_act[gbase] = active ? ig : 0.f;
  gx_act[gbase + H] = active ? fg : 0.f;
  gx_act[gbase + 2 * H] = active ? gg : 0.f;
  gx_act[gbase + 3 * H] = active ? og : 0.f;
  hbuf[((long long)(s & 1) * 2 + dir) * BH + (long long)b * H + j] = f2bf(h);
}

// backward: WG = 16 units x 16 utterances, 8 waves split K = 4H.
constexpr int BMB = 16;
template <int MAXKS>
__global__ void __launch_bounds__(512) lstm_bwd_step_fast(
    int q, int B, int T, int H, const int32_t* __restrict__ lens,
    const uint16_t* __restrict__ wt, const float* __restrict__ dy,
    float* __restrict__ act_dg, const float* __restrict__ cst, uint16_t* __restrict__ dgbuf,
    float* __restrict__ dc) {
  __shared__ float part[8][BMB][16];
  const int dir = blockIdx.y;
  const int u0 = blockIdx.x * BU;
  const int b0 = blockIdx.z * BMB;
  const int t = dir == 0 ? T - 1 - q : q;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H4 = 4 * H;
  const long long BG = (long long)B * H4;

  // epilogue prefetch (threads < 256: one (utterance, unit) each)
  const int row = tid >> 4, uu = tid & 15;
  const int b = b0 + row, j = u0 + uu;
  const bool own = tid < BMB * BU && b < B && j < H;
  const int bc = own ? b : 0, jc = own ? j : 0;
  const long long gbase = ((long long)bc * T + t) * 8 * H + (long long)dir * H4 + jc;
  const long long sidx = ((long long)bc * T + t) * 2 * H + (long long)dir * H + jc;
  const long long cidx = ((long long)dir * B + bc) * H + jc;
  const int tp = dir == 0 ? t - 1 : t + 1;
  float av[4] = {0.f, 0.f, 0.f, 0.f}, c = 0.f, cp = 0.f, dyv = 0.f, dcv = 0.f;
  int len = 0;
  if (own) {
#pragma unroll
    for (int k = 0; k < 4; ++k) av[k] = act_dg[gbase + (long long)k * H];
    c = cst[sidx];
    cp = (tp >= 0 && tp < T) ? cst[sidx + (long long)(tp - t) * 2 * H] : 0.f;
    dyv = dy ? dy[sidx] : 0.f;
    dcv = dc[cidx];
    len = lens[bc];
  }

  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (q > 0) {
    const uint16_t* gprev = dgbuf + ((long long)((q + 1) & 1) * 2 + dir) * BG;
    const uint16_t* W = wt + (long long)dir * H * H4;
    const int ra = min(b0 + (lane & 15), B - 1);
    const int jl = min(u0 + (lane & 15), H - 1);
    const uint16_t* pa = gprev + (long long)ra * H4 + 8 * (lane >> 4);
    const uint16_t* pb = W + (long long)jl * H4 + 8 * (lane >> 4);
    const int nks = H4 >> 5;
    bf16x8 fa[MAXKS], fb[MAXKS];
#pragma unroll
    for (int i = 0; i < MAXKS; ++i) {   // unconditional (clamped) loads: no branch, one wait
      const int kc = min(wave + 8 * i, nks - 1) * 32;
      fa[i] = load_bf16x8(pa + kc);
      fb[i] = load_bf16x8(pb + kc);
    }
#pragma unroll
    for (int i = 0; i < MAXKS; ++i)
      if (wave + 8 * i < nks) acc = mfma_bf16(fa[i], fb[i], acc);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) part[tid >> 6][4 * (lane >> 4) + r][lane & 15] = acc[r];
  __syncthreads();
  if (!own) return;
  uint16_t* gn = dgbuf + ((long long)(q & 1) * 2 + dir) * BG + (long long)b * H4 + j;
  if (t >= len) {
    act_dg[gbase] = 0.f; act_dg[gbase + H] = 0.f; act_dg[gbase + 2 * H] = 0.f;
    act_dg[gbase + 3 * H] = 0.f;
    gn[0] = 0; gn[H] = 0; gn[2 * H] = 0; gn[3 * H] = 0;
    dc[cidx] = 0.f;
    return;
  }
  float dh = dyv;
#pragma unroll
  for (int w = 0; w < 8; ++w) dh += part[w][row][uu];
  const float ig = av[0], fg = av[1], gg = av[2], og = av[3];
  const float tc = tanhf_(c);
  const float dcell = dcv + dh * og * (1.f - tc * tc);
  const float d_i = dcell * gg * ig * (1.f - ig);
  const float d_f = dcell * cp * fg * (1.f - fg);
  const float d_g = dcell * ig * (1.f - gg * gg);
  const float d_o = dh * tc * og * (1.f - og);
  dc[cidx] = dcell * fg;
  act_dg[gbase] = d_i; act_dg[gbase + H] = d_f; act_dg[gbase + 2 * H] = d_g;
  act_dg[gbase + 3 * H] = d_o;
  gn[0] = f2bf(d_i); gn[H] = f2bf(d_f); gn[2 * H] = f2bf(d_g); gn[3 * H] = f2bf(d_o);
}

// ---------------------------------------------------------------------------
// backward step (processing index q: forward dir at t = T-1-q, reverse at t = q)
// grid = (ceil(H/BU), 2, ceil(B/MB)), block = 256
// ---------------------------------------------------------------------------
template <bool BF16, typename TS>
__global__ void __launch_bounds__(256) lstm_bwd_step(
    int q, int B, int T, int H, const int32_t* __restrict__ lens, const TS* __restrict__ wt,
    const float* __restrict__ dy, float* __restrict__ act_dg, const float* __restrict__ cst,
    TS* __restrict__ dgbuf, float* __restrict__ dc, int vec) {
  __shared__ float part[4][MB][16];
  const int dir = blockIdx.y;
  const int u0 = blockIdx.x * BU;
  const int b0 = blockIdx.z * MB;
  const int t = dir == 0 ? T - 1 - q : q;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int H4 = 4 * H;
  const long long BG = (long long)B * H4;
  const TS* gprev = dgbuf + ((long long)((q + 1) & 1) * 2 + dir) * BG;
  TS* gnext = dgbuf + ((long long)(q & 1) * 2 + dir) * BG;
  const TS* W = wt + (long long)dir * H * H4;   // W_hh^T: [H][4H]

  const int ra = b0 + (lane & 15), rb = b0 + 16 + (lane & 15);
  const TS* a_row0 = ra < B ? gprev + (long long)ra * H4 : nullptr;
  const TS* a_row1 = rb < B ? gprev + (long long)rb * H4 : nullptr;
  const int j_l = u0 + (lane & 15);
  const TS* b_row = j_l < H ? W + (long long)j_l * H4 : nullptr;

  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if (q > 0) wave_dot<BF16, TS, TS>(a_row0, a_row1, b_row, H4, wave, vec != 0, acc0, acc1);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    part[wave][4 * (lane >> 4) + r][lane & 15] = acc0[r];
    part[wave][16 + 4 * (lane >> 4) + r][lane & 15] = acc1[r];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < MB * BU; idx += 256) {
    const int row = idx / BU, uu = idx % BU;
    const int b = b0 + row, j = u0 + uu;
    if (b >= B || j >= H) continue;
    const long long gbase = ((long long)b * T + t) * 8 * H + (long long)dir * H4 + j;
    const long long sidx = ((long long)b * T + t) * 2 * H + (long long)dir * H + j;
    const long long cidx = ((long long)dir * B + b) * H + j;
    TS* gn = gnext + (long long)b * H4 + j;
    if (t >= lens[b]) {
      act_dg[gbase] = 0.f; act_dg[gbase + H] = 0.f; act_dg[gbase + 2 * H] = 0.f;
      act_dg[gbase + 3 * H] = 0.f;
      store_state(gn, 0, 0.f); store_state(gn, H, 0.f); store_state(gn, 2 * H, 0.f);
      store_state(gn, 3 * H, 0.f);
      dc[cidx] = 0.f;
      continue;
    }
    const float dh = part[0][row][uu] + part[1][row][uu] + part[2][row][uu] + part[3][row][uu] +
                     (dy ? dy[sidx] : 0.f);
    const float ig = act_dg[gbase], fg = act_dg[gbase + H], gg = act_dg[gbase + 2 * H],
                og = act_dg[gbase + 3 * H];
    const float c = cst[sidx];
    const int tp = dir == 0 ? t - 1 : t + 1;
    const float cprev = (tp >= 0 && tp < T) ? cst[sidx + (long long)(tp - t) * 2 * H] : 0.f;
    const float tc = tanhf_(c);
    const float dcell = dc[cidx] + dh * og * (1.f - tc * tc);
    const float d_i = dcell * gg * ig * (1.f - ig);
    const float d_f = dcell * cprev * fg * (1.f - fg);
    const float d_g = dcell * ig * (1.f - gg * gg);
    const float d_o = dh * tc * og * (1.f - og);
    dc[cidx] = dcell * fg;
    act_dg[gbase] = d_i; act_dg[gbase + H] = d_f; act_dg[gbase + 2 * H] = d_g;
    act_dg[gbase + 3 * H] = d_o;
    store_state(gn, 0, d_i); store_state(gn, H, d_f); store_state(gn, 2 * H, d_g);
    store_state(gn, 3 * H, d_o);
  }
}

// W_hh [4H][H] (f32 or bf16) -> W_hh^T [H][4H] in the compute dtype, both dirs.
template <typename TW, typename TS>
__global__ void transpose_whh(const TW* __restrict__ wf, const TW* __restrict__ wr, int H,
                              TS* __restrict__ out) {
  __shared__ float tile[32][33];
  const int dir = blockIdx.z;
  const TW* w = dir == 0 ? wf : wr;
  const int R = 4 * H, C = H;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? ldf<TW>(w, (long long)r * C + c) : 0.f;
  }
  __syncthreads();
  TS* o = out + (long long)dir * C * R;
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (c < C && r < R) store_state(o, (long long)c * R + r, tile[tx][i]);
  }
}

// [fwd W_hh (n) ; rev W_hh (n)] f32 -> bf16, n = 4H*H each
__global__ void convert_bf16(const float* __restrict__ wf, const float* __restrict__ wr,
                             long long n, uint16_t* __restrict__ out) {
  const long long i0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long long i = i0 + j;
    if (i < n) {
      out[i] = f2bf(wf[i]);
      out[n + i] = f2bf(wr[i]);
    }
  }
}

size_t al256(size_t n) { return (n + 255) & ~size_t(255); }

__global__ void to_bf16(const float* __restrict__ x, uint16_t* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

// Forward workspace: [hand-off counters][ping-pong h: 2 parity x 2 dir x Bp x H,
// compute dtype][bf16 copy of W_hh (bf16 mode)], Bp = B rounded up to 16.
size_t fwd_ctr_bytes(int B) { return al256(persist_ctr_bytes(B)); }
size_t fwd_state_bytes(int B, int H, int cdt) {
  return fwd_ctr_bytes(B) + al256((size_t)4 * persist_rows(B) * H * (cdt == ASR_DT_BF16 ? 2 : 4));
}

size_t fwd_ws(int B, int H, int cdt) {
  size_t w = cdt == ASR_DT_BF16 ? (size_t)2 * 4 * H * H * 2 : 0;  // bf16 copy of W_hh
  const size_t xg = cdt == ASR_DT_BF16 ? lstm_xg_fwd_bytes(B, H) : lstm_xg32_fwd_bytes(B, H);
  return std::max(fwd_state_bytes(B, H, cdt) + w, xg);
}

// Backward workspace: [counters][W_hh^T][ping-pong dgates: 2 x 2 x Bp x 4H][dc f32 2 x B x H]
struct BwdLayout {
  size_t ctr, wt, dg, dcb, total;
};
BwdLayout bwd_layout(int B, int H, int cdt) {
  const size_t es = cdt == ASR_DT_BF16 ? 2 : 4;
  BwdLayout l;
  l.ctr = 0;
  l.wt = fwd_ctr_bytes(B);
  l.dg = l.wt + al256((size_t)2 * H * 4 * H * es);
  l.dcb = l.dg + al256((size_t)4 * persist_rows(B) * 4 * H * es);
  l.total = l.dcb + (size_t)2 * B * H * 4;
  return l;
}
size_t bwd_ws(int B, int H, int cdt) {
  const size_t xg = cdt == ASR_DT_BF16 ? lstm_xg_bwd_bytes(B, H) : lstm_xg32_bwd_bytes(B, H);
  return std::max(bwd_layout(B, H, cdt).total, xg);
}
// Bias-gradient scratch behind the backward workspace: [max(B, 64)][8H] f32
// (per-utterance partials of the fused path, or the colsum chunks otherwise).
size_t bias_ws_off(int B, int H, int cdt) { return al256(bwd_ws(B, H, cdt)); }
size_t bwd_ws_bias(int B, int H, int cdt) {
  return bias_ws_off(B, H, cdt) + (size_t)std::max(B, 64) * 8 * H * sizeof(float);
}

}  // namespace
}  // namespace asr

using namespace asr;

extern "C" size_t asr_colsum_workspace_bytes(int M, int N);
extern "C" int asr_colsum_accumulate(const float* g, long long ld, int M, int N, float alpha,
                                     float* out0, float* out1, void* workspace, size_t ws_bytes,
                                     void* stream);

namespace asr {
// Which recurrence implementation the last layer pass ran, per direction of
// the pass {forward, backward} (host-side record; asr_lstm_last_path):
// 0 per-step kernels, 1 tagged-granule bf16 (lstm_xg.hip), 2 tagged-granule
// f32, 3 tagged-granule bf16 with the fused input projection, 4 counter form.
int g_lstm_last_path[2];
}  // namespace asr

extern "C" int asr_lstm_last_path(int* out2) {
  ASR_REQUIRE(out2, ASR_ERR_ARG, "lstm_last_path: null pointer");
  out2[0] = asr::g_lstm_last_path[0];
  out2[1] = asr::g_lstm_last_path[1];
  return ASR_OK;
}

// backward: 0 forward, 1 backward, 2 backward with bias gradients (asr_lstm_backward_db)
extern "C" size_t asr_lstm_workspace_bytes(int B, int H, int compute_dtype, int backward) {
  if (backward == 2) return bwd_ws_bias(B, H, compute_dtype);
  return backward ? bwd_ws(B, H, compute_dtype) : fwd_ws(B, H, compute_dtype);
}

extern "C" int asr_lstm_forward(float* gx_act, const void* whh_f, const void* whh_r, int w_dtype,
                                const int32_t* lens, int B, int T, int H, int compute_dtype,
                                float* y, float* cst, uint16_t* ybf, void* workspace,
                                size_t ws_bytes, void* stream) {
  ASR_REQUIRE(gx_act && whh_f && whh_r && lens && y && cst && workspace, ASR_ERR_ARG,
              "lstm_forward: null pointer");
  ASR_REQUIRE(B > 0 && T > 0 && H > 0, ASR_ERR_ARG, "lstm_forward: bad shape");
  ASR_REQUIRE(ws_bytes >= fwd_ws(B, H, compute_dtype), ASR_ERR_WORKSPACE,
              "lstm_forward: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const bool bf = compute_dtype == ASR_DT_BF16;
  int* ctr = (int*)workspace;
  void* hbuf = (char*)workspace + fwd_ctr_bytes(B);
  const int vec = (H % 8 == 0) ? 1 : 0;
  dim3 grid(ceil_div(H, FU), 2, ceil_div(B, MB));
  ASR_REQUIRE(bf || w_dtype == ASR_DT_F32, ASR_ERR_ARG, "lstm_forward: f32 compute needs f32 W");
  if (bf && w_dtype == ASR_DT_F32 &&
      lstm_fwd_xg_launch(B, T, H, lens, (const float*)whh_f, (const float*)whh_r, gx_act, y, cst,
                         workspace, ybf, s, true) == 1) {
    // one persistent launch, tagged-granule hand-off (lstm_xg.hip)
    const int slot = prof_begin_launch(ASR_PROF_LSTM_FWD_SEQ, s, 0.0, ASR_PTAG_LSTM_FWD_XG);
    const int rc = lstm_fwd_xg_launch(B, T, H, lens, (const float*)whh_f, (const float*)whh_r,
                                      gx_act, y, cst, workspace, ybf, s, false);
    ASR_REQUIRE(rc == 1, ASR_ERR_HIP, "lstm_forward: tagged-granule launch failed");
    prof_end_launch(ASR_PROF_LSTM_FWD_SEQ, slot, s);
    g_lstm_last_path[0] = 1;
    return ASR_OK;
  }
  if (!bf && lstm_fwd_xg32_launch(B, T, H, lens, (const float*)whh_f, (const float*)whh_r, gx_act,
                                  y, cst, workspace, s, true) == 1) {
    // reference precision: the same persistent hand-off with f32 granules
    const int slot = prof_begin_launch(ASR_PROF_LSTM_FWD_SEQ, s, 0.0, ASR_PTAG_LSTM_FWD_XG);
    const int rc = lstm_fwd_xg32_launch(B, T, H, lens, (const float*)whh_f, (const float*)whh_r,
                                        gx_act, y, cst, workspace, s, false);
    ASR_REQUIRE(rc == 1, ASR_ERR_HIP, "lstm_forward: f32 tagged-granule launch failed");
    prof_end_launch(ASR_PROF_LSTM_FWD_SEQ, slot, s);
    g_lstm_last_path[0] = 2;
    if (ybf) {
      const long long n = (long long)B * T * 2 * H;
      hipLaunchKernelGGL(to_bf16, dim3((unsigned)min(4096LL, (n + 255) / 256)), dim3(256), 0, s, y,
                         ybf, n);
      ASR_LAUNCH_CHECK();
    }
    return ASR_OK;
  }
  // bf16 mode with f32 weights: one conversion pass so the T step launches
  // stream 2 bytes per weight instead of 4.
  const uint16_t* wbf_f = (const uint16_t*)whh_f;
  const uint16_t* wbf_r = (const uint16_t*)whh_r;
  if (bf && w_dtype == ASR_DT_F32) {
    uint16_t* wb = (uint16_t*)((char*)workspace + fwd_state_bytes(B, H, compute_dtype));
    const long long n = 4LL * H * H;
    hipLaunchKernelGGL(convert_bf16, dim3(ceil_div(n, 256 * 4)), dim3(256), 0, s,
                       (const float*)whh_f, (const float*)whh_r, n, wb);
    ASR_LAUNCH_CHECK();
    wbf_f = wb;
    wbf_r = wb + n;
  }
  if (bf && wbf_r == wbf_f + 4LL * H * H &&
      lstm_fwd_persistent(B, T, H, lens, wbf_f, gx_act, y, cst, (uint16_t*)hbuf, ctr, ybf, s,
                          true)) {
    // one persistent launch for the whole pass
    ASR_CHECK_HIP(hipMemsetAsync(ctr, 0, fwd_ctr_bytes(B), s));
    const int slot = prof_begin_launch(ASR_PROF_LSTM_FWD_SEQ, s, 0.0, ASR_PTAG_LSTM_PERSIST);
    const int rc = lstm_fwd_persistent(B, T, H, lens, wbf_f, gx_act, y, cst, (uint16_t*)hbuf,
                                       ctr, ybf, s, false);
    ASR_REQUIRE(rc == 1, ASR_ERR_HIP, "lstm_forward: persistent launch failed");
    prof_end_launch(ASR_PROF_LSTM_FWD_SEQ, slot, s);
    g_lstm_last_path[0] = 4;
    return ASR_OK;
  }
  g_lstm_last_path[0] = 0;
  ASR_CHECK_HIP(hipMemsetAsync(workspace, 0, fwd_state_bytes(B, H, compute_dtype), s));
  const int nks = H / 32;
  const int fast_ks = (bf && H % 32 == 0) ? (nks <= 4 ? 1 : nks <= 8 ? 2 : nks <= 16 ? 4 :
                                             nks <= 32 ? 8 : 0) : 0;
  for (int st = 0; st < T; ++st) {
    const int slot = prof_begin_launch(ASR_PROF_LSTM_FWD, s);
    if (fast_ks) {
#define ASR_FWD_FAST(KS)                                                                       \
  hipLaunchKernelGGL(lstm_fwd_step_fast<KS>, grid, dim3(256), 0, s, st, B, T, H, lens, wbf_f,  \
                     wbf_r, gx_act, y, cst, (uint16_t*)hbuf)
      switch (fast_ks) {
        case 1: ASR_FWD_FAST(1); break;
        case 2: ASR_FWD_FAST(2); break;
        case 4: ASR_FWD_FAST(4); break;
        default: ASR_FWD_FAST(8); break;
      }
#undef ASR_FWD_FAST
    } else if (bf) {
      hipLaunchKernelGGL((lstm_fwd_step<true, uint16_t, uint16_t>), grid, dim3(256), 0, s, st, B,
                         T, H, lens, wbf_f, wbf_r, gx_act, y, cst, (uint16_t*)hbuf, vec);
    } else {
      hipLaunchKernelGGL((lstm_fwd_step<false, float, float>), grid, dim3(256), 0, s, st, B, T, H,
                         lens, (const float*)whh_f, (const float*)whh_r, gx_act, y, cst,
                         (float*)hbuf, vec);
    }
    ASR_LAUNCH_CHECK();
    prof_end_launch(ASR_PROF_LSTM_FWD, slot, s);
  }
  if (ybf) {  // bf16 copy of y (the persistent path writes it in-kernel)
    const long long n = (long long)B * T * 2 * H;
    hipLaunchKernelGGL(to_bf16, dim3((unsigned)min(4096LL, (n + 255) / 256)), dim3(256), 0, s, y,
                       ybf, n);
    ASR_LAUNCH_CHECK();
  }
  return ASR_OK;
}

static int lstm_backward_impl(const float* dy, const void* whh_f, const void* whh_r,
                              int w_dtype, const int32_t* lens, int B, int T, int H,
                              int compute_dtype, float* act_dg, const float* cst,
                              uint16_t* dgbf, float* dbpart, void* workspace, size_t ws_bytes,
                              void* stream, bool* fused_bias, bool dg_f32 = true) {
  *fused_bias = false;
  ASR_REQUIRE(whh_f && whh_r && lens && act_dg && cst && workspace, ASR_ERR_ARG,
              "lstm_backward: null pointer");
  ASR_REQUIRE(B > 0 && T > 0 && H > 0, ASR_ERR_ARG, "lstm_backward: bad shape");
  ASR_REQUIRE(ws_bytes >= bwd_ws(B, H, compute_dtype), ASR_ERR_WORKSPACE,
              "lstm_backward: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const bool bf = compute_dtype == ASR_DT_BF16;
  if (bf && w_dtype == ASR_DT_F32 &&
      lstm_bwd_xg_launch(B, T, H, lens, (const float*)whh_f, (const float*)whh_r, dy, act_dg, cst,
                         workspace, dgbf, dbpart, s, true, dg_f32) == 1) {
    const int slot = prof_begin_launch(ASR_PROF_LSTM_BWD_SEQ, s, 0.0, ASR_PTAG_LSTM_BWD_XG);
    const int rc = lstm_bwd_xg_launch(B, T, H, lens, (const float*)whh_f, (const float*)whh_r, dy,
                                      act_dg, cst, workspace, dgbf, dbpart, s, false, dg_f32);
    ASR_REQUIRE(rc == 1, ASR_ERR_HIP, "lstm_backward: tagged-granule launch failed");
    prof_end_launch(ASR_PROF_LSTM_BWD_SEQ, slot, s);
    *fused_bias = dbpart != nullptr;
    g_lstm_last_path[1] = 1;
    return ASR_OK;
  }
  if (!bf && w_dtype == ASR_DT_F32 && dg_f32 &&
      lstm_bwd_xg32_launch(B, T, H, lens, (const float*)whh_f, (const float*)whh_r, dy, act_dg, cst,
                           workspace, dbpart, s, true) == 1) {
    const int slot = prof_begin_launch(ASR_PROF_LSTM_BWD_SEQ, s, 0.0, ASR_PTAG_LSTM_BWD_XG);
    const int rc = lstm_bwd_xg32_launch(B, T, H, lens, (const float*)whh_f, (const float*)whh_r, dy,
                                        act_dg, cst, workspace, dbpart, s, false);
    ASR_REQUIRE(rc == 1, ASR_ERR_HIP, "lstm_backward: f32 tagged-granule launch failed");
    prof_end_launch(ASR_PROF_LSTM_BWD_SEQ, slot, s);
    *fused_bias = dbpart != nullptr;
    g_lstm_last_path[1] = 2;
    if (dgbf) {
      const long long n = (long long)B * T * 8 * H;
      hipLaunchKernelGGL(to_bf16, dim3((unsigned)min(4096LL, (n + 255) / 256)), dim3(256), 0, s,
                         act_dg, dgbf, n);
      ASR_LAUNCH_CHECK();
    }
    return ASR_OK;
  }
  const BwdLayout L = bwd_layout(B, H, compute_dtype);
  char* base = (char*)workspace;
  int* ctr = (int*)base;
  void* wt = base + L.wt;
  void* dg = base + L.dg;
  float* dcb = (float*)(base + L.dcb);
  const bool persist = bf && lstm_bwd_persistent(B, T, H, lens, (const uint16_t*)wt, dy, act_dg,
                                                 cst, (uint16_t*)dg, ctr, dgbf, s, true);
  if (persist)
    ASR_CHECK_HIP(hipMemsetAsync(ctr, 0, L.wt, s));
  else
    ASR_CHECK_HIP(hipMemsetAsync(dg, 0, L.total - L.dg, s));
  dim3 tg(ceil_div(H, 32), ceil_div(4 * H, 32), 2);
  if (bf) {
    if (w_dtype == ASR_DT_BF16)
      hipLaunchKernelGGL((transpose_whh<uint16_t, uint16_t>), tg, dim3(256), 0, s,
                         (const uint16_t*)whh_f, (const uint16_t*)whh_r, H, (uint16_t*)wt);
    else
      hipLaunchKernelGGL((transpose_whh<float, uint16_t>), tg, dim3(256), 0, s,
                         (const float*)whh_f, (const float*)whh_r, H, (uint16_t*)wt);
  } else {
    ASR_REQUIRE(w_dtype == ASR_DT_F32, ASR_ERR_ARG, "lstm_backward: f32 compute needs f32 W");
    hipLaunchKernelGGL((transpose_whh<float, float>), tg, dim3(256), 0, s, (const float*)whh_f,
                       (const float*)whh_r, H, (float*)wt);
  }
  ASR_LAUNCH_CHECK();
  if (persist) {  // one persistent launch for the whole pass
    const int slot = prof_begin_launch(ASR_PROF_LSTM_BWD_SEQ, s, 0.0, ASR_PTAG_LSTM_PERSIST);
    const int rc = lstm_bwd_persistent(B, T, H, lens, (const uint16_t*)wt, dy, act_dg, cst,
                                       (uint16_t*)dg, ctr, dgbf, s, false);
    ASR_REQUIRE(rc == 1, ASR_ERR_HIP, "lstm_backward: persistent launch failed");
    prof_end_launch(ASR_PROF_LSTM_BWD_SEQ, slot, s);
    g_lstm_last_path[1] = 4;
    return ASR_OK;
  }
  g_lstm_last_path[1] = 0;
  const int vec = (H % 8 == 0) ? 1 : 0;
  dim3 grid(ceil_div(H, BU), 2, ceil_div(B, MB));
  const int nks = 4 * H / 32;
  const int fast_ks = (bf && H % 32 == 0) ? (nks <= 8 ? 1 : nks <= 16 ? 2 : nks <= 32 ? 4 :
                                             nks <= 64 ? 8 : nks <= 128 ? 16 : 0) : 0;
  const dim3 fgrid(ceil_div(H, BU), 2, ceil_div(B, BMB));
  for (int q = 0; q < T; ++q) {
    const int slot = prof_begin_launch(ASR_PROF_LSTM_BWD, s);
    if (fast_ks) {
#define ASR_BWD_FAST(KS)                                                                       \
  hipLaunchKernelGGL(lstm_bwd_step_fast<KS>, fgrid, dim3(512), 0, s, q, B, T, H, lens,         \
                     (const uint16_t*)wt, dy, act_dg, cst, (uint16_t*)dg, dcb)
      switch (fast_ks) {
        case 1: ASR_BWD_FAST(1); break;
        case 2: ASR_BWD_FAST(2); break;
        case 4: ASR_BWD_FAST(4); break;
        case 8: ASR_BWD_FAST(8); break;
        default: ASR_BWD_FAST(16); break;
      }
#undef ASR_BWD_FAST
    } else if (bf)
      hipLaunchKernelGGL((lstm_bwd_step<true, uint16_t>), grid, dim3(256), 0, s, q, B, T, H, lens,
                         (const uint16_t*)wt, dy, act_dg, cst, (uint16_t*)dg, dcb, vec);
    else
      hipLaunchKernelGGL((lstm_bwd_step<false, float>), grid, dim3(256), 0, s, q, B, T, H, lens,
                         (const float*)wt, dy, act_dg, cst, (float*)dg, dcb, vec);
    ASR_LAUNCH_CHECK();
    prof_end_launch(ASR_PROF_LSTM_BWD, slot, s);
  }
  if (dgbf) {  // bf16 copy of the gate gradients (the persistent path writes it in-kernel)
    const long long n = (long long)B * T * 8 * H;
    hipLaunchKernelGGL(to_bf16, dim3((unsigned)min(4096LL, (n + 255) / 256)), dim3(256), 0, s,
                       act_dg, dgbf, n);
    ASR_LAUNCH_CHECK();
  }
  return ASR_OK;
}

extern "C" int asr_lstm_backward(const float* dy, const void* whh_f, const void* whh_r,
                                 int w_dtype, const int32_t* lens, int B, int T, int H,
                                 int compute_dtype, float* act_dg, const float* cst,
                                 uint16_t* dgbf, void* workspace, size_t ws_bytes,
                                 void* stream) {
  bool fused = false;
  return lstm_backward_impl(dy, whh_f, whh_r, w_dtype, lens, B, T, H, compute_dtype, act_dg, cst,
                            dgbf, nullptr, workspace, ws_bytes, stream, &fused);
}

// asr_lstm_backward plus the bias gradients: db_ih[n] += sum_{b,t} dG[b][t][n] and
// db_hh[n] += the same (both biases feed the same gate pre-activation).  The
// tagged-granule path sums them inside the recurrence (no pass over dG);
// other paths reduce the written dG.
static int lstm_backward_db_impl(const float* dy, const void* whh_f, const void* whh_r,
                                 int w_dtype, const int32_t* lens, int B, int T, int H,
                                 int compute_dtype, float* act_dg, const float* cst,
                                 uint16_t* dgbf, float* db_ih, float* db_hh, void* workspace,
                                 size_t ws_bytes, void* stream, bool dg_f32) {
  ASR_REQUIRE(db_ih, ASR_ERR_ARG, "lstm_backward_db: null bias gradient");
  ASR_REQUIRE(B > 0 && T > 0 && H > 0, ASR_ERR_ARG, "lstm_backward_db: bad shape");
  ASR_REQUIRE(ws_bytes >= bwd_ws_bias(B, H, compute_dtype), ASR_ERR_WORKSPACE,
              "lstm_backward_db: workspace too small");
  float* part = (float*)((char*)workspace + bias_ws_off(B, H, compute_dtype));
  bool fused = false;
  const int rc = lstm_backward_impl(dy, whh_f, whh_r, w_dtype, lens, B, T, H, compute_dtype,
                                    act_dg, cst, dgbf, part, workspace, ws_bytes, stream, &fused,
                                    dg_f32);
  if (rc != ASR_OK) return rc;
  hipStream_t s = (hipStream_t)stream;
  const int N = 8 * H;
  if (fused) {
    hipLaunchKernelGGL(bias_from_partials, dim3(ceil_div(N, 256)), dim3(256), 0, s, part, B, N,
                       db_ih, db_hh);
    ASR_LAUNCH_CHECK();
    return ASR_OK;
  }
  const int M = B * T;
  return asr_colsum_accumulate(act_dg, N, M, N, 1.f, db_ih, db_hh, part,
                               asr_colsum_workspace_bytes(M, N), stream);
}

extern "C" int asr_lstm_backward_db(const float* dy, const void* whh_f, const void* whh_r,
                                    int w_dtype, const int32_t* lens, int B, int T, int H,
                                    int compute_dtype, float* act_dg, const float* cst,
                                    uint16_t* dgbf, float* db_ih, float* db_hh, void* workspace,
                                    size_t ws_bytes, void* stream) {
  return lstm_backward_db_impl(dy, whh_f, whh_r, w_dtype, lens, B, T, H, compute_dtype, act_dg,
                               cst, dgbf, db_ih, db_hh, workspace, ws_bytes, stream, true);
}

// asr_lstm_backward_dgbf reading the packed fp16 gate activations of
// asr_lstm_forward_xh (act_h [B][T][2][H][4]).  Only the tagged-granule
// recurrence reads that layout: ASR_ERR_UNSUPPORTED when it does not take
// this shape (the caller unpacks with asr_lstm_unpack_act_h and runs
// asr_lstm_backward_dgbf).
extern "C" int asr_lstm_backward_dgbf_h(const float* dy, const void* whh_f, const void* whh_r,
                                        int w_dtype, const int32_t* lens, int B, int T, int H,
                                        int compute_dtype, const uint16_t* act_h, const float* cst,
                                        uint16_t* dgbf, float* db_ih, float* db_hh,
                                        void* workspace, size_t ws_bytes, void* stream) {
  ASR_REQUIRE(whh_f && whh_r && lens && act_h && cst && dgbf && db_ih && workspace, ASR_ERR_ARG,
              "lstm_backward_dgbf_h: null pointer");
  ASR_REQUIRE(B > 0 && T > 0 && H > 0, ASR_ERR_ARG, "lstm_backward_dgbf_h: bad shape");
  ASR_REQUIRE(compute_dtype == ASR_DT_BF16 && w_dtype == ASR_DT_F32, ASR_ERR_ARG,
              "lstm_backward_dgbf_h: bf16 compute with f32 W_hh only");
  ASR_REQUIRE(ws_bytes >= bwd_ws_bias(B, H, compute_dtype), ASR_ERR_WORKSPACE,
              "lstm_backward_dgbf_h: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)((char*)workspace + bias_ws_off(B, H, compute_dtype));
  if (lstm_bwd_xg_launch(B, T, H, lens, (const float*)whh_f, (const float*)whh_r, dy, nullptr, cst,
                         workspace, dgbf, part, s, true, false, act_h) != 1)
    return ASR_ERR_UNSUPPORTED;
  const int slot = prof_begin_launch(ASR_PROF_LSTM_BWD_SEQ, s, 0.0, ASR_PTAG_LSTM_BWD_XG);
  const int rc = lstm_bwd_xg_launch(B, T, H, lens, (const float*)whh_f, (const float*)whh_r, dy,
                                    nullptr, cst, workspace, dgbf, part, s, false, false, act_h);
  ASR_REQUIRE(rc == 1, ASR_ERR_HIP, "lstm_backward_dgbf_h: tagged-granule launch failed");
  prof_end_launch(ASR_PROF_LSTM_BWD_SEQ, slot, s);
  g_lstm_last_path[1] = 1;
  hipLaunchKernelGGL(bias_from_partials, dim3(ceil_div(8 * H, 256)), dim3(256), 0, s, part, B,
                     8 * H, db_ih, db_hh);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

// asr_lstm_backward_db for callers that consume only the bf16 gate gradients
// (dgbf, required): the tagged-granule recurrence then skips the f32 dG stores
// (B*T*8H*4 bytes per pass) and act_dg's contents are unspecified on exit.
// ASR_XG_DG_F32=1 keeps the f32 stores (A/B).
extern "C" int asr_lstm_backward_dgbf(const float* dy, const void* whh_f, const void* whh_r,
                                      int w_dtype, const int32_t* lens, int B, int T, int H,
                                      int compute_dtype, float* act_dg, const float* cst,
                                      uint16_t* dgbf, float* db_ih, float* db_hh, void* workspace,
                                      size_t ws_bytes, void* stream) {
  ASR_REQUIRE(dgbf, ASR_ERR_ARG, "lstm_backward_dgbf: null dgbf");
  const char* e = getenv("ASR_XG_DG_F32");
  const bool keep = e && e[0] == '1';
  return lstm_backward_db_impl(dy, whh_f, whh_r, w_dtype, lens, B, T, H, compute_dtype, act_dg,
                               cst, dgbf, db_ih, db_hh, workspace, ws_bytes, stream, keep);
}
