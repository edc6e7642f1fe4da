// Bidirectional GRU recurrence for the encoder (gfx950), replacing the packed
// nn.GRU(bidirectional=True) of models/pytorch_v3/encoders/rnn.py (:173-191
// fast path, :226-233 per-layer path, packing :343-358, :377-390).
//
// torch's GRU, gate order r, z, n (h0 = 0):
//   r = sig(gx_r + W_hr h + b_hr)      gx = x W_ih^T + b_ih  (one GEMM, outside)
//   z = sig(gx_z + W_hz h + b_hz)
//   n = tanh(gx_n + r * (W_hn h + b_hn))
//   h' = (1 - z) n + z h
// b_hh is added here because b_hn sits inside the r product.  Packed-sequence
// behaviour: for t >= len[b] the output and the carried state are 0, so the
// reverse direction starts at each utterance's own last frame.
//
// One launch per time step processes BOTH directions (forward at t = s,
// reverse at t = T-1-s).  Forward work-group: 32 utterances x 4 hidden units
// (16 MFMA columns = 4 gate slots x 4 units, slot 3 empty), its 4 waves split
// K = H on the exact-f32 MFMA and combine through LDS; the cell is fused.  h of
// the previous step is read straight from y (the layer output), so no separate
// state buffer exists.  The saved activations (r, z, n over gx, and
// gh_n = W_hn h + b_hn) feed the backward.
//
// Backward (one launch per step, reverse processing order): work-group =
// 32 utterances x 16 units; the recurrent carry dh_prev = dgh W_hh (K = 3H, a
// transposed W_hh so fragments are contiguous) + dh z of the later step, then
//   dn = dh (1 - z), dz = dh (h_prev - n), dp_n = dn (1 - n^2),
//   dp_r = dp_n gh_n r (1 - r), dp_z = dz z (1 - z)
//   dgx = [dp_r, dp_z, dp_n] (over the activations), dgh = [dp_r, dp_z, dp_n r]
// dW_ih = dgx^T x, dW_hh = dgh^T h_prev, the bias sums and dx = dgx W_ih are
// GEMMs / column sums outside (native_ops.BGRULayerFn).
#include "mfma.h"
#include "prof.h"

namespace asr {
namespace {

constexpr int GFU = 4;    // forward: hidden units per work-group
constexpr int GBU = 16;   // backward: hidden units per work-group
constexpr int GMB = 32;   // utterances per work-group (two 16-row MFMA blocks)

__device__ __forceinline__ float ld0(const float* row, int k, int klim) {
  return (row != nullptr && k < klim) ? row[k] : 0.f;
}

// acc[block] += A[rows][k] * B[k][col] over this wave's k-slice (exact f32 MFMA)
__device__ __forceinline__ void wave_dot_f32(const float* a0, const float* a1, const float* bcol,
                                             int K, int wave, f32x4& acc0, f32x4& acc1) {
  const int lane = threadIdx.x & 63;
  for (int k0 = wave * 4; k0 < K; k0 += 16) {
    const int k = k0 + (lane >> 4);
    const float bv = ld0(bcol, k, K);
    acc0 = mfma_f32(ld0(a0, k, K), bv, acc0);
    acc1 = mfma_f32(ld0(a1, k, K), bv, acc1);
  }
}

// grid = (ceil(H / GFU), 2, ceil(B / GMB)), block 256
__global__ void __launch_bounds__(256) gru_fwd_step(
    int s, int B, int T, int H, const int32_t* __restrict__ lens, const float* __restrict__ whh,
    const float* __restrict__ bhh, float* __restrict__ gx_act, float* __restrict__ y,
    float* __restrict__ ghn) {
  __shared__ float part[4][GMB][16];
  const int dir = blockIdx.y;
  const int u0 = blockIdx.x * GFU, b0 = blockIdx.z * GMB;
  const int t = dir == 0 ? s : T - 1 - s;
  const int tp = dir == 0 ? t - 1 : t + 1;   // the previous step's frame (valid when s > 0)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long H2 = 2LL * H, H6 = 6LL * H;
  const float* W = whh + (long long)dir * 3 * H * H;
  const int ra = b0 + (lane & 15), rb = ra + 16;
  const float* a0 = (s > 0 && ra < B) ? y + ((long long)ra * T + tp) * H2 + (long long)dir * H : nullptr;
  const float* a1 = (s > 0 && rb < B) ? y + ((long long)rb * T + tp) * H2 + (long long)dir * H : nullptr;
  const int n = lane & 15, g = n >> 2, u = u0 + (n & 3);
  const float* bcol = (g < 3 && u < H) ? W + (long long)(g * H + u) * H : nullptr;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if (s > 0) wave_dot_f32(a0, a1, bcol, H, wave, acc0, acc1);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    part[wave][4 * (lane >> 4) + r][n] = acc0[r];
    part[wave][16 + 4 * (lane >> 4) + r][n] = acc1[r];
  }
  __syncthreads();
  if (threadIdx.x >= GMB * GFU) return;
  const int row = threadIdx.x >> 2, uu = threadIdx.x & 3;
  const int b = b0 + row, j = u0 + uu;
  if (b >= B || j >= H) return;
  float hg[3];
#pragma unroll
  for (int q = 0; q < 3; ++q)
    hg[q] = part[0][row][4 * q + uu] + part[1][row][4 * q + uu] + part[2][row][4 * q + uu] +
            part[3][row][4 * q + uu];
  const long long gb = ((long long)b * T + t) * H6 + (long long)dir * 3 * H + j;
  const long long si = ((long long)b * T + t) * H2 + (long long)dir * H + j;
  const float* bh = bhh + (long long)dir * 3 * H;
  const float hprev = s > 0 ? y[si + (long long)(tp - t) * H2] : 0.f;
  float r = sigmoidf_(gx_act[gb] + hg[0] + bh[j]);
  float z = sigmoidf_(gx_act[gb + H] + hg[1] + bh[H + j]);
  float gn = hg[2] + bh[2 * H + j];
  float nn = tanhf_(gx_act[gb + 2 * H] + r * gn);
  float h = (1.f - z) * nn + z * hprev;
  if (t >= lens[b]) { r = z = gn = nn = h = 0.f; }
  y[si] = h;
  ghn[si] = gn;
  gx_act[gb] = r;
  gx_act[gb + H] = z;
  gx_act[gb + 2 * H] = nn;
}

// wt[dir][j][k] = whh[dir][k][j]  (k < 3H, j < H); grid (ceil(H/32), ceil(3H/32), 2)
__global__ void gru_transpose_whh(const float* __restrict__ whh, int H, float* __restrict__ wt) {
  __shared__ float tile[32][33];
  const int dir = blockIdx.z;
  const int R = 3 * H, C = H;
  const float* w = whh + (long long)dir * R * C;
  float* o = wt + (long long)dir * R * C;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? w[(long long)r * C + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (c < C && r < R) o[(long long)c * R + r] = tile[tx][i];
  }
}

// grid = (ceil(H / GBU), 2, ceil(B / GMB)), block 256.  dhz: [2 parity][B][2H].
__global__ void __launch_bounds__(256) gru_bwd_step(
    int q, int B, int T, int H, const int32_t* __restrict__ lens, const float* __restrict__ wt,
    const float* __restrict__ dy, float* __restrict__ act, const float* __restrict__ ghn,
    const float* __restrict__ y, float* __restrict__ dgh, float* __restrict__ dhz) {
  __shared__ float part[4][GMB][16];
  const int dir = blockIdx.y;
  const int u0 = blockIdx.x * GBU, b0 = blockIdx.z * GMB;
  const int t = dir == 0 ? T - 1 - q : q;
  const int tn = dir == 0 ? t + 1 : t - 1;   // frame of the previous processing step (q > 0)
  const int tp = dir == 0 ? t - 1 : t + 1;   // h_prev's frame in the forward recursion
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long H2 = 2LL * H, H6 = 6LL * H;
  const int K = 3 * H;
  const int ra = b0 + (lane & 15), rb = ra + 16;
  const float* a0 = (q > 0 && ra < B) ? dgh + ((long long)ra * T + tn) * H6 + (long long)dir * K : nullptr;
  const float* a1 = (q > 0 && rb < B) ? dgh + ((long long)rb * T + tn) * H6 + (long long)dir * K : nullptr;
  const int n = lane & 15, u = u0 + n;
  const float* bcol = u < H ? wt + ((long long)dir * H + u) * K : nullptr;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if (q > 0) wave_dot_f32(a0, a1, bcol, K, wave, acc0, acc1);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    part[wave][4 * (lane >> 4) + r][n] = acc0[r];
    part[wave][16 + 4 * (lane >> 4) + r][n] = acc1[r];
  }
  __syncthreads();
  const float* dhz_in = dhz + (long long)((q + 1) & 1) * B * H2;
  float* dhz_out = dhz + (long long)(q & 1) * B * H2;
  for (int e = threadIdx.x; e < GMB * GBU; e += 256) {
    const int row = e >> 4, uu = e & 15;
    const int b = b0 + row, j = u0 + uu;
    if (b >= B || j >= H) continue;
    const long long si = ((long long)b * T + t) * H2 + (long long)dir * H + j;
    const long long gb = ((long long)b * T + t) * H6 + (long long)dir * K + j;
    float dh = dy ? dy[si] : 0.f;
    if (q > 0)
      dh += part[0][row][uu] + part[1][row][uu] + part[2][row][uu] + part[3][row][uu] +
            dhz_in[(long long)b * H2 + (long long)dir * H + j];
    float dpr = 0.f, dpz = 0.f, dpn = 0.f, r = 0.f, z = 0.f;
    if (t < lens[b]) {
      r = act[gb];
      z = act[gb + H];
      const float nn = act[gb + 2 * H];
      const float gn = ghn[si];
      const float hprev = (tp >= 0 && tp < T) ? y[si + (long long)(tp - t) * H2] : 0.f;
      const float dn = dh * (1.f - z);
      const float dz = dh * (hprev - nn);
      dpn = dn * (1.f - nn * nn);
      dpr = dpn * gn * r * (1.f - r);
      dpz = dz * z * (1.f - z);
    } else {
      dh = 0.f;
    }
    act[gb] = dpr;
    act[gb + H] = dpz;
    act[gb + 2 * H] = dpn;
    dgh[gb] = dpr;
    dgh[gb + H] = dpz;
    dgh[gb + 2 * H] = dpn * r;
    dhz_out[(long long)b * H2 + (long long)dir * H + j] = dh * z;
  }
}

size_t gru_dhz_bytes(int B, int H) { return (((size_t)2 * B * 2 * H * 4) + 255) / 256 * 256; }

// nn.GRUCell nonlinearity (the decoder cell, rnn_decoder.py:91-95):
// gi = x W_ih^T + b_ih, gh = h W_hh^T + b_hh [B][3D] (GEMMs outside).
__global__ void gru_cell_fwd(const float* __restrict__ gi, const float* __restrict__ gh,
                             const float* __restrict__ h, int B, int D, float* __restrict__ act,
                             float* __restrict__ hout) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)B * D) return;
  const long long b = e / D, j = e - b * D;
  const long long g = b * 3 * D + j;
  const float r = sigmoidf_(gi[g] + gh[g]);
  const float z = sigmoidf_(gi[g + D] + gh[g + D]);
  const float n = tanhf_(gi[g + 2 * D] + r * gh[g + 2 * D]);
  hout[e] = (1.f - z) * n + z * h[e];
  act[g] = r;
  act[g + D] = z;
  act[g + 2 * D] = n;
}

__global__ void gru_cell_bwd(const float* __restrict__ act, const float* __restrict__ gh,
                             const float* __restrict__ h, const float* __restrict__ dh, int B,
                             int D, float* __restrict__ dgi, float* __restrict__ dgh,
                             float* __restrict__ dh_prev) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)B * D) return;
  const long long b = e / D, j = e - b * D;
  const long long g = b * 3 * D + j;
  const float r = act[g], z = act[g + D], n = act[g + 2 * D];
  const float d = dh[e];
  const float dn = d * (1.f - z);
  const float dz = d * (h[e] - n);
  const float dpn = dn * (1.f - n * n);
  const float dpr = dpn * gh[g + 2 * D] * r * (1.f - r);
  const float dpz = dz * z * (1.f - z);
  dgi[g] = dpr;
  dgi[g + D] = dpz;
  dgi[g + 2 * D] = dpn;
  dgh[g] = dpr;
  dgh[g + D] = dpz;
  dgh[g + 2 * D] = dpn * r;
  dh_prev[e] = d * z;
}

}  // namespace
}  // namespace asr

using namespace asr;

extern "C" size_t asr_gru_workspace_bytes(int B, int H) {
  if (B <= 0 || H <= 0) return 0;
  return gru_dhz_bytes(B, H) + (size_t)2 * 3 * H * H * 4;
}

extern "C" int asr_gru_forward(float* gx_act, const float* whh, const float* bhh,
                               const int32_t* lens, int B, int T, int H, float* y, float* ghn,
                               void* stream) {
  ASR_REQUIRE(gx_act && whh && bhh && lens && y && ghn, ASR_ERR_ARG, "gru_forward: null pointer");
  ASR_REQUIRE(B > 0 && T > 0 && H > 0, ASR_ERR_ARG, "gru_forward: bad shape");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(ceil_div(H, GFU), 2, ceil_div(B, GMB));
  for (int s = 0; s < T; ++s) {
    hipLaunchKernelGGL(gru_fwd_step, grid, dim3(256), 0, st, s, B, T, H, lens, whh, bhh, gx_act,
                       y, ghn);
    ASR_LAUNCH_CHECK();
  }
  return ASR_OK;
}

extern "C" int asr_gru_backward(const float* dy, const float* whh, const int32_t* lens, int B,
                                int T, int H, float* act_dgx, const float* ghn, const float* y,
                                float* dgh, void* workspace, size_t ws_bytes, void* stream) {
  ASR_REQUIRE(whh && lens && act_dgx && ghn && y && dgh && workspace, ASR_ERR_ARG,
              "gru_backward: null pointer");
  ASR_REQUIRE(B > 0 && T > 0 && H > 0, ASR_ERR_ARG, "gru_backward: bad shape");
  ASR_REQUIRE(ws_bytes >= asr_gru_workspace_bytes(B, H), ASR_ERR_WORKSPACE,
              "gru_backward: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* dhz = (float*)workspace;
  float* wt = (float*)((char*)workspace + gru_dhz_bytes(B, H));
  hipLaunchKernelGGL(gru_transpose_whh, dim3(ceil_div(H, 32), ceil_div(3 * H, 32), 2), dim3(256),
                     0, st, whh, H, wt);
  ASR_LAUNCH_CHECK();
  const dim3 grid(ceil_div(H, GBU), 2, ceil_div(B, GMB));
  for (int q = 0; q < T; ++q) {
    hipLaunchKernelGGL(gru_bwd_step, grid, dim3(256), 0, st, q, B, T, H, lens, wt, dy, act_dgx,
                       ghn, y, dgh, dhz);
    ASR_LAUNCH_CHECK();
  }
  return ASR_OK;
}

extern "C" int asr_gru_cell_forward(const float* gi, const float* gh, const float* h, int B, int D,
                                    float* act, float* hout, void* stream) {
  ASR_REQUIRE(gi && gh && h && act && hout && B > 0 && D > 0, ASR_ERR_ARG, "gru_cell: bad args");
  const long long n = (long long)B * D;
  hipLaunchKernelGGL(gru_cell_fwd, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, gi,
                     gh, h, B, D, act, hout);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_gru_cell_backward(const float* act, const float* gh, const float* h,
                                     const float* dh, int B, int D, float* dgi, float* dgh,
                                     float* dh_prev, void* stream) {
  ASR_REQUIRE(act && gh && h && dh && dgi && dgh && dh_prev && B > 0 && D > 0, ASR_ERR_ARG,
              "gru_cell: bad args");
  const long long n = (long long)B * D;
  hipLaunchKernelGGL(gru_cell_bwd, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, act,
                     gh, h, dh, B, D, dgi, dgh, dh_prev);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}
