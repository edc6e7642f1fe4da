// Persistent (one launch per layer pass) bidirectional LSTM recurrence, bf16
// MFMA, gfx950.  Same semantics as the per-step kernels in lstm.hip (nn.LSTM
// bidirectional with pack/pad behaviour, models/pytorch_v3/encoders/rnn.py
// :166-172, :218-224, :343-390), without T kernel boundaries per pass.
//
// Layout: every work-group owns a fixed tile of (16 utterances x U hidden units)
// of one direction for the whole sequence.  Its slice of W_hh lives in VGPRs
// (MFMA B fragments, loaded once), its cell states live in registers, and only
// the recurrent vector crosses work-groups each step:
//   forward : h_t   [16 rows][H]  bf16, published 16 B per (row, 8 units)
//   backward: dg_t  [16 rows][4H] bf16 (gate gradients, K of dh = dg W_hh)
// Hand-off (cdna_hip_programming.md §6 Guideline 16, valid-form row 1 of
// MI355X_MICROARCH.md § visibility): payload stored write-through (sc1) by one
// wave, that wave's s_waitcnt vmcnt(0), then one lane's agent-scope atomic add
// on the (direction, row-group) counter; consumers poll the counter relaxed
// (sc1) from one lane, join a workgroup barrier, and read the payload with sc1
// buffer loads only.  Counters are monotonic within a call (step s waits for
// s * units_groups arrivals) and zeroed by a memset before every launch; the
// exchange is ping-pong by step parity.  One work-group per CU is enforced
// with a large dynamic LDS request, and the host launches this path only when
// the whole grid is co-resident (occupancy query); spins are bounded and set
// g_persist_status + an abort word instead of hanging.
#include "mfma.h"
#include "prof.h"

namespace asr {

__device__ int g_persist_status;  // bit 0: a bounded spin gave up (results invalid)

namespace {

constexpr int PRB = 16;          // utterances per work-group (one MFMA row block)
constexpr int PFU = 8;           // forward: hidden units per work-group (32 gate columns)
constexpr int PBU = 16;          // backward: hidden units per work-group
constexpr int CTR_STRIDE = 64;   // ints between polled words (own 256-B line each)
constexpr unsigned SPIN_LIMIT = 1u << 18;
constexpr size_t PIN_LDS = 96 * 1024;   // forward: > 80 KB dynamic LDS -> one work-group per CU
constexpr size_t PIN_LDS_B = 140 * 1024; // backward: also leaves no room for a GEMM work-group
                                         // (20 KB) running beside it on another stream

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((address_space(1))) int gint;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)bytes, 0x00020000);
}

// One lane: wait until *ctr >= target.  false = gave up (abort word set / timeout).
__device__ __forceinline__ bool wait_count(int* ctr, int target, int* abort_w) {
  gint* c = (gint*)ctr;
  gint* a = (gint*)abort_w;
  for (unsigned spins = 0;; ++spins) {
    if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    if (__hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
    if (spins >= SPIN_LIMIT) {
      __hip_atomic_store(a, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicOr(&g_persist_status, 1);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

__device__ __forceinline__ void arrive(int* ctr) {
  __hip_atomic_fetch_add((gint*)ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bf16x8 as_frag(const u32x4& v) { return __builtin_bit_cast(bf16x8, v); }

// ---------------------------------------------------------------------------
// forward.  grid = NUG * 2 * NRG work-groups (NUG = H/8, NRG = ceil(B/16)),
// block 256 = 4 waves splitting K = H; wave w takes k-steps w, w+4, ...
// hx: [2 parity][2 dir][NRG*16][H] bf16; ctr: abort word at 0, counters at
// (1 + dir*NRG + rg) * CTR_STRIDE.
// ---------------------------------------------------------------------------
template <int KSW>
__global__ void __launch_bounds__(256) lstm_fwd_persist(
    int B, int T, int H, const int32_t* __restrict__ lens, const uint16_t* __restrict__ wbf,
    float* __restrict__ gx_act, float* __restrict__ y, float* __restrict__ cst, uint16_t* hx,
    int* ctr, int pubw, uint16_t* __restrict__ ybf) {
  __shared__ float part[4][PRB][2 * PRB];
  __shared__ __attribute__((aligned(16))) uint16_t hrow[PRB][PFU];
  __shared__ int s_ok;
  const int NUG = H / PFU, NRG = (B + PRB - 1) / PRB, Bp = NRG * PRB;
  const int ug = blockIdx.x % NUG, rest = blockIdx.x / NUG;
  const int dir = rest & 1, rg = rest >> 1;
  const int u0 = ug * PFU, b0 = rg * PRB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nks = H >> 5;
  int* my_ctr = ctr + (1 + dir * NRG + rg) * CTR_STRIDE;

  // this wave's W_hh fragments: col = cb*16 + (lane&15) -> gate col>>3, unit u0 + (col&7)
  bf16x8 wf[2][KSW];
  {
    const uint16_t* W = wbf + (long long)dir * 4 * H * H;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int col = cb * 16 + (lane & 15);
      const uint16_t* wr = W + (long long)((col >> 3) * H + u0 + (col & 7)) * H + 8 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < KSW; ++i) wf[cb][i] = load_bf16x8(wr + min(wave + 4 * i, nks - 1) * 32);
    }
  }
  // owned cell (threads 0..127): row r = tid>>3, unit uu = tid&7
  const int r = tid >> 3, uu = tid & 7;
  const int b = b0 + r, j = u0 + uu;
  const bool own = tid < PRB * PFU && b < B;
  const int len = own ? lens[b] : 0;
  float c = 0.f;

  const unsigned hx_bytes = (unsigned)(4ull * Bp * H * 2);
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(hx, hx_bytes);
  const long long H8 = 8LL * H;

  for (int s = 0; s < T; ++s) {
    const int t = dir == 0 ? s : T - 1 - s;
    float gxv[4] = {0.f, 0.f, 0.f, 0.f};
    const long long gbase = ((long long)(own ? b : 0) * T + t) * H8 + (long long)dir * 4 * H + j;
    if (own) {
#pragma unroll
      for (int q = 0; q < 4; ++q) gxv[q] = gx_act[gbase + (long long)q * H];
    }
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    if (s > 0) {
      if (tid == 0) s_ok = wait_count(my_ctr, s * NUG, ctr);
      __syncthreads();
      if (!s_ok) return;
      const int par = (s - 1) & 1;
      const unsigned rowoff =
          (unsigned)((((par * 2 + dir) * Bp) + b0 + (lane & 15)) * (long long)H * 2);
      u32x4 fa[KSW];
#pragma unroll
      for (int i = 0; i < KSW; ++i) {
        const int kc = min(wave + 4 * i, nks - 1) * 32 + 8 * (lane >> 4);
        fa[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, rowoff + kc * 2, 0, 16);
      }
#pragma unroll
      for (int i = 0; i < KSW; ++i) {
        if (wave + 4 * i < nks) {
          acc0 = mfma_bf16(as_frag(fa[i]), wf[0][i], acc0);
          acc1 = mfma_bf16(as_frag(fa[i]), wf[1][i], acc1);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      part[wave][4 * (lane >> 4) + q][lane & 15] = acc0[q];
      part[wave][4 * (lane >> 4) + q][16 + (lane & 15)] = acc1[q];
    }
    __syncthreads();
    if (tid < PRB * PFU) {
      uint16_t hb = 0;
      if (own) {
        float pre[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int col = q * PFU + uu;
          pre[q] = part[0][r][col] + part[1][r][col] + part[2][r][col] + part[3][r][col] + gxv[q];
        }
        const bool active = t < len;
        const float ig = sigmoidf_(pre[0]), fg = sigmoidf_(pre[1]);
        const float gg = tanhf_(pre[2]), og = sigmoidf_(pre[3]);
        float cn = fg * c + ig * gg;
        float h = og * tanhf_(cn);
        if (!active) { cn = 0.f; h = 0.f; }
        c = cn;
        const long long sidx = ((long long)b * T + t) * 2 * H + (long long)dir * H + j;
        y[sidx] = h;
        cst[sidx] = cn;
        gx_act[gbase] = active ? ig : 0.f;
        gx_act[gbase + H] = active ? fg : 0.f;
        gx_act[gbase + 2 * H] = active ? gg : 0.f;
        gx_act[gbase + 3 * H] = active ? og : 0.f;
        hb = f2bf(h);
      }
      hrow[r][uu] = hb;
    }
    __syncthreads();
    // publish h_t: 16 rows x 16 B, write-through; drain; one arrival (by wave
    // pubw: 0 by default, see pub_last_wave)
    if (wave == pubw) {
      if (lane < PRB) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(&hrow[lane][0]);
        const unsigned off =
            (unsigned)(((((s & 1) * 2 + dir) * Bp + b0 + lane) * (long long)H + u0) * 2);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) arrive(my_ctr);
      // bf16 copy of y for the weight-gradient GEMMs (after the arrival: off the
      // hand-off's critical path)
      if (ybf && lane < PRB && b0 + lane < B) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(&hrow[lane][0]);
        *reinterpret_cast<u32x4*>(ybf + ((long long)(b0 + lane) * T + t) * 2 * H + dir * H + u0) = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward.  grid = NUG * 2 * NRG (NUG = H/16), block 512 = 8 waves splitting
// K = 4H; wave w takes k-steps w, w+8, ...  Processing step q handles the
// forward direction at t = T-1-q and the reverse direction at t = q.
// wt: [2][H][4H] (W_hh^T, bf16); dgx: [2 parity][2 dir][NRG*16][4H] bf16.
// ---------------------------------------------------------------------------
template <int KSW>
__global__ void __launch_bounds__(512) lstm_bwd_persist(
    int B, int T, int H, const int32_t* __restrict__ lens, const uint16_t* __restrict__ wt,
    const float* __restrict__ dy, float* __restrict__ act_dg, const float* __restrict__ cst,
    uint16_t* dgx, int* ctr, int pubw, uint16_t* __restrict__ dgbf) {
  __shared__ float part[8][PRB][PBU];
  __shared__ __attribute__((aligned(16))) uint16_t dgrow[PRB][4][PBU];
  __shared__ int s_ok;
  const int NUG = H / PBU, NRG = (B + PRB - 1) / PRB, Bp = NRG * PRB;
  const int ug = blockIdx.x % NUG, rest = blockIdx.x / NUG;
  const int dir = rest & 1, rg = rest >> 1;
  const int u0 = ug * PBU, b0 = rg * PRB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H4 = 4 * H, nks = H4 >> 5;
  int* my_ctr = ctr + (1 + dir * NRG + rg) * CTR_STRIDE;

  bf16x8 wf[KSW];
  {
    const uint16_t* wr = wt + (long long)dir * H * H4 + (long long)(u0 + (lane & 15)) * H4 +
                         8 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < KSW; ++i) wf[i] = load_bf16x8(wr + min(wave + 8 * i, nks - 1) * 32);
  }
  // owned cell (threads 0..255): row r = tid>>4, unit uu = tid&15
  const int r = tid >> 4, uu = tid & 15;
  const int b = b0 + r, j = u0 + uu;
  const bool own = tid < PRB * PBU && b < B;
  const int len = own ? lens[b] : 0;
  float dc = 0.f;

  const unsigned dg_bytes = (unsigned)(4ull * Bp * H4 * 2);
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(dgx, dg_bytes);

  for (int q = 0; q < T; ++q) {
    const int t = dir == 0 ? T - 1 - q : q;
    const int tp = dir == 0 ? t - 1 : t + 1;
    const long long gbase = ((long long)(own ? b : 0) * T + t) * 8 * H + (long long)dir * H4 + j;
    const long long sidx = ((long long)(own ? b : 0) * T + t) * 2 * H + (long long)dir * H + j;
    float av[4] = {0.f, 0.f, 0.f, 0.f}, cc = 0.f, cp = 0.f, dyv = 0.f;
    if (own) {
#pragma unroll
      for (int k = 0; k < 4; ++k) av[k] = act_dg[gbase + (long long)k * H];
      cc = cst[sidx];
      cp = (tp >= 0 && tp < T) ? cst[sidx + (long long)(tp - t) * 2 * H] : 0.f;
      dyv = dy ? dy[sidx] : 0.f;
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (q > 0) {
      if (tid == 0) s_ok = wait_count(my_ctr, q * NUG, ctr);
      __syncthreads();
      if (!s_ok) return;
      const int par = (q - 1) & 1;
      const unsigned rowoff =
          (unsigned)((((par * 2 + dir) * Bp) + b0 + (lane & 15)) * (long long)H4 * 2);
      u32x4 fa[KSW];
#pragma unroll
      for (int i = 0; i < KSW; ++i) {
        const int kc = min(wave + 8 * i, nks - 1) * 32 + 8 * (lane >> 4);
        fa[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, rowoff + kc * 2, 0, 16);
      }
#pragma unroll
      for (int i = 0; i < KSW; ++i)
        if (wave + 8 * i < nks) acc = mfma_bf16(as_frag(fa[i]), wf[i], acc);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) part[wave][4 * (lane >> 4) + k][lane & 15] = acc[k];
    __syncthreads();
    if (tid < PRB * PBU) {
      float d_i = 0.f, d_f = 0.f, d_g = 0.f, d_o = 0.f;
      if (own) {
        if (t < len) {
          float dh = dyv;
#pragma unroll
          for (int w = 0; w < 8; ++w) dh += part[w][r][uu];
          const float ig = av[0], fg = av[1], gg = av[2], og = av[3];
          const float tc = tanhf_(cc);
          const float dcell = dc + dh * og * (1.f - tc * tc);
          d_i = dcell * gg * ig * (1.f - ig);
          d_f = dcell * cp * fg * (1.f - fg);
          d_g = dcell * ig * (1.f - gg * gg);
          d_o = dh * tc * og * (1.f - og);
          dc = dcell * fg;
        } else {
          dc = 0.f;
        }
        act_dg[gbase] = d_i;
        act_dg[gbase + H] = d_f;
        act_dg[gbase + 2 * H] = d_g;
        act_dg[gbase + 3 * H] = d_o;
      }
      dgrow[r][0][uu] = f2bf(d_i);
      dgrow[r][1][uu] = f2bf(d_f);
      dgrow[r][2][uu] = f2bf(d_g);
      dgrow[r][3][uu] = f2bf(d_o);
    }
    __syncthreads();
    // publish dg_t: 16 rows x 4 gates x 32 B = 128 x 16 B, write-through; drain;
    // one arrival (by wave pubw)
    if (wave == pubw) {
      const unsigned rowbase = (unsigned)((((q & 1) * 2 + dir) * Bp + b0) * (long long)H4 * 2);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int e = lane + 64 * p;             // 0..127
        const int rr = e >> 3, g = (e >> 1) & 3, half = e & 1;
        const u32x4 v = *reinterpret_cast<const u32x4*>(&dgrow[rr][g][half * 8]);
        const unsigned off = rowbase + (unsigned)((rr * H4 + g * H + u0 + half * 8) * 2);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) arrive(my_ctr);
      if (dgbf) {  // bf16 gate gradients [B][T][8H] for the weight-gradient GEMMs
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int e = lane + 64 * p;
          const int rr = e >> 3, g = (e >> 1) & 3, half = e & 1;
          if (b0 + rr < B) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(&dgrow[rr][g][half * 8]);
            *reinterpret_cast<u32x4*>(dgbf + ((long long)(b0 + rr) * T + t) * 8 * H +
                                      dir * H4 + g * H + u0 + half * 8) = v;
          }
        }
      }
    }
  }
}

int g_num_cus = 0;

int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) !=
        hipSuccess)
      g_num_cus = 0;
  }
  return g_num_cus;
}

// ASR_LSTM_PERSIST=0 selects the per-step kernels (read per call: A/B tests).
bool persist_enabled() {
  const char* e = getenv("ASR_LSTM_PERSIST");
  return !(e && e[0] == '0');
}

// Which wave publishes the hand-off payload: wave 0 (owns cells; default, it
// measured 4 % faster per pass in an interleaved A/B) or, with
// ASR_LSTM_PUBW=1, the last wave (owns no cells).
bool pub_last_wave() {
  const char* e = getenv("ASR_LSTM_PUBW");
  return e && e[0] == '1';
}

template <typename K>
bool fits(K kernel, int threads, int grid, size_t lds) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds) !=
      hipSuccess)
    return false;
  return per_cu >= 1 && grid <= num_cus();  // one work-group per CU (PIN_LDS)
}

}  // namespace

size_t persist_ctr_bytes(int B) {
  const int NRG = (B + PRB - 1) / PRB;
  return (size_t)(1 + 2 * NRG) * CTR_STRIDE * sizeof(int);
}

int persist_rows(int B) { return ((B + PRB - 1) / PRB) * PRB; }

// dry: 1 if this shape / device can take the persistent path (else the caller
// uses the per-step kernels), launching nothing.  Otherwise launches and
// returns 1, or 0 / -1 if not eligible / the launch failed.
int lstm_fwd_persistent(int B, int T, int H, const int32_t* lens, const uint16_t* wbf,
                        float* gx_act, float* y, float* cst, uint16_t* hx, int* ctr,
                        uint16_t* ybf, hipStream_t s, bool dry) {
  if (!persist_enabled() || H % 32 != 0) return 0;
  const int nks = H / 32;
  const int ksw = (nks + 3) / 4;
  const int grid = (H / PFU) * 2 * ((B + PRB - 1) / PRB);
  const int pw = pub_last_wave() ? 3 : 0;
#define ASR_FWD_P(KS)                                                                          \
  do {                                                                                         \
    if (!fits(lstm_fwd_persist<KS>, 256, grid, PIN_LDS)) return 0;                                      \
    if (dry) return 1;                                                                         \
    hipLaunchKernelGGL(lstm_fwd_persist<KS>, dim3(grid), dim3(256), PIN_LDS, s, B, T, H, lens, \
                       wbf, gx_act, y, cst, hx, ctr, pw, ybf);                                  \
  } while (0)
  if (ksw <= 1) ASR_FWD_P(1);
  else if (ksw <= 2) ASR_FWD_P(2);
  else if (ksw <= 4) ASR_FWD_P(4);
  else if (ksw <= 8) ASR_FWD_P(8);
  else return 0;
#undef ASR_FWD_P
  return hipGetLastError() == hipSuccess ? 1 : -1;
}

int lstm_bwd_persistent(int B, int T, int H, const int32_t* lens, const uint16_t* wt,
                        const float* dy, float* act_dg, const float* cst, uint16_t* dgx, int* ctr,
                        uint16_t* dgbf, hipStream_t s, bool dry) {
  if (!persist_enabled() || H % 32 != 0) return 0;
  const int nks = H / 8;
  const int ksw = (nks + 7) / 8;
  const int grid = (H / PBU) * 2 * ((B + PRB - 1) / PRB);
  const int pw = pub_last_wave() ? 7 : 0;
#define ASR_BWD_P(KS)                                                                          \
  do {                                                                                         \
    if (!fits(lstm_bwd_persist<KS>, 512, grid, PIN_LDS_B)) return 0;                                      \
    if (dry) return 1;                                                                         \
    hipLaunchKernelGGL(lstm_bwd_persist<KS>, dim3(grid), dim3(512), PIN_LDS_B, s, B, T, H, lens, \
                       wt, dy, act_dg, cst, dgx, ctr, pw, dgbf);                                  \
  } while (0)
  if (ksw <= 2) ASR_BWD_P(2);
  else if (ksw <= 4) ASR_BWD_P(4);
  else if (ksw <= 8) ASR_BWD_P(8);
  else if (ksw <= 16) ASR_BWD_P(16);
  else return 0;
#undef ASR_BWD_P
  return hipGetLastError() == hipSuccess ? 1 : -1;
}

// Device address of the counter form's status word (the persistent decoder
// pass reports its give-ups there too).
int* lstm_persist_status_word() {
  void* p = nullptr;
  return hipGetSymbolAddress(&p, HIP_SYMBOL(g_persist_status)) == hipSuccess ? (int*)p : nullptr;
}

}  // namespace asr

namespace asr {
int lstm_xg_status(int* status, int clear, hipStream_t s);  // lstm_xg.hip
int* lstm_xg_status_word();                                  // lstm_xg.hip
}

using namespace asr;

extern "C" int asr_lstm_persist_status(int* status, int clear, void* stream) {
  ASR_REQUIRE(status, ASR_ERR_ARG, "persist_status: null pointer");
  hipStream_t s = (hipStream_t)stream;
  ASR_CHECK_HIP(hipMemcpyFromSymbolAsync(status, HIP_SYMBOL(g_persist_status), sizeof(int), 0,
                                         hipMemcpyDeviceToHost, s));
  ASR_CHECK_HIP(hipStreamSynchronize(s));
  if (clear) {
    const int zero = 0;
    ASR_CHECK_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_persist_status), &zero, sizeof(int), 0,
                                         hipMemcpyHostToDevice, s));
    ASR_CHECK_HIP(hipStreamSynchronize(s));
  }
  ASR_REQUIRE(lstm_xg_status(status, clear, s) == 0, ASR_ERR_HIP,
              "persist_status: tagged-granule status read failed");
  return ASR_OK;
}

// Stream-ordered, sync-free form for the training step: dst[0] = the counter
// form's status word, dst[1] = the tagged-granule form's, copied device to
// device after the recurrences that precede it on the stream; clear = 1 then
// zeroes both words (also stream-ordered).  dst feeds asr_optim_step_guarded
// (directly, or after a MAX all-reduce over the data-parallel ranks).
namespace asr {
namespace {
// both status words copied (and cleared) by one thread: one launch where two
// copies and two fills were four (each a dispatch on the step's stream)
__global__ void status_gather_k(int* dst, int* pp, int* xg, int clear) {
  if (threadIdx.x == 0) {
    const int a = __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int b = __hip_atomic_load(xg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    dst[0] = a;
    dst[1] = b;
    if (clear) {
      __hip_atomic_store(pp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(xg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
}  // namespace
}  // namespace asr

extern "C" int asr_lstm_status_gather(int* dst, int clear, void* stream) {
  ASR_REQUIRE(dst, ASR_ERR_ARG, "status_gather: null pointer");
  hipStream_t s = (hipStream_t)stream;
  int* xg = lstm_xg_status_word();
  static void* pp = nullptr;
  ASR_REQUIRE(xg, ASR_ERR_HIP, "status_gather: no tagged-granule status word");
  if (!pp) ASR_CHECK_HIP(hipGetSymbolAddress(&pp, HIP_SYMBOL(g_persist_status)));
  hipLaunchKernelGGL(asr::status_gather_k, dim3(1), dim3(64), 0, s, dst, (int*)pp, xg, clear);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

// Test hook: mark the tagged-granule recurrence as having given up (what a
// bounded spin that ran out does), stream-ordered.
extern "C" int asr_lstm_status_inject(int bits, void* stream) {
  int* xg = lstm_xg_status_word();
  ASR_REQUIRE(xg, ASR_ERR_HIP, "status_inject: no tagged-granule status word");
  ASR_CHECK_HIP(hipMemsetAsync(xg, bits & 0xff, 1, (hipStream_t)stream));
  return ASR_OK;
}
