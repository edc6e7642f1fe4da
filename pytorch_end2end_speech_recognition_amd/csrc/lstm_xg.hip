// Bidirectional LSTM recurrence, one persistent launch per layer pass, with the
// recurrent hand-off done by tagged granules (gfx950, bf16 MFMA, f32 state).
// Same semantics as lstm.hip / lstm_persist.hip (nn.LSTM bidirectional with
// pack/pad behaviour, models/pytorch_v3/encoders/rnn.py:166-172, :218-224,
// :343-390): gate order i,f,g,o; h0 = c0 = 0; the reverse direction starts at
// each utterance's own last frame; padded frames produce zeros.
//
// Why a second persistent design (lstm_persist.hip is the counter form): a
// hand-off there is payload store -> drain -> atomic arrival on a counter that
// 64 producers share -> relaxed poll -> workgroup barrier -> payload loads,
// i.e. three dependent fabric round trips plus a 64-way atomic fan-in per time
// step.  Here the data IS the flag (cdna_hip_programming.md §6 Guideline 16,
// form R2): every 8-byte granule is {32-bit payload, 32-bit tag = step + 1},
// written by ONE sc1 store and swept by the consumer with sc1 loads until all
// its tags match, so one step costs one store->load round trip.  Granule words
// are zeroed by a memset before every launch (tag 0 never matches).
//
// Work split.  Groups of R utterances x one direction (R = 8, or 16 for larger
// batches); a group is H/16 work-groups, each owning 16 hidden units for the
// whole pass, its slice of W_hh held in VGPRs as MFMA fragments (converted to
// bf16 once at kernel start), its cell states in registers.  Work-groups are
// pinned one per CU and the grid is launched only when it is co-resident.
//
//   forward  (256 threads, 4 waves split K = H): publishes h_t [R][16] as
//            granules of FOUR bf16 whose step tag is one bit (the LSB of the
//            first value, tag_bit); consumers gather the group's whole h_t
//            [R][H] (K of the recurrent product) -- 8 KB of granules per
//            work-group per step at R = 8, H = 512 (the hop's cost grows with
//            the bytes each consumer CU loads).
//   backward (512 threads): the owner of units J turns dh_t(J) into the gate
//            gradients dg_t [R][4 x 16] and multiplies them by ITS OWN 64 rows of
//            W_hh, publishing partial sums of dh_{t-1} for ALL H units in the
//            forward's granule format (four bf16, one-bit tag: 8 KB per
//            consumer work-group per step at R = 8, H = 512).  A consumer sums
//            the WPG partials of its 16 units in f32.  No transposed copy of
//            W_hh is needed.
//
// Spins are bounded; on give-up a work-group sets the abort word (seen by every
// other spinner) and g_xg_status, and exits: results are then invalid and
// asr_lstm_persist_status reports it.
#include <algorithm>
#include <cstdlib>

#include "mfma.h"
#include "prof.h"

namespace asr {

extern int g_lstm_last_path[2];   // lstm.hip: {forward, backward} implementation of the last pass
__device__ int g_xg_status;  // bit 0: a bounded spin gave up (results invalid)
__device__ int g_xg_mode;    // bit 0: a launch ran write-through (sc1); bit 1: XCD-local
// Sequence number of the last backward launch whose work-groups were all
// resident (written by its block 0 after placement); the wgrad gate waits on it.
__device__ unsigned g_xg_resident;
// Diagnostics only (ASR_XG_TRACE=1): per-step phase timestamps (100 MHz
// s_memrealtime) of work-groups 0..XG_TR_WG-1, steps 0..XG_TR_STEPS-1.
__device__ unsigned long long* g_xg_trace;
// Diagnostics only (asr_lstm_debug_dh): when set, the backward's cell waves
// record every dh_t they form, [B][T][2][H] f32 (the swept partial sums + dy),
// and the spin count of the sweep that fed it, [B/R groups][T][2][H/16] u32.
__device__ float* g_xg_dbg_dh;
__device__ unsigned* g_xg_dbg_spins;
// ... and per cell and step [B][T][2][H][12] f32: the four gate gradients it
// computed, the four gate activations it used, c_t, c_{t-1}, dy and the
// incoming dc carry.
__device__ float* g_xg_dbg_cell;
#define XG_TR_WG 64
#define XG_TR_STEPS 128
#define XG_TR_K 12
#define XG_TR_AT(step, k, val)                                                           \
  do {                                                                                  \
    if (tr && (step) < XG_TR_STEPS)                                                    \
      tr[((long long)blockIdx.x * XG_TR_STEPS + (step)) * XG_TR_K + (k)] = (val);      \
  } while (0)
#define XG_TR(step, k, val)                                                              \
  do {                                                                                  \
    if (tr && (step) < XG_TR_STEPS && lane == 0 && wave == 0)                          \
      tr[((long long)blockIdx.x * XG_TR_STEPS + (step)) * XG_TR_K + (k)] = (val);      \
  } while (0)

namespace {

constexpr int XU = 16;                 // hidden units per work-group
constexpr unsigned XG_SPIN_LIMIT = 1u << 20;
constexpr size_t XG_PIN_FWD = 96 * 1024;   // > 80 KB dynamic LDS: one work-group per CU
constexpr size_t XG_PIN_FWD8 = 64 * 1024;  // 8 sweeper waves: static `part` is >= 34 KB
constexpr size_t XG_PIN_BWD = 140 * 1024;
// ASR_XG_PIN_BWD_KB (read per launch): the backward's dynamic-LDS pin.  Any
// value above 80 KB still keeps one work-group per CU; 96 leaves 64 KB beside
// it, room for one 128 x 128 GEMM work-group (the co-resident weight-gradient
// mode of native_ops, ASR_OVERLAP_WGRAD=2).
int g_pin_bwd_kb = 0;   // asr_lstm_set_bwd_pin_kb (0: ASR_XG_PIN_BWD_KB or the default)
size_t xg_pin_bwd() {
  if (g_pin_bwd_kb > 80 && g_pin_bwd_kb <= 160) return (size_t)g_pin_bwd_kb * 1024;
  const char* e = getenv("ASR_XG_PIN_BWD_KB");
  const int kb = e ? atoi(e) : 0;
  static bool warned = false;
  if (e && !(kb > 80 && kb <= 160) && !warned) {
    warned = true;
    fprintf(stderr, "[lstm_xg] warning: ASR_XG_PIN_BWD_KB=%s outside (80, 160]; using %d KB\n", e,
            (int)(XG_PIN_BWD / 1024));
  }
  return (kb > 80 && kb <= 160) ? (size_t)kb * 1024 : XG_PIN_BWD;
}

// Units per backward work-group (lstm_bwd_xg's XB): asr_lstm_set_bwd_units, else
// ASR_XG_BWD_XU, else 16.  32 only where it is supported: H % 32 == 0, R = 8 and
// at most 32 A fragments per MFMA lane (H <= 512).
int g_bwd_xu = 0;
int xg_bwd_xu(int R, int H) {
  int xu = g_bwd_xu;
  if (!xu) {
    const char* e = getenv("ASR_XG_BWD_XU");
    xu = e ? atoi(e) : 16;
  }
  if (xu == 32 && R == 8 && H % 32 == 0 && (H / 16 + 3) / 4 <= 8) return 32;
  return 16;
}

// asr_lstm_set_dy_flags: dy of the next packed-activation backward launch
// arrives chunk by chunk (see lstm_bwd_xg's sweepers); NULL = off.
const int* g_dyflag = nullptr;
// asr_lstm_set_bwd_progress: the next packed-activation backward launch reports
// when the gate gradients of processing steps <= g_prog_q are stored (every
// cell wave adds 1 to *g_prog_ctr after a release), so the input-gradient GEMM
// of the rows complete by then can start beside the rest of the pass.
unsigned long long* g_prog_ctr = nullptr;
int g_prog_q = -1;
int g_prog_q2 = -1;   // a second reporting step (asr_lstm_set_bwd_progress2), -1: none
int g_dyc0 = 16;
unsigned g_dyepoch = 0;

// The backward's pin leaves no room for the kernel's static LDS: the layer
// would silently take the slower counter-form recurrence -- say so once.
static void xg_warn_pin_unfit(size_t pin) {
  static bool warned = false;
  if (warned) return;
  warned = true;
  fprintf(stderr, "[lstm_xg] warning: backward LDS pin %zu KB + static LDS exceeds the CU's "
          "160 KB; the tagged-granule backward recurrence is skipped and the counter-form "
          "recurrence runs instead (ASR_XG_PIN_BWD_KB <= 150 keeps it)\n", pin / 1024);
}
constexpr unsigned AUX_SC1_VOL = 16u | (1u << 31);  // sc1; volatile (never hoisted from a spin)
constexpr unsigned AUX_SC1 = 16u;

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
// packed gate activations of one (utterance, frame, direction, unit): i, f, g, o
typedef __attribute__((ext_vector_type(4))) _Float16 h16x4;
typedef __attribute__((address_space(1))) int gint;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) float gfloat;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t xg_rsrc(void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ u32x4 ld_sc1(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX_SC1_VOL);
}

__device__ __forceinline__ int tags_ok(const u32x4& v, unsigned tag) {
  return (int)(v[1] == tag) & (int)(v[3] == tag);
}

// Called by a whole wave after a failed sweep; false = give up (abort word set
// by someone, or this wave's spin budget is spent).
__device__ int g_xg_cell_sc1;  // backward cell inputs by sc1 (L2) loads (ASR_XG_CELL_SC1)
__device__ int g_xg_sleep;   // s_sleep(1) units between polls (ASR_XG_SLEEP, default 1)
__device__ int g_xg_delay;   // s_sleep(1) units before a step's first poll (ASR_XG_DELAY)

__device__ __forceinline__ void nap(int n) {
  for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(1);
}

__device__ __forceinline__ bool keep_spinning(unsigned spins, int* abortw, int nsleep) {
  if ((spins & 31u) == 31u) {
    if (__hip_atomic_load((gint*)abortw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
    if (spins >= XG_SPIN_LIMIT) {
      __hip_atomic_store((gint*)abortw, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicOr(&g_xg_status, 1);
      return false;
    }
  }
  nap(nsleep);
  return true;
}

// Work-group placement, decided once per launch.  tid 0 reads its XCD
// (HW_REG_XCC_ID) and registers with ONE 64-bit agent-scope atomic add of
// 1 << (8 * xcc) on the header's registry word, so a single word holds every
// XCD's count consistently; it then waits until all gridDim.x work-groups
// have registered.  If every XCD holds a whole number of groups, groups are
// formed per XCD ("local" mode: a group's producers and consumers share one
// L2, so hand-offs are plain stores into that L2 and sc1 loads that bypass
// only the CU's L1).  Otherwise (or with allow_local = 0) groups follow
// blockIdx and every granule is stored write-through (sc1), which is correct
// for any placement.  Results never depend on placement: placement only
// selects which of the two correct protocols runs.
__device__ __forceinline__ void xg_place(int WPG, int allow_local, int* hdr, int* s_pl,
                                         unsigned seq = 0) {
  if (threadIdx.x == 0) {
    int* abortw = hdr;
    typedef __attribute__((address_space(1))) unsigned long long gu64r;
    gu64r* regw = (gu64r*)(hdr + 16);
    const unsigned xcc =
        __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;  // XCC_ID[3:0]
    int ok = xcc < 8;
    unsigned long long old = 0, now = 0;
    if (ok) old = __hip_atomic_fetch_add(regw, 1ull << (8 * xcc), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    for (unsigned spins = 0; ok; ++spins) {
      now = __hip_atomic_load(regw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned tot = 0;
      for (int x = 0; x < 8; ++x) tot += (unsigned)((now >> (8 * x)) & 255u);
      if (tot >= gridDim.x) break;
      if (__hip_atomic_load((gint*)abortw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
          spins >= XG_SPIN_LIMIT) {
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok) {
      __hip_atomic_store((gint*)abortw, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicOr(&g_xg_status, 1);
    }
    int local = ok && allow_local;
    int before = 0;
    for (int x = 0; x < 8; ++x) {
      const int c = (int)((now >> (8 * x)) & 255u);
      if (c % WPG) local = 0;
      if (x < (int)xcc) before += c / WPG;
    }
    const int slot = (int)((old >> (8 * xcc)) & 255u);
    if (local) {
      s_pl[0] = before + slot / WPG;
      s_pl[1] = slot % WPG;
    } else {
      s_pl[0] = blockIdx.x / WPG;
      s_pl[1] = blockIdx.x % WPG;
    }
    s_pl[2] = local;
    s_pl[3] = ok;
    if (blockIdx.x == 0 && ok) atomicOr(&g_xg_mode, local ? 2 : 1);
    if (blockIdx.x == 0 && ok && seq)
      __hip_atomic_store(&g_xg_resident, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
}

// Forward granules carry FOUR bf16 (units 4q..4q+3 of one row) and no tag
// word: the tag is the least significant bit of the first value, the bf16
// next to h (truncated or one ulp further out) whose LSB is tag_bit(step).
// Steps s and s-2 share a buffer and have different bits; the memset's zeros
// never match the first use (bit 1).  Error <= 1 bf16 ulp on one value in four
// of the recurrent input; y / ybf keep the plain values.
__device__ __forceinline__ unsigned tag_bit(int step) { return (((unsigned)step >> 1) & 1u) ^ 1u; }
__device__ __forceinline__ unsigned bf_with_lsb(float h, unsigned bit) {
  const unsigned t = __float_as_uint(h) >> 16;
  return (t & 1u) == bit ? t : t + 1u;
}
// lane i <- lane i+n inside its row of 16 (DPP row_shl:n); the row's last n
// lanes receive 0
template <int N>
__device__ __forceinline__ unsigned row_from_upper(unsigned x) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x100 + N, 0xf, 0xf, false);
}

__device__ __forceinline__ bf16x8 frag_lo(const u32x4& a, const u32x4& b) {
  // payload words of two 16-B granule pairs -> 8 bf16 (units in order)
  u32x4 w = {a[0], a[2], b[0], b[2]};
  return __builtin_bit_cast(bf16x8, w);
}

__device__ __forceinline__ bf16x8 cvt_f32x8(const float* p) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  u16x8 r;
  r[0] = f2bf(a.x); r[1] = f2bf(a.y); r[2] = f2bf(a.z); r[3] = f2bf(a.w);
  r[4] = f2bf(b.x); r[5] = f2bf(b.y); r[6] = f2bf(b.z); r[7] = f2bf(b.w);
  return as_bf16x8(r);
}

__device__ __forceinline__ float fsig(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
// ftanh's error is absolute (~1e-7 near 0, where tanh(x) ~ x): fine for the
// bf16 paths, not for reference precision -- the F32 kernels take tanhf (an
// LSTM with tiny inputs and forget-gate bias 1 carries h ~ 1e-6 for many steps,
// where ftanh's error was 5 % per step)
__device__ __forceinline__ float ftanh(float x) { return 2.f * fsig(2.f * x) - 1.f; }

// Packed fp16 gate activations (act_h) that keep precision near saturation.
// The backward needs s and 1 - s of each sigmoid gate and g and 1 - g^2 of
// the tanh gate; fp16's spacing just below 1.0 (4.9e-4) would make 1 - s of a
// saturated gate coarse or zero.  A sigmoid gate is stored as s when s < 0.5
// and as -(1 - s) otherwise (s > 0, so the sign bit is free); the tanh gate as
// g when |g| <= 0.499 and as sign(g) * (1 - |g|) * 2^14 otherwise (magnitudes
// >= 0.5 mark the complement form; 1 - |g| is clamped to >= 2^-15, so the
// stored magnitude is >= 0.5 exactly, while direct values round to < 0.5).
// Both forms carry fp16's relative precision for the small factor.
// (-(1 - s), not s - 1: a saturated s == 1 must store -0, whose sign bit marks
// the complement form; s - 1 would give +0 and decode as s = 0)
#ifndef ASR_ACTH_PLAIN
__device__ __forceinline__ float enc_sig(float s) { return s < 0.5f ? s : -(1.f - s); }
__device__ __forceinline__ float enc_tanh(float g) {
  const float a = fabsf(g);
  return a <= 0.499f ? g : copysignf(fmaxf(1.f - a, 1.f / 32768.f) * 16384.f, g);
}
__device__ __forceinline__ void dec_sig(float e, float& s, float& om) {
  const bool neg = (__float_as_uint(e) >> 31) != 0u;   // -0 (s == 1) included
  s = neg ? 1.f + e : e;
  om = neg ? -e : 1.f - e;
}
__device__ __forceinline__ void dec_tanh(float e, float& g, float& om2) {   // om2 = 1 - g^2
  const float a = fabsf(e);
  const float c = a * (1.f / 16384.f);
  const bool cm = a >= 0.5f;
  g = cm ? copysignf(1.f - c, e) : e;
  om2 = cm ? c * (2.f - c) : 1.f - e * e;
}
#else   // A/B builds only: the gates stored as plain fp16 (round 3)
__device__ __forceinline__ float enc_sig(float s) { return s; }
__device__ __forceinline__ float enc_tanh(float g) { return g; }
__device__ __forceinline__ void dec_sig(float e, float& s, float& om) { s = e; om = 1.f - e; }
__device__ __forceinline__ void dec_tanh(float e, float& g, float& om2) { g = e; om2 = 1.f - e * e; }
#endif

// ---------------------------------------------------------------------------
// forward.  grid = G * WPG (G = 2 * ceil(B / R) groups, WPG = H / 16).
// Block -> (group, member); group -> (direction = grp & 1, row group).
// Granules: xg[par][grp][row][H/2] u64 = {bf16 pair (units 2p, 2p+1), tag}.
// Wave roles (each wave's vector-memory counter only waits for its own ops):
//   waves 0..3 (sweepers): poll h_{t-1} granules, MFMA over their K quarter,
//     partial gate sums -> LDS, barrier, next poll.  They issue nothing else,
//     so a poll never waits behind output stores or input prefetches.
//   waves 4.. (R/4 cell waves, one thread per (row, unit)): barrier, sum the
//     partials + the prefetched input projection, cell update, publish h_t
//     granules FIRST, then the y / c / activation / bf16-y stores and the next
//     step's input-projection prefetch.
// One __syncthreads per step; `part` is double-buffered by step parity.
//
// F32 (the reference-precision configs): h_{t-1} travels as f32 and the
// sweepers multiply it by f32 W_hh on v_mfma_f32_16x16x4_f32.  Granules:
// xg[par][grp][row][H/2] u64 = {h(2p) with its LSB the step tag, h(2p+1)}
// (<= 1 f32 ulp on every other value of the recurrent input; y keeps the plain
// values).  The K range is split into 16 contiguous slices of H / 16 units, one
// per (sweeper wave, lane group): lane group kq of wave w covers units
// [(4 w + kq) H / 16, ...), so each 16-B poll of four consecutive units feeds
// four successive k-steps and the W_hh fragments are loaded in that same k
// order.  KSW is then the number of 16-B polls per lane (H = 64 KSW, NSW = 4).
// ---------------------------------------------------------------------------
template <int R, int KSW, int NSW, bool F32 = false, int XUF = XU>
__global__ void __launch_bounds__(64 * NSW + R * XUF) lstm_fwd_xg(
    int B, int T, int H, const int32_t* __restrict__ lens, const float* __restrict__ whh_f,
    const float* __restrict__ whh_r, float* __restrict__ gx_act, float* __restrict__ y,
    float* __restrict__ cst, unsigned long long* xg, int* hdr, uint16_t* __restrict__ ybf,
    unsigned epoch, int allow_local) {
  __shared__ float part[2][NSW][R][4 * XUF + 4];
  __shared__ int s_dead;  // a sweeper gave up: every wave exits after the next barrier
  __shared__ int s_pl[4];
  int* abortw = hdr;
  const int WPG = H / XUF;
  const int G = gridDim.x / WPG;
  if (threadIdx.x == 0) s_dead = 0;
  xg_place(WPG, allow_local, hdr, s_pl);
  if (!s_pl[3]) return;
  const int grp = s_pl[0], mem = s_pl[1];
  const bool local = s_pl[2] != 0;
  (void)epoch;  // forward granules carry a 1-bit step tag (tag_bit) instead
  const int dir = grp & 1, rg = grp >> 1;
  const int u0 = mem * XUF, b0 = rg * R;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nks = H >> 5;
  const unsigned quarter = (unsigned)(H / 4);   // granules per row
  unsigned long long* tr = blockIdx.x < XG_TR_WG ? g_xg_trace : nullptr;

  if constexpr (F32) {
    if (wave < NSW) {
      // --------------------------- f32 sweeper ----------------------------
      static_assert(NSW == 4, "f32 sweepers: 16 K slices = 4 waves x 4 lane groups");
      const int kq = lane >> 4, ln = lane & 15;
      const bool sweeper = ln < R;
      const int kb = (4 * wave + kq) * 4 * KSW;   // this lane group's first unit of K
      // NBK blocks of 16 gate columns: column c = 16 blk + ln is gate c / XUF,
      // unit u0 + c % XUF (XUF = 16: one gate per block; 8: two)
      constexpr int NBK = XUF / 4;
      // B fragments: B[k][n] = W_hh[gate row of column 16 blk + n][kb + k-step]
      float wf[4 * KSW][NBK];
      {
        const float* W = dir ? whh_r : whh_f;
#pragma unroll
        for (int g = 0; g < NBK; ++g)
#pragma unroll
          for (int i = 0; i < KSW; ++i) {
            const int c = 16 * g + ln;
            const float4 w4 = *reinterpret_cast<const float4*>(
                W + (long long)((c / XUF) * H + u0 + c % XUF) * H + kb + 4 * i);
            wf[4 * i][g] = w4.x;
            wf[4 * i + 1][g] = w4.y;
            wf[4 * i + 2][g] = w4.z;
            wf[4 * i + 3][g] = w4.w;
          }
      }
      const __amdgpu_buffer_rsrc_t rs = xg_rsrc(xg, (unsigned)(2ull * G * R * H * 4));
      const int nsleep = __builtin_amdgcn_readfirstlane(g_xg_sleep);
      const int ndelay = __builtin_amdgcn_readfirstlane(g_xg_delay);
      for (int s = 0; s < T; ++s) {
        XG_TR(s, 0, __builtin_amdgcn_s_memrealtime());
        f32x4 acc[NBK];
#pragma unroll
        for (int g = 0; g < NBK; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (s > 0) {
          const unsigned ebit = tag_bit(s - 1);
          const unsigned rowoff =
              (unsigned)(((((s - 1) & 1) * G + grp) * R + (sweeper ? ln : 0)) * (long long)H * 4);
          u32x4 v[KSW];
          nap(ndelay);
          for (unsigned spins = 0;; ++spins) {
            int ok = 1;
            if (sweeper) {
#pragma unroll
              for (int i = 0; i < KSW; ++i) v[i] = ld_sc1(rs, rowoff + (unsigned)((kb + 4 * i) * 4));
#pragma unroll
              for (int i = 0; i < KSW; ++i)
                ok &= (int)((((v[i][0] ^ ebit) | (v[i][2] ^ ebit)) & 1u) == 0u);
            }
            if (__all(ok)) {
              XG_TR(s, 1, __builtin_amdgcn_s_memrealtime());
              XG_TR(s, 5, spins);
              break;
            }
            if (!keep_spinning(spins, abortw, nsleep)) {
              s_dead = 1;
              break;
            }
          }
          // whole-wave MFMAs; rows >= R (lanes that did not sweep) multiply zeros
#pragma unroll
          for (int i = 0; i < KSW; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float a = sweeper ? __uint_as_float(v[i][e]) : 0.f;
#pragma unroll
              for (int g = 0; g < NBK; ++g) acc[g] = mfma_f32(a, wf[4 * i + e][g], acc[g]);
            }
        }
        if (4 * kq < R) {
#pragma unroll
          for (int g = 0; g < NBK; ++g)
#pragma unroll
            for (int r = 0; r < 4; ++r) part[s & 1][wave][4 * kq + r][16 * g + ln] = acc[g][r];
        }
        __syncthreads();  // B(s)
        if (s_dead) return;
        __syncthreads();  // Bp(s)
      }
      return;
    }
  } else if (wave < NSW) {
    // ------------------------------ sweeper -------------------------------
    const int kq = lane >> 4, ln = lane & 15;
    const bool sweeper = ln < R;
    // B fragments: B[k][n] = W_hh[g*H + u0 + n][k], n = ln, k = 32 ks + 8 kq + j
    bf16x8 wf[KSW][4];
    {
      const float* W = dir ? whh_r : whh_f;
#pragma unroll
      for (int i = 0; i < KSW; ++i) {
        const int ks = min(wave + NSW * i, nks - 1);
#pragma unroll
        for (int g = 0; g < 4; ++g)
          wf[i][g] = cvt_f32x8(W + (long long)(g * H + u0 + ln) * H + 32 * ks + 8 * kq);
      }
    }
    const unsigned xg_bytes = (unsigned)(2ull * G * R * quarter * 8);
    const __amdgpu_buffer_rsrc_t rs = xg_rsrc(xg, xg_bytes);
    const int nsleep = __builtin_amdgcn_readfirstlane(g_xg_sleep);
    const int ndelay = __builtin_amdgcn_readfirstlane(g_xg_delay);
    for (int s = 0; s < T; ++s) {
      XG_TR(s, 0, __builtin_amdgcn_s_memrealtime());
      f32x4 acc[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (s > 0) {
        const unsigned ebit = tag_bit(s - 1);
        const unsigned rowoff = (unsigned)((((((s - 1) & 1) * G + grp) * R + (sweeper ? ln : 0)) *
                                            (long long)quarter) * 8);
        u32x4 v[KSW];
        nap(ndelay);
        for (unsigned spins = 0;; ++spins) {
          const unsigned long long t_iss = tr ? __builtin_amdgcn_s_memrealtime() : 0;
          int ok = 1;  // bitwise ANDs: every load is issued before the first wait
          if (sweeper) {
            // k-steps past nks re-read the last one (no branch between the loads)
            // k = 32 ks + 8 kq + 0..7: two granules, one 16-B load
#pragma unroll
            for (int i = 0; i < KSW; ++i)
              v[i] = ld_sc1(rs, rowoff + (unsigned)((8 * min(wave + NSW * i, nks - 1) + 2 * kq) * 8));
#pragma unroll
            for (int i = 0; i < KSW; ++i)
              ok &= (int)((((v[i][0] ^ ebit) | (v[i][2] ^ ebit)) & 1u) == 0u);
          }
          if (__all(ok)) {
            XG_TR(s, 1, __builtin_amdgcn_s_memrealtime());
            XG_TR(s, 5, spins);
            XG_TR(s, 6, t_iss);
            XG_TR(s, 7, (unsigned long long)(grp * 256 + mem));
            break;
          }
          if (!keep_spinning(spins, abortw, nsleep)) {
            s_dead = 1;
            break;
          }
        }
        // MFMA is a whole-wave operation: never under a lane-divergent branch.
        // Rows >= R (lanes that did not sweep) multiply zeros.
#pragma unroll
        for (int i = 0; i < KSW; ++i) {
          if (wave + NSW * i < nks) {  // wave-uniform
            u32x4 z = {0u, 0u, 0u, 0u};
            const bf16x8 a = __builtin_bit_cast(bf16x8, sweeper ? v[i] : z);
#pragma unroll
            for (int g = 0; g < 4; ++g) acc[g] = mfma_bf16(a, wf[i][g], acc[g]);
          }
        }
      }
      // partial gate sums -> LDS (rows 4 kq + r; only rows < R are real)
      if (4 * kq < R) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int r = 0; r < 4; ++r) part[s & 1][wave][4 * kq + r][g * XUF + ln] = acc[g][r];
      }
      XG_TR(s, 4, __builtin_amdgcn_s_memrealtime());
      __syncthreads();  // B(s): partial sums in LDS
      XG_TR(s, 2, __builtin_amdgcn_s_memrealtime());
      if (s_dead) return;
      // Bp(s): this block's cell waves have issued their h_s granules.  Polling
      // for h_s before that cannot succeed, and would only queue this CU's
      // vector-memory pipe ahead of those stores.
      __syncthreads();
    }
    return;
  }

  // -------------------------------- cell ----------------------------------
  const int ct = tid - 64 * NSW;
  static_assert(XUF == 16 || XUF == 8, "units per work-group");
  const int row = ct >> (XUF == 16 ? 4 : 3), unit = ct & (XUF - 1);
  const int b = b0 + row, j = u0 + unit;
  const bool own = b < B;
  const int len = own ? lens[b] : 0;
  float c = 0.f;
  const long long H8 = 8LL * H;
  const long long gcol = (long long)dir * 4 * H + j;
  gu64* xgg = (gu64*)xg;
  float gxv[4] = {0.f, 0.f, 0.f, 0.f};
  if (own) {
    const int t0 = dir ? T - 1 : 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) gxv[q] = gx_act[((long long)b * T + t0) * H8 + gcol + (long long)q * H];
  }
  __builtin_amdgcn_s_setprio(2);  // the cell update + publish is the critical path
  const int cw = wave - NSW;  // trace as this block's first cell wave
  for (int s = 0; s < T; ++s) {
    const int t = dir ? T - 1 - s : s;
    __syncthreads();
    if (s_dead) return;
    float h = 0.f, cn = 0.f, ig = 0.f, fg = 0.f, gg = 0.f, og = 0.f;
    const bool active = own && t < len;
    if (active) {
      float pre[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = q * XUF + unit;
        float a = part[s & 1][0][row][col];
#pragma unroll
        for (int w = 1; w < NSW; ++w) a += part[s & 1][w][row][col];
        pre[q] = a + gxv[q];
      }
      ig = fsig(pre[0]);
      fg = fsig(pre[1]);
      gg = F32 ? tanhf(pre[2]) : ftanh(pre[2]);
      og = fsig(pre[3]);
      cn = fg * c + ig * gg;
      h = og * (F32 ? tanhf(cn) : ftanh(cn));
    }
    c = cn;
    const unsigned hb = f2bf(h);
    const unsigned h1 = row_from_upper<1>(hb);
    const unsigned val = hb | (h1 << 16);                 // bf16 pair for ybf
    if constexpr (F32) {
      // {h(j) with the tag in its LSB, h(j + 1)}: one 8-B granule per unit pair
      const unsigned fb = __float_as_uint(h);
      const unsigned f1 = row_from_upper<1>(fb);
      if ((unit & 1) == 0) {
        const unsigned long long gr =
            ((unsigned long long)f1 << 32) | ((fb & ~1u) | tag_bit(s));
        gu64* p = xgg + ((((long long)(s & 1) * G + grp) * R + row) * (H >> 1) + (j >> 1));
        if (local)
          __hip_atomic_store(p, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
          __hip_atomic_store(p, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
    const unsigned h2 = row_from_upper<2>(hb), h3 = row_from_upper<3>(hb);
    const unsigned h0t = bf_with_lsb(h, tag_bit(s));
    if ((unit & 3) == 0) {
      const unsigned long long gr =
          ((unsigned long long)(h2 | (h3 << 16)) << 32) | (h0t | (h1 << 16));
      gu64* p = xgg + ((((long long)(s & 1) * G + grp) * R + row) * quarter + (j >> 2));
      if (local)  // plain 8-B store: into this XCD's L2, where the group reads
        __hip_atomic_store(p, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else        // write-through (sc1) 8-B store
        __hip_atomic_store(p, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    }
    if (cw == 0 && lane == 0 && tr && s < XG_TR_STEPS)
      tr[((long long)blockIdx.x * XG_TR_STEPS + s) * XG_TR_K + 3] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();  // Bp(s)
    if (own) {
      const long long sidx = ((long long)b * T + t) * 2 * H + (long long)dir * H + j;
      y[sidx] = h;
      cst[sidx] = cn;
      const long long gb = ((long long)b * T + t) * H8 + gcol;
      gx_act[gb] = ig;
      gx_act[gb + H] = fg;
      gx_act[gb + 2 * H] = gg;
      gx_act[gb + 3 * H] = og;
      if (ybf && (unit & 1) == 0)
        *reinterpret_cast<uint32_t*>(ybf + ((long long)b * T + t) * 2 * H + dir * H + j) = val;
      if (s + 1 < T) {
        const int tn = dir ? t - 1 : t + 1;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          gxv[q] = gx_act[((long long)b * T + tn) * H8 + gcol + (long long)q * H];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// forward with the input projection fused (lstm_fwd_xgx).  Same hand-off,
// sweepers and cell waves as lstm_fwd_xg, but gx = x W_ih^T + b_ih + b_hh is
// not precomputed by a GEMM: NPW producer waves hold this work-group's 64 rows
// of W_ih as bf16 MFMA B fragments (k-steps p, p + NPW, ... of K = Din) in
// VGPRs and, one step ahead of the recurrence, multiply the bf16 input rows
// x[b, t] of the group's R utterances (loaded a further step ahead).  Their
// partial gate inputs go to LDS (double-buffered by step parity) before
// barrier B(s); the cell waves sum them with the biases for step s + 1 after
// publishing h_s -- where lstm_fwd_xg prefetched gx from HBM -- so nothing is
// added to the hand-off chain.  `act` receives the post-activation gates for
// the backward and is never read here.
//
// LDS hazards (producers write pre(s+1) into xpart[(s+1)&1] between Bp(s-1)
// and B(s); cells read pre(s+1) between Bp(s) and B(s+1)): the buffer a
// producer overwrites at iteration s was last read before B(s-1).
// ---------------------------------------------------------------------------
constexpr int XGX_DMAX = 1024;   // largest input width of the fused projection
typedef __attribute__((address_space(3))) void lds_void_t;

template <int R, int KSW, int NSW, int NPW, int KPW>
__global__ void __launch_bounds__(64 * NSW + R * XU + 64 * NPW) lstm_fwd_xgx(
    int B, int T, int H, const int32_t* __restrict__ lens, const float* __restrict__ whh_f,
    const float* __restrict__ whh_r, const uint16_t* __restrict__ x, int Din,
    const uint16_t* __restrict__ wih, const float* __restrict__ b_ih,
    const float* __restrict__ b_hh, float* __restrict__ act, float* __restrict__ y,
    float* __restrict__ cst, unsigned long long* xg, int* hdr, uint16_t* __restrict__ ybf,
    int allow_local, int late_load, int defer_st, h16x4* __restrict__ acth,
    uint16_t* __restrict__ ydrop, float drop_p, unsigned long long drop_seed) {
  (void)late_load;   // input rows now staged by LDS DMA three steps ahead
  // partial gate inputs, row r of a step at prow(r).  (A bank-conflict-free
  // pitch -- rows 80 floats apart, rows 4..7 a further 16 on -- measured
  // 1457 vs 1450 us per 5x512 launch against this 68-float pitch: the cell's
  // partial-sum reads are not what bounds the step.)
  constexpr int PROW = 4 * XU + 4;
  constexpr int PSZ = R * PROW;
  auto prow = [](int r) { return r * PROW; };
  // the sweepers' partials column-major: a lane's four rows of one gate column
  // (its MFMA accumulator) are one 16-B store -- four per lane instead of
  // sixteen 4-B stores between the MFMAs and barrier B(s); a 12-float column
  // pitch keeps the cells' reads (4 rows x 16 units per wave) conflict-free.
  // Measured (same-box A/B): 303 -> 289 us per launch at H = 320 (KSW = 3),
  // 1442 -> 1450 at H = 512 (KSW = 4), so H = 512 keeps the row-major form.
  constexpr bool PCM = KSW < 4;
  constexpr int PCOL = R + 4;
  static_assert(!PCM || R == 8, "column pitch chosen for 8 rows");
  __shared__ __attribute__((aligned(16))) float part[2][NSW][PCM ? 4 * XU * PCOL : PSZ];
  __shared__ float xpart[2][NPW][PSZ];
  // input rows of steps s+1 .. s+3: [3 slots][R rows][XGX_DMAX] bf16, filled by
  // buffer -> LDS DMA three steps ahead (16-B chunks XOR-swizzled by row when
  // Din % 64 == 0, so a fragment read of 8 rows hits distinct banks)
  __shared__ __attribute__((aligned(16))) uint16_t xs[3][R * XGX_DMAX];
  __shared__ int s_dead;
  __shared__ int s_pl[4];
  int* abortw = hdr;
  const int WPG = H / XU;
  const int G = gridDim.x / WPG;
  if (threadIdx.x == 0) s_dead = 0;
  xg_place(WPG, allow_local, hdr, s_pl);
  if (!s_pl[3]) return;
  const int grp = s_pl[0], mem = s_pl[1];
  const bool local = s_pl[2] != 0;
  const int dir = grp & 1, rg = grp >> 1;
  const int u0 = mem * XU, b0 = rg * R;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nks = H >> 5;
  const unsigned quarter = (unsigned)(H / 4);
  constexpr int NCW = R * XU / 64;
#ifdef ASR_XG_TRACE_FWD   // phase stamps (tools/xg_trace.py); they cost ~5 % of the step
  unsigned long long* tr = blockIdx.x < XG_TR_WG ? g_xg_trace : nullptr;
#else
  constexpr unsigned long long* tr = nullptr;
#endif

  if (wave < NSW) {
    // ------------------------------ sweeper (as lstm_fwd_xg) ------------------
    const int kq = lane >> 4, ln = lane & 15;
    const bool sweeper = ln < R;
    bf16x8 wf[KSW][4];
    {
      const float* W = dir ? whh_r : whh_f;
#pragma unroll
      for (int i = 0; i < KSW; ++i) {
        const int ks = min(wave + NSW * i, nks - 1);
#pragma unroll
        for (int g = 0; g < 4; ++g)
          wf[i][g] = cvt_f32x8(W + (long long)(g * H + u0 + ln) * H + 32 * ks + 8 * kq);
      }
    }
    const unsigned xg_bytes = (unsigned)(2ull * G * R * quarter * 8);
    const __amdgpu_buffer_rsrc_t rs = xg_rsrc(xg, xg_bytes);
    const int nsleep = __builtin_amdgcn_readfirstlane(g_xg_sleep);
    const int ndelay = __builtin_amdgcn_readfirstlane(g_xg_delay);
    __syncthreads();  // B_pre: the first three steps' input rows are in LDS
    __syncthreads();  // B_init: the producers' pre(0) is in LDS
    for (int s = 0; s < T; ++s) {
      XG_TR(s, 0, __builtin_amdgcn_s_memrealtime());
      f32x4 acc[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (s > 0) {
        const unsigned ebit = tag_bit(s - 1);
        const unsigned rowoff = (unsigned)((((((s - 1) & 1) * G + grp) * R + (sweeper ? ln : 0)) *
                                            (long long)quarter) * 8);
        u32x4 v[KSW];
        nap(ndelay);
        for (unsigned spins = 0;; ++spins) {
          const unsigned long long t_iss = tr ? __builtin_amdgcn_s_memrealtime() : 0;
          int ok = 1;
          if (sweeper) {
#pragma unroll
            for (int i = 0; i < KSW; ++i)
              v[i] = ld_sc1(rs, rowoff + (unsigned)((8 * min(wave + NSW * i, nks - 1) + 2 * kq) * 8));
#pragma unroll
            for (int i = 0; i < KSW; ++i)
              ok &= (int)((((v[i][0] ^ ebit) | (v[i][2] ^ ebit)) & 1u) == 0u);
          }
          if (__all(ok)) {
            XG_TR(s, 1, __builtin_amdgcn_s_memrealtime());
            XG_TR(s, 5, spins);
            XG_TR(s, 6, t_iss);
            XG_TR(s, 7, (unsigned long long)(grp * 256 + mem));
            break;
          }
          if (!keep_spinning(spins, abortw, nsleep)) {
            s_dead = 1;
            break;
          }
        }
#pragma unroll
        for (int i = 0; i < KSW; ++i) {
          if (wave + NSW * i < nks) {  // wave-uniform
            u32x4 z = {0u, 0u, 0u, 0u};
            const bf16x8 a = __builtin_bit_cast(bf16x8, sweeper ? v[i] : z);
#pragma unroll
            for (int g = 0; g < 4; ++g) acc[g] = mfma_bf16(a, wf[i][g], acc[g]);
          }
        }
      }
      if (tr && wave == 0 && lane == 0) {
        asm volatile("" ::"v"(acc[0][0]), "v"(acc[1][0]), "v"(acc[2][0]), "v"(acc[3][0]));
        XG_TR_AT(s, 11, __builtin_amdgcn_s_memrealtime());
      }
      if (4 * kq < R) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
          if constexpr (PCM) {
            *reinterpret_cast<f32x4*>(&part[s & 1][wave][(g * XU + ln) * PCOL + 4 * kq]) = acc[g];
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) part[s & 1][wave][prow(4 * kq + r) + g * XU + ln] = acc[g][r];
          }
      }
      XG_TR(s, 4, __builtin_amdgcn_s_memrealtime());
      __syncthreads();  // B(s)
      XG_TR(s, 2, __builtin_amdgcn_s_memrealtime());
      if (s_dead) return;
      __syncthreads();  // Bp(s)
    }
    return;
  }

  if (wave >= NSW + NCW) {
    // ------------------------------ producer ----------------------------------
    const int pw = wave - NSW - NCW;
    const int kq = lane >> 4, ln = lane & 15;
    const int nkx = (Din + 31) >> 5;
    const u16x8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
    // B fragments: B[k][n] = W_ih[dir*4H + g*H + u0 + n][k], n = ln, k = 32 ks + 8 kq + j
    bf16x8 wb[KPW][4];
#pragma unroll
    for (int i = 0; i < KPW; ++i) {
      const int k = 32 * (pw + NPW * i) + 8 * kq;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const long long row = (long long)dir * 4 * H + (long long)g * H + u0 + ln;
        wb[i][g] = k < Din ? load_bf16x8(wih + row * Din + k) : as_bf16x8(z8);
      }
    }
    const bool swz = (Din & 63) == 0;
    const __amdgpu_buffer_rsrc_t xr = xg_rsrc((void*)x, (unsigned)((long long)B * T * Din * 2));
    const int slot_elems = R * Din;
    constexpr int NI = (R * XGX_DMAX * 2 + NPW * 1024 - 1) / (NPW * 1024);  // DMAs per wave
    // buffer -> LDS DMA of step st's R input rows into ring slot st % 3
    auto stage_x = [&](int st) {
      const int t = dir ? T - 1 - st : st;
      uint16_t* slot = &xs[st % 3][0];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int blk = pw * NI + i;
        const int e = blk * 512 + lane * 8;        // element of the slot this lane fills
        unsigned voff = 0x7ffffff0u;               // out of range: zeros
        if (e < slot_elems) {
          const int r = e / Din, c = (e - r * Din) >> 3;
          const int cs = swz ? (c ^ (r & 7)) : c;  // source chunk of LDS chunk c
          if (b0 + r < B) voff = (unsigned)((((long long)(b0 + r) * T + t) * Din + 8 * cs) * 2);
        }
        if (blk * 512 < slot_elems) {              // wave-uniform
          const unsigned lds_addr = (unsigned)(uintptr_t)(lds_void_t*)(slot + blk * 512);
          unsigned keep;
          asm volatile(
              "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
              "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
              : "=&s"(keep)
              : "v"(voff), "s"(xr), "s"(lds_addr)
              : "memory");
        }
      }
    };
    auto produce = [&](int st) {
      const uint16_t* slot = &xs[st % 3][0];
      f32x4 acc[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < KPW; ++i) {
#ifdef ASR_XGX_HALF_TEST   // timing experiment only: half the projection (wrong results)
        if ((i & 1) && st > 0) continue;
#endif
        if (pw + NPW * i < nkx) {  // wave-uniform
          const int k = 32 * (pw + NPW * i) + 8 * kq;
          bf16x8 a = as_bf16x8(z8);
          if (ln < R && k < Din) {
            const int c = (k >> 3) ^ (swz ? (ln & 7) : 0);
            a = *reinterpret_cast<const bf16x8*>(slot + ln * Din + 8 * c);
          }
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[g] = mfma_bf16(a, wb[i][g], acc[g]);
        }
      }
      if (4 * kq < R) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int r = 0; r < 4; ++r) xpart[st & 1][pw][prow(4 * kq + r) + g * XU + ln] = acc[g][r];
      }
    };
    for (int st = 0; st < 3 && st < T; ++st) stage_x(st);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // B_pre
    produce(0);
    __syncthreads();  // B_init
    // Step s+1's gate inputs before B(s); after B(s) wait for this wave's DMA
    // of step s+2 (issued one step ago) and issue step s+3's: the barrier Bp(s)
    // then publishes every wave's rows of step s+2 for produce(s+2).
    for (int s = 0; s < T; ++s) {
      if (s + 1 < T) produce(s + 1);
      if (pw == 0 && lane == 0) XG_TR_AT(s, 8, __builtin_amdgcn_s_memrealtime());
      __syncthreads();  // B(s)
      if (s_dead) return;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (s + 3 < T) stage_x(s + 3);
      __syncthreads();  // Bp(s)
    }
    return;
  }

  // -------------------------------- cell ----------------------------------
  const int ct = tid - 64 * NSW;
  const int row = ct >> 4, unit = ct & 15;
  const int b = b0 + row, j = u0 + unit;
  const bool own = b < B;
  const int len = own ? lens[b] : 0;
  float c = 0.f;
  const long long H8 = 8LL * H;
  const long long gcol = (long long)dir * 4 * H + j;
  gu64* xgg = (gu64*)xg;
  float bsum[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) bsum[q] = b_ih[gcol + (long long)q * H] + b_hh[gcol + (long long)q * H];
  float gxv[4];
  __syncthreads();  // B_pre
  __syncthreads();  // B_init
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float v = bsum[q];
#pragma unroll
    for (int p = 0; p < NPW; ++p) v += xpart[0][p][prow(row) + q * XU + unit];
    gxv[q] = v;
  }
  __builtin_amdgcn_s_setprio(2);  // the cell update + publish is the critical path
  // defer_st: step s's y / c / gate / bf16-y stores are issued after B(s+1)
  // (ahead of step s+1's cell math) instead of right after Bp(s), where they
  // share the CU's vector-memory path with the sweepers' polls for step s+1
  float pv[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  unsigned pval = 0u, pdval = 0u;
  int pt = -1;
  // ydrop: bf16 dropout(y) with asr_dropout's mask over [B][T][2H] -- the next
  // layer's staged input, written here instead of from an f32 y (y may be null)
  const float dscale = 1.f / (1.f - drop_p);
  auto store_step = [&](int tt, const float* v, unsigned bv, unsigned dv) {
    const long long sidx = ((long long)b * T + tt) * 2 * H + (long long)dir * H + j;
    if (y) y[sidx] = v[0];
    cst[sidx] = v[1];
    if (acth) {   // the four gates of (b, t, dir, j) as one 8-B fp16 store (enc_sig / enc_tanh)
      const h16x4 hv = {(_Float16)enc_sig(v[2]), (_Float16)enc_sig(v[3]), (_Float16)enc_tanh(v[4]),
                        (_Float16)enc_sig(v[5])};
      acth[(((long long)b * T + tt) * 2 + dir) * H + j] = hv;
    } else {
      const long long gb = ((long long)b * T + tt) * H8 + gcol;
      act[gb] = v[2];
      act[gb + H] = v[3];
      act[gb + 2 * H] = v[4];
      act[gb + 3 * H] = v[5];
    }
    if (ybf && (unit & 1) == 0)
      *reinterpret_cast<uint32_t*>(ybf + ((long long)b * T + tt) * 2 * H + dir * H + j) = bv;
    if (ydrop && (unit & 1) == 0)
      *reinterpret_cast<uint32_t*>(ydrop + ((long long)b * T + tt) * 2 * H + dir * H + j) = dv;
  };
  for (int s = 0; s < T; ++s) {
    const int t = dir ? T - 1 - s : s;
    __syncthreads();  // B(s)
    // the abort word is tested after the step's math: its LDS read overlaps
    // the partial-sum reads instead of preceding them
    const int dead = s_dead;
    if (defer_st && own && pt >= 0) store_step(pt, pv, pval, pdval);
    float h = 0.f, cn = 0.f, ig = 0.f, fg = 0.f, gg = 0.f, og = 0.f;
    const bool active = own && t < len;
    if (active) {
      float pre[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = q * XU + unit;
        const int pi = PCM ? col * PCOL + row : prow(row) + col;
        float a = part[s & 1][0][pi];
#pragma unroll
        for (int w = 1; w < NSW; ++w) a += part[s & 1][w][pi];
        pre[q] = a + gxv[q];
      }
      if (ct == 0 && tr) {   // (trace) the partial sums are in registers
        asm volatile("" ::"v"(pre[0]), "v"(pre[1]), "v"(pre[2]), "v"(pre[3]));
        XG_TR_AT(s, 9, __builtin_amdgcn_s_memrealtime());
      }
      ig = fsig(pre[0]);
      fg = fsig(pre[1]);
      gg = ftanh(pre[2]);
      og = fsig(pre[3]);
      cn = fg * c + ig * gg;
      h = og * ftanh(cn);
      if (ct == 0 && tr) {
        asm volatile("" ::"v"(h));
        XG_TR_AT(s, 10, __builtin_amdgcn_s_memrealtime());
      }
    }
    c = cn;
    if (dead) return;
    const unsigned hb = f2bf(h);
    const unsigned h1 = row_from_upper<1>(hb);
    const unsigned val = hb | (h1 << 16);
    const unsigned h2 = row_from_upper<2>(hb), h3 = row_from_upper<3>(hb);
    const unsigned h0t = bf_with_lsb(h, tag_bit(s));
    if ((unit & 3) == 0) {
      const unsigned long long gr =
          ((unsigned long long)(h2 | (h3 << 16)) << 32) | (h0t | (h1 << 16));
      gu64* p = xgg + ((((long long)(s & 1) * G + grp) * R + row) * quarter + (j >> 2));
      if (local)
        __hip_atomic_store(p, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else
        __hip_atomic_store(p, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (ct == 0 && tr && s < XG_TR_STEPS)
      tr[((long long)blockIdx.x * XG_TR_STEPS + s) * XG_TR_K + 3] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();  // Bp(s)
    pv[0] = h; pv[1] = cn; pv[2] = ig; pv[3] = fg; pv[4] = gg; pv[5] = og;
    pval = val;
    pt = t;
    if (ydrop) {   // off the hand-off chain: the sweepers are polling for step s + 1
      const long long sidx = ((long long)b * T + t) * 2 * H + (long long)dir * H + j;
      const unsigned db = f2bf(u01(drop_seed, (unsigned long long)sidx) >= drop_p ? h * dscale : 0.f);
      pdval = db | (row_from_upper<1>(db) << 16);
    }
    if (own && (!defer_st || s + 1 == T)) store_step(t, pv, pval, pdval);
    if (s + 1 < T) {  // the producers wrote pre(s+1) before B(s)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v = bsum[q];
#pragma unroll
        for (int p = 0; p < NPW; ++p) v += xpart[(s + 1) & 1][p][prow(row) + q * XU + unit];
        gxv[q] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward.  grid = G * WPG, WPG = H / XB work-groups per group, each owning
// XB units (16, or 32 to leave half of a 256-CU chip to the weight-gradient
// GEMMs at 5x512: the group's fan-in halves and the MFMA phase doubles).
// Processing step q handles the forward direction at t = T-1-q and the reverse
// direction at t = q.
// Granules: pg[par][grp][producer][row][H/4] u64 = four bf16 partials of dh
// (units 4p .. 4p+3), the first one's LSB the step tag bit -- the partials are
// sums of bf16 dg x bf16 W_hh products accumulated in f32 and rounded once for
// transport; the consumer sums the WPG partials in f32.
// Wave roles, two barriers per step (B1: partials summed; B2: dg in LDS):
//   waves 0..3 (sweepers): poll the partials of dh for this block's XB units
//     from every producer of the group, sum per producer subset -> LDS, B1, B2.
//   R XB / 64 cell waves: B1, dh = dy + sum, cell backward -> dg (bf16 -> LDS),
//     B2, then the f32 / bf16 dg stores and the next step's prefetch.
//   XB / 4 MFMA waves: B1, B2, partial dh_{t-1}[rows][all units] = dg x (this
//     block's 4 XB rows of W_hh) -> write-through granules.
// A fragments (VGPRs): A[m][k] = W_hh[gaterow(k)][m] for output unit m (M block
// mb = mw + (XB / 4) i) and local gate row k in [0, 4 XB): gate k / XB, unit u0 + k % XB.
//
// F32 (reference-precision configs; XB = 16, f32 activations, f32 dG): the
// partials of dh travel as f32 pairs (pg[par][grp][producer][row][H/2] u64 =
// {partial(2p) with the tag in its LSB, partial(2p + 1)}), dG sits in LDS as
// f32 and the MFMA waves run v_mfma_f32_16x16x4_f32 over 16 k-steps; lane
// group kq takes gate kq's 16 units in order (k = 16 kq + k-step), so its B
// operand is four 16-B LDS reads of one dG row and its A fragments are
// W_hh[kq H + u0 + k-step][m].
// ---------------------------------------------------------------------------
template <int R, int MB, bool AH, int XB, bool F32 = false>
__global__ void __launch_bounds__(256 + R * XB + 64 * (F32 ? 4 : XB / 4)) lstm_bwd_xg(
    int B, int T, int H, const int32_t* __restrict__ lens, const float* __restrict__ whh_f,
    const float* __restrict__ whh_r, const float* __restrict__ dy, float* __restrict__ act_dg,
    const float* __restrict__ cst, unsigned long long* pg, int* hdr,
    uint16_t* __restrict__ dgbf, float* __restrict__ dbpart, unsigned epoch, int allow_local,
    int dg_f32, int io_pos, int dg_st16, const h16x4* __restrict__ acth,
    const int* __restrict__ dyflag, int dyc0, int dyepoch, unsigned long long* prog,
    int prog_q, int prog_q2) {
  static_assert(!F32 || ((XB == 16 || XB == 8) && !AH), "f32 backward: 8 or 16 units, f32 activations");
  constexpr int UPL = F32 ? 4 : 8;     // units per 16-B load
  constexpr int SQ = XB / UPL;         // 16-B loads per row of a producer's slice
  constexpr int LPS = R * SQ;          // sweeper lanes per producer subset
  constexpr int NPG = 256 / LPS;       // producer subsets swept in parallel
  constexpr int NKS = F32 ? XB : XB / 8;   // MFMA k-steps: 4 gates x XB units / (4 or 32)
  // MFMA waves (bf16: XB / 4, 8 at XB = 32 with 64 fragment VGPRs each; f32: 4,
  // one per SIMD, whatever XB)
  constexpr int NMW = F32 ? 4 : XB / 4;
  constexpr int WPGMAX = 16 * NMW * MB / XB;   // producers: H / XB <= 16 NMW MB / XB
  typedef typename std::conditional<F32, float, uint16_t>::type dgt_t;
  // row pitch XB + 4: a sweeper lane's 8 partial sums are two 16-B stores
  __shared__ __attribute__((aligned(16))) float red[NPG][R][XB + 4];
  __shared__ __attribute__((aligned(16))) dgt_t dgt[16][4 * XB + (F32 ? 4 : 8)];
  __shared__ int s_dead;
  __shared__ int s_pl[4];
  int* abortw = hdr;
  const int WPG = H / XB;
  const int G = gridDim.x / WPG;
  if (threadIdx.x == 0) s_dead = 0;
  xg_place(WPG, allow_local, hdr, s_pl, epoch);  // epoch: the launch's sequence number
  if (!s_pl[3]) return;
  const int grp = s_pl[0], mem = s_pl[1];
  const bool local = s_pl[2] != 0;  // granules carry a 1-bit step tag (tag_bit)
  const int dir = grp & 1, rg = grp >> 1;
  const int u0 = mem * XB, b0 = rg * R;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int HB = H / 16;                 // output M blocks
  const int H4 = 4 * H;
  const int hq = F32 ? H / 2 : H / 4;    // granules per producer row
  const unsigned pg_bytes = (unsigned)(2ull * G * WPG * R * hq * 8);
  const __amdgpu_buffer_rsrc_t rs = xg_rsrc(pg, pg_bytes);
  unsigned long long* tr = blockIdx.x < XG_TR_WG ? g_xg_trace : nullptr;
  for (int e = tid; e < (int)(sizeof(dgt) / sizeof(dgt_t)); e += blockDim.x) (&dgt[0][0])[e] = 0;
  const int NCW = R * XB / 64;                // cell waves: 4 .. 4 + NCW - 1; MFMA waves after

  if (wave < 4) {
    // ------------------------------ sweeper -------------------------------
    const int sl = tid & (LPS - 1);
    const int srow = sl / SQ, sq = sl % SQ;   // row, units UPL sq .. UPL (sq + 1) - 1
    const int pgi = tid / LPS;
    // producers per sweeper lane
    constexpr int NLD = (WPGMAX + NPG - 1) / NPG;
    unsigned* dspin = g_xg_dbg_spins;
    const int nsleep = __builtin_amdgcn_readfirstlane(g_xg_sleep);
    const int ndelay = __builtin_amdgcn_readfirstlane(g_xg_delay);
    // dyflag (non-null): dy is being written while this kernel runs -- by the
    // layer above's input-gradient GEMMs, chunk by chunk from both ends of the
    // sequence (chunk k = processing steps [c0 k, c0 (k + 1)), signalled in
    // order up to the middle step).  The cell waves load step
    // q + 2's dy after B2 of step q, so the sweepers make sure of chunk
    // (q + 2) -- clamped to the middle step, whose chunk covers the rows of
    // every later step -- before B1 of step q; the flag's load is issued
    // before the step's poll and checked after it.
    const int qmid = (T + 1) / 2 - 1;
    int dyk = -1, dynext = 0, dyv = 0;
    auto dy_need = [&](int q) { return min(q, qmid) >= dynext; };
    if (dyflag && dy_need(min(1, T - 1))) {   // steps 0 and 1 (loaded before the loop)
      for (unsigned spins = 0;; ++spins) {
        if (__hip_atomic_load(dyflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == dyepoch) break;
        if (!keep_spinning(spins, abortw, nsleep)) { s_dead = 1; break; }
      }
      dyk = 0;
      dynext = dyc0;
    }
    __syncthreads();  // B0: the cell waves load steps 0 and 1 after it
    for (int q = 0; q < T; ++q) {
      XG_TR(q, 0, __builtin_amdgcn_s_memrealtime());
      const bool dyw = dyflag && q + 2 < T && dy_need(q + 2);
      if (dyw) dyv = __hip_atomic_load(dyflag + dyk + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (q > 0) {
        const unsigned ebit = tag_bit(q - 1);
        const long long base = ((long long)((q - 1) & 1) * G + grp) * WPG;
        float sm[8];
        nap(ndelay);
        // every load of the sweep is in flight before the first wait: slots
        // past the group's last producer read beyond the buffer's extent, which
        // a buffer load returns as zeros without a memory access (a guarded
        // load per slot made the compiler wait for each one in turn: one L2
        // round trip per slot instead of one per sweep)
        auto issue = [&](u32x4 (&vv)[NLD]) {
#pragma unroll
          for (int l = 0; l < NLD; ++l) {
            const int w = pgi + l * NPG;
            // two granules = this block's units 8 sq .. 8 sq + 7 from producer w
            const unsigned off =
                w < WPG ? (unsigned)((((base + w) * R + srow) * (long long)hq + u0 / (UPL / 2) + 2 * sq) * 8)
                        : 0x7ffffff0u;
            vv[l] = ld_sc1(rs, off);
          }
        };
        auto check = [&](const u32x4 (&vv)[NLD]) {
          int ok = 1;
#pragma unroll
          for (int e = 0; e < 8; ++e) sm[e] = 0.f;
#pragma unroll
          for (int l = 0; l < NLD; ++l) {
            const u32x4 v = vv[l];
            ok &= (int)(pgi + l * NPG >= WPG) | (int)((((v[0] ^ ebit) | (v[2] ^ ebit)) & 1u) == 0u);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              if constexpr (F32) {
                sm[e] += __uint_as_float(v[e]);
              } else {
                sm[2 * e] += bf2f((uint16_t)(v[e] & 0xffffu));
                sm[2 * e + 1] += bf2f((uint16_t)(v[e] >> 16));
              }
            }
          }
          return __all(ok);
        };
        for (unsigned spins = 0;; ++spins) {
          const unsigned long long t_iss = tr ? __builtin_amdgcn_s_memrealtime() : 0;
          u32x4 vv[NLD];
          issue(vv);
          if (check(vv)) {
            XG_TR(q, 1, __builtin_amdgcn_s_memrealtime());
            XG_TR(q, 5, spins);
            XG_TR(q, 6, t_iss);
            XG_TR(q, 7, (unsigned long long)(grp * 256 + mem));
            if (dspin && tid == 0)
              dspin[(((long long)rg * T + q) * 2 + dir) * WPG + mem] = spins + 1;
            break;
          }
          if (!keep_spinning(spins, abortw, nsleep)) {
            s_dead = 1;
            break;
          }
        }
#pragma unroll
        for (int e = 0; e < UPL; e += 4)
          *reinterpret_cast<f32x4*>(&red[pgi][srow][UPL * sq + e]) =
              f32x4{sm[e], sm[e + 1], sm[e + 2], sm[e + 3]};
      }
      if (dyw) {   // chunk dyk + 1 (one step may cross at most one boundary)
        for (unsigned spins = 0; dyv != dyepoch; ++spins) {
          if (!keep_spinning(spins, abortw, nsleep)) { s_dead = 1; break; }
          dyv = __hip_atomic_load(dyflag + dyk + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        ++dyk;
        dynext = dyc0 * (dyk + 1);
      }
      __syncthreads();  // B1
      XG_TR(q, 2, __builtin_amdgcn_s_memrealtime());
      if (s_dead) return;
      __syncthreads();  // B2
      XG_TR(q, 3, __builtin_amdgcn_s_memrealtime());
      __syncthreads();  // B3: this block's MFMA waves have issued their partials
    }
    return;
  }

  if (wave < 4 + NCW) {
    // -------------------------------- cell --------------------------------
    __builtin_amdgcn_s_setprio(2);
    const int ct = tid - 256;
#ifdef ASR_XG_DIAG_CELL_T   // diagnostics build: rows across lanes, units across lane groups
    const int row = ct % R, unit = ct / R;
#else
    const int row = ct / XB, unit = ct % XB;
#endif
    const int b = b0 + row, j = u0 + unit;
    const bool own = b < B;
    const int len = own ? lens[b] : 0;
    float dc = 0.f;
    float* ddh = g_xg_dbg_dh;
    float* dcl = g_xg_dbg_cell;
    // c_t of step q is c_{tp} of step q - 1: with `carry` it is taken from there
    // bit 0: every cell input by agent-scope loads (ASR_XG_CELL_SC1); bit 1: dy
    // only -- it is written by another stream's GEMMs while this launch runs
    const int lsc1 = __builtin_amdgcn_readfirstlane(g_xg_cell_sc1) | (dyflag ? 2 : 0);
    auto ldf = [&](const float* p) {
      return (lsc1 & 1) ? __hip_atomic_load((const gfloat*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                  : *p;
    };
    auto load_cell = [&](int q, float (&av)[4], h16x4& avh, float& cc, float& cp, float& dyv,
                         const float* carry) {
      const int t = dir == 0 ? T - 1 - q : q;
      const int tp = dir == 0 ? t - 1 : t + 1;
      const long long gb = ((long long)b * T + t) * 8 * H + (long long)dir * H4 + j;
      const long long si = ((long long)b * T + t) * 2 * H + (long long)dir * H + j;
      if constexpr (AH) {   // one 8-B load of the four fp16 gates, converted when used
        const h16x4* pa = acth + (((long long)b * T + t) * 2 + dir) * H + j;
        if (lsc1)
          avh = __builtin_bit_cast(h16x4, __hip_atomic_load((const gu64*)pa, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT));
        else
          avh = *pa;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) av[k] = ldf(act_dg + gb + (long long)k * H);
      }
      cc = carry ? *carry : ldf(cst + si);
      cp = (tp >= 0 && tp < T) ? ldf(cst + si + (long long)(tp - t) * 2 * H) : 0.f;
      if (!dy)
        dyv = 0.f;
      else if (lsc1)   // bit 1: dy written by another stream's GEMMs during the launch
        dyv = __hip_atomic_load((const gfloat*)(dy + si), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        dyv = *(dy + si);
    };
    // inputs of step q (av, cc, cp, dyv) and q + 1 (n*): loaded two steps ahead
    float av[4] = {0.f, 0.f, 0.f, 0.f}, cc = 0.f, cp = 0.f, dyv = 0.f;
    float nav[4] = {0.f, 0.f, 0.f, 0.f}, ncc = 0.f, ncp = 0.f, ndyv = 0.f;
    h16x4 avh = {0, 0, 0, 0}, navh = {0, 0, 0, 0};
    // bias gradient: sum over t of this (utterance, unit)'s four gate gradients
    float sb_i = 0.f, sb_f = 0.f, sb_g = 0.f, sb_o = 0.f;
    __syncthreads();  // B0 (the sweepers have seen dy's first chunk)
    if (own) load_cell(0, av, avh, cc, cp, dyv, nullptr);
#ifndef ASR_XG_DIAG_PREF1
    if (own && T > 1) load_cell(1, nav, navh, ncc, ncp, ndyv, nullptr);
#endif
    // io_pos: where the cell waves issue a step's dG stores and the loads of
    // step q + 2 in the CU's vector-memory queue.  0: after B2 (beside the
    // partial-dh stores); 1: after B3 (beside the next poll: measured +2.4 ms /
    // step at 5x512; stores after B1 of the next step: +0.25 ms).
    // bf16 dG leaves from the dgt tile (stable from B2 until the next step's B1)
    // as ONE 16-B store per lane of the first R / 8 cell waves -- R rows x 4
    // gates x 2 halves of 8 units -- instead of four 2-B stores per (row, unit)
    // lane on every cell wave (dg_st16; ASR_XG_DG_ST16=0: the per-lane stores).
    const int srow = ct / (4 * SQ), sg = (ct / SQ) & 3, sh = ct % SQ;
    const bool st16 = !F32 && dg_st16 && dgbf && ct < 4 * SQ * R && b0 + srow < B;
    auto step_io = [&](int q, int t, float d_i, float d_f, float d_g, float d_o, uint16_t bi,
                       uint16_t bff, uint16_t bg, uint16_t bo) {
      if (own) {
        const long long gb = ((long long)b * T + t) * 8 * H + (long long)dir * H4 + j;
        if (dg_f32) {  // f32 dG in place (not needed when only the bf16 copy feeds the GEMMs)
          act_dg[gb] = d_i;
          act_dg[gb + H] = d_f;
          act_dg[gb + 2 * H] = d_g;
          act_dg[gb + 3 * H] = d_o;
        }
        if (dgbf && !dg_st16) {
          dgbf[gb] = bi;
          dgbf[gb + H] = bff;
          dgbf[gb + 2 * H] = bg;
          dgbf[gb + 3 * H] = bo;
        }
      }
      if constexpr (!F32) {
        if (st16) {
          const uint4 v = *reinterpret_cast<const uint4*>(&dgt[srow][sg * XB + 8 * sh]);
          *reinterpret_cast<uint4*>(dgbf + ((long long)(b0 + srow) * T + t) * 8 * H +
                                    (long long)dir * H4 + (long long)sg * H + u0 + 8 * sh) = v;
        }
      }
#ifdef ASR_XG_DIAG_PREF1   // diagnostics build: inputs one step ahead, straight into place
      if (own && q + 1 < T) load_cell(q + 1, av, avh, cc, cp, dyv, &cp);
#else
      if (own && q + 2 < T) load_cell(q + 2, nav, navh, ncc, ncp, ndyv, &cp);   // cp: step q + 1's
#endif
    };
    for (int q = 0; q < T; ++q) {
      const int t = dir == 0 ? T - 1 - q : q;
      const bool act = own && t < len;
      float ig, fg, gg, og, omi, omf, omg2, omo;   // gates and 1 - s / 1 - g^2
      if constexpr (AH) {
        dec_sig((float)avh[0], ig, omi);
        dec_sig((float)avh[1], fg, omf);
        dec_tanh((float)avh[2], gg, omg2);
        dec_sig((float)avh[3], og, omo);
      } else {
        ig = av[0]; fg = av[1]; gg = av[2]; og = av[3];
        omi = 1.f - ig; omf = 1.f - fg; omg2 = 1.f - gg * gg; omo = 1.f - og;
      }
#ifndef ASR_XG_BWD_NOPRE
      // everything that does not depend on dh_t, formed while this wave waits
      // at B1 for the sweepers (the step's inputs are in registers since the
      // previous step): after B1 only dcell = dc + dh k_d and four products
      // remain on the step's critical path
      const float tc = F32 ? tanhf(cc) : ftanh(cc);
      float k_d = og * (1.f - tc * tc);
      float k_i = gg * ig * omi, k_f = cp * fg * omf, k_g = ig * omg2;
      float k_o = tc * og * omo;
      // pinned here: the compiler would otherwise sink them past B1 into the
      // active-cell branch, back onto the critical path
      asm volatile("" : "+v"(k_d), "+v"(k_i), "+v"(k_f), "+v"(k_g), "+v"(k_o), "+v"(fg));
#endif
      if (ct == 0) XG_TR_AT(q, 8, __builtin_amdgcn_s_memrealtime());
      __syncthreads();  // B1
      if (ct == 0) XG_TR_AT(q, 9, __builtin_amdgcn_s_memrealtime());
      // the abort word is tested after the step's math, so its LDS read
      // overlaps the partial-sum reads instead of preceding them
      const int dead = s_dead;
      float d_i = 0.f, d_f = 0.f, d_g = 0.f, d_o = 0.f;
      if (act) {
        float dh = dyv;
        if (q > 0) {   // in order: a pairwise tree measured slower (same-box A/B)
#pragma unroll
          for (int p = 0; p < NPG; ++p) dh += red[p][row][unit];
        }
        if (ddh) ddh[(((long long)b * T + t) * 2 + dir) * H + j] = dh;
#ifndef ASR_XG_BWD_NOPRE
        float dcell = __builtin_fmaf(dh, k_d, dc);
        // dcell as an opaque value, so the vectoriser cannot splat it out of
        // the HIGH half of a packed pair (op_sel:[x,1] -- the gfx950
        // co-residency hazard, tools/isa_check.py)
        asm volatile("" : "+v"(dcell));
        d_i = dcell * k_i;
        d_f = dcell * k_f;
        d_g = dcell * k_g;
        d_o = dh * k_o;
#else
        const float tc = F32 ? tanhf(cc) : ftanh(cc);
        float dcell = dc + dh * og * (1.f - tc * tc);
        if constexpr (!AH) asm volatile("" : "+v"(dcell));
        d_i = dcell * gg * ig * omi;
        d_f = dcell * cp * fg * omf;
        d_g = dcell * ig * omg2;
        d_o = dh * tc * og * omo;
#endif
        if (dcl) {
          float* o = dcl + ((((long long)b * T + t) * 2 + dir) * H + j) * 12;
          o[0] = d_i; o[1] = d_f; o[2] = d_g; o[3] = d_o;
          o[4] = ig; o[5] = fg; o[6] = gg; o[7] = og;
          o[8] = cc; o[9] = cp; o[10] = dyv; o[11] = dc;
        }
        dc = dcell * fg;
        sb_i += d_i;
        sb_f += d_f;
        sb_g += d_g;
        sb_o += d_o;
      } else {
        dc = 0.f;
      }
      if (dead) return;
      const uint16_t bi = f2bf(d_i), bff = f2bf(d_f), bg = f2bf(d_g), bo = f2bf(d_o);
      if constexpr (F32) {
        dgt[row][unit] = d_i;
        dgt[row][XB + unit] = d_f;
        dgt[row][2 * XB + unit] = d_g;
        dgt[row][3 * XB + unit] = d_o;
      } else {
        dgt[row][unit] = bi;
        dgt[row][XB + unit] = bff;
        dgt[row][2 * XB + unit] = bg;
        dgt[row][3 * XB + unit] = bo;
      }
#ifndef ASR_XG_DIAG_PREF1
      // step q + 1's inputs (loaded two steps ahead)
#pragma unroll
      for (int k = 0; k < 4; ++k) av[k] = nav[k];
      avh = navh;
      cc = ncc;
      cp = ncp;
      dyv = ndyv;
#endif
      if (ct == 0) XG_TR_AT(q, 10, __builtin_amdgcn_s_memrealtime());
      __syncthreads();  // B2
      if (io_pos == 0) step_io(q, t, d_i, d_f, d_g, d_o, bi, bff, bg, bo);
      __syncthreads();  // B3
      if (io_pos == 1) step_io(q, t, d_i, d_f, d_g, d_o, bi, bff, bg, bo);
      if (prog && (q == prog_q || q == prog_q2)) {
        // every dG store of steps <= q by this wave is complete and released
        // at agent scope (written back from this XCD's L2), then counted: a
        // reader on another stream that sees all arrivals reads final rows
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (lane == 0)
          __hip_atomic_fetch_add((gu64*)prog, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (own && dbpart) {  // per-utterance bias-gradient partials [B][8H]
      float* o = dbpart + (long long)b * 8 * H + (long long)dir * H4 + j;
      o[0] = sb_i;
      o[H] = sb_f;
      o[2 * H] = sb_g;
      o[3 * H] = sb_o;
    }
    return;
  }

  // --------------------------------- MFMA -----------------------------------
  __builtin_amdgcn_s_setprio(2);
  const int mw = wave - 4 - NCW;         // 0 .. NMW - 1
  const int kq = lane >> 4, ln = lane & 15;
  if constexpr (F32) {
    // A[m][k] = W_hh[kq H + u0 + k-step][16 mb + ln]: lane group kq = gate kq
    float wa[MB][NKS];
    {
      const float* W = dir ? whh_r : whh_f;
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const int mb = min(mw + NMW * i, HB - 1);
#pragma unroll
        for (int kst = 0; kst < NKS; ++kst)
          wa[i][kst] = W[(long long)(kq * H + u0 + kst) * H + 16 * mb + ln];
      }
    }
    __syncthreads();  // B0
    for (int q = 0; q < T; ++q) {
      __syncthreads();  // B1
      if (s_dead) return;
      __syncthreads();  // B2
      float bfk[NKS];   // B[k][n] = dG[row n][gate kq, unit k-step]
#pragma unroll
      for (int c = 0; c < NKS; c += 4) {
        const f32x4 d = *reinterpret_cast<const f32x4*>(&dgt[ln][XB * kq + c]);
        bfk[c] = d[0];
        bfk[c + 1] = d[1];
        bfk[c + 2] = d[2];
        bfk[c + 3] = d[3];
      }
      const unsigned tb = tag_bit(q);
      const long long obase = (((long long)(q & 1) * G + grp) * WPG + mem) * R;
      f32x4 acc[MB];
      auto mm = [&](int i) {
        acc[i] = mfma_f32(wa[i][0], bfk[0], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int kst = 1; kst < NKS; ++kst) acc[i] = mfma_f32(wa[i][kst], bfk[kst], acc[i]);
      };
      // two granules of (row ln, block mb): units 16 mb + 4 kq .. + 3
      const unsigned off0 = (unsigned)(((obase + ln) * (long long)H + 16 * mw + 4 * kq) * 4);
      auto publish = [&](auto aux) {
        auto st = [&](int i) {
          const int mb = mw + NMW * i;
          if (ln < R && mb < HB) {
            const u32x4 v = {(__float_as_uint(acc[i][0]) & ~1u) | tb, __float_as_uint(acc[i][1]),
                             (__float_as_uint(acc[i][2]) & ~1u) | tb, __float_as_uint(acc[i][3])};
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, off0 + 64u * NMW * i, 0,
                                                   decltype(aux)::value);
          }
        };
        mm(0);
#pragma unroll
        for (int i = 1; i < MB; ++i) {
          mm(i);
          __builtin_amdgcn_sched_barrier(0);
          st(i - 1);
          __builtin_amdgcn_sched_barrier(0);
        }
        st(MB - 1);
      };
      if (local)
        publish(std::integral_constant<int, 0>());
      else
        publish(std::integral_constant<int, (int)AUX_SC1>());
      __syncthreads();  // B3
    }
    return;
  }
  bf16x8 wa[MB][NKS];
  {
    const float* W = dir ? whh_r : whh_f;
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int mb = min(mw + NMW * i, HB - 1);
      const int m = 16 * mb + ln;
#pragma unroll
      for (int kst = 0; kst < NKS; ++kst) {
        u16x8 r;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const int k = 32 * kst + 8 * kq + jj;
          r[jj] = f2bf(W[(long long)((k / XB) * H + u0 + (k % XB)) * H + m]);
        }
        wa[i][kst] = as_bf16x8(r);
      }
    }
  }
  __syncthreads();  // B0
  for (int q = 0; q < T; ++q) {
    __syncthreads();  // B1
    if (s_dead) return;
    __syncthreads();  // B2
    if (mw == 0 && lane == 0) XG_TR_AT(q, 11, __builtin_amdgcn_s_memrealtime());
    bf16x8 bfk[NKS];
#pragma unroll
    for (int kst = 0; kst < NKS; ++kst)
      bfk[kst] = *reinterpret_cast<const bf16x8*>(&dgt[ln][32 * kst + 8 * kq]);
    const unsigned tb = tag_bit(q);
    const long long obase = (((long long)(q & 1) * G + grp) * WPG + mem) * R;
    // block by block, one block of lag: the MFMA pair of block i is issued
    // before block i - 1 is converted and stored, so the pair's latency hides
    // behind the previous block's conversion (a block's MFMAs, convert and store
    // back to back serialised the phase).  All MFMAs first and then the stores
    // (every granule leaves in one burst) measured 0.7 ms / step slower at 5x512.
    // Blocks past HB (wave-uniform) compute on a clamped fragment and store
    // nothing.
    f32x4 acc[MB];
    auto mm = [&](int i) {
      acc[i] = mfma_bf16(wa[i][0], bfk[0], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int kst = 1; kst < NKS; ++kst) acc[i] = mfma_bf16(wa[i][kst], bfk[kst], acc[i]);
    };
    // granule of (row ln, block mb): units 16 mb + 4 kq .. + 3
    const unsigned off0 = (unsigned)(((obase + ln) * (long long)hq + 4 * mw + kq) * 8);
    auto publish = [&](auto aux) {
      auto st = [&](int i) {
        const int mb = mw + NMW * i;
        if (ln < R && mb < HB) {  // C[m][n]: n = ln (row), m = 16 mb + 4 kq + r
          // one granule: units 16 mb + 4 kq .. + 3, tag bit in the first value
          const unsigned off = off0 + 32u * NMW * i;
          // (packed v_cvt_pk_bf16_f32 conversions here, three VALU instead of
          // about twelve, measured 35 us / launch SLOWER in a same-box A/B)
          const unsigned p01 = bf_with_lsb(acc[i][0], tb) | ((unsigned)f2bf(acc[i][1]) << 16);
          const unsigned p23 = f2bf(acc[i][2]) | ((unsigned)f2bf(acc[i][3]) << 16);
          const u32x2 v0 = {p01, p23};
          __builtin_amdgcn_raw_buffer_store_b64(v0, rs, off, 0, decltype(aux)::value);
        }
      };
      mm(0);
#pragma unroll
      for (int i = 1; i < MB; ++i) {
        mm(i);
        __builtin_amdgcn_sched_barrier(0);
        st(i - 1);
        __builtin_amdgcn_sched_barrier(0);
      }
      st(MB - 1);
    };
    if (local)  // plain: into this XCD's L2
      publish(std::integral_constant<int, 0>());
    else        // write-through
      publish(std::integral_constant<int, (int)AUX_SC1>());
    if (mw == 0 && lane == 0 && tr && q < XG_TR_STEPS)
      tr[((long long)blockIdx.x * XG_TR_STEPS + q) * XG_TR_K + 4] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();  // B3
  }
}

int xg_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 0;
  }
  return n;
}

// ASR_LSTM_XG=0 disables this path (A/B tests against lstm_persist.hip).
bool xg_enabled() {
  const char* e = getenv("ASR_LSTM_XG");
  return !(e && e[0] == '0') && !(getenv("ASR_LSTM_PERSIST") && getenv("ASR_LSTM_PERSIST")[0] == '0');
}

// rows per group for this shape, or 0 if the grid cannot be co-resident
int xg_rows(int B, int H) {
  if (H % 32 != 0 || H / XU > 64) return 0;
  const int ncu = xg_num_cus();
  const int wpg = H / XU;
  for (int R : {8, 16}) {
    const int G = 2 * ((B + R - 1) / R);
    if (G * wpg <= ncu) return R;
  }
  return 0;
}

template <typename K>
bool xg_fits(K kernel, int threads, size_t lds) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds) != hipSuccess)
    return false;
  return per_cu >= 1;
}

}  // namespace

void xg_trace_setup(hipStream_t s);

constexpr size_t XG_HDR = 256;  // abort word + placement registry, zeroed with the granules

// The caller's workspace is already zero (a per-step arena cleared by one fill
// for every layer pass, native_ops.rec_arena_begin): the next launch skips its
// own memset.  Thread-local like the other per-call settings.
thread_local int g_ws_zeroed = 0;

hipError_t xg_ws_clear(void* ws, size_t n, hipStream_t s) {
  if (g_ws_zeroed) {
    g_ws_zeroed = 0;
    return hipSuccess;
  }
  return hipMemsetAsync(ws, 0, n, s);
}

unsigned xg_next_epoch() {
  static unsigned e = 0;
  e = (e + 1) & 0xFFFu;
  return e;
}

// Backward launches are numbered 1, 2, ... (never 0: 0 means "no signal").
unsigned xg_bwd_seq(bool next) {
  static unsigned n = 0;
  if (next) n = n + 1 ? n + 1 : 1;
  return n;
}

// Gate for the weight-gradient GEMMs of ASR_OVERLAP_WGRAD=2: one 64-thread
// work-group (no LDS) that waits until backward launch `want` is resident, or
// about `max_ticks` of s_memrealtime (100 MHz) have passed.  The GEMMs queued
// behind it on the same stream then fill the room beside the recurrence's
// work-groups instead of taking CUs before the recurrence is placed.  Only
// timing depends on it.
__global__ void xg_wgrad_gate(unsigned want, unsigned long long max_ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    const unsigned v = __hip_atomic_load(&g_xg_resident, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((int)(v - want) >= 0) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(8);
  }
}

int xg_allow_local() {
  const char* e = getenv("ASR_XG_LOCAL");
  return !(e && e[0] == '0');
}

size_t lstm_xg_fwd_bytes(int B, int H) {
  const int R = xg_rows(B, H);
  if (!R) return 0;
  const long long rows = 2LL * ((B + R - 1) / R) * R;
  return XG_HDR + (size_t)2 * rows * (H / 4) * 8;
}

size_t lstm_xg_bwd_bytes(int B, int H) {
  const int R = xg_rows(B, H);
  if (!R) return 0;
  const long long rows = 2LL * ((B + R - 1) / R) * R;
  return XG_HDR + (size_t)2 * rows * (H / XU) * (H / 4) * 8;
}

// f32 layouts.  16 units per work-group with the row groups of the bf16 path
// (xg_rows), or, with ASR_XG32_XU=8, 16-row groups of 8 units where the chip
// holds that grid: every column of the f32 MFMA is then a real row and each
// work-group does half the MFMAs per step -- but the hand-offs carry twice the
// rows per poll and the backward sweep twice the producers, and the step
// measured SLOWER (att4x320 fp32: forward 1.90 -> 2.56 ms, backward 1.72 ->
// 2.90 ms per launch): the f32 recurrence is hand-off bound, not MFMA bound.
int xg32_units(int B, int H) {
  const char* e = getenv("ASR_XG32_XU");
  if (!(e && atoi(e) == 8)) return 16;
  if (H % 64 != 0 || H / 8 > 64) return 16;
  const int G = 2 * ((B + 15) / 16);
  return G * (H / 8) <= xg_num_cus() ? 8 : 16;
}
int xg32_rows(int B, int H) { return xg32_units(B, H) == 8 ? 16 : xg_rows(B, H); }

// f32 granules: two values per 8 B; rows rounded up to 16 covers every layout
size_t lstm_xg32_fwd_bytes(int B, int H) {
  if (!xg_rows(B, H)) return 0;
  const long long rows = 2LL * ((B + 15) / 16) * 16;
  return XG_HDR + (size_t)2 * rows * H * 4;
}
size_t lstm_xg32_bwd_bytes(int B, int H) {
  if (!xg_rows(B, H)) return 0;
  const long long rows = 2LL * ((B + 15) / 16) * 16;
  return XG_HDR + (size_t)2 * rows * (H / 8) * H * 4;
}

// f32 shapes: H a multiple of 64 (16 K slices of whole 16-B polls) up to 512
// forward, up to 384 backward (MB <= 6 M blocks per MFMA wave: 16 f32 A
// fragments per block must stay in registers beside the other roles' waves).
bool xg32_shape_ok(int H, bool backward) { return H % 64 == 0 && H <= (backward ? 384 : 512); }

// Reference-precision (f32) forward: 1 launched / eligible (dry), 0 not, -1 error.
int lstm_fwd_xg32_launch(int B, int T, int H, const int32_t* lens, const float* whh_f,
                         const float* whh_r, float* gx_act, float* y, float* cst, void* ws,
                         hipStream_t s, bool dry) {
  if (!xg_enabled()) return 0;
  const char* e = getenv("ASR_LSTM_XG32");
  if (e && e[0] == '0') return 0;
  if (!xg_rows(B, H) || !xg32_shape_ok(H, false)) return 0;
  const int xu = xg32_units(B, H);
  const int R = xg32_rows(B, H);
  const int nl = H / 64;
  const int grid = 2 * ((B + R - 1) / R) * (H / xu);
  int* hdr = (int*)ws;
  unsigned long long* g = (unsigned long long*)((char*)ws + XG_HDR);
  const int al = xg_allow_local();
#define ASR_XGF32(RR, NL, XV)                                                                    \
  do {                                                                                           \
    if (!xg_fits(lstm_fwd_xg<RR, NL, 4, true, XV>, 256 + RR * XV, XG_PIN_FWD)) return 0;          \
    if (dry) return 1;                                                                           \
    if (xg_ws_clear(ws, lstm_xg32_fwd_bytes(B, H), s) != hipSuccess) return -1;                  \
    xg_trace_setup(s);                                                                           \
    hipLaunchKernelGGL((lstm_fwd_xg<RR, NL, 4, true, XV>), dim3(grid), dim3(256 + RR * XV),      \
                       XG_PIN_FWD, s, B, T, H, lens, whh_f, whh_r, gx_act, y, cst, g, hdr,       \
                       (uint16_t*)nullptr, 0u, al);                                              \
  } while (0)
#define ASR_XGF32_N(RR, XV)                   \
  do {                                        \
    switch (nl) {                             \
      case 1: ASR_XGF32(RR, 1, XV); break;    \
      case 2: ASR_XGF32(RR, 2, XV); break;    \
      case 3: ASR_XGF32(RR, 3, XV); break;    \
      case 4: ASR_XGF32(RR, 4, XV); break;    \
      case 5: ASR_XGF32(RR, 5, XV); break;    \
      case 6: ASR_XGF32(RR, 6, XV); break;    \
      case 7: ASR_XGF32(RR, 7, XV); break;    \
      default: ASR_XGF32(RR, 8, XV); break;   \
    }                                         \
  } while (0)
  if (xu == 8) ASR_XGF32_N(16, 8);
  else if (R == 8) ASR_XGF32_N(8, 16);
  else ASR_XGF32_N(16, 16);
#undef ASR_XGF32_N
#undef ASR_XGF32
  return hipGetLastError() == hipSuccess ? 1 : -1;
}

// Reference-precision (f32) backward: f32 dG in place of the activations,
// per-utterance bias partials into dbpart (if given).
int lstm_bwd_xg32_launch(int B, int T, int H, const int32_t* lens, const float* whh_f,
                         const float* whh_r, const float* dy, float* act_dg, const float* cst,
                         void* ws, float* dbpart, hipStream_t s, bool dry) {
  if (!xg_enabled()) return 0;
  const char* e = getenv("ASR_LSTM_XG32");
  if (e && e[0] == '0') return 0;
  if (!xg_rows(B, H) || !xg32_shape_ok(H, true)) return 0;
  const int xb = xg32_units(B, H);
  const int R = xg32_rows(B, H);
  const int mb = (H / 16 + 3) / 4;
  const int grid = 2 * ((B + R - 1) / R) * (H / xb);
  int* hdr = (int*)ws;
  unsigned long long* g = (unsigned long long*)((char*)ws + XG_HDR);
  const unsigned ep = xg_bwd_seq(true);
  const int al = xg_allow_local();
  const size_t pin = XG_PIN_BWD;
#define ASR_XGB32(RR, M, XV)                                                                     \
  do {                                                                                           \
    if (!xg_fits(lstm_bwd_xg<RR, M, false, XV, true>, 256 + RR * XV + 256, pin)) return 0;       \
    if (dry) return 1;                                                                           \
    if (xg_ws_clear(ws, lstm_xg32_bwd_bytes(B, H), s) != hipSuccess) return -1;                  \
    xg_trace_setup(s);                                                                           \
    hipLaunchKernelGGL((lstm_bwd_xg<RR, M, false, XV, true>), dim3(grid),                        \
                       dim3(256 + RR * XV + 256), pin, s, B, T, H, lens, whh_f, whh_r, dy,      \
                       act_dg, cst, g, hdr, (uint16_t*)nullptr, dbpart, ep, al, 1, 0, 0,        \
                       (const h16x4*)nullptr, (const int*)nullptr, 0, 0, nullptr, -1, -1);       \
  } while (0)
#define ASR_XGB32_M(RR, XV)                 \
  do {                                      \
    if (mb <= 1) ASR_XGB32(RR, 1, XV);      \
    else if (mb <= 2) ASR_XGB32(RR, 2, XV); \
    else if (mb <= 3) ASR_XGB32(RR, 3, XV); \
    else if (mb <= 4) ASR_XGB32(RR, 4, XV); \
    else if (mb <= 5) ASR_XGB32(RR, 5, XV); \
    else ASR_XGB32(RR, 6, XV);              \
  } while (0)
  if (xb == 8) ASR_XGB32_M(16, 8);
  else if (R == 8) ASR_XGB32_M(8, 16);
  else ASR_XGB32_M(16, 16);
#undef ASR_XGB32_M
#undef ASR_XGB32
  return hipGetLastError() == hipSuccess ? 1 : -1;
}


// Returns 1 if launched (or, with dry, if this shape/device can take the
// path), 0 if not eligible, -1 on a launch error.  ws must hold
// lstm_xg_{fwd,bwd}_bytes; it is zeroed here before the launch.
int lstm_fwd_xg_launch(int B, int T, int H, const int32_t* lens, const float* whh_f,
                       const float* whh_r, float* gx_act, float* y, float* cst, void* ws,
                       uint16_t* ybf, hipStream_t s, bool dry) {
  if (!xg_enabled()) return 0;
  const int R = xg_rows(B, H);
  if (!R) return 0;
  // sweeper waves: 4 (ASR_XG_NSW=8: eight -- the MFMA phase after the hop
  // drops 0.32 -> 0.24 us but the cell's 8-way partial sum adds 0.08: no gain)
  const char* ns = getenv("ASR_XG_NSW");
  const int nsw = (ns && atoi(ns) == 8) ? 8 : 4;
  int ksw = (H / 32 + nsw - 1) / nsw;
  if (ksw > 8) return 0;
  if (getenv("ASR_XG_KSW")) ksw = std::max(ksw, atoi(getenv("ASR_XG_KSW")));  // diagnostics
  const int grid = 2 * ((B + R - 1) / R) * (H / XU);
  int* hdr = (int*)ws;
  unsigned long long* g = (unsigned long long*)((char*)ws + XG_HDR);
  const unsigned ep = xg_next_epoch();
  const int al = xg_allow_local();
#define ASR_XGF_N(RR, KS, NS, PIN)                                                              \
  do {                                                                                          \
    if (!xg_fits(lstm_fwd_xg<RR, KS, NS>, 64 * NS + RR * XU, PIN)) return 0;                     \
    if (dry) return 1;                                                                          \
    if (xg_ws_clear(ws, lstm_xg_fwd_bytes(B, H), s) != hipSuccess) return -1;                   \
    xg_trace_setup(s);                                                                          \
    hipLaunchKernelGGL((lstm_fwd_xg<RR, KS, NS>), dim3(grid), dim3(64 * NS + RR * XU), PIN, s,   \
                       B, T, H, lens, whh_f, whh_r, gx_act, y, cst, g, hdr, ybf, ep, al);        \
  } while (0)
#define ASR_XGF(RR, KS)                                            \
  do {                                                             \
    if (nsw == 8) ASR_XGF_N(RR, KS, 8, XG_PIN_FWD8);               \
    else ASR_XGF_N(RR, KS, 4, XG_PIN_FWD);                         \
  } while (0)
#define ASR_XGF_K(RR)                   \
  do {                                  \
    if (ksw <= 1) ASR_XGF(RR, 1);       \
    else if (ksw <= 2) ASR_XGF(RR, 2);  \
    else if (ksw <= 3) ASR_XGF(RR, 3);  \
    else if (ksw <= 4) ASR_XGF(RR, 4);  \
    else ASR_XGF(RR, 8);                \
  } while (0)
  if (R == 8) ASR_XGF_K(8);
  else ASR_XGF_K(16);
#undef ASR_XGF_K
#undef ASR_XGF
#undef ASR_XGF_N
  return hipGetLastError() == hipSuccess ? 1 : -1;
}

int lstm_bwd_xg_launch(int B, int T, int H, const int32_t* lens, const float* whh_f,
                       const float* whh_r, const float* dy, float* act_dg, const float* cst,
                       void* ws, uint16_t* dgbf, float* dbpart, hipStream_t s, bool dry,
                       bool dg_f32, const uint16_t* acth) {
  if (acth && (dg_f32 || !dgbf)) return 0;   // packed activations: bf16 dG only
  if (!xg_enabled()) return 0;
  const int R = xg_rows(B, H);
  if (!R) return 0;
  const int xb = xg_bwd_xu(R, H);
  const int mb = (H / 16 + xb / 4 - 1) / (xb / 4);   // M blocks per MFMA wave
  if (mb > 16) return 0;
  const int grid = 2 * ((B + R - 1) / R) * (H / xb);
  int* hdr = (int*)ws;
  unsigned long long* g = (unsigned long long*)((char*)ws + XG_HDR);
  const unsigned ep = xg_bwd_seq(true);
  const int al = xg_allow_local();
  const size_t pin = xg_pin_bwd();
  const char* li = getenv("ASR_XG_BWD_IO");   // cell I/O position (lstm_bwd_xg), A/B
  const int io_pos = (li && atoi(li) == 1) ? 1 : 0;
  const char* s16 = getenv("ASR_XG_DG_ST16");   // A/B: bf16 dG by 16-B stores from LDS
  const int st16 = (s16 && s16[0] == '0') ? 0 : 1;
#define ASR_XGB3(RR, M, AHV, XBV)                                                               \
  do {                                                                                          \
    if (!xg_fits(lstm_bwd_xg<RR, M, AHV, XBV>, 256 + (RR + 16) * XBV, pin)) {                   \
      if (pin != XG_PIN_BWD) xg_warn_pin_unfit(pin);                                             \
      return 0;                                                                                 \
    }                                                                                           \
    if (dry) return 1;                                                                          \
    if (xg_ws_clear(ws, lstm_xg_bwd_bytes(B, H), s) != hipSuccess) return -1;                   \
    xg_trace_setup(s);                                                                          \
    hipLaunchKernelGGL((lstm_bwd_xg<RR, M, AHV, XBV>), dim3(grid), dim3(256 + (RR + 16) * XBV),   \
                       pin, s,                                                                  \
                       B, T, H, lens, whh_f, whh_r, dy, act_dg, cst, g, hdr, dgbf, dbpart, ep,   \
                       al, (dg_f32 || !dgbf) ? 1 : 0, io_pos, st16, (const h16x4*)acth,         \
                       acth ? g_dyflag : nullptr, g_dyc0, (int)g_dyepoch,                        \
                       acth ? g_prog_ctr : nullptr, g_prog_q, g_prog_q2);                        \
  } while (0)
#define ASR_XGB2(RR, M, AHV)                                  \
  do {                                                        \
    bool done32 = false;                                      \
    if constexpr (RR == 8 && M <= 4) {                        \
      if (xb == 32) {                                         \
        ASR_XGB3(RR, M, AHV, 32);                             \
        done32 = true;                                        \
      }                                                       \
    }                                                         \
    if (!done32) ASR_XGB3(RR, M, AHV, 16);                    \
  } while (0)
#define ASR_XGB(RR, M)                        \
  do {                                        \
    if (acth) ASR_XGB2(RR, M, true);          \
    else ASR_XGB2(RR, M, false);              \
  } while (0)
#define ASR_XGB_M(RR)                  \
  do {                                 \
    if (mb <= 1) ASR_XGB(RR, 1);       \
    else if (mb <= 2) ASR_XGB(RR, 2);  \
    else if (mb <= 4) ASR_XGB(RR, 4);  \
    else if (mb <= 5) ASR_XGB(RR, 5);  \
    else if (mb <= 8) ASR_XGB(RR, 8);  \
    else ASR_XGB(RR, 16);              \
  } while (0)
  if (R == 8) ASR_XGB_M(8);
  else ASR_XGB_M(16);
#undef ASR_XGB_M
#undef ASR_XGB
#undef ASR_XGB2
#undef ASR_XGB3
  return hipGetLastError() == hipSuccess ? 1 : -1;
}


// Fused-projection forward (lstm_fwd_xgx): 1 if launched (dry: eligible), 0 if
// not eligible (ASR_FUSE_XPROJ=0, shape, Din % 8 or Din > 32 * 8 * KPW_MAX),
// -1 on a launch error.
constexpr int XGX_NPW = 6;   // 12 waves: 3 per SIMD, 170 registers per wave (8: 4 per SIMD, 128: spills)
int lstm_fwd_xgx_launch(int B, int T, int H, const int32_t* lens, const float* whh_f,
                        const float* whh_r, const uint16_t* x, int Din, const uint16_t* wih,
                        const float* b_ih, const float* b_hh, float* act, float* y, float* cst,
                        void* ws, uint16_t* ybf, hipStream_t s, bool dry, uint16_t* acth,
                        uint16_t* ydrop = nullptr, float drop_p = 0.f,
                        unsigned long long drop_seed = 0) {
  if (!xg_enabled()) return 0;
  const char* e = getenv("ASR_FUSE_XPROJ");
  if (e && e[0] == '0') return 0;
  const int R = xg_rows(B, H);
  if (R != 8) return 0;
  if (Din <= 0 || Din % 8 || Din > XGX_DMAX) return 0;
  if ((long long)B * T * Din * 2 >= 0x7fff0000LL) return 0;   // one buffer resource
  const int nkx = (Din + 31) / 32;
  const int kpw = (nkx + XGX_NPW - 1) / XGX_NPW;
  if (kpw > 6) return 0;
  const int nks = H / 32;
  const int ksw = (nks + 3) / 4;
  if (ksw > 4) return 0;   // H > 512: the W_hh + W_ih fragments would spill
  const int grid = 2 * ((B + R - 1) / R) * (H / XU);
  const int threads = 64 * 4 + R * XU + 64 * XGX_NPW;
  int* hdr = (int*)ws;
  unsigned long long* g = (unsigned long long*)((char*)ws + XG_HDR);
  const int al = xg_allow_local();
  const char* ll = getenv("ASR_XGX_LATE_LOAD");   // measured: -0.1..-0.35 ms/step (default)
  const int late = ll ? atoi(ll) : 1;
  const char* ds = getenv("ASR_XGX_DEFER_STORES");
  const int defer = ds ? atoi(ds) : 0;
#define ASR_XGX(KS, KP)                                                                         \
  do {                                                                                          \
    auto kfn = lstm_fwd_xgx<8, KS, 4, XGX_NPW, KP>;                                              \
    hipFuncAttributes fa;                                                                       \
    if (hipFuncGetAttributes(&fa, (const void*)kfn) != hipSuccess) return 0;                   \
    const size_t pin = fa.sharedSizeBytes >= 84 * 1024 ? 0 : 84 * 1024 - fa.sharedSizeBytes;   \
    if (!xg_fits(kfn, threads, pin)) return 0;                                                  \
    if (dry) return 1;                                                                          \
    if (xg_ws_clear(ws, lstm_xg_fwd_bytes(B, H), s) != hipSuccess) return -1;                   \
    xg_trace_setup(s);                                                                          \
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(threads), pin, s, B, T, H, lens, whh_f, whh_r, x,  \
                       Din, wih, b_ih, b_hh, act, y, cst, g, hdr, ybf, al, late, defer,          \
                       (h16x4*)acth, ydrop, drop_p, drop_seed);                                  \
  } while (0)
#define ASR_XGX_P(KS)                    \
  do {                                   \
    if (kpw <= 1) ASR_XGX(KS, 1);        \
    else if (kpw <= 2) ASR_XGX(KS, 2);   \
    else if (kpw <= 4) ASR_XGX(KS, 4);   \
    else ASR_XGX(KS, 6);                 \
  } while (0)
  if (ksw <= 2) ASR_XGX_P(2);
  else if (ksw <= 3) ASR_XGX_P(3);
  else ASR_XGX_P(4);
#undef ASR_XGX_P
#undef ASR_XGX
  return hipGetLastError() == hipSuccess ? 1 : -1;
}

// ASR_XG_TRACE=1: allocate the trace buffer once and publish its pointer.
void xg_tuning_setup(hipStream_t s) {
  static bool done = false;
  if (done) return;
  done = true;
  const char* a = getenv("ASR_XG_SLEEP");
  const char* b = getenv("ASR_XG_DELAY");
  const int sl = a ? atoi(a) : 1, dl = b ? atoi(b) : 0;
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_xg_sleep), &sl, sizeof(int), 0, hipMemcpyHostToDevice, s);
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_xg_delay), &dl, sizeof(int), 0, hipMemcpyHostToDevice, s);
}

void xg_trace_setup(hipStream_t s) {
  xg_tuning_setup(s);
  {  // read per launch (A/B within one process)
    static int last = -1;
    const char* c1 = getenv("ASR_XG_CELL_SC1");
    const int sc1 = c1 ? atoi(c1) : 0;
    if (sc1 != last) {
      last = sc1;
      (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_xg_cell_sc1), &sc1, sizeof(int), 0,
                                   hipMemcpyHostToDevice, s);
    }
  }
  static unsigned long long* buf = nullptr;
  if (!getenv("ASR_XG_TRACE") || buf) return;
  const size_t n = (size_t)XG_TR_WG * XG_TR_STEPS * XG_TR_K;
  if (hipMalloc(&buf, n * 8) != hipSuccess) return;
  (void)hipMemsetAsync(buf, 0, n * 8, s);
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_xg_trace), &buf, sizeof(buf), 0, hipMemcpyHostToDevice, s);
}

int lstm_xg_status(int* status, int clear, hipStream_t s) {
  int v = 0;
  if (hipMemcpyFromSymbolAsync(&v, HIP_SYMBOL(g_xg_status), sizeof(int), 0,
                               hipMemcpyDeviceToHost, s) != hipSuccess)
    return -1;
  if (hipStreamSynchronize(s) != hipSuccess) return -1;
  *status |= v;
  if (clear) {
    const int zero = 0;
    if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_xg_status), &zero, sizeof(int), 0,
                               hipMemcpyHostToDevice, s) != hipSuccess)
      return -1;
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
  }
  return 0;
}

// Device address of g_xg_status (stream-ordered gathers and clears, no host sync).
int* lstm_xg_status_word() {
  static void* p = nullptr;
  if (!p && hipGetSymbolAddress(&p, HIP_SYMBOL(g_xg_status)) != hipSuccess) p = nullptr;
  return (int*)p;
}

}  // namespace asr

// Diagnostics: copy the phase-timestamp trace (ASR_XG_TRACE=1) to host memory
// (XG_TR_WG * XG_TR_STEPS * XG_TR_K u64).  Returns the element count, 0 if off.
extern "C" long long asr_xg_trace_read(unsigned long long* host) {
  unsigned long long* buf = nullptr;
  if (hipMemcpyFromSymbol(&buf, HIP_SYMBOL(asr::g_xg_trace), sizeof(buf)) != hipSuccess || !buf)
    return 0;
  const size_t n = (size_t)XG_TR_WG * XG_TR_STEPS * XG_TR_K;
  if (host && hipMemcpy(host, buf, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (long long)n;
}

// The backward recurrence's dynamic-LDS pin for the launches that follow
// (kb in (80, 160]; 0 = ASR_XG_PIN_BWD_KB or the 140 KB default).  native_ops
// sets 84 while weight-gradient GEMMs are meant to co-reside (opt-in
// ASR_OVERLAP_WGRAD=2) and 0 otherwise: at 140 KB (+ 11 KB static) no kernel
// with more than 9 KB of LDS -- every GEMM / convolution kernel -- can share a
// CU with the recurrence.
extern "C" int asr_lstm_set_bwd_pin_kb(int kb) {
  ASR_REQUIRE(kb == 0 || (kb > 80 && kb <= 160), ASR_ERR_ARG, "lstm pin: %d KB", kb);
  asr::g_pin_bwd_kb = kb;
  return ASR_OK;
}

// dy of the backward recurrence launches that follow (asr_lstm_backward_dgbf_h
// only) is written concurrently by input-gradient GEMMs on another stream:
// processing steps [c0 k, c0 (k + 1)) -- dy rows t = q and t = T - 1 - q for
// those steps q -- are complete once flags[k] == epoch
// (set by asr_lstm_dy_signal after the chunk's GEMMs).  flags NULL: off.
extern "C" int asr_lstm_set_dy_flags(const int* flags, int c0, int epoch) {
  ASR_REQUIRE(!flags || (c0 > 0 && epoch != 0), ASR_ERR_ARG, "dy flags: c0 %d epoch %d", c0,
              epoch);
  asr::g_dyflag = flags;
  asr::g_dyc0 = c0;
  asr::g_dyepoch = (unsigned)epoch;
  return ASR_OK;
}

namespace asr {
namespace {
__global__ void dy_signal(int* flags, int k, int epoch) {
  if (threadIdx.x == 0)
    __hip_atomic_store(flags + k, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace
}  // namespace asr

// Stream-ordered: flags[k] = epoch once the work enqueued before it on
// `stream` is complete (one thread; the chunk's dy rows are then visible).
extern "C" int asr_lstm_dy_signal(int* flags, int k, int epoch, void* stream) {
  ASR_REQUIRE(flags && k >= 0 && epoch != 0, ASR_ERR_ARG, "dy signal");
  hipLaunchKernelGGL(asr::dy_signal, dim3(1), dim3(64), 0, (hipStream_t)stream, flags, k, epoch);
  return hipGetLastError() == hipSuccess ? ASR_OK : ASR_ERR_HIP;
}

// The next packed-activation backward launch (asr_lstm_backward_dgbf_h) adds 1
// to *counter per cell wave once the gate gradients of processing steps <= q
// are stored and released; counter NULL: off.  Stream-ordered launches only
// ever add, so a reader waits for the running total (asr_lstm_progress_gate).
// The workspace of the next tagged-granule launch on this thread is already
// zero (on: 1): it skips its memset.  Consumed by that launch; callers reset
// it after the call (a call that took another path leaves it set).
extern "C" int asr_lstm_ws_prezeroed(int on) {
  asr::g_ws_zeroed = on ? 1 : 0;
  return ASR_OK;
}

// Leading bytes of a recurrence workspace that a tagged-granule launch of
// [B, *, H] zeroes (header + granules; the rest of asr_lstm_workspace_bytes
// belongs to the per-step kernels, which clear their own).
extern "C" size_t asr_lstm_ws_zero_bytes(int B, int H) {
  if (B <= 0 || H <= 0) return 0;
  return std::max(std::max(asr::lstm_xg_fwd_bytes(B, H), asr::lstm_xg_bwd_bytes(B, H)),
                  std::max(asr::lstm_xg32_fwd_bytes(B, H), asr::lstm_xg32_bwd_bytes(B, H)));
}

extern "C" int asr_lstm_set_bwd_progress(unsigned long long* counter, int q) {
  ASR_REQUIRE(!counter || q >= 0, ASR_ERR_ARG, "bwd progress: q %d", q);
  asr::g_prog_ctr = counter;
  asr::g_prog_q = counter ? q : -1;
  asr::g_prog_q2 = -1;
  return ASR_OK;
}

// Two reporting steps q1 < q2: the counter gains one launch's arrivals at each.
extern "C" int asr_lstm_set_bwd_progress2(unsigned long long* counter, int q1, int q2) {
  ASR_REQUIRE(!counter || (q1 >= 0 && q2 > q1), ASR_ERR_ARG, "bwd progress: q %d, %d", q1, q2);
  asr::g_prog_ctr = counter;
  asr::g_prog_q = counter ? q1 : -1;
  asr::g_prog_q2 = counter ? q2 : -1;
  return ASR_OK;
}

// Arrivals one backward launch of this shape adds to the progress counter
// (cell waves x work-groups), 0 if the shape does not take the tagged-granule
// backward with the current units setting.
extern "C" long long asr_lstm_bwd_progress_arrivals(int B, int H) {
  const int R = asr::xg_rows(B, H);
  if (!R) return 0;
  const int xb = asr::xg_bwd_xu(R, H);
  return (long long)(2 * ((B + R - 1) / R) * (H / xb)) * (R * xb / 64);
}

namespace asr {
namespace {
// one lane waits (acquire, agent scope) until *ctr >= target; bounded by
// `ticks` of the 100 MHz clock: a timeout marks the recurrence as given up
// (g_xg_status: the training step that needed these rows is skipped, never
// computed from incomplete rows)
__global__ void progress_gate(const unsigned long long* ctr, unsigned long long target,
                              unsigned long long ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load((const gu64*)ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      atomicOr(&g_xg_status, 2);
      return;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}
}  // namespace
}  // namespace asr

// Enqueue on `stream`: return once the progress counter reaches `target`
// (bounded at ~2 s; a timeout sets the recurrence status word).
extern "C" int asr_lstm_progress_gate(const unsigned long long* counter, long long target,
                                      void* stream) {
  ASR_REQUIRE(counter && target > 0, ASR_ERR_ARG, "progress gate: args");
  hipLaunchKernelGGL(asr::progress_gate, dim3(1), dim3(64), 0, (hipStream_t)stream, counter,
                     (unsigned long long)target, 200000000ull);
  return hipGetLastError() == hipSuccess ? ASR_OK : ASR_ERR_HIP;
}

// Units per work-group of the backward recurrence for the launches that follow
// (0: ASR_XG_BWD_XU or 16; 16; 32 -- half the work-groups, see lstm_bwd_xg).
extern "C" int asr_lstm_set_bwd_units(int xu) {
  ASR_REQUIRE(xu == 0 || xu == 16 || xu == 32, ASR_ERR_ARG, "lstm units: %d", xu);
  asr::g_bwd_xu = xu;
  return ASR_OK;
}

// Work-groups of the tagged-granule backward recurrence for [B, *, H] with xu
// units per work-group (0: the current setting), 0 if the shape cannot take it.
extern "C" int asr_lstm_backward_grid(int B, int H, int xu) {
  const int R = asr::xg_rows(B, H);
  if (!R) return 0;
  int xb = 16;
  if (xu == 0) xb = asr::xg_bwd_xu(R, H);
  else if (xu == 32) xb = (R == 8 && H % 32 == 0 && (H / 16 + 3) / 4 <= 8) ? 32 : 0;
  else if (xu != 16) return 0;
  if (!xb) return 0;
  return 2 * ((B + R - 1) / R) * (H / xb);
}

// Diagnostics: the backward recurrence's dh / spin-count recorders (NULL: off).
// Stream-ordered: launches enqueued after this call on `stream` record into the
// given buffers ([B][T][2][H] f32; [ceil(B/R)][T][2][H/16] u32).
extern "C" int asr_lstm_debug_dh(float* dh, unsigned* spins, float* cell, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (hipMemcpyToSymbolAsync(HIP_SYMBOL(asr::g_xg_dbg_dh), &dh, sizeof(dh), 0,
                             hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyToSymbolAsync(HIP_SYMBOL(asr::g_xg_dbg_cell), &cell, sizeof(cell), 0,
                             hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyToSymbolAsync(HIP_SYMBOL(asr::g_xg_dbg_spins), &spins, sizeof(spins), 0,
                             hipMemcpyHostToDevice, s) != hipSuccess)
    return ASR_ERR_HIP;
  return ASR_OK;
}

// Which hand-off protocols the tagged-granule recurrence used since the last
// clear: bit 0 write-through (sc1, any placement), bit 1 XCD-local.
extern "C" int asr_lstm_xg_mode(int* mode, int clear) {
  if (!mode) return ASR_ERR_ARG;
  if (hipDeviceSynchronize() != hipSuccess) return ASR_ERR_HIP;
  if (hipMemcpyFromSymbol(mode, HIP_SYMBOL(asr::g_xg_mode), sizeof(int)) != hipSuccess)
    return ASR_ERR_HIP;
  if (clear) {
    const int zero = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(asr::g_xg_mode), &zero, sizeof(int)) != hipSuccess)
      return ASR_ERR_HIP;
  }
  return ASR_OK;
}

// Enqueue the wgrad gate on `stream`: it releases once the NEXT persistent
// backward recurrence launched on any stream is resident (bounded at ~5 ms).
// Diagnostics only (ASR_DIAG_SPIN, native_ops): work-groups that fill `lds`
// bytes of LDS with a pattern and rewrite / check it for `iters` rounds, as a
// stand-in for the co-resident weight-gradient GEMMs (no global memory
// traffic).  bad[0] counts pattern mismatches.
namespace asr {
__global__ void diag_lds_spin(int iters, int* bad) {
  extern __shared__ unsigned dl[];
  const int words = 16384;   // 64 KB
  unsigned err = 0;
  for (int it = 0; it < iters; ++it) {
    for (int i = threadIdx.x; i < words; i += blockDim.x) dl[i] = (unsigned)(i * 2654435761u) ^ it;
    __syncthreads();
    for (int i = threadIdx.x; i < words; i += blockDim.x)
      err += dl[(i * 7 + 1) % words] != ((unsigned)(((i * 7 + 1) % words) * 2654435761u) ^ it);
    __syncthreads();
  }
  if (err) atomicAdd(bad, (int)err);
}
}  // namespace asr

extern "C" int asr_diag_lds_spin(int nwg, int iters, int* bad, void* stream) {
  hipLaunchKernelGGL(asr::diag_lds_spin, dim3(nwg), dim3(256), 64 * 1024, (hipStream_t)stream,
                     iters, bad);
  return hipGetLastError() == hipSuccess ? ASR_OK : ASR_ERR_HIP;
}

// Diagnostics only (tests/test_coresidency_gpu.py): nwg work-groups of 256
// threads, each holding `lds_bytes` of dynamic LDS, that stay resident for
// `usec` microseconds (s_memrealtime, 100 MHz) and exit -- a stand-in for a
// long-lived kernel (an RCCL collective spinning on its peer) occupying CUs
// when a persistent recurrence is launched.  Bounded by its own clock.
namespace asr {
__global__ void diag_hold(unsigned long long ticks) {
  extern __shared__ unsigned hl[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) hl[0] = 0u;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}
}  // namespace asr

extern "C" int asr_diag_hold_cus(int nwg, int lds_bytes, int usec, void* stream) {
  ASR_REQUIRE(nwg > 0 && nwg <= 4096 && lds_bytes >= 4 && lds_bytes <= 160 * 1024 && usec >= 0 &&
                  usec <= 10000000, ASR_ERR_ARG, "diag_hold_cus: nwg %d lds %d usec %d", nwg,
              lds_bytes, usec);
  hipLaunchKernelGGL(asr::diag_hold, dim3(nwg), dim3(256), (size_t)lds_bytes, (hipStream_t)stream,
                     (unsigned long long)usec * 100ull);
  return hipGetLastError() == hipSuccess ? ASR_OK : ASR_ERR_HIP;
}

extern "C" int asr_lstm_wgrad_gate(void* stream) {
  const unsigned want = asr::xg_bwd_seq(false) + 1;
  hipLaunchKernelGGL(asr::xg_wgrad_gate, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     want ? want : 1u, 500000ull);
  return hipGetLastError() == hipSuccess ? ASR_OK : ASR_ERR_HIP;
}

// Forward layer pass with the input projection fused into the persistent
// recurrence (bf16 mode): x [B*T][Din] bf16 (rows (b, t) of the layer input,
// the dense staged GEMM operand), wih [8H][Din] bf16 ([W_ih fwd; W_ih rev]),
// b_ih / b_hh [8H]; act [B][T][8H] receives the post-activation gates (as
// gx_act of asr_lstm_forward after the call).  Returns ASR_ERR_UNSUPPORTED when
// the shape does not take this path (the caller then runs the GEMM +
// asr_lstm_forward).
extern "C" int asr_lstm_forward_x(const uint16_t* x, int Din, const uint16_t* wih,
                                  const float* b_ih, const float* b_hh, const float* whh_f,
                                  const float* whh_r, const int32_t* lens, int B, int T, int H,
                                  float* act, float* y, float* cst, uint16_t* ybf,
                                  void* workspace, size_t ws_bytes, void* stream) {
  ASR_REQUIRE(x && wih && b_ih && b_hh && whh_f && whh_r && lens && act && y && cst && workspace,
              ASR_ERR_ARG, "lstm_forward_x: null pointer");
  ASR_REQUIRE(B > 0 && T > 0 && H > 0 && Din > 0, ASR_ERR_ARG, "lstm_forward_x: bad shape");
  hipStream_t s = (hipStream_t)stream;
  if (asr::lstm_fwd_xgx_launch(B, T, H, lens, whh_f, whh_r, x, Din, wih, b_ih, b_hh, act, y, cst,
                               workspace, ybf, s, true, nullptr) != 1)
    return ASR_ERR_UNSUPPORTED;
  ASR_REQUIRE(ws_bytes >= asr::lstm_xg_fwd_bytes(B, H), ASR_ERR_WORKSPACE,
              "lstm_forward_x: workspace too small");
  const int slot = asr::prof_begin_launch(ASR_PROF_LSTM_FWD_SEQ, s, 0.0, ASR_PTAG_LSTM_FWD_XGX);
  const int rc = asr::lstm_fwd_xgx_launch(B, T, H, lens, whh_f, whh_r, x, Din, wih, b_ih, b_hh,
                                          act, y, cst, workspace, ybf, s, false, nullptr);
  ASR_REQUIRE(rc == 1, ASR_ERR_HIP, "lstm_forward_x: launch failed");
  asr::prof_end_launch(ASR_PROF_LSTM_FWD_SEQ, slot, s);
  asr::g_lstm_last_path[0] = 3;
  return ASR_OK;
}

// asr_lstm_forward_x writing the gate activations packed as fp16 (act_h
// [B][T][2][H][4]: i, f, g, o of one (utterance, frame, direction, unit) in
// one 8-B word) instead of f32 [B][T][8H]; the backward then reads them with
// asr_lstm_backward_dgbf_h.
extern "C" int asr_lstm_forward_xh(const uint16_t* x, int Din, const uint16_t* wih,
                                   const float* b_ih, const float* b_hh, const float* whh_f,
                                   const float* whh_r, const int32_t* lens, int B, int T, int H,
                                   uint16_t* act_h, float* y, float* cst, uint16_t* ybf,
                                   void* workspace, size_t ws_bytes, void* stream) {
  ASR_REQUIRE(x && wih && b_ih && b_hh && whh_f && whh_r && lens && act_h && y && cst &&
              workspace, ASR_ERR_ARG, "lstm_forward_xh: null pointer");
  ASR_REQUIRE(B > 0 && T > 0 && H > 0 && Din > 0, ASR_ERR_ARG, "lstm_forward_xh: bad shape");
  ASR_REQUIRE(((uintptr_t)act_h & 7) == 0, ASR_ERR_ARG, "lstm_forward_xh: act_h not 8-B aligned");
  hipStream_t s = (hipStream_t)stream;
  if (asr::lstm_fwd_xgx_launch(B, T, H, lens, whh_f, whh_r, x, Din, wih, b_ih, b_hh, nullptr, y,
                               cst, workspace, ybf, s, true, act_h) != 1)
    return ASR_ERR_UNSUPPORTED;
  ASR_REQUIRE(ws_bytes >= asr::lstm_xg_fwd_bytes(B, H), ASR_ERR_WORKSPACE,
              "lstm_forward_xh: workspace too small");
  const int slot = asr::prof_begin_launch(ASR_PROF_LSTM_FWD_SEQ, s, 0.0, ASR_PTAG_LSTM_FWD_XGX);
  const int rc = asr::lstm_fwd_xgx_launch(B, T, H, lens, whh_f, whh_r, x, Din, wih, b_ih, b_hh,
                                          nullptr, y, cst, workspace, ybf, s, false, act_h);
  ASR_REQUIRE(rc == 1, ASR_ERR_HIP, "lstm_forward_xh: launch failed");
  asr::prof_end_launch(ASR_PROF_LSTM_FWD_SEQ, slot, s);
  asr::g_lstm_last_path[0] = 3;
  return ASR_OK;
}

// asr_lstm_forward_xh for a layer whose consumer is the next BLSTM layer's
// staged bf16 input: y (the f32 output) may be NULL -- not written -- and ydrop
// (non-NULL) receives bf16(dropout(y)) with asr_dropout's mask for (drop_p,
// drop_seed) over the [B][T][2H] output, i.e. exactly what
// asr_convert_rows_bf16_dropout would stage from y.  ybf (bf16 y, the dW_hh
// operand) is required.
extern "C" int asr_lstm_forward_xh_drop(const uint16_t* x, int Din, const uint16_t* wih,
                                        const float* b_ih, const float* b_hh, const float* whh_f,
                                        const float* whh_r, const int32_t* lens, int B, int T,
                                        int H, uint16_t* act_h, float* y, float* cst,
                                        uint16_t* ybf, uint16_t* ydrop, float drop_p,
                                        unsigned long long drop_seed, void* workspace,
                                        size_t ws_bytes, void* stream) {
  ASR_REQUIRE(x && wih && b_ih && b_hh && whh_f && whh_r && lens && act_h && cst && ybf &&
              workspace, ASR_ERR_ARG, "lstm_forward_xh_drop: null pointer");
  ASR_REQUIRE(B > 0 && T > 0 && H > 0 && Din > 0, ASR_ERR_ARG, "lstm_forward_xh_drop: bad shape");
  ASR_REQUIRE(drop_p >= 0.f && drop_p < 1.f, ASR_ERR_ARG, "lstm_forward_xh_drop: p=%f",
              (double)drop_p);
  ASR_REQUIRE(((uintptr_t)act_h & 7) == 0 && ((uintptr_t)ybf & 3) == 0 &&
              ((uintptr_t)ydrop & 3) == 0, ASR_ERR_ARG, "lstm_forward_xh_drop: misaligned");
  hipStream_t s = (hipStream_t)stream;
  if (asr::lstm_fwd_xgx_launch(B, T, H, lens, whh_f, whh_r, x, Din, wih, b_ih, b_hh, nullptr, y,
                               cst, workspace, ybf, s, true, act_h) != 1)
    return ASR_ERR_UNSUPPORTED;
  ASR_REQUIRE(ws_bytes >= asr::lstm_xg_fwd_bytes(B, H), ASR_ERR_WORKSPACE,
              "lstm_forward_xh_drop: workspace too small");
  const int slot = asr::prof_begin_launch(ASR_PROF_LSTM_FWD_SEQ, s, 0.0, ASR_PTAG_LSTM_FWD_XGX);
  const int rc = asr::lstm_fwd_xgx_launch(B, T, H, lens, whh_f, whh_r, x, Din, wih, b_ih, b_hh,
                                          nullptr, y, cst, workspace, ybf, s, false, act_h, ydrop,
                                          drop_p, drop_seed);
  ASR_REQUIRE(rc == 1, ASR_ERR_HIP, "lstm_forward_xh_drop: launch failed");
  asr::prof_end_launch(ASR_PROF_LSTM_FWD_SEQ, slot, s);
  asr::g_lstm_last_path[0] = 3;
  return ASR_OK;
}

// act [B][T][8H] f32 (forward columns [0, 4H), reverse [4H, 8H)) from the
// packed fp16 activations of asr_lstm_forward_xh (for a backward that cannot
// take the tagged-granule recurrence).
namespace asr {
namespace {
__global__ void unpack_act_h(const h16x4* __restrict__ a, long long n, int H,
                             float* __restrict__ act) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long bt = i / (2LL * H);
    const int r = (int)(i - bt * 2LL * H), dir = r / H, j = r - dir * H;
    const h16x4 v = a[i];
    float* o = act + bt * 8LL * H + (long long)dir * 4 * H + j;
    float s, om;
    dec_sig((float)v[0], s, om);
    o[0] = s;
    dec_sig((float)v[1], s, om);
    o[H] = s;
    dec_tanh((float)v[2], s, om);
    o[2LL * H] = s;
    dec_sig((float)v[3], s, om);
    o[3LL * H] = s;
  }
}
}  // namespace
}  // namespace asr

extern "C" int asr_lstm_unpack_act_h(const uint16_t* act_h, int B, int T, int H, float* act,
                                     void* stream) {
  ASR_REQUIRE(act_h && act && B > 0 && T > 0 && H > 0, ASR_ERR_ARG, "lstm_unpack_act_h: args");
  const long long n = (long long)B * T * 2 * H;
  hipLaunchKernelGGL(asr::unpack_act_h, dim3((unsigned)std::min(8192LL, (n + 255) / 256)),
                     dim3(256), 0, (hipStream_t)stream, (const asr::h16x4*)act_h, n, H, act);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

// 1 when asr_lstm_forward_x takes this shape on this device, else 0.
extern "C" int asr_lstm_forward_x_ok(int B, int H, int Din) {
  if (B <= 0 || H <= 0 || Din <= 0) return 0;
  return asr::lstm_fwd_xgx_launch(B, 1, H, nullptr, nullptr, nullptr, nullptr, Din, nullptr,
                                  nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                  nullptr, true, nullptr) == 1;
}
