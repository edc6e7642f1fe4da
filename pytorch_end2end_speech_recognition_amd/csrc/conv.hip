// Tap-resident 3x3 convolution over zero-haloed channels-last pixels (the VGG
// front-end's convolutions, models/pytorch_v3/encoders/cnn.py:124-165) for
// gfx950, bf16 operands, f32 accumulation.
//
// The layer input is [P][Cin] bf16 over the padded pixel grid [B][T+2][F+2]
// (row pitch Fp = F + 2 pixels), so tap (kt, kf) of a 3x3 kernel is a constant
// row shift sign * ((kt - 1) Fp + (kf - 1)), and
//   out[p][n] = bias[n] + sum_tap sum_c in[p + shift(tap)][c] * w[n][tap Cin + c]
// is the implicit GEMM M = P, N = Cout, K = 9 Cin that asr_gemm runs with
// tap-addressed operands (cnn.hip).  There every 64-deep k-tile is a fresh
// global -> LDS load of the tile's rows at that tap's shift (nine reads of the
// same pixel rows per tile, one L2 round trip per k-tile: the 64-channel
// layers ran at 235 TF/s).  Here a persistent work-group owns a contiguous run
// of pixel tiles and keeps the input rows in an LDS ring of pixel rows: a tile
// of BM output pixels needs rows [m0 - Fp - 1, m0 + BM + Fp + 1); consecutive
// tiles share all but BM of them, so each tile loads only its BM new rows
// (issued one tile ahead), and all nine taps read the ring at their shift.
// The weights stream through a ring of 64-deep k-slices ([Cout][64] bf16,
// L2-resident: every work-group reads the same few hundred KB).
//
// Roles: out^T = W X^T on the MFMA (A = weight rows = output channels, B =
// pixel rows), so a lane's accumulator holds four consecutive channels of one
// pixel and the epilogue writes 16-B (f32) / 8-B (bf16) pieces of pixel rows.
// The k order (tap-major, 32-deep MFMA steps in increasing k) is the tap GEMM's,
// so the f32 sums equal asr_gemm's (bit-equal on integer operands; the MFMA is
// order-insensitive to swapping its A and B roles).
#include <algorithm>
#include <cstdlib>

#include "mfma.h"
#include "prof.h"

namespace asr {
namespace {

constexpr int TR_NT = 256;   // four waves, one per SIMD
constexpr unsigned TR_OOB = 0x7ffffff0u;

typedef __attribute__((address_space(3))) void tr_lds_void_t;
typedef __attribute__((ext_vector_type(4))) unsigned int tr_u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int tr_u32x2;

struct TrArgs {
  const void* in;
  const void* w;
  const float* bias;
  void* out;
  int P;        // padded pixel rows
  int Fp;       // row pitch of the pixel grid (F + 2)
  int sign;     // +1: forward taps, -1: mirrored (input gradient)
  int ntiles;   // ceil(P / BM)
  int RC;       // LDS ring capacity in pixel rows (multiple of 16)
  int RCB;      // a multiple of RC >= Fp + 17 (keeps ring slots of negative rows >= 0)
  unsigned in_bytes, w_bytes, out_bytes;
};

// One 16-B-per-lane buffer -> LDS DMA: lane l's 16 bytes land at LDS byte
// lds_addr + 16 l.  (In inline asm: hipcc keeps neither M0 nor the DMA's
// counter across it; completion is waited for by the caller's vmcnt.)
__device__ __forceinline__ void tr_dma16(unsigned voff, __amdgpu_buffer_rsrc_t rs,
                                         unsigned lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(lds_addr)
      : "memory");
}

__device__ __forceinline__ unsigned tr_lds(const char* p) {
  return (unsigned)(uintptr_t)(const tr_lds_void_t*)p;
}

template <int N>
__device__ __forceinline__ void tr_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most n vector-memory operations of this wave are outstanding
// (n is one of the few values the schedule below produces)
__device__ __forceinline__ void tr_wait(int n) {
  switch (n) {
    case 0: tr_vmcnt<0>(); break;
    case 2: tr_vmcnt<2>(); break;
    case 4: tr_vmcnt<4>(); break;
    case 6: tr_vmcnt<6>(); break;
    case 8: tr_vmcnt<8>(); break;
    case 10: tr_vmcnt<10>(); break;
    case 12: tr_vmcnt<12>(); break;
    case 14: tr_vmcnt<14>(); break;
    case 16: tr_vmcnt<16>(); break;
    case 18: tr_vmcnt<18>(); break;
    case 20: tr_vmcnt<20>(); break;
    case 22: tr_vmcnt<22>(); break;
    case 24: tr_vmcnt<24>(); break;
    case 26: tr_vmcnt<26>(); break;
    case 28: tr_vmcnt<28>(); break;
    case 30: tr_vmcnt<30>(); break;
    case 32: tr_vmcnt<32>(); break;
    case 36: tr_vmcnt<36>(); break;
    case 40: tr_vmcnt<40>(); break;
    default: tr_vmcnt<0>(); break;   // unreachable for the shapes below; safe
  }
}

// 16 rows x 32 k fragment of a [rows][64] bf16 image with 128-B rows whose
// 16-B chunk c of row r sits at chunk c ^ ((r >> 1) & 7) (conflict-free
// ds_read_b128 over 16 consecutive rows); `row` is this lane's row.
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int row, int kk, int lane) {
  const int c = (4 * kk + (lane >> 4)) ^ ((row >> 1) & 7);
  return __builtin_bit_cast(bf16x8, *(const tr_u32x4*)(img + row * 128 + c * 16));
}

// CIN, COUT in {64, 128}; WPX pixels per wave (BM = 4 WPX per tile); NW
// weight-ring slots (NW - 1 k-slices in flight), or NW = 0: the whole weight
// image resident in LDS (loaded once; one barrier per tile instead of one per
// k-slice -- the 64 -> 64 layers, whose 72 KB image fits beside the ring).
template <int CIN, int COUT, int WPX, int NW, bool OUT_BF16>
__global__ void __launch_bounds__(TR_NT) conv3x3_tr(TrArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NCB = CIN / 64;            // 64-channel blocks of a pixel row
  constexpr int BM = 4 * WPX;              // output pixels per tile
  constexpr int KT = 9 * NCB;              // 64-deep k-slices per tile
  constexpr int NI = COUT / 16, NJ = WPX / 16;
  constexpr int WSLOT = COUT * 128;        // bytes per weight slot
  constexpr int NBW = COUT / 32;           // weight DMAs per wave per slot (COUT / 8 blocks)
  constexpr int NH = BM * NCB / 32;        // halo DMAs per wave per tile (BM / 8 blocks x NCB)
  constexpr int NST = NI * NJ;             // epilogue stores per wave per tile
  static_assert(NH * 4 * 8 == BM * NCB, "halo blocks split evenly over the waves");

  const int RC = a.RC;
  char* halo = smem;                               // [NCB][RC][64] bf16
  char* wring = smem + (size_t)NCB * RC * 128;     // [NW][COUT][64] bf16
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = gridDim.x, g = blockIdx.x;
  const int t_beg = (int)((long long)a.ntiles * g / G);
  const int t_end = (int)((long long)a.ntiles * (g + 1) / G);
  if (t_beg >= t_end) return;
  const __amdgpu_buffer_rsrc_t rin =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.in), 0, (int)a.in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rwt =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, (int)a.w_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rout =
      __builtin_amdgcn_make_buffer_rsrc(a.out, 0, (int)a.out_bytes, 0x00020000);
  const int H1 = a.Fp + 1;   // largest |shift|

  // pixel rows [p0, p0 + 8 nblk) (p0 a multiple of 8, may be negative) into the
  // ring: DMA d of the work-group covers rows p0 + 8 (d / NCB) .. + 7, channel
  // block d % NCB; wave w issues d = w, w + 4, ...
  auto load_rows = [&](int p0, int nblk) {
    for (int d = w; d < nblk * NCB; d += 4) {
      const int blk = d / NCB, cb = d - blk * NCB;
      const int q0 = p0 + 8 * blk;
      const int s0 = (q0 + a.RCB) % RC;   // multiple of 8
      const int p = q0 + (lane >> 3), s = s0 + (lane >> 3);
      const int lc = (lane & 7) ^ ((s >> 1) & 7);
      unsigned voff = TR_OOB;
      if (p >= 0 && p < a.P) voff = (unsigned)(((long long)p * CIN + cb * 64 + 8 * lc) * 2);
      tr_dma16(voff, rin, tr_lds(halo + ((size_t)cb * RC + s0) * 128));
    }
  };
  // weight k-slice kq (k = 64 kq .. 64 kq + 63 of every output channel) into slot
  auto load_w = [&](int kq, int slot) {
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      const int blk = w * NBW + i;
      const int r = blk * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const unsigned voff = (unsigned)((r * (9 * CIN) + kq * 64 + 8 * c) * 2);
      tr_dma16(voff, rwt, tr_lds(wring + slot * WSLOT + blk * 1024));
    }
  };
  auto lo_row = [&](int m) { return ((m * BM - H1) >> 3) << 3; };          // floor to 8
  auto hi_row = [&](int m) { return ((m * BM + BM + H1 + 7) >> 3) << 3; };  // ceil to 8

  // prologue: the first tile's rows, weight slices 0 .. NW - 2 (all of them
  // when resident)
  load_rows(lo_row(t_beg), (hi_row(t_beg) - lo_row(t_beg)) >> 3);
  const int NKT = (t_end - t_beg) * KT;
  if constexpr (NW == 0) {
#pragma unroll
    for (int j = 0; j < KT; ++j) load_w(j, j);
  } else {
#pragma unroll
    for (int j = 0; j < NW - 1; ++j)
      if (j < NKT) load_w(j % KT, j);
  }

  // bias of this lane's channels, read before the loop (a global load inside it
  // would make the compiler drain the DMAs in flight before the epilogue)
  float bias4[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias4[i][r] = a.bias ? a.bias[16 * i + 4 * (lane >> 4) + r] : 0.f;
  // per-lane fragment addresses that never change: the weight rows (bytes
  // within a slot) and the swizzle-free chunk part of the pixel-row reads
  int woff[NI][2];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r = 16 * i + (lane & 15);
      woff[i][kk] = r * 128 + (((4 * kk + (lane >> 4)) ^ ((r >> 1) & 7)) << 4);
    }
  const int cpart0 = (lane >> 4) << 4, cpart1 = (4 + (lane >> 4)) << 4;
  const int sh_t = a.Fp * a.sign, sh_f = a.sign;   // tap (kt, kf) shift = (kt-1) sh_t + (kf-1) sh_f

  for (int m = t_beg; m < t_end; ++m) {
    const bool more = m + 1 < t_end, prev = m > t_beg;
    const int it0 = (m - t_beg) * KT;
    const int pb = m * BM + w * WPX + (lane & 15);
    int bslot[NJ];   // ring slot of this lane's pixel row of fragment j (shift 0)
#pragma unroll
    for (int j = 0; j < NJ; ++j) bslot[j] = (pb + 16 * j + a.RCB) % RC;
    f32x4 acc[NI][NJ];
#pragma unroll
    for (int kq = 0; kq < KT; ++kq) {
      const int it = it0 + kq;
      if constexpr (NW == 0) {
        // resident weights: per tile, wait for this tile's rows (the previous
        // tile's epilogue stores may stay in flight), one barrier, then the
        // next tile's rows go out
        if (kq == 0) {
          if (prev) tr_vmcnt<NST>();
          else tr_vmcnt<0>();
          __syncthreads();
          if (more) load_rows(hi_row(m), BM / 8);
        }
      } else {
        // wait for weight slice `it`: everything this wave issued after it may stay
        // in flight -- later slices, the halo batch of the next tile (issued right
        // after slice it0 + NW - 1) and the previous tile's epilogue stores
        {
          int n = NBW * min(NW - 2, NKT - 1 - it);
          if (kq >= 1 && kq <= NW - 1 && more) n += NH;
          if (kq <= NW - 2 && prev) n += NST;
          tr_wait(n);
        }
        __syncthreads();
        if (it + NW - 1 < NKT) load_w((kq + NW - 1) % KT, (it + NW - 1) % NW);
        if (kq == 0 && more) load_rows(hi_row(m), BM / 8);
      }

      const int tap = kq / NCB, cb = kq % NCB;
      const int sh = (tap / 3 - 1) * sh_t + (tap % 3 - 1) * sh_f;
      const char* hb = halo + (size_t)cb * RC * 128;
      const char* wb = wring + (NW == 0 ? kq : it % (NW == 0 ? 1 : NW)) * WSLOT;
      int ra[NJ], sw[NJ];   // row byte address and swizzle (<< 4) of fragment j's rows
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        int s = bslot[j] + sh;
        s = s >= RC ? s - RC : s;
        s = s < 0 ? s + RC : s;
        ra[j] = s << 7;
        sw[j] = (s << 3) & 0x70;
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 fa[NI], fb[NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i)
          fa[i] = __builtin_bit_cast(bf16x8, *(const tr_u32x4*)(wb + woff[i][kk]));
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          fb[j] = __builtin_bit_cast(
              bf16x8, *(const tr_u32x4*)(hb + ra[j] + ((kk ? cpart1 : cpart0) ^ sw[j])));
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = mfma_bf16(fa[i], fb[j],
                                  (kq == 0 && kk == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j]);
      }
    }

    // epilogue: lane = (pixel 16 j + lane & 15, channels 16 i + 4 (lane >> 4) .. + 3);
    // every lane issues every store (out-of-range pixels at an out-of-range
    // offset, dropped by the buffer) so the store count the waits assume holds
    const int c4 = 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const float* b4 = bias4[i];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int p = pb + 16 * j;
        const long long e = (long long)p * COUT + 16 * i + c4;
        const f32x4 v = acc[i][j];
        if constexpr (OUT_BF16) {
          const unsigned voff = p < a.P ? (unsigned)(e * 2) : TR_OOB;
          const tr_u32x2 pk = {(unsigned)f2bf(v[0] + b4[0]) | ((unsigned)f2bf(v[1] + b4[1]) << 16),
                               (unsigned)f2bf(v[2] + b4[2]) | ((unsigned)f2bf(v[3] + b4[3]) << 16)};
          __builtin_amdgcn_raw_buffer_store_b64(pk, rout, voff, 0, 0);
        } else {
          const unsigned voff = p < a.P ? (unsigned)(e * 4) : TR_OOB;
          const tr_u32x4 pk = {__float_as_uint(v[0] + b4[0]), __float_as_uint(v[1] + b4[1]),
                               __float_as_uint(v[2] + b4[2]), __float_as_uint(v[3] + b4[3])};
          __builtin_amdgcn_raw_buffer_store_b128(pk, rout, voff, 0, 0);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Weight gradient of the same convolution, tap-resident:
//   packed[n][tap Cin + c] = sum_p dz[p][n] * x[p + shift(tap)][c]   (shift sign +1)
// (the dW image asr_gemm forms as dz^T X over K = P pixel rows; unpacked into
// the Conv2d weight gradient by asr_conv_weight_unpack_acc_pad).  A work-group
// owns one block of 64 output channels (n) and a contiguous chunk of pixels:
// it streams 64-pixel tiles of dz (its 64 channels) and the chunk's x rows
// through LDS rings and holds the block's whole 64 x 9 Cin partial image in
// accumulators (Cin / 16 waves, each 64 x 144: nine 16-column tiles of the
// tap-major columns); the per-chunk partials go to a slab, summed in a fixed
// order by tr_wgrad_reduce.  Both MFMA operands are pixel-major (k = pixel
// row), read as transposed fragments (ds_read_b64_tr_b16) from images with
// 128-B rows whose 32-B granule G sits at G ^ trh(row) -- conflict-free for
// the eight rows of a transposed read at ANY row alignment (the nine taps
// read the x ring at nine different shifts).
// ---------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(4))) short tr_v4s;
typedef __attribute__((address_space(3))) tr_v4s tr_lds_v4s;
typedef __attribute__((ext_vector_type(8))) short tr_v8s;

__device__ __forceinline__ int trh(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }

// transposed fragment: lane l gets [m = 16 G + (l & 15)][k = 8 (l >> 4) + 0..7] of an image
// whose k-rows (pixels) are 128-B rows; s_lo / s_hi: this lane's rows for k = 8 (l >> 4) + q
// and + 4 + q, q = (l >> 2) & 3
__device__ __forceinline__ bf16x8 tr_tfrag(const char* img, int s_lo, int s_hi, int G, int lane) {
  const int p = lane & 3;
  const char* a0 = img + s_lo * 128 + ((G ^ trh(s_lo)) << 5) + 8 * p;
  const char* a1 = img + s_hi * 128 + ((G ^ trh(s_hi)) << 5) + 8 * p;
  const tr_v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_lds_v4s*)a0);
  const tr_v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_lds_v4s*)a1);
  const tr_v8s v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

struct TrwArgs {
  const void* x;     // [P][CIN] bf16
  const void* dz;    // [P][COUT] bf16
  float* slab;       // [S][NG][64][9 CIN] f32
  int P, Fp, S, RC, RCB;
  unsigned x_bytes, dz_bytes;
};

constexpr int TRW_BK = 64;   // pixels per k-tile
constexpr int TRW_D = 3;     // k-tiles in flight ahead of the one computed

// CIN / 16 waves; grid = S chunks x NG = COUT / 64 channel blocks
template <int CIN, int COUT>
__global__ void __launch_bounds__(CIN * 4) conv3x3_tr_wgrad(TrwArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NCB = CIN / 64, NWV = CIN / 16, NG = COUT / 64;
  constexpr int NDZ = TRW_D + 1;                 // dz ring slots
  constexpr int DZSLOT = TRW_BK * 128;           // [64 pixels][64 channels] bf16
  constexpr int NLX = 8 * NCB / NWV, NLZ = 8 / NWV;   // DMAs per wave per k-tile (x rows, dz rows)
  static_assert(NLX * NWV == 8 * NCB && NLZ * NWV == 8, "DMAs split evenly over the waves");
  constexpr int NL = NLX + NLZ;
  const int RC = a.RC;
  char* xr = smem;                                  // [NCB][RC][64]
  char* zr = smem + (size_t)NCB * RC * 128;         // [NDZ][64][64]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cob = blockIdx.x % NG, split = blockIdx.x / NG;
  if (split >= a.S) return;
  const int cbeg = (int)(((long long)a.P * split / a.S) >> 3) << 3;
  const int cend = split + 1 == a.S ? a.P : (int)(((long long)a.P * (split + 1) / a.S) >> 3) << 3;
  const int H1 = a.Fp + 1;
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rz =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.dz), 0, (int)a.dz_bytes, 0x00020000);
  const int nkt = (cend - cbeg + TRW_BK - 1) / TRW_BK;

  // 8 pixel rows [q0, q0 + 8) of x, channel block cb, into the x ring
  auto dma_x = [&](int q0, int cb) {
    const int s0 = (q0 + a.RCB) % RC;
    const int p = q0 + (lane >> 3), s = s0 + (lane >> 3);
    const int lg = ((lane & 7) >> 1) ^ trh(s);          // logical 32-B granule
    const int lc = 2 * lg + (lane & 1);
    unsigned voff = TR_OOB;
    if (p >= 0 && p < a.P) voff = (unsigned)(((long long)p * CIN + cb * 64 + 8 * lc) * 2);
    tr_dma16(voff, rx, tr_lds(xr + ((size_t)cb * RC + s0) * 128));
  };
  // 8 pixel rows of dz (this block's 64 channels) into row r0 of dz slot
  auto dma_z = [&](int q0, int slot, int r0) {
    const int p = q0 + (lane >> 3), r = r0 + (lane >> 3);
    const int lg = ((lane & 7) >> 1) ^ trh(r);
    const int lc = 2 * lg + (lane & 1);
    unsigned voff = TR_OOB;
    if (p < cend) voff = (unsigned)(((long long)p * COUT + cob * 64 + 8 * lc) * 2);
    tr_dma16(voff, rz, tr_lds(zr + slot * DZSLOT + r0 * 128));
  };
  // k-tile t's loads: the x rows new to it and its dz rows, NL DMAs per wave
  const int lo0 = ((cbeg - H1) >> 3) << 3;
  const int hi0 = ((cbeg + TRW_BK + H1 + 7) >> 3) << 3;
  auto load_tile = [&](int t) {
    const int xb = hi0 + (t - 1) * TRW_BK;   // x rows [xb, xb + 64) (t >= 1)
#pragma unroll
    for (int i = 0; i < NLX; ++i) {
      const int d = w * NLX + i, blk = d / NCB, cb = d - blk * NCB;
      dma_x(xb + 8 * blk, cb);
    }
#pragma unroll
    for (int i = 0; i < NLZ; ++i) {
      const int blk = w * NLZ + i;
      dma_z(cbeg + t * TRW_BK + 8 * blk, t % NDZ, 8 * blk);
    }
  };
  // prologue: x rows [lo0, hi0) (tile 0's), dz of tile 0; then tiles 1 .. D - 1
  for (int d = w; d < ((hi0 - lo0) >> 3) * NCB; d += NWV) dma_x(lo0 + 8 * (d / NCB), d % NCB);
  for (int blk = w; blk < 8; blk += NWV) dma_z(cbeg + 8 * blk, 0, 8 * blk);
  for (int t = 1; t < TRW_D; ++t)
    if (t < nkt) load_tile(t);

  // wave w owns channel tile w of x (16 channels: 64-channel half w >> 2,
  // granule w & 3) for all nine taps: acc[i][tap] = rows 16 i .. of the block,
  // columns tap CIN + 16 w ..
  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kq = (lane >> 2) & 3, kg = lane >> 4, p8 = 8 * (lane & 3);
  const int G = w & 3;
  const char* xh = xr + (size_t)(w >> 2) * RC * 128;
  // the swizzle of a row depends on its bits 1 and 3 only, which neither the
  // 64-row advance per k-tile nor the ring wrap (RC % 16 == 0) changes: per tap
  // the granule offsets of this lane's lo / hi rows are fixed for the kernel
  int tzl[9], tzh[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int r0 = cbeg + 8 * kg + kq + a.RCB + (tap / 3 - 1) * a.Fp + (tap % 3 - 1);
    tzl[tap] = ((G ^ trh(r0)) << 5) + p8;
    tzh[tap] = ((G ^ trh(r0 + 4)) << 5) + p8;
  }
  // dz fragment offsets within a slot (rows 32 kk + 8 kg + kq and + 4, granule i)
  int zo[4][2][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = 32 * kk + 8 * kg + kq + 4 * h;
        zo[i][kk][h] = r * 128 + ((i ^ trh(r)) << 5) + p8;
      }
  int xb = (cbeg + 8 * kg + kq + a.RCB) % RC;   // ring slot of this lane's row (shift 0)
  auto rd = [&](const char* base, int off_lo, int off_hi) {
    const tr_v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_lds_v4s*)(base + off_lo));
    const tr_v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_lds_v4s*)(base + off_hi));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto up = [&](int v) { return v >= RC ? v - RC : v; };

  for (int t = 0; t < nkt; ++t) {
    // wait for tile t: tiles t + 1 .. t + D - 1 may stay in flight
    {
      const int after = min(TRW_D - 1, nkt - 1 - t);
      if (after >= 2) tr_vmcnt<2 * NL>();
      else if (after == 1) tr_vmcnt<NL>();
      else tr_vmcnt<0>();
    }
    __syncthreads();
    if (t + TRW_D < nkt) load_tile(t + TRW_D);
    const char* zs = zr + (t % NDZ) * DZSLOT;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = rd(zs, zo[i][kk][0], zo[i][kk][1]);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int sh = (tap / 3 - 1) * a.Fp + (tap % 3 - 1);
        int s = xb + sh + 32 * kk;
        s = s < 0 ? s + RC : up(s);
        const int s4 = up(s + 4);
        const bf16x8 fb = rd(xh, (s << 7) + tzl[tap], (s4 << 7) + tzh[tap]);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][tap] = mfma_bf16(fa[i], fb, acc[i][tap]);
      }
    }
    xb = up(xb + TRW_BK);
  }
  // partial image of this chunk: rows n = 16 i + 4 (l >> 4) + r, columns 16 jt + (l & 15)
  float* o = a.slab + ((size_t)split * NG + cob) * 64 * (9 * CIN);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jn = 0; jn < 9; ++jn)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        o[(size_t)(16 * i + 4 * (lane >> 4) + r) * (9 * CIN) + jn * CIN + 16 * w + (lane & 15)] =
            acc[i][jn][r];
}

// packed[n][k] = sum over chunks s of slab[s][n / 64][n % 64][k], fixed order:
// thread (column group cg = tid % 16, chunk lane q = tid / 16) of a 256-thread
// block sums chunks q, q + 16, ... of its float4 column in order, the 16 lanes
// are then summed in order q = 0 .. 15 (deterministic; every chunk row is read
// by 16 x more threads than one sequential sum per column)
__global__ void __launch_bounds__(256) tr_wgrad_reduce(const float* __restrict__ slab, int S,
                                                       int NG, int K, float* __restrict__ packed) {
  __shared__ float4 part[16][16];
  const int cg = threadIdx.x & 15, q = threadIdx.x >> 4;
  const long long i4 = (long long)blockIdx.x * 16 + cg;   // float4 column
  const long long n4 = (long long)NG * 64 * K / 4;
  const long long blk4 = n4;                              // float4s per chunk
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < n4)
    for (int c = q; c < S; c += 16) {
      const float4 v = reinterpret_cast<const float4*>(slab)[c * blk4 + i4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  part[q][cg] = s;
  __syncthreads();
  if (q == 0 && i4 < n4) {
    float4 t = part[0][cg];
#pragma unroll
    for (int j = 1; j < 16; ++j) {
      const float4 v = part[j][cg];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    reinterpret_cast<float4*>(packed)[i4] = t;
  }
}

// zero the one-pixel halo of a channels-last padded grid [B][T+2][F+2][C]
// (the interior is written by the producing kernel): 16-B stores
__global__ void zero_halo(char* __restrict__ buf, int B, int T, int F, int rowbytes) {
  const int per_b = 2 * (F + 2) + 2 * T;   // border pixels of one utterance
  const int chunks = rowbytes / 16;
  const long long n = (long long)B * per_b * chunks;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % chunks);
    const long long k = e / chunks;
    const int b = (int)(k / per_b), j = (int)(k % per_b);
    int t, f;
    if (j < F + 2) { t = 0; f = j; }
    else if (j < 2 * (F + 2)) { t = T + 1; f = j - (F + 2); }
    else { const int r = j - 2 * (F + 2); t = 1 + (r >> 1); f = (r & 1) ? F + 1 : 0; }
    const long long pix = ((long long)b * (T + 2) + t) * (F + 2) + f;
    *reinterpret_cast<uint4*>(buf + pix * rowbytes + ch * 16) = make_uint4(0u, 0u, 0u, 0u);
  }
}

struct TrwPlan {
  int RC;
  size_t lds;
};

bool trw_plan(int Cin, int Cout, int Fp, TrwPlan* pl) {
  if (!((Cin == 64 || Cin == 128) && (Cout == 64 || Cout == 128)) || Fp < 3) return false;
  pl->RC = ((TRW_D + 1) * TRW_BK + 2 * Fp + 16 + 15) / 16 * 16;
  pl->lds = (size_t)(Cin / 64) * pl->RC * 128 + (size_t)(TRW_D + 1) * TRW_BK * 128;
  return pl->lds <= 160 * 1024;
}

struct TrPlan {
  int wpx, nw;
  size_t lds;
  int RC;
};

template <int CIN, int COUT, int WPX, int NW>
int tr_launch(const TrArgs& a0, int out_bf16, hipStream_t s, size_t lds) {
  TrArgs a = a0;
  const void* k = out_bf16 ? (const void*)conv3x3_tr<CIN, COUT, WPX, NW, true>
                           : (const void*)conv3x3_tr<CIN, COUT, WPX, NW, false>;
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return ASR_ERR_UNSUPPORTED;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, TR_NT, lds) != hipSuccess ||
      per_cu < 1)
    return ASR_ERR_UNSUPPORTED;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return ASR_ERR_HIP;
  }
  int grid = std::min(a.ntiles, ncu * per_cu);
  // tests: fewer work-groups, so each runs long chains of tiles through its ring
  if (const char* e = getenv("ASR_CONV_TR_GRID")) grid = std::max(1, std::min(grid, atoi(e)));
  if (out_bf16)
    hipLaunchKernelGGL((conv3x3_tr<CIN, COUT, WPX, NW, true>), dim3(grid), dim3(TR_NT), lds, s, a);
  else
    hipLaunchKernelGGL((conv3x3_tr<CIN, COUT, WPX, NW, false>), dim3(grid), dim3(TR_NT), lds, s, a);
  return ASR_OK;
}

// (wpx, nw) per channel pair: 64 x 64 waves for Cout = 64 at Cin = 64, 128 x 32
// otherwise; four weight slots where the LDS allows, else three.
bool tr_plan(int Cin, int Cout, int Fp, TrPlan* pl) {
  if (!((Cin == 64 || Cin == 128) && (Cout == 64 || Cout == 128)) || Fp < 3) return false;
  pl->wpx = (Cin == 64 && Cout == 64) ? 64 : 32;
  const int BM = 4 * pl->wpx;
  pl->RC = ((2 * BM + 2 * Fp + 16) + 15) / 16 * 16;
  const size_t halo = (size_t)(Cin / 64) * pl->RC * 128;
  const size_t wslot = (size_t)Cout * 128;
  const size_t cap = 160 * 1024;
  const char* wr = getenv("ASR_CONV_TR_WRES");   // A/B: 0 keeps the weight ring
  if (Cin == 64 && Cout == 64 && halo + 9 * wslot <= cap && !(wr && wr[0] == '0')) pl->nw = 0;
  else if (halo + 4 * wslot <= cap) pl->nw = 4;
  else if (halo + 3 * wslot <= cap) pl->nw = 3;
  else return false;
  pl->lds = halo + (pl->nw ? pl->nw : 9 * (Cin / 64)) * wslot;
  return true;
}

}  // namespace
}  // namespace asr

using namespace asr;

extern "C" int asr_conv3x3_tr_supported(int Cin, int Cout, int Fp) {
  TrPlan pl;
  return tr_plan(Cin, Cout, Fp, &pl) ? 1 : 0;
}

extern "C" int asr_conv3x3_tr(const void* in, long long P, int Cin, int Fp, int sign,
                              const void* w, int Cout, const float* bias, void* out,
                              int out_dtype, void* stream) {
  ASR_REQUIRE(in && w && out && P > 0 && (sign == 1 || sign == -1), ASR_ERR_ARG,
              "conv3x3_tr: bad args");
  ASR_REQUIRE(out_dtype == ASR_DT_F32 || out_dtype == ASR_DT_BF16, ASR_ERR_ARG,
              "conv3x3_tr: out dtype %d", out_dtype);
  ASR_REQUIRE(((uintptr_t)in & 15) == 0 && ((uintptr_t)w & 15) == 0 && ((uintptr_t)out & 15) == 0,
              ASR_ERR_ARG, "conv3x3_tr: operands must be 16-B aligned");
  TrPlan pl;
  ASR_REQUIRE(tr_plan(Cin, Cout, Fp, &pl), ASR_ERR_UNSUPPORTED,
              "conv3x3_tr: Cin %d Cout %d Fp %d not supported", Cin, Cout, Fp);
  const int osz = out_dtype == ASR_DT_BF16 ? 2 : 4;
  ASR_REQUIRE(P * Cin * 2 < (1LL << 31) && P * Cout * osz < (1LL << 31), ASR_ERR_UNSUPPORTED,
              "conv3x3_tr: operands above 2 GiB");
  TrArgs a;
  a.in = in;
  a.w = w;
  a.bias = bias;
  a.out = out;
  a.P = (int)P;
  a.Fp = Fp;
  a.sign = sign;
  const int BM = 4 * pl.wpx;
  a.ntiles = (int)((P + BM - 1) / BM);
  a.RC = pl.RC;
  a.RCB = pl.RC * ((Fp + 17 + pl.RC - 1) / pl.RC);
  a.in_bytes = (unsigned)(P * Cin * 2);
  a.w_bytes = (unsigned)((size_t)Cout * 9 * Cin * 2);
  a.out_bytes = (unsigned)(P * Cout * osz);
  hipStream_t s = (hipStream_t)stream;
  const int slot = prof_begin_launch(ASR_PROF_GEMM, s, 2.0 * P * Cout * 9.0 * Cin,
                                     4 * ASR_PTAG_CONV_TR);
  const int bf = out_dtype == ASR_DT_BF16;
  int rc = ASR_ERR_UNSUPPORTED;
#define TR_CASE(CI, CO, WPX, NW)                                                         \
  if (Cin == CI && Cout == CO && pl.wpx == WPX && pl.nw == NW) rc = tr_launch<CI, CO, WPX, NW>(a, bf, s, pl.lds)
  TR_CASE(64, 64, 64, 0);
  else TR_CASE(64, 64, 64, 4);
  else TR_CASE(64, 128, 32, 4);
  else TR_CASE(128, 64, 32, 4);
  else TR_CASE(128, 128, 32, 4);
  else TR_CASE(128, 128, 32, 3);
#undef TR_CASE
  prof_end_launch(ASR_PROF_GEMM, slot, s);
  if (rc != ASR_OK) {
    set_error("conv3x3_tr: no kernel for Cin %d Cout %d Fp %d", Cin, Cout, Fp);
    return rc;
  }
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" size_t asr_conv3x3_tr_wgrad_workspace_bytes(long long P, int Cin, int Cout, int Fp) {
  TrwPlan pl;
  if (!trw_plan(Cin, Cout, Fp, &pl) || P <= 0) return 0;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  const int NG = Cout / 64;
  const int S = std::max(1, std::min(ncu / NG, (int)(P / 512)));
  return (size_t)S * NG * 64 * 9 * Cin * 4;
}

extern "C" int asr_conv3x3_tr_wgrad(const void* x, const void* dz, long long P, int Cin, int Fp,
                                    int Cout, float* packed, void* ws, size_t ws_bytes,
                                    void* stream) {
  ASR_REQUIRE(x && dz && packed && ws && P > 0, ASR_ERR_ARG, "conv3x3_tr_wgrad: bad args");
  ASR_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)dz & 15) == 0 &&
                  ((uintptr_t)packed & 15) == 0 && ((uintptr_t)ws & 15) == 0,
              ASR_ERR_ARG, "conv3x3_tr_wgrad: operands must be 16-B aligned");
  TrwPlan pl;
  ASR_REQUIRE(trw_plan(Cin, Cout, Fp, &pl), ASR_ERR_UNSUPPORTED,
              "conv3x3_tr_wgrad: Cin %d Cout %d Fp %d not supported", Cin, Cout, Fp);
  ASR_REQUIRE(P * Cin * 2 < (1LL << 31) && P * Cout * 2 < (1LL << 31), ASR_ERR_UNSUPPORTED,
              "conv3x3_tr_wgrad: operands above 2 GiB");
  const size_t need = asr_conv3x3_tr_wgrad_workspace_bytes(P, Cin, Cout, Fp);
  ASR_REQUIRE(need > 0 && ws_bytes >= need, ASR_ERR_WORKSPACE, "conv3x3_tr_wgrad: workspace");
  const int NG = Cout / 64;
  TrwArgs a;
  a.x = x;
  a.dz = dz;
  a.slab = (float*)ws;
  a.P = (int)P;
  a.Fp = Fp;
  a.S = (int)(need / ((size_t)NG * 64 * 9 * Cin * 4));
  if (const char* e = getenv("ASR_CONV_TR_SPLITS")) a.S = std::max(1, std::min(a.S, atoi(e)));
  a.RC = pl.RC;
  a.RCB = pl.RC * ((Fp + 17 + pl.RC - 1) / pl.RC);
  a.x_bytes = (unsigned)(P * Cin * 2);
  a.dz_bytes = (unsigned)(P * Cout * 2);
  hipStream_t s = (hipStream_t)stream;
  const int slot = prof_begin_launch(ASR_PROF_GEMM, s, 2.0 * P * Cout * 9.0 * Cin,
                                     4 * ASR_PTAG_CONV_TR_WGRAD);
  const void* k = nullptr;
  if (Cin == 64 && Cout == 64) k = (const void*)conv3x3_tr_wgrad<64, 64>;
  else if (Cin == 64) k = (const void*)conv3x3_tr_wgrad<64, 128>;
  else if (Cout == 64) k = (const void*)conv3x3_tr_wgrad<128, 64>;
  else k = (const void*)conv3x3_tr_wgrad<128, 128>;
  ASR_CHECK_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl.lds));
  const dim3 grid(a.S * NG), block(Cin * 4);
  if (Cin == 64 && Cout == 64) hipLaunchKernelGGL((conv3x3_tr_wgrad<64, 64>), grid, block, pl.lds, s, a);
  else if (Cin == 64) hipLaunchKernelGGL((conv3x3_tr_wgrad<64, 128>), grid, block, pl.lds, s, a);
  else if (Cout == 64) hipLaunchKernelGGL((conv3x3_tr_wgrad<128, 64>), grid, block, pl.lds, s, a);
  else hipLaunchKernelGGL((conv3x3_tr_wgrad<128, 128>), grid, block, pl.lds, s, a);
  ASR_LAUNCH_CHECK();
  const long long n4 = (long long)NG * 64 * 9 * Cin / 4;
  hipLaunchKernelGGL(tr_wgrad_reduce, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, s,
                     (const float*)ws, a.S, NG, 9 * Cin, packed);
  prof_end_launch(ASR_PROF_GEMM, slot, s);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_vgg_zero_halo(void* buf, int dtype, int B, int T, int F, int C, void* stream) {
  ASR_REQUIRE(buf && B > 0 && T > 0 && F > 0 && C > 0, ASR_ERR_ARG, "vgg_zero_halo: bad args");
  const int rowbytes = C * (dtype == ASR_DT_BF16 ? 2 : 4);
  ASR_REQUIRE(rowbytes % 16 == 0 && ((uintptr_t)buf & 15) == 0, ASR_ERR_ARG,
              "vgg_zero_halo: rows must be 16-B multiples");
  const long long n = (long long)B * (2 * (F + 2) + 2 * T) * (rowbytes / 16);
  const int grid = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(zero_halo, dim3(grid), dim3(256), 0, (hipStream_t)stream, (char*)buf, B, T, F,
                     rowbytes);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

// ---------------------------------------------------------------------------
// Weight gradient of the first VGG layer (one input channel), direct from the
// raw features: packed[n][tap Cip + c] = sum_p dz[p][n] * x[p + shift(tap)][c]
// with x the padded operand the tap GEMM would read -- channel 0 = xs (bf16-
// rounded when round_bf16), channels 1 .. Cip-1 zero -- so the image equals
// the tap GEMM's (the padded 16-channel operand and its 48 GFLOP product at
// vgg_hier are no longer needed: the work is 2 x 9 x Co MACs per pixel).
// A work-group per contiguous pixel chunk, 256-pixel tiles: dz rows and the
// tile's x window (+- Fp + 1 rows) in LDS, the next tile's dz prefetched into
// registers; thread (n = tid % Co, kernel row kt = tid / Co < 3) accumulates
// its three taps; per-chunk partials summed in a fixed order.
// ---------------------------------------------------------------------------
namespace asr {
namespace {
constexpr int C1W_TP = 256;    // pixels per tile
constexpr int C1W_MAXS = 1024; // work-groups (4 per CU: 34 KB of LDS each)

template <int CO>
__global__ void __launch_bounds__(256) c1_wgrad_xs(const float* __restrict__ xs, int round_bf16,
                                                    int B, int T, int F,
                                                    const uint16_t* __restrict__ dz, int P, int S,
                                                    float* __restrict__ slab) {
  constexpr int NV = C1W_TP * CO * 2 / 16 / 256;   // 16-B dz pieces per thread per tile
  extern __shared__ __attribute__((aligned(16))) char sm[];
  uint16_t* dzt = (uint16_t*)sm;                              // [TP][CO]
  const int Fp = F + 2, H1 = Fp + 1;
  float* xw = (float*)(sm + C1W_TP * CO * 2);                 // [TP + 2 H1]
  const int tid = threadIdx.x;
  const int beg = (int)((long long)P * blockIdx.x / S), end = (int)((long long)P * (blockIdx.x + 1) / S);
  const int n = tid % CO, kt = tid / CO;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  const int per_b = (T + 2) * Fp;
  auto xval = [&](int q) {   // padded operand channel 0 at padded row q
    if (q < 0 || q >= P) return 0.f;
    const int b = q / per_b, r = q - b * per_b, tp = r / Fp, fp = r - tp * Fp;
    if (tp < 1 || tp > T || fp < 1 || fp > F) return 0.f;
    const float v = xs[((long long)b * T + tp - 1) * F + fp - 1];
    return round_bf16 ? bf2f(f2bf(v)) : v;
  };
  uint4 pre[NV];
  auto fetch = [&](int p0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int e = (j * 256 + tid) * 8;        // bf16 element within the tile
      const int p = p0 + e / CO;
      pre[j] = p < end ? *reinterpret_cast<const uint4*>(dz + (long long)p0 * CO + e)
                       : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  if (beg < end) fetch(beg);
  for (int p0 = beg; p0 < end; p0 += C1W_TP) {
    __syncthreads();   // the previous tile's reads are done
#pragma unroll
    for (int j = 0; j < NV; ++j)
      *reinterpret_cast<uint4*>(dzt + (j * 256 + tid) * 8) = pre[j];
    for (int i = tid; i < C1W_TP + 2 * H1; i += 256) xw[i] = xval(p0 - H1 + i);
    __syncthreads();
    if (p0 + C1W_TP < end) fetch(p0 + C1W_TP);   // in flight during this tile's sums
    if (kt < 3) {
      const int np = min(C1W_TP, end - p0);
      const float* xr = xw + H1 + (kt - 1) * Fp - 1;   // tap (kt, kf): x[i + (kt-1) Fp + kf - 1]
      // the three taps' x values slide through registers: one LDS read of x
      // and one of dz per three FMAs
      float x0 = xr[0], x1 = xr[1];
#pragma unroll 4
      for (int i = 0; i < np; ++i) {
        const float x2 = xr[i + 2];
        const float d = bf2f(dzt[i * CO + n]);
        a0 += d * x0;
        a1 += d * x1;
        a2 += d * x2;
        x0 = x1;
        x1 = x2;
      }
    }
  }
  if (kt < 3) {
    float* o = slab + ((size_t)blockIdx.x * CO + n) * 9 + 3 * kt;
    o[0] = a0;
    o[1] = a1;
    o[2] = a2;
  }
}

// packed[n][tap Cip + c] = (c == 0) * sum_s slab[s][n][tap] (fixed order): a
// block per 16 (n, tap) columns, 16 interleaved phases per column with four
// accumulators each, combined in order through LDS (one thread per column
// summing all S partials serially took 60 us)
__global__ void __launch_bounds__(256) c1_wgrad_reduce(const float* __restrict__ slab, int S,
                                                       int CO, int Cip,
                                                       float* __restrict__ packed) {
  __shared__ float red[256];
  const int tid = threadIdx.x, cl = tid % 16, q0 = tid / 16;
  const int k = blockIdx.x * 16 + cl;   // (n, tap) = (k / 9, k % 9)
  const int K = CO * 9;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (k < K) {
    int q = q0;
    for (; q + 48 < S; q += 64) {
      s0 += slab[(size_t)q * K + k];
      s1 += slab[(size_t)(q + 16) * K + k];
      s2 += slab[(size_t)(q + 32) * K + k];
      s3 += slab[(size_t)(q + 48) * K + k];
    }
    for (; q < S; q += 16) s0 += slab[(size_t)q * K + k];
  }
  red[tid] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (q0 == 0 && k < K) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) t += red[j * 16 + cl];
    red[cl] = t;   // (own slot: read above by this thread only)
  }
  __syncthreads();
  for (int e = tid; e < 16 * Cip; e += 256) {   // the block's 16 columns x Cip channels
    const int kk = blockIdx.x * 16 + e / Cip, c = e % Cip;
    if (kk < K) packed[(size_t)kk * Cip + c] = c == 0 ? red[kk - blockIdx.x * 16] : 0.f;
  }
}
}  // namespace
}  // namespace asr

extern "C" size_t asr_conv3x3_c1_wgrad_workspace_bytes(int Co) {
  return (size_t)C1W_MAXS * Co * 9 * sizeof(float);
}

extern "C" int asr_conv3x3_c1_wgrad_xs(const float* xs, int round_bf16, int B, int T, int F,
                                       int Co, const void* dz, int Cip, float* packed, void* ws,
                                       size_t ws_bytes, void* stream) {
  ASR_REQUIRE(xs && dz && packed && ws && B > 0 && T > 0 && F > 0 && Cip >= 1, ASR_ERR_ARG,
              "conv3x3_c1_wgrad_xs: bad args");
  ASR_REQUIRE(Co == 64, ASR_ERR_UNSUPPORTED, "conv3x3_c1_wgrad_xs: Co %d (64 only)", Co);
  ASR_REQUIRE(((uintptr_t)dz & 15) == 0, ASR_ERR_ARG, "conv3x3_c1_wgrad_xs: dz not 16-B aligned");
  const long long P = (long long)B * (T + 2) * (F + 2);
  ASR_REQUIRE(P * Co * 2 < (1LL << 31), ASR_ERR_UNSUPPORTED, "conv3x3_c1_wgrad_xs: too large");
  const int S = (int)std::min<long long>(C1W_MAXS, std::max<long long>(1, P / 1024));
  ASR_REQUIRE(ws_bytes >= (size_t)S * Co * 9 * sizeof(float), ASR_ERR_WORKSPACE,
              "conv3x3_c1_wgrad_xs: workspace");
  const size_t lds = (size_t)C1W_TP * Co * 2 + (size_t)(C1W_TP + 2 * (F + 3)) * 4;
  ASR_REQUIRE(lds <= 64 * 1024, ASR_ERR_UNSUPPORTED, "conv3x3_c1_wgrad_xs: F too large");
  hipStream_t s = (hipStream_t)stream;
  const int slot = prof_begin_launch(ASR_PROF_GEMM, s, 2.0 * P * Co * 9.0, 4 * ASR_PTAG_CONV_C1_WGRAD);
  hipLaunchKernelGGL(c1_wgrad_xs<64>, dim3(S), dim3(256), lds, s, xs, round_bf16, B, T, F,
                     (const uint16_t*)dz, (int)P, S, (float*)ws);
  ASR_LAUNCH_CHECK();
  hipLaunchKernelGGL(c1_wgrad_reduce, dim3((Co * 9 + 15) / 16), dim3(256), 0, s, (const float*)ws,
                     S, Co, Cip, packed);
  prof_end_launch(ASR_PROF_GEMM, slot, s);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}
