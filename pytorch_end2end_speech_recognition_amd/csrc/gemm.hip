// General MFMA GEMM for the ASR step (gfx950):
//   C(m,n) = alpha * sum_k A(m,k) * B(n,k) + beta * C(m,n) + bias[n]
// Operands are addressed through a RowMap so the encoder's row gathers fuse into
// the operand loads instead of separate copy passes:
//   * batch permutation (length sort, rnn.py:319-326)       -> perm
//   * pyramidal "drop" subsampling xs[:, 1::2] (rnn.py:417)  -> t_mul=2, t_add=1
//   * h_{t-1} / h_{t+1} for dW_hh with zero boundary rows   -> t_add=-1/+1, t_limit
// Element (i,k) of an operand lives at row(i)+k (trans=0, k contiguous) or at
// row(k)+i (trans=1, i contiguous).  Loads are f32 or bf16; compute is exact-f32
// MFMA (v_mfma_f32_16x16x4_f32, parity mode) or bf16 MFMA
// (v_mfma_f32_16x16x32_bf16, fp32 accumulate, performance mode).
//
// Tile 128x128x32, 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4 MFMA
// blocks.  Register-staged double buffering: the next K tile's global loads are
// issued before the MFMAs of the current tile and written to LDS after the
// barrier.  Block ids are remapped so consecutive tiles share an XCD's L2.
#include <stdio.h>
#include <string.h>

#include "mfma.h"
#include "prof.h"

namespace asr {
namespace {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;
constexpr int LDB16 = BK + 8;  // bf16 LDS row pitch (80 B: 16-B aligned fragment reads)
constexpr int LDF32 = BK + 1;  // f32 LDS row pitch

struct RowMap {
  const void* base;
  long long stride_b, stride_t;
  int rows_per_b, t_mul, t_add, t_limit;
  const int32_t* perm;
};

struct Operand {
  RowMap map;
  int dtype;  // ASR_DT_F32 / ASR_DT_BF16
  int trans;
  int vec_ok; // 16-element vector loads legal (alignment of base and strides)
  long long bytes;  // readable bytes from base (0 = unknown)
  int tap_g, tap_w, tap_s;  // 3x3 tap addressing (asr_operand_t), tap_g = 0: off
  int sf;     // division-free staging of the 128x128 kernel applies (StageF)
  int plain;  // row map is r * stride_t, valid for 0 <= r < t_limit
};

// Tap addressing: contiguous index x -> (tap, x'), row shifted by the tap's offset.
__device__ __forceinline__ void tap_adjust(const Operand& op, int& row, int& col) {
  if (op.tap_g) {
    const int tap = col / op.tap_g;
    col -= tap * op.tap_g;
    row += op.tap_s * ((tap / 3 - 1) * op.tap_w + (tap % 3 - 1));
  }
}

struct Problem {
  Operand a, b;
  RowMap c;
  const float* bias;
  const float* bias2;
  int M, N, K;
  float alpha, beta;
  int batch;
  int c_bf16;   // C written as bf16 (beta 0, no split-K, store_acc kernels); fills padding
  long long sA, sB, sC;
  int ksplit;   // > 1: split-K into f32 slabs [ksplit][M][N], reduced by splitk_reduce
  int kchunk;   // K elements per split (multiple of BK)
  float* slab;
  float drop_p;                  // > 0: C element at offset i from C's base is kept iff
  unsigned long long drop_seed;  // u01(drop_seed, i) >= drop_p, scaled by 1 / (1 - p)
  // non-null (asr_gemm_lse_ws): per row m and 64-column slab q of C, the online
  // log-sum-exp pair (max, sum exp(c - max)) of the written values ->
  // lse[2 (q M + m)], lse[2 (q M + m) + 1] (beta 0, no dropout, f32 C, no split)
  float* lse;
};

// Dropout mask of the epilogue (asr_dropout's mask over C's flat offsets).
__device__ __forceinline__ float drop_scale(const Problem& pr, long long i) {
  return u01(pr.drop_seed, (unsigned long long)i) >= pr.drop_p ? 1.f / (1.f - pr.drop_p) : 0.f;
}

struct Params {
  Problem p[2];
  int nprob;
};

// Tile order within an XCD's contiguous id range: groups of GM row-tiles x
// every column-tile, walked column-minor, so the ~64 tiles an XCD holds at once
// form an 8 x 8 block whose A rows and B columns stay in that XCD's L2 (a
// row-major walk re-streams the whole A operand from MALL / HBM once per
// column tile).
constexpr int GM = 8;
__device__ __forceinline__ void tile_coords(int id, int gm, int gn, int* tm, int* tn) {
  const int per = GM * gn;
  const int g = id / per, r = id - g * per;
  const int m0 = g * GM;
  const int gs = min(GM, gm - m0);
  *tm = (m0 + r % gs) * BM;
  *tn = (r / gs) * BN;
}

// Element offset of logical row r, or -1 when the row maps outside [0, t_limit).
__device__ __forceinline__ long long row_off(const RowMap& m, int r) {
  const int b = r / m.rows_per_b;
  const int t = r - b * m.rows_per_b;
  const int tp = t * m.t_mul + m.t_add;
  if (tp < 0 || tp >= m.t_limit) return -1;
  const int bp = m.perm ? m.perm[b] : b;
  return (long long)bp * m.stride_b + (long long)tp * m.stride_t;
}

// Load 16 contiguous elements (along the contiguous dim) starting at logical
// (row r, col c0) of the stored matrix; `ncols` bounds the contiguous dim.
__device__ __forceinline__ void load16(const Operand& op, int r, int nrows, int c0, int ncols,
                                       float (&v)[16]) {
  long long off = (r < nrows) ? row_off(op.map, r) : -1;
  if (off < 0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = 0.f;
    return;
  }
  if (op.dtype == ASR_DT_F32) {
    const float* p = (const float*)op.map.base + off + c0;
    if (op.vec_ok && c0 + 16 <= ncols) {
#pragma unroll
      for (int j = 0; j < 16; j += 4) {
        float4 x = *reinterpret_cast<const float4*>(p + j);
        v[j] = x.x; v[j + 1] = x.y; v[j + 2] = x.z; v[j + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = (c0 + j < ncols) ? p[j] : 0.f;
    }
  } else {
    const uint16_t* p = (const uint16_t*)op.map.base + off + c0;
    if (op.vec_ok && c0 + 16 <= ncols) {
#pragma unroll
      for (int j = 0; j < 16; j += 8) {
        u16x8 x = *reinterpret_cast<const u16x8*>(p + j);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[j + q] = bf2f(x[q]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = (c0 + j < ncols) ? bf2f(p[j]) : 0.f;
    }
  }
}

// 4 contiguous elements starting at logical (row r, col c0) of the stored matrix.
__device__ __forceinline__ void load4(const Operand& op, int r, int nrows, int c0, int ncols,
                                      float* v) {
  long long off = (r < nrows) ? row_off(op.map, r) : -1;
  if (off < 0) {
    v[0] = v[1] = v[2] = v[3] = 0.f;
    return;
  }
  if (op.dtype == ASR_DT_F32) {
    const float* p = (const float*)op.map.base + off + c0;
    if (op.vec_ok && c0 + 4 <= ncols) {
      float4 x = *reinterpret_cast<const float4*>(p);
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (c0 + j < ncols) ? p[j] : 0.f;
    }
  } else {
    const uint16_t* p = (const uint16_t*)op.map.base + off + c0;
    if (op.vec_ok && c0 + 4 <= ncols) {
      uint2 x = *reinterpret_cast<const uint2*>(p);
      v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xffff0000u);
      v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xffff0000u);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (c0 + j < ncols) ? bf2f(p[j]) : 0.f;
    }
  }
}

// Thread -> its 16 elements of a tile.
//   trans=0: tile is 128 logical rows x 32 k: row = tid/2, k = (tid&1)*16..+15
//   trans=1: tile is 32 k-rows x 128 logical rows (contiguous): a 4(k) x 4(row)
//            block per thread, k = 4*(tid/32)..+3, row = 4*(tid%32)..+3, so each
//            row's 4 k land as one 8-B (bf16) LDS store instead of 4 scalars.
//            v[kk*4 + mi] = element (k0 + 4*(tid/32) + kk, row tile0 + 4*(tid%32) + mi)
// K: end of this work-group's k range (split-K chunk end); Ktot: the operand's
// full k extent (a tap-shifted k-row may read past the chunk, never past Ktot).
__device__ __forceinline__ void load_tile(const Operand& op, int tile0, int nrows_logical, int k0,
                                          int K, int Ktot, float (&v)[16]) {
  const int tid = threadIdx.x;
  if (!op.trans) {
    int r = tile0 + (tid >> 1), c = k0 + (tid & 1) * 16;
    if (op.tap_g) {
      const int kv = K - c;   // elements of this chunk inside K
      tap_adjust(op, r, c);
      if (kv <= 0) r = nrows_logical;   // past K: zeros
      load16(op, r, nrows_logical, c, c + min(kv, 16), v);
    } else {
      load16(op, r, nrows_logical, c, K, v);
    }
  } else {
    const int kb = k0 + 4 * (tid >> 5), m4 = tile0 + 4 * (tid & 31);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (op.tap_g) {
        int r = kb + kk, c = m4;
        const int nv = nrows_logical - c;
        tap_adjust(op, r, c);
        if (nv <= 0 || kb + kk >= K) r = Ktot;
        load4(op, r, Ktot, c, c + min(nv, 4), v + 4 * kk);
      } else {
        load4(op, kb + kk, K, m4, nrows_logical, v + 4 * kk);
      }
    }
  }
}

template <bool BF16>
__device__ __forceinline__ void store_tile(const Operand& op, void* lds, const float (&v)[16]) {
  const int tid = threadIdx.x;
  if (BF16) {
    uint16_t* s = (uint16_t*)lds;
    if (!op.trans) {
      uint16_t* d = s + (tid >> 1) * LDB16 + (tid & 1) * 16;
      u16x8 x0, x1;
#pragma unroll
      for (int j = 0; j < 8; ++j) { x0[j] = f2bf(v[j]); x1[j] = f2bf(v[8 + j]); }
      *reinterpret_cast<u16x8*>(d) = x0;
      *reinterpret_cast<u16x8*>(d + 8) = x1;
    } else {
      const int kk0 = 4 * (tid >> 5), m0 = 4 * (tid & 31);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        uint2 w;
        w.x = (uint32_t)f2bf(v[mi]) | ((uint32_t)f2bf(v[4 + mi]) << 16);
        w.y = (uint32_t)f2bf(v[8 + mi]) | ((uint32_t)f2bf(v[12 + mi]) << 16);
        *reinterpret_cast<uint2*>(s + (m0 + mi) * LDB16 + kk0) = w;
      }
    }
  } else {
    float* s = (float*)lds;
    if (!op.trans) {
      float* d = s + (tid >> 1) * LDF32 + (tid & 1) * 16;
#pragma unroll
      for (int j = 0; j < 16; ++j) d[j] = v[j];
    } else {
      const int kk0 = 4 * (tid >> 5), m0 = 4 * (tid & 31);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) s[(m0 + mi) * LDF32 + kk0 + kk] = v[4 * kk + mi];
    }
  }
}

// One row's (max, sum exp) over a 64-column slab held by the 16 lanes of a
// lane group (4 values each, -inf where the column is past N): reduce across
// the group, lane 0 of it stores.  Every lane of the wave calls it (shuffles).
// All-reduce over a 16-lane DPP row: lane ^ 1, lane ^ 2 (quad_perm), then the
// row rotated by 4 and by 8 -- VALU only (ds_bpermute shuffles made the
// 8-wave kernel's epilogue 66 us slower per 8000 x 10001 product).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row16_max(float x) {
  x = fmaxf(x, dpp_f<0xB1>(x));    // quad_perm [1,0,3,2]
  x = fmaxf(x, dpp_f<0x4E>(x));    // quad_perm [2,3,0,1]
  x = fmaxf(x, dpp_f<0x124>(x));   // row_ror:4
  return fmaxf(x, dpp_f<0x128>(x));   // row_ror:8
}
__device__ __forceinline__ float row16_sum(float x) {
  x += dpp_f<0xB1>(x);
  x += dpp_f<0x4E>(x);
  x += dpp_f<0x124>(x);
  return x + dpp_f<0x128>(x);
}

__device__ __forceinline__ void lse_pair_store(const Problem& pr, int q, int m, const float (&v)[4],
                                               float mx, int lane) {
  mx = row16_max(mx);
  // fmaxf drops NaN, so a NaN logit is carried by the sum instead: with the
  // slab's max -inf (every column -inf, past N, or NaN) the exponentials are
  // taken against 0, which gives 0 for -inf and NaN for NaN.  Every slab of
  // the row's extent stores its pair (a skipped store left the
  // partials uninitialised, so a diverged forward could fold a finite loss);
  // the fold (ctc_lse_from_parts) adds an empty slab's sum as is.
  const float base = mx == neg_inf() ? 0.f : mx;
  float sm = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) sm += __expf(v[e] - base);
  sm = row16_sum(sm);
  if ((lane & 15) == 0 && m < pr.M && 64 * q < pr.N) {
    float* p = pr.lse + 2 * ((long long)q * pr.M + m);
    p[0] = mx;
    p[1] = sm;
  }
}

// Epilogue shared by the GEMM kernels.  C/D layout: col = lane&15, row = 4*(lane>>4) + r.
__device__ __forceinline__ void store_acc(const Problem& pr, const f32x4 (&acc)[4][4], int tm,
                                          int tn, int wr, int wc, int lane, int split,
                                          int nsplit) {
  if (nsplit > 1) {  // raw partial sums into this split's slab; splitk_reduce finishes
    float* slab = pr.slab + (long long)split * pr.M * pr.N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = tm + wr + i * 16 + 4 * (lane >> 4) + r;
        if (m >= pr.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = tn + wc + j * 16 + (lane & 15);
          if (n < pr.N) slab[(long long)m * pr.N + n] = acc[i][j][r];
        }
      }
    return;
  }
  if (pr.lse) {   // row log-sum-exp partials of this wave's 64-column slab
    const int q = (tn + wc) >> 6;
    float bj[4];    // this lane's four columns' bias, loaded once
    bool inj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = tn + wc + j * 16 + (lane & 15);
      inj[j] = n < pr.N;
      bj[j] = 0.f;
      if (inj[j] && pr.bias) bj[j] += pr.bias[n];
      if (inj[j] && pr.bias2) bj[j] += pr.bias2[n];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v[4];
        float mx = neg_inf();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = inj[j] ? pr.alpha * acc[i][j][r] + bj[j] : neg_inf();
          mx = fmaxf(mx, v[j]);
        }
        lse_pair_store(pr, q, tm + wr + i * 16 + 4 * (lane >> 4) + r, v, mx, lane);
      }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = tm + wr + i * 16 + 4 * (lane >> 4) + r;
      if (m >= pr.M) continue;
      const long long off = row_off(pr.c, m);
      if (off < 0) continue;
      float* crow = (float*)pr.c.base + off;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = tn + wc + j * 16 + (lane & 15);
        if (n >= pr.N) continue;
        float v = pr.alpha * acc[i][j][r];
        if (pr.bias) v += pr.bias[n];
        if (pr.bias2) v += pr.bias2[n];
        if (pr.beta != 0.f) v += pr.beta * crow[n];
        if (pr.drop_p > 0.f) v *= drop_scale(pr, off + n);
        if (pr.c_bf16)   // bf16 C (beta 0): element offsets of the same map, 2-B stores
          ((uint16_t*)pr.c.base)[off + n] = f2bf(v);
        else
          crow[n] = v;
      }
    }
  }
}

template <bool BF16>
__global__ void __launch_bounds__(NT) gemm_kernel(Params P) {
  constexpr int TILE_ELEMS = BF16 ? BM * LDB16 : BM * LDF32;
  constexpr int ESZ = BF16 ? 2 : 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  void* As = smem;
  void* Bs = smem + TILE_ELEMS * ESZ;

  const int zb = blockIdx.z / P.nprob, zp = blockIdx.z % P.nprob;
  Problem pr = P.p[zp];
  if (zb >= pr.batch) return;
  if (zb > 0) {  // batched product: shift every base by its batch stride
    pr.a.map.base = (const char*)pr.a.map.base + zb * pr.sA * (pr.a.dtype == ASR_DT_F32 ? 4 : 2);
    pr.b.map.base = (const char*)pr.b.map.base + zb * pr.sB * (pr.b.dtype == ASR_DT_F32 ? 4 : 2);
    pr.c.base = (const char*)pr.c.base + zb * pr.sC * (pr.c_bf16 ? 2 : 4);
  }
  const int gm = (pr.M + BM - 1) / BM, gn = (pr.N + BN - 1) / BN;
  const int nwg = gm * gn;
  const int nsplit = pr.ksplit > 1 ? pr.ksplit : 1;
  const int ntot = nwg * nsplit;
  int id = blockIdx.x;
  if (id >= ntot) return;
  {  // bijective XCD-grouping remap: blocks b, b+8, ... land on one XCD
    const int q = ntot / 8, r = ntot % 8, x = id % 8;
    id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
  }
  const int split = id / nwg;
  id -= split * nwg;
  int tm, tn;
  tile_coords(id, gm, gn, &tm, &tn);
  const int kbeg = nsplit > 1 ? split * pr.kchunk : 0;
  const int kend = nsplit > 1 ? min(pr.K, kbeg + pr.kchunk) : pr.K;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = (w >> 1) * 64, wc = (w & 1) * 64;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + BK - 1) / BK;
  float va[16], vb[16];
  load_tile(pr.a, tm, pr.M, kbeg, kend, pr.K, va);
  load_tile(pr.b, tn, pr.N, kbeg, kend, pr.K, vb);
  store_tile<BF16>(pr.a, As, va);
  store_tile<BF16>(pr.b, Bs, vb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      load_tile(pr.a, tm, pr.M, kbeg + (kt + 1) * BK, kend, pr.K, va);
      load_tile(pr.b, tn, pr.N, kbeg + (kt + 1) * BK, kend, pr.K, vb);
    }
    if (BF16) {
      const uint16_t* a = (const uint16_t*)As;
      const uint16_t* b = (const uint16_t*)Bs;
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[i] = load_bf16x8(a + (wr + i * 16 + (lane & 15)) * LDB16 + 8 * (lane >> 4));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = load_bf16x8(b + (wc + j * 16 + (lane & 15)) * LDB16 + 8 * (lane >> 4));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma_bf16(fa[i], fb[j], acc[i][j]);
    } else {
      const float* a = (const float*)As;
      const float* b = (const float*)Bs;
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        float fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = a[(wr + i * 16 + (lane & 15)) * LDF32 + kk + (lane >> 4)];
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = b[(wc + j * 16 + (lane & 15)) * LDF32 + kk + (lane >> 4)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma_f32(fa[i], fb[j], acc[i][j]);
      }
    }
    __syncthreads();
    if (more) {
      store_tile<BF16>(pr.a, As, va);
      store_tile<BF16>(pr.b, Bs, vb);
    }
    __syncthreads();
  }

  store_acc(pr, acc, tm, tn, wr, wc, lane, split, nsplit);
}

// ---------------------------------------------------------------------------
// bf16 fast path: both operands bf16 in memory with known extents (< 2 GiB).
// Tiles go global -> LDS by range-checked buffer loads (buffer_load ... lds,
// 16 B per lane, no pass through VGPRs); rows outside the row map, k outside
// the split's range and bytes past the allocation read as zeros.
//   R mode (trans=0, k contiguous): LDS image [128 rows][64 k], 128-B rows;
//     16-B chunk c of row r sits at chunk c ^ ((r>>1)&7), so one ds_read_b128
//     fragment read of 16 consecutive rows touches 16 distinct bank slots.
//   K mode (trans=1, rows contiguous): LDS image [64 k][128 rows], 256-B
//     k-rows; 32-B granule g of k-row k sits at g ^ h(k), h(k) = (k&3) |
//     ((k>>3)&1)<<2, and fragments come from two ds_read_b64_tr_b16 (hardware
//     transpose) per 16 x 32 block -- conflict-free across each 32-lane half.
//     This is how dW = dG^T X (K = B*T rows) runs without transposed copies.
// 128x128x64 tiles, 4 waves (2x2, 64x64 each), two LDS stages (64 KB): the
// next k-tile's loads are issued before this tile's MFMAs, one vmcnt(0) +
// barrier per k-tile.  The swizzle is applied on the global source address
// (the LDS destination of a buffer->LDS load is lane-linear) and on the read.
// ---------------------------------------------------------------------------
constexpr int FBK = 64;
constexpr int FTILE = 128 * FBK * 2;   // bytes per operand tile (16 KB)
constexpr unsigned OOB_OFF = 0x7ffffff0u;

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((ext_vector_type(4))) short v4s_t;
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

__device__ __forceinline__ int swz_h(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// row_off without the batch permutation (the fast path requires perm == NULL,
// so the staging code issues no global load the compiler would wait for).
__device__ __forceinline__ long long row_off_np(const RowMap& m, int r) {
  const int b = r / m.rows_per_b;
  const int t = r - b * m.rows_per_b;
  const int tp = t * m.t_mul + m.t_add;
  if (tp < 0 || tp >= m.t_limit) return -1;
  return (long long)b * m.stride_b + (long long)tp * m.stride_t;
}

// This thread's 4 buffer->LDS loads of one operand tile.  Instruction i of
// wave w fills LDS bytes [1024*(4w+i), +1024): R mode tile rows (4w+i)*8..+7,
// K mode tile k-rows (4w+i)*4..+3.
template <int MODE, int NB = 4>
__device__ __forceinline__ void stage_tile(const Operand& op, __amdgpu_buffer_rsrc_t rs,
                                           char* lds_tile, int tile0, int nrows, int k0, int kend,
                                           int wave, int lane) {
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int blk = wave * NB + i;
    unsigned voff = OOB_OFF;
    if (MODE == 0) {
      const int r = blk * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      int row = tile0 + r, k = k0 + 8 * c;
      if (row < nrows && k < kend) {
        tap_adjust(op, row, k);
        const long long off = row_off_np(op.map, row);
        if (off >= 0) voff = (unsigned)((off + k) * 2);
      }
    } else {
      const int kr = blk * 4 + (lane >> 4);
      const int j = lane & 15;
      const int c = 2 * ((j >> 1) ^ swz_h(kr)) + (j & 1);
      int k = k0 + kr, col = tile0 + 8 * c;
      if (k < kend) {
        tap_adjust(op, k, col);
        const long long off = row_off_np(op.map, k);
        if (off >= 0) voff = (unsigned)((off + col) * 2);
      }
    }
    // LDS-DMA in inline asm: hipcc neither counts it (so it does not drain it
    // with vmcnt(0) before the current stage's ds_reads) nor keeps M0; the
    // statement saves / restores M0 itself.  Completion: the caller's vmcnt(0).
    const unsigned lds_addr =
        (unsigned)(uintptr_t)(lds_void_t*)(lds_tile + blk * 1024);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rs), "s"(lds_addr)
        : "memory");
  }
}

// Division-free staging for the 128x128 kernel (the Stage8 scheme, with tap
// addressing): per DMA slot the row / k-row state is computed once per tile
// and advanced by FBK per k-tile, so the k-loop does no integer division --
// the division-based row_off_np + tap split per DMA was VALU work comparable
// to the MFMA work of a k-tile.  R mode: the rows are fixed; with taps on k the
// slot carries (tap, k within the tap group) and the row shift of its tap.
// K mode: the columns are fixed (their tap split and row shift once); the
// k-row advances (plain map) or carries its (utterance, frame) pair.
struct StageF {
  int x[4];   // R: k within the tap group (taps) | K: current k-row (+ tap shift), plain map
  int y[4];   // R: current tap (taps) | K: frame of the k-row (general map)
  int z[4];   // R: pixel row (taps) | K: utterance of the k-row (general map)
  unsigned base[4];   // R: row byte offset (no taps) | K: column byte offset
  int valid;
};

__device__ __forceinline__ int tap_shift(const Operand& op, int tap) {
  return op.tap_s * ((tap / 3 - 1) * op.tap_w + (tap % 3 - 1));
}

template <int MODE, int NB = 4>
__device__ __forceinline__ void stagef_init(const Operand& op, StageF& st, int tile0, int nrows,
                                            int kbeg, int wave, int lane) {
  st.valid = 0;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int blk = wave * NB + i;
    if (MODE == 0) {
      const int r = blk * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int row = tile0 + r, k = kbeg + 8 * c;
      if (row < nrows) st.valid |= 1 << i;
      if (op.tap_g) {
        st.y[i] = k / op.tap_g;
        st.x[i] = k - st.y[i] * op.tap_g;
        st.z[i] = row;
        st.base[i] = 0u;
      } else {
        const long long off = row < nrows ? row_off_np(op.map, row) : -1;
        if (off < 0) st.valid &= ~(1 << i);
        st.base[i] = off >= 0 ? (unsigned)(off * 2) : 0u;
        st.x[i] = 8 * c;
        st.y[i] = st.z[i] = 0;
      }
    } else {
      const int kr = blk * 4 + (lane >> 4);
      const int j = lane & 15;
      const int c = 2 * ((j >> 1) ^ swz_h(kr)) + (j & 1);
      int col = tile0 + 8 * c, shift = 0;
      if (op.tap_g) {
        const int tap = col / op.tap_g;
        col -= tap * op.tap_g;
        shift = tap_shift(op, tap);
      }
      st.base[i] = (unsigned)(col * 2);
      const int k = kbeg + kr;
      if (op.plain) {
        st.x[i] = k + shift;
        st.y[i] = st.z[i] = 0;
      } else {
        st.z[i] = k / op.map.rows_per_b;
        st.y[i] = k - st.z[i] * op.map.rows_per_b;
        st.x[i] = 0;
      }
    }
  }
}

template <int MODE, int NB = 4>
__device__ __forceinline__ void stagef(const Operand& op, __amdgpu_buffer_rsrc_t rs, StageF& st,
                                       char* lds_tile, int k0, int kend, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int blk = wave * NB + i;
    unsigned voff = OOB_OFF;
    if (MODE == 0) {
      const int r = blk * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int k = k0 + 8 * c;
      if (op.tap_g) {
        const int rr = st.z[i] + tap_shift(op, st.y[i]);
        if (((st.valid >> i) & 1) && k < kend && rr >= 0 && rr < op.map.t_limit)
          voff = (unsigned)(((long long)rr * op.map.stride_t + st.x[i]) * 2);
        st.x[i] += FBK;   // this slot's k in the next k-tile
        while (st.x[i] >= op.tap_g) {
          st.x[i] -= op.tap_g;
          ++st.y[i];
        }
      } else if (((st.valid >> i) & 1) && k < kend) {
        voff = st.base[i] + (unsigned)(k * 2);
      }
    } else {
      const int kr = blk * 4 + (lane >> 4);
      const int k = k0 + kr;
      if (op.plain) {
        const int rr = st.x[i];
        if (k < kend && rr >= 0 && rr < op.map.t_limit)
          voff = (unsigned)((long long)rr * op.map.stride_t * 2) + st.base[i];
        st.x[i] += FBK;
      } else {
        const int tp = st.y[i] * op.map.t_mul + op.map.t_add;
        if (k < kend && tp >= 0 && tp < op.map.t_limit)
          voff = (unsigned)(((long long)st.z[i] * op.map.stride_b +
                             (long long)tp * op.map.stride_t) * 2) + st.base[i];
        st.y[i] += FBK;
        while (st.y[i] >= op.map.rows_per_b) {
          st.y[i] -= op.map.rows_per_b;
          ++st.z[i];
        }
      }
    }
    const unsigned lds_addr = (unsigned)(uintptr_t)(lds_void_t*)(lds_tile + blk * 1024);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rs), "s"(lds_addr)
        : "memory");
  }
}

// One operand's tile of the 128x128 kernel: StageF when the operand allows it
// (wave-uniform branch), else the per-DMA row map.
template <int MODE, int NB = 4>
__device__ __forceinline__ void stage_any(const Operand& op, __amdgpu_buffer_rsrc_t rs,
                                          StageF& st, char* lds_tile, int tile0, int nrows,
                                          int k0, int kend, int wave, int lane) {
  if (op.sf) stagef<MODE, NB>(op, rs, st, lds_tile, k0, kend, wave, lane);
  else stage_tile<MODE, NB>(op, rs, lds_tile, tile0, nrows, k0, kend, wave, lane);
}

// MFMA fragment (16 rows x 32 k) of the block starting at tile row rb, k-half kk.
template <int MODE>
__device__ __forceinline__ bf16x8 frag_bf16(const char* lds_tile, int rb, int kk, int lane) {
  if (MODE == 0) {
    const int r = rb + (lane & 15);
    const int c = (4 * kk + (lane >> 4)) ^ ((r >> 1) & 7);
    return __builtin_bit_cast(bf16x8, *(const u32x4_t*)(lds_tile + r * 128 + c * 16));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int G = rb >> 4;
    const int k0 = 32 * kk + 8 * g + q, k1 = k0 + 4;
    const char* a0 = lds_tile + k0 * 256 + ((G ^ swz_h(k0)) << 5) + 8 * p;
    const char* a1 = lds_tile + k1 * 256 + ((G ^ swz_h(k1)) << 5) + 8 * p;
    const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)a0);
    const v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)a1);
    typedef __attribute__((ext_vector_type(8))) short v8s_t;
    const v8s_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
  }
}

template <int AMODE, int BMODE>
__device__ __forceinline__ void mma_ktile(const char* cur, f32x4 (&acc)[4][4], int wr, int wc,
                                          int lane) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    bf16x8 fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag_bf16<AMODE>(cur, wr + 16 * i, kk, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = frag_bf16<BMODE>(cur + FTILE, wc + 16 * j, kk, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma_bf16(fa[i], fb[j], acc[i][j]);
  }
}

// NSTAGE = 2: double buffer (64 KB LDS, 2 blocks / CU), one tile of prefetch;
// NSTAGE = 4: ring (128 KB, 1 block / CU), three tiles of prefetch.
template <int AMODE, int BMODE, int NSTAGE>
__global__ void __launch_bounds__(NT) gemm_bf16_fast(Params P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 stages x (A, B) tiles

  const int zb = blockIdx.z / P.nprob, zp = blockIdx.z % P.nprob;
  Problem pr = P.p[zp];
  if (zb >= pr.batch) return;
  if (zb > 0) {
    pr.a.map.base = (const char*)pr.a.map.base + zb * pr.sA * 2;
    pr.b.map.base = (const char*)pr.b.map.base + zb * pr.sB * 2;
    pr.a.bytes -= zb * pr.sA * 2;
    pr.b.bytes -= zb * pr.sB * 2;
    pr.c.base = (const char*)pr.c.base + zb * pr.sC * (pr.c_bf16 ? 2 : 4);
  }
  const int gm = (pr.M + BM - 1) / BM, gn = (pr.N + BN - 1) / BN;
  const int nwg = gm * gn;
  const int nsplit = pr.ksplit > 1 ? pr.ksplit : 1;
  const int ntot = nwg * nsplit;
  int id = blockIdx.x;
  if (id >= ntot) return;
  {
    const int q = ntot / 8, r = ntot % 8, x = id % 8;
    id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
  }
  const int split = id / nwg;
  id -= split * nwg;
  int tm, tn;
  tile_coords(id, gm, gn, &tm, &tn);
  const int kbeg = nsplit > 1 ? split * pr.kchunk : 0;
  const int kend = nsplit > 1 ? min(pr.K, kbeg + pr.kchunk) : pr.K;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = (w >> 1) * 64, wc = (w & 1) * 64;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)pr.a.map.base, 0, (int)pr.a.bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)pr.b.map.base, 0, (int)pr.b.bytes, 0x00020000);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + FBK - 1) / FBK;
  StageF sa, sb;
  if (pr.a.sf) stagef_init<AMODE>(pr.a, sa, tm, pr.M, kbeg, w, lane);
  if (pr.b.sf) stagef_init<BMODE>(pr.b, sb, tn, pr.N, kbeg, w, lane);
  if (NSTAGE == 2) {
    stage_any<AMODE>(pr.a, ra, sa, smem, tm, pr.M, kbeg, kend, w, lane);
    stage_any<BMODE>(pr.b, rb, sb, smem + FTILE, tn, pr.N, kbeg, kend, w, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < nk; ++kt) {
      const char* cur = smem + (kt & 1) * 2 * FTILE;
      if (kt + 1 < nk) {
        char* nxt = smem + ((kt + 1) & 1) * 2 * FTILE;
        const int k0 = kbeg + (kt + 1) * FBK;
        stage_any<AMODE>(pr.a, ra, sa, nxt, tm, pr.M, k0, kend, w, lane);
        stage_any<BMODE>(pr.b, rb, sb, nxt + FTILE, tn, pr.N, k0, kend, w, lane);
      }
      mma_ktile<AMODE, BMODE>(cur, acc, wr, wc, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  } else {
    // Ring of NSTAGE stages, tiles issued NSTAGE - 1 ahead.  Iteration kt:
    // counted wait for tile kt (the tiles issued after it may stay in flight:
    // 8 loads each), barrier (every wave's tile-kt data visible, and every wave
    // done reading stage (kt - 1) % NSTAGE), refill that stage with tile
    // kt + NSTAGE - 1, compute tile kt.  One barrier per k-tile.
#pragma unroll
    for (int j = 0; j < NSTAGE - 1; ++j) {
      if (j < nk) {
        char* st = smem + j * 2 * FTILE;
        const int k0 = kbeg + j * FBK;
        stage_any<AMODE>(pr.a, ra, sa, st, tm, pr.M, k0, kend, w, lane);
        stage_any<BMODE>(pr.b, rb, sb, st + FTILE, tn, pr.N, k0, kend, w, lane);
      }
    }
    for (int kt = 0; kt < nk; ++kt) {
      const int after = min(NSTAGE - 2, nk - 1 - kt);   // tiles issued after tile kt
      if (after >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if (after == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + NSTAGE - 1 < nk) {
        char* st = smem + ((kt + NSTAGE - 1) % NSTAGE) * 2 * FTILE;
        const int k0 = kbeg + (kt + NSTAGE - 1) * FBK;
        stage_any<AMODE>(pr.a, ra, sa, st, tm, pr.M, k0, kend, w, lane);
        stage_any<BMODE>(pr.b, rb, sb, st + FTILE, tn, pr.N, k0, kend, w, lane);
      }
      mma_ktile<AMODE, BMODE>(smem + (kt % NSTAGE) * 2 * FTILE, acc, wr, wc, lane);
    }
  }
  store_acc(pr, acc, tm, tn, wr, wc, lane, split, nsplit);
}

// ---------------------------------------------------------------------------
// f32 fast path (reference precision): gemm_bf16_fast's structure -- LDS-DMA
// staging (buffer_load ... lds, 16 B per lane), division-free per-slot row
// state (taps included), double-buffered k-tiles -- with f32 elements (32-k
// tiles) and v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulate).
// The generic register-staged kernel ran these products at 45-90 TF/s (157
// peak).  Work-group tile (64 TMW) x (64 TNW), TMW TNW = 4 waves of 64 x 64:
// 128 x 128, or 256 x 64 for N <= 64 (the 64-channel convolutions) and
// 64 x 256 for M <= 64 (their weight gradients), so no tile is half empty.
//   R mode (k contiguous): LDS [ROWS][32 k], 128-B rows; 16-B chunk c of row r
//     at chunk c ^ ((r >> 1) & 7) (the bf16 image's swizzle).  A k extent that
//     is not a multiple of 4 is allowed: the one 16-B chunk straddling the end
//     of k (inside the row: rows are 16-B aligned and at least k long) has its
//     elements past the end zeroed in LDS by the lane that loaded it, after
//     its wait and before the barrier.
//   K mode (rows contiguous): LDS [32 k-rows][ROWS], ROWS 4-B k-rows; 16-B
//     chunk c of k-row k at chunk c ^ (4 ((k >> 3) & 3)).
// k order inside a k-tile: at MFMA s (0..7) lane group g = lane >> 4 supplies
// k = 8 g + s, so an R-mode fragment is two ds_read_b128 of one row and a
// K-mode fragment eight ds_read_b32 down one column (the swizzle puts the four
// lane groups' k-rows in different bank quarters).  Summation order differs
// from gemm_kernel<false>; every product is still one f32 FMA into an f32 sum.
// ---------------------------------------------------------------------------
constexpr int FBK32 = 32;

__device__ __forceinline__ int swz32(int k) { return ((k >> 3) & 3) << 2; }

template <int NB>
struct StageF32 {
  int x[NB], y[NB], z[NB];
  int zp[NB];      // K mode, general map: perm[z] (the batch permutation), or z
  unsigned base[NB];
  int valid;
  int tmask, tn;   // R mode: slots whose chunk straddles the end of k, valid elements
};

template <int MODE, int ROWS>
__device__ __forceinline__ void stagef32_init(const Operand& op, StageF32<ROWS / 32>& st,
                                              int tile0, int nrows, int kbeg, int kend0, int wave,
                                              int lane) {
  constexpr int NB = ROWS / 32, KPD = 256 / ROWS, LPK = ROWS / 4;
  st.valid = 0;
  st.tmask = 0;
  st.tn = 4;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int blk = wave * NB + i;
    if (MODE == 0) {
      const int r = blk * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int row = tile0 + r, k = kbeg + 4 * c;
      if (row < nrows) st.valid |= 1 << i;
      if (op.tap_g) {
        st.y[i] = k / op.tap_g;
        st.x[i] = k - st.y[i] * op.tap_g;
        st.z[i] = row;
        st.base[i] = 0u;
      } else {
        // rows are fixed in R mode: the batch permutation is applied once here
        const long long off = row < nrows ? row_off(op.map, row) : -1;
        if (off < 0) st.valid &= ~(1 << i);
        st.base[i] = off >= 0 ? (unsigned)(off * 4) : 0u;
        st.x[i] = 4 * c;
        st.y[i] = st.z[i] = 0;
      }
    } else {
      const int kr = blk * KPD + lane / LPK;
      const int c = (lane % LPK) ^ swz32(kr);
      int col = tile0 + 4 * c, shift = 0;
      if (op.tap_g) {
        const int tap = col / op.tap_g;
        col -= tap * op.tap_g;
        shift = tap_shift(op, tap);
      }
      st.base[i] = (unsigned)(col * 4);
      const int k = kbeg + kr;
      if (op.plain) {
        st.x[i] = k + shift;
        st.y[i] = st.z[i] = 0;
      } else {
        st.z[i] = k / op.map.rows_per_b;
        st.y[i] = k - st.z[i] * op.map.rows_per_b;
        st.x[i] = 0;
        st.zp[i] = (op.map.perm && k < kend0) ? op.map.perm[st.z[i]] : st.z[i];
      }
    }
  }
}

template <int MODE, int ROWS>
__device__ __forceinline__ void stagef32(const Operand& op, __amdgpu_buffer_rsrc_t rs,
                                         StageF32<ROWS / 32>& st, char* lds_tile, int k0, int kend,
                                         int wave, int lane) {
  constexpr int NB = ROWS / 32, KPD = 256 / ROWS, LPK = ROWS / 4;
  st.tmask = 0;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int blk = wave * NB + i;
    unsigned voff = OOB_OFF;
    if (MODE == 0) {
      const int r = blk * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int k = k0 + 4 * c;
      bool on = false;
      if (op.tap_g) {
        const int rr = st.z[i] + tap_shift(op, st.y[i]);
        on = ((st.valid >> i) & 1) && k < kend && rr >= 0 && rr < op.map.t_limit;
        if (on) voff = (unsigned)(((long long)rr * op.map.stride_t + st.x[i]) * 4);
        st.x[i] += FBK32;
        while (st.x[i] >= op.tap_g) {
          st.x[i] -= op.tap_g;
          ++st.y[i];
        }
      } else if (((st.valid >> i) & 1) && k < kend) {
        on = true;
        voff = st.base[i] + (unsigned)(k * 4);
      }
      if (on && k + 4 > kend) {
        st.tmask |= 1 << i;
        st.tn = kend - k;
      }
    } else {
      const int kr = blk * KPD + lane / LPK;
      const int k = k0 + kr;
      if (op.plain) {
        const int rr = st.x[i];
        if (k < kend && rr >= 0 && rr < op.map.t_limit)
          voff = (unsigned)((long long)rr * op.map.stride_t * 4) + st.base[i];
        st.x[i] += FBK32;
      } else {
        const int tp = st.y[i] * op.map.t_mul + op.map.t_add;
        if (k < kend && tp >= 0 && tp < op.map.t_limit)
          voff = (unsigned)(((long long)st.zp[i] * op.map.stride_b +
                             (long long)tp * op.map.stride_t) * 4) + st.base[i];
        st.y[i] += FBK32;
        bool moved = false;
        while (st.y[i] >= op.map.rows_per_b) {
          st.y[i] -= op.map.rows_per_b;
          ++st.z[i];
          moved = true;
        }
        // the permuted utterance of this slot's next k-row, read only when it
        // changes and exists (k-tiles cross an utterance every rows_per_b / 32)
        if (moved) st.zp[i] = (op.map.perm && k + FBK32 < kend) ? op.map.perm[st.z[i]] : st.z[i];
      }
    }
    const unsigned lds_addr = (unsigned)(uintptr_t)(lds_void_t*)(lds_tile + blk * 1024);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rs), "s"(lds_addr)
        : "memory");
  }
}

// After the wait for a tile's DMAs, before its barrier: zero the elements past
// the end of k in this lane's straddling R-mode chunks (see above).
template <int ROWS>
__device__ __forceinline__ void tailfix32(const StageF32<ROWS / 32>& st, char* lds_tile, int wave,
                                          int lane) {
  constexpr int NB = ROWS / 32;
  if (!st.tmask) return;
#pragma unroll
  for (int i = 0; i < NB; ++i)
    if ((st.tmask >> i) & 1) {
      float* p = (float*)(lds_tile + (wave * NB + i) * 1024 + lane * 16);
      for (int e = st.tn; e < 4; ++e) p[e] = 0.f;
    }
}

// The four k values 8 g + 4 h .. + 3 (g = lane >> 4) of tile row / column
// rb + (lane & 15); ROWS: the tile's extent along the operand's outer dim.
template <int MODE, int ROWS>
__device__ __forceinline__ f32x4 frag_f32(const char* lds_tile, int rb, int h, int lane) {
  const int g = lane >> 4;
  if (MODE == 0) {
    const int r = rb + (lane & 15);
    const int c = (2 * g + h) ^ ((r >> 1) & 7);
    return *(const f32x4*)(lds_tile + r * 128 + c * 16);
  } else {
    const int j = rb + (lane & 15);
    const int cb = (((j >> 2) ^ (g << 2)) << 4) + 4 * (j & 3);
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      v[e] = *(const float*)(lds_tile + (8 * g + 4 * h + e) * (ROWS * 4) + cb);
    return v;
  }
}

// s_waitcnt vmcnt(n) with expcnt / lgkmcnt left at their maxima (gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// NSTAGE = 2: double buffer, two work-groups per CU; 3: a ring with two
// k-tiles in flight (one work-group per CU), counted waits.
template <int AMODE, int BMODE, int TMW, int NSTAGE = 2>
__global__ void __launch_bounds__(NT) gemm_f32_fast(Params P) {
  constexpr int TNW = 4 / TMW, TM = 64 * TMW, TN = 64 * TNW;
  constexpr int ATILE = TM * FBK32 * 4, STAGE = (TM + TN) * FBK32 * 4;
  constexpr int DPT = (TM + TN) / 32;   // DMAs per wave per k-tile
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 stages x (A, B) tiles
  const int zb = blockIdx.z / P.nprob, zp = blockIdx.z % P.nprob;
  Problem pr = P.p[zp];
  if (zb >= pr.batch) return;
  if (zb > 0) {
    pr.a.map.base = (const char*)pr.a.map.base + zb * pr.sA * 4;
    pr.b.map.base = (const char*)pr.b.map.base + zb * pr.sB * 4;
    pr.a.bytes -= zb * pr.sA * 4;
    pr.b.bytes -= zb * pr.sB * 4;
    pr.c.base = (const char*)pr.c.base + zb * pr.sC * 4;
  }
  const int gm = (pr.M + TM - 1) / TM, gn = (pr.N + TN - 1) / TN;
  const int nwg = gm * gn;
  const int nsplit = pr.ksplit > 1 ? pr.ksplit : 1;
  const int ntot = nwg * nsplit;
  int id = blockIdx.x;
  if (id >= ntot) return;
  {
    const int q = ntot / 8, r = ntot % 8, x = id % 8;
    id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
  }
  const int split = id / nwg;
  id -= split * nwg;
  int tm, tn;
  {   // tile_coords with this kernel's tile extents
    const int per = GM * gn;
    const int g = id / per, r = id - g * per;
    const int m0 = g * GM;
    const int gs = min(GM, gm - m0);
    tm = (m0 + r % gs) * TM;
    tn = (r / gs) * TN;
  }
  const int kbeg = nsplit > 1 ? split * pr.kchunk : 0;
  const int kend = nsplit > 1 ? min(pr.K, kbeg + pr.kchunk) : pr.K;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = (w / TNW) * 64, wc = (w % TNW) * 64;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)pr.a.map.base, 0, (int)pr.a.bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)pr.b.map.base, 0, (int)pr.b.bytes, 0x00020000);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + FBK32 - 1) / FBK32;
  StageF32<TM / 32> sa;
  StageF32<TN / 32> sb;
  stagef32_init<AMODE, TM>(pr.a, sa, tm, pr.M, kbeg, kend, w, lane);
  stagef32_init<BMODE, TN>(pr.b, sb, tn, pr.N, kbeg, kend, w, lane);
  auto mma = [&](const char* cur) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x4 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag_f32<AMODE, TM>(cur, wr + 16 * i, h, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag_f32<BMODE, TN>(cur + ATILE, wc + 16 * j, h, lane);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma_f32(fa[i][e], fb[j][e], acc[i][j]);
    }
  };
  auto stage = [&](char* st, int k0) {
    stagef32<AMODE, TM>(pr.a, ra, sa, st, k0, kend, w, lane);
    stagef32<BMODE, TN>(pr.b, rb, sb, st + ATILE, k0, kend, w, lane);
  };
  // the last k-tile's straddling R-mode chunks (the only ones), once landed
  auto tail = [&](char* st) {
    if (AMODE == 0) tailfix32<TM>(sa, st, w, lane);
    if (BMODE == 0) tailfix32<TN>(sb, st + ATILE, w, lane);
  };
  if constexpr (NSTAGE == 2) {
    stage(smem, kbeg);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tail(smem);
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < nk; ++kt) {
      const char* cur = smem + (kt & 1) * STAGE;
      char* nxt = smem + ((kt + 1) & 1) * STAGE;
      if (kt + 1 < nk) stage(nxt, kbeg + (kt + 1) * FBK32);
      mma(cur);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (kt + 1 < nk) tail(nxt);
      __builtin_amdgcn_s_barrier();
    }
  } else {
#pragma unroll
    for (int j = 0; j < NSTAGE - 1; ++j)
      if (j < nk) stage(smem + j * STAGE, kbeg + j * FBK32);
    for (int kt = 0; kt < nk; ++kt) {
      const int after = min(NSTAGE - 2, nk - 1 - kt);   // tiles issued after tile kt
      if (after >= 1) wait_vmcnt<DPT>();
      else wait_vmcnt<0>();
      asm volatile("" ::: "memory");
      char* cur = smem + (kt % NSTAGE) * STAGE;
      if (kt == nk - 1) tail(cur);
      __builtin_amdgcn_s_barrier();
      if (kt + NSTAGE - 1 < nk)
        stage(smem + ((kt + NSTAGE - 1) % NSTAGE) * STAGE, kbeg + (kt + NSTAGE - 1) * FBK32);
      mma(cur);
    }
  }
  store_acc(pr, acc, tm, tn, wr, wc, lane, split, nsplit);
}

// 256 x 64 tiles for products with N <= 64 and B in R mode (B stored [N][K]:
// the 3x3 convolutions of the 64-channel VGG layers, forward and input
// gradient).  The 128 x 128 kernel computed those with half of every B tile
// and of every MFMA empty.  Four waves stacked along M (64 x 64 each, the
// same fragments and MFMA order as gemm_bf16_fast), the A tile staged as two
// 128-row halves (own StageF states), the B tile as 64 rows (two DMAs per
// wave); double-buffered, 80 KB of LDS (two work-groups per CU).
constexpr int N64_BM = 256;
// stage bytes: A (32 KB) + B (R mode: 64 rows, 8 KB; K mode: the 128-column
// k-row layout of the 128 x 128 kernel with columns 64.. zero, 16 KB)
__host__ __device__ constexpr int n64_stage(int bmode) { return 2 * FTILE + (bmode ? FTILE : FTILE / 2); }

// NSTAGE = 2: double buffer (80 KB, two work-groups per CU), one k-tile of
// prefetch; NSTAGE = 3: a ring (120 KB, one work-group per CU), two k-tiles in
// flight (the tap-addressed convolutions wait on L2 for every k-tile).
template <int AMODE, int BMODE, int NSTAGE = 2>
__global__ void __launch_bounds__(NT) gemm_bf16_n64(Params P) {
  constexpr int N64_STAGE = n64_stage(BMODE);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int zb = blockIdx.z / P.nprob, zp = blockIdx.z % P.nprob;
  Problem pr = P.p[zp];
  if (zb >= pr.batch) return;
  if (zb > 0) {
    pr.a.map.base = (const char*)pr.a.map.base + zb * pr.sA * 2;
    pr.b.map.base = (const char*)pr.b.map.base + zb * pr.sB * 2;
    pr.a.bytes -= zb * pr.sA * 2;
    pr.b.bytes -= zb * pr.sB * 2;
    pr.c.base = (const char*)pr.c.base + zb * pr.sC * (pr.c_bf16 ? 2 : 4);
  }
  const int gm = (pr.M + N64_BM - 1) / N64_BM;
  const int nsplit = pr.ksplit > 1 ? pr.ksplit : 1;
  const int ntot = gm * nsplit;
  int id = blockIdx.x;
  if (id >= ntot) return;
  {
    const int q = ntot / 8, r = ntot % 8, x = id % 8;
    id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
  }
  const int split = id / gm;
  const int tm = (id - split * gm) * N64_BM, tn = 0;
  const int kbeg = nsplit > 1 ? split * pr.kchunk : 0;
  const int kend = nsplit > 1 ? min(pr.K, kbeg + pr.kchunk) : pr.K;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w * 64, wc = 0;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)pr.a.map.base, 0, (int)pr.a.bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)pr.b.map.base, 0, (int)pr.b.bytes, 0x00020000);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + FBK - 1) / FBK;
  StageF sa0, sa1, sb;
  if (pr.a.sf) {
    stagef_init<AMODE>(pr.a, sa0, tm, pr.M, kbeg, w, lane);
    stagef_init<AMODE>(pr.a, sa1, tm + 128, pr.M, kbeg, w, lane);
  }
  if (pr.b.sf) stagef_init<BMODE, BMODE ? 4 : 2>(pr.b, sb, tn, pr.N, kbeg, w, lane);
  auto stage = [&](char* st, int k0) {
    stage_any<AMODE>(pr.a, ra, sa0, st, tm, pr.M, k0, kend, w, lane);
    stage_any<AMODE>(pr.a, ra, sa1, st + FTILE, tm + 128, pr.M, k0, kend, w, lane);
    stage_any<BMODE, BMODE ? 4 : 2>(pr.b, rb, sb, st + 2 * FTILE, tn, pr.N, k0, kend, w, lane);
  };
  auto compute = [&](const char* cur) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)   // waves 2, 3 read the second 128-row half
        fa[i] = frag_bf16<AMODE>(cur + (wr >> 7) * FTILE, (wr & 127) + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag_bf16<BMODE>(cur + 2 * FTILE, wc + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma_bf16(fa[i], fb[j], acc[i][j]);
    }
  };
  static_assert(NSTAGE == 2 || NSTAGE == 3, "n64: two or three stages");
  if constexpr (NSTAGE == 2) {
    stage(smem, kbeg);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < nk; ++kt) {
      const char* cur = smem + (kt & 1) * N64_STAGE;
      if (kt + 1 < nk) stage(smem + ((kt + 1) & 1) * N64_STAGE, kbeg + (kt + 1) * FBK);
      compute(cur);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  } else {
    // ring: k-tiles issued NSTAGE - 1 ahead; iteration kt waits for tile kt
    // (each k-tile is N64_DMA buffer->LDS loads per wave; the later tiles stay
    // in flight), one barrier (tile kt visible to every wave, and every wave
    // done with slot (kt - 1) % NSTAGE), refills that slot, computes tile kt
    constexpr int N64_DMA = 8 + (BMODE ? 4 : 2);
#pragma unroll
    for (int j = 0; j < NSTAGE - 1; ++j)
      if (j < nk) stage(smem + j * N64_STAGE, kbeg + j * FBK);
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N64_DMA) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + NSTAGE - 1 < nk)
        stage(smem + ((kt + NSTAGE - 1) % NSTAGE) * N64_STAGE, kbeg + (kt + NSTAGE - 1) * FBK);
      compute(smem + (kt % NSTAGE) * N64_STAGE);
    }
  }
  store_acc(pr, acc, tm, tn, wr, wc, lane, split, nsplit);
}

// ---------------------------------------------------------------------------
// 256 x 256 tiles for K-major x K-major products (the weight gradients
// dW = dG^T X, K = B*T): four waves, each a 128 x 128 sub-tile (8 x 8 MFMA
// accumulators, 256 registers, in AGPRs), so each wave reads half the LDS
// bytes per MFMA of the 128 x 128 kernel (whose 64 x 64 wave tiles put the
// LDS read rate at the MFMA rate) and each work-group streams half the
// L2 bytes per flop.  Same staging scheme: swizzled K-mode tiles (here 512-B
// k-rows) filled by buffer->LDS DMA, hardware-transpose fragment reads; a
// four-stage ring of 32-deep k-tiles (128 KB: one work-group per CU, three
// k-tiles in flight), one barrier per k-tile.
// ---------------------------------------------------------------------------
constexpr int BT2 = 256;
constexpr int BK2 = 32;                 // k-tile depth
constexpr int NST2 = 4;                 // LDS ring stages (3 k-tiles in flight)
constexpr int FTILE2 = BT2 * BK2 * 2;   // 16 KB per operand tile

__device__ __forceinline__ void stage_tile_k256(const Operand& op, __amdgpu_buffer_rsrc_t rs,
                                                char* lds_tile, int tile0, int k0, int kend,
                                                int wave, int lane) {
#pragma unroll
  for (int i = 0; i < BK2 / 8; ++i) {
    const int blk = wave * (BK2 / 8) + i;  // 1 KB = two 512-B k-rows
    const int kr = blk * 2 + (lane >> 5);
    const int j = lane & 31;               // 16-B chunk of the k-row
    const int c = 2 * ((j >> 1) ^ swz_h(kr)) + (j & 1);
    unsigned voff = OOB_OFF;
    int k = k0 + kr, col = tile0 + 8 * c;
    if (k < kend) {
      tap_adjust(op, k, col);
      const long long off = row_off_np(op.map, k);
      if (off >= 0) voff = (unsigned)((off + col) * 2);
    }
    const unsigned lds_addr = (unsigned)(uintptr_t)(lds_void_t*)(lds_tile + blk * 1024);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rs), "s"(lds_addr)
        : "memory");
  }
}

__device__ __forceinline__ bf16x8 frag_k256(const char* lds_tile, int rb, int kk, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int G = rb >> 4;
  const int k0 = 32 * kk + 8 * g + q, k1 = k0 + 4;
  const char* a0 = lds_tile + k0 * 512 + ((G ^ swz_h(k0)) << 5) + 8 * p;
  const char* a1 = lds_tile + k1 * 512 + ((G ^ swz_h(k1)) << 5) + 8 * p;
  const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)a0);
  const v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)a1);
  typedef __attribute__((ext_vector_type(8))) short v8s_t;
  const v8s_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm_bf16_kk256(Params P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 stages x (A, B) tiles

  const int zb = blockIdx.z / P.nprob, zp = blockIdx.z % P.nprob;
  Problem pr = P.p[zp];
  if (zb >= pr.batch) return;
  if (zb > 0) {
    pr.a.map.base = (const char*)pr.a.map.base + zb * pr.sA * 2;
    pr.b.map.base = (const char*)pr.b.map.base + zb * pr.sB * 2;
    pr.a.bytes -= zb * pr.sA * 2;
    pr.b.bytes -= zb * pr.sB * 2;
    pr.c.base = (const char*)pr.c.base + zb * pr.sC * (pr.c_bf16 ? 2 : 4);
  }
  const int gm = (pr.M + BT2 - 1) / BT2, gn = (pr.N + BT2 - 1) / BT2;
  const int nwg = gm * gn;
  const int nsplit = pr.ksplit > 1 ? pr.ksplit : 1;
  const int ntot = nwg * nsplit;
  int id = blockIdx.x;
  if (id >= ntot) return;
  {
    const int q = ntot / 8, r = ntot % 8, x = id % 8;
    id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
  }
  const int split = id / nwg;
  id -= split * nwg;
  // column-minor walk inside groups of 4 row tiles (an XCD's resident tiles share operands)
  int tm, tn;
  {
    const int per = 4 * gn;
    const int g = id / per, r = id - g * per;
    const int m0 = g * 4;
    const int gs = min(4, gm - m0);
    tm = (m0 + r % gs) * BT2;
    tn = (r / gs) * BT2;
  }
  const int kbeg = nsplit > 1 ? split * pr.kchunk : 0;
  const int kend = nsplit > 1 ? min(pr.K, kbeg + pr.kchunk) : pr.K;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = (w >> 1) * 128, wc = (w & 1) * 128;
  // descriptors built from wave-uniform values (readfirstlane) so they live in SGPRs
  auto uni_ptr = [](const void* p) {
    const unsigned long long v = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (void*)(((unsigned long long)hi << 32) | lo);
  };
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      uni_ptr(pr.a.map.base), 0, __builtin_amdgcn_readfirstlane((int)pr.a.bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      uni_ptr(pr.b.map.base), 0, __builtin_amdgcn_readfirstlane((int)pr.b.bytes), 0x00020000);

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Ring of NST2 stages, k-tiles issued NST2 - 1 ahead; iteration kt: counted
  // wait for tile kt (each tile is 2 * BK2 / 8 DMA instructions per thread),
  // barrier, refill the stage read in iteration kt - 1, compute tile kt.
  constexpr int PER = 2 * (BK2 / 8);
  const int nk = (kend - kbeg + BK2 - 1) / BK2;
#pragma unroll
  for (int j = 0; j < NST2 - 1; ++j) {
    if (j < nk) {
      char* st = smem + j * 2 * FTILE2;
      stage_tile_k256(pr.a, ra, st, tm, kbeg + j * BK2, kend, w, lane);
      stage_tile_k256(pr.b, rb, st + FTILE2, tn, kbeg + j * BK2, kend, w, lane);
    }
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int after = min(NST2 - 2, nk - 1 - kt);
    if (after >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + NST2 - 1 < nk) {
      char* st = smem + ((kt + NST2 - 1) % NST2) * 2 * FTILE2;
      const int k0 = kbeg + (kt + NST2 - 1) * BK2;
      stage_tile_k256(pr.a, ra, st, tm, k0, kend, w, lane);
      stage_tile_k256(pr.b, rb, st + FTILE2, tn, k0, kend, w, lane);
    }
    const char* cur = smem + (kt % NST2) * 2 * FTILE2;
#pragma unroll
    for (int kk = 0; kk < BK2 / 32; ++kk) {
      bf16x8 fb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) fb[j] = frag_k256(cur + FTILE2, wc + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const bf16x8 fa = frag_k256(cur, wr + 16 * i, kk, lane);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = mfma_bf16(fa, fb[j], acc[i][j]);
      }
    }
  }

  if (nsplit > 1) {  // raw partial sums into this split's slab; splitk_reduce finishes
    float* slab = pr.slab + (long long)split * pr.M * pr.N;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = tm + wr + i * 16 + 4 * (lane >> 4) + r;
        if (m >= pr.M) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int n = tn + wc + j * 16 + (lane & 15);
          if (n < pr.N) slab[(long long)m * pr.N + n] = acc[i][j][r];
        }
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = tm + wr + i * 16 + 4 * (lane >> 4) + r;
      if (m >= pr.M) continue;
      const long long off = row_off(pr.c, m);
      if (off < 0) continue;
      float* crow = (float*)pr.c.base + off;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int n = tn + wc + j * 16 + (lane & 15);
        if (n >= pr.N) continue;
        float v = pr.alpha * acc[i][j][r];
        if (pr.bias) v += pr.bias[n];
        if (pr.bias2) v += pr.bias2[n];
        if (pr.beta != 0.f) v += pr.beta * crow[n];
        if (pr.drop_p > 0.f) v *= drop_scale(pr, off + n);
        crow[n] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// 256 x 256 x 64 tiles, 8 waves (2 x 4, each wave 128 x 64 = 8 x 4 MFMA
// accumulators), two 64-KB LDS buffers (one work-group per CU, two waves per
// SIMD): every plain bf16 product of the encoder (input projections R x R,
// input gradients R x K, weight gradients K x K).  Why it beats the 128 x 128
// kernel (one barrier + vmcnt(0) per k-tile, the "step-3 structure" whose
// ceiling is ~900 TF/s): the staging pipeline is two k-tiles deep and never
// drains inside the loop, and the LDS reads of one k-half overlap the MFMAs of
// the other:
//   prologue : DMA k-tiles 0, 1 -> buffers 0, 1; wait tile 0; kk = 0 fragments
//   k-tile t : read kk = 1 fragments of t | MFMA kk = 0 of t
//              lgkmcnt(0) + barrier          (buffer t & 1 fully read by all)
//              DMA k-tile t + 2 -> buffer t & 1
//              vmcnt(8) + barrier            (k-tile t + 1 landed: only t + 2's
//                                             eight DMAs may stay in flight)
//              read kk = 0 fragments of t + 1 | MFMA kk = 1 of t
// Staging is the buffer -> LDS DMA of the 128 x 128 kernel (inline asm: hipcc
// neither counts nor drains it; the counted waits above are the only ones),
// with the same source-address swizzles (R mode: 128-B rows, chunk c of row r
// at c ^ ((r >> 1) & 7); K mode: 512-B k-rows, 32-B granule g of k-row k at
// g ^ swz_h(k), read by ds_read_b64_tr_b16).
// ---------------------------------------------------------------------------
constexpr int T8 = 256, BK8 = 64, NT8 = 512;
constexpr int TILE8 = T8 * BK8 * 2;   // 32 KB per operand k-tile

// Per-thread staging state of one operand: the byte offsets of this thread's
// four 16-B DMA sources, computed once (R mode: the rows never change, only
// k advances) or advanced incrementally (K mode: the k-rows move by 64 per
// k-tile; their (utterance, frame) pair is carried, so the row map costs no
// division inside the k-loop -- the division-based row_off per DMA was most of
// the kernel's VALU work).
struct Stage8 {
  unsigned base[4];   // R: row byte offset + chunk; K: column byte offset
  int b[4], t[4];     // K: utterance / frame of the current k-row
  int kr[4];          // R: chunk k offset (8c); K: k-row within the tile
  int valid;          // R: bit i = row i inside the operand
};

template <int MODE>
__device__ __forceinline__ void stage8_init(const Operand& op, Stage8& st, int tile0, int nrows,
                                            int kbeg, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int blk = wave * 4 + i;
    if (MODE == 0) {
      const int r = blk * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int row = tile0 + r;
      long long off = row < nrows ? row_off_np(op.map, row) : -1;
      st.base[i] = off >= 0 ? (unsigned)(off * 2) : 0u;
      st.kr[i] = 8 * c;
      if (i == 0) st.valid = 0;
      if (off >= 0) st.valid |= 1 << i;
    } else {
      const int kr = blk * 2 + (lane >> 5);
      const int j = lane & 31;
      const int c = 2 * ((j >> 1) ^ swz_h(kr)) + (j & 1);
      st.base[i] = (unsigned)((tile0 + 8 * c) * 2);
      st.kr[i] = kr;
      const int k = kbeg + kr;
      st.b[i] = k / op.map.rows_per_b;
      st.t[i] = k - st.b[i] * op.map.rows_per_b;
    }
  }
}

template <int MODE>
__device__ __forceinline__ void stage8(const Operand& op, __amdgpu_buffer_rsrc_t rs, Stage8& st,
                                       char* lds_tile, int k0, int kend, int wave) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int blk = wave * 4 + i;          // 1 KB of the 32-KB image
    unsigned voff = OOB_OFF;
    if (MODE == 0) {
      const int k = k0 + st.kr[i];
      if (((st.valid >> i) & 1) && k < kend) voff = st.base[i] + (unsigned)(k * 2);
    } else {
      const int k = k0 + st.kr[i];
      const int tp = st.t[i] * op.map.t_mul + op.map.t_add;
      if (k < kend && tp >= 0 && tp < op.map.t_limit)
        voff = (unsigned)(((long long)st.b[i] * op.map.stride_b +
                           (long long)tp * op.map.stride_t) * 2) + st.base[i];
      // advance to this k-row of the next k-tile
      st.t[i] += BK8;
      while (st.t[i] >= op.map.rows_per_b) {
        st.t[i] -= op.map.rows_per_b;
        ++st.b[i];
      }
    }
    const unsigned lds_addr = (unsigned)(uintptr_t)(lds_void_t*)(lds_tile + blk * 1024);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rs), "s"(lds_addr)
        : "memory");
  }
}

// R-mode fragment read with the lane-dependent part of the address hoisted:
// rb is a multiple of 16, so the chunk swizzle ((r >> 1) & 7) of row
// r = rb + (lane & 15) depends on the lane only and the address is
// tile + rb * 128 (uniform) + lane_off(kk) (one VGPR per k-half).
__device__ __forceinline__ unsigned r_lane_off(int kk, int lane) {
  const int r = lane & 15;
  return (unsigned)(r * 128 + (((4 * kk + (lane >> 4)) ^ ((r >> 1) & 7)) * 16));
}

template <int MODE>
__device__ __forceinline__ bf16x8 frag8(const char* lds_tile, int rb, int kk, int lane) {
  if (MODE == 0)
    return __builtin_bit_cast(bf16x8,
                              *(const u32x4_t*)(lds_tile + rb * 128 + r_lane_off(kk, lane)));
  return frag_k256(lds_tile, rb, kk, lane);
}

// Fragments of one k-half (kk) of a k-tile: B for the wave's 64 columns (4
// blocks), A for 64 of its 128 rows (half ih: 4 blocks).
template <int BMODE>
__device__ __forceinline__ void fragsB8(const char* buf, int kk, int wc, int lane, bf16x8 (&fb)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) fb[j] = frag8<BMODE>(buf + TILE8, wc + 16 * j, kk, lane);
}
template <int AMODE>
__device__ __forceinline__ void fragsA8(const char* buf, int kk, int r0, int lane, bf16x8 (&fa)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) fa[i] = frag8<AMODE>(buf, r0 + 16 * i, kk, lane);
}

// 16 MFMAs: rows [ih*64, +64) of the wave's tile x its 64 columns, one k-half
__device__ __forceinline__ void mma8(const bf16x8 (&fa)[4], const bf16x8 (&fb)[4],
                                     f32x4 (&acc)[8][4], int ih) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[ih * 4 + i][j] = mfma_bf16(fa[i], fb[j], acc[ih * 4 + i][j]);
  __builtin_amdgcn_s_setprio(0);
}

// Epilogue of the 8-wave kernel through LDS: each wave's 128 x 64 f32 tile is
// written to LDS in four 32-row quarters (pitch 68 floats: the 4-row lane
// groups of a ds_write land on distinct banks; 8 waves x 8.5 KB) and read
// back as 16-B row chunks, so the global stores (and the bias / beta reads)
// are dwordx4 over whole 256-B row segments instead of 4-B lanes.
// C(m, n) = alpha acc + bias[n] + bias2[n] + beta C(m, n) through C's row map;
// raw = 1 writes acc alone to a dense [M][N] slab (split-K partials).
constexpr int EP8 = 68;
__device__ __forceinline__ void epi8(const Problem& pr, const RowMap& cm, bool raw,
                                     f32x4 (&acc)[8][4], int tm, int tn, int wr, int wc,
                                     int w, int lane, char* smem) {
  float* tile = (float*)smem + w * 32 * EP8;
  // a plain C map (every row valid, no batch split) needs no division per row
  const bool plain = cm.rows_per_b == 0x7fffffff && cm.t_mul == 1 && cm.t_add == 0 &&
                     cm.t_limit == 0x7fffffff && !cm.perm;
  const bool bias_vec = ((uintptr_t)pr.bias & 15) == 0 && ((uintptr_t)pr.bias2 & 15) == 0;
  // the row-LSE pass: this lane's four columns (fixed over the quarters) and
  // their bias, loaded once
  float lb[4] = {0.f, 0.f, 0.f, 0.f};
  bool lin[4] = {false, false, false, false};
  if (!raw && pr.lse) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = tn + wc + 4 * (lane & 15) + e;
      lin[e] = n < pr.N;
      if (lin[e] && pr.bias) lb[e] += pr.bias[n];
      if (lin[e] && pr.bias2) lb[e] += pr.bias2[n];
    }
  }
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    __syncthreads();   // LDS free (k-loop done / previous quarter read back)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          tile[(16 * i + 4 * (lane >> 4) + r) * EP8 + 16 * j + (lane & 15)] = acc[2 * h + i][j][r];
    __syncthreads();
    if (!raw && pr.lse) {   // row log-sum-exp partials of this wave's 64-column slab
      for (int it = 0; it < 8; ++it) {
        const int row = it * 4 + (lane >> 4), ch = lane & 15;
        const float4 t4 = *reinterpret_cast<const float4*>(tile + row * EP8 + 4 * ch);
        const float tv[4] = {t4.x, t4.y, t4.z, t4.w};
        float v[4];
        float mx = neg_inf();
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = lin[e] ? tv[e] * pr.alpha + lb[e] : neg_inf();
          mx = fmaxf(mx, v[e]);
        }
        lse_pair_store(pr, (tn + wc) >> 6, tm + wr + 32 * h + row, v, mx, lane);
      }
    }
#pragma unroll 4
    for (int it = 0; it < 8; ++it) {
      const int row = it * 4 + (lane >> 4), ch = lane & 15;
      const int m = tm + wr + 32 * h + row;
      const int n = tn + wc + 4 * ch;
      if (m >= pr.M || n >= pr.N) continue;
      const float4 v = *reinterpret_cast<const float4*>(tile + row * EP8 + 4 * ch);
      const long long off = plain ? (long long)m * cm.stride_t : row_off(cm, m);
      if (off < 0) continue;
      float* cp = (float*)cm.base + off + n;
      float o[4] = {v.x, v.y, v.z, v.w};
      const bool full = n + 4 <= pr.N;
      if (!raw) {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] *= pr.alpha;
        if (full && bias_vec) {   // the bias pair as two 16-B loads
          if (pr.bias) {
            const float4 b = *reinterpret_cast<const float4*>(pr.bias + n);
            o[0] += b.x; o[1] += b.y; o[2] += b.z; o[3] += b.w;
          }
          if (pr.bias2) {
            const float4 b = *reinterpret_cast<const float4*>(pr.bias2 + n);
            o[0] += b.x; o[1] += b.y; o[2] += b.z; o[3] += b.w;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (n + e < pr.N) {
              if (pr.bias) o[e] += pr.bias[n + e];
              if (pr.bias2) o[e] += pr.bias2[n + e];
            }
          }
        }
      }
      if (full && ((uintptr_t)cp & 15) == 0) {
        if (!raw && pr.beta != 0.f) {
          const float4 c = *reinterpret_cast<const float4*>(cp);
          o[0] += pr.beta * c.x; o[1] += pr.beta * c.y; o[2] += pr.beta * c.z; o[3] += pr.beta * c.w;
        }
        if (!raw && pr.drop_p > 0.f) drop_n<4>(o, pr.drop_p, pr.drop_seed, (unsigned long long)(off + n));
        *reinterpret_cast<float4*>(cp) = make_float4(o[0], o[1], o[2], o[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n + e < pr.N) {
            float x = (!raw && pr.beta != 0.f) ? o[e] + pr.beta * cp[e] : o[e];
            if (!raw && pr.drop_p > 0.f) x *= drop_scale(pr, off + n + e);
            cp[e] = x;
          }
      }
    }
  }
}

template <int AMODE, int BMODE>
__global__ void __launch_bounds__(NT8) __attribute__((amdgpu_waves_per_eu(2, 2)))
gemm_bf16_8w(Params P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 buffers x (A, B)

  const int zb = blockIdx.z / P.nprob, zp = blockIdx.z % P.nprob;
  Problem pr = P.p[zp];
  if (zb >= pr.batch) return;
  if (zb > 0) {
    pr.a.map.base = (const char*)pr.a.map.base + zb * pr.sA * 2;
    pr.b.map.base = (const char*)pr.b.map.base + zb * pr.sB * 2;
    pr.a.bytes -= zb * pr.sA * 2;
    pr.b.bytes -= zb * pr.sB * 2;
    pr.c.base = (const char*)pr.c.base + zb * pr.sC * (pr.c_bf16 ? 2 : 4);
  }
  const int gm = (pr.M + T8 - 1) / T8, gn = (pr.N + T8 - 1) / T8;
  const int nwg = gm * gn;
  const int nsplit = pr.ksplit > 1 ? pr.ksplit : 1;
  const int ntot = nwg * nsplit;
  int id = blockIdx.x;
  if (id >= ntot) return;
  {  // bijective XCD remap: an XCD's blocks take a contiguous id range
    const int q = ntot / 8, r = ntot % 8, x = id % 8;
    id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
  }
  const int split = id / nwg;
  id -= split * nwg;
  int tm, tn;
  {  // column-minor walk inside groups of 4 row tiles
    const int per = 4 * gn;
    const int g = id / per, r = id - g * per;
    const int m0 = g * 4;
    const int gs = min(4, gm - m0);
    tm = (m0 + r % gs) * T8;
    tn = (r / gs) * T8;
  }
  const int kbeg = nsplit > 1 ? split * pr.kchunk : 0;
  const int kend = nsplit > 1 ? min(pr.K, kbeg + pr.kchunk) : pr.K;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = (w >> 2) * 128, wc = (w & 3) * 64;
  auto uni_ptr = [](const void* p) {
    const unsigned long long v = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (void*)(((unsigned long long)hi << 32) | lo);
  };
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      uni_ptr(pr.a.map.base), 0, __builtin_amdgcn_readfirstlane((int)pr.a.bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      uni_ptr(pr.b.map.base), 0, __builtin_amdgcn_readfirstlane((int)pr.b.bytes), 0x00020000);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + BK8 - 1) / BK8;
  Stage8 sa, sb;
  stage8_init<AMODE>(pr.a, sa, tm, pr.M, kbeg, w, lane);
  stage8_init<BMODE>(pr.b, sb, tn, pr.N, kbeg, w, lane);
  stage8<AMODE>(pr.a, ra, sa, smem, kbeg, kend, w);
  stage8<BMODE>(pr.b, rb, sb, smem + TILE8, kbeg, kend, w);
  if (nk > 1) {
    stage8<AMODE>(pr.a, ra, sa, smem + 2 * TILE8, kbeg + BK8, kend, w);
    stage8<BMODE>(pr.b, rb, sb, smem + 3 * TILE8, kbeg + BK8, kend, w);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  // four phases per k-tile, (k-half, row-half) = (0,0) (0,1) (1,0) (1,1); the
  // fragments of the next phase are read while the current phase's 16 MFMAs run
  bf16x8 b0[4], b1[4], a00[4], a01[4], a10[4], a11[4];
  fragsB8<BMODE>(smem, 0, wc, lane, b0);
  fragsA8<AMODE>(smem, 0, wr, lane, a00);
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * 2 * TILE8;
    fragsA8<AMODE>(cur, 0, wr + 64, lane, a01);
    mma8(a00, b0, acc, 0);
    fragsB8<BMODE>(cur, 1, wc, lane, b1);
    fragsA8<AMODE>(cur, 1, wr, lane, a10);
    mma8(a01, b0, acc, 1);
    fragsA8<AMODE>(cur, 1, wr + 64, lane, a11);
    mma8(a10, b1, acc, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                         // buffer kt & 1 read by all waves
    if (kt + 2 < nk) {
      const int k0 = kbeg + (kt + 2) * BK8;
      stage8<AMODE>(pr.a, ra, sa, cur, k0, kend, w);
      stage8<BMODE>(pr.b, rb, sb, cur + TILE8, k0, kend, w);
    }
    if (kt + 1 < nk) {
      if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();                       // k-tile kt + 1 landed for all
      const char* nxt = smem + ((kt + 1) & 1) * 2 * TILE8;
      fragsB8<BMODE>(nxt, 0, wc, lane, b0);
      fragsA8<AMODE>(nxt, 0, wr, lane, a00);
    }
    mma8(a11, b1, acc, 1);
  }

  if (nsplit > 1) {  // raw partial sums into this split's slab; splitk_reduce finishes
    RowMap sm;
    sm.base = pr.slab + (long long)split * pr.M * pr.N;
    sm.stride_b = 0;
    sm.stride_t = pr.N;
    sm.rows_per_b = 0x7fffffff;
    sm.t_mul = 1;
    sm.t_add = 0;
    sm.t_limit = 0x7fffffff;
    sm.perm = nullptr;
    epi8(pr, sm, true, acc, tm, tn, wr, wc, w, lane, smem);
    return;
  }
  epi8(pr, pr.c, false, acc, tm, tn, wr, wc, w, lane, smem);
}

// ---------------------------------------------------------------------------
// Ring form of the 8-wave kernel (the default; ASR_GEMM_8R=0 selects the
// two-buffer form above): 32-deep k-tiles in a
// five-slot LDS ring (5 x 32 KB = 160 KB), three k-tiles in flight behind the
// one being read (the 64-deep two-buffer form keeps one).  Per k-tile:
//   read A rows 64-127 | MFMA rows 0-63
//   lgkmcnt(0) + barrier (slot free) -> DMA k-tile t + 4 into it
//   counted vmcnt + barrier (k-tile t + 1 landed) -> read its B, A rows 0-63
//   | MFMA rows 64-127
// R-mode image [256 rows][32 k]: 64-B rows, 16-B chunk c of row r at slot
// c ^ swz8r(r) with swz8r = 0, 0, 3, 3 for (r >> 2) & 3 = 0..3.  A 64-B row
// covers 16 of the 64 banks, so rows r and r + 4 share banks; ds_read_b128
// serves a wave in four fixed 16-lane groups (MI355X_MICROARCH.md §LDS), and
// each group's (row % 4, slot) pairs must be distinct: the round-2 swizzle
// (r >> 2) & 3 put two lanes of every group on the same banks (PMC: 46 % of
// the fwd product's LDS cycles were conflict cycles); this one clears all four
// groups.  K-mode image [32 k][256 rows] as the 256 x 256 kernel's.
__device__ __forceinline__ int swz8r(int r) { return ((r >> 3) & 1) * 3; }
// K-mode image [32 k][256 rows] as the 256 x 256 kernel's.
// ---------------------------------------------------------------------------
constexpr int BKR = 32, NSLOT = 5;
constexpr int TILER = T8 * BKR * 2;    // 16 KB per operand k-tile

struct StageR {
  unsigned base[2];
  int b[2], t[2], kr[2];
  int valid;
};

template <int MODE>
__device__ __forceinline__ void stager_init(const Operand& op, StageR& st, int tile0, int nrows,
                                            int kbeg, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = wave * 2 + i;          // 1 KB of the 16-KB image
    if (MODE == 0) {
      const int r = blk * 16 + (lane >> 2);
      const int c = (lane & 3) ^ swz8r(r);
      const int row = tile0 + r;
      long long off = row < nrows ? row_off_np(op.map, row) : -1;
      st.base[i] = off >= 0 ? (unsigned)(off * 2) : 0u;
      st.kr[i] = 8 * c;
      if (i == 0) st.valid = 0;
      if (off >= 0) st.valid |= 1 << i;
    } else {
      const int kr = blk * 2 + (lane >> 5);
      const int j = lane & 31;
      const int c = 2 * ((j >> 1) ^ swz_h(kr)) + (j & 1);
      st.base[i] = (unsigned)((tile0 + 8 * c) * 2);
      st.kr[i] = kr;
      const int k = kbeg + kr;
      st.b[i] = k / op.map.rows_per_b;
      st.t[i] = k - st.b[i] * op.map.rows_per_b;
    }
  }
}

// a K-mode operand whose k-rows are consecutive rows of one group (no time
// offset / stride / limit): row k sits at k * stride_t -- one 32-bit multiply-add
// per DMA instead of the (b, t) walk with 64-bit products (the weight-gradient
// operands dG and X; the shifted h_{t-1} rows of dW_hh keep the walk)
__device__ __forceinline__ bool kmode_dense(const RowMap& m) {
  return m.t_mul == 1 && m.t_add == 0 && !m.perm &&
         (m.rows_per_b >= 0x40000000 || m.stride_b == (long long)m.rows_per_b * m.stride_t) &&
         m.t_limit >= m.rows_per_b;
}

template <int MODE>
__device__ __forceinline__ void stager(const Operand& op, __amdgpu_buffer_rsrc_t rs, StageR& st,
                                       char* lds_tile, int k0, int kend, int wave) {
  const bool dense = MODE == 1 && kmode_dense(op.map);
  const unsigned kst = (unsigned)(op.map.stride_t * 2);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = wave * 2 + i;
    unsigned voff = OOB_OFF;
    const int k = k0 + st.kr[i];
    if (MODE == 0) {
      if (((st.valid >> i) & 1) && k < kend) voff = st.base[i] + (unsigned)(k * 2);
    } else if (dense) {
      if (k < kend) voff = (unsigned)k * kst + st.base[i];
    } else {
      const int tp = st.t[i] * op.map.t_mul + op.map.t_add;
      if (k < kend && tp >= 0 && tp < op.map.t_limit)
        voff = (unsigned)(((long long)st.b[i] * op.map.stride_b +
                           (long long)tp * op.map.stride_t) * 2) + st.base[i];
      st.t[i] += BKR;
      while (st.t[i] >= op.map.rows_per_b) {
        st.t[i] -= op.map.rows_per_b;
        ++st.b[i];
      }
    }
    const unsigned lds_addr = (unsigned)(uintptr_t)(lds_void_t*)(lds_tile + blk * 1024);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rs), "s"(lds_addr)
        : "memory");
  }
}

template <int MODE>
__device__ __forceinline__ bf16x8 fragr(const char* lds_tile, int rb, int lane) {
  if (MODE == 0) {
    const int r = lane & 15;
    const unsigned lo = (unsigned)(r * 64 + (((lane >> 4) ^ swz8r(r)) * 16));
    return __builtin_bit_cast(bf16x8, *(const u32x4_t*)(lds_tile + rb * 64 + lo));
  }
  return frag_k256(lds_tile, rb, 0, lane);
}

template <int AMODE, int BMODE>
__device__ __forceinline__ void fragsr(const char* slot, int r0, int wc, int lane, bool withb,
                                       bf16x8 (&fa)[4], bf16x8 (&fb)[4]) {
  if (withb) {
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = fragr<BMODE>(slot + TILER, wc + 16 * j, lane);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) fa[i] = fragr<AMODE>(slot, r0 + 16 * i, lane);
}

template <int AMODE, int BMODE>
__global__ void __launch_bounds__(NT8) __attribute__((amdgpu_waves_per_eu(2, 2)))
gemm_bf16_8r(Params P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // NSLOT x (A, B)

  const int zb = blockIdx.z / P.nprob, zp = blockIdx.z % P.nprob;
  Problem pr = P.p[zp];
  if (zb >= pr.batch) return;
  if (zb > 0) {
    pr.a.map.base = (const char*)pr.a.map.base + zb * pr.sA * 2;
    pr.b.map.base = (const char*)pr.b.map.base + zb * pr.sB * 2;
    pr.a.bytes -= zb * pr.sA * 2;
    pr.b.bytes -= zb * pr.sB * 2;
    pr.c.base = (const char*)pr.c.base + zb * pr.sC * (pr.c_bf16 ? 2 : 4);
  }
  const int gm = (pr.M + T8 - 1) / T8, gn = (pr.N + T8 - 1) / T8;
  const int nwg = gm * gn;
  const int nsplit = pr.ksplit > 1 ? pr.ksplit : 1;
  const int ntot = nwg * nsplit;
  int id = blockIdx.x;
  if (id >= ntot) return;
  {
    const int q = ntot / 8, r = ntot % 8, x = id % 8;
    id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
  }
  const int split = id / nwg;
  id -= split * nwg;
  int tm, tn;
  {
    const int per = 4 * gn;
    const int g = id / per, r = id - g * per;
    const int m0 = g * 4;
    const int gs = min(4, gm - m0);
    tm = (m0 + r % gs) * T8;
    tn = (r / gs) * T8;
  }
  const int kbeg = nsplit > 1 ? split * pr.kchunk : 0;
  const int kend = nsplit > 1 ? min(pr.K, kbeg + pr.kchunk) : pr.K;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = (w >> 2) * 128, wc = (w & 3) * 64;
  auto uni_ptr = [](const void* p) {
    const unsigned long long v = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (void*)(((unsigned long long)hi << 32) | lo);
  };
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      uni_ptr(pr.a.map.base), 0, __builtin_amdgcn_readfirstlane((int)pr.a.bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      uni_ptr(pr.b.map.base), 0, __builtin_amdgcn_readfirstlane((int)pr.b.bytes), 0x00020000);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + BKR - 1) / BKR;
  StageR sa, sb;
  stager_init<AMODE>(pr.a, sa, tm, pr.M, kbeg, w, lane);
  stager_init<BMODE>(pr.b, sb, tn, pr.N, kbeg, w, lane);
  constexpr int SLOT = 2 * TILER;
#pragma unroll
  for (int j = 0; j < NSLOT - 1; ++j) {
    if (j < nk) {
      stager<AMODE>(pr.a, ra, sa, smem + j * SLOT, kbeg + j * BKR, kend, w);
      stager<BMODE>(pr.b, rb, sb, smem + j * SLOT + TILER, kbeg + j * BKR, kend, w);
    }
  }
  {
    const int after = min(NSLOT - 2, nk - 1);          // k-tiles issued after tile 0
    if (after >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (after == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  bf16x8 b0[4], b1[4], a0[4], a1[4];
  fragsr<AMODE, BMODE>(smem, wr, wc, lane, true, a0, b0);
  // one k-tile; bc: its B fragments, bn: receives the next tile's (the loop
  // runs two tiles per trip with the roles swapped, so the B fragments are
  // never copied -- 16 v_mov per k-tile and wave otherwise)
  auto ktile = [&](int kt, bf16x8 (&bc)[4], bf16x8 (&bn)[4]) {
    const char* cur = smem + (kt % NSLOT) * SLOT;
    // slot (kt - 1) % NSLOT was last read before iteration kt - 1's barrier
    // the DMA of k-tile kt + 4 is spread over the two MFMA phases (A before the
    // first, B before the second): an LDS-DMA issue stalls the wave for tens of
    // cycles, so a burst of four would open a gap in the MFMA stream
    const bool dma = kt + NSLOT - 1 < nk;
    char* fre = smem + ((kt + NSLOT - 1) % NSLOT) * SLOT;
    const int kd = kbeg + (kt + NSLOT - 1) * BKR;
    if (dma) stager<AMODE>(pr.a, ra, sa, fre, kd, kend, w);
    fragsr<AMODE, BMODE>(cur, wr + 64, wc, lane, false, a1, bc);
    mma8(a0, bc, acc, 0);
    if (dma) stager<BMODE>(pr.b, rb, sb, fre + TILER, kd, kend, w);
    if (kt + 1 < nk) {
      const int after = min(NSLOT - 2, nk - 2 - kt);    // k-tiles issued after tile kt + 1
      if (after >= 3) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
      else if (after == 2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
      else if (after == 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      // k-tile kt + 1 landed for all waves; every wave's reads of slot kt done
      __builtin_amdgcn_s_barrier();
      const char* nxt = smem + ((kt + 1) % NSLOT) * SLOT;
      fragsr<AMODE, BMODE>(nxt, wr, wc, lane, true, a0, bn);
    }
    mma8(a1, bc, acc, 1);
  };
  for (int kt = 0; kt < nk; kt += 2) {
    ktile(kt, b0, b1);
    if (kt + 1 < nk) ktile(kt + 1, b1, b0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  if (nsplit > 1) {
    RowMap sm;
    sm.base = pr.slab + (long long)split * pr.M * pr.N;
    sm.stride_b = 0;
    sm.stride_t = pr.N;
    sm.rows_per_b = 0x7fffffff;
    sm.t_mul = 1;
    sm.t_add = 0;
    sm.t_limit = 0x7fffffff;
    sm.perm = nullptr;
    epi8(pr, sm, true, acc, tm, tn, wr, wc, w, lane, smem);
    return;
  }
  epi8(pr, pr.c, false, acc, tm, tn, wr, wc, w, lane, smem);
}

// Split-K finish: C(m,n) = alpha * sum_s slab[s][m][n] (fixed order s = 0..) +
// bias + bias2 + beta * C, through C's row map.
__global__ void splitk_reduce(const float* __restrict__ slab, int ksplit, int M, int N, RowMap c,
                              float alpha, float beta, const float* __restrict__ bias,
                              const float* __restrict__ bias2, float drop_p,
                              unsigned long long drop_seed) {
  const long long MN = (long long)M * N;
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= MN) return;
  const int m = (int)(e / N), n = (int)(e - (long long)m * N);
  const long long off = row_off(c, m);
  if (off < 0) return;
  float s = 0.f;
  for (int k = 0; k < ksplit; ++k) s += slab[k * MN + e];
  float v = alpha * s;
  if (bias) v += bias[n];
  if (bias2) v += bias2[n];
  float* crow = (float*)c.base + off;
  if (beta != 0.f) v += beta * crow[n];
  if (drop_p > 0.f)
    v *= u01(drop_seed, (unsigned long long)(off + n)) >= drop_p ? 1.f / (1.f - drop_p) : 0.f;
  crow[n] = v;
}

// splitk_reduce over 4 columns per thread (N % 4 == 0, C rows 16-B aligned):
// 16-B slab / C accesses, 32-bit index math (M * N < 2^31), same fixed order.
__global__ void splitk_reduce4(const float* __restrict__ slab, int ksplit, int M, int N, RowMap c,
                               float alpha, float beta, const float* __restrict__ bias,
                               const float* __restrict__ bias2, float drop_p,
                               unsigned long long drop_seed) {
  const int MN = M * N;
  const int e = 4 * (blockIdx.x * 256 + threadIdx.x);
  if (e >= MN) return;
  const int m = e / N, n = e - m * N;
  const long long off = row_off(c, m);
  if (off < 0) return;
  float4 s = *reinterpret_cast<const float4*>(slab + e);
  for (int k = 1; k < ksplit; ++k) {
    const float4 t = *reinterpret_cast<const float4*>(slab + (long long)k * MN + e);
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  }
  float v[4] = {alpha * s.x, alpha * s.y, alpha * s.z, alpha * s.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (bias) v[q] += bias[n + q];
    if (bias2) v[q] += bias2[n + q];
  }
  float* crow = (float*)c.base + off + n;
  if (beta != 0.f) {
    const float4 o = *reinterpret_cast<const float4*>(crow);
    v[0] += beta * o.x; v[1] += beta * o.y; v[2] += beta * o.z; v[3] += beta * o.w;
  }
  if (drop_p > 0.f) drop_n<4>(v, drop_p, drop_seed, (unsigned long long)(off + n));
  *reinterpret_cast<float4*>(crow) = make_float4(v[0], v[1], v[2], v[3]);
}

// Column sums: partial[chunk][n] = sum over rows of chunk; then ordered final sum.
// One (64-column, row chunk) tile per work-group: 4 waves split the chunk's
// rows (wave w takes rows w, w + 4, ...), each lane keeps eight rows' loads in
// flight; the waves' sums are combined in LDS in wave order (deterministic).
__device__ __forceinline__ float colsum_ld(const float* g, long long i) { return g[i]; }
__device__ __forceinline__ float colsum_ld(const uint16_t* g, long long i) { return bf2f(g[i]); }

template <typename TG>
__global__ void __launch_bounds__(256) colsum_partial(const TG* __restrict__ g, long long ld,
                                                      int M, int N, int rows_per_chunk,
                                                      float* __restrict__ partial) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + lane;
  const int chunk = blockIdx.y;
  const int m0 = chunk * rows_per_chunk, m1 = min(M, m0 + rows_per_chunk);
  float s0 = 0.f, s1 = 0.f;
  if (n < N) {
    int m = m0 + w;
    for (; m + 28 < m1; m += 32) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = colsum_ld(g, (long long)(m + 4 * j) * ld + n);
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        s0 += v[j];
        s1 += v[j + 1];
      }
    }
    for (; m < m1; m += 4) s0 += colsum_ld(g, (long long)m * ld + n);
  }
  red[w][lane] = s0 + s1;
  __syncthreads();
  if (w == 0 && n < N)
    partial[(long long)chunk * N + n] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}
// 16 columns x 16 phases per 256-thread block (phase q sums chunks q, q + 16,
// ... in order; phases combined in order): one thread per column walking all
// chunks was a latency chain for the narrow bias vectors (~11 us per call)
__global__ void __launch_bounds__(256) colsum_final(const float* __restrict__ partial, int nchunk,
                                                    int N, float alpha, float* __restrict__ out0,
                                                    float* __restrict__ out1) {
  __shared__ float red[256];
  const int cl = threadIdx.x & 15, q0 = threadIdx.x >> 4;
  const int n = blockIdx.x * 16 + cl;
  float s0 = 0.f, s1 = 0.f;
  if (n < N) {
    int c = q0;
    for (; c + 16 < nchunk; c += 32) {
      s0 += partial[(long long)c * N + n];
      s1 += partial[(long long)(c + 16) * N + n];
    }
    for (; c < nchunk; c += 16) s0 += partial[(long long)c * N + n];
  }
  red[threadIdx.x] = s0 + s1;
  __syncthreads();
  if (q0 == 0 && n < N) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += red[j * 16 + cl];
    s *= alpha;
    out0[n] += s;
    if (out1) out1[n] += s;
  }
}

RowMap make_map(const asr_rowmap_t& m, const void* base) {
  RowMap r;
  r.base = base;
  r.stride_b = m.stride_b;
  r.stride_t = m.stride_t;
  r.rows_per_b = m.rows_per_b > 0 ? m.rows_per_b : 0x7fffffff;
  r.t_mul = m.t_mul == 0 ? 1 : m.t_mul;
  r.t_add = m.t_add;
  r.t_limit = m.t_limit > 0 ? m.t_limit : 0x7fffffff;
  r.perm = m.perm;
  return r;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int fill_operand(const asr_operand_t& o, Operand* op, const char* name) {
  ASR_REQUIRE(o.ptr, ASR_ERR_ARG, "gemm: operand %s is null", name);
  ASR_REQUIRE(o.dtype == ASR_DT_F32 || o.dtype == ASR_DT_BF16, ASR_ERR_ARG,
              "gemm: operand %s bad dtype", name);
  op->map = make_map(o.map, o.ptr);
  op->dtype = o.dtype;
  op->trans = o.trans;
  const int esz = o.dtype == ASR_DT_F32 ? 4 : 2;
  const int vec = o.dtype == ASR_DT_F32 ? 4 : 8;
  op->vec_ok = aligned16(o.ptr) && (o.map.stride_t % vec == 0) && (o.map.stride_b % vec == 0);
  op->bytes = o.bytes;
  op->tap_g = o.tap_group;
  op->tap_w = o.tap_pitch;
  op->tap_s = o.tap_sign ? o.tap_sign : 1;
  op->plain = (o.map.rows_per_b <= 0 && (o.map.t_mul == 0 || o.map.t_mul == 1) &&
               o.map.t_add == 0 && !o.map.perm) ? 1 : 0;
  // StageF: tap operands need the plain map; ASR_GEMM_STAGEF=0 keeps the
  // per-DMA row map (A/B)
  {
    const char* e = getenv("ASR_GEMM_STAGEF");
    op->sf = !(e && e[0] == '0') && (!o.tap_group || op->plain) && !o.map.perm;
  }
  if (o.tap_group)
    ASR_REQUIRE(o.tap_group > 0 && o.tap_group % (o.trans ? 8 : 16) == 0 && !o.map.perm,
                ASR_ERR_ARG, "gemm: operand %s tap_group %d unsupported", name, o.tap_group);
  (void)esz;
  return ASR_OK;
}

// Split-K plan (pure function of the shapes): a launch with fewer than two
// waves of 128x128 tiles over 256 CUs and K >= 1024 is split into ~1024 work
// groups, each K chunk >= 128 (a multiple of the fast path's k-tile).
struct SplitPlan {
  int ksplit[2], kchunk[2];
  size_t slab_off[2];
  size_t bytes;
};

// asr_gemm_set_nosplit(1): launches from this host thread take no split-K
// slabs until reset (products whose rows are computed in several launches
// that must sum each output element in the same order as one launch would)
thread_local int g_nosplit = 0;

SplitPlan plan_split(const asr_gemm_t* g, int nprob) {
  SplitPlan sp{};
  const char* ns = getenv("ASR_GEMM_NOSPLIT");   // diagnostics: no split-K slabs
  const bool nosplit = (ns && ns[0] == '1') || g_nosplit;
  for (int i = 0; i < nprob; ++i) {
    // per problem: the problems of one launch run side by side (blockIdx.z), so
    // a few-tile dW next to a many-tile dX still gets its own K split
    const int tiles = ceil_div(g[i].M, BM) * ceil_div(g[i].N, BN);
    int ks = 1;
    if (!nosplit && g[i].c_dtype != ASR_DT_BF16 && g[i].batch <= 1 && tiles > 0 &&
        tiles < 512 && g[i].K >= 1024) {
      // a few-tile, long-K product (the decoder / projection weight gradients,
      // K = B*S or B*T) is latency-bound per work-group: chunks >= 128
      ks = min(ceil_div(1024, tiles), g[i].K / 128);
      const long long mn = (long long)g[i].M * g[i].N;
      while (ks > 1 && (long long)ks * mn * 4 > (64LL << 20)) --ks;  // slab <= 64 MB
      ks = max(ks, 1);
    }
    int kc = g[i].K;
    if (ks > 1) {
      kc = ceil_div(ceil_div(g[i].K, ks), 64) * 64;  // whole fast-path k-tiles
      ks = ceil_div(g[i].K, kc);
    }
    sp.ksplit[i] = ks;
    sp.kchunk[i] = kc;
    sp.slab_off[i] = sp.bytes;
    if (ks > 1) sp.bytes += ((size_t)ks * g[i].M * g[i].N * sizeof(float) + 255) & ~(size_t)255;
  }
  return sp;
}

// The bf16 fast path's operand mode pair (2*a.trans + b.trans) when every
// problem of the launch qualifies and all share it, else -1 (generic kernel).
bool fast_operand_ok(const asr_operand_t& o, const Operand& op, long long batch_stride,
                     int batch, int kdim) {
  if (o.dtype != ASR_DT_BF16 || o.bytes <= 0 || o.bytes > 0x7fff0000LL) return false;
  if (o.map.perm) return false;
  if (!aligned16(o.ptr) || o.map.stride_t % 8 || o.map.stride_b % 8) return false;
  if (batch > 1 && batch_stride % 8) return false;
  if (!o.trans && kdim % 8) return false;
  (void)op;
  return true;
}

// LDS stages of the bf16 fast path (ASR_GEMM_STAGES = 2 | 4, default 2: the
// 4-deep ring halves occupancy and measured 226 vs 391 TF/s on the encoder
// products); the 128 KB ring needs the dynamic-LDS limit raised once per kernel.
int fast_stages() {
  static int n = 0;
  if (n == 0) {
    const char* e = getenv("ASR_GEMM_STAGES");
    n = (e && atoi(e) == 4) ? 4 : 2;
    if (n == 4) {
      const int bytes = 4 * 2 * FTILE;
      bool ok = true;
      ok &= hipFuncSetAttribute((const void*)gemm_bf16_fast<0, 0, 4>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess;
      ok &= hipFuncSetAttribute((const void*)gemm_bf16_fast<0, 1, 4>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess;
      ok &= hipFuncSetAttribute((const void*)gemm_bf16_fast<1, 0, 4>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess;
      ok &= hipFuncSetAttribute((const void*)gemm_bf16_fast<1, 1, 4>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess;
      if (!ok) n = 2;
    }
  }
  return n;
}

// The f32 fast path's operand mode pair, or -1 (gemm_kernel<false>).  Every
// operand f32 with a known extent < 2 GiB and 16-B aligned rows; a batch
// permutation is allowed, taps need a plain map.  ASR_GEMM_F32FAST=0 keeps
// the generic kernel.
bool fast32_operand_ok(const asr_operand_t& o, const Operand& op, long long batch_stride,
                       int batch, int kdim) {
  if (o.dtype != ASR_DT_F32 || o.bytes <= 0 || o.bytes > 0x7fff0000LL) return false;
  // the division-free staging (taps only on a plain map); a batch permutation
  // is applied once per R-mode row and once per utterance crossing in K mode
  if (o.tap_group && !op.plain) return false;
  if (!aligned16(o.ptr) || o.map.stride_t % 4 || o.map.stride_b % 4) return false;
  if (batch > 1 && batch_stride % 4) return false;
  (void)kdim;   // R mode: a k extent that is not a multiple of 4 is zero-filled in LDS
  return true;
}

int fast32_modes(const asr_gemm_t* g, const Params& P) {
  const char* e = getenv("ASR_GEMM_F32FAST");
  if (e && e[0] == '0') return -1;
  // diagnostics: ASR_GEMM_F32FAST_MASK (bit m: layout mode m may take the
  // kernel), ASR_GEMM_F32FAST_NOTAP=1 (no tap-addressed operand)
  const char* em = getenv("ASR_GEMM_F32FAST_MASK");
  const int mask = em ? atoi(em) : 15;
  const char* et = getenv("ASR_GEMM_F32FAST_NOTAP");
  const bool notap = et && et[0] == '1';
  int modes = -1;
  for (int i = 0; i < P.nprob; ++i) {
    const Problem& p = P.p[i];
    if (!fast32_operand_ok(g[i].a, p.a, p.sA, p.batch, p.K) ||
        !fast32_operand_ok(g[i].b, p.b, p.sB, p.batch, p.K))
      return -1;
    if (notap && (g[i].a.tap_group || g[i].b.tap_group)) return -1;
    const int m = 2 * (g[i].a.trans ? 1 : 0) + (g[i].b.trans ? 1 : 0);
    if (modes >= 0 && m != modes) return -1;
    modes = m;
  }
  if (modes >= 0 && !((mask >> modes) & 1)) return -1;
  return modes;
}

int fast_modes(const asr_gemm_t* g, const Params& P) {
  if (getenv("ASR_GEMM_FAST") && getenv("ASR_GEMM_FAST")[0] == '0') return -1;
  int modes = -1;
  for (int i = 0; i < P.nprob; ++i) {
    const Problem& p = P.p[i];
    if (!fast_operand_ok(g[i].a, p.a, p.sA, p.batch, p.K) ||
        !fast_operand_ok(g[i].b, p.b, p.sB, p.batch, p.K))
      return -1;
    const int m = 2 * (g[i].a.trans ? 1 : 0) + (g[i].b.trans ? 1 : 0);
    if (modes >= 0 && m != modes) return -1;
    modes = m;
  }
  return modes;
}

// K-major x K-major problems with both output extents >= 256 take the 256 x 256
// kernel when ASR_GEMM_KK256=1 (read per launch).  Off by default: at the
// 5x512 weight-gradient shapes it measured 511 vs 482 TF/s (tools/gemm_bench.py)
// but the whole step did not move beyond noise, and the 4x320 / VGG configs
// ran 0.2-0.5 ms/step slower with it (fewer work-groups per product).
bool kk256_ok(const asr_gemm_t* g, int nprob) {
  for (int i = 0; i < nprob; ++i)
    if (g[i].c_dtype == ASR_DT_BF16) return false;   // its own f32 epilogue
  const char* e = getenv("ASR_GEMM_KK256");
  if (!(e && e[0] == '1')) return false;
  for (int i = 0; i < nprob; ++i)
    if (g[i].M < BT2 || g[i].N < BT2) return false;
  return true;
}

// Problems whose output extents both reach a 256-row tile take the 8-wave
// 256 x 256 kernel (ASR_GEMM_8W=0 keeps them on the 128 x 128 kernel; read per
// launch, for A/B runs).
// Work-groups a split-K product of the 8-wave kernel aims for (ASR_GEMM_SPLITWG,
// default 512: two per CU); fewer splits mean smaller f32 slabs to reduce.
int split_target() {
  const char* e = getenv("ASR_GEMM_SPLITWG");
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : 512;
}

// asr_gemm_set_small_tiles(1): launches from this host thread keep to the
// 128 x 128 kernel (64 KB of LDS) until reset -- the weight-gradient GEMMs that
// run co-resident with the persistent backward recurrence (native_ops,
// ASR_OVERLAP_WGRAD=2) must fit beside its work-group on every CU.
thread_local int g_small_tiles = 0;
thread_local float* g_row_lse = nullptr;   // asr_gemm_lse_ws: the product's row-LSE partials
thread_local int g_n64_kmode = 0;

// Products with N <= 64 and many rows take the 256 x 64 kernel (B in R mode;
// ASR_GEMM_N64=0 keeps them on the 128 x 128 kernel; read per launch).
bool n64_ok(const asr_gemm_t* g, int nprob, int bmode) {
  if (g_small_tiles) return false;
  const char* e = getenv("ASR_GEMM_N64");
  if (e && e[0] == '0') return false;
  // K-mode B (its tile keeps the 128-column layout, 96 KB of LDS): opt-in per
  // launch thread (asr_gemm_set_n64_kmode), used by the VGG weight gradients
  if (bmode && !g_n64_kmode) return false;
  for (int i = 0; i < nprob; ++i)   // many rows, or a long K that split-K spreads
    if (g[i].N > 64 || (g[i].M < 4096 && g[i].K < 65536)) return false;
  return true;
}


bool big8_ok(const asr_gemm_t* g, int nprob) {
  const char* e = getenv("ASR_GEMM_8W");
  if (e && e[0] == '0') return false;
  if (g_small_tiles) return false;
  for (int i = 0; i < nprob; ++i) {
    if (g[i].c_dtype == ASR_DT_BF16) return false;   // its own f32 epilogue
    if (g[i].M < T8 || g[i].N < T8) return false;
    if (g[i].a.tap_group || g[i].b.tap_group) return false;     // taps: 128 x 128 kernel
    // K-mode operands advance their (utterance, frame) pair by 64 k-rows per tile
    for (const asr_operand_t* o : {&g[i].a, &g[i].b})
      if (o->trans && o->map.rows_per_b > 0 && o->map.rows_per_b < BK8) return false;
  }
  return true;
}

int gemm_launch_own(const asr_gemm_t* problems, int nprob, int compute_dtype, void* workspace,
                    size_t ws_bytes, void* stream) {
  SplitPlan sp{};
  if (workspace) {
    sp = plan_split(problems, nprob);
    ASR_REQUIRE(ws_bytes >= sp.bytes, ASR_ERR_WORKSPACE, "gemm: workspace too small");
  } else {
    for (int i = 0; i < nprob; ++i) { sp.ksplit[i] = 1; sp.kchunk[i] = problems[i].K; }
  }
  Params P;
  P.nprob = nprob;
  int maxwg = 0, maxb = 1;
  for (int i = 0; i < nprob; ++i) {
    const asr_gemm_t& g = problems[i];
    ASR_REQUIRE(g.M >= 0 && g.N >= 0 && g.K >= 0, ASR_ERR_ARG, "gemm: negative size");
    Problem& p = P.p[i];
    int rc = fill_operand(g.a, &p.a, "A");
    if (rc) return rc;
    rc = fill_operand(g.b, &p.b, "B");
    if (rc) return rc;
    ASR_REQUIRE(g.c, ASR_ERR_ARG, "gemm: C is null");
    p.c = make_map(g.c_map, g.c);
    p.bias = g.bias;
    p.bias2 = g.bias2;
    p.M = g.M; p.N = g.N; p.K = g.K;
    p.alpha = g.alpha;
    p.beta = g.beta;
    ASR_REQUIRE(g.drop_p >= 0.f && g.drop_p < 1.f, ASR_ERR_ARG, "gemm: dropout p outside [0, 1)");
    ASR_REQUIRE(g.drop_p == 0.f || g.batch <= 1, ASR_ERR_ARG, "gemm: dropout on a batched product");
    p.drop_p = g.drop_p;
    p.drop_seed = g.drop_seed;
    p.lse = nullptr;
    ASR_REQUIRE(g.c_dtype == ASR_DT_F32 || g.c_dtype == ASR_DT_BF16, ASR_ERR_ARG,
                "gemm: C dtype %d", g.c_dtype);
    p.c_bf16 = g.c_dtype == ASR_DT_BF16;
    ASR_REQUIRE(!p.c_bf16 || (g.beta == 0.f && compute_dtype == ASR_DT_BF16), ASR_ERR_ARG,
                "gemm: bf16 C needs beta 0 and bf16 compute");
    p.batch = g.batch > 1 ? g.batch : 1;
    p.sA = g.batch_stride_a;
    p.sB = g.batch_stride_b;
    p.sC = g.batch_stride_c;
    if (p.batch > 1)  // vector loads stay legal only if every batch base stays 16-B aligned
      ASR_REQUIRE(p.sA >= 0 && p.sB >= 0 && p.sC >= 0, ASR_ERR_ARG, "gemm: batch strides");
    if (p.batch > 1 && (p.sA % 8 || p.sB % 8)) { p.a.vec_ok = 0; p.b.vec_ok = 0; }
    p.ksplit = sp.ksplit[i];
    p.kchunk = sp.kchunk[i];
    p.slab = p.ksplit > 1 ? (float*)((char*)workspace + sp.slab_off[i]) : nullptr;
    maxwg = max(maxwg, ceil_div(g.M, BM) * ceil_div(g.N, BN) * p.ksplit);
    maxb = max(maxb, p.batch);
  }
  if (g_row_lse) {   // asr_gemm_lse_ws: one product, whole-K tiles (no split slabs)
    P.p[0].lse = g_row_lse;
    P.p[0].ksplit = 1;
    P.p[0].kchunk = P.p[0].K;
    P.p[0].slab = nullptr;
    maxwg = ceil_div(problems[0].M, BM) * ceil_div(problems[0].N, BN);
  }
  if (nprob == 1) { P.p[1] = P.p[0]; P.p[1].batch = 0; }
  if (maxwg == 0) return ASR_OK;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(maxwg, 1, nprob * maxb);
  ASR_REQUIRE(grid.z <= 65535, ASR_ERR_ARG, "gemm: batch too large");
  double flops = 0.0;
  for (int i = 0; i < nprob; ++i)
    flops += 2.0 * problems[i].M * problems[i].N * problems[i].K * P.p[i].batch;
  const int slot = prof_begin_launch(ASR_PROF_GEMM, s, flops);
  const int fast = compute_dtype == ASR_DT_BF16 ? fast_modes(problems, P) : -1;
  if (fast >= 0 && big8_ok(problems, nprob)) {
    // 256 x 256 8-wave kernel; the split never exceeds the workspace plan's
    int maxwg8 = 0;
    for (int i = 0; i < nprob; ++i) {
      Problem& p = P.p[i];
      const int tiles8 = ceil_div(p.M, T8) * ceil_div(p.N, T8);
      int ks = 1;
      if (p.ksplit > 1) {
        ks = min(p.ksplit, max(1, ceil_div(split_target(), tiles8)));
        const int kc = ceil_div(ceil_div(p.K, ks), BK8) * BK8;
        ks = ceil_div(p.K, kc);
        p.kchunk = kc;
      }
      if (ks <= 1) { ks = 1; p.kchunk = p.K; }
      p.ksplit = ks;
      maxwg8 = max(maxwg8, tiles8 * ks);
    }
    static bool attr8 = false;
    if (!attr8) {
      bool ok = true;
      ok &= hipFuncSetAttribute((const void*)gemm_bf16_8w<0, 0>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 4 * TILE8) == hipSuccess;
      ok &= hipFuncSetAttribute((const void*)gemm_bf16_8w<0, 1>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 4 * TILE8) == hipSuccess;
      ok &= hipFuncSetAttribute((const void*)gemm_bf16_8w<1, 0>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 4 * TILE8) == hipSuccess;
      ok &= hipFuncSetAttribute((const void*)gemm_bf16_8w<1, 1>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 4 * TILE8) == hipSuccess;
      ASR_REQUIRE(ok, ASR_ERR_HIP, "gemm: cannot raise the LDS limit of the 8-wave kernel");
      attr8 = true;
    }
    const dim3 g8(maxwg8, 1, nprob * maxb);
    const size_t lds8 = 4 * TILE8;
    const char* er = getenv("ASR_GEMM_8R");   // ring form by default (ASR_GEMM_8R=0: two buffers)
    prof_set_tag(ASR_PROF_GEMM, slot, 4 * ((er && er[0] == '0') ? ASR_PTAG_GEMM_8W : ASR_PTAG_GEMM_8R) + fast);
    if (!(er && er[0] == '0')) {
      static bool attrr = false;
      const int ldsr = NSLOT * 2 * TILER;
      if (!attrr) {
        bool ok = true;
        ok &= hipFuncSetAttribute((const void*)gemm_bf16_8r<0, 0>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, ldsr) == hipSuccess;
        ok &= hipFuncSetAttribute((const void*)gemm_bf16_8r<0, 1>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, ldsr) == hipSuccess;
        ok &= hipFuncSetAttribute((const void*)gemm_bf16_8r<1, 0>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, ldsr) == hipSuccess;
        ok &= hipFuncSetAttribute((const void*)gemm_bf16_8r<1, 1>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, ldsr) == hipSuccess;
        ASR_REQUIRE(ok, ASR_ERR_HIP, "gemm: cannot raise the LDS limit of the ring kernel");
        attrr = true;
      }
      switch (fast) {
        case 0: hipLaunchKernelGGL((gemm_bf16_8r<0, 0>), g8, dim3(NT8), ldsr, s, P); break;
        case 1: hipLaunchKernelGGL((gemm_bf16_8r<0, 1>), g8, dim3(NT8), ldsr, s, P); break;
        case 2: hipLaunchKernelGGL((gemm_bf16_8r<1, 0>), g8, dim3(NT8), ldsr, s, P); break;
        default: hipLaunchKernelGGL((gemm_bf16_8r<1, 1>), g8, dim3(NT8), ldsr, s, P); break;
      }
    } else switch (fast) {
      case 0: hipLaunchKernelGGL((gemm_bf16_8w<0, 0>), g8, dim3(NT8), lds8, s, P); break;
      case 1: hipLaunchKernelGGL((gemm_bf16_8w<0, 1>), g8, dim3(NT8), lds8, s, P); break;
      case 2: hipLaunchKernelGGL((gemm_bf16_8w<1, 0>), g8, dim3(NT8), lds8, s, P); break;
      default: hipLaunchKernelGGL((gemm_bf16_8w<1, 1>), g8, dim3(NT8), lds8, s, P); break;
    }
  } else if (fast == 3 && !g_row_lse && kk256_ok(problems, nprob)) {
    // 256 x 256 tiles; the split never exceeds the workspace plan's (128 x 128) split
    int maxwg2 = 0;
    for (int i = 0; i < nprob; ++i) {
      Problem& p = P.p[i];
      const int tiles2 = ceil_div(p.M, BT2) * ceil_div(p.N, BT2);
      int ks = 1;
      if (p.ksplit > 1) {
        ks = min(p.ksplit, max(1, ceil_div(256, tiles2)));
        const int kc = ceil_div(ceil_div(p.K, ks), BK2) * BK2;
        ks = ceil_div(p.K, kc);
        p.kchunk = kc;
      }
      if (ks <= 1) { ks = 1; p.kchunk = p.K; }
      p.ksplit = ks;
      maxwg2 = max(maxwg2, tiles2 * ks);
    }
    static bool attr = false;
    if (!attr) {
      ASR_REQUIRE(hipFuncSetAttribute((const void*)gemm_bf16_kk256,
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      NST2 * 2 * FTILE2) == hipSuccess,
                  ASR_ERR_HIP, "gemm: cannot raise the LDS limit of the 256x256 kernel");
      attr = true;
    }
    prof_set_tag(ASR_PROF_GEMM, slot, 4 * ASR_PTAG_GEMM_KK256 + fast);
    hipLaunchKernelGGL(gemm_bf16_kk256, dim3(maxwg2, 1, nprob * maxb), dim3(NT),
                       (size_t)NST2 * 2 * FTILE2, s, P);
  } else if (fast >= 0 && n64_ok(problems, nprob, fast & 1)) {
    // ASR_GEMM_N64_STAGES=3: the three-stage ring (read per launch)
    const char* n64e = getenv("ASR_GEMM_N64_STAGES");
    const int n64st = (n64e && n64e[0] == '3') ? 3 : 2;
    static bool attr64 = false;
    if (!attr64) {
      bool ok = true;
#define ASR_N64_ATTR(A, B, NS)                                                               \
  ok &= hipFuncSetAttribute((const void*)gemm_bf16_n64<A, B, NS>,                            \
                            hipFuncAttributeMaxDynamicSharedMemorySize, NS * n64_stage(B)) ==   \
        hipSuccess
      ASR_N64_ATTR(0, 0, 2); ASR_N64_ATTR(1, 0, 2); ASR_N64_ATTR(0, 1, 2); ASR_N64_ATTR(1, 1, 2);
      ASR_N64_ATTR(0, 0, 3); ASR_N64_ATTR(1, 0, 3); ASR_N64_ATTR(0, 1, 3); ASR_N64_ATTR(1, 1, 3);
#undef ASR_N64_ATTR
      ASR_REQUIRE(ok, ASR_ERR_HIP, "gemm: cannot raise the LDS limit of the 256x64 kernel");
      attr64 = true;
    }
    int maxwg64 = 0;
    for (int i = 0; i < nprob; ++i)
      maxwg64 = max(maxwg64, ceil_div(P.p[i].M, N64_BM) * max(1, P.p[i].ksplit));
    const dim3 g64(maxwg64, 1, nprob * maxb);
    prof_set_tag(ASR_PROF_GEMM, slot, 4 * ASR_PTAG_GEMM_N64 + fast);
#define ASR_N64(A, B)                                                                          \
  do {                                                                                         \
    if (n64st == 3)                                                                            \
      hipLaunchKernelGGL((gemm_bf16_n64<A, B, 3>), g64, dim3(NT), 3 * n64_stage(B), s, P);     \
    else                                                                                       \
      hipLaunchKernelGGL((gemm_bf16_n64<A, B, 2>), g64, dim3(NT), 2 * n64_stage(B), s, P);     \
  } while (0)
    switch (fast) {
      case 0: ASR_N64(0, 0); break;
      case 2: ASR_N64(1, 0); break;
      case 1: ASR_N64(0, 1); break;
      default: ASR_N64(1, 1); break;
    }
#undef ASR_N64
  } else if (fast >= 0) {
    const int nst = g_small_tiles ? 2 : fast_stages();
    const size_t lds = (size_t)nst * 2 * FTILE;
    prof_set_tag(ASR_PROF_GEMM, slot,
                 4 * (nst == 4 ? ASR_PTAG_GEMM_FAST4 : ASR_PTAG_GEMM_FAST2) + fast);
    switch (fast) {
#define ASR_FAST(A, B)                                                                   \
  do {                                                                                   \
    if (nst == 4) hipLaunchKernelGGL((gemm_bf16_fast<A, B, 4>), grid, dim3(NT), lds, s, P); \
    else hipLaunchKernelGGL((gemm_bf16_fast<A, B, 2>), grid, dim3(NT), lds, s, P);          \
  } while (0)
      case 0: ASR_FAST(0, 0); break;
      case 1: ASR_FAST(0, 1); break;
      case 2: ASR_FAST(1, 0); break;
      default: ASR_FAST(1, 1); break;
#undef ASR_FAST
    }
  } else if (compute_dtype == ASR_DT_BF16) {
    static bool warned = false;   // a bf16-mode product of real size on the slow path: say so once
    if (!warned && !getenv("ASR_GEMM_DEBUG")) {
      for (int i = 0; i < nprob; ++i) {
        const double fl = 2.0 * problems[i].M * problems[i].N * problems[i].K * problems[i].batch;
        if (fl >= 32e6) {
          warned = true;
          fprintf(stderr, "[asr_gemm] warning: a bf16-mode product (M=%d N=%d K=%d batch=%d) runs "
                  "on the generic register-staged kernel, not the LDS-DMA fast kernels "
                  "(ASR_GEMM_DEBUG=1 lists every such product)\n", problems[i].M, problems[i].N,
                  problems[i].K, problems[i].batch);
          break;
        }
      }
    }
    if (getenv("ASR_GEMM_DEBUG"))   // which bf16-mode products miss the fast kernels
      for (int i = 0; i < nprob; ++i)
        fprintf(stderr, "[asr_gemm generic] M=%d N=%d K=%d batch=%d a(dt=%d tr=%d tap=%d perm=%d) "
                "b(dt=%d tr=%d tap=%d perm=%d)\n", problems[i].M, problems[i].N, problems[i].K,
                problems[i].batch, problems[i].a.dtype, problems[i].a.trans,
                problems[i].a.tap_group, problems[i].a.map.perm != nullptr, problems[i].b.dtype,
                problems[i].b.trans, problems[i].b.tap_group, problems[i].b.map.perm != nullptr);
    const size_t lds = 2 * BM * LDB16 * 2;
    prof_set_tag(ASR_PROF_GEMM, slot, 4 * ASR_PTAG_GEMM_GEN_BF16);
    hipLaunchKernelGGL(gemm_kernel<true>, grid, dim3(NT), lds, s, P);
  } else if (const int f32m = fast32_modes(problems, P); f32m >= 0) {
    // tile shape: 256 x 64 when every N <= 64, 64 x 256 when every M <= 64
    bool n64 = true, m64 = true;
    for (int i = 0; i < nprob; ++i) {
      n64 &= problems[i].N <= 64;
      m64 &= problems[i].M <= 64;
    }
    const int tmw = n64 ? 4 : m64 ? 1 : 2;
    const int tmr = 64 * tmw, tnr = 256 / tmw;
    int wg32 = 0;
    for (int i = 0; i < nprob; ++i)
      wg32 = max(wg32, ceil_div(P.p[i].M, tmr) * ceil_div(P.p[i].N, tnr) * max(1, P.p[i].ksplit));
    const dim3 g32(wg32, 1, nprob * maxb);
    const size_t lds = 2 * (size_t)(tmr + tnr) * FBK32 * 4;
    prof_set_tag(ASR_PROF_GEMM, slot, 4 * ASR_PTAG_GEMM_F32F + f32m);
    const char* fst = getenv("ASR_GEMM_F32_STAGES");   // 3: the ring (A/B; read per launch)
    const bool ring = fst && fst[0] == '3';
    if (ring) {
      static bool attr = false;
      if (!attr) {
        attr = true;
#define ASR_F32R_ATTR(A, B, TW)                                                                  \
  (void)hipFuncSetAttribute((const void*)gemm_f32_fast<A, B, TW, 3>,                             \
                            hipFuncAttributeMaxDynamicSharedMemorySize, 3 * 320 * FBK32 * 4)
        ASR_F32R_ATTR(0, 0, 1); ASR_F32R_ATTR(0, 0, 2); ASR_F32R_ATTR(0, 0, 4);
        ASR_F32R_ATTR(0, 1, 1); ASR_F32R_ATTR(0, 1, 2); ASR_F32R_ATTR(0, 1, 4);
        ASR_F32R_ATTR(1, 0, 1); ASR_F32R_ATTR(1, 0, 2); ASR_F32R_ATTR(1, 0, 4);
        ASR_F32R_ATTR(1, 1, 1); ASR_F32R_ATTR(1, 1, 2); ASR_F32R_ATTR(1, 1, 4);
#undef ASR_F32R_ATTR
      }
    }
    const size_t ldsr = ring ? lds / 2 * 3 : lds;
#define ASR_F32F(A, B)                                                                           \
  do {                                                                                           \
    if (ring) {                                                                                  \
      if (tmw == 4) hipLaunchKernelGGL((gemm_f32_fast<A, B, 4, 3>), g32, dim3(NT), ldsr, s, P);   \
      else if (tmw == 1) hipLaunchKernelGGL((gemm_f32_fast<A, B, 1, 3>), g32, dim3(NT), ldsr, s, P); \
      else hipLaunchKernelGGL((gemm_f32_fast<A, B, 2, 3>), g32, dim3(NT), ldsr, s, P);            \
    } else if (tmw == 4) hipLaunchKernelGGL((gemm_f32_fast<A, B, 4>), g32, dim3(NT), lds, s, P);  \
    else if (tmw == 1) hipLaunchKernelGGL((gemm_f32_fast<A, B, 1>), g32, dim3(NT), lds, s, P);    \
    else hipLaunchKernelGGL((gemm_f32_fast<A, B, 2>), g32, dim3(NT), lds, s, P);                  \
  } while (0)
    switch (f32m) {
      case 0: ASR_F32F(0, 0); break;
      case 1: ASR_F32F(0, 1); break;
      case 2: ASR_F32F(1, 0); break;
      default: ASR_F32F(1, 1); break;
    }
#undef ASR_F32F
  } else {
    if (getenv("ASR_GEMM_DEBUG"))   // which fp32-mode products miss the f32 fast kernel
      for (int i = 0; i < nprob; ++i)
        fprintf(stderr, "[asr_gemm generic f32] M=%d N=%d K=%d batch=%d a(dt=%d tr=%d tap=%d "
                "perm=%d ld=%lld al=%d) b(dt=%d tr=%d tap=%d perm=%d ld=%lld al=%d)\n",
                problems[i].M, problems[i].N, problems[i].K, problems[i].batch,
                problems[i].a.dtype, problems[i].a.trans, problems[i].a.tap_group,
                problems[i].a.map.perm != nullptr, problems[i].a.map.stride_t,
                (int)aligned16(problems[i].a.ptr), problems[i].b.dtype, problems[i].b.trans,
                problems[i].b.tap_group, problems[i].b.map.perm != nullptr,
                problems[i].b.map.stride_t, (int)aligned16(problems[i].b.ptr));
    const size_t lds = 2 * BM * LDF32 * 4;
    prof_set_tag(ASR_PROF_GEMM, slot, 4 * ASR_PTAG_GEMM_GEN_F32);
    hipLaunchKernelGGL(gemm_kernel<false>, grid, dim3(NT), lds, s, P);
  }
  ASR_LAUNCH_CHECK();
  prof_end_launch(ASR_PROF_GEMM, slot, s);
  for (int i = 0; i < nprob; ++i) {
    const Problem& p = P.p[i];
    if (p.ksplit <= 1) continue;
    const long long mn = (long long)p.M * p.N;
    if (mn == 0) continue;
    const bool v4 = p.N % 4 == 0 && mn < 0x7fffffffLL && ((uintptr_t)p.c.base & 15) == 0 &&
                    p.c.stride_t % 4 == 0 && p.c.stride_b % 4 == 0;
    if (v4)
      hipLaunchKernelGGL(splitk_reduce4, dim3((unsigned)((mn / 4 + 255) / 256)), dim3(256), 0, s,
                         p.slab, p.ksplit, p.M, p.N, p.c, p.alpha, p.beta, p.bias, p.bias2,
                         p.drop_p, p.drop_seed);
    else
      hipLaunchKernelGGL(splitk_reduce, dim3((unsigned)((mn + 255) / 256)), dim3(256), 0, s,
                         p.slab, p.ksplit, p.M, p.N, p.c, p.alpha, p.beta, p.bias, p.bias2,
                         p.drop_p, p.drop_seed);
    ASR_LAUNCH_CHECK();
  }
  return ASR_OK;
}

// bf16 staging of f32 operands.  In bf16 mode a product with an f32 operand
// (the decoder / bottleneck / attention projections fed by f32 activations)
// would run on the generic register-staged kernel, converting inside its
// loads (30-50 TF/s at these shapes).  A product of at least STAGE_FLOPS
// instead stages each f32 operand once into a dense bf16 copy in the workspace
// (one convert_rows pass through the operand's row map) and takes the fast /
// 8-wave kernels; the arithmetic is unchanged (bf16 operands, f32 accumulate).
// ASR_GEMM_STAGE=0 keeps the generic kernel (A/B).
constexpr double STAGE_FLOPS = 3.2e7;
}  // namespace
// elementwise.hip: up to four conversions in one launch (1), or 0 (not eligible)
int convert_rows_bf16_multi(const float* const* src, const asr_rowmap_t* maps, const int* nrows,
                            const int* ncols, uint16_t* const* dst, int n, void* stream);
namespace {

struct StagePlan {
  bool on[2][2];
  int rows[2][2], cols[2][2], ld[2][2];
  size_t off[2][2];
  size_t bytes;
};

StagePlan plan_stage(const asr_gemm_t* g, int nprob, size_t base) {
  StagePlan sp{};
  const char* e = getenv("ASR_GEMM_STAGE");
  if (e && e[0] == '0') return sp;
  bool any = false;
  for (int i = 0; i < nprob; ++i) {
    // batched products (the attention context's per-utterance products): each
    // operand staged as [batch][rows][ld] through a row map whose utterance
    // stride is the operand's batch stride; a K that is not a multiple of 8
    // only when both operands are K-major (the fast kernels' R-mode rows need it)
    const int nb = g[i].batch > 1 ? g[i].batch : 1;
    const bool kk = g[i].a.trans && g[i].b.trans;
    if ((g[i].K % 8 && !kk) || 2.0 * g[i].M * g[i].N * g[i].K * nb < STAGE_FLOPS) return sp;
    for (int j = 0; j < 2; ++j) {
      const asr_operand_t& op = j ? g[i].b : g[i].a;
      if (op.dtype != ASR_DT_F32) continue;
      if (op.tap_group) return sp;
      if (nb > 1 && (op.map.rows_per_b > 0 || op.map.perm || (op.map.t_mul != 0 && op.map.t_mul != 1) ||
                     (j ? g[i].batch_stride_b : g[i].batch_stride_a) % 4))
        return sp;
      const int outer = j ? g[i].N : g[i].M;
      const int cols = op.trans ? outer : g[i].K;
      if (cols % 8 == 0 && (!aligned16(op.ptr) || op.map.stride_t % 4 || op.map.stride_b % 4))
        return sp;   // the conversion's vector path needs aligned rows
      any = true;
    }
  }
  if (!any) return sp;
  size_t o = base;
  for (int i = 0; i < nprob; ++i)
    for (int j = 0; j < 2; ++j) {
      const asr_operand_t& op = j ? g[i].b : g[i].a;
      if (op.dtype != ASR_DT_F32) continue;
      const int outer = j ? g[i].N : g[i].M;
      sp.on[i][j] = true;
      sp.rows[i][j] = op.trans ? g[i].K : outer;
      sp.cols[i][j] = op.trans ? outer : g[i].K;
      sp.ld[i][j] = (sp.cols[i][j] + 7) / 8 * 8;
      sp.off[i][j] = o;
      const int nb = g[i].batch > 1 ? g[i].batch : 1;
      o += ((size_t)nb * sp.rows[i][j] * sp.ld[i][j] * 2 + 255) & ~(size_t)255;
    }
  sp.bytes = o - base;
  return sp;
}

// the conversion's row map of operand j of g: the operand's own map, and for a
// batched product its utterances as blocks of `rows` rows at the batch stride
asr_rowmap_t stage_map(const asr_gemm_t& g, int j, int rows) {
  const asr_operand_t& op = j ? g.b : g.a;
  asr_rowmap_t m = op.map;
  if (g.batch > 1) {
    m.rows_per_b = rows;
    m.stride_b = j ? g.batch_stride_b : g.batch_stride_a;
  }
  return m;
}

size_t split_bytes_aligned(const asr_gemm_t* g, int nprob) {
  return (plan_split(g, nprob).bytes + 255) & ~(size_t)255;
}

int gemm_launch(const asr_gemm_t* problems, int nprob, int compute_dtype, void* workspace,
                size_t ws_bytes, void* stream) {
  ASR_REQUIRE(problems && nprob >= 1 && nprob <= 2, ASR_ERR_ARG, "gemm: nprob must be 1 or 2");
  // The fast kernels take one operand-layout pair per launch: two products with
  // different layouts (a Linear backward's dX + dW) run as two launches, one
  // after the other on the stream (each within the pair's workspace), instead
  // of one launch of the generic kernel.
  if (nprob == 2 && compute_dtype == ASR_DT_BF16 &&
      2 * problems[0].a.trans + problems[0].b.trans !=
          2 * problems[1].a.trans + problems[1].b.trans) {
    const int rc = gemm_launch(problems, 1, compute_dtype, workspace, ws_bytes, stream);
    if (rc) return rc;
    return gemm_launch(problems + 1, 1, compute_dtype, workspace, ws_bytes, stream);
  }
  if (compute_dtype == ASR_DT_BF16 && workspace) {
    const size_t base = split_bytes_aligned(problems, nprob);
    const StagePlan st = plan_stage(problems, nprob, base);
    if (st.bytes > 0 && ws_bytes >= base + st.bytes) {
      // every staged operand in one launch when all take the vector form
      // (ASR_GEMM_STAGE_MULTI=0: one launch per operand)
      const float* msrc[4];
      asr_rowmap_t mmap[4];
      int mrows[4], mcols[4], nm = 0;
      uint16_t* mdst[4];
      bool multi = !(getenv("ASR_GEMM_STAGE_MULTI") && getenv("ASR_GEMM_STAGE_MULTI")[0] == '0');
      for (int i = 0; i < nprob && multi; ++i)
        for (int j = 0; j < 2; ++j) {
          if (!st.on[i][j]) continue;
          const asr_operand_t& op = j ? problems[i].b : problems[i].a;
          if (st.cols[i][j] != st.ld[i][j]) multi = false;
          msrc[nm] = (const float*)op.ptr;
          mmap[nm] = stage_map(problems[i], j, st.rows[i][j]);
          mrows[nm] = st.rows[i][j] * (problems[i].batch > 1 ? problems[i].batch : 1);
          mcols[nm] = st.cols[i][j];
          mdst[nm] = (uint16_t*)((char*)workspace + st.off[i][j]);
          ++nm;
        }
      int done = 0;
      if (multi && nm > 1) {
        done = convert_rows_bf16_multi(msrc, mmap, mrows, mcols, mdst, nm, stream);
        ASR_REQUIRE(done >= 0, ASR_ERR_HIP, "gemm: operand staging launch failed");
      }
      asr_gemm_t g2[2];
      for (int i = 0; i < nprob; ++i) {
        g2[i] = problems[i];
        for (int j = 0; j < 2; ++j) {
          if (!st.on[i][j]) continue;
          asr_operand_t& op = j ? g2[i].b : g2[i].a;
          uint16_t* dst = (uint16_t*)((char*)workspace + st.off[i][j]);
          const int nbt = problems[i].batch > 1 ? problems[i].batch : 1;
          const int rc = done ? 0
                              : asr_convert_rows_bf16_ld((const float*)op.ptr,
                                                         stage_map(problems[i], j, st.rows[i][j]),
                                                         st.rows[i][j] * nbt, st.cols[i][j],
                                                         st.ld[i][j], dst, stream);
          if (rc) return rc;
          op.ptr = dst;
          op.dtype = ASR_DT_BF16;
          memset(&op.map, 0, sizeof(op.map));
          op.map.stride_t = st.ld[i][j];
          op.bytes = (long long)nbt * st.rows[i][j] * st.ld[i][j] * 2;
          if (nbt > 1) (j ? g2[i].batch_stride_b : g2[i].batch_stride_a) =
              (long long)st.rows[i][j] * st.ld[i][j];
        }
      }
      return gemm_launch_own(g2, nprob, compute_dtype, workspace, ws_bytes, stream);
    }
  }
  return gemm_launch_own(problems, nprob, compute_dtype, workspace, ws_bytes, stream);
}

}  // namespace
}  // namespace asr

using namespace asr;

extern "C" int asr_gemm_set_nosplit(int on) {
  g_nosplit = on ? 1 : 0;
  return ASR_OK;
}

extern "C" int asr_gemm_set_small_tiles(int on) {
  g_small_tiles = on ? 1 : 0;
  return ASR_OK;
}

// asr_gemm_set_n64_kmode(1): products with N <= 64 and a K-major B (the VGG
// weight gradients computed transposed) take the 256 x 64 kernel too.
extern "C" int asr_gemm_set_n64_kmode(int on) {
  g_n64_kmode = on ? 1 : 0;
  return ASR_OK;
}

extern "C" int asr_gemm(const asr_gemm_t* problems, int nprob, int compute_dtype, void* stream) {
  return gemm_launch(problems, nprob, compute_dtype, nullptr, 0, stream);
}

extern "C" size_t asr_gemm_workspace_bytes(const asr_gemm_t* problems, int nprob) {
  if (!problems || nprob < 1 || nprob > 2) return 0;
  // split-K slabs, then the bf16 staging copies (used in bf16 mode only)
  const size_t base = split_bytes_aligned(problems, nprob);
  const size_t stage = plan_stage(problems, nprob, base).bytes;
  return stage ? base + stage : plan_split(problems, nprob).bytes;
}

extern "C" int asr_gemm_lse_ws(const asr_gemm_t* problem, int compute_dtype, float* lse,
                               void* workspace, size_t ws_bytes, void* stream) {
  ASR_REQUIRE(problem && lse, ASR_ERR_ARG, "gemm_lse: null pointer");
  ASR_REQUIRE(problem->beta == 0.f && problem->drop_p == 0.f && problem->c_dtype == ASR_DT_F32 &&
                  problem->batch <= 1,
              ASR_ERR_ARG, "gemm_lse: needs beta 0, no dropout, f32 C, one batch");
  g_row_lse = lse;
  const int rc = gemm_launch(problem, 1, compute_dtype, workspace, ws_bytes, stream);
  g_row_lse = nullptr;
  return rc;
}

extern "C" int asr_gemm_ws(const asr_gemm_t* problems, int nprob, int compute_dtype,
                           void* workspace, size_t ws_bytes, void* stream) {
  if (!workspace) ASR_REQUIRE(plan_split(problems, nprob).bytes == 0, ASR_ERR_WORKSPACE,
                              "gemm: split-K workspace required");   // (staging is optional)
  return gemm_launch(problems, nprob, compute_dtype, workspace, ws_bytes, stream);
}

// Row chunks of a column sum: enough (64-column, chunk) work-groups to cover
// the chip (~512), chunks of >= 64 rows, at most 64 partial rows.
int colsum_chunks(int M, int N) {
  const int cblocks = (N + 63) / 64;
  int nc = max(1, 512 / max(cblocks, 1));
  nc = min(nc, max(1, M / 64));
  return min(nc, 64);
}

extern "C" size_t asr_colsum_workspace_bytes(int M, int N) {
  return (size_t)colsum_chunks(M, N) * N * sizeof(float);
}

template <typename TG>
static int colsum_accumulate_impl(const TG* g, long long ld, int M, int N, float alpha,
                                  float* out0, float* out1, void* workspace, size_t ws_bytes,
                                  void* stream) {
  ASR_REQUIRE(g && out0 && workspace, ASR_ERR_ARG, "colsum: null pointer");
  if (M <= 0 || N <= 0) return ASR_OK;
  const int nchunk = colsum_chunks(M, N);
  ASR_REQUIRE(ws_bytes >= asr_colsum_workspace_bytes(M, N), ASR_ERR_WORKSPACE,
              "colsum: workspace too small");
  const int rpc = (M + nchunk - 1) / nchunk;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(colsum_partial<TG>, dim3(ceil_div(N, 64), nchunk), dim3(256), 0, s, g, ld, M,
                     N, rpc, (float*)workspace);
  ASR_LAUNCH_CHECK();
  hipLaunchKernelGGL(colsum_final, dim3(ceil_div(N, 16)), dim3(256), 0, s,
                     (const float*)workspace, nchunk, N, alpha, out0, out1);
  ASR_LAUNCH_CHECK();
  return ASR_OK;
}

extern "C" int asr_colsum_accumulate(const float* g, long long ld, int M, int N, float alpha,
                                     float* out0, float* out1, void* workspace, size_t ws_bytes,
                                     void* stream) {
  return colsum_accumulate_impl(g, ld, M, N, alpha, out0, out1, workspace, ws_bytes, stream);
}

// The same over a bf16 matrix (the fused CTC head's dY operand), f32 sums.
extern "C" int asr_colsum_accumulate_bf16(const uint16_t* g, long long ld, int M, int N,
                                          float alpha, float* out0, float* out1, void* workspace,
                                          size_t ws_bytes, void* stream) {
  return colsum_accumulate_impl(g, ld, M, N, alpha, out0, out1, workspace, ws_bytes, stream);
}
