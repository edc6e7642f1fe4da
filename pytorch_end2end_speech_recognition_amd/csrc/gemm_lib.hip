// Plain bf16 GEMMs on hipBLASLt.  asr_gemm sends a problem here only when it is
// a plain library GEMM -- bf16 operands in dense row-major / column-major
// layouts, no row map (no permutation, subsampling, time shift, tap
// addressing), no batching, f32 bias vectors -- and it is large enough
// to matter; everything with a fused row map stays on the hand-written MFMA
// kernels of gemm.hip.  Two bias vectors (nn.LSTM's b_ih + b_hh) are summed
// into the workspace first and enter through the BIAS epilogue.  Our row-major C[M][ldc] = A op B^T is hipBLASLt's
// column-major D (N x M) = op(X) op(Y) with X = B, Y = A.
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"

namespace asr {
namespace {

constexpr size_t kLibWs = 32u << 20;     // hipBLASLt workspace offered to the heuristics
constexpr size_t kBiasWs = 64u << 10;    // summed bias (N <= 16384 floats), before it

__global__ void bias_sum(const float* __restrict__ b1, const float* __restrict__ b2,
                         float* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = b1[i] + b2[i];
}

struct LibPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t lx = nullptr, ly = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  bool ok = false;
};

typedef std::tuple<int, int, int, int, int, long long, long long, long long, int, int> Key;

hipblasLtHandle_t handle() {
  static hipblasLtHandle_t h = nullptr;
  static bool tried = false;
  if (!tried) {
    tried = true;
    if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) h = nullptr;
  }
  return h;
}

bool plain(const asr_rowmap_t& m, long long rows) {
  if (m.perm || m.t_add != 0 || (m.t_mul != 0 && m.t_mul != 1)) return false;
  if (m.rows_per_b > 0 && m.stride_b != (long long)m.rows_per_b * m.stride_t) return false;
  // t_limit bounds the time index inside a group (rows_per_b rows), else the row
  if (m.t_limit > 0 && m.t_limit < (m.rows_per_b > 0 ? m.rows_per_b : rows)) return false;
  return true;
}

}  // namespace

bool gemm_lib_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("ASR_GEMM_LIB");
    on = !(e && e[0] == '0');
  }
  return on == 1;
}

// Whether asr_gemm may run problem g on hipBLASLt (pure function of the
// problem; the split-K planner and the launcher agree through it).
bool gemm_lib_eligible(const asr_gemm_t& g, int compute_dtype) {
  if (!gemm_lib_enabled() || compute_dtype != ASR_DT_BF16) return false;
  if (g.a.dtype != ASR_DT_BF16 || g.b.dtype != ASR_DT_BF16 || g.batch > 1) return false;
  if (g.a.tap_group || g.b.tap_group) return false;
  if (g.bias2 && (!g.bias || g.N > (int)(kBiasWs / 4))) return false;
  if (2.0 * g.M * g.N * g.K < 4.0e9) return false;            // small: own kernels
  // K-major x K-major (the weight gradients, K = B*T): the library's first
  // choice runs at ~300 TF/s, the own split-K kernel at ~520
  if (g.a.trans && g.b.trans) return false;
  const long long ra = g.a.trans ? g.K : g.M, rb = g.b.trans ? g.K : g.N;
  if (!plain(g.a.map, ra) || !plain(g.b.map, rb) || !plain(g.c_map, g.M)) return false;
  const long long lda = g.a.map.stride_t, ldb = g.b.map.stride_t, ldc = g.c_map.stride_t;
  if (lda % 8 || ldb % 8 || ldc % 4) return false;
  if (lda < (g.a.trans ? g.M : g.K) || ldb < (g.b.trans ? g.N : g.K) || ldc < g.N) return false;
  if (((uintptr_t)g.a.ptr & 15) || ((uintptr_t)g.b.ptr & 15) || ((uintptr_t)g.c & 15))
    return false;
  return handle() != nullptr;
}

size_t gemm_lib_workspace_bytes() { return kBiasWs + kLibWs; }

// Runs g on hipBLASLt.  Returns 1 when done, 0 when no algorithm fits (the
// caller falls back to its own kernel), < 0 on error.
int gemm_lib_run(const asr_gemm_t& g, void* ws, size_t ws_bytes, hipStream_t s) {
  if (g.bias2 && (!ws || ws_bytes < kBiasWs)) return 0;
  const float* bias = g.bias;
  if (ws && ws_bytes >= kBiasWs) {
    if (g.bias2) {
      hipLaunchKernelGGL(bias_sum, dim3((g.N + 255) / 256), dim3(256), 0, s, g.bias, g.bias2,
                         (float*)ws, g.N);
      ASR_LAUNCH_CHECK();
      bias = (const float*)ws;
    }
    ws = (char*)ws + kBiasWs;
    ws_bytes -= kBiasWs;
  } else {
    ws = nullptr;
    ws_bytes = 0;
  }
  static std::mutex mu;
  static std::map<Key, LibPlan> cache;
  const hipblasLtHandle_t h = handle();
  if (!h) return 0;
  const long long lda = g.a.map.stride_t, ldb = g.b.map.stride_t, ldc = g.c_map.stride_t;
  const Key key(g.M, g.N, g.K, g.a.trans, g.b.trans, lda, ldb, ldc, g.bias != nullptr,
                ws_bytes >= kLibWs);
  LibPlan* pl;
  {
    std::lock_guard<std::mutex> lock(mu);
    pl = &cache[key];
    if (!pl->desc) {
      // X = B: trans=0 -> col-major (K x N, ld) used transposed; trans=1 -> (N x K, ld)
      // Y = A: trans=0 -> col-major (K x M, ld) as is;           trans=1 -> (M x K, ld) transposed
      const hipblasOperation_t tx = g.b.trans ? HIPBLAS_OP_N : HIPBLAS_OP_T;
      const hipblasOperation_t ty = g.a.trans ? HIPBLAS_OP_T : HIPBLAS_OP_N;
      bool ok = hipblasLtMatmulDescCreate(&pl->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) ==
                HIPBLAS_STATUS_SUCCESS;
      ok = ok && hipblasLtMatmulDescSetAttribute(pl->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &tx,
                                                 sizeof(tx)) == HIPBLAS_STATUS_SUCCESS;
      ok = ok && hipblasLtMatmulDescSetAttribute(pl->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &ty,
                                                 sizeof(ty)) == HIPBLAS_STATUS_SUCCESS;
      if (g.bias) {
        const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
        const hipDataType bt = HIP_R_32F;
        ok = ok && hipblasLtMatmulDescSetAttribute(pl->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep,
                                                   sizeof(ep)) == HIPBLAS_STATUS_SUCCESS;
        ok = ok && hipblasLtMatmulDescSetAttribute(pl->desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE,
                                                   &bt, sizeof(bt)) == HIPBLAS_STATUS_SUCCESS;
      }
      const uint64_t xr = g.b.trans ? g.N : g.K, xc = g.b.trans ? g.K : g.N;
      const uint64_t yr = g.a.trans ? g.M : g.K, yc = g.a.trans ? g.K : g.M;
      ok = ok && hipblasLtMatrixLayoutCreate(&pl->lx, HIP_R_16BF, xr, xc, ldb) ==
                     HIPBLAS_STATUS_SUCCESS;
      ok = ok && hipblasLtMatrixLayoutCreate(&pl->ly, HIP_R_16BF, yr, yc, lda) ==
                     HIPBLAS_STATUS_SUCCESS;
      ok = ok && hipblasLtMatrixLayoutCreate(&pl->ld, HIP_R_32F, g.N, g.M, ldc) ==
                     HIPBLAS_STATUS_SUCCESS;
      if (ok) {
        hipblasLtMatmulPreference_t pref;
        const uint64_t maxws = ws_bytes >= kLibWs ? kLibWs : 0;
        ok = hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS;
        ok = ok && hipblasLtMatmulPreferenceSetAttribute(
                       pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &maxws,
                       sizeof(maxws)) == HIPBLAS_STATUS_SUCCESS;
        // the first choice only: the process runs torch's bundled hipBLASLt
        // (same soname, loaded first), and timing the further candidates of
        // that build ended in a GPU memory fault
        hipblasLtMatmulHeuristicResult_t res[1];
        int n = 0;
        ok = ok && hipblasLtMatmulAlgoGetHeuristic(h, pl->desc, pl->lx, pl->ly, pl->ld, pl->ld,
                                                   pref, 1, res, &n) == HIPBLAS_STATUS_SUCCESS;
        ok = ok && n > 0 && res[0].state == HIPBLAS_STATUS_SUCCESS;
        if (ok) {
          pl->algo = res[0].algo;
          pl->ws = res[0].workspaceSize;
        }
        hipblasLtMatmulPreferenceDestroy(pref);
      }
      pl->ok = ok;
    }
  }
  if (!pl->ok || pl->ws > ws_bytes) return 0;
  if (bias &&
      hipblasLtMatmulDescSetAttribute(pl->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias,
                                      sizeof(void*)) != HIPBLAS_STATUS_SUCCESS)
    return ASR_ERR_HIP;
  const float alpha = g.alpha, beta = g.beta;
  const hipblasStatus_t st =
      hipblasLtMatmul(h, pl->desc, &alpha, g.b.ptr, pl->lx, g.a.ptr, pl->ly, &beta, g.c, pl->ld,
                      g.c, pl->ld, &pl->algo, pl->ws ? ws : nullptr, pl->ws, s);
  if (st != HIPBLAS_STATUS_SUCCESS) {
    set_error("gemm: hipblasLtMatmul failed (%d)", (int)st);
    return ASR_ERR_HIP;
  }
  return 1;
}

}  // namespace asr

extern "C" int asr_gemm_library_ready(void) {
  return asr::gemm_lib_enabled() && asr::handle() != nullptr;
}
