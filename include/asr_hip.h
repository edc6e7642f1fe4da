/*
 * libasr_hip.so -- C ABI of the MI355X (gfx950) hot path of the hybrid
 * CTC/attention ASR training step.
 *
 * Plain pointers and sizes only: no torch / C++ types cross this boundary.
 * All device pointers are HIP device memory owned by the caller; the library
 * never allocates, frees or synchronises inside an entry point (graph-capture
 * safe).  Every entry point is stream-ordered on `stream` (a hipStream_t
 * passed as void*), re-entrant, and returns ASR_OK (0) or a negative error
 * code; asr_last_error() gives the text (thread-local).
 *
 * Reference interfaces replaced (paths into carolinebear/pytorch_end2end_speech_recognition):
 *   CTC           warpctc_pytorch.gpu_ctc / cpu_ctc as bound by
 *                 models/pytorch_v3/ctc/ctc.py:30-66 (my_warpctc)
 *   LSTM layer    torch.nn.LSTM(bidirectional) + pack/pad in
 *                 models/pytorch_v3/encoders/rnn.py:166-172,218-224,343-390
 *   LinearND      models/pytorch_v3/linear.py:15-47 (and every nn.Linear GEMM)
 *   attention     AttentionMechanism.forward (location) in
 *                 models/pytorch_v3/attention/attention_layer.py:123-251
 *   LSTMCell      models/pytorch_v3/attention/rnn_decoder.py:63-113
 *   optimizer     torch.optim.Adam / SGD + clip_grad_norm in
 *                 models/pytorch_v3/base.py:141-213, utils/training/training_loop.py:42-51
 *   best path     GreedyDecoder in models/pytorch_v3/ctc/decoders/greedy_decoder.py:19-47
 */
#ifndef ASR_HIP_H_
#define ASR_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ASR_OK 0
#define ASR_ERR_ARG (-1)      /* bad pointer / size / shape argument */
#define ASR_ERR_WORKSPACE (-2) /* workspace too small */
#define ASR_ERR_HIP (-3)      /* HIP runtime error (launch / memset) */
#define ASR_ERR_UNSUPPORTED (-4)

#define ASR_DT_F32 0
#define ASR_DT_BF16 1

/* ---------------------------------------------------------------- info */
const char* asr_version(void);
const char* asr_last_error(void);
/* 1 when the current device is a gfx950 (the only code-object target of the
 * library), 0 for another device, -1 when no device can be queried. */
int asr_arch_is_gfx950(void);

/* A HIP stream restricted to CUs [cu_begin, cu_begin + cu_count) of the
 * current device (hipExtStreamCreateWithCUMask).  The weight-gradient GEMMs
 * of encoder layer l run on it beside the persistent backward recurrence of
 * layer l-1, which keeps the remaining CUs to itself. */
int asr_stream_create_cu_masked(int cu_begin, int cu_count, void** stream_out);
int asr_stream_destroy(void* stream);

/* ----------------------------------------------------------------- CTC
 * Replaces warpctc_pytorch.gpu_ctc(acts, grads, labels, label_lens,
 * act_lens, minibatch, costs) (models/pytorch_v3/ctc/ctc.py:35-45).
 *
 * acts: unnormalised f32 activations, element (t, b, v) at
 *   acts[t*stride_t + b*stride_b + v]  -- time-major [T,B,V] as warp-ctc
 *   (stride_t = B*V, stride_b = V) or batch-major [B,T,V] (stride_t = V,
 *   stride_b = T*V) without a transpose copy.
 * labels_flat: int32 [sum(label_lens)], device, values in [0,V) != blank.
 * label_lens, act_lens: int32 [B], device.  max_label_len >= max(label_lens).
 * Softmax is applied inside; blank index `blank` (reference: 0).
 * costs: f32 [B] = -log P(y_b|x_b) (0 if infeasible and zero_infinity, +inf
 *   otherwise).  loss_out (nullable): f32 [1] = loss_scale * sum_b costs[b].
 * Gradient (w.r.t. the unnormalised activations, zero for t >= act_lens[b],
 *   zero for infeasible utterances) is produced by asr_ctc_backward from the
 *   state kept in `workspace` (so it is written exactly once, already scaled),
 *   scaled by scale * (*grad_scale) (grad_scale: device f32 scalar, e.g. the
 *   upstream dLoss; NULL means 1.0).
 */
size_t asr_ctc_workspace_bytes(int T, int B, int V, int max_label_len);
int asr_ctc_forward(const float* acts, long long stride_t, long long stride_b, int T, int B,
                    int V, const int32_t* labels_flat, const int32_t* label_lens,
                    const int32_t* act_lens, int max_label_len, int blank, int zero_infinity,
                    float* costs, float* loss_out, float loss_scale, void* workspace,
                    size_t ws_bytes, void* stream);
/* asr_ctc_forward with the per-frame log-sum-exp already formed by the output
 * layer's GEMM (asr_gemm_lse_ws): lse_part holds, for every frame row b*T + t
 * and 64-class slab q < nslab = ceil(V / 64), the pair (max, sum exp(x - max))
 * at lse_part[2 (q B T + b T + t)].  The activations are then read only at
 * the label columns; costs, loss and the workspace state for asr_ctc_backward
 * are those of asr_ctc_forward. */
int asr_ctc_forward_lse(const float* acts, long long stride_t, long long stride_b, int T, int B,
                        int V, const float* lse_part, int nslab, const int32_t* labels_flat,
                        const int32_t* label_lens, const int32_t* act_lens, int max_label_len,
                        int blank, int zero_infinity, float* costs, float* loss_out,
                        float loss_scale, void* workspace, size_t ws_bytes, void* stream);
int asr_ctc_backward(const float* acts, long long stride_t, long long stride_b, int T, int B,
                     int V, const int32_t* labels_flat, const int32_t* label_lens,
                     const int32_t* act_lens, int max_label_len, int blank,
                     const float* grad_scale, float scale, float* grads, long long gstride_t,
                     long long gstride_b, const void* workspace, size_t ws_bytes, void* stream);
/* asr_ctc_backward writing the gradient as bf16 rows of gld columns (gld >= V,
 * gld % 8 == 0, 16-B aligned rows, strides in elements), columns [V, gld)
 * zero: the zero-padded dY operand of the output layer's staged bf16 GEMMs
 * (the fused CTC head, native_ops.LinearCTCFn; no f32 gradient pass). */
int asr_ctc_backward_bf16(const float* acts, long long stride_t, long long stride_b, int T, int B,
                          int V, const int32_t* labels_flat, const int32_t* label_lens,
                          const int32_t* act_lens, int max_label_len, int blank,
                          const float* grad_scale, float scale, uint16_t* grads,
                          long long gstride_t, long long gstride_b, int gld,
                          const void* workspace, size_t ws_bytes, void* stream);
/* asr_ctc_backward_bf16 that also ADDS the f32 column sums of the gradient,
 * formed before the bf16 rounding, into dbias [V] (the output layer's bias
 * gradient of the fused CTC head: the reference's LinearND bias gradient,
 * linear.py:32-47, summed from dY = ctc.py:30-52's gradient).  Deterministic
 * (fixed-order per-block partials); bias_ws holds
 * asr_ctc_bias_workspace_bytes(T, B, V, gld) bytes.  V <= 16384. */
size_t asr_ctc_bias_workspace_bytes(int T, int B, int V, int gld);
int asr_ctc_backward_bf16_db(const float* acts, long long stride_t, long long stride_b, int T,
                             int B, int V, const int32_t* labels_flat, const int32_t* label_lens,
                             const int32_t* act_lens, int max_label_len, int blank,
                             const float* grad_scale, float scale, uint16_t* grads,
                             long long gstride_t, long long gstride_b, int gld,
                             const void* workspace, size_t ws_bytes, float* dbias, void* bias_ws,
                             size_t bias_ws_bytes, void* stream);
/* warp-ctc drop-in: forward + backward with scale 1 in one call. */
int asr_ctc_fwd_bwd(const float* acts, long long stride_t, long long stride_b, int T, int B,
                    int V, const int32_t* labels_flat, const int32_t* label_lens,
                    const int32_t* act_lens, int max_label_len, int blank, int zero_infinity,
                    float* costs, float* grads, void* workspace, size_t ws_bytes, void* stream);

/* Which kernels the last CTC forward / gradient ran (host-side record), out2 =
 * {normaliser: 0 the emission pass over the logits, 1 the head GEMM
 * epilogue's partials; gradient: 0 f32 ctc_grad, 1 ctc_grad_bf16, 2 narrow
 * (V <= 256), 3 pipelined, 4 streamed}. */
int asr_ctc_last_path(int* out2);
/* Waves per direction of the last CTC forward's lattice (round 6): 1 = the
 * one-wave ctc_lattice, 2 / 4 = ctc_lattice_w (ASR_CTC_LATTICE_W=1 forces 1). */
int asr_ctc_last_lattice_waves(void);
/* Tag of the last GEMM launch (4 x kernel family + operand mode, the
 * ASR_PTAG_GEMM_* families of csrc/prof.h): diagnostics, tools/gemm_log.py. */
int asr_gemm_last_family(void);

/* ---------------------------------------------------------------- GEMM
 * C(m,n) = alpha * sum_k A(m,k) B(n,k) + beta * C(m,n) + bias[n] + bias2[n]  (f32 C)
 * Replaces every nn.Linear / LinearND GEMM (linear.py:15-47) and the LSTM
 * input-projection and weight-gradient GEMMs inside nn.LSTM.
 *
 * A row map turns a logical row index r into memory:
 *   g = r / rows_per_b, t = r % rows_per_b, tp = t*t_mul + t_add,
 *   row(r) = base + perm[g]*stride_b + tp*stride_t   (perm NULL = identity)
 *   rows with tp outside [0, t_limit) read as zeros (A/B) / are not stored (C).
 * This fuses the length-sort gather (rnn.py:319-326), the pyramidal drop
 * subsampling xs[:,1::2] (rnn.py:415-419) and the h_{t-1} shift of dW_hh
 * into the operand loads.  Operand element (i,k) is at row(i)+k (trans=0) or
 * row(k)+i (trans=1); operands are f32 or bf16 in memory.
 * compute_dtype ASR_DT_F32: exact-f32 MFMA (v_mfma_f32_16x16x4_f32);
 * ASR_DT_BF16: bf16 MFMA with f32 accumulation.  Up to 2 independent
 * problems per launch (e.g. the two LSTM directions).
 */
typedef struct {
  long long stride_b;
  long long stride_t;
  int rows_per_b; /* <= 0: a single group */
  int t_mul;      /* 0 means 1 */
  int t_add;
  int t_limit;    /* <= 0: unlimited */
  const int32_t* perm;
} asr_rowmap_t;

typedef struct {
  const void* ptr;
  int dtype;
  int trans;
  asr_rowmap_t map;
  /* bytes readable from ptr (the rest of its allocation), 0 = unknown.  Known
   * extents < 2 GiB let bf16 operands use the range-checked buffer-load path
   * (out-of-range and masked rows read as zeros straight into LDS). */
  long long bytes;
  /* 3x3 "tap" addressing (implicit-GEMM convolution over a zero-haloed
   * [rows = padded pixels][channels] layout), 0 = off.  The contiguous index x
   * (k for trans=0, the output index for trans=1) splits into tap = x /
   * tap_group and x' = x % tap_group; the element is read at column x' of row
   * r + tap_sign * ((tap / 3 - 1) * tap_pitch + tap % 3 - 1).  Needs
   * tap_group % 16 == 0 (trans=0) or % 8 == 0 (trans=1). */
  int tap_group;
  int tap_pitch;
  int tap_sign;
} asr_operand_t;

typedef struct {
  asr_operand_t a;
  asr_operand_t b;
  float* c;
  asr_rowmap_t c_map;
  const float* bias;  /* nullable, f32 [N] */
  const float* bias2; /* nullable, f32 [N], added too (nn.LSTM b_ih + b_hh) */
  int M, N, K;
  float alpha, beta;
  int batch;          /* <= 1: single; else `batch` independent products */
  long long batch_stride_a, batch_stride_b, batch_stride_c; /* elements */
  /* drop_p > 0: the written value is multiplied by asr_dropout's mask for the
   * element's offset i from c (kept iff u01(drop_seed, i) >= drop_p, scale
   * 1 / (1 - drop_p)): dropout's backward fused into the producing GEMM. */
  float drop_p;
  unsigned long long drop_seed;
  /* ASR_DT_F32 (0, the default of a zeroed struct) or ASR_DT_BF16: C is
   * written as bf16 (bf16 compute, beta 0; the product is not split over K;
   * the 128 x 128 / 256 x 64 / generic kernels). */
  int c_dtype;
} asr_gemm_t;

int asr_gemm(const asr_gemm_t* problems, int nprob, int compute_dtype, void* stream);

/* Same product with a workspace for deterministic split-K: weight-gradient
 * GEMMs (dW = dgates^T x over B*T rows, K ~ 32000) have few output tiles and
 * a long K; they are split along K into fixed f32 slabs and summed in a fixed
 * order by a second kernel (bit-reproducible run to run).  The split is a pure
 * function of the shapes; asr_gemm_workspace_bytes returns 0 when no problem
 * splits (then workspace may be NULL and this equals asr_gemm). */
size_t asr_gemm_workspace_bytes(const asr_gemm_t* problems, int nprob);
int asr_gemm_ws(const asr_gemm_t* problems, int nprob, int compute_dtype, void* workspace,
                size_t ws_bytes, void* stream);
/* asr_gemm_ws of ONE product (beta 0, no dropout, f32 C, batch 1) whose
 * epilogue also writes, for every row m < M and 64-column slab q < ceil(N/64),
 * the online log-sum-exp pair of the values written to C: lse[2 (q M + m)] =
 * max, lse[2 (q M + m) + 1] = sum exp(c - max) (the CTC normaliser of an
 * output layer, formed where the logits are produced; asr_ctc_forward_lse). */
int asr_gemm_lse_ws(const asr_gemm_t* problem, int compute_dtype, float* lse, void* workspace,
                    size_t ws_bytes, void* stream);

/* on != 0: later asr_gemm / asr_gemm_ws calls FROM THIS HOST THREAD use only the
 * 128 x 128 kernel (64 KB of LDS per work-group) until reset with 0, so that
 * their work-groups fit beside a persistent recurrence work-group on every CU
 * (weight gradients co-resident with the backward recurrence). */
int asr_gemm_set_small_tiles(int on);
/* on != 0: later asr_gemm calls FROM THIS HOST THREAD take no split-K slabs
 * (rows of one product computed by several launches then sum every output
 * element in the order one launch would: bitwise the same dX either way). */
int asr_gemm_set_nosplit(int on);
/* asr_gemm_set_n64_kmode(1): products with N <= 64 (M >= 4096) whose B is
 * K-major also take the 256 x 64 kernel (launches from this host thread). */
int asr_gemm_set_n64_kmode(int on);

/* Enqueue on `stream` a one-wave gate that releases once the NEXT persistent
 * backward recurrence (asr_lstm_backward*, any stream) has all its work-groups
 * resident, or after ~5 ms.  Work queued behind it on `stream` (the small-tile
 * weight-gradient GEMMs) then runs beside that recurrence.  Timing only. */
int asr_lstm_wgrad_gate(void* stream);

/* out0[n] (+ out1[n] if non-NULL) += alpha * sum_m g[m*ld + n]  (bias grads of
 * nn.Linear / nn.LSTM bias_ih and bias_hh); fixed-order, deterministic. */
size_t asr_colsum_workspace_bytes(int M, int N);
int asr_colsum_accumulate(const float* g, long long ld, int M, int N, float alpha, float* out0,
                          float* out1, void* workspace, size_t ws_bytes, void* stream);
/* asr_colsum_accumulate over a bf16 matrix (f32 sums). */
int asr_colsum_accumulate_bf16(const uint16_t* g, long long ld, int M, int N, float alpha,
                               float* out0, float* out1, void* workspace, size_t ws_bytes,
                               void* stream);

/* ---------------------------------------------------------- LSTM layer
 * Bidirectional recurrence of one encoder layer (nn.LSTM bidirectional with
 * pack/pad semantics, rnn.py:166-172,218-224,343-390).  Gate order i,f,g,o.
 * gx_act: f32 [B][T][8H]; on entry x@W_ih^T + b_ih + b_hh (forward dir in
 *   columns [0,4H), reverse in [4H,8H)); on exit the post-activation gates
 *   (i,f,g,o) needed by backward.  whh: [2][4H][H] (forward then reverse),
 *   f32 or bf16 (w_dtype).  lens: int32 [B] device (frames >= lens[b] give
 *   zero state / output).  y: f32 [B][T][2H] = [h_fwd ; h_bwd]; cst: f32
 *   [B][T][2H] cell states.  compute_dtype selects bf16 or exact-f32 MFMA for
 *   h @ W_hh^T (state and accumulation always f32).
 * Backward: dy f32 [B][T][2H] (nullable = 0); act_dg holds the saved gates on
 *   entry and the pre-activation gate gradients dG on exit (feeds the weight
 *   gradient GEMMs: dW_ih = dG^T x, dW_hh = dG^T h_prev, db = colsum dG).
 * ybf / dgbf (nullable): bf16 copies of y [B][T][2H] / dG [B][T][8H], written by
 *   the persistent kernels as they go, for the bf16 weight-gradient GEMMs.
 * bf16 mode runs each pass as ONE persistent launch when the grid is
 *   co-resident (see lstm_persist.hip), else one launch per time step.
 */
size_t asr_lstm_workspace_bytes(int B, int H, int compute_dtype, int backward);
int asr_lstm_forward(float* gx_act, const void* whh_f, const void* whh_r, int w_dtype,
                     const int32_t* lens, int B, int T, int H, int compute_dtype, float* y,
                     float* cst, uint16_t* ybf, void* workspace, size_t ws_bytes, void* stream);
int asr_lstm_backward(const float* dy, const void* whh_f, const void* whh_r, int w_dtype,
                      const int32_t* lens, int B, int T, int H, int compute_dtype, float* act_dg,
                      const float* cst, uint16_t* dgbf, void* workspace, size_t ws_bytes,
                      void* stream);
/* asr_lstm_backward plus the bias gradients of nn.LSTM's bias_ih / bias_hh
 * (both [2 dirs x 4H], accumulated +=, identical values: both biases feed the
 * same gate pre-activation, rnn.py:166-172).  The tagged-granule recurrence
 * sums them inside the pass; other paths reduce dG afterwards.  workspace:
 * asr_lstm_workspace_bytes(B, H, compute_dtype, 2). */
int asr_lstm_backward_db(const float* dy, const void* whh_f, const void* whh_r, int w_dtype,
                         const int32_t* lens, int B, int T, int H, int compute_dtype,
                         float* act_dg, const float* cst, uint16_t* dgbf, float* db_ih,
                         float* db_hh, void* workspace, size_t ws_bytes, void* stream);
/* asr_lstm_backward_db for a caller that feeds only the bf16 gate gradients
 * (dgbf, required) to its weight / input gradient GEMMs: the tagged-granule
 * recurrence skips the f32 dG stores and act_dg's contents are unspecified on
 * exit.  Same workspace as asr_lstm_backward_db. */
int asr_lstm_backward_dgbf(const float* dy, const void* whh_f, const void* whh_r, int w_dtype,
                           const int32_t* lens, int B, int T, int H, int compute_dtype,
                           float* act_dg, const float* cst, uint16_t* dgbf, float* db_ih,
                           float* db_hh, void* workspace, size_t ws_bytes, void* stream);

/* Forward layer pass with the input projection fused into the persistent
 * recurrence (bf16 mode; replaces asr_gemm(gx = x W_ih^T + b_ih + b_hh) +
 * asr_lstm_forward): x [B*T][Din] bf16 rows (b, t) of the layer input, wih
 * [8H][Din] bf16 = [W_ih fwd; W_ih rev], b_ih / b_hh f32 [8H], whh f32 [4H][H]
 * per direction.  act [B][T][8H] f32 receives the post-activation gates (the
 * backward's input, as gx_act after asr_lstm_forward); y, cst, ybf as there.
 * ASR_ERR_UNSUPPORTED: this shape / device does not take the path
 * (asr_lstm_forward_x_ok tells beforehand). */
int asr_lstm_forward_x(const uint16_t* x, int Din, const uint16_t* wih, const float* b_ih,
                       const float* b_hh, const float* whh_f, const float* whh_r,
                       const int32_t* lens, int B, int T, int H, float* act, float* y, float* cst,
                       uint16_t* ybf, void* workspace, size_t ws_bytes, void* stream);
int asr_lstm_forward_x_ok(int B, int H, int Din);
/* asr_lstm_forward_x with the gate activations stored packed as fp16:
 * act_h [B][T][2][H][4] (i, f, g, o of one (utterance, frame, direction,
 * unit) in one 8-B word; 8 B per cell instead of 16, one store instead of
 * four).  Read back by asr_lstm_backward_dgbf_h (or unpacked to the f32
 * [B][T][8H] layout by asr_lstm_unpack_act_h).  Replaces the same nn.LSTM
 * forward as asr_lstm_forward_x (models/pytorch_v3/encoders/rnn.py:166-172). */
int asr_lstm_forward_xh(const uint16_t* x, int Din, const uint16_t* wih, const float* b_ih,
                        const float* b_hh, const float* whh_f, const float* whh_r,
                        const int32_t* lens, int B, int T, int H, uint16_t* act_h, float* y,
                        float* cst, uint16_t* ybf, void* workspace, size_t ws_bytes,
                        void* stream);
/* asr_lstm_forward_xh for a layer whose output feeds only the next BLSTM
 * layer's staged bf16 input (the stacked nn.LSTM layers of
 * models/pytorch_v3/encoders/rnn.py:343-390 with dropout between them,
 * rnn.py:398): y may be NULL (the f32 output is then not written); ydrop,
 * when non-NULL, receives bf16(dropout(y)) [B][T][2H] with asr_dropout's mask
 * for (drop_p, drop_seed) -- what asr_convert_rows_bf16_dropout would stage
 * from y; ybf (bf16 y) is required. */
int asr_lstm_forward_xh_drop(const uint16_t* x, int Din, const uint16_t* wih, const float* b_ih,
                             const float* b_hh, const float* whh_f, const float* whh_r,
                             const int32_t* lens, int B, int T, int H, uint16_t* act_h,
                             float* y, float* cst, uint16_t* ybf, uint16_t* ydrop, float drop_p,
                             unsigned long long drop_seed, void* workspace, size_t ws_bytes,
                             void* stream);
/* asr_lstm_backward_dgbf reading act_h of asr_lstm_forward_xh (tagged-granule
 * recurrence only; ASR_ERR_UNSUPPORTED otherwise).  Same workspace. */
int asr_lstm_backward_dgbf_h(const float* dy, const void* whh_f, const void* whh_r, int w_dtype,
                             const int32_t* lens, int B, int T, int H, int compute_dtype,
                             const uint16_t* act_h, const float* cst, uint16_t* dgbf,
                             float* db_ih, float* db_hh, void* workspace, size_t ws_bytes,
                             void* stream);
int asr_lstm_unpack_act_h(const uint16_t* act_h, int B, int T, int H, float* act, void* stream);
/* Diagnostics only (tools/buckets_diag.py, ASR_DIAG_SPIN): nwg work-groups of
 * 256 threads that fill 64 KB of LDS with a pattern and check it `iters`
 * times; mismatches are added to *bad (device int). */
int asr_diag_lds_spin(int nwg, int iters, int* bad, void* stream);

/* Diagnostics only (tests/test_coresidency_gpu.py): nwg work-groups of 256
 * threads holding lds_bytes of LDS each stay resident for usec microseconds
 * (a long-lived kernel beside the next persistent recurrence launch). */
int asr_diag_hold_cus(int nwg, int lds_bytes, int usec, void* stream);

/* ------------------------------------------------------------ GRU layer
 * Replaces the packed nn.GRU(bidirectional=True) of
 * models/pytorch_v3/encoders/rnn.py:173-191 (fast path) / :226-233 (per layer).
 * Gate order r, z, n; h0 = 0; outputs and state are 0 for t >= lens[b].
 *   gx_act [B][T][6H] f32: in  x W_ih^T + b_ih (forward cols [0,3H), reverse [3H,6H))
 *                          out r, z, n (post-activation), then dgx after backward
 *   whh    [2][3H][H] f32 (forward then reverse), bhh [2][3H] f32
 *   y      [B][T][2H] f32 out = [h_fwd ; h_rev];  ghn [B][T][2H] f32 out = W_hn h + b_hn
 * Backward: dy [B][T][2H] (nullable = 0); writes dgx over gx_act and
 * dgh [B][T][6H] = the gate gradients of W_hh h + b_hh; the weight / bias /
 * input gradients are GEMMs and column sums of dgx and dgh.  One launch per
 * time step (both directions), exact-f32 MFMA. */
size_t asr_gru_workspace_bytes(int B, int H);
int asr_gru_forward(float* gx_act, const float* whh, const float* bhh, const int32_t* lens, int B,
                    int T, int H, float* y, float* ghn, void* stream);
int asr_gru_backward(const float* dy, const float* whh, const int32_t* lens, int B, int T, int H,
                     float* act_dgx, const float* ghn, const float* y, float* dgh,
                     void* workspace, size_t ws_bytes, void* stream);

/* nn.GRUCell nonlinearity (decoder cells, rnn_decoder.py:91-95): gi = x W_ih^T +
 * b_ih, gh = h W_hh^T + b_hh [B][3D] (GEMMs by the caller); act [B][3D] out =
 * r, z, n; hout = (1 - z) n + z h.  Backward: dgi, dgh [B][3D] (the gate
 * gradients of the two GEMMs' outputs) and dh_prev = dh z (the direct term;
 * the caller adds dgh W_hh). */
int asr_gru_cell_forward(const float* gi, const float* gh, const float* h, int B, int D,
                         float* act, float* hout, void* stream);
int asr_gru_cell_backward(const float* act, const float* gh, const float* h, const float* dh,
                          int B, int D, float* dgi, float* dgh, float* dh_prev, void* stream);

/* ------------------------------------------------------------ optimizer
 * Replaces torch.nn.utils.clip_grad_norm(params, max_norm)
 * (utils/training/training_loop.py:46-50) + torch.optim Adam / SGD /
 * momentum / nesterov (models/pytorch_v3/base.py:141-194) over the model's
 * flat f32 parameter and gradient buffers.
 * asr_grad_sqnorm: out[0] = sum g^2 (deterministic; g 16-B aligned).
 * asr_optim_step: kind 0 adam (m, v), 1 sgd, 2 momentum (m), 3 nesterov (m);
 *   the clip coefficient min(1, max_norm / (sqrt(*grad_sqnorm) + 1e-6)) is
 *   computed on device (grad_sqnorm NULL or max_norm <= 0: no clipping);
 *   weight decay is L2 added to the gradient (torch semantics); step is the
 *   1-based step count for Adam bias correction; bf16_shadow (nullable)
 *   receives a bf16 copy of the updated parameters.
 */
size_t asr_grad_sqnorm_workspace_bytes(void);
int asr_grad_sqnorm(const float* g, long long n, float* out, void* workspace, size_t ws_bytes,
                    void* stream);
/* asr_optim_step_guarded: the same with guard (device int32[2], nullable):
 * when guard[0] | guard[1] != 0 (asr_lstm_status_gather's words) the kernel
 * leaves params and state untouched. */
int asr_optim_step_guarded(int kind, float* params, const float* grads, float* m, float* v,
                           long long n, float lr, float beta1, float beta2, float eps,
                           float weight_decay, long long step, float momentum, float dampening,
                           const float* grad_sqnorm, float max_norm, uint16_t* bf16_shadow,
                           const int* guard, void* stream);
int asr_optim_step(int kind, float* params, const float* grads, float* m, float* v, long long n,
                   float lr, float beta1, float beta2, float eps, float weight_decay,
                   long long step, float momentum, float dampening, const float* grad_sqnorm,
                   float max_norm, uint16_t* bf16_shadow, void* stream);

/* ------------------------------------------------------- elementwise
 * asr_dropout: y = x * (u(seed, i) >= p) / (1 - p), u a counter hash (the
 *   mask is recomputed from (seed, i) in backward: call again on dy).  u(seed,
 *   i) is 16-bit field i % 2 of lowbias32(((i / 2) * 0x9E3779B9) ^ key), key =
 *   lowbias32((uint32)seed ^ (uint32)(seed >> 32) * 0x85EBCA6B), divided by
 *   65536 (two elements per 32-bit hash; one stream covers 2^33 elements;
 *   oracle/rng.py restates it).
 *   Replaces nn.Dropout on the encoder / decoder activations.
 * asr_embedding_*: nn.Embedding(padding_idx) lookup / gradient (linear.py:50-77;
 *   trans=1: weight stored [E][V], the one-hot @ W^T of Embedding_LS,
 *   linear.py:80-116).  idx int64 [n].  Backward is deterministic and skips
 *   padding_idx (pass -1 for none).
 * asr_tanh_*: F.tanh of the encoder projection / attention bottleneck.
 */
int asr_dropout(const float* x, float* y, long long n, float p, unsigned long long seed,
                void* stream);
int asr_embedding_forward(const long long* idx, const float* weight, int n, int V, int E,
                          int trans, float* out, void* stream);
int asr_embedding_backward(const long long* idx, const float* dout, int n, int V, int E,
                           int trans, int padding_idx, float* grad_weight, void* stream);
/* The embedding gradient with the rows grouped by token (CSR built on the host
 * from the label array the caller already holds: rows order[starts[v] ..
 * starts[v+1]) carry token v in ascending order).  Same sums, O(n E). */
int asr_embedding_backward_csr(const int32_t* order, const int32_t* starts, const float* dout,
                               int V, int E, int trans, int padding_idx, float* grad_weight,
                               void* stream);
/* nn.LSTMCell nonlinearity (RNNDecoder.forward, rnn_decoder.py:80-86): pre
 * [B][4D] gate pre-activations (i, f, g, o) -> h, c [B][D]; act [B][4D] the
 * activated gates kept for the backward.  c_prev nullable (zero state).
 * Backward: dh / dc nullable cotangents -> dpre [B][4D], dc_prev [B][D]
 * (nullable). */
int asr_lstm_cell_forward(const float* pre, const float* c_prev, int B, int D, float* act,
                          float* h, float* c, void* stream);
int asr_lstm_cell_backward(const float* act, const float* c_prev, const float* c,
                           const float* dh, const float* dc, int B, int D, float* dpre,
                           float* dc_prev, void* stream);
int asr_tanh_forward(const float* x, float* y, long long n, void* stream);
int asr_tanh_backward(const float* y, const float* dy, float* dx, long long n, void* stream);
/* y = tanh(a + b) (attention bottleneck with per-branch dropout,
 * attention_seq2seq.py:788-790); its backward is asr_tanh_backward for both. */
int asr_add_tanh_forward(const float* a, const float* b, float* y, long long n, void* stream);
/* y = a + b: the encoder's residual / dense-residual sums (rnn.py:456-462);
 * the backward is the identity to both inputs. */
int asr_add_forward(const float* a, const float* b, float* y, long long n, void* stream);

/* dst[r][0:ncols] = bf16(src[row(r) + 0:ncols]) (round to nearest even) for r <
 * nrows, rows through an asr_rowmap_t (perm / subsample gathers; rows outside
 * [0, t_limit) become zeros).  Builds the dense bf16 GEMM operands of the
 * encoder layer (its input X, W_ih) in bf16 mode. */
int asr_convert_rows_bf16(const float* src, asr_rowmap_t map, int nrows, int ncols,
                          uint16_t* dst, void* stream);
/* Same with an output row pitch ld >= ncols; columns [ncols, ld) are zeros (a
 * bf16 operand whose leading dimension is padded to a multiple of 8). */
int asr_convert_rows_bf16_ld(const float* src, asr_rowmap_t map, int nrows, int ncols, int ld,
                             uint16_t* dst, void* stream);
/* Up to four asr_convert_rows_bf16 conversions in one launch (round 6: a
 * staged linear layer's input, weight and zero pad rows).  Each needs ncols % 8
 * == 0, 16-B aligned rows (src, dst, map strides); returns 1 when launched, 0
 * when a job does not qualify (nothing launched: convert one by one), < 0 on
 * a launch error.  The same bits as the one-by-one conversions. */
int asr_convert_rows_bf16_multi(int n, const float* const* src, const asr_rowmap_t* maps,
                                const int* nrows, const int* ncols, uint16_t* const* dst,
                                void* stream);
/* asr_convert_rows_bf16 of dropout(src): element at linear offset i of src is
 * kept iff u(seed, i) >= p and scaled by 1/(1-p) -- the mask asr_dropout(src,
 * ., n, p, seed) applies -- so a layer's dropped output is staged as the next
 * layer's bf16 GEMM operand in one pass (nn.Dropout after each BLSTM layer,
 * models/pytorch_v3/encoders/rnn.py:392-393, fused with the input staging). */
int asr_convert_rows_bf16_dropout(const float* src, asr_rowmap_t map, int nrows, int ncols,
                                  uint16_t* dst, float p, unsigned long long seed, void* stream);

/* ------------------------------------------------------------ decoding
 * asr_ctc_best_path: CTC greedy best path (greedy_decoder.py:19-47): per
 *   utterance argmax over V for t < lens[b] (first maximum wins ties, as
 *   np.argmax), collapse repeats, drop `blank`.  hyps int32 [B][T] (first
 *   hyp_lens[b] valid), hyp_lens int32 [B].  Bit-exact with the reference.
 * asr_row_argmax: out[r] = argmax_v x[r*V + v] (int64; first max on ties).
 */
int asr_ctc_best_path(const float* logits, long long stride_t, long long stride_b, int T, int B,
                      int V, const int32_t* lens, int blank, int32_t* hyps, int32_t* hyp_lens,
                      void* stream);
int asr_row_argmax(const float* x, int rows, int V, long long* out, void* stream);

/* -------------------------------------------------------------- losses
 * Fused softmax cross-entropy + uniform label smoothing over rows of V logits
 * (attention_seq2seq.py:588-601, criterion.py:51-80, ctc.py:329-337):
 *   loss = ce_scale * sum_{r: tgt[r]>=0} (lse_r - x[r,tgt[r]])
 *        + ls_scale * sum_{r in LS rows} -(1/V) sum_v (x[r,v] - lse_r)
 * LS rows: r = b*T + t with t < lens[b] if lens != NULL, else tgt[r] >= 0.
 * targets int64 (nullable), -1 = ignore.  workspace keeps the row lse for
 * backward (asr_xent_workspace_bytes(R)).  Backward writes
 * dlogits = scale * (*grad_scale) * dloss/dlogits.
 */
size_t asr_xent_workspace_bytes(int R);
int asr_xent_forward(const float* logits, int R, int V, int T, const long long* targets,
                     const int32_t* lens, float ce_scale, float ls_scale, float* loss_out,
                     void* workspace, size_t ws_bytes, void* stream);
int asr_xent_backward(const float* logits, int R, int V, int T, const long long* targets,
                      const int32_t* lens, float ce_scale, float ls_scale,
                      const float* grad_scale, float scale, float* dlogits,
                      const void* workspace, size_t ws_bytes, void* stream);
int asr_softmax(const float* x, int R, int V, float* y, void* stream);

/* ---------------------------------------------------- attention decoder
 * Teacher-forced decoder loop of AttentionSeq2seq._decode_train
 * (attention_seq2seq.py:704-799; bahdanau order, 1-layer LSTMCell decoder
 * rnn_decoder.py:63-113, location attention attention_layer.py:74-251, 1 head).
 * Dims: B utterances, T encoder frames, E encoder width, A attention dim,
 * C conv channels, K conv width (odd), D decoder units, S decoder steps (L+1).
 * Inputs: enc [B][T][E], enc_a [B][T][A] (= W_enc enc + b), lens [B] (the
 *   multiplicative energy mask, :216-225), w_ih_ctx = &W_ih[0][emb] with row
 *   stride ld_ih (the context columns of the decoder LSTMCell W_ih), w_hh
 *   [4D][D], w_dec [A][D], w_conv [A][C], conv_w [C][K], v [A],
 *   pre_emb [B][S][4D] (= emb(y_in) W_ih_emb^T + b_ih + b_hh, one GEMM for all
 *   steps), h0 [B][D] (nullable = zeros; init_dec_state).
 * Forward outputs (all saved for backward): dec [B][S][D] (dec_out_t; t=0:
 *   h0), c [B][S][D], gates [B][S][4D], x [B][S][E+D] (= [ctx_{t-1}; h_{t-1}]),
 *   ctx [B][S][E], aw [B][S][T].
 * Backward inputs: d_dec_in [B][S][D], d_ctx_in [B][S][E] (from the hoisted
 *   W_d / W_c GEMMs).  Outputs: gates_dg (dgates over the saved gates; feeds
 *   dW_ih, dW_hh, db and the embedding gradient), dctx_tot [B][S][E] (feeds
 *   d enc = aw^T dctx_tot), d_enc_a [B][T][A], d_h0 [B][D] (nullable),
 *   dwd_all [B][S][A] (dW_dec = dwd^T dec), per-(utterance, frame chunk)
 *   partials summed over the steps dv_part [B][NC][A], dwc_part [B][NC][A*C],
 *   dcw_part [B][NC][C*K] with NC = asr_attdec_chunks(dims) (column sums give
 *   dV, dW_conv, d conv kernel; fixed summation order, deterministic).
 */
typedef struct {
  int B, T, E, A, C, K, D, S;
  float sharpening;
  int sigmoid_smoothing;
} asr_attdec_dims_t;

/* Training-mode options of the decoder loop (NULL = none of them).
 * dropout_hidden: RNNDecoder dropout on h after the LSTMCell
 *   (rnn_decoder.py:97-98); the dropped h is both dec_out and the recurrent
 *   state.  Mask of element (b, t, j): asr dropout RNG, seed_hidden, index
 *   (b*S + t)*D + j (regenerated in backward).
 * Scheduled sampling (attention_seq2seq.py:744-748): ss_steps_host[t] != 0
 *   (host memory, [S], t >= 1) feeds step t with embed(argmax logits_{t-1})
 *   instead of the teacher token, where logits_{t-1} = fc(tanh(drop_d(W_d
 *   dec_{t-1} + b_d) + drop_c(W_c ctx_{t-1} + b_c))) -- the same logits the loss
 *   sees when the caller applies its post-loop dropouts with seed_d / seed_c
 *   over [B][S][Dz] (index (b*S + t)*Dz + k).  The sampled embedding (row of
 *   emb_w [V][Y], or column of emb_w [Y][V] when emb_trans) is dropped with
 *   drop_emb / seed_emb (index (b*S + t)*Y + y), written to emb_ss [B][S][Y]
 *   (caller zeroes it; teacher steps stay 0) and projected:
 *   pre_ss[b,t] = W_ih[:, :Y] e + b_ih + b_hh (w_ih_emb row stride ld_ih).
 *   tok_ss [B][S] (nullable) receives the sampled tokens.  In backward,
 *   d_pre [B][S][4D] = dG with sampled steps zeroed (the gradient of pre_emb)
 *   and dg_ss [B][S][4D] = dG at sampled steps only (for W_ih[:, :Y] and the
 *   biases through emb_ss); both NULL when no step is sampled. */
typedef struct {
  float dropout_hidden;
  unsigned long long seed_hidden;
  const int32_t* ss_steps_host;
  int Y, Dz, V;
  const float* w_d;
  const float* b_d;
  float drop_d;
  unsigned long long seed_d;
  const float* w_c;
  const float* b_c;
  float drop_c;
  unsigned long long seed_c;
  const float* w_fc;
  const float* b_fc;
  const float* emb_w;
  int emb_trans;
  float drop_emb;
  unsigned long long seed_emb;
  const float* w_ih_emb;
  long long ld_ih;
  const float* b_ih;
  const float* b_hh;
  float* pre_ss;
  float* emb_ss;
  long long* tok_ss;
  float* d_pre;
  float* dg_ss;
} asr_attdec_opts_t;

/* Diagnostics: phase stamps (s_memrealtime ticks, 100 MHz) of the per-step
 * attention kernels' work-group (0, 0) at decoder step 10 of the last pass;
 * host must hold 64 values. */
int asr_att_trace_read(unsigned long long* host);
size_t asr_attdec_workspace_bytes(const asr_attdec_dims_t* dims, int compute_dtype,
                                  int backward);
int asr_attdec_chunks(const asr_attdec_dims_t* dims);
int asr_attdec_forward(const asr_attdec_dims_t* dims, int compute_dtype, const float* enc,
                       const float* enc_a, const int32_t* lens, const float* w_ih_ctx,
                       long long ld_ih, const float* w_hh, const float* w_dec,
                       const float* w_conv, const float* conv_w, const float* v,
                       const float* pre_emb, const float* h0, float* dec, float* c, float* gates,
                       float* x, float* ctx, float* aw, void* workspace, size_t ws_bytes,
                       void* stream);
int asr_attdec_backward(const asr_attdec_dims_t* dims, int compute_dtype, const float* enc,
                        const float* enc_a, const int32_t* lens, const float* w_ih_ctx,
                        long long ld_ih, const float* w_hh, const float* w_dec,
                        const float* w_conv, const float* conv_w, const float* v,
                        const float* dec, const float* c, const float* aw,
                        const float* d_dec_in, const float* d_ctx_in, float* gates_dg,
                        float* dctx_tot, float* d_enc_a, float* d_h0, float* dwd_all,
                        float* dv_part, float* dwc_part, float* dcw_part, void* workspace,
                        size_t ws_bytes, void* stream);
/* The same two calls with training-mode options (asr_attdec_opts_t above). */
int asr_attdec_forward_ex(const asr_attdec_dims_t* dims, const asr_attdec_opts_t* opts,
                          int compute_dtype, const float* enc, const float* enc_a,
                          const int32_t* lens, const float* w_ih_ctx, long long ld_ih,
                          const float* w_hh, const float* w_dec, const float* w_conv,
                          const float* conv_w, const float* v, const float* pre_emb,
                          const float* h0, float* dec, float* c, float* gates, float* x,
                          float* ctx, float* aw, void* workspace, size_t ws_bytes, void* stream);
/* One location-attention step as a standalone op (AttentionMechanism.forward,
 * attention_layer.py:123-251; the layer boundary of SURVEY §8(b)); the same
 * kernels as the decoder loop.  dims->S is ignored.  Forward: conv of aw_prev
 * [B][T], energies from enc_a [B][T][A] + W_dec dec_out [B][D] + W_conv f,
 * multiplicative length mask, sharpening, softmax / sigmoid -> aw_out [B][T],
 * ctx_out [B][E] = aw_out . enc.  Backward (cotangents d_ctx [B][E],
 * d_aw_out [B][T] nullable): d_enc_a, d_dec, d_aw_prev, dctx_tot, dwd (d of
 * W_dec dec_out) written; dv_part / dwc_part / dcw_part hold
 * B * asr_attdec_chunks rows whose column sums are dV, dW_conv and the
 * conv-kernel gradient.  The caller forms dW_dec = dwd^T dec_out and
 * d enc = aw_out^T dctx_tot. */
size_t asr_att_step_workspace_bytes(const asr_attdec_dims_t* dims);
int asr_att_step_forward(const asr_attdec_dims_t* dims, const float* enc, const float* enc_a,
                         const int32_t* lens, const float* w_dec, const float* w_conv,
                         const float* conv_w, const float* v, const float* dec_out,
                         const float* aw_prev, float* ctx_out, float* aw_out, void* workspace,
                         size_t ws_bytes, void* stream);
int asr_att_step_backward(const asr_attdec_dims_t* dims, const float* enc, const float* enc_a,
                          const int32_t* lens, const float* w_dec, const float* w_conv,
                          const float* conv_w, const float* v, const float* dec_out,
                          const float* aw_prev, const float* aw_out, const float* d_ctx,
                          const float* d_aw_out, float* d_enc_a, float* d_dec, float* d_aw_prev,
                          float* dctx_tot, float* dwd, float* dv_part, float* dwc_part,
                          float* dcw_part, void* workspace, size_t ws_bytes, void* stream);

/* Test / diagnostics: the attention-step kernel instantiations the last
 * asr_attdec_forward_ex / _backward_ex launched: out4 = {forward conv-channel
 * template (10 or 3; 0 = generic), forward 32-frame chunks per utterance,
 * backward template, backward chunks}. */
int asr_attdec_last_launch(int* out4);
/* {forward, backward}: 1 if the last decoder pass of that direction ran as one
 * persistent launch (bf16, B <= 32, no scheduled sampling; ASR_ATT_PERSIST=0
 * disables it). */
int asr_attdec_persist_last(int* out2);
/* Round 6: the conv features of every decoder step kept by the next
 * persistent forward pass from this host thread and read back by the next
 * persistent backward pass (instead of recomputing them from aw); buf holds
 * asr_attdec_conv_feat_bytes(dims) bytes, NULL turns it off.  The caller sets
 * it before each pass and resets it after; a backward may only be given the
 * buffer of a forward that ran persistent (asr_attdec_persist_last). */
int asr_attdec_set_conv_feat(float* buf);
size_t asr_attdec_conv_feat_bytes(const asr_attdec_dims_t* dims);
int asr_attdec_backward_ex(const asr_attdec_dims_t* dims, const asr_attdec_opts_t* opts,
                           int compute_dtype, const float* enc, const float* enc_a,
                           const int32_t* lens, const float* w_ih_ctx, long long ld_ih,
                           const float* w_hh, const float* w_dec, const float* w_conv,
                           const float* conv_w, const float* v, const float* dec,
                           const float* c, const float* aw, const float* d_dec_in,
                           const float* d_ctx_in, float* gates_dg, float* dctx_tot,
                           float* d_enc_a, float* d_h0, float* dwd_all, float* dv_part,
                           float* dwc_part, float* dcw_part, void* workspace, size_t ws_bytes,
                           void* stream);

/* ------------------------------------------------------------- VGG front-end
 * Replaces CNNEncoder (models/pytorch_v3/encoders/cnn.py:124-165): Conv2d 3x3
 * (padding 1) -> ReLU -> MaxPool (first floor mode, later ceil) -> BatchNorm2d
 * -> Dropout per layer, input viewed [B, 1, F, T] (cnn.py:143-149), output
 * [B, T', F'*C] (cnn.py:155-157).  Layer tensors are channels-last with a zero
 * halo: [B][T+2][F+2][C] ("padded pixels").  Layers with C_in >= 16 run the
 * 3x3 convolution as one asr_gemm with tap addressing (asr_operand_t);
 * C_in = 1 (and channel counts that are not multiples of 16) use
 * asr_conv_direct_*.
 * asr_vgg_pool_dims: output extent of a pool (kernel = stride), torch's
 *   floor / ceil rules.
 * asr_vgg_block_forward / _backward: ReLU + pool + BatchNorm (training batch
 *   statistics over every (b, f, t) incl. padding frames, running stats with
 *   momentum / unbiased variance; or eval with running stats) + dropout (asr
 *   dropout RNG, index = element of [B][T'][F'][C]).  See cnn.hip. */
int asr_vgg_pad_input(const float* xs, int B, int T, int F, float* out, void* stream);
/* ... as a Cp-channel image (channel 0 = xs, the rest 0; out_dtype f32 / bf16):
 * the first conv layer on the GEMM path with its one input channel padded to 16 */
int asr_vgg_pad_input_ch(const float* xs, int B, int T, int F, int Cp, int out_dtype, void* out,
                         void* stream);
/* GEMM images of a Conv2d weight W [Co][Ci][3][3] (tap j = kw*3 + kh):
 * mode 0 out[co][j*Ci + ci] (forward B operand), mode 1 out[ci][j*Co + co]
 * (input-gradient B operand); unpack_acc: dW [Co][Ci][3][3] += [Co][9 Ci]. */
int asr_conv_weight_pack(const float* w, int Co, int Ci, int mode, int out_dtype, void* out,
                         void* stream);
int asr_conv_weight_unpack_acc(const float* packed, int Co, int Ci, float* dw, void* stream);
/* mode-0 image / unpack with an input-channel pitch Cip >= Ci (padded channels
 * stay as the caller zeroed them) */
int asr_conv_weight_pack_pad(const float* w, int Co, int Ci, int Cip, int mode, int out_dtype,
                             void* out, void* stream);
/* The same from the transposed image packed_t [9 Cip][Co] (the weight
 * gradient computed as X^T dZ, so that C_out is the product's narrow N). */
int asr_conv_weight_unpack_acc_pad_t(const float* packed_t, int Co, int Ci, int Cip, float* dw,
                                     void* stream);
int asr_conv_weight_unpack_acc_pad(const float* packed, int Co, int Ci, int Cip, float* dw,
                                   void* stream);
/* Direct 3x3 convolution (layers the tap-addressed GEMM cannot take: C_in = 1,
 * channel counts not multiples of 16): x [padded pixels][Ci] f32, w the torch
 * weight [Co][Ci][3][3]; z / dx over valid pixels; dw / dbias accumulate. */
int asr_conv_direct_forward(const float* x, int B, int T, int F, int Ci, int Co, const float* w,
                            const float* bias, float* z, void* stream);
/* Single-input-channel 3x3 convolution forward (the first VGG layer) from
 * channel 0 of a padded operand x [B][T+2][F+2][cstride] (x_dtype ASR_DT_F32
 * or ASR_DT_BF16, e.g. the GEMM path's 16-channel bf16 staging): z
 * [B][T+2][F+2][Co] f32 at valid pixels (+ bias); Co % 4 == 0, Co <= 512.
 * Same sum as asr_conv_direct_forward with Ci = 1 (CNNEncoder's first Conv2d,
 * cnn.py:124-165). */
int asr_conv3x3_c1_forward(const void* x, int x_dtype, int cstride, int B, int T, int F, int Co,
                           const float* w, const float* bias, float* z, void* stream);
/* asr_conv3x3_c1_forward reading the raw features xs [B][T][F] f32 (the first
 * VGG layer, encoders/cnn.py:124-165), each value rounded to bf16 first when
 * round_bf16 (the bf16 operand's values); Co / 4 must divide 256. */
int asr_conv3x3_c1_forward_xs(const float* xs, int round_bf16, int B, int T, int F, int Co,
                              const float* w, const float* bias, void* z, int z_dtype,
                              void* stream);
/* 3x3 convolution of a zero-haloed channels-last bf16 operand, tap-resident
 * (csrc/conv.hip; replaces the tap-addressed asr_gemm product of the VGG
 * convolutions, encoders/cnn.py:124-165 Conv2d 3x3 padding 1):
 *   out[p][n] = bias[n] + sum_{tap < 9} sum_{c < Cin} in[p + s(tap)][c] * w[n][tap Cin + c],
 *   s(tap) = sign * ((tap / 3 - 1) * Fp + (tap % 3 - 1)), rows outside [0, P) zero,
 * for every padded pixel row p < P (Fp = F + 2: the grid's row pitch).  in bf16
 * [P][Cin], w bf16 [Cout][9 Cin] (asr_conv_weight_pack_pad / _pack images),
 * bias f32 [Cout] or NULL, out [P][Cout] f32 or bf16 (out_dtype).  sign = 1:
 * the forward; sign = -1 with the mirrored weight image: the input gradient.
 * The f32 sums are asr_gemm's (same k order).  Cin, Cout in {64, 128};
 * ASR_ERR_UNSUPPORTED otherwise (asr_conv3x3_tr_supported says which). */
int asr_conv3x3_tr_supported(int Cin, int Cout, int Fp);
int asr_conv3x3_tr(const void* in, long long P, int Cin, int Fp, int sign, const void* w,
                   int Cout, const float* bias, void* out, int out_dtype, void* stream);
/* Weight-gradient image of the same convolution (csrc/conv.hip, replaces the
 * dz^T X tap GEMM): packed[n][tap Cin + c] = sum_p dz[p][n] * x[p + s(tap)][c]
 * (sign +1), overwritten, f32 [Cout][9 Cin] -- the image
 * asr_conv_weight_unpack_acc_pad accumulates into the Conv2d weight gradient.
 * x bf16 [P][Cin], dz bf16 [P][Cout]; per-chunk partials in the workspace
 * (asr_conv3x3_tr_wgrad_workspace_bytes, 0 = shape not supported), summed in a
 * fixed order (deterministic).  Cin, Cout in {64, 128}. */
/* Weight-gradient image of the first VGG layer (one input channel) straight
 * from the raw features xs [B][T][F] f32 (rounded to bf16 when round_bf16):
 * packed [Co][9 Cip] f32 (overwritten) = the tap GEMM's dz^T X image over the
 * Cip-channel padded operand whose channel 0 holds xs (channels >= 1 zero);
 * dz bf16 [B (T+2) (F+2)][Co].  Co = 64; workspace
 * asr_conv3x3_c1_wgrad_workspace_bytes(Co). */
size_t asr_conv3x3_c1_wgrad_workspace_bytes(int Co);
int asr_conv3x3_c1_wgrad_xs(const float* xs, int round_bf16, int B, int T, int F, int Co,
                            const void* dz, int Cip, float* packed, void* ws, size_t ws_bytes,
                            void* stream);
/* Zero the one-pixel halo (rows t = 0, T + 1 and columns f = 0, F + 1) of a
 * channels-last padded grid [B][T+2][F+2][C] of dtype (ASR_DT_F32 / _BF16;
 * C * size % 16 == 0): the producers of the VGG layer operands write only the
 * interior, so the buffer need not be zero-filled whole. */
int asr_vgg_zero_halo(void* buf, int dtype, int B, int T, int F, int C, void* stream);
size_t asr_conv3x3_tr_wgrad_workspace_bytes(long long P, int Cin, int Cout, int Fp);
int asr_conv3x3_tr_wgrad(const void* x, const void* dz, long long P, int Cin, int Fp, int Cout,
                         float* packed, void* ws, size_t ws_bytes, void* stream);
int asr_conv_direct_dgrad(const float* dz, int B, int T, int F, int Ci, int Co, const float* w,
                          float* dx, void* stream);
size_t asr_conv_direct_wgrad_workspace_bytes(int B, int T, int F, int Ci, int Co);
int asr_conv_direct_wgrad(const float* x, const float* dz, int B, int T, int F, int Ci, int Co,
                          float* dw, float* dbias, void* workspace, size_t ws_bytes,
                          void* stream);
int asr_vgg_accumulate(const float* a, float* dst, int n, const float* a2, float* dst2, int n2,
                       void* stream);
int asr_vgg_pool_dims(int T, int F, int pt, int pf, int ceil_mode, int* To, int* Fo);
size_t asr_vgg_block_workspace_bytes(int B, int To, int Fo, int C);
int asr_vgg_block_forward(const float* z, int B, int T, int F, int C, int pt, int pf,
                          int ceil_mode, float* P, uint8_t* slot, const float* gamma,
                          const float* beta, float* run_mean, float* run_var, int training,
                          float momentum, float eps, float* bn_mean, float* bn_rstd, float drop,
                          unsigned long long seed, void* out, int out_dtype, int flat,
                          void* workspace, size_t ws_bytes, void* stream);
int asr_vgg_block_backward(const float* dnext, int flat, const float* z, int B, int T, int F,
                           int C, int pt, int pf, int ceil_mode, const float* P,
                           const uint8_t* slot, const float* gamma, const float* bn_mean,
                           const float* bn_rstd, float* dgamma, float* dbeta, float drop,
                           unsigned long long seed, void* dz, int dz_dtype, void* workspace,
                           size_t ws_bytes, void* stream);
/* ... and dbias (nullable) += the conv bias gradient (per-channel sum of the
 * f32 dZ values, fixed order), so dZ can be stored as a bf16 GEMM operand. */
int asr_vgg_block_backward_ex(const float* dnext, int flat, const float* z, int B, int T, int F,
                              int C, int pt, int pf, int ceil_mode, const float* P,
                              const uint8_t* slot, const float* gamma, const float* bn_mean,
                              const float* bn_rstd, float* dgamma, float* dbeta, float drop,
                              unsigned long long seed, void* dz, int dz_dtype, float* dbias,
                              void* workspace, size_t ws_bytes, void* stream);
/* asr_vgg_block_forward / asr_vgg_block_backward_ex with the conv output z of
 * dtype z_dtype (ASR_DT_F32 or ASR_DT_BF16, C % 4 == 0): in bf16 mode the
 * convolution GEMMs write z as bf16 (asr_gemm_t.c_dtype), halving its
 * write and its two reads (ReLU + pool forward, ReLU mask backward). */
int asr_vgg_block_forward_z(const void* z, int z_dtype, int B, int T, int F, int C, int pt,
                            int pf, int ceil_mode, float* P, uint8_t* slot, const float* gamma,
                            const float* beta, float* run_mean, float* run_var, int training,
                            float momentum, float eps, float* bn_mean, float* bn_rstd, float drop,
                            unsigned long long seed, void* out, int out_dtype, int flat,
                            void* workspace, size_t ws_bytes, void* stream);
int asr_vgg_block_backward_z(const float* dnext, int flat, const void* z, int z_dtype, int B,
                             int T, int F, int C, int pt, int pf, int ceil_mode, const float* P,
                             const uint8_t* slot, const float* gamma, const float* bn_mean,
                             const float* bn_rstd, float* dgamma, float* dbeta, float drop,
                             unsigned long long seed, void* dz, int dz_dtype, float* dbias,
                             void* workspace, size_t ws_bytes, void* stream);
/* asr_vgg_block_backward_z with the incoming gradient's dtype: dnext_dtype
 * ASR_DT_BF16 (C % 4 == 0, bf16 z and dz, full-resolution pass) reads a bf16
 * dnext (the input-gradient convolution of the layer above writes it so). */
int asr_vgg_block_backward_zd(const void* dnext, int dnext_dtype, int flat, const void* z,
                              int z_dtype, int B, int T, int F, int C, int pt, int pf,
                              int ceil_mode, const float* P, const uint8_t* slot,
                              const float* gamma, const float* bn_mean, const float* bn_rstd,
                              float* dgamma, float* dbeta, float drop, unsigned long long seed,
                              void* dz, int dz_dtype, float* dbias, void* workspace,
                              size_t ws_bytes, void* stream);
/* The two above with the pooled-value store P of dtype p_dtype: ASR_DT_BF16
 * (bf16 z, C % 4 == 0, P 8-B aligned) stores P = max(0, max z) as bf16 --
 * exact, since every candidate is a bf16 value -- halving P's write and its
 * four reads (BN moments, BN apply, BN backward moments, ReLU mask). */
int asr_vgg_block_forward_zp(const void* z, int z_dtype, int B, int T, int F, int C, int pt,
                             int pf, int ceil_mode, void* P, int p_dtype, uint8_t* slot,
                             const float* gamma, const float* beta, float* run_mean,
                             float* run_var, int training, float momentum, float eps,
                             float* bn_mean, float* bn_rstd, float drop, unsigned long long seed,
                             void* out, int out_dtype, int flat, void* workspace,
                             size_t ws_bytes, void* stream);
int asr_vgg_block_backward_zdp(const void* dnext, int dnext_dtype, int flat, const void* z,
                               int z_dtype, int B, int T, int F, int C, int pt, int pf,
                               int ceil_mode, const void* P, int p_dtype, const uint8_t* slot,
                               const float* gamma, const float* bn_mean, const float* bn_rstd,
                               float* dgamma, float* dbeta, float drop, unsigned long long seed,
                               void* dz, int dz_dtype, float* dbias, void* workspace,
                               size_t ws_bytes, void* stream);
/* The first VGG layer (one input channel, stencil from the raw features as
 * asr_conv3x3_c1_forward_xs) when it is unpooled and followed by batch norm:
 * writes P = max(0, bf16(z)) [B][T][F][Co] bf16 directly -- the value the
 * ReLU pass would store -- and, with mpart / qpart, per-block partial sums of
 * P - shift and its square ([asr_vgg_c1_relu_p_blocks(B, T)][Co] each; shift =
 * the running mean), so no conv output z is written or read back
 * (cnn.py:124-165's Conv2d -> ReLU -> BatchNorm2d of layer 0). */
int asr_vgg_c1_relu_p_blocks(int B, int T);
int asr_vgg_c1_forward_relu_p(const float* xs, int round_bf16, int B, int T, int F, int Co,
                              const float* w, const float* bias, uint16_t* P, const float* shift,
                              float* mpart, float* qpart, void* stream);
/* asr_vgg_block_forward_zp from that P and its partials: batch statistics
 * (training) or running statistics, the running-stat update, and the next
 * layer's input (bf16 padded rows, or flat f32).  workspace >= C floats. */
int asr_vgg_block_forward_given_p(const uint16_t* P, int B, int T, int F, int C,
                                  const float* gamma, const float* beta, float* run_mean,
                                  float* run_var, int training, float momentum, float eps,
                                  float* bn_mean, float* bn_rstd, float drop,
                                  unsigned long long seed, void* out, int out_dtype, int flat,
                                  const float* mpart, const float* qpart, int nblk,
                                  void* workspace, size_t ws_bytes, void* stream);

/* ----------------------------------------------------------- profiling
 * Sampled HIP-event timing of the recurrence step kernels on their own stream
 * (bench.py's live roofline measurement).  asr_prof_begin(stride): bracket
 * every stride-th launch of each tracked kernel with an event pair.
 * asr_prof_end: synchronises on the recorded events (the only entry point
 * that does), fills mean_us[k] (mean launch duration, microseconds) and
 * launches[k] (all launches seen) for k = 0 lstm forward step, 1 lstm
 * backward step (per-step kernels, sampled), 2 lstm forward pass, 3 lstm
 * backward pass (persistent kernels, one launch per layer pass, all timed),
 * 4 the asr_gemm main kernel (all timed; mean_work[4] = mean algorithmic
 * flops 2*M*N*K per timed launch).  mean_work may be NULL.
 */
int asr_prof_begin(int stride);
int asr_prof_end(double* mean_us, long long* launches, double* mean_work, int nkinds);
/* Every timed sample of kind `kind` after asr_prof_end: per sample the tag
 * naming the kernel instantiation (GEMM / convolution family x 4 + operand
 * modes, the CTC vocabulary V, the persistent LSTM pass form; prof.h
 * ASR_PTAG_*), its algorithmic work and its duration in microseconds, up to
 * `max` samples.  Returns the sample count, -1 before asr_prof_end. */
long long asr_prof_samples(int kind, int* tags, double* work, double* us, long long max);

/* Status word of the persistent recurrence kernels: bit 0 set when a bounded
 * inter-work-group wait gave up (a co-residency failure; that pass's outputs
 * are invalid).  Synchronises `stream`; clear != 0 resets the word. */
int asr_lstm_persist_status(int* status, int clear, void* stream);

/* The same two status words, stream-ordered and without a host sync:
 * dst (device int32[2]) = {counter-form word, tagged-granule word}; clear != 0
 * then zeroes both.  The training step gathers them after its backward and
 * hands dst (MAX-all-reduced over data-parallel ranks) to
 * asr_optim_step_guarded, so a pass whose spin gave up never updates the
 * weights; the host reads dst at the step's loss read-back and skips the
 * batch (training_loop.py:69-76 semantics).  asr_lstm_status_inject sets the
 * tagged-granule word (test hook: what a spin give-up does). */
int asr_lstm_status_gather(int* dst, int clear, void* stream);
int asr_lstm_status_inject(int bits, void* stream);

/* Hand-off protocols the tagged-granule recurrence (lstm_xg.hip) has run
 * since the last clear: bit 0 write-through (sc1, any placement), bit 1
 * XCD-local (every group's work-groups registered on one XCD).  Synchronises
 * the device. */
int asr_lstm_xg_mode(int* mode, int clear);

/* Which recurrence implementation the last BLSTM layer pass ran (host-side
 * record), out2 = {forward pass, backward pass}: 0 per-step kernels, 1
 * tagged-granule bf16, 2 tagged-granule f32 (reference precision), 3
 * tagged-granule bf16 with the fused input projection, 4 counter-form
 * persistent. */
int asr_lstm_last_path(int* out2);

/* Diagnostics (ASR_XG_TRACE=1 at the first recurrence launch): copies the
 * per-step phase timestamps of work-groups 0..63 (64 x 128 steps x 12 u64) to
 * `host` (may be NULL); returns the element count, 0 when tracing is off. */
long long asr_xg_trace_read(unsigned long long* host);
/* The persistent backward recurrence's dynamic-LDS pin (KB, in (80, 160]; 0 =
 * ASR_XG_PIN_BWD_KB or the 140 KB default) for the launches that follow.  At
 * the default no kernel with more than 9 KB of LDS -- every GEMM and
 * convolution kernel -- can be co-resident with it. */
int asr_lstm_set_bwd_pin_kb(int kb);
/* Hidden units per work-group of the tagged-granule backward recurrence for the
 * launches that follow: 0 (ASR_XG_BWD_XU, else 16), 16, or 32 -- half the
 * work-groups, so a layer of 2 x 8 rows x 512 units takes 128 of 256 CUs and
 * the weight-gradient GEMMs of the layer above run beside it (native_ops'
 * ASR_OVERLAP_WGRAD mode 3).  32 applies only where H % 32 == 0, H <= 512 and
 * 8 rows per group fit; elsewhere 16 is used. */
int asr_lstm_set_bwd_units(int xu);
/* Work-groups that backward recurrence launches for [B, *, H] with xu units per
 * work-group (0: the current setting); 0 if the shape cannot take that path. */
int asr_lstm_backward_grid(int B, int H, int xu);
/* Pipelined input gradients (the layer above's dX GEMMs overlapping this
 * layer's backward recurrence, rnn.py:343-390's stacked layers): dy of the
 * asr_lstm_backward_dgbf_h launches that follow is written concurrently, in
 * chunks of processing steps q in [c0 k, c0 (k + 1)) -- rows t = q and
 * t = T - 1 - q -- complete once flags[k] == epoch (chunks up to the middle
 * step (T + 1) / 2 - 1).  The recurrence
 * waits for each chunk's flag before reading its dy rows.  flags NULL: off. */
int asr_lstm_set_dy_flags(const int* flags, int c0, int epoch);

/* Split input gradient (round 6): the next asr_lstm_backward_dgbf_h launch
 * adds 1 to *counter per cell wave once the gate gradients of processing steps
 * <= q are stored and released at agent scope (NULL: off; applies to launches
 * from the calling host thread until reset).  asr_lstm_bwd_progress_arrivals:
 * what one launch of [B, *, H] adds.  asr_lstm_progress_gate enqueues a wait
 * on another stream until *counter >= target (bounded; a timeout sets the
 * recurrence status word, so the step is skipped).  Processing step q covers
 * t = T-1-q (forward direction) and t = q (reverse): rows t in [T-1-q, q] of
 * dG are final once q >= T/2. */
int asr_lstm_set_bwd_progress(unsigned long long* counter, int q);
/* Two reporting steps q1 < q2 (round 6, the two-chunk split): one launch's
 * arrivals are added at each. */
int asr_lstm_set_bwd_progress2(unsigned long long* counter, int q1, int q2);
long long asr_lstm_bwd_progress_arrivals(int B, int H);
int asr_lstm_progress_gate(const unsigned long long* counter, long long target, void* stream);
/* Per-step workspace arena (round 6): the workspace handed to the next
 * tagged-granule launch from this host thread is already zero (on = 1), so
 * the launch skips its own memset.  Consumed by that launch; reset it after
 * the call.  Replaces asr_lstm_workspace_bytes' "zeroed before every launch"
 * with one fill per training step (native_ops.rec_arena_begin). */
int asr_lstm_ws_prezeroed(int on);
/* Leading bytes of such a workspace a tagged-granule launch of [B, *, H]
 * zeroes (the arena clears only these). */
size_t asr_lstm_ws_zero_bytes(int B, int H);
/* Stream-ordered: flags[k] = epoch after the work enqueued before it. */
int asr_lstm_dy_signal(int* flags, int k, int epoch, void* stream);
/* Diagnostics only (tools/cores_locate.py): backward recurrence launches
 * enqueued on `stream` after this call record every dh_t their cell waves form
 * into dh ([B][T][2][H] f32), each step's sweep spin count into spins
 * ([ceil(B/R)][T][2][H/16] u32) and, per cell and step, the four gate
 * gradients computed, the four activations, c_t, c_{t-1}, dy and the incoming
 * dc into cell ([B][T][2][H][12] f32); NULL pointers switch recording off. */
int asr_lstm_debug_dh(float* dh, unsigned* spins, float* cell, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ASR_HIP_H_ */
