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
/* Number of gfx950 code objects linked in (sanity check for loaders). */
int asr_arch_is_gfx950(void);

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
int asr_ctc_backward(const float* acts, long long stride_t, long long stride_b, int T, int B,
                     int V, const int32_t* labels_flat, const int32_t* label_lens,
                     const int32_t* act_lens, int max_label_len, int blank,
                     const float* grad_scale, float scale, float* grads, long long gstride_t,
                     long long gstride_b, const void* workspace, size_t ws_bytes, void* stream);
/* warp-ctc drop-in: forward + backward with scale 1 in one call. */
int asr_ctc_fwd_bwd(const float* acts, long long stride_t, long long stride_b, int T, int B,
                    int V, const int32_t* labels_flat, const int32_t* label_lens,
                    const int32_t* act_lens, int max_label_len, int blank, int zero_infinity,
                    float* costs, float* grads, void* workspace, size_t ws_bytes, void* stream);

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
} asr_gemm_t;

int asr_gemm(const asr_gemm_t* problems, int nprob, int compute_dtype, void* stream);

/* out0[n] (+ out1[n] if non-NULL) += alpha * sum_m g[m*ld + n]  (bias grads of
 * nn.Linear / nn.LSTM bias_ih and bias_hh); fixed-order, deterministic. */
size_t asr_colsum_workspace_bytes(int M, int N);
int asr_colsum_accumulate(const float* g, long long ld, int M, int N, float alpha, float* out0,
                          float* out1, void* workspace, size_t ws_bytes, void* stream);

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
 */
size_t asr_lstm_workspace_bytes(int B, int H, int compute_dtype, int backward);
int asr_lstm_forward(float* gx_act, const void* whh_f, const void* whh_r, int w_dtype,
                     const int32_t* lens, int B, int T, int H, int compute_dtype, float* y,
                     float* cst, void* workspace, size_t ws_bytes, void* stream);
int asr_lstm_backward(const float* dy, const void* whh_f, const void* whh_r, int w_dtype,
                      const int32_t* lens, int B, int T, int H, int compute_dtype, float* act_dg,
                      const float* cst, void* workspace, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ASR_HIP_H_ */
