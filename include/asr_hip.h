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

#ifdef __cplusplus
}
#endif
#endif /* ASR_HIP_H_ */
