// Internal: sampled per-launch event timing hooks (see prof.hip).
#pragma once
#include <hip/hip_runtime.h>

#define ASR_PROF_LSTM_FWD 0      /* per-step forward kernel (sampled every `stride`) */
#define ASR_PROF_LSTM_BWD 1      /* per-step backward kernel (sampled) */
#define ASR_PROF_LSTM_FWD_SEQ 2  /* persistent forward pass (every launch timed) */
#define ASR_PROF_LSTM_BWD_SEQ 3  /* persistent backward pass (every launch timed) */
#define ASR_PROF_GEMM 4          /* asr_gemm main kernel and the convolutions (flops recorded) */
#define ASR_PROF_CTC_FWD 5       /* CTC emissions + lattice (algorithmic bytes recorded) */
#define ASR_PROF_CTC_GRAD 6      /* CTC gradient pass (algorithmic bytes recorded) */
#define ASR_PROF_ATT_FWD 7       /* persistent attention-decoder forward pass (bytes recorded) */
#define ASR_PROF_ATT_BWD 8       /* persistent attention-decoder backward pass (bytes recorded) */
#define ASR_PROF_NKINDS 9

// Per-sample tags naming the kernel instantiation (bench.py turns them into
// the rocprof kernel names).  GEMM family: tag = 4 * family + operand modes
// (2 * a.trans + b.trans); the CTC kinds: tag = V; the persistent LSTM passes:
// one of ASR_PTAG_LSTM_*.
#define ASR_PTAG_GEMM_8R 1
#define ASR_PTAG_GEMM_8W 2
#define ASR_PTAG_GEMM_KK256 3
#define ASR_PTAG_GEMM_N64 4
#define ASR_PTAG_GEMM_FAST2 5
#define ASR_PTAG_GEMM_FAST4 6
#define ASR_PTAG_GEMM_GEN_BF16 7
#define ASR_PTAG_GEMM_GEN_F32 8
#define ASR_PTAG_CONV_TR 9        /* modes: 0 */
#define ASR_PTAG_CONV_TR_WGRAD 10
#define ASR_PTAG_CONV_C1_WGRAD 11
#define ASR_PTAG_GEMM_F32F 12      /* gemm_f32_fast<a, b> */
#define ASR_PTAG_LSTM_FWD_XG 1
#define ASR_PTAG_LSTM_FWD_XGX 2
#define ASR_PTAG_LSTM_BWD_XG 3
#define ASR_PTAG_LSTM_PERSIST 4

namespace asr {
bool prof_on();
int prof_begin_launch(int kind, hipStream_t s, double work = 0.0, int tag = 0);
void prof_set_tag(int kind, int slot, int tag);
void prof_end_launch(int kind, int slot, hipStream_t s);
}  // namespace asr
