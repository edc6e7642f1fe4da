// Internal: sampled per-launch event timing hooks (see prof.hip).
#pragma once
#include <hip/hip_runtime.h>

#define ASR_PROF_LSTM_FWD 0      /* per-step forward kernel (sampled every `stride`) */
#define ASR_PROF_LSTM_BWD 1      /* per-step backward kernel (sampled) */
#define ASR_PROF_LSTM_FWD_SEQ 2  /* persistent forward pass (every launch timed) */
#define ASR_PROF_LSTM_BWD_SEQ 3  /* persistent backward pass (every launch timed) */
#define ASR_PROF_GEMM 4          /* asr_gemm main kernel (every launch timed, flops recorded) */
#define ASR_PROF_CTC_FWD 5       /* CTC emissions + lattice (algorithmic bytes recorded) */
#define ASR_PROF_CTC_GRAD 6      /* CTC gradient pass (algorithmic bytes recorded) */
#define ASR_PROF_ATT_FWD 7       /* persistent attention-decoder forward pass (bytes recorded) */
#define ASR_PROF_ATT_BWD 8       /* persistent attention-decoder backward pass (bytes recorded) */
#define ASR_PROF_NKINDS 9

namespace asr {
bool prof_on();
int prof_begin_launch(int kind, hipStream_t s, double work = 0.0);
void prof_end_launch(int kind, int slot, hipStream_t s);
}  // namespace asr
