// Internal: sampled per-launch event timing hooks (see prof.hip).
#pragma once
#include <hip/hip_runtime.h>

#define ASR_PROF_LSTM_FWD 0
#define ASR_PROF_LSTM_BWD 1
#define ASR_PROF_NKINDS 2

namespace asr {
bool prof_on();
int prof_begin_launch(int kind, hipStream_t s);
void prof_end_launch(int kind, int slot, hipStream_t s);
}  // namespace asr
