// Sampled per-launch HIP-event timing of the recurrence step kernels, used by
// bench.py to measure the dominant kernel's average launch duration live, on
// the stream the kernel is launched on (torch.cuda.Event only sees torch's own
// stream ops).  Every `stride`-th launch of a tracked kernel is bracketed by an
// event pair; asr_prof_end synchronises on the recorded events and returns the
// mean duration per tracked kernel.  Off by default (zero cost).
#include <vector>

#include "common.h"
#include "prof.h"

namespace asr {
namespace {
constexpr int kMaxPairs = 4096;

struct KindState {
  std::vector<hipEvent_t> ev;  // 2 per sample
  int used = 0;
  long long seen = 0;
  long long launches = 0;
  double work = 0.0;  // summed over the timed launches
};

struct Prof {
  bool on = false;
  int stride = 8;
  KindState k[ASR_PROF_NKINDS];
};

Prof& prof() {
  static Prof p;
  return p;
}
}  // namespace

bool prof_on() { return prof().on; }

int prof_begin_launch(int kind, hipStream_t s, double work) {
  Prof& p = prof();
  if (!p.on) return -1;
  KindState& k = p.k[kind];
  k.launches++;
  const int stride = kind >= ASR_PROF_LSTM_FWD_SEQ ? 1 : p.stride;   // passes: every launch
  if ((k.seen++ % stride) != 0 || k.used >= kMaxPairs) return -1;
  const int slot = k.used++;
  k.work += work;
  (void)hipEventRecord(k.ev[2 * slot], s);
  return slot;
}

void prof_end_launch(int kind, int slot, hipStream_t s) {
  if (slot < 0) return;
  (void)hipEventRecord(prof().k[kind].ev[2 * slot + 1], s);
}
}  // namespace asr

using namespace asr;

extern "C" int asr_prof_begin(int stride) {
  Prof& p = prof();
  p.stride = stride > 0 ? stride : 1;
  for (int i = 0; i < ASR_PROF_NKINDS; ++i) {
    KindState& k = p.k[i];
    if (k.ev.empty()) {
      k.ev.resize(2 * kMaxPairs);
      for (auto& e : k.ev) ASR_CHECK_HIP(hipEventCreate(&e));
    }
    k.used = 0;
    k.seen = 0;
    k.launches = 0;
    k.work = 0.0;
  }
  p.on = true;
  return ASR_OK;
}

extern "C" int asr_prof_end(double* mean_us, long long* launches, double* mean_work,
                            int nkinds) {
  Prof& p = prof();
  p.on = false;
  for (int i = 0; i < ASR_PROF_NKINDS && i < nkinds; ++i) {
    KindState& k = p.k[i];
    double tot = 0.0;
    for (int j = 0; j < k.used; ++j) {
      ASR_CHECK_HIP(hipEventSynchronize(k.ev[2 * j + 1]));
      float ms = 0.f;
      ASR_CHECK_HIP(hipEventElapsedTime(&ms, k.ev[2 * j], k.ev[2 * j + 1]));
      tot += ms;
    }
    mean_us[i] = k.used ? 1000.0 * tot / k.used : 0.0;
    launches[i] = k.launches;
    if (mean_work) mean_work[i] = k.used ? k.work / k.used : 0.0;
  }
  return ASR_OK;
}
