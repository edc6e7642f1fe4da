// Sampled per-launch HIP-event timing of the hot kernels, used by bench.py to
// measure each kernel's average launch duration live, on the stream the kernel
// is launched on (torch.cuda.Event only sees torch's own stream ops).  Every
// `stride`-th launch of a per-step kind (every launch of the other kinds) is
// bracketed by an event pair and carries its algorithmic work and a tag that
// names the kernel instantiation (GEMM family + operand modes, CTC vocabulary,
// ...), so bench.py can report one roofline row per kernel rather than per
// family.  asr_prof_end synchronises on the recorded events and returns the
// per-kind means; asr_prof_samples then returns every timed sample.  Off by
// default (zero cost).
#include <vector>

#include "common.h"
#include "prof.h"

namespace asr {
namespace {
constexpr int kMaxPairs = 4096;

struct KindState {
  std::vector<hipEvent_t> ev;  // 2 per sample
  std::vector<int> tag;        // per sample
  std::vector<double> work;    // per sample
  std::vector<double> us;      // per sample, filled by asr_prof_end
  int used = 0;
  long long seen = 0;
  long long launches = 0;
};

struct Prof {
  bool on = false;
  bool done = false;   // asr_prof_end has resolved the samples
  int stride = 8;
  KindState k[ASR_PROF_NKINDS];
};

Prof& prof() {
  static Prof p;
  return p;
}
}  // namespace

bool prof_on() { return prof().on; }

int prof_begin_launch(int kind, hipStream_t s, double work, int tag) {
  Prof& p = prof();
  if (!p.on) return -1;
  KindState& k = p.k[kind];
  k.launches++;
  const int stride = kind >= ASR_PROF_LSTM_FWD_SEQ ? 1 : p.stride;   // passes: every launch
  if ((k.seen++ % stride) != 0 || k.used >= kMaxPairs) return -1;
  const int slot = k.used++;
  k.work[slot] = work;
  k.tag[slot] = tag;
  (void)hipEventRecord(k.ev[2 * slot], s);
  return slot;
}

int g_last_tag[ASR_PROF_NKINDS];   // the last launch's tag per kind, sampled or not

void prof_set_tag(int kind, int slot, int tag) {
  g_last_tag[kind] = tag;
  if (slot < 0) return;
  prof().k[kind].tag[slot] = tag;
}

void prof_end_launch(int kind, int slot, hipStream_t s) {
  if (slot < 0) return;
  (void)hipEventRecord(prof().k[kind].ev[2 * slot + 1], s);
}
}  // namespace asr

// Tag of the last GEMM launch from any host thread (4 x kernel family + mode,
// csrc/prof.h ASR_PTAG_GEMM_*): diagnostics (tools/gemm_log.py).
extern "C" int asr_gemm_last_family(void) { return asr::g_last_tag[ASR_PROF_GEMM]; }

using namespace asr;

extern "C" int asr_prof_begin(int stride) {
  Prof& p = prof();
  p.stride = stride > 0 ? stride : 1;
  for (int i = 0; i < ASR_PROF_NKINDS; ++i) {
    KindState& k = p.k[i];
    if (k.ev.empty()) {
      k.ev.resize(2 * kMaxPairs);
      for (auto& e : k.ev) ASR_CHECK_HIP(hipEventCreate(&e));
      k.tag.assign(kMaxPairs, 0);
      k.work.assign(kMaxPairs, 0.0);
      k.us.assign(kMaxPairs, 0.0);
    }
    k.used = 0;
    k.seen = 0;
    k.launches = 0;
  }
  p.on = true;
  p.done = false;
  return ASR_OK;
}

extern "C" int asr_prof_end(double* mean_us, long long* launches, double* mean_work,
                            int nkinds) {
  Prof& p = prof();
  p.on = false;
  for (int i = 0; i < ASR_PROF_NKINDS; ++i) {
    KindState& k = p.k[i];
    double tot = 0.0, work = 0.0;
    for (int j = 0; j < k.used; ++j) {
      ASR_CHECK_HIP(hipEventSynchronize(k.ev[2 * j + 1]));
      float ms = 0.f;
      ASR_CHECK_HIP(hipEventElapsedTime(&ms, k.ev[2 * j], k.ev[2 * j + 1]));
      k.us[j] = 1000.0 * ms;
      tot += ms;
      work += k.work[j];
    }
    if (i < nkinds) {
      if (mean_us) mean_us[i] = k.used ? 1000.0 * tot / k.used : 0.0;
      if (launches) launches[i] = k.launches;
      if (mean_work) mean_work[i] = k.used ? work / k.used : 0.0;
    }
  }
  p.done = true;
  return ASR_OK;
}

// Every timed sample of `kind` after asr_prof_end: tag, algorithmic work and
// duration (µs) per sample, up to `max`.  Returns the sample count (which may
// exceed max), or -1 before asr_prof_end / for a bad kind.
extern "C" long long asr_prof_samples(int kind, int* tags, double* work, double* us,
                                      long long max) {
  Prof& p = prof();
  if (!p.done || kind < 0 || kind >= ASR_PROF_NKINDS) return -1;
  const KindState& k = p.k[kind];
  for (long long j = 0; j < k.used && j < max; ++j) {
    if (tags) tags[j] = k.tag[j];
    if (work) work[j] = k.work[j];
    if (us) us[j] = k.us[j];
  }
  return k.used;
}
