// prof.h -- optional cycle accounting for control-plane tuning (compile with -DTAMD_PROF).
// Zero cost otherwise.  Used by tests/native/cp_bench.
#pragma once

#ifdef TAMD_PROF
#include <stdint.h>
#include <x86intrin.h>

namespace tamd {
namespace prof {
enum Slot {
    kEncAdd, kEncEncode, kEncAck, kDecAddOrig, kDecAddRec, kDecDecode, kDecAck, kDecIsReady,
    kGenMatrix, kGE, kElim, kLowerTri, kBackSub, kChainFlush, kSymMerge, kFlushAll, kFinish, kRelease,
    kEncDense, kEncLight, kEncEmit, kElimSums, kElimPairs, kElimFold, kEncCauchy, kEncRemove, kElimStart, kLaneRead, kLaneDyn, kCombine, kFoldMerge, kAlloc,
    kX1, kX2, kX3, kX4, kSlots  // kX*: ad-hoc probes
};
extern thread_local uint64_t cycles[kSlots];
extern thread_local uint64_t calls[kSlots];
extern const char* const names[kSlots];
struct Scope {
    Slot s;
    uint64_t t0;
    explicit Scope(Slot slot) : s(slot), t0(__rdtsc()) {}
    ~Scope() { cycles[s] += __rdtsc() - t0; calls[s]++; }
};
}  // namespace prof
}  // namespace tamd
#define TAMD_PROF_CAT2(a, b) a##b
#define TAMD_PROF_CAT(a, b) TAMD_PROF_CAT2(a, b)
#define TAMD_PROF_SCOPE(slot) ::tamd::prof::Scope TAMD_PROF_CAT(tamd_prof_scope_, __LINE__)(::tamd::prof::slot)
#else
#define TAMD_PROF_SCOPE(slot) do {} while (0)
#endif
