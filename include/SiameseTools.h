/* SiameseTools.h -- header-compatible helpers for code built against the siamese.h drop-in.

   Tonk includes SiameseTools.h beside siamese.h (TonkineseTools.h:61) for a handful of helpers
   that are not part of the codec ABI: the PCG generator (SiameseTools.h:79-102 of the
   reference), the microsecond / millisecond clocks (:108-110, SiameseTools.cpp:81-117) and the
   windowed minimum / maximum filter of its bandwidth and time-sync code (:116-236).  This header
   provides the same names, members and results for tonk_amd; the two clocks
   are exported by libtonk_amd.so (tonk_amd/csrc/siamese_tools.cpp).

   Users: TonkineseBandwidth.h:683-700, TonkineseTools.h:140-141 (WindowedMinMax with the two
   compare functors), TonkineseSession/Outgoing/Incoming (GetTimeUsec/GetTimeMsec, PCGRandom). */
#ifndef TONK_AMD_SIAMESE_TOOLS_H
#define TONK_AMD_SIAMESE_TOOLS_H

#include <stdint.h>
#include <string.h>
#include <new>

// Debug checks (active with _DEBUG / DEBUG, as the reference's SIAMESE_DEBUG_ASSERT).
#if defined(_DEBUG) || defined(DEBUG)
#define SIAMESE_DEBUG
#define SIAMESE_DEBUG_BREAK() __builtin_trap()
#define SIAMESE_DEBUG_ASSERT(cond) { if (!(cond)) { SIAMESE_DEBUG_BREAK(); } }
#else
#define SIAMESE_DEBUG_BREAK() do {} while (false);
#define SIAMESE_DEBUG_ASSERT(cond) do {} while (false);
#endif

#define SIAMESE_FORCE_INLINE inline __attribute__((always_inline))

namespace siamese {

/// PCG32 (XSH-RR output, 64-bit LCG state), seeded as the reference seeds it: the stream
/// selector y picks the increment, x offsets the state after one step.
class PCGRandom {
public:
    void Seed(uint64_t y, uint64_t x = 0) {
        Inc = (y << 1u) | 1u;
        State = 0;
        Next();
        State += x;
        Next();
    }

    uint32_t Next() {
        const uint64_t s = State;
        State = s * UINT64_C(6364136223846793005) + Inc;
        const uint32_t mixed = (uint32_t)(((s >> 18) ^ s) >> 27);
        const uint32_t r = (uint32_t)(s >> 59);
        return (mixed >> r) | (mixed << ((32u - r) & 31u));
    }

    uint64_t State = 0, Inc = 0;
};

/// Wall-clock time (gettimeofday) in microseconds and milliseconds.  Exported by libtonk_amd.so.
uint64_t GetTimeUsec();
uint64_t GetTimeMsec();

/// Orderings for WindowedMinMax: "x is at least as good as y".
template <typename T>
struct WindowedMinCompare {
    SIAMESE_FORCE_INLINE bool operator()(const T x, const T y) const { return x <= y; }
};
template <typename T>
struct WindowedMaxCompare {
    SIAMESE_FORCE_INLINE bool operator()(const T x, const T y) const { return x >= y; }
};

/// Running minimum (or maximum) over a sliding time window, kept as the best, second-best and
/// third-best samples of three successive sub-windows (K. Nichols' windowed filter, as used by
/// BBR): O(1) time and space per update.  Samples[0] is the current best.
template <typename T, class CompareT>
class WindowedMinMax {
public:
    typedef uint64_t TimeT;
    CompareT Compare;

    struct Sample {
        T Value;
        TimeT Timestamp;

        explicit Sample(T value = 0, TimeT timestamp = 0) : Value(value), Timestamp(timestamp) {}

        /// More than `timeout` has passed since the sample was taken (wrapping arithmetic).
        inline bool TimeoutExpired(TimeT now, TimeT timeout) { return (TimeT)(now - Timestamp) > timeout; }
    };

    static const unsigned kSampleCount = 3;
    Sample Samples[kSampleCount];

    /// A zero best value means "no sample yet".
    bool IsValid() const { return Samples[0].Value != 0; }
    T GetBest() const { return Samples[0].Value; }

    void Reset(const Sample sample = Sample()) {
        for (unsigned i = 0; i < kSampleCount; ++i) Samples[i] = sample;
    }

    void Update(T value, TimeT timestamp, const TimeT windowLengthTime) {
        const Sample s(value, timestamp);
        Sample& best = Samples[0];
        Sample& second = Samples[1];
        Sample& third = Samples[2];

        // Empty filter, a new overall best, or even the newest kept sample is out of the
        // window: start over from this one.
        if (!IsValid() || Compare(value, best.Value) || third.TimeoutExpired(timestamp, windowLengthTime)) {
            Reset(s);
            return;
        }

        // Keep the sub-window candidates ordered.
        if (Compare(value, second.Value)) {
            second = s;
            third = s;
        } else if (Compare(value, third.Value)) {
            third = s;
        }

        // The best sample left the window: promote the candidates that are still inside it.
        if (best.TimeoutExpired(timestamp, windowLengthTime)) {
            if (second.TimeoutExpired(timestamp, windowLengthTime)) {
                best = third;
                second = s;
            } else {
                best = second;
                second = third;
            }
            third = s;
            return;
        }

        // A quarter window without a better second candidate: refresh it (and the third).
        if (second.Value == best.Value && second.TimeoutExpired(timestamp, windowLengthTime / 4)) {
            second = s;
            third = s;
            return;
        }

        // Half a window without a better third candidate: refresh it.
        if (third.Value == second.Value && third.TimeoutExpired(timestamp, windowLengthTime / 2)) third = s;
    }
};

}  // namespace siamese

#endif  // TONK_AMD_SIAMESE_TOOLS_H
