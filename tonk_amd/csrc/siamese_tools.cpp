// siamese_tools.cpp -- the two clocks declared by include/SiameseTools.h, exported by
// libtonk_amd.so for code built against the drop-in headers (Tonk calls siamese::GetTimeUsec /
// GetTimeMsec from its session, bandwidth and time-sync code; the reference defines them in
// SiameseTools.cpp:81-117 on gettimeofday).
#include "../../include/SiameseTools.h"

#include <sys/time.h>

namespace siamese {

uint64_t GetTimeUsec() {
    timeval tv;
    gettimeofday(&tv, nullptr);
    return 1000000ull * (uint64_t)tv.tv_sec + (uint64_t)tv.tv_usec;
}

uint64_t GetTimeMsec() { return GetTimeUsec() / 1000u; }

}  // namespace siamese
