// gf256.h -- host-side GF(2^8) field and Siamese coefficient generators for the control plane.
//
// The bulk byte arithmetic never runs on the host: it is emitted as device programs.  The host
// needs only scalar field operations (matrix generation and Gaussian elimination in the
// decoder, coefficient folding in the symbolic row algebra) and the small per-coefficient
// tables that the HIP kernels stage in LDS.
//
// Field: polynomial 0x14D, generator 2 (gf256.cpp:358-403).
#pragma once
#include <stdint.h>

namespace tamd {

struct GF {
    uint8_t mul[256][256];  // mul[y][x] = x * y
    uint8_t div[256][256];  // div[y][x] = x / y  (0 when y == 0, as gf256.cpp:410-442)
    uint8_t inv[256];
    uint8_t sqr[256];
    // Per-coefficient product tables for the device: x * c = T0[x & 7] ^ T1[(x >> 3) & 7] ^
    // T2[x >> 6], each table 8 bytes (T2 uses 4).  Laid out as 6 dwords per coefficient.
    uint32_t perm[256][8];
    bool ready = false;
};

extern GF g_gf;

// Builds the tables and runs the field self-test; returns true on success.  Idempotent.
bool gf_init();

inline uint8_t gf_mul(uint8_t x, uint8_t y) { return g_gf.mul[y][x]; }
inline uint8_t gf_div(uint8_t x, uint8_t y) { return g_gf.div[y][x]; }
inline uint8_t gf_inv(uint8_t x) { return g_gf.inv[x]; }
inline uint8_t gf_sqr(uint8_t x) { return g_gf.sqr[x]; }

// ---- Siamese code parameters (SiameseCommon.h:80-218) ----
static const unsigned kMaxLossRecovery = 255;       // kMaximumLossRecoveryCount
static const unsigned kColumnPeriod    = 0x400000;  // 22-bit packet numbers
static const unsigned kRowPeriod       = 255;
static const unsigned kLanes           = 8;         // kColumnLaneCount
static const unsigned kSums            = 3;         // kColumnSumCount
static const unsigned kPairRate        = 16;        // kPairAddRate
static const unsigned kSubwindow       = 64;        // kSubwindowSize
static const unsigned kCauchyThreshold = 64;        // SIAMESE_CAUCHY_THRESHOLD
static const unsigned kSumResetThreshold = 32;      // SIAMESE_SUM_RESET_THRESHOLD
static const unsigned kCauchyMaxColumns = 64;
static const unsigned kCauchyMaxRows   = 256 - 64;
static const unsigned kMaxPackets      = 16000;     // SIAMESE_MAX_PACKETS
static const unsigned kRemoveThreshold = 2 * kSubwindow; // encoder/decoder removal threshold

inline uint8_t column_value(unsigned column) { return (uint8_t)(3u + (column * 199u) % 253u); }
inline uint8_t row_value(unsigned row) { return (uint8_t)(1u + (row + 1u) % 255u); }

inline unsigned row_opcode(unsigned lane, unsigned row) {
    uint32_t k = lane + (row + 3u) * kLanes;
    k += ~(k << 15);
    k ^= (k >> 10);
    k += (k << 3);
    k ^= (k >> 6);
    k += ~(k << 11);
    k ^= (k >> 16);
    const uint32_t op = k & 63u;
    return op == 0 ? 16u : op;
}

inline uint8_t cauchy_element(unsigned row, unsigned column) {
    return gf_inv((uint8_t)((uint8_t)column ^ (uint8_t)(row + kCauchyMaxColumns)));
}

// Column arithmetic modulo the 22-bit packet-number period (SiameseCommon.h:105-127).
inline bool col_delta_negative(unsigned d) { return d >= kColumnPeriod / 2; }
inline unsigned col_sub(unsigned a, unsigned b) { return (a - b) % kColumnPeriod; }
inline unsigned col_add(unsigned a, unsigned b) { return (a + b) % kColumnPeriod; }
inline unsigned col_inc(unsigned a) { return col_add(a, 1); }

// PCG32 (SiameseTools.h:79-101): drives the LDPC column choice.
struct Pcg32 {
    uint64_t state = 0, inc = 0;
    void seed(uint64_t y, uint64_t x) {
        state = 0;
        inc = (y << 1u) | 1u;
        next();
        state += x;
        next();
    }
    uint32_t next() {
        const uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        const uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
        const uint32_t rot = (uint32_t)(old >> 59);
        return (xs >> rot) | (xs << ((uint32_t)(-(int32_t)rot) & 31u));
    }
};

// x mod d for a divisor fixed over many draws (the LDPC pair columns, `next() % count`): two
// multiplications instead of a division, exact for every 32-bit x and d > 0 (Lemire, Kaser &
// Kurz, "Faster remainder by direct computation", 2019).
struct FastMod {
    uint64_t m;
    uint32_t d;
    explicit FastMod(uint32_t divisor) : m(divisor ? ~0ull / divisor + 1 : 0), d(divisor) {}  // (d = 0: never called)
    uint32_t operator()(uint32_t x) const { return (uint32_t)(((unsigned __int128)(m * x) * d) >> 64); }
};

} // namespace tamd
