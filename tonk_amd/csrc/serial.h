// serial.h -- Siamese wire formats (SiameseSerializers.h), restated for the control plane.
//
//   packet number  : 1-3 bytes, header form (front) and footer form (back)        :330-448
//   packet count   : 1-2 bytes, footer form                                        :510-551
//   packet length  : 1-4 byte varint prefixed to every original row                :566-640
//   recovery footer: [Row, LDPCCount] ColumnStart SumCount-1, parsed from the end  :736-800
//   NACK loss range: 1-7 bytes                                                     :861-994
#pragma once
#include <stdint.h>

namespace tamd {

struct RecoveryMeta {
    unsigned Row = 0;          // recovery row number (0 = parity/single)
    unsigned ColumnStart = 0;  // first column of the sum
    unsigned SumCount = 0;     // columns in the sum
    unsigned LDPCCount = 0;    // columns in the LDPC / Cauchy range (right-aligned in the sum)
};

static const unsigned kMaxLengthFieldBytes = 4;
static const unsigned kMaxRecoveryFooterBytes = 8;
static const unsigned kMaxLossRangeBytes = 7;

inline unsigned put_pnum_header(unsigned v, uint8_t* b) {
    if (v <= 0x7f) { b[0] = (uint8_t)v; return 1; }
    if (v <= 0x3fff) { b[0] = (uint8_t)(0x80 | (v >> 8)); b[1] = (uint8_t)v; return 2; }
    b[0] = (uint8_t)(0xC0 | (v >> 16)); b[1] = (uint8_t)(v >> 8); b[2] = (uint8_t)v; return 3;
}

inline int get_pnum_header(const uint8_t* b, int avail, unsigned& v) {
    if (!b || avail < 1) return -1;
    const int n = b[0] >> 6;
    if (n <= 1) { v = b[0]; return 1; }
    if (avail < n) return -1;
    if (n == 2) v = (((unsigned)b[0] << 8) | b[1]) & 0x3fff;
    else        v = (((unsigned)b[0] << 16) | ((unsigned)b[1] << 8) | b[2]) & 0x3fffff;
    return n;
}

inline unsigned put_pnum_footer(unsigned v, uint8_t* b) {
    if (v <= 0x7f) { b[0] = (uint8_t)v; return 1; }
    if (v <= 0x3fff) { b[0] = (uint8_t)v; b[1] = (uint8_t)(0x80 | (v >> 8)); return 2; }
    b[0] = (uint8_t)v; b[1] = (uint8_t)(v >> 8); b[2] = (uint8_t)(0xC0 | (v >> 16)); return 3;
}

inline int get_pnum_footer(const uint8_t* b, int avail, unsigned& v) {
    if (!b || avail < 1) return -1;
    const uint8_t* p = b + avail - 1;
    const int n = p[0] >> 6;
    if (n <= 1) { v = p[0]; return 1; }
    if (avail < n) return -1;
    if (n == 2) v = (((unsigned)p[0] << 8) | p[-1]) & 0x3fff;
    else        v = (((unsigned)p[0] << 16) | ((unsigned)p[-1] << 8) | p[-2]) & 0x3fffff;
    return n;
}

inline unsigned put_count_footer(unsigned v, uint8_t* b) {
    if (v <= 127) { b[0] = (uint8_t)v; return 1; }
    b[0] = (uint8_t)v; b[1] = (uint8_t)(0x80 | (v >> 8)); return 2;
}

inline int get_count_footer(const uint8_t* b, unsigned avail, unsigned& v) {
    if (avail < 1) return -1;
    const uint8_t* p = b + avail - 1;
    if ((p[0] & 0x80) == 0) { v = p[0]; return 1; }
    if (avail < 2) return -1;
    v = (((unsigned)p[0] << 8) | p[-1]) & 0x7fff;
    return 2;
}

inline unsigned put_length_header(unsigned len, uint8_t* b) {
    if (len <= 0x7f) { b[0] = (uint8_t)len; return 1; }
    if (len <= 0x3fff) { b[0] = (uint8_t)(0x80 | (len >> 8)); b[1] = (uint8_t)len; return 2; }
    if (len <= 0x1fffff) {
        b[0] = (uint8_t)(0xC0 | (len >> 16)); b[1] = (uint8_t)(len >> 8); b[2] = (uint8_t)len; return 3;
    }
    b[0] = (uint8_t)(0xE0 | (len >> 24)); b[1] = (uint8_t)(len >> 16);
    b[2] = (uint8_t)(len >> 8); b[3] = (uint8_t)len; return 4;
}

inline unsigned length_header_bytes(unsigned len) {
    return len <= 0x7f ? 1 : len <= 0x3fff ? 2 : len <= 0x1fffff ? 3 : 4;
}

inline int get_length_header(const uint8_t* b, unsigned avail, unsigned& len) {
    if (!b || avail < 1) return -1;
    const int n = b[0] >> 6;
    if (n <= 1) { len = b[0]; return 1; }
    if (n == 2) {
        if (avail < 2) return -1;
        len = (((unsigned)b[0] << 8) | b[1]) & 0x3fff; return 2;
    }
    if ((b[0] & 0xE0) == 0xC0) {
        if (avail < 3) return -1;
        len = (((unsigned)b[0] << 16) | ((unsigned)b[1] << 8) | b[2]) & 0x1fffff; return 3;
    }
    if (avail < 4) return -1;
    len = (((unsigned)b[0] << 24) | ((unsigned)b[1] << 16) | ((unsigned)b[2] << 8) | b[3]) & 0x1fffffff;
    return 4;
}

inline unsigned put_recovery_footer(const RecoveryMeta& m, uint8_t* b) {
    unsigned n = 0;
    if (m.SumCount > 1) {
        b[n++] = (uint8_t)m.Row;
        n += put_count_footer(m.LDPCCount, b + n);
    }
    n += put_pnum_footer(m.ColumnStart, b + n);
    n += put_count_footer(m.SumCount - 1, b + n);
    return n;
}

inline int get_recovery_footer(const uint8_t* b, unsigned bytes, RecoveryMeta& m) {
    unsigned avail = bytes;
    int f = get_count_footer(b, avail, m.SumCount);
    if (f < 0) return -1;
    avail -= (unsigned)f;
    m.SumCount++;
    f = get_pnum_footer(b, (int)avail, m.ColumnStart);
    if (f < 0) return -1;
    avail -= (unsigned)f;
    if (m.SumCount <= 1) {
        m.LDPCCount = 1;
        m.Row = 0;
    } else {
        f = get_count_footer(b, avail, m.LDPCCount);
        if (f < 0) return -1;
        avail -= (unsigned)f;
        if (m.SumCount < m.LDPCCount) return -1;
        if (avail < 1) return -1;
        m.Row = b[--avail];
    }
    return (int)(bytes - avail);
}

inline unsigned put_nack_range(unsigned rel, unsigned lossM1, uint8_t* b) {
    unsigned b0 = lossM1 <= 2 ? lossM1 : 3;
    b0 |= rel << 3;
    unsigned n = 1;
    if (rel >= (1u << 5)) {
        unsigned b1 = rel >> 5;
        if (rel >= (1u << 12)) {
            unsigned b2 = rel >> 12;
            if (rel >= (1u << 19)) { b[3] = (uint8_t)(rel >> 19); b2 |= 0x80; ++n; }
            b[2] = (uint8_t)b2;
            b1 |= 0x80;
            ++n;
        }
        b[1] = (uint8_t)b1;
        b0 |= 4;
        ++n;
    }
    b[0] = (uint8_t)b0;
    if (lossM1 >= 3) {
        uint8_t* q = b + n;
        const unsigned c = lossM1 - 3;
        unsigned c1 = c;
        if (c >= (1u << 7)) {
            unsigned c2 = c >> 7;
            if (c >= (1u << 14)) { q[2] = (uint8_t)(c >> 14); c2 |= 0x80; ++n; }
            q[1] = (uint8_t)c2;
            c1 |= 0x80;
            ++n;
        }
        q[0] = (uint8_t)c1;
        ++n;
    }
    return n;
}

// Requires 7 readable bytes at b (callers pad), like the reference (:934-941).
inline int get_nack_range(const uint8_t* b, unsigned avail, unsigned& rel, unsigned& lossM1) {
    if (!b || avail < kMaxLossRangeBytes) return -1;
    const unsigned b0 = b[0];
    unsigned lc = b0 & 3, rs = b0 >> 3, n = 1;
    if (b0 & 4) {
        ++n;
        const unsigned b1 = b[1];
        rs |= (b1 & 0x7f) << 5;
        if (b1 & 0x80) {
            ++n;
            const unsigned b2 = b[2];
            rs |= (b2 & 0x7f) << 12;
            if (b2 & 0x80) { ++n; rs |= (unsigned)b[3] << 19; }
        }
    }
    if (lc == 3) {
        const uint8_t* q = b + n;
        lc += q[0] & 0x7f;
        if (q[0] & 0x80) {
            lc += (q[1] & 0x7fu) << 7;
            if (q[1] & 0x80) { lc += (unsigned)q[2] << 14; ++n; }
            ++n;
        }
        ++n;
    }
    rel = rs;
    lossM1 = lc;
    return (int)n;
}

} // namespace tamd
