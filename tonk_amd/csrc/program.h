// program.h -- the device program format shared by the host control plane (emitter), the HIP
// executor (kernels.hip) and the test-only CPU interpreter (oracle/siamese_oracle.c).
//
// A program is a flat list of independent ops.  Each op owns an accumulator the width of its
// span and runs its instruction list in order:
//
//   ACC   (row, coef, len, a)          acc_a[j] ^= coef * row[j]        for j < len
//   ACC3  (row, c1, c2, len)           acc_0[j] ^= row[j], acc_1[j] ^= c1 * row[j],
//                                      acc_2[j] ^= c2 * row[j]          for j < len
//   STORE (row, len, footer, cap, a)   row[j] = acc_a[j]                for j < len
//                                      row[j] = footer[j - len]         for len <= j < len + F
//                                      row[j] = 0                       for len + F <= j < cap
//   STOREC(row, len, cap, c0, c1, c2)  row[j] = c0*acc_0[j] ^ c1*acc_1[j] ^ c2*acc_2[j] for j < len,
//                                      0 for len <= j < cap       (no FOOTER word follows)
//   CLEAR                              acc_0 = acc_1 = acc_2 = 0
//   ACCR  (mode, p, row0, count, len) + RANGE (stride, col0, cstep)
//         for k < count: row_k = row0 + k*stride (64-B units), col_k = (col0 + k*cstep) mod 2^22
//         LANE3:  acc_0 ^= row_k, acc_1 ^= cx*row_k, acc_2 ^= cx^2*row_k, cx = 3 + (199*col_k mod 253)
//         CAUCHY: acc_0 ^= inv((col_k mod 64) ^ (p + 64)) * row_k
//         CONST:  acc_0 ^= p * row_k
//         MULTI:  + TARGETS (t_0, t_1, t_2), t_a = kind | p << 2 | lo << 10 | hi << 21 (kind 0:
//                 unused): for lo <= k < hi: CAUCHY: acc_a ^= inv((col_k mod 64) ^ (p + 64)) * row_k,
//                                            CONST:  acc_a ^= row_k
//                 (up to three Cauchy / parity rows over overlapping windows: each row of the
//                 run is read once for all of them)
//         DENSE:  + COEFS (row = o bits 0..31, len = o bits 32..47 | rx << 16): o holds the 6-bit
//                 opcode of each lane (bits 6l .. 6l + 5, SiameseCommon.h:160 GetRowOpcode); row k
//                 (lane l = col_k mod 8, opcode b, cx = CX(col_k)) adds
//                 acc_0 ^= (b0 ^ b1*cx ^ b2*cx^2  ^  rx * (b3 ^ b4*cx ^ b5*cx^2)) * row_k
//                 -- a Siamese row's dense part straight from the packets of its sum range: the
//                 lane-sum combination the row reads (SiameseEncoder.cpp:1046-1098), without sums
//                 One target: ACCR w0 bits 24..31 = s > 1 scales every row's coefficient (a decoder's
//                 elimination of received originals from a Siamese row, scaled by its solve).
//                 With p = 2 or 3 (ACCR w0 bits 16..23): p targets, each a COEFS word (cap = its
//                 ADJ words | hi << 16) followed by its ADJ words; target t adds rows k < hi_t
//                 into acc_t -- rows of nested sum ranges, each packet loaded once for all
//         (runs of equally long packets stored at a fixed stride: the window's originals, whose
//         rows sit in a contiguous ring in HBM, become one instruction per run)
//
// An op owns three accumulators; plain combines use acc_0 only, lane running-sum scans use all
// three (sum s of a lane accumulates cx^s * packet, one ACC3 per packet) and a read of a lane's
// sums in a recovery row is one STOREC of the combination the row's opcode selects.
//
// Rows are addressed in 64-byte units from the arena base.  Byte positions are independent in
// GF(2^8) arithmetic, so an op is split into byte slices that the device runs in parallel with
// no synchronisation.  Ops in one launch never read a row another op of the same launch writes
// (the host orders dependent ops into later launches: "levels").
#pragma once
#include <stdint.h>

#define TAMD_ROW_UNIT 64u
/* A work item (one wave) covers one slice of an op: 1536 bytes (16 + 8 B per lane, tamd_exec24,
   the default: a packet row of up to 1536 bytes is one item) or 1024 bytes (16 B per lane,
   tamd_exec16; TONK_AMD_SLICE=1024). */
#define TAMD_SLICE_BYTES 1024u
#define TAMD_SLICE_BYTES_X 1536u

enum tamd_instr_kind {
    TAMD_I_ACC    = 1,
    TAMD_I_STORE  = 2,
    TAMD_I_FOOTER = 3,  // payload word that always follows a STORE
    TAMD_I_CLEAR  = 4,
    TAMD_I_ACC3   = 5,
    TAMD_I_STOREC = 6,  // w0 = kind | c0 << 8 | c1 << 16 | c2 << 24
    TAMD_I_ACCR   = 7,  // w0 = kind | mode << 8 | p << 16 (| s << 24: CAUCHY scale); row = row0, len, cap = count
    TAMD_I_RANGE  = 8,  // payload word after ACCR: row = stride (units), len = col0, cap = cstep
    TAMD_I_TARGETS = 9, // payload word after the RANGE of a MULTI ACCR: row, len, cap = t_0, t_1, t_2
    TAMD_I_COEFS  = 10, // payload word after the RANGE of a DENSE ACCR: lane opcodes and rx; cap =
                        // the number of ADJ words that follow it
    TAMD_I_ADJ    = 11, // payload of a DENSE ACCR: four coefficient additions, each dword
                        // idx << 16 | delta << 8 (| kind in dword 0): row idx of the run gets
                        // coefficient ^ delta (delta 0: an empty entry)
};

enum tamd_range_mode {
    TAMD_R_LANE3  = 1,
    TAMD_R_CAUCHY = 2,
    TAMD_R_CONST  = 3,
    TAMD_R_MULTI  = 4,
    TAMD_R_DENSE  = 5,
};

// Ops of a level are grouped into classes: class 0 holds the long pure combines (ACC into acc_0,
// CONST/CAUCHY runs, one final STORE), which a whole workgroup executes together (each wave
// takes every fourth batch of rows, partial sums reduced through LDS); classes 1..4 hold the
// other ops by cost, most expensive first, each run by one wave.  Long chains start first.
#define TAMD_COST_CLASSES 5u

#define TAMD_COLUMN_PERIOD 0x400000u  /* packet numbers are 22-bit (SiameseCommon.h:105) */

// 16-byte instruction word.
typedef struct tamd_instr {
    uint32_t w0;   // kind | (coef, c1 or footer_len) << 8 | (accumulator or c2) << 16
    uint32_t row;  // row offset in TAMD_ROW_UNIT units (ACC/STORE); footer bytes 0..3 (FOOTER)
    uint32_t len;  // byte length (ACC/STORE);                      footer bytes 4..7 (FOOTER)
    uint32_t cap;  // zero-fill end (STORE)
} tamd_instr;

// 16-byte op header.
typedef struct tamd_op {
    uint32_t first;  // index of first instruction
    uint32_t count;  // instruction count
    uint32_t span;   // bytes covered by the op's accumulator
    uint32_t full;   // min(span, every length the op's instructions use): slices below it need no
                     // per-lane length handling (the executor's fast path)
} tamd_op;

// The item segments of one executor launch (level pipelining: one level each of up to
// TAMD_MAX_SEGMENTS programs; items are numbered across the segments in order).  Passed by
// value; byte offsets into the device's program memory.
#define TAMD_MAX_SEGMENTS 6
typedef struct tamd_segment {
    uint32_t ops, instrs, items;  // offsets of the program's ops / instructions / this level's items
    uint32_t count;               // items ((op index, slice) uint32 pairs)
    uint32_t cls[5];              // items per cost class (TAMD_COST_CLASSES), in that order
} tamd_segment;
typedef struct tamd_segments {
    tamd_segment s[TAMD_MAX_SEGMENTS];
    uint32_t n;
    uint32_t flags;  // bit 0: items are taken class by class across the segments (the launch's
                     // longest first), else segment by segment
} tamd_segments;

static inline uint32_t tamd_w0(uint32_t kind, uint32_t arg, uint32_t arg2 = 0) {
    return kind | (arg << 8) | (arg2 << 16);
}
