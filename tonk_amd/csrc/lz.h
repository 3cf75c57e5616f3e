// lz.h -- layouts shared by the compression kernel (lz.hip) and its host side (compress.cpp):
// job and message descriptors, the FSE table blob, and the zstd length-code tables
// (RFC 8878 s3.1.1.3.2.1.1, the literal-length and match-length codes; offsets are coded as
// Offset_Value = offset + 3, code = highbit(Offset_Value), value bits = the rest).
#pragma once
#include <math.h>
#include <stdint.h>

#define TAMD_LZ_MAX_MESSAGE 1536u  // messages up to this size are compressed entirely in LDS
#define TAMD_LZ_WAVES 8u           // jobs (waves) per workgroup of tamd_lz_compress: 2 waves per SIMD
#define TAMD_LZ_MAX_BLOCK 131071u  // larger ones (up to zstd's block limit, 128 KB) use global scratch
#define TAMD_LZ_NO_SCRATCH 0xffffffffu
#define TAMD_LZ_WINDOW 32768u      // history bytes inserted into a job's hash table
#define TAMD_LZ_RING 65536u        // per-compressor device ring of the stream's bytes (the drop-in)
#define TAMD_LZ_MIRROR 64u         // the ring's first bytes repeated after it (wide loads at its end)
#define TAMD_LZ_PHASES 8u          // (profiling: 100 MHz ticks per job and phase, TONK_AMD_LZ_PROF)

// The drop-in's staging: message bytes land in their compressor's ring (one workgroup each).
typedef struct tamd_lz_scatter {
    uint8_t* ring;
    uint32_t slot, bytes, src, pad;
} tamd_lz_scatter;

// A run of consecutive messages of one stream.  `buf` holds the stream's bytes at their linear
// positions (masked by `mask`: a power-of-two ring, or ~0 for a linear array).
typedef struct tamd_lz_job {
    const uint8_t* buf;
    uint32_t mask, first, count, pad;
} tamd_lz_job;

// One message: linear position and length, the start of the bytes the decompressor holds when it
// decodes it (previous history segment start), its output slot, and for a message above
// TAMD_LZ_MAX_MESSAGE the byte offset of its scratch area (tamd_lz_scratch_bytes, 16-byte
// aligned; TAMD_LZ_NO_SCRATCH: none, the message is stored uncompressed).
typedef struct tamd_lz_msg {
    uint32_t pos, len, win, out, cap, scratch, pad[2];
} tamd_lz_msg;

// Sequences of a message of n bytes: at most n / 4 (every match is at least 4 bytes).
static inline
#ifdef __HIPCC__
__host__ __device__
#endif
uint32_t tamd_lz_big_seqs(uint32_t n) { return n / 4u + 1u; }
// Scratch of a message above TAMD_LZ_MAX_MESSAGE (lz.hip lz_message<true>): sequences and offsets
// (2 x S words), the bit stream ((n + 64) / 4 + 4 words) and three chains of state updates
// (3 x S halfwords).
static inline
#ifdef __HIPCC__
__host__ __device__
#endif
uint32_t tamd_lz_scratch_bytes(uint32_t n) {
    const uint32_t S = tamd_lz_big_seqs(n);
    return (8u * S + 4u * ((n + 64u) / 4u + 4u) + 6u * S + 15u) & ~15u;
}

// FSE tables of the predefined distributions, one blob:
//   *_ENC[symbol][next_state] = the state of `symbol` whose bit range holds next_state
//   *_DEC[state] = {nbBits, newState} of the decoding table (FSE_buildDTable's layout)
#define TAMD_FSE_LL_ENC 0u
#define TAMD_FSE_ML_ENC (TAMD_FSE_LL_ENC + 36u * 64u)
#define TAMD_FSE_OF_ENC (TAMD_FSE_ML_ENC + 53u * 64u)
#define TAMD_FSE_LL_DEC (TAMD_FSE_OF_ENC + 29u * 32u)
#define TAMD_FSE_ML_DEC (TAMD_FSE_LL_DEC + 64u * 2u)
#define TAMD_FSE_OF_DEC (TAMD_FSE_ML_DEC + 64u * 2u)
// The same encoder maps with the decoding info folded in, one 16-bit word per (symbol, next
// state): state | nbBits << 6 | (next state - base) << 10 (the kernel's chains read only these).
#define TAMD_FSE_E16 (TAMD_FSE_OF_DEC + 32u * 2u)
#define TAMD_FSE_LL_E16 0u  // (word offsets inside the E16 section)
#define TAMD_FSE_ML_E16 (36u * 64u)
#define TAMD_FSE_OF_E16 (TAMD_FSE_ML_E16 + 53u * 64u)
#define TAMD_FSE_E16_WORDS (TAMD_FSE_OF_E16 + 29u * 32u)
// Symbol costs in 1/16 bit for choosing each block's table (tamd_seq_choose): the predefined
// distributions' per symbol (64 bytes per table: LL, ML, OF; 0 past the last symbol), and a
// block-fitted table's by normalized count 0..32.
#define TAMD_FSE_PCOST (TAMD_FSE_E16 + 2u * TAMD_FSE_E16_WORDS)
#define TAMD_FSE_FCOST (TAMD_FSE_PCOST + 3u * 64u)
#define TAMD_FSE_FLAGS (TAMD_FSE_FCOST + 63u)  // (an unused cost slot)
#define TAMD_FSE_PREDEFINED_ONLY 1u              // flag: every block keeps the predefined tables
#define TAMD_FSE_BYTES (TAMD_FSE_FCOST + 64u)

#ifdef __HIPCC__
#define TAMD_HD __host__ __device__
#else
#define TAMD_HD
#endif

// literal length codes 16..24 have the irregular bases; from 25 on, base 2^(code-19)
TAMD_HD static inline uint32_t tamd_ll_bits(uint32_t code) {
    if (code < 16) return 0;
    if (code < 20) return 1;
    if (code < 22) return 2;
    if (code < 24) return 3;
    if (code == 24) return 4;
    return code - 19;
}
TAMD_HD static inline uint32_t tamd_ll_base(uint32_t code) {
    if (code < 16) return code;
    if (code < 20) return 16 + 2 * (code - 16);
    if (code < 22) return 24 + 4 * (code - 20);
    if (code < 24) return 32 + 8 * (code - 22);
    if (code == 24) return 48;
    return 1u << (code - 19);
}
// match length codes: 0..31 are lengths 3..34; 32..42 irregular; from 43 on, base 2^(code-36)+3
TAMD_HD static inline uint32_t tamd_ml_bits(uint32_t code) {
    if (code < 32) return 0;
    if (code < 36) return 1;
    if (code < 38) return 2;
    if (code < 40) return 3;
    if (code < 42) return 4;
    if (code == 42) return 5;
    return code - 36;
}
TAMD_HD static inline uint32_t tamd_ml_base(uint32_t code) {
    if (code < 32) return code + 3;
    if (code < 36) return 35 + 2 * (code - 32);
    if (code < 38) return 43 + 4 * (code - 36);
    if (code < 40) return 51 + 8 * (code - 38);
    if (code < 42) return 67 + 16 * (code - 40);
    if (code == 42) return 99;
    return (1u << (code - 36)) + 3;
}

// Code of a literal length / match length (the inverse of the tables above).
TAMD_HD static inline uint32_t tamd_ll_code(uint32_t ll) {
    if (ll < 16) return ll;
    if (ll < 24) return 16 + ((ll - 16) >> 1);
    if (ll < 32) return 20 + ((ll - 24) >> 2);
    if (ll < 48) return 22 + ((ll - 32) >> 3);
    if (ll < 64) return 24;
    return 19 + (31 - (uint32_t)__builtin_clz(ll));  // 64-127: 25, 128-255: 26, ...
}
TAMD_HD static inline uint32_t tamd_ml_code(uint32_t ml) {  // ml >= 3
    if (ml < 35) return ml - 3;
    if (ml < 43) return 32 + ((ml - 35) >> 1);
    if (ml < 51) return 36 + ((ml - 43) >> 2);
    if (ml < 67) return 38 + ((ml - 51) >> 3);
    if (ml < 99) return 40 + ((ml - 67) >> 4);
    if (ml < 131) return 42;
    return 36 + (31 - (uint32_t)__builtin_clz(ml - 3));  // 131-258: 43, 259-514: 44, ...
}

// Literals section header of raw literals (RFC 8878 s3.1.1.3.1.1): 1, 2 or 3 bytes, packed
// little-endian into a word (*len bytes).
TAMD_HD static inline uint32_t tamd_lits_header_word(uint32_t lits, uint32_t* len) {
    if (lits < 32) {
        *len = 1;
        return lits << 3;
    }
    if (lits < 4096) {
        *len = 2;
        return 0x04u | ((lits & 15u) << 4) | ((lits >> 4) << 8);
    }
    *len = 3;
    return 0x0cu | ((lits & 15u) << 4) | (((lits >> 4) & 0xffu) << 8) | ((lits >> 12) << 16);
}

// Sequences section header (s3.1.1.3.2.1): the count, then the modes byte (0: the predefined
// distributions for all three codes) when there are sequences; packed like the above.
TAMD_HD static inline uint32_t tamd_seq_header_word(uint32_t n, uint32_t* len) {
    if (n == 0) {
        *len = 1;
        return 0;
    }
    if (n < 128) {
        *len = 2;
        return n;
    }
    if (n < 0x7f00) {
        *len = 3;
        return (0x80u + (n >> 8)) | ((n & 0xffu) << 8);
    }
    *len = 4;
    return 0xffu | (((n - 0x7f00u) & 0xffu) << 8) | (((n - 0x7f00u) >> 8) << 16);
}

TAMD_HD static inline uint32_t tamd_lits_header(uint32_t lits, uint8_t* h) {
    uint32_t len = 0;
    const uint32_t w = tamd_lits_header_word(lits, &len);
    for (uint32_t k = 0; k < len; ++k) h[k] = (uint8_t)(w >> (8 * k));
    return len;
}

TAMD_HD static inline uint32_t tamd_seq_header(uint32_t n, uint8_t* h) {
    uint32_t len = 0;
    const uint32_t w = tamd_seq_header_word(n, &len);
    for (uint32_t k = 0; k < len; ++k) h[k] = (uint8_t)(w >> (8 * k));
    return len;
}

// The sequences' bit stream (s3.1.1.3.2.2 / 4.1): written forward here, read backward by the
// decoder.  The decoder reads the initial LL, OF, ML states, then per sequence the offset, match
// length and literal length value bits followed (except after the last sequence) by the LL, ML,
// OF state updates; so the writer starts from the last sequence and emits everything in the
// reverse order.  Sequence k: seq_lo[k] = literal length | match length << 16, seq_off[k] =
// offset (no repeat codes: Offset_Value = offset + 3).  Returns the bytes written (end mark
// included), 0 when they would exceed cap.
TAMD_HD static inline uint32_t tamd_fse_sequences(const uint32_t* seq_lo, const uint32_t* seq_off, uint32_t nseq,
                                                 const uint8_t* tabs, uint8_t* out, uint32_t cap) {
    uint64_t acc = 0;
    uint32_t nbits = 0, pos = 0;
    bool over = false;
    auto add = [&](uint32_t v, uint32_t bits) {
        if (!bits) return;
        acc |= (uint64_t)(v & ((1u << bits) - 1u)) << nbits;
        nbits += bits;
        while (nbits >= 8) {
            if (pos < cap) out[pos] = (uint8_t)acc;
            else over = true;
            ++pos;
            acc >>= 8;
            nbits -= 8;
        }
    };
    const uint8_t* ll_enc = tabs + TAMD_FSE_LL_ENC;
    const uint8_t* ml_enc = tabs + TAMD_FSE_ML_ENC;
    const uint8_t* of_enc = tabs + TAMD_FSE_OF_ENC;
    const uint8_t* ll_dec = tabs + TAMD_FSE_LL_DEC;
    const uint8_t* ml_dec = tabs + TAMD_FSE_ML_DEC;
    const uint8_t* of_dec = tabs + TAMD_FSE_OF_DEC;
    uint32_t s = nseq - 1;
    uint32_t ll = seq_lo[s] & 0xffffu, ml = seq_lo[s] >> 16, off = seq_off[s] + 3u;
    uint32_t llc = tamd_ll_code(ll), mlc = tamd_ml_code(ml), ofc = 31u - (uint32_t)__builtin_clz(off);
    // any state of the symbol can start: take the one whose range holds next-state 0
    uint32_t st_ll = ll_enc[llc * 64], st_ml = ml_enc[mlc * 64], st_of = of_enc[ofc * 32];
    add(ll - tamd_ll_base(llc), tamd_ll_bits(llc));
    add(ml - tamd_ml_base(mlc), tamd_ml_bits(mlc));
    add(off, ofc);
    while (s-- > 0) {
        ll = seq_lo[s] & 0xffffu;
        ml = seq_lo[s] >> 16;
        off = seq_off[s] + 3u;
        llc = tamd_ll_code(ll);
        mlc = tamd_ml_code(ml);
        ofc = 31u - (uint32_t)__builtin_clz(off);
        // into the states of sequence s + 1: offsets, match lengths, literal lengths
        uint32_t u = of_enc[ofc * 32 + st_of];
        add(st_of - of_dec[2 * u + 1], of_dec[2 * u]);
        st_of = u;
        u = ml_enc[mlc * 64 + st_ml];
        add(st_ml - ml_dec[2 * u + 1], ml_dec[2 * u]);
        st_ml = u;
        u = ll_enc[llc * 64 + st_ll];
        add(st_ll - ll_dec[2 * u + 1], ll_dec[2 * u]);
        st_ll = u;
        add(ll - tamd_ll_base(llc), tamd_ll_bits(llc));
        add(ml - tamd_ml_base(mlc), tamd_ml_bits(mlc));
        add(off, ofc);
    }
    add(st_ml, 6);  // the initial states, read first by the decoder: LL, OF, ML
    add(st_of, 5);
    add(st_ll, 6);
    add(1, 1);  // end mark
    if (nbits) add(0, 8 - nbits);
    return over ? 0 : pos;
}

// ---- Block-fitted sequence tables (RFC 8878 s3.1.1.3.2.1.2: RLE_Mode, FSE_Compressed_Mode) -----
// A block may replace each of the three predefined distributions by one fitted to its own codes:
// RLE (every sequence has the same code: one byte, no state bits) or an FSE table described in
// the block (s4.1.1, as zstd's FSE_readNCount reads it, entropy_common.c:61-155), which the
// decoder builds as ZSTD_buildFSETable does (zstd_decompress.c:804-863, the spread of
// tamd_build_fse).  Fitted tables here have accuracy log 5 (32 states, the format's minimum):
// on Tonk-like messages (tens of sequences per block) a finer table never paid for its longer
// description.  No table is ever "repeat" mode, so blocks still carry no entropy state.
#define TAMD_FIT_LOG 5u
#define TAMD_FIT_SIZE 32u
#define TAMD_FIT_STEP 23u      // (32 >> 1) + (32 >> 3) + 3, FSE_TABLESTEP
#define TAMD_FIT_STEP_INV 7u   // 23 * 7 = 1 (mod 32): the spread slot of state u is (u * 7) & 31
#define TAMD_MODE_PREDEF 0u
#define TAMD_MODE_RLE 1u
#define TAMD_MODE_FSE 2u
#define TAMD_FIT_DESC 48u      // description bytes per table (a 53-symbol table needs at most 45)
#define TAMD_FIT_MIN_SEQS 8u   // fewer sequences: no fitted table (its description never pays)

// Normalized count of a symbol seen `count` of `total` times: the nearest share of the 32 states,
// at least one for a present symbol.  The sum is brought to exactly 32 on the largest share
// (lowest symbol on ties), which must stay >= 1 (else no fitted table).
TAMD_HD static inline uint32_t tamd_fit_norm(uint32_t count, uint32_t total) {
    if (!count) return 0;
    const uint32_t n = (2u * TAMD_FIT_SIZE * count + total) / (2u * total);
    return n ? n : 1u;
}

// One symbol's field in the table description (s4.1.1): the value count + 1 in a width set by
// the states not yet given out ("remaining" = 33 - cum, cum = the counts of the symbols before
// it); a zero count is followed by 2-bit repeat flags for the zero counts after it (3 = three
// more and continue).  A zero inside such a run writes nothing itself.  `lead` = first symbol or
// the previous one's count was not zero; `zeros_after` = zero counts following a zero.  Returns
// the width in bits (<= 44) and the bits in *v (first bit = least significant).
TAMD_HD static inline uint32_t tamd_ncount_item(uint32_t n, uint32_t cum, bool lead, uint32_t zeros_after,
                                               uint64_t* v) {
    *v = 0;
    if (n == 0 && !lead) return 0;
    const uint32_t R = TAMD_FIT_SIZE + 1u - cum;
    const uint32_t hb = 31u - (uint32_t)__builtin_clz(R);
    const uint32_t T = 1u << hb, nb = hb + 1u, mx = 2u * T - 1u - R;
    uint32_t x = n + 1u;
    if (x >= T) x += mx;
    uint32_t w = nb - (x < mx ? 1u : 0u);
    uint64_t val = x;
    if (n == 0) {
        const uint32_t q = zeros_after / 3u;
        const uint64_t flags = ((1ull << (2u * q)) - 1ull) | ((uint64_t)(zeros_after % 3u) << (2u * q));
        val |= flags << w;
        w += 2u * q + 2u;
    }
    *v = val;
    return w;
}

// The encoder's view of a fitted table (FSE_buildCTable_wksp, fse_compress.c:85-170, restated):
// cum[s] = states of the symbols before s; state[cum[s] + k] = the k-th state (ascending) that
// decodes s -- the one the decoder reaches with next-state value norm[s] + k.
TAMD_HD static inline void tamd_fit_states(const uint8_t* norm, uint32_t nsym, uint8_t* cum, uint8_t* state) {
    uint8_t sym[TAMD_FIT_SIZE];
    uint8_t rank[64];
    uint32_t c = 0, pos = 0;
    for (uint32_t s = 0; s < nsym; ++s) {
        cum[s] = (uint8_t)c;
        rank[s] = 0;
        c += norm[s];
        for (uint32_t i = 0; i < norm[s]; ++i) {
            sym[pos] = (uint8_t)s;
            pos = (pos + TAMD_FIT_STEP) & (TAMD_FIT_SIZE - 1u);
        }
    }
    for (uint32_t u = 0; u < TAMD_FIT_SIZE; ++u) {
        const uint32_t s = sym[u];
        state[cum[s] + rank[s]++] = (uint8_t)u;
    }
}

// One step of a fitted table's state chain (FSE_encodeSymbol): the decoder must reach state `st`
// after the symbol (norm n, cum c); returns the state that decodes it, *upd = the bits the decoder
// reads to get from there to `st` | their number << 8.
// (the most bits a step out of one of the symbol's states reads: the accuracy log for a single
// state, else log - highbit(n - 1); a state value S below n << mbo reads one bit fewer)
TAMD_HD static inline uint32_t tamd_fit_mbo(uint32_t n) {
    return n > 1u ? TAMD_FIT_LOG - (31u - (uint32_t)__builtin_clz(n - 1u)) : TAMD_FIT_LOG;
}
TAMD_HD static inline uint32_t tamd_fit_step_m(uint32_t n, uint32_t c, uint32_t mbo, const uint8_t* state, uint32_t st,
                                              uint32_t* upd) {
    const uint32_t S = TAMD_FIT_SIZE + st;
    const uint32_t nb = S >= (n << mbo) ? mbo : mbo - 1u;
    *upd = (S & ((1u << nb) - 1u)) | (nb << 8);
    return state[c + (S >> nb) - n];
}
TAMD_HD static inline uint32_t tamd_fit_step(uint32_t n, uint32_t c, const uint8_t* state, uint32_t st, uint32_t* upd) {
    return tamd_fit_step_m(n, c, tamd_fit_mbo(n), state, st, upd);
}

// A block's three tables (index 0 literal lengths, 1 match lengths, 2 offsets, as the codes are
// packed: LL | ML << 8 | OF << 16).
typedef struct tamd_seq_tables {
    uint32_t mode[3];       // TAMD_MODE_*
    uint32_t desc_len[3];   // description bytes (RLE: 1, FSE: the NCount bytes)
    uint8_t desc[3][TAMD_FIT_DESC];
    uint8_t norm[3][64], cum[3][64], state[3][TAMD_FIT_SIZE];
} tamd_seq_tables;

// Choose each table for the codes of a block (sequential; the kernel computes the same choice a
// lane per symbol): the cheapest of the predefined distribution, RLE when one code is used, and a
// fitted table, by costs in 1/16 bit from the blob (state bits of every sequence + the initial
// state + the description).  Returns the descriptions' total bytes.
TAMD_HD static inline uint32_t tamd_seq_choose(const uint32_t* codes, uint32_t nseq, const uint8_t* blob,
                                              tamd_seq_tables* t) {
    uint32_t total = 0;
    for (uint32_t k = 0; k < 3; ++k) {
        const uint32_t nsym = k == 0 ? 36u : k == 1 ? 53u : 32u, plog = k == 2 ? 5u : 6u;
        uint32_t count[64];
        for (uint32_t s = 0; s < 64; ++s) count[s] = 0;
        for (uint32_t q = 0; q < nseq; ++q) ++count[(codes[q] >> (8u * k)) & 0xffu];
        uint32_t present = 0, last = 0, only = 0, sum = 0, big = 0;
        uint64_t pre = 16u * plog;
        for (uint32_t s = 0; s < nsym; ++s) {
            pre += (uint64_t)count[s] * blob[TAMD_FSE_PCOST + 64u * k + s];
            const uint32_t n = tamd_fit_norm(count[s], nseq);
            t->norm[k][s] = (uint8_t)n;
            sum += n;
            if (n > t->norm[k][big]) big = s;
            if (count[s]) {
                ++present;
                last = s;
                only = s;
            }
        }
        t->mode[k] = TAMD_MODE_PREDEF;
        t->desc_len[k] = 0;
        uint64_t best = pre;
        if (present == 1 && 16u * 8u < best) {
            t->mode[k] = TAMD_MODE_RLE;
            t->desc_len[k] = 1;
            t->desc[k][0] = (uint8_t)only;
            best = 16u * 8u;
        }
        const int32_t fixed = (int32_t)t->norm[k][big] + (int32_t)TAMD_FIT_SIZE - (int32_t)sum;
        if (present >= 2 && present <= TAMD_FIT_SIZE && nseq >= TAMD_FIT_MIN_SEQS && fixed >= 1) {
            t->norm[k][big] = (uint8_t)fixed;
            uint64_t fit = 0, bits = 4;  // (4 bits: accuracy log - 5 = 0)
            uint8_t d[TAMD_FIT_DESC];
            for (uint32_t i = 0; i < TAMD_FIT_DESC; ++i) d[i] = 0;
            uint32_t cum = 0;
            for (uint32_t s = 0; s <= last; ++s) {
                const uint32_t n = t->norm[k][s];
                fit += (uint64_t)count[s] * blob[TAMD_FSE_FCOST + n];
                uint32_t z = 0;
                if (n == 0)
                    while (s + 1u + z <= last && t->norm[k][s + 1u + z] == 0) ++z;
                uint64_t v;
                const uint32_t w = tamd_ncount_item(n, cum, s == 0 || t->norm[k][s - 1] != 0, z, &v);
                for (uint32_t b = 0; b < w; ++b)
                    if ((v >> b) & 1u) d[(bits + b) / 8u] |= (uint8_t)(1u << ((bits + b) % 8u));
                bits += w;
                cum += n;
            }
            fit += 16u * (TAMD_FIT_LOG + bits);
            if (fit < best) {
                t->mode[k] = TAMD_MODE_FSE;
                t->desc_len[k] = (uint32_t)((bits + 7u) / 8u);
                for (uint32_t i = 0; i < t->desc_len[k]; ++i) t->desc[k][i] = d[i];
                tamd_fit_states(t->norm[k], last + 1u, t->cum[k], t->state[k]);
            }
        }
        total += t->desc_len[k];
    }
    return total;
}

// The sequences section's modes byte (s3.1.1.3.2.1.2): LL << 6 | OF << 4 | ML << 2.
TAMD_HD static inline uint32_t tamd_modes_byte(const uint32_t* mode) {
    return (mode[0] << 6) | (mode[2] << 4) | (mode[1] << 2);
}

// tamd_fse_sequences with the block's tables: the descriptions are not written here (they follow
// the modes byte: LL, OF, ML); `modes` null = all predefined.
TAMD_HD static inline uint32_t tamd_fse_sequences_t(const uint32_t* seq_lo, const uint32_t* seq_off, uint32_t nseq,
                                                   const uint8_t* tabs, const tamd_seq_tables* tt, uint8_t* out,
                                                   uint32_t cap) {
    uint64_t acc = 0;
    uint32_t nbits = 0, pos = 0;
    bool over = false;
    auto add = [&](uint32_t v, uint32_t bits) {
        if (!bits) return;
        acc |= (uint64_t)(v & ((1u << bits) - 1u)) << nbits;
        nbits += bits;
        while (nbits >= 8) {
            if (pos < cap) out[pos] = (uint8_t)acc;
            else over = true;
            ++pos;
            acc >>= 8;
            nbits -= 8;
        }
    };
    const uint16_t* e16 = (const uint16_t*)(tabs + TAMD_FSE_E16);
    const uint32_t e16_at[3] = {TAMD_FSE_LL_E16, TAMD_FSE_ML_E16, TAMD_FSE_OF_E16};
    const uint32_t psize[3] = {64u, 64u, 32u};
    uint32_t mode[3] = {0, 0, 0};
    if (tt)
        for (uint32_t k = 0; k < 3; ++k) mode[k] = tt->mode[k];
    auto code_of = [&](uint32_t q, uint32_t k) {
        if (k == 0) return tamd_ll_code(seq_lo[q] & 0xffffu);
        if (k == 1) return tamd_ml_code(seq_lo[q] >> 16);
        return 31u - (uint32_t)__builtin_clz(seq_off[q] + 3u);
    };
    // one step of table k into the symbol of sequence q, from the decoder's next state st
    auto step = [&](uint32_t k, uint32_t q, uint32_t st, uint32_t* upd) -> uint32_t {
        const uint32_t c = code_of(q, k);
        if (mode[k] == TAMD_MODE_RLE) {
            *upd = 0;
            return 0;
        }
        if (mode[k] == TAMD_MODE_FSE) return tamd_fit_step(tt->norm[k][c], tt->cum[k][c], tt->state[k], st, upd);
        const uint32_t e = e16[e16_at[k] + c * psize[k] + st];
        *upd = (e >> 10) | (((e >> 6) & 15u) << 8);
        return e & 63u;
    };
    const uint32_t init_bits[3] = {mode[0] == TAMD_MODE_PREDEF ? 6u : mode[0] == TAMD_MODE_FSE ? TAMD_FIT_LOG : 0u,
                                   mode[1] == TAMD_MODE_PREDEF ? 6u : mode[1] == TAMD_MODE_FSE ? TAMD_FIT_LOG : 0u,
                                   mode[2] == TAMD_MODE_PREDEF ? 5u : mode[2] == TAMD_MODE_FSE ? TAMD_FIT_LOG : 0u};
    uint32_t s = nseq - 1, st[3], upd;
    for (uint32_t k = 0; k < 3; ++k) st[k] = step(k, s, 0, &upd);
    auto values = [&](uint32_t q) {
        const uint32_t ll = seq_lo[q] & 0xffffu, ml = seq_lo[q] >> 16, off = seq_off[q] + 3u;
        const uint32_t llc = tamd_ll_code(ll), mlc = tamd_ml_code(ml), ofc = 31u - (uint32_t)__builtin_clz(off);
        add(ll - tamd_ll_base(llc), tamd_ll_bits(llc));
        add(ml - tamd_ml_base(mlc), tamd_ml_bits(mlc));
        add(off, ofc);
    };
    values(s);
    while (s-- > 0) {
        const uint32_t order[3] = {2u, 1u, 0u};  // offsets, match lengths, literal lengths
        for (uint32_t i = 0; i < 3; ++i) {
            const uint32_t k = order[i];
            st[k] = step(k, s, st[k], &upd);
            add(upd & 0xffu, upd >> 8);
        }
        values(s);
    }
    add(st[1], init_bits[1]);  // the initial states, read first by the decoder: LL, OF, ML
    add(st[2], init_bits[2]);
    add(st[0], init_bits[0]);
    add(1, 1);  // end mark
    if (nbits) add(0, 8 - nbits);
    return over ? 0 : pos;
}

// Host: the FSE blob of the predefined distributions (RFC 8878 s3.1.1.3.2.2; zstd_internal.h
// LL/ML/OF_defaultNorm).  Each decoding table is laid out as FSE_buildDTable does
// (fse_decompress.c:93-148 restated: probability -1 symbols at the top, the others spread with
// step 5/8 of the table + 3, then per state its bit count and next-state base); the encoder's map
// inverts it: for a symbol and the state the decoder must reach next, the state to be in now.
static inline void tamd_build_fse(const int16_t* norm, uint32_t nsym, uint32_t log, uint8_t* enc, uint8_t* dec,
                                  uint16_t* e16) {
    const uint32_t size = 1u << log;
    uint32_t sym[64], next[64];
    uint32_t high = size - 1;
    for (uint32_t s = 0; s < nsym; ++s) {
        if (norm[s] == -1) {
            sym[high--] = s;
            next[s] = 1;
        } else {
            next[s] = (uint32_t)norm[s];
        }
    }
    const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    uint32_t pos = 0;
    for (uint32_t s = 0; s < nsym; ++s)
        for (int i = 0; i < norm[s]; ++i) {
            sym[pos] = s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    for (uint32_t u = 0; u < size; ++u) {
        const uint32_t s = sym[u];
        const uint32_t ns = next[s]++;
        const uint32_t nb = log - (31u - (uint32_t)__builtin_clz(ns));
        const uint32_t base = (ns << nb) - size;
        dec[2 * u] = (uint8_t)nb;
        dec[2 * u + 1] = (uint8_t)base;
        for (uint32_t y = base; y < base + (1u << nb); ++y) {
            enc[s * size + y] = (uint8_t)u;
            e16[s * size + y] = (uint16_t)(u | (nb << 6) | ((y - base) << 10));
        }
    }
}

static inline void tamd_fse_blob(uint8_t* blob) {
    static const int16_t ll[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
    static const int16_t ml[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
    static const int16_t of[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
    for (uint32_t i = 0; i < TAMD_FSE_BYTES; ++i) blob[i] = 0;
    uint16_t* e16 = (uint16_t*)(blob + TAMD_FSE_E16);
    tamd_build_fse(ll, 36, 6, blob + TAMD_FSE_LL_ENC, blob + TAMD_FSE_LL_DEC, e16 + TAMD_FSE_LL_E16);
    tamd_build_fse(ml, 53, 6, blob + TAMD_FSE_ML_ENC, blob + TAMD_FSE_ML_DEC, e16 + TAMD_FSE_ML_E16);
    tamd_build_fse(of, 29, 5, blob + TAMD_FSE_OF_ENC, blob + TAMD_FSE_OF_DEC, e16 + TAMD_FSE_OF_E16);
    // costs: log - log2(probability slots), a -1 symbol holding one slot
    const struct { const int16_t* norm; uint32_t nsym, log; } t[3] = {{ll, 36, 6}, {ml, 53, 6}, {of, 29, 5}};
    for (uint32_t k = 0; k < 3; ++k)
        for (uint32_t s = 0; s < t[k].nsym; ++s) {
            const double p = t[k].norm[s] > 0 ? (double)t[k].norm[s] : 1.0;
            blob[TAMD_FSE_PCOST + 64 * k + s] = (uint8_t)(16.0 * ((double)t[k].log - log2(p)) + 0.5);
        }
    for (uint32_t n = 1; n <= TAMD_FIT_SIZE; ++n)
        blob[TAMD_FSE_FCOST + n] = (uint8_t)(16.0 * ((double)TAMD_FIT_LOG - log2((double)n)) + 0.5);
}

// ---- Huffman-coded literals (RFC 8878 s3.1.1.3.1, s4.2) ----------------------------------------
// Literal byte values 0..128 only (the direct weight representation, s4.2.1.1 headerByte >= 128);
// code lengths limited to TAMD_HUF_MAX_BITS and complete (the decoder completes the last weight
// to a power of two).
#define TAMD_HUF_MAX_BITS 11u
#define TAMD_HUF_SYMS 129u

// Code lengths from the histogram `count[0..129)`; returns the longest length (0: fewer than two
// symbols, or a symbol above 128 occurs: no Huffman block).  Scratch: arrays of 2 * 129 entries.
TAMD_HD static inline uint32_t tamd_huf_lengths(const uint32_t* count, uint8_t* len, uint32_t* w, uint16_t* sym,
                                               uint16_t* parent) {
    uint32_t n = 0;
    for (uint32_t s = 0; s < TAMD_HUF_SYMS; ++s) {
        len[s] = 0;
        if (count[s]) sym[n++] = (uint16_t)s;
    }
    if (n < 2) return 0;
    for (uint32_t i = 1; i < n; ++i) {  // ascending count, then symbol (insertion sort, n <= 129)
        const uint16_t x = sym[i];
        uint32_t j = i;
        while (j > 0 && count[sym[j - 1]] > count[x]) {
            sym[j] = sym[j - 1];
            --j;
        }
        sym[j] = x;
    }
    // two-queue Huffman: leaves 0..n-1 (sorted), internal nodes n.. in creation order
    for (uint32_t i = 0; i < n; ++i) w[i] = count[sym[i]];
    uint32_t leaf = 0, node = n, made = n;
    for (uint32_t k = 0; k + 1 < n; ++k) {
        uint32_t pick[2];
        for (uint32_t t = 0; t < 2; ++t) {
            if (leaf < n && (node >= made || w[leaf] <= w[node])) pick[t] = leaf++;
            else pick[t] = node++;
        }
        w[made] = w[pick[0]] + w[pick[1]];
        parent[pick[0]] = parent[pick[1]] = (uint16_t)made;
        ++made;
    }
    // depths from the root (the last node) down; a leaf's depth is its code length
    w[made - 1] = 0;
    for (uint32_t k = made - 1; k-- > 0;) w[k] = w[parent[k]] + 1;
    uint32_t maxlen = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t l = w[i];
        if (l > TAMD_HUF_MAX_BITS) l = TAMD_HUF_MAX_BITS;
        len[sym[i]] = (uint8_t)l;
    }
    // length limit: restore Kraft equality at 2^MAX (longer codes for the rarest, shorter for the
    // most frequent)
    const uint32_t target = 1u << TAMD_HUF_MAX_BITS;
    uint32_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += 1u << (TAMD_HUF_MAX_BITS - len[sym[i]]);
    while (total > target) {
        for (uint32_t i = 0; i < n && total > target; ++i) {  // rarest first
            const uint32_t s = sym[i];
            if (len[s] < TAMD_HUF_MAX_BITS) {
                total -= 1u << (TAMD_HUF_MAX_BITS - len[s] - 1);
                ++len[s];
            }
        }
    }
    bool changed = true;
    while (total < target && changed) {
        changed = false;
        for (uint32_t i = n; i-- > 0 && total < target;) {  // most frequent first
            const uint32_t s = sym[i];
            if (len[s] > 1 && total + (1u << (TAMD_HUF_MAX_BITS - len[s])) <= target) {
                total += 1u << (TAMD_HUF_MAX_BITS - len[s]);
                --len[s];
                changed = true;
            }
        }
    }
    if (total != target) return 0;
    for (uint32_t s = 0; s < TAMD_HUF_SYMS; ++s)
        if (len[s] > maxlen) maxlen = len[s];
    return maxlen;
}

// Canonical codes (s4.2.1.3: by increasing weight = decreasing length, then by symbol value,
// values counting up from 0 at the longest length).
TAMD_HD static inline void tamd_huf_codes(const uint8_t* len, uint32_t maxlen, uint16_t* code) {
    uint32_t c = 0;
    for (uint32_t l = maxlen; l >= 1; --l) {
        for (uint32_t s = 0; s < TAMD_HUF_SYMS; ++s)
            if (len[s] == l) code[s] = (uint16_t)c++;
        c >>= 1;
    }
}

// Tree description, direct representation: header byte 127 + N, then the weights of symbols
// 0..N-1 two per byte (high nibble first); N = the largest symbol present, whose weight the
// decoder deduces.  Returns its size.
TAMD_HD static inline uint32_t tamd_huf_tree(const uint8_t* len, uint32_t maxlen, uint8_t* out) {
    uint32_t top = 0;
    for (uint32_t s = 0; s < TAMD_HUF_SYMS; ++s)
        if (len[s]) top = s;
    out[0] = (uint8_t)(127u + top);
    for (uint32_t s = 0; s < top; s += 2) {
        const uint32_t w0 = len[s] ? maxlen + 1 - len[s] : 0;
        const uint32_t w1 = s + 1 < top && len[s + 1] ? maxlen + 1 - len[s + 1] : 0;
        out[1 + s / 2] = (uint8_t)((w0 << 4) | w1);
    }
    return 1 + (top + 1) / 2;
}

// One Huffman stream of lits[0..n) (the decoder reads the first literal first, so the writer goes
// from the last), end mark and padding.  Returns its bytes, 0 when they would exceed cap.
TAMD_HD static inline uint32_t tamd_huf_stream(const uint8_t* lits, uint32_t n, const uint8_t* len,
                                              const uint16_t* code, uint8_t* out, uint32_t cap) {
    uint64_t acc = 0;
    uint32_t nbits = 0, pos = 0;
    for (uint32_t i = n; i-- > 0;) {
        const uint32_t s = lits[i];
        acc |= (uint64_t)code[s] << nbits;
        nbits += len[s];
        while (nbits >= 8) {
            if (pos >= cap) return 0;
            out[pos++] = (uint8_t)acc;
            acc >>= 8;
            nbits -= 8;
        }
    }
    acc |= 1ull << nbits;  // end mark
    ++nbits;
    while (nbits > 0) {
        if (pos >= cap) return 0;
        out[pos++] = (uint8_t)acc;
        acc >>= 8;
        nbits = nbits > 8 ? nbits - 8 : 0;
    }
    return pos;
}

// The whole Huffman literals section (header, tree, one or four streams) of lits[0..n) into out;
// returns its size, 0 when Huffman does not apply or the section would not beat `cap` bytes.
TAMD_HD static inline uint32_t tamd_huf_section(const uint8_t* lits, uint32_t n, const uint32_t* count,
                                               uint8_t* out, uint32_t cap) {
    uint8_t len[TAMD_HUF_SYMS];
    uint16_t code[TAMD_HUF_SYMS], sym[TAMD_HUF_SYMS], parent[2 * TAMD_HUF_SYMS];
    uint32_t w[2 * TAMD_HUF_SYMS];
    if (n < 16 || n > 16383 || cap < 8) return 0;
    const uint32_t maxlen = tamd_huf_lengths(count, len, w, sym, parent);
    if (!maxlen) return 0;
    tamd_huf_codes(len, maxlen, code);
    const bool single = n <= 1023;
    const uint32_t hsize = single ? 3u : (n <= 1023 ? 3u : 4u);
    uint32_t at = hsize;
    at += tamd_huf_tree(len, maxlen, out + at);
    if (at >= cap) return 0;
    if (single) {
        const uint32_t b = tamd_huf_stream(lits, n, len, code, out + at, cap - at);
        if (!b) return 0;
        at += b;
    } else {
        const uint32_t seg = (n + 3) / 4, jt = at;
        at += 6;
        if (at >= cap) return 0;
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t a = k * seg, e = a + seg < n ? a + seg : n;
            const uint32_t b = tamd_huf_stream(lits + a, e - a, len, code, out + at, cap - at);
            if (!b) return 0;
            if (k < 3) {
                out[jt + 2 * k] = (uint8_t)b;
                out[jt + 2 * k + 1] = (uint8_t)(b >> 8);
            }
            at += b;
        }
    }
    const uint32_t comp = at - hsize;  // tree + (jump table +) streams
    if (single) {
        if (comp > 1023) return 0;
        const uint32_t v = 2u | (n << 4) | (comp << 14);
        out[0] = (uint8_t)v;
        out[1] = (uint8_t)(v >> 8);
        out[2] = (uint8_t)(v >> 16);
    } else if (hsize == 3) {
        if (comp > 1023) return 0;
        const uint32_t v = 2u | (1u << 2) | (n << 4) | (comp << 14);
        out[0] = (uint8_t)v;
        out[1] = (uint8_t)(v >> 8);
        out[2] = (uint8_t)(v >> 16);
    } else {
        if (comp > 16383) return 0;
        const uint32_t v = 2u | (2u << 2) | (n << 4) | (comp << 18);
        out[0] = (uint8_t)v;
        out[1] = (uint8_t)(v >> 8);
        out[2] = (uint8_t)(v >> 16);
        out[3] = (uint8_t)(v >> 24);
    }
    return at;
}
