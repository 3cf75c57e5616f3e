// lz.hip -- Tonk's upstream compression step (MessageCompressor, PacketCompression.h:92-140 /
// PacketCompression.cpp:70-118) on gfx950: every message becomes one zstd *compressed block*
// (RFC 8878 s3.1.1.3) that the reference's MessageDecompressor (ZSTD_decompressBlock against its
// 24 KB history ring) decodes unchanged.
//
// One wave per job; a job is a run of consecutive messages of one stream.  Matches come from the
// bytes the decompressor will hold when it decodes the message: the current history segment and
// the one before it (zstd keeps the previous contiguous segment as its external dictionary,
// zstd_decompress.c ZSTD_checkContinuity).  The block uses raw literals and the predefined FSE
// distributions for literal lengths, match lengths and offsets, or per block the cheaper of an RLE
// code or an FSE table fitted to the block's codes and described in it (round 6; no repeat
// offsets or repeat tables, so no state carries from block to block).
//
// Eight waves per workgroup (two per SIMD: a wave's LDS is 17.5 KB, the FSE maps are shared).
// Per message: (1) candidate positions from a hash table of 8-byte keys in LDS (16-bit positions
// relative to the job's base; the window's positions are inserted once per job, each message's
// after it is scanned, 64 at a time), (2) every lane
// extends its own candidate, (3) a ballot-driven greedy parse, (4) lane 0 writes the backward
// FSE bit stream of the sequences into LDS, (5) the wave copies header, literals and bit stream
// to the output when the block is smaller than the message (else written = 0, as
// ZSTD_compressBlock's "not compressible" result, PacketCompression.cpp:96-101).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz.h"

#define LZ_HASH_LOG 12  // 4K entries of 16 bits: 8 KB per wave, so that 8 waves (2 per SIMD) fit a CU
#ifndef LZ_WINDOW_LANE16
#define LZ_WINDOW_LANE16 1
#endif
#define LZ_REL_MAX 65535u
#ifndef LZ_NO_EXTEND
#define LZ_NO_EXTEND 0  // (measurement only: matches stop at the probe's LZ_PROBE bytes)
#endif
#ifndef LZ_PROBE_BATCH
#define LZ_PROBE_BATCH 3u  // groups of 64 positions whose candidate loads go out together
#endif  // job-relative positions (+ 1) the table can hold
#define LZ_HASH (1u << LZ_HASH_LOG)
#define LZ_MIN_MATCH 4u
#ifndef LZ_PROBE
#define LZ_PROBE 16u  // bytes a lane compares per candidate; a chosen match is extended by the wave
#endif
#define LZ_MAX_SEQS (TAMD_LZ_MAX_MESSAGE / LZ_MIN_MATCH)
// Candidates are found and parsed LZ_CH positions at a time; after the parse the same words
// hold the three state-update chains (3 x LZ_MAX_SEQS halfwords).  A sequence's codes are
// recomputed from its lengths and offset wherever they are needed instead of being stored.
#define LZ_CH (3u * LZ_MAX_SEQS / 2u)
#define LZ_WAVES TAMD_LZ_WAVES  // jobs per workgroup: the waves share the FSE maps (1 workgroup per CU)
#define LZ_COST_BYTES (TAMD_FSE_BYTES - TAMD_FSE_PCOST)  // costs and flags, in LDS after the maps
static_assert(TAMD_FSE_PCOST == TAMD_FSE_E16 + 2u * TAMD_FSE_E16_WORDS && LZ_COST_BYTES % 4u == 0u, "blob layout");

// Byte loads of a stream: `buf` at linear position p & mask.  Multi-byte loads are unaligned
// global loads; the buffers carry readable slack past their end (a linear stream: 32 bytes past
// its last message, tamd_compress_batch; the 64 KB ring: its first 64 bytes mirrored after it).
typedef uint64_t lz_u64u __attribute__((aligned(1)));

static __device__ __forceinline__ uint64_t lz_dword(const uint8_t* __restrict__ buf, uint32_t mask, uint32_t p) {
    return *(const lz_u64u*)(buf + (p & mask));
}

// Candidates are keyed by the 8 bytes at a position (a match still needs only LZ_MIN_MATCH equal
// bytes): on text a 4-byte key's most recent occurrence is mostly a short match inside a common
// word, an 8-byte key's mostly the long one (fewer, longer sequences: the ratio of zstd level 1).
// Bytes past the message end may enter a key; the probe compares only the message's bytes.
static __device__ __forceinline__ uint32_t lz_hash(uint64_t w) {
    return (uint32_t)((w * 0x9E3779B185EBCA87ull) >> (64 - LZ_HASH_LOG));
}

// The waves of a workgroup run unrelated jobs: they synchronise only with themselves (LDS and
// scratch writes complete before any lane reads them).
#define LZ_SYNC()                                                \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   \
        __builtin_amdgcn_wave_barrier();                         \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   \
    } while (0)

// One wave's LDS.
struct LzWave {
    uint16_t htab[LZ_HASH];  // (position - job base + 1), 0 = empty
    uint32_t mword[LZ_CH];  // per chunk position: the match there, length | distance << 16
    uint32_t seq_lo[LZ_MAX_SEQS];                             // literal length | match length << 16
    uint32_t seq_off[LZ_MAX_SEQS];                            // offset
    uint32_t bitw[(TAMD_LZ_MAX_MESSAGE + 64) / 4];            // backward FSE bit stream
    __attribute__((aligned(16))) uint8_t mbuf[TAMD_LZ_MAX_MESSAGE + LZ_PROBE + 16];  // the message
    uint32_t sh_init[3], sh_bytes, sh_ok;
    // the block's sequence tables (tamd_seq_choose, a lane per symbol): descriptions, and the
    // fitted tables' normalized counts, state offsets and states (tamd_fit_states)
    uint32_t fdesc[3][TAMD_FIT_DESC / 4];
    uint32_t fstarts[3];  // bit g: some symbol's share of the 32 states starts at occurrence g
    uint8_t fnorm[3][64], fcum[3][64], fstate[3][TAMD_FIT_SIZE], gsym[3][TAMD_FIT_SIZE];
};

// The hash table keeps each bucket's most recent position, relative to the job's base (lz_rebase).
// Positions enter it in increasing order, 64 consecutive ones per store (the window, each
// message's scan), so a later store is always more recent; lanes of one store that share a bucket
// leave one of theirs (LDS resolves same-address lanes in a fixed order: the output does not
// vary from run to run, and its ratio equals that of a version that re-stored until the largest
// stayed, profiles/r06q_lz_occupancy_ab.txt).
static __device__ __forceinline__ void lz_insert(uint16_t* htab, bool ins, uint32_t h, uint32_t rel) {
    if (ins) htab[h] = (uint16_t)rel;
}

// Moves the job's base forward to `to` (> base): entries keep their positions, the ones before
// `to` become empty.  Only jobs that span more than LZ_REL_MAX bytes (large messages) need it.
static __device__ __forceinline__ void lz_rebase(uint16_t* htab, uint32_t& base, uint32_t to, uint32_t lane) {
    const uint32_t d = to - base;
    for (uint32_t k = lane; k < LZ_HASH; k += 64) {
        const uint32_t e = htab[k];
        htab[k] = (uint16_t)(e > d ? e - d : 0u);
    }
    LZ_SYNC();
    base = to;
}

// Wave sums (DPP row shifts: a few instructions) and exclusive prefix sums of B-bit values, a bit
// plane at a time (one ballot and a lane's mbcnt per bit).
static __device__ __forceinline__ uint32_t lz_wave_sum(uint32_t x) { return __reduce_add_sync(~0ull, x); }
template <uint32_t B>
static __device__ __forceinline__ uint32_t lz_wave_excl(uint32_t x) {  // sum over the lanes below
    uint32_t s = 0;
#pragma unroll
    for (uint32_t b = 0; b < B; ++b) {
        const uint64_t m = __ballot((x >> b) & 1u);
        s += __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << b;
    }
    return s;
}


// One message.  BIG: the message is read from the stream buffer and its per-sequence arrays live
// in global scratch; otherwise all of it is in the wave's LDS.
template <bool BIG>
static __device__ __forceinline__ void lz_message(LzWave& L, const uint16_t* __restrict__ e16,
                                                  const uint8_t* __restrict__ fse, const tamd_lz_msg m,
                                                  const uint8_t* __restrict__ buf, uint32_t mask,
                                                  uint8_t* __restrict__ scratch, uint8_t* __restrict__ out,
                                                  uint32_t* __restrict__ written, uint32_t mi, uint32_t lane, uint32_t& jb,
                                                  unsigned long long* ph, unsigned long long& t_ph, bool prof) {
#define LZ_PHASE(k)                                                          \
    if (prof) {                                                              \
        const unsigned long long t_now = __builtin_amdgcn_s_memrealtime();   \
        ph[k] += t_now - t_ph;                                               \
        t_ph = t_now;                                                        \
    }
    const uint32_t n = m.len;
    const uint32_t S = BIG ? tamd_lz_big_seqs(n) : LZ_MAX_SEQS;
    uint32_t *seq_lo, *seq_off, *bitw;
    uint16_t* upd;
    uint32_t bw_cap;  // bit-stream words
    if constexpr (BIG) {
        uint32_t* w = (uint32_t*)(scratch + m.scratch);
        seq_lo = w;
        seq_off = w + S;
        bitw = w + 2 * S;
        bw_cap = (n + 64u) / 4u;
        upd = (uint16_t*)(bitw + bw_cap + 4u);
    } else {
        seq_lo = L.seq_lo;
        seq_off = L.seq_off;
        upd = (uint16_t*)L.mword;  // (free after the parse)
        bitw = L.bitw;
        bw_cap = (TAMD_LZ_MAX_MESSAGE + 64u) / 4u;
    }
    const uint8_t* mb = L.mbuf;
    // the literal-length, match-length and offset codes of sequence sq (bytes 0, 1, 2)
    auto seq_code = [&](uint32_t sq) -> uint32_t {
        const uint32_t lo = seq_lo[sq];
        return tamd_ll_code(lo & 0xffffu) | (tamd_ml_code(lo >> 16) << 8) |
               ((31u - (uint32_t)__builtin_clz(seq_off[sq] + 3u)) << 16);
    };
    // the message's bytes at offset i (LDS copy, or the stream buffer for BIG messages)
    auto msg_dword = [&](uint32_t i) -> uint64_t {
        if constexpr (BIG) return lz_dword(buf, mask, m.pos + i);
        else return *(const lz_u64u*)(mb + i);
    };
    auto msg_byte = [&](uint32_t i) -> uint8_t {
        if constexpr (BIG) return buf[(m.pos + i) & mask];
        else return mb[i];
    };
    if constexpr (!BIG) {
        // the message into LDS (16 bytes per lane per step; the slack past it is readable)
        for (uint32_t k = 16u * lane; k < n; k += 1024) {
            const uint64_t a = lz_dword(buf, mask, m.pos + k), b = lz_dword(buf, mask, m.pos + k + 8);
            *(uint64_t*)(L.mbuf + k) = a;
            *(uint64_t*)(L.mbuf + k + 8) = b;
        }
        LZ_SYNC();
    }
    // Chunks of LZ_CH positions: (1)+(2) candidates and match lengths, 64 positions at a time (a
    // group's positions are inserted after it is scanned: matches reach back to earlier groups),
    // then (3) the greedy parse of the chunk: from p, the first position with a match starts the
    // next sequence.  The wave holds the match words of 64 positions from `wb` in registers; the
    // window moves only when p leaves it.  Sequences collect in registers (lane j keeps sequence
    // j of each group of 64) and are stored a group at a time.
    uint32_t p = 0, lit_start = 0, nseq = 0, lits = 0;
    uint32_t my_lo = 0, my_off = 0;
    for (uint32_t c0 = 0; c0 < n; c0 += LZ_CH) {
        const uint32_t cend = n - c0 < LZ_CH ? n : c0 + LZ_CH;
        // (the chunk's positions must fit the table: a job past 64 KB moves its base up to the
        // last TAMD_LZ_WINDOW bytes before the chunk)
        if (m.pos + cend - jb >= LZ_REL_MAX) lz_rebase(L.htab, jb, m.pos + c0 - TAMD_LZ_WINDOW, lane);
        // LZ_PROBE_BATCH groups of 64 positions at a time: the table is read and written group
        // after group in LDS order (group g's lookups see groups < g, not g itself), and only then
        // do the candidates' loads go out, every group's together.  Lanes without a candidate load
        // from the message start and drop the result (no exec-masked loads).
        for (uint32_t c = c0; c < cend; c += 64u * LZ_PROBE_BATCH) {
            uint64_t key[LZ_PROBE_BATCH];
#pragma unroll
            for (uint32_t b = 0; b < LZ_PROBE_BATCH; ++b) {
                const uint32_t i = c + 64u * b + lane;
                key[b] = 0;
                if (i < cend && i + LZ_MIN_MATCH <= n) key[b] = msg_dword(i);
            }
            uint32_t src[LZ_PROBE_BATCH];
#pragma unroll
            for (uint32_t b = 0; b < LZ_PROBE_BATCH; ++b) {
                const uint32_t i = c + 64u * b + lane;
                const bool look = i < cend && i + LZ_MIN_MATCH <= n;  // (= i + 3 < n: inserted too)
                const uint32_t h = lz_hash(key[b]);
                uint32_t e = 0;
                if (look) e = L.htab[h];
                lz_insert(L.htab, look, h, m.pos + i + 1 - jb);
                src[b] = e ? jb + e - 1 : 0u;
            }
#pragma unroll
            for (uint32_t b = 0; b < LZ_PROBE_BATCH; ++b) {
                const uint32_t i = c + 64u * b + lane;
                const bool cand = i < cend && i + LZ_MIN_MATCH <= n && src[b] && src[b] >= m.win && src[b] < m.pos + i;
                const uint32_t lim = cand ? (n - i < LZ_PROBE ? n - i : LZ_PROBE) : 0u;
                const uint32_t s0 = cand ? src[b] : m.pos;
                uint64_t xs[LZ_PROBE / 8];
#pragma unroll
                for (uint32_t k = 0; k < LZ_PROBE / 8; ++k) {  // (no load past the message)
                    const bool in = 8 * k < lim;
                    xs[k] = lz_dword(buf, mask, s0 + (in ? 8 * k : 0u)) ^ msg_dword(in ? i + 8 * k : 0u);
                    if (!in) xs[k] = 0;
                }
                uint32_t len = LZ_PROBE;
#pragma unroll
                for (uint32_t k = LZ_PROBE / 8; k-- > 0;)
                    if (xs[k]) len = 8 * k + ((uint32_t)__builtin_ctzll(xs[k]) >> 3);
                if (len > lim) len = lim;
                if (len < LZ_MIN_MATCH) len = 0;
                if (i < cend) L.mword[i - c0] = len ? len | ((m.pos + i - src[b]) << 16) : 0u;
            }
        }
        LZ_SYNC();
        LZ_PHASE(1)
        if (p < cend) {
            uint32_t wb = p > c0 ? p : c0;  // (positions in [p, c0) were scanned with the last chunk)
            uint32_t mine = wb + lane < cend ? L.mword[wb + lane - c0] : 0u;
            // the window's positions with a match, once per window: a step only masks off the
            // positions below p (scalar work)
            uint64_t mm = __ballot((mine & 0xffffu) != 0);
            for (;;) {
                const uint32_t sh = p > wb ? p - wb : 0u;
                const uint64_t b = sh < 64u ? mm & (~0ull << sh) : 0ull;
                if (!b) {
                    wb = __builtin_amdgcn_readfirstlane(wb + 64);
                    if (wb >= cend) break;
                    if (p < wb) p = wb;
                    mine = wb + lane < cend ? L.mword[wb + lane - c0] : 0u;
                    mm = __ballot((mine & 0xffffu) != 0);
                    continue;
                }
                const uint32_t first = (uint32_t)__builtin_ctzll(b);
                const uint32_t at = __builtin_amdgcn_readfirstlane(wb + first);
                const uint32_t word = (uint32_t)__builtin_amdgcn_readlane((int)mine, (int)first);
                const uint32_t dist = word >> 16;
                uint32_t ml = word & 0xffffu;
                if (!LZ_NO_EXTEND && ml == LZ_PROBE && at + ml < n) {
                    // the probe matched in full: the wave extends the match 512 bytes per step
                    const uint32_t q = m.pos + at;
                    for (;;) {
                        const uint32_t k = ml + 8u * lane;
                        uint64_t x = 0;
                        if (k < n - at) x = lz_dword(buf, mask, q - dist + k) ^ lz_dword(buf, mask, q + k);
                        const uint64_t bad = __ballot(k >= n - at || x != 0);
                        if (!bad) {
                            ml += 512;
                            continue;
                        }
                        const uint32_t fb = (uint32_t)__builtin_ctzll(bad);
                        const uint64_t xf = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)fb) |
                                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), (int)fb) << 32);
                        const uint32_t kf = ml + 8u * fb;
                        ml = kf < n - at ? kf + ((uint32_t)__builtin_ctzll(xf) >> 3) : n - at;
                        break;
                    }
                    if (ml > n - at) ml = n - at;
                    ml = __builtin_amdgcn_readfirstlane(ml);
                }
                const bool slot = lane == (nseq & 63u);  // (selects, no branch)
                my_lo = slot ? (at - lit_start) | (ml << 16) : my_lo;
                my_off = slot ? dist : my_off;
                lits += at - lit_start;
                ++nseq;
                if ((nseq & 63u) == 0) {
                    seq_lo[nseq - 64 + lane] = my_lo;
                    seq_off[nseq - 64 + lane] = my_off;
                }
                p = __builtin_amdgcn_readfirstlane(at + ml);
                lit_start = p;
                if (p >= cend) break;
                if (p >= wb + 64) {
                    wb = p;
                    mine = wb + lane < cend ? L.mword[wb + lane - c0] : 0u;
                    mm = __ballot((mine & 0xffffu) != 0);
                }
            }
        }
        LZ_SYNC();  // (the next chunk rewrites mword)
        LZ_PHASE(2)
    }
    if ((nseq & 63u) != 0 && lane < (nseq & 63u)) {
        const uint32_t g = nseq & ~63u;
        seq_lo[g + lane] = my_lo;
        seq_off[g + lane] = my_off;
    }
    if (prof) ph[7] += nseq;  // (profiling: sequences, not ticks)
    const uint32_t last_lits = n - lit_start;  // literals after the last sequence
    lits += last_lits;
    LZ_SYNC();

    // (4) the sequence bit stream, as tamd_fse_sequences_t (lz.h) writes it, built in parallel:
    // codes per sequence (all lanes), each table's choice (a lane per symbol), the three state
    // chains (lanes 0-2, one chain each, from the last sequence back), then every sequence's bit
    // fields placed at their offsets (a prefix sum of the field widths in stream order: the last
    // sequence first).
    uint32_t lh = 0, shb = 0;
    const uint32_t lits_word = tamd_lits_header_word(lits, &lh);
    uint32_t seq_word = tamd_seq_header_word(nseq, &shb);
    const uint32_t limit = n - 1u < m.cap ? n - 1u : m.cap;  // smaller than the message, fits
    uint32_t head = lh + lits + shb;
    bool ok = head < limit && nseq > 0;
    uint32_t total = 0;
    uint32_t mode[3] = {TAMD_MODE_PREDEF, TAMD_MODE_PREDEF, TAMD_MODE_PREDEF}, dlen[3] = {0, 0, 0};
    if (ok) {
        uint32_t* hist = L.bitw;  // (3 x 64 counts; the bit stream's words are zeroed after)
        for (uint32_t k = lane; k < 3u * 64u; k += 64) hist[k] = 0;
        if (lane < 3u * TAMD_FIT_DESC / 4u) (&L.fdesc[0][0])[lane] = 0;
        if (lane < 3u) L.fstarts[lane] = 0;
        LZ_SYNC();
        for (uint32_t sq = lane; sq < nseq; sq += 64) {
            const uint32_t cd = seq_code(sq);
            atomicAdd(&hist[cd & 0xffu], 1u);
            atomicAdd(&hist[64u + ((cd >> 8) & 0xffu)], 1u);
            atomicAdd(&hist[128u + (cd >> 16)], 1u);
        }
        LZ_SYNC();
        // each table's mode (tamd_seq_choose restated a lane per symbol), the three tables side by
        // side: their chains of wave operations are independent, so each one's latency hides the
        // others' (one wave per SIMD here)
        const uint8_t* costs = (const uint8_t*)(e16 + TAMD_FSE_E16_WORDS);  // (LDS: the blob from TAMD_FSE_PCOST)
        const bool fit_on = !(costs[TAMD_FSE_FLAGS - TAMD_FSE_PCOST] & TAMD_FSE_PREDEFINED_ONLY);
        uint32_t cnt[3], nrm[3], present[3], last[3], best[3], cum[3] = {0, 0, 0}, w[3] = {0, 0, 0};
        uint64_t pres[3], v[3] = {0, 0, 0};
        bool cand[3];
#pragma unroll
        for (uint32_t k = 0; k < 3; ++k) {
            const uint32_t nsym = k == 0 ? 36u : k == 1 ? 53u : 32u, plog = k == 2 ? 5u : 6u;
            cnt[k] = lane < nsym ? hist[64u * k + lane] : 0u;
            nrm[k] = tamd_fit_norm(cnt[k], nseq);
            pres[k] = __ballot(cnt[k] != 0);
            present[k] = (uint32_t)__builtin_popcountll(pres[k]);
            last[k] = 63u - (uint32_t)__builtin_clzll(pres[k]);
            best[k] = lz_wave_sum(cnt[k] * costs[64u * k + lane]) + 16u * plog;
            if (present[k] == 1u && 16u * 8u < best[k] && fit_on) {
                mode[k] = TAMD_MODE_RLE;
                best[k] = 16u * 8u;
                dlen[k] = 1;
            }
            cand[k] = present[k] >= 2u && present[k] <= TAMD_FIT_SIZE && nseq >= TAMD_FIT_MIN_SEQS && fit_on;
        }
        if (cand[0] || cand[1] || cand[2]) {
            uint32_t sum[3], big[3];
            uint64_t top[3];
#pragma unroll
            for (uint32_t k = 0; k < 3; ++k) {
                sum[k] = lz_wave_sum(nrm[k]);
                top[k] = pres[k];
            }
            // the largest share, lowest symbol on ties: bit planes from the top
#pragma unroll
            for (uint32_t b = 6; b-- > 0;)
#pragma unroll
                for (uint32_t k = 0; k < 3; ++k) {
                    const uint64_t m = top[k] & __ballot((nrm[k] >> b) & 1u);
                    if (m) top[k] = m;
                }
#pragma unroll
            for (uint32_t k = 0; k < 3; ++k) {
                big[k] = (uint32_t)__builtin_ctzll(top[k]);
                const int32_t fixed = (int32_t)__builtin_amdgcn_readlane((int)nrm[k], (int)big[k]) + (int32_t)TAMD_FIT_SIZE - (int32_t)sum[k];
                cand[k] = cand[k] && fixed >= 1;
                if (cand[k] && lane == big[k]) nrm[k] = (uint32_t)fixed;
            }
            uint32_t wsum[3], fit[3];
#pragma unroll
            for (uint32_t k = 0; k < 3; ++k) {
                cum[k] = lz_wave_excl<6>(nrm[k]);
                const uint64_t nz = __ballot(nrm[k] != 0);
                const bool lead = lane == 0 || ((nz >> (lane - 1u)) & 1ull) != 0;
                const uint64_t above = nz & ~((2ull << lane) - 1ull);
                const uint32_t z = nrm[k] == 0 && above ? (uint32_t)__builtin_ctzll(above) - lane - 1u : 0u;
                w[k] = cand[k] && lane <= last[k] ? tamd_ncount_item(nrm[k], cum[k], lead, z, &v[k]) : 0u;
            }
#pragma unroll
            for (uint32_t k = 0; k < 3; ++k) {
                wsum[k] = lz_wave_sum(w[k]);
                fit[k] = lz_wave_sum(cnt[k] * costs[TAMD_FSE_FCOST - TAMD_FSE_PCOST + nrm[k]]) +
                         16u * (TAMD_FIT_LOG + 4u + wsum[k]);
                if (cand[k] && fit[k] < best[k]) {
                    mode[k] = TAMD_MODE_FSE;
                    dlen[k] = (4u + wsum[k] + 7u) / 8u;
                }
            }
            // the fitted tables' descriptions, then the encoder's states (tamd_fit_states)
            bool any = false;
#pragma unroll
            for (uint32_t k = 0; k < 3; ++k) {
                if (mode[k] != TAMD_MODE_FSE) continue;
                any = true;
                const uint32_t at = 4u + lz_wave_excl<6>(w[k]);
                if (w[k]) {
                    uint32_t* d = L.fdesc[k];
                    const uint32_t w0 = at / 32u, sh = at % 32u;
                    atomicOr(&d[w0], (uint32_t)(v[k] << sh));
                    if (sh + w[k] > 32u) atomicOr(&d[w0 + 1], (uint32_t)(v[k] >> (32u - sh)));
                    if (sh + w[k] > 64u) atomicOr(&d[w0 + 2], (uint32_t)(v[k] >> (64u - sh)));
                }
                L.fnorm[k][lane] = (uint8_t)nrm[k];
                L.fcum[k][lane] = (uint8_t)cum[k];
                // occurrence g belongs to the symbol whose share starts at the last start <= g
                if (nrm[k]) {
                    L.gsym[k][cum[k]] = (uint8_t)lane;
                    atomicOr(&L.fstarts[k], 1u << cum[k]);
                }
            }
            if (any) {
                LZ_SYNC();
                // state u decodes the symbol spread to slot u: occurrence g = u * 7 (mod 32); its
                // rank among that symbol's states is the number of smaller u with it
                const bool in = lane < TAMD_FIT_SIZE;
                const uint32_t g = (lane * TAMD_FIT_STEP_INV) & (TAMD_FIT_SIZE - 1u);
#pragma unroll
                for (uint32_t k = 0; k < 3; ++k) {
                    if (mode[k] != TAMD_MODE_FSE) continue;
                    const uint32_t starts = L.fstarts[k];
                    const uint32_t sym = in ? L.gsym[k][31u - (uint32_t)__builtin_clz(starts & ((2u << g) - 1u))] : 0u;
                    uint64_t same = __ballot(in);
#pragma unroll
                    for (uint32_t b = 0; b < 6; ++b) {
                        const uint64_t bb = __ballot(in && ((sym >> b) & 1u));
                        same &= ((sym >> b) & 1u) ? bb : ~bb;
                    }
                    const uint32_t rank = (uint32_t)__builtin_popcountll(same & ((1ull << lane) - 1ull));
                    if (in) L.fstate[k][L.fcum[k][sym] + rank] = (uint8_t)lane;
                }
            }
        }
        if (lane == 0)
#pragma unroll
            for (uint32_t k = 0; k < 3; ++k)
                if (mode[k] == TAMD_MODE_RLE) L.fdesc[k][0] = 63u - __builtin_clzll(pres[k]);
        LZ_SYNC();
        seq_word |= tamd_modes_byte(mode) << (8u * (shb - 1u));
        head += dlen[0] + dlen[1] + dlen[2];
        ok = head < limit;
    }
    LZ_PHASE(5)
    if (ok) {
        // every sequence's code in its update slot of each table's chain: for a predefined table the
        // code itself, for a fitted one its share | offset << 6 | step bits << 11
        for (uint32_t sq = lane; sq < nseq; sq += 64) {
            const uint32_t cd = seq_code(sq);
#pragma unroll
            for (uint32_t t = 0; t < 3; ++t) {
                const uint32_t c = (cd >> (8u * t)) & 0xffu;
                if (mode[t] == TAMD_MODE_FSE) {
                    const uint32_t nn = L.fnorm[t][c];
                    upd[S * t + sq] = (uint16_t)(nn | (uint32_t)L.fcum[t][c] << 6 | tamd_fit_mbo(nn) << 11);
                } else if (mode[t] == TAMD_MODE_PREDEF) {
                    upd[S * t + sq] = (uint16_t)c;
                }
            }
        }
        LZ_SYNC();
        if (lane < 3) {
            const uint32_t size = lane == 2 ? 32u : 64u;
            const uint32_t md = lane == 0 ? mode[0] : lane == 1 ? mode[1] : mode[2];
            const uint16_t* enc = e16 + (lane == 0 ? TAMD_FSE_LL_E16 : lane == 1 ? TAMD_FSE_ML_E16 : TAMD_FSE_OF_E16);
            uint16_t* u_out = upd + S * lane;
            uint32_t st = 0;
            if (md == TAMD_MODE_FSE) {
                const uint8_t* sv = L.fstate[lane];
                uint32_t u;
                const uint32_t inf0 = u_out[nseq - 1];
                st = tamd_fit_step_m(inf0 & 63u, (inf0 >> 6) & 31u, inf0 >> 11, sv, 0, &u);
                // (each step's symbol share and offset were put in its update slot beforehand: the
                // only load that waits for the previous step is the state's)
#pragma unroll 4
                for (uint32_t sq = nseq - 1; sq-- > 0;) {
                    const uint32_t inf = u_out[sq];
                    st = tamd_fit_step_m(inf & 63u, (inf >> 6) & 31u, inf >> 11, sv, st, &u);
                    u_out[sq] = (uint16_t)u;
                }
            } else if (md == TAMD_MODE_PREDEF) {
                st = enc[u_out[nseq - 1] * size] & 63u;
                for (uint32_t sq = nseq - 1; sq-- > 0;) {
                    const uint32_t e = enc[u_out[sq] * size + st];
                    u_out[sq] = (uint16_t)((e >> 10) | (((e >> 6) & 15u) << 8));
                    st = e & 63u;
                }
            }  // (RLE: no state bits)
            L.sh_init[lane] = st;
        }
        LZ_PHASE(6)
        // zero the bit buffer words the stream can use
        const uint32_t cap_words = (limit - head + 3u) / 4u + 1u;
        const uint32_t wcap = cap_words < bw_cap ? cap_words : bw_cap;
        for (uint32_t k = lane; k < wcap; k += 64) bitw[k] = 0;
        LZ_SYNC();
        uint32_t carry = 0;
        for (uint32_t base = 0; base < nseq; base += 64) {
            const uint32_t r = base + lane;  // stream order: sequence nseq - 1 - r
            uint64_t v = 0;
            uint32_t nbits = 0;
            if (r < nseq) {
                const uint32_t sq = nseq - 1u - r;
                const uint32_t cd = seq_code(sq), llc = cd & 0xffu, mlc = (cd >> 8) & 0xffu, ofc = cd >> 16;
                auto put = [&](uint32_t val, uint32_t nb) {
                    v |= (uint64_t)(val & ((1u << nb) - 1u)) << nbits;
                    nbits += nb;
                };
                if (sq != nseq - 1u) {
                    const uint32_t o = mode[2] != TAMD_MODE_RLE ? upd[2u * S + sq] : 0u;
                    const uint32_t ml_u = mode[1] != TAMD_MODE_RLE ? upd[S + sq] : 0u;
                    const uint32_t l_u = mode[0] != TAMD_MODE_RLE ? upd[sq] : 0u;
                    put(o & 0xffu, o >> 8);
                    put(ml_u & 0xffu, ml_u >> 8);
                    put(l_u & 0xffu, l_u >> 8);
                }
                put((seq_lo[sq] & 0xffffu) - tamd_ll_base(llc), tamd_ll_bits(llc));
                put((seq_lo[sq] >> 16) - tamd_ml_base(mlc), tamd_ml_bits(mlc));
                put(seq_off[sq] + 3u, ofc);
            }
            uint32_t x = nbits;
#pragma unroll
            for (uint32_t d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d);
                if (lane >= d) x += y;
            }
            const uint32_t at = carry + x - nbits;
            if (nbits && (at + nbits + 31u) / 32u < wcap) {
                const uint32_t w0 = at / 32u, sh = at % 32u;
                atomicOr(&bitw[w0], (uint32_t)(v << sh));
                if (sh + nbits > 32u) atomicOr(&bitw[w0 + 1], (uint32_t)(v >> (32u - sh)));
                if (sh + nbits > 64u) atomicOr(&bitw[w0 + 2], (uint32_t)(v >> (64u - sh)));
            }
            carry += __shfl(x, 63);
        }
        LZ_SYNC();
        // the initial states (ML, OF, LL: the decoder reads LL first) and the end mark
        auto init_w = [&](uint32_t k) {
            return mode[k] == TAMD_MODE_PREDEF ? (k == 2 ? 5u : 6u) : mode[k] == TAMD_MODE_FSE ? TAMD_FIT_LOG : 0u;
        };
        const uint32_t w_ml = init_w(1), w_of = init_w(2), w_ll = init_w(0);
        const uint64_t tail = (uint64_t)L.sh_init[1] | ((uint64_t)L.sh_init[2] << w_ml) |
                              ((uint64_t)L.sh_init[0] << (w_ml + w_of)) | (1ull << (w_ml + w_of + w_ll));
        const uint32_t tail_bits = w_ml + w_of + w_ll + 1u;
        const uint32_t bits_total = carry + tail_bits;
        total = head + (bits_total + 7u) / 8u;
        ok = total <= limit;
        if (ok && lane == 0) {
            const uint32_t w0 = carry / 32u, sh = carry % 32u;
            bitw[w0] |= (uint32_t)(tail << sh);
            if (sh + tail_bits > 32u) bitw[w0 + 1] |= (uint32_t)(tail >> (32u - sh));
        }
    }
    if (lane == 0) {
        L.sh_bytes = ok ? total : 0;
        L.sh_ok = ok;
        written[mi] = ok ? total : 0;
    }
    LZ_SYNC();
    LZ_PHASE(3)
    // (5) the block: literals section header, literals, sequences header, bit stream
    if (L.sh_ok) {
        uint8_t* o = out + m.out;
        uint32_t w = lh;
        if (lane < w) o[lane] = (uint8_t)(lits_word >> (8u * lane));
        // literals: lane j copies the literal run of sequences j, j + 64, ... (and the final run)
        // to its place, found by a wave prefix sum of the run lengths; where it starts in the
        // message, by a prefix sum of the sequences' spans (literals + match)
        uint32_t carry = 0, mcarry = 0;
        for (uint32_t base = 0; base <= nseq; base += 64) {
            const uint32_t sq = base + lane;
            uint32_t ll = 0, span = 0;
            if (sq < nseq) {
                const uint32_t lo = seq_lo[sq];
                ll = lo & 0xffffu;
                span = ll + (lo >> 16);
            } else if (sq == nseq) {
                ll = last_lits;
            }
            uint32_t x = ll, y = span;
#pragma unroll
            for (uint32_t d = 1; d < 64; d <<= 1) {
                const uint32_t xu = __shfl_up(x, d), yu = __shfl_up(y, d);
                if (lane >= d) {
                    x += xu;
                    y += yu;
                }
            }
            const uint32_t at = w + carry + x - ll, from = mcarry + y - span;
            for (uint32_t k = 0; k < ll; ++k) o[at + k] = msg_byte(from + k);
            carry += __shfl(x, 63);
            mcarry += __shfl(y, 63);
        }
        w += lits;
        const uint32_t hs = shb;
        if (lane < hs) o[w + lane] = (uint8_t)(seq_word >> (8u * lane));
        w += hs;
        // the tables' descriptions: literal lengths, offsets, match lengths
        const uint32_t order[3] = {0u, 2u, 1u};
#pragma unroll
        for (uint32_t i = 0; i < 3; ++i) {
            const uint32_t k = order[i];
            if (lane < dlen[k]) o[w + lane] = ((const uint8_t*)L.fdesc[k])[lane];
            w += dlen[k];
        }
        const uint32_t nb = L.sh_bytes - w;
        const uint8_t* bits = (const uint8_t*)bitw;
        for (uint32_t k = lane; k < nb; k += 64) o[w + k] = bits[k];
    }
    LZ_SYNC();
    LZ_PHASE(4)
#undef LZ_PHASE
}

extern "C" __global__ void __launch_bounds__(64 * LZ_WAVES)
tamd_lz_compress(const tamd_lz_job* __restrict__ jobs, uint32_t n_jobs, const tamd_lz_msg* __restrict__ msgs,
                 const uint8_t* __restrict__ fse, uint8_t* __restrict__ out, uint32_t* __restrict__ written,
                 uint8_t* __restrict__ scratch, unsigned long long* __restrict__ prof) {
    __shared__ LzWave W[LZ_WAVES];
    // FSE encode maps with decode info, then the table costs and flags (lz.h: the blob from
    // TAMD_FSE_E16 to its end, contiguous)
    __shared__ uint16_t e16[TAMD_FSE_E16_WORDS + LZ_COST_BYTES / 2];
    for (uint32_t i = threadIdx.x; i < (TAMD_FSE_E16_WORDS + LZ_COST_BYTES / 2) / 2; i += blockDim.x)
        ((uint32_t*)e16)[i] = ((const uint32_t*)(fse + TAMD_FSE_E16))[i];
    __syncthreads();  // (the only workgroup barrier: from here on the waves are independent)
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t ji = blockIdx.x * LZ_WAVES + wave;
    if (ji >= n_jobs) return;
    LzWave& L = W[wave];
    const tamd_lz_job job = jobs[ji];
    // profiling only (TONK_AMD_LZ_PROF): per job, 100 MHz ticks spent in each phase
    unsigned long long ph[TAMD_LZ_PHASES] = {0, 0, 0, 0, 0, 0, 0, 0}, t_ph = prof ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint8_t* __restrict__ buf = job.buf;
    const uint32_t mask = job.mask;
    uint32_t jb = 0;  // the job's base position: table entries are relative to it
    for (uint32_t i = lane; i < LZ_HASH; i += 64) L.htab[i] = 0;
    LZ_SYNC();

    // The job's window: the positions before its first message, last TAMD_LZ_WINDOW bytes of it.
    {
        const tamd_lz_msg m0 = msgs[job.first];
        uint32_t w0 = m0.win;
        if (m0.pos - w0 > TAMD_LZ_WINDOW) w0 = m0.pos - TAMD_LZ_WINDOW;
        jb = w0;
#if LZ_WINDOW_LANE16
        // 16 consecutive positions per lane: 24 bytes loaded once, 16 keys from registers (one
        // load per 64 positions, per lane, made the window phase 3x longer); inside a block of 1024
        // positions a bucket may keep an older one of its positions
        for (uint32_t q = w0; q < m0.pos; q += 1024) {
            const uint32_t p0 = q + 16u * lane;
            uint64_t a = 0, b = 0, c = 0;
            if (p0 < m0.pos) {
                a = lz_dword(buf, mask, p0);
                b = lz_dword(buf, mask, p0 + 8);
                c = lz_dword(buf, mask, p0 + 16);
            }
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) {
                uint64_t w;
                if (k == 0) w = a;
                else if (k < 8) w = (a >> (8 * k)) | (b << (64 - 8 * k));
                else if (k == 8) w = b;
                else w = (b >> (8 * (k - 8))) | (c << (64 - 8 * (k - 8)));
                lz_insert(L.htab, p0 + k < m0.pos, lz_hash(w), p0 + k + 1 - jb);
            }
        }
#else
        // 64 consecutive positions per store (in increasing order), the keys of eight stores
        // loaded at once
        for (uint32_t q = w0; q < m0.pos; q += 512) {
            uint64_t w[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) {
                const uint32_t p = q + 64u * k + lane;
                w[k] = p < m0.pos ? lz_dword(buf, mask, p) : 0ull;
            }
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) {
                const uint32_t p = q + 64u * k + lane;
                lz_insert(L.htab, p < m0.pos, lz_hash(w[k]), p + 1 - jb);
            }
        }
#endif
        LZ_SYNC();
    }
    if (prof) {
        const unsigned long long t_now = __builtin_amdgcn_s_memrealtime();
        ph[0] += t_now - t_ph;
        t_ph = t_now;
    }

    for (uint32_t mi = job.first; mi < job.first + job.count; ++mi) {
        const tamd_lz_msg m = msgs[mi];
        const uint32_t n = m.len;
        const bool big = n > TAMD_LZ_MAX_MESSAGE;
        if (n < 8 || n > TAMD_LZ_MAX_BLOCK || (big && m.scratch == TAMD_LZ_NO_SCRATCH)) {
            // (outside the kernel's bounds: stored uncompressed; its positions still enter the table)
            if (lane == 0) written[mi] = 0;
            for (uint32_t q = m.pos; q + 3 < m.pos + n; q += 64) {
                if (q + 64u - jb >= LZ_REL_MAX) lz_rebase(L.htab, jb, q - TAMD_LZ_WINDOW, lane);
                const uint32_t pp = q + lane;
                const bool ins = pp + 3 < m.pos + n;
                uint32_t h = 0;
                if (ins) h = lz_hash(lz_dword(buf, mask, pp));
                lz_insert(L.htab, ins, h, pp + 1 - jb);
            }
            LZ_SYNC();
            continue;
        }
        if (big) lz_message<true>(L, e16, fse, m, buf, mask, scratch, out, written, mi, lane, jb, ph, t_ph, prof != nullptr);
        else lz_message<false>(L, e16, fse, m, buf, mask, scratch, out, written, mi, lane, jb, ph, t_ph, prof != nullptr);
    }
    if (prof && lane == 0)
#pragma unroll
        for (uint32_t k = 0; k < TAMD_LZ_PHASES; ++k) prof[TAMD_LZ_PHASES * ji + k] = ph[k];
}

// The per-message drop-in's staging (compress.cpp): each message of a combined batch is copied
// from the batch upload into its compressor's ring at its slot, wrapping at the ring's end, with
// the ring's first TAMD_LZ_MIRROR bytes mirrored after it.  One workgroup per message.
extern "C" __global__ void __launch_bounds__(256)
tamd_lz_scatter_ring(const tamd_lz_scatter* __restrict__ d, const uint8_t* __restrict__ src) {
    const tamd_lz_scatter s = d[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < s.bytes; i += blockDim.x) {
        const uint32_t p = (s.slot + i) & (TAMD_LZ_RING - 1u);
        const uint8_t b = src[s.src + i];
        s.ring[p] = b;
        if (p < TAMD_LZ_MIRROR) s.ring[TAMD_LZ_RING + p] = b;
    }
}
