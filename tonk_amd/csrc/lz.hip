// lz.hip -- Tonk's upstream compression step (MessageCompressor, PacketCompression.h:92-140 /
// PacketCompression.cpp:70-118) on gfx950: every message becomes one zstd *compressed block*
// (RFC 8878 s3.1.1.3) that the reference's MessageDecompressor (ZSTD_decompressBlock against its
// 24 KB history ring) decodes unchanged.
//
// One wave per job; a job is a run of consecutive messages of one stream.  Matches come from the
// bytes the decompressor will hold when it decodes the message: the current history segment and
// the one before it (zstd keeps the previous contiguous segment as its external dictionary,
// zstd_decompress.c ZSTD_checkContinuity).  The block uses raw literals and the predefined FSE
// distributions for literal lengths, match lengths and offsets (no repeat offsets, so no state
// carries from block to block).
//
// Per message: (1) candidate positions from a 4-byte hash table in LDS (the window's positions
// are inserted once per job, each message's after it is scanned, 64 at a time), (2) every lane
// extends its own candidate, (3) a ballot-driven greedy parse, (4) lane 0 writes the backward
// FSE bit stream of the sequences into LDS, (5) the wave copies header, literals and bit stream
// to the output when the block is smaller than the message (else written = 0, as
// ZSTD_compressBlock's "not compressible" result, PacketCompression.cpp:96-101).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz.h"

#define LZ_HASH_LOG 12
#define LZ_HASH (1u << LZ_HASH_LOG)
#define LZ_MIN_MATCH 4u
#define LZ_MAX_SEQS (TAMD_LZ_MAX_MESSAGE / LZ_MIN_MATCH)

static __device__ __forceinline__ uint32_t lz_byte(const uint8_t* __restrict__ buf, uint32_t mask, uint32_t p) {
    return buf[p & mask];
}

static __device__ __forceinline__ uint32_t lz_word(const uint8_t* __restrict__ buf, uint32_t mask, uint32_t p) {
    return lz_byte(buf, mask, p) | (lz_byte(buf, mask, p + 1) << 8) | (lz_byte(buf, mask, p + 2) << 16) |
           (lz_byte(buf, mask, p + 3) << 24);
}

static __device__ __forceinline__ uint32_t lz_hash(uint32_t w) { return (w * 2654435761u) >> (32 - LZ_HASH_LOG); }

extern "C" __global__ void __launch_bounds__(64)
tamd_lz_compress(const tamd_lz_job* __restrict__ jobs, const tamd_lz_msg* __restrict__ msgs,
                 const uint8_t* __restrict__ fse, uint8_t* __restrict__ out, uint32_t* __restrict__ written) {
    __shared__ uint32_t htab[LZ_HASH];                       // (position + 1), 0 = empty
    __shared__ uint32_t cand[TAMD_LZ_MAX_MESSAGE];           // match source position per message byte
    __shared__ uint16_t mlen[TAMD_LZ_MAX_MESSAGE];           // match length there (0: none)
    __shared__ uint32_t seq_lo[LZ_MAX_SEQS];                 // literal length | match length << 16
    __shared__ uint32_t seq_off[LZ_MAX_SEQS];                // offset
    __shared__ uint8_t bits[TAMD_LZ_MAX_MESSAGE + 64];       // backward FSE bit stream
    __shared__ uint8_t tabs[TAMD_FSE_BYTES];                 // encode maps + decode-state info
    __shared__ uint32_t sh_nseq, sh_bytes, sh_ok;

    const uint32_t lane = threadIdx.x;
    const tamd_lz_job job = jobs[blockIdx.x];
    const uint8_t* __restrict__ buf = job.buf;
    const uint32_t mask = job.mask;

    for (uint32_t i = lane; i < TAMD_FSE_BYTES / 4; i += 64) ((uint32_t*)tabs)[i] = ((const uint32_t*)fse)[i];
    for (uint32_t i = lane; i < LZ_HASH; i += 64) htab[i] = 0;
    __syncthreads();

    // The job's window: the positions before its first message, last TAMD_LZ_WINDOW bytes of it.
    {
        const tamd_lz_msg m0 = msgs[job.first];
        uint32_t w0 = m0.win;
        if (m0.pos - w0 > TAMD_LZ_WINDOW) w0 = m0.pos - TAMD_LZ_WINDOW;
        for (uint32_t q = w0; q < m0.pos; q += 64) {
            const uint32_t p = q + lane;
            if (p < m0.pos) atomicMax(&htab[lz_hash(lz_word(buf, mask, p))], p + 1);
        }
        __syncthreads();
    }

    for (uint32_t mi = job.first; mi < job.first + job.count; ++mi) {
        const tamd_lz_msg m = msgs[mi];
        const uint32_t n = m.len;
        if (n > TAMD_LZ_MAX_MESSAGE || n < 8) {  // (outside the kernel's bounds: stored uncompressed)
            if (lane == 0) written[mi] = 0;
            for (uint32_t q = m.pos; q + 3 < m.pos + n; q += 64) {
                const uint32_t p = q + lane;
                if (p + 3 < m.pos + n) atomicMax(&htab[lz_hash(lz_word(buf, mask, p))], p + 1);
            }
            __syncthreads();
            continue;
        }
        // (1)+(2) candidates and match lengths, 64 positions at a time; a chunk's positions are
        // inserted after the chunk is scanned (matches reach back to the previous chunks)
        for (uint32_t c = 0; c < n; c += 64) {
            const uint32_t i = c + lane;
            uint32_t len = 0, src = 0;
            if (i + LZ_MIN_MATCH <= n) {
                const uint32_t p = m.pos + i;
                const uint32_t e = htab[lz_hash(lz_word(buf, mask, p))];
                if (e) {
                    src = e - 1;
                    if (src >= m.win && src < p) {
                        const uint32_t lim = n - i;
                        while (len < lim && lz_byte(buf, mask, src + len) == lz_byte(buf, mask, p + len)) ++len;
                        if (len < LZ_MIN_MATCH) len = 0;
                    }
                }
            }
            if (i < n) {
                cand[i] = src;
                mlen[i] = (uint16_t)len;
            }
            __syncthreads();
            if (i + 3 < n) atomicMax(&htab[lz_hash(lz_word(buf, mask, m.pos + i))], m.pos + i + 1);
            __syncthreads();
        }
        // (3) greedy parse: from p, the first position with a match starts the next sequence
        if (lane == 0) sh_nseq = 0;
        __syncthreads();
        uint32_t p = 0, lit_start = 0, nseq = 0;
        while (p < n) {
            const uint32_t i = p + lane;
            const bool has = i < n && mlen[i] != 0;
            const uint64_t b = __ballot(has);
            if (!b) {
                p += 64;
                continue;
            }
            const uint32_t at = p + (uint32_t)__builtin_ctzll(b);
            const uint32_t ml = mlen[at];
            if (lane == 0) {
                seq_lo[nseq] = (at - lit_start) | (ml << 16);
                seq_off[nseq] = m.pos + at - cand[at];
            }
            ++nseq;
            p = at + ml;
            lit_start = p;
        }
        const uint32_t last_lits = n - lit_start;  // literals after the last sequence
        __syncthreads();

        // (4) sizes and the sequence bit stream (lane 0)
        if (lane == 0) {
            uint32_t lits = last_lits;
            for (uint32_t s = 0; s < nseq; ++s) lits += seq_lo[s] & 0xffffu;
            uint8_t hdr[4];
            const uint32_t lh = tamd_lits_header(lits, hdr);
            const uint32_t sh = tamd_seq_header(nseq, hdr);
            const uint32_t limit = n - 1u < m.cap ? n - 1u : m.cap;  // smaller than the message, fits
            uint32_t total = lh + lits + sh;
            bool ok = total < limit && nseq > 0;
            if (ok) {
                const uint32_t nb = tamd_fse_sequences(seq_lo, seq_off, nseq, tabs, bits, limit - total);
                total += nb;
                ok = nb != 0 && total <= limit;
            }
            sh_nseq = nseq;
            sh_bytes = ok ? total : 0;
            sh_ok = ok;
            written[mi] = ok ? total : 0;
        }
        __syncthreads();
        // (5) the block: literals section header, literals, sequences header, bit stream
        if (sh_ok) {
            uint8_t* o = out + m.out;
            uint32_t lits = last_lits;
            for (uint32_t s = 0; s < sh_nseq; ++s) lits += seq_lo[s] & 0xffffu;
            uint8_t hdr[4];
            uint32_t w = tamd_lits_header(lits, hdr);
            if (lane < w) o[lane] = hdr[lane];
            // literals: the message bytes outside the matches, in order
            uint32_t src = 0;
            for (uint32_t s = 0; s <= sh_nseq; ++s) {
                const uint32_t ll = s < sh_nseq ? (seq_lo[s] & 0xffffu) : last_lits;
                for (uint32_t k = lane; k < ll; k += 64) o[w + k] = (uint8_t)lz_byte(buf, mask, m.pos + src + k);
                w += ll;
                if (s < sh_nseq) src += ll + (seq_lo[s] >> 16);
            }
            const uint32_t hs = tamd_seq_header(sh_nseq, hdr);
            if (lane < hs) o[w + lane] = hdr[lane];
            w += hs;
            const uint32_t nb = sh_bytes - w;
            for (uint32_t k = lane; k < nb; k += 64) o[w + k] = bits[k];
        }
        __syncthreads();
    }
}
