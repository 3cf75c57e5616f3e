// lz_check.cpp -- TEST ONLY.  Checks the zstd block writer the compression kernel uses (the
// host+device helpers of tonk_amd/csrc/lz.h: FSE tables of the predefined distributions,
// literal/sequence headers, the backward sequence bit stream) against the reference's zstd
// decoder (oracle/_ref/libmsgcodec_ref.so, MessageDecompressor restated over thirdparty/zstd),
// with a plain greedy matcher standing in for the kernel's parse.  The GPU tests run the kernel
// itself against the same decoder.
//
// usage: lz_check [messages] [seed]   -> prints "ok <compressed> <total>" or the first mismatch
#include "../../tonk_amd/csrc/lz.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

extern "C" {
void* ref_decomp_new(unsigned max);
void ref_insert(void* d, const uint8_t* data, unsigned bytes);
int ref_decomp(void* d, const uint8_t* src, unsigned bytes, uint8_t* out, unsigned cap);
void ref_decomp_free(void* d);
}

static uint32_t rng_state = 1;
static bool g_huffman = true;
static uint32_t g_minmatch = 4;
static bool g_fitted = true;  // block-fitted sequence tables (tamd_seq_choose)
static unsigned fitted_tables[3] = {0, 0, 0}, rle_tables[3] = {0, 0, 0};
static unsigned huffman_blocks = 0;
static uint64_t lit_bytes = 0, seq_bytes = 0, n_seqs = 0, lit_small = 0;
static double est_fitted = 0;  // estimated bytes of the sequence streams with block-fitted tables
#include <math.h>
static uint32_t rnd() {
    rng_state = rng_state * 1664525u + 1013904223u;
    return rng_state >> 8;
}

int main(int argc, char** argv) {
    const unsigned n_msgs = argc > 1 ? (unsigned)atoi(argv[1]) : 400;
    rng_state = argc > 2 ? (uint32_t)atoi(argv[2]) : 1;
    g_huffman = argc > 3 ? atoi(argv[3]) != 0 : true;
    g_minmatch = argc > 4 ? (uint32_t)atoi(argv[4]) : 4;
    g_fitted = argc > 5 ? atoi(argv[5]) != 0 : true;
    const unsigned kMax = 1300, kDict = 24000;
    uint8_t fse[TAMD_FSE_BYTES];
    tamd_fse_blob(fse);
    {  // the kernel's packed maps agree with the encoder/decoder tables the host writer uses
        const uint16_t* e16 = (const uint16_t*)(fse + TAMD_FSE_E16);
        const struct { uint32_t enc, dec, e, nsym, size; } t[3] = {
            {TAMD_FSE_LL_ENC, TAMD_FSE_LL_DEC, TAMD_FSE_LL_E16, 36, 64},
            {TAMD_FSE_ML_ENC, TAMD_FSE_ML_DEC, TAMD_FSE_ML_E16, 53, 64},
            {TAMD_FSE_OF_ENC, TAMD_FSE_OF_DEC, TAMD_FSE_OF_E16, 29, 32}};
        for (const auto& c : t)
            for (uint32_t sy = 0; sy < c.nsym; ++sy)
                for (uint32_t y = 0; y < c.size; ++y) {
                    const uint32_t u = fse[c.enc + sy * c.size + y], w = e16[c.e + sy * c.size + y];
                    if ((w & 63u) != u || ((w >> 6) & 15u) != fse[c.dec + 2 * u] || (w >> 10) != y - fse[c.dec + 2 * u + 1]) {
                        printf("packed FSE map differs (symbol %u, state %u)\n", sy, y);
                        return 1;
                    }
                }
    }
    // a stream of messages: words from a small vocabulary, random bytes, repeats of old messages
    std::vector<uint8_t> stream;
    std::vector<unsigned> lens;
    const char* words[] = {"siamese ", "tonk ", "packet ", "recovery ", "window ", "lane ", "sum ", "ack ", "0123 "};
    for (unsigned k = 0; k < n_msgs; ++k) {
        const unsigned n = 8 + rnd() % (kMax - 8);
        const unsigned kind = rnd() % 4;
        const size_t at = stream.size();
        if (kind == 3 && at > 4000) {  // repeat an earlier stretch
            const size_t from = at - 1 - rnd() % (at < 40000 ? at - 1 : 40000);
            for (unsigned i = 0; i < n; ++i) stream.push_back(stream[from + i < at ? from + i : at - 1]);
        } else {
            for (unsigned i = 0; i < n;) {
                if (kind == 0) {
                    stream.push_back((uint8_t)rnd());
                    ++i;
                } else if (kind == 2) {  // novel text: skewed letters (Huffman-coded literals)
                    const uint32_t r = rnd() % 100;
                    stream.push_back((uint8_t)(r < 40 ? 'e' + r % 4 : r < 80 ? 'a' + r % 12 : ' ' + r % 64));
                    ++i;
                } else {
                    const char* w = words[rnd() % 9];
                    for (const char* c = w; *c && i < n; ++c, ++i) stream.push_back((uint8_t)*c);
                }
            }
        }
        lens.push_back(n);
    }
    void* dec = ref_decomp_new(kMax);
    // ring bookkeeping of compress.cpp (RingTrack) restated for the check
    unsigned next = 0;
    uint64_t lin = 0, seg = 0, prev = 0;
    bool have_prev = false;
    std::vector<int64_t> table(1u << 14, -1);
    uint64_t total_in = 0, total_out = 0;
    unsigned compressed = 0;
    std::vector<uint8_t> out(2 * kMax + 64), got(kMax + 64);
    for (unsigned k = 0; k < n_msgs; ++k) {
        const unsigned n = lens[k];
        if (next + kMax > kDict) {
            if (next) {
                prev = seg;
                have_prev = true;
                seg = lin;
            }
            next = 0;
        }
        const uint64_t pos = lin;
        uint64_t win = seg;
        if (have_prev) win = prev + next + n < seg ? prev + next + n : seg;
        // greedy parse
        std::vector<uint32_t> lo, off;
        const uint8_t* s = stream.data();
        auto hash = [&](uint64_t p) {
            uint32_t w;
            memcpy(&w, s + p, 4);
            return (w * 2654435761u) >> 18;
        };
        uint32_t lit_start = 0, i = 0;
        while (i + 4 <= n) {
            const uint64_t p = pos + i;
            const int64_t c = table[hash(p)];
            table[hash(p)] = (int64_t)p;
            uint32_t len = 0;
            if (c >= 0 && (uint64_t)c >= win && (uint64_t)c < p)
                while (len < n - i && s[c + len] == s[p + len]) ++len;
            if (len >= g_minmatch) {
                lo.push_back((i - lit_start) | (len << 16));
                off.push_back((uint32_t)(p - (uint64_t)c));
                for (uint32_t j = 1; j < len && i + j + 4 <= n; ++j) table[hash(p + j)] = (int64_t)(p + j);
                i += len;
                lit_start = i;
            } else {
                ++i;
            }
        }
        unsigned w = 0;
        if (!lo.empty()) {
            uint32_t lits = n - lit_start;
            for (uint32_t v : lo) lits += v & 0xffffu;
            uint8_t h[4];
            // the literals in order, then the smaller of the raw and Huffman sections
            std::vector<uint8_t> litbuf;
            uint32_t src = 0;
            for (size_t q = 0; q <= lo.size(); ++q) {
                const uint32_t ll = q < lo.size() ? (lo[q] & 0xffffu) : n - lit_start;
                litbuf.insert(litbuf.end(), s + pos + src, s + pos + src + ll);
                if (q < lo.size()) src += ll + (lo[q] >> 16);
            }
            uint32_t count[TAMD_HUF_SYMS] = {0};
            bool small = true;
            for (uint8_t c : litbuf) {
                if (c >= TAMD_HUF_SYMS) small = false;
                else ++count[c];
            }
            const uint32_t raw = tamd_lits_header(lits, out.data()) + lits;
            lit_bytes += lits;
            n_seqs += lo.size();
            if (small) lit_small += lits;
            uint32_t huf = 0;
            std::vector<uint8_t> hsec(raw + 64);
            if (g_huffman && small) huf = tamd_huf_section(litbuf.data(), lits, count, hsec.data(), raw);
            if (huf && huf < raw) {
                memcpy(out.data(), hsec.data(), huf);
                w = huf;
                ++huffman_blocks;
            } else {
                w = tamd_lits_header(lits, out.data());
                memcpy(&out[w], litbuf.data(), lits);
                w += lits;
            }
            const uint32_t hs = tamd_seq_header((uint32_t)lo.size(), h);
            // the block's tables: codes packed as the kernel packs them
            tamd_seq_tables tt;
            std::vector<uint32_t> codes(lo.size());
            for (size_t q = 0; q < lo.size(); ++q)
                codes[q] = tamd_ll_code(lo[q] & 0xffffu) | (tamd_ml_code(lo[q] >> 16) << 8) |
                           ((31u - (uint32_t)__builtin_clz(off[q] + 3u)) << 16);
            uint32_t dl = 0;
            if (g_fitted) {
                dl = tamd_seq_choose(codes.data(), (uint32_t)codes.size(), fse, &tt);
                h[hs - 1] = (uint8_t)tamd_modes_byte(tt.mode);
                for (uint32_t k = 0; k < 3; ++k) {
                    if (tt.mode[k] == TAMD_MODE_FSE) ++fitted_tables[k];
                    if (tt.mode[k] == TAMD_MODE_RLE) ++rle_tables[k];
                }
            }
            memcpy(&out[w], h, hs);
            w += hs;
            if (g_fitted) {
                const uint32_t order[3] = {0u, 2u, 1u};  // descriptions: LL, OF, ML
                for (uint32_t k : order) {
                    memcpy(&out[w], tt.desc[k], tt.desc_len[k]);
                    w += tt.desc_len[k];
                }
            }
            if (w < n - 1) {
                const uint32_t nb = tamd_fse_sequences_t(lo.data(), off.data(), (uint32_t)lo.size(), fse,
                                                         g_fitted ? &tt : nullptr, &out[w], n - 1 - w);
                if (!g_fitted) {  // the packed-map writer agrees with the table writer
                    std::vector<uint8_t> alt(n);
                    const uint32_t nb2 = tamd_fse_sequences(lo.data(), off.data(), (uint32_t)lo.size(), fse, alt.data(),
                                                            n - 1 - w);
                    if (nb2 != nb || memcmp(alt.data(), &out[w], nb) != 0) {
                        printf("sequence writers differ at message %u\n", k);
                        return 1;
                    }
                }
                seq_bytes += nb + hs + dl;
                {  // entropy of the three code streams per block + the same extra bits + ~8 B of table headers each
                    uint32_t hl[64] = {0}, hm[64] = {0}, ho[32] = {0};
                    double extra = 0;
                    for (size_t q = 0; q < lo.size(); ++q) {
                        const uint32_t llc = tamd_ll_code(lo[q] & 0xffffu), mlc = tamd_ml_code(lo[q] >> 16);
                        const uint32_t ofc = 31u - (uint32_t)__builtin_clz(off[q] + 3u);
                        ++hl[llc]; ++hm[mlc]; ++ho[ofc];
                        extra += tamd_ll_bits(llc) + tamd_ml_bits(mlc) + ofc;
                    }
                    auto ent = [&](const uint32_t* h, int k) {
                        double e = 0, t = (double)lo.size();
                        for (int i = 0; i < k; ++i) if (h[i]) e -= h[i] * log2(h[i] / t);
                        return e;
                    };
                    est_fitted += (ent(hl, 64) + ent(hm, 64) + ent(ho, 32) + extra) / 8.0 + 3 * 8 + hs;
                }
                w = nb ? w + nb : 0;
            } else {
                w = 0;
            }
        }
        if (w && w < n) {
            const int r = ref_decomp(dec, out.data(), w, got.data(), (unsigned)got.size());
            if (r != (int)n || memcmp(got.data(), s + pos, n) != 0) {
                printf("mismatch at message %u (n %u, block %u bytes, %zu sequences, rc %d)\n", k, n, w, lo.size(), r);
                return 1;
            }
            ++compressed;
            total_out += w;
        } else {
            ref_insert(dec, s + pos, n);
            total_out += n;
        }
        total_in += n;
        next += n;
        lin += n;
    }
    ref_decomp_free(dec);
    fprintf(stderr, "sequence sections now %llu bytes, with block-fitted tables about %.0f\n",
            (unsigned long long)seq_bytes, est_fitted);
    fprintf(stderr, "literal bytes %llu (in Huffman-able sections %llu), sequences %llu in %llu bytes\n",
            (unsigned long long)lit_bytes, (unsigned long long)lit_small, (unsigned long long)n_seqs,
            (unsigned long long)seq_bytes);
    fprintf(stderr, "fitted tables LL/ML/OF %u/%u/%u, RLE %u/%u/%u\n", fitted_tables[0], fitted_tables[1],
            fitted_tables[2], rle_tables[0], rle_tables[1], rle_tables[2]);
    printf("ok %u/%u compressed (%u with Huffman literals), %llu -> %llu bytes\n", compressed, n_msgs,
           huffman_blocks, (unsigned long long)total_in, (unsigned long long)total_out);
    return 0;
}
