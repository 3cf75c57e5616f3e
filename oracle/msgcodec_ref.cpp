// msgcodec_ref.cpp -- TEST INFRASTRUCTURE (oracle for the compression step).
// Tonk's MessageCompressor / MessageDecompressor (PacketCompression.cpp:28-216) restated over
// the reference's own zstd (thirdparty/zstd, compiled from /root/reference by oracle/Makefile):
// the same 24,000-byte history ring with the Allocate(max)/Commit rule (PacketCompression.h:36-63),
// ZSTD_compressBlock at level 1 with the same parameters, ZSTD_decompressBlock /
// ZSTD_insertBlock on the receive side.  Used only by tests/ (decompressing the GPU's blocks) and
// by bench.py's cpu_baseline leg (timing the reference compressor); never by the product.
#define ZSTD_STATIC_LINKING_ONLY
#include "zstd/zstd.h"
#include "zstd/zstd_errors.h"

#include <stdint.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

namespace {

const unsigned kDictBytes = 24 * 1000;  // kCompressionDictBytes (PacketCompression.h:40)
const int kLevel = 1;                   // kCompressionLevel (PacketCompression.h:39)

struct Ring {  // RingBuffer<kBufferBytes> (PacketCompression.h:44-63)
    uint8_t buf[kDictBytes];
    unsigned next = 0;
    uint8_t* allocate(unsigned bytes) {
        if (next + bytes > kDictBytes) next = 0;
        return buf + next;
    }
    void commit(unsigned bytes) { next += bytes; }
};

struct Comp {
    Ring hist;
    ZSTD_CCtx* cctx = nullptr;
    unsigned max = 0;
};

struct Decomp {
    Ring hist;
    ZSTD_DCtx* dctx = nullptr;
    unsigned max = 0;
};

}  // namespace

extern "C" {

// MessageCompressor::Initialize (PacketCompression.cpp:28-61)
void* ref_comp_new(unsigned max) {
    Comp* c = new Comp();
    c->max = max;
    c->cctx = ZSTD_createCCtx();
    ZSTD_parameters zp;
    zp.cParams = ZSTD_getCParams(kLevel, max, kDictBytes);
    zp.fParams.checksumFlag = 0;
    zp.fParams.contentSizeFlag = 0;
    zp.fParams.noDictIDFlag = 1;
    if (!c->cctx || ZSTD_isError(ZSTD_compressBegin_advanced(c->cctx, nullptr, 0, zp, ZSTD_CONTENTSIZE_UNKNOWN)) ||
        ZSTD_getBlockSize(c->cctx) < max) {
        if (c->cctx) ZSTD_freeCCtx(c->cctx);
        delete c;
        return nullptr;
    }
    return c;
}

// MessageCompressor::Compress (PacketCompression.cpp:70-118): 0 ok (written 0 = uncompressed)
int ref_comp(void* cp, const uint8_t* data, unsigned bytes, uint8_t* dest, unsigned* written) {
    Comp* c = (Comp*)cp;
    *written = 0;
    uint8_t* h = c->hist.allocate(c->max);
    memcpy(h, data, bytes);
    c->hist.commit(bytes);
    const size_t r = ZSTD_compressBlock(c->cctx, dest, c->max, h, bytes);
    if (r == 0 || r == (size_t)-ZSTD_error_dstSize_tooSmall || r >= bytes) return 0;
    if (ZSTD_isError(r)) return -1;
    *written = (unsigned)r;
    return 0;
}

void ref_comp_free(void* cp) {
    Comp* c = (Comp*)cp;
    if (!c) return;
    ZSTD_freeCCtx(c->cctx);
    delete c;
}

// MessageDecompressor::Initialize (PacketCompression.cpp:136-152)
void* ref_decomp_new(unsigned max) {
    Decomp* d = new Decomp();
    d->max = max;
    d->dctx = ZSTD_createDCtx();
    if (!d->dctx || ZSTD_isError(ZSTD_decompressBegin(d->dctx))) {
        if (d->dctx) ZSTD_freeDCtx(d->dctx);
        delete d;
        return nullptr;
    }
    return d;
}

// MessageDecompressor::InsertUncompressed (PacketCompression.cpp:162-176)
void ref_insert(void* dp, const uint8_t* data, unsigned bytes) {
    Decomp* d = (Decomp*)dp;
    if (bytes > d->max) return;
    uint8_t* h = d->hist.allocate(d->max);
    memcpy(h, data, bytes);
    ZSTD_insertBlock(d->dctx, h, bytes);
    d->hist.commit(bytes);
}

// MessageDecompressor::Decompress (PacketCompression.cpp:178-208): bytes restored into out, or -1
int ref_decomp(void* dp, const uint8_t* src, unsigned bytes, uint8_t* out, unsigned out_cap) {
    Decomp* d = (Decomp*)dp;
    uint8_t* h = d->hist.allocate(d->max);
    const size_t r = ZSTD_decompressBlock(d->dctx, h, d->max, src, bytes);
    if (r == 0 || ZSTD_isError(r) || r > out_cap) return -1;
    memcpy(out, h, r);
    d->hist.commit((unsigned)r);
    return (int)r;
}

void ref_decomp_free(void* dp) {
    Decomp* d = (Decomp*)dp;
    if (!d) return;
    ZSTD_freeDCtx(d->dctx);
    delete d;
}

// CPU baseline: n_streams fresh compressors, stream s's n_msgs messages back to back at
// data + s * stride (lens per message), split over `threads` host threads, repeated `reps`
// times.  Returns seconds; *in_bytes / *out_bytes (optional) sum the last repetition.
double ref_comp_bench(const uint8_t* data, uint64_t stride, unsigned n_streams, unsigned n_msgs,
                      const unsigned* lens, unsigned max, unsigned threads, unsigned reps, uint64_t* in_bytes,
                      uint64_t* out_bytes) {
    std::atomic<uint64_t> tin(0), tout(0);
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned rep = 0; rep < reps; ++rep) {
        std::atomic<unsigned> next(0);
        tin = 0;
        tout = 0;
        auto work = [&]() {
            std::vector<uint8_t> dest(max + 64);
            for (;;) {
                const unsigned s = next++;
                if (s >= n_streams) break;
                void* c = ref_comp_new(max);
                if (!c) break;
                const uint8_t* p = data + (uint64_t)s * stride;
                uint64_t i = 0, o = 0;
                for (unsigned k = 0; k < n_msgs; ++k) {
                    const unsigned n = lens[(uint64_t)s * n_msgs + k];
                    unsigned w = 0;
                    ref_comp(c, p, n, dest.data(), &w);
                    p += n;
                    i += n;
                    o += w ? w : n;
                }
                ref_comp_free(c);
                tin += i;
                tout += o;
            }
        };
        std::vector<std::thread> ts;
        for (unsigned t = 0; t < threads; ++t) ts.emplace_back(work);
        for (auto& t : ts) t.join();
    }
    if (in_bytes) *in_bytes = tin;
    if (out_bytes) *out_bytes = tout;
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // extern "C"
