// transcript.h -- text transcript of one workload stream, written the
// same way for every backend so runs can be compared line by line against the reference.
//
// Lines:
//   E rc len row cs sc ldpc h     encode: packet bytes (data+footer), footer metadata, FNV-1a
//   D rc n [num:len:h ...]        decode result and recovered packets (len = payload bytes)
//   K rd used h re next           decoder ack (result, bytes, digest) -> encoder ack result
//   a|O|R|X|T rc x y              add/original/recovery/ARQ/retransmit-delivery events with a
//                                 non-zero result
//   T rc [num bytes h]            siamese_encoder_retransmit: result, packet, payload digest
//   S e0..e7 d0..d9               final stats (the allocator-dependent MemoryUsed is omitted)
#pragma once
#include <stdio.h>
#include <stdarg.h>
#include <stdint.h>
#include <string>
#include <vector>

namespace tamd {
namespace wl {

struct TextSink {
    std::string text;
    void line(const char* s) { text += s; text += '\n'; }
    void put(const char* fmt, ...) __attribute__((format(printf, 2, 3))) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        text += buf;
    }
};

inline void fmt_retransmit(TextSink& t, int rc, uint32_t num, uint32_t bytes, uint64_t h) {
    if (rc != 0) t.put("T %d\n", rc);
    else t.put("T 0 %u %u %016llx\n", num, bytes, (unsigned long long)h);
}

inline void fmt_stats(TextSink& t, const uint64_t enc[9], const uint64_t dec[11]) {
    t.put("S");
    for (int i = 0; i < 8; ++i) t.put(" %llu", (unsigned long long)enc[i]);
    t.put(" |");
    for (int i = 0; i < 10; ++i) t.put(" %llu", (unsigned long long)dec[i]);
    t.put("\n");
}

} // namespace wl
} // namespace tamd
