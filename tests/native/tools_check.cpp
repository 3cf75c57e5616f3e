// tools_check.cpp -- TEST ONLY.  Exercises the helpers Tonk takes from SiameseTools.h and
// SiameseSerializers.h (PCGRandom, the LE readers/writers, Write/ReadByteStream, WindowedMinMax
// with both orderings) on seeded random inputs and prints every result.  Built twice: against
// include/ (tonk_amd's header-compatible versions: tests/native/_build/tools_check) and against
// the reference headers (oracle/Makefile: oracle/_ref/tools_check_ref); tests/test_tools_headers.py
// requires identical output.  Clocks are not compared (they read the wall clock).
#include "SiameseSerializers.h"
#include "SiameseTools.h"

#include <stdio.h>
#include <stdint.h>
#include <string.h>

using namespace siamese;

static uint64_t g_hash = 1469598103934665603ULL;
static void mix(uint64_t v) {
    for (int i = 0; i < 8; ++i) {
        g_hash ^= (uint8_t)(v >> (8 * i));
        g_hash *= 1099511628211ULL;
    }
}

int main() {
    // PCGRandom: several seeds, first outputs printed, the rest hashed.
    for (uint64_t y = 0; y < 6; ++y) {
        PCGRandom p;
        p.Seed(y * 0x9E3779B97F4A7C15ull, y * 7 + 1);
        printf("pcg %llu:", (unsigned long long)y);
        for (int i = 0; i < 4; ++i) printf(" %08x", p.Next());
        for (int i = 0; i < 10000; ++i) mix(p.Next());
        printf(" | %016llx %016llx\n", (unsigned long long)p.State, (unsigned long long)p.Inc);
        PCGRandom q;
        q.Seed(y);  // default x
        mix(q.Next());
    }
    printf("pcg hash %016llx\n", (unsigned long long)g_hash);

    // Serializers: every reader over random bytes, every writer into a poisoned buffer.
    PCGRandom r;
    r.Seed(12345, 678);
    g_hash = 1469598103934665603ULL;
    for (int it = 0; it < 20000; ++it) {
        uint8_t buf[16];
        for (int i = 0; i < 16; ++i) buf[i] = (uint8_t)r.Next();
        const unsigned o = r.Next() % 8;
        mix(ReadU16_LE(buf + o));
        mix(ReadU24_LE(buf + o));
        mix(ReadU24_LE_Min4Bytes(buf + o));
        mix(ReadU32_LE(buf + o));
        mix(ReadU64_LE(buf + o));
        const uint64_t v = ((uint64_t)r.Next() << 32) | r.Next();
        uint8_t out[16];
        memset(out, 0xA5, sizeof(out));
        switch (it % 6) {
            case 0: WriteU16_LE(out + o, (uint16_t)v); break;
            case 1: WriteU24_LE(out + o, (uint32_t)v); break;
            case 2: WriteU24_LE_Min4Bytes(out + o, (uint32_t)v); break;
            case 3: WriteU32_LE(out + o, (uint32_t)v); break;
            case 4: WriteU64_LE(out + o, v); break;
            default: WriteU24_LE_Min4Bytes(out + o, (uint32_t)v & 0xFFFFFF); break;
        }
        for (int i = 0; i < 16; ++i) mix(out[i]);
    }
    printf("serial hash %016llx\n", (unsigned long long)g_hash);

    // Byte streams: a random script of writes, then the same reads.
    g_hash = 1469598103934665603ULL;
    for (int it = 0; it < 2000; ++it) {
        uint8_t buf[512];
        memset(buf, 0x5A, sizeof(buf));
        WriteByteStream w(buf, sizeof(buf));
        uint8_t ops[64];
        int n = 0;
        while (n < 64) {
            const uint8_t op = (uint8_t)(r.Next() % 6);
            const unsigned need = op == 0 ? 1 : op == 1 ? 2 : op == 2 ? 3 : op == 3 ? 4 : op == 4 ? 8 : 5;
            if (w.Remaining() < need) break;
            const uint64_t v = ((uint64_t)r.Next() << 32) | r.Next();
            switch (op) {
                case 0: w.Write8((uint8_t)v); break;
                case 1: w.Write16((uint16_t)v); break;
                case 2: w.Write24((uint32_t)v); break;
                case 3: w.Write32((uint32_t)v); break;
                case 4: w.Write64(v); break;
                default: { uint8_t src[5]; memcpy(src, &v, 5); w.WriteBuffer(src, 5); break; }
            }
            ops[n++] = op;
        }
        mix(w.WrittenBytes);
        mix(w.Remaining());
        mix((uint64_t)(w.Peek() - buf));
        for (int i = 0; i < 512; ++i) mix(buf[i]);
        ReadByteStream rd(buf, w.WrittenBytes);
        for (int i = 0; i < n; ++i) {
            switch (ops[i]) {
                case 0: mix(rd.Read8()); break;
                case 1: mix(rd.Read16()); break;
                case 2: mix(rd.Read24()); break;
                case 3: mix(rd.Read32()); break;
                case 4: mix(rd.Read64()); break;
                default: { const uint8_t* p = rd.Read(5); for (int k = 0; k < 5; ++k) mix(p[k]); break; }
            }
            mix(rd.Remaining());
            mix(rd.BytesRead);
        }
        rd.Skip(0);
        mix((uint64_t)(rd.Peek() - buf));
    }
    printf("stream hash %016llx\n", (unsigned long long)g_hash);

    // WindowedMinMax, both orderings, with timestamps that jump, stall and wrap, and resets.
    typedef WindowedMinMax<unsigned, WindowedMinCompare<unsigned> > WinMin;
    typedef WindowedMinMax<unsigned, WindowedMaxCompare<unsigned> > WinMax;
    typedef WindowedMinMax<uint32_t, WindowedMinCompare<uint32_t> > WinMin32;
    for (int variant = 0; variant < 4; ++variant) {
        WinMin mn;
        WinMax mx;
        WinMin32 m32;
        mn.Reset();
        mx.Reset();
        m32.Reset();
        g_hash = 1469598103934665603ULL;
        uint64_t t = variant == 3 ? ~0ull - 5000 : 1000;  // variant 3: the clock wraps
        const uint64_t window = variant == 0 ? 100 : variant == 1 ? 1000 : 250;
        for (int i = 0; i < 50000; ++i) {
            const uint32_t step = r.Next() % (variant == 2 ? 200 : 40);
            t += step;
            const unsigned vmin = 1 + r.Next() % (variant == 1 ? 1000 : 60);
            const unsigned vmax = r.Next() % 500;
            mn.Update(vmin, t, window);
            mx.Update(vmax, t, window);
            m32.Update((uint32_t)(vmin * 3 + (i & 7)), t, window / 2);
            mix(mn.GetBest());
            mix(mx.GetBest());
            mix(m32.GetBest());
            mix(mn.IsValid());
            mix(mx.IsValid());
            for (unsigned k = 0; k < WinMin::kSampleCount; ++k) {
                mix(mn.Samples[k].Value);
                mix(mn.Samples[k].Timestamp);
                mix(mx.Samples[k].Value);
                mix(mx.Samples[k].Timestamp);
            }
            if (r.Next() % 5000 == 0) mx.Reset(WinMax::Sample(vmax, t));
            if (r.Next() % 7000 == 0) mn.Reset();
        }
        printf("winminmax %d: min %u max %u m32 %u hash %016llx\n", variant, mn.GetBest(), mx.GetBest(), m32.GetBest(),
               (unsigned long long)g_hash);
    }
    printf("SIAMESE_PACKET_NUM_INC %u %u\n", (unsigned)SIAMESE_PACKET_NUM_INC(5u), (unsigned)SIAMESE_PACKET_NUM_INC(0x3fffffu));
    return 0;
}
