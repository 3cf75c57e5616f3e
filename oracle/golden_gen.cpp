// golden_gen.cpp -- TEST INFRASTRUCTURE.  Runs the synthetic workload (tonk_amd/csrc/workload.h)
// against the REFERENCE codec compiled from /root/reference (oracle/_ref/libsiamese_ref.so) and
//   * writes the per-stream transcript (tests/golden fixtures), or
//   * times the reference CPU path over many streams on host threads (bench.py cpu_baseline).
//
// Only siamese.h API calls are made; nothing of the reference is copied.  Every recovered
// packet is also checked against the true payload so a fixture can never pin a wrong decode.
//
// usage: golden_gen transcript <out.txt> key=value...
//        golden_gen transcripts <prefix> threads=T streams=S key=value...
//                   (streams stream..stream+S-1 concurrently on T threads, one codec pair each;
//                    <prefix><id>.txt per stream -- the C ABI's concurrent-codec check)
//        golden_gen time threads=T streams=S reps=R key=value...
#include "siamese.h"

#include "../tonk_amd/csrc/workload.h"
#include "../tonk_amd/csrc/transcript.h"

#include <algorithm>
#include <chrono>
#include <dlfcn.h>
#include <sys/resource.h>
#include <functional>
#include <thread>
#include <atomic>
#include <memory>
#include <stdlib.h>
#include <string.h>

using namespace tamd::wl;

// Virtual millisecond clock of retransmit scenarios (workload.h rtx_every): per thread, so
// concurrent streams each run on their own clock.  The reference codec reads the time through
// siamese::GetTimeMsec (SiameseTools.h:110; SiameseEncoder.cpp:142, 595, 905); this executable
// defines that symbol (linked with -rdynamic) so the reference library's calls resolve here.
// The MI355X library takes the same clock through its tamd_set_clock hook (looked up at run
// time, since this driver is linked against either library).
static thread_local bool g_vclock_on = false;
static thread_local uint64_t g_vclock_ms = 0;
static uint64_t real_usec() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}
static uint64_t vclock_msec() { return g_vclock_on ? g_vclock_ms : real_usec() / 1000; }
namespace siamese {
uint64_t GetTimeUsec() { return g_vclock_on ? g_vclock_ms * 1000 : real_usec(); }
uint64_t GetTimeMsec() { return vclock_msec(); }
}  // namespace siamese

// `lat=1` (time mode): the duration of every siamese_encode and siamese_decode call, per thread
// (the drop-in's per-call latency: TonkineseOutgoing.cpp:1284-1328 calls siamese_encode inline).
static bool g_lat = false;
struct LatLog { std::vector<uint32_t> enc_ns, dec_ns; };
static thread_local LatLog* g_latlog = nullptr;
static inline uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}
// `prof=1` (time mode): nanoseconds spent in each kind of siamese.h call, summed per thread, and
// each thread's busy time -- where a pass's time goes (diagnostics; adds two clock reads per call).
enum { P_ADD, P_ENCODE, P_EACK, P_DADD, P_DREC, P_READY, P_DECODE, P_DACK, P_N };
static bool g_prof = false;
static thread_local uint64_t* g_profv = nullptr;
struct ProfScope {
    int k;
    uint64_t t0;
    explicit ProfScope(int kind) : k(kind), t0(g_profv ? now_ns() : 0) {}
    ~ProfScope() { if (g_profv) g_profv[k] += now_ns() - t0; }
};

struct RefBackend {
    struct RecRef { std::vector<uint8_t> bytes; };
    struct DecRef { std::vector<std::vector<uint8_t>> data; };

    const Params& p;
    SiameseEncoder enc = nullptr;
    SiameseDecoder dec = nullptr;
    std::vector<uint8_t> payloads;   // all payloads, pregenerated (index * stride)
    std::vector<uint32_t> lens;
    uint32_t stride = 0;
    uint64_t bad_recoveries = 0;
    uint32_t top = 0;  // originals added (recovered packet numbers are 22-bit columns)

    // `pool` > 0 (timing only): payloads of the first `pool` indices, reused cyclically (original
    // i carries the bytes of i mod pool), so a long stream does not need its whole payload set in
    // host memory; the codec's work does not depend on the bytes, and recovered packets are
    // still checked against what was sent.
    uint32_t pool = 0;
    explicit RefBackend(const Params& prm, uint32_t pool_n = 0) : p(prm) {
        enc = siamese_encoder_create();
        dec = siamese_decoder_create();
        stride = prm.payload_max;
        // (equal lengths only: the runner passes payload_length(i) with every packet)
        pool = pool_n && pool_n < prm.n_originals && prm.payload_min == prm.payload_max ? pool_n : prm.n_originals;
        payloads.resize((size_t)stride * pool);
        lens.resize(pool);
        for (uint32_t i = 0; i < pool; ++i) {
            lens[i] = payload_length(prm, i);
            payload_bytes(prm, i, payloads.data() + (size_t)i * stride, lens[i]);
        }
    }
    uint32_t len_of(uint32_t i) const { return lens[i % pool]; }
    ~RefBackend() {
        siamese_encoder_free(enc);
        siamese_decoder_free(dec);
    }
    // Fresh codecs for a repeated run over the same (already generated) payloads.
    void reset_codecs() {
        siamese_encoder_free(enc);
        siamese_decoder_free(dec);
        enc = siamese_encoder_create();
        dec = siamese_decoder_create();
    }
    const uint8_t* pay(uint32_t i) const { return payloads.data() + (size_t)(i % pool) * stride; }

    int enc_add(uint32_t index, uint32_t len, uint32_t* col) {
        SiameseOriginalPacket o;
        o.PacketNum = 0;
        o.Data = pay(index);
        o.DataBytes = len;
        ProfScope ps(P_ADD);
        const int rc = siamese_encoder_add(enc, &o);
        *col = o.PacketNum;
        if (rc == 0) top = index + 1;
        return rc;
    }
    int enc_is_ready() { return siamese_encoder_is_ready(enc); }
    int enc_encode(RecRef& r) {
        SiameseRecoveryPacket rp;
        rp.Data = nullptr;
        rp.DataBytes = 0;
        const uint64_t t0 = g_latlog ? now_ns() : 0;
        ProfScope ps(P_ENCODE);
        const int rc = siamese_encode(enc, &rp);
        if (g_latlog) g_latlog->enc_ns.push_back((uint32_t)std::min<uint64_t>(now_ns() - t0, 0xffffffffu));
        if (rc == 0) r.bytes.assign(rp.Data, rp.Data + rp.DataBytes);
        return rc;
    }
    int enc_ack(const uint8_t* buf, uint32_t n, uint32_t* next) {
        ProfScope ps(P_EACK);
        return siamese_encoder_ack(enc, buf, n, next);
    }
    int dec_add_original(uint32_t col, uint32_t index, uint32_t len) {
        SiameseOriginalPacket o;
        o.PacketNum = col;
        o.Data = pay(index);
        o.DataBytes = len;
        ProfScope ps(P_DADD);
        return siamese_decoder_add_original(dec, &o);
    }
    int dec_add_recovery(const RecRef& r) {
        SiameseRecoveryPacket rp;
        rp.Data = r.bytes.data();
        rp.DataBytes = (unsigned)r.bytes.size();
        ProfScope ps(P_DREC);
        return siamese_decoder_add_recovery(dec, &rp);
    }
    void recovery_lost(const RecRef&) {}
    int dec_is_ready() {
        ProfScope ps(P_READY);
        return siamese_decoder_is_ready(dec);
    }
    int dec_decode(std::vector<uint32_t>& nums, DecRef& out) {
        SiameseOriginalPacket* pk = nullptr;
        unsigned count = 0;
        const uint64_t t0 = g_latlog ? now_ns() : 0;
        ProfScope ps(P_DECODE);
        const int rc = siamese_decode(dec, &pk, &count);
        if (g_latlog) g_latlog->dec_ns.push_back((uint32_t)std::min<uint64_t>(now_ns() - t0, 0xffffffffu));
        if (rc == 0) {
            for (unsigned k = 0; k < count; ++k) {
                nums.push_back(pk[k].PacketNum);
                out.data.emplace_back(pk[k].Data, pk[k].Data + pk[k].DataBytes);
                const uint32_t idx = index_of_column(pk[k].PacketNum, top);
                if (idx >= p.n_originals || len_of(idx) != pk[k].DataBytes ||
                    memcmp(pay(idx), pk[k].Data, pk[k].DataBytes) != 0)
                    ++bad_recoveries;
            }
        }
        return rc;
    }
    int dec_ack(uint8_t* buf, uint32_t limit, uint32_t* used) {
        ProfScope ps(P_DACK);
        return siamese_decoder_ack(dec, buf, limit, used);
    }
    // the reference is always driven one call at a time
    bool enc_add_run(uint32_t, uint32_t, uint32_t, uint32_t*) { return false; }
    bool dec_add_run(uint32_t, uint32_t, uint32_t, uint32_t) { return false; }
    void set_time(uint64_t ms) {
        g_vclock_on = true;
        g_vclock_ms = ms;
    }
    int enc_retransmit(uint32_t* num, uint32_t* bytes, const uint8_t** data) {
        SiameseOriginalPacket o;
        o.PacketNum = 0;
        o.Data = nullptr;
        o.DataBytes = 0;
        const int rc = siamese_encoder_retransmit(enc, &o);
        *num = o.PacketNum;
        *bytes = o.DataBytes;
        *data = o.Data;
        return rc;
    }
    void stats(uint64_t e[9], uint64_t d[11]) {
        siamese_encoder_stats(enc, e, 9);
        siamese_decoder_stats(dec, d, 11);
    }
};

struct RefTranscript {
    TextSink t;
    bool enabled = true;
    void on_encode(int rc, const RefBackend::RecRef& r) {
        if (!enabled) return;
        if (rc != 0) { t.put("E %d\n", rc); return; }
        RecoveryMetadataView m;
        decode_footer(r.bytes, m);
        t.put("E 0 %zu %u %u %u %u %016llx\n", r.bytes.size(), m.row, m.cs, m.sc, m.ldpc,
              (unsigned long long)fnv1a(r.bytes.data(), r.bytes.size()));
    }
    void on_decode(int rc, const std::vector<uint32_t>& nums, const RefBackend::DecRef& d) {
        if (!enabled) return;
        t.put("D %d %zu", rc, nums.size());
        for (size_t k = 0; k < nums.size(); ++k)
            t.put(" %u:%zu:%016llx", nums[k], d.data[k].size(),
                  (unsigned long long)fnv1a(d.data[k].data(), d.data[k].size()));
        t.put("\n");
    }
    void on_ack(int rd, const uint8_t* buf, uint32_t used, int re, uint32_t next) {
        if (!enabled) return;
        t.put("K %d %u %016llx %d %u\n", rd, used, (unsigned long long)fnv1a(buf, used), re, next);
    }
    void on_event(char kind, int rc, uint32_t a, uint32_t b) {
        if (!enabled) return;
        if (rc != 0) t.put("%c %d %u %u\n", kind, rc, a, b);
    }
    void on_retransmit(int rc, uint32_t num, uint32_t bytes, uint64_t h) {
        if (enabled) fmt_retransmit(t, rc, num, bytes, h);
    }
    void on_stats(const uint64_t e[9], const uint64_t d[11]) {
        if (enabled) fmt_stats(t, e, d);
    }

    struct RecoveryMetadataView { unsigned row = 0, cs = 0, sc = 0, ldpc = 0; };
    // Footer parse (SiameseSerializers.h:759-800), restated for transcript labelling only.
    static void decode_footer(const std::vector<uint8_t>& b, RecoveryMetadataView& m) {
        size_t n = b.size();
        auto cnt = [&](unsigned& v) {
            const uint8_t x = b[n - 1];
            if ((x & 0x80) == 0) { v = x; n -= 1; }
            else { v = (((unsigned)x << 8) | b[n - 2]) & 0x7fff; n -= 2; }
        };
        auto pnum = [&](unsigned& v) {
            const uint8_t x = b[n - 1];
            const unsigned k = x >> 6;
            if (k <= 1) { v = x; n -= 1; }
            else if (k == 2) { v = (((unsigned)x << 8) | b[n - 2]) & 0x3fff; n -= 2; }
            else { v = (((unsigned)x << 16) | ((unsigned)b[n - 2] << 8) | b[n - 3]) & 0x3fffff; n -= 3; }
        };
        cnt(m.sc); m.sc += 1;
        pnum(m.cs);
        if (m.sc <= 1) { m.ldpc = 1; m.row = 0; }
        else { cnt(m.ldpc); m.row = b[n - 1]; }
    }
};

static uint32_t g_pool = 0;  // time mode: payload pool per stream (RefBackend::pool)
static int g_runs = 1;        // time mode: timed passes
static bool parse_kv(Params& p, int& threads, int& streams, int& reps, const char* kv) {
    const char* eq = strchr(kv, '=');
    if (!eq) return false;
    std::string k(kv, eq - kv);
    const unsigned long long v = strtoull(eq + 1, nullptr, 0);
    if (k == "pool") g_pool = (uint32_t)v;
    else if (k == "lat") g_lat = v != 0;
    else if (k == "prof") g_prof = v != 0;
    else if (k == "runs") g_runs = (int)v;
    else if (k == "threads") threads = (int)v;
    else if (k == "streams") streams = (int)v;
    else if (k == "reps") reps = (int)v;
    else return parse_param(p, k, v);
    return true;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s transcript <out> k=v... | time k=v...\n", argv[0]);
        return 2;
    }
    if (siamese_init() != 0) { fprintf(stderr, "siamese_init failed\n"); return 3; }
    typedef void (*SetClock)(uint64_t (*)(void));
    if (SetClock set_clock = (SetClock)dlsym(RTLD_DEFAULT, "tamd_set_clock")) set_clock(vclock_msec);
    Params base;
    int threads = 1, streams = 1, reps = 1;
    const bool timing = strcmp(argv[1], "time") == 0;
    const bool multi = strcmp(argv[1], "transcripts") == 0;
    const int first_kv = timing ? 2 : 3;
    if (!timing && argc < 3) { fprintf(stderr, "missing output path\n"); return 2; }
    for (int i = first_kv; i < argc; ++i) {
        if (!parse_kv(base, threads, streams, reps, argv[i])) { fprintf(stderr, "bad arg %s\n", argv[i]); return 2; }
    }

    auto write_transcript = [](const char* path, const RefTranscript& tr, const Summary& s, uint64_t bad) {
        FILE* f = fopen(path, "wb");
        if (!f) return false;
        fwrite(tr.t.text.data(), 1, tr.t.text.size(), f);
        fprintf(f, "Z originals=%llu lost=%llu recoveries=%llu lostrec=%llu recovered=%llu arq=%llu "
                   "acks=%llu decodes=%llu flush=%llu missing=%llu bad=%llu\n",
                (unsigned long long)s.originals, (unsigned long long)s.lost_originals,
                (unsigned long long)s.recoveries, (unsigned long long)s.lost_recoveries,
                (unsigned long long)s.recovered, (unsigned long long)s.arq_redelivered,
                (unsigned long long)s.acks, (unsigned long long)s.decode_calls,
                (unsigned long long)s.flush_encodes, (unsigned long long)s.missing_at_end,
                (unsigned long long)bad);
        fclose(f);
        return true;
    };
    if (multi) {
        std::atomic<int> next{0};
        std::atomic<unsigned long long> bad{0};
        std::atomic<int> fails{0};
        std::vector<std::thread> pool;
        const std::string prefix = argv[2];
        for (int t = 0; t < threads; ++t) {
            pool.emplace_back([&]() {
                for (;;) {
                    const int s = next++;
                    if (s >= streams) break;
                    Params p = base;
                    p.stream_id = base.stream_id + s;
                    p.seed_data = 1000 + p.stream_id;
                    p.seed_loss = 2000 + p.stream_id;
                    RefBackend be(p);
                    RefTranscript tr;
                    const Summary sum = run_stream(p, be, tr);
                    const std::string path = prefix + std::to_string(p.stream_id) + ".txt";
                    if (!write_transcript(path.c_str(), tr, sum, be.bad_recoveries)) ++fails;
                    bad += be.bad_recoveries;
                }
            });
        }
        for (auto& th : pool) th.join();
        return fails.load() ? 4 : (bad.load() ? 5 : 0);
    }
    if (!timing) {
        RefBackend be(base);
        RefTranscript tr;
        Summary s = run_stream(base, be, tr);
        if (!write_transcript(argv[2], tr, s, be.bad_recoveries)) return 4;
        return be.bad_recoveries ? 5 : 0;
    }

    // Timing: `streams` independent streams (stream id s uses seeds 1000+s / 2000+s) spread
    // over `threads` host threads, each stream's workload run `reps` times with fresh codecs.
    // Scenario generation -- payloads and every run's loss draws -- happens before the clock
    // starts; the timed region is the siamese.h calls and the runner's
    // bookkeeping between them.
    // `runs=R` repeats the whole timed pass R times (fresh codecs and pregenerated runners each
    // time) and prints one line per pass.
    typedef Runner<RefBackend, RefTranscript> RefRunner;
    std::atomic<unsigned long long> bad{0};
    std::vector<std::unique_ptr<RefBackend>> bes(streams);
    std::vector<Params> ps(streams, base);
    RefTranscript quiet;
    quiet.enabled = false;
    // setup on the worker threads too (the payload pools are the bulk of it)
    // (prof=1: each thread's first and last stream start / end, ns after the pass started)
    std::vector<uint64_t> th_first(threads), th_end(threads);
    uint64_t pass_t0 = 0;
    auto parallel = [&](const std::function<void(int)>& f) {
        std::atomic<int> at{0};
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t)
            pool.emplace_back([&, t]() {
                th_first[t] = now_ns() - pass_t0;
                for (int s; (s = at++) < streams;) f(s);
                th_end[t] = now_ns() - pass_t0;
            });
        for (auto& th : pool) th.join();
    };
    parallel([&](int s) {
        ps[s].stream_id = base.stream_id + s;
        ps[s].seed_data = 1000 + ps[s].stream_id;
        ps[s].seed_loss = 2000 + ps[s].stream_id;
        bes[s].reset(new RefBackend(ps[s], g_pool));
    });
    for (int pass = 0; pass < g_runs; ++pass) {
        std::vector<std::vector<std::unique_ptr<RefRunner>>> runs(streams);
        parallel([&](int s) {
            if (pass) bes[s]->reset_codecs();
            for (int r = 0; r < reps; ++r) {
                runs[s].emplace_back(new RefRunner(ps[s], *bes[s], quiet));
                runs[s].back()->pregenerate();
            }
        });
        std::atomic<unsigned long long> bytes{0};
        std::vector<LatLog> logs(streams);
        std::vector<std::vector<uint64_t>> prof(streams, std::vector<uint64_t>(P_N + 1, 0));
        struct rusage ru0, ru1;
        getrusage(RUSAGE_SELF, &ru0);
        pass_t0 = now_ns();
        const auto t0 = std::chrono::steady_clock::now();
        parallel([&](int s) {
            if (g_lat) g_latlog = &logs[s];
            if (g_prof) g_profv = prof[s].data();
            const uint64_t s0 = g_prof ? now_ns() : 0;
            unsigned long long b = 0;
            for (uint32_t i = 0; i < ps[s].n_originals; ++i) b += bes[s]->len_of(i);
            for (int r = 0; r < reps; ++r) {
                if (r) bes[s]->reset_codecs();
                runs[s][r]->finish();
                bytes += b;
            }
            g_latlog = nullptr;
            if (g_prof) prof[s][P_N] += now_ns() - s0;
            g_profv = nullptr;
        });
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (int s = 0; s < streams; ++s) bad += bes[s]->bad_recoveries;
        std::string lat;
        if (g_lat) {
            auto pct = [&](bool enc) {
                std::vector<uint32_t> all;
                for (const LatLog& l : logs) {
                    const std::vector<uint32_t>& v = enc ? l.enc_ns : l.dec_ns;
                    all.insert(all.end(), v.begin(), v.end());
                }
                if (all.empty()) return std::string("null");
                std::sort(all.begin(), all.end());
                auto at = [&](double q) { return all[std::min(all.size() - 1, (size_t)(q * (double)all.size()))] / 1e3; };
                double sum = 0;
                for (uint32_t x : all) sum += x;
                char b[200];
                snprintf(b, sizeof(b), "{\"calls\": %zu, \"mean\": %.2f, \"p50\": %.2f, \"p90\": %.2f, \"p99\": %.2f, \"max\": %.2f}",
                         all.size(), sum / all.size() / 1e3, at(0.5), at(0.9), at(0.99), all.back() / 1e3);
                return std::string(b);
            };
            lat = ", \"encode_us\": " + pct(true) + ", \"decode_us\": " + pct(false);
        }
        if (g_prof) {
            getrusage(RUSAGE_SELF, &ru1);
            char rb[256];
            snprintf(rb, sizeof(rb), ", \"rusage\": {\"minflt\": %ld, \"majflt\": %ld, \"nvcsw\": %ld, \"nivcsw\": %ld, "
                     "\"utime_s\": %.3f, \"stime_s\": %.3f}", ru1.ru_minflt - ru0.ru_minflt, ru1.ru_majflt - ru0.ru_majflt,
                     ru1.ru_nvcsw - ru0.ru_nvcsw, ru1.ru_nivcsw - ru0.ru_nivcsw,
                     (ru1.ru_utime.tv_sec - ru0.ru_utime.tv_sec) + 1e-6 * (ru1.ru_utime.tv_usec - ru0.ru_utime.tv_usec),
                     (ru1.ru_stime.tv_sec - ru0.ru_stime.tv_sec) + 1e-6 * (ru1.ru_stime.tv_usec - ru0.ru_stime.tv_usec));
            lat += rb;
            const uint64_t fmax = *std::max_element(th_first.begin(), th_first.end());
            const uint64_t emin = *std::min_element(th_end.begin(), th_end.end());
            const uint64_t emax = *std::max_element(th_end.begin(), th_end.end());
            snprintf(rb, sizeof(rb), ", \"threads_ms\": {\"last_start\": %.2f, \"first_end\": %.2f, \"last_end\": %.2f}",
                     fmax / 1e6, emin / 1e6, emax / 1e6);
            lat += rb;
            static const char* names[P_N + 1] = {"enc_add", "encode", "enc_ack", "dec_add", "dec_recovery", "is_ready",
                                                 "decode", "dec_ack", "stream_total"};
            // the slowest stream (it sets the pass time): its id, ms per call kind, call counts
            int worst = 0;
            for (int s = 1; s < streams; ++s)
                if (prof[s][P_N] > prof[worst][P_N]) worst = s;
            lat += ", \"slowest_stream\": {\"stream\": " + std::to_string(ps[worst].stream_id) + ", \"encodes\": " +
                   std::to_string(logs[worst].enc_ns.size()) + ", \"decodes\": " + std::to_string(logs[worst].dec_ns.size());
            for (int k = 0; k <= P_N; ++k) {
                char b[96];
                snprintf(b, sizeof(b), ", \"%s\": %.2f", names[k], prof[worst][k] / 1e6);
                lat += b;
            }
            lat += "}";
            lat += ", \"call_ms\": {";
            for (int k = 0; k <= P_N; ++k) {
                uint64_t t = 0;
                for (int s = 0; s < streams; ++s) t += prof[s][k];
                char b[96];
                snprintf(b, sizeof(b), "%s\"%s\": %.1f", k ? ", " : "", names[k], t / 1e6);
                lat += b;
            }
            lat += "}";
        }
        printf("{\"seconds\": %.6f, \"payload_bytes\": %llu, \"gib_per_s\": %.6f, \"threads\": %d, "
               "\"streams\": %d, \"reps\": %d, \"bad\": %llu%s}\n",
               sec, (unsigned long long)bytes.load(), bytes.load() / sec / (1024.0 * 1024 * 1024),
               threads, streams, reps, (unsigned long long)bad.load(), lat.c_str());
        fflush(stdout);
    }
    return bad.load() ? 5 : 0;
}
