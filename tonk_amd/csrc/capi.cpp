// capi.cpp -- the siamese.h C ABI over the MI355X engine (drop-in for the reference siamese.cpp).
//
// Argument validation and result codes follow siamese.cpp:43-299 exactly.  Data crosses the
// device boundary where the API forces it:
//   encoder_add / decoder_add_original / decoder_add_recovery : H2D of the packet into a row
//   siamese_encode                                            : run program, D2H recovery row
//   siamese_decode                                            : run program, D2H recovered rows
// Host mirrors of originals back siamese_encoder_get/retransmit and siamese_decoder_get.
#define SIAMESE_BUILDING 1
#include "../../include/siamese.h"

#include "decoder.h"
#include "device.h"

#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>

using namespace tamd;

namespace {

struct Runtime {
    std::mutex mu;
    Device dev;
    Context ctx;
    bool ok = false;
};

Runtime* g_rt = nullptr;
std::mutex g_init_mu;

// Call accounting for the watchdog (TONK_AMD_CAPI_WATCH=<seconds>): a thread prints to stderr how
// many API calls and device waits ran, the longest lock wait, and whether a call is inside a
// device wait right now -- to tell a slow path from a stuck one under a real caller (Tonk).
std::atomic<uint64_t> g_calls{0}, g_waits{0}, g_wait_ns{0}, g_lock_wait_max_ns{0};
std::atomic<int64_t> g_in_wait_since{0};
bool g_watch = false;
std::atomic<uint64_t> g_prepare_ns{0}, g_run_ns{0};
int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// Per-entry-point accounting: calls and time spent holding the lock.
struct Site {
    const char* name;
    std::atomic<uint64_t> calls{0}, held_ns{0};
    Site* next;
    explicit Site(const char* n);
};
std::atomic<Site*> g_sites{nullptr};
Site::Site(const char* n) : name(n), next(nullptr) {
    Site* head = g_sites.load();
    do { next = head; } while (!g_sites.compare_exchange_weak(head, this));
}

struct ApiLock {
    std::unique_lock<std::mutex> lk;
    Site& site;
    int64_t t_in = 0;
    explicit ApiLock(Site& s) : lk(g_rt->mu, std::defer_lock), site(s) {
        if (!lk.try_lock()) {
            const int64_t t0 = now_ns();
            lk.lock();
            const uint64_t w = (uint64_t)(now_ns() - t0);
            uint64_t m = g_lock_wait_max_ns.load(std::memory_order_relaxed);
            while (w > m && !g_lock_wait_max_ns.compare_exchange_weak(m, w)) {}
        }
        g_calls.fetch_add(1, std::memory_order_relaxed);
        if (g_watch) t_in = now_ns();
    }
    ~ApiLock() {
        site.calls.fetch_add(1, std::memory_order_relaxed);
        if (g_watch) site.held_ns.fetch_add((uint64_t)(now_ns() - t_in), std::memory_order_relaxed);
    }
};
#define API_LOCK()                   \
    static Site api_site_(__func__); \
    ApiLock lk(api_site_)

void watch_loop(double period_s) {
    const int64_t start = now_ns();
    for (;;) {
        std::this_thread::sleep_for(std::chrono::duration<double>(period_s));
        const int64_t since = g_in_wait_since.load();
        fprintf(stderr, "[tonk_amd capi] t=%.1fs calls=%llu device_waits=%llu wait_ms=%.1f lock_wait_max_ms=%.2f%s\n",
                (now_ns() - start) * 1e-9, (unsigned long long)g_calls.load(), (unsigned long long)g_waits.load(),
                g_wait_ns.load() * 1e-6, g_lock_wait_max_ns.exchange(0) * 1e-6,
                since ? (" IN DEVICE WAIT for " + std::to_string((now_ns() - since) / 1000000) + " ms").c_str() : "");
        fprintf(stderr, "[tonk_amd capi]   flush: prepare_ms=%.1f launch_ms=%.1f programs=%llu launches=%llu\n",
                g_prepare_ns.load() * 1e-6, g_run_ns.load() * 1e-6, (unsigned long long)g_rt->dev.stats().programs,
                (unsigned long long)g_rt->dev.stats().launches);
        for (Site* st = g_sites.load(); st; st = st->next) {
            const uint64_t c = st->calls.load();
            if (c)
                fprintf(stderr, "[tonk_amd capi]   %-28s calls=%llu held_ms=%.1f\n", st->name, (unsigned long long)c,
                        st->held_ns.load() * 1e-6);
        }
    }
}

void release_host(void* host, void*) { free(host); }

struct CEncoder {
    Encoder* enc = nullptr;
    uint8_t* recovery = nullptr;  // pinned: the D2H of each recovery packet lands here
    size_t recovery_cap = 0;
};

struct CDecoder {
    Decoder* dec = nullptr;
    std::vector<SiameseOriginalPacket> out;
};

uint64_t row_byte_offset(RowId r) { return (uint64_t)g_rt->ctx.rows.offset(r) * TAMD_ROW_UNIT; }

// Enqueues the pending program (caller holds the lock); reads of its results may be enqueued
// behind it with Device::download_async before flush_complete() waits once for all of it.
uint64_t flush_enqueue() {
    Context& ctx = g_rt->ctx;
    uint64_t ticket = 0;
    const int64_t t0 = g_watch ? now_ns() : 0;
    ctx.prepare_flush();
    const int64_t t1 = g_watch ? now_ns() : 0;
    if (!ctx.pb.empty()) ticket = g_rt->dev.run(&ctx);
    if (g_watch) {
        g_prepare_ns.fetch_add((uint64_t)(t1 - t0), std::memory_order_relaxed);
        g_run_ns.fetch_add((uint64_t)(now_ns() - t1), std::memory_order_relaxed);
    }
    return ticket;
}

void flush_complete() {
    Context& ctx = g_rt->ctx;
    const uint64_t done = ctx.epoch;
    const int64_t t0 = now_ns();
    g_in_wait_since.store(t0);
    g_rt->dev.synchronize();
    g_in_wait_since.store(0);
    g_waits.fetch_add(1, std::memory_order_relaxed);
    g_wait_ns.fetch_add((uint64_t)(now_ns() - t0), std::memory_order_relaxed);
    ctx.finish_flush();
    ctx.rows.release_up_to(done);
}

// varint(len) || payload into a malloc'd host buffer and a device row.
bool store_framed(const unsigned char* data, unsigned len, uint8_t** host_out, RowId* row_out,
                  uint32_t* framed_out, uint32_t* header_out) {
    uint8_t hdr[4];
    const uint32_t hb = put_length_header(len, hdr);
    const uint32_t framed = hb + len;
    uint8_t* host = (uint8_t*)malloc(framed);
    if (!host) return false;
    memcpy(host, hdr, hb);
    memcpy(host + hb, data, len);
    const RowId row = g_rt->ctx.alloc(framed);
    if (row == kNoRow) { free(host); return false; }
    g_rt->dev.upload(row_byte_offset(row), host, framed);
    *host_out = host;
    *row_out = row;
    *framed_out = framed;
    *header_out = hb;
    return true;
}

} // namespace

extern "C" {

SIAMESE_EXPORT int siamese_init_(int version) {
    if (version != SIAMESE_VERSION) return Siamese_Disabled;
    std::lock_guard<std::mutex> lk(g_init_mu);
    if (g_rt) return g_rt->ok ? Siamese_Success : Siamese_Disabled;
    g_rt = new Runtime();
    if (!gf_init()) return Siamese_Disabled;
    int device = 0;
    if (const char* d = getenv("TONK_AMD_DEVICE")) device = atoi(d);
    uint64_t arena_mb = 2048;
    if (const char* a = getenv("TONK_AMD_ARENA_MB")) arena_mb = strtoull(a, nullptr, 10);
    if (!g_rt->dev.init(device, arena_mb << 20)) {
        fprintf(stderr, "%s\n", g_rt->dev.error().c_str());
        return Siamese_Disabled;
    }
    if (!g_rt->dev.gf_selftest()) {
        fprintf(stderr, "tonk_amd: device GF(256) self test failed\n");
        return Siamese_Disabled;
    }
    g_rt->ctx.rows.init(g_rt->dev.arena_bytes(), 0);
    g_rt->ctx.track_dirty = true;
    g_rt->ok = true;
    if (const char* w = getenv("TONK_AMD_CAPI_WATCH")) {
        const double period = atof(w) > 0 ? atof(w) : 5.0;
        g_watch = true;
        std::thread(watch_loop, period).detach();
    }
    return Siamese_Success;
}

// ---------------------------------------------------------------------------- Encoder API

SIAMESE_EXPORT SiameseEncoder siamese_encoder_create() {
    if (!g_rt || !g_rt->ok) return nullptr;
    API_LOCK();
    CEncoder* e = new (std::nothrow) CEncoder();
    if (!e) return nullptr;
    e->enc = new Encoder(&g_rt->ctx, 0, release_host, nullptr);
    return reinterpret_cast<SiameseEncoder>(e);
}

SIAMESE_EXPORT void siamese_encoder_free(SiameseEncoder encoder_t) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e) return;
    API_LOCK();
    if (e->recovery) {
        g_rt->dev.synchronize();  // no copy may still be landing in the buffer
        Device::host_free(e->recovery);
    }
    delete e->enc;
    delete e;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_is_ready(SiameseEncoder encoder_t) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e) return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(e->enc);
    if (e->enc->remaining_slots() <= 2) return Siamese_MaxPacketsReached;
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_add(SiameseEncoder encoder_t, SiameseOriginalPacket* packet) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || !packet || !packet->Data || packet->DataBytes <= 0 || packet->DataBytes > SIAMESE_MAX_PACKET_BYTES)
        return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(e->enc);
    if (e->enc->disabled()) return Siamese_Disabled;
    if (e->enc->remaining_slots() <= 0) return Siamese_MaxPacketsReached;
    uint8_t* host = nullptr;
    RowId row = kNoRow;
    uint32_t framed = 0, hb = 0;
    if (!store_framed(packet->Data, packet->DataBytes, &host, &row, &framed, &hb)) return Siamese_Disabled;
    uint32_t pn = 0;
    const Result r = e->enc->add(row, framed, hb, packet->DataBytes, host, &pn);
    if (r != kSuccess) {
        g_rt->ctx.rows.free_deferred(row);
        free(host);
        return (SiameseResult)r;
    }
    packet->PacketNum = pn;
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_get(SiameseEncoder encoder_t, SiameseOriginalPacket* packet) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || !packet || packet->PacketNum > SIAMESE_PACKET_NUM_MAX) return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(e->enc);
    const StoredOriginal* o = nullptr;
    const Result r = e->enc->get(packet->PacketNum, &o);
    if (r != kSuccess) {
        packet->Data = nullptr;
        packet->DataBytes = 0;
        return (SiameseResult)r;
    }
    packet->Data = (const unsigned char*)o->host + o->header_bytes;
    packet->DataBytes = o->bytes - o->header_bytes;
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_remove_before(SiameseEncoder encoder_t, unsigned packetNum) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || packetNum > SIAMESE_PACKET_NUM_MAX) return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(e->enc);
    e->enc->remove_before(packetNum);
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_ack(SiameseEncoder encoder_t, const void* buffer, unsigned bytes,
                                                 unsigned* nextExpectedPacketNum) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || !buffer || bytes < 1 || !nextExpectedPacketNum) return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(e->enc);
    uint32_t next = 0;
    const Result r = e->enc->acknowledge((const uint8_t*)buffer, bytes, &next);
    if (r == kSuccess) *nextExpectedPacketNum = next;
    return (SiameseResult)r;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_retransmit(SiameseEncoder encoder_t, SiameseOriginalPacket* original) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || !original) return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(e->enc);
    original->Data = nullptr;
    original->DataBytes = 0;
    const StoredOriginal* o = nullptr;
    const Result r = e->enc->retransmit(&o);
    if (r != kSuccess) return (SiameseResult)r;
    original->PacketNum = o->column;
    original->Data = (const unsigned char*)o->host + o->header_bytes;
    original->DataBytes = o->bytes - o->header_bytes;
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_encode(SiameseEncoder encoder_t, SiameseRecoveryPacket* recovery) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || !recovery) return Siamese_InvalidInput;
    void* ev = nullptr;
    uint64_t done = 0, ticket = 0;
    uint32_t total = 0;
    {
        API_LOCK();
        g_rt->ctx.touch(e->enc);
        RecoveryOut out;
        const Result r = e->enc->encode(out);
        if (r != kSuccess) {
            if (r == kNeedMoreData) recovery->DataBytes = 0;
            return (SiameseResult)r;
        }
        total = out.total();
        if (total > e->recovery_cap) {
            if (e->recovery) {
                g_rt->dev.synchronize();
                Device::host_free(e->recovery);
            }
            e->recovery_cap = total < 2048 ? 2048 : total;
            e->recovery = (uint8_t*)Device::host_alloc(e->recovery_cap);
            if (!e->recovery) {
                e->recovery_cap = 0;
                g_rt->ctx.rows.free_deferred(out.row);
                e->enc->set_disabled();
                return Siamese_Disabled;
            }
        }
        // Enqueue the program and the read of the recovery row behind it, close the program's
        // host bookkeeping (later programs are stream-ordered after it), and wait for the copy
        // without the lock so other codecs' calls proceed meanwhile.
        ticket = flush_enqueue();
        g_rt->dev.download_pinned(e->recovery, row_byte_offset(out.row), total);
        ev = g_rt->dev.record_event();
        done = g_rt->ctx.epoch;
        g_rt->ctx.finish_flush();
        g_rt->ctx.rows.free_deferred(out.row);  // released once the next program completes
    }
    const int64_t t0 = now_ns();
    Device::event_wait(ev);
    g_waits.fetch_add(1, std::memory_order_relaxed);
    g_wait_ns.fetch_add((uint64_t)(now_ns() - t0), std::memory_order_relaxed);
    {
        API_LOCK();
        g_rt->dev.event_release(ev);
        g_rt->dev.completed(ticket);  // retire finished programs' events
        g_rt->ctx.rows.release_up_to(done);
    }
    recovery->Data = e->recovery;
    recovery->DataBytes = total;
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_stats(SiameseEncoder encoder_t, uint64_t* statsOut, unsigned statsCount) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || !statsOut || statsCount <= 0) return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(e->enc);
    e->enc->stats(statsOut, statsCount);
    return Siamese_Success;
}

// ---------------------------------------------------------------------------- Decoder API

SIAMESE_EXPORT SiameseDecoder siamese_decoder_create() {
    if (!g_rt || !g_rt->ok) return nullptr;
    API_LOCK();
    CDecoder* d = new (std::nothrow) CDecoder();
    if (!d) return nullptr;
    d->dec = new Decoder(&g_rt->ctx, 0, release_host, nullptr);
    return reinterpret_cast<SiameseDecoder>(d);
}

SIAMESE_EXPORT void siamese_decoder_free(SiameseDecoder decoder_t) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d) return;
    API_LOCK();
    delete d->dec;
    delete d;
}

SIAMESE_EXPORT SiameseResult siamese_decoder_add_original(SiameseDecoder decoder_t, const SiameseOriginalPacket* packet) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d || !packet || packet->DataBytes <= 0 || packet->DataBytes > SIAMESE_MAX_PACKET_BYTES ||
        packet->PacketNum > SIAMESE_PACKET_NUM_MAX)
        return Siamese_InvalidInput;
    if (!packet->Data) return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(d->dec);
    if (d->dec->disabled()) return Siamese_Disabled;
    uint8_t* host = nullptr;
    RowId row = kNoRow;
    uint32_t framed = 0, hb = 0;
    if (!store_framed(packet->Data, packet->DataBytes, &host, &row, &framed, &hb)) {
        d->dec->set_disabled();
        return Siamese_Disabled;
    }
    bool took = false;
    const Result r = d->dec->add_original(packet->PacketNum, row, framed, hb, packet->DataBytes, host, &took);
    if (!took) {
        g_rt->ctx.rows.free_deferred(row);
        free(host);
    }
    return (SiameseResult)r;
}

SIAMESE_EXPORT SiameseResult siamese_decoder_add_recovery(SiameseDecoder decoder_t, const SiameseRecoveryPacket* packet) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d || !packet || !packet->Data || packet->DataBytes <= 0 || packet->DataBytes > SIAMESE_MAX_PACKET_BYTES)
        return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(d->dec);
    if (d->dec->disabled()) return Siamese_Disabled;
    const uint32_t total = packet->DataBytes;
    const RowId row = g_rt->ctx.alloc(total);
    if (row == kNoRow) { d->dec->set_disabled(); return Siamese_Disabled; }
    g_rt->dev.upload(row_byte_offset(row), packet->Data, total);
    const uint32_t tl = total < 8 ? total : 8;
    bool took = false;
    const Result r = d->dec->add_recovery(row, total, packet->Data + total - tl, packet->Data, &took);
    if (!took) g_rt->ctx.rows.free_deferred(row);
    return (SiameseResult)r;
}

SIAMESE_EXPORT SiameseResult siamese_decoder_get(SiameseDecoder decoder_t, SiameseOriginalPacket* packet) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d || !packet || packet->PacketNum > SIAMESE_PACKET_NUM_MAX) return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(d->dec);
    StoredOriginal* o = nullptr;
    const Result r = d->dec->get(packet->PacketNum, &o);
    if (r != kSuccess) {
        packet->Data = nullptr;
        packet->DataBytes = 0;
        return (SiameseResult)r;
    }
    if (!o->host) {  // recovered data not read back yet
        flush_enqueue();
        uint8_t* host = (uint8_t*)malloc(o->bytes);
        if (!host) { flush_complete(); return Siamese_Disabled; }
        g_rt->dev.download_async(host, row_byte_offset(o->row), o->bytes);
        flush_complete();
        unsigned len = 0;
        const int hb = get_length_header(host, o->bytes, len);
        if (hb < 1 || len == 0 || (uint32_t)hb + len > o->bytes) { free(host); d->dec->set_disabled(); return Siamese_Disabled; }
        o->host = host;
        o->header_bytes = (uint32_t)hb;
        o->bytes = (uint32_t)hb + len;
    }
    packet->Data = (const unsigned char*)o->host + o->header_bytes;
    packet->DataBytes = o->bytes - o->header_bytes;
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_decoder_is_ready(SiameseDecoder decoder_t) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d) return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(d->dec);
    return (SiameseResult)d->dec->is_ready();
}

SIAMESE_EXPORT SiameseResult siamese_decode(SiameseDecoder decoder_t, SiameseOriginalPacket** packetsPtrOut,
                                            unsigned* countOut) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d || (!packetsPtrOut != !countOut)) return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(d->dec);
    if (packetsPtrOut) {
        *packetsPtrOut = nullptr;
        *countOut = 0;
    }
    std::vector<RecoveredPacket*> got;
    const Result r = d->dec->decode(got);
    if (r != kSuccess) return (SiameseResult)r;
    flush_enqueue();
    // every recovered row not read back yet: one D2H each behind the program, then one wait
    std::vector<std::pair<StoredOriginal*, uint8_t*>> reads;
    std::vector<StoredOriginal*> outs;
    bool failed = false;
    for (RecoveredPacket* rp : got) {
        StoredOriginal* o = nullptr;
        if (d->dec->get(rp->packet_num, &o) != kSuccess || !o) { failed = true; break; }
        outs.push_back(o);
        if (!o->host) {
            const uint32_t upper = rp->framed_upper;
            uint8_t* host = (uint8_t*)malloc(upper ? upper : 1);
            if (!host) { failed = true; break; }
            g_rt->dev.download_async(host, row_byte_offset(rp->row), upper);
            reads.push_back(std::make_pair(o, host));
            o->bytes = upper;  // the upper bound until the header is parsed below
        }
    }
    flush_complete();
    for (auto& rd : reads) {
        StoredOriginal* o = rd.first;
        uint8_t* host = rd.second;
        if (failed) { free(host); continue; }
        const uint32_t upper = o->bytes;
        unsigned len = 0;
        const int hb = get_length_header(host, upper, len);
        // BackSubstitution's length check (SiameseDecoder.cpp:1139-1154).
        if (hb < 1 || len == 0 || (uint32_t)hb + len > upper) {
            free(host);
            failed = true;
            continue;
        }
        o->host = host;
        o->header_bytes = (uint32_t)hb;
        o->bytes = (uint32_t)hb + len;
    }
    if (failed) { d->dec->set_disabled(); return Siamese_Disabled; }
    d->out.clear();
    for (size_t i = 0; i < got.size(); ++i) {
        SiameseOriginalPacket p;
        p.PacketNum = got[i]->packet_num;
        p.Data = (const unsigned char*)outs[i]->host + outs[i]->header_bytes;
        p.DataBytes = outs[i]->bytes - outs[i]->header_bytes;
        d->out.push_back(p);
    }
    if (packetsPtrOut) {
        *packetsPtrOut = d->out.empty() ? nullptr : d->out.data();
        *countOut = (unsigned)d->out.size();
    }
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_decoder_ack(SiameseDecoder decoder_t, void* buffer, unsigned byteLimit,
                                                 unsigned* usedBytes) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d || !buffer || !usedBytes || byteLimit < SIAMESE_ACK_MIN_BYTES) return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(d->dec);
    uint32_t used = 0;
    const Result r = d->dec->ack((uint8_t*)buffer, byteLimit, &used);
    *usedBytes = used;
    return (SiameseResult)r;
}

SIAMESE_EXPORT SiameseResult siamese_decoder_stats(SiameseDecoder decoder_t, uint64_t* statsOut, unsigned statsCount) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d || !statsOut || statsCount <= 0) return Siamese_InvalidInput;
    API_LOCK();
    g_rt->ctx.touch(d->dec);
    d->dec->stats(statsOut, statsCount);
    return Siamese_Success;
}

} // extern "C"
