// capi.cpp -- the siamese.h C ABI over the MI355X engine (drop-in for the reference siamese.cpp).
//
// Argument validation and result codes follow siamese.cpp:43-299 exactly.  Data crosses the
// device boundary where the API forces it:
//   encoder_add / decoder_add_original / decoder_add_recovery : H2D of the packet into a row
//   siamese_encode                                            : run program, D2H recovery row
//   siamese_decode                                            : run program, D2H recovered rows
// Host mirrors of originals back siamese_encoder_get/retransmit and siamese_decoder_get.
//
// Concurrency follows the reference contract (siamese.h:58-59): the caller serialises calls on
// one codec, different codecs run concurrently.  Every codec owns its Context (pending program,
// row table); their rows come from arena segments of a shared pool, and the arena grows by
// mapping more memory into a reserved address range (no fixed cap short of the reservation).
// Only Device calls (program upload/launch, copies, events) take the process-wide device lock,
// and no lock is held while a call waits for the GPU.
#define SIAMESE_BUILDING 1
#include "../../include/siamese.h"

#include "decoder.h"
#include "device.h"
#include "server.h"

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>

using namespace tamd;

namespace {

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// ---- call accounting for the watchdog (TONK_AMD_CAPI_WATCH=<seconds>) ----
// A thread prints to stderr how many API calls and device waits ran, the longest device-lock
// wait, and how many calls are inside a device wait right now -- to tell a slow path from a
// stuck one under a real caller (Tonk).  Everything it reads is an atomic.
std::atomic<uint64_t> g_calls{0}, g_waits{0}, g_wait_ns{0}, g_lock_wait_max_ns{0}, g_lock_hold_max_ns{0};
std::atomic<uint64_t> g_programs{0}, g_launches{0}, g_prepare_ns{0}, g_run_ns{0};
std::atomic<uint64_t> g_batches{0}, g_batched{0};  // combined launches and the calls they served
std::atomic<uint64_t> g_ph_up_ns{0}, g_ph_run_ns{0}, g_ph_read_ns{0}, g_ph_lock_ns{0};  // batch phases (watch)
std::atomic<int> g_in_wait{0};
std::atomic<int64_t> g_in_wait_since{0};  // start of the current run of overlapping waits
bool g_watch = false;

struct Site {
    const char* name;
    std::atomic<uint64_t> calls{0}, ns{0};
    std::atomic<uint64_t> rc[8] = {};  // result codes, for the sites that record them (API_RC)
    Site* next;
    explicit Site(const char* n);
};
std::atomic<Site*> g_sites{nullptr};
Site::Site(const char* n) : name(n), next(nullptr) {
    Site* head = g_sites.load();
    do { next = head; } while (!g_sites.compare_exchange_weak(head, this));
}
// (only with the watchdog on: shared counters bumped by every call of every thread cost the
// drop-in ~1.6 us per call once 16 threads contend for their cache lines)
struct CallScope {
    Site& site;
    int64_t t0;
    explicit CallScope(Site& s) : site(s), t0(0) {
        if (!g_watch) return;
        t0 = now_ns();
        g_calls.fetch_add(1, std::memory_order_relaxed);
    }
    ~CallScope() {
        if (!g_watch) return;
        site.calls.fetch_add(1, std::memory_order_relaxed);
        site.ns.fetch_add((uint64_t)(now_ns() - t0), std::memory_order_relaxed);
    }
};
#define API_CALL()                   \
    static Site api_site_(__func__); \
    CallScope api_scope_(api_site_)
// Return `r`, counting it in the site's result histogram (watchdog diagnostics).
#define API_RC(r) do { const int rc_ = (int)(r); if (g_watch) api_site_.rc[(unsigned)rc_ & 7u].fetch_add(1, std::memory_order_relaxed); return (SiameseResult)rc_; } while (0)

// ---- the process runtime: one device, one arena, a segment pool over it ----
struct Runtime;
Runtime* g_rt = nullptr;
std::mutex g_init_mu;

struct SegmentPool final : SegmentSource {
    std::mutex mu;
    uint64_t bump_units = 0;                                 // first never-used unit
    std::vector<std::pair<uint64_t, uint32_t>> free_list;  // returned ranges
    uint32_t seg_units = 1u << 16;                          // 4 MiB ranges by default
    bool get(uint32_t min_units, uint64_t* base, uint32_t* units) override;
    void put(uint64_t base, uint32_t units) override;
};

struct Runtime {
    std::mutex dev_mu;  // every Device call
    Device dev;
    SegmentPool pool;
    bool ok = false;
};
// The launch-free path (server.h): null when off (TONK_AMD_SERVE=0) or when it failed its checks.
Server* g_srv = nullptr;
// The codecs' staging halves and command buffers in device memory the host writes through the
// PCIe BAR (Device::bar_alloc): the executor then copies commands and lands packets at HBM
// latency instead of pulling them across PCIe.  TONK_AMD_CAPI_BAR: a mask of what goes there
// (1 staging halves, 2 command buffers, 4 the executor's ring -- server.cpp; 0: all in pinned
// host memory).  Default 6: staging in BAR memory makes every add a PCIe write on the caller's
// thread, which cost more than the faster landing saved (profiles/r06m_capi_bar_placement.txt).
unsigned g_bar = 0;

struct DevLock {
    std::unique_lock<std::mutex> lk;
    int64_t held_since = 0;
    const char* site;
    explicit DevLock(const char* where = __builtin_FUNCTION()) : lk(g_rt->dev_mu, std::defer_lock), site(where) {
        // Tonk calls from many threads; every Device call targets this GPU.  Bound outside the lock:
        // a thread's first hipSetDevice can take tens of ms while the driver is busy (e.g. right
        // after another GPU process exited), which under the lock stalls every codec.
        g_rt->dev.bind_thread();
        if (!lk.try_lock()) {
            const int64_t t0 = now_ns();
            lk.lock();
            const uint64_t w = (uint64_t)(now_ns() - t0);
            uint64_t m = g_lock_wait_max_ns.load(std::memory_order_relaxed);
            while (w > m && !g_lock_wait_max_ns.compare_exchange_weak(m, w)) {}
        }
        if (g_watch) held_since = now_ns();
    }
    ~DevLock() {
        if (!g_watch) return;
        const uint64_t h = (uint64_t)(now_ns() - held_since);
        uint64_t m = g_lock_hold_max_ns.load(std::memory_order_relaxed);
        while (h > m && !g_lock_hold_max_ns.compare_exchange_weak(m, h)) {}
        if (h >= 10000000) fprintf(stderr, "tonk_amd: device lock held %.1f ms in %s\n", h * 1e-6, site);
    }
};

bool SegmentPool::get(uint32_t min_units, uint64_t* base, uint32_t* units) {
    std::lock_guard<std::mutex> lk(mu);
    for (size_t i = 0; i < free_list.size(); ++i) {
        if (free_list[i].second >= min_units) {
            *base = free_list[i].first;
            *units = free_list[i].second;
            free_list[i] = free_list.back();
            free_list.pop_back();
            return true;
        }
    }
    const uint32_t n = min_units > seg_units ? min_units : seg_units;
    const uint64_t end_bytes = (bump_units + n) * TAMD_ROW_UNIT;
    // Growth maps memory past everything in use: it takes no device lock, so other codecs'
    // programs keep going (a growth costs ~170-190 ms); and it normally happened already, in the
    // background, once three quarters of the mapped arena were handed out.
    if (end_bytes > g_rt->dev.arena_bytes() && !g_rt->dev.grow_arena(end_bytes)) {
        static std::atomic<int> reported{0};
        if (!reported.exchange(1))
            fprintf(stderr, "tonk_amd: the arena cannot grow to %llu MB (mapped %llu MB)\n",
                    (unsigned long long)(end_bytes >> 20), (unsigned long long)(g_rt->dev.arena_bytes() >> 20));
        return false;
    }
    *base = bump_units;
    *units = n;
    bump_units += n;
    if (bump_units * TAMD_ROW_UNIT > g_rt->dev.arena_bytes() / 4 * 3) g_rt->dev.grow_arena_async();
    return true;
}

void SegmentPool::put(uint64_t base, uint32_t units) {
    std::lock_guard<std::mutex> lk(mu);
    free_list.push_back(std::make_pair(base, units));
}

// Live encoders, for the watchdog's state dump (TONK_AMD_CAPI_WATCH_STATE=1).  The dump reads
// scalar fields of codecs other threads may be using: diagnostics only.
struct CEncoder;
std::mutex g_enc_mu;
std::vector<CEncoder*> g_encs;
void dump_encoders();

void watch_loop(double period_s) {
    const int64_t start = now_ns();
    for (;;) {
        std::this_thread::sleep_for(std::chrono::duration<double>(period_s));
        const int waiting = g_in_wait.load();
        const int64_t since = g_in_wait_since.load();
        std::string w;
        if (waiting > 0 && since)
            w = " IN DEVICE WAIT: " + std::to_string(waiting) + " call(s), for " +
                std::to_string((now_ns() - since) / 1000000) + " ms";
        fprintf(stderr, "[tonk_amd capi] t=%.1fs calls=%llu device_waits=%llu wait_ms=%.1f lock_wait_max_ms=%.2f lock_hold_max_ms=%.2f%s\n",
                (now_ns() - start) * 1e-9, (unsigned long long)g_calls.load(), (unsigned long long)g_waits.load(),
                g_wait_ns.load() * 1e-6, g_lock_wait_max_ns.exchange(0) * 1e-6, g_lock_hold_max_ns.exchange(0) * 1e-6,
                w.c_str());
        fprintf(stderr, "[tonk_amd capi]   flush: prepare_ms=%.1f launch_ms=%.1f programs=%llu launches=%llu batches=%llu calls_batched=%llu\n",
                g_prepare_ns.load() * 1e-6, g_run_ns.load() * 1e-6, (unsigned long long)g_programs.load(),
                (unsigned long long)g_launches.load(), (unsigned long long)g_batches.load(),
                (unsigned long long)g_batched.load());
        {
            DeviceStats& ds = g_rt->dev.stats();  // (read unlocked: diagnostics)
            fprintf(stderr, "[tonk_amd capi]   batch phases (device lock held): bind+take_ms=%.1f uploads_ms=%.1f programs_ms=%.1f reads_ms=%.1f; slot_wait_ms=%.1f program_h2d_enqueue_ms=%.1f\n",
                    g_ph_lock_ns.load() * 1e-6, g_ph_up_ns.load() * 1e-6, g_ph_run_ns.load() * 1e-6,
                    g_ph_read_ns.load() * 1e-6, ds.slot_wait_ms, ds.upload_enqueue_ms);
        }
        for (Site* st = g_sites.load(); st; st = st->next) {
            const uint64_t c = st->calls.load();
            if (!c) continue;
            std::string h;
            for (int k = 0; k < 8; ++k)
                if (const uint64_t v = st->rc[k].load()) h += " rc" + std::to_string(k) + "=" + std::to_string(v);
            fprintf(stderr, "[tonk_amd capi]   %-28s calls=%llu ms=%.1f%s\n", st->name, (unsigned long long)c,
                    st->ns.load() * 1e-6, h.c_str());
        }
        if (g_srv)
            fprintf(stderr, "[tonk_amd capi]   server: posted=%llu launches=%llu parked_waits=%llu slow_waits=%llu gpu_ms=%.1f\n",
                    (unsigned long long)g_srv->posted.load(), (unsigned long long)g_srv->launches.load(),
                    (unsigned long long)g_srv->waits_parked.load(), (unsigned long long)g_srv->waits_slow.load(),
                    g_srv->gpu_ns_sum.load() * 1e-6);
        if (g_srv) fprintf(stderr, "[tonk_amd capi]   server phases: %s\n", g_srv->phase_report().c_str());
        dump_encoders();
    }
}

void release_host(void* host, void*) { free(host); }

// A codec goes to Disabled (sticky, siamese.h:147-150): say why on stderr, once per reason.
void report_disable(const char* where) {
    static std::mutex mu;
    static std::vector<const char*> seen;
    std::lock_guard<std::mutex> lk(mu);
    for (const char* w : seen)
        if (w == where) return;
    seen.push_back(where);
    fprintf(stderr, "tonk_amd: codec disabled in %s%s\n", where, g_rt && g_rt->dev.failed() ? " (device failure)" : "");
}
#define DISABLE(codec) (report_disable(__func__), (codec)->set_disabled())

bool capi_combine();

// Packets added to a codec wait in the codec's own pinned staging (two halves) and reach the
// arena in one H2D copy + one scatter launch: before the codec's next program, or when a half
// fills up.  Adds never take the device lock.
struct Staging {
    static const size_t kFlushBytes = 1u << 20;  // packet bytes per half before it is sent
    unsigned stream = 0;             // the codec's launch stream (Device::select_stream)
    uint8_t* half[2] = {nullptr, nullptr};
    size_t cap = 0;                  // bytes per half (packets + descriptors)
    void* sent[2] = {nullptr, nullptr};  // event behind a sent half's copy (not yet waited for)
    int cur = 0;
    size_t used = 0;                 // packet bytes in the current half (16-B aligned)
    std::vector<Device::ScatterIn> descs;
    // The launch-free path: one command buffer per half.  A half that fills up goes out as an
    // upload-only command from its buffer; a program's command is built in the current half's.
    CmdBuf cmd[2];
    // A command of this codec did not complete (the server timed out or died): it may still run,
    // reading these halves and writing the codec's rows and pinned buffer, so none of them is
    // ever freed or reused (the codec is disabled; Codec::~Codec leaks its segments too).
    bool stalled = false;
    bool bar = false;  // halves in BAR-written device memory (g_bar)

    size_t need(size_t bytes, size_t n_desc) const { return ((bytes + 15) & ~(size_t)15) + n_desc * 16 + 16; }
    // The current half's packets as zero-copy sources of one batched host_copy (combined
    // launches): the half is reused by the codec's next adds, which cannot come before the batch
    // has completed (the codec's caller waits for it).
    void take_uploads(std::vector<Device::HostCopy>& out) {
        peek_uploads(out);
        descs.clear();
        used = 0;
    }
    void peek_uploads(std::vector<Device::HostCopy>& out) const {
        for (const Device::ScatterIn& d : descs)
            out.push_back(Device::HostCopy{half[cur] + d.src, (uint64_t)d.row * TAMD_ROW_UNIT, d.len});
    }
    // Every command of this codec's halves has completed (launch-free path).
    bool settle_cmds() {
        bool ok = true;
        for (CmdBuf& b : cmd) ok = g_srv->settle(b) && ok;
        if (!ok) stalled = true;
        return ok;
    }
    bool settle_cmd(int h) {
        if (!g_srv || g_srv->settle(cmd[h])) return true;
        stalled = true;
        return false;
    }
    // Enqueue the current half (caller holds the device lock).
    void send_locked(Device& dev) {
        if (descs.empty()) return;
        dev.scatter_upload(half[cur], used, descs.data(), (uint32_t)descs.size());
        descs.clear();
        used = 0;
    }
    // Wait for (and forget) a half's pending copy.
    static void settle(void*& ev) {
        if (!ev) return;
        Device::event_wait(ev);
        DevLock dl;
        g_rt->dev.event_release(ev);
        ev = nullptr;
    }
    // After the codec waited for work enqueued behind every sent half: all halves are free.
    void all_settled() {
        for (void*& ev : sent)
            if (ev) {
                DevLock dl;
                g_rt->dev.event_release(ev);
                ev = nullptr;
            }
    }
    bool grow(size_t want) {
        settle(sent[0]);
        settle(sent[1]);
        if (g_srv && !settle_cmds()) return false;
        for (uint8_t*& h : half) {
            if (bar) Device::bar_free(h);
            else Device::host_free(h);
            h = nullptr;
        }
        cap = want < (256u << 10) ? (256u << 10) : want;
        for (uint8_t*& h : half)
            if (!(h = (uint8_t*)(bar ? Device::bar_alloc(cap) : Device::host_alloc(cap)))) { cap = 0; return false; }
        return true;
    }
    // Copy a packet into the staging for arena unit offset `row`.
    bool stage(uint32_t row, const uint8_t* data, uint32_t n) {
        if (stalled) return false;
        if (used && (used + n > kFlushBytes || need(used + n, descs.size() + 1) > cap) && g_srv && g_srv->live()) {
            // launch-free: the full half lands by an upload-only command; the other half is
            // reused once its own command -- and a launch-path copy from it -- has completed
            thread_local std::vector<Device::HostCopy> ups, none;
            ups.clear();
            peek_uploads(ups);
            if (!settle_cmd(cur)) return false;
            if (Server::build(cmd[cur], ups, nullptr, none)) {
                g_srv->post(cmd[cur]);
                descs.clear();
                used = 0;
                cur ^= 1;
                if (!settle_cmd(cur)) return false;
                settle(sent[cur]);
            }
        }
        if (used && (used + n > kFlushBytes || need(used + n, descs.size() + 1) > cap)) {
            {
                DevLock dl;
                g_rt->dev.select_stream(stream);
                send_locked(g_rt->dev);
                sent[cur] = g_rt->dev.record_event();
                if (g_rt->dev.failed()) return false;
            }
            cur ^= 1;
            settle(sent[cur]);
            if (!settle_cmd(cur)) return false;
        }
        if (need(used + n, descs.size() + 1) > cap) {  // (only while the half is empty)
            if (used) return false;
            if (!grow(need(n, 1) + (64u << 10))) return false;
        }
        memcpy(half[cur] + used, data, n);
        Device::ScatterIn d;
        d.row = row;
        d.len = n;
        d.src = (uint32_t)used;
        descs.push_back(d);
        used = (used + n + 15) & ~(size_t)15;
        return true;
    }
    ~Staging() {
        if (stalled) return;  // (kept for good: a command may still read or write them)
        for (uint8_t* h : half) {
            if (bar) Device::bar_free(h);
            else Device::host_free(h);
        }
        for (CmdBuf& b : cmd) b.release();
    }
};

// Per-codec state: its own Context (pending program + row table over pool segments).
struct Codec {
    Context ctx;
    Staging staging;
    uint8_t* pinned = nullptr;  // D2H landing buffer (recovery packet / recovered rows)
    size_t pinned_cap = 0;
    // Codecs are spread over the device's launch streams round robin (a codec's work stays on
    // its stream, in order; different codecs' programs overlap instead of queueing behind each
    // other on one stream).
    Codec() {
        ctx.rows.init_segmented(&g_rt->pool);
        // Per-call programs stay small (the few-stream session's policies, Context): a decode of L
        // unknowns solves over materialized eliminated rows from L = 2 on, and expansions of more
        // than 16 terms are read as rows -- inlining both grows a program quadratically with L
        // (a burst of losses under Tonk made single programs of 8 MB, and the slot growth that
        // follows stalls every codec).
        static const uint32_t bs = getenv("TONK_AMD_CAPI_BACKSUB") ? (uint32_t)atoi(getenv("TONK_AMD_CAPI_BACKSUB")) : 2u;
        static const uint32_t ex = getenv("TONK_AMD_CAPI_EXPAND") ? (uint32_t)atoi(getenv("TONK_AMD_CAPI_EXPAND")) : 16u;
        ctx.backsub_rows = bs ? bs : ~0u;  // (0: never materialize / always inline)
        ctx.ex.expand_limit = ex ? ex : ~0u;
        static const bool short_scans = !getenv("TONK_AMD_CAPI_SHORT_SCANS") || atoi(getenv("TONK_AMD_CAPI_SHORT_SCANS")) != 0;
        ctx.short_scans = short_scans;  // (A/B: 0 restores the chain level)
        static std::atomic<unsigned> next{0};
        staging.stream = next.fetch_add(1) % g_rt->dev.stream_count();
        staging.bar = (g_bar & 1u) != 0;
        staging.cmd[0].bar = staging.cmd[1].bar = (g_bar & 2u) != 0;
    }
    uint64_t byte_offset(RowId r) const { return (uint64_t)ctx.rows.offset(r) * TAMD_ROW_UNIT; }
    // The pinned buffer holds at least n bytes (no copy can be landing in it: every read into it
    // was waited for before the call that issued it returned).
    bool ensure_pinned(size_t n) {
        if (staging.stalled) return false;  // (a stalled command may still write the old one)
        if (n <= pinned_cap) return true;
        Device::host_free(pinned);
        pinned_cap = n < 4096 ? 4096 : n + n / 2;
        pinned = (uint8_t*)Device::host_alloc(pinned_cap);
        if (!pinned) pinned_cap = 0;
        return pinned != nullptr;
    }
    // Before the codec's rows go back to the pool: nothing of its may still be in flight.
    bool used_launch = false;  // a program of this codec went through the launch path
    void quiesce() {
        if (g_srv && !staging.settle_cmds()) return;  // stalled: ~Codec keeps everything
        if (g_srv && !used_launch && !staging.sent[0] && !staging.sent[1]) return;
        DevLock dl;
        g_rt->dev.synchronize();
        for (void*& ev : staging.sent)
            if (ev) {
                g_rt->dev.event_release(ev);
                ev = nullptr;
            }
    }
    ~Codec() {
        if (staging.stalled) {
            // a command that never completed may still write these rows and the pinned buffer:
            // they never go back to the pool (a leak, bounded by one codec per stalled command)
            ctx.rows.leak_segments();
            return;
        }
        Device::host_free(pinned);
    }
};

// Encode-ahead.  A caller that encodes twice with no other call on the encoder between (the
// end of a transfer: recovery packets until the receiver has everything, workload.h finish;
// Tonk's flush of a quiet connection) is likely to encode again: from then on the same command
// also encodes the next `depth` recovery packets while Encoder::encode_is_quiet (their encodes
// change nothing but row counters and statistics), and reads them all back; the next calls
// return them without a device round trip.  Any other call on the encoder first takes the
// unused ones back (Encoder::rewind), so every result and statistic is the one a call-by-call
// run gives.  The depth doubles (to TONK_AMD_CAPI_AHEAD, default 63; 0: off) while the packets
// are all used and drops to 1 after a take-back.
struct CEncoder : Codec {
    Encoder* enc = nullptr;
    struct Ahead { size_t off; uint32_t total; };  // in `pinned`
    std::vector<Ahead> ahead;
    std::vector<Encoder::Mark> marks;  // marks[i]: the encoder before ahead[i] was encoded
    size_t ahead_next = 0;
    uint32_t depth = 1;
    bool last_encode = false;  // the previous call on the encoder was a successful encode
    void cancel_ahead() {
        if (ahead_next < ahead.size()) {
            enc->rewind(marks[ahead_next]);
            depth = 1;
        }
        ahead.clear();
        marks.clear();
        ahead_next = 0;
        last_encode = false;
    }
};

void dump_encoders() {
    static const bool on = getenv("TONK_AMD_CAPI_WATCH_STATE") != nullptr;
    if (!on) return;
    std::lock_guard<std::mutex> lk(g_enc_mu);
    char line[512];
    for (size_t i = 0; i < g_encs.size(); ++i) {
        if (!g_encs[i]->enc) continue;
        g_encs[i]->enc->debug_state(line, sizeof(line));
        fprintf(stderr, "[tonk_amd capi]   encoder %zu: %s\n", i, line);
    }
}

struct CDecoder : Codec {
    Decoder* dec = nullptr;
    std::vector<SiameseOriginalPacket> out;
};

// Combined launches (TONK_AMD_CAPI_COMBINE=0 turns them off).  Codecs of different connections
// call siamese_encode / siamese_decode concurrently, and each call needs its program run and read
// back before it returns (siamese.cpp:158-167; TonkineseOutgoing.cpp:1284-1328 sends the result
// at once).  A caller whose program is ready queues it; the first caller to find no leader
// becomes the leader and launches every queued program as ONE merged program (Device::run over
// their contexts: one executor launch per level for all of them), with each caller's reads and
// event behind it; it hands leadership on once its own program is launched, so no connection's
// send path serves the others for long (the compressor's pattern, compress.cpp).  Every caller
// then waits for its own event without a lock.  There is one such queue per launch stream and a
// codec keeps its stream, so its staged uploads, programs and reads stay in order while the
// streams' batches overlap on the device.
bool capi_combine() {
    static const bool on = !(getenv("TONK_AMD_CAPI_COMBINE") && atoi(getenv("TONK_AMD_CAPI_COMBINE")) == 0);
    return on;
}
// The event behind a combined batch, released by the last of its callers to finish waiting.
struct BatchDone {
    void* ev = nullptr;
    std::atomic<int> left{0};
};
struct RunReq {
    Codec* c = nullptr;
    const std::vector<Device::HostCopy>* reads = nullptr;
    BatchDone* done = nullptr;
    bool launched = false, ok = true;
    std::condition_variable cv;  // its caller waits here (woken alone: no herd of hundreds of threads)
};
// One combining queue per launch stream: a codec keeps its stream, so its uploads, programs and
// reads stay in order, and the streams' batches run side by side.
struct RunQueue {
    std::mutex mu;
    std::vector<RunReq*> q;
    bool leader = false;
};
RunQueue g_run[Device::kMaxStreams];

// One batch = one zero-copy upload launch for every codec's staged packets, the merged program's
// level launches, one zero-copy read-back launch for every caller's reads and one event: a fixed
// handful of commands however many callers it serves (per-codec copies would queue one H2D and
// one D2H command per caller on the stream).
// The batch is taken from the stream's queue only once the device lock is held: the lock is
// shared by every stream's leader, and callers that queue while a leader waits for it join that
// leader's batch instead of forming batches of one behind it (under a Tonk server's load the lock
// is busy most of the time, and batches of ~1.3 calls made every call pay a launch of its own).
void launch_batch(std::vector<RunReq*>& b, unsigned stream) {
    DevLock dl;
    {
        std::lock_guard<std::mutex> g(g_run[stream].mu);
        b.clear();
        b.swap(g_run[stream].q);
    }
    if (b.empty()) return;
    Device& dev = g_rt->dev;
    dev.select_stream(stream);
    std::vector<Context*> ctxs;
    thread_local std::vector<Device::HostCopy> up;
    up.clear();
    const uint64_t launches = dev.stats().launches;
    for (RunReq* r : b) {
        r->c->staging.take_uploads(up);  // packets added since the codec's last program land first
        if (!r->c->ctx.pb.empty()) ctxs.push_back(&r->c->ctx);
    }
    const int64_t p0 = g_watch ? now_ns() : 0;
    dev.host_copy(up.data(), (uint32_t)up.size(), false);
    const int64_t p1 = g_watch ? now_ns() : 0;
    // the merged program, in parts that fit a staging slot as it is (a part of one codec's
    // program may still need the oversize slot)
    const size_t cap = dev.slot_capacity(), pad = 64 * 16;
    size_t at = 0;
    while (at < ctxs.size()) {
        size_t end = at + 1, bytes = Device::program_bytes(ctxs[at]->pb) + pad;
        while (end < ctxs.size()) {
            const size_t more = Device::program_bytes(ctxs[end]->pb);
            if (bytes + more > cap) break;
            bytes += more;
            ++end;
        }
        dev.run(ctxs.data() + at, end - at);
        at = end;
    }
    const int64_t p2 = g_watch ? now_ns() : 0;
    if (!ctxs.empty()) {
        g_programs.fetch_add(ctxs.size(), std::memory_order_relaxed);
        g_launches.fetch_add(dev.stats().launches - launches, std::memory_order_relaxed);
    }
    g_batches.fetch_add(1, std::memory_order_relaxed);
    g_batched.fetch_add(b.size(), std::memory_order_relaxed);
    dev.collect_host_reads(true);
    for (RunReq* r : b)
        for (const Device::HostCopy& x : *r->reads) dev.download_pinned(x.host, x.arena_off, x.len);
    dev.collect_host_reads(false);
    dev.flush_host_reads();
    BatchDone* done = new BatchDone();
    done->ev = dev.record_event();
    if (g_watch) {
        g_ph_lock_ns.fetch_add((uint64_t)(p0 - dl.held_since), std::memory_order_relaxed);
        g_ph_up_ns.fetch_add((uint64_t)(p1 - p0), std::memory_order_relaxed);
        g_ph_run_ns.fetch_add((uint64_t)(p2 - p1), std::memory_order_relaxed);
        g_ph_read_ns.fetch_add((uint64_t)(now_ns() - p2), std::memory_order_relaxed);
    }
    if (g_watch && now_ns() - p0 >= 10000000) {
        size_t bytes = 0;
        for (Context* c : ctxs) bytes += Device::program_bytes(c->pb);
        fprintf(stderr, "tonk_amd: slow batch: uploads %.1f ms (%zu), programs %.1f ms (%zu, %zu KB), reads %.1f ms\n",
                (p1 - p0) * 1e-6, up.size(), (p2 - p1) * 1e-6, ctxs.size(), bytes >> 10, (now_ns() - p2) * 1e-6);
    }
    done->left.store((int)b.size());
    const bool ok = !dev.failed();
    for (RunReq* r : b) {
        r->done = done;
        r->ok = ok;
    }
}

// Close the codec's pending program and run it with `reads` (arena rows into the caller's
// pinned buffer) behind it, then wait for all of it without any lock.  Returns false on a device
// failure.  Launch-free when the command fits a worker of the persistent executor (server.h);
// otherwise, or with the server off, through kernel launches on the codec's launch stream.
bool run_and_read(Codec& c, const std::vector<Device::HostCopy>& reads) {
    Context& ctx = c.ctx;
    const int64_t t0 = g_watch ? now_ns() : 0;
    if (c.staging.stalled) return false;
    ctx.prepare_flush();
    const int64_t t1 = g_watch ? now_ns() : 0;
    if (g_srv) {
        Staging& sg = c.staging;
        // (upload-only commands of full halves -- or launch-path scatters of halves whose command
        // did not fit -- landed before this program reads their rows)
        if (!sg.settle_cmds()) return false;
        Staging::settle(sg.sent[0]);
        Staging::settle(sg.sent[1]);
        thread_local std::vector<Device::HostCopy> ups;
        ups.clear();
        sg.peek_uploads(ups);
        CmdBuf& b = sg.cmd[sg.cur];
        // Test hook (as Device::begin's): every program after the n-th fails like a device failure.
        static const long long fail_after =
            getenv("TONK_AMD_FAIL_AFTER_PROGRAMS") ? atoll(getenv("TONK_AMD_FAIL_AFTER_PROGRAMS")) : -1;
        static std::atomic<long long> programs_run{0};
        if (fail_after >= 0 && !ctx.pb.empty() && programs_run.fetch_add(1) >= fail_after) {
            ctx.finish_flush();
            return false;
        }
        if (g_srv->live() && Server::build(b, ups, &ctx.pb, reads)) {
            sg.descs.clear();
            sg.used = 0;
            g_srv->post(b);
            if (g_watch) g_programs.fetch_add(ctx.pb.empty() ? 0 : 1, std::memory_order_relaxed);
            const uint64_t done = ctx.epoch;
            ctx.finish_flush();
            const int64_t w0 = g_watch ? now_ns() : 0;
            const bool ok = g_srv->wait(b);
            if (g_watch) {
                g_waits.fetch_add(1, std::memory_order_relaxed);
                g_wait_ns.fetch_add((uint64_t)(now_ns() - w0), std::memory_order_relaxed);
                g_prepare_ns.fetch_add((uint64_t)(t1 - t0), std::memory_order_relaxed);
            }
            if (!ok) {  // still in flight: nothing it may touch is released (Staging::stalled)
                sg.stalled = true;
                return false;
            }
            ctx.rows.release_up_to(done);
            return true;
        }
        c.used_launch = true;
    }
    void* ev = nullptr;
    BatchDone* batch = nullptr;
    bool ok = true;
    if (capi_combine()) {
        RunReq req;
        req.c = &c;
        req.reads = &reads;
        {
            const unsigned st = c.staging.stream;
            RunQueue& rq = g_run[st];
            std::unique_lock<std::mutex> lk(rq.mu);
            rq.q.push_back(&req);
            req.cv.wait(lk, [&req, &rq] { return req.launched || !rq.leader; });
            if (!req.launched) {
                rq.leader = true;
                std::vector<RunReq*> b;
                while (!req.launched) {
                    lk.unlock();
                    launch_batch(b, st);  // (takes the queue under the device lock)
                    lk.lock();
                    for (RunReq* r : b) {
                        r->launched = true;
                        if (r != &req) r->cv.notify_one();
                    }
                }
                rq.leader = false;
                if (!rq.q.empty()) rq.q.front()->cv.notify_one();  // the next caller queued leads
            }
        }
        ok = req.ok;
        batch = req.done;
    } else {
        DevLock dl;
        Device& dev = g_rt->dev;
        dev.select_stream(c.staging.stream);
        const uint64_t launches = dev.stats().launches;
        c.staging.send_locked(dev);  // packets added since the last program land first
        if (!ctx.pb.empty()) {
            dev.run(&ctx);
            g_programs.fetch_add(1, std::memory_order_relaxed);
            g_launches.fetch_add(dev.stats().launches - launches, std::memory_order_relaxed);
        }
        for (const Device::HostCopy& x : reads) dev.download_pinned(x.host, x.arena_off, x.len);
        ev = dev.record_event();
        ok = !dev.failed();
    }
    if (g_watch) {
        g_prepare_ns.fetch_add((uint64_t)(t1 - t0), std::memory_order_relaxed);
        g_run_ns.fetch_add((uint64_t)(now_ns() - t1), std::memory_order_relaxed);
    }
    const uint64_t done = ctx.epoch;
    ctx.finish_flush();
    const int64_t w0 = now_ns();
    if (g_in_wait.fetch_add(1) == 0) g_in_wait_since.store(w0);
    ok = Device::event_wait(batch ? batch->ev : ev) && ok;
    if (g_in_wait.fetch_sub(1) == 1) g_in_wait_since.store(0);
    g_waits.fetch_add(1, std::memory_order_relaxed);
    g_wait_ns.fetch_add((uint64_t)(now_ns() - w0), std::memory_order_relaxed);
    if (!batch || batch->left.fetch_sub(1) == 1) {
        DevLock dl;
        g_rt->dev.event_release(batch ? batch->ev : ev);
        ok = ok && !g_rt->dev.failed();
        delete batch;
    } else {
        ok = ok && !g_rt->dev.failed();
    }
    c.staging.all_settled();         // every staged copy was enqueued before `ev`
    ctx.rows.release_up_to(done);  // every program of this codec up to `done` has completed
    return ok;
}

// varint(len) || payload into a malloc'd host buffer and a device row of `c`.
bool store_framed(Codec& c, const unsigned char* data, unsigned len, uint8_t** host_out, RowId* row_out,
                  uint32_t* framed_out, uint32_t* header_out) {
    uint8_t hdr[4];
    const uint32_t hb = put_length_header(len, hdr);
    const uint32_t framed = hb + len;
    uint8_t* host = (uint8_t*)malloc(framed);
    if (!host) return false;
    memcpy(host, hdr, hb);
    memcpy(host + hb, data, len);
    const RowId row = c.ctx.alloc(framed);
    if (row == kNoRow) { free(host); return false; }
    if (!c.staging.stage(c.ctx.rows.offset(row), host, framed)) {
        c.ctx.rows.free_deferred(row);
        free(host);
        return false;
    }
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
    // Initial arena (grown on demand up to TONK_AMD_ARENA_MAX_MB of reserved address space) and
    // the size of the ranges codecs take from it.
    // (4 GB mapped up front: every growth remaps device memory while codecs run; 288 GB per GPU)
    uint64_t arena_mb = 4096, max_mb = 64 << 10, seg_kb = 4096;
    if (const char* a = getenv("TONK_AMD_ARENA_MB")) arena_mb = strtoull(a, nullptr, 10);
    if (const char* a = getenv("TONK_AMD_ARENA_MAX_MB")) max_mb = strtoull(a, nullptr, 10);
    if (const char* a = getenv("TONK_AMD_SEGMENT_KB")) seg_kb = strtoull(a, nullptr, 10);
    if (arena_mb < 2) arena_mb = 2;
    if (seg_kb < 64) seg_kb = 64;
    g_rt->pool.seg_units = (uint32_t)(seg_kb * 1024 / TAMD_ROW_UNIT);
    // Many slots of modest size: a codec waits for its own program before its next one, so with
    // hundreds of codecs (a Tonk server) hundreds of programs are in flight, and a slot still in
    // use is waited for under the device lock, which stalls every codec behind it.  4 MB each
    // (512 MB pinned): combined batches are split to fit a slot, and a growth of all 128 slots
    // (drain + reallocation, 0.1-0.5 s with every codec waiting) inflates the round trips Tonk
    // measures for its retransmission timeouts.  A single program above 4 MB (a decode solving
    // hundreds of unknowns) takes the 32 MB oversize slot instead of growing them all: one such
    // growth stalled every codec of a Tonk test for 317 ms, and the losses the peers piled up
    // meanwhile made an acknowledgement too long for a Tonk datagram.
    size_t slot_kb = 4096, big_kb = 32768;  // (test hooks: small slots send programs to the oversize one)
    if (const char* a = getenv("TONK_AMD_CAPI_SLOT_KB")) slot_kb = strtoull(a, nullptr, 10);
    if (const char* a = getenv("TONK_AMD_CAPI_OVERSIZE_KB")) big_kb = strtoull(a, nullptr, 10);
    g_rt->dev.set_program_slots(128, slot_kb << 10, big_kb << 10);
    g_rt->dev.set_small_uploads(true);  // per-call programs are small
    if (!g_rt->dev.init_growable(device, arena_mb << 20, max_mb << 20)) {
        fprintf(stderr, "%s\n", g_rt->dev.error().c_str());
        return Siamese_Disabled;
    }
    // events and pinned staging for the codecs to come, created now: creating either later makes
    // a driver call that can block for milliseconds, and it would happen under the device lock
    g_rt->dev.reserve_events(1024);
    Device::host_prefill(4);  // (a Tonk process with 100 connections uses ~250 MB of staging)
    if (!Device::host_reserve(1)) {
        fprintf(stderr, "tonk_amd: pinned host memory unavailable\n");
        return Siamese_Disabled;
    }
    if (!g_rt->dev.gf_selftest()) {
        fprintf(stderr, "tonk_amd: device GF(256) self test failed\n");
        return Siamese_Disabled;
    }
    // One launch stream per hardware queue the runtime gives a process (GPU_MAX_HW_QUEUES, 4 by
    // default); TONK_AMD_CAPI_STREAMS overrides (1: every codec on one stream).
    unsigned nstreams = 4;
    if (const char* a = getenv("TONK_AMD_CAPI_STREAMS")) nstreams = (unsigned)atoi(a);
    if (nstreams > 1) g_rt->dev.add_streams(nstreams);
    g_rt->dev.warm_streams();
    g_rt->ok = true;
    // The launch-free path (TONK_AMD_SERVE=0: kernel launches for every call): the persistent
    // executor on TONK_AMD_SERVE_WORKERS CUs (default 64), ending after TONK_AMD_SERVE_IDLE_MS
    // (default 50) without a command and relaunched on demand.
    if (!(getenv("TONK_AMD_SERVE") && atoi(getenv("TONK_AMD_SERVE")) == 0)) {
        unsigned workers = 64;
        double idle_ms = 50;
        if (const char* a = getenv("TONK_AMD_SERVE_WORKERS")) workers = (unsigned)atoi(a);
        if (const char* a = getenv("TONK_AMD_SERVE_IDLE_MS")) idle_ms = atof(a);
        Server* srv = new Server();
        if (srv->init(g_rt->dev, workers, 4096, idle_ms)) {
            // the launch streams must not queue behind the resident kernel (a shared hardware
            // queue): each completes an empty kernel while it runs
            const double worst = g_rt->dev.probe_streams();
            if (worst > 20.0) {
                fprintf(stderr, "tonk_amd: launch streams wait %.1f ms behind the persistent executor; using kernel launches\n", worst);
                srv->stop();
            } else {
                g_srv = srv;
                atexit([] { if (g_srv) g_srv->stop(); });
                const unsigned want = getenv("TONK_AMD_CAPI_BAR") ? (unsigned)atoi(getenv("TONK_AMD_CAPI_BAR")) : 6u;
                if (want & 3u) {
                    void* p = Device::bar_alloc(4096);  // (maps the first slab now)
                    g_bar = p ? want : 0u;
                    Device::bar_free(p);
                }
            }
        } else {
            srv->stop();
        }
    }
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
    API_CALL();
    CEncoder* e = new (std::nothrow) CEncoder();
    if (!e) return nullptr;
    e->enc = new Encoder(&e->ctx, 0, release_host, nullptr);
    if (g_watch) {
        std::lock_guard<std::mutex> lk(g_enc_mu);
        g_encs.push_back(e);
    }
    return reinterpret_cast<SiameseEncoder>(e);
}

SIAMESE_EXPORT void siamese_encoder_free(SiameseEncoder encoder_t) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e) return;
    API_CALL();
    if (g_watch) {
        std::lock_guard<std::mutex> lk(g_enc_mu);
        g_encs.erase(std::remove(g_encs.begin(), g_encs.end(), e), g_encs.end());
    }
    delete e->enc;  // (the destructor may still close scans into the pending program)
    e->enc = nullptr;
    e->quiesce();
    delete e;       // rows and segments go back to the pool
}

SIAMESE_EXPORT SiameseResult siamese_encoder_is_ready(SiameseEncoder encoder_t) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e) return Siamese_InvalidInput;
    API_CALL();
    if (e->enc->remaining_slots() <= 2) API_RC(Siamese_MaxPacketsReached);
    API_RC(Siamese_Success);
}

SIAMESE_EXPORT SiameseResult siamese_encoder_add(SiameseEncoder encoder_t, SiameseOriginalPacket* packet) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || !packet || !packet->Data || packet->DataBytes <= 0 || packet->DataBytes > SIAMESE_MAX_PACKET_BYTES)
        return Siamese_InvalidInput;
    API_CALL();
    e->cancel_ahead();
    if (e->enc->disabled()) return Siamese_Disabled;
    if (e->enc->remaining_slots() <= 0) return Siamese_MaxPacketsReached;
    uint8_t* host = nullptr;
    RowId row = kNoRow;
    uint32_t framed = 0, hb = 0;
    if (!store_framed(*e, packet->Data, packet->DataBytes, &host, &row, &framed, &hb)) {
        DISABLE(e->enc);
        return Siamese_Disabled;
    }
    uint32_t pn = 0;
    const Result r = e->enc->add(row, framed, hb, packet->DataBytes, host, &pn);
    if (r != kSuccess) {
        e->ctx.rows.free_deferred(row);
        free(host);
        return (SiameseResult)r;
    }
    packet->PacketNum = pn;
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_get(SiameseEncoder encoder_t, SiameseOriginalPacket* packet) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || !packet || packet->PacketNum > SIAMESE_PACKET_NUM_MAX) return Siamese_InvalidInput;
    API_CALL();
    StoredOriginal ov;
    const StoredOriginal* o = &ov;
    const Result r = e->enc->get(packet->PacketNum, &ov);
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
    API_CALL();
    e->cancel_ahead();
    e->enc->remove_before(packetNum);
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_ack(SiameseEncoder encoder_t, const void* buffer, unsigned bytes,
                                                 unsigned* nextExpectedPacketNum) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || !buffer || bytes < 1 || !nextExpectedPacketNum) return Siamese_InvalidInput;
    API_CALL();
    e->cancel_ahead();
    uint32_t next = 0;
    const Result r = e->enc->acknowledge((const uint8_t*)buffer, bytes, &next);
    if (r == kSuccess) *nextExpectedPacketNum = next;
    return (SiameseResult)r;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_retransmit(SiameseEncoder encoder_t, SiameseOriginalPacket* original) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || !original) return Siamese_InvalidInput;
    API_CALL();
    e->cancel_ahead();
    original->Data = nullptr;
    original->DataBytes = 0;
    StoredOriginal ov;
    const StoredOriginal* o = &ov;
    const Result r = e->enc->retransmit(&ov);
    if (r != kSuccess) API_RC(r);
    original->PacketNum = o->column;
    original->Data = (const unsigned char*)o->host + o->header_bytes;
    original->DataBytes = o->bytes - o->header_bytes;
    API_RC(Siamese_Success);
}

SIAMESE_EXPORT SiameseResult siamese_encode(SiameseEncoder encoder_t, SiameseRecoveryPacket* recovery) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || !recovery) return Siamese_InvalidInput;
    API_CALL();
    if (e->ahead_next < e->ahead.size()) {  // encoded ahead (CEncoder)
        const CEncoder::Ahead& a = e->ahead[e->ahead_next++];
        recovery->Data = e->pinned + a.off;
        recovery->DataBytes = a.total;
        return Siamese_Success;
    }
    static const uint32_t kAheadMax = getenv("TONK_AMD_CAPI_AHEAD") ? (uint32_t)atoi(getenv("TONK_AMD_CAPI_AHEAD")) : 63u;
    if (!e->ahead.empty()) {  // all of them used
        e->depth = 2 * e->depth < kAheadMax ? 2 * e->depth : kAheadMax;
        e->ahead.clear();
        e->marks.clear();
        e->ahead_next = 0;
    }
    thread_local std::vector<RecoveryOut> outs;
    outs.resize(1);
    const Result r = e->enc->encode(outs[0]);
    if (r == kDisabled) report_disable("Encoder::encode");
    if (r != kSuccess) {
        e->last_encode = false;
        if (r == kNeedMoreData) recovery->DataBytes = 0;
        return (SiameseResult)r;
    }
    if (kAheadMax && e->last_encode) {
        // (within what one executor command holds: 16 B an instruction in its 64 KB)
        for (uint32_t k = 0; k < e->depth && e->ctx.pb.instrs().size() < 2500 && e->enc->encode_is_quiet(); ++k) {
            const Encoder::Mark m = e->enc->mark();
            RecoveryOut o;
            if (e->enc->encode(o) != kSuccess) {
                e->enc->rewind(m);
                break;
            }
            e->marks.push_back(m);
            outs.push_back(o);
        }
    }
    e->last_encode = true;
    size_t bytes = 0;
    for (const RecoveryOut& o : outs) bytes += (o.total() + 63u) & ~(size_t)63;
    bool ok = e->ensure_pinned(bytes);
    // the program and the read of the recovery rows behind it, waited for without a lock
    if (ok) {
        thread_local std::vector<Device::HostCopy> rd;
        rd.clear();
        size_t at = 0;
        for (size_t i = 0; i < outs.size(); ++i) {
            rd.push_back(Device::HostCopy{e->pinned + at, e->byte_offset(outs[i].row), outs[i].total()});
            if (i) e->ahead.push_back(CEncoder::Ahead{at, outs[i].total()});
            at += (outs[i].total() + 63u) & ~(size_t)63;
        }
        ok = run_and_read(*e, rd);
    }
    for (const RecoveryOut& o : outs) e->ctx.rows.free_deferred(o.row);  // released once the codec's next program completes
    if (!ok) {
        e->ahead.clear();
        e->marks.clear();
        DISABLE(e->enc);
        return Siamese_Disabled;
    }
    recovery->Data = e->pinned;
    recovery->DataBytes = outs[0].total();
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_stats(SiameseEncoder encoder_t, uint64_t* statsOut, unsigned statsCount) {
    CEncoder* e = reinterpret_cast<CEncoder*>(encoder_t);
    if (!e || !statsOut || statsCount <= 0) return Siamese_InvalidInput;
    API_CALL();
    e->cancel_ahead();
    e->enc->stats(statsOut, statsCount);
    return Siamese_Success;
}

// ---------------------------------------------------------------------------- Decoder API

SIAMESE_EXPORT SiameseDecoder siamese_decoder_create() {
    if (!g_rt || !g_rt->ok) return nullptr;
    API_CALL();
    CDecoder* d = new (std::nothrow) CDecoder();
    if (!d) return nullptr;
    d->dec = new Decoder(&d->ctx, 0, release_host, nullptr);
    return reinterpret_cast<SiameseDecoder>(d);
}

SIAMESE_EXPORT void siamese_decoder_free(SiameseDecoder decoder_t) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d) return;
    API_CALL();
    delete d->dec;
    d->dec = nullptr;
    d->quiesce();
    delete d;
}

SIAMESE_EXPORT SiameseResult siamese_decoder_add_original(SiameseDecoder decoder_t, const SiameseOriginalPacket* packet) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d || !packet || packet->DataBytes <= 0 || packet->DataBytes > SIAMESE_MAX_PACKET_BYTES ||
        packet->PacketNum > SIAMESE_PACKET_NUM_MAX)
        return Siamese_InvalidInput;
    if (!packet->Data) return Siamese_InvalidInput;
    API_CALL();
    if (d->dec->disabled()) return Siamese_Disabled;
    uint8_t* host = nullptr;
    RowId row = kNoRow;
    uint32_t framed = 0, hb = 0;
    if (!store_framed(*d, packet->Data, packet->DataBytes, &host, &row, &framed, &hb)) {
        DISABLE(d->dec);
        return Siamese_Disabled;
    }
    bool took = false;
    const Result r = d->dec->add_original(packet->PacketNum, row, framed, hb, packet->DataBytes, host, &took);
    if (!took) {
        d->ctx.rows.free_deferred(row);
        free(host);
    }
    return (SiameseResult)r;
}

SIAMESE_EXPORT SiameseResult siamese_decoder_add_recovery(SiameseDecoder decoder_t, const SiameseRecoveryPacket* packet) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d || !packet || !packet->Data || packet->DataBytes <= 0 || packet->DataBytes > SIAMESE_MAX_PACKET_BYTES)
        return Siamese_InvalidInput;
    API_CALL();
    if (d->dec->disabled()) return Siamese_Disabled;
    const uint32_t total = packet->DataBytes;
    const RowId row = d->ctx.alloc(total);
    if (row == kNoRow) { DISABLE(d->dec); return Siamese_Disabled; }
    if (!d->staging.stage(d->ctx.rows.offset(row), packet->Data, total)) {
        d->ctx.rows.free_deferred(row);
        DISABLE(d->dec);
        return Siamese_Disabled;
    }
    const uint32_t tl = total < 8 ? total : 8;
    bool took = false;
    const Result r = d->dec->add_recovery(row, total, packet->Data + total - tl, packet->Data, &took);
    if (!took) d->ctx.rows.free_deferred(row);
    return (SiameseResult)r;
}

namespace {

// The host copy of recovered rows: `rows` read back behind the decoder's pending program into
// the decoder's pinned buffer, then each framed row's length header parsed (BackSubstitution's
// length check, SiameseDecoder.cpp:1139-1154) and its bytes copied to a malloc'd mirror.
bool read_back(CDecoder& d, const std::vector<std::pair<StoredOriginal*, RowId>>& rows, const std::vector<uint32_t>& upper) {
    size_t total = 0;
    std::vector<size_t> at(rows.size());
    for (size_t i = 0; i < rows.size(); ++i) {
        at[i] = total;
        total += (upper[i] + 63) & ~(size_t)63;
    }
    if (!d.ensure_pinned(total ? total : 64)) return false;
    thread_local std::vector<Device::HostCopy> rd;
    rd.clear();
    for (size_t i = 0; i < rows.size(); ++i)
        rd.push_back(Device::HostCopy{d.pinned + at[i], d.byte_offset(rows[i].second), upper[i]});
    const bool ok = run_and_read(d, rd);
    if (!ok) return false;
    for (size_t i = 0; i < rows.size(); ++i) {
        StoredOriginal* o = rows[i].first;
        const uint8_t* src = d.pinned + at[i];
        unsigned len = 0;
        const int hb = get_length_header(src, upper[i], len);
        if (hb < 1 || len == 0 || (uint32_t)hb + len > upper[i]) return false;
        uint8_t* host = (uint8_t*)malloc((size_t)hb + len);
        if (!host) return false;
        memcpy(host, src, (size_t)hb + len);
        o->host = host;
        o->header_bytes = (uint32_t)hb;
        o->bytes = (uint32_t)hb + len;
    }
    return true;
}

} // namespace

SIAMESE_EXPORT SiameseResult siamese_decoder_get(SiameseDecoder decoder_t, SiameseOriginalPacket* packet) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d || !packet || packet->PacketNum > SIAMESE_PACKET_NUM_MAX) return Siamese_InvalidInput;
    API_CALL();
    StoredOriginal* o = nullptr;
    const Result r = d->dec->get(packet->PacketNum, &o);
    if (r != kSuccess) {
        packet->Data = nullptr;
        packet->DataBytes = 0;
        return (SiameseResult)r;
    }
    if (!o->host) {  // recovered data not read back yet
        std::vector<std::pair<StoredOriginal*, RowId>> rows(1, std::make_pair(o, o->row));
        std::vector<uint32_t> upper(1, o->bytes);
        if (!read_back(*d, rows, upper)) { DISABLE(d->dec); return Siamese_Disabled; }
    }
    packet->Data = (const unsigned char*)o->host + o->header_bytes;
    packet->DataBytes = o->bytes - o->header_bytes;
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_decoder_is_ready(SiameseDecoder decoder_t) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d) return Siamese_InvalidInput;
    API_CALL();
    return (SiameseResult)d->dec->is_ready();
}

SIAMESE_EXPORT SiameseResult siamese_decode(SiameseDecoder decoder_t, SiameseOriginalPacket** packetsPtrOut,
                                            unsigned* countOut) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d || (!packetsPtrOut != !countOut)) return Siamese_InvalidInput;
    API_CALL();
    if (packetsPtrOut) {
        *packetsPtrOut = nullptr;
        *countOut = 0;
    }
    std::vector<RecoveredPacket*> got;
    const Result r = d->dec->decode(got);
    if (r == kDisabled) report_disable("Decoder::decode");
    if (r != kSuccess) return (SiameseResult)r;
    // every recovered row not read back yet: one D2H each behind the program, one wait
    std::vector<std::pair<StoredOriginal*, RowId>> rows;
    std::vector<uint32_t> upper;
    std::vector<StoredOriginal*> outs;
    for (RecoveredPacket* rp : got) {
        StoredOriginal* o = nullptr;
        if (d->dec->get(rp->packet_num, &o, true) != kSuccess || !o) { DISABLE(d->dec); return Siamese_Disabled; }
        outs.push_back(o);
        if (!o->host) {
            rows.push_back(std::make_pair(o, rp->row));
            upper.push_back(rp->framed_upper);
        }
    }
    if (!read_back(*d, rows, upper)) { DISABLE(d->dec); return Siamese_Disabled; }
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
    API_CALL();
    uint32_t used = 0;
    const Result r = d->dec->ack((uint8_t*)buffer, byteLimit, &used);
    *usedBytes = used;
    return (SiameseResult)r;
}

SIAMESE_EXPORT SiameseResult siamese_decoder_stats(SiameseDecoder decoder_t, uint64_t* statsOut, unsigned statsCount) {
    CDecoder* d = reinterpret_cast<CDecoder*>(decoder_t);
    if (!d || !statsOut || statsCount <= 0) return Siamese_InvalidInput;
    API_CALL();
    d->dec->stats(statsOut, statsCount);
    return Siamese_Success;
}

} // extern "C"
