// session.cpp -- batched device-resident runner (include/tonk_amd.h).
//
// Every stream (encoder + decoder + lossy channel) owns one Context: a disjoint range of the
// HBM arena and its own pending program.  A step: host threads take streams dynamically and
// advance each by N originals (control planes emit symbolic ops), then the streams' programs are
// merged into one and enqueued level by level on the device stream.  The host then starts the next step while the device
// executes; rows freed during a step are reused only once that step's program has completed.
#include "../../include/tonk_amd.h"

#include "decoder.h"
#include "device.h"
#include "workload.h"
#include "transcript.h"

#include <hip/hip_runtime.h>

#include <chrono>
#include <atomic>
#include <algorithm>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

using namespace tamd;

namespace {

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}
std::vector<int> parse_cpulist(const char* text) {
    std::vector<int> out;
    std::string line(text ? text : "");
    size_t at = 0;
    while (at < line.size()) {
        size_t end = line.find_first_of(",\n", at);
        if (end == std::string::npos) end = line.size();
        int a = 0, b = 0;
        const int n = sscanf(line.substr(at, end - at).c_str(), "%d-%d", &a, &b);
        if (n >= 1) {
            if (n == 1) b = a;
            for (int c = a; c <= b && c >= 0 && c < CPU_SETSIZE; ++c) out.push_back(c);
        }
        at = end + 1;
    }
    return out;
}

// The share of a NUMA node's cores that one GPU's pool takes when several GPUs hang off the same
// node (4 per socket on an 8-GPU MI355X node): the devices whose local_cpulist equals this
// device's split `node_cores` into equal contiguous shares in device order (the remainder to
// the first), so the ranks of one node never pin their threads to the same cores (the
// reference's equivalent is one worker pool per process over all cores,
// TonkineseSession.cpp:71-102).  `slot_override` "k/n" (TONK_AMD_CPU_SLOT) replaces the device
// scan, for launchers that give each rank only its own GPU.  Pure: tested on CPU.
std::vector<int> node_core_share(const std::vector<std::string>& dev_cpulists, unsigned device,
                                 const std::vector<int>& node_cores, const char* slot_override,
                                 unsigned* slot_out = nullptr, unsigned* nslots_out = nullptr) {
    unsigned slot = 0, nslots = 1;
    unsigned k = 0, n = 0;
    if (slot_override && sscanf(slot_override, "%u/%u", &k, &n) == 2 && n >= 1 && k < n) {
        slot = k;
        nslots = n;
    } else if (device < dev_cpulists.size()) {
        nslots = 0;
        for (size_t d = 0; d < dev_cpulists.size(); ++d) {
            if (dev_cpulists[d] != dev_cpulists[device]) continue;
            if (d < device) ++slot;
            ++nslots;
        }
    }
    if (slot_out) *slot_out = slot;
    if (nslots_out) *nslots_out = nslots;
    const size_t N = node_cores.size();
    if (nslots <= 1 || N < nslots) return node_cores;
    const size_t base = N / nslots, extra = N % nslots;
    const size_t begin = slot * base + (slot < extra ? slot : extra);
    const size_t len = base + (slot < extra ? 1 : 0);
    return std::vector<int>(node_cores.begin() + begin, node_cores.begin() + begin + len);
}

std::string read_line(const std::string& path) {
    FILE* f = fopen(path.c_str(), "r");
    if (!f) return std::string();
    char line[4096] = {0};
    const bool ok = fgets(line, sizeof(line), f) != nullptr;
    fclose(f);
    std::string s = ok ? std::string(line) : std::string();
    while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
    return s;
}

std::string device_cpulist(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return std::string();
    for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
    return read_line(std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist");
}

// CPUs of the device's NUMA node (the PCI device's local_cpulist) that this process may run on,
// one hardware thread per core, and of those this device's share (node_core_share);
// TONK_AMD_AFFINITY=node keeps both SMT threads, =none returns nothing (no pinning).  The
// control-plane threads run there so their stream state lives in the node next to the GPU.
// Bench A/B on one box (40 steps, twice each): 224-227 GiB/s with one thread per core, 212-226
// with the node's CPUs, 199-217 unpinned.
std::vector<int> device_local_cpus(int device) {
    const char* mode = getenv("TONK_AMD_AFFINITY");
    std::vector<int> out;
    if (mode && !strcmp(mode, "none")) return out;
    const std::string mine = device_cpulist(device);
    if (mine.empty()) return out;
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return out;
    const bool one_per_core = !(mode && !strcmp(mode, "node"));
    for (int c : parse_cpulist(mine.c_str())) {
        if (!CPU_ISSET(c, &allowed)) continue;
        if (one_per_core) {
            char tp[128];
            snprintf(tp, sizeof(tp), "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", c);
            const std::vector<int> sib = parse_cpulist(read_line(tp).c_str());
            if (!sib.empty() && sib[0] != c) continue;
        }
        out.push_back(c);
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    std::vector<std::string> lists;
    for (int d = 0; d < n; ++d) lists.push_back(device_cpulist(d));
    return node_core_share(lists, (unsigned)device, out, getenv("TONK_AMD_CPU_SLOT"));
}

// Busy jiffies of each CPU so far (/proc/stat: every process on the host), indexed by CPU.
std::vector<uint64_t> cpu_busy_jiffies() {
    std::vector<uint64_t> busy;
    FILE* f = fopen("/proc/stat", "r");
    if (!f) return busy;
    char line[512];
    while (fgets(line, sizeof(line), f)) {
        if (strncmp(line, "cpu", 3) != 0 || line[3] < '0' || line[3] > '9') continue;
        unsigned c = 0;
        unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (sscanf(line + 3, "%u %llu %llu %llu %llu %llu %llu %llu %llu", &c, &v[0], &v[1], &v[2], &v[3], &v[4],
                   &v[5], &v[6], &v[7]) < 5)
            continue;
        if (c >= busy.size()) busy.resize(c + 1, 0);
        busy[c] = v[0] + v[1] + v[2] + v[5] + v[6] + v[7];  // user nice system irq softirq steal
    }
    fclose(f);
    return busy;
}

// The `want` least busy CPUs of `share` over a short sampling window (ties: lower CPU first),
// in ascending order.  The GPU box's CPUs are shared with other jobs' threads; a pool thread
// pinned to a core another job keeps busy is descheduled for milliseconds at a time, and the
// step waits for it.  Pure selection in pick_idle(); the sampling reads /proc/stat.
std::vector<int> pick_idle(const std::vector<int>& share, const std::vector<uint64_t>& busy_delta, size_t want) {
    if (share.size() <= want) return share;
    std::vector<int> order(share);
    auto busy = [&](int c) { return (size_t)c < busy_delta.size() ? busy_delta[c] : 0; };
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return busy(a) < busy(b); });
    order.resize(want);
    std::sort(order.begin(), order.end());
    return order;
}

std::vector<int> idle_cpus(const std::vector<int>& share, size_t want) {
    static const bool off = getenv("TONK_AMD_NO_IDLE_PICK") != nullptr;  // A/B switch
    if (off || share.size() <= want) return share.size() > want ? std::vector<int>(share.begin(), share.begin() + want) : share;
    const std::vector<uint64_t> a = cpu_busy_jiffies();
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    const std::vector<uint64_t> b = cpu_busy_jiffies();
    std::vector<uint64_t> d(b.size(), 0);
    for (size_t i = 0; i < b.size() && i < a.size(); ++i) d[i] = b[i] - a[i];
    return pick_idle(share, d, want);
}

struct Stream;

// Transcript in the oracle's format (record mode).  The digests of device rows are computed on
// the device (Device::verify_next) right after the launch that completes their program, and
// filled into the lines at the end of the run.
struct SessTranscript {
    bool on = false;
    std::vector<std::string> lines;
    // rows whose digest goes into line `pos`; `v` = index of the digest among the session's
    // verification results (assigned when the rows are registered after their pass)
    struct PendEnc { RowId row; uint32_t total; RecoveryMeta meta; size_t pos; uint64_t v; };
    struct PendDec { RowId row; uint32_t upper; size_t pos; uint64_t v; };
    std::vector<PendEnc> pend_enc;
    std::vector<PendDec> pend_dec;
    size_t reg_enc = 0, reg_dec = 0;  // entries [0, reg_*) are registered
};

struct Stream {
    wl::Params p;
    Context* ctx = nullptr;
    std::unique_ptr<Encoder> enc;
    std::unique_ptr<Decoder> dec;
    std::vector<RowId> enc_rows, dec_rows;
    uint32_t pool = 0;        // input rows per side (original i reads row i mod pool)
    bool pool_affine = false; // each side's pool rows are consecutive handles at one arena stride:
    uint32_t pool_off[2] = {0, 0}, pool_stride = 0;  // row i mod pool at pool_off[side] + (i mod pool) * stride
    std::vector<uint32_t> framed;
    std::vector<uint8_t> dec_row_used;
    SessTranscript tr;
    uint64_t alg_bytes = 0, payload_bytes = 0;
    // stage_host: rows this step produced that leave through PCIe (recovery packets, recovered
    // originals) and the recovery bytes the decoder received (which arrived through PCIe)
    uint32_t stage = 0;  // stage_host mask: 1 sender side staged, 2 receiver side
    std::vector<std::pair<RowId, uint32_t>> out_rows;
    uint64_t recv_bytes = 0;

    // ---- workload backend ----
    struct RecRef { RecoveryOut out; };
    struct DecRef {};

    int enc_add(uint32_t index, uint32_t len, uint32_t* col) {
        const uint32_t hb = length_header_bytes(len);
        // input rows are generated once in HBM and borrowed by the codecs (never freed)
        const Result r = enc->add(enc_rows[index], hb + len, hb, len, nullptr, col, true);
        if (r == kSuccess) {
            alg_bytes += hb + len;
            payload_bytes += len;
        }
        return r;
    }
    // Input rows were allocated back to back per side (generate), so a run that does not wrap
    // the input pool is consecutive handles at one stride: the codecs get its layout instead of
    // checking and looking it up (the row table is cold).
    uint64_t layout(int side, uint32_t index, uint32_t k) const {
        if (!pool_affine || index % pool + k > pool) return 0;
        return (uint64_t)(pool_off[side] + (index % pool) * pool_stride) << 32 | pool_stride;
    }
    bool enc_add_run(uint32_t index, uint32_t k, uint32_t len, uint32_t* col0) {
        const uint32_t hb = length_header_bytes(len);
        if (!enc->add_run(&enc_rows[index], k, hb + len, hb, len, true, col0, layout(0, index, k))) return false;
        alg_bytes += (uint64_t)(hb + len) * k;
        payload_bytes += (uint64_t)len * k;
        return true;
    }
    bool dec_add_run(uint32_t col0, uint32_t index, uint32_t k, uint32_t len) {
        const uint32_t hb = length_header_bytes(len);
        if (!dec->add_run_inorder(col0, &dec_rows[index], k, hb + len, hb, len, true, layout(1, index, k))) return false;
        alg_bytes += (uint64_t)(hb + len) * k;
        return true;
    }
    int enc_encode(RecRef& r) {
        const Result rc = enc->encode(r.out);
        if (rc == kSuccess) {
            alg_bytes += r.out.total();
            if (stage & 1u) out_rows.push_back(std::make_pair(r.out.row, r.out.total()));
        }
        return rc;
    }
    int enc_ack(const uint8_t* buf, uint32_t n, uint32_t* next) { return enc->acknowledge(buf, n, next); }
    int enc_is_ready() { return enc->remaining_slots() <= 2 ? (int)kMaxPacketsReached : 0; }
    int dec_add_original(uint32_t col, uint32_t index, uint32_t len) {
        const uint32_t hb = length_header_bytes(len);
        bool took = false;
        const Result r = dec->add_original(col, dec_rows[index], hb + len, hb, len, nullptr, &took, true);
        alg_bytes += hb + len;
        return r;
    }
    void recovery_lost(const RecRef& r) { ctx->rows.free_deferred(r.out.row); }
    int dec_add_recovery(const RecRef& r) {
        uint8_t tail[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const uint32_t tl = r.out.total() < 8 ? r.out.total() : 8;
        memcpy(tail + tl - r.out.footer_len, r.out.footer, r.out.footer_len);
        bool took = false;
        const Result rc = dec->add_recovery(r.out.row, r.out.total(), tail, nullptr, &took);
        if (!took) ctx->rows.free_deferred(r.out.row);
        alg_bytes += r.out.total();
        if (stage & 2u) recv_bytes += r.out.total();
        return rc;
    }
    int dec_is_ready() { return dec->is_ready(); }
    std::vector<RecoveredPacket*> got_;
    int dec_decode(std::vector<uint32_t>& nums, DecRef&) {
        got_.clear();
        const Result rc = dec->decode(got_);
        if (rc == kSuccess) {
            for (RecoveredPacket* rp : got_) {
                nums.push_back(rp->packet_num);
                alg_bytes += rp->framed_upper;
                if (stage & 2u) out_rows.push_back(std::make_pair(rp->row, rp->framed_upper));
                if (tr.on) tr.pend_dec.push_back(SessTranscript::PendDec{rp->row, rp->framed_upper, tr.lines.size(), 0});
            }
        }
        return rc;
    }
    int dec_ack(uint8_t* buf, uint32_t limit, uint32_t* used) { return dec->ack(buf, limit, used); }
    void stats(uint64_t e[9], uint64_t d[11]) { enc->stats(e, 9); dec->stats(d, 11); }
    uint64_t vclock = 0;
    void set_time(uint64_t ms) {
        if (!vclock) enc->set_clock(&vclock);
        vclock = ms;
    }
    int enc_retransmit(uint32_t* num, uint32_t* bytes, const uint8_t** data) {
        StoredOriginal ov;
        const StoredOriginal* o = &ov;
        const Result rc = enc->retransmit(&ov);
        if (rc == kSuccess) {
            *num = o->column;
            *bytes = o->bytes - o->header_bytes;
            *data = nullptr;  // the payload lives in HBM; the runner regenerates it for the digest
        }
        return rc;
    }

    // ---- transcript ----
    void on_encode(int rc, const RecRef& r) {
        if (!tr.on) return;
        if (rc != 0) { tr.lines.push_back("E " + std::to_string(rc)); return; }
        tr.pend_enc.push_back(SessTranscript::PendEnc{r.out.row, r.out.total(), r.out.meta, tr.lines.size(), 0});
        tr.lines.push_back("E ?");
    }
    void on_decode(int rc, const std::vector<uint32_t>& nums, const DecRef&) {
        if (!tr.on) return;
        std::string ln = "D " + std::to_string(rc) + " " + std::to_string(nums.size());
        for (uint32_t n : nums) ln += " " + std::to_string(n) + "#";
        // pend_dec entries were pushed with pos = lines.size() before this line is appended
        tr.lines.push_back(ln);
    }
    void on_ack(int rd, const uint8_t* buf, uint32_t used, int re, uint32_t next) {
        if (!tr.on) return;
        char b[128];
        snprintf(b, sizeof(b), "K %d %u %016llx %d %u", rd, used, (unsigned long long)wl::fnv1a(buf, used), re, next);
        tr.lines.push_back(b);
    }
    void on_event(char kind, int rc, uint32_t a, uint32_t b) {
        if (!tr.on || rc == 0) return;
        char t[64];
        snprintf(t, sizeof(t), "%c %d %u %u", kind, rc, a, b);
        tr.lines.push_back(t);
    }
    void on_retransmit(int rc, uint32_t num, uint32_t bytes, uint64_t h) {
        if (!tr.on) return;
        wl::TextSink t;
        wl::fmt_retransmit(t, rc, num, bytes, h);
        t.text.pop_back();
        tr.lines.push_back(t.text);
    }
    void on_stats(const uint64_t e[9], const uint64_t d[11]) {
        if (!tr.on) return;
        std::string s = "S";
        for (int i = 0; i < 8; ++i) s += " " + std::to_string(e[i]);
        s += " |";
        for (int i = 0; i < 10; ++i) s += " " + std::to_string(d[i]);
        tr.lines.push_back(s);
    }

    std::unique_ptr<wl::Runner<Stream, Stream>> runner;

    // free-running schedule (Session::fr_*): the next step this stream runs, a claim flag (one
    // thread at a time), the send clock of the step being run, and its part of each open program
    std::atomic<uint32_t> next_step{0};
    std::atomic<uint8_t> busy{0};
    uint64_t clock = 0;
    static const unsigned kParts = 8;
    Device::Part parts[kParts];
};

// One stream = one Context (its own arena range and pending program), so host threads can take
// streams dynamically and a stream's ops are laid out contiguously in the merged program.
struct Session {
    tamd_session_params prm;
    Device dev;
    std::vector<std::unique_ptr<Stream>> streams;
    std::vector<std::unique_ptr<Context>> ctxs;     // ctxs[i] belongs to streams[i]
    std::vector<double> busy_ms;                    // per thread, control-plane time of a step
    std::vector<double> fill_ms;                    // per thread, program fill time (deferred mode)
    std::vector<std::pair<uint64_t, uint64_t>> epoch_ticket;  // (epoch, ticket) awaiting release
    uint64_t last_ticket = 0, released_epoch = 0;
    double host_ms[6] = {0, 0, 0, 0, 0, 0};
    uint64_t clock_msec = 0;  // packet send times of a step (RTO bookkeeping only)
    uint32_t row_cap = 0;
    // stage_host: every stream's inputs (both sides, packet order) in pinned host memory, and
    // the pinned landing buffer of a step's outgoing rows
    uint8_t* host_in = nullptr;
    size_t host_in_bytes = 0;
    uint8_t* host_out = nullptr;
    size_t host_out_cap = 0;
    uint64_t h2d_bytes = 0, d2h_bytes = 0;
    bool finished = false;
    std::string error;

    // thread pool: run_all(f) calls f(stream index, thread index) for every stream, streams
    // handed out dynamically (an atomic counter) so uneven streams balance across threads
    std::vector<std::thread> threads;
    std::vector<int> cpus;  // pool threads' CPU set (device_local_cpus), empty = not pinned
    size_t threads_wanted = 0;
    std::mutex mu;
    std::condition_variable cv_start, cv_done;
    std::atomic<bool> main_sleeping{false};
    const std::function<void(size_t, size_t)>* job = nullptr;  // the pass being run (run_all)
    std::atomic<size_t> next_item{0};
    std::atomic<bool> quit{false};

    ~Session() {
        if (fr_running) fr_drain();
        quit.store(true);
        {
            std::lock_guard<std::mutex> lk(mu);
            gen.fetch_add(1);
        }
        cv_start.notify_all();
        for (auto& t : threads) t.join();
        dev.synchronize();
        dev.sync_staging();
        if (host_in) hipHostFree(host_in);
        if (host_out) hipHostFree(host_out);
        for (auto& s : streams) {
            s->runner.reset();
            s->enc.reset();
            s->dec.reset();
        }
    }

    // Streams are handed out longest first (by their control-plane time in the previous step),
    // so the step does not end waiting for one expensive stream picked up last.
    std::vector<uint32_t> order;
    std::vector<double> stream_ms;

    // Sticky mode (default): thread t first runs its own streams (s % T == t), longest first, so
    // a stream's state stays in the same core's caches from step to step, then takes any stream
    // still unclaimed, longest first.  Without it streams are handed out longest first only.
    std::vector<std::atomic<uint8_t>> claimed;
    bool sticky_job = false;
    void drain(const std::function<void(size_t, size_t)>& f, size_t ti) {
        if (sticky_job) {
            // own streams longest first (by the previous pass), so what is left for others to
            // steal at the end of a pass is a slow thread's shortest streams
            static const bool own_fifo = getenv("TONK_AMD_OWN_FIFO") != nullptr;  // A/B switch (profiling)
            const size_t T = threads.size(), n = streams.size();
            if (own_fifo || order.empty()) {
                for (size_t s = ti; s < n; s += T)
                    if (!claimed[s].exchange(1)) f(s, ti);
            } else {
                for (size_t k = 0; k < n; ++k) {
                    const size_t s = order[k];
                    if (s % T == ti && !claimed[s].exchange(1)) f(s, ti);
                }
            }
            for (size_t k = 0; k < n; ++k) {
                const size_t s = order.empty() ? k : order[k];
                if (!claimed[s].exchange(1)) f(s, ti);
            }
            return;
        }
        for (;;) {
            const size_t i = next_item.fetch_add(1);
            if (i >= streams.size()) break;
            f(order.empty() ? i : order[i], ti);
        }
    }

    // Workers spin on the job generation for a while before sleeping on the condition variable,
    // and the main thread spins for the end of a pass: a step is a few hundred microseconds, so
    // a futex wake-up of 16 threads (and of the main thread) per pass is a visible share of it.
    // TONK_AMD_SPIN_US sets the spin window (0: always sleep); 100 us covers the caller's work
    // between passes (launch + layout, ~0.05 ms) without keeping 16 spinning threads beside the
    // caller for long (the job's CPU quota counts them).
    static uint64_t spin_ns() {
        static const uint64_t v = getenv("TONK_AMD_SPIN_US") ? 1000ull * strtoull(getenv("TONK_AMD_SPIN_US"), nullptr, 10)
                                                            : 100000ull;
        return v;
    }
    std::atomic<uint64_t> gen{0};
    std::atomic<size_t> left{0};
    std::atomic<int> sleepers{0};

    void pool_loop(size_t ti) {
        // A pool thread may launch the step's program (early launch): its HIP calls (events,
        // launches) must target the session's device, not device 0.
        dev.bind_thread();
        // Each pool thread on a core of its own (with sticky streams its streams' state stays in
        // that core's caches); TONK_AMD_PIN=set lets every thread float over the whole CPU set.
        static const bool pin_set = getenv("TONK_AMD_PIN") && !strcmp(getenv("TONK_AMD_PIN"), "set");
        if (!cpus.empty()) {
            cpu_set_t set;
            CPU_ZERO(&set);
            if (pin_set || cpus.size() < threads_wanted) {
                for (int c : cpus) CPU_SET(c, &set);
            } else {
                CPU_SET(cpus[ti % cpus.size()], &set);
            }
            pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
        }
        uint64_t seen = 0;
        for (;;) {
            if (gen.load(std::memory_order_acquire) == seen) {
                const auto until = std::chrono::steady_clock::now() + std::chrono::nanoseconds(spin_ns());
                unsigned k = 0;
                while (gen.load(std::memory_order_acquire) == seen) {
                    __builtin_ia32_pause();
                    if ((++k & 255) == 0 && std::chrono::steady_clock::now() > until) break;
                }
            }
            if (gen.load(std::memory_order_acquire) == seen) {
                std::unique_lock<std::mutex> lk(mu);
                sleepers.fetch_add(1);
                cv_start.wait(lk, [&] { return gen.load() != seen; });
                sleepers.fetch_sub(1);
            }
            seen = gen.load(std::memory_order_acquire);
            if (quit.load(std::memory_order_acquire)) return;
            if (job_kind.load(std::memory_order_acquire) == 1) fr_loop(ti);
            else drain(*job, ti);
            if (left.fetch_sub(1, std::memory_order_acq_rel) == 1 && main_sleeping.load()) {
                std::lock_guard<std::mutex> lk(mu);
                cv_done.notify_one();
            }
        }
    }

    void run_all(const std::function<void(size_t, size_t)>& f) {
        if (fr_running) fr_drain();  // (the pool leaves the free-running loop first)
        static const bool sticky = getenv("TONK_AMD_NO_STICKY") == nullptr;  // A/B switch (profiling)
        next_item = 0;
        sticky_job = sticky && !threads.empty();
        if (sticky_job) {
            if (claimed.size() != streams.size()) claimed = std::vector<std::atomic<uint8_t>>(streams.size());
            for (auto& c : claimed) c.store(0, std::memory_order_relaxed);
        }
        if (threads.empty()) {
            drain(f, 0);
            return;
        }
        job = &f;
        job_kind.store(0, std::memory_order_relaxed);
        left.store(threads.size(), std::memory_order_relaxed);
        gen.fetch_add(1, std::memory_order_seq_cst);
        if (sleepers.load(std::memory_order_seq_cst) > 0) {
            std::lock_guard<std::mutex> lk(mu);
            cv_start.notify_all();
        }
        wait_pass_end();
    }

    // The caller blocks for the end of the pass (after a short spin): the workers already
    // occupy the job's CPU share (cpu.max on the GPU box), a spinning 17th thread would push the
    // process over its quota and get it throttled.
    void wait_pass_end() {
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(20);
        unsigned k = 0;
        while (left.load(std::memory_order_acquire) != 0) {
            __builtin_ia32_pause();
            if ((++k & 255) == 0 && std::chrono::steady_clock::now() > until) {
                std::unique_lock<std::mutex> lk(mu);
                main_sleeping.store(true);
                cv_done.wait(lk, [&] { return left.load() == 0; });
                main_sleeping.store(false);
                break;
            }
        }
    }

    // ---- free-running schedule (sessions with worker threads, level pipelining) ----
    // tamd_session_step publishes a step and returns; the workers run every stream through every
    // published step, each stream's steps in order, a thread's own streams first (s % T == t: its
    // state stays in that core's caches) and any other runnable stream when it has none, with no
    // barrier between steps: a thread that finishes its streams of step k goes on with step k + 1
    // while others finish k.  Right after a stream's control plane for step k, its thread adds
    // the stream's part to program k (Device::add_part: an atomic reservation in the program's
    // slot, no global layout); the caller launches program k once every stream has added its part
    // (Device::close_program), programs in order.  Steps run at most fr_ahead ahead of the last
    // launched program.  All HIP calls stay on the caller's thread.
    struct FrProg {
        uint32_t originals = 0;
        bool finish = false;
        int handle = -1;
        uint64_t epoch = 0, clock = 0;
        std::atomic<uint32_t> remaining{0};
    };
    static const unsigned kFrRing = Stream::kParts;
    FrProg fr_progs[kFrRing];
    bool fr_mode = false, fr_running = false;
    std::atomic<int> job_kind{0};             // pool job: 0 run_all pass, 1 fr_loop
    std::atomic<bool> fr_stop{false};
    std::atomic<uint32_t> fr_published{0};
    uint32_t fr_launched = 0, fr_ahead = 2;
    uint64_t fr_next_epoch = 1;
    std::atomic<uint64_t> fr_released{0};     // completed epoch (rows freed up to it are reusable)
    std::mutex fr_mu;
    std::condition_variable cv_fr, cv_main;
    std::atomic<int> fr_sleepers{0};
    std::atomic<bool> fr_main_waiting{false};
    std::vector<std::vector<uint64_t>> fr_vbase;  // record mode: per program, per stream: first digest index

    void start_fr() {
        if (fr_running) return;
        fr_stop.store(false);
        job_kind.store(1, std::memory_order_relaxed);
        left.store(threads.size(), std::memory_order_relaxed);
        gen.fetch_add(1, std::memory_order_seq_cst);
        if (sleepers.load(std::memory_order_seq_cst) > 0) {
            std::lock_guard<std::mutex> lk(mu);
            cv_start.notify_all();
        }
        fr_running = true;
    }

    void stop_fr() {
        if (!fr_running) return;
        fr_stop.store(true, std::memory_order_seq_cst);
        {
            std::lock_guard<std::mutex> lk(fr_mu);
            cv_fr.notify_all();
        }
        wait_pass_end();
        fr_running = false;
        job_kind.store(0);
        double sum = 0, mx = 0;
        for (double b : busy_ms) {
            sum += b;
            if (b > mx) mx = b;
        }
        host_ms[1] += sum;
        host_ms[5] += mx;
        std::fill(busy_ms.begin(), busy_ms.end(), 0.0);
        for (double f : fill_ms) host_ms[3] += f;  // stolen stream steps
        std::fill(fill_ms.begin(), fill_ms.end(), 0.0);
    }

    // A runnable stream for thread ti (claimed), or -1.  Its own streams first, the one furthest
    // behind.  Otherwise a stream of a thread in its group of 8 (neighbouring cores: the stream's
    // state is still in the shared L3), and beyond the group only a stream that holds up the
    // oldest unlaunched program: a stolen stream's state moves to another core's caches, which
    // costs more than it saves unless the launch waits for it (TONK_AMD_STEAL=0: steal anything).
    std::atomic<uint32_t> fr_launched_pub{0};
    int fr_pick(size_t ti) {
        const int best = fr_scan(ti);
        if (best < 0) return -1;
        const uint32_t pub = fr_published.load(std::memory_order_acquire);
        Stream& st = *streams[best];
        if (st.busy.exchange(1, std::memory_order_acq_rel)) return -2;  // raced: look again
        if (st.next_step.load(std::memory_order_acquire) < pub) return best;
        st.busy.store(0, std::memory_order_release);
        return -2;
    }
    // The stream fr_pick would take for thread ti (not claimed), or -1.
    int fr_scan(size_t ti) {
        static const int steal_mode = getenv("TONK_AMD_STEAL") ? atoi(getenv("TONK_AMD_STEAL")) : 1;  // A/B
        const uint32_t pub = fr_published.load(std::memory_order_acquire);
        const uint32_t oldest = fr_launched_pub.load(std::memory_order_acquire);
        const size_t T = threads.size(), n = streams.size();
        const size_t group = ti / 8;
        for (int pass = 0; pass < 3; ++pass) {
            if (pass == 1 && steal_mode == 0) continue;
            int best = -1;
            uint32_t bk = ~0u;
            for (size_t s = pass ? 0 : ti; s < n; s += pass ? 1 : T) {
                if (pass == 1 && (s % T) / 8 != group) continue;
                Stream& st = *streams[s];
                const uint32_t k = st.next_step.load(std::memory_order_acquire);
                if (pass == 2 && steal_mode != 0 && k != oldest) continue;
                if (k < pub && k < bk && !st.busy.load(std::memory_order_relaxed)) {
                    best = (int)s;
                    bk = k;
                }
            }
            if (best >= 0) return best;
        }
        return -1;
    }

    void fr_loop(size_t ti) {
        for (;;) {
            if (fr_stop.load(std::memory_order_acquire)) return;
            const int s = fr_pick(ti);
            if (s >= 0) {
                fr_run(s, ti);
                continue;
            }
            if (s == -2) continue;
            // idle: spin a while, then sleep until a step is published, a program is launched
            // (its successor's streams become stealable) or a stolen stream is handed back
            const uint32_t seen = fr_published.load(std::memory_order_acquire);
            const uint32_t seen_l = fr_launched_pub.load(std::memory_order_acquire);
            const uint32_t seen_h = fr_handback.load(std::memory_order_acquire);
            auto changed = [&] {
                return fr_stop.load(std::memory_order_acquire) || fr_published.load(std::memory_order_acquire) != seen ||
                       fr_launched_pub.load(std::memory_order_acquire) != seen_l ||
                       fr_handback.load(std::memory_order_acquire) != seen_h;
            };
            const auto until = std::chrono::steady_clock::now() + std::chrono::nanoseconds(spin_ns());
            unsigned k = 0;
            bool woke = false;
            while (!(woke = changed())) {
                __builtin_ia32_pause();
                if ((++k & 255) == 0 && std::chrono::steady_clock::now() > until) break;
            }
            if (woke) continue;
            std::unique_lock<std::mutex> lk(fr_mu);
            fr_sleepers.fetch_add(1);
            cv_fr.wait(lk, [&] { return changed() || fr_scan(ti) >= 0; });
            fr_sleepers.fetch_sub(1);
        }
    }
    std::atomic<uint32_t> fr_handback{0};  // bumped when a thief leaves a stream runnable
    void fr_wake_workers() {
        if (fr_sleepers.load(std::memory_order_seq_cst) > 0) {
            std::lock_guard<std::mutex> lk(fr_mu);
            cv_fr.notify_all();
        }
    }

    // Stream s's next step (claimed by the caller): control plane, then its part of the program.
    void fr_run(int s, size_t ti) {
        typedef std::chrono::steady_clock clk;
        const auto w0 = clk::now();
        Stream& st = *streams[s];
        const uint32_t k = st.next_step.load(std::memory_order_relaxed);
        FrProg& P = fr_progs[k % kFrRing];
        Context& c = *ctxs[s];
        c.rows.release_up_to(fr_released.load(std::memory_order_acquire));
        st.clock = P.clock;
        if (P.finish) st.runner->finish();
        else st.runner->advance(P.originals);
        c.prepare_flush();
        Device::Part& part = st.parts[k % kFrRing];
        dev.add_part(P.handle, c.pb, part);
        part.verify.clear();
        if (st.tr.on) {
            // record mode: the digests of this step's rows, taken once program k completes;
            // an entry's index is (program, position in this stream's part)
            SessTranscript& t = st.tr;
            uint64_t local = 0;
            for (size_t e = t.reg_enc; e < t.pend_enc.size(); ++e) {
                t.pend_enc[e].v = ((uint64_t)k << 32) | local++;
                part.verify.push_back(Device::VerifyDesc{(uint32_t)c.rows.offset(t.pend_enc[e].row), t.pend_enc[e].total, 0, 0});
            }
            for (size_t e = t.reg_dec; e < t.pend_dec.size(); ++e) {
                t.pend_dec[e].v = ((uint64_t)k << 32) | local++;
                part.verify.push_back(Device::VerifyDesc{(uint32_t)c.rows.offset(t.pend_dec[e].row), t.pend_dec[e].upper, 1, 0});
            }
            t.reg_enc = t.pend_enc.size();
            t.reg_dec = t.pend_dec.size();
        }
        c.finish_flush(false);
        busy_ms[ti] += std::chrono::duration<double, std::milli>(clk::now() - w0).count();
        const bool stolen = (size_t)s % threads.size() != ti;
        if (stolen) fill_ms[ti] += 1.0;  // (fr: counts steps run by a thief)
        st.next_step.store(k + 1, std::memory_order_release);
        st.busy.store(0, std::memory_order_release);
        if (stolen && k + 1 < fr_published.load(std::memory_order_acquire)) {
            fr_handback.fetch_add(1, std::memory_order_seq_cst);  // its owner may be asleep
            fr_wake_workers();
        }
        if (P.remaining.fetch_sub(1, std::memory_order_acq_rel) == 1 && fr_main_waiting.load()) {
            std::lock_guard<std::mutex> lk(fr_mu);
            cv_main.notify_one();
        }
    }

    // Launch every program whose parts are all in, in order.
    void fr_launch_ready() {
        typedef std::chrono::steady_clock clk;
        const uint32_t pub = fr_published.load(std::memory_order_relaxed);
        std::vector<Device::Part*> parts(streams.size());
        while (fr_launched < pub) {
            FrProg& P = fr_progs[fr_launched % kFrRing];
            if (P.remaining.load(std::memory_order_acquire) != 0) break;
            const auto t0 = clk::now();
            for (size_t i = 0; i < streams.size(); ++i) parts[i] = &streams[i]->parts[fr_launched % kFrRing];
            if (prm.record) {
                std::vector<uint64_t> base(streams.size());
                for (size_t i = 0; i < streams.size(); ++i) {
                    base[i] = verify_count;
                    verify_count += parts[i]->verify.size();
                }
                if (fr_vbase.size() <= fr_launched) fr_vbase.resize(fr_launched + 1);
                fr_vbase[fr_launched].swap(base);
            }
            last_ticket = dev.close_program(P.handle, parts.data(), parts.size());
            epoch_ticket.push_back(std::make_pair(P.epoch, last_ticket));
            ++fr_launched;
            fr_launched_pub.store(fr_launched, std::memory_order_seq_cst);
            fr_wake_workers();  // (the next program's streams are now stealable)
            fr_released.store(completed_epoch(), std::memory_order_release);
            host_ms[4] += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        }
    }

    // Block until the oldest unlaunched program has all its parts, then launch what is ready.
    void fr_wait_one() {
        typedef std::chrono::steady_clock clk;
        const auto t0 = clk::now();
        FrProg& P = fr_progs[fr_launched % kFrRing];
        const auto until = t0 + std::chrono::microseconds(20);
        unsigned k = 0;
        while (P.remaining.load(std::memory_order_acquire) != 0) {
            __builtin_ia32_pause();
            if ((++k & 255) == 0 && clk::now() > until) {
                std::unique_lock<std::mutex> lk(fr_mu);
                fr_main_waiting.store(true);
                cv_main.wait(lk, [&] { return P.remaining.load() == 0; });
                fr_main_waiting.store(false);
                break;
            }
        }
        host_ms[0] += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        fr_launch_ready();
    }

    // Upper bounds of one stream's program for a step of `originals` (records = instructions +
    // ops; measured up to ~12 records per original on the decoder-stress stream and ~1.5 on the
    // batched ones) and the end-of-stream flush (remaining originals + flush_max recoveries).
    void fr_bounds(uint32_t originals, bool finish, size_t* recs, size_t* items) const {
        uint64_t n = originals;
        if (finish) {
            n = 0;
            for (const auto& sp : streams) {
                const uint64_t left = sp->p.n_originals - sp->runner->position() + sp->p.flush_max;
                if (left > n) n = left;
            }
        }
        *recs = streams.size() * (size_t)(16 * n + 8192);
        *items = streams.size() * (size_t)(n / 2 + 2048);
    }

    void fr_step(uint32_t originals, bool finish) {
        typedef std::chrono::steady_clock clk;
        size_t recs = 0, items = 0;
        fr_bounds(originals, finish, &recs, &items);
        if (!dev.assembly_fits(recs, items)) {
            // A step larger than the staging slots were sized for: launch what is published, then
            // grow every slot (nothing in flight) before this step's program is opened.
            fr_drain();
            if (!dev.ensure_assembly(recs, items)) error = dev.error();
        }
        start_fr();
        while (fr_published.load(std::memory_order_relaxed) - fr_launched >= fr_ahead) fr_wait_one();
        const uint32_t k = fr_published.load(std::memory_order_relaxed);
        FrProg& P = fr_progs[k % kFrRing];
        P.originals = originals;
        P.finish = finish;
        P.clock = time_msec();
        P.epoch = fr_next_epoch++;
        const auto t0 = clk::now();
        P.handle = dev.open_program();
        host_ms[2] += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        P.remaining.store((uint32_t)streams.size(), std::memory_order_relaxed);
        fr_published.store(k + 1, std::memory_order_seq_cst);
        fr_wake_workers();
        fr_launch_ready();
    }

    // Every published step run and launched; the workers leave their loop.
    void fr_drain() {
        if (!fr_mode) return;
        while (fr_launched < fr_published.load(std::memory_order_relaxed)) fr_wait_one();
        stop_fr();
    }

    // Highest epoch whose program has completed on the device (its freed rows are reusable).
    uint64_t completed_epoch() {
        size_t k = 0;
        while (k < epoch_ticket.size() && dev.completed(epoch_ticket[k].second)) {
            released_epoch = epoch_ticket[k].first;
            ++k;
        }
        epoch_ticket.erase(epoch_ticket.begin(), epoch_ticket.begin() + k);
        return released_epoch;
    }

    // Advance every stream by `originals` (or finish it), then merge the streams' programs into
    // one and enqueue it.  The per-stream phases run on the pool threads:
    //   1. release rows of completed programs, run the control planes, emit the running-sum scans
    //   2. (main) lay out the merged program, wait for a free staging slot
    //   3. copy each stream's ops into the pinned staging buffer, close the stream's epoch
    //   4. (main) upload the program and launch it level by level
    // Deferred mode (the default with level pipelining): phase 3 of a program runs at the start
    // of the NEXT step's phase 1, in the same per-stream job (the stream's closed program is
    // still in that core's caches), and the program is launched after it.  A step is then one
    // pass over the pool instead of two; the device runs one program behind the host, which
    // costs nothing while the host sets the pace.
    bool deferred = false;       // set at create: pipelined and not host-staged
    bool have_closed = false;    // a closed program is laid out (dev.begin) and awaits its fill
    std::atomic<size_t> fills_left{0};  // early launch: streams of the pass not yet filled
    uint64_t closed_epoch = 0;

    void step(uint32_t originals, bool finish) {
        if (fr_mode) { fr_step(originals, finish); return; }
        if (deferred) { step_deferred(originals, finish); return; }
        typedef std::chrono::steady_clock clk;
        auto ms = [](clk::time_point a, clk::time_point b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
        };
        const auto t0 = clk::now();
        clock_msec = time_msec();
        if (host_in && !finish) stage_inputs(originals);
        const uint64_t rel = completed_epoch();
        std::fill(busy_ms.begin(), busy_ms.end(), 0.0);
        init_order();
        run_all([this, originals, finish, rel, &ms](size_t i, size_t ti) {
            const auto w0 = clk::now();
            Context& c = *ctxs[i];
            streams[i]->clock = clock_msec;
            c.rows.release_up_to(rel);
            if (finish) streams[i]->runner->finish();
            else streams[i]->runner->advance(originals);
            c.prepare_flush();
            const double t = ms(w0, clk::now());
            busy_ms[ti] += t;
            stream_ms[i] = t;
        });
        sort_order();
        const auto t1 = clk::now();
        account_busy();
        std::vector<Context*> cs;
        for (auto& c : ctxs) cs.push_back(c.get());
        dev.begin(cs.data(), cs.size());
        const auto t2 = clk::now();
        const uint64_t epoch = ctxs.empty() ? 0 : ctxs[0]->epoch;
        run_all([this](size_t i, size_t) {
            dev.fill(i);
            ctxs[i]->finish_flush();
        });
        const auto t3 = clk::now();
        if (host_in) dev.h2d_fence();  // the program reads the rows copied in above
        if (prm.record) register_verify();
        last_ticket = dev.launch();
        if (host_in) stage_outputs();
        const auto t4 = clk::now();
        host_ms[0] += ms(t0, t1);
        host_ms[2] += ms(t1, t2);
        host_ms[3] += ms(t2, t3);
        host_ms[4] += ms(t3, t4);
        epoch_ticket.push_back(std::make_pair(epoch, last_ticket));
    }

    void init_order() {
        if (order.size() != streams.size()) {
            order.resize(streams.size());
            for (size_t i = 0; i < order.size(); ++i) order[i] = (uint32_t)i;
            stream_ms.assign(streams.size(), 0.0);
        }
    }
    void sort_order() {
        static const bool lpt = getenv("TONK_AMD_STREAM_FIFO") == nullptr;  // A/B switch (profiling)
        if (lpt)
            std::sort(order.begin(), order.end(), [this](uint32_t a, uint32_t b) { return stream_ms[a] > stream_ms[b]; });
    }
    void account_busy() {
        double mx = 0;
        for (double b : busy_ms) {
            host_ms[1] += b;
            if (b > mx) mx = b;
        }
        host_ms[5] += mx;
    }

    // One pass over the pool: fill the closed program of the previous step (if any), then the
    // control planes of this step, each stream closing its new program; then (main) launch the
    // filled program and lay out the new one.  host_ms[3] (fill) is the fill part of the pass.
    void step_deferred(uint32_t originals, bool finish) {
        typedef std::chrono::steady_clock clk;
        auto ms = [](clk::time_point a, clk::time_point b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
        };
        const auto t0 = clk::now();
        clock_msec = time_msec();
        const uint64_t rel = completed_epoch();
        std::fill(busy_ms.begin(), busy_ms.end(), 0.0);
        std::fill(fill_ms.begin(), fill_ms.end(), 0.0);
        init_order();
        const bool fill = have_closed;
        // Early launch: the thread that fills the last stream launches the program at once
        // (the other threads only run control planes, which touch no device state) instead of the
        // caller after the pass.  Record mode runs the same schedule (its digests are enqueued by
        // the launches themselves).
        // A session without workers runs the same order: its one stream's previous program is
        // filled and launched before this step's control plane, which then overlaps its levels.
        static const bool early_ok = getenv("TONK_AMD_LATE_LAUNCH") == nullptr;  // A/B switch
        const bool early = fill && early_ok;
        if (early) fills_left.store(streams.size(), std::memory_order_relaxed);
        run_all([this, originals, finish, rel, fill, early, &ms](size_t i, size_t ti) {
            const auto w0 = clk::now();
            Context& c = *ctxs[i];
            if (fill) {
                dev.fill(i);
                fill_ms[ti] += ms(w0, clk::now());
                if (early && fills_left.fetch_sub(1, std::memory_order_acq_rel) == 1) launch_closed();
            }
            c.rows.release_up_to(rel);
            streams[i]->clock = clock_msec;
            if (finish) streams[i]->runner->finish();
            else streams[i]->runner->advance(originals);
            c.prepare_flush();
            c.finish_flush(true);
            const double t = ms(w0, clk::now());
            busy_ms[ti] += t;
            stream_ms[i] = t;
        });
        sort_order();
        const auto t1 = clk::now();
        account_busy();
        for (double f : fill_ms) host_ms[3] += f / (double)fill_ms.size();
        if (fill && !early) launch_closed();
        const auto t2 = clk::now();
        std::vector<Context*> cs;
        for (auto& c : ctxs) cs.push_back(c.get());
        dev.begin(cs.data(), cs.size(), true);
        if (prm.record) register_verify();  // rows of the program just closed (launched next pass)
        have_closed = true;
        closed_epoch = ctxs.empty() ? 0 : ctxs[0]->epoch - 1;
        const auto t3 = clk::now();
        host_ms[0] += ms(t0, t1);
        host_ms[4] += ms(t1, t2);
        host_ms[2] += ms(t2, t3);
    }

    // Launch the closed program (filled).
    void launch_closed() {
        last_ticket = dev.launch();
        have_closed = false;
        epoch_ticket.push_back(std::make_pair(closed_epoch, last_ticket));
    }

    // Fill and launch a closed program still waiting (end of a run: wait / finish).
    void flush_closed() {
        fr_drain();
        if (!have_closed) return;
        run_all([this](size_t i, size_t) { dev.fill(i); });
        launch_closed();
    }

    // H2D of the next `originals` input rows of every stream, both codec sides (each side's
    // rows are one contiguous range of the arena in packet order, see generate()).
    void stage_inputs(uint32_t originals) {
        const size_t side_bytes = (size_t)streams[0]->p.n_originals * row_cap;
        for (size_t i = 0; i < streams.size(); ++i) {
            Stream& st = *streams[i];
            const uint32_t next = (uint32_t)st.runner->summary().originals;
            const uint32_t n = next + originals <= st.p.n_originals ? originals : st.p.n_originals - next;
            if (!n) continue;
            for (int side = 0; side < 2; ++side) {
                if (!((prm.stage_host >> side) & 1u)) continue;  // (that end's packets are resident)
                const RowId r = (side ? st.dec_rows : st.enc_rows)[next];
                const uint8_t* src = host_in + (2 * i + side) * side_bytes + (size_t)next * row_cap;
                dev.h2d((uint64_t)st.ctx->rows.offset(r) * TAMD_ROW_UNIT, src, (size_t)n * row_cap);
                h2d_bytes += (uint64_t)n * row_cap;
            }
        }
    }

    // D2H of the step's recovery packets and recovered originals (packed by a gather kernel
    // after the step's program), then H2D of the recovery bytes the decoders received.
    void stage_outputs() {
        std::vector<Device::GatherDesc> d;
        size_t bytes = 0, recv = 0;
        for (auto& sp : streams) {
            for (const auto& o : sp->out_rows) {
                Device::GatherDesc g;
                g.row = sp->ctx->rows.offset(o.first);
                g.len = o.second;
                g.out = (uint32_t)bytes;
                d.push_back(g);
                bytes += (o.second + 15u) & ~15u;
            }
            sp->out_rows.clear();
            recv += sp->recv_bytes;
            sp->recv_bytes = 0;
        }
        if (bytes > host_out_cap) {
            dev.sync_staging();
            if (host_out) hipHostFree(host_out);
            host_out_cap = bytes + bytes / 2 + 4096;
            if (hipHostMalloc((void**)&host_out, host_out_cap, hipHostMallocDefault) != hipSuccess) {
                host_out = nullptr;
                host_out_cap = 0;
                error = "pinned staging allocation failed";
                return;
            }
        }
        dev.d2h_gather(d, bytes, host_out);
        d2h_bytes += bytes;
        if (recv > bytes) recv = bytes;
        dev.h2d_after_d2h(host_out, recv);
        h2d_bytes += recv;
    }

    void release_all() {
        const uint64_t rel = completed_epoch();
        run_all([this, rel](size_t i, size_t) { ctxs[i]->rows.release_up_to(rel); });
    }

    // Record mode: hand the rows of the program about to be launched (every transcript entry
    // not registered yet) to the device's verification, which digests them right after the
    // launch that completes the program.  Main thread, between passes (no stream is running).
    uint64_t verify_count = 0, verify_base = 0;
    void register_verify() {
        std::vector<Device::VerifyDesc> d;
        for (auto& sp : streams) {
            SessTranscript& t = sp->tr;
            for (size_t k = t.reg_enc; k < t.pend_enc.size(); ++k) {
                auto& e = t.pend_enc[k];
                e.v = verify_count++;
                d.push_back(Device::VerifyDesc{(uint32_t)sp->ctx->rows.offset(e.row), e.total, 0, 0});
            }
            for (size_t k = t.reg_dec; k < t.pend_dec.size(); ++k) {
                auto& e = t.pend_dec[k];
                e.v = verify_count++;
                d.push_back(Device::VerifyDesc{(uint32_t)sp->ctx->rows.offset(e.row), e.upper, 1, 0});
            }
            t.reg_enc = t.pend_enc.size();
            t.reg_dec = t.pend_dec.size();
        }
        dev.verify_next(d);
    }

    // Fill the transcript lines from the device digests (end of a run: every program done).
    void resolve_transcripts() {
        if (!fr_mode) register_verify();  // (entries of a program never launched: none, unless the run failed)
        std::vector<Device::VerifyOut> res;
        dev.verify_results(res);
        if (verify_base + res.size() != verify_count) {
            error = "verification digests missing";
            return;
        }
        size_t si = 0;
        auto get = [&](uint64_t v) -> const Device::VerifyOut& {
            // free-running schedule: v = (program, position in the stream's part)
            if (fr_mode) v = fr_vbase[v >> 32][si] + (v & 0xffffffffu);
            return res[v - verify_base];
        };
        for (auto& sp : streams) {
            Stream& s = *sp;
            char line[256];
            for (auto& e : s.tr.pend_enc) {
                const Device::VerifyOut& o = get(e.v);
                snprintf(line, sizeof(line), "E 0 %u %u %u %u %u %016llx", e.total, e.meta.Row, e.meta.ColumnStart,
                         e.meta.SumCount, e.meta.LDPCCount, (unsigned long long)o.hash);
                s.tr.lines[e.pos] = line;
            }
            for (auto& d : s.tr.pend_dec) {
                const Device::VerifyOut& o = get(d.v);
                if (!o.ok) {
                    error = "recovered row with a corrupt length header";
                    continue;
                }
                std::string& ln = s.tr.lines[d.pos];
                snprintf(line, sizeof(line), ":%u:%016llx", o.len, (unsigned long long)o.hash);
                const size_t at = ln.find('#');
                if (at != std::string::npos) ln.replace(at, 1, line);
            }
            s.tr.pend_enc.clear();
            s.tr.pend_dec.clear();
            s.tr.reg_enc = s.tr.reg_dec = 0;
            ++si;
        }
        verify_base = verify_count;
        dev.verify_reset();
    }
};

} // namespace

extern "C" {

void* tamd_session_create(const tamd_session_params* p, char* err, size_t err_len) {
    auto fail = [&](const std::string& m) -> void* {
        if (err && err_len) snprintf(err, err_len, "%s", m.c_str());
        return nullptr;
    };
    if (!p || p->n_streams == 0) return fail("bad parameters");
    if (!gf_init()) return fail("gf self test failed");
    std::unique_ptr<Session> s(new Session());
    s->prm = *p;
    // Level pipelining (Device::set_pipelined): off when packets are staged through the host
    // (the D2H gather right after a program needs all of its levels) and for A/B runs.  A
    // program stays in flight for as many launches as it has levels: 6 staging slots.
    const bool pipe = !p->stage_host && getenv("TONK_AMD_NO_PIPELINE") == nullptr;
    uint32_t nthreads = p->n_threads ? (p->n_threads < p->n_streams ? p->n_threads : p->n_streams) : 1;
    // The worker pool's cores: this GPU's share of its NUMA node (device_local_cpus).  A share
    // smaller than the pool (a node with fewer usable cores per GPU than workers) shrinks the pool
    // to one worker per core rather than putting two workers on one core: the rank's rate then
    // degrades in proportion to its cores, and config.host_cores shows them.
    std::vector<int> share;
    if (nthreads > 1) {
        share = device_local_cpus((int)p->device);
        if (!share.empty() && share.size() < nthreads) nthreads = (uint32_t)share.size();
    }
    // The free-running schedule (worker threads, pipelined levels): programs assembled in
    // parallel (Device::add_part) in 8 slots -- up to fr_ahead open, the rest in flight; otherwise
    // one laid-out program per step in 6 slots (TONK_AMD_PASSES=1 keeps the pass schedule).
    // TONK_AMD_FR_SINGLE=1 runs it for one-thread sessions too (one worker beside the caller:
    // the worker's control plane of step k + 1 overlaps the caller's assembly and launch of
    // program k).  Off by default: on the decoder-stress stream the worker's control plane ran
    // 25-40 % slower than the caller's own (configs[4]: 2.8 vs 3.6 GiB/s at 512 originals per
    // program, 3.6 vs 4.2 at 1024), which costs more than the overlap gains.
    static const bool fr_single = getenv("TONK_AMD_FR_SINGLE") != nullptr;
    s->fr_mode = pipe && (nthreads > 1 || fr_single) && getenv("TONK_AMD_NO_DEFER") == nullptr &&
                 getenv("TONK_AMD_PASSES") == nullptr;
    if (const char* a = getenv("TONK_AMD_RUNAHEAD")) {
        // (programs k .. k + fr_ahead are open at once: each needs its own FrProg, Part and slot)
        const int v = atoi(a);
        s->fr_ahead = v < 1 ? 1u : v > (int)Session::kFrRing - 1 ? Session::kFrRing - 1 : (uint32_t)v;
    }
    s->dev.set_small_uploads(p->n_streams <= 4);
    if (s->fr_mode) s->dev.set_assembly_slots(8, p->n_streams <= 4 ? 8 : 24);
    else {
        // (TONK_AMD_SLOTS: A/B knob for the slot count of the pass schedule)
        // (few streams: a program's levels stay in flight until later programs launch beside
        // them; with 6 slots a decoder-stress stream's deep programs drained the device for a slot
        // every program: configs[4] 5.50 -> 5.83 GiB/s with 12)
        const size_t slots = getenv("TONK_AMD_SLOTS") ? (size_t)atoi(getenv("TONK_AMD_SLOTS"))
                                                      : (pipe ? (p->n_streams <= 4 ? 12 : 6) : 2);
        s->dev.set_program_slots(slots, (p->n_streams <= 4 ? 2u : 16u) << 20);
    }
    if (!s->dev.init((int)p->device, p->arena_bytes)) return fail(s->dev.error());
    s->dev.set_pipelined(pipe);
    if (!s->dev.gf_selftest()) return fail("device GF(256) self test failed");

    const uint64_t range = (s->dev.arena_bytes() / p->n_streams) & ~(uint64_t)(TAMD_ROW_UNIT - 1);
    s->row_cap = ((p->payload_max + 4 + 63) / 64) * 64;
    s->busy_ms.assign(nthreads, 0.0);
    s->fill_ms.assign(nthreads, 0.0);
    s->deferred = pipe && getenv("TONK_AMD_NO_DEFER") == nullptr;
    Session* raw = s.get();
    if (nthreads > 1 || s->fr_mode) {
        raw->cpus = idle_cpus(share.empty() ? device_local_cpus((int)p->device) : share, nthreads);
        raw->threads_wanted = nthreads;
        for (uint32_t t = 0; t < nthreads; ++t) raw->threads.emplace_back([raw, t] { raw->pool_loop(t); });
    }
    // Streams are built on the pool threads (first touch of their state on the device's node).
    s->streams.resize(p->n_streams);
    s->ctxs.resize(p->n_streams);
    s->run_all([raw, p, range, pipe](size_t i, size_t) {
        std::unique_ptr<Context> ctx(new Context());
        ctx->rows.init(range, (range / TAMD_ROW_UNIT) * i);
        ctx->pipeline = pipe;
        // Pipelined sessions of one or a few streams reference expansions of more than 16 terms
        // as rows: their launches are small, so the extra levels cost little, while inlining
        // grows with the solves per program and sets the host time (configs[4] decoder stress:
        // 1.84 -> 3.63 GiB/s).  Batched sessions keep inlining: there the extra levels are extra
        // full-width launches (configs[3]: 33 -> 57 launches per 30 steps, device time per step
        // +11 %, no host gain).  TONK_AMD_EXPAND=<terms> overrides (A/B knob).
        static const char* expand_env = getenv("TONK_AMD_EXPAND");
        const uint32_t expand = expand_env ? (uint32_t)atoi(expand_env) : (p->n_streams <= 4 ? 16u : ~0u);
        if (pipe) ctx->ex.expand_limit = expand;
        // The same split for back substitution over materialized rows (configs[4]: host time per
        // program -12 %, device -6 %; configs[2]/[3]: +1 level, +20 % launches, no fewer bytes).
        // TONK_AMD_BACKSUB_ROWS=<unknowns> overrides (A/B knob).
        static const char* bs_env = getenv("TONK_AMD_BACKSUB_ROWS");
        ctx->backsub_rows = bs_env ? (uint32_t)atoi(bs_env) : (p->n_streams <= 4 ? 2u : ~0u);
        // (TONK_AMD_DENSE_SPLIT=<packets> overrides: A/B knob)
        static const char* split_env = getenv("TONK_AMD_DENSE_SPLIT");
        ctx->dense_split = split_env ? (uint32_t)atoi(split_env) : (p->n_streams <= 4 ? 0u : Encoder::kDenseSplit);
        // Few-stream sessions also take the C ABI's lane scan levels (Context::short_scans): a
        // snapshot read while its scan is one op long is promised level 1, which takes a level off
        // configs[1]'s program (4 -> 3 launches, 17.4 -> 19.3 GiB/s; configs[4] 5.9 -> 6.2).
        // Batched sessions keep the chain level: a promised snapshot makes its whole scan one op,
        // a long item in a full-width launch.  TONK_AMD_SHORT_SCANS=0|1 overrides (A/B knob).
        static const char* short_env = getenv("TONK_AMD_SHORT_SCANS");
        ctx->short_scans = short_env ? atoi(short_env) != 0 : p->n_streams <= 4;
        std::unique_ptr<Stream> st(new Stream());
        st->ctx = ctx.get();
        wl::Params& q = st->p;
        q.stream_id = p->stream_base + (uint32_t)i;
        q.n_originals = p->n_originals;
        q.payload_min = p->payload_min;
        q.payload_max = p->payload_max;
        q.loss_thresh = p->loss_thresh;
        q.ge_enable = p->ge_enable;
        q.gb_thresh = p->gb_thresh;
        q.bg_thresh = p->bg_thresh;
        q.loss_on_recovery = p->loss_on_recovery;
        q.fec_rate_q16 = p->fec_rate_q16;
        q.ack_every = p->ack_every;
        q.ack_bytes = p->ack_bytes ? p->ack_bytes : 256;
        q.arq_lag = p->arq_lag;
        q.flush_max = p->flush_max;
        q.rtx_every = p->rtx_every;
        q.rtx_msec = p->rtx_msec ? p->rtx_msec : 1;
        q.hold_full = p->hold_full;
        q.batch_adds = getenv("TONK_AMD_SINGLE_ADDS") ? 0 : 1;  // A/B switch (profiling)
        q.seed_data = 1000 + q.stream_id;
        q.seed_loss = 2000 + q.stream_id;
        st->enc.reset(new Encoder(ctx.get(), raw->row_cap));
        st->enc->set_clock(&st->clock);
        st->dec.reset(new Decoder(ctx.get(), raw->row_cap));
        st->tr.on = p->record != 0;
        st->runner.reset(new wl::Runner<Stream, Stream>(st->p, *st, *st));
        raw->streams[i] = std::move(st);
        raw->ctxs[i] = std::move(ctx);
    });
    return s.release();
}

int tamd_session_generate(void* sp) {
    Session* s = (Session*)sp;
    // Per stream on the pool threads (the row tables and row lists are that stream's state).
    std::vector<std::vector<Device::GenDesc>> per(s->streams.size());
    std::atomic<bool> full{false};
    s->run_all([s, &per, &full](size_t si, size_t) {
        Stream& st = *s->streams[si];
        std::vector<Device::GenDesc>& d = per[si];
        const uint32_t n = st.p.n_originals;
        st.runner->pregenerate();  // the stream's loss draws (scenario generation, untimed)
        st.enc_rows.assign(n, kNoRow);
        st.dec_rows.assign(n, kNoRow);
        // (an input pool: rows for the first `pool` originals; original i reads row i mod pool)
        // (equal payload lengths only: a pooled row's length header must be original i's)
        const uint32_t pool = s->prm.input_pool && s->prm.input_pool < n && !s->prm.record &&
                                      !s->prm.stage_host && st.p.payload_min == st.p.payload_max
                                  ? s->prm.input_pool : n;
        d.reserve(2 * (size_t)pool);
        // Each side's inputs are an array of equal slots (row_cap bytes) in packet order, so runs of
        // a window's packets sit at a fixed stride (one ACCR instruction per run).
        for (int side = 0; side < 2; ++side) {
            for (uint32_t i = 0; i < pool; ++i) {
                const uint32_t len = wl::payload_length(st.p, i);
                const RowId r = st.ctx->alloc(s->row_cap);
                if (r == kNoRow) { full = true; return; }
                (side ? st.dec_rows : st.enc_rows)[i] = r;
                Device::GenDesc g;
                g.row = st.ctx->rows.offset(r);
                g.index = i;
                g.len = len;
                g.pad = st.ctx->rows.cap_bytes(r);
                g.seed = st.p.seed_data;
                d.push_back(g);
            }
            std::vector<RowId>& rows = side ? st.dec_rows : st.enc_rows;
            for (uint32_t i = pool; i < n; ++i) rows[i] = rows[i - pool];
        }
        st.pool = pool;
        st.pool_affine = pool >= 2;
        for (int side = 0; side < 2 && st.pool_affine; ++side) {
            const std::vector<RowId>& rows = side ? st.dec_rows : st.enc_rows;
            const uint32_t o0 = st.ctx->rows.offset(rows[0]), stride = st.ctx->rows.offset(rows[1]) - o0;
            st.pool_affine = consecutive_handles(rows.data(), pool) && stride > 0 &&
                             st.ctx->rows.affine(rows[0], pool, stride) && (!side || stride == st.pool_stride);
            st.pool_off[side] = o0;
            st.pool_stride = stride;
        }
    });
    if (full) { s->error = "arena too small for the session inputs"; return -1; }
    std::vector<Device::GenDesc> d;
    size_t total = 0;
    for (auto& v : per) total += v.size();
    d.reserve(total);
    for (auto& v : per) {
        d.insert(d.end(), v.begin(), v.end());
        std::vector<Device::GenDesc>().swap(v);
    }
    s->dev.generate_rows(d, s->row_cap);
    if (!s->dev.error().empty()) return -2;
    if (s->prm.stage_host) {
        // the pinned host copy of every input row: the bytes the steps copy in again
        const size_t side_bytes = (size_t)s->streams[0]->p.n_originals * s->row_cap;
        s->host_in_bytes = 2 * s->streams.size() * side_bytes;
        if (!s->dev.enable_staging() ||
            hipHostMalloc((void**)&s->host_in, s->host_in_bytes, hipHostMallocDefault) != hipSuccess) {
            s->host_in = nullptr;
            s->error = "pinned input staging allocation failed";
            return -3;
        }
        for (size_t i = 0; i < s->streams.size(); ++i) {
            Stream& st = *s->streams[i];
            st.stage = s->prm.stage_host & 3u;
            for (int side = 0; side < 2; ++side) {
                const std::vector<RowId>& rows = side ? st.dec_rows : st.enc_rows;
                const uint64_t base = st.ctx->rows.offset(rows[0]);
                for (uint32_t k = 0; k < st.p.n_originals; ++k)
                    if (st.ctx->rows.offset(rows[k]) != base + (uint64_t)k * (s->row_cap / TAMD_ROW_UNIT)) {
                        s->error = "input rows are not contiguous";
                        return -3;
                    }
                s->dev.download(s->host_in + (2 * i + side) * side_bytes, base * TAMD_ROW_UNIT, side_bytes);
            }
        }
    }
    return 0;
}

int tamd_session_step(void* sp, uint32_t originals) {
    Session* s = (Session*)sp;
    s->step(originals, false);
    for (auto& c : s->ctxs) if (c->oom) { s->error = "arena exhausted"; return -1; }
    return s->error.empty() && s->dev.error().empty() ? 0 : -1;
}

int tamd_session_wait(void* sp) {
    Session* s = (Session*)sp;
    s->flush_closed();
    s->dev.synchronize();
    s->dev.sync_staging();
    if (s->prm.record) s->resolve_transcripts();
    s->release_all();
    return s->dev.error().empty() && s->error.empty() ? 0 : -1;
}

int tamd_session_finish(void* sp) {
    Session* s = (Session*)sp;
    if (!s->finished) {
        s->step(0, true);
        s->finished = true;
    }
    return tamd_session_wait(sp);
}

int tamd_session_summary(void* sp, uint64_t* out, unsigned n) {
    Session* s = (Session*)sp;
    uint64_t v[TAMD_SUM_COUNT] = {0};
    for (auto& stp : s->streams) {
        const wl::Summary& q = stp->runner->summary();
        v[TAMD_SUM_ORIGINALS] += q.originals;
        v[TAMD_SUM_LOST_ORIGINALS] += q.lost_originals;
        v[TAMD_SUM_RECOVERIES] += q.recoveries;
        v[TAMD_SUM_LOST_RECOVERIES] += q.lost_recoveries;
        v[TAMD_SUM_RECOVERED] += q.recovered;
        v[TAMD_SUM_ARQ] += q.arq_redelivered;
        v[TAMD_SUM_MISSING_AT_END] += q.missing_at_end;
        v[TAMD_SUM_PAYLOAD_BYTES] += stp->payload_bytes;
        v[TAMD_SUM_ALG_BYTES] += stp->alg_bytes;
        v[TAMD_SUM_DISABLED_CODECS] += (stp->enc->disabled() ? 1 : 0) + (stp->dec->disabled() ? 1 : 0);
    }
    const DeviceStats& ds = s->dev.stats();
    v[TAMD_SUM_PROGRAMS] = ds.programs;
    v[TAMD_SUM_LAUNCHES] = ds.launches;
    v[TAMD_SUM_OPS] = ds.ops;
    v[TAMD_SUM_INSTRS] = ds.instrs;
    v[TAMD_SUM_UPLOAD_BYTES] = ds.upload_bytes;
    v[TAMD_SUM_ACC_BYTES] = ds.acc_bytes;
    v[TAMD_SUM_STORE_BYTES] = ds.store_bytes;
    v[TAMD_SUM_H2D_BYTES] = s->h2d_bytes;
    v[TAMD_SUM_D2H_BYTES] = s->d2h_bytes;
    v[TAMD_SUM_D2H_COPY_US] = (uint64_t)(ds.d2h_copy_ms * 1e3);
    if (n > TAMD_SUM_COUNT) n = TAMD_SUM_COUNT;
    for (unsigned i = 0; i < n; ++i) out[i] = v[i];
    return s->error.empty() ? 0 : -1;
}

void tamd_session_set_timing(void* sp, int on) { ((Session*)sp)->dev.set_timing(on != 0); }

double tamd_session_kernel_ms(void* sp, uint64_t* launches) {
    Session* s = (Session*)sp;
    s->dev.collect_timing();
    if (launches) *launches = s->dev.stats().timed_launches;
    return s->dev.stats().kernel_ms;
}

size_t tamd_session_transcript(void* sp, uint32_t stream, char* buf, size_t cap) {
    Session* s = (Session*)sp;
    if (stream >= s->streams.size()) return 0;
    std::string all;
    for (const std::string& l : s->streams[stream]->tr.lines) { all += l; all += '\n'; }
    if (buf && cap) {
        const size_t n = all.size() < cap - 1 ? all.size() : cap - 1;
        memcpy(buf, all.data(), n);
        buf[n] = 0;
    }
    return all.size() + 1;
}

void tamd_session_host_ms(void* sp, double out[10]) {
    Session* s = (Session*)sp;
    for (int i = 0; i < 6; ++i) out[i] = s->host_ms[i];
    out[6] = s->dev.stats().slot_wait_ms;
    out[7] = s->dev.stats().upload_enqueue_ms;
    out[8] = s->dev.stats().upload_enqueue_max_ms;
    out[9] = (double)s->dev.stats().slot_reallocs;
}

void tamd_session_arena(void* sp, uint64_t* base, uint64_t* bytes) {
    Session* s = (Session*)sp;
    if (base) *base = (uint64_t)(uintptr_t)s->dev.arena();
    if (bytes) *bytes = s->dev.arena_bytes();
}

void tamd_session_destroy(void* sp) { delete (Session*)sp; }

const char* tamd_session_error(void* sp) {
    Session* s = (Session*)sp;
    if (!s->error.empty()) return s->error.c_str();
    return s->dev.error().c_str();
}

void tamd_set_clock(uint64_t (*fn)(void)) { set_clock_source(fn); }

int tamd_session_schedule(void* sp) { return ((Session*)sp)->fr_mode ? 1 : 0; }

unsigned tamd_session_cpus(void* sp, int* out, unsigned cap) {
    Session* s = (Session*)sp;
    for (unsigned i = 0; i < cap && i < s->cpus.size(); ++i) out[i] = s->cpus[i];
    return (unsigned)s->cpus.size();
}

unsigned tamd_cpu_share(const char* dev_cpulists, unsigned device, const char* node_cores, const char* slot_override,
                        int* out, unsigned cap) {
    std::vector<std::string> lists;
    const std::string all(dev_cpulists ? dev_cpulists : "");
    size_t at = 0;
    while (at <= all.size() && !all.empty()) {
        size_t end = all.find(';', at);
        if (end == std::string::npos) end = all.size();
        lists.push_back(all.substr(at, end - at));
        at = end + 1;
    }
    const std::vector<int> share = node_core_share(lists, device, parse_cpulist(node_cores), slot_override);
    for (unsigned i = 0; i < cap && i < share.size(); ++i) out[i] = share[i];
    return (unsigned)share.size();
}

int tamd_device_selftest(uint32_t device, char* err, size_t err_len) {
    Device d;
    if (!d.init((int)device, 1 << 20)) {
        if (err && err_len) snprintf(err, err_len, "%s", d.error().c_str());
        return -1;
    }
    if (!d.gf_selftest()) {
        if (err && err_len) snprintf(err, err_len, "v_perm GF(256) multiply mismatch");
        return -2;
    }
    return 0;
}

} // extern "C"
