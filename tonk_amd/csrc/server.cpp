// server.cpp -- host side of the launch-free submission path (server.h, serve.h).
#include "server.h"

#include <hip/hip_runtime.h>
#include <chrono>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <thread>
#include <immintrin.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <time.h>

extern "C" __global__ void tamd_serve(const tamd_serve_args);

namespace tamd {

namespace {
std::atomic<int> g_spinners{0};  // callers spinning in Server::wait
int spinners_max() {  // (TONK_AMD_SPINNERS overrides)
    // (default: no cap in practice.  Capping at 8 kept Tonk's slow start-ups slow -- they are not
    // the spinners' doing -- and cost the C ABI bench 16 % with its 16 calling threads)
    static const int n = getenv("TONK_AMD_SPINNERS") ? atoi(getenv("TONK_AMD_SPINNERS")) : 1024;
    return n;
}
long futex_wait(std::atomic<uint32_t>* w, uint32_t expect, long timeout_ns) {
    timespec ts{timeout_ns / 1000000000L, timeout_ns % 1000000000L};
    return syscall(SYS_futex, (uint32_t*)w, FUTEX_WAIT_PRIVATE, expect, &ts, nullptr, 0);
}
void futex_wake(std::atomic<uint32_t>* w) { syscall(SYS_futex, (uint32_t*)w, FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0); }
double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
void* coherent_alloc(size_t n) {
    void* p = nullptr;
    if (hipHostMalloc(&p, n, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
    memset(p, 0, n);
    return p;
}
}  // namespace

bool Server::init(Device& dev, unsigned workers, unsigned ring_size, double idle_ms) {
    dev_ = &dev;
    dev.bind_thread();
    ring_size_ = 1;
    while (ring_size_ < ring_size) ring_size_ <<= 1;
    workers_ = workers ? workers : 1;
    idle_ticks_ = (uint64_t)(idle_ms * 1e5);  // s_memrealtime: 100 MHz
    if (const char* e = getenv("TONK_AMD_SERVE_DEBUG")) debug_ = (uint32_t)atoi(e);
    if (const char* e = getenv("TONK_AMD_SERVE_STALL_POST_MS")) stall_post_ms_ = (uint32_t)atoi(e);
    if (const char* e = getenv("TONK_AMD_WAIT_SPIN_US")) spin_us_ = atof(e);
    if (const char* e = getenv("TONK_AMD_WAIT_YIELD_US")) yield_us_ = atof(e);
    if (yield_us_ < spin_us_) yield_us_ = spin_us_;
    if (const char* e = getenv("TONK_AMD_WAIT_PARK")) park_ = atoi(e) != 0;
    stamps_ = getenv("TONK_AMD_CAPI_WATCH") != nullptr;
    // The ring in device memory the host writes through the BAR (the dispatcher then polls HBM,
    // not host memory across PCIe), unless TONK_AMD_CAPI_BAR leaves out bit 4 or that memory is
    // unavailable.
    const size_t ring_bytes = (size_t)ring_size_ * sizeof(tamd_serve_slot);
    if ((getenv("TONK_AMD_CAPI_BAR") ? (atoi(getenv("TONK_AMD_CAPI_BAR")) & 4) != 0 : true) &&
        (ring_ = (tamd_serve_slot*)Device::bar_alloc(ring_bytes))) {
        for (size_t i = 0; i < ring_bytes / 8; ++i) ((volatile uint64_t*)ring_)[i] = 0;
        _mm_sfence();
    } else {
        ring_ = (tamd_serve_slot*)coherent_alloc(ring_bytes);
    }
    host_ = (volatile tamd_serve_host*)coherent_alloc(sizeof(tamd_serve_host));
    if (!ring_ || !host_) return false;
    const size_t dbytes = sizeof(tamd_serve_dev) + (size_t)ring_size_ * sizeof(tamd_serve_slot);
    if (hipMalloc((void**)&dstate_, dbytes) != hipSuccess) return false;
    int least = 0, greatest = 0;
    hipDeviceGetStreamPriorityRange(&least, &greatest);
    hipStream_t st = nullptr;
    if (hipStreamCreateWithPriority(&st, hipStreamNonBlocking, greatest) != hipSuccess) return false;
    stream_ = st;
    if (hipMemsetAsync(dstate_, 0, dbytes, st) != hipSuccess) return false;
    {
        std::lock_guard<std::mutex> lk(launch_mu_);
        if (!launch_locked(0)) return false;
    }
    ok_ = true;
    // An empty command through the ring must come back.
    CmdBuf probe;
    if (debug_ & 1u) {
        dbg_done_ = (uint64_t*)coherent_alloc(4096);
        probe.done_at = dbg_done_;
    }
    std::vector<Device::HostCopy> none;
    if (!build(probe, none, nullptr, none)) return false;
    post(probe);
    const bool answered = wait(probe);
    if (!answered) {
        // (the probe's buffer stays allocated: the executor may still write its completion words)
        fprintf(stderr, "tonk_amd: the persistent executor did not answer; using kernel launches\n");
        ok_ = false;
        return false;
    }
    probe.release();
    // (test hook: a short timeout makes a loaded command time out, to exercise the dead server)
    if (const char* e = getenv("TONK_AMD_SERVE_TIMEOUT_US")) timeout_us_ = atof(e);
    return true;
}

bool Server::launch_locked(uint64_t tail0) {
    hipStream_t st = (hipStream_t)stream_;
    tamd_serve_args a;
    memset(&a, 0, sizeof(a));
    a.ring = ring_;
    a.host = (tamd_serve_host*)host_;
    a.dev = dstate_;
    a.arena = dev_->arena();
    a.gf = dev_->gf_tables();
    a.zrow = dev_->zero_row();
    a.tail0 = tail0;
    a.idle_ticks = idle_ticks_;
    a.ring_mask = ring_size_ - 1;
    a.wl_mask = ring_size_ - 1;
    a.gen = gen_.load() + 1;
    // (A/B bits of TONK_AMD_SERVE_DEBUG >> 2: 1 no release fence before the completion word,
    // 2 the dispatcher polls one slot at a time, 4 commands copied with plain 16-byte loads,
    // 8 reads stored with system-scope 8-byte stores)
    a.pad = debug_ >> 2;
    // the instance's claim counter and quit flag start from zero (stream order: after the
    // previous instance has ended)
    if (hipMemsetAsync(dstate_, 0, sizeof(tamd_serve_dev), st) != hipSuccess) return false;
    hipLaunchKernelGGL(tamd_serve, dim3(1 + workers_), dim3(TAMD_SERVE_THREADS), 0, st, a);
    if (hipGetLastError() != hipSuccess) return false;
    gen_.store(a.gen);
    launches.fetch_add(1, std::memory_order_relaxed);
    return true;
}

bool Server::ensure_running() {
    std::lock_guard<std::mutex> lk(launch_mu_);
    if (dead_.load()) return false;
    if (host_->exited_gen != gen_.load()) return true;  // the current instance runs (or a relaunch won)
    dev_->bind_thread();
    const uint64_t tail = host_->exit_tail;
    const double t0 = now_us();
    if (launch_locked(tail)) {
        const double us = now_us() - t0;
        if (stamps_ && us > 2000.0)  // (watchdog: a relaunch every waiting caller sits behind)
            fprintf(stderr, "tonk_amd: slow executor relaunch: %.1f ms (launch %llu)\n", us * 1e-3,
                    (unsigned long long)launches.load());
        return true;
    }
    // Nothing will consume the ring: later calls take the launch path, and the waits of commands
    // already posted end at once (their codecs are disabled and keep their buffers).
    fprintf(stderr, "tonk_amd: relaunching the persistent executor failed; using kernel launches\n");
    dead_.store(true);
    return false;
}

bool Server::build(CmdBuf& b, const std::vector<Device::HostCopy>& up, const ProgramBuilder* pb,
                   const std::vector<Device::HostCopy>& rd) {
    uint32_t levels = 0, n_items = 0, n_instr = 0, n_ops = 0, B = 0;
    if (pb && !pb->empty()) {
        B = (uint32_t)pb->level_ops().size();
        B = (B + TAMD_COST_CLASSES - 1) / TAMD_COST_CLASSES * TAMD_COST_CLASSES;
        levels = B / TAMD_COST_CLASSES;
        for (uint32_t c : pb->level_items()) n_items += c;
        n_instr = (uint32_t)pb->instrs().size();
        n_ops = (uint32_t)pb->ops().size();
    }
    if (levels > TAMD_SERVE_MAX_LEVELS) return false;
    for (const Device::HostCopy& x : up)
        if (((uintptr_t)x.host & 15u) || (x.arena_off & 63u) || x.arena_off / 64 > 0xffffffffull) return false;
    for (const Device::HostCopy& x : rd)
        if (((uintptr_t)x.host & 15u) || (x.arena_off & 63u) || x.arena_off / 64 > 0xffffffffull) return false;
    const uint32_t off_up = (uint32_t)((sizeof(tamd_cmd) + 15) & ~(size_t)15);
    const uint32_t off_rd = off_up + 16u * (uint32_t)up.size();
    const uint32_t off_instr = off_rd + 16u * (uint32_t)rd.size();
    const uint32_t off_ops = off_instr + 16u * (n_instr + 8u);  // (the executor reads a batch past the end)
    const uint32_t off_items = off_ops + 16u * n_ops;
    const uint32_t bytes = (off_items + 8u * n_items + 15u) & ~15u;
    if ((size_t)bytes + 256 > TAMD_SERVE_CMD_BYTES) return false;
    if (CmdBuf::kHead + bytes > b.cap) {
        if (b.bar) Device::bar_free(b.mem);
        else Device::host_free(b.mem);
        b.cap = 4096;
        while (b.cap < CmdBuf::kHead + bytes) b.cap <<= 1;
        b.mem = (uint8_t*)(b.bar ? Device::bar_alloc(b.cap) : Device::host_alloc(b.cap));
        if (b.bar && !b.head) {
            b.head = (uint8_t*)Device::host_alloc(4096);
            if (b.head) memset(b.head, 0, CmdBuf::kHead);
            b.done_at = (volatile uint64_t*)b.head;
        }
        if (!b.mem || (b.bar && !b.head)) {
            b.cap = 0;
            return false;
        }
        if (!b.bar) memset(b.mem, 0, CmdBuf::kHead);
    }
    b.bytes = bytes;
    b.shape[0] = levels;
    b.shape[1] = n_items;
    b.shape[2] = n_instr;
    b.shape[3] = (uint32_t)up.size();
    uint8_t* base = (uint8_t*)b.cmd();
    tamd_cmd* c = b.cmd();
    memset(c, 0, sizeof(tamd_cmd));
    c->bytes = bytes;
    c->n_up = (uint32_t)up.size();
    c->n_rd = (uint32_t)rd.size();
    c->levels = levels;
    c->off_up = off_up;
    c->off_rd = off_rd;
    c->off_instr = off_instr;
    c->off_ops = off_ops;
    c->off_items = off_items;
    c->n_items = n_items;
    c->n_instr = n_instr;
    c->n_ops = n_ops;
    tamd_xfer* xu = (tamd_xfer*)(base + off_up);
    uint64_t chunks = 0;
    bool ordered = true;
    for (size_t i = 0; i < up.size(); ++i) {
        xu[i] = tamd_xfer{(uint64_t)(uintptr_t)up[i].host, (uint32_t)(up[i].arena_off / 64), up[i].len};
        chunks += (up[i].len + 15u) / 16u;
        if (i && (uintptr_t)up[i].host < (uintptr_t)up[i - 1].host + up[i - 1].len) ordered = false;
    }
    if (!up.empty() && ordered) {
        const uint64_t span = ((uintptr_t)up.back().host + up.back().len + 15u - (uintptr_t)up[0].host) / 16u;
        if (span <= 2 * chunks + 64 && span < (1u << 24)) c->up_chunks = (uint32_t)span;
    }
    tamd_xfer* xr = (tamd_xfer*)(base + off_rd);
    for (size_t i = 0; i < rd.size(); ++i)
        xr[i] = tamd_xfer{(uint64_t)(uintptr_t)rd[i].host, (uint32_t)(rd[i].arena_off / 64), rd[i].len};
    if (!levels) return true;
    // Multi-target DENSE runs are not built into the executor (its registers are at the limit);
    // a program with one takes the launch path (per-call programs hold one encode each, so their
    // rows are never grouped).
    for (const tamd_instr& in : pb->instrs())
        if ((in.w0 & 0xffu) == TAMD_I_ACCR && ((in.w0 >> 8) & 0xffu) == TAMD_R_DENSE && ((in.w0 >> 16) & 0xffu) > 1u)
            return false;
    // The program as Device::begin / fill lay out one context's: ops grouped by bucket (level,
    // then cost class, most expensive first), each op's work items (op, slice) in that order.
    memcpy(base + off_instr, pb->instrs().data(), (size_t)n_instr * sizeof(tamd_instr));
    memset(base + off_instr + 16u * n_instr, 0, 16u * 8u);
    uint32_t op_fill[TAMD_SERVE_MAX_LEVELS * TAMD_COST_CLASSES], item_fill[TAMD_SERVE_MAX_LEVELS * TAMD_COST_CLASSES];
    uint32_t op_at = 0, item_at = 0;
    const std::vector<uint32_t>& lo = pb->level_ops();
    const std::vector<uint32_t>& li = pb->level_items();
    for (uint32_t k = 0; k < B; ++k) {
        if (k % TAMD_COST_CLASSES == 0) c->level_base[k / TAMD_COST_CLASSES] = item_at;
        op_fill[k] = op_at;
        item_fill[k] = item_at;
        if (k < lo.size()) {
            op_at += lo[k];
            item_at += li[k];
        }
    }
    c->level_base[levels] = item_at;
    tamd_op* ho = (tamd_op*)(base + off_ops);
    uint32_t* hi = (uint32_t*)(base + off_items);
    const std::vector<tamd_op>& ops = pb->ops();
    const std::vector<uint32_t>& lv = pb->op_levels();
    const std::vector<uint8_t>& pure = pb->op_pure();
    for (size_t i = 0; i < ops.size(); ++i) {
        const uint32_t k = lv[i];
        const uint32_t oi = op_fill[k]++;
        ho[oi] = ops[i];
        const uint32_t slices = op_slices(ops[i].span);
        uint32_t ii = item_fill[k];
        item_fill[k] += slices;
        // (bit 31 of the slice word: a pure combine, whose row batches a group of waves may split)
        const uint32_t share = pure[i] == 1 ? 0x80000000u : 0u;  // (2: several accumulators, one wave)
        for (uint32_t s = 0; s < slices; ++s, ++ii) {
            hi[2 * ii] = oi;
            hi[2 * ii + 1] = s | share;
        }
    }
    return true;
}

void Server::post(CmdBuf& b) {
    const uint64_t idx = head_.fetch_add(1, std::memory_order_relaxed);
    tamd_serve_slot* s = &ring_[idx & (ring_size_ - 1)];
    // the slot's previous command (idx - ring size) must have been handed on
    for (uint32_t spin = 0; idx >= host_->consumed + ring_size_; ++spin) {
        if ((spin & 255) == 255) {
            if (host_->exited_gen == gen_.load()) ensure_running();
            if (dead_.load(std::memory_order_relaxed)) break;
            sched_yield();
        }
        _mm_pause();
    }
    if (idx >= host_->consumed + ring_size_) {  // dead server, slot still taken: never written
        b.ticket = idx;
        b.busy = true;
        return;
    }
    const bool stall = stall_post_ms_ && idx == 100;
    if (stall) {  // (test hook: a poster descheduled between its ticket and its descriptor)
        stall_pending_.store(true);
        std::this_thread::sleep_for(std::chrono::milliseconds(stall_post_ms_));
    }
    // six tagged granules, 8-byte stores (each one atomic): the dispatcher takes the slot once
    // every tag is this command's
    const uint64_t cmd = (uint64_t)(uintptr_t)b.cmd(), done = (uint64_t)(uintptr_t)b.done();
    // the command and the packets it lands, when they were written through the BAR
    // (write-combined), leave the CPU before its descriptor does (PCIe keeps posted writes in order)
    _mm_sfence();
    volatile uint64_t* g = s->g;
    g[0] = tamd_granule(idx, (uint32_t)cmd);
    g[1] = tamd_granule(idx, (uint32_t)(cmd >> 32));
    g[2] = tamd_granule(idx, (uint32_t)done);
    g[3] = tamd_granule(idx, (uint32_t)(done >> 32));
    g[4] = tamd_granule(idx, (uint32_t)(idx + 1));
    g[5] = tamd_granule(idx, b.bytes);
    if (stall) stall_pending_.store(false);
    b.ticket = idx;
    b.busy = true;
    if (stamps_) {
        b.posted_us = now_us();
        std::lock_guard<std::mutex> lk(stamp_mu_);
        shape_[0] += b.shape[0];
        shape_[1] += b.shape[1];
        shape_[2] += b.shape[2];
        shape_[3] += b.shape[3];
        shape_[4] += b.bytes;
        shape_n_++;
    }
    posted.fetch_add(1, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    if (host_->exited_gen == gen_.load()) ensure_running();
}

bool Server::wait(CmdBuf& b) {
    const uint64_t want = (uint32_t)(b.ticket + 1);  // (the worker stores the 32-bit tag)
    volatile uint64_t* d = b.done();
    if (*d == want) {
        b.busy = false;
        std::atomic_thread_fence(std::memory_order_acquire);
        return true;
    }
    const double t0 = now_us();
    if (park_) return wait_parked(b, t0);
    // At most spinners_max() callers spin (and yield) at a time; the others poll with short sleeps
    // (TONK_AMD_SPINNERS: a bound on the CPU that waiting callers burn in processes with hundreds
    // of calling threads on a few cores).
    struct SpinSlot {
        bool mine;
        SpinSlot() : mine(g_spinners.fetch_add(1, std::memory_order_relaxed) < spinners_max()) {
            if (!mine) g_spinners.fetch_sub(1, std::memory_order_relaxed);
        }
        ~SpinSlot() { if (mine) g_spinners.fetch_sub(1, std::memory_order_relaxed); }
    } slot;
    for (uint32_t spin = 1;; ++spin) {
        if (*d == want) break;
        if (dead_.load(std::memory_order_relaxed)) return false;  // (b stays busy: never reused)
        if (!slot.mine && (spin & 63) != 0) {
            std::this_thread::sleep_for(std::chrono::microseconds(10));
            spin |= 63;  // (every poll of a sleeper also takes the checks below)
            continue;
        }
        if ((spin & 63) == 0) {
            const double t = now_us() - t0;
            // the executor ended on an idle spell without taking this command: start the next one
            if (host_->exited_gen == gen_.load() && host_->exit_tail <= b.ticket && !ensure_running()) return false;
            if (t > timeout_us_) {
                // The command is still posted and may run later: the server goes dead (new
                // commands take the launch path), and the caller keeps `b`, its codec's pinned
                // buffers and rows for good (capi.cpp Codec::stalled).
                dead_.store(true);
                fprintf(stderr, "tonk_amd: command %llu not completed after %.0f us (done word %llu); dispatcher: start %llu "
                        "polls/1024 %llu waits for %llu; command 0: stage %llu block %llu; consumed %llu exited_gen %llu "
                        "(launched %u) exit_tail %llu\n",
                        (unsigned long long)b.ticket, timeout_us_, (unsigned long long)*d, (unsigned long long)host_->dbg[0],
                        (unsigned long long)host_->dbg[1], (unsigned long long)host_->dbg[2],
                        (unsigned long long)host_->dbg[3], (unsigned long long)host_->dbg[4],
                        (unsigned long long)host_->consumed, (unsigned long long)host_->exited_gen, gen_.load(),
                        (unsigned long long)host_->exit_tail);
                fprintf(stderr, "tonk_amd: the persistent executor is off; using kernel launches\n");
                return false;
            }
            // a short spin, then give the core to other threads between polls (a Tonk process
            // has hundreds of threads on a few cores)
            if (t > 30.0) {
                if (t > 2000.0) {
                    waits_slow.fetch_add(1, std::memory_order_relaxed);
                    std::this_thread::sleep_for(std::chrono::microseconds(20));
                } else {
                    sched_yield();
                }
            }
        }
        _mm_pause();
    }
    return completed(b);
}

// The command in `b` is done (its completion word seen).
bool Server::completed(CmdBuf& b) {
    volatile uint64_t* d = b.done();
    std::atomic_thread_fence(std::memory_order_acquire);
    b.busy = false;
    if (stamps_) {  // (watchdog: where a command's time goes, 100 MHz stamps -> ns)
        const double wall = now_us() - b.posted_us;
        std::lock_guard<std::mutex> lk(stamp_mu_);
        phase_ns_[0] += (d[3] - d[1]) * 10;  // start -> command in LDS
        phase_ns_[1] += (d[4] - d[3]) * 10;  // -> packets landed
        phase_ns_[2] += (d[5] - d[4]) * 10;  // -> program run
        phase_ns_[3] += (d[6] - d[5]) * 10;  // -> reads written
        phase_ns_[4] += (d[2] - d[6]) * 10;  // -> completion stored (fence)
        phase_ns_[5] += (uint64_t)(wall * 1e3) - (d[2] - d[1]) * 10;  // host wall outside the worker
        phase_n_++;
    }
    gpu_ns_sum.fetch_add((d[2] - d[1]) * 10, std::memory_order_relaxed);
    if (stall_post_ms_ && b.ticket > 100 && stall_pending_.load()) stall_passed_.fetch_add(1);
    return true;
}

// Spin on the completion word for spin_us_, spin and yield up to yield_us_ (a command that lands
// just after the spin costs no wake-up), then park (server.h Parked): the poller wakes the caller
// when the word is written; the caller also wakes every millisecond to check the executor's life
// (idle exit, timeout, dead server) as the spinning loop does.
bool Server::wait_parked(CmdBuf& b, double t0) {
    const uint64_t want = (uint32_t)(b.ticket + 1);
    volatile uint64_t* d = b.done();
    Parked p;
    p.done = d;
    p.want = want;
    p.ticket = b.ticket;
    bool parked = false;
    for (uint32_t spin = 1;; ++spin) {
        if (*d == want) break;
        if (dead_.load(std::memory_order_relaxed)) {
            if (parked) unpark(p);
            return false;  // (b stays busy: never reused)
        }
        if (parked) {
            if (!p.woken.load(std::memory_order_acquire)) futex_wait(&p.woken, 0, 1000000L);
            if (p.woken.load(std::memory_order_acquire)) break;
        } else if ((spin & 63) != 0) {
            _mm_pause();
            continue;
        }
        const double t = now_us() - t0;
        if (host_->exited_gen == gen_.load() && host_->exit_tail <= b.ticket && !ensure_running()) {
            if (parked) unpark(p);
            return false;
        }
        if (t > timeout_us_) {
            if (parked) unpark(p);
            dead_.store(true);
            fprintf(stderr, "tonk_amd: command %llu not completed after %.0f us (done word %llu); dispatcher: start %llu "
                    "polls/1024 %llu waits for %llu; command 0: stage %llu block %llu; consumed %llu exited_gen %llu "
                    "(launched %u) exit_tail %llu\n",
                    (unsigned long long)b.ticket, timeout_us_, (unsigned long long)*d, (unsigned long long)host_->dbg[0],
                    (unsigned long long)host_->dbg[1], (unsigned long long)host_->dbg[2],
                    (unsigned long long)host_->dbg[3], (unsigned long long)host_->dbg[4],
                    (unsigned long long)host_->consumed, (unsigned long long)host_->exited_gen, gen_.load(),
                    (unsigned long long)host_->exit_tail);
            fprintf(stderr, "tonk_amd: the persistent executor is off; using kernel launches\n");
            return false;
        }
        if (!parked && t > spin_us_ && t <= yield_us_) {
            sched_yield();
            continue;
        }
        if (!parked && t > yield_us_) {
            std::call_once(poller_once_, [this] { poller_ = std::thread([this] { poller_loop(); }); });
            {
                std::lock_guard<std::mutex> lk(park_mu_);
                parked_.push_back(&p);
            }
            park_seq_.fetch_add(1, std::memory_order_release);
            futex_wake(&park_seq_);
            waits_parked.fetch_add(1, std::memory_order_relaxed);
            parked = true;
        }
    }
    if (parked) {
        unpark(p);
        if (now_us() - t0 > 2000.0) waits_slow.fetch_add(1, std::memory_order_relaxed);
    }
    return completed(b);
}

// Off the poller's list (a no-op when the poller took it): after this the poller no longer
// touches `p` (it wakes under the same lock).
void Server::unpark(Parked& p) {
    std::lock_guard<std::mutex> lk(park_mu_);
    for (size_t i = 0; i < parked_.size(); ++i)
        if (parked_[i] == &p) {
            parked_[i] = parked_.back();
            parked_.pop_back();
            break;
        }
}

// The poller: while callers are parked, rescan their completion words (about every microsecond)
// and wake the done ones; with none parked, sleep on park_seq_.  It also relaunches the executor
// when it ended on an idle spell with parked commands still unconsumed.
void Server::poller_loop() {
    while (!poller_stop_.load(std::memory_order_relaxed)) {
        const uint32_t seq = park_seq_.load(std::memory_order_acquire);
        size_t left;
        uint64_t low_ticket = ~0ull;
        {
            std::lock_guard<std::mutex> lk(park_mu_);
            for (size_t i = 0; i < parked_.size();) {
                Parked* p = parked_[i];
                if (*p->done == p->want) {
                    p->woken.store(1, std::memory_order_release);
                    futex_wake(&p->woken);
                    parked_[i] = parked_.back();
                    parked_.pop_back();
                } else {
                    if (p->ticket < low_ticket) low_ticket = p->ticket;
                    ++i;
                }
            }
            left = parked_.size();
        }
        if (!left) {
            futex_wait(&park_seq_, seq, 10000000L);
            continue;
        }
        if (host_->exited_gen == gen_.load() && host_->exit_tail <= low_ticket) ensure_running();
        for (int i = 0; i < 64; ++i) _mm_pause();
    }
}

std::string Server::phase_report() {
    std::lock_guard<std::mutex> lk(stamp_mu_);
    if (!phase_n_) return std::string();
    char b[320];
    const double n = (double)phase_n_ * 1e3;
    snprintf(b, sizeof(b), "commands %llu, us each: copy %.2f land %.2f program %.2f reads %.2f fence+done %.2f; host wall outside the worker %.2f",
             (unsigned long long)phase_n_, phase_ns_[0] / n, phase_ns_[1] / n, phase_ns_[2] / n, phase_ns_[3] / n,
             phase_ns_[4] / n, phase_ns_[5] / n);
    std::string r = b;
    if (shape_n_) {
        const double k = (double)shape_n_;
        snprintf(b, sizeof(b), "; per command: levels %.2f items %.1f instrs %.1f packets landed %.1f bytes %.0f",
                 shape_[0] / k, shape_[1] / k, shape_[2] / k, shape_[3] / k, shape_[4] / k);
        r += b;
    }
    return r;
}

void Server::stop() {
    if (!ring_) return;
    if (stall_post_ms_)
        fprintf(stderr, "tonk_amd: %llu commands completed behind the stalled post\n",
                (unsigned long long)stall_passed_.load());
    if (stamps_)  // (watchdog: the executor's life at process exit)
        fprintf(stderr, "tonk_amd: executor stop: posted=%llu launches=%llu; %s\n", (unsigned long long)posted.load(),
                (unsigned long long)launches.load(), phase_report().c_str());
    if (poller_.joinable()) {
        poller_stop_.store(true);
        park_seq_.fetch_add(1);
        futex_wake(&park_seq_);
        poller_.join();
    }
    host_->stop = 1;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    hipStream_t st = (hipStream_t)stream_;
    for (int i = 0; i < 2000 && hipStreamQuery(st) == hipErrorNotReady; ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    ok_ = false;
}

}  // namespace tamd
