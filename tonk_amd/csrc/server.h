// server.h -- host side of the launch-free submission path (serve.h): the command ring, the
// persistent executor's life cycle and the completion waits of the siamese.h C ABI.
//
// Calls never launch, record or wait on HIP objects: a call writes its command into its codec's
// pinned buffer, stores the command's address into the ring (a release store of the slot's
// sequence word) and spins on the command's completion word.  The only HIP calls left are the
// executor's (re)launches -- at start, and after it ended on an idle spell -- made under the
// server's own mutex, never under the device lock.
#pragma once

#include "device.h"
#include "serve.h"

#include <atomic>
#include <mutex>
#include <thread>
#include <stdint.h>
#include <string>
#include <vector>

namespace tamd {

// A codec's command buffer: [0, 128) completion words (done, start, end), then the command.
// With `bar` the buffer is device memory the host writes through the PCIe BAR (Device::bar_alloc:
// the executor copies the command at HBM latency); its completion words, which the host polls,
// then live in a pinned block of their own (`head`).  The host never reads a BAR buffer.
struct CmdBuf {
    uint8_t* mem = nullptr;
    size_t cap = 0;
    uint64_t ticket = 0;   // ring index of the command in flight from this buffer
    double posted_us = 0;  // (watchdog stamps)
    bool busy = false;     // posted and not yet waited for
    bool bar = false;
    uint8_t* head = nullptr;  // (bar) pinned completion words
    uint32_t bytes = 0;       // the command's size (Server::build)
    uint32_t shape[4] = {0, 0, 0, 0};  // levels, items, instructions, uploads (watchdog stamps)
    static const size_t kHead = 128;
    volatile uint64_t* done_at = nullptr;  // completion words (null: the buffer's head)
    volatile uint64_t* done() const { return done_at ? done_at : (volatile uint64_t*)mem; }
    tamd_cmd* cmd() const { return (tamd_cmd*)(mem + kHead); }
    void release() {  // (the command must be complete)
        if (bar) {
            Device::bar_free(mem);
            Device::host_free(head);
            head = nullptr;
            done_at = nullptr;
        } else {
            Device::host_free(mem);
        }
        mem = nullptr;
        cap = 0;
    }
};

class Server {
public:
    // Ring, control words and device state; the executor's first instance is launched on a
    // stream of its own (high priority, non-blocking: it must not share a hardware queue with
    // the launch streams, whose work would queue behind a resident kernel).  False: no server,
    // the C ABI keeps its launch path.
    bool init(Device& dev, unsigned workers, unsigned ring_size, double idle_ms);
    bool ok() const { return ok_; }
    // Whether new commands may be posted.  False once a command timed out or a relaunch of the
    // executor failed: later calls take the launch path, and commands already posted are only
    // checked, never waited for again (wait() returns false at once for one not done).
    bool live() const { return ok_ && !dead_.load(std::memory_order_relaxed); }
    // Build a command into `b` (grown as needed): `up` packets to land, the program of `pb`
    // (may be null or empty), `rd` rows to read back.  False when it does not fit the worker's
    // LDS (TAMD_SERVE_CMD_BYTES) or has too many levels: the caller takes the launch path.
    static bool build(CmdBuf& b, const std::vector<Device::HostCopy>& up, const ProgramBuilder* pb,
                      const std::vector<Device::HostCopy>& rd);
    // Post the command in `b` (after build); wait for it.  wait() returns false on a timeout
    // (the executor stopped answering: the server goes dead, the codec is disabled and keeps
    // the command's buffers and rows for good -- the command may still run later).
    void post(CmdBuf& b);
    bool wait(CmdBuf& b);
    bool settle(CmdBuf& b) { return b.busy ? wait(b) : true; }
    void stop();  // process exit: the executor ends and the stream drains (bounded wait)
    std::string phase_report();  // (watchdog) mean time per command phase

    // counters for the C ABI's watchdog
    std::atomic<uint64_t> posted{0}, launches{0}, waits_slow{0}, waits_parked{0};
    std::atomic<uint64_t> gpu_ns_sum{0};  // executor time of the commands waited for

private:
    bool ok_ = false;
    Device* dev_ = nullptr;
    void* stream_ = nullptr;
    tamd_serve_slot* ring_ = nullptr;
    volatile tamd_serve_host* host_ = nullptr;
    tamd_serve_dev* dstate_ = nullptr;
    uint32_t ring_size_ = 0, workers_ = 0;
    uint64_t idle_ticks_ = 0;
    std::atomic<uint64_t> head_{0};
    std::mutex launch_mu_;
    std::atomic<uint32_t> gen_{0};  // generation of the instance launched last
    std::atomic<bool> dead_{false};
    double timeout_us_ = 3e6;  // a command not completed after this long kills the server
    bool ensure_running();      // false (and the server dead) when a relaunch failed
    uint32_t debug_ = 0;  // TONK_AMD_SERVE_DEBUG bits (diagnostics): 1 the probe's completion words in
                          // the server's own coherent page, 4 a release fence before every completion word
    uint64_t* dbg_done_ = nullptr;
    // Test hook (TONK_AMD_SERVE_STALL_POST_MS): command 100's poster sleeps this long between
    // taking its ticket and writing its descriptor; commands completed meanwhile behind it are
    // counted and reported when the server stops (the ring hands slots on out of order).
    uint32_t stall_post_ms_ = 0;
    std::atomic<bool> stall_pending_{false};
    std::atomic<uint64_t> stall_passed_{0};
    bool stamps_ = false;
    std::mutex stamp_mu_;
    uint64_t phase_ns_[6] = {0, 0, 0, 0, 0, 0}, phase_n_ = 0;
    uint64_t shape_[5] = {0, 0, 0, 0, 0}, shape_n_ = 0;
    bool launch_locked(uint64_t tail0);

    // Completion waits that outlast a short spin are parked: the caller sleeps on a futex word and
    // one poller thread watches the completion words of every parked caller, waking each when its
    // command is done.  A Tonk process has hundreds of calling threads on a CPU quota of a few
    // cores: waiters that poll (yield or short sleeps) burn that quota as a group, and a burst of
    // them starves the threads that post and consume (a start-up that never recovers speed).
    struct Parked {
        volatile uint64_t* done;
        uint64_t want, ticket;
        std::atomic<uint32_t> woken{0};
    };
    std::mutex park_mu_;
    std::vector<Parked*> parked_;
    std::atomic<uint32_t> park_seq_{0};  // futex word of the poller while nothing is parked
    std::thread poller_;
    std::once_flag poller_once_;
    std::atomic<bool> poller_stop_{false};
    double spin_us_ = 30.0;   // TONK_AMD_WAIT_SPIN_US: spin this long,
    double yield_us_ = 150.0; // TONK_AMD_WAIT_YIELD_US: then spin and yield up to this long, then park
    bool park_ = true;       // TONK_AMD_WAIT_PARK=0: the round-5 yield/sleep polling (A/B)
    void poller_loop();
    void unpark(Parked& p);
    bool wait_parked(CmdBuf& b, double t0);
    bool completed(CmdBuf& b);
};

}  // namespace tamd
