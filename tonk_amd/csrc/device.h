// device.h -- HIP runtime of the engine: device arena, GF tables, program upload and
// level-by-level execution on one HIP stream.  All byte work of the codec runs here.
#pragma once

#include "engine.h"

#include <stdint.h>
#include <atomic>
#include <deque>
#include <mutex>
#include <vector>
#include <string>

namespace tamd {

struct DeviceStats {
    uint64_t programs = 0, launches = 0, ops = 0, items = 0, instrs = 0;
    uint64_t upload_bytes = 0;
    uint64_t acc_bytes = 0, store_bytes = 0;  // op-trace bytes of all programs run
    double kernel_ms = 0;  // sum of tamd_exec durations (when timing is enabled)
    double slot_wait_ms = 0, upload_enqueue_ms = 0;  // host time in begin() waits / H2D enqueue
    double upload_enqueue_max_ms = 0;
    uint64_t slot_reallocs = 0;
    uint64_t timed_launches = 0;
    double d2h_copy_ms = 0;  // stage_host: duration of the D2H copies (events around each copy)
};

class Device {
public:
    ~Device();
    // Opens `device`, allocates the arena and uploads the GF tables.  Returns false (with a
    // message in error()) when no usable gfx950 device is present: the engine has no CPU path.
    bool init(int device, uint64_t arena_bytes);
    // The same with a growable arena: `max_bytes` of address space reserved, `arena_bytes`
    // mapped now, grow_arena() maps more (HIP virtual memory management).  Falls back to a
    // fixed arena of `arena_bytes` where the device does not support it.
    bool init_growable(int device, uint64_t arena_bytes, uint64_t max_bytes);
    // arena_bytes() >= min_bytes afterwards, or false.  Thread safe, and independent of every
    // other Device call (it maps memory into the reserved range past everything in use), so the
    // C ABI grows without its device lock.
    bool grow_arena(uint64_t min_bytes);
    // Start growing the arena by half on a background thread (at most one growth at a time),
    // so codecs find the memory mapped before they need it.
    void grow_arena_async();
    uint64_t reserved_bytes() const { return reserved_bytes_; }
    // Program staging: `count` pinned/device slot pairs of `bytes` each (grown on demand), used
    // round robin; a program waits only for the program `count` back.  Call before init.
    // Default 2 x 16 MB (the session's big step programs); the C ABI runs many small ones.
    // `oversize` > 0 adds one more slot of that size for the rare program larger than a regular
    // slot (the C ABI: a decode that solves hundreds of unknowns in one call), so such a program
    // waits only for the previous oversize one instead of draining the device to grow every slot.
    void set_program_slots(size_t count, size_t bytes, size_t oversize = 0) {
        slots_.assign(count < 2 ? 2 : count, Slot());
        slot_bytes_ = bytes;
        big_cap_ = oversize;
    }
    // Staging bytes a program of these builders needs (Device::begin's layout) and the slots'
    // current capacity: a caller merging programs (the C ABI's batches) keeps a merge within it,
    // since growing the slots drains the device and reallocates every slot.
    static size_t program_bytes(const ProgramBuilder& pb) {
        size_t items = 0;
        for (uint32_t c : pb.level_items()) items += c;
        return (pb.instrs().size() + pb.ops().size()) * 16 + items * 8;
    }
    size_t slot_capacity() const { return slot_cap_ ? slot_cap_ : slot_bytes_; }
    size_t oversize_capacity() const { return big_cap_; }
    const std::string& error() const { return error_; }
    bool failed() const { return failed_; }  // any HIP call failed (sticky; safe to read unlocked)
    uint64_t arena_bytes() const { return arena_bytes_; }
    int device() const { return device_; }
    // Make this device current on the calling thread: HIP's current device is
    // per thread, and events, streams and allocations of a call belong to the current one.
    void bind_thread() const;
    uint8_t* arena() const { return arena_; }
    const uint32_t* gf_tables() const { return d_gf_; }  // the executor's LDS table image (kernels.hip)
    const uint8_t* zero_row() const { return d_zero_; }
    // An empty kernel on every launch stream; returns the longest any took to complete (ms,
    // capped near 2000): a stream that shares a hardware queue with a resident kernel waits.
    double probe_streams();
    void* stream() const { return stream_; }
    // Several launch streams (the C ABI): add_streams(k) creates k - 1 more streams beside the
    // first; select_stream(i) makes stream i the one every following enqueue uses (the caller
    // serialises Device calls).  Work of one codec stays on one stream, so it stays ordered;
    // work of different codecs overlaps.  synchronize() and slot growth wait for all streams;
    // completed()/wait() tickets assume one stream (the session), callers with several streams
    // wait on their own events (record_event / event_wait).
    void add_streams(unsigned k);
    void select_stream(unsigned i) {
        if (i < streams_.size()) { stream_ = streams_[i]; cur_stream_ = i; }
    }
    unsigned stream_count() const { return streams_.empty() ? 1u : (unsigned)streams_.size(); }
    void warm_streams();  // first kernel and copies on every launch stream now (queue creation)
    static const unsigned kMaxStreams = 16;  // add_streams clamps to it

    // Enqueue the pending programs of `ctxs` as one merged program (asynchronous).  Returns the
    // completion ticket (monotonic); call completed() / wait() with it.
    uint64_t run(Context* const* ctxs, size_t n);
    uint64_t run(Context* ctx) { return run(&ctx, 1); }
    // The same in three phases so host threads can fill their part of the merged program in
    // parallel: begin() lays the program out (ops grouped by level, then by context) and waits
    // for the staging slot; fill(i) copies context i (thread safe for distinct i); launch()
    // uploads the program and enqueues one tamd_exec per level.  Returns the ticket.  With
    // `closed` the program is each context's closed program (Context::close_flush) instead of
    // its pending one, so the next program can be built while this one is filled.
    void begin(Context* const* ctxs, size_t n, bool closed = false);
    void fill(size_t i);
    uint64_t launch();
    // (verification descriptors, see verify_next below)
    struct VerifyDesc { uint32_t row, len, mode, pad; };
    struct VerifyOut { uint64_t hash; uint32_t len, ok; };

    // Parallel assembly without a layout pass (the session's free-running schedule).  A program
    // is opened (its staging slot: the slot's previous program must have completed), then any
    // number of threads add parts concurrently -- one context's pending program each -- and the
    // caller closes it: the parts' work items are merged level by level (cost class, then part),
    // the program is uploaded and launched like launch().  A part reserves its instructions and
    // ops with an atomic bump inside the slot, so no part waits for another; indices in the
    // program are relative to the slot's record area.  open/close: the launching thread only;
    // add_part: thread safe, no HIP call.
    struct Part {
        std::vector<uint32_t> bucket_start;  // buckets + 1 offsets into items
        std::vector<uint64_t> items;         // op record index | slice << 32, by bucket
        uint64_t acc_bytes = 0, store_bytes = 0;
        uint32_t n_instr = 0, n_ops = 0;
        std::vector<VerifyDesc> verify;      // rows to digest once the program completes
    };
    int open_program();
    bool add_part(int h, const ProgramBuilder& pb, Part& out);
    uint64_t close_program(int h, Part* const* parts, size_t n);
    // Parallel-assembly slots: `count` slots of `host_mb` MB pinned staging (the record area a
    // program can fill) and 4x that on the device, plus an item area; call before init.
    void set_assembly_slots(size_t count, size_t host_mb);
    // Small programs (few-stream sessions, the C ABI) are uploaded by a copy kernel instead of DMA
    // (its latency, not its rate, is what a single program waits for); call before init.
    void set_small_uploads(bool on) { small_uploads_ = on && small_upload_limit() > 0; }
    static size_t small_upload_limit();
    // Whether a program of `recs` records (instructions + ops) and `items` work items fits a slot;
    // ensure_assembly grows every slot to fit (drains the device first: no program may be open).
    bool assembly_fits(size_t recs, size_t items) const;
    bool ensure_assembly(size_t recs, size_t items);
    // Level pipelining across programs (the session; Context::kPipeDepth): a program's levels
    // above the depth are launched beside the next program's first levels.
    void set_pipelined(bool on) { pipelined_ = on; }
    bool pending_levels() const { return !progs_.empty(); }
    bool completed(uint64_t ticket);
    void wait(uint64_t ticket);
    void synchronize();

    // Host <-> arena copies (stream ordered).  upload() copies `src` into a pinned staging
    // buffer so the caller may reuse it immediately; staged packets reach the arena in one H2D
    // copy + one tamd_scatter_rows launch, enqueued before the next program, download or sync
    // (flush_uploads()).  download() is synchronous; download_async() only enqueues the copy
    // (the destination is valid after synchronize()).
    void upload(uint64_t arena_offset, const void* src, size_t n);
    void flush_uploads();
    // A caller-staged batch of packets: `bytes` of packet data in pinned `src`, followed there by
    // room for `n` descriptors (written here); one H2D copy and one tamd_scatter_rows launch
    // put packet k at arena unit offset rows[k].  `src` must stay untouched until an event
    // recorded after this call has completed.
    struct ScatterIn { uint32_t row, len, src; };
    void scatter_upload(uint8_t* pinned_src, size_t bytes, const ScatterIn* d, uint32_t n);
    void download(void* dst, uint64_t arena_offset, size_t n);
    // Synchronous copy that waits only for work already enqueued (deferred program levels stay
    // deferred, unlike download()).
    void download_now(void* dst, uint64_t arena_offset, size_t n);
    void download_async(void* dst, uint64_t arena_offset, size_t n);
    // Reads that complete outside the caller's lock (the C ABI's encode): D2H straight into the
    // caller's pinned buffer, then an event recorded behind it.  event_wait() may run without
    // any lock; record/release must hold the same lock as every other Device call.
    void download_pinned(void* pinned_dst, uint64_t arena_offset, size_t n);
    // Zero-copy transfers between pinned host memory and the arena: one tamd_host_copy launch
    // moves every listed packet (the kernel reads or writes the host pages over the link), instead
    // of a copy command per packet.  Host addresses must be pinned (host_alloc) and 16-B aligned;
    // arena offsets 64-B aligned.  to_host = false: the host bytes must stay untouched until an
    // event recorded after this call has completed; true: they are valid once it has.
    struct HostCopy { void* host; uint64_t arena_off; uint32_t len; };
    void host_copy(const HostCopy* d, uint32_t n, bool to_host);
    // While collecting, download_pinned() only lists its copy; flush_host_reads() then runs every
    // listed copy as one host_copy(to_host) launch (the C ABI's combined batches).
    void collect_host_reads(bool on) { collect_reads_ = on; }
    void flush_host_reads();
    void* record_event();
    void reserve_events(size_t n);  // pre-create events for record_event (no creation later)
    static bool event_wait(void* ev);  // false when the wait failed
    void event_release(void* ev) { free_events_.push_back(ev); }
    static void* host_alloc(size_t n);  // pinned (pooled; see device.cpp)
    static bool host_reserve(size_t n);  // map a pinned slab now if fewer than n bytes are left in it
    static void host_prefill(unsigned slabs);  // map (and warm) that many 64 MB slabs ahead of use
    static void host_free(void* p);
    // Device memory the host writes directly (fine-grained, through the PCIe BAR; pooled as the
    // pinned blocks): the C ABI's staging and commands when TONK_AMD_CAPI_BAR is on.  The host must
    // only store into it (a host load is an uncached PCIe round trip).
    static void* bar_alloc(size_t n);
    static void bar_free(void* p);

    // Bench helpers (kernels.hip).
    struct GenDesc { uint32_t row, index, len, pad; uint64_t seed; };
    void generate_rows(const std::vector<GenDesc>& d, uint32_t row_cap);
    struct DigestDesc { uint32_t row, skip, len, pad; };
    void digest_rows(const std::vector<DigestDesc>& d, std::vector<uint64_t>& out);

    // Output verification of the schedule as it runs (the session's record mode): the rows of
    // the next launched program are digested on the launch stream right after the launch that
    // completes that program, i.e. before any later launch can rewrite or reuse them, so the
    // timed schedule (early launch, release at completion) is checked unchanged.  `mode` 0:
    // FNV-1a over `len` bytes; 1: a length-prefixed original (`len` = its upper bound), FNV-1a
    // over the payload the header announces.  Results are read after synchronize(), in the
    // order the descriptors were given over all calls.
    void verify_next(const std::vector<VerifyDesc>& d);
    void verify_results(std::vector<VerifyOut>& out);  // all results so far (synchronizes)
    void verify_reset();                               // drop results read (after verify_results)
    bool gf_selftest();  // device v_perm multiply vs host tables, all 65536 products

    // Host staging (the PCIe-inclusive path): packets start and end in pinned host
    // memory.  h2d() copies on a dedicated stream; h2d_fence() makes every later launch wait for
    // the copies enqueued so far.  d2h_gather() packs rows (after everything enqueued on the
    // compute stream) into a device buffer and copies it to `pinned_dst` on a third stream;
    // h2d_after_d2h() then copies `n` bytes of it back (the received-recovery direction).
    struct GatherDesc { uint32_t row, len, out; };
    bool enable_staging();
    void h2d(uint64_t arena_offset, const void* pinned_src, size_t n);
    void h2d_fence();
    void d2h_gather(const std::vector<GatherDesc>& d, size_t bytes, void* pinned_dst);
    void h2d_after_d2h(const void* pinned_src, size_t n);
    void sync_staging();

    // Kernel timing with HIP events around every tamd_exec launch (on the launch stream).
    // Turning timing on or off also launches the empty kernel tamd_timed_region, so a kernel
    // trace of the run can average exactly the timed launches (tools/trace_region.py).
    void set_timing(bool on);
    DeviceStats& stats() { return stats_; }
    void collect_timing();  // adds pending event pairs into stats().kernel_ms

private:
    std::string error_;
    volatile bool failed_ = false;
    // growable arena (init_growable): reserved range, mapped prefix, physical chunks
    uint64_t reserved_bytes_ = 0, granule_ = 0;
    std::vector<std::pair<unsigned long long, uint64_t>> chunks_;  // (hipMemGenericAllocationHandle_t, bytes)
    bool map_chunk(uint64_t bytes);
    int device_ = -1;
    uint8_t* arena_ = nullptr;
    std::atomic<uint64_t> arena_bytes_{0};
    std::mutex grow_mu_;
    std::atomic<bool> growing_{false};
    uint32_t* d_gf_ = nullptr;
    uint8_t* d_zero_ = nullptr;
    bool small_uploads_ = false;
    uint32_t max_grid_ = 256;
    const void* exec_kernel_ = nullptr;  // tamd_exec16
    // host staging
    void* h2d_stream_ = nullptr;
    void* d2h_stream_ = nullptr;
    void* h2d_done_ = nullptr;   // hipEvent_t
    void* gather_done_ = nullptr;
    void* d2h_done_ = nullptr;
    uint8_t* gather_dev_ = nullptr;  // packed rows
    size_t gather_cap_ = 0;
    uint8_t* recv_dev_ = nullptr;    // received-recovery landing area
    size_t recv_cap_ = 0;
    std::vector<std::pair<void*, void*>> d2h_timing_;  // (start, end) events of D2H copies not yet read
    GatherDesc* gdesc_host_ = nullptr;
    GatherDesc* gdesc_dev_ = nullptr;
    size_t gdesc_cap_ = 0;
    void* stream_ = nullptr;
    // program staging: pinned host buffers and device buffers, double buffered
    // Program memory: every slot's device half is a part of ONE allocation (prog_dev_, slot k
    // at k * slot_cap_), so launches address programs by 32-bit offsets (tamd_segments).
    struct Slot {
        uint8_t* host = nullptr;   // pinned staging
        uint8_t* dev = nullptr;    // prog_dev_ + dev_off
        uint32_t dev_off = 0;
        void* done = nullptr;  // hipEvent_t
        uint64_t ticket = 0;
        std::atomic<uint32_t> bump{0};  // parallel assembly: records reserved in the record area
        bool failed = false;            // a part did not fit
        Slot() {}
        Slot(const Slot& o) : host(o.host), dev(o.dev), dev_off(o.dev_off), done(o.done), ticket(o.ticket) {}
        Slot& operator=(const Slot& o) {
            host = o.host; dev = o.dev; dev_off = o.dev_off; done = o.done; ticket = o.ticket;
            return *this;
        }
    };
    // parallel assembly geometry (set_assembly_slots): per slot, the item area then the records
    size_t asm_items_ = 0;        // item capacity (8 B each)
    size_t asm_host_recs_ = 0;    // records (16 B) staged in pinned memory
    size_t asm_dev_recs_ = 0;     // records the device slot holds (parts past the pinned area are
                                  // staged in heap buffers and copied separately)
    struct Spill { uint32_t rec; std::vector<uint8_t> bytes; };
    std::mutex spill_mu_;
    std::vector<Spill> spills_;   // parts of the open programs past their pinned area (rare)
    std::vector<int> spill_slot_;
    std::vector<Slot> slots_ = std::vector<Slot>(2);
    size_t slot_bytes_ = 16u << 20;  // requested initial capacity
    size_t slot_cap_ = 0;            // current capacity of every slot
    Slot big_;                       // the oversize slot (set_program_slots), after the regular ones
    size_t big_cap_ = 0;
    uint8_t* prog_dev_ = nullptr;
    uint8_t* prog_host_ = nullptr;   // pinned twin of prog_dev_
    bool alloc_slots(size_t cap);    // (re)allocate every slot; nothing may be in flight
    // layout of the program being assembled (begin/fill/launch)
    struct Plan {
        std::vector<const ProgramBuilder*> pbs;      // per context
        std::vector<uint32_t> instr_base;          // per context
        std::vector<uint32_t> op_start, item_start; // [context * levels + level]
        std::vector<uint32_t> level_items, item_base, level_coop;  // level_coop: class-0 items (first)
        std::vector<uint32_t> class_items;                       // per bucket (level, cost class)
        uint32_t levels = 0, buckets = 0;
        size_t n_instr = 0, n_ops = 0, n_items = 0, bytes_instr = 0, bytes_ops = 0, total = 0;
        Slot* slot = nullptr;
        bool empty = true;
    } plan_;
    int next_slot_ = 0;
    // Programs with levels still to launch (level pipelining), oldest first.  Every launch runs
    // the next level of each of them beside level 1 of the newest program; a program completes
    // (slot event, ticket) once its last level is launched and every older one has completed.
    struct Inflight {
        uint32_t ops = 0, instrs = 0, items = 0;  // offsets into prog_dev_
        uint32_t levels = 0, next = 1;
        std::vector<uint32_t> level_items, item_base, level_coop;
        std::vector<uint32_t> class_items;  // per level and cost class (TAMD_COST_CLASSES * level + class)
        Slot* slot = nullptr;
        uint64_t ticket = 0;
        int verify = -1;  // index into vbatches_ (digested when the program completes)
        bool done() const { return next >= levels; }
    };
    // verification batches (verify_next): descriptors and results in device memory
    struct VerifyBatch {
        std::vector<VerifyDesc> host;  // kept until the end: the H2D copy reads it asynchronously
        VerifyDesc* dev_desc = nullptr;
        VerifyOut* dev_out = nullptr;
        uint32_t count = 0;
    };
    std::vector<VerifyBatch> vbatches_;
    size_t vread_ = 0;       // batches whose results verify_results() has returned
    int pending_verify_ = -1;
    void run_verify(int batch);
    std::deque<Inflight> progs_;
    bool pipelined_ = false;
    uint64_t start_program(Inflight& cur, size_t n_instr, size_t n_ops, size_t n_items, size_t bytes);
    // one launch: the next level of every program in progs_ (+ `fresh`'s level 1 when given)
    void launch_step(Inflight* fresh, unsigned long long* stamps);
    void retire_done();
    void drain_programs();  // launch every remaining level, complete every program
    uint64_t ticket_ = 0, completed_ = 0;
    std::deque<std::pair<uint64_t, void*>> inflight_;  // (ticket, hipEvent_t) in stream order
    std::vector<void*> free_events_;
    bool ticket_is_empty_ = false;
    void mark(uint64_t ticket);
    // upload staging: packets at [up_flushed_, up_used_) of up_host_ are not enqueued yet
    struct ScatterDesc { uint32_t row, len, src, pad; };
    uint8_t* up_host_ = nullptr;
    uint8_t* up_dev_ = nullptr;
    uint8_t* sc_dev_ = nullptr;  // scatter_upload landing area (of the current stream)
    // host_copy: descriptor buffers (pinned, read by the kernel over the link), used in turn; each
    // is reused once the event recorded behind its launch has completed
    struct HcBuf { void* p = nullptr; size_t cap = 0; void* ev = nullptr; };
    HcBuf hc_[32];
    unsigned hc_next_ = 0;
    bool collect_reads_ = false;
    std::vector<HostCopy> reads_;
    size_t sc_cap_ = 0;
    std::vector<void*> streams_;  // all launch streams (add_streams), streams_[0] = the first
    std::vector<std::pair<uint8_t*, size_t>> sc_per_stream_;  // landing areas of the others
    unsigned cur_stream_ = 0;
    void sync_all_streams();
    size_t up_cap_ = 0, up_used_ = 0, up_flushed_ = 0;
    std::vector<ScatterDesc> up_pending_;
    // readback staging: download_async() lands rows in pinned rb_host_; synchronize() copies
    // them to the callers' buffers
    struct Readback { void* dst; size_t off, n; };
    uint8_t* rb_host_ = nullptr;
    size_t rb_cap_ = 0, rb_used_ = 0;
    std::vector<Readback> rb_pending_;
    void* up_event_ = nullptr;
    bool timing_ = false;
    std::vector<std::pair<void*, void*>> timing_events_;
    std::vector<void*> timing_pool_;
    void* timing_event();
    DeviceStats stats_;
    bool ensure_slot(Slot& s, size_t bytes);  // every slot grows (after a full drain) when short
};

} // namespace tamd
