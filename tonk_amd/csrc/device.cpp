// device.cpp -- HIP runtime of the engine (see device.h).
#include "device.h"

#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <chrono>
#include <unordered_map>
#include <thread>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

extern "C" __global__ void tamd_exec24(tamd_segments, const uint8_t*, uint32_t, uint8_t*, const uint32_t*,
                                        const uint8_t*, unsigned long long*);
extern "C" __global__ void tamd_exec16(tamd_segments, const uint8_t*, uint32_t, uint8_t*, const uint32_t*,
                                       const uint8_t*, unsigned long long*);
typedef void (*ExecFn)(tamd_segments, const uint8_t*, uint32_t, uint8_t*, const uint32_t*, const uint8_t*,
                       unsigned long long*);
extern "C" __global__ void tamd_gf_selftest(const uint32_t*, uint8_t*);
extern "C" __global__ void tamd_timed_region();
extern "C" __global__ void tamd_nop();
extern "C" __global__ void tamd_gather_rows(const tamd::Device::GatherDesc*, uint32_t, const uint8_t*, uint8_t*);
struct ScatterDescDev { uint32_t row, len, src, pad; };
extern "C" __global__ void tamd_scatter_rows(const ScatterDescDev*, uint32_t, const uint8_t*, uint8_t*);
struct HostCopyDev { uint64_t host; uint32_t unit, len; };
extern "C" __global__ void tamd_host_copy(const HostCopyDev*, uint32_t, uint8_t*, uint32_t);
extern "C" __global__ void tamd_copy_in(const uint4*, uint4*, uint32_t, const uint4*, uint4*, uint32_t);
namespace {
// Program uploads below this many bytes go through tamd_copy_in (a launch whose threads read the
// pinned bytes) instead of the DMA engine, on devices that asked for it (set_small_uploads: few
// streams, the C ABI); TONK_AMD_SMALL_UPLOAD overrides the size (0: never, A/B).
size_t small_upload() {
    static const size_t v = getenv("TONK_AMD_SMALL_UPLOAD") ? (size_t)atoll(getenv("TONK_AMD_SMALL_UPLOAD")) : (256u << 10);
    return v;
}
// Two host -> device ranges, by the copy kernel when small, else by DMA.
void upload2(bool small_ok, void* d0, const void* h0, size_t b0, void* d1, const void* h1, size_t b1, hipStream_t st) {
    if (small_ok && b0 + b1 < small_upload()) {
        const uint32_t n0 = (uint32_t)((b0 + 15) / 16), n1 = (uint32_t)((b1 + 15) / 16);
        const uint32_t blocks = std::min<uint32_t>(256u, (n0 + n1 + 255) / 256);
        if (n0 + n1)
            hipLaunchKernelGGL(tamd_copy_in, dim3(blocks), dim3(256), 0, st, (const uint4*)h0, (uint4*)d0, n0,
                               (const uint4*)h1, (uint4*)d1, n1);
        return;
    }
    if (b0) hipMemcpyAsync(d0, h0, b0, hipMemcpyHostToDevice, st);
    if (b1) hipMemcpyAsync(d1, h1, b1, hipMemcpyHostToDevice, st);
}
}  // namespace
size_t tamd::Device::small_upload_limit() { return small_upload(); }

struct GenDescDev { uint32_t row, index, len, pad; unsigned long long seed; };
struct DigestDescDev { uint32_t row, skip, len, pad; };
extern "C" __global__ void tamd_gen_rows(const GenDescDev*, uint32_t, uint8_t*, uint32_t);
extern "C" __global__ void tamd_digest_rows(const DigestDescDev*, uint32_t, const uint8_t*, unsigned long long*);
struct VerifyDescDev { uint32_t row, len, mode, pad; };
struct VerifyOutDev { unsigned long long hash; uint32_t len, ok; };
extern "C" __global__ void tamd_verify_rows(const VerifyDescDev*, uint32_t, const uint8_t*, VerifyOutDev*);

namespace tamd {

namespace {
int g_pin_device = -1;  // the device pinned slabs are mapped for (Device::init): bound before their HIP calls
}

// With the C ABI watchdog on (TONK_AMD_CAPI_WATCH), every runtime call through HIPCHK / HIPT
// that blocks for 10 ms or more is named on stderr.
static bool hip_watch() {
    static const bool on = getenv("TONK_AMD_CAPI_WATCH") != nullptr;
    return on;
}
struct HipTimer {
    const char* what;
    std::chrono::steady_clock::time_point t0;
    explicit HipTimer(const char* w) : what(w) { if (hip_watch()) t0 = std::chrono::steady_clock::now(); }
    ~HipTimer() {
        if (!hip_watch()) return;
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (ms >= 10.0) fprintf(stderr, "tonk_amd: slow HIP call %.1f ms: %.60s\n", ms, what);
    }
};
#define HIPT(x)                  \
    do {                         \
        HipTimer ht_(#x);        \
        x;                       \
    } while (0)
#define HIPCHK(x)                                                                        \
    do {                                                                                 \
        HipTimer ht_(#x);                                                                \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "tonk_amd: %s failed: %s\n", #x, hipGetErrorString(e_));     \
            error_ = std::string(#x) + ": " + hipGetErrorString(e_);                    \
            failed_ = true;                                                              \
        }                                                                                \
    } while (0)


Device::~Device() {
    if (device_ < 0) return;
    hipSetDevice(device_);
    if (streams_.empty()) hipStreamSynchronize((hipStream_t)stream_);
    else for (void* st : streams_) hipStreamSynchronize((hipStream_t)st);
    for (Slot& s : slots_)
        if (s.done) hipEventDestroy((hipEvent_t)s.done);
    if (big_.done) hipEventDestroy((hipEvent_t)big_.done);
    if (prog_host_) hipHostFree(prog_host_);
    if (prog_dev_) hipFree(prog_dev_);
    for (auto& p : inflight_) hipEventDestroy((hipEvent_t)p.second);
    for (void* e : free_events_) hipEventDestroy((hipEvent_t)e);
    for (auto& p : timing_events_) { hipEventDestroy((hipEvent_t)p.first); hipEventDestroy((hipEvent_t)p.second); }
    for (void* e : timing_pool_) hipEventDestroy((hipEvent_t)e);
    if (h2d_stream_) hipStreamSynchronize((hipStream_t)h2d_stream_);
    if (d2h_stream_) hipStreamSynchronize((hipStream_t)d2h_stream_);
    if (h2d_stream_) hipStreamDestroy((hipStream_t)h2d_stream_);
    if (d2h_stream_) hipStreamDestroy((hipStream_t)d2h_stream_);
    for (void* e : {h2d_done_, gather_done_, d2h_done_})
        if (e) hipEventDestroy((hipEvent_t)e);
    if (gather_dev_) hipFree(gather_dev_);
    if (recv_dev_) hipFree(recv_dev_);
    if (gdesc_dev_) hipFree(gdesc_dev_);
    if (gdesc_host_) hipHostFree(gdesc_host_);
    if (up_host_) hipHostFree(up_host_);
    if (up_dev_) hipFree(up_dev_);
    if (sc_dev_ && sc_per_stream_.empty()) hipFree(sc_dev_);
    if (rb_host_) hipHostFree(rb_host_);
    if (up_event_) hipEventDestroy((hipEvent_t)up_event_);
    for (HcBuf& b : hc_) {
        if (b.ev) hipEventDestroy((hipEvent_t)b.ev);
        host_free(b.p);
    }
    if (d_gf_) hipFree(d_gf_);
    if (d_zero_) hipFree(d_zero_);
    for (VerifyBatch& b : vbatches_)
        if (b.dev_desc) hipFree(b.dev_desc);
    if (reserved_bytes_) {
        hipMemUnmap(arena_, arena_bytes_);
        for (auto& c : chunks_) hipMemRelease((hipMemGenericAllocationHandle_t)c.first);
        hipMemAddressFree(arena_, reserved_bytes_);
    } else if (arena_) {
        hipFree(arena_);
    }
    if (streams_.empty()) {
        if (stream_) hipStreamDestroy((hipStream_t)stream_);
    } else {
        for (void* st : streams_) hipStreamDestroy((hipStream_t)st);
        for (auto& a : sc_per_stream_)
            if (a.first) hipFree(a.first);
    }
}

void Device::bind_thread() const {
    if (device_ >= 0) hipSetDevice(device_);  // (a thread-local assignment in HIP: cheap)
}

void Device::add_streams(unsigned k) {
    if (k > kMaxStreams) k = kMaxStreams;
    if (!stream_ || !streams_.empty() || k < 2) return;
    streams_.push_back(stream_);
    for (unsigned i = 1; i < k; ++i) {
        hipStream_t st = nullptr;
        HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        streams_.push_back(st);
    }
    sc_per_stream_.assign(k, std::make_pair((uint8_t*)nullptr, (size_t)0));
}

void Device::warm_streams() {
    // The runtime creates a stream's hardware queues on its first kernel and its first copy
    // (~80 ms each, blocking); do both on every launch stream now instead of under the device
    // lock of the first codecs to use them.
    uint8_t* h = (uint8_t*)host_alloc(4096);
    uint8_t* d = nullptr;
    HIPCHK(hipMalloc((void**)&d, 4096));
    if (!h || !d) return;
    std::vector<void*> all = streams_;
    if (all.empty()) all.push_back(stream_);
    // Then many commands in flight at once, so the runtime's per-queue pools (kernel arguments,
    // completion signals) grow to a working size now: under load each growth blocked ~80 ms.
    for (int round = 0; round < 2; ++round)
        for (void* s : all) {
            hipStream_t st = (hipStream_t)s;
            const int n = round ? 1024 : 1;
            for (int i = 0; i < n; ++i) {
                hipLaunchKernelGGL(tamd_nop, dim3(1), dim3(64), 0, st);
                if (i % 8 == 0) {
                    HIPCHK(hipMemcpyAsync(d, h, 64, hipMemcpyHostToDevice, st));
                    HIPCHK(hipMemcpyAsync(h, d, 64, hipMemcpyDeviceToHost, st));
                }
            }
            if (!round) HIPCHK(hipStreamSynchronize(st));
        }
    sync_all_streams();
    HIPCHK(hipFree(d));
    host_free(h);
    // scatter_upload's landing areas at their working size (a staged half: up to 1 MB of packets
    // and its descriptors), so none grows -- hipFree + hipMalloc -- while codecs run
    const size_t land = 2u << 20;
    if (!sc_per_stream_.empty()) {
        for (auto& a : sc_per_stream_)
            if (a.second < land) {
                if (a.first) HIPCHK(hipFree(a.first));
                HIPCHK(hipMalloc((void**)&a.first, land));
                a.second = land;
            }
    } else if (sc_cap_ < land) {
        if (sc_dev_) HIPCHK(hipFree(sc_dev_));
        HIPCHK(hipMalloc((void**)&sc_dev_, land));
        sc_cap_ = land;
    }
}

double Device::probe_streams() {
    std::vector<void*> all = streams_;
    if (all.empty()) all.push_back(stream_);
    const auto t0 = std::chrono::steady_clock::now();
    auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    for (void* s : all) hipLaunchKernelGGL(tamd_nop, dim3(1), dim3(64), 0, (hipStream_t)s);
    double worst = 0;
    for (void* s : all) {
        while (hipStreamQuery((hipStream_t)s) == hipErrorNotReady) {
            if (ms() > 2000.0) return ms();
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        worst = std::max(worst, ms());
    }
    return worst;
}

void Device::sync_all_streams() {
    if (streams_.empty()) {
        HIPCHK(hipStreamSynchronize((hipStream_t)stream_));
        return;
    }
    for (void* st : streams_) HIPCHK(hipStreamSynchronize((hipStream_t)st));
}

bool Device::init(int device, uint64_t arena_bytes) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) {
        error_ = "tonk_amd: no HIP device available (the Siamese engine runs only on MI355X/gfx950)";
        return false;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) { error_ = "hipGetDeviceProperties failed"; return false; }
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        error_ = std::string("tonk_amd: device is ") + prop.gcnArchName + ", kernels are built for gfx950";
        return false;
    }
    device_ = device;
    g_pin_device = device;
    // Persistent grid: exactly the workgroups that are resident at once (occupancy x CUs), so
    // every workgroup stages the GF tables once and no workgroup starts late (kernels.hip).
    int per_cu = 0;
    exec_kernel_ = slice_bytes() == TAMD_SLICE_BYTES ? (const void*)tamd_exec16 : (const void*)tamd_exec24;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, exec_kernel_, 256, 0) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    // The occupancy API ignores the SGPR limit (MI355X_MICROARCH.md, Correctness boundaries): at
    // tamd_exec16's ~106 SGPRs a SIMD holds floor(800 / 128) = 6 waves, i.e. 6 workgroups per CU.
    if (per_cu > 6) per_cu = 6;
    max_grid_ = (uint32_t)per_cu * (uint32_t)prop.multiProcessorCount;
    HIPCHK(hipSetDevice(device));
    hipStream_t s = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    stream_ = s;
    if (!reserved_bytes_) {  // (init_growable mapped the arena already)
        arena_bytes_ = (arena_bytes + 255) & ~255ull;
        HIPCHK(hipMalloc((void**)&arena_, arena_bytes_));
    }
    HIPCHK(hipMemsetAsync(arena_, 0, arena_bytes_, s));
    if (getenv("TONK_AMD_DEBUG_ALLOC"))  // (diagnostics: placement of the arena)
        fprintf(stderr, "tonk_amd: arena %p, %llu bytes\n", (void*)arena_, (unsigned long long)arena_bytes_);
    if (!gf_init()) { error_ = "gf self test failed"; return false; }
    // kernels.hip TAMD_GF_DWORDS: perm tables, inv[256], sqr[256], then the lane table: for
    // i = 0..252 (column value cx = 3 + i) the perm dwords of cx and of cx^2, then the Cauchy table
    std::vector<uint8_t> tables(sizeof(g_gf.perm) + 512 + 253 * 12 * 4 + 192 * 32);
    memcpy(tables.data(), g_gf.perm, sizeof(g_gf.perm));
    memcpy(tables.data() + sizeof(g_gf.perm), g_gf.inv, 256);
    memcpy(tables.data() + sizeof(g_gf.perm) + 256, g_gf.sqr, 256);
    for (unsigned i = 0; i < 253; ++i) {
        const uint8_t cx = (uint8_t)(3 + i);
        uint8_t* dst = tables.data() + sizeof(g_gf.perm) + 512 + i * 48;
        memcpy(dst, g_gf.perm[cx], 24);
        memcpy(dst + 24, g_gf.perm[gf_sqr(cx)], 24);
    }
    // then the Cauchy table: for x = 64..255 the perm tables of inv(x), 32 bytes each
    for (unsigned x = 64; x < 256; ++x)
        memcpy(tables.data() + sizeof(g_gf.perm) + 512 + 253 * 48 + (x - 64) * 32, g_gf.perm[gf_inv((uint8_t)x)], 32);
    HIPCHK(hipMalloc((void**)&d_zero_, 4096));  // the executor's dummy-load target (kernels.hip)
    HIPCHK(hipMemsetAsync(d_zero_, 0, 4096, s));
    HIPCHK(hipMalloc((void**)&d_gf_, tables.size()));
    HIPCHK(hipMemcpy(d_gf_, tables.data(), tables.size(), hipMemcpyHostToDevice));
    for (Slot& sl : slots_) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        sl.done = e;
    }
    if (big_cap_) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        big_.done = e;
    }
    hipEvent_t ue;
    HIPCHK(hipEventCreateWithFlags(&ue, hipEventDisableTiming));
    up_event_ = ue;
    up_cap_ = 4u << 20;
    HIPCHK(hipHostMalloc((void**)&up_host_, up_cap_, hipHostMallocDefault));
    HIPCHK(hipMalloc((void**)&up_dev_, up_cap_));
    rb_cap_ = 2u << 20;
    HIPCHK(hipHostMalloc((void**)&rb_host_, rb_cap_, hipHostMallocDefault));
    // Staging slots up front, each touched by one copy, so no step pays first-use costs.
    if (!alloc_slots(slot_bytes_)) { error_ = "program staging allocation failed"; return false; }
    for (Slot& sl : slots_) {
        memset(sl.host, 0, 4096);
        HIPCHK(hipMemcpyAsync(sl.dev, sl.host, 4096, hipMemcpyHostToDevice, s));
    }
    stats_.slot_reallocs = 0;
    HIPCHK(hipStreamSynchronize(s));
    return error_.empty();
}

bool Device::init_growable(int device, uint64_t arena_bytes, uint64_t max_bytes) {
    int vmm = 0;
    if (max_bytes <= arena_bytes ||
        hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, device) != hipSuccess || !vmm)
        return init(device, arena_bytes);
    // reserve the address range, map the first chunk, then the usual setup on top of it
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    size_t gran = 0;
    if (hipSetDevice(device) != hipSuccess ||
        hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum) != hipSuccess || !gran)
        return init(device, arena_bytes);
    granule_ = gran < (2u << 20) ? (2u << 20) : gran;
    const uint64_t maxb = (max_bytes + granule_ - 1) / granule_ * granule_;
    void* base = nullptr;
    if (hipMemAddressReserve(&base, maxb, 0, nullptr, 0) != hipSuccess || !base) return init(device, arena_bytes);
    arena_ = (uint8_t*)base;
    reserved_bytes_ = maxb;
    arena_bytes_ = 0;
    device_ = device;
    if (!grow_arena(arena_bytes)) {
        hipMemAddressFree(base, maxb);
        arena_ = nullptr;
        reserved_bytes_ = 0;
        return init(device, arena_bytes);
    }
    return init(device, 0);
}

bool Device::map_chunk(uint64_t bytes) {
    bytes = (bytes + granule_ - 1) / granule_ * granule_;
    if (arena_bytes_ + bytes > reserved_bytes_) return false;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device_ >= 0 ? device_ : 0;
    hipMemGenericAllocationHandle_t h;
    hipError_t e = hipMemCreate(&h, bytes, &prop, 0);
    if (e != hipSuccess) {
        fprintf(stderr, "tonk_amd: hipMemCreate(%llu) failed: %s\n", (unsigned long long)bytes, hipGetErrorString(e));
        return false;
    }
    e = hipMemMap(arena_ + arena_bytes_, bytes, 0, h, 0);
    if (e != hipSuccess) {
        fprintf(stderr, "tonk_amd: hipMemMap(+%llu, %llu) failed: %s\n", (unsigned long long)arena_bytes_,
                (unsigned long long)bytes, hipGetErrorString(e));
        hipMemRelease(h);
        return false;
    }
    hipMemAccessDesc ad = {};
    ad.location = prop.location;
    ad.flags = hipMemAccessFlagsProtReadWrite;
    e = hipMemSetAccess(arena_ + arena_bytes_, bytes, &ad, 1);
    if (e != hipSuccess) {
        fprintf(stderr, "tonk_amd: hipMemSetAccess failed: %s\n", hipGetErrorString(e));
        hipMemUnmap(arena_ + arena_bytes_, bytes);
        hipMemRelease(h);
        return false;
    }
    chunks_.push_back(std::make_pair((unsigned long long)h, bytes));
    arena_bytes_ += bytes;
    return true;
}

// Diagnostics (TONK_AMD_CAPI_WATCH): device operations that block for long (they run under the
// C ABI's device lock) are reported on stderr.
static void report_slow(const char* what, std::chrono::steady_clock::time_point t0, uint64_t a, uint64_t b) {
    static const bool on = getenv("TONK_AMD_CAPI_WATCH") != nullptr;
    if (!on) return;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms >= 10.0) fprintf(stderr, "tonk_amd: slow %s: %.1f ms (%llu, %llu)\n", what, ms, (unsigned long long)a, (unsigned long long)b);
}

bool Device::grow_arena(uint64_t min_bytes) {
    if (!reserved_bytes_) return min_bytes <= arena_bytes_;
    std::lock_guard<std::mutex> g(grow_mu_);
    if (arena_bytes_ >= min_bytes && min_bytes) return true;  // (another thread grew it meanwhile)
    bind_thread();
    const auto t0 = std::chrono::steady_clock::now();
    struct Report {
        std::chrono::steady_clock::time_point t0;
        const std::atomic<uint64_t>* mapped;
        ~Report() { report_slow("arena growth", t0, mapped->load() >> 20, 0); }
    } rep{t0, &arena_bytes_};
    // Physical 256 MiB chunks mapped back to back.  A growth maps at least half the size mapped so
    // far, so a window-filling Tonk server takes a handful of growths, not one per 256 MiB (the C
    // ABI starts them in the background ahead of need: SegmentPool::get).
    const uint64_t chunk = ((256ull << 20) + granule_ - 1) / granule_ * granule_;
    uint64_t target = arena_bytes_ + arena_bytes_ / 2;
    if (target < min_bytes) target = min_bytes;
    while (arena_bytes_ < target) {
        if (arena_bytes_ + chunk > reserved_bytes_) return arena_bytes_ >= min_bytes;
        if (!map_chunk(chunk)) return arena_bytes_ >= min_bytes;
    }
    return true;
}

void Device::grow_arena_async() {
    if (!reserved_bytes_ || arena_bytes_ >= reserved_bytes_ || growing_.exchange(true)) return;
    std::thread([this] {
        grow_arena(0);  // (a growth maps at least half the size mapped so far)
        growing_.store(false);
    }).detach();
}

bool Device::alloc_slots(size_t cap) {
    // parallel-assembly slots: the device half is larger than the pinned half (parts past the
    // pinned record area are staged separately, close_program)
    size_t hcap = cap, dcap = cap;
    if (asm_items_) {
        hcap = asm_items_ * 8 + asm_host_recs_ * 16;
        dcap = asm_items_ * 8 + asm_dev_recs_ * 16;
    }
    hcap = (hcap + 255) & ~(size_t)255;
    dcap = (dcap + 255) & ~(size_t)255;
    const size_t big = asm_items_ ? 0 : (big_cap_ + 255) & ~(size_t)255;  // (after the regular slots)
    if (dcap * slots_.size() + big > 0xfffff000ull) return false;  // 32-bit program offsets
    for (Slot& s : slots_) {
        s.host = nullptr;
        s.dev = nullptr;
    }
    big_.host = big_.dev = nullptr;
    if (prog_host_) hipHostFree(prog_host_);
    if (prog_dev_) hipFree(prog_dev_);
    prog_host_ = nullptr;
    prog_dev_ = nullptr;
    slot_cap_ = 0;
    // one pinned and one device allocation, split into the slots
    if (hipMalloc((void**)&prog_dev_, dcap * slots_.size() + big) != hipSuccess) return false;
    // (coherent where small programs are read by the device's threads, tamd_copy_in: a slot is
    // rewritten for later programs and no device cache may keep an older program's bytes.  Only
    // there: the batched sessions' multi-MB programs go by DMA, and their host fill into
    // coherent memory cost 2 % of the control time, 4 % of the headline)
    if (hipHostMalloc((void**)&prog_host_, hcap * slots_.size() + big,
                      small_uploads_ ? hipHostMallocMapped | hipHostMallocCoherent : hipHostMallocDefault) != hipSuccess)
        return false;
    for (size_t k = 0; k < slots_.size(); ++k) {
        Slot& s = slots_[k];
        s.host = prog_host_ + k * hcap;
        s.dev_off = (uint32_t)(k * dcap);
        s.dev = prog_dev_ + s.dev_off;
    }
    if (big) {
        big_.host = prog_host_ + slots_.size() * hcap;
        big_.dev_off = (uint32_t)(slots_.size() * dcap);
        big_.dev = prog_dev_ + big_.dev_off;
    }
    slot_cap_ = hcap;
    return true;
}

void Device::set_assembly_slots(size_t count, size_t host_mb) {
    slots_.assign(count < 2 ? 2 : count, Slot());
    asm_items_ = 1u << 20;                  // 8 MB of work items per program
    asm_host_recs_ = (host_mb << 20) / 16;  // pinned record area
    asm_dev_recs_ = 4 * asm_host_recs_;
    slot_bytes_ = 0;
}

bool Device::assembly_fits(size_t recs, size_t items) const {
    return recs + 64 <= asm_dev_recs_ && items <= asm_items_;
}

bool Device::ensure_assembly(size_t recs, size_t items) {
    if (assembly_fits(recs, items)) return true;
    stats_.slot_reallocs++;
    const auto t0 = std::chrono::steady_clock::now();
    drain_programs();
    sync_all_streams();  // a program on any stream may still read its slot
    for (Slot& sl : slots_) sl.ticket = 0;
    if (items > asm_items_) asm_items_ = items + items / 4;
    if (recs + 64 > asm_dev_recs_) asm_dev_recs_ = (recs + 64) + (recs + 64) / 4;
    // (every slot lies within 4 GB of the program base: 32-bit offsets; a bound above that is
    // clamped -- the callers' bounds are generous, and a real overflow still fails loudly)
    const size_t per_slot = (0xfffff000ull / slots_.size()) & ~(size_t)255;
    const size_t max_recs = per_slot > asm_items_ * 8 + 4096 ? (per_slot - asm_items_ * 8 - 4096) / 16 : 0;
    if (asm_dev_recs_ > max_recs) asm_dev_recs_ = max_recs;
    const bool ok = alloc_slots(0);
    if (!ok) {
        error_ = "program staging allocation failed (assembly slots)";
        failed_ = true;
    }
    report_slow("assembly slot growth", t0, asm_dev_recs_ >> 6, recs >> 6);
    return ok;
}

int Device::open_program() {
    const int h = next_slot_;
    Slot& slot = slots_[h];
    next_slot_ = (next_slot_ + 1) % (int)slots_.size();
    for (const Inflight& p : progs_)
        if (p.slot == &slot) { drain_programs(); break; }  // (the slot still holds a program in flight)
    if (slot.ticket) {
        const auto w0 = std::chrono::steady_clock::now();
        HIPCHK(hipEventSynchronize((hipEvent_t)slot.done));
        stats_.slot_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
        if (streams_.empty() && slot.ticket > completed_) completed_ = slot.ticket;
        slot.ticket = 0;
    }
    slot.bump.store(0, std::memory_order_relaxed);
    slot.failed = false;
    return h;
}

bool Device::add_part(int h, const ProgramBuilder& pb, Part& out) {
    Slot& slot = slots_[h];
    const InstrVec& ins = pb.instrs();
    const std::vector<tamd_op>& ops = pb.ops();
    const std::vector<uint32_t>& lv = pb.op_levels();
    const std::vector<uint32_t>& li = pb.level_items();
    const uint32_t ni = (uint32_t)ins.size(), no = (uint32_t)ops.size();
    out.n_instr = ni;
    out.n_ops = no;
    out.acc_bytes = pb.acc_bytes();
    out.store_bytes = pb.store_bytes();
    out.bucket_start.assign(li.size() + 1, 0);
    for (size_t b = 0; b < li.size(); ++b) out.bucket_start[b + 1] = out.bucket_start[b] + li[b];
    out.items.resize(out.bucket_start.back());
    if (!no) return true;
    // the executor reads up to a batch past an op's last instruction: every part's instructions
    // are followed by its ops, and the record area keeps 64 records of slack at its end
    const uint32_t recs = ni + no;
    const uint32_t base = slot.bump.fetch_add(recs, std::memory_order_relaxed);
    if ((size_t)base + recs + 64 > asm_dev_recs_) {
        slot.failed = true;
        return false;
    }
    std::vector<uint8_t> spill;
    tamd_instr* dst;
    if ((size_t)base + recs <= asm_host_recs_) {
        dst = (tamd_instr*)(slot.host + asm_items_ * 8) + base;
    } else {
        spill.resize((size_t)recs * 16);
        dst = (tamd_instr*)spill.data();
    }
    memcpy(dst, ins.data(), (size_t)ni * sizeof(tamd_instr));
    tamd_op* od = (tamd_op*)(dst + ni);
    uint32_t cur_small[64];
    std::vector<uint32_t> cur_big;
    uint32_t* cur = cur_small;
    if (li.size() > 64) {
        cur_big.assign(out.bucket_start.begin(), out.bucket_start.end() - 1);
        cur = cur_big.data();
    } else {
        for (size_t b = 0; b < li.size(); ++b) cur[b] = out.bucket_start[b];
    }
    uint64_t* it = out.items.data();
    for (uint32_t i = 0; i < no; ++i) {
        tamd_op op = ops[i];
        op.first += base;
        od[i] = op;
        const uint64_t rec = base + ni + i;
        const uint32_t slices = op_slices(op.span);
        uint32_t& c = cur[lv[i]];
        for (uint32_t k = 0; k < slices; ++k) it[c++] = rec | ((uint64_t)k << 32);
    }
    if (!spill.empty()) {
        std::lock_guard<std::mutex> g(spill_mu_);
        spills_.push_back(Spill{base, std::move(spill)});
        spill_slot_.push_back(h);
    }
    return true;
}

uint64_t Device::close_program(int h, Part* const* parts, size_t n) {
    flush_uploads();
    Slot& slot = slots_[h];
    if (slot.failed) {
        error_ = "a program exceeds its staging slot";
        failed_ = true;
    }
    uint32_t B = 0;
    size_t n_instr = 0, n_ops = 0;
    std::vector<VerifyDesc> ver;
    for (size_t i = 0; i < n; ++i) {
        const Part& p = *parts[i];
        if (p.bucket_start.size() > B + 1) B = (uint32_t)p.bucket_start.size() - 1;
        n_instr += p.n_instr;
        n_ops += p.n_ops;
        stats_.acc_bytes += p.acc_bytes;
        stats_.store_bytes += p.store_bytes;
        ver.insert(ver.end(), p.verify.begin(), p.verify.end());
    }
    if (!ver.empty()) verify_next(ver);
    B = (B + TAMD_COST_CLASSES - 1) / TAMD_COST_CLASSES * TAMD_COST_CLASSES;
    const uint32_t L = B / TAMD_COST_CLASSES;
    Inflight cur;
    cur.levels = L;
    cur.level_items.assign(L, 0);
    cur.level_coop.assign(L, 0);
    cur.class_items.assign(B, 0);
    cur.item_base.assign(L + 1, 0);
    // Items of a level: cost class by cost class.  Inside a class, part i (one context: a stream)
    // has XCD affinity i mod 8: its items go to positions p with p mod 8 == i mod 8 as far as the
    // counts allow, and the executor runs position p of a class block on a workgroup of XCD p mod 8
    // (exec_level), so one stream's ops -- which read the same packets -- share that XCD's L2.
    // (TONK_AMD_XCD_AFFINITY=0: parts in order, A/B.)
    static const bool affinity = !getenv("TONK_AMD_XCD_AFFINITY") || atoi(getenv("TONK_AMD_XCD_AFFINITY")) != 0;
    uint64_t* items = (uint64_t*)slot.host;
    size_t at = 0;
    for (uint32_t b = 0; b < B && !failed_; ++b) {
        const uint32_t l = b / TAMD_COST_CLASSES;
        if (b % TAMD_COST_CLASSES == 0) cur.item_base[l] = (uint32_t)at;
        size_t total = 0;
        for (size_t i = 0; i < n; ++i) {
            const Part& p = *parts[i];
            if (b + 1 < p.bucket_start.size()) total += p.bucket_start[b + 1] - p.bucket_start[b];
        }
        if (!total) continue;
        if (at + total > asm_items_) {
            error_ = "a program exceeds its work-item area";
            failed_ = true;
            break;
        }
        if (!affinity || n < 2) {
            for (size_t i = 0; i < n; ++i) {
                const Part& p = *parts[i];
                if (b + 1 >= p.bucket_start.size()) continue;
                const uint32_t c = p.bucket_start[b + 1] - p.bucket_start[b];
                memcpy(items + at, p.items.data() + p.bucket_start[b], (size_t)c * 8);
                at += c;
            }
        } else {
            // per residue r: a cursor over the items of parts r, r + 8, ... (part, next item)
            size_t part_of[8], next[8], left[8];
            for (uint32_t r = 0; r < 8; ++r) {
                part_of[r] = r;
                next[r] = 0;
                left[r] = 0;
                for (size_t i = r; i < n; i += 8) {
                    const Part& p = *parts[i];
                    if (b + 1 < p.bucket_start.size()) left[r] += p.bucket_start[b + 1] - p.bucket_start[b];
                }
            }
            auto take = [&](uint32_t r) -> uint64_t {
                for (;;) {
                    const Part& p = *parts[part_of[r]];
                    const uint32_t c = b + 1 < p.bucket_start.size() ? p.bucket_start[b + 1] - p.bucket_start[b] : 0u;
                    if (next[r] < c) {
                        --left[r];
                        return p.items[p.bucket_start[b] + next[r]++];
                    }
                    part_of[r] += 8;
                    next[r] = 0;
                }
            };
            for (size_t j = 0; j < total; ++j) {
                uint32_t r = (uint32_t)(j & 7u);
                if (!left[r]) {  // this residue's parts are done: the residue with most left
                    for (uint32_t q = 0; q < 8; ++q)
                        if (left[q] > left[r]) r = q;
                }
                items[at + j] = take(r);
            }
            at += total;
        }
        cur.level_items[l] += (uint32_t)total;
        cur.class_items[b] += (uint32_t)total;
        if (b % TAMD_COST_CLASSES == 0) cur.level_coop[l] += (uint32_t)total;
    }
    cur.item_base[L] = (uint32_t)at;
    if (at == 0 || failed_) {  // nothing to run: complete once everything before it is done
        const uint64_t ticket = ++ticket_;
        drain_programs();
        ticket_is_empty_ = true;
        mark(ticket);
        ticket_is_empty_ = false;
        if (pending_verify_ >= 0) run_verify(pending_verify_);
        pending_verify_ = -1;
        return ticket;
    }
    hipStream_t st = (hipStream_t)stream_;
    const size_t ibytes = asm_items_ * 8;
    const uint32_t recs = slot.bump.load(std::memory_order_relaxed);
    const size_t hrecs = recs < asm_host_recs_ ? recs : asm_host_recs_;
    const auto u0 = std::chrono::steady_clock::now();
    upload2(small_uploads_, slot.dev, slot.host, at * 8, slot.dev + ibytes, slot.host + ibytes, hrecs * 16, st);
    HIPCHK(hipGetLastError());
    {
        std::lock_guard<std::mutex> g(spill_mu_);
        size_t keep = 0;
        for (size_t i = 0; i < spills_.size(); ++i) {
            if (spill_slot_[i] != h) {
                spills_[keep] = std::move(spills_[i]);
                spill_slot_[keep++] = spill_slot_[i];
                continue;
            }
            // (rare: a program larger than the pinned area; a synchronous copy of the spilled part)
            HIPCHK(hipStreamSynchronize(st));
            HIPCHK(hipMemcpy(slot.dev + ibytes + (size_t)spills_[i].rec * 16, spills_[i].bytes.data(),
                             spills_[i].bytes.size(), hipMemcpyHostToDevice));
        }
        spills_.resize(keep);
        spill_slot_.resize(keep);
    }
    const double up_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - u0).count();
    stats_.upload_enqueue_ms += up_ms;
    if (up_ms > stats_.upload_enqueue_max_ms) stats_.upload_enqueue_max_ms = up_ms;
    cur.instrs = cur.ops = slot.dev_off + (uint32_t)ibytes;
    cur.items = slot.dev_off;
    cur.slot = &slot;
    return start_program(cur, n_instr, n_ops, at, at * 8 + (size_t)recs * 16);
}

bool Device::ensure_slot(Slot& s, size_t bytes) {
    const bool big = &s == &big_;
    if ((big ? big_cap_ : slot_cap_) >= bytes) return true;
    stats_.slot_reallocs++;
    // a bench step's program is ~8 MB: avoid reallocating mid-run
    size_t cap = slot_cap_ ? slot_cap_ : slot_bytes_;
    if (big) {
        while (big_cap_ < bytes) big_cap_ *= 2;
    } else {
        while (cap < bytes) cap *= 2;
    }
    const auto t0 = std::chrono::steady_clock::now();
    drain_programs();
    sync_all_streams();  // a program on any stream may still read its slot
    for (Slot& sl : slots_) sl.ticket = 0;
    big_.ticket = 0;
    const bool ok = alloc_slots(cap);
    report_slow(big ? "oversize slot growth" : "program slot growth", t0, (big ? big_cap_ : cap) >> 10, bytes >> 10);
    return ok;
}

uint64_t Device::run(Context* const* ctxs, size_t n) {
    begin(ctxs, n);
    for (size_t i = 0; i < n; ++i) fill(i);
    return launch();
}

void Device::begin(Context* const* ctxs, size_t n, bool closed) {
    Plan& P = plan_;
    P.pbs.resize(n);
    for (size_t c = 0; c < n; ++c) P.pbs[c] = closed ? &ctxs[c]->closed : &ctxs[c]->pb;
    P.levels = 0;
    P.n_instr = P.n_ops = P.n_items = 0;
    uint32_t B = 0;  // buckets: TAMD_COST_CLASSES per level (expensive ops first), see ProgramBuilder::op_levels
    for (size_t c = 0; c < n; ++c) {
        const ProgramBuilder& pb = *P.pbs[c];
        P.n_instr += pb.instrs().size();
        P.n_ops += pb.ops().size();
        stats_.acc_bytes += pb.acc_bytes();
        stats_.store_bytes += pb.store_bytes();
        if (pb.level_ops().size() > B) B = (uint32_t)pb.level_ops().size();
    }
    B = (B + TAMD_COST_CLASSES - 1) / TAMD_COST_CLASSES * TAMD_COST_CLASSES;
    P.levels = B / TAMD_COST_CLASSES;
    P.buckets = B;
    P.empty = P.n_ops == 0;
    if (P.empty) return;
    const uint32_t L = P.levels;
    // Ops grouped by bucket (level, then long before short); inside a bucket, by context.
    P.op_start.assign(n * B, 0);
    P.item_start.assign(n * B, 0);
    P.level_items.assign(L, 0);
    P.level_coop.assign(L, 0);
    P.class_items.assign(B, 0);
    P.item_base.assign(L + 1, 0);
    P.instr_base.assign(n, 0);
    uint32_t op_at = 0, item_at = 0, instr_at = 0;
    for (uint32_t b = 0; b < B; ++b) {
        if (b % TAMD_COST_CLASSES == 0) P.item_base[b / TAMD_COST_CLASSES] = item_at;
        for (size_t c = 0; c < n; ++c) {
            const ProgramBuilder& pb = *P.pbs[c];
            P.op_start[c * B + b] = op_at;
            P.item_start[c * B + b] = item_at;
            if (b < pb.level_ops().size()) {
                op_at += pb.level_ops()[b];
                item_at += pb.level_items()[b];
                P.level_items[b / TAMD_COST_CLASSES] += pb.level_items()[b];
                P.class_items[b] += pb.level_items()[b];
                if (b % TAMD_COST_CLASSES == 0) P.level_coop[b / TAMD_COST_CLASSES] += pb.level_items()[b];
            }
        }
    }
    P.item_base[L] = item_at;
    for (size_t c = 0; c < n; ++c) {
        P.instr_base[c] = instr_at;
        instr_at += (uint32_t)P.pbs[c]->instrs().size();
    }
    P.n_items = item_at;
    // the executor reads a 64-instruction window without bounds checks: pad the region
    P.bytes_instr = (P.n_instr + 64) * sizeof(tamd_instr);
    P.bytes_ops = P.n_ops * sizeof(tamd_op);
    P.total = P.bytes_instr + P.bytes_ops + P.n_items * sizeof(uint32_t) * 2;

    // (a program larger than a regular slot takes the oversize slot when there is one)
    const bool big = big_.dev && P.total > slot_capacity();
    Slot& slot = big ? big_ : slots_[next_slot_];
    if (!big) next_slot_ = (next_slot_ + 1) % (int)slots_.size();
    for (const Inflight& p : progs_)
        if (p.slot == &slot) { drain_programs(); break; }  // (the slot still holds a program in flight)
    if (slot.ticket) {
        const auto w0 = std::chrono::steady_clock::now();
        HIPCHK(hipEventSynchronize((hipEvent_t)slot.done));
        stats_.slot_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
        report_slow("program slot wait", w0, 0, 0);
        // (ticket order is completion order only on a single stream)
        if (streams_.empty() && slot.ticket > completed_) completed_ = slot.ticket;
        slot.ticket = 0;
    }
    P.slot = &slot;
    // Test hook: TONK_AMD_FAIL_AFTER_PROGRAMS=<n> makes every program after the n-th fail as a
    // staging allocation failure would (the C ABI must then report Siamese_Disabled).
    static const long long fail_after = getenv("TONK_AMD_FAIL_AFTER_PROGRAMS") ? atoll(getenv("TONK_AMD_FAIL_AFTER_PROGRAMS")) : -1;
    if (!ensure_slot(slot, P.total) || (fail_after >= 0 && (long long)stats_.programs >= fail_after)) {
        error_ = "program staging allocation failed";
        failed_ = true;
        P.empty = true;
    }
}

void Device::fill(size_t c) {
    Plan& P = plan_;
    if (P.empty) return;
    const ProgramBuilder& pb = *P.pbs[c];
    const uint32_t L = P.buckets;
    tamd_instr* hi = (tamd_instr*)P.slot->host;
    tamd_op* ho = (tamd_op*)(P.slot->host + P.bytes_instr);
    uint32_t* hitems = (uint32_t*)(P.slot->host + P.bytes_instr + P.bytes_ops);
    const uint32_t ibase = P.instr_base[c];
    memcpy(hi + ibase, pb.instrs().data(), pb.instrs().size() * sizeof(tamd_instr));
    uint32_t op_fill[64], item_fill[64];
    std::vector<uint32_t> big_op, big_item;
    uint32_t* of = op_fill;
    uint32_t* itf = item_fill;
    if (L > 64) {
        big_op.resize(L);
        big_item.resize(L);
        of = big_op.data();
        itf = big_item.data();
    }
    for (uint32_t l = 0; l < L; ++l) {
        of[l] = P.op_start[c * L + l];
        itf[l] = P.item_start[c * L + l];
    }
    const std::vector<tamd_op>& ops = pb.ops();
    const std::vector<uint32_t>& lv = pb.op_levels();
    for (size_t i = 0; i < ops.size(); ++i) {
        const uint32_t l = lv[i];
        tamd_op op = ops[i];
        op.first += ibase;
        const uint32_t oi = of[l]++;
        ho[oi] = op;
        const uint32_t slices = op_slices(op.span);
        uint32_t ii = itf[l];
        itf[l] += slices;
        for (uint32_t s = 0; s < slices; ++s, ++ii) {
            hitems[2 * ii] = oi;
            hitems[2 * ii + 1] = s;
        }
    }
}

// One executor launch: the next level of every program with levels left (oldest first), then
// level 1 of `fresh` (the program being launched) if given.
void Device::launch_step(Inflight* fresh, unsigned long long* stamps) {
    tamd_segments sg;
    memset(&sg, 0, sizeof(sg));
    uint32_t cnt = 0, coop = 0;
    uint32_t seg_level[TAMD_MAX_SEGMENTS], seg_coop[TAMD_MAX_SEGMENTS];
    auto add = [&](Inflight& p) {
        if (p.done()) return;
        const uint32_t l = p.next++;
        const uint32_t c = p.level_items[l];
        if (!c) return;
        seg_level[sg.n] = l;
        seg_coop[sg.n] = p.level_coop[l];
        tamd_segment& g = sg.s[sg.n++];
        g.ops = p.ops;
        g.instrs = p.instrs;
        g.items = p.items + 8u * p.item_base[l];
        g.count = c;
        for (uint32_t k = 0; k < TAMD_COST_CLASSES; ++k) g.cls[k] = p.class_items[TAMD_COST_CLASSES * l + k];
        cnt += c;
    };
    for (Inflight& p : progs_) add(p);
    if (fresh) add(*fresh);
    if (!cnt) return;
    // Segment order = the order waves claim items in (A/B, TONK_AMD_SEG_ORDER): 0 programs
    // oldest first (deepest level first, the new program's level 1 last); 1 level 2, level 1,
    // then the rest; 2 level 1, level 2, then the rest; 3 the rest, then level 1, then level 2.
    static const int seg_order = getenv("TONK_AMD_SEG_ORDER") ? atoi(getenv("TONK_AMD_SEG_ORDER")) : 0;
    if (seg_order && sg.n > 1) {
        static const uint32_t rank_of[4][3] = {{0, 0, 0}, {1, 0, 2}, {0, 1, 2}, {1, 2, 0}};  // [order][L1, L2, rest]
        tamd_segment tmp[TAMD_MAX_SEGMENTS];
        uint32_t tl[TAMD_MAX_SEGMENTS], tc[TAMD_MAX_SEGMENTS], m = 0;
        for (uint32_t pass = 0; pass < 3; ++pass)
            for (uint32_t k = 0; k < sg.n; ++k) {
                const uint32_t cls = seg_level[k] == 1 ? 0u : seg_level[k] == 2 ? 1u : 2u;
                if (rank_of[seg_order & 3][cls] != pass) continue;
                tmp[m] = sg.s[k];
                tl[m] = seg_level[k];
                tc[m] = seg_coop[k];
                ++m;
            }
        for (uint32_t k = 0; k < sg.n; ++k) {
            sg.s[k] = tmp[k];
            seg_level[k] = tl[k];
            seg_coop[k] = tc[k];
        }
    }
    coop = seg_coop[0];
    // Items class by class across the segments: the launch's long items (every level's class 0)
    // are taken first (TONK_AMD_CLASS_MAJOR=0: segment by segment, A/B)
    static const bool class_major = !getenv("TONK_AMD_CLASS_MAJOR") || atoi(getenv("TONK_AMD_CLASS_MAJOR")) != 0;
    sg.flags = class_major ? 1u : 0u;
    hipStream_t st = (hipStream_t)stream_;
    // Class-0 ops are shared by a workgroup only in launches too small to fill the chip twice
    // over with single-wave items; in the big ones they run as ordinary (first) items.  Only the
    // first segment's class-0 items (they lead it) can be shared.  A shared item gets a
    // workgroup of its own, the single-wave items four to a workgroup beside them.
    static const int share_mode = getenv("TONK_AMD_SHARE") ? atoi(getenv("TONK_AMD_SHARE")) : 0;  // A/B (profiling)
    const uint32_t shared = (share_mode == 1 || (share_mode == 0 && cnt < 2u * 4u * max_grid_)) ? coop : 0u;
    uint32_t grid = shared + (cnt - shared + 3) / 4;
    if (grid > max_grid_) grid = max_grid_;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (timing_) {
        e0 = (hipEvent_t)timing_event();
        e1 = (hipEvent_t)timing_event();
    }
    const ExecFn fn = (ExecFn)exec_kernel_;
    // Profiling only: TONK_AMD_LAUNCH_STAMPS=<launch number> records per-item stamps of every
    // segment of that launch (a pipelined one) into tonk_amd_launch_stamps.txt.
    static const char* lstamp_env = getenv("TONK_AMD_LAUNCH_STAMPS");
    unsigned long long* lstamps = nullptr;
    if (lstamp_env && !stamps && (uint64_t)atoll(lstamp_env) == stats_.launches) {
        if (hipMalloc((void**)&lstamps, (size_t)cnt * 24) == hipSuccess) {
            hipMemsetAsync(lstamps, 0, (size_t)cnt * 24, st);
            stamps = lstamps;
        }
    }
    // Timed: the events carry the dispatch's own start and end (hipExtLaunchKernelGGL), as a
    // kernel trace does; events recorded around the launch would add the dispatch latency.
    if (timing_)
        HIPT(hipExtLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, st, e0, e1, 0, sg, (const uint8_t*)prog_dev_, shared,
                              arena_, d_gf_, d_zero_, stamps));
    else
        HIPT(hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, st, sg, (const uint8_t*)prog_dev_, shared, arena_, d_gf_,
                           d_zero_, stamps));
    if (timing_) {
        timing_events_.push_back(std::make_pair((void*)e0, (void*)e1));
    }
    if (lstamps) {
        std::vector<unsigned long long> h((size_t)cnt * 3);
        hipMemcpyAsync(h.data(), lstamps, h.size() * 8, hipMemcpyDeviceToHost, st);
        hipStreamSynchronize(st);
        hipFree(lstamps);
        if (FILE* f = fopen("tonk_amd_launch_stamps.txt", "w")) {
            fprintf(f, "# seg level class t0 t1 block_wave (100 MHz ticks); shared items %u, grid %u\n", shared, grid);
            size_t at = 0;
            for (uint32_t k = 0; k < sg.n; ++k) {
                uint32_t c = 0, left = sg.s[k].cls[0];
                for (uint32_t i = 0; i < sg.s[k].count; ++i, ++at) {
                    while (!left && c + 1 < TAMD_COST_CLASSES) left = sg.s[k].cls[++c];
                    if (left) --left;
                    fprintf(f, "%u %u %u %llu %llu %llu\n", k, seg_level[k], c, h[3 * at], h[3 * at + 1], h[3 * at + 2]);
                }
            }
            fclose(f);
        }
    }
    stats_.launches++;
}

void Device::set_timing(bool on) {
    if (on == timing_) return;
    if (stream_) hipLaunchKernelGGL(tamd_timed_region, dim3(1), dim3(64), 0, (hipStream_t)stream_);
    timing_ = on;
}

// Complete the oldest programs whose levels have all been launched (in ticket order).
void Device::retire_done() {
    while (!progs_.empty() && progs_.front().done()) {
        Inflight& p = progs_.front();
        HIPCHK(hipEventRecord((hipEvent_t)p.slot->done, (hipStream_t)stream_));
        p.slot->ticket = p.ticket;
        mark(p.ticket);
        if (p.verify >= 0) run_verify(p.verify);
        progs_.pop_front();
    }
}

void Device::drain_programs() {
    while (!progs_.empty()) {
        launch_step(nullptr, nullptr);
        retire_done();
    }
    HIPCHK(hipGetLastError());
}

uint64_t Device::launch() {
    flush_uploads();  // staged packets land before the program reads them
    Plan& P = plan_;
    if (P.empty) {
        const uint64_t ticket = ++ticket_;
        drain_programs();
        ticket_is_empty_ = true;
        mark(ticket);  // done once everything enqueued before it is done
        ticket_is_empty_ = false;
        if (pending_verify_ >= 0) run_verify(pending_verify_);
        pending_verify_ = -1;
        return ticket;
    }
    hipStream_t st = (hipStream_t)stream_;
    Slot& slot = *P.slot;
    const auto u0 = std::chrono::steady_clock::now();
    upload2(small_uploads_, slot.dev, slot.host, P.total, nullptr, nullptr, 0, st);
    HIPCHK(hipGetLastError());
    const double up_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - u0).count();
    stats_.upload_enqueue_ms += up_ms;
    if (up_ms > 1.0 && getenv("TONK_AMD_TRACE_UPLOADS"))
        fprintf(stderr, "tonk_amd: program %llu: H2D enqueue of %zu bytes took %.3f ms\n",
                (unsigned long long)(ticket_ + 1), P.total, up_ms);
    if (up_ms > stats_.upload_enqueue_max_ms) stats_.upload_enqueue_max_ms = up_ms;
    Inflight cur;
    cur.instrs = slot.dev_off;
    cur.ops = slot.dev_off + (uint32_t)P.bytes_instr;
    cur.items = slot.dev_off + (uint32_t)(P.bytes_instr + P.bytes_ops);
    cur.levels = P.levels;
    cur.level_items = P.level_items;
    cur.item_base = P.item_base;
    cur.level_coop = P.level_coop;
    cur.class_items = P.class_items;
    cur.slot = &slot;
    return start_program(cur, P.n_instr, P.n_ops, P.n_items, P.total);
}

// Enqueue a program whose memory is uploaded (launch, close_program): its first level now (with
// the next level of every program in flight) when pipelined, all of its levels otherwise.
uint64_t Device::start_program(Inflight& cur, size_t n_instr, size_t n_ops, size_t n_items, size_t bytes) {
    hipStream_t st = (hipStream_t)stream_;
    Slot& slot = *cur.slot;
    const uint64_t ticket = ++ticket_;
    cur.ticket = ticket;
    cur.verify = pending_verify_;
    pending_verify_ = -1;
    // Profiling only: TONK_AMD_STAMPS=<program number> records per-item start/end stamps of that
    // program's launches and writes them to tonk_amd_stamps.bin (u64 triples per item; levels
    // delimited by the item bases printed to stderr).  A stamped program runs alone.
    unsigned long long* stamps = nullptr;
    static const char* stamp_env = getenv("TONK_AMD_STAMPS");
    const bool stamp_this = stamp_env && (uint64_t)atoll(stamp_env) == stats_.programs;
    const bool pipe = pipelined_ && !stamp_this;
    if (!pipe) drain_programs();
    if (stamp_this) HIPCHK(hipMalloc((void**)&stamps, n_items * 24 + 24));
    // a launch holds at most TAMD_MAX_SEGMENTS levels: the oldest programs finish first if needed
    while (progs_.size() + 1 > TAMD_MAX_SEGMENTS) {
        launch_step(nullptr, nullptr);
        retire_done();
    }
    if (pipe) {
        // Pipelined: this program's level 1 beside the next level of every program in flight;
        // its level d runs d - 1 launches later (Context::kPipeDepth, inherited levels).
        launch_step(&cur, nullptr);
        progs_.push_back(cur);
        retire_done();
    } else {
        for (uint32_t l = 1; l < cur.levels; ++l) {
            progs_.push_back(cur);  // (a single-program launch per level)
            progs_.back().next = l;
            progs_.back().levels = l + 1;
            launch_step(nullptr, stamps ? stamps + 3 * cur.item_base[l] : nullptr);
            progs_.pop_back();
        }
        HIPCHK(hipEventRecord((hipEvent_t)slot.done, st));
        slot.ticket = ticket;
        mark(ticket);
        if (cur.verify >= 0) run_verify(cur.verify);
    }
    HIPCHK(hipGetLastError());
    if (stamp_this) {
        std::vector<unsigned long long> h(n_items * 3);
        HIPCHK(hipMemcpyAsync(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        hipFree(stamps);
        // items (op record, slice), the table item.x indexes (op records) and the one op.first
        // indexes (instructions); with parallel assembly both are the slot's record area
        const size_t io = cur.instrs - slot.dev_off, oo = cur.ops - slot.dev_off, it = cur.items - slot.dev_off;
        const bool merged = io == oo;
        const size_t rec_bytes = merged ? bytes - n_items * 8 : 0;
        auto dump = [](const char* name, const void* p, size_t n) {
            FILE* f = fopen(name, "wb");
            if (f) {
                fwrite(p, 1, n, f);
                fclose(f);
            }
        };
        dump("tonk_amd_stamps.bin", h.data(), h.size() * 8);
        dump("tonk_amd_items.bin", slot.host + it, n_items * 8);
        dump("tonk_amd_ops.bin", slot.host + oo, merged ? rec_bytes : n_ops * 16);
        dump("tonk_amd_instrs.bin", slot.host + io, merged ? rec_bytes : n_instr * 16);
        fprintf(stderr, "stamps: n_instr %zu n_ops %zu n_items %zu\n", n_instr, n_ops, n_items);
        for (uint32_t k = 0; k <= cur.levels; ++k) fprintf(stderr, "stamps level %u item_base %u\n", k, cur.item_base[k]);
    }
    stats_.programs++;
    stats_.ops += n_ops;
    stats_.items += n_items;
    stats_.instrs += n_instr;
    stats_.upload_bytes += bytes;
    return ticket;
}

void Device::mark(uint64_t ticket) {
    if (inflight_.empty() && ticket_is_empty_) {
        completed_ = ticket;
        return;
    }
    void* e = nullptr;
    if (!free_events_.empty()) {
        e = free_events_.back();
        free_events_.pop_back();
    } else {
        hipEvent_t he;
        HIPCHK(hipEventCreateWithFlags(&he, hipEventDisableTiming));
        e = he;
    }
    HIPCHK(hipEventRecord((hipEvent_t)e, (hipStream_t)stream_));
    inflight_.push_back(std::make_pair(ticket, e));
    // Callers that wait on their own events (the C ABI) never poll completed(): retire finished
    // entries here so the list (and the events it holds) stays short.
    while (inflight_.size() > 64 && hipEventQuery((hipEvent_t)inflight_.front().second) == hipSuccess) {
        if (streams_.empty() && inflight_.front().first > completed_) completed_ = inflight_.front().first;
        free_events_.push_back(inflight_.front().second);
        inflight_.pop_front();
    }
}

bool Device::completed(uint64_t ticket) {
    while (!inflight_.empty() && ticket > completed_) {
        if (hipEventQuery((hipEvent_t)inflight_.front().second) != hipSuccess) break;
        if (inflight_.front().first > completed_) completed_ = inflight_.front().first;
        free_events_.push_back(inflight_.front().second);
        inflight_.pop_front();
    }
    return ticket <= completed_;
}

void Device::wait(uint64_t ticket) {
    if (!progs_.empty() && ticket >= progs_.front().ticket) drain_programs();
    while (!inflight_.empty() && ticket > completed_) {
        HIPCHK(hipEventSynchronize((hipEvent_t)inflight_.front().second));
        if (inflight_.front().first > completed_) completed_ = inflight_.front().first;
        free_events_.push_back(inflight_.front().second);
        inflight_.pop_front();
    }
}

void Device::synchronize() {
    drain_programs();
    flush_uploads();
    sync_all_streams();
    for (auto& p : inflight_) free_events_.push_back(p.second);
    inflight_.clear();
    completed_ = ticket_;
    up_used_ = up_flushed_ = 0;
    for (const Readback& r : rb_pending_) memcpy(r.dst, rb_host_ + r.off, r.n);
    rb_pending_.clear();
    rb_used_ = 0;
}

void Device::upload(uint64_t off, const void* src, size_t n) {
    if (n == 0) return;
    hipStream_t st = (hipStream_t)stream_;
    const size_t desc_room = (up_pending_.size() + 1) * sizeof(ScatterDesc);
    if (n + 16 + desc_room > up_cap_ / 2 || off % TAMD_ROW_UNIT != 0 || off / TAMD_ROW_UNIT > 0xffffffffull) {
        synchronize();
        HIPCHK(hipMemcpyAsync(arena_ + off, src, n, hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
        return;
    }
    // packets and (at flush) their descriptors share the staging buffer
    if (up_used_ + n + 16 + desc_room > up_cap_) synchronize();
    memcpy(up_host_ + up_used_, src, n);
    ScatterDesc d;
    d.row = (uint32_t)(off / TAMD_ROW_UNIT);
    d.len = (uint32_t)n;
    d.src = (uint32_t)up_used_;
    d.pad = 0;
    up_pending_.push_back(d);
    up_used_ += (n + 15) & ~(size_t)15;
}

void Device::flush_uploads() {
    if (up_pending_.empty()) return;
    hipStream_t st = (hipStream_t)stream_;
    const uint32_t cnt = (uint32_t)up_pending_.size();
    const size_t dbytes = cnt * sizeof(ScatterDesc);
    memcpy(up_host_ + up_used_, up_pending_.data(), dbytes);
    const size_t begin = up_flushed_;
    const size_t end = up_used_ + dbytes;
    HIPCHK(hipMemcpyAsync(up_dev_ + begin, up_host_ + begin, end - begin, hipMemcpyHostToDevice, st));
    // descriptor sources are offsets into up_dev_ (the same offsets as in up_host_)
    HIPT(hipLaunchKernelGGL(tamd_scatter_rows, dim3(cnt), dim3(64), 0, st, (const ScatterDescDev*)(up_dev_ + up_used_), cnt,
                       (const uint8_t*)up_dev_, arena_));
    HIPCHK(hipGetLastError());
    up_used_ = (end + 15) & ~(size_t)15;
    up_flushed_ = up_used_;
    up_pending_.clear();
}

void Device::scatter_upload(uint8_t* src, size_t bytes, const ScatterIn* d, uint32_t n) {
    if (!n) return;
    flush_uploads();  // (stream order of the shared staging buffer)
    hipStream_t st = (hipStream_t)stream_;
    const size_t at = (bytes + 15) & ~(size_t)15;
    ScatterDesc* sd = (ScatterDesc*)(src + at);
    for (uint32_t k = 0; k < n; ++k) {
        sd[k].row = d[k].row;
        sd[k].len = d[k].len;
        sd[k].src = d[k].src;
        sd[k].pad = 0;
    }
    const size_t total = at + (size_t)n * sizeof(ScatterDesc);
    // each stream has its own landing area (reused batch after batch in that stream's order)
    if (!sc_per_stream_.empty()) {
        sc_dev_ = sc_per_stream_[cur_stream_].first;
        sc_cap_ = sc_per_stream_[cur_stream_].second;
    }
    if (total > sc_cap_) {  // the device landing area grows (after the stream drains)
        HIPCHK(hipStreamSynchronize(st));
        if (sc_dev_) hipFree(sc_dev_);
        sc_cap_ = total + total / 2;
        HIPCHK(hipMalloc((void**)&sc_dev_, sc_cap_));
        if (!sc_per_stream_.empty()) sc_per_stream_[cur_stream_] = std::make_pair(sc_dev_, sc_cap_);
    }
    // (the landing area is reused batch after batch: copies and scatters are stream ordered)
    // (hipMemcpyDefault: the C ABI's staging may be BAR-written device memory, whose
    // write-combined stores -- packets and the descriptors above -- must be out before the copy)
    _mm_sfence();
    HIPCHK(hipMemcpyAsync(sc_dev_, src, total, hipMemcpyDefault, st));
    HIPT(hipLaunchKernelGGL(tamd_scatter_rows, dim3(n), dim3(64), 0, st, (const ScatterDescDev*)(sc_dev_ + at), n,
                       (const uint8_t*)sc_dev_, arena_));
    HIPCHK(hipGetLastError());
    stats_.upload_bytes += total;
}

void Device::download_now(void* dst, uint64_t off, size_t n) {
    if (n == 0) return;
    flush_uploads();
    hipStream_t st = (hipStream_t)stream_;
    HIPCHK(hipMemcpyAsync(dst, arena_ + off, n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
}

void Device::download(void* dst, uint64_t off, size_t n) {
    if (n == 0) return;
    download_async(dst, off, n);
    synchronize();
}

void Device::download_async(void* dst, uint64_t off, size_t n) {
    if (n == 0) return;
    flush_uploads();
    hipStream_t st = (hipStream_t)stream_;
    if (n > rb_cap_) {  // larger than the pinned buffer: a plain (synchronous) copy
        synchronize();
        HIPCHK(hipMemcpyAsync(dst, arena_ + off, n, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        return;
    }
    if (rb_used_ + n > rb_cap_) synchronize();
    HIPCHK(hipMemcpyAsync(rb_host_ + rb_used_, arena_ + off, n, hipMemcpyDeviceToHost, st));
    Readback r;
    r.dst = dst;
    r.off = rb_used_;
    r.n = n;
    rb_pending_.push_back(r);
    rb_used_ += (n + 63) & ~(size_t)63;
}

void Device::download_pinned(void* dst, uint64_t off, size_t n) {
    if (collect_reads_) {
        if (n) reads_.push_back(HostCopy{dst, off, (uint32_t)n});
        return;
    }
    flush_uploads();
    if (n) HIPCHK(hipMemcpyAsync(dst, arena_ + off, n, hipMemcpyDeviceToHost, (hipStream_t)stream_));
}

void Device::flush_host_reads() {
    if (!reads_.empty()) host_copy(reads_.data(), (uint32_t)reads_.size(), true);
    reads_.clear();
}

void Device::host_copy(const HostCopy* d, uint32_t n, bool to_host) {
    if (!n) return;
    _mm_sfence();  // (sources the host wrote through the BAR, write-combined: out before the launch)
    flush_uploads();
    hipStream_t st = (hipStream_t)stream_;
    // a descriptor buffer whose previous launch has read it: the next one in turn that is free,
    // or (all busy) the next one in turn once it is (the ring is shared by every stream, and a
    // buffer's last launch may be queued behind another stream's work)
    const unsigned nb = (unsigned)(sizeof(hc_) / sizeof(hc_[0]));
    unsigned pick = hc_next_ % nb;
    for (unsigned k = 0; k < nb; ++k) {
        const unsigned i = (hc_next_ + k) % nb;
        if (!hc_[i].ev || hipEventQuery((hipEvent_t)hc_[i].ev) == hipSuccess) { pick = i; break; }
    }
    hc_next_ = pick + 1;
    HcBuf& b = hc_[pick];
    if (b.ev) HIPCHK(hipEventSynchronize((hipEvent_t)b.ev));  // (its previous launch has read it)
    const size_t need = (size_t)n * sizeof(HostCopyDev);
    if (need > b.cap) {  // (pooled: hipHostFree would wait for the whole device)
        host_free(b.p);
        b.cap = need + need / 2 + 4096;
        if (!(b.p = host_alloc(b.cap))) {
            b.cap = 0;
            error_ = "host copy descriptor allocation failed";
            failed_ = true;
            return;
        }
    }
    HostCopyDev* hd = (HostCopyDev*)b.p;
    for (uint32_t k = 0; k < n; ++k) {
        if (((uintptr_t)d[k].host & 15u) || (d[k].arena_off & 63u) || d[k].arena_off / 64 > 0xffffffffull) {
            error_ = "host copy: unaligned host buffer or arena offset";
            failed_ = true;
            return;
        }
        hd[k].host = (uint64_t)(uintptr_t)d[k].host;
        hd[k].unit = (uint32_t)(d[k].arena_off / 64);
        hd[k].len = d[k].len;
    }
    HIPT(hipLaunchKernelGGL(tamd_host_copy, dim3(n), dim3(128), 0, st, (const HostCopyDev*)b.p, n, arena_, to_host ? 1u : 0u));
    HIPCHK(hipGetLastError());
    if (!b.ev) {
        hipEvent_t he;
        HIPCHK(hipEventCreateWithFlags(&he, hipEventDisableTiming));
        b.ev = he;
    }
    HIPCHK(hipEventRecord((hipEvent_t)b.ev, st));
}

void* Device::record_event() {
    void* e = nullptr;
    if (!free_events_.empty()) {
        e = free_events_.back();
        free_events_.pop_back();
    } else {
        hipEvent_t he;
        HIPCHK(hipEventCreateWithFlags(&he, hipEventDisableTiming));
        e = he;
    }
    HIPCHK(hipEventRecord((hipEvent_t)e, (hipStream_t)stream_));
    return e;
}

void Device::reserve_events(size_t n) {
    while (free_events_.size() < n) {
        hipEvent_t he;
        if (hipEventCreateWithFlags(&he, hipEventDisableTiming) != hipSuccess) return;
        free_events_.push_back(he);
    }
}

bool Device::event_wait(void* ev) {
    const hipError_t e = hipEventSynchronize((hipEvent_t)ev);
    if (e != hipSuccess) fprintf(stderr, "tonk_amd: hipEventSynchronize failed: %s\n", hipGetErrorString(e));
    return e == hipSuccess;
}

// Pinned buffers (the C ABI's per-codec staging and landing buffers) are power-of-two blocks cut
// from pinned slabs of 64 MB, and go back to per-size free lists, never to HIP while the process
// runs: hipHostFree waits for the whole device, so a codec growing its buffer (or a connection
// closing) would stall every other codec's work behind it; and on some hosts every hipHostMalloc
// takes 10+ ms while blocking other HIP calls -- hundreds of codecs starting together (a Tonk test
// opening 100 connections) then spent seconds in allocations.  host_reserve() maps slabs up front.
// The same pool kind serves device memory the host writes through the PCIe BAR (bar_alloc):
// fine-grained device allocations, which the host stores into directly (write-combined) and the
// executor reads at HBM latency instead of across PCIe.
namespace {
const size_t kPinSlab = 64u << 20;

struct SlabPool {
    bool bar = false;  // device memory (BAR-writable) instead of pinned host memory
    std::mutex mu;
    std::vector<void*> free_[64];
    std::unordered_map<void*, unsigned> cls;
    uint8_t* slab = nullptr;  // the slab blocks are cut from
    size_t used = kPinSlab;
    std::vector<void*> spare;  // mapped and warmed ahead (prefill)

    void* raw(size_t n) {
        void* p = nullptr;
        if (g_pin_device >= 0) hipSetDevice(g_pin_device);  // (a codec thread may not have bound it yet)
        if (bar) return hipExtMallocWithFlags(&p, n, hipDeviceMallocFinegrained) == hipSuccess ? p : nullptr;
        // (coherent: the persistent executor reads staged packets and commands, and writes results
        // and completion words, while the host works on the same pages -- server.h)
        return hipHostMalloc(&p, n, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess ? p : nullptr;
    }
    // A new slab, and one small copy out of it and back: the first transfer touching a new pinned
    // allocation has been seen to block for ~80 ms, which should not happen under the device lock.
    void* new_slab() {
        const auto t0 = std::chrono::steady_clock::now();
        void* p = raw(kPinSlab);
        if (!p) return nullptr;
        static uint8_t* d = nullptr;
        if (!d && hipMalloc((void**)&d, 4096) != hipSuccess) d = nullptr;
        if (d && !bar) {
            memset(p, 0, 4096);
            hipMemcpy(d, p, 4096, hipMemcpyHostToDevice);
            hipMemcpy(p, d, 4096, hipMemcpyDeviceToHost);
        }
        report_slow(bar ? "BAR slab" : "pinned slab", t0, kPinSlab >> 20, 0);
        return p;
    }
    void prefill(unsigned slabs) {
        std::vector<void*> got;
        for (unsigned i = 0; i < slabs; ++i)
            if (void* p = new_slab()) got.push_back(p);
        std::lock_guard<std::mutex> g(mu);
        spare.insert(spare.end(), got.begin(), got.end());
    }
    bool reserve(size_t bytes) {
        void* p = nullptr;
        {
            std::lock_guard<std::mutex> g(mu);
            // (one slab at a time: the current one is only replaced once used up)
            if (slab && used + bytes <= kPinSlab) return true;
            if (!spare.empty()) {
                p = spare.back();
                spare.pop_back();
            }
        }
        // A new slab is mapped and warmed outside the mutex (the allocation and its copies can take
        // tens of ms, which under the mutex would stall every codec allocating meanwhile), then
        // published under it; a thread that lost the race parks its slab as a spare.
        if (!p && !(p = new_slab())) return false;
        std::lock_guard<std::mutex> g(mu);
        if (slab && used + bytes <= kPinSlab) {
            spare.push_back(p);
            return true;
        }
        if (slab) {  // the rest of the old slab becomes free blocks
            for (unsigned c = 63; c >= 12; --c)
                while (used + ((size_t)1 << c) <= kPinSlab) {
                    void* b = slab + used;
                    cls[b] = c;
                    free_[c].push_back(b);
                    used += (size_t)1 << c;
                }
        }
        slab = (uint8_t*)p;
        used = 0;
        return true;
    }
    void* alloc(size_t n) {
        unsigned c = 12;
        while (((size_t)1 << c) < n) ++c;
        const size_t sz = (size_t)1 << c;
        {
            std::lock_guard<std::mutex> g(mu);
            if (!free_[c].empty()) {
                void* p = free_[c].back();
                free_[c].pop_back();
                return p;
            }
        }
        if (sz > kPinSlab / 4) {  // (large blocks: their own allocation)
            const auto t0 = std::chrono::steady_clock::now();
            void* p = raw(sz);
            if (!p) return nullptr;
            report_slow(bar ? "BAR allocation" : "pinned allocation", t0, sz >> 10, 0);
            std::lock_guard<std::mutex> g(mu);
            cls[p] = c;
            return p;
        }
        for (;;) {
            {
                std::lock_guard<std::mutex> g(mu);
                if (slab && used + sz <= kPinSlab) {  // (4 KB aligned: every size is a multiple)
                    void* p = slab + used;
                    used += sz;
                    cls[p] = c;
                    return p;
                }
            }
            if (!reserve(sz)) return nullptr;
        }
    }
    void release(void* p) {
        if (!p) return;
        std::lock_guard<std::mutex> g(mu);
        auto it = cls.find(p);
        if (it != cls.end()) free_[it->second].push_back(p);
    }
};
SlabPool g_pin;
SlabPool& bar_pool() {
    static SlabPool* p = [] {
        SlabPool* q = new SlabPool();
        q->bar = true;
        return q;
    }();
    return *p;
}
}  // namespace

void Device::host_prefill(unsigned slabs) { g_pin.prefill(slabs); }
bool Device::host_reserve(size_t bytes) { return g_pin.reserve(bytes); }
void* Device::host_alloc(size_t n) { return g_pin.alloc(n); }
void Device::host_free(void* p) { g_pin.release(p); }
void* Device::bar_alloc(size_t n) { return bar_pool().alloc(n); }
void Device::bar_free(void* p) { bar_pool().release(p); }

bool Device::enable_staging() {
    if (h2d_stream_) return true;
    hipStream_t a, b;
    hipEvent_t e0, e1, e2;
    if (hipStreamCreateWithFlags(&a, hipStreamNonBlocking) != hipSuccess) return false;
    if (hipStreamCreateWithFlags(&b, hipStreamNonBlocking) != hipSuccess) return false;
    if (hipEventCreateWithFlags(&e0, hipEventDisableTiming) != hipSuccess) return false;
    if (hipEventCreateWithFlags(&e1, hipEventDisableTiming) != hipSuccess) return false;
    if (hipEventCreateWithFlags(&e2, hipEventDisableTiming) != hipSuccess) return false;
    h2d_stream_ = a;
    d2h_stream_ = b;
    h2d_done_ = e0;
    gather_done_ = e1;
    d2h_done_ = e2;
    return true;
}

void Device::h2d(uint64_t off, const void* src, size_t n) {
    if (n) HIPCHK(hipMemcpyAsync(arena_ + off, src, n, hipMemcpyHostToDevice, (hipStream_t)h2d_stream_));
}

void Device::h2d_fence() {
    HIPCHK(hipEventRecord((hipEvent_t)h2d_done_, (hipStream_t)h2d_stream_));
    HIPCHK(hipStreamWaitEvent((hipStream_t)stream_, (hipEvent_t)h2d_done_, 0));
}

void Device::d2h_gather(const std::vector<GatherDesc>& d, size_t bytes, void* dst) {
    flush_uploads();
    if (d.empty()) return;
    hipStream_t st = (hipStream_t)stream_;
    // the previous gather's copy-out must be done before the buffers are reused
    HIPCHK(hipStreamWaitEvent(st, (hipEvent_t)d2h_done_, 0));
    if (bytes > gather_cap_) {
        HIPCHK(hipStreamSynchronize((hipStream_t)d2h_stream_));
        HIPCHK(hipStreamSynchronize(st));
        if (gather_dev_) hipFree(gather_dev_);
        gather_cap_ = bytes + bytes / 2 + 4096;
        HIPCHK(hipMalloc((void**)&gather_dev_, gather_cap_));
    }
    if (d.size() > gdesc_cap_) {
        HIPCHK(hipStreamSynchronize(st));
        if (gdesc_dev_) hipFree(gdesc_dev_);
        if (gdesc_host_) hipHostFree(gdesc_host_);
        gdesc_cap_ = d.size() + d.size() / 2 + 64;
        HIPCHK(hipMalloc((void**)&gdesc_dev_, gdesc_cap_ * sizeof(GatherDesc)));
        HIPCHK(hipHostMalloc((void**)&gdesc_host_, gdesc_cap_ * sizeof(GatherDesc), hipHostMallocDefault));
    } else {
        // the descriptor staging buffer is reused: wait for the previous gather to have read it
        HIPCHK(hipEventSynchronize((hipEvent_t)gather_done_));
    }
    memcpy(gdesc_host_, d.data(), d.size() * sizeof(GatherDesc));
    HIPCHK(hipMemcpyAsync(gdesc_dev_, gdesc_host_, d.size() * sizeof(GatherDesc), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(tamd_gather_rows, dim3((uint32_t)d.size()), dim3(256), 0, st, gdesc_dev_, (uint32_t)d.size(),
                       arena_, gather_dev_);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord((hipEvent_t)gather_done_, st));
    hipStream_t ds = (hipStream_t)d2h_stream_;
    HIPCHK(hipStreamWaitEvent(ds, (hipEvent_t)gather_done_, 0));
    void* ta = timing_event();
    void* tb = timing_event();
    HIPCHK(hipEventRecord((hipEvent_t)ta, ds));  // (the copy's own duration: D2H effective rate)
    HIPCHK(hipMemcpyAsync(dst, gather_dev_, bytes, hipMemcpyDeviceToHost, ds));
    HIPCHK(hipEventRecord((hipEvent_t)tb, ds));
    d2h_timing_.push_back(std::make_pair(ta, tb));
    HIPCHK(hipEventRecord((hipEvent_t)d2h_done_, ds));
}

void Device::h2d_after_d2h(const void* src, size_t n) {
    if (!n) return;
    hipStream_t hs = (hipStream_t)h2d_stream_;
    if (n > recv_cap_) {
        HIPCHK(hipStreamSynchronize(hs));
        if (recv_dev_) hipFree(recv_dev_);
        recv_cap_ = n + n / 2 + 4096;
        HIPCHK(hipMalloc((void**)&recv_dev_, recv_cap_));
    }
    HIPCHK(hipStreamWaitEvent(hs, (hipEvent_t)d2h_done_, 0));
    HIPCHK(hipMemcpyAsync(recv_dev_, src, n, hipMemcpyHostToDevice, hs));
}

void Device::sync_staging() {
    if (h2d_stream_) HIPCHK(hipStreamSynchronize((hipStream_t)h2d_stream_));
    if (d2h_stream_) HIPCHK(hipStreamSynchronize((hipStream_t)d2h_stream_));
    for (auto& p : d2h_timing_) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, (hipEvent_t)p.first, (hipEvent_t)p.second) == hipSuccess) stats_.d2h_copy_ms += ms;
        timing_pool_.push_back(p.first);
        timing_pool_.push_back(p.second);
    }
    d2h_timing_.clear();
}

void Device::generate_rows(const std::vector<GenDesc>& d, uint32_t row_cap) {
    flush_uploads();
    if (d.empty()) return;
    hipStream_t st = (hipStream_t)stream_;
    GenDescDev* dd = nullptr;
    HIPCHK(hipMalloc((void**)&dd, d.size() * sizeof(GenDescDev)));
    HIPCHK(hipMemcpyAsync(dd, d.data(), d.size() * sizeof(GenDescDev), hipMemcpyHostToDevice, st));
    const uint32_t n = (uint32_t)d.size();
    hipLaunchKernelGGL(tamd_gen_rows, dim3((n + 255) / 256), dim3(256), 0, st, dd, n, arena_, row_cap);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    hipFree(dd);
}

void Device::digest_rows(const std::vector<DigestDesc>& d, std::vector<uint64_t>& out) {
    flush_uploads();
    out.assign(d.size(), 0);
    if (d.empty()) return;
    hipStream_t st = (hipStream_t)stream_;
    DigestDescDev* dd = nullptr;
    unsigned long long* dout = nullptr;
    HIPCHK(hipMalloc((void**)&dd, d.size() * sizeof(DigestDescDev)));
    HIPCHK(hipMalloc((void**)&dout, d.size() * 8));
    HIPCHK(hipMemcpyAsync(dd, d.data(), d.size() * sizeof(DigestDescDev), hipMemcpyHostToDevice, st));
    const uint32_t n = (uint32_t)d.size();
    hipLaunchKernelGGL(tamd_digest_rows, dim3((n + 255) / 256), dim3(256), 0, st, dd, n, arena_, dout);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out.data(), dout, d.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    hipFree(dd);
    hipFree(dout);
}

void Device::verify_next(const std::vector<VerifyDesc>& d) {
    if (d.empty()) return;
    VerifyBatch b;
    b.host = d;
    b.count = (uint32_t)d.size();
    uint8_t* mem = nullptr;
    HIPCHK(hipMalloc((void**)&mem, d.size() * (sizeof(VerifyDesc) + sizeof(VerifyOut))));
    if (!mem) return;
    b.dev_desc = (VerifyDesc*)mem;
    b.dev_out = (VerifyOut*)(mem + d.size() * sizeof(VerifyDesc));
    HIPCHK(hipMemcpyAsync(b.dev_desc, b.host.data(), d.size() * sizeof(VerifyDesc), hipMemcpyHostToDevice,
                          (hipStream_t)stream_));
    vbatches_.push_back(std::move(b));
    if (pending_verify_ >= 0) run_verify(pending_verify_);  // (a batch no launch took: digest now)
    pending_verify_ = (int)vbatches_.size() - 1;
}

void Device::run_verify(int batch) {
    const VerifyBatch& b = vbatches_[batch];
    hipLaunchKernelGGL(tamd_verify_rows, dim3((b.count + 63) / 64), dim3(64), 0, (hipStream_t)stream_,
                       (const VerifyDescDev*)b.dev_desc, b.count, (const uint8_t*)arena_, (VerifyOutDev*)b.dev_out);
    HIPCHK(hipGetLastError());
}

void Device::verify_results(std::vector<VerifyOut>& out) {
    if (pending_verify_ >= 0) {  // registered but never launched: its rows exist already
        run_verify(pending_verify_);
        pending_verify_ = -1;
    }
    synchronize();
    out.clear();
    for (size_t k = vread_; k < vbatches_.size(); ++k) {
        const VerifyBatch& b = vbatches_[k];
        const size_t at = out.size();
        out.resize(at + b.count);
        HIPCHK(hipMemcpy(out.data() + at, b.dev_out, b.count * sizeof(VerifyOut), hipMemcpyDeviceToHost));
    }
}

void Device::verify_reset() {
    for (size_t k = vread_; k < vbatches_.size(); ++k) {
        if (vbatches_[k].dev_desc) hipFree(vbatches_[k].dev_desc);
        vbatches_[k] = VerifyBatch();
    }
    vread_ = vbatches_.size();
}

bool Device::gf_selftest() {
    hipStream_t st = (hipStream_t)stream_;
    uint8_t* dout = nullptr;
    HIPCHK(hipMalloc((void**)&dout, 65536));
    hipLaunchKernelGGL(tamd_gf_selftest, dim3(256), dim3(64), 0, st, d_gf_, dout);
    std::vector<uint8_t> h(65536);
    HIPCHK(hipMemcpyAsync(h.data(), dout, 65536, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    hipFree(dout);
    for (unsigned y = 0; y < 256; ++y)
        for (unsigned x = 0; x < 256; ++x)
            if (h[y * 256 + x] != gf_mul((uint8_t)x, (uint8_t)y)) return false;
    return error_.empty();
}

void* Device::timing_event() {
    if (!timing_pool_.empty()) {
        void* e = timing_pool_.back();
        timing_pool_.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    HIPCHK(hipEventCreate(&e));
    return e;
}

void Device::collect_timing() {
    for (auto& p : timing_events_) {
        float ms = 0;
        hipEventSynchronize((hipEvent_t)p.second);
        if (hipEventElapsedTime(&ms, (hipEvent_t)p.first, (hipEvent_t)p.second) == hipSuccess) {
            stats_.kernel_ms += ms;
            stats_.timed_launches++;
        }
        timing_pool_.push_back(p.first);
        timing_pool_.push_back(p.second);
    }
    timing_events_.clear();
}

} // namespace tamd
