// compress.cpp -- host side of the compression step (include/tonk_compress.h): the FSE tables
// of zstd's predefined distributions, MessageCompressor's history-ring bookkeeping, and the
// launches of tamd_lz_compress (lz.hip).
#include "../../include/tonk_compress.h"
#include "lz.h"

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <mutex>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

extern "C" __global__ void tamd_lz_compress(const tamd_lz_job*, const tamd_lz_msg*, const uint8_t*, uint8_t*,
                                            uint32_t*, unsigned long long*);

namespace tamd {
namespace {

// History ring of PacketCompression.h:36-63 (kCompressionDictBytes = 24 * 1000).
const uint32_t kDictBytes = 24 * 1000;

struct DeviceTables {
    std::mutex mu;
    int device = -1;
    uint8_t* fse = nullptr;
};
DeviceTables g_tables;

const uint8_t* device_fse(int device) {
    std::lock_guard<std::mutex> g(g_tables.mu);
    if (g_tables.fse && g_tables.device == device) return g_tables.fse;
    std::vector<uint8_t> blob(TAMD_FSE_BYTES, 0);
    tamd_fse_blob(blob.data());
    uint8_t* d = nullptr;
    if (hipMalloc((void**)&d, TAMD_FSE_BYTES) != hipSuccess) return nullptr;
    if (hipMemcpy(d, blob.data(), TAMD_FSE_BYTES, hipMemcpyHostToDevice) != hipSuccess) {
        hipFree(d);
        return nullptr;
    }
    g_tables.fse = d;  // (kept for the process; one device per process in practice)
    g_tables.device = device;
    return d;
}

bool device_ok() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return false;
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

// MessageCompressor's ring (PacketCompression.h:44-63 Allocate/Commit, used by Compress at
// PacketCompression.cpp:79-83 and identically by the decompressor): every message is placed at
// the write offset unless `max` bytes would not fit, in which case the ring restarts at 0 and a
// new contiguous segment begins.  In linear stream positions, the decompressor decoding a message
// holds the current segment before it and, as zstd's external dictionary, the previous segment's
// bytes that the current segment has not overwritten yet (ring offsets past the message's end).
struct RingTrack {
    uint32_t max = 0, next = 0;  // ring write offset
    uint64_t lin = 0;            // linear position of the next message
    uint64_t seg = 0;            // linear start of the current segment
    uint64_t prev = 0;           // linear start of the previous segment (seg when none)
    bool have_prev = false;
    // place a message of n bytes; returns its linear position and window start
    void place(uint32_t n, uint64_t* pos, uint64_t* win) {
        if (next + max > kDictBytes) {
            if (next != 0) {
                prev = seg;
                have_prev = true;
                seg = lin;
            }
            next = 0;
        }
        *pos = lin;
        if (have_prev) {
            // previous segment bytes at ring offsets >= next + n are still intact
            const uint64_t w = prev + next + n;
            *win = w < seg ? w : seg;
        } else {
            *win = seg;
        }
        next += n;
        lin += n;
    }
};

}  // namespace

struct Compressor {
    uint32_t max = 0;
    int device = 0;
    const uint8_t* fse = nullptr;
    uint8_t* ring = nullptr;  // 64 KB device ring of the stream's bytes (linear position & 0xffff)
    tamd_lz_job* d_job = nullptr;
    tamd_lz_msg* d_msg = nullptr;
    uint8_t* d_out = nullptr;
    uint32_t* d_written = nullptr;
    uint8_t* h_stage = nullptr;  // pinned: message in, then {written, block} out
    RingTrack ring_track;
    bool failed = false;
};

static const uint32_t kRing = 1u << 16;
static const uint32_t kMirror = 64;  // the ring's first bytes repeated after it (wide loads at its end)
// pinned staging of the per-message path: [message | descriptor | written | compressed block]
static size_t stage_msg(uint32_t max) { return ((size_t)max + 63u) & ~(size_t)63u; }
static size_t stage_written(uint32_t max) { return stage_msg(max) + 64u; }
static size_t stage_out(uint32_t max) { return stage_written(max) + 64u; }
static size_t stage_bytes(uint32_t max) { return stage_out(max) + max + 64u; }

}  // namespace tamd

using namespace tamd;

// Every compressor of the process enqueues on one stream (each call is a synchronous round trip);
// Tonk creates a compressor per connection, most of which may never compress, so a compressor's
// device buffers are made on its first message.
static std::mutex g_lz_mu;
static hipStream_t g_lz_stream = nullptr;

static bool ensure_device(Compressor* c) {
    if (c->ring) return true;
    bool ok = (c->fse = device_fse(c->device)) != nullptr;
    if (ok && !g_lz_stream) ok = hipStreamCreateWithFlags(&g_lz_stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipMalloc((void**)&c->d_job, sizeof(tamd_lz_job)) == hipSuccess;
    ok = ok && hipMalloc((void**)&c->d_msg, sizeof(tamd_lz_msg)) == hipSuccess;
    ok = ok && hipMalloc((void**)&c->d_out, c->max + 64) == hipSuccess;
    ok = ok && hipMalloc((void**)&c->d_written, 64) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&c->h_stage, stage_bytes(c->max), hipHostMallocDefault) == hipSuccess;
    uint8_t* ring = nullptr;
    ok = ok && hipMalloc((void**)&ring, kRing + kMirror) == hipSuccess;
    if (ok) {
        tamd_lz_job job;
        memset(&job, 0, sizeof(job));
        job.buf = ring;
        job.mask = kRing - 1;
        job.first = 0;
        job.count = 1;
        ok = hipMemcpy(c->d_job, &job, sizeof(job), hipMemcpyHostToDevice) == hipSuccess;
    }
    if (!ok) {
        if (ring) hipFree(ring);
        return false;
    }
    c->ring = ring;
    return true;
}

extern "C" void* tamd_compressor_create(unsigned max_bytes) {
    if (max_bytes == 0 || max_bytes + max_bytes > kRing || max_bytes > kDictBytes) return nullptr;
    if (!device_ok()) return nullptr;
    Compressor* c = new Compressor();
    c->max = max_bytes;
    c->ring_track.max = max_bytes;
    hipGetDevice(&c->device);
    return c;
}

extern "C" void tamd_compressor_destroy(void* cp) {
    Compressor* c = (Compressor*)cp;
    if (!c) return;
    {
        std::lock_guard<std::mutex> g(g_lz_mu);  // (no call of this compressor is in flight)
    }
    if (c->ring) hipFree(c->ring);
    if (c->d_job) hipFree(c->d_job);
    if (c->d_msg) hipFree(c->d_msg);
    if (c->d_out) hipFree(c->d_out);
    if (c->d_written) hipFree(c->d_written);
    if (c->h_stage) hipHostFree(c->h_stage);
    delete c;
}

extern "C" int tamd_compressor_compress(void* cp, const uint8_t* data, unsigned bytes, uint8_t* dest,
                                        unsigned* written) {
    Compressor* c = (Compressor*)cp;
    if (written) *written = 0;
    if (!c || !data || !dest || !written || bytes == 0 || bytes > c->max) return -1;
    if (c->failed) return -2;
    std::lock_guard<std::mutex> lock(g_lz_mu);
    if (!ensure_device(c)) {
        c->failed = true;
        return -2;
    }
    hipStream_t const stream = g_lz_stream;
    uint64_t pos = 0, win = 0;
    c->ring_track.place(bytes, &pos, &win);
    // positions passed to the kernel are rebased to a multiple of the ring size below the window
    // (same ring slots, small numbers)
    const uint64_t base = win & ~(uint64_t)(kRing - 1);
    tamd_lz_msg& m = *(tamd_lz_msg*)(c->h_stage + stage_msg(c->max));
    memset(&m, 0, sizeof(m));
    m.pos = (uint32_t)(pos - base);
    m.len = bytes;
    m.win = (uint32_t)(win - base);
    m.out = 0;
    m.cap = c->max;
    memcpy(c->h_stage, data, bytes);
    const uint32_t slot = (uint32_t)(pos & (kRing - 1));
    const uint32_t first = bytes < kRing - slot ? bytes : kRing - slot;
    bool ok = hipMemcpyAsync(c->ring + slot, c->h_stage, first, hipMemcpyHostToDevice, stream) == hipSuccess;
    if (first < bytes)
        ok = ok && hipMemcpyAsync(c->ring, c->h_stage + first, bytes - first, hipMemcpyHostToDevice, stream) ==
                       hipSuccess;
    // ring bytes [0, kMirror) also live at [kRing, kRing + kMirror)
    if (first < bytes) {
        const uint32_t k = bytes - first < kMirror ? bytes - first : kMirror;
        ok = ok && hipMemcpyAsync(c->ring + kRing, c->h_stage + first, k, hipMemcpyHostToDevice, stream) ==
                       hipSuccess;
    }
    if (slot < kMirror) {
        const uint32_t k = (kMirror - slot) < first ? kMirror - slot : first;
        ok = ok && hipMemcpyAsync(c->ring + kRing + slot, c->h_stage, k, hipMemcpyHostToDevice, stream) ==
                       hipSuccess;
    }
    ok = ok && hipMemcpyAsync(c->d_msg, &m, sizeof(m), hipMemcpyHostToDevice, stream) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(tamd_lz_compress, dim3(1), dim3(64), 0, stream, c->d_job, c->d_msg, c->fse, c->d_out,
                           c->d_written, (unsigned long long*)nullptr);
        ok = hipGetLastError() == hipSuccess;
    }
    uint32_t* h_written = (uint32_t*)(c->h_stage + stage_written(c->max));
    uint8_t* h_out = c->h_stage + stage_out(c->max);
    ok = ok && hipMemcpyAsync(h_written, c->d_written, 4, hipMemcpyDeviceToHost, stream) == hipSuccess;
    ok = ok && hipMemcpyAsync(h_out, c->d_out, c->max, hipMemcpyDeviceToHost, stream) == hipSuccess;
    ok = ok && hipStreamSynchronize(stream) == hipSuccess;
    if (!ok) {
        c->failed = true;
        return -2;
    }
    const uint32_t w = *h_written;
    if (w > c->max) {
        c->failed = true;
        return -2;
    }
    if (w) memcpy(dest, h_out, w);
    *written = w;
    return 0;
}

extern "C" int tamd_compress_batch(const void* dev_data, uint64_t stride, uint32_t n_streams, uint32_t n_msgs,
                                   const uint32_t* lens, uint32_t max_bytes, void* dev_out, uint32_t* written_host,
                                   uint32_t msgs_per_job, float* kernel_ms) {
    if (!dev_data || !lens || !dev_out || !written_host || !n_streams || !n_msgs || !max_bytes ||
        max_bytes > kDictBytes)
        return -1;
    if (stride > 0xffffffffull) return -1;  // linear positions are 32-bit per stream
    if (!msgs_per_job) msgs_per_job = 16;
    int dev = 0;
    if (!device_ok()) return -3;
    hipGetDevice(&dev);
    const uint8_t* fse = device_fse(dev);
    if (!fse) return -3;
    const uint64_t total = (uint64_t)n_streams * n_msgs;
    std::vector<tamd_lz_msg> msgs(total);
    std::vector<tamd_lz_job> jobs;
    for (uint32_t s = 0; s < n_streams; ++s) {
        RingTrack rt;
        rt.max = max_bytes;
        for (uint32_t k = 0; k < n_msgs; ++k) {
            const uint32_t n = lens[(uint64_t)s * n_msgs + k];
            if (n == 0 || n > max_bytes) return -1;
            uint64_t pos = 0, win = 0;
            rt.place(n, &pos, &win);
            if (pos + n + 8 > stride) return -1;  // (8 readable bytes past the last message)
            tamd_lz_msg& m = msgs[(uint64_t)s * n_msgs + k];
            memset(&m, 0, sizeof(m));
            m.pos = (uint32_t)pos;
            m.len = n;
            m.win = (uint32_t)win;
            m.out = 0;  // (set below: out is a 32-bit offset per stream chunk)
            m.cap = max_bytes;
        }
        for (uint32_t k = 0; k < n_msgs; k += msgs_per_job) {
            tamd_lz_job j;
            memset(&j, 0, sizeof(j));
            j.buf = (const uint8_t*)dev_data + (uint64_t)s * stride;
            j.mask = ~0u;
            j.first = (uint32_t)((uint64_t)s * n_msgs + k);
            j.count = n_msgs - k < msgs_per_job ? n_msgs - k : msgs_per_job;
            jobs.push_back(j);
        }
    }
    if (total * max_bytes > 0xffffffffull) return -1;  // output offsets are 32-bit
    for (uint64_t i = 0; i < total; ++i) msgs[i].out = (uint32_t)(i * max_bytes);
    // persistent launch state (grown on demand): stream, descriptor and result buffers, events
    static std::mutex mu;
    static hipStream_t st = nullptr;
    static tamd_lz_job* d_jobs = nullptr;
    static tamd_lz_msg* d_msgs = nullptr;
    static uint32_t* d_written = nullptr;
    static size_t cap_jobs = 0, cap_msgs = 0;
    static hipEvent_t e0 = nullptr, e1 = nullptr;
    std::lock_guard<std::mutex> g(mu);
    bool ok = true;
    if (!st) ok = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
                  hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess;
    if (ok && jobs.size() > cap_jobs) {
        if (d_jobs) hipFree(d_jobs);
        d_jobs = nullptr;
        cap_jobs = jobs.size() + jobs.size() / 2;
        ok = hipMalloc((void**)&d_jobs, cap_jobs * sizeof(tamd_lz_job)) == hipSuccess;
        if (!ok) cap_jobs = 0;
    }
    if (ok && total > cap_msgs) {
        if (d_msgs) hipFree(d_msgs);
        if (d_written) hipFree(d_written);
        d_msgs = nullptr;
        d_written = nullptr;
        cap_msgs = total + total / 2;
        ok = hipMalloc((void**)&d_msgs, cap_msgs * sizeof(tamd_lz_msg)) == hipSuccess &&
             hipMalloc((void**)&d_written, cap_msgs * 4) == hipSuccess;
        if (!ok) cap_msgs = 0;
    }
    ok = ok && hipMemcpyAsync(d_jobs, jobs.data(), jobs.size() * sizeof(tamd_lz_job), hipMemcpyHostToDevice, st) ==
                   hipSuccess;
    ok = ok && hipMemcpyAsync(d_msgs, msgs.data(), total * sizeof(tamd_lz_msg), hipMemcpyHostToDevice, st) ==
                   hipSuccess;
    // profiling only: TONK_AMD_LZ_PROF=1 prints the phase totals of the launch (lz.hip LZ_PHASE)
    static const bool prof_on = getenv("TONK_AMD_LZ_PROF") != nullptr;
    unsigned long long* d_prof = nullptr;
    if (ok && prof_on) ok = hipMalloc((void**)&d_prof, jobs.size() * 5 * 8) == hipSuccess;
    if (ok) {
        hipExtLaunchKernelGGL(tamd_lz_compress, dim3((uint32_t)jobs.size()), dim3(64), 0, st, e0, e1, 0, d_jobs,
                              d_msgs, fse, (uint8_t*)dev_out, d_written, d_prof);
        ok = hipGetLastError() == hipSuccess;
    }
    if (ok && d_prof) {
        std::vector<unsigned long long> h(jobs.size() * 5);
        ok = hipMemcpyAsync(h.data(), d_prof, h.size() * 8, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess;
        double t[5] = {0, 0, 0, 0, 0};
        for (size_t j = 0; j < jobs.size(); ++j)
            for (int k = 0; k < 5; ++k) t[k] += (double)h[5 * j + k];
        fprintf(stderr, "lz phases (us per job): window %.1f probe %.1f parse %.1f fse %.1f out %.1f\n",
                t[0] / jobs.size() / 100.0, t[1] / jobs.size() / 100.0, t[2] / jobs.size() / 100.0,
                t[3] / jobs.size() / 100.0, t[4] / jobs.size() / 100.0);
        hipFree(d_prof);
    }
    ok = ok && hipMemcpyAsync(written_host, d_written, total * 4, hipMemcpyDeviceToHost, st) == hipSuccess;
    ok = ok && hipStreamSynchronize(st) == hipSuccess;
    if (ok && kernel_ms) {
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        *kernel_ms = ms;
    }
    return ok ? 0 : -2;
}

extern "C" int tamd_compress_batch_host(const void* host_data, uint64_t stride, uint32_t n_streams, uint32_t n_msgs,
                                        const uint32_t* lens, uint32_t max_bytes, void* host_out,
                                        uint32_t* written_host, uint32_t msgs_per_job, float* kernel_ms) {
    if (!host_data || !host_out || !n_streams || !n_msgs || !max_bytes) return -1;
    if (!device_ok()) return -3;
    const size_t in_bytes = (size_t)stride * n_streams, out_bytes = (size_t)n_streams * n_msgs * max_bytes;
    void *d_in = nullptr, *d_out = nullptr;
    int rc = -2;
    if (hipMalloc(&d_in, in_bytes) == hipSuccess && hipMalloc(&d_out, out_bytes) == hipSuccess &&
        hipMemcpy(d_in, host_data, in_bytes, hipMemcpyHostToDevice) == hipSuccess) {
        rc = tamd_compress_batch(d_in, stride, n_streams, n_msgs, lens, max_bytes, d_out, written_host, msgs_per_job,
                                 kernel_ms);
        if (rc == 0 && hipMemcpy(host_out, d_out, out_bytes, hipMemcpyDeviceToHost) != hipSuccess) rc = -2;
    }
    if (d_in) hipFree(d_in);
    if (d_out) hipFree(d_out);
    return rc;
}
