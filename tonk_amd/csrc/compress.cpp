// compress.cpp -- host side of the compression step (include/tonk_compress.h): the FSE tables
// of zstd's predefined distributions, MessageCompressor's history-ring bookkeeping, and the
// launches of tamd_lz_compress (lz.hip).
#include "../../include/tonk_compress.h"
#include "lz.h"

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <condition_variable>
#include <mutex>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

extern "C" __global__ void tamd_lz_compress(const tamd_lz_job*, uint32_t, const tamd_lz_msg*, const uint8_t*,
                                            uint8_t*, uint32_t*, uint8_t*, unsigned long long*);
// (lz.hip: two jobs per 128-thread workgroup)
static const uint32_t kLzJobsPerGroup = TAMD_LZ_WAVES;
extern "C" __global__ void tamd_lz_scatter_ring(const tamd_lz_scatter*, const uint8_t*);

namespace tamd {
namespace {

// History ring of PacketCompression.h:36-63 (kCompressionDictBytes = 24 * 1000).
const uint32_t kDictBytes = 24 * 1000;

// The FSE table blob on each device (uploaded once per device, kept for the process).
struct DeviceTables {
    std::mutex mu;
    std::vector<uint8_t*> fse;  // by device index
};
DeviceTables g_tables;

const uint8_t* device_fse(int device) {
    std::lock_guard<std::mutex> g(g_tables.mu);
    if (device < 0) return nullptr;
    if ((size_t)device < g_tables.fse.size() && g_tables.fse[device]) return g_tables.fse[device];
    std::vector<uint8_t> blob(TAMD_FSE_BYTES, 0);
    tamd_fse_blob(blob.data());
    // (TONK_AMD_LZ_FIT=0: the predefined sequence tables only, as before round 6 -- A/B knob)
    if (getenv("TONK_AMD_LZ_FIT") && atoi(getenv("TONK_AMD_LZ_FIT")) == 0) blob[TAMD_FSE_FLAGS] |= TAMD_FSE_PREDEFINED_ONLY;
    uint8_t* d = nullptr;
    if (hipSetDevice(device) != hipSuccess || hipMalloc((void**)&d, TAMD_FSE_BYTES) != hipSuccess) return nullptr;
    if (hipMemcpy(d, blob.data(), TAMD_FSE_BYTES, hipMemcpyHostToDevice) != hipSuccess) {
        hipFree(d);
        return nullptr;
    }
    if ((size_t)device >= g_tables.fse.size()) g_tables.fse.resize(device + 1, nullptr);
    g_tables.fse[device] = d;
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
    uint8_t* ring = nullptr;  // device ring of the stream's bytes (linear position & 0xffff) + mirror
    RingTrack ring_track;
    bool failed = false;
    bool queued = false;      // a call of this compressor is in the current batch
};

}  // namespace tamd

using namespace tamd;

// ---- the per-message drop-in: concurrent calls combined into one launch ----
//
// Tonk compresses each message on the connection's own thread and waits for the result
// (PacketCompression.cpp:70-118).  One GPU round trip per message is slow next to zstd on the
// calling thread, so calls from different connections are combined: a caller queues its
// request; the first caller becomes the leader and runs every queued request as ONE batch (one
// upload of all messages and descriptors, a scatter into the compressors' rings, one compression
// launch with a wave per message, one download), then completes them and serves the requests
// that queued meanwhile.  A batch costs about one round trip however many connections it serves.
namespace {
struct LzRequest {
    Compressor* c;
    const uint8_t* data;
    uint32_t bytes;
    uint8_t* dest;
    unsigned* written;
    int rc = 0;
    bool done = false;
    std::condition_variable cv;  // its caller waits here: a batch wakes only its own callers
};
std::mutex g_req_mu;
std::condition_variable g_req_cv;  // tamd_compressor_destroy waits here for its last call
std::vector<LzRequest*> g_pending;
bool g_leader = false;

// leader-only launch state (grown on demand)
struct LzBatchState {
    int device = -1;
    hipStream_t st = nullptr;
    uint8_t* h_in = nullptr;   // pinned: scatter descs | msgs | jobs | message bytes
    uint8_t* d_in = nullptr;
    size_t in_cap = 0;
    uint8_t* h_out = nullptr;  // pinned: written[] | compressed blocks
    uint8_t* d_out = nullptr;
    size_t out_cap = 0;
    uint8_t* d_scratch = nullptr;  // messages above TAMD_LZ_MAX_MESSAGE
    size_t scratch_cap = 0;
} g_batch;

size_t align16(size_t n) { return (n + 15) & ~(size_t)15; }

// Device rings of destroyed compressors are kept for the next ones: hipFree waits for the whole
// device (every stream of the process, the Siamese codecs' too), and Tonk destroys a compressor
// with every connection it closes.
std::mutex g_ring_mu;
std::vector<std::pair<int, uint8_t*>> g_free_rings;  // (device, ring)
uint8_t* take_ring(int device) {
    std::lock_guard<std::mutex> g(g_ring_mu);
    for (size_t i = 0; i < g_free_rings.size(); ++i)
        if (g_free_rings[i].first == device) {
            uint8_t* r = g_free_rings[i].second;
            g_free_rings[i] = g_free_rings.back();
            g_free_rings.pop_back();
            return r;
        }
    return nullptr;
}

bool grow(uint8_t*& h, uint8_t*& d, size_t& cap, size_t need) {
    if (need <= cap) return true;
    if (h) hipHostFree(h);
    if (d) hipFree(d);
    h = d = nullptr;
    cap = need + need / 2;
    if (hipHostMalloc((void**)&h, cap, hipHostMallocDefault) != hipSuccess || hipMalloc((void**)&d, cap) != hipSuccess) {
        cap = 0;
        return false;
    }
    return true;
}

// Runs one batch (leader, no lock held); every request of `b` belongs to device b[0]->c->device
// and names a distinct compressor.
void run_batch(const std::vector<LzRequest*>& in) {
    LzBatchState& S = g_batch;
    const int dev = in[0]->c->device;
    bool ok = hipSetDevice(dev) == hipSuccess;
    if (ok && S.device != dev) {  // (a process compresses on one device in practice)
        if (S.st) hipStreamDestroy(S.st);
        S.st = nullptr;
        ok = hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking) == hipSuccess;
        S.device = ok ? dev : -1;
    }
    const uint8_t* fse = ok ? device_fse(dev) : nullptr;
    ok = ok && fse;
    // A compressor whose device ring cannot be allocated fails on its own (rc -2, sticky) and is
    // left out of the launch: nothing is ever placed into a null ring.
    std::vector<LzRequest*> live;
    live.reserve(in.size());
    for (LzRequest* r : in) {
        if (ok && !r->c->ring && !r->c->failed) {
            uint8_t* ring = take_ring(dev);
            if (!ring && hipMalloc((void**)&ring, TAMD_LZ_RING + TAMD_LZ_MIRROR) != hipSuccess) r->c->failed = true;
            else r->c->ring = ring;
        }
        if (ok && r->c->ring && !r->c->failed) {
            live.push_back(r);
        } else {
            if (ok) r->c->failed = true;
            r->rc = -2;
        }
    }
    if (ok && live.empty()) return;
    const std::vector<LzRequest*>& b = ok ? live : in;
    const size_t n = b.size();
    size_t data_bytes = 0, out_bytes = 0, scratch_bytes = 0;
    for (LzRequest* r : b) {
        data_bytes += align16(r->bytes);
        out_bytes += align16(r->c->max);
        if (r->bytes > TAMD_LZ_MAX_MESSAGE) scratch_bytes += tamd_lz_scratch_bytes(r->bytes);
    }
    const size_t o_msgs = align16(n * sizeof(tamd_lz_scatter));
    const size_t o_jobs = o_msgs + align16(n * sizeof(tamd_lz_msg));
    const size_t o_data = o_jobs + align16(n * sizeof(tamd_lz_job));
    const size_t o_blocks = align16(n * 4);
    ok = ok && grow(S.h_in, S.d_in, S.in_cap, o_data + data_bytes) && grow(S.h_out, S.d_out, S.out_cap, o_blocks + out_bytes);
    if (ok && scratch_bytes > S.scratch_cap) {
        if (S.d_scratch) hipFree(S.d_scratch);
        S.d_scratch = nullptr;
        S.scratch_cap = scratch_bytes + scratch_bytes / 2;
        if (hipMalloc((void**)&S.d_scratch, S.scratch_cap) != hipSuccess) {
            S.scratch_cap = 0;
            ok = false;
        }
    }
    if (ok) {
        size_t scr = 0;
        tamd_lz_scatter* sc = (tamd_lz_scatter*)S.h_in;
        tamd_lz_msg* ms = (tamd_lz_msg*)(S.h_in + o_msgs);
        tamd_lz_job* jb = (tamd_lz_job*)(S.h_in + o_jobs);
        size_t din = 0, dout = o_blocks;
        for (size_t i = 0; i < n; ++i) {
            LzRequest* r = b[i];
            Compressor* c = r->c;
            uint64_t pos = 0, win = 0;
            c->ring_track.place(r->bytes, &pos, &win);
            // positions are rebased to a multiple of the ring size below the window (same ring
            // slots, small numbers)
            const uint64_t base = win & ~(uint64_t)(TAMD_LZ_RING - 1);
            memcpy(S.h_in + o_data + din, r->data, r->bytes);
            sc[i].ring = c->ring;
            sc[i].slot = (uint32_t)(pos & (TAMD_LZ_RING - 1));
            sc[i].bytes = r->bytes;
            sc[i].src = (uint32_t)din;
            sc[i].pad = 0;
            memset(&ms[i], 0, sizeof(ms[i]));
            ms[i].pos = (uint32_t)(pos - base);
            ms[i].len = r->bytes;
            ms[i].win = (uint32_t)(win - base);
            ms[i].out = (uint32_t)(dout - o_blocks);
            ms[i].cap = c->max;
            ms[i].scratch = TAMD_LZ_NO_SCRATCH;
            if (r->bytes > TAMD_LZ_MAX_MESSAGE) {
                ms[i].scratch = (uint32_t)scr;
                scr += tamd_lz_scratch_bytes(r->bytes);
            }
            memset(&jb[i], 0, sizeof(jb[i]));
            jb[i].buf = c->ring;
            jb[i].mask = TAMD_LZ_RING - 1;
            jb[i].first = (uint32_t)i;
            jb[i].count = 1;
            din += align16(r->bytes);
            dout += align16(c->max);
        }
        ok = hipMemcpyAsync(S.d_in, S.h_in, o_data + data_bytes, hipMemcpyHostToDevice, S.st) == hipSuccess;
        if (ok) {
            hipLaunchKernelGGL(tamd_lz_scatter_ring, dim3((uint32_t)n), dim3(256), 0, S.st,
                               (const tamd_lz_scatter*)S.d_in, (const uint8_t*)(S.d_in + o_data));
            hipLaunchKernelGGL(tamd_lz_compress, dim3((uint32_t)((n + kLzJobsPerGroup - 1) / kLzJobsPerGroup)),
                               dim3(64 * kLzJobsPerGroup), 0, S.st, (const tamd_lz_job*)(S.d_in + o_jobs), (uint32_t)n,
                               (const tamd_lz_msg*)(S.d_in + o_msgs), fse, S.d_out + o_blocks, (uint32_t*)S.d_out,
                               S.d_scratch, (unsigned long long*)nullptr);
            ok = hipGetLastError() == hipSuccess;
        }
        ok = ok && hipMemcpyAsync(S.h_out, S.d_out, o_blocks + out_bytes, hipMemcpyDeviceToHost, S.st) == hipSuccess;
        ok = ok && hipStreamSynchronize(S.st) == hipSuccess;
    }
    size_t dout = o_blocks;
    for (size_t i = 0; i < n; ++i) {
        LzRequest* r = b[i];
        Compressor* c = r->c;
        const uint32_t w = ok ? ((const uint32_t*)S.h_out)[i] : 0;
        if (!ok || c->failed || w > c->max) {
            c->failed = true;
            r->rc = -2;
        } else {
            if (w) memcpy(r->dest, S.h_out + dout, w);
            *r->written = w;
            r->rc = 0;
        }
        dout += align16(c->max);
    }
}
}  // namespace

extern "C" void* tamd_compressor_create(unsigned max_bytes) {
    if (max_bytes == 0 || max_bytes + max_bytes > TAMD_LZ_RING || max_bytes > kDictBytes) return nullptr;
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
        // (no call of this compressor is queued or in flight: its owner is not calling it)
        std::unique_lock<std::mutex> g(g_req_mu);
        g_req_cv.wait(g, [c] { return !c->queued; });
    }
    if (c->ring) {  // (no launch reads it any more: its last call was waited for)
        std::lock_guard<std::mutex> g(g_ring_mu);
        g_free_rings.push_back(std::make_pair(c->device, c->ring));
    }
    delete c;
}

extern "C" int tamd_compressor_compress(void* cp, const uint8_t* data, unsigned bytes, uint8_t* dest,
                                        unsigned* written) {
    Compressor* c = (Compressor*)cp;
    if (written) *written = 0;
    if (!c || !data || !dest || !written || bytes == 0 || bytes > c->max) return -1;
    if (c->failed) return -2;
    LzRequest req;
    req.c = c;
    req.data = data;
    req.bytes = bytes;
    req.dest = dest;
    req.written = written;
    std::unique_lock<std::mutex> lk(g_req_mu);
    g_pending.push_back(&req);
    // Wait while another caller leads; take over when it steps down with this request unserved.
    req.cv.wait(lk, [&req] { return req.done || !g_leader; });
    if (req.done) return req.rc;
    g_leader = true;
    std::vector<LzRequest*> batch, later;
    // The leader serves batches only until its own request is done, then hands leadership to a
    // waiting caller: its own send path is never held by other connections' traffic.
    while (!req.done) {
        // one request per compressor and one device per batch (a compressor's messages are
        // placed in its ring in call order); the rest waits for the next batch
        batch.clear();
        later.clear();
        for (LzRequest* r : g_pending) {
            if (r->c->queued || r->c->device != g_pending[0]->c->device) later.push_back(r);
            else {
                r->c->queued = true;
                batch.push_back(r);
            }
        }
        g_pending.swap(later);
        lk.unlock();
        run_batch(batch);
        lk.lock();
        for (LzRequest* r : batch) {
            r->c->queued = false;
            r->done = true;
            if (r != &req) r->cv.notify_one();
        }
        g_req_cv.notify_all();
    }
    g_leader = false;
    if (!g_pending.empty()) g_pending.front()->cv.notify_one();  // the next queued caller leads
    return req.rc;
}

extern "C" int tamd_compress_batch(const void* dev_data, uint64_t stride, uint32_t n_streams, uint32_t n_msgs,
                                   const uint32_t* lens, uint32_t max_bytes, void* dev_out, uint32_t* written_host,
                                   uint32_t msgs_per_job, float* kernel_ms) {
    if (!dev_data || !lens || !dev_out || !written_host || !n_streams || !n_msgs || !max_bytes ||
        max_bytes > kDictBytes)
        return -1;
    if (stride > 0xffffffffull) return -1;  // linear positions are 32-bit per stream
    int dev = 0;
    if (!device_ok()) return -3;
    hipGetDevice(&dev);
    if (!msgs_per_job) {
        // auto: the fewest messages per job that keep every stream's jobs within one job per wave
        // slot (CUs x TAMD_LZ_WAVES): one round of jobs, each seeding its window once
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        const uint32_t slots = (uint32_t)cus * TAMD_LZ_WAVES;
        const uint32_t per_stream = slots / n_streams ? slots / n_streams : 1u;
        msgs_per_job = (n_msgs + per_stream - 1) / per_stream;
    }
    const uint8_t* fse = device_fse(dev);
    if (!fse) return -3;
    const uint64_t total = (uint64_t)n_streams * n_msgs;
    std::vector<tamd_lz_msg> msgs(total);
    std::vector<tamd_lz_job> jobs;
    uint64_t scratch_bytes = 0;
    for (uint32_t s = 0; s < n_streams; ++s) {
        RingTrack rt;
        rt.max = max_bytes;
        for (uint32_t k = 0; k < n_msgs; ++k) {
            const uint32_t n = lens[(uint64_t)s * n_msgs + k];
            if (n == 0 || n > max_bytes) return -1;
            uint64_t pos = 0, win = 0;
            rt.place(n, &pos, &win);
            if (pos + n + 32 > stride) return -1;  // (32 readable bytes past the last message: the
                                                   // kernel's wide loads, lz.hip)
            tamd_lz_msg& m = msgs[(uint64_t)s * n_msgs + k];
            memset(&m, 0, sizeof(m));
            m.pos = (uint32_t)pos;
            m.len = n;
            m.win = (uint32_t)win;
            m.out = 0;  // (set below: out is a 32-bit offset per stream chunk)
            m.cap = max_bytes;
            m.scratch = TAMD_LZ_NO_SCRATCH;
            if (n > TAMD_LZ_MAX_MESSAGE) {
                m.scratch = (uint32_t)scratch_bytes;
                scratch_bytes += tamd_lz_scratch_bytes(n);
            }
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
    if (total * max_bytes > 0xffffffffull || scratch_bytes > 0xffffffffull) return -1;  // 32-bit offsets
    for (uint64_t i = 0; i < total; ++i) msgs[i].out = (uint32_t)(i * max_bytes);
    // persistent launch state (grown on demand): stream, descriptor and result buffers, events
    static std::mutex mu;
    static hipStream_t st = nullptr;
    static tamd_lz_job* d_jobs = nullptr;
    static tamd_lz_msg* d_msgs = nullptr;
    static uint32_t* d_written = nullptr;
    static size_t cap_jobs = 0, cap_msgs = 0;
    static hipEvent_t e0 = nullptr, e1 = nullptr;
    static uint8_t* d_scratch = nullptr;
    static size_t cap_scratch = 0;
    std::lock_guard<std::mutex> g(mu);
    bool ok = true;
    if (scratch_bytes > cap_scratch) {
        if (d_scratch) hipFree(d_scratch);
        d_scratch = nullptr;
        cap_scratch = scratch_bytes + scratch_bytes / 2;
        ok = hipMalloc((void**)&d_scratch, cap_scratch) == hipSuccess;
        if (!ok) cap_scratch = 0;
    }
    if (ok && !st) ok = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
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
    if (ok && prof_on) ok = hipMalloc((void**)&d_prof, jobs.size() * TAMD_LZ_PHASES * 8) == hipSuccess;
    if (ok) {
        const uint32_t nj = (uint32_t)jobs.size();
        hipExtLaunchKernelGGL(tamd_lz_compress, dim3((nj + kLzJobsPerGroup - 1) / kLzJobsPerGroup),
                              dim3(64 * kLzJobsPerGroup), 0, st, e0, e1, 0, d_jobs, nj, d_msgs, fse, (uint8_t*)dev_out,
                              d_written, d_scratch, d_prof);
        ok = hipGetLastError() == hipSuccess;
    }
    if (ok && d_prof) {
        std::vector<unsigned long long> h(jobs.size() * TAMD_LZ_PHASES);
        ok = hipMemcpyAsync(h.data(), d_prof, h.size() * 8, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess;
        double t[TAMD_LZ_PHASES] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (size_t j = 0; j < jobs.size(); ++j)
            for (uint32_t k = 0; k < TAMD_LZ_PHASES; ++k) t[k] += (double)h[TAMD_LZ_PHASES * j + k];
        const double q = 100.0 * (double)jobs.size();
        fprintf(stderr, "lz phases (us per job): window %.1f probe %.1f parse %.1f codes+tables %.1f chains %.1f "
                "stream %.1f out %.1f; sequences per job %.1f\n", t[0] / q, t[1] / q, t[2] / q, t[5] / q, t[6] / q,
                t[3] / q, t[4] / q, t[7] / (double)jobs.size());
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
