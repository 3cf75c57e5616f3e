// device.cpp -- HIP runtime of the engine (see device.h).
#include "device.h"

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

extern "C" __global__ void tamd_exec(const tamd_op*, const tamd_instr*, const uint2*, uint32_t, uint8_t*,
                                     const uint32_t*);
extern "C" __global__ void tamd_gf_selftest(const uint32_t*, uint8_t*);

struct GenDescDev { uint32_t row, index, len, pad; unsigned long long seed; };
struct DigestDescDev { uint32_t row, skip, len, pad; };
extern "C" __global__ void tamd_gen_rows(const GenDescDev*, uint32_t, uint8_t*, uint32_t);
extern "C" __global__ void tamd_digest_rows(const DigestDescDev*, uint32_t, const uint8_t*, unsigned long long*);

namespace tamd {

#define HIPCHK(x)                                                                        \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "tonk_amd: %s failed: %s\n", #x, hipGetErrorString(e_));     \
            error_ = std::string(#x) + ": " + hipGetErrorString(e_);                    \
        }                                                                                \
    } while (0)

static const uint32_t kSlice = 512;   // bytes per work item (64 lanes x 8 bytes)
static const uint32_t kMaxGrid = 4096;

Device::~Device() {
    if (device_ < 0) return;
    hipSetDevice(device_);
    hipStreamSynchronize((hipStream_t)stream_);
    for (Slot& s : slots_) {
        if (s.host) hipHostFree(s.host);
        if (s.dev) hipFree(s.dev);
        if (s.done) hipEventDestroy((hipEvent_t)s.done);
    }
    for (void* e : ticket_events_) if (e) hipEventDestroy((hipEvent_t)e);
    for (auto& p : timing_events_) { hipEventDestroy((hipEvent_t)p.first); hipEventDestroy((hipEvent_t)p.second); }
    if (up_host_) hipHostFree(up_host_);
    if (up_event_) hipEventDestroy((hipEvent_t)up_event_);
    if (d_gf_) hipFree(d_gf_);
    if (arena_) hipFree(arena_);
    if (stream_) hipStreamDestroy((hipStream_t)stream_);
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
    HIPCHK(hipSetDevice(device));
    hipStream_t s = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    stream_ = s;
    arena_bytes_ = (arena_bytes + 255) & ~255ull;
    HIPCHK(hipMalloc((void**)&arena_, arena_bytes_));
    HIPCHK(hipMemsetAsync(arena_, 0, arena_bytes_, s));
    if (!gf_init()) { error_ = "gf self test failed"; return false; }
    HIPCHK(hipMalloc((void**)&d_gf_, sizeof(g_gf.perm)));
    HIPCHK(hipMemcpy(d_gf_, g_gf.perm, sizeof(g_gf.perm), hipMemcpyHostToDevice));
    for (Slot& sl : slots_) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        sl.done = e;
    }
    hipEvent_t ue;
    HIPCHK(hipEventCreateWithFlags(&ue, hipEventDisableTiming));
    up_event_ = ue;
    up_cap_ = 4u << 20;
    HIPCHK(hipHostMalloc((void**)&up_host_, up_cap_, hipHostMallocDefault));
    HIPCHK(hipStreamSynchronize(s));
    return error_.empty();
}

bool Device::ensure_slot(Slot& s, size_t bytes) {
    if (s.cap >= bytes) return true;
    if (s.host) hipHostFree(s.host);
    if (s.dev) hipFree(s.dev);
    size_t cap = 1u << 20;
    while (cap < bytes) cap *= 2;
    s.host = nullptr;
    s.dev = nullptr;
    s.cap = 0;
    if (hipHostMalloc((void**)&s.host, cap, hipHostMallocDefault) != hipSuccess) return false;
    if (hipMalloc((void**)&s.dev, cap) != hipSuccess) return false;
    s.cap = cap;
    return true;
}

uint64_t Device::run(Context* const* ctxs, size_t n) {
    hipStream_t st = (hipStream_t)stream_;
    // Count everything first.
    size_t n_instr = 0, n_ops = 0;
    uint32_t max_level = 0;
    for (size_t c = 0; c < n; ++c) {
        const ProgramBuilder& pb = ctxs[c]->pb;
        n_instr += pb.instrs().size();
        n_ops += pb.ops().size();
        stats_.acc_bytes += pb.acc_bytes();
        stats_.store_bytes += pb.store_bytes();
        if (pb.max_level() > max_level) max_level = pb.max_level();
    }
    const uint64_t ticket = ++ticket_;
    if (n_ops == 0) {
        completed_ = ticket;
        return ticket;
    }

    // Items per op and per level.
    std::vector<uint32_t> level_ops(max_level + 2, 0), level_items(max_level + 2, 0);
    size_t n_items = 0;
    for (size_t c = 0; c < n; ++c) {
        const ProgramBuilder& pb = ctxs[c]->pb;
        for (size_t i = 0; i < pb.ops().size(); ++i) {
            const uint32_t l = pb.op_levels()[i];
            const uint32_t slices = (pb.ops()[i].span + kSlice - 1) / kSlice;
            level_ops[l]++;
            level_items[l] += slices ? slices : 1;
            n_items += slices ? slices : 1;
        }
    }
    const size_t bytes_instr = n_instr * sizeof(tamd_instr);
    const size_t bytes_ops = n_ops * sizeof(tamd_op);
    const size_t bytes_items = n_items * sizeof(uint32_t) * 2;
    const size_t total = bytes_instr + bytes_ops + bytes_items;

    Slot& slot = slots_[next_slot_];
    next_slot_ ^= 1;
    if (slot.ticket) {
        HIPCHK(hipEventSynchronize((hipEvent_t)slot.done));
        if (slot.ticket > completed_) completed_ = slot.ticket;
    }
    if (!ensure_slot(slot, total)) { error_ = "program staging allocation failed"; return ticket; }

    tamd_instr* hi = (tamd_instr*)slot.host;
    tamd_op* ho = (tamd_op*)(slot.host + bytes_instr);
    uint32_t* hitems = (uint32_t*)(slot.host + bytes_instr + bytes_ops);

    // Level-ordered placement.
    std::vector<uint32_t> op_base(max_level + 2, 0), item_base(max_level + 2, 0);
    for (uint32_t l = 1; l <= max_level; ++l) {
        op_base[l + 1] = op_base[l] + level_ops[l];
        item_base[l + 1] = item_base[l] + level_items[l];
    }
    std::vector<uint32_t> op_fill(op_base), item_fill(item_base);
    uint32_t instr_base = 0;
    for (size_t c = 0; c < n; ++c) {
        const ProgramBuilder& pb = ctxs[c]->pb;
        memcpy(hi + instr_base, pb.instrs().data(), pb.instrs().size() * sizeof(tamd_instr));
        for (size_t i = 0; i < pb.ops().size(); ++i) {
            const uint32_t l = pb.op_levels()[i];
            tamd_op op = pb.ops()[i];
            op.first += instr_base;
            const uint32_t oi = op_fill[l]++;
            ho[oi] = op;
            uint32_t slices = (op.span + kSlice - 1) / kSlice;
            if (!slices) slices = 1;
            for (uint32_t s = 0; s < slices; ++s) {
                const uint32_t ii = item_fill[l]++;
                hitems[2 * ii] = oi;
                hitems[2 * ii + 1] = s;
            }
        }
        instr_base += (uint32_t)pb.instrs().size();
    }
    HIPCHK(hipMemcpyAsync(slot.dev, slot.host, total, hipMemcpyHostToDevice, st));
    const tamd_instr* di = (const tamd_instr*)slot.dev;
    const tamd_op* dops = (const tamd_op*)(slot.dev + bytes_instr);
    const uint2* ditems = (const uint2*)(slot.dev + bytes_instr + bytes_ops);
    for (uint32_t l = 1; l <= max_level; ++l) {
        const uint32_t cnt = level_items[l];
        if (!cnt) continue;
        uint32_t grid = (cnt + 3) / 4;
        if (grid > kMaxGrid) grid = kMaxGrid;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (timing_) {
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0, st);
        }
        hipLaunchKernelGGL(tamd_exec, dim3(grid), dim3(256), 0, st, dops, di, ditems + item_base[l], cnt,
                           arena_, d_gf_);
        if (timing_) {
            hipEventRecord(e1, st);
            timing_events_.push_back(std::make_pair((void*)e0, (void*)e1));
        }
        stats_.launches++;
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord((hipEvent_t)slot.done, st));
    slot.ticket = ticket;
    stats_.programs++;
    stats_.ops += n_ops;
    stats_.items += n_items;
    stats_.instrs += n_instr;
    stats_.upload_bytes += total;
    return ticket;
}

bool Device::completed(uint64_t ticket) {
    if (ticket <= completed_) return true;
    for (Slot& s : slots_) {
        if (s.ticket == ticket) {
            if (hipEventQuery((hipEvent_t)s.done) == hipSuccess) {
                completed_ = ticket;
                return true;
            }
            return false;
        }
    }
    // Older than both slots: finished when the slots' older ticket is done.
    return ticket <= completed_;
}

void Device::wait(uint64_t ticket) {
    if (ticket <= completed_) return;
    for (Slot& s : slots_) {
        if (s.ticket == ticket) {
            HIPCHK(hipEventSynchronize((hipEvent_t)s.done));
            completed_ = ticket;
            return;
        }
    }
    synchronize();
}

void Device::synchronize() {
    HIPCHK(hipStreamSynchronize((hipStream_t)stream_));
    completed_ = ticket_;
    up_used_ = 0;
}

void Device::upload(uint64_t off, const void* src, size_t n) {
    if (n == 0) return;
    hipStream_t st = (hipStream_t)stream_;
    if (n > up_cap_) {
        HIPCHK(hipMemcpyAsync(arena_ + off, src, n, hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
        return;
    }
    if (up_used_ + n > up_cap_) {
        HIPCHK(hipStreamSynchronize(st));
        completed_ = ticket_;
        up_used_ = 0;
    }
    memcpy(up_host_ + up_used_, src, n);
    HIPCHK(hipMemcpyAsync(arena_ + off, up_host_ + up_used_, n, hipMemcpyHostToDevice, st));
    up_used_ += (n + 63) & ~(size_t)63;
}

void Device::download(void* dst, uint64_t off, size_t n) {
    if (n == 0) return;
    hipStream_t st = (hipStream_t)stream_;
    HIPCHK(hipMemcpyAsync(dst, arena_ + off, n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    completed_ = ticket_;
    up_used_ = 0;
}

void Device::generate_rows(const std::vector<GenDesc>& d, uint32_t row_cap) {
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

void Device::collect_timing() {
    for (auto& p : timing_events_) {
        float ms = 0;
        hipEventSynchronize((hipEvent_t)p.second);
        if (hipEventElapsedTime(&ms, (hipEvent_t)p.first, (hipEvent_t)p.second) == hipSuccess) {
            stats_.kernel_ms += ms;
            stats_.timed_launches++;
        }
        hipEventDestroy((hipEvent_t)p.first);
        hipEventDestroy((hipEvent_t)p.second);
    }
    timing_events_.clear();
}

} // namespace tamd
