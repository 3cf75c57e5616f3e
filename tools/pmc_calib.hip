// pmc_calib.hip -- calibration for rocprofv3 FETCH_SIZE / WRITE_SIZE with the executors' access
// patterns: tamd_exec reads/writes 512 contiguous bytes per wave as 8 bytes per lane,
// tamd_exec16 1024 bytes as 16 bytes per lane.  These kernels move a known byte count with each
// width so tools/pmc_traffic.py can scale the executor's counters by a measured factor (the
// guide's gfx950 correction is stated for 16-B/lane loads).  Sizes are far beyond the 256 MiB
// Infinity Cache.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned long long u64;

extern "C" __global__ void calib_read8(const u64* __restrict__ src, size_t n_words, u64* __restrict__ sink) {
    u64 acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_words; i += (size_t)gridDim.x * blockDim.x)
        acc ^= src[i];
    if (acc == 0x123456789abcdefull) sink[0] = acc;  // keep the loads
}

extern "C" __global__ void calib_write8(u64* __restrict__ dst, size_t n_words) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_words; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = i;
}

typedef u64 u64x2 __attribute__((ext_vector_type(2)));

extern "C" __global__ void calib_read16(const u64x2* __restrict__ src, size_t n_pairs, u64* __restrict__ sink) {
    u64 acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pairs; i += (size_t)gridDim.x * blockDim.x) {
        const u64x2 v = src[i];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x123456789abcdefull) sink[0] = acc;
}

extern "C" __global__ void calib_write16(u64x2* __restrict__ dst, size_t n_pairs) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pairs; i += (size_t)gridDim.x * blockDim.x) {
        u64x2 v;
        v.x = i;
        v.y = ~i;
        dst[i] = v;
    }
}

// tamd_exec24's pattern: one wave per 1344-byte row, 16 B per lane over its first 1024 bytes and
// 8 B per lane over bytes 1024..1535 (lanes past the row's 1302 bytes re-read its first bytes).
extern "C" __global__ void calib_read_row24(const unsigned char* __restrict__ src, size_t n_rows, u64* __restrict__ sink) {
    const uint32_t lane = threadIdx.x & 63u;
    u64 acc = 0;
    for (size_t r = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; r < n_rows; r += (size_t)gridDim.x * (blockDim.x / 64)) {
        const unsigned char* row = src + r * 1344;
        const u64x2 v = *(const u64x2*)(row + lane * 16u);
        const uint32_t ox = 1024u + lane * 8u;
        const u64 w = *(const u64*)(row + (ox < 1302u ? ox : 0u));
        acc ^= v.x ^ v.y ^ w;
    }
    if (acc == 0x123456789abcdefull) sink[0] = acc;
}

extern "C" __global__ void calib_write_row24(unsigned char* __restrict__ dst, size_t n_rows) {
    const uint32_t lane = threadIdx.x & 63u;
    for (size_t r = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; r < n_rows; r += (size_t)gridDim.x * (blockDim.x / 64)) {
        unsigned char* row = dst + r * 1344;
        u64x2 v;
        v.x = r;
        v.y = ~r;
        *(u64x2*)(row + lane * 16u) = v;
        const uint32_t ox = 1024u + lane * 8u;
        if (ox < 1344u) *(u64*)(row + ox) = r ^ lane;
    }
}

int main() {
    const size_t read_bytes = 2ull << 30, write_bytes = 1ull << 30;
    u64 *src = nullptr, *dst = nullptr, *sink = nullptr;
    if (hipMalloc((void**)&src, read_bytes) != hipSuccess || hipMalloc((void**)&dst, write_bytes) != hipSuccess ||
        hipMalloc((void**)&sink, 64) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    (void)hipMemset(src, 1, read_bytes);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(calib_read8, dim3(4096), dim3(256), 0, 0, src, read_bytes / 8, sink);
        hipLaunchKernelGGL(calib_write8, dim3(4096), dim3(256), 0, 0, dst, write_bytes / 8);
        hipLaunchKernelGGL(calib_read16, dim3(4096), dim3(256), 0, 0, (const u64x2*)src, read_bytes / 16, sink);
        hipLaunchKernelGGL(calib_write16, dim3(4096), dim3(256), 0, 0, (u64x2*)dst, write_bytes / 16);
        hipLaunchKernelGGL(calib_read_row24, dim3(4096), dim3(256), 0, 0, (const unsigned char*)src, read_bytes / 1344, sink);
        hipLaunchKernelGGL(calib_write_row24, dim3(4096), dim3(256), 0, 0, (unsigned char*)dst, write_bytes / 1344);
    }
    (void)hipDeviceSynchronize();
    printf("{\"calib_read_bytes\": %zu, \"calib_write_bytes\": %zu, \"row24_read_bytes\": %zu, \"row24_write_bytes\": %zu}\n",
           read_bytes, write_bytes, (read_bytes / 1344) * 1302, (write_bytes / 1344) * 1344);
    (void)hipFree(src);
    (void)hipFree(dst);
    (void)hipFree(sink);
    return 0;
}
