// membench.hip -- PROFILING ONLY.  Ceiling of the executor's access pattern: waves gathering
// rows of 1344 B (the arena's row pitch) 512 B at a time (8 B per lane), B loads in flight per
// wave, XOR-combined.  Compares 8-byte and 16-byte-per-lane loads and batch depths.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <random>
typedef unsigned long long u64;

template <int B, int W>  // B loads in flight, W = bytes per lane (8 or 16)
__global__ void __launch_bounds__(256) gather(const uint8_t* __restrict__ buf, const uint32_t* __restrict__ rows,
                                              uint32_t n_items, uint32_t rows_per_item, u64* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u64 acc = 0;
    for (uint32_t it = blockIdx.x * 4 + wave; it < n_items; it += gridDim.x * 4) {
        const uint32_t slice = it % (W == 8 ? 3 : 2);
        const uint32_t* rl = rows + (size_t)it * rows_per_item;
        for (uint32_t e = 0; e < rows_per_item; e += B) {
            if (W == 8) {
                u64 d[B];
#pragma unroll
                for (int q = 0; q < B; ++q)
                    d[q] = *(const u64*)(buf + (size_t)__builtin_amdgcn_readfirstlane(rl[e + q]) * 1344 + slice * 512 + lane * 8);
#pragma unroll
                for (int q = 0; q < B; ++q) acc ^= d[q];
            } else {
                uint4 d[B];
#pragma unroll
                for (int q = 0; q < B; ++q)
                    d[q] = *(const uint4*)(buf + (size_t)__builtin_amdgcn_readfirstlane(rl[e + q]) * 1344 + slice * 1024 + lane * 16);
#pragma unroll
                for (int q = 0; q < B; ++q) acc ^= ((u64)d[q].x | ((u64)d[q].y << 32)) ^ ((u64)d[q].z | ((u64)d[q].w << 32));
            }
        }
    }
    if (acc == 0x1234567) out[0] = acc;
}

template <int B, int W>
void run(const char* name, const uint8_t* buf, const uint32_t* rows, uint32_t n_items, uint32_t rpi, u64* out, int grid) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    gather<B, W><<<grid, 256>>>(buf, rows, n_items, rpi, out);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) gather<B, W><<<grid, 256>>>(buf, rows, n_items, rpi, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double bytes = 5.0 * n_items * rpi * (W == 8 ? 512.0 : 1024.0);
    printf("%-28s grid %5d: %.1f us/launch, %.2f TB/s requested\n", name, grid, ms * 1e3 / 5, bytes / (ms * 1e-3) / 1e12);
}

int main() {
    const size_t nrows = 1u << 20;  // 1.4 GB of 1344-B rows
    uint8_t* buf;
    hipMalloc(&buf, nrows * 1344 + 4096);
    hipMemset(buf, 1, nrows * 1344 + 4096);
    const uint32_t rpi = 32, n_items = 48000;
    std::vector<uint32_t> h((size_t)n_items * rpi);
    std::mt19937 g(1);
    for (auto& x : h) x = g() % nrows;
    uint32_t* rows;
    hipMalloc(&rows, h.size() * 4);
    hipMemcpy(rows, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    u64* out;
    hipMalloc(&out, 8);
    for (int grid : {1024, 1536, 2048}) {
        run<8, 8>("8B/lane, 8 in flight", buf, rows, n_items, rpi, out, grid);
        run<16, 8>("8B/lane, 16 in flight", buf, rows, n_items, rpi, out, grid);
        run<32, 8>("8B/lane, 32 in flight", buf, rows, n_items, rpi, out, grid);
        run<8, 16>("16B/lane, 8 in flight", buf, rows, n_items, rpi, out, grid);
        run<16, 16>("16B/lane, 16 in flight", buf, rows, n_items, rpi, out, grid);
    }
    // sequential rows (a window's originals) instead of random
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)((i / rpi) * 7 + (i % rpi)) % nrows;
    hipMemcpy(rows, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    run<8, 8>("seq 8B/lane, 8 in flight", buf, rows, n_items, rpi, out, 1536);
    run<16, 16>("seq 16B/lane, 16 in flight", buf, rows, n_items, rpi, out, 1536);
    return 0;
}
