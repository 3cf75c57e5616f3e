// h2d_probe.hip -- measures how long hipMemcpyAsync H2D from pinned memory blocks the caller
// (enqueue time) for program-sized transfers, while a kernel is running on the stream.
#include <hip/hip_runtime.h>
#include <chrono>
#include <stdio.h>
#include <string.h>

__global__ void spin(unsigned long long cycles) {
    const unsigned long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
}

int main() {
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    const size_t sizes[] = {1 << 16, 1 << 20, 4 << 20, 8 << 20, 16 << 20};
    for (int mode = 0; mode < 2; ++mode) {
        for (size_t n : sizes) {
            void* h = nullptr;
            void* d = nullptr;
            if (mode == 0) hipHostMalloc(&h, n, hipHostMallocDefault);
            else hipHostMalloc(&h, n, hipHostMallocNonCoherent);
            hipMalloc(&d, n);
            memset(h, 1, n);
            double best = 1e9, total = 0;
            for (int rep = 0; rep < 5; ++rep) {
                hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, st, 2000000ull);  // ~1 ms
                const auto t0 = std::chrono::steady_clock::now();
                hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st);
                const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                hipStreamSynchronize(st);
                const auto t1 = std::chrono::steady_clock::now();
                hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st);
                hipStreamSynchronize(st);
                total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
                if (ms < best) best = ms;
            }
            printf("mode=%s bytes=%zu enqueue_ms=%.3f copy_ms=%.3f\n", mode ? "noncoherent" : "default", n, best, total);
            hipHostFree(h);
            hipFree(d);
        }
    }
    return 0;
}
