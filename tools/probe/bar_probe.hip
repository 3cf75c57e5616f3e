// bar_probe.hip -- TEST ONLY: can the host write device memory directly (large BAR), and how
// fast?  Allocates device memory a few ways, reports whether a host pointer exists, times host
// stores into it and checks a kernel sees them.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <chrono>
#include <vector>
#include <immintrin.h>

__global__ void sum_kernel(const uint32_t* p, size_t n, unsigned long long* out) {
    unsigned long long s = 0;
    for (size_t i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
    atomicAdd(out, s);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void try_one(const char* name, void* dev, void* host, size_t bytes) {
    printf("%s: dev %p host %p\n", name, dev, host);
    if (!host) return;
    std::vector<uint32_t> src(bytes / 4);
    for (size_t i = 0; i < src.size(); ++i) src[i] = (uint32_t)i;
    for (size_t chunk : {(size_t)2048, (size_t)49152, bytes}) {
        double best = 1e30;
        for (int r = 0; r < 20; ++r) {
            const double t0 = now_us();
            memcpy(host, src.data(), chunk);
            _mm_sfence();
            const double t = now_us() - t0;
            if (t < best) best = t;
        }
        printf("  host memcpy %zu B: %.2f us (%.2f GB/s)\n", chunk, best, chunk / best * 1e-3);
    }
    // read-back latency from the host (uncached?)
    {
        volatile uint32_t* v = (volatile uint32_t*)host;
        const double t0 = now_us();
        uint32_t x = 0;
        for (int i = 0; i < 100; ++i) x += v[i * 1024];
        printf("  host read x100: %.2f us each (x=%u)\n", (now_us() - t0) / 100, x);
    }
    unsigned long long* out;
    hipMalloc(&out, 8);
    hipMemset(out, 0, 8);
    hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, 0, (const uint32_t*)dev, bytes / 4, out);
    unsigned long long got = 0;
    hipMemcpy(&got, out, 8, hipMemcpyDeviceToHost);
    unsigned long long want = 0;
    for (size_t i = 0; i < bytes / 4; ++i) want += (uint32_t)i;
    printf("  kernel sum %s (%llu vs %llu)\n", got == want ? "ok" : "MISMATCH", got, want);
    hipFree(out);
}

int main() {
    const size_t bytes = 1 << 20;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    printf("device %s, large BAR? pciBus %d\n", prop.gcnArchName, prop.pciBusID);
    {
        void* p = nullptr;
        hipError_t e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained);
        printf("hipExtMallocWithFlags(fine): %s\n", hipGetErrorString(e));
        if (e == hipSuccess) {
            hipPointerAttribute_t a;
            memset(&a, 0, sizeof(a));
            hipPointerGetAttributes(&a, p);
            printf("  attr type %d hostPointer %p devicePointer %p\n", (int)a.type, a.hostPointer, a.devicePointer);
            try_one("fine-grained device (same pointer)", p, p, bytes);
        }
    }
    {
        void* p = nullptr;
        hipError_t e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
        printf("hipExtMallocWithFlags(uncached): %s\n", hipGetErrorString(e));
        if (e == hipSuccess) try_one("uncached device (same pointer)", p, p, bytes);
    }
    {
        void* p = nullptr;
        hipError_t e = hipMallocManaged(&p, bytes);
        printf("hipMallocManaged: %s\n", hipGetErrorString(e));
        if (e == hipSuccess) {
            hipMemAdvise(p, bytes, hipMemAdviseSetPreferredLocation, 0);
            hipMemPrefetchAsync(p, bytes, 0, 0);
            hipDeviceSynchronize();
            try_one("managed, preferred on device", p, p, bytes);
        }
    }
    return 0;
}
