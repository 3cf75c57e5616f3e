// bar_coherence.hip -- TEST ONLY: host writes into fine-grained device memory (hipExtMallocWithFlags
// hipDeviceMallocFinegrained, host-writable through the BAR) read by a persistent kernel.
// Protocol as the C ABI would use it: the host rewrites a 49 KB "staging" area and a 2 KB
// "command" in device memory, sfence, then bumps a sequence word (also in device memory); the
// kernel (one workgroup, polling the word with system-scope loads) sums the staging with PLAIN
// 16-byte loads and the command with system-scope loads, and writes both sums to host memory.
// Any stale line (an L2 copy of an earlier round) shows as a wrong sum.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <chrono>
#include <immintrin.h>

struct Host { unsigned long long seq_seen, sum_plain, sum_sys, pad[5]; };

__global__ void poll_kernel(const uint32_t* stage, const uint64_t* cmd, const uint64_t* seq, Host* out, int rounds,
                            size_t n_stage, size_t n_cmd) {
    __shared__ unsigned long long s_plain, s_sys;
    __shared__ unsigned long long s_seq;
    for (int r = 1; r <= rounds; ++r) {
        if (threadIdx.x == 0) {
            unsigned long long v;
            long spins = 0;
            do {
                v = __hip_atomic_load((uint64_t*)seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            } while (v < (unsigned long long)r && ++spins < 200000000L);
            s_seq = v;
            s_plain = 0;
            s_sys = 0;
            asm volatile("buffer_inv sc1" ::: "memory");
        }
        __syncthreads();
        if (s_seq < (unsigned long long)r) return;  // (host stopped: exit)
        unsigned long long a = 0, b = 0;
        for (size_t i = threadIdx.x; i < n_stage / 4; i += blockDim.x) {
            const uint4 v = ((const uint4*)stage)[i];
            a += (unsigned long long)v.x + v.y + v.z + v.w;
        }
        for (size_t i = threadIdx.x; i < n_cmd; i += blockDim.x)
            b += __hip_atomic_load((uint64_t*)(cmd + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        atomicAdd(&s_plain, a);
        atomicAdd(&s_sys, b);
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_store(&out->sum_plain, s_plain, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&out->sum_sys, s_sys, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __atomic_thread_fence(__ATOMIC_RELEASE);
            __hip_atomic_store(&out->seq_seen, (unsigned long long)r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
    }
}

int main() {
    const size_t stage_bytes = 49152, cmd_words = 256;
    uint32_t* stage = nullptr;
    uint64_t *cmd = nullptr, *seq = nullptr;
    if (hipExtMallocWithFlags((void**)&stage, stage_bytes, hipDeviceMallocFinegrained) != hipSuccess ||
        hipExtMallocWithFlags((void**)&cmd, cmd_words * 8, hipDeviceMallocFinegrained) != hipSuccess ||
        hipExtMallocWithFlags((void**)&seq, 64, hipDeviceMallocFinegrained) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    Host* out = nullptr;
    hipHostMalloc((void**)&out, sizeof(Host), hipHostMallocMapped | hipHostMallocCoherent);
    memset(out, 0, sizeof(Host));
    *(volatile uint64_t*)seq = 0;
    _mm_sfence();
    const int rounds = 2000;
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipLaunchKernelGGL(poll_kernel, dim3(1), dim3(256), 0, st, stage, cmd, seq, out, rounds, stage_bytes / 4, cmd_words);
    int bad_plain = 0, bad_sys = 0;
    double lat_sum = 0, lat_max = 0;
    for (int r = 1; r <= rounds; ++r) {
        // new contents (a different value every round)
        uint32_t tmp[stage_bytes / 4];
        unsigned long long want_plain = 0, want_sys = 0;
        for (size_t i = 0; i < stage_bytes / 4; ++i) {
            tmp[i] = (uint32_t)(i * 2654435761u + r * 97u);
            want_plain += tmp[i];
        }
        uint64_t c[cmd_words];
        for (size_t i = 0; i < cmd_words; ++i) {
            c[i] = (uint64_t)r * 1000003ull + i;
            want_sys += c[i];
        }
        const auto t0 = std::chrono::steady_clock::now();
        memcpy(stage, tmp, stage_bytes);
        memcpy(cmd, c, sizeof(c));
        _mm_sfence();
        *(volatile uint64_t*)seq = (uint64_t)r;
        _mm_sfence();
        long spins = 0;
        while (__atomic_load_n(&out->seq_seen, __ATOMIC_ACQUIRE) < (unsigned long long)r && ++spins < 2000000000L) _mm_pause();
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        lat_sum += us;
        if (us > lat_max) lat_max = us;
        if (out->sum_plain != want_plain) ++bad_plain;
        if (out->sum_sys != want_sys) ++bad_sys;
        if (out->seq_seen < (unsigned long long)r) { printf("timeout at round %d\n", r); break; }
    }
    hipStreamSynchronize(st);
    printf("rounds %d: stale plain-load sums %d, stale system-scope sums %d; host round trip mean %.2f us max %.2f us\n",
           rounds, bad_plain, bad_sys, lat_sum / rounds, lat_max);
    return 0;
}
