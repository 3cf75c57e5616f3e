// kernels.hip -- CDNA4 (gfx950) kernels of the Siamese engine.
//
// tamd_exec runs one level of a device program (program.h).  Work item = (op, 512-byte slice):
// one 64-lane wave owns 8 bytes per lane of the op's three accumulators and walks the op's
// instruction list (wave-uniform, scalar loads).  GF(2^8) byte multiplication by the
// instruction's coefficient uses three 8-entry product tables per coefficient staged in LDS
// and v_perm_b32 byte lookups (x*c = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6]), so a muladd costs
// ~11 VALU ops per dword and no divergent LDS gathers.  Coefficient 1 is a plain XOR.
// No MFMA: this is GF(2^8) table/XOR work.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "program.h"

#define TAMD_WAVES_PER_WG 4
#define TAMD_LANE_BYTES 8
#define TAMD_BATCH 8    // instructions whose loads are issued together (memory-level parallelism)
#define TAMD_RBATCH 16  // rows of an ACCR run loaded together
static_assert(TAMD_SLICE_BYTES == 64 * TAMD_LANE_BYTES, "one wave covers one slice");

typedef unsigned long long u64;

__device__ __forceinline__ uint32_t gf_mul4(uint32_t x, uint32_t t0lo, uint32_t t0hi, uint32_t t1lo,
                                            uint32_t t1hi, uint32_t t2lo, uint32_t t2hi) {
    const uint32_t s0 = x & 0x07070707u;
    const uint32_t s1 = (x >> 3) & 0x07070707u;
    const uint32_t s2 = (x >> 6) & 0x03030303u;
    return __builtin_amdgcn_perm(t0hi, t0lo, s0) ^ __builtin_amdgcn_perm(t1hi, t1lo, s1) ^
           __builtin_amdgcn_perm(t2hi, t2lo, s2);
}

__device__ __forceinline__ u64 byte_mask(uint32_t nbytes) {  // low `nbytes` bytes set (nbytes < 8)
    return (1ull << (8u * nbytes)) - 1ull;
}

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ u64 gf_mul8(u64 v, uint32_t coef, const uint32_t* __restrict__ lds_perm) {
    const uint32_t* t = &lds_perm[coef * 8u];
    const uint32_t t0lo = t[0], t0hi = t[1], t1lo = t[2], t1hi = t[3], t2lo = t[4], t2hi = t[5];
    const uint32_t lo = gf_mul4((uint32_t)v, t0lo, t0hi, t1lo, t1hi, t2lo, t2hi);
    const uint32_t hi = gf_mul4((uint32_t)(v >> 32), t0lo, t0hi, t1lo, t1hi, t2lo, t2hi);
    return ((u64)hi << 32) | lo;
}

__device__ __forceinline__ void store_slice(uint8_t* __restrict__ arena, const tamd_instr& in, const tamd_instr& f,
                                            uint32_t o, u64 acc) {
    const uint32_t len = in.len, cap = in.cap;
    if (o >= cap) return;
    const u64 footer = ((u64)f.len << 32) | f.row;
    u64 keep;
    if (o + 8u <= len) keep = ~0ull;
    else if (o >= len) keep = 0;
    else keep = byte_mask(len - o);
    u64 fpart = 0;
    if (o >= len) {
        const uint32_t sh = o - len;
        if (sh < 8u) fpart = footer >> (8u * sh);
    } else {
        const uint32_t sh = len - o;
        if (sh < 8u) fpart = footer << (8u * sh);
    }
    *(u64*)(arena + (size_t)in.row * TAMD_ROW_UNIT + o) = (acc & keep) | fpart;
}

// LDS image of the device tables (device.cpp uploads the same layout):
//   [0, 2048)        perm tables, 8 dwords per coefficient (6 used)
//   [2048, 2112)     inv[256] as bytes
//   [2112, 2176)     sqr[256] as bytes
//   [2176, +253*12)  lane table: for i = 0..252 (cx = 3 + i) the 6 perm dwords of cx, then of cx^2
#define TAMD_LDS_INV 2048
#define TAMD_LDS_LANE 2176
#define TAMD_GF_DWORDS (TAMD_LDS_LANE + 253 * 12)

__device__ __forceinline__ uint32_t lds_byte(const uint32_t* __restrict__ lds, uint32_t byte_index) {
    return (lds[byte_index >> 2] >> (8u * (byte_index & 3u))) & 0xffu;
}

__device__ __forceinline__ u64 gf_mul8_t(u64 v, const uint32_t* __restrict__ t) {
    const uint32_t t0lo = t[0], t0hi = t[1], t1lo = t[2], t1hi = t[3], t2lo = t[4], t2hi = t[5];
    const uint32_t lo = gf_mul4((uint32_t)v, t0lo, t0hi, t1lo, t1hi, t2lo, t2hi);
    const uint32_t hi = gf_mul4((uint32_t)(v >> 32), t0lo, t0hi, t1lo, t1hi, t2lo, t2hi);
    return ((u64)hi << 32) | lo;
}

// ACCR: a strided run of rows (program.h).  TAMD_RBATCH row loads are issued together; every
// element's coefficient table is found with one uniform LDS address: lane runs step the column
// value index (cx = 3 + (199*col mod 253)) on the scalar unit and read the precomputed
// (cx, cx^2) tables; Cauchy runs fetch their inverses for the whole batch first.
__device__ __forceinline__ void run_accr(const tamd_instr& a, const tamd_instr& r, uint32_t o,
                                         const uint8_t* __restrict__ arena, const uint32_t* __restrict__ lds,
                                         u64& a0, u64& a1, u64& a2) {
    const uint32_t mode = uniform((a.w0 >> 8) & 0xffu), p = uniform((a.w0 >> 16) & 0xffu);
    const uint32_t row0 = uniform(a.row), len = uniform(a.len), count = uniform(a.cap);
    const uint32_t stride = uniform(r.row), col0 = uniform(r.len), cstep = uniform(r.cap);
    const bool live = o < len;
    const u64 tail = (o + 8u > len && live) ? byte_mask(len - o) : ~0ull;
    uint32_t ci = uniform((199u * (col0 % 253u)) % 253u);     // column value index of element 0
    const uint32_t cstep_i = uniform((199u * (cstep % 253u)) % 253u);
    uint32_t col = col0;
    for (uint32_t e = 0; e < count; e += TAMD_RBATCH) {
        u64 d[TAMD_RBATCH];
#pragma unroll
        for (uint32_t q = 0; q < TAMD_RBATCH; ++q) {
            d[q] = 0;
            if (live && e + q < count)
                d[q] = *(const u64*)(arena + ((size_t)row0 + (size_t)(e + q) * stride) * TAMD_ROW_UNIT + o);
        }
        if (mode == TAMD_R_LANE3) {
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q) {
                if (e + q < count) {
                    const uint32_t* t = lds + TAMD_LDS_LANE + ci * 12u;
                    const u64 x = d[q] & tail;
                    a0 ^= x;
                    a1 ^= gf_mul8_t(x, t);
                    a2 ^= gf_mul8_t(x, t + 6);
                }
                ci += cstep_i;
                if (ci >= 253u) ci -= 253u;
            }
        } else if (mode == TAMD_R_CAUCHY) {
            uint32_t c[TAMD_RBATCH];
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q) {  // CauchyElement(p, col mod 64)
                c[q] = uniform(lds_byte(lds + TAMD_LDS_INV, ((col & 63u) ^ (p + 64u)) & 0xffu));
                col = (col + cstep) & (TAMD_COLUMN_PERIOD - 1u);
            }
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q)
                if (e + q < count) a0 ^= gf_mul8_t(d[q] & tail, lds + c[q] * 8u);
        } else {
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q)
                if (e + q < count) a0 ^= p == 1u ? (d[q] & tail) : gf_mul8_t(d[q] & tail, lds + p * 8u);
        }
    }
}

// Ops of one level never read a row written by an op of the same level, so every ACC load of
// a batch can be issued before the batch's STOREs: TAMD_BATCH loads in flight per wave.
extern "C" __global__ void __launch_bounds__(256)
tamd_exec(const tamd_op* __restrict__ ops, const tamd_instr* __restrict__ instrs,
          const uint2* __restrict__ items, uint32_t n_items, uint8_t* __restrict__ arena,
          const uint32_t* __restrict__ gf_perm) {
    __shared__ uint32_t lds_perm[TAMD_GF_DWORDS];
    for (uint32_t i = threadIdx.x; i < TAMD_GF_DWORDS; i += blockDim.x) lds_perm[i] = gf_perm[i];
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = uniform(threadIdx.x >> 6);
    const uint32_t stride = gridDim.x * TAMD_WAVES_PER_WG;

    for (uint32_t it = blockIdx.x * TAMD_WAVES_PER_WG + wave; it < n_items; it += stride) {
        const uint2 item = items[it];
        const tamd_op op = ops[uniform(item.x)];
        const uint32_t o = uniform(item.y) * TAMD_SLICE_BYTES + lane * TAMD_LANE_BYTES;
        u64 a0 = 0, a1 = 0, a2 = 0;  // the op's three accumulators (program.h)
        const uint32_t first = uniform(op.first), end = uniform(op.first + op.count);
        for (uint32_t k = first; k < end;) {
            tamd_instr in[TAMD_BATCH];
            u64 v[TAMD_BATCH];
            // A batch runs up to (not including) the next ACCR; an ACCR at the head runs alone.
            uint32_t nb = TAMD_BATCH;
#pragma unroll
            for (uint32_t j = 0; j < TAMD_BATCH; ++j) {
                in[j].w0 = 0;
                if (k + j < end) {
                    in[j] = instrs[k + j];
                    if ((in[j].w0 & 0xffu) == TAMD_I_ACCR && j < nb) nb = j;
                }
            }
            if (nb == 0) {
                run_accr(in[0], in[1], o, arena, lds_perm, a0, a1, a2);  // in[1] is its RANGE word
                k += 2;
                continue;
            }
#pragma unroll
            for (uint32_t j = 0; j < TAMD_BATCH; ++j) {
                v[j] = 0;
                const uint32_t kind = in[j].w0 & 0xffu;
                if (j < nb && (kind == TAMD_I_ACC || kind == TAMD_I_ACC3) && o < in[j].len)
                    v[j] = *(const u64*)(arena + (size_t)in[j].row * TAMD_ROW_UNIT + o);
            }
#pragma unroll
            for (uint32_t j = 0; j < TAMD_BATCH; ++j) {
                const uint32_t kind = j < nb ? (in[j].w0 & 0xffu) : 0u;
                if (kind == TAMD_I_ACC) {
                    const uint32_t len = in[j].len;
                    if (o < len) {
                        u64 x = v[j];
                        if (o + 8u > len) x &= byte_mask(len - o);
                        const uint32_t coef = (in[j].w0 >> 8) & 0xffu;
                        if (coef != 1u) x = gf_mul8(x, coef, lds_perm);
                        const uint32_t a = (in[j].w0 >> 16) & 0xffu;
                        if (a == 0) a0 ^= x;
                        else if (a == 1) a1 ^= x;
                        else a2 ^= x;
                    }
                } else if (kind == TAMD_I_ACC3) {
                    const uint32_t len = in[j].len;
                    if (o < len) {
                        u64 x = v[j];
                        if (o + 8u > len) x &= byte_mask(len - o);
                        a0 ^= x;
                        a1 ^= gf_mul8(x, (in[j].w0 >> 8) & 0xffu, lds_perm);
                        a2 ^= gf_mul8(x, (in[j].w0 >> 16) & 0xffu, lds_perm);
                    }
                } else if (kind == TAMD_I_STORE) {
                    // the FOOTER word follows the STORE (possibly in the next batch)
                    const tamd_instr f = (j + 1 < TAMD_BATCH) ? in[j + 1 < TAMD_BATCH ? j + 1 : j] : instrs[k + j + 1];
                    const uint32_t a = (in[j].w0 >> 16) & 0xffu;
                    store_slice(arena, in[j], f, o, a == 0 ? a0 : (a == 1 ? a1 : a2));
                } else if (kind == TAMD_I_STOREC) {
                    const uint32_t w = in[j].w0;
                    const uint32_t c0 = (w >> 8) & 0xffu, c1 = (w >> 16) & 0xffu, c2 = w >> 24;
                    u64 x = 0;
                    if (c0 == 1u) x = a0; else if (c0) x = gf_mul8(a0, c0, lds_perm);
                    if (c1 == 1u) x ^= a1; else if (c1) x ^= gf_mul8(a1, c1, lds_perm);
                    if (c2 == 1u) x ^= a2; else if (c2) x ^= gf_mul8(a2, c2, lds_perm);
                    tamd_instr f;
                    f.w0 = TAMD_I_FOOTER;
                    f.row = f.len = f.cap = 0;
                    store_slice(arena, in[j], f, o, x);
                } else if (kind == TAMD_I_CLEAR) {
                    a0 = a1 = a2 = 0;
                }
            }
            k += nb;
        }
    }
}

// GF self test: out[y * 256 + x] = x * y through the same v_perm path the executor uses.
extern "C" __global__ void tamd_gf_selftest(const uint32_t* __restrict__ gf_perm, uint8_t* __restrict__ out) {
    const uint32_t y = blockIdx.x;
    const uint32_t x4 = threadIdx.x;  // 64 threads x 4 bytes
    const uint32_t* t = &gf_perm[y * 8u];
    const uint32_t xs = (x4 * 4u) | ((x4 * 4u + 1u) << 8) | ((x4 * 4u + 2u) << 16) | ((x4 * 4u + 3u) << 24);
    const uint32_t r = gf_mul4(xs, t[0], t[1], t[2], t[3], t[4], t[5]);
    *(uint32_t*)(out + y * 256u + x4 * 4u) = r;
}

// PCG32 (SiameseTools.h:79-101), used to generate the synthetic payloads on the device.
struct DevPcg {
    u64 state, inc;
    __device__ void seed(u64 y, u64 x) {
        state = 0;
        inc = (y << 1u) | 1u;
        next();
        state += x;
        next();
    }
    __device__ uint32_t next() {
        const u64 old = state;
        state = old * 6364136223846793005ULL + inc;
        const uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
        const uint32_t rot = (uint32_t)(old >> 59);
        return (xs >> rot) | (xs << ((uint32_t)(-(int32_t)rot) & 31u));
    }
};

// Synthetic input rows (tonk_amd/csrc/workload.h payload_bytes): for each descriptor
// {row offset (64-B units), packet index, payload length, row capacity, seed_data}, write
// varint(len) || PCG bytes and zero-fill to the capacity.  One thread per packet (setup only).
struct GenDesc { uint32_t row, index, len, cap; u64 seed; };

extern "C" __global__ void tamd_gen_rows(const GenDesc* __restrict__ d, uint32_t n, uint8_t* __restrict__ arena,
                                          uint32_t row_cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const GenDesc g = d[i];
    uint8_t* dst = arena + (size_t)g.row * TAMD_ROW_UNIT;
    uint8_t hdr[4];
    uint32_t hb;
    const uint32_t len = g.len;
    if (len <= 0x7f) { hdr[0] = (uint8_t)len; hb = 1; }
    else if (len <= 0x3fff) { hdr[0] = (uint8_t)(0x80 | (len >> 8)); hdr[1] = (uint8_t)len; hb = 2; }
    else if (len <= 0x1fffff) { hdr[0] = (uint8_t)(0xC0 | (len >> 16)); hdr[1] = (uint8_t)(len >> 8); hdr[2] = (uint8_t)len; hb = 3; }
    else { hdr[0] = (uint8_t)(0xE0 | (len >> 24)); hdr[1] = (uint8_t)(len >> 16); hdr[2] = (uint8_t)(len >> 8); hdr[3] = (uint8_t)len; hb = 4; }
    for (uint32_t k = 0; k < hb; ++k) dst[k] = hdr[k];
    DevPcg p;
    p.seed(g.seed, g.index);
    uint32_t k = 0;
    for (; k + 4 <= len; k += 4) {
        const uint32_t w = p.next();
        dst[hb + k] = (uint8_t)w; dst[hb + k + 1] = (uint8_t)(w >> 8);
        dst[hb + k + 2] = (uint8_t)(w >> 16); dst[hb + k + 3] = (uint8_t)(w >> 24);
    }
    if (k < len) {
        const uint32_t w = p.next();
        for (uint32_t b = 0; k + b < len; ++b) dst[hb + k + b] = (uint8_t)(w >> (8 * b));
    }
    const uint32_t cap = g.cap < row_cap ? g.cap : row_cap;
    for (uint32_t z = hb + len; z < cap; ++z) dst[z] = 0;
}

// Digest of rows (FNV-1a 64 over `len` bytes starting `skip` bytes into the row): one thread
// per row, for output verification after a timed run (not on the timed path).
struct DigestDesc { uint32_t row, skip, len, pad; };

extern "C" __global__ void tamd_digest_rows(const DigestDesc* __restrict__ d, uint32_t n,
                                             const uint8_t* __restrict__ arena, u64* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const DigestDesc g = d[i];
    const uint8_t* p = arena + (size_t)g.row * TAMD_ROW_UNIT + g.skip;
    u64 h = 1469598103934665603ULL;
    for (uint32_t k = 0; k < g.len; ++k) { h ^= p[k]; h *= 1099511628211ULL; }
    out[i] = h;
}
