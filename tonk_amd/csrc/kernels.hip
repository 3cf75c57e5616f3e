// kernels.hip -- CDNA4 (gfx950) kernels of the Siamese engine.
//
// tamd_exec16 runs one level of a device program (program.h).  A work item is one op over a
// 1024-byte slice of its rows: one 64-lane wave owns 16 bytes per lane of the op's three
// accumulators and walks the op's instruction list (wave-uniform, scalar loads).  GF(2^8)
// multiplication by a wave-uniform coefficient uses three 8-entry product tables per
// coefficient staged in LDS and v_perm_b32 byte lookups (x*c = T0[x&7] ^ T1[(x>>3)&7] ^
// T2[x>>6]): ~11 VALU ops per dword, no divergent LDS gathers.  Coefficient 1 is a plain XOR.
// No MFMA: this is GF(2^8) table/XOR work.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "program.h"
#include "serve.h"

#define TAMD_WAVES_PER_WG 4
#ifndef TAMD_BITOP3
#define TAMD_BITOP3 1  // three-input XORs as v_bitop3_b32 (mul_sel)
#endif
#ifndef TAMD_ROLL
#define TAMD_ROLL 1  // rolling row loads in ACCR runs (run_accr)
#endif

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
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ u64 ballot(bool p) { return __builtin_amdgcn_uicmp((uint32_t)p, 0u, 33 /*ne*/); }

// An instruction word of the op's list.  LDSI: the list sits in LDS (the persistent C-ABI
// executor, tamd_serve, copies each command's program there); its fields are wave uniform, so
// they move to SGPRs and every row address keeps its scalar base.  Otherwise a scalar load.
template <bool LDSI>
__device__ __forceinline__ tamd_instr fetch_instr(const tamd_instr* __restrict__ p, uint32_t i) {
    if constexpr (!LDSI) {
        return p[i];
    } else {
        const uint4 v = *(const uint4*)(p + i);
        tamd_instr r;
        r.w0 = uniform(v.x);
        r.row = uniform(v.y);
        r.len = uniform(v.z);
        r.cap = uniform(v.w);
        return r;
    }
}

// A wave-uniform value moved into a VGPR: LDS addresses built from it need no v_readfirstlane /
// v_mov round trip.
__device__ __forceinline__ uint32_t vgpr(uint32_t s) {
    uint32_t v;
    asm("v_mov_b32 %0, %1" : "=v"(v) : "s"(s));
    return v;
}

// Bytes of this lane's 8 that lie below `len` (FULL: the whole slice does).
template <bool FULL>
__device__ __forceinline__ u64 keep_mask(uint32_t o, uint32_t len) {
    if (FULL) return ~0ull;
    if (o + 8u <= len) return ~0ull;
    if (o >= len) return 0ull;
    return byte_mask(len - o);
}

// Offset of this lane's load inside a row of `len` bytes: lanes past the end read the row's
// first bytes (a valid address) and mask them to zero, so no load is exec-masked.
template <bool FULL>
__device__ __forceinline__ uint32_t load_off(uint32_t o, uint32_t len) { return (FULL || o < len) ? o : 0u; }

// row[len, len + 8) = footer, row[len + 8, cap) = 0 around acc (one lane's 8 bytes at offset o).
// An 8-byte arena store; WT: write-through (an agent-scope relaxed atomic store, `sc1`), so the
// row is visible to every CU and XCD once the storing wave has drained (the persistent C-ABI
// executor's commands need no L2 write-back fence for the next command of the codec).
template <bool WT>
__device__ __forceinline__ void st_u64(uint8_t* p, u64 v) {
    if constexpr (WT) __hip_atomic_store((u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *(u64*)p = v;
}

template <bool WT = false>
__device__ __forceinline__ void store_slice(uint8_t* __restrict__ arena, uint32_t row, uint32_t len, uint32_t cap,
                                            u64 footer, uint32_t o, u64 acc) {
    if (o >= cap) return;
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
    st_u64<WT>(arena + (size_t)row * TAMD_ROW_UNIT + o, (acc & keep) | fpart);
}

// LDS image of the device tables (device.cpp uploads the same layout):
//   [0, 2048)        perm tables, 8 dwords per coefficient (6 used)
//   [2048, 2112)     inv[256] as bytes
//   [2112, 2176)     sqr[256] as bytes
//   [2176, +253*12)  lane table: for i = 0..252 (cx = 3 + i) the 6 perm dwords of cx, then of cx^2
//   [5212, +192*8)   Cauchy table: for x = 64..255 the perm tables of inv(x) (CauchyElement(p, c)
//                    = inv(c ^ (p + 64)) in one lookup instead of two dependent ones)
#define TAMD_LDS_INV 2048
#define TAMD_LDS_LANE 2176
#define TAMD_LDS_CINV (TAMD_LDS_LANE + 253 * 12)  // 5212, a multiple of 4
#define TAMD_GF_DWORDS (TAMD_LDS_CINV + 192 * 8)  // 6748

// v_perm product tables of one coefficient from LDS (6 dwords at a 16-byte aligned address).
struct PermT { uint32_t t[6]; };
__device__ __forceinline__ PermT perm_at(const uint32_t* __restrict__ lds, uint32_t dword_index) {
    PermT p;
    const uint4 a = *(const uint4*)(lds + dword_index);
    const uint2 b = *(const uint2*)(lds + dword_index + 4);
    p.t[0] = a.x; p.t[1] = a.y; p.t[2] = a.z; p.t[3] = a.w; p.t[4] = b.x; p.t[5] = b.y;
    return p;
}
// The same for tables at an 8-byte (not 16-byte) aligned address: the cx^2 half of a lane entry.
__device__ __forceinline__ PermT perm_at_hi(const uint32_t* __restrict__ lds, uint32_t dword_index) {
    PermT p;
    const uint2 a = *(const uint2*)(lds + dword_index);
    const uint4 b = *(const uint4*)(lds + dword_index + 2);
    p.t[0] = a.x; p.t[1] = a.y; p.t[2] = b.x; p.t[3] = b.y; p.t[4] = b.z; p.t[5] = b.w;
    return p;
}

// Selectors of x shared by every product of x (ACC3 multiplies one row by two coefficients).
struct Sel { uint32_t s0, s1, s2; };
__device__ __forceinline__ Sel sel4(uint32_t x) {
    Sel s;
    s.s0 = x & 0x07070707u;
    s.s1 = (x >> 3) & 0x07070707u;
    s.s2 = (x >> 6) & 0x03030303u;
    return s;
}
// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96); the compiler emits two v_xor_b32.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if TAMD_BITOP3
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return a ^ b ^ c;
#endif
}
__device__ __forceinline__ uint32_t mul_sel(const Sel& s, const PermT& p) {
    return xor3(__builtin_amdgcn_perm(p.t[1], p.t[0], s.s0), __builtin_amdgcn_perm(p.t[3], p.t[2], s.s1),
                __builtin_amdgcn_perm(p.t[5], p.t[4], s.s2));
}
__device__ __forceinline__ u64 mul8(u64 x, const PermT& p) {
    const Sel lo = sel4((uint32_t)x), hi = sel4((uint32_t)(x >> 32));
    return ((u64)mul_sel(hi, p) << 32) | mul_sel(lo, p);
}

// A lane's bytes of a slice: NH 8-byte words.  NH = 1: 8 B per lane, 512-byte slices; NH = 2:
// 16 B per lane, 1024-byte slices, one dwordx4 load per row (a 1302-byte row is two work items
// instead of three, so the instruction walk, coefficient-table reads and selector math of an
// item cover twice the bytes).
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
template <int NH>
struct LV {
    u64 h[NH];
    __device__ __forceinline__ LV& operator^=(const LV& b) {
#pragma unroll
        for (int i = 0; i < NH; ++i) h[i] ^= b.h[i];
        return *this;
    }
};
template <int NH>
__device__ __forceinline__ LV<NH> lv_zero() {
    LV<NH> r;
#pragma unroll
    for (int i = 0; i < NH; ++i) r.h[i] = 0;
    return r;
}
// NH = 3: a 1536-byte slice, 16 B per lane at `o` (the slice's first 1024 bytes) and 8 B per lane
// at `ox` = slice + 1024 + 8 * lane (its last 512): one wave covers a whole 1302-byte packet row,
// one dwordx4 and one dwordx2 load per row, instead of a 1024-byte item plus a tail item that
// repeats the instruction walk and memory round trips for 278 bytes.  `px` is the row's address
// at ox (unused for NH < 3).
template <int NH>
__device__ __forceinline__ LV<NH> lv_load(const uint8_t* p, const uint8_t* px = nullptr) {
    LV<NH> r;
    if constexpr (NH == 1) {
        r.h[0] = *(const u64*)p;
    } else {
        const u64x2 t = *(const u64x2*)p;
        r.h[0] = t.x;
        r.h[1] = t.y;
        if constexpr (NH == 3) r.h[2] = *(const u64*)px;
    }
    return r;
}
// The same from a wave-uniform row base and the lane's offsets (scalar-base addressing).
template <int NH>
__device__ __forceinline__ LV<NH> lv_load_at(const uint8_t* base, uint32_t off, uint32_t offx) {
    // (the empty asm keeps the 32-bit offsets from being widened once outside the loop, which
    // would turn every load into a 64-bit per-lane address add)
    asm volatile("" : "+v"(off));
    if constexpr (NH == 3) asm volatile("" : "+v"(offx));
    return lv_load<NH>(base + off, base + offx);
}
template <int NH>
__device__ __forceinline__ void lv_store(uint8_t* p, const LV<NH>& v) {
    if constexpr (NH == 1) {
        *(u64*)p = v.h[0];
    } else {
        u64x2 t;
        t.x = v.h[0];
        t.y = v.h[1];
        *(u64x2*)p = t;
    }
}
// x with the bytes at or past `len` cleared (lane bytes start at offset o)
// (NH = 3: FULL covers the 16-byte part only; the extension word is always masked)
template <bool FULL, int NH>
__device__ __forceinline__ LV<NH> lv_keep(LV<NH> x, uint32_t o, uint32_t len, uint32_t ox = 0) {
    if (!FULL) {
#pragma unroll
        for (int i = 0; i < (NH < 3 ? NH : 2); ++i) x.h[i] &= keep_mask<false>(o + 8u * i, len);
    }
    if constexpr (NH == 3) x.h[2] &= keep_mask<false>(ox, len);
    return x;
}
template <int NH>
__device__ __forceinline__ LV<NH> lv_mul(const LV<NH>& x, const PermT& p) {
    LV<NH> r;
#pragma unroll
    for (int i = 0; i < NH; ++i) r.h[i] = mul8(x.h[i], p);
    return r;
}
// acc_0 ^= x, acc_1 ^= c1 * x, acc_2 ^= c2 * x (one lane running-sum step, selectors shared)
template <int NH>
__device__ __forceinline__ void lv_acc3(const LV<NH>& x, const PermT& c1, const PermT& c2, LV<NH>& a0, LV<NH>& a1,
                                        LV<NH>& a2) {
#pragma unroll
    for (int i = 0; i < NH; ++i) {
        const Sel lo = sel4((uint32_t)x.h[i]), hi = sel4((uint32_t)(x.h[i] >> 32));
        a0.h[i] ^= x.h[i];
        a1.h[i] ^= ((u64)mul_sel(hi, c1) << 32) | mul_sel(lo, c1);
        a2.h[i] ^= ((u64)mul_sel(hi, c2) << 32) | mul_sel(lo, c2);
    }
}
template <bool FULL, int NH, bool WT = false>
__device__ __forceinline__ void lv_store_row(uint8_t* __restrict__ arena, uint32_t row, uint32_t len, uint32_t cap,
                                             u64 footer, uint32_t o, const LV<NH>& x, uint32_t ox = 0) {
    constexpr int NM = NH < 3 ? NH : 2;
    if (FULL) {
        if constexpr (NH == 3 && WT) {
            st_u64<true>(arena + (size_t)row * TAMD_ROW_UNIT + o, x.h[0]);
            st_u64<true>(arena + (size_t)row * TAMD_ROW_UNIT + o + 8u, x.h[1]);
        } else if constexpr (NH == 3) {
            u64x2 t;
            t.x = x.h[0];
            t.y = x.h[1];
            *(u64x2*)(arena + (size_t)row * TAMD_ROW_UNIT + o) = t;
        } else {
            lv_store<NH>(arena + (size_t)row * TAMD_ROW_UNIT + o, x);
        }
    } else {
#pragma unroll
        for (int i = 0; i < NM; ++i) store_slice<WT>(arena, row, len, cap, footer, o + 8u * i, x.h[i]);
    }
    if constexpr (NH == 3) store_slice<WT>(arena, row, len, cap, footer, ox, x.h[2]);
}

// Rolling row loads over one wave's batches of a run: batch b (rows b*R .. b*R + R - 1) is
// this wave's when (unit + b) mod nw == wid -- every batch when the wave runs the op alone, every
// nw-th when nw waves share it.  The rows of the wave's next batch are loaded as soon as a half of
// the current one has been combined, so a wave keeps 3-6 row loads in flight while it computes
// instead of waiting a full memory round trip per batch.  body(i, v): row i's slice bytes.
template <bool FULL, int NH, uint32_t R, class F>
__device__ __forceinline__ void roll_rows(const uint8_t* rbase, size_t step, uint32_t lo, uint32_t lox,
                                          uint32_t count, uint32_t o, uint32_t len, uint32_t ox, uint32_t& unit,
                                          uint32_t nw, uint32_t wid, F&& body) {
    const uint32_t nbat = (count + R - 1) / R;
    const uint32_t b0 = (wid - unit) & (nw - 1u), jump = nw * R;
    unit += nbat;
    if (b0 >= nbat) return;
    constexpr uint32_t H = R / 2;
    LV<NH> d[R];
    uint32_t e = b0 * R;
#pragma unroll
    for (uint32_t q = 0; q < R; ++q) d[q] = lv_load_at<NH>(rbase + (size_t)min(e + q, count - 1u) * step, lo, lox);
    for (; e < count; e += jump) {
        const bool more = e + jump < count;
#pragma unroll
        for (uint32_t h = 0; h < 2; ++h) {
#pragma unroll
            for (uint32_t q = h * H; q < (h ? R : H); ++q)
                if (e + q < count) body(e + q, lv_keep<FULL, NH>(d[q], o, len, ox));
            if (more) {
#pragma unroll
                for (uint32_t q = h * H; q < (h ? R : H); ++q)
                    d[q] = lv_load_at<NH>(rbase + (size_t)min(e + jump + q, count - 1u) * step, lo, lox);
            }
        }
    }
}

// ACCR: a strided run of equally long rows (program.h).  TAMD_RBATCH row loads are issued
// together (the row index is clamped to the run, so no load is branched around); the per-row
// table address stepping runs on the vector ALU: lane runs step the column value index
// (cx = 3 + (199 col mod 253)) through the lane table, Cauchy runs fetch their inverses for the
// whole batch first.
// Batches of rows are numbered across the op (`unit`); with nw > 1 waves sharing the op, a
// wave combines only the batches with unit mod nw == wid (the coefficient stepping still walks
// every row).
template <bool FULL, int NH, uint32_t TAMD_RBATCH, bool LDSI = false>
__device__ __forceinline__ void run_accr(const tamd_instr& a, const tamd_instr& r, const tamd_instr& tg,
                                         const tamd_instr* __restrict__ adj, uint32_t o, uint32_t ox,
                                         const uint8_t* __restrict__ arena, const uint32_t* __restrict__ lds,
                                         uint32_t& unit, uint32_t nw, uint32_t wid, LV<NH>& a0, LV<NH>& a1,
                                         LV<NH>& a2) {
    const uint32_t mode = (a.w0 >> 8) & 0xffu, p = (a.w0 >> 16) & 0xffu;
    const uint32_t row0 = a.row, len = a.len, count = a.cap;
    const uint32_t stride = r.row, col0 = r.len, cstep = r.cap;
    // a row's address: a wave-uniform base (SGPRs) plus the lane's 32-bit offsets, so the loads
    // use the scalar-base addressing mode and no 64-bit per-lane address math per row
    const uint8_t* rbase = arena + (size_t)row0 * TAMD_ROW_UNIT;
    const uint32_t lo = load_off<FULL>(o, len), lox = NH == 3 ? load_off<false>(ox, len) : 0u;
    const size_t step = (size_t)stride * TAMD_ROW_UNIT;
#define TAMD_RUN_LD(idx) lv_load_at<NH>(rbase + (size_t)(idx) * step, lo, lox)
    // loads past the run's end re-read its last row (never consumed)
#define TAMD_RUN_ROW(q) TAMD_RUN_LD(min(e + (q), count - 1u))
    if (mode == TAMD_R_LANE3) {
        // byte offset of the (cx, cx^2) tables in the lane table: 48 bytes per column value index
        const uint32_t W = 253u * 48u;
        uint32_t t = vgpr(((199u * (col0 % 253u)) % 253u) * 48u);
        const uint32_t tstep = vgpr(((199u * (cstep % 253u)) % 253u) * 48u);
        if (TAMD_ROLL && nw == 1u) {
            // Rolling loads: the rows of the next batch half are loaded as soon as a half has been
            // combined, so a wave keeps 3-6 row loads in flight while it computes instead of
            // waiting a full memory round trip per batch (same registers as a plain batch).
            constexpr uint32_t H = TAMD_RBATCH / 2;
            LV<NH> d[TAMD_RBATCH];
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q) d[q] = TAMD_RUN_LD(min(q, count - 1u));
            for (uint32_t e = 0; e < count; e += TAMD_RBATCH) {
                const bool more = e + TAMD_RBATCH < count;
#pragma unroll
                for (uint32_t h = 0; h < 2; ++h) {
#pragma unroll
                    for (uint32_t q = h * H; q < (h ? TAMD_RBATCH : H); ++q) {
                        if (e + q < count) {
                            const uint32_t ti = TAMD_LDS_LANE + (t >> 2);
                            const PermT c1 = perm_at(lds, ti), c2 = perm_at_hi(lds, ti + 6u);
                            lv_acc3<NH>(lv_keep<FULL, NH>(d[q], o, len, ox), c1, c2, a0, a1, a2);
                            t += tstep;
                            t = min(t, t - W);
                        }
                    }
                    if (more) {
#pragma unroll
                        for (uint32_t q = h * H; q < (h ? TAMD_RBATCH : H); ++q)
                            d[q] = TAMD_RUN_LD(min(e + TAMD_RBATCH + q, count - 1u));
                    }
                }
            }
            unit += (count + TAMD_RBATCH - 1) / TAMD_RBATCH;
            return;
        }
        for (uint32_t e = 0; e < count; e += TAMD_RBATCH) {
            if ((unit++ & (nw - 1u)) != wid) {
#pragma unroll
                for (uint32_t q = 0; q < TAMD_RBATCH; ++q) {
                    t += tstep;
                    t = min(t, t - W);
                }
                continue;
            }
            LV<NH> d[TAMD_RBATCH];
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q) d[q] = TAMD_RUN_ROW(q);
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q) {
                if (e + q < count) {
                    const uint32_t ti = TAMD_LDS_LANE + (t >> 2);
                    const PermT c1 = perm_at(lds, ti), c2 = perm_at_hi(lds, ti + 6u);
                    lv_acc3<NH>(lv_keep<FULL, NH>(d[q], o, len, ox), c1, c2, a0, a1, a2);
                    t += tstep;
                    t = min(t, t - W);  // t - W wraps above t while t < W
                }
            }
        }
    } else if (mode == TAMD_R_MULTI) {
        // Up to three Cauchy / parity rows over overlapping windows: row i of the run goes to
        // every target a with lo_a <= i < hi_a, loaded once (the op is never shared: nw == 1).
        uint32_t col = vgpr(col0);
        const uint32_t cs = vgpr(cstep);
        const uint32_t w0 = tg.row, w1 = tg.len, w2 = tg.cap;
        // target a takes rows lo_a <= i < hi_a: (i - lo_a) < n_a, unsigned
        const uint32_t l0 = (w0 >> 10) & 0x7ffu, l1 = (w1 >> 10) & 0x7ffu, l2 = (w2 >> 10) & 0x7ffu;
        const uint32_t h0 = (w0 >> 21) - l0, h1 = (w1 >> 21) - l1, h2 = (w2 >> 21) - l2;
        const uint32_t x0 = ((w0 >> 2) & 0xffu) + 64u, x1 = ((w1 >> 2) & 0xffu) + 64u, x2 = ((w2 >> 2) & 0xffu) + 64u;
        const bool k0 = (w0 & 3u) == TAMD_R_CONST, k1 = (w1 & 3u) == TAMD_R_CONST, k2 = (w2 & 3u) == TAMD_R_CONST;
        constexpr uint32_t H = TAMD_RBATCH / 2;
        LV<NH> d[TAMD_RBATCH];
#pragma unroll
        for (uint32_t q = 0; q < TAMD_RBATCH; ++q) d[q] = TAMD_RUN_LD(min(q, count - 1u));
#define TAMD_MULTI_TARGET(l, h, k, x, acc)                                                 \
    if (i - l < h) {                                                                       \
        if (k) acc ^= v;                                                                   \
        else acc ^= lv_mul<NH>(v, perm_at(lds, TAMD_LDS_CINV - 512u + (((col & 63u) ^ x) << 3)));  \
    }
        for (uint32_t e = 0; e < count; e += TAMD_RBATCH) {
            const bool more = e + TAMD_RBATCH < count;
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
#pragma unroll
                for (uint32_t q = h * H; q < (h ? TAMD_RBATCH : H); ++q) {
                    const uint32_t i = e + q;
                    if (i < count) {
                        const LV<NH> v = lv_keep<FULL, NH>(d[q], o, len, ox);
                        TAMD_MULTI_TARGET(l0, h0, k0, x0, a0)
                        TAMD_MULTI_TARGET(l1, h1, k1, x1, a1)
                        TAMD_MULTI_TARGET(l2, h2, k2, x2, a2)
                    }
                    col += cs;
                }
                if (more) {
#pragma unroll
                    for (uint32_t q = h * H; q < (h ? TAMD_RBATCH : H); ++q)
                        d[q] = TAMD_RUN_LD(min(e + TAMD_RBATCH + q, count - 1u));
                }
            }
        }
#undef TAMD_MULTI_TARGET
        unit += (count + TAMD_RBATCH - 1) / TAMD_RBATCH;
        return;
    } else if (!LDSI && mode == TAMD_R_DENSE && p > 1u) {  // (not in tamd_serve: Server::build)
        // p (2 or 3) Siamese rows of one encoder over nested sum ranges (program.h DENSE with
        // targets): every packet of the run is loaded once and multiplied by each target's
        // coefficient; target t takes rows i < hi_t into acc_t.  Coefficients as for one target
        // (below), 64 rows at a time, the column value shared by the targets.
        const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        const uint8_t* sqr = (const uint8_t*)(lds + TAMD_LDS_INV + 64u);
        // COEFS_t and its ADJ words: COEFS_0 is `tg`, the others follow the previous one's ADJ
        const uint32_t n0 = tg.cap & 0xffffu;
        const tamd_instr c1 = fetch_instr<LDSI>(adj, n0);
        const uint32_t n1 = c1.cap & 0xffffu;
        const tamd_instr c2 = p > 2u ? fetch_instr<LDSI>(adj, n0 + 1u + n1) : c1;
        const uint32_t n2 = p > 2u ? c2.cap & 0xffffu : 0u;
        const uint32_t* __restrict__ ad0 = (const uint32_t*)adj;
        const uint32_t* __restrict__ ad1 = (const uint32_t*)(adj + n0 + 1u);
        const uint32_t* __restrict__ ad2 = (const uint32_t*)(adj + n0 + n1 + 2u);
        const uint32_t hi0 = tg.cap >> 16, hi1 = c1.cap >> 16, hi2 = p > 2u ? c2.cap >> 16 : 0u;
        uint32_t cur0 = 0, cur1 = 0, cur2 = 0, gv0 = 0, gv1 = 0, gv2 = 0, gblk = ~0u;
        // lane j's table indices for row 64 * gblk + j, one per target
        auto block = [&](uint32_t i) __attribute__((always_inline)) {
            gblk = i >> 6;
            const uint32_t base = i & ~63u, mine = base + lane;
            const uint32_t c = (col0 + mine * cstep) & (TAMD_COLUMN_PERIOD - 1u);
            const uint32_t cx = 3u + (199u * (c % 253u)) % 253u, cx2 = sqr[cx], sh = 6u * (c & 7u);
            // (the rx tables are read here, once per 64 rows, not kept across the rows)
            auto one = [&](const tamd_instr& cw, const uint32_t* __restrict__ ad, uint32_t nadj,
                           uint32_t& cur) __attribute__((always_inline)) -> uint32_t {
                const PermT prx = perm_at(lds, ((cw.len >> 16) & 0xffu) * 8u);
                const u64 opw = (u64)cw.row | ((u64)(cw.len & 0xffffu) << 32);
                const uint32_t b = (uint32_t)(opw >> sh) & 63u;
                const uint32_t sd = (b & 1u) ^ ((b & 2u) ? cx : 0u) ^ ((b & 4u) ? cx2 : 0u);
                const uint32_t tp = ((b >> 3) & 1u) ^ ((b & 16u) ? cx : 0u) ^ ((b & 32u) ? cx2 : 0u);
                uint32_t g = (sd ^ mul_sel(sel4(tp), prx)) & 0xffu;
                for (; cur < 4u * nadj; ++cur) {
                    const uint32_t d = LDSI ? uniform(ad[cur]) : ad[cur];
                    if ((d >> 16) >= base + 64u) break;
                    if ((d >> 16) == mine) g ^= (d >> 8) & 0xffu;
                }
                return g * 8u;
            };
            gv0 = one(tg, ad0, n0, cur0);
            gv1 = one(c1, ad1, n1, cur1);
            if (p > 2u) gv2 = one(c2, ad2, n2, cur2);
        };
        // row i (its slice bytes v) into every target whose range holds it, one product table
        // live at a time
        auto row = [&](uint32_t i, const LV<NH>& v) __attribute__((always_inline)) {
            if ((i >> 6) != gblk) block(i);
            const int l = (int)(i & 63u);
            if (i < hi0) a0 ^= lv_mul<NH>(v, perm_at(lds, (uint32_t)__builtin_amdgcn_readlane((int)gv0, l)));
            if (i < hi1) a1 ^= lv_mul<NH>(v, perm_at(lds, (uint32_t)__builtin_amdgcn_readlane((int)gv1, l)));
            if (i < hi2) a2 ^= lv_mul<NH>(v, perm_at(lds, (uint32_t)__builtin_amdgcn_readlane((int)gv2, l)));
        };
        // (4-row batches: the three accumulators leave no registers for a fifth row in flight)
        roll_rows<FULL, NH, 4>(rbase, step, lo, lox, count, o, len, ox, unit, nw, wid, row);
        return;
    } else if (mode == TAMD_R_DENSE || (mode == TAMD_R_CAUCHY && (a.w0 >> 24) > 1u)) {
        // Rows with a per-row coefficient, then one product per byte:
        //  - DENSE: a Siamese row's dense part packet by packet (program.h); row k's coefficient
        //    is the lane-sum combination the recovery row reads, from its lane's opcode bits, cx
        //    and rx;
        //  - scaled CAUCHY (a decoder elimination run): s * CauchyElement(p, col mod 64).
        // The coefficients of 64 rows are computed at once, lane j taking row base + j (the table
        // lookups of one row depend on each other; across rows they do not); each row then reads
        // its product table at the index broadcast from its lane, so no row waits on the LDS
        // round trips of its own coefficient.
        const bool dense = mode == TAMD_R_DENSE;
        const u64 opw = (u64)tg.row | ((u64)(tg.len & 0xffffu) << 32);
        // DENSE w0 bits 24..31: s > 1 scales every coefficient (a decoder's scaled elimination run)
        const uint32_t dscale = dense ? a.w0 >> 24 : 0u;
        const PermT prx = perm_at(lds, (dense ? (tg.len >> 16) & 0xffu : a.w0 >> 24) * 8u);
        const uint8_t* sqr = (const uint8_t*)(lds + TAMD_LDS_INV + 64u);
        const uint8_t* inv = (const uint8_t*)(lds + TAMD_LDS_INV);
        const uint32_t px = p + 64u;
        const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        auto coef = [&](uint32_t c) -> uint32_t {
            if (!dense) return mul_sel(sel4(inv[(c & 63u) ^ px]), prx) & 0xffu;
            const uint32_t b = (uint32_t)(opw >> (6u * (c & 7u))) & 63u;
            const uint32_t cx = 3u + (199u * (c % 253u)) % 253u, cx2 = sqr[cx];
            const uint32_t sd = (b & 1u) ^ ((b & 2u) ? cx : 0u) ^ ((b & 4u) ? cx2 : 0u);
            const uint32_t tp = ((b >> 3) & 1u) ^ ((b & 16u) ? cx : 0u) ^ ((b & 32u) ? cx2 : 0u);
            return (sd ^ mul_sel(sel4(tp), prx)) & 0xffu;
        };
        // DENSE: COEFS.cap ADJ words follow, coefficient additions for single rows (the LDPC pair
        // columns of the recovery row, SiameseEncoder.cpp:1100-1144, folded into the run)
        // The additions come sorted by row (empty entries, row 0, only at the end): a cursor walks
        // them once per run, each block taking the ones below its end.
        const uint32_t nadj = dense ? 4u * tg.cap : 0u;
        const uint32_t* __restrict__ adw = (const uint32_t*)adj;
        uint32_t acur = 0;
        uint32_t gv = 0, gblk = ~0u;  // gv: lane j's table index for row 64 * gblk + j
        auto row_tab = [&](uint32_t i) -> PermT {
            if ((i >> 6) != gblk) {
                gblk = i >> 6;
                const uint32_t base = i & ~63u, mine = base + lane;
                uint32_t g = coef((col0 + mine * cstep) & (TAMD_COLUMN_PERIOD - 1u));
                for (; acur < nadj; ++acur) {
                    const uint32_t d = LDSI ? uniform(adw[acur]) : adw[acur];
                    if ((d >> 16) >= base + 64u) break;
                    if ((d >> 16) == mine) g ^= (d >> 8) & 0xffu;
                }
                if (dscale > 1u) g = mul_sel(sel4(g), perm_at(lds, dscale * 8u)) & 0xffu;
                gv = g * 8u;
            }
            return perm_at(lds, (uint32_t)__builtin_amdgcn_readlane((int)gv, (int)(i & 63u)));
        };
        if (TAMD_ROLL) {  // rolling loads over this wave's batches
            roll_rows<FULL, NH, TAMD_RBATCH>(rbase, step, lo, lox, count, o, len, ox, unit, nw, wid,
                                             [&](uint32_t i, const LV<NH>& v) __attribute__((always_inline)) {
                                                 a0 ^= lv_mul<NH>(v, row_tab(i));
                                             });
            return;
        }
        for (uint32_t e = 0; e < count; e += TAMD_RBATCH) {
            if ((unit++ & (nw - 1u)) != wid) continue;
            LV<NH> d[TAMD_RBATCH];
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q) d[q] = TAMD_RUN_ROW(q);
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q)
                if (e + q < count) a0 ^= lv_mul<NH>(lv_keep<FULL, NH>(d[q], o, len, ox), row_tab(e + q));
        }
    } else if (mode == TAMD_R_CAUCHY) {
        // CauchyElement(p, col mod 64) = inv((col mod 64) ^ (p + 64)) (SiameseCommon.h:212-218)
        uint32_t col = vgpr(col0);
        const uint32_t cs = vgpr(cstep), px = vgpr(p + 64u);
        const uint8_t* inv = (const uint8_t*)(lds + TAMD_LDS_INV);
        if (TAMD_ROLL) {  // rolling loads over this wave's batches
            roll_rows<FULL, NH, TAMD_RBATCH>(rbase, step, lo, lox, count, o, len, ox, unit, nw, wid,
                                             [&](uint32_t i, const LV<NH>& v) __attribute__((always_inline)) {
                                                 // the perm tables of inv((col mod 64) ^ (p + 64)), one LDS lookup
                                                 const uint32_t ti = TAMD_LDS_CINV - 512u + ((((col + i * cs) & 63u) ^ px) << 3);
                                                 a0 ^= lv_mul<NH>(v, perm_at(lds, ti));
                                             });
            return;
        }
        for (uint32_t e = 0; e < count; e += TAMD_RBATCH) {
            if ((unit++ & (nw - 1u)) != wid) {
                col += cs * TAMD_RBATCH;
                continue;
            }
            LV<NH> d[TAMD_RBATCH];
            uint32_t c[TAMD_RBATCH];
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q) {
                d[q] = TAMD_RUN_ROW(q);
                c[q] = inv[(col & 63u) ^ px];
                col += cs;
            }
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q)
                if (e + q < count) a0 ^= lv_mul<NH>(lv_keep<FULL, NH>(d[q], o, len, ox), perm_at(lds, c[q] * 8u));
        }
    } else {
        const bool plain = p == 1u;
        const PermT cp = perm_at(lds, p * 8u);
        if (TAMD_ROLL) {
            // rolling loads over this wave's batches: the rows are summed as they arrive and the
            // sum multiplied once (a parity row: p = 1, no multiply at all)
            LV<NH> x = lv_zero<NH>();
            roll_rows<FULL, NH, TAMD_RBATCH>(rbase, step, lo, lox, count, o, len, ox, unit, nw, wid,
                                             [&](uint32_t, const LV<NH>& v) __attribute__((always_inline)) { x ^= v; });
            a0 ^= plain ? x : lv_mul<NH>(x, cp);
            return;
        }
        for (uint32_t e = 0; e < count; e += TAMD_RBATCH) {
            if ((unit++ & (nw - 1u)) != wid) continue;
            LV<NH> d[TAMD_RBATCH];
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q) d[q] = TAMD_RUN_ROW(q);
            LV<NH> x = lv_zero<NH>();
#pragma unroll
            for (uint32_t q = 0; q < TAMD_RBATCH; ++q)
                if (e + q < count) x ^= lv_keep<FULL, NH>(d[q], o, len, ox);
            a0 ^= plain ? x : lv_mul<NH>(x, cp);  // one coefficient: sum the batch's rows, one product
        }
    }
#undef TAMD_RUN_ROW
#undef TAMD_RUN_LD
}

// One work item: the op's instruction list over this wave's slice.  FULL items lie below every
// length the op uses (op.full), so they need no per-lane length handling at all.
//
// Shared ops (nw = 4, the class-0 pure combines): every wave walks the instruction list, combines
// only its share of the row batches and skips the final STORE; the caller reduces the waves'
// acc_0 through LDS and stores.  Returns acc_0.
template <bool FULL, int NH, uint32_t TAMD_BATCH, bool LDSI = false>
__device__ __forceinline__ LV<NH> run_item(const tamd_instr* __restrict__ instrs, uint32_t first, uint32_t end,
                                           uint32_t o, uint32_t ox, uint32_t laneb, uint8_t* __restrict__ arena,
                                           const uint8_t* __restrict__ zrow, const uint32_t* __restrict__ lds,
                                           uint32_t nw, uint32_t wid, LV<NH>* __restrict__ r1 = nullptr,
                                           LV<NH>* __restrict__ r2 = nullptr) {
    LV<NH> a0 = lv_zero<NH>(), a1 = lv_zero<NH>(), a2 = lv_zero<NH>();  // the op's accumulators (program.h)
    uint32_t unit = 0;
    for (uint32_t k = first; k < end;) {
        tamd_instr in[TAMD_BATCH];
#pragma unroll
        for (uint32_t j = 0; j < TAMD_BATCH; ++j) in[j] = fetch_instr<LDSI>(instrs, k + j);  // region padded
        // A batch runs up to (not including) the next ACCR; an ACCR at the head runs alone.
        uint32_t nb = end - k < TAMD_BATCH ? end - k : TAMD_BATCH;
#pragma unroll
        for (uint32_t j = TAMD_BATCH; j-- > 0;)
            if ((in[j].w0 & 0xffu) == TAMD_I_ACCR && j < nb) nb = j;
        if (nb == 0) {
            // in[1]: the RANGE word, in[2]: TARGETS (MULTI runs) or COEFS (DENSE runs, followed by
            // COEFS.cap ADJ words)
            run_accr<FULL, NH, TAMD_BATCH, LDSI>(in[0], in[1], in[2], instrs + k + 3, o, ox, arena, lds, unit, nw, wid, a0,
                                           a1, a2);
            const uint32_t rmode = (in[0].w0 >> 8) & 0xffu, np = (in[0].w0 >> 16) & 0xffu;
            if (rmode == TAMD_R_DENSE && np > 1u) {
                // COEFS_t + its ADJ words for each of the np targets
                uint32_t skip = 3u + (in[2].cap & 0xffffu);
                for (uint32_t t = 1; t < np; ++t) skip += 1u + (fetch_instr<LDSI>(instrs, k + skip).cap & 0xffffu);
                k += skip;
                continue;
            }
            k += rmode == TAMD_R_DENSE ? 3u + in[2].cap : rmode == TAMD_R_MULTI ? 3u : 2u;
            continue;
        }
        if ((unit++ & (nw - 1u)) != wid) {  // another wave's batch (shared ops only)
            k += nb;
            continue;
        }
        // Every slot of the batch loads: ACC/ACC3 their row, the others the zero row (no branches,
        // no exec changes; the values are never consumed).
        LV<NH> v[TAMD_BATCH];
#pragma unroll
        for (uint32_t j = 0; j < TAMD_BATCH; ++j) {
            const uint32_t kind = in[j].w0 & 0xffu;
            const bool ld = j < nb && (kind == TAMD_I_ACC || kind == TAMD_I_ACC3);
            const uint8_t* rp = ld ? arena + (size_t)in[j].row * TAMD_ROW_UNIT : zrow;  // wave-uniform
            const uint32_t lo = ld ? load_off<FULL>(o, in[j].len) : laneb;
            const uint32_t lox = NH < 3 ? 0u : ld ? load_off<false>(ox, in[j].len) : (laneb >> 1);
            v[j] = lv_load_at<NH>(rp, lo, lox);
        }
#pragma unroll
        for (uint32_t j = 0; j < TAMD_BATCH; ++j) {
            const uint32_t w = in[j].w0, kind = j < nb ? (w & 0xffu) : 0u;
            if (kind == TAMD_I_ACC) {
                LV<NH> x = lv_keep<FULL, NH>(v[j], o, in[j].len, ox);
                const uint32_t coef = (w >> 8) & 0xffu;
                if (coef != 1u) x = lv_mul<NH>(x, perm_at(lds, coef * 8u));
                const uint32_t a = (w >> 16) & 0xffu;
                if (a == 0) a0 ^= x;
                else if (a == 1) a1 ^= x;
                else a2 ^= x;
            } else if (kind == TAMD_I_STOREC) {
                const uint32_t c0 = (w >> 8) & 0xffu, c1 = (w >> 16) & 0xffu, c2 = w >> 24;
                LV<NH> x = lv_zero<NH>();
                if (c0 == 1u) x = a0; else if (c0) x = lv_mul<NH>(a0, perm_at(lds, c0 * 8u));
                if (c1 == 1u) x ^= a1; else if (c1) x ^= lv_mul<NH>(a1, perm_at(lds, c1 * 8u));
                if (c2 == 1u) x ^= a2; else if (c2) x ^= lv_mul<NH>(a2, perm_at(lds, c2 * 8u));
                lv_store_row<FULL, NH, LDSI>(arena, in[j].row, in[j].len, in[j].cap, 0, o, x, ox);
            } else if (kind == TAMD_I_ACC3) {
                const LV<NH> x = lv_keep<FULL, NH>(v[j], o, in[j].len, ox);
                const PermT c1 = perm_at(lds, ((w >> 8) & 0xffu) * 8u), c2 = perm_at(lds, ((w >> 16) & 0xffu) * 8u);
                lv_acc3<NH>(x, c1, c2, a0, a1, a2);
            } else if (kind == TAMD_I_STORE && nw == 1u) {
                const uint32_t a = (w >> 16) & 0xffu;
                const LV<NH> x = a == 0 ? a0 : (a == 1 ? a1 : a2);
                if (FULL && NH < 3) {
                    lv_store<NH>(arena + (size_t)in[j].row * TAMD_ROW_UNIT + o, x);
                } else {
                    // the FOOTER word follows the STORE (possibly past this batch)
                    const tamd_instr f = fetch_instr<LDSI>(instrs, k + j + 1);
                    lv_store_row<FULL, NH, LDSI>(arena, in[j].row, in[j].len, in[j].cap, ((u64)f.len << 32) | f.row, o, x, ox);
                }
            } else if (kind == TAMD_I_CLEAR) {
                a0 = a1 = a2 = lv_zero<NH>();
            }
        }
        k += nb;
    }
    if (r1) {  // (shared multi-target ops: the caller reduces acc_1 and acc_2 too)
        *r1 = a1;
        *r2 = a2;
    }
    return a0;
}

// Ops of one level never read a row written by an op of the same level, so every load of a
// batch can be issued before the batch's stores.  Persistent grid: each workgroup stages the
// tables in LDS once and then claims items.  A slice is 64 lanes x 8*NH bytes.
// A launch runs one level each of up to TAMD_MAX_SEGMENTS programs (level pipelining,
// Device::launch): segment k holds program k's items; items are numbered across segments.
// Programs live in one device allocation (`prog`); segments address them by byte offsets, so
// every instruction fetch derives from one noalias argument and stays a scalar load (pointers
// inside an argument struct would turn them into vector loads: +11 VGPRs, 4 waves/SIMD).
template <int NH, uint32_t B>
__device__ __forceinline__ void exec_level(const tamd_segments& sg, const uint8_t* __restrict__ pbase,
                                           uint32_t n_shared, uint8_t* __restrict__ arena,
                                           const uint32_t* __restrict__ gf_perm, const uint8_t* __restrict__ zrow,
                                           unsigned long long* __restrict__ stamps) {
    constexpr uint32_t SLICE = 64u * 8u * NH;
    // bytes of a slice at the lanes' 16-byte offsets (NH = 3: the first 1024, FULL's extent)
    constexpr uint32_t MAIN = NH == 3 ? 1024u : SLICE;
    __shared__ __attribute__((aligned(16))) uint32_t lds_perm[TAMD_GF_DWORDS];
    __shared__ LV<NH> partial[TAMD_WAVES_PER_WG][64];  // shared ops: the waves' acc_0
    __shared__ uint32_t claim, shared_claim, shared_item;
    __shared__ tamd_segment lds_seg[TAMD_MAX_SEGMENTS];
    // the launch's items in the order waves take them: blocks of (segment, cost class) items,
    // class by class across the segments (flags bit 0) or segment by segment; + a sentinel
    __shared__ uint4 lds_blk[TAMD_MAX_SEGMENTS * TAMD_COST_CLASSES + 1];  // {segment, first item, count, -}
    // this workgroup's items of block b: positions r_b, r_b + G, ... (.x = r_b, .y = how many)
    __shared__ uint2 lds_wg[TAMD_MAX_SEGMENTS * TAMD_COST_CLASSES + 1];
    for (uint32_t i = threadIdx.x; i < TAMD_GF_DWORDS / 4; i += blockDim.x)
        ((uint4*)lds_perm)[i] = ((const uint4*)gf_perm)[i];
    if (threadIdx.x == 0) {
        claim = shared_claim = 0;
        // constant indices only (a dynamic index into the arguments would copy them to scratch)
#pragma unroll
        for (uint32_t k = 0; k < TAMD_MAX_SEGMENTS; ++k) {
            lds_seg[k] = sg.s[k];
            if (k >= sg.n) lds_seg[k].count = 0;
        }
        // (.w: the segment's first item in segment order, where the stamps of an item go)
        uint32_t nb = 0, base = 0;
        if (sg.flags & 1u) {
            uint32_t first[TAMD_MAX_SEGMENTS] = {0, 0, 0, 0, 0, 0};
            for (uint32_t c = 0; c < TAMD_COST_CLASSES; ++c) {
                base = 0;
                for (uint32_t k = 0; k < sg.n; ++k) {
                    const uint32_t m = lds_seg[k].cls[c];
                    if (m) lds_blk[nb++] = make_uint4(k, first[k], m, base);
                    first[k] += m;
                    base += lds_seg[k].count;
                }
            }
        } else {
            for (uint32_t k = 0; k < sg.n; ++k) {
                if (lds_seg[k].count) lds_blk[nb++] = make_uint4(k, 0, lds_seg[k].count, base);
                base += lds_seg[k].count;
            }
        }
        lds_blk[nb] = make_uint4(0, 0, ~0u, 0);
        // Single-wave items (the shared ones, the first n_shared of the first block, excepted):
        // workgroup g takes positions p = (g - o_b) mod G + m G of block b, o_b = the items before
        // the block rounded down to a multiple of 8.  So position p runs on an XCD p mod 8 (g mod 8)
        // -- the host lays out each class with every stream's items on one residue (XCD affinity,
        // Device::close_program) -- and the rotation o_b spreads the blocks' remainders.
        if (n_shared) {
            lds_blk[0].y += n_shared;
            lds_blk[0].z -= n_shared;
        }
        // (a small launch gives the shared items workgroups of their own, the first n_shared:
        // the single-wave items then go to the others, none waiting behind a shared one)
        const bool apart = n_shared && gridDim.x > n_shared;
        const uint32_t G = apart ? gridDim.x - n_shared : gridDim.x, g = apart ? blockIdx.x - n_shared : blockIdx.x;
        const bool none = apart && blockIdx.x < n_shared;
        uint32_t before = 0;
        for (uint32_t b = 0; b < nb; ++b) {
            const uint32_t cnt = lds_blk[b].z, r = (g + G - (before & ~7u) % G) % G;
            lds_wg[b] = make_uint2(r, !none && cnt > r ? (cnt - 1u - r) / G + 1u : 0u);
            before += cnt;
        }
        lds_wg[nb] = make_uint2(0, ~0u);
    }
    __syncthreads();
    const tamd_op* __restrict__ ops = (const tamd_op*)(pbase + sg.s[0].ops);
    const tamd_instr* __restrict__ instrs = (const tamd_instr*)(pbase + sg.s[0].instrs);
    const uint2* __restrict__ items = (const uint2*)(pbase + sg.s[0].items);

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = uniform(threadIdx.x >> 6);
    const uint32_t laneb = lane * 8u * (NH < 3 ? NH : 2);
    const uint32_t laneb_x = MAIN + lane * 8u;  // (NH = 3) the extension word's offset in the slice

    // Items [0, n_shared) are class-0 pure combines: the workgroup takes them one at a time
    // (items g, g + G, ...), each wave combining every fourth batch of rows; wave 0 reduces the
    // partial sums through LDS and executes the op's final STORE.
    for (;;) {
        if (threadIdx.x == 0) shared_item = shared_claim++;
        __syncthreads();
        const uint32_t it = blockIdx.x + shared_item * gridDim.x;
        __syncthreads();  // every wave has read shared_item before it is claimed again
        if (it >= n_shared) break;
        const uint2 item = items[it];
        const tamd_op op = ops[uniform(item.x)];
        const uint32_t s0 = uniform(item.y) * SLICE;
        const uint32_t o = s0 + laneb, ox = s0 + laneb_x;
        const uint32_t first = uniform(op.first), end = uniform(op.first + op.count);
        const bool full = s0 + MAIN <= uniform(op.full);
        const u64 t0 = stamps ? __builtin_amdgcn_s_memrealtime() : 0;
        LV<NH> x1, x2;
        const LV<NH> x = full ? run_item<true, NH, B>(instrs, first, end, o, ox, laneb, arena, zrow, lds_perm, TAMD_WAVES_PER_WG, wave, &x1, &x2)
                              : run_item<false, NH, B>(instrs, first, end, o, ox, laneb, arena, zrow, lds_perm, TAMD_WAVES_PER_WG, wave, &x1, &x2);
        // The op ends with one STORE + FOOTER per accumulator it fills: one for a pure combine, up
        // to three for a multi-target dense op; each is reduced through `partial` in turn.
        uint32_t nst = 1;
        while (nst < 3u && end >= first + 2u * (nst + 1u) && (instrs[end - 2u * (nst + 1u)].w0 & 0xffu) == TAMD_I_STORE) ++nst;
        for (uint32_t s = 0; s < nst; ++s) {
            const tamd_instr st = instrs[end - 2u * (nst - s)], f = instrs[end - 2u * (nst - s) + 1u];
            const uint32_t acc = (st.w0 >> 16) & 0xffu;
            if (s) __syncthreads();  // wave 0 has read the previous accumulator's partial sums
            LV<NH> mine = x;
            if (acc == 1u) mine = x1;
            if (acc == 2u) mine = x2;
            partial[wave][lane] = mine;
            __syncthreads();
            if (wave == 0) {
                LV<NH> sum = partial[0][lane];
                sum ^= partial[1][lane];
                sum ^= partial[2][lane];
                sum ^= partial[3][lane];
                const u64 foot = ((u64)f.len << 32) | f.row;
                if (full) lv_store_row<true, NH>(arena, st.row, st.len, st.cap, foot, o, sum, ox);
                else lv_store_row<false, NH>(arena, st.row, st.len, st.cap, foot, o, sum, ox);
            }
        }
        if (wave == 0) {
            if (stamps && lane == 0) {
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                stamps[3 * it] = t0;
                stamps[3 * it + 1] = __builtin_amdgcn_s_memrealtime();
                stamps[3 * it + 2] = ((u64)blockIdx.x << 32) | 4u;
            }
        }
        // (the next claim's barriers order partial[] reuse)
    }

    // Items [n_shared, n_items): one wave per item.  Workgroup g owns items g, g + G, ... of
    // them (a stratified sample of the level: ordered by cost class, most expensive first); its
    // waves claim them one at a time through an LDS counter, so a wave that drew a long op does
    // not hold up the others.
    const uint32_t wg_stride = n_shared && gridDim.x > n_shared ? gridDim.x - n_shared : gridDim.x;
    for (;;) {
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(&claim, 1u);
        k = uniform(__shfl(k, 0));
        // this workgroup's k-th item: its block and position there (wave-uniform LDS reads)
        uint32_t b = 0;
        while (k >= lds_wg[b].y) k -= lds_wg[b++].y;
        if (lds_wg[b].y == ~0u) break;
        const uint32_t seg = uniform(lds_blk[b].x);
        const uint32_t rel = uniform(lds_blk[b].y) + uniform(lds_wg[b].x) + k * wg_stride;
        const uint32_t at = uniform(lds_blk[b].w) + rel;  // (stamps)
        const tamd_segment sd = lds_seg[seg];
        const tamd_op* __restrict__ sops = (const tamd_op*)(pbase + uniform(sd.ops));
        const tamd_instr* __restrict__ ins = (const tamd_instr*)(pbase + uniform(sd.instrs));
        const uint2 item = ((const uint2*)(pbase + uniform(sd.items)))[uniform(rel)];
        const tamd_op op = sops[uniform(item.x)];
        const uint32_t s0 = uniform(item.y) * SLICE;
        const uint32_t o = s0 + laneb, ox = s0 + laneb_x;
        const uint32_t first = uniform(op.first), end = uniform(op.first + op.count);
        const u64 t0 = stamps ? __builtin_amdgcn_s_memrealtime() : 0;
        if (s0 + MAIN <= uniform(op.full))
            run_item<true, NH, B>(ins, first, end, o, ox, laneb, arena, zrow, lds_perm, 1u, 0u);
        else
            run_item<false, NH, B>(ins, first, end, o, ox, laneb, arena, zrow, lds_perm, 1u, 0u);
        if (stamps && lane == 0) {  // profiling only (TONK_AMD_STAMPS): vector stores of 100 MHz stamps
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            const u64 t1 = __builtin_amdgcn_s_memrealtime();
            stamps[3 * at] = t0;
            stamps[3 * at + 1] = t1;
            stamps[3 * at + 2] = ((u64)blockIdx.x << 32) | (threadIdx.x >> 6);
        }
    }
}

// tamd_exec16: 16 B per lane, 1024-byte slices, 6 rows per load batch (94 VGPRs, 5 waves/SIMD).
// Measured on the bench program (round 1): 61.6-62.2 us per launch, against 62.7-63.5 us for
// 8 B per lane / 512-byte slices / 8-row batches and 67 us for 16 B per lane with 8-row batches
// (108 VGPRs, 4 waves/SIMD); only this variant is built.
#define TAMD_EXEC_KERNEL(name, NH, B)                                                                  \
    extern "C" __global__ void __launch_bounds__(256)                                                   \
    name(const tamd_segments segments, const uint8_t* __restrict__ prog, uint32_t n_shared,            \
         uint8_t* __restrict__ arena,                                                                  \
         const uint32_t* __restrict__ gf_perm, const uint8_t* __restrict__ zrow,                       \
         unsigned long long* __restrict__ stamps) {                                                    \
        exec_level<NH, B>(segments, prog, n_shared, arena, gf_perm, zrow, stamps);                    \
    }
TAMD_EXEC_KERNEL(tamd_exec16, 2, 6)
// tamd_exec24: 1536-byte slices (16 + 8 B per lane), so a 1302-byte packet row is one work item
// (program.h TAMD_SLICE_BYTES_X; chosen by Device::init, tonk_amd::slice_bytes()).
TAMD_EXEC_KERNEL(tamd_exec24, 3, 5)


// ---------------------------------------------------------------------------------------------
// tamd_serve: the persistent executor of the siamese.h C ABI (serve.h; host side serve.cpp).
// Block 0 is the dispatcher: one lane polls the host ring in order and publishes each command in
// the device work list.  Every other block is a worker (16 waves, one per CU): it claims the next
// work-list index, waits for it, and runs the command -- copy it into LDS, land its packets in
// the arena, run the program's levels (waves claim items through an LDS counter; a workgroup
// barrier between levels: an op only reads rows of lower levels), write the reads to the host
// and store the completion word.  Memory: the worker's system-scope acquire at the start of a
// command (this CU's L1, and host data the L2 may hold) and release at its end (the XCD's L2
// written back before the completion word) make a codec's rows visible to its next command on
// any CU or XCD, and to the ordinary executor launches.  The dispatcher ends after
// `idle_ticks` without a command (or when the host sets `stop`); the workers drain every
// published command and end too, so the grid always empties; the host relaunches on demand.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ u64 ld_sys(const uint64_t* p) {
    return __hip_atomic_load((uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint64_t* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ u64 ld_agent(const uint64_t* p) {
    return __hip_atomic_load((uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Copy `len` bytes between host memory (16-B aligned) and an arena row, one wave: 16 B per lane
// per chunk, four chunks in flight per lane, the tail (len mod 16) byte by byte.
template <bool TO_HOST, bool PLAIN = false>
__device__ __forceinline__ void serve_xfer(uint8_t* __restrict__ arena, u64 host, uint32_t unit, uint32_t len,
                                           uint32_t lane) {
    uint8_t* a = arena + (size_t)unit * TAMD_ROW_UNIT;
    uint8_t* h = (uint8_t*)host;
    const uint8_t* src = TO_HOST ? a : h;
    uint8_t* dst = TO_HOST ? h : a;
    const uint32_t n16 = len >> 4;
    // (every lane loads -- a clamped chunk when past the end -- and only in-range lanes store:
    // four loads in flight, no exec-masked loads, no private array)
    for (uint32_t b = 0; b < n16; b += 256u) {
        const uint32_t c0 = b + lane, c1 = c0 + 64u, c2 = c0 + 128u, c3 = c0 + 192u, m = n16 - 1u;
        const uint4 v0 = *(const uint4*)(src + 16u * min(c0, m));
        const uint4 v1 = *(const uint4*)(src + 16u * min(c1, m));
        const uint4 v2 = *(const uint4*)(src + 16u * min(c2, m));
        const uint4 v3 = *(const uint4*)(src + 16u * min(c3, m));
        // Arena rows: write-through (agent scope), visible to the codec's next command on any
        // XCD; host memory: system-scope stores, written through to the host before the completion
        // word (plain stores there can still sit in the L2 when it is seen: wrong packets)
        const uint4 v[4] = {v0, v1, v2, v3};
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q)
            if (c0 + 64u * q < n16) {
                uint8_t* d = dst + 16u * (c0 + 64u * q);
                const u64 lo = ((u64)v[q].y << 32) | v[q].x, hi = ((u64)v[q].w << 32) | v[q].z;
                if constexpr (PLAIN) {
                    *(uint4*)d = v[q];
                } else if constexpr (TO_HOST) {
                    st_sys((uint64_t*)d, lo);
                    st_sys((uint64_t*)(d + 8), hi);
                } else {
                    st_u64<true>(d, lo);
                    st_u64<true>(d + 8, hi);
                }
            }
    }
    const uint32_t tail = len & 15u;
    if (TO_HOST) {
        // the last partial 8-byte words as whole words: the landing buffers are in 64-byte units
        // (capi.cpp) and arena rows too, so the bytes past `len` stay inside both
        const uint32_t w0 = 16u * n16, nw = (tail + 7u) / 8u;
        if (lane < nw) st_sys((uint64_t*)(dst + w0 + 8u * lane), *(const u64*)(src + w0 + 8u * lane));
    } else if (tail) {  // the last partial 8-byte words of the row, merged with the bytes already there
        const uint32_t w0 = 16u * n16, nw = (tail + 7u) / 8u;
        if (lane < nw) {
            const uint32_t at = w0 + 8u * lane, nb = min(8u, len - at);
            u64 x = 0;
            for (uint32_t b = 0; b < nb; ++b) x |= (u64)src[at + b] << (8u * b);
            if (nb < 8u) x |= *(const u64*)(dst + at) & ~byte_mask(nb);
            st_u64<true>(dst + at, x);
        }
    }
}

__device__ __forceinline__ tamd_xfer lds_xfer(const uint8_t* base, uint32_t i) {
    const uint4 v = ((const uint4*)base)[i];
    tamd_xfer x;
    x.host = ((u64)uniform(v.y) << 32) | uniform(v.x);
    x.unit = uniform(v.z);
    x.len = uniform(v.w);
    return x;
}

extern "C" __global__ void __launch_bounds__(TAMD_SERVE_THREADS) tamd_serve(const tamd_serve_args a) {
    tamd_serve_slot* wl = (tamd_serve_slot*)(a.dev + 1);
    if (blockIdx.x == 0) {
        // ---- the dispatcher: one wave ----
        // Each poll reads ten slots (lane = 6 * slot + granule, lanes 60..63 idle) from t + scan,
        // t being the first slot not yet handed on, and hands on every complete one among them, in
        // any order: its granules are copied unchanged into the work list with write-through
        // stores (no fence: the tags are the flags).  `ahead` marks the slots past t already
        // handed on, so a poster descheduled between taking its ticket and writing its granules
        // holds up only its own command: the ones behind it go on (the workers claim work-list
        // indices in order but wait only on their own entry).  While every slot of the window
        // but t is handed on, the next poll looks ten slots further (up to 60 past t).
        if (threadIdx.x >= 64) return;
        const uint32_t lane = threadIdx.x, j = lane / TAMD_SERVE_GRANULES, k = lane - TAMD_SERVE_GRANULES * j;
        // (A/B, pad bit 1: one slot per poll)
        const uint32_t width = (a.pad & 2u) ? 1u : 10u;
        const uint32_t wmask = (1u << width) - 1u;
        const bool mine = lane < width * TAMD_SERVE_GRANULES;
        u64 t = a.tail0, ahead = 0;  // ahead bit i: slot t + i handed on (bit 0 never set)
        uint32_t scan = 0;
        u64 last = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) st_sys(&a.host->dbg[0], last);
        for (uint32_t polls = 0;; ++polls) {
            if ((polls & 1023u) == 0 && lane == 0) {
                st_sys(&a.host->dbg[1], polls >> 10);
                st_sys(&a.host->dbg[2], t);
            }
            const u64 ti = t + scan + (mine ? j : 0u);
            const u64 gv = ld_sys(&a.ring[ti & a.ring_mask].g[mine ? k : 0u]);
            const u64 okm = ballot(mine && (uint32_t)(gv >> 32) == (uint32_t)(ti + 1));
            uint32_t comp = 0;
            for (uint32_t n = 0; n < width; ++n)
                if (((okm >> (TAMD_SERVE_GRANULES * n)) & 0x3full) == 0x3full) comp |= 1u << n;
            const uint32_t done = (uint32_t)(ahead >> scan) & wmask;
            const uint32_t fresh = comp & ~done;
            if (fresh) {
                if (mine && ((fresh >> j) & 1u))
                    __hip_atomic_store(&wl[ti & a.wl_mask].g[k], gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ahead |= (u64)fresh << scan;
                // t moves past the handed-on prefix
                const uint32_t n = ~ahead ? (uint32_t)__builtin_ctzll(~ahead) : 64u;
                ahead = n < 64u ? ahead >> n : 0ull;
                t += n;
                if (lane == 0 && n) st_sys(&a.host->consumed, t);
                last = __builtin_amdgcn_s_memrealtime();
                scan = 0;
                continue;
            }
            // nothing new here: while the window is handed on but for slot t, look further
            const uint32_t open = ~done & wmask & (scan ? wmask : wmask & ~1u);
            if (!open && scan + 2u * width <= 64u) {
                scan += width;
                continue;
            }
            scan = 0;
            // (the instance never ends with commands past t handed on: the next one starts at t)
            if (!ahead && (__builtin_amdgcn_s_memrealtime() - last > a.idle_ticks)) break;
            if (ld_sys(&a.host->stop)) break;
            __builtin_amdgcn_s_sleep(2);
        }
        // End: the workers drain what was published, then end; the host learns where the next
        // instance starts (exit_tail) before it learns that this one ended (exited_gen).
        vm_drain();
        if (lane == 0) {
            __hip_atomic_store(&a.dev->quit, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            st_sys(&a.host->exit_tail, t);
            vm_drain();
            st_sys(&a.host->exited_gen, a.gen);
        }
        return;
    }

    // ---- a worker ----
    constexpr int NH = 3;
    constexpr uint32_t SLICE = 64u * 8u * NH, MAIN = 1024u;
    __shared__ __attribute__((aligned(16))) uint32_t lds_perm[TAMD_GF_DWORDS];
    __shared__ __attribute__((aligned(16))) uint4 cbuf[TAMD_SERVE_CMD_BYTES / 16];
    __shared__ u64 sh_cmd;
    __shared__ uint32_t sh_state, sh_bytes, sh_item;
    __shared__ LV<3> partial[TAMD_SERVE_WAVES][64];  // grouped levels: each wave's acc_0
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = uniform(tid >> 6);
    for (uint32_t i = tid; i < TAMD_GF_DWORDS / 4; i += TAMD_SERVE_THREADS)
        ((uint4*)lds_perm)[i] = ((const uint4*)a.gf)[i];
    const uint32_t laneb = lane * 16u, laneb_x = MAIN + lane * 8u;
    const uint8_t* cb = (const uint8_t*)cbuf;
    // Wave 0 completes the previous command (its completion words) and claims the next one in
    // ONE wave-uniform region at the top of the loop, right before the barrier (a lane-divergent
    // region before the back edge was rotated by the compiler so that the other lanes of wave 0
    // looped through the barrier without lane 0: a hang).
    u64 prev_done = 0, prev_start = 0;
    u64 prev_t[4] = {0, 0, 0, 0};  // stamps: command in LDS, packets landed, program run, reads written
    uint32_t prev_val = 0, prev_dbg = 0;
    for (;;) {
        if (wave == 0) {
            if (prev_done) {
                // every wave drained its stores (rows write-through, reads to the host) before
                // the barrier that ended the command: the completion word goes last
                if (lane == 0) {
                    uint64_t* done = (uint64_t*)prev_done;
                    st_sys(done + 1, prev_start);
                    st_sys(done + 2, __builtin_amdgcn_s_memrealtime());
                    // the reads' lines and anything else of the command still in the L2 go to
                    // memory before the completion word (pad bit 0: no fence, A/B)
                    if (!(a.pad & 1u)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                    vm_drain();
                    st_sys(done + 3, prev_t[0]);
                    st_sys(done + 4, prev_t[1]);
                    st_sys(done + 5, prev_t[2]);
                    st_sys(done + 6, prev_t[3]);
                    st_sys(done, prev_val);
                    if (prev_dbg) st_sys(&a.host->dbg[3], 7);
                }
                prev_done = 0;
            }
            u64 k = 0;
            if (lane == 0) k = __hip_atomic_fetch_add(&a.dev->claim, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            k = ((u64)uniform((uint32_t)(rdl((uint32_t)(k >> 32), 0))) << 32) | uniform(rdl((uint32_t)k, 0));
            const u64 idx = a.tail0 + k;
            const uint64_t* en = wl[idx & a.wl_mask].g;
            const uint32_t tag = (uint32_t)(idx + 1);
            if (idx == 0 && lane == 0) {  // (diagnostics: the first command, the server's start-up probe)
                st_sys(&a.host->dbg[3], 1);
                st_sys(&a.host->dbg[4], blockIdx.x);
            }
            uint32_t st = 0;
            u64 gv = 0;
            for (;;) {
                gv = ld_agent(en + min(lane, TAMD_SERVE_GRANULES - 1u));
                if (ballot((uint32_t)(gv >> 32) != tag) == 0) { st = 1; break; }
                if (ld_agent(&a.dev->quit)) {
                    gv = ld_agent(en + min(lane, TAMD_SERVE_GRANULES - 1u));
                    st = ballot((uint32_t)(gv >> 32) != tag) == 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (st) {
                const uint32_t v = (uint32_t)gv;
                prev_done = ((u64)uniform(rdl(v, 3)) << 32) | uniform(rdl(v, 2));
                prev_val = uniform(rdl(v, 4));
                prev_start = __builtin_amdgcn_s_memrealtime();
                prev_dbg = idx == 0;
                if (lane == 0) {
                    sh_cmd = ((u64)rdl(v, 1) << 32) | rdl(v, 0);
                    sh_bytes = rdl(v, 5);
                }
                // this CU's L1 drops lines another CU may have rewritten since (the codec's rows);
                // it completes while the command is copied (through uncached loads) and is waited
                // for before the barrier below, ahead of every arena access
                asm volatile("buffer_inv sc1" ::: "memory");
            }
            if (lane == 0) sh_state = st ? (idx == 0 ? 2u : 1u) : 0u;
        }
        __syncthreads();
        // (read through readfirstlane: a loop exit the compiler sees as divergent would put the
        // workgroup barriers below under divergent control flow)
        const uint32_t state = uniform(sh_state);
        if (!state) break;
        const bool dbg = state == 2u && tid == 0;
        if (dbg) st_sys(&a.host->dbg[3], 2);
        const u64 cmd_addr = ((u64)uniform((uint32_t)(sh_cmd >> 32)) << 32) | uniform((uint32_t)sh_cmd);
        const uint32_t cmd_bytes = uniform(sh_bytes);
        // 1. the command into LDS (8-byte system-scope loads: they bypass the L1, whose invalidation
        // runs meanwhile)
        if (a.pad & 4u) {
            vm_drain();
            __syncthreads();
            const uint32_t n16 = (cmd_bytes + 15u) >> 4, m = n16 - 1u;
            const uint4* src = (const uint4*)cmd_addr;
            constexpr uint32_t T = TAMD_SERVE_THREADS;
            for (uint32_t b = tid; b < n16; b += 4u * T) {
                const uint4 v0 = src[min(b, m)], v1 = src[min(b + T, m)], v2 = src[min(b + 2u * T, m)],
                            v3 = src[min(b + 3u * T, m)];
                cbuf[b] = v0;
                if (b + T < n16) cbuf[b + T] = v1;
                if (b + 2u * T < n16) cbuf[b + 2u * T] = v2;
                if (b + 3u * T < n16) cbuf[b + 3u * T] = v3;
            }
        } else {
            const uint32_t n8 = (cmd_bytes + 7u) >> 3, m = n8 - 1u;
            const uint64_t* src = (const uint64_t*)cmd_addr;
            constexpr uint32_t T = TAMD_SERVE_THREADS;
            u64* dst = (u64*)cbuf;
            for (uint32_t b = tid; b < n8; b += 4u * T) {
                const u64 v0 = ld_sys(src + min(b, m)), v1 = ld_sys(src + min(b + T, m)),
                          v2 = ld_sys(src + min(b + 2u * T, m)), v3 = ld_sys(src + min(b + 3u * T, m));
                dst[b] = v0;
                if (b + T < n8) dst[b + T] = v1;
                if (b + 2u * T < n8) dst[b + 2u * T] = v2;
                if (b + 3u * T < n8) dst[b + 3u * T] = v3;
            }
        }
        vm_drain();  // (wave 0: its L1 invalidation too)
        __syncthreads();
        prev_t[0] = __builtin_amdgcn_s_memrealtime();
        if (dbg) st_sys(&a.host->dbg[3], 3);
        const tamd_cmd* c = (const tamd_cmd*)cb;
        const uint32_t n_up = uniform(c->n_up), n_rd = uniform(c->n_rd), levels = uniform(c->levels);
        // 2. packets staged since the codec's last program land in their rows
        const uint32_t up_chunks = uniform(c->up_chunks);
        if (up_chunks) {
            // one staging half: every thread copies 16-byte chunks of it, four loads in flight,
            // each chunk to the packet it falls in (binary search over the uploads, in LDS);
            // chunks in the alignment gaps between packets are dropped, a packet's last chunk
            // may write bytes past its end inside its row (rows are whole 64-byte units)
            const uint8_t* xs = cb + uniform(c->off_up);
            const u64 base = lds_xfer(xs, 0).host;
            constexpr uint32_t T = TAMD_SERVE_THREADS;
            const uint32_t m = up_chunks - 1u;
            for (uint32_t b = tid; b < up_chunks; b += 4u * T) {
                uint4 v[4];
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) v[q] = *(const uint4*)(base + 16ull * min(b + q * T, m));
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    const uint32_t ch = b + q * T;
                    if (ch >= up_chunks) break;
                    const u64 at = base + 16ull * ch;
                    uint32_t lo = 0, hi = n_up;  // last upload whose host address is <= at
                    while (hi - lo > 1u) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (((const tamd_xfer*)xs)[mid].host <= at) lo = mid; else hi = mid;
                    }
                    const tamd_xfer x = ((const tamd_xfer*)xs)[lo];
                    const u64 off = at - x.host;
                    if (off < x.len) {
                        uint8_t* d = a.arena + (size_t)x.unit * TAMD_ROW_UNIT + off;
                        st_u64<true>(d, ((u64)v[q].y << 32) | v[q].x);
                        st_u64<true>(d + 8, ((u64)v[q].w << 32) | v[q].z);
                    }
                }
            }
        } else {
            for (uint32_t u = wave; u < n_up; u += TAMD_SERVE_WAVES) {
                const tamd_xfer x = lds_xfer(cb + uniform(c->off_up), u);
                serve_xfer<false>(a.arena, x.host, x.unit, x.len, lane);
            }
        }
        vm_drain();
        __syncthreads();
        if (dbg) st_sys(&a.host->dbg[3], 4);
        prev_t[1] = __builtin_amdgcn_s_memrealtime();
        // 3. the program, level by level
        const tamd_instr* ins = (const tamd_instr*)(cb + uniform(c->off_instr));
        const uint4* ops = (const uint4*)(cb + uniform(c->off_ops));
        const uint2* items = (const uint2*)(cb + uniform(c->off_items));
        for (uint32_t l = 0; l < levels; ++l) {
            const uint32_t b0 = uniform(c->level_base[l]), b1 = uniform(c->level_base[l + 1]), n = b1 - b0;
            if (n && 2u * n <= TAMD_SERVE_WAVES) {
                // Few items: a group of G waves per item (G = 16, 8, 4, 2 for 1, 2, 3-4, 5-8 items).
                // A pure combine's row batches are split over its group (every G-th batch per
                // wave, run_item's shared mode) and the group's first wave sums the partial
                // accumulators through LDS and stores the row; any other op runs on that wave alone.
                // (A per-call program is one to three such levels of one to a few ops: a single
                // wave walking a 50-row op was most of a command's time.)
                const uint32_t G = TAMD_SERVE_WAVES >> (32u - __builtin_clz(n - 1u | 1u) - (n == 1u ? 1u : 0u));
                const uint32_t grp = wave / G, rank = wave % G;
                const bool active = grp < n;
                uint32_t shared = 0, full = 0, first = 0, end = 0, o = 0, ox = 0;
                LV<NH> x = lv_zero<NH>();
                if (active) {
                    const uint2 item = items[b0 + grp];
                    const uint4 op = ops[uniform(item.x)];
                    shared = uniform(item.y) >> 31;
                    const uint32_t s0 = (uniform(item.y) & 0x7fffffffu) * SLICE;
                    o = s0 + laneb;
                    ox = s0 + laneb_x;
                    first = uniform(op.x);
                    end = first + uniform(op.y);
                    full = s0 + MAIN <= uniform(op.w);
                    if (shared || rank == 0) {
                        const uint32_t nw = shared ? G : 1u, wid = shared ? rank : 0u;
                        if (full)
                            x = run_item<true, NH, 5, true>(ins, first, end, o, ox, laneb, a.arena, a.zrow, lds_perm, nw, wid);
                        else
                            x = run_item<false, NH, 5, true>(ins, first, end, o, ox, laneb, a.arena, a.zrow, lds_perm, nw, wid);
                    }
                }
                partial[wave][lane] = x;
                __syncthreads();
                if (active && shared && rank == 0) {
                    LV<NH> sum = x;
                    for (uint32_t w = 1; w < G; ++w) sum ^= partial[wave + w][lane];
                    const tamd_instr st = fetch_instr<true>(ins, end - 2u), f = fetch_instr<true>(ins, end - 1u);
                    const u64 foot = ((u64)f.len << 32) | f.row;  // STORE (acc_0) + FOOTER end every pure op
                    if (full) lv_store_row<true, NH, true>(a.arena, st.row, st.len, st.cap, foot, o, sum, ox);
                    else lv_store_row<false, NH, true>(a.arena, st.row, st.len, st.cap, foot, o, sum, ox);
                }
                vm_drain();
                __syncthreads();
                continue;
            }
            if (tid == 0) sh_item = c->level_base[l];
            __syncthreads();
            for (;;) {
                uint32_t it = 0;
                if (lane == 0) it = atomicAdd(&sh_item, 1u);
                it = uniform(rdl(it, 0));
                if (it >= b1) break;
                const uint2 item = items[it];
                const uint4 op = ops[uniform(item.x)];
                const uint32_t s0 = (uniform(item.y) & 0x7fffffffu) * SLICE;
                const uint32_t o = s0 + laneb, ox = s0 + laneb_x;
                const uint32_t first = uniform(op.x), end = first + uniform(op.y);
                if (s0 + MAIN <= uniform(op.w))
                    run_item<true, NH, 5, true>(ins, first, end, o, ox, laneb, a.arena, a.zrow, lds_perm, 1u, 0u);
                else
                    run_item<false, NH, 5, true>(ins, first, end, o, ox, laneb, a.arena, a.zrow, lds_perm, 1u, 0u);
            }
            vm_drain();
            __syncthreads();
        }
        if (dbg) st_sys(&a.host->dbg[3], 5);
        prev_t[2] = __builtin_amdgcn_s_memrealtime();
        // 4. the reads into the caller's pinned buffer
        for (uint32_t r = wave; r < n_rd; r += TAMD_SERVE_WAVES) {
            const tamd_xfer x = lds_xfer(cb + uniform(c->off_rd), r);
            // (plain stores into the host buffer, written back by the release fence ahead of the
            // completion word: 8-byte system-scope stores, one fabric write each, made a
            // recovery-packet read ~10x slower; pad bit 3 restores them for A/B)
            if (a.pad & 8u) serve_xfer<true>(a.arena, x.host, x.unit, x.len, lane);
            else serve_xfer<true, true>(a.arena, x.host, x.unit, x.len, lane);
        }
        vm_drain();
        __syncthreads();
        if (dbg) st_sys(&a.host->dbg[3], 6);
        prev_t[3] = __builtin_amdgcn_s_memrealtime();
        // 5. completion: at the top of the next iteration (lane 0 of wave 0)
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

// Host staging (device.cpp d2h_gather): pack rows {arena row, bytes, output offset} into one
// buffer for a single D2H copy.  One workgroup per row, 16-byte stores where aligned.
struct GatherDesc { uint32_t row, len, out; };

extern "C" __global__ void tamd_gather_rows(const GatherDesc* __restrict__ d, uint32_t n,
                                            const uint8_t* __restrict__ arena, uint8_t* __restrict__ out) {
    const GatherDesc g = d[blockIdx.x];
    const uint8_t* src = arena + (size_t)g.row * TAMD_ROW_UNIT;  // rows are 64-B aligned
    uint8_t* dst = out + g.out;                                   // outputs are 16-B aligned
    const uint32_t n16 = g.len / 16u;
    for (uint32_t i = threadIdx.x; i < n16; i += blockDim.x) ((uint4*)dst)[i] = ((const uint4*)src)[i];
    for (uint32_t i = n16 * 16u + threadIdx.x; i < g.len; i += blockDim.x) dst[i] = src[i];
}

// Coalesced uploads of the siamese.h C ABI (Device::upload): packets staged back to back in one
// buffer (16-B aligned), one workgroup per packet copies it into its arena row (64-B aligned).
struct ScatterDesc { uint32_t row, len, src, pad; };

extern "C" __global__ void tamd_scatter_rows(const ScatterDesc* __restrict__ d, uint32_t n,
                                             const uint8_t* __restrict__ in, uint8_t* __restrict__ arena) {
    const ScatterDesc g = d[blockIdx.x];
    const uint8_t* src = in + g.src;
    uint8_t* dst = arena + (size_t)g.row * TAMD_ROW_UNIT;
    const uint32_t n16 = g.len / 16u;
    for (uint32_t i = threadIdx.x; i < n16; i += blockDim.x) ((uint4*)dst)[i] = ((const uint4*)src)[i];
    for (uint32_t i = n16 * 16u + threadIdx.x; i < g.len; i += blockDim.x) dst[i] = src[i];
}

// Zero-copy transfers between pinned host memory and the arena (Device::host_copy): one
// workgroup per packet reads (to_host = 0) or writes (1) the host bytes over the link directly.
// Host addresses are 16-B aligned, arena rows 64-B aligned.
struct HostCopyDesc { u64 host; uint32_t unit, len; };

extern "C" __global__ void __launch_bounds__(128)
tamd_host_copy(const HostCopyDesc* __restrict__ d, uint32_t n, uint8_t* __restrict__ arena, uint32_t to_host) {
    const HostCopyDesc c = d[blockIdx.x];
    uint8_t* a = arena + (size_t)c.unit * TAMD_ROW_UNIT;
    uint8_t* h = (uint8_t*)c.host;
    uint8_t* dst = to_host ? h : a;
    const uint8_t* src = to_host ? a : h;
    const uint32_t n16 = c.len / 16u;
    for (uint32_t i = threadIdx.x; i < n16; i += blockDim.x) ((uint4*)dst)[i] = ((const uint4*)src)[i];
    for (uint32_t i = n16 * 16u + threadIdx.x; i < c.len; i += blockDim.x) dst[i] = src[i];
}

// A small program's upload (Device::close_program / run, below kSmallUpload bytes): two ranges of
// pinned host memory into program memory, read over the link by the threads of one launch -- a
// DMA-engine copy costs tens of microseconds of latency before the first level can start, which
// a single stream or a per-call program waits out in full.
extern "C" __global__ void __launch_bounds__(256)
tamd_copy_in(const uint4* __restrict__ s0, uint4* __restrict__ d0, uint32_t n0, const uint4* __restrict__ s1,
             uint4* __restrict__ d1, uint32_t n1) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n0 + n1; i += stride) {
        if (i < n0) d0[i] = s0[i];
        else d1[i - n0] = s1[i - n0];
    }
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

// Verification digests of a program's output rows (Device::verify_next): enqueued on the launch
// stream right after the launch that completes the program.  mode 0: FNV-1a over `len` bytes
// (a recovery packet, footer included); mode 1: a recovered original -- parse its length
// prefix (serial.h get_length_header, `len` bytes available) and hash the payload it announces.
// One thread per row; verification only, never in a timed region.
struct VerifyDesc { uint32_t row, len, mode, pad; };
struct VerifyOut { u64 hash; uint32_t len, ok; };

extern "C" __global__ void tamd_verify_rows(const VerifyDesc* __restrict__ d, uint32_t n,
                                            const uint8_t* __restrict__ arena, VerifyOut* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const VerifyDesc g = d[i];
    const uint8_t* p = arena + (size_t)g.row * TAMD_ROW_UNIT;
    uint32_t skip = 0, len = g.len, ok = 1;
    if (g.mode == 1) {
        const uint32_t b0 = g.len >= 1 ? p[0] : 0u;
        const uint32_t top = b0 >> 6;
        uint32_t hb = 0;
        if (g.len < 1) ok = 0;
        else if (top <= 1) { len = b0; hb = 1; }
        else if (top == 2) { hb = 2; len = ((b0 << 8) | p[1]) & 0x3fffu; }
        else if ((b0 & 0xE0u) == 0xC0u) { hb = 3; len = ((b0 << 16) | ((uint32_t)p[1] << 8) | p[2]) & 0x1fffffu; }
        else { hb = 4; len = ((b0 << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]) & 0x1fffffffu; }
        if (ok && (hb > g.len || len > g.len - hb)) ok = 0;
        skip = hb;
        if (!ok) len = 0;
    }
    u64 h = 1469598103934665603ULL;
    for (uint32_t k = 0; k < len; ++k) { h ^= p[skip + k]; h *= 1099511628211ULL; }
    VerifyOut o;
    o.hash = h;
    o.len = len;
    o.ok = ok;
    out[i] = o;
}

// Marks the start and end of a bench's timed region in kernel traces (Device::set_timing).
extern "C" __global__ void tamd_timed_region() {}
// Empty kernel of the C ABI's start-up warming (Device::warm_streams): not a trace marker.
extern "C" __global__ void tamd_nop() {}
