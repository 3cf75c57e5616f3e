/*
    siamese_oracle.c -- TEST INFRASTRUCTURE ONLY (see siamese_oracle.h).

    A deliberately plain, scalar restatement of the reference math.  Every function cites the
    reference file:line it restates.  No SIMD, no allocator, no state machine: just the field,
    the coefficient generators, the wire formats, the definition of a recovery row, and an
    interpreter for the device program format so the host control plane can be checked on a
    machine without a GPU.
*/
#include "siamese_oracle.h"

#include <string.h>
#include <stdlib.h>

/* ------------------------------------------------------------------------------------------
   GF(2^8) tables.  gf256.cpp:358-372 picks GF256_GEN_POLY[3] = 0xa6 and uses (0xa6 << 1) | 1
   = 0x14D.  EXP/LOG follow gf256_explog_init (gf256.cpp:379-403): LOG[0] = 512 so that any
   product with zero lands in the zero tail of EXP (indices 510+ are 0 except EXP[510] = 1).
   MUL/DIV follow gf256_muldiv_init (gf256.cpp:410-442); INV = DIV(1, x) (gf256.cpp:449);
   SQR = MUL(x, x) (gf256.cpp:460).
   ------------------------------------------------------------------------------------------ */
static unsigned g_poly;
static uint8_t  g_exp[1025];
static uint16_t g_log[256];
static uint8_t  g_mul[256][256]; /* [y][x] */
static uint8_t  g_div[256][256]; /* [y][x] = x / y */
static uint8_t  g_inv[256];
static uint8_t  g_sqr[256];
static int      g_ready;

static void build_tables(void)
{
    g_poly = (0xa6u << 1) | 1u;

    g_log[0] = 512;
    g_exp[0] = 1;
    for (unsigned j = 1; j < 255; ++j) {
        unsigned v = (unsigned)g_exp[j - 1] << 1;
        if (v >= 256) v ^= g_poly;
        g_exp[j] = (uint8_t)v;
        g_log[g_exp[j]] = (uint16_t)j;
    }
    g_exp[255] = g_exp[0];
    g_log[g_exp[255]] = 255;            /* LOG[1] ends up 255 (gf256.cpp:395) */
    for (unsigned j = 256; j < 510; ++j) g_exp[j] = g_exp[j % 255];
    g_exp[510] = 1;
    for (unsigned j = 511; j < 1020; ++j) g_exp[j] = 0;

    for (unsigned x = 0; x < 256; ++x) { g_mul[0][x] = 0; g_div[0][x] = 0; }
    for (unsigned y = 1; y < 256; ++y) {
        const uint8_t ly  = (uint8_t)g_log[y];
        const uint8_t lyn = (uint8_t)(255 - ly);
        g_mul[y][0] = 0; g_div[y][0] = 0;
        for (unsigned x = 1; x < 256; ++x) {
            g_mul[y][x] = g_exp[g_log[x] + ly];
            g_div[y][x] = g_exp[g_log[x] + lyn];
        }
    }
    for (unsigned x = 0; x < 256; ++x) g_inv[x] = g_div[x][1];
    for (unsigned x = 0; x < 256; ++x) g_sqr[x] = g_mul[x][x];
}

uint8_t  oracle_gf_mul(uint8_t x, uint8_t y) { return g_mul[y][x]; }
uint8_t  oracle_gf_div(uint8_t x, uint8_t y) { return g_div[y][x]; }
uint8_t  oracle_gf_inv(uint8_t x) { return g_inv[x]; }
uint8_t  oracle_gf_sqr(uint8_t x) { return g_sqr[x]; }
unsigned oracle_gf_polynomial(void) { return g_poly; }
uint8_t  oracle_gf_exp(unsigned i) { return i < 1025 ? g_exp[i] : 0; }
uint16_t oracle_gf_log(uint8_t x) { return g_log[x]; }

/* Bulk ops: gf256_add_mem (gf256.cpp:653), gf256_muladd_mem (gf256.cpp:1268, y=0 no-op,
   y=1 xor), gf256_mul_mem (gf256.cpp:1104, y=0 memset, y=1 memcpy). */
void oracle_add_mem(uint8_t* x, const uint8_t* y, size_t n)
{
    for (size_t i = 0; i < n; ++i) x[i] ^= y[i];
}

void oracle_muladd_mem(uint8_t* z, uint8_t y, const uint8_t* x, size_t n)
{
    if (y == 0) return;
    for (size_t i = 0; i < n; ++i) z[i] ^= g_mul[y][x[i]];
}

void oracle_mul_mem(uint8_t* z, const uint8_t* x, uint8_t y, size_t n)
{
    for (size_t i = 0; i < n; ++i) z[i] = g_mul[y][x[i]];
}

/* Reference self test (gf256.cpp:84-189): mul/div consistency over all pairs and the bulk
   operations on a 63-byte buffer with a guard byte. */
static int gf_self_test(void)
{
    for (unsigned i = 0; i < 256; ++i) {
        for (unsigned j = 0; j < 256; ++j) {
            const uint8_t p = oracle_gf_mul((uint8_t)i, (uint8_t)j);
            if (i && j) {
                if (oracle_gf_div(p, (uint8_t)i) != j) return -1;
                if (oracle_gf_div(p, (uint8_t)j) != i) return -2;
            } else if (p != 0) {
                return -3;
            }
            if (j == 1 && p != i) return -4;
        }
    }
    enum { N = 63 };
    uint8_t a[N + 1], b[N + 1];
    a[N] = b[N] = 0x5a;
    memset(a, 0x1f, N); memset(b, 0xf7, N);
    oracle_add_mem(a, b, N);
    for (unsigned i = 0; i < N; ++i) if (a[i] != (0x1f ^ 0xf7)) return -5;
    memset(a, 0xff, N); memset(b, 0xaa, N);
    oracle_muladd_mem(a, 0x6c, b, N);
    for (unsigned i = 0; i < N; ++i) if (a[i] != (uint8_t)(oracle_gf_mul(0xaa, 0x6c) ^ 0xff)) return -6;
    memset(a, 0xff, N); memset(b, 0x55, N);
    oracle_mul_mem(a, b, 0xa2, N);
    for (unsigned i = 0; i < N; ++i) if (a[i] != oracle_gf_mul(0xa2, 0x55)) return -7;
    if (a[N] != 0x5a || b[N] != 0x5a) return -8;
    return 0;
}

int oracle_gf_init(void)
{
    if (!g_ready) {
        build_tables();
        g_ready = 1;
    }
    return gf_self_test();
}

/* ------------------------------------------------------------------------------------------
   Coefficient generators.
   ------------------------------------------------------------------------------------------ */

/* GetColumnValue, SiameseCommon.h:89-93: LCG over 3..255 (period 253). */
uint8_t oracle_column_value(unsigned column)
{
    return (uint8_t)(3u + (column * 199u) % 253u);
}

/* GetRowValue, SiameseCommon.h:95-98. */
uint8_t oracle_row_value(unsigned row)
{
    return (uint8_t)(1u + (row + 1u) % 255u);
}

/* Int32Hash (Thomas Wang), SiameseCommon.h:150-159. */
static uint32_t int32_hash(uint32_t key)
{
    key += ~(key << 15);
    key ^= (key >> 10);
    key += (key << 3);
    key ^= (key >> 6);
    key += ~(key << 11);
    key ^= (key >> 16);
    return key;
}

/* GetRowOpcode, SiameseCommon.h:162-174: 6 low bits of the hash of lane + (row + 3) * 8;
   a zero opcode is replaced by 1 << 4 (kZeroValue). */
unsigned oracle_row_opcode(unsigned lane, unsigned row)
{
    const uint32_t op = int32_hash(lane + (row + 3u) * 8u) & 63u;
    return op == 0 ? 16u : op;
}

/* CauchyElement, SiameseCommon.h:212-218: 1 / ((row + 64) ^ column). */
uint8_t oracle_cauchy_element(unsigned row, unsigned column)
{
    return oracle_gf_inv((uint8_t)((uint8_t)column ^ (uint8_t)(row + 64u)));
}

/* PCGRandom, SiameseTools.h:79-101. */
uint32_t oracle_pcg_next(oracle_pcg* p)
{
    const uint64_t old = p->state;
    p->state = old * UINT64_C(6364136223846793005) + p->inc;
    const uint32_t xs  = (uint32_t)(((old >> 18) ^ old) >> 27);
    const uint32_t rot = (uint32_t)(old >> 59);
    return (xs >> rot) | (xs << ((uint32_t)(-(int32_t)rot) & 31u));
}

void oracle_pcg_seed(oracle_pcg* p, uint64_t y, uint64_t x)
{
    p->state = 0;
    p->inc = (y << 1u) | 1u;
    oracle_pcg_next(p);
    p->state += x;
    oracle_pcg_next(p);
}

/* ------------------------------------------------------------------------------------------
   Serializers.
   ------------------------------------------------------------------------------------------ */

/* SerializeHeader_PacketLength, SiameseSerializers.h:566-593. */
unsigned oracle_serialize_length_header(unsigned length, uint8_t* out)
{
    if (length <= 0x7f) { out[0] = (uint8_t)length; return 1; }
    if (length <= 0x3fff) { out[0] = (uint8_t)(0x80 | (length >> 8)); out[1] = (uint8_t)length; return 2; }
    if (length <= 0x1fffff) {
        out[0] = (uint8_t)(0xC0 | (length >> 16)); out[1] = (uint8_t)(length >> 8);
        out[2] = (uint8_t)length; return 3;
    }
    out[0] = (uint8_t)(0xE0 | (length >> 24)); out[1] = (uint8_t)(length >> 16);
    out[2] = (uint8_t)(length >> 8); out[3] = (uint8_t)length; return 4;
}

/* DeserializeHeader_PacketLength, SiameseSerializers.h:598-640. */
int oracle_deserialize_length_header(const uint8_t* in, unsigned avail, unsigned* length)
{
    if (!in || avail < 1) return -1;
    const unsigned n = in[0] >> 6;
    if (n <= 1) { *length = in[0]; return 1; }
    if (n == 2) {
        if (avail < 2) return -1;
        *length = (((unsigned)in[0] << 8) | in[1]) & 0x3fff; return 2;
    }
    if ((in[0] & 0xE0) == 0xC0) {
        if (avail < 3) return -1;
        *length = (((unsigned)in[0] << 16) | ((unsigned)in[1] << 8) | in[2]) & 0x1fffff; return 3;
    }
    if (avail < 4) return -1;
    *length = (((unsigned)in[0] << 24) | ((unsigned)in[1] << 16) | ((unsigned)in[2] << 8) | in[3]) & 0x1fffffff;
    return 4;
}

/* Footer forms: SerializeFooter_PacketCount (:510) and SerializeFooter_PacketNum (:383). */
static unsigned footer_count(unsigned v, uint8_t* out)
{
    if (v <= 127) { out[0] = (uint8_t)v; return 1; }
    out[0] = (uint8_t)v; out[1] = (uint8_t)(0x80 | (v >> 8)); return 2;
}

static unsigned footer_pnum(unsigned v, uint8_t* out)
{
    if (v <= 0x7f) { out[0] = (uint8_t)v; return 1; }
    if (v <= 0x3fff) { out[0] = (uint8_t)v; out[1] = (uint8_t)(0x80 | (v >> 8)); return 2; }
    out[0] = (uint8_t)v; out[1] = (uint8_t)(v >> 8); out[2] = (uint8_t)(0xC0 | (v >> 16)); return 3;
}

/* SerializeFooter_RecoveryMetadata, SiameseSerializers.h:736-754. */
unsigned oracle_serialize_recovery_footer(const oracle_recovery_meta* m, uint8_t* out)
{
    unsigned n = 0;
    if (m->SumCount > 1) {
        out[n++] = (uint8_t)m->Row;
        n += footer_count(m->LDPCCount, out + n);
    }
    n += footer_pnum(m->ColumnStart, out + n);
    n += footer_count(m->SumCount - 1, out + n);
    return n;
}

/* DeserializeFooter_PacketCount (:528), DeserializeFooter_PacketNum (:407) and
   DeserializeFooter_RecoveryMetadata (:759-800). */
static int rfooter_count(const uint8_t* buf, unsigned avail, unsigned* v)
{
    if (avail < 1) return -1;
    const uint8_t* p = buf + avail - 1;
    if ((p[0] & 0x80) == 0) { *v = p[0]; return 1; }
    if (avail < 2) return -1;
    *v = (((unsigned)p[0] << 8) | p[-1]) & 0x7fff;
    return 2;
}

static int rfooter_pnum(const uint8_t* buf, unsigned avail, unsigned* v)
{
    if (avail < 1) return -1;
    const uint8_t* p = buf + avail - 1;
    const unsigned n = p[0] >> 6;
    if (n <= 1) { *v = p[0]; return 1; }
    if (avail < n) return -1;
    if (n == 2) *v = (((unsigned)p[0] << 8) | p[-1]) & 0x3fff;
    else        *v = (((unsigned)p[0] << 16) | ((unsigned)p[-1] << 8) | p[-2]) & 0x3fffff;
    return (int)n;
}

int oracle_deserialize_recovery_footer(const uint8_t* buf, unsigned bytes, oracle_recovery_meta* m)
{
    unsigned avail = bytes;
    int f = rfooter_count(buf, avail, &m->SumCount);
    if (f < 0) return -1;
    avail -= (unsigned)f;
    m->SumCount++;
    f = rfooter_pnum(buf, avail, &m->ColumnStart);
    if (f < 0) return -1;
    avail -= (unsigned)f;
    if (m->SumCount <= 1) {
        m->LDPCCount = 1;
        m->Row = 0;
    } else {
        f = rfooter_count(buf, avail, &m->LDPCCount);
        if (f < 0) return -1;
        avail -= (unsigned)f;
        if (m->SumCount < m->LDPCCount) return -1;
        if (avail < 1) return -1;
        m->Row = buf[--avail];
    }
    return (int)(bytes - avail);
}

/* SerializeHeader_NACKLossRange, SiameseSerializers.h:861-928. */
unsigned oracle_serialize_nack_range(unsigned relStart, unsigned lossCountM1, uint8_t* out)
{
    unsigned b0 = lossCountM1 <= 2 ? lossCountM1 : 3;
    b0 |= relStart << 3;
    unsigned n = 1;
    if (relStart >= (1u << 5)) {
        unsigned b1 = relStart >> 5;
        if (relStart >= (1u << 12)) {
            unsigned b2 = relStart >> 12;
            if (relStart >= (1u << 19)) {
                out[3] = (uint8_t)(relStart >> 19);
                b2 |= 0x80;
                ++n;
            }
            out[2] = (uint8_t)b2;
            b1 |= 0x80;
            ++n;
        }
        out[1] = (uint8_t)b1;
        b0 |= 4;
        ++n;
    }
    out[0] = (uint8_t)b0;
    if (lossCountM1 >= 3) {
        uint8_t* q = out + n;
        unsigned c = lossCountM1 - 3;
        unsigned c1 = c;
        if (c >= (1u << 7)) {
            unsigned c2 = c >> 7;
            if (c >= (1u << 14)) {
                q[2] = (uint8_t)(c >> 14);
                c2 |= 0x80;
                ++n;
            }
            q[1] = (uint8_t)c2;
            c1 |= 0x80;
            ++n;
        }
        q[0] = (uint8_t)c1;
        ++n;
    }
    return n;
}

/* DeserializeHeader_NACKLossRange, SiameseSerializers.h:934-994 (needs 7 readable bytes). */
int oracle_deserialize_nack_range(const uint8_t* in, unsigned avail, unsigned* relStart, unsigned* lossCountM1)
{
    if (!in || avail < 7) return -1;
    const unsigned b0 = in[0];
    unsigned lc = b0 & 3, rs = b0 >> 3, n = 1;
    if (b0 & 4) {
        ++n;
        const unsigned b1 = in[1];
        rs |= (b1 & 0x7f) << 5;
        if (b1 & 0x80) {
            ++n;
            const unsigned b2 = in[2];
            rs |= (b2 & 0x7f) << 12;
            if (b2 & 0x80) {
                ++n;
                rs |= (unsigned)in[3] << 19;
            }
        }
    }
    if (lc == 3) {
        const uint8_t* q = in + n;
        lc += q[0] & 0x7f;
        if (q[0] & 0x80) {
            lc += (q[1] & 0x7fu) << 7;
            if (q[1] & 0x80) {
                lc += (unsigned)q[2] << 14;
                ++n;
            }
            ++n;
        }
        ++n;
    }
    *relStart = rs;
    *lossCountM1 = lc;
    return (int)n;
}

/* ------------------------------------------------------------------------------------------
   Direct recovery-row definition.

   Siamese row (SumCount > 64; SiameseEncoder.cpp:1046-1254):
     lane(c) = c % 8, op = GetRowOpcode(lane, Row), CX = GetColumnValue(c), RX = GetRowValue(Row)
     dense:   rec  += [op&1] row_c + [op&2] CX row_c + [op&4] CX^2 row_c   for c in sum range
              prod += [op&8] row_c + [op&16] CX row_c + [op&32] CX^2 row_c
     LDPC:    PCG.Seed(Row, LDPCCount); ceil(LDPCCount/16) pairs over the last LDPCCount
              columns: rec += row_{e1}; prod += row_{eRX}
     result:  rec += RX * prod, everything truncated to the recovery data length.
   Parity row (Row == 0, SumCount <= 64; SiameseEncoder.cpp:1356-1389): XOR of all rows.
   Cauchy row (Row = k + 1; SiameseEncoder.cpp:1390-1427): sum of CauchyElement(k, c % 64) row_c.
   Single (SumCount == 1; SiameseEncoder.cpp:1296-1329): the framed row itself.
   ------------------------------------------------------------------------------------------ */
static void acc_row(uint8_t* out, unsigned out_bytes, const uint8_t* row, unsigned bytes, uint8_t coef)
{
    unsigned n = bytes < out_bytes ? bytes : out_bytes;
    if (coef == 1) oracle_add_mem(out, row, n);
    else           oracle_muladd_mem(out, coef, row, n);
}

int oracle_recovery_row(const oracle_recovery_meta* m, oracle_get_row_fn get_row, void* ctx,
                        uint8_t* out, unsigned out_bytes)
{
    memset(out, 0, out_bytes);
    const unsigned period = 0x400000u;
    if (m->SumCount <= 64) {
        for (unsigned i = 0; i < m->SumCount; ++i) {
            const unsigned c = (m->ColumnStart + i) % period;
            unsigned bytes = 0;
            const uint8_t* row = get_row(ctx, c, &bytes);
            if (!row) return -1;
            uint8_t coef = 1;
            if (m->SumCount > 1 && m->Row != 0)
                coef = oracle_cauchy_element(m->Row - 1, c % 64u);
            acc_row(out, out_bytes, row, bytes, coef);
        }
        return 0;
    }

    uint8_t* prod = (uint8_t*)calloc(out_bytes ? out_bytes : 1, 1);
    if (!prod) return -1;
    const uint8_t rx = oracle_row_value(m->Row);
    for (unsigned i = 0; i < m->SumCount; ++i) {
        const unsigned c = (m->ColumnStart + i) % period;
        unsigned bytes = 0;
        const uint8_t* row = get_row(ctx, c, &bytes);
        if (!row) { free(prod); return -1; }
        const unsigned op = oracle_row_opcode(c % 8u, m->Row);
        const uint8_t cx = oracle_column_value(c);
        const uint8_t cx2 = oracle_gf_sqr(cx);
        const uint8_t k[3] = { 1, cx, cx2 };
        for (unsigned s = 0; s < 3; ++s) {
            if (op & (1u << s))       acc_row(out, out_bytes, row, bytes, k[s]);
            if (op & (1u << (s + 3))) acc_row(prod, out_bytes, row, bytes, k[s]);
        }
    }
    oracle_pcg prng;
    oracle_pcg_seed(&prng, m->Row, m->LDPCCount);
    const unsigned ldpcStart = m->ColumnStart + m->SumCount - m->LDPCCount;
    const unsigned pairs = (m->LDPCCount + 15u) / 16u;
    for (unsigned i = 0; i < pairs; ++i) {
        const unsigned c1  = (ldpcStart + oracle_pcg_next(&prng) % m->LDPCCount) % period;
        const unsigned crx = (ldpcStart + oracle_pcg_next(&prng) % m->LDPCCount) % period;
        unsigned b1 = 0, brx = 0;
        const uint8_t* r1 = get_row(ctx, c1, &b1);
        const uint8_t* rrx = get_row(ctx, crx, &brx);
        if (!r1 || !rrx) { free(prod); return -1; }
        acc_row(out, out_bytes, r1, b1, 1);
        acc_row(prod, out_bytes, rrx, brx, 1);
    }
    oracle_muladd_mem(out, rx, prod, out_bytes);
    free(prod);
    return 0;
}

/* ------------------------------------------------------------------------------------------
   CPU interpreter for the device program (tonk_amd/csrc/program.h).  Word layouts are
   restated here (not included) so this file stays a stand-alone checker.
   ------------------------------------------------------------------------------------------ */
enum { I_ACC = 1, I_STORE = 2, I_FOOTER = 3, I_CLEAR = 4, I_ACC3 = 5, I_STOREC = 6, I_ACCR = 7, I_RANGE = 8,
       I_TARGETS = 9, I_COEFS = 10 };
enum { R_LANE3 = 1, R_CAUCHY = 2, R_CONST = 3, R_MULTI = 4, R_DENSE = 5 };

/* Each op owns three accumulators of `span` bytes (program.h):
     ACC   w0 = 1 | coef << 8 | a << 16       acc_a ^= coef * row[0:len]
     ACC3  w0 = 5 | c1 << 8 | c2 << 16        acc_0 ^= row, acc_1 ^= c1 * row, acc_2 ^= c2 * row
     STORE w0 = 2 | flen << 8 | a << 16       row = acc_a[0:len] || footer || zeros to cap
     STOREC w0 = 6 | c0 << 8 | c1 << 16 | c2 << 24
                                              row = (c0*acc_0 ^ c1*acc_1 ^ c2*acc_2)[0:len] || zeros
     CLEAR                                    all accumulators = 0
     ACCR  w0 = 7 | mode << 8 | p << 16, row0, len, count; then RANGE w0 = 8, stride, col0, cstep:
           row_k = row0 + k*stride, col_k = (col0 + k*cstep) mod 2^22, k < count
           LANE3: as ACC3 with cx = CX(col_k); CAUCHY: acc_0 ^= CauchyElement(p, col_k mod 64)*row_k;
           CONST: acc_0 ^= p*row_k
           MULTI: then TARGETS w0 = 9, t_0, t_1, t_2 with t_a = kind | p << 2 | lo << 10 | hi << 21: for
           lo <= k < hi,
           kind CAUCHY: acc_a ^= CauchyElement(p, col_k mod 64)*row_k, kind CONST: acc_a ^= row_k
           DENSE: then COEFS w0 = 10, o[0:32], o[32:48] | rx << 16: with b = (o >> 6*(col_k mod 8)) & 63
           and cx = CX(col_k), acc_0 ^= (b0 ^ b1 cx ^ b2 cx^2 ^ rx (b3 ^ b4 cx ^ b5 cx^2)) * row_k, the
           lane-sum combination of a Siamese row (SiameseEncoder.cpp:1046-1098) packet by packet;
           with p = 2 or 3 targets: p COEFS words (cap = ADJ words | hi << 16), each followed by its
           ADJ words, target t adding rows k < hi_t into acc_t (rows of nested sum ranges); one
           target: w0 bits 24..31 = s > 1 scales every coefficient (decoder eliminations) */
int oracle_run_program(uint8_t* arena, size_t arena_bytes,
                       const uint32_t* ops, unsigned n_ops,
                       const uint32_t* instrs, unsigned n_instrs)
{
    uint8_t* acc = NULL;
    size_t acc_cap = 0;
    for (unsigned o = 0; o < n_ops; ++o) {
        const uint32_t first = ops[4 * o + 0], count = ops[4 * o + 1], span = ops[4 * o + 2];
        if ((size_t)first + count > n_instrs) { free(acc); return -1; }
        if (span > acc_cap) {
            free(acc);
            acc_cap = span;
            acc = (uint8_t*)malloc(3 * acc_cap);
            if (!acc) return -2;
        }
        if (span) memset(acc, 0, 3 * (size_t)span);
        for (uint32_t k = 0; k < count; ++k) {
            const uint32_t* w = instrs + 4 * (size_t)(first + k);
            const uint32_t kind = w[0] & 0xff;
            if (kind == I_CLEAR) {
                if (span) memset(acc, 0, 3 * (size_t)span);
            } else if (kind == I_ACC) {
                const uint8_t coef = (uint8_t)(w[0] >> 8);
                const uint32_t a = (w[0] >> 16) & 0xff;
                const size_t base = (size_t)w[1] * 64u;
                const uint32_t len = w[2];
                if (a > 2 || len > span || base + len > arena_bytes) { free(acc); return -3; }
                uint8_t* dst = acc + (size_t)a * span;
                if (coef == 1) oracle_add_mem(dst, arena + base, len);
                else           oracle_muladd_mem(dst, coef, arena + base, len);
            } else if (kind == I_ACC3) {
                const uint8_t c1 = (uint8_t)(w[0] >> 8), c2 = (uint8_t)(w[0] >> 16);
                const size_t base = (size_t)w[1] * 64u;
                const uint32_t len = w[2];
                if (len > span || base + len > arena_bytes) { free(acc); return -8; }
                oracle_add_mem(acc, arena + base, len);
                oracle_muladd_mem(acc + span, c1, arena + base, len);
                oracle_muladd_mem(acc + 2 * (size_t)span, c2, arena + base, len);
            } else if (kind == I_ACCR) {
                if (k + 1 >= count) { free(acc); return -10; }
                const uint32_t* r = w + 4;
                if ((r[0] & 0xff) != I_RANGE) { free(acc); return -11; }
                const uint32_t mode = (w[0] >> 8) & 0xff, p = (w[0] >> 16) & 0xff;
                const uint32_t len = w[2], n = w[3], stride = r[1], col0 = r[2], cstep = r[3];
                if (len > span) { free(acc); return -12; }
                const uint32_t* tg = NULL;
                if (mode == R_MULTI || mode == R_DENSE) {
                    if (k + 2 >= count) { free(acc); return -15; }
                    tg = w + 8;
                    if ((tg[0] & 0xff) != (mode == R_MULTI ? I_TARGETS : I_COEFS)) { free(acc); return -16; }
                    if (mode == R_DENSE && p < 2 && k + 2 + tg[3] >= count) { free(acc); return -18; }
                }
                if (mode == R_DENSE && p >= 2) {
                    /* p targets: COEFS_t (cap = ADJ words | hi << 16) + its ADJ words each; target t
                       takes rows e < hi_t into acc_t */
                    const uint32_t* cw[3] = { NULL, NULL, NULL };
                    uint32_t at = k + 2;
                    if (p > 3) { free(acc); return -19; }
                    for (uint32_t t = 0; t < p; ++t) {
                        if (at >= count) { free(acc); return -20; }
                        cw[t] = instrs + 4 * (size_t)(first + at);
                        if ((cw[t][0] & 0xff) != I_COEFS) { free(acc); return -21; }
                        at += 1 + (cw[t][3] & 0xffffu);
                    }
                    if (at > count) { free(acc); return -22; }
                    for (uint32_t e = 0; e < n; ++e) {
                        const size_t base = ((size_t)w[1] + (size_t)e * stride) * 64u;
                        const unsigned col = (unsigned)(((uint64_t)col0 + (uint64_t)e * cstep) % 0x400000u);
                        if (base + len > arena_bytes) { free(acc); return -13; }
                        const uint8_t cx = oracle_column_value(col), cx2 = oracle_gf_sqr(cx);
                        for (uint32_t t = 0; t < p; ++t) {
                            if (e >= (cw[t][3] >> 16)) continue;
                            const uint64_t ow = (uint64_t)cw[t][1] | ((uint64_t)(cw[t][2] & 0xffffu) << 32);
                            const uint8_t rx = (uint8_t)(cw[t][2] >> 16);
                            const unsigned b = (unsigned)(ow >> (6u * (col % 8u))) & 63u;
                            const uint8_t sdir = (uint8_t)((b & 1u) ^ ((b & 2u) ? cx : 0u) ^ ((b & 4u) ? cx2 : 0u));
                            const uint8_t tprod = (uint8_t)(((b >> 3) & 1u) ^ ((b & 16u) ? cx : 0u) ^ ((b & 32u) ? cx2 : 0u));
                            uint8_t g = (uint8_t)(sdir ^ oracle_gf_mul(rx, tprod));
                            for (uint32_t aw = 0; aw < (cw[t][3] & 0xffffu); ++aw)
                                for (unsigned q = 0; q < 4; ++q) {
                                    const uint32_t d = cw[t][4 + 4 * aw + q];
                                    if ((d >> 16) == e) g ^= (uint8_t)(d >> 8);
                                }
                            if (g) oracle_muladd_mem(acc + (size_t)t * span, g, arena + base, len);
                        }
                    }
                    k = at - 1;  /* the loop's ++k moves past the last ADJ word */
                    continue;
                }
                for (uint32_t e = 0; e < n; ++e) {
                    const size_t base = ((size_t)w[1] + (size_t)e * stride) * 64u;
                    const unsigned col = (unsigned)(((uint64_t)col0 + (uint64_t)e * cstep) % 0x400000u);
                    if (base + len > arena_bytes) { free(acc); return -13; }
                    const uint8_t* row = arena + base;
                    if (mode == R_LANE3) {
                        const uint8_t cx = oracle_column_value(col);
                        oracle_add_mem(acc, row, len);
                        oracle_muladd_mem(acc + span, cx, row, len);
                        oracle_muladd_mem(acc + 2 * (size_t)span, oracle_gf_sqr(cx), row, len);
                    } else if (mode == R_CAUCHY) {
                        /* w0 bits 24..31: scale s (0 or 1: none) -- decoder elimination runs */
                        const uint8_t s = (uint8_t)(w[0] >> 24), ce = oracle_cauchy_element(p, col % 64u);
                        oracle_muladd_mem(acc, s > 1 ? oracle_gf_mul(s, ce) : ce, row, len);
                    } else if (mode == R_CONST) {
                        oracle_muladd_mem(acc, (uint8_t)p, row, len);
                    } else if (mode == R_DENSE) {
                        const uint64_t ow = (uint64_t)tg[1] | ((uint64_t)(tg[2] & 0xffffu) << 32);
                        const uint8_t rx = (uint8_t)(tg[2] >> 16);
                        const unsigned b = (unsigned)(ow >> (6u * (col % 8u))) & 63u;
                        const uint8_t cx = oracle_column_value(col), cx2 = oracle_gf_sqr(cx);
                        const uint8_t sdir = (uint8_t)((b & 1u) ^ ((b & 2u) ? cx : 0u) ^ ((b & 4u) ? cx2 : 0u));
                        const uint8_t tprod = (uint8_t)(((b >> 3) & 1u) ^ ((b & 16u) ? cx : 0u) ^ ((b & 32u) ? cx2 : 0u));
                        uint8_t g = (uint8_t)(sdir ^ oracle_gf_mul(rx, tprod));
                        /* ADJ words (COEFS.cap of them): idx << 16 | delta << 8 additions */
                        for (uint32_t w = 0; w < tg[3]; ++w)
                            for (unsigned q = 0; q < 4; ++q) {
                                const uint32_t d = tg[4 + 4 * w + q];
                                if ((d >> 16) == e) g ^= (uint8_t)(d >> 8);
                            }
                        /* w0 bits 24..31 (one target): scale s of every coefficient (0 or 1: none) --
                           a decoder elimination run scaled by the solve */
                        const uint8_t s = (uint8_t)(w[0] >> 24);
                        if (s > 1) g = oracle_gf_mul(s, g);
                        if (g) oracle_muladd_mem(acc, g, row, len);
                    } else if (mode == R_MULTI) {
                        for (unsigned a = 0; a < 3; ++a) {
                            const uint32_t t = tg[1 + a], kind = t & 3, tp = (t >> 2) & 0xff;
                            if (e < ((t >> 10) & 0x7ff) || e >= (t >> 21)) continue;
                            uint8_t* dst = acc + (size_t)a * span;
                            if (kind == R_CONST) oracle_add_mem(dst, row, len);
                            else if (kind == R_CAUCHY) oracle_muladd_mem(dst, oracle_cauchy_element(tp, col % 64u), row, len);
                            else { free(acc); return -17; }
                        }
                    } else {
                        free(acc); return -14;
                    }
                }
                k += mode == R_DENSE ? 2 + tg[3] : mode == R_MULTI ? 2 : 1; /* RANGE (+ TARGETS / COEFS + ADJ) */
            } else if (kind == I_STOREC) {
                const uint8_t c[3] = { (uint8_t)(w[0] >> 8), (uint8_t)(w[0] >> 16), (uint8_t)(w[0] >> 24) };
                const size_t base = (size_t)w[1] * 64u;
                const uint32_t len = w[2], cap = w[3];
                if (len > span || len > cap || base + cap > arena_bytes) { free(acc); return -9; }
                memset(arena + base, 0, cap);
                for (unsigned a = 0; a < 3; ++a)
                    if (c[a]) oracle_muladd_mem(arena + base, c[a], acc + (size_t)a * span, len);
            } else if (kind == I_STORE) {
                if (k + 1 >= count) { free(acc); return -4; }
                const uint32_t* f = w + 4;
                if ((f[0] & 0xff) != I_FOOTER) { free(acc); return -5; }
                const uint32_t flen = (w[0] >> 8) & 0xff;
                const uint32_t a = (w[0] >> 16) & 0xff;
                const size_t base = (size_t)w[1] * 64u;
                const uint32_t len = w[2], cap = w[3];
                if (a > 2 || len > span || flen > 8 || len + flen > cap || base + cap > arena_bytes) {
                    free(acc); return -6;
                }
                uint8_t footer[8];
                for (unsigned b = 0; b < 4; ++b) {
                    footer[b]     = (uint8_t)(f[1] >> (8 * b));
                    footer[4 + b] = (uint8_t)(f[2] >> (8 * b));
                }
                memcpy(arena + base, acc + (size_t)a * span, len);
                memcpy(arena + base + len, footer, flen);
                memset(arena + base + len + flen, 0, cap - len - flen);
                ++k; /* consumed the FOOTER word */
            } else {
                free(acc); return -7;
            }
        }
    }
    free(acc);
    return 0;
}

/* ------------------------------------------------------------------------------------------
   Known answers (computed from the reference binary).
   ------------------------------------------------------------------------------------------ */
int oracle_self_test(void)
{
    int r = oracle_gf_init();
    if (r) return r;
    if (oracle_gf_polynomial() != 0x14d) return -20;
    if (oracle_gf_mul(2, 0x80) != 0x4d) return -21;
    if (oracle_gf_mul(0xaa, 0x6c) != 0x7c) return -22;
    if (oracle_gf_inv(2) != 0xa6) return -23;
    if (oracle_gf_sqr(3) != 0x05) return -24;
    if (oracle_gf_exp(1) != 2 || oracle_gf_exp(2) != 4 || oracle_gf_exp(3) != 8 || oracle_gf_exp(8) != 77) return -25;
    static const unsigned op0[8] = { 23, 54, 36, 54, 56, 48, 41, 2 };
    static const unsigned op1[8] = { 1, 1, 20, 6, 1, 14, 50, 26 };
    for (unsigned l = 0; l < 8; ++l) {
        if (oracle_row_opcode(l, 0) != op0[l]) return -26;
        if (oracle_row_opcode(l, 1) != op1[l]) return -27;
    }
    static const unsigned cx[8] = { 3, 202, 148, 94, 40, 239, 185, 131 };
    for (unsigned c = 0; c < 8; ++c) if (oracle_column_value(c) != cx[c]) return -28;
    for (unsigned rr = 0; rr < 4; ++rr) if (oracle_row_value(rr) != rr + 2) return -29;
    if (oracle_cauchy_element(0, 0) != 107 || oracle_cauchy_element(1, 5) != 255) return -30;
    oracle_pcg p;
    oracle_pcg_seed(&p, 0, 100);
    /* Values printed by the reference PCGRandom (SURVEY.md lists them in reverse order). */
    if (oracle_pcg_next(&p) != 1435445633u) return -31;
    if (oracle_pcg_next(&p) != 2998190369u) return -32;
    if (oracle_pcg_next(&p) != 1706867612u) return -33;
    return 0;
}
