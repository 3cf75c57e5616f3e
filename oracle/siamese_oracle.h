/*
    siamese_oracle.h -- TEST INFRASTRUCTURE ONLY.

    Plain-C CPU restatement of the Siamese FEC math used as the parity checker for the
    MI355X engine.  Nothing in the product (tonk_amd/, include/, the C-ABI library) links or
    calls this; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg do.

    Parity pinning: the restatement is checked against (a) the reference's own gf256 self-test
    and the known-answer values listed in SURVEY.md s8(c), and (b) golden fixtures produced by
    the reference codec itself compiled from /root/reference (oracle/Makefile -> oracle/_ref/).
*/
#ifndef SIAMESE_ORACLE_H
#define SIAMESE_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- GF(2^8), polynomial 0x14D (gf256.cpp:358-372) ---- */
int      oracle_gf_init(void);                 /* builds tables + runs the self-test; 0 = ok */
uint8_t  oracle_gf_mul(uint8_t x, uint8_t y);
uint8_t  oracle_gf_div(uint8_t x, uint8_t y);
uint8_t  oracle_gf_inv(uint8_t x);
uint8_t  oracle_gf_sqr(uint8_t x);
unsigned oracle_gf_polynomial(void);
uint8_t  oracle_gf_exp(unsigned i);            /* EXP table entry (0..1024) */
uint16_t oracle_gf_log(uint8_t x);             /* LOG table entry (LOG[0] = 512) */

void oracle_add_mem(uint8_t* x, const uint8_t* y, size_t n);             /* x ^= y      */
void oracle_muladd_mem(uint8_t* z, uint8_t y, const uint8_t* x, size_t n);/* z ^= y * x  */
void oracle_mul_mem(uint8_t* z, const uint8_t* x, uint8_t y, size_t n);  /* z  = y * x  */

/* ---- Code parameters / coefficient generators (SiameseCommon.h:80-218) ---- */
uint8_t  oracle_column_value(unsigned column);           /* CX */
uint8_t  oracle_row_value(unsigned row);                 /* RX */
unsigned oracle_row_opcode(unsigned lane, unsigned row); /* 6-bit opcode */
uint8_t  oracle_cauchy_element(unsigned row, unsigned column);

/* ---- PCG (SiameseTools.h:79-101) ---- */
typedef struct { uint64_t state, inc; } oracle_pcg;
void     oracle_pcg_seed(oracle_pcg* p, uint64_t y, uint64_t x);
uint32_t oracle_pcg_next(oracle_pcg* p);

/* ---- Serializers (SiameseSerializers.h) ---- */
typedef struct {
    unsigned Row, ColumnStart, SumCount, LDPCCount;
} oracle_recovery_meta;

unsigned oracle_serialize_length_header(unsigned length, uint8_t* out);       /* :566 */
int      oracle_deserialize_length_header(const uint8_t* in, unsigned avail, unsigned* length); /* :598 */
unsigned oracle_serialize_recovery_footer(const oracle_recovery_meta* m, uint8_t* out); /* :736 */
int      oracle_deserialize_recovery_footer(const uint8_t* buf, unsigned bytes,
                                            oracle_recovery_meta* m);          /* :759 */
unsigned oracle_serialize_nack_range(unsigned relStart, unsigned lossCountM1, uint8_t* out); /* :861 */
int      oracle_deserialize_nack_range(const uint8_t* in, unsigned avail,
                                       unsigned* relStart, unsigned* lossCountM1);      /* :934 */

/* ---- Direct (non-incremental) recovery-row definition ----
   Computes the data part of a recovery packet straight from its metadata and the framed
   original rows, without running sums (SiameseEncoder.cpp:1046-1254,
   :1296-1441).  get_row(ctx, column, &bytes) returns the framed row (length prefix + payload)
   for any column in [ColumnStart, ColumnStart + SumCount).  out must hold out_bytes bytes,
   where out_bytes is the recovery data length (packet bytes minus footer).  Returns 0 on
   success, -1 if a needed row is missing. */
typedef const uint8_t* (*oracle_get_row_fn)(void* ctx, unsigned column, unsigned* bytes);
int oracle_recovery_row(const oracle_recovery_meta* m, oracle_get_row_fn get_row, void* ctx,
                        uint8_t* out, unsigned out_bytes);

/* ---- CPU interpreter of the device program format (tonk_amd/csrc/program.h) ----
   Evaluates the same op/instruction stream the HIP executor runs, over a host arena whose
   rows are addressed in 64-byte units.  Used only to check the control plane on hosts
   without a GPU. */
int oracle_run_program(uint8_t* arena, size_t arena_bytes,
                       const uint32_t* ops, unsigned n_ops,
                       const uint32_t* instrs, unsigned n_instrs);

/* Known-answer self test of everything above; returns 0 when all pass. */
int oracle_self_test(void);

#ifdef __cplusplus
}
#endif
#endif
