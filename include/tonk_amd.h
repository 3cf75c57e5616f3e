/*
    tonk_amd.h -- additive batched API of the MI355X Siamese engine (not part of siamese.h).

    A session runs many independent connection streams (encoder + decoder + lossy channel per
    stream, tonk_amd/csrc/workload.h) whose packets live in HBM.  Host worker threads run the
    codec control planes; every step's byte work is one merged device program executed level
    by level on the GPU while the host builds the next step.  This is the device-resident path
    the benchmark measures; the siamese.h ABI is the drop-in path.
*/
#ifndef TONK_AMD_H
#define TONK_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tamd_session_params {
    uint32_t device;
    uint32_t n_streams;        /* streams on this device */
    uint32_t stream_base;      /* global id of the first stream (seeds 1000+id / 2000+id) */
    uint32_t n_threads;        /* host worker threads */
    uint32_t n_originals;      /* originals per stream for the whole session */
    uint32_t payload_min, payload_max;
    uint32_t loss_thresh, ge_enable, gb_thresh, bg_thresh, loss_on_recovery;
    uint32_t fec_rate_q16, ack_every, ack_bytes, arq_lag, flush_max;
    uint32_t record;           /* 1: keep per-stream transcripts (parity checks, not timed).  The
                                  schedule is the timed one (early launch, rows released at their
                                  program's completion); the rows are digested on the launch
                                  stream right after the launch that completes their program. */
    uint32_t stage_host;       /* packets start and end in pinned host memory (the PCIe-inclusive
                                  rate), a bit mask of the connection's two ends:
                                  1 the sender (originals H2D into the encoder, recovery packets
                                  D2H), 2 the receiver (originals and received recovery packets
                                  H2D into the decoder, recovered originals D2H); 3 both */
    uint64_t arena_bytes;
    uint32_t rtx_every;        /* retransmission tick every rtx_every originals (0: off) under a
                                  virtual clock advancing rtx_msec per original (workload.h) */
    uint32_t rtx_msec;
    uint32_t input_pool;       /* > 0: only this many input rows per side are generated and original
                                  i reads row i mod input_pool (the bench's long streams: the codecs'
                                  work does not depend on the payload bytes, as the reference
                                  timing leg's payload pool).  Ignored with record or stage_host. */
    uint32_t hold_full;        /* 1: window-full behaviour of the workload (workload.h hold_full): the
                                  sender asks siamese_encoder_is_ready before every add and a refused
                                  add waits for an acknowledgement; single adds only */
} tamd_session_params;

/* Summary counters (tamd_session_summary indices). */
enum {
    TAMD_SUM_ORIGINALS, TAMD_SUM_LOST_ORIGINALS, TAMD_SUM_RECOVERIES, TAMD_SUM_LOST_RECOVERIES,
    TAMD_SUM_RECOVERED, TAMD_SUM_ARQ, TAMD_SUM_MISSING_AT_END, TAMD_SUM_PAYLOAD_BYTES,
    TAMD_SUM_ALG_BYTES,        /* algorithmic HBM bytes (SURVEY.md s8(d) B_alg) */
    TAMD_SUM_ACC_BYTES,        /* bytes read by ACC instructions (op-trace diagnostic) */
    TAMD_SUM_STORE_BYTES,      /* bytes written by STORE instructions */
    TAMD_SUM_PROGRAMS, TAMD_SUM_LAUNCHES, TAMD_SUM_OPS, TAMD_SUM_INSTRS, TAMD_SUM_UPLOAD_BYTES,
    TAMD_SUM_DISABLED_CODECS,
    TAMD_SUM_H2D_BYTES,        /* stage_host: bytes copied host -> device */
    TAMD_SUM_D2H_BYTES,        /* stage_host: bytes copied device -> host */
    TAMD_SUM_D2H_COPY_US,      /* stage_host: duration of the D2H copies themselves (HIP events) */
    TAMD_SUM_COUNT
};

void* tamd_session_create(const tamd_session_params* p, char* err, size_t err_len);
int   tamd_session_generate(void* s);                 /* write all input rows in HBM (untimed) */
int   tamd_session_step(void* s, uint32_t originals); /* host work + enqueue; device is async */
int   tamd_session_wait(void* s);                     /* wait for every enqueued program */
int   tamd_session_finish(void* s);                   /* end-of-stream flush, then wait */
int   tamd_session_summary(void* s, uint64_t* out, unsigned n);
void  tamd_session_set_timing(void* s, int on);       /* HIP events around every launch */
double tamd_session_kernel_ms(void* s, uint64_t* launches);
/* Host time split of the steps so far, milliseconds (summed over steps).  Pass schedule:
   [0] control planes (wall, all workers)   [1] sum over workers of their own control-plane time
   [2] program layout + staging-slot wait    [3] parallel program fill + epoch close
   [4] upload + launch enqueue               [5] max over workers of their control-plane time
   Free-running schedule (tamd_session_schedule = 1):
   [0] caller waiting for a program's parts [1] sum over workers of control plane + part
   [2] opening a program (its slot's wait)   [3] stream steps run by another thread (count)
   [4] closing (item merge, upload) + launch [5] max over workers of [1]'s share
   Both: [6] wait for the staging slot        [7] H2D copy enqueue
   [8] longest single H2D enqueue             [9] staging-slot reallocations (count) */
void  tamd_session_host_ms(void* s, double out[10]);
/* The session's device arena: base address and mapped bytes (diagnostics: placement studies). */
void  tamd_session_arena(void* s, uint64_t* base, uint64_t* bytes);
/* Transcript of one stream in the oracle's text format (record mode). Returns bytes needed. */
size_t tamd_session_transcript(void* s, uint32_t stream, char* buf, size_t cap);
void  tamd_session_destroy(void* s);
/* The session's last error ("" when none). */
const char* tamd_session_error(void* s);

/* Test hook: the codecs' millisecond clock (GetTimeMsec: send times, RTO, retransmit) is read
   from `fn` instead of the monotonic clock (null restores it).  Used to compare
   siamese_encoder_retransmit with the reference under a virtual clock. */
void  tamd_set_clock(uint64_t (*fn)(void));

/* The CPUs the session's worker threads are pinned to (count returned; empty = not pinned). */
unsigned tamd_session_cpus(void* s, int* out, unsigned cap);
/* The session's host schedule: 1 = free-running streams with parallel program assembly (worker
   threads beside the caller, level pipelining), 0 = one pass over the streams per step.  It
   decides what tamd_session_host_ms's entries hold (tonk_amd.Session.host_phases). */
int tamd_session_schedule(void* s);
/* Host-core plan of one GPU's worker pool (pure, no device needed): `dev_cpulists` holds every
   device's NUMA local_cpulist separated by ';', `node_cores` the usable cores of `device`'s node
   (one CPU per core).  The devices sharing that node split its cores into equal contiguous
   shares in device order; `slot_override` "k/n" (TONK_AMD_CPU_SLOT) fixes the share instead.
   Returns the number of CPUs of the share (written to out[0..cap)). */
unsigned tamd_cpu_share(const char* dev_cpulists, unsigned device, const char* node_cores,
                        const char* slot_override, int* out, unsigned cap);

/* Device self test: v_perm GF(2^8) multiply against the host tables (all 65536 products). */
int   tamd_device_selftest(uint32_t device, char* err, size_t err_len);

#ifdef __cplusplus
}
#endif
#endif
