// serve.h -- the launch-free submission path of the siamese.h C ABI: the records shared by the
// host (serve.cpp, capi.cpp) and the persistent executor kernel tamd_serve (kernels.hip).
//
// A codec's call builds ONE command in host memory -- the packets to land in the arena (staged
// since the codec's last program), the codec's pending program (its levels, ops, instructions
// and work items) and the rows to read back into the caller's pinned buffer -- posts its address
// into a ring in host-coherent pinned memory and spins on a completion word.  No HIP call, no
// kernel launch, no event: the resident kernel's dispatcher (block 0, one lane) polls the ring,
// hands each command to a worker workgroup through device memory, and the worker copies the
// command into its LDS, lands the packets, runs the program's levels with workgroup barriers
// between them, writes the reads to the host and stores the completion word.
#pragma once
#include <stdint.h>

#define TAMD_SERVE_THREADS 1024u          /* one worker = one 16-wave workgroup = one CU */
#define TAMD_SERVE_WAVES (TAMD_SERVE_THREADS / 64u)
#define TAMD_SERVE_CMD_BYTES (64u << 10)  /* LDS area one command fits in (else: launch path) */
#define TAMD_SERVE_MAX_LEVELS 32u

/* A command's descriptor is 6 tagged granules, each one 8-byte word {tag = low 32 bits of
   index + 1, value}: 0/1 the command's host address (low/high half), 2/3 the completion word's,
   4 the value the worker stores there (the tag), 5 the command's bytes.  The host writes them
   into the ring slot with 8-byte stores in any order; the dispatcher copies them unchanged into
   the device work list with write-through stores; a reader takes a descriptor once all six tags
   match -- the data is the flag, no fence on either hand-off (MI355X_MICROARCH.md, R2). */
#define TAMD_SERVE_GRANULES 6u
typedef struct tamd_serve_slot {  /* host ring slot and device work-list entry, 64 B */
    uint64_t g[TAMD_SERVE_GRANULES];
    uint64_t pad[2];
} tamd_serve_slot;
static inline uint64_t tamd_granule(uint64_t index, uint32_t value) {
    return ((uint64_t)(uint32_t)(index + 1) << 32) | value;
}

/* Host-side control words (coherent pinned memory), each on a line of its own. */
typedef struct tamd_serve_host {
    uint64_t stop;        /* host: the dispatcher ends at its next poll (process exit) */
    uint64_t pad0[15];
    uint64_t consumed;    /* dispatcher: ring slots below this index have been handed on */
    uint64_t pad1[15];
    uint64_t exit_tail;   /* dispatcher, when it ends: the first index it did not take ... */
    uint64_t exited_gen;  /* ... and then its instance's generation (release-stored after) */
    uint64_t pad2[14];
    /* diagnostics (printed when a command times out): [0] dispatcher start stamp, [1] its polls /
       1024, [2] the index it waits for; [3] the stage of command 0 (the start-up probe: 1 claimed,
       2 seen, 3 in LDS, 4 landed, 5 program run, 6 reads written, 7 done stored), [4] its block */
    uint64_t dbg[16];
} tamd_serve_host;

/* Device state of one kernel instance (hipMalloc; reset before each launch). */
typedef struct tamd_serve_dev {
    uint64_t claim;       /* workers' next relative index (atomic add) */
    uint64_t pad0[15];
    uint64_t quit;        /* dispatcher: no further command comes in this instance */
    uint64_t pad1[15];
    /* then: tamd_serve_slot wl[wl_size], the work list */
} tamd_serve_dev;

/* A command (16-B aligned, host memory; copied whole into the worker's LDS). */
typedef struct tamd_cmd {
    uint32_t bytes;       /* the whole command, this head included */
    uint32_t n_up, n_rd, levels;
    uint32_t off_up, off_rd, off_instr, off_ops;  /* byte offsets from the command's start */
    uint32_t off_items, n_items, n_instr, n_ops;
    uint32_t up_chunks;   /* > 0: the uploads' host bytes lie in increasing order within this many
                             16-byte chunks from the first one's address (one staging half), which
                             the worker's threads copy chunk by chunk, all in flight at once */
    uint32_t level_base[TAMD_SERVE_MAX_LEVELS + 3]; /* item index where level l starts (levels + 1) */
} tamd_cmd;

/* A transfer between host memory and an arena row: upload (host -> row) or read (row -> host).
   Host addresses and lengths are arbitrary; arena rows are 64-B aligned. */
typedef struct tamd_xfer {
    uint64_t host;
    uint32_t unit, len;   /* arena row (64-B units), bytes */
} tamd_xfer;

/* Kernel arguments (by value). */
typedef struct tamd_serve_args {
    const tamd_serve_slot* ring;   /* host ring (coherent) */
    tamd_serve_host* host;         /* host control words (coherent) */
    tamd_serve_dev* dev;           /* this instance's device state */
    uint8_t* arena;
    const uint32_t* gf;            /* device GF tables (kernels.hip TAMD_GF_DWORDS) */
    const uint8_t* zrow;           /* a zero row (the executor's dummy loads) */
    uint64_t tail0;                /* first ring index this instance dispatches */
    uint64_t idle_ticks;           /* the dispatcher ends after this long without a command (100 MHz ticks) */
    uint32_t ring_mask, wl_mask;
    uint32_t gen, pad;
} tamd_serve_args;
