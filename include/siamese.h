/*
    siamese.h -- C ABI of the MI355X Siamese FEC engine (tonk_amd).

    Drop-in replacement for the reference codec's public header (catid/tonk siamese.h,
    SIAMESE_VERSION 5): identical function names, argument meaning, result codes, struct
    layouts and constants, so TonkineseOutgoing.cpp / TonkineseIncoming.cpp compile and link
    against libtonk_amd.so unchanged.  Every declaration below cites the reference interface it
    replaces (/root/reference/siamese.h line numbers).

    Execution: the codec state machines run on the host; all GF(2^8) byte work (running sums,
    recovery rows, elimination, triangular solve) runs as HIP kernels on an MI355X (gfx950).
    There is no CPU fallback: siamese_init() fails with Siamese_Disabled when no gfx950 device
    is present.

    Threading: as in the reference, one codec object must not be used from two threads at once;
    different codecs may be used concurrently (calls are serialized internally).
*/
#ifndef CAT_SIAMESE_H
#define CAT_SIAMESE_H

/* Library header version (siamese.h:91). */
#define SIAMESE_VERSION 5

/* Export macros (siamese.h:97-109). */
#if defined(SIAMESE_BUILDING)
# if defined(SIAMESE_DLL)
#  define SIAMESE_EXPORT __declspec(dllexport)
# else
#  define SIAMESE_EXPORT __attribute__((visibility("default")))
# endif
#else
# if defined(SIAMESE_DLL)
#  define SIAMESE_EXPORT __declspec(dllimport)
# else
#  define SIAMESE_EXPORT extern
# endif
#endif

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Initialization (siamese.h:122-129) ---- */
SIAMESE_EXPORT int siamese_init_(int version);
#define siamese_init() siamese_init_(SIAMESE_VERSION)

/* ---- Shared constants and types (siamese.h:135-199) ---- */
typedef enum SiameseResultT
{
    Siamese_Success           = 0,
    Siamese_InvalidInput      = 1,
    Siamese_NeedMoreData      = 2,
    Siamese_MaxPacketsReached = 3,
    Siamese_DuplicateData     = 4,
    Siamese_Disabled          = 5,
    SiameseResult_Count,
    SiameseResult_Padding = 0x7fffffff
} SiameseResult;

#define SIAMESE_RECOVERY_NUM_MIN         0
#define SIAMESE_RECOVERY_NUM_MAX       255
#define SIAMESE_RECOVERY_NUM_COUNT     256
#define SIAMESE_MAX_PACKETS          16000
#define SIAMESE_PACKET_NUM_MIN           0
#define SIAMESE_PACKET_NUM_MAX    0x3fffff
#define SIAMESE_PACKET_NUM_COUNT  0x400000
#define SIAMESE_PACKET_NUM_BITS         22
#define SIAMESE_PACKET_NUM_INC(x)  ( (x + 1) & (SIAMESE_PACKET_NUM_COUNT - 1) )
#define SIAMESE_MIN_PACKET_BYTES         1
#define SIAMESE_MAX_PACKET_BYTES 536870911 /* 0x1fffffff */
#define SIAMESE_MAX_ENCODE_OVERHEAD     8
#define SIAMESE_ACK_MIN_BYTES          16

struct SiameseOriginalPacket
{
    unsigned PacketNum;
    unsigned DataBytes;
    const unsigned char* Data;
};

struct SiameseRecoveryPacket
{
    unsigned DataBytes;
    const unsigned char* Data;
};

/* ---- Encoder (siamese.h:205-352) ---- */
typedef struct SiameseEncoderImpl { int impl; }* SiameseEncoder;

SIAMESE_EXPORT SiameseEncoder siamese_encoder_create();                               /* :213 */
SIAMESE_EXPORT void siamese_encoder_free(SiameseEncoder encoder);                     /* :216 */
SIAMESE_EXPORT SiameseResult siamese_encoder_is_ready(SiameseEncoder encoder);        /* :230 */
SIAMESE_EXPORT SiameseResult siamese_encoder_add(SiameseEncoder encoder,
                                                 SiameseOriginalPacket* packet);      /* :248 */
SIAMESE_EXPORT SiameseResult siamese_encoder_get(SiameseEncoder encoder,
                                                 SiameseOriginalPacket* packet);      /* :262 */
SIAMESE_EXPORT SiameseResult siamese_encoder_remove_before(SiameseEncoder encoder,
                                                           unsigned firstKeptPacketNum); /* :278 */
SIAMESE_EXPORT SiameseResult siamese_encoder_ack(SiameseEncoder encoder, const void* buffer,
                                                 unsigned bytes,
                                                 unsigned* nextExpectedPacketNum);    /* :299 */
SIAMESE_EXPORT SiameseResult siamese_encoder_retransmit(SiameseEncoder encoder,
                                                        SiameseOriginalPacket* original); /* :327 */
SIAMESE_EXPORT SiameseResult siamese_encode(SiameseEncoder encoder,
                                            SiameseRecoveryPacket* recovery);         /* :349 */

/* ---- Decoder (siamese.h:358-483) ---- */
typedef struct SiameseDecoderImpl { int impl; }* SiameseDecoder;

SIAMESE_EXPORT SiameseDecoder siamese_decoder_create();                               /* :366 */
SIAMESE_EXPORT void siamese_decoder_free(SiameseDecoder decoder);                     /* :369 */
SIAMESE_EXPORT SiameseResult siamese_decoder_add_original(SiameseDecoder decoder,
                                                          const SiameseOriginalPacket* packet); /* :381 */
SIAMESE_EXPORT SiameseResult siamese_decoder_add_recovery(SiameseDecoder decoder,
                                                          const SiameseRecoveryPacket* packet); /* :399 */
SIAMESE_EXPORT SiameseResult siamese_decoder_get(SiameseDecoder decoder,
                                                 SiameseOriginalPacket* packet);      /* :420 */
SIAMESE_EXPORT SiameseResult siamese_decoder_is_ready(SiameseDecoder decoder);        /* :430 */
SIAMESE_EXPORT SiameseResult siamese_decode(SiameseDecoder decoder,
                                            SiameseOriginalPacket** packetsPtrOut,
                                            unsigned* countOut);                      /* :457 */
SIAMESE_EXPORT SiameseResult siamese_decoder_ack(SiameseDecoder decoder, void* buffer,
                                                 unsigned byteLimit, unsigned* usedBytes); /* :478 */

/* ---- Statistics (siamese.h:489-583) ---- */
typedef enum SiameseEncoderStatsT
{
    SiameseEncoderStats_OriginalCount,
    SiameseEncoderStats_OriginalBytes,
    SiameseEncoderStats_RecoveryCount,
    SiameseEncoderStats_RecoveryBytes,
    SiameseEncoderStats_RetransmitCount,
    SiameseEncoderStats_RetransmitBytes,
    SiameseEncoderStats_AckCount,
    SiameseEncoderStats_AckBytes,
    SiameseEncoderStats_MemoryUsed,   /* engine: host + device bytes held by the codec */
    SiameseEncoderStats_Count
} SiameseEncoderStats;

SIAMESE_EXPORT SiameseResult siamese_encoder_stats(SiameseEncoder encoder, uint64_t* statsOut,
                                                   unsigned statsCount);              /* :527 */

typedef enum SiameseDecoderStatsT
{
    SiameseDecoderStats_OriginalCount,
    SiameseDecoderStats_OriginalBytes,
    SiameseDecoderStats_RecoveryCount,
    SiameseDecoderStats_RecoveryBytes,
    SiameseDecoderStats_AckCount,
    SiameseDecoderStats_AckBytes,
    SiameseDecoderStats_DupedOriginalCount,
    SiameseDecoderStats_SolveSuccessCount,
    SiameseDecoderStats_SolveFailCount,
    SiameseDecoderStats_DupedRecoveryCount,
    SiameseDecoderStats_MemoryUsed,   /* engine: host + device bytes held by the codec */
    SiameseDecoderStats_Count
} SiameseDecoderStats;

SIAMESE_EXPORT SiameseResult siamese_decoder_stats(SiameseDecoder decoder, uint64_t* statsOut,
                                                   unsigned statsCount);              /* :579 */

#ifdef __cplusplus
}
#endif

#endif /* CAT_SIAMESE_H */
