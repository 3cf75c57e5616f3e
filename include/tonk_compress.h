/*
    tonk_compress.h -- Tonk's upstream compression step on MI355X.

    Replaces tonk::MessageCompressor (PacketCompression.h:92-140, PacketCompression.cpp:28-118):
    messages of a reliable in-order stream are compressed against the stream's history so that
    the reference's tonk::MessageDecompressor (PacketCompression.cpp:120-216: zstd
    ZSTD_decompressBlock / ZSTD_insertBlock over a 24,000-byte history ring) restores them
    unchanged.  Each compressed message is one zstd compressed block (RFC 8878) built on the GPU
    (tonk_amd/csrc/lz.hip); a message that does not shrink is reported with written = 0 and is
    sent as is (the decompressor then calls InsertUncompressed), exactly the reference contract.
    There is no CPU fallback: without a gfx950 device creation fails.
*/
#ifndef TONK_COMPRESS_H
#define TONK_COMPRESS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* MessageCompressor::Initialize (PacketCompression.cpp:28-61): null when no device is usable. */
void* tamd_compressor_create(unsigned max_compressed_message_bytes);

/* MessageCompressor::Compress (PacketCompression.cpp:70-118): 0 on success with *written = the
   compressed bytes in dest (at most max_compressed_message_bytes), or 0 when the message should be
   sent uncompressed; negative on a device error (the compressor then stays failed, as the
   reference's "compressor has stopped unexpectedly").  bytes must be 1..max. */
int   tamd_compressor_compress(void* c, const uint8_t* data, unsigned bytes, uint8_t* dest, unsigned* written);

void  tamd_compressor_destroy(void* c);

/* The device-resident batch (bench.py --workload compress): n_streams independent compressor
   streams, stream s's messages back to back at dev_data + s * stride (device memory, with at
   least 32 readable bytes after a stream's last message), message k of stream s is
   lens[s * n_msgs + k] bytes (1..max_bytes).  Every stream starts fresh (history
   empty) and applies MessageCompressor's Allocate(max)/Commit ring rule.  Outputs: message
   (s, k) compressed at dev_out + (s * n_msgs + k) * max_bytes, written_host[s * n_msgs + k]
   (0: send uncompressed).  msgs_per_job consecutive messages of a stream share one wave's hash
   table (0: chosen so that the jobs fill the device's wave slots once).  *kernel_ms (optional) = the compression kernel's duration.  Returns 0 or negative. */
int   tamd_compress_batch(const void* dev_data, uint64_t stride, uint32_t n_streams, uint32_t n_msgs,
                          const uint32_t* lens, uint32_t max_bytes, void* dev_out, uint32_t* written_host,
                          uint32_t msgs_per_job, float* kernel_ms);

/* The same batch from host memory: host_data is copied to the device first and the compressed
   messages come back to host_out (n_streams * n_msgs * max_bytes bytes). */
int   tamd_compress_batch_host(const void* host_data, uint64_t stride, uint32_t n_streams, uint32_t n_msgs,
                               const uint32_t* lens, uint32_t max_bytes, void* host_out, uint32_t* written_host,
                               uint32_t msgs_per_job, float* kernel_ms);

#ifdef __cplusplus
}
#endif

#endif
