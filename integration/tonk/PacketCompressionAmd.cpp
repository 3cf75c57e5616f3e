// PacketCompressionAmd.cpp -- Tonk-side binding of the MI355X compressor (include/tonk_compress.h).
// A maintainer builds this file in place of the reference's PacketCompression.cpp; it defines the
// members of the classes declared by the reference's PacketCompression.h, which it includes
// unchanged, so Tonk's sources (TonkineseOutgoing.cpp:462, 865; TonkineseIncoming.cpp) link
// as they are:
//   * tonk::MessageCompressor (PacketCompression.h:92-140) -> tamd_compressor_* on the GPU.  The
//     class's zstd context slot carries the GPU handle; its History ring is still kept, as the
//     reference's Compress does (PacketCompression.cpp:79-83), for code that inspects it.
//   * tonk::MessageDecompressor (PacketCompression.h:210-260) stays the reference's receive side:
//     zstd block decoding against the same 24,000-byte ring (PacketCompression.cpp:120-216).
// oracle/tonk.mk links Tonk's unit_tests with this file (unit_tests_amd_lz).
#include "PacketCompression.h"

#include "tonk_compress.h"  // include/ (oracle/tonk.mk: -I../include)

#include <string.h>

namespace tonk {

Result MessageCompressor::Initialize(unsigned maxCompressedMessagesBytes) {
    MaxCompressedMessagesBytes = maxCompressedMessagesBytes;
    void* handle = tamd_compressor_create(maxCompressedMessagesBytes);
    if (!handle)
        return Result("MessageCompressor::Initialize", "tamd_compressor_create failed (no gfx950 device?)",
                      ErrorType::Zstd);
    CCtx = reinterpret_cast<ZSTD_CCtx*>(handle);
    return Result::Success();
}

MessageCompressor::~MessageCompressor() {
    if (CCtx) tamd_compressor_destroy(CCtx);
}

Result MessageCompressor::Compress(const uint8_t* data, unsigned bytes, uint8_t* destBuffer, unsigned& writtenBytes) {
    writtenBytes = 0;
    void* slot = History.Allocate(MaxCompressedMessagesBytes);
    memcpy(slot, data, bytes);
    History.Commit(bytes);
    unsigned written = 0;
    const int rc = tamd_compressor_compress(CCtx, data, bytes, destBuffer, &written);
    if (rc != 0)
        return Result("MessageCompressor::Compress", "tamd_compressor_compress failed", ErrorType::Zstd, rc);
    writtenBytes = written;  // 0: send the message as is (the peer calls InsertUncompressed)
    return Result::Success();
}

Result MessageDecompressor::Initialize(unsigned maxCompressedMessagesBytes) {
    MaxCompressedMessagesBytes = maxCompressedMessagesBytes;
    DCtx = ZSTD_createDCtx();
    if (!DCtx) return Result("MessageDecompressor::Initialize", "ZSTD_createDCtx failed", ErrorType::Zstd);
    const size_t r = ZSTD_decompressBegin(DCtx);
    if (ZSTD_isError(r))
        return Result("MessageDecompressor::Initialize", "ZSTD_decompressBegin failed", ErrorType::Zstd, r);
    return Result::Success();
}

MessageDecompressor::~MessageDecompressor() {
    if (DCtx) ZSTD_freeDCtx(DCtx);
}

void MessageDecompressor::InsertUncompressed(const uint8_t* data, unsigned bytes) {
    if (bytes > MaxCompressedMessagesBytes) return;
    void* slot = History.Allocate(MaxCompressedMessagesBytes);
    memcpy(slot, data, bytes);
    ZSTD_insertBlock(DCtx, slot, bytes);
    History.Commit(bytes);
}

Result MessageDecompressor::Decompress(const void* data, unsigned bytes, Decompressed& decompressed) {
    void* slot = History.Allocate(MaxCompressedMessagesBytes);
    const size_t r = ZSTD_decompressBlock(DCtx, slot, MaxCompressedMessagesBytes, data, bytes);
    if (r == 0 || ZSTD_isError(r))
        return Result("MessageDecompressor::Decompress", std::string("ZSTD_decompressBlock failed: ") +
                      ZSTD_getErrorName(r), ErrorType::Zstd, r);
    History.Commit((unsigned)r);
    decompressed.Data = reinterpret_cast<const uint8_t*>(slot);
    decompressed.Bytes = (unsigned)r;
    return Result::Success();
}

} // namespace tonk
