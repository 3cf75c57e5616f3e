/* SiameseSerializers.h -- header-compatible little-endian field helpers and byte streams.

   Tonk includes SiameseSerializers.h beside siamese.h (TonkineseTools.h:62) and uses its POD
   readers/writers (the reference's SiameseSerializers.h:58-153) and the WriteByteStream /
   ReadByteStream cursors (:160-313) to build and parse its datagrams (TonkineseIncoming.cpp:251,
   TonkineseOutgoing.cpp:1352-1399, TonkineseSession.cpp, tests/BandwidthControlTest.cpp).  This
   header provides the same names and wire results for tonk_amd.  The codec's
   own packet-number, length and recovery-footer encodings live in the engine
   (tonk_amd/csrc/serial.h); they are not part of what Tonk calls.

   All helpers are little-endian and alignment-free (memcpy of the host's little-endian value:
   x86-64 and the GPU hosts are little-endian).  The *_Min4Bytes forms read or write four bytes
   of which the value uses three, as the reference's do: the buffer must hold four. */
#ifndef TONK_AMD_SIAMESE_SERIALIZERS_H
#define TONK_AMD_SIAMESE_SERIALIZERS_H

#include "siamese.h"
#include "SiameseTools.h"

#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace siamese {

template <typename T>
SIAMESE_FORCE_INLINE T LoadLE(const uint8_t* p) {
    T v;
    memcpy(&v, p, sizeof(T));
    return v;
}
template <typename T>
SIAMESE_FORCE_INLINE void StoreLE(uint8_t* p, T v) {
    memcpy(p, &v, sizeof(T));
}

SIAMESE_FORCE_INLINE uint16_t ReadU16_LE(const uint8_t* data) { return LoadLE<uint16_t>(data); }
SIAMESE_FORCE_INLINE uint32_t ReadU24_LE(const uint8_t* data) {
    return (uint32_t)data[0] | ((uint32_t)data[1] << 8) | ((uint32_t)data[2] << 16);
}
SIAMESE_FORCE_INLINE uint32_t ReadU24_LE_Min4Bytes(const uint8_t* data) { return LoadLE<uint32_t>(data) & 0xFFFFFFu; }
SIAMESE_FORCE_INLINE uint32_t ReadU32_LE(const uint8_t* data) { return LoadLE<uint32_t>(data); }
SIAMESE_FORCE_INLINE uint64_t ReadU64_LE(const uint8_t* data) { return LoadLE<uint64_t>(data); }

SIAMESE_FORCE_INLINE void WriteU16_LE(uint8_t* data, uint16_t value) { StoreLE<uint16_t>(data, value); }
SIAMESE_FORCE_INLINE void WriteU24_LE(uint8_t* data, uint32_t value) {
    data[0] = (uint8_t)value;
    data[1] = (uint8_t)(value >> 8);
    data[2] = (uint8_t)(value >> 16);
}
/// Writes all four bytes of `value` (its top byte included), like the reference.
SIAMESE_FORCE_INLINE void WriteU24_LE_Min4Bytes(uint8_t* data, uint32_t value) { StoreLE<uint32_t>(data, value); }
SIAMESE_FORCE_INLINE void WriteU32_LE(uint8_t* data, uint32_t value) { StoreLE<uint32_t>(data, value); }
SIAMESE_FORCE_INLINE void WriteU64_LE(uint8_t* data, uint64_t value) { StoreLE<uint64_t>(data, value); }

/// Output cursor over a caller's buffer: Write* append at WrittenBytes.
struct WriteByteStream {
    uint8_t* Data = nullptr;
    unsigned BufferBytes = 0;
    unsigned WrittenBytes = 0;

    explicit WriteByteStream() {}
    explicit WriteByteStream(uint8_t* data, uint64_t bytes) : Data(data), BufferBytes((unsigned)bytes) {
        SIAMESE_DEBUG_ASSERT(data != nullptr && bytes > 0);
    }

    SIAMESE_FORCE_INLINE uint8_t* Peek() { return Data + WrittenBytes; }
    SIAMESE_FORCE_INLINE unsigned Remaining() { return BufferBytes - WrittenBytes; }

    SIAMESE_FORCE_INLINE void Write8(uint8_t value) { put(value, 1); }
    SIAMESE_FORCE_INLINE void Write16(uint16_t value) { put(value, 2); }
    SIAMESE_FORCE_INLINE void Write24(uint32_t value) {
        SIAMESE_DEBUG_ASSERT(WrittenBytes + 3 <= BufferBytes);
        WriteU24_LE(Peek(), value);
        WrittenBytes += 3;
    }
    SIAMESE_FORCE_INLINE void Write32(uint32_t value) { put(value, 4); }
    SIAMESE_FORCE_INLINE void Write64(uint64_t value) { put(value, 8); }
    SIAMESE_FORCE_INLINE void WriteBuffer(const void* source, size_t bytes) {
        SIAMESE_DEBUG_ASSERT(source != nullptr || bytes == 0);
        SIAMESE_DEBUG_ASSERT(WrittenBytes + bytes <= BufferBytes);
        if (bytes) memcpy(Peek(), source, bytes);
        WrittenBytes += (unsigned)bytes;
    }

private:
    template <typename T>
    SIAMESE_FORCE_INLINE void put(T value, unsigned n) {
        SIAMESE_DEBUG_ASSERT(WrittenBytes + n <= BufferBytes);
        StoreLE<T>(Peek(), value);
        WrittenBytes += n;
    }
};

/// Input cursor over a received buffer: Read* consume from BytesRead.
struct ReadByteStream {
    const uint8_t* const Data;
    const unsigned BufferBytes;
    unsigned BytesRead;

    ReadByteStream(const uint8_t* data, uint64_t bytes) : Data(data), BufferBytes((unsigned)bytes), BytesRead(0) {
        SIAMESE_DEBUG_ASSERT(data != nullptr);
    }

    SIAMESE_FORCE_INLINE const uint8_t* Peek() { return Data + BytesRead; }
    SIAMESE_FORCE_INLINE unsigned Remaining() { return BufferBytes - BytesRead; }
    SIAMESE_FORCE_INLINE void Skip(unsigned bytes) {
        SIAMESE_DEBUG_ASSERT(BytesRead + bytes <= BufferBytes);
        BytesRead += bytes;
    }
    SIAMESE_FORCE_INLINE const uint8_t* Read(unsigned bytes) {
        const uint8_t* p = Peek();
        Skip(bytes);
        return p;
    }

    SIAMESE_FORCE_INLINE uint8_t Read8() { return take<uint8_t>(1); }
    SIAMESE_FORCE_INLINE uint16_t Read16() { return take<uint16_t>(2); }
    SIAMESE_FORCE_INLINE uint32_t Read24() {
        const uint32_t v = ReadU24_LE(Peek());
        Skip(3);
        return v;
    }
    SIAMESE_FORCE_INLINE uint32_t Read32() { return take<uint32_t>(4); }
    SIAMESE_FORCE_INLINE uint64_t Read64() { return take<uint64_t>(8); }

private:
    template <typename T>
    SIAMESE_FORCE_INLINE T take(unsigned n) {
        SIAMESE_DEBUG_ASSERT(BytesRead + n <= BufferBytes);
        const T v = LoadLE<T>(Peek());
        BytesRead += n;
        return v;
    }
};

}  // namespace siamese

#endif  // TONK_AMD_SIAMESE_SERIALIZERS_H
