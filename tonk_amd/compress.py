"""Tonk's upstream compression step on MI355X (include/tonk_compress.h).

`MessageCompressor` mirrors tonk::MessageCompressor (PacketCompression.h:92-140): construct with the
maximum compressed message size (Initialize), then `compress(message)` returns the compressed
block, or b"" when the message should be sent as is (the reference's writtenBytes = 0; the
receiver then calls MessageDecompressor::InsertUncompressed).  `compress_batch` is the
device-resident batch the bench measures: many independent streams in one kernel launch.
"""
from __future__ import annotations

import ctypes

from . import lib as _lib_loader

_bound = False


def _lib() -> ctypes.CDLL:
    global _bound
    L = _lib_loader()
    if not _bound:
        vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.tamd_compressor_create.restype = vp
        L.tamd_compressor_create.argtypes = [ctypes.c_uint]
        L.tamd_compressor_compress.restype = ctypes.c_int
        L.tamd_compressor_compress.argtypes = [vp, ctypes.c_char_p, ctypes.c_uint, ctypes.c_void_p,
                                               ctypes.POINTER(ctypes.c_uint)]
        L.tamd_compressor_destroy.restype = None
        L.tamd_compressor_destroy.argtypes = [vp]
        L.tamd_compress_batch.restype = ctypes.c_int
        L.tamd_compress_batch.argtypes = [vp, u64, u32, u32, ctypes.POINTER(u32), u32, vp, ctypes.POINTER(u32), u32,
                                          ctypes.POINTER(ctypes.c_float)]
        L.tamd_compress_batch_host.restype = ctypes.c_int
        L.tamd_compress_batch_host.argtypes = [vp, u64, u32, u32, ctypes.POINTER(u32), u32, vp, ctypes.POINTER(u32),
                                               u32, ctypes.POINTER(ctypes.c_float)]
        _bound = True
    return L


class MessageCompressor:
    """tonk::MessageCompressor on the GPU.  Raises when no gfx950 device is usable."""

    def __init__(self, max_compressed_message_bytes: int):
        self.max = int(max_compressed_message_bytes)
        self._h = _lib().tamd_compressor_create(self.max)
        if not self._h:
            raise RuntimeError("tonk_amd: tamd_compressor_create failed (no gfx950 device, or bad size)")
        self._dest = ctypes.create_string_buffer(self.max + 64)

    def compress(self, message: bytes) -> bytes:
        w = ctypes.c_uint(0)
        rc = _lib().tamd_compressor_compress(self._h, message, len(message), self._dest, ctypes.byref(w))
        if rc != 0:
            raise RuntimeError(f"tonk_amd: compress failed (rc={rc})")
        return self._dest.raw[:w.value]

    def close(self) -> None:
        if self._h:
            _lib().tamd_compressor_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def compress_batch(dev_data: int, stride: int, n_streams: int, n_msgs: int, lens, max_bytes: int, dev_out: int,
                   msgs_per_job: int = 0):
    """Compress every message of `n_streams` fresh streams (device pointers from the caller, e.g.
    torch tensors' data_ptr()).  `lens`: uint32 per message (any sequence; a contiguous numpy
    uint32 array is passed without a copy).  Returns (written bytes per message as a numpy array,
    0 = uncompressed; kernel ms)."""
    import numpy as np
    total = n_streams * n_msgs
    L = np.ascontiguousarray(lens, dtype=np.uint32)
    W = np.zeros(total, dtype=np.uint32)
    ms = ctypes.c_float(0.0)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    rc = _lib().tamd_compress_batch(dev_data, stride, n_streams, n_msgs, L.ctypes.data_as(u32p), max_bytes, dev_out,
                                    W.ctypes.data_as(u32p), msgs_per_job, ctypes.byref(ms))
    if rc != 0:
        raise RuntimeError(f"tonk_amd: compress_batch failed (rc={rc})")
    return W, ms.value


def compress_batch_host(data, stride: int, n_streams: int, n_msgs: int, lens, max_bytes: int,
                        msgs_per_job: int = 0) -> tuple[bytes, list[int], float]:
    """compress_batch from a host buffer (bytes-like of n_streams * stride): returns (the output
    slots, max_bytes per message; written per message; kernel ms)."""
    total = n_streams * n_msgs
    L = (ctypes.c_uint32 * total)(*lens)
    W = (ctypes.c_uint32 * total)()
    src = ctypes.create_string_buffer(bytes(data), n_streams * stride)
    out = ctypes.create_string_buffer(total * max_bytes)
    ms = ctypes.c_float(0.0)
    rc = _lib().tamd_compress_batch_host(src, stride, n_streams, n_msgs, L, max_bytes, out, W, msgs_per_job,
                                         ctypes.byref(ms))
    if rc != 0:
        raise RuntimeError(f"tonk_amd: compress_batch_host failed (rc={rc})")
    return out.raw, list(W), ms.value
