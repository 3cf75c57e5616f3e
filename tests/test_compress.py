"""The compression step (Tonk's MessageCompressor, PacketCompression.h:92).

Parity here is the reference's own receive side: every block the GPU writes must be restored
byte for byte by tonk::MessageDecompressor (PacketCompression.cpp:120-216, restated over the
reference's zstd in oracle/msgcodec_ref.cpp and compiled from /root/reference into oracle/_ref),
with uncompressed messages fed to InsertUncompressed as Tonk does.  The blocks themselves differ
from zstd level 1's (raw literals, predefined FSE tables, our own parse); their sizes are
reported beside the reference compressor's.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import NATIVE, ROOT, _make

REF = os.path.join(ROOT, "oracle", "_ref", "libmsgcodec_ref.so")
MAX = 1300  # kMaxCompressedBytes of TonkUnitTest.cpp:604 (Tonk's datagram budget)


def ref_lib():
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/libmsgcodec_ref.so not built (needs /root/reference at build time)")
    L = ctypes.CDLL(REF)
    vp, cu = ctypes.c_void_p, ctypes.c_uint
    L.ref_comp_new.restype = vp
    L.ref_comp_new.argtypes = [cu]
    L.ref_comp.restype = ctypes.c_int
    L.ref_comp.argtypes = [vp, ctypes.c_char_p, cu, ctypes.c_void_p, ctypes.POINTER(cu)]
    L.ref_comp_free.argtypes = [vp]
    L.ref_decomp_new.restype = vp
    L.ref_decomp_new.argtypes = [cu]
    L.ref_insert.argtypes = [vp, ctypes.c_char_p, cu]
    L.ref_decomp.restype = ctypes.c_int
    L.ref_decomp.argtypes = [vp, ctypes.c_char_p, cu, ctypes.c_void_p, cu]
    L.ref_decomp_free.argtypes = [vp]
    return L


class RefDecompressor:
    def __init__(self, L, max_bytes=MAX):
        self.L, self.h = L, L.ref_decomp_new(max_bytes)
        self.buf = ctypes.create_string_buffer(max_bytes + 64)

    def feed(self, block: bytes, original: bytes) -> bytes:
        """Tonk's receive side: Decompress a compressed block, InsertUncompressed otherwise."""
        if not block:
            self.L.ref_insert(self.h, original, len(original))
            return original
        n = self.L.ref_decomp(self.h, block, len(block), self.buf, len(self.buf))
        assert n >= 0, "reference zstd rejected the block"
        return self.buf.raw[:n]


class RefCompressor:
    def __init__(self, L, max_bytes=MAX):
        self.L, self.h = L, L.ref_comp_new(max_bytes)
        self.buf = ctypes.create_string_buffer(max_bytes + 64)

    def compress(self, msg: bytes) -> bytes:
        w = ctypes.c_uint(0)
        assert self.L.ref_comp(self.h, msg, len(msg), self.buf, ctypes.byref(w)) == 0
        return self.buf.raw[:w.value]


class Pcg:
    """siamese::PCGRandom (SiameseTools.h:80-102)."""
    M = (1 << 64) - 1

    def __init__(self, y, x=0):
        self.state, self.inc = 0, ((y << 1) | 1) & self.M
        self.next()
        self.state = (self.state + x) & self.M
        self.next()

    def next(self) -> int:
        old = self.state
        self.state = (old * 6364136223846793005 + self.inc) & self.M
        xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xs >> rot) | (xs << ((-rot) & 31))) & 0xFFFFFFFF


def tonk_unit_messages():
    """TestCompression's stream (TonkUnitTest.cpp:599-700): 100 messages of 400 PCG bytes, seeds
    0..49 then 50..1 (the second half repeats the first in reverse)."""
    out = []
    for i in range(100):
        seed = 100 - i if i >= 50 else i
        p = Pcg(seed)
        out.append(b"".join(p.next().to_bytes(4, "little") for _ in range(100)))
    return out


def mixed_messages(n, seed):
    """Text-like runs, random bytes and repeats of earlier stretches; lengths 8..MAX."""
    rng = np.random.default_rng(seed)
    words = [b"siamese ", b"tonk ", b"packet ", b"recovery ", b"window ", b"lane ", b"sum ", b"ack ", b"0123 "]
    stream = bytearray()
    msgs = []
    for _ in range(n):
        ln = int(rng.integers(8, MAX + 1))
        kind = int(rng.integers(0, 4))
        if kind == 3 and len(stream) > 4000:
            start = len(stream) - 1 - int(rng.integers(0, min(len(stream) - 1, 40000)))
            m = bytes(stream[start:start + ln]).ljust(ln, b"x")
        elif kind == 0:
            m = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        else:
            parts = []
            while sum(map(len, parts)) < ln:
                parts.append(words[int(rng.integers(0, len(words)))])
            m = b"".join(parts)[:ln]
        stream += m
        msgs.append(m)
    return msgs


# --------------------------------------------------------------------------------------- CPU

def test_reference_msgcodec_roundtrip():
    """Pins the oracle: the reference compressor's blocks restore through the restated
    decompressor over Tonk's own unit-test stream and a long mixed stream (ring wraps)."""
    L = ref_lib()
    for msgs in (tonk_unit_messages(), mixed_messages(300, 5)):
        comp, dec = RefCompressor(L), RefDecompressor(L)
        n_comp = 0
        for m in msgs:
            blk = comp.compress(m)
            n_comp += bool(blk)
            assert dec.feed(blk, m) == m
        assert n_comp > 0


def test_block_writer_decodes_with_reference_zstd():
    """The block writer shared by the kernel (lz.h) against the reference's zstd decoder: with
    block-fitted / RLE sequence tables (tamd_seq_choose, the kernel's choice), and with the
    predefined tables only (where the table writer must also equal the packed-map writer)."""
    ref_lib()
    _make(NATIVE, "_build/lz_check")
    exe = os.path.join(NATIVE, "_build", "lz_check")
    for seed in (1, 2, 3):
        for extra in ([], ["0", "4", "0"]):
            r = subprocess.run([exe, "300", str(seed)] + extra, capture_output=True, text=True, timeout=120)
            assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
            if not extra:
                assert "fitted tables LL/ML/OF 0/0/0," not in r.stderr, r.stderr


def test_compress_abi_exports_and_no_cpu_fallback():
    import tonk_amd
    path = tonk_amd.LIB_PATH
    if not os.path.exists(path):
        pytest.skip("library not built")
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
    for sym in ("tamd_compressor_create", "tamd_compressor_compress", "tamd_compressor_destroy",
                "tamd_compress_batch", "tamd_compress_batch_host"):
        assert f" T {sym}" in out, sym
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from tonk_amd.compress import MessageCompressor
    with pytest.raises(RuntimeError):
        MessageCompressor(MAX)


# --------------------------------------------------------------------------------------- GPU

@pytest.mark.gpu
def test_gpu_compressor_tonk_unit_stream():
    """TonkUnitTest.cpp TestCompression through the GPU compressor: every message restored, and
    the repeated second half compresses wherever the decompressor still holds its source."""
    from tonk_amd.compress import MessageCompressor
    L = ref_lib()
    msgs = tonk_unit_messages()
    comp, dec = MessageCompressor(MAX), RefDecompressor(L)
    rcomp = RefCompressor(L)
    ours = theirs = 0
    for m in msgs:
        blk = comp.compress(m)
        assert len(blk) < len(m)
        ours += bool(blk)
        assert dec.feed(blk, m) == m
        theirs += bool(rcomp.compress(m))
    print(f"compressed messages: gpu {ours}, reference zstd-1 {theirs}")
    assert ours >= 20


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [5, 6])
def test_gpu_compressor_mixed_stream(seed):
    """A long mixed stream (several ring wraps, external-dictionary matches) through the GPU
    compressor, restored by the reference decompressor; sizes beside zstd level 1."""
    from tonk_amd.compress import MessageCompressor
    L = ref_lib()
    msgs = mixed_messages(400, seed)
    comp, dec, rcomp = MessageCompressor(MAX), RefDecompressor(L), RefCompressor(L)
    out_gpu = out_ref = inp = 0
    for m in msgs:
        blk = comp.compress(m)
        assert dec.feed(blk, m) == m
        out_gpu += len(blk) if blk else len(m)
        r = rcomp.compress(m)
        out_ref += len(r) if r else len(m)
        inp += len(m)
    print(f"bytes in {inp}: gpu {out_gpu} ({inp / out_gpu:.2f}x), zstd-1 {out_ref} ({inp / out_ref:.2f}x)")
    assert out_gpu < 0.75 * inp


@pytest.mark.gpu
def test_gpu_compress_batch_streams():
    """The device-resident batch: 16 streams x 120 messages in one launch; every stream restored
    in order by its own reference decompressor."""
    from tonk_amd.compress import compress_batch_host
    L = ref_lib()
    n_streams, n_msgs = 16, 120
    streams = [mixed_messages(n_msgs, 100 + s) for s in range(n_streams)]
    stride = max(sum(map(len, s)) for s in streams) + 64
    host = np.zeros((n_streams, stride), dtype=np.uint8)
    lens = []
    for s, ms in enumerate(streams):
        blob = b"".join(ms)
        host[s, :len(blob)] = np.frombuffer(blob, dtype=np.uint8)
        lens += [len(m) for m in ms]
    raw, written, ms = compress_batch_host(host.tobytes(), stride, n_streams, n_msgs, lens, MAX, msgs_per_job=8)
    out_h = np.frombuffer(raw, dtype=np.uint8)
    total_in = total_out = 0
    for s, msgs in enumerate(streams):
        dec = RefDecompressor(L)
        for k, m in enumerate(msgs):
            i = s * n_msgs + k
            w = written[i]
            assert w < len(m)
            blk = out_h[i * MAX:i * MAX + w].tobytes() if w else b""
            assert dec.feed(blk, m) == m, (s, k)
            total_in += len(m)
            total_out += w if w else len(m)
    print(f"batch: {total_in} -> {total_out} bytes, kernel {ms:.3f} ms")
    assert total_out < 0.8 * total_in


@pytest.mark.gpu
@pytest.mark.parametrize("max_bytes", [1300, 4000, 24000])
def test_gpu_compressor_edge_cases(max_bytes):
    """Tiny messages (below the kernel's 8-byte floor: sent as is), runs of one byte (matches that
    overlap their own output, distance 1), messages of exactly max bytes, messages above 2048
    bytes (compressed through global scratch instead of LDS) up to the 24,000-byte history, and
    enough of them to restart the ring many times; every one restored by the reference
    decompressor."""
    from tonk_amd.compress import MessageCompressor
    L = ref_lib()
    rng = np.random.default_rng(max_bytes)
    top = max_bytes
    msgs = []
    for k in range(300):
        kind = k % 6
        if kind == 0:
            msgs.append(bytes(rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8)))
        elif kind == 1:
            msgs.append(bytes([k & 0xFF]) * int(rng.integers(9, top + 1)))
        elif kind == 2:
            msgs.append((b"abc" * top)[:top])
        elif kind == 3:
            msgs.append(bytes(rng.integers(0, 4, top, dtype=np.uint8)))
        elif kind == 4 and max_bytes > 2048:
            msgs.append((b"tonk siamese " * 400)[:int(rng.integers(2049, max_bytes + 1))])
        else:
            msgs.append(msgs[-1] if msgs else b"x" * 20)
    comp, dec = MessageCompressor(max_bytes), RefDecompressor(L, max_bytes)
    n_comp = 0
    for m in msgs:
        blk = comp.compress(m)
        assert len(blk) < len(m) or not blk
        if len(m) < 8:
            assert blk == b""
        n_comp += bool(blk)
        if len(m) > 2048 and len(set(m)) <= 3:
            assert blk, len(m)  # (repetitive text and one-byte runs compress at any size)
        assert dec.feed(blk, m) == m
    assert n_comp > 100


@pytest.mark.gpu
@pytest.mark.parametrize("per_job", [4, 0])
def test_gpu_compress_batch_large_messages(per_job):
    """The batch API with messages of 64 B .. 24,000 B (the history size) mixed in one launch:
    the large ones go through global scratch, jobs longer than 64 KB move their hash table's base;
    per_job 0: the library's job size (one round of jobs over the wave slots: here one message
    per job); every stream restored by the reference."""
    from tonk_amd.compress import compress_batch_host
    L = ref_lib()
    max_bytes, n_streams, n_msgs = 24000, 4, 24
    rng = np.random.default_rng(11)
    text = b"".join(rng.choice([b"siamese ", b"tonk ", b"window ", b"lane "], 6000))
    streams = []
    for s in range(n_streams):
        ms = []
        for k in range(n_msgs):
            n = int(rng.integers(64, 2049)) if k % 3 else int(rng.integers(2049, max_bytes + 1))
            if k % 4 == 3:
                ms.append(bytes(rng.integers(0, 256, n, dtype=np.uint8)))
            else:
                o = int(rng.integers(0, len(text) - n))
                ms.append(text[o:o + n])
        streams.append(ms)
    stride = max(sum(map(len, s)) for s in streams) + 64
    host = np.zeros((n_streams, stride), dtype=np.uint8)
    lens = []
    for s, ms in enumerate(streams):
        blob = b"".join(ms)
        host[s, :len(blob)] = np.frombuffer(blob, dtype=np.uint8)
        lens += [len(m) for m in ms]
    raw, written, _ = compress_batch_host(host.tobytes(), stride, n_streams, n_msgs, lens, max_bytes, msgs_per_job=per_job)
    out_h = np.frombuffer(raw, dtype=np.uint8)
    big = 0
    for s, msgs in enumerate(streams):
        dec = RefDecompressor(L, max_bytes)
        for k, m in enumerate(msgs):
            i = s * n_msgs + k
            w = written[i]
            assert w < len(m)
            big += bool(w) and len(m) > 2048
            blk = out_h[i * max_bytes:i * max_bytes + w].tobytes() if w else b""
            assert dec.feed(blk, m) == m, (s, k)
    assert big >= n_streams * n_msgs // 6


@pytest.mark.gpu
def test_gpu_compressor_concurrent_callers():
    """Several threads, each with its own compressor, call the synchronous per-message API at the
    same time (Tonk's connection threads): the calls are combined into shared launches, a leader
    hands leadership on once its own message is done, and every stream is restored in order by
    its own reference decompressor."""
    import threading
    from tonk_amd.compress import MessageCompressor
    L = ref_lib()
    n_threads, n_msgs = 8, 150
    streams = [mixed_messages(n_msgs, 300 + t) for t in range(n_threads)]
    blocks = [[None] * n_msgs for _ in range(n_threads)]
    errors = []

    def worker(t):
        try:
            comp = MessageCompressor(MAX)
            for k, m in enumerate(streams[t]):
                blocks[t][k] = comp.compress(m)
        except Exception as e:  # (surfaced below)
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not any(x.is_alive() for x in th), "a compressor call did not return"
    assert not errors, errors
    for t in range(n_threads):
        dec = RefDecompressor(L)
        for k, m in enumerate(streams[t]):
            assert dec.feed(blocks[t][k], m) == m, (t, k)
