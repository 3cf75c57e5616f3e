"""oracle_py.py -- TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench cpu_baseline).

Python side of the parity checker: the synthetic payload definition of the workload
(tonk_amd/csrc/workload.h payload_length / payload_bytes, vectorised PCG32 of
SiameseTools.h:79-101), the varint length prefix (SiameseSerializers.h:566-596), the FNV-1a
digests the transcripts use, and a ctypes wrapper over the plain-C oracle
(oracle/siamese_oracle.c) that recomputes a recovery packet from its metadata with the direct,
non-incremental definition.  Nothing in the product imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_M = np.uint64(6364136223846793005)


def _pcg_seed(y, x):
    """Vectorised PCG32 seeding (SiameseTools.h:79-101): returns (state, inc) arrays."""
    y = np.asarray(y, dtype=np.uint64)
    x = np.asarray(x, dtype=np.uint64)
    inc = (y << np.uint64(1)) | np.uint64(1)
    state = np.zeros(np.broadcast(y, x).shape, dtype=np.uint64)
    state = state * _M + inc
    state = state + x
    state = state * _M + inc
    return state, inc


def _pcg_next(state, inc):
    old = state
    state = old * _M + inc
    xs = (((old >> np.uint64(18)) ^ old) >> np.uint64(27)).astype(np.uint32)
    rot = (old >> np.uint64(59)).astype(np.uint32)
    out = (xs >> rot) | (xs << ((np.uint32(32) - rot) & np.uint32(31)))
    return state, out.astype(np.uint32)


def payload_lengths(kv: dict, n: int) -> np.ndarray:
    """workload.h payload_length for originals 0..n-1 (kv: pmin, pmax, seed_data)."""
    if kv["pmin"] == kv["pmax"]:
        return np.full(n, kv["pmin"], dtype=np.int64)
    with np.errstate(over="ignore"):
        st, inc = _pcg_seed(np.full(n, kv["seed_data"] ^ 0x5BD1E995, dtype=np.uint64), np.arange(n, dtype=np.uint64))
        st, r = _pcg_next(st, inc)
    return kv["pmin"] + (r.astype(np.int64) % (kv["pmax"] - kv["pmin"] + 1))


def payloads(kv: dict, n: int):
    """(lengths, byte matrix [n, pmax rounded up to 4]) of originals 0..n-1 of a stream."""
    lens = payload_lengths(kv, n)
    with np.errstate(over="ignore"):
        words = (int(kv["pmax"]) + 3) // 4
        st, inc = _pcg_seed(np.full(n, kv["seed_data"], dtype=np.uint64), np.arange(n, dtype=np.uint64))
        out = np.zeros((n, words), dtype=np.uint32)
        for w in range(words):
            st, out[:, w] = _pcg_next(st, inc)
    data = out.view(np.uint8).reshape(n, words * 4)
    col = np.arange(words * 4)[None, :]
    data = np.where(col < lens[:, None], data, 0).astype(np.uint8)
    return lens, data


def length_header(n: int) -> bytes:
    """Varint length prefix (SiameseSerializers.h:566-596)."""
    if n <= 0x7F:
        return bytes([n])
    if n <= 0x3FFF:
        return bytes([0x80 | (n >> 8), n & 0xFF])
    if n <= 0x1FFFFF:
        return bytes([0xC0 | (n >> 16), (n >> 8) & 0xFF, n & 0xFF])
    return bytes([0xE0 | (n >> 24), (n >> 16) & 0xFF, (n >> 8) & 0xFF, n & 0xFF])


def fnv1a(b: bytes) -> int:
    h = 1469598103934665603
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


class Meta(ctypes.Structure):
    _fields_ = [("Row", ctypes.c_uint), ("ColumnStart", ctypes.c_uint), ("SumCount", ctypes.c_uint),
                ("LDPCCount", ctypes.c_uint)]


GET_ROW = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint, ctypes.POINTER(ctypes.c_uint))
_LIB = None


def load(build: bool = True):
    """oracle/liboracle.so (built on demand), self-tested."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = os.path.join(HERE, "liboracle.so")
    if build:
        subprocess.run(["make", "-C", HERE, "liboracle.so"], check=True, stdout=subprocess.DEVNULL)
    L = ctypes.CDLL(path)
    if L.oracle_self_test() != 0:
        raise RuntimeError("oracle self test failed")
    L.oracle_recovery_row.argtypes = [ctypes.POINTER(Meta), GET_ROW, ctypes.c_void_p,
                                      ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint]
    _LIB = L
    return L


class RecoveryChecker:
    """Recomputes recovery packets of one stream from their footer metadata (oracle direct
    definition) and compares their FNV-1a digests with a transcript's `E 0 ...` lines."""

    PERIOD = 0x400000

    def __init__(self, kv: dict, n: int):
        self.L = load()
        lens, data = payloads(kv, n)
        self.rows = []
        for i in range(n):
            framed = length_header(int(lens[i])) + bytes(data[i, : lens[i]])
            self.rows.append((ctypes.c_uint8 * len(framed)).from_buffer_copy(framed))
        self.n = n

        def get_row(_ctx, column, nbytes):
            c = column % self.PERIOD
            if c >= self.n:
                return None
            nbytes[0] = len(self.rows[c])
            return ctypes.addressof(self.rows[c])

        self._cb = GET_ROW(get_row)
        self._footer = (ctypes.c_uint8 * 16)()

    def packet(self, total: int, row: int, cs: int, sc: int, ldpc: int) -> bytes:
        meta = Meta(row, cs, sc, ldpc)
        flen = self.L.oracle_serialize_recovery_footer(ctypes.byref(meta), self._footer)
        dlen = total - flen
        out = (ctypes.c_uint8 * max(dlen, 1))()
        if self.L.oracle_recovery_row(ctypes.byref(meta), self._cb, None, out, dlen) != 0:
            raise ValueError("recovery references a column outside the stream")
        return bytes(out[:dlen]) + bytes(self._footer[:flen])

    def check_lines(self, lines) -> int:
        """Number of `E 0` lines verified; raises AssertionError on the first mismatch."""
        checked = 0
        for ln in lines:
            f = ln.split()
            if len(f) < 8 or f[0] != "E" or f[1] != "0":
                continue
            pkt = self.packet(int(f[2]), int(f[3]), int(f[4]), int(f[5]), int(f[6]))
            if fnv1a(pkt) != int(f[7], 16):
                raise AssertionError(f"recovery packet differs from the oracle: {ln}")
            checked += 1
        return checked
