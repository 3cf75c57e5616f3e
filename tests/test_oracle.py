"""CPU tests of the oracle (oracle/siamese_oracle.c), the parity checker of the MI355X engine.

The oracle is pinned two ways before anything is compared with it:
* its known-answer self test (gf256 self test of the reference, SURVEY.md s8(c) values);
* the golden transcripts produced by the REFERENCE codec (tests/golden, oracle/gen_golden.py):
  every recovery packet the reference emitted is recomputed from its footer metadata with the
  oracle's direct (non-incremental) definition and must hash identically, and every packet the
  reference decoder recovered must be the true payload.
"""
from __future__ import annotations

import ctypes
import gzip
import os

import oracle_py
import pytest

from conftest import GOLDEN, fnv1a, length_header, payloads, scenario_params


Meta = oracle_py.Meta


def test_self_test(oracle_lib):
    assert oracle_lib.oracle_self_test() == 0


def test_gf_field(oracle_lib):
    L = oracle_lib
    L.oracle_gf_mul.restype = ctypes.c_uint8
    L.oracle_gf_div.restype = ctypes.c_uint8
    L.oracle_gf_inv.restype = ctypes.c_uint8
    L.oracle_gf_polynomial.restype = ctypes.c_uint
    assert L.oracle_gf_polynomial() == 0x14D  # gf256.cpp:358-372
    for x in range(1, 256):
        ix = L.oracle_gf_inv(x)
        assert L.oracle_gf_mul(x, ix) == 1
        for y in (1, 2, 3, 0x53, 0xCA, 255):
            p = L.oracle_gf_mul(x, y)
            assert L.oracle_gf_div(p, y) == x
    assert L.oracle_gf_mul(0, 77) == 0


def test_serializers_roundtrip(oracle_lib):
    L = oracle_lib
    buf = (ctypes.c_uint8 * 16)()
    for n in (0, 1, 0x7F, 0x80, 0x3FFF, 0x4000, 0x1FFFFF, 0x200000):
        k = L.oracle_serialize_length_header(n, buf)
        assert bytes(buf[:k]) == length_header(n)
        out = ctypes.c_uint(0)
        assert L.oracle_deserialize_length_header(buf, k, ctypes.byref(out)) == k
        assert out.value == n
    for m in [(0, 5, 1, 1), (0, 100, 17, 17), (3, 4000, 60, 60), (7, 0x3FFFFF, 300, 250), (255, 12345, 2000, 700)]:
        meta = Meta(*m)
        k = L.oracle_serialize_recovery_footer(ctypes.byref(meta), buf)
        back = Meta()
        assert L.oracle_deserialize_recovery_footer(buf, k, ctypes.byref(back)) == k
        if m[2] > 1:
            assert (back.Row, back.ColumnStart, back.SumCount, back.LDPCCount) == m
        else:
            assert (back.ColumnStart, back.SumCount) == (m[1], 1)
    for rel, lm1 in [(0, 0), (5, 2), (200, 0), (70000, 9), (3, 300)]:
        k = L.oracle_serialize_nack_range(rel, lm1, buf)
        a, b = ctypes.c_uint(0), ctypes.c_uint(0)
        assert L.oracle_deserialize_nack_range(buf, 16, ctypes.byref(a), ctypes.byref(b)) == k
        assert (a.value, b.value) == (rel, lm1)


def _golden_lines(name):
    with gzip.open(os.path.join(GOLDEN, f"{name}.txt.gz"), "rt") as f:
        return f.read().splitlines()


RECOVERY_SCENARIOS = ["c1_256_p3", "c2_4096_p1_noack", "c3_4096_p2_ack64_s1", "var_1_1500_p2_ack32",
                      "tiny_1_20_p5_ack16", "big_9000_p3_ack64", "single_p0"]


@pytest.mark.parametrize("name", RECOVERY_SCENARIOS)
def test_recovery_packets_match_reference(oracle_lib, golden_index, name):
    """Every recovery packet of the reference transcript == the oracle's direct definition."""
    kv = scenario_params(golden_index, name)
    chk = oracle_py.RecoveryChecker(kv, kv["n"])
    assert chk.check_lines(_golden_lines(name)) > 0


@pytest.mark.parametrize("name", ["c1_256_p3", "c3_4096_p2_ack64_s63", "var_1_1500_p2_ack32", "hiloss_p20_arq"])
def test_reference_recoveries_are_true_payloads(golden_index, name):
    """The fixtures pin real decodes: every payload the reference recovered is the original."""
    kv = scenario_params(golden_index, name)
    lens, data = payloads(kv, kv["n"])
    seen = 0
    for ln in _golden_lines(name):
        f = ln.split()
        if f[0] != "D" or f[1] != "0":
            continue
        for ent in f[3:]:
            num, ln_, h = ent.split(":")
            num, ln_ = int(num), int(ln_)
            assert ln_ == lens[num]
            assert fnv1a(bytes(data[num, :ln_])) == int(h, 16)
            seen += 1
    assert seen > 0
