"""CPU checks of the C-ABI boundary (no GPU, no compute calls).

* libtonk_amd.so loads and exports every function include/*.h declares (the drop-in surface
  the reference's siamese.h users link against, plus the session API the bench uses);
* the library refuses to run without an MI355X instead of falling back to a CPU path.
"""
from __future__ import annotations

import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADERS = [os.path.join(ROOT, "include", h) for h in ("siamese.h", "tonk_amd.h")]
DECL = re.compile(r"^\s*(?:SIAMESE_EXPORT\s+)?[A-Za-z_][\w\s\*]*?\b((?:siamese|tamd)_\w+)\s*\(", re.M)


def declared_functions():
    names = set()
    for h in HEADERS:
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        text = re.sub(r"#define[^\n]*", "", text)
        names.update(DECL.findall(text))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    import tonk_amd
    path = os.path.join(ROOT, "tonk_amd", "libtonk_amd.so")
    if not os.path.exists(path):
        tonk_amd.build()
    return ctypes.CDLL(path)


def test_headers_declare_the_reference_api():
    names = declared_functions()
    # siamese.h:213-443 of the reference: the entry points Tonk calls
    for n in ["siamese_init_", "siamese_encoder_create", "siamese_encoder_free", "siamese_encoder_add",
              "siamese_encoder_get", "siamese_encoder_remove_before", "siamese_encoder_ack",
              "siamese_encoder_retransmit", "siamese_encode", "siamese_encoder_is_ready",
              "siamese_decoder_create", "siamese_decoder_free", "siamese_decoder_add_original",
              "siamese_decoder_add_recovery", "siamese_decoder_get", "siamese_decoder_is_ready",
              "siamese_decode", "siamese_decoder_ack", "siamese_encoder_stats", "siamese_decoder_stats"]:
        assert n in names, n
    assert len(names) >= 30


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"declared in include/ but not exported: {missing}"


def test_no_cpu_fallback_without_gpu(lib):
    """With no MI355X visible the engine must refuse, not silently compute on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    err = ctypes.create_string_buffer(256)
    assert lib.tamd_device_selftest(0, err, 256) != 0
    assert b"no HIP device" in err.value or b"gfx950" in err.value
    lib.siamese_encoder_create.restype = ctypes.c_void_p
    lib.siamese_decoder_create.restype = ctypes.c_void_p
    assert not lib.siamese_encoder_create()
    assert not lib.siamese_decoder_create()
