"""Drives the siamese.h C ABI of one library through its argument checks and edge cases
(siamese.cpp:43-299 of the reference) and prints every result code and returned value as JSON.
tests/test_capi_boundary.py runs it once against the reference codec (oracle/_ref) and once
against libtonk_amd.so and requires identical output.  Test infrastructure only.

usage: python capi_boundary_driver.py <library.so>
"""
import ctypes
import json
import sys

MAX_PN = 0x3FFFFF


class Orig(ctypes.Structure):
    _fields_ = [("PacketNum", ctypes.c_uint), ("DataBytes", ctypes.c_uint), ("Data", ctypes.c_void_p)]


class Rec(ctypes.Structure):
    _fields_ = [("DataBytes", ctypes.c_uint), ("Data", ctypes.c_void_p)]


def main(path: str) -> None:
    L = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    for n in ("siamese_encoder_create", "siamese_decoder_create"):
        getattr(L, n).restype = vp
    for n in ("siamese_encoder_free", "siamese_decoder_free"):
        getattr(L, n).argtypes = [vp]
        getattr(L, n).restype = None
    out = []

    def rec(name, v):
        out.append([name, v])

    def data(p, n):
        return list(ctypes.string_at(p, n)) if p and n else None

    rec("init_v4", L.siamese_init_(4))
    rec("init", L.siamese_init_(5))
    enc = vp(L.siamese_encoder_create())
    dec = vp(L.siamese_decoder_create())
    rec("enc_created", bool(enc.value))
    rec("dec_created", bool(dec.value))
    null = vp(None)

    rec("enc_is_ready_null", L.siamese_encoder_is_ready(null))
    rec("enc_is_ready", L.siamese_encoder_is_ready(enc))
    r = Rec()
    rec("encode_empty", L.siamese_encode(enc, ctypes.byref(r)))
    rec("encode_null_rec", L.siamese_encode(enc, None))

    bufs = [bytes((i * 7 + j) & 0xFF for j in range(n)) for i, n in enumerate((1, 100, 1300, 37))]
    keep = [ctypes.create_string_buffer(b, len(b)) for b in bufs]
    o = Orig(0, 0, None)
    rec("add_null_packet", L.siamese_encoder_add(enc, None))
    rec("add_null_data", L.siamese_encoder_add(enc, ctypes.byref(Orig(0, 5, None))))
    rec("add_zero_bytes", L.siamese_encoder_add(enc, ctypes.byref(Orig(0, 0, ctypes.cast(keep[0], vp)))))
    rec("add_too_big", L.siamese_encoder_add(enc, ctypes.byref(Orig(0, 0x20000000, ctypes.cast(keep[0], vp)))))
    for i, b in enumerate(keep):
        o = Orig(0, len(bufs[i]), ctypes.cast(b, vp))
        rec(f"add_{i}", [L.siamese_encoder_add(enc, ctypes.byref(o)), o.PacketNum])

    g = Orig(MAX_PN + 1, 0, None)
    rec("get_bad_num", L.siamese_encoder_get(enc, ctypes.byref(g)))
    g = Orig(1, 0, None)
    rc = L.siamese_encoder_get(enc, ctypes.byref(g))
    rec("get_1", [rc, g.DataBytes, data(g.Data, g.DataBytes)])
    g = Orig(9, 0, None)
    rec("get_missing", L.siamese_encoder_get(enc, ctypes.byref(g)))

    r = Rec()
    rc = L.siamese_encode(enc, ctypes.byref(r))
    rec("encode_1", [rc, r.DataBytes, data(r.Data, r.DataBytes)])
    rbytes = ctypes.string_at(r.Data, r.DataBytes) if rc == 0 else b""
    rbuf = ctypes.create_string_buffer(rbytes, len(rbytes))

    # decoder: originals 0, 2, 3 arrive, 1 is lost (the reference does not check an original's Data
    # pointer, siamese.cpp:212-214: no null-data case here)
    rec("dec_add_orig_null", L.siamese_decoder_add_original(dec, None))
    rec("dec_add_orig_zero", L.siamese_decoder_add_original(dec, ctypes.byref(Orig(0, 0, ctypes.cast(keep[0], vp)))))
    for i in (0, 2, 3):
        rec(f"dec_add_orig_{i}",
            L.siamese_decoder_add_original(dec, ctypes.byref(Orig(i, len(bufs[i]), ctypes.cast(keep[i], vp)))))
    rec("dec_add_orig_dup", L.siamese_decoder_add_original(dec, ctypes.byref(Orig(0, 1, ctypes.cast(keep[0], vp)))))
    g = Orig(1, 0, None)
    rec("dec_get_missing", L.siamese_decoder_get(dec, ctypes.byref(g)))
    g = Orig(MAX_PN + 1, 0, None)
    rec("dec_get_bad_num", L.siamese_decoder_get(dec, ctypes.byref(g)))
    g = Orig(2, 0, None)
    rc = L.siamese_decoder_get(dec, ctypes.byref(g))
    rec("dec_get_2", [rc, g.DataBytes, data(g.Data, g.DataBytes)])
    rec("dec_is_ready_null", L.siamese_decoder_is_ready(null))
    rec("dec_is_ready_0", L.siamese_decoder_is_ready(dec))
    rec("dec_add_rec_null", L.siamese_decoder_add_recovery(dec, None))
    rec("dec_add_rec_zero", L.siamese_decoder_add_recovery(dec, ctypes.byref(Rec(0, ctypes.cast(rbuf, vp)))))
    rec("dec_add_rec", L.siamese_decoder_add_recovery(dec, ctypes.byref(Rec(len(rbytes), ctypes.cast(rbuf, vp)))))
    rec("dec_add_rec_dup", L.siamese_decoder_add_recovery(dec, ctypes.byref(Rec(len(rbytes), ctypes.cast(rbuf, vp)))))
    rec("dec_is_ready_1", L.siamese_decoder_is_ready(dec))
    pp = ctypes.POINTER(Orig)()
    cnt = ctypes.c_uint(0)
    rec("decode_mismatch", L.siamese_decode(dec, ctypes.byref(pp), None))
    rc = L.siamese_decode(dec, ctypes.byref(pp), ctypes.byref(cnt))
    got = [[pp[i].PacketNum, pp[i].DataBytes, data(pp[i].Data, pp[i].DataBytes)] for i in range(cnt.value)] if rc == 0 else []
    rec("decode", [rc, cnt.value, got])
    rec("decode_again", L.siamese_decode(dec, ctypes.byref(pp), ctypes.byref(cnt)))

    ack = ctypes.create_string_buffer(256)
    used = ctypes.c_uint(0)
    rec("dec_ack_small", L.siamese_decoder_ack(dec, ack, 15, ctypes.byref(used)))
    rec("dec_ack_null_used", L.siamese_decoder_ack(dec, ack, 64, None))
    rc = L.siamese_decoder_ack(dec, ack, 64, ctypes.byref(used))
    rec("dec_ack", [rc, used.value, list(ack.raw[:used.value])])
    nxt = ctypes.c_uint(0)
    rec("enc_ack_zero", L.siamese_encoder_ack(enc, ack, 0, ctypes.byref(nxt)))
    rec("enc_ack_null_next", L.siamese_encoder_ack(enc, ack, used.value, None))
    rc = L.siamese_encoder_ack(enc, ack, used.value, ctypes.byref(nxt))
    rec("enc_ack", [rc, nxt.value])

    st = (ctypes.c_uint64 * 11)()
    rec("enc_stats_null", L.siamese_encoder_stats(enc, None, 9))
    rec("enc_stats_zero", L.siamese_encoder_stats(enc, st, 0))
    rc = L.siamese_encoder_stats(enc, st, 9)
    rec("enc_stats", [rc, list(st)[:8]])  # [8] MemoryUsed is allocator dependent
    rec("dec_stats_null", L.siamese_decoder_stats(dec, None, 11))
    rc = L.siamese_decoder_stats(dec, st, 11)
    rec("dec_stats", [rc, list(st)[:10]])  # [10] MemoryUsed is allocator dependent

    rec("remove_before_bad", L.siamese_encoder_remove_before(enc, MAX_PN + 1))
    rec("remove_before_2", L.siamese_encoder_remove_before(enc, 2))
    g = Orig(0, 0, None)
    rec("get_removed", L.siamese_encoder_get(enc, ctypes.byref(g)))
    g = Orig(3, 0, None)
    rc = L.siamese_encoder_get(enc, ctypes.byref(g))
    rec("get_3", [rc, g.DataBytes, data(g.Data, g.DataBytes)])

    L.siamese_encoder_free(enc)
    L.siamese_decoder_free(dec)
    L.siamese_encoder_free(null)
    L.siamese_decoder_free(null)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
