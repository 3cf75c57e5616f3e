"""tonk_amd -- MI355X-native Siamese FEC engine (catid/tonk's FEC hot path).

The engine is a C-ABI shared library built in-tree (tonk_amd/libtonk_amd.so) that exports

* the reference's ``siamese.h`` API (drop-in for TonkineseOutgoing/Incoming.cpp), and
* a batched device-resident session API (``include/tonk_amd.h``) used by ``bench.py``.

Python only loads the library and marshals arguments (ctypes); there is no Python or CPU
implementation of the codec here.  Importing works without a GPU; creating a codec or a
session on a host without an MI355X raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

__all__ = ["LIB_PATH", "build", "lib", "Session", "WorkloadParams", "loss_threshold", "ge_thresholds",
           "fec_q16", "device_selftest", "cpu_share", "SUMMARY_FIELDS"]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libtonk_amd.so")
# A/B runs of two builds on one box (tools/gpu_ab_lib.sh): another in-tree build of the library.
if os.environ.get("TONK_AMD_LIB"):
    LIB_PATH = os.path.join(_HERE, os.path.basename(os.environ["TONK_AMD_LIB"]))
_lib = None


def build(jobs: int = 8) -> str:
    """Compile libtonk_amd.so for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-C", _HERE, f"-j{jobs}"], check=True, stdout=subprocess.DEVNULL)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    """Load the in-tree engine library.  Raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"tonk_amd: {LIB_PATH} missing -- run tonk_amd.build() (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
        vp, u32, u64, cp, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_size_t
        L.tamd_session_create.restype = vp
        L.tamd_session_create.argtypes = [ctypes.POINTER(_SessionParams), cp, sz]
        for name in ("tamd_session_generate", "tamd_session_wait", "tamd_session_finish"):
            getattr(L, name).restype = ctypes.c_int
            getattr(L, name).argtypes = [vp]
        L.tamd_session_step.restype = ctypes.c_int
        L.tamd_session_step.argtypes = [vp, u32]
        L.tamd_session_summary.restype = ctypes.c_int
        L.tamd_session_summary.argtypes = [vp, ctypes.POINTER(u64), ctypes.c_uint]
        L.tamd_session_set_timing.restype = None
        L.tamd_session_set_timing.argtypes = [vp, ctypes.c_int]
        L.tamd_session_kernel_ms.restype = ctypes.c_double
        L.tamd_session_kernel_ms.argtypes = [vp, ctypes.POINTER(u64)]
        L.tamd_session_host_ms.restype = None
        L.tamd_session_host_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        L.tamd_session_transcript.restype = sz
        L.tamd_session_transcript.argtypes = [vp, u32, ctypes.c_char_p, sz]
        L.tamd_session_error.restype = ctypes.c_char_p
        L.tamd_session_error.argtypes = [vp]
        L.tamd_session_destroy.restype = None
        L.tamd_session_destroy.argtypes = [vp]
        L.tamd_session_schedule.restype = ctypes.c_int
        L.tamd_session_schedule.argtypes = [vp]
        L.tamd_session_arena.restype = None
        L.tamd_session_arena.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.tamd_session_cpus.restype = ctypes.c_uint
        L.tamd_session_cpus.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.c_uint]
        L.tamd_cpu_share.restype = ctypes.c_uint
        L.tamd_cpu_share.argtypes = [cp, ctypes.c_uint, cp, cp, ctypes.POINTER(ctypes.c_int), ctypes.c_uint]
        L.tamd_device_selftest.restype = ctypes.c_int
        L.tamd_device_selftest.argtypes = [u32, cp, sz]
        _lib = L
    return _lib


class _SessionParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "device", "n_streams", "stream_base", "n_threads", "n_originals", "payload_min", "payload_max",
        "loss_thresh", "ge_enable", "gb_thresh", "bg_thresh", "loss_on_recovery", "fec_rate_q16",
        "ack_every", "ack_bytes", "arq_lag", "flush_max", "record", "stage_host")] + [
            ("arena_bytes", ctypes.c_uint64), ("rtx_every", ctypes.c_uint32), ("rtx_msec", ctypes.c_uint32),
            ("input_pool", ctypes.c_uint32), ("hold_full", ctypes.c_uint32)]


SUMMARY_FIELDS = ["originals", "lost_originals", "recoveries", "lost_recoveries", "recovered", "arq",
                  "missing_at_end", "payload_bytes", "alg_bytes", "acc_bytes", "store_bytes", "programs",
                  "launches", "ops", "instrs", "upload_bytes", "disabled_codecs", "h2d_bytes", "d2h_bytes",
                  "d2h_copy_us"]


def loss_threshold(p: float) -> int:
    """Uniform loss probability -> 32-bit threshold of the workload's PCG draw."""
    return min(int(p * 2**32), 2**32 - 1)


def ge_thresholds(p: float, burst: float) -> tuple[int, int]:
    """Gilbert-Elliott channel with mean loss p and mean burst length b."""
    p_gb = p / (burst * (1.0 - p))
    p_bg = 1.0 / burst
    return int(p_gb * 2**32), int(p_bg * 2**32)


def fec_q16(p: float, rate: float | None = None) -> int:
    """Tonk's recovery rate f = max(2p, 1%) (TonkineseBandwidth.cpp:770) in 1/65536 units."""
    f = rate if rate is not None else max(2.0 * p, 0.01)
    return int(round(f * 65536))


class WorkloadParams:
    """Synthetic workload parameters (tonk_amd/csrc/workload.h Params)."""

    KEYS = ("n", "pmin", "pmax", "loss", "ge", "gb", "bg", "lossrec", "fec", "ack", "ackbytes", "arq", "flush")
    # retransmission ticks under a virtual clock (workload.h) and the window-full behaviour; each
    # written to args() only when on
    OPTIONAL = ("rtx", "rtxms", "full")

    def __init__(self, n=4096, payload=1300, payload_max=None, loss=0.01, burst=None, fec=None, ack=64,
                 ack_bytes=256, arq=0, flush=4096, loss_on_recovery=True, rtx=0, rtx_msec=1, full=0):
        self.n = n
        self.pmin = payload
        self.pmax = payload_max if payload_max is not None else payload
        if burst:
            self.ge = 1
            self.gb, self.bg = ge_thresholds(loss, burst)
            self.loss = 0
        else:
            self.ge, self.gb, self.bg = 0, 0, 0
            self.loss = loss_threshold(loss)
        self.fec = fec_q16(loss, fec)
        self.ack = ack
        self.ackbytes = ack_bytes
        self.arq = arq
        self.flush = flush
        self.lossrec = 1 if loss_on_recovery else 0
        self.rtx = rtx
        self.rtxms = rtx_msec
        self.full = full

    def args(self) -> list[str]:
        keys = self.KEYS + (("rtx", "rtxms") if self.rtx else ()) + (("full",) if self.full else ())
        return [f"{k}={getattr(self, k)}" for k in keys]

    @classmethod
    def from_args(cls, args: list[str]) -> "WorkloadParams":
        """The inverse of args() (fixture argument lists)."""
        wp = cls()
        kv = dict(a.split("=") for a in args)
        for k in cls.KEYS + cls.OPTIONAL:
            if k in kv:
                setattr(wp, k, int(kv[k]))
        return wp


def cpu_share(dev_cpulists: list[str], device: int, node_cores: str, slot_override: str | None = None) -> list[int]:
    """Host cores of `device`'s worker pool (include/tonk_amd.h tamd_cpu_share; pure, no GPU):
    the devices with the same NUMA local_cpulist split `node_cores` in device order."""
    out = (ctypes.c_int * 4096)()
    n = lib().tamd_cpu_share(";".join(dev_cpulists).encode(), device, node_cores.encode(),
                             slot_override.encode() if slot_override else None, out, 4096)
    return [int(out[i]) for i in range(min(n, 4096))]


def device_selftest(device: int = 0) -> None:
    err = ctypes.create_string_buffer(512)
    rc = lib().tamd_device_selftest(device, err, len(err))
    if rc != 0:
        raise RuntimeError(f"tonk_amd device self test failed: {err.value.decode()}")


class Session:
    """Batched device-resident Siamese streams on one MI355X (include/tonk_amd.h)."""

    def __init__(self, wp: WorkloadParams, n_streams: int, device: int = 0, stream_base: int = 0,
                 threads: int = 1, arena_bytes: int = 4 << 30, record: bool = False, stage_host: bool = False,
                 input_pool: int = 0):
        p = _SessionParams()
        p.device, p.n_streams, p.stream_base, p.n_threads = device, n_streams, stream_base, threads
        p.n_originals, p.payload_min, p.payload_max = wp.n, wp.pmin, wp.pmax
        p.loss_thresh, p.ge_enable, p.gb_thresh, p.bg_thresh = wp.loss, wp.ge, wp.gb, wp.bg
        p.loss_on_recovery, p.fec_rate_q16, p.ack_every, p.ack_bytes = wp.lossrec, wp.fec, wp.ack, wp.ackbytes
        p.arq_lag, p.flush_max, p.record, p.arena_bytes = wp.arq, wp.flush, 1 if record else 0, arena_bytes
        # stage_host: True (both ends), or the tonk_amd.h mask (1 sender end, 2 receiver end)
        p.stage_host = 3 if stage_host is True else int(stage_host or 0)
        p.rtx_every, p.rtx_msec = wp.rtx, wp.rtxms
        p.input_pool = input_pool
        p.hold_full = wp.full
        self.n_streams = n_streams
        err = ctypes.create_string_buffer(512)
        self._h = lib().tamd_session_create(ctypes.byref(p), err, len(err))
        if not self._h:
            raise RuntimeError(f"tonk_amd: session creation failed: {err.value.decode()}")

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            err = lib().tamd_session_error(self._h).decode()
            raise RuntimeError(f"tonk_amd: {what} failed (rc={rc}): {err}; summary={self.summary()}")

    def generate(self) -> None:
        self._check(lib().tamd_session_generate(self._h), "input generation")

    def step(self, originals: int) -> None:
        self._check(lib().tamd_session_step(self._h, originals), "step")

    def wait(self) -> None:
        self._check(lib().tamd_session_wait(self._h), "wait")

    def finish(self) -> None:
        self._check(lib().tamd_session_finish(self._h), "finish")

    def summary(self) -> dict:
        out = (ctypes.c_uint64 * len(SUMMARY_FIELDS))()
        lib().tamd_session_summary(self._h, out, len(SUMMARY_FIELDS))
        return dict(zip(SUMMARY_FIELDS, [int(v) for v in out]))

    def set_timing(self, on: bool) -> None:
        lib().tamd_session_set_timing(self._h, 1 if on else 0)

    def arena(self) -> tuple[int, int]:
        """(device base address, mapped bytes) of the session's arena (diagnostics)."""
        base, n = ctypes.c_uint64(0), ctypes.c_uint64(0)
        lib().tamd_session_arena(self._h, ctypes.byref(base), ctypes.byref(n))
        return int(base.value), int(n.value)

    def kernel_ms(self) -> tuple[float, int]:
        n = ctypes.c_uint64(0)
        ms = lib().tamd_session_kernel_ms(self._h, ctypes.byref(n))
        return ms, int(n.value)

    HOST_PHASES = ("control_wall", "control_sum", "layout", "fill", "launch", "control_max", "slot_wait",
                   "upload_enqueue", "upload_enqueue_max", "slot_reallocs")

    # the same entries under the free-running schedule (include/tonk_amd.h)
    HOST_PHASES_FR = ("parts_wait", "control_sum", "open_wait", "stolen_steps", "close_launch", "control_max",
                      "slot_wait", "upload_enqueue", "upload_enqueue_max", "slot_reallocs")

    def free_running(self) -> bool:
        return lib().tamd_session_schedule(self._h) == 1

    def host_ms(self) -> dict:
        out = (ctypes.c_double * 10)()
        lib().tamd_session_host_ms(self._h, out)
        names = self.HOST_PHASES_FR if self.free_running() else self.HOST_PHASES
        return dict(zip(names, [float(v) for v in out]))

    def cpus(self) -> list[int]:
        """CPUs the worker threads are pinned to (empty: not pinned)."""
        out = (ctypes.c_int * 1024)()
        n = lib().tamd_session_cpus(self._h, out, 1024)
        return [int(out[i]) for i in range(min(n, 1024))]

    def transcript(self, stream: int) -> str:
        need = lib().tamd_session_transcript(self._h, stream, None, 0)
        buf = ctypes.create_string_buffer(need)
        lib().tamd_session_transcript(self._h, stream, buf, need)
        return buf.value.decode()

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().tamd_session_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
