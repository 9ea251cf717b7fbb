"""Loads libmicksum.so (the HIP extension) and declares the C ABI of
include/mi_cksum.h for ctypes.

The library is built in-tree (``make -C libunsod_amd/csrc`` or
``__graft_entry__.build()``) into ``libunsod_amd/lib/libmicksum.so``.  There is no
fallback: if the library is missing, importing the package raises.
"""
from __future__ import annotations

import ctypes as C
import os

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.environ.get("MI_CKSUM_LIB") or os.path.join(LIB_DIR, "libmicksum.so")  # override: A/B builds

MI_SPAN_STREAM = 0
MI_SPAN_ABS = 1
MI_ST_IP_BAD = 1
MI_ST_L4_BAD = 2
MI_ST_MALFORMED = 4
MI_ST_L4_NONE = 8
MI_BATCH_PACKED = 1
MI_BATCH_DEMUX = 2
MI_BATCH_HOST_STAGED = 4
MI_BATCH_OFFS32 = 8
MI_BATCH_MAX_BYTES = 0xFFFFE000  # include/mi_cksum.h
MI_TIME_NONE = 0
MI_TIME_REGION = 1
MI_TIME_PER_PASS = 2
MI_REPEAT_GRAPH = 0x100
MI_REPEAT_AFTER_DEFAULT = 0x200
MI_REPEAT_ASYNC = 0x400
MI_REPEAT_OP_VERIFY = 0
MI_REPEAT_OP_FINALIZE = 1
MI_CHAIN_SKIP = 0
MI_CHAIN_PSEUDO = 1
MI_CSUM_IP_CHECKED = 0x100
MI_CSUM_IP_VALID = 0x200
MI_CSUM_DATA_VALID = 0x400
MI_CSUM_PSEUDO_HDR = 0x800
MI_CSUM_IP = 0x1
MI_CSUM_TCP = 0x2
MI_CSUM_UDP = 0x4
MI_TX_NOBUFS = 1
MI_TX_SHORT = 2
MI_TX_NOSUM = 4
MI_TX_L4_SKIPPED = 8


class MiCksumError(RuntimeError):
    """A libmicksum batch call returned -errno."""

    def __init__(self, fn: str, rc: int, msg: str):
        super().__init__(f"{fn} failed ({rc} {os.strerror(-rc) if rc < 0 else ''}): {msg}")
        self.rc = rc


class PktBatchC(C.Structure):
    """struct mi_pkt_batch (include/mi_cksum.h)."""
    _fields_ = [
        ("base", C.c_void_p),
        ("bytes", C.c_uint64),
        ("offs", C.c_void_p),
        ("stride", C.c_uint64),
        ("first_off", C.c_uint64),
        ("lens", C.c_void_p),
        ("fixed_len", C.c_uint32),
        ("n", C.c_uint32),
        ("max_len", C.c_uint32),
        ("flags", C.c_uint32),
    ]


class SpanSeedsC(C.Structure):
    """struct mi_span_seeds (include/mi_cksum.h)."""
    _fields_ = [(k, C.c_void_p) for k in ("seeds", "src", "dst", "proto", "plens")]


class ChainBatchC(C.Structure):
    """struct mi_chain_batch (include/mi_cksum.h)."""
    _fields_ = [
        ("base", C.c_void_p),
        ("bytes", C.c_uint64),
        ("seg_off", C.c_void_p),
        ("seg_len", C.c_void_p),
        ("pkt_seg", C.c_void_p),
        ("n", C.c_uint32),
        ("mode", C.c_uint32),
        ("len", C.c_void_p),
        ("skip", C.c_void_p),
        ("src", C.c_void_p),
        ("dst", C.c_void_p),
        ("proto", C.c_void_p),
        ("max_seg", C.c_uint32),
        ("nseg", C.c_uint32),
    ]


class TxBatchC(C.Structure):
    """struct mi_tx_batch (include/mi_cksum.h)."""
    _fields_ = [
        ("src", C.c_void_p),
        ("src_bytes", C.c_uint64),
        ("seg_off", C.c_void_p),
        ("seg_len", C.c_void_p),
        ("pkt_seg", C.c_void_p),
        ("pkt_len", C.c_void_p),
        ("csum_flags", C.c_void_p),
        ("csum_data", C.c_void_p),
        ("dst", C.c_void_p),
        ("dst_bytes", C.c_uint64),
        ("dst_stride", C.c_uint64),
        ("dst_first", C.c_uint64),
        ("room", C.c_uint32),
        ("l3_off", C.c_uint32),
        ("n", C.c_uint32),
        ("max_len", C.c_uint32),
    ]


# Every symbol include/mi_cksum.h declares -> (restype, argtypes).
SIGNATURES = {
    "in_cksum_skip": (C.c_ushort, [C.c_void_p, C.c_int, C.c_int]),
    "in_cksum_pseudo_header": (C.c_uint16, [C.c_void_p, C.c_int, C.c_int, C.c_uint32, C.c_uint32, C.c_uint8]),
    "in_cksum_hdr": (C.c_uint, [C.c_void_p]),
    "in_pseudo": (C.c_ushort, [C.c_uint, C.c_uint, C.c_uint]),
    "in_addword": (C.c_ushort, [C.c_ushort, C.c_ushort]),
    "mi_cksum_device_count": (C.c_int, []),
    "mi_cksum_init": (C.c_int, [C.c_int]),
    "mi_cksum_strerror": (C.c_char_p, []),
    "mi_cksum_version": (C.c_char_p, []),
    "mi_cksum_set_shape": (C.c_int, [C.c_int, C.c_int, C.c_int]),
    "mi_cksum_set_run_kernel": (C.c_int, [C.c_int, C.c_int]),
    "mi_cksum_span_batch": (C.c_int, [C.POINTER(PktBatchC), C.c_uint32, C.POINTER(SpanSeedsC), C.c_void_p,
                                      C.c_void_p]),
    "mi_cksum_chain_batch": (C.c_int, [C.POINTER(ChainBatchC), C.c_void_p, C.c_void_p]),
    "mi_cksum_ipv4_verify": (C.c_int, [C.POINTER(PktBatchC), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p]),
    "mi_cksum_ipv4_finalize": (C.c_int, [C.POINTER(PktBatchC), C.c_void_p]),
    "mi_cksum_ipv4_verify_multi": (C.c_int, [C.POINTER(PktBatchC), C.c_uint32, C.POINTER(C.c_void_p),
                                             C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_void_p,
                                             C.c_void_p]),
    "mi_cksum_tx_copy": (C.c_int, [C.POINTER(TxBatchC), C.c_void_p, C.c_void_p]),
    "mi_cksum_tx_copy_host": (C.c_int, [C.POINTER(TxBatchC), C.c_void_p, C.c_uint32]),
    "mi_cksum_tx_repeat_create": (C.c_int, [C.POINTER(TxBatchC), C.c_uint32, C.POINTER(C.c_void_p), C.c_uint32,
                                            C.POINTER(C.c_void_p)]),
    "mi_cksum_verify_plan": (C.c_char_p, [C.POINTER(PktBatchC)]),
    "mi_cksum_rx_offload": (C.c_int, [C.POINTER(PktBatchC), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mi_cksum_ipv4_verify_repeat": (C.c_int, [C.POINTER(PktBatchC), C.c_uint32, C.POINTER(C.c_void_p),
                                              C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_uint32,
                                              C.c_uint32, C.c_uint32, C.POINTER(C.c_float),
                                              C.POINTER(C.c_float)]),
    "mi_cksum_repeat_create": (C.c_int, [C.POINTER(PktBatchC), C.c_uint32, C.POINTER(C.c_void_p),
                                         C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_uint32,
                                         C.POINTER(C.c_void_p)]),
    "mi_cksum_repeat_run": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_float)]),
    "mi_cksum_repeat_span": (C.c_int, [C.c_void_p, C.POINTER(C.c_float)]),
    "mi_cksum_repeat_destroy": (None, [C.c_void_p]),
    "mi_cksum_set_busy_wait": (C.c_int, [C.c_int]),
    "mi_cksum_repeat_set_op": (C.c_int, [C.c_void_p, C.c_uint32]),
    "mi_cksum_repeat_set_engine": (C.c_int, [C.c_void_p, C.c_uint32]),
    "mi_cksum_ipv4_verify_host": (C.c_int, [C.POINTER(PktBatchC), C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_void_p]),
    "mi_cksum_rx_offload_host": (C.c_int, [C.POINTER(PktBatchC), C.c_void_p, C.c_void_p, C.c_void_p]),
    "mi_cksum_host_register": (C.c_int, [C.c_void_p, C.c_uint64]),
    "mi_cksum_host_unregister": (C.c_int, [C.c_void_p]),
    "mi_cksum_synth_ipv4": (C.c_int, [C.POINTER(PktBatchC), C.c_uint64, C.c_void_p]),
    "mi_cksum_hsa_queues": (C.c_int, []),
    "mi_cksum_set_dropin_error_handler": (None, [C.c_void_p]),
    "mi_cksum_set_dropin_mode": (C.c_int, [C.c_int]),
    "mi_cksum_dropin_degraded": (C.c_uint64, []),
}
# (b1) serving modes (include/mi_cksum.h)
MI_DROPIN_HOST, MI_DROPIN_GPU = 0, 1

# mi_cksum_error_fn: void (*)(const char *what, const char *err)
DROPIN_ERROR_FN = C.CFUNCTYPE(None, C.c_char_p, C.c_char_p)

_lib = None


def load() -> C.CDLL:
    """Load libmicksum.so once; raise if it is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: the HIP extension must be built "
            "(python -c 'import __graft_entry__ as g; g.build()' or make -C libunsod_amd/csrc)")
    # torch bundles its own libamdhip64 (SONAME libamdhip64.so.7, NEEDED by torch
    # as "libamdhip64.so"): load it first so libmicksum binds to that same
    # runtime instead of pulling a second HIP runtime into the process.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(fn: str, rc: int) -> None:
    if rc != 0:
        raise MiCksumError(fn, rc, load().mi_cksum_strerror().decode(errors="replace"))
