"""libunsod_amd -- MI355X-native RFC 1071 checksum path of iamyb/libunsod.

The product is the C-ABI library ``lib/libmicksum.so`` (HIP kernels for gfx950
+ the drop-in ``in_cksum*`` symbols, include/mi_cksum.h).  This package loads it
(and raises if it is missing: the batch path has no CPU fallback) and mirrors the
reference interface in Python for tests and the bench.
"""
from ._lib import (LIB_PATH, MI_SPAN_ABS, MI_SPAN_STREAM, MI_ST_IP_BAD, MI_ST_L4_BAD, MI_ST_MALFORMED, MI_ST_L4_NONE,
                   MiCksumError, load)
from .api import (ChainBatch, MbufChain, chain_batch, PktBatch, device_count, host_register, host_unregister, in_addword, in_cksum,
                  in_cksum_hdr, in_cksum_pseudo_header, in_cksum_skip, in_pseudo, init, ipv4_finalize,
                  ipv4_verify, ipv4_verify_multi, ipv4_verify_host, rx_offload_host, ipv4_verify_repeat, VerifyRepeat, rx_offload, set_busy_wait, set_shape, set_run_kernel, verify_plan, span_batch, synth_ipv4, version,
                  TxBatch, TxRepeat, tx_copy, tx_copy_host, page_buffer, set_dropin_mode, dropin_degraded)

load()

__all__ = [
    "LIB_PATH", "MI_SPAN_ABS", "MI_SPAN_STREAM", "MI_ST_IP_BAD", "MI_ST_L4_BAD", "MI_ST_MALFORMED", "MI_ST_L4_NONE",
    "MiCksumError", "load", "ChainBatch", "MbufChain", "chain_batch", "PktBatch", "device_count", "host_register", "host_unregister",
    "in_addword", "in_cksum", "in_cksum_hdr", "in_cksum_pseudo_header", "in_cksum_skip", "in_pseudo", "init",
    "ipv4_finalize", "ipv4_verify", "ipv4_verify_multi", "ipv4_verify_host", "rx_offload_host", "ipv4_verify_repeat", "VerifyRepeat", "rx_offload", "set_busy_wait", "span_batch", "verify_plan", "synth_ipv4", "version",
    "TxBatch", "TxRepeat", "tx_copy", "tx_copy_host", "page_buffer", "set_dropin_mode", "dropin_degraded",
]
