import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden", "cksum_golden.npz")
DEMUX_GOLDEN = os.path.join(ROOT, "tests", "golden", "demux_golden.npz")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmicksum's HIP kernels)")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        have_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        have_gpu = False
    if have_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment (gpu tests run on the MI355X box)")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def demux_golden():
    with np.load(DEMUX_GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def chain_segments(g, seg0: int, nseg: int):
    """[(bytes, addr_mod)] of a golden chain."""
    out = []
    for s in range(seg0, seg0 + nseg):
        off, ln, mod = int(g["seg_off"][s]), int(g["seg_len"][s]), int(g["seg_mod"][s])
        out.append((g["blob"][off:off + ln].tobytes(), mod))
    return out


def aligned(a: np.ndarray, align: int = 64):
    """Copy of ``a`` at an address == 0 (mod align); returns (keepalive, view)."""
    raw = np.zeros(a.size + 2 * align, np.uint8)
    s = (-raw.ctypes.data) % align
    v = raw[s:s + a.size]
    v[:] = a
    return raw, v


@pytest.fixture(params=["host", "dispatch", "service"])
def dropin_mode(request):
    """The (b1) drop-ins on the CPU (MI_DROPIN_HOST, the default), as one AQL
    dispatch per call, or through the device's resident drop-in service
    (MI_DROPIN_GPU; MI_CKSUM_DROPIN_SERVICE); restored afterwards.  In the GPU
    modes no call may have been served by the host fold (a GPU error degrades
    to it): the results checked came from the GPU."""
    import ctypes as C

    import libunsod_amd as mi
    from libunsod_amd._lib import load
    lib = load()
    lib.mi__set_dropin_service.restype = C.c_int
    lib.mi__set_dropin_service.argtypes = [C.c_int]
    gpu = request.param != "host"
    mode_was = mi.set_dropin_mode("gpu" if gpu else "host")
    was = lib.mi__set_dropin_service(1 if request.param == "service" else 0)
    assert was in (0, 1)
    degraded = mi.dropin_degraded()
    yield request.param
    assert lib.mi__set_dropin_service(was) in (0, 1)
    mi.set_dropin_mode(mode_was)
    if gpu:
        assert mi.dropin_degraded() == degraded, "a GPU-mode drop-in was served by the host fold"


@pytest.fixture
def gpu_dropins():
    """The (b1) drop-ins through the GPU (MI_DROPIN_GPU) for one test, and no
    call served by the host fold."""
    import libunsod_amd as mi
    was = mi.set_dropin_mode("gpu")
    degraded = mi.dropin_degraded()
    yield
    mi.set_dropin_mode(was)
    assert mi.dropin_degraded() == degraded, "a GPU-mode drop-in was served by the host fold"
