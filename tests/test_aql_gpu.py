"""The repeat handle's AQL engine (mi_cksum_repeat_set_engine,
MI_REPEAT_ENGINE_AQL): passes submitted as prebuilt AQL packets into the
handle's own HSA queue(s) must write exactly what the HIP launches write --
every verify plan it serves (lane-group shapes, flat run, 64-byte slots),
one or two queues, runs longer than the queue, asynchronous runs -- checked
against the CPU oracle (ip_input.c:459-471 + tcp_input.c:697-720)."""
import numpy as np
import pytest
import torch

from oracle.pyoracle import Oracle

import libunsod_amd as mi
from libunsod_amd import synth

pytestmark = pytest.mark.gpu
ORC = Oracle("port")


def dev_tensor(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def cpu(t):
    return t.cpu().numpy()


def _uniform(n, L, stride, first, seed, corrupt=True):
    b0 = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=seed)
    h = b0["buf"]
    ORC.ipv4_finalize_batch(h, n, stride=stride, first_off=first, fixed_flen=L)
    if corrupt:
        rng = np.random.default_rng(seed)
        for i in rng.choice(n, max(1, n // 40), replace=False):
            h[first + int(i) * stride + int(rng.integers(0, L))] ^= 0x41
    want = ORC.ipv4_verify_batch(h, n, stride=stride, first_off=first, fixed_flen=L)
    return mi.PktBatch(dev_tensor(h), n, stride=stride, first_off=first, fixed_len=L), want


def _packed(n, seed):
    lens = synth.pareto_lengths(n, seed=seed)
    offs = synth.packed_offsets(lens, first_off=2)
    h = synth.build_ipv4_batch(n, lens, offs=offs.astype(np.int64), seed=seed + 1)["buf"]
    ORC.ipv4_finalize_batch(h, n, offs=offs, flen=lens.astype(np.uint32))
    h[offs[::29].astype(np.int64) + 25] ^= 4
    want = ORC.ipv4_verify_batch(h, n, offs=offs, flen=lens.astype(np.uint32))
    return mi.PktBatch(dev_tensor(h), n, offs=dev_tensor(offs.astype(np.int64)),
                       lens=dev_tensor(lens.astype(np.int32)), packed=True), want


def _outs(n):
    return dict(ip=torch.zeros(n, dtype=torch.uint16, device="cuda"),
                l4=torch.zeros(n, dtype=torch.uint16, device="cuda"),
                status=torch.zeros(n, dtype=torch.uint8, device="cuda"))


def _check(outs, wants):
    for o, w in zip(outs, wants):
        assert np.array_equal(cpu(o["ip"]), w[0])
        assert np.array_equal(cpu(o["l4"]), w[1])
        assert np.array_equal(cpu(o["status"]), w[2])


@pytest.mark.parametrize("nq", [1, 2])
def test_aql_uniform_rotation_and_span(nq):
    bs, wants = zip(*[_uniform(4096, 1500, 2176, 142, 300 + r) for r in range(3)])
    outs = [_outs(4096) for _ in bs]
    torch.cuda.synchronize()
    rep = mi.VerifyRepeat(list(bs), outs, nstreams=nq, engine="aql")
    try:
        rep.run(2)  # batches 0, 1
        assert not cpu(outs[2]["status"]).any() and not cpu(outs[2]["ip"]).any()
        rep.run(1, timed=True)  # batch 2: the rotation continues
        assert rep.span() > 0
        _check(outs, wants)
        # a timed multi-pass run: span covers all passes
        for o in outs:
            for t in o.values():
                t.zero_()
        torch.cuda.synchronize()
        rep.run(6, timed=True)
        assert rep.span() > 0
        _check(outs, wants)
    finally:
        rep.close()


# every plan the engine serves: lane-group shapes picked by length, the flat
# run over dense slots and packed mixed lengths, one lane per 64-byte slot
@pytest.mark.parametrize("spec", [
    (2048, 46, 64, 14),        # 64-byte slots -> mi_aql_slot64
    (2048, 100, 128, 2),       # dense slots -> flat run (U = 4)
    (2048, 40, 2176, 142),     # 1x4
    (2048, 100, 2176, 142),    # 1x8
    (2048, 200, 2176, 142),    # 4x4
    (2048, 700, 2176, 142),    # 8x4
    (2048, 1500, 2176, 142),   # 16x6
    (1024, 3000, 4096, 142),   # 8x8
    (512, 9000, 9216, 142),    # 8x12
    "packed",                  # Pareto, packed -> flat run (U = 8)
])
def test_aql_every_plan_bit_exact(spec):
    if spec == "packed":
        b, w = _packed(3000, 41)
        n = 3000
    else:
        n, L, stride, first = spec
        b, w = _uniform(n, L, stride, first, 17 + L)
    o = _outs(n)
    torch.cuda.synchronize()
    rep = mi.VerifyRepeat([b], [o], nstreams=1, engine="aql")
    try:
        rep.run(1)
        _check([o], [w])
        # the HIP engine on the same handle gives the same bytes
        hip = {k: t.clone() for k, t in o.items()}
        for t in o.values():
            t.zero_()
        torch.cuda.synchronize()
    finally:
        rep.close()
    rep2 = mi.VerifyRepeat([b], [o], nstreams=1)
    rep2.run(1)
    rep2.close()
    for k in o:
        assert torch.equal(o[k], hip[k])


def test_aql_runs_longer_than_the_queue_and_async():
    """5000 passes through one 4096-packet queue (the submitter waits for
    free slots), then an asynchronous run completed by span()."""
    bs, wants = zip(*[_uniform(256, 1500, 2176, 142, 900 + r) for r in range(2)])
    outs = [_outs(256) for _ in bs]
    torch.cuda.synchronize()
    rep = mi.VerifyRepeat(list(bs), outs, nstreams=1, engine="aql")
    try:
        rep.run(5000, timed=True)
        assert rep.span() > 0
        _check(outs, wants)
        for o in outs:
            for t in o.values():
                t.zero_()
        torch.cuda.synchronize()
        rep.run(2, timed=True, wait=False)
        assert rep.span() > 0  # waits for the asynchronous run
        _check(outs, wants)
    finally:
        rep.close()


def test_aql_refuses_what_it_cannot_serve():
    # length-class batch (per-packet lengths, not packed): several launches per pass
    lens = np.full(64, 1500, np.int32)
    lens[::2] = 60
    buf = torch.zeros(64 * 2176, dtype=torch.uint8, device="cuda")
    offs = torch.arange(64, dtype=torch.int64, device="cuda") * 2176
    b = mi.PktBatch(buf, 64, offs=offs, lens=dev_tensor(lens), max_len=1500)
    with pytest.raises(mi.MiCksumError):
        mi.VerifyRepeat([b], [_outs(64)], nstreams=1, engine="aql")
    # finalize op
    b2, _ = _uniform(64, 1500, 2176, 142, 5, corrupt=False)
    with pytest.raises(mi.MiCksumError):
        mi.VerifyRepeat([b2], None, nstreams=1, op="finalize", engine="aql")


@pytest.mark.parametrize("nq", [2, 4])
def test_aql_rewritten_batches_between_runs(nq):
    """every queue's first packet acquires at system scope, so a
    run sees batch bytes rewritten between runs (a re-filled RX ring: here a
    host-to-device copy of different datagrams into the same buffers) on
    every queue, not stale lines of the previous run.  The outputs are checked
    after each run against the oracle of the bytes the run saw."""
    n, L, stride, first = 4096, 1500, 2176, 142
    nb = 2 * nq
    gens = [[_uniform(n, L, stride, first, 900 + 17 * g + r) for r in range(nb)] for g in range(3)]
    bs = [b for b, _ in gens[0]]
    outs = [_outs(n) for _ in bs]
    torch.cuda.synchronize()
    rep = mi.VerifyRepeat(bs, outs, nstreams=nq, engine="aql")
    try:
        for g in range(3):
            if g:
                for b, (bg, _) in zip(bs, gens[g]):
                    b.buf.copy_(bg.buf)  # new datagrams into the same device buffers
                for o in outs:
                    for t in o.values():
                        t.fill_(0xEE)
                torch.cuda.synchronize()
            rep.run(nb)  # one pass over every batch, spread over the nq queues
            _check(outs, [w for _, w in gens[g]])
    finally:
        rep.close()
