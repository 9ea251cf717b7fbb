"""Multi-GPU partitioning on the CPU: the path shards with no
data-path collective.  World-size-2 gloo run: each rank takes its byte-balanced
contiguous range of one mixed-length batch, verifies it on its own (here with
the CPU oracle standing in for the rank's GPU), and only timing / counters are
reduced.  The union of the ranks' results must equal the whole-batch result."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import aligned
from libunsod_amd import shard, synth
from oracle.pyoracle import Oracle


def test_shard_uniform():
    for n in (0, 1, 7, 65536):
        for w in (1, 2, 3, 8):
            r = [shard.shard_uniform(n, w, k) for k in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(r[k][1] == r[k + 1][0] for k in range(w - 1))
            assert max(b - a for a, b in r) - min(b - a for a, b in r) <= 1
    with pytest.raises(ValueError):
        shard.shard_uniform(10, 2, 2)


def test_shard_by_bytes():
    lens = synth.pareto_lengths(1 << 16)
    assert 64 <= lens.min() and lens.max() <= 9000
    total = int(lens.sum())
    for w in (1, 2, 4, 8):
        r = shard.all_shards(lens, w)
        assert r[0][0] == 0 and r[-1][1] == len(lens)
        assert all(r[k][1] == r[k + 1][0] for k in range(w - 1))
        sizes = [int(lens[a:b].sum()) for a, b in r]
        assert sum(sizes) == total
        assert max(sizes) - total / w <= 9000  # balanced to within one packet
    assert shard.shard_by_bytes([], 4, 3) == (0, 0)
    # more ranks than packets: empty shards, still a partition
    r = shard.all_shards([100, 200], 4)
    assert sum(b - a for a, b in r) == 2 and r[-1][1] == 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 6000
        lens = synth.pareto_lengths(n, seed=0x9A7E70)
        offs = synth.packed_offsets(lens, first_off=2)
        full = synth.build_ipv4_batch(n, lens, offs=offs.astype(np.int64), seed=77, payload="pattern")
        buf = full["buf"]
        orc = Oracle("port")
        _, whole = aligned(buf)
        orc.ipv4_finalize_batch(whole, n, offs=offs, flen=lens.astype(np.uint32))
        # corrupt a few packets everywhere
        bad = np.arange(5, n, 397)
        whole[offs[bad].astype(np.int64) + 30] ^= 0x40
        lo, hi = shard.shard_by_bytes(lens, world, rank)
        # this rank's shard lives in its own buffer (what it would hold in its HBM)
        base = int(offs[lo]) & ~15 if hi > lo else 0
        end = int(offs[hi - 1] + lens[hi - 1]) if hi > lo else 0
        _, mine = aligned(whole[base:end + 16].copy() if hi > lo else np.zeros(16, np.uint8))
        ip, l4, st = orc.ipv4_verify_batch(mine, hi - lo, offs=(offs[lo:hi] - base), flen=lens[lo:hi].astype(np.uint32))
        elapsed, nbytes, npkts = shard.job_totals(0.001 * (rank + 1), float(lens[lo:hi].sum()), float(hi - lo))
        gathered = [None] * world
        dist.all_gather_object(gathered, (lo, hi, ip, l4, st))
        nbad = int((st != 0).sum())
        import torch
        t = torch.tensor([nbad])
        dist.all_reduce(t)
        if rank == 0:
            ip_w, l4_w, st_w = orc.ipv4_verify_batch(whole, n, offs=offs, flen=lens.astype(np.uint32))
            got_ip = np.concatenate([g[2] for g in gathered])
            got_l4 = np.concatenate([g[3] for g in gathered])
            got_st = np.concatenate([g[4] for g in gathered])
            ok = (np.array_equal(got_ip, ip_w) and np.array_equal(got_l4, l4_w) and np.array_equal(got_st, st_w)
                  and int(t.item()) == int((st_w != 0).sum()) == len(bad)
                  and elapsed == pytest.approx(0.001 * world) and nbytes == float(lens.sum()) and npkts == n
                  and [g[:2] for g in gathered] == shard.all_shards(lens, world))
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_byte_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def _rank_uniform(rank, world, port, q):
    """The uniform configs' strong split (bench.py 1500_split / 9000_split):
    one batch of fixed slots, contiguous packet ranges of N/G packets."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, L, stride, first = 3001, 1500, 2176, 142
        full = synth.build_ipv4_batch(n, L, stride=stride, first_off=first, seed=91)
        orc = Oracle("port")
        _, whole = aligned(full["buf"])
        orc.ipv4_finalize_batch(whole, n, stride=stride, first_off=first, fixed_flen=L)
        bad = np.arange(3, n, 211)
        whole[first + bad * stride + 700] ^= 0x08
        lo, hi = shard.shard_uniform(n, world, rank)
        # this rank's range in a buffer of its own, same slot geometry
        _, mine = aligned(whole[lo * stride:hi * stride + first + L].copy())
        ip, l4, st = orc.ipv4_verify_batch(mine, hi - lo, stride=stride, first_off=first, fixed_flen=L)
        elapsed, nbytes, npkts = shard.job_totals(0.001 * (rank + 1), float(L * (hi - lo)), float(hi - lo))
        gathered = [None] * world
        dist.all_gather_object(gathered, (lo, hi, ip, l4, st))
        if rank == 0:
            ip_w, l4_w, st_w = orc.ipv4_verify_batch(whole, n, stride=stride, first_off=first, fixed_flen=L)
            ok = (np.array_equal(np.concatenate([g[2] for g in gathered]), ip_w)
                  and np.array_equal(np.concatenate([g[3] for g in gathered]), l4_w)
                  and np.array_equal(np.concatenate([g[4] for g in gathered]), st_w)
                  and int((st_w != 0).sum()) == len(bad) and nbytes == float(L * n) and npkts == n
                  and elapsed == pytest.approx(0.001 * world)
                  and [g[:2] for g in gathered] == [shard.shard_uniform(n, world, k) for k in range(world)])
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_uniform_split():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_uniform, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True
