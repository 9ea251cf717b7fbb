"""Multi-GPU sharding on the HIP path, world size 2 over gloo.

Each rank takes its byte-balanced contiguous range of the 2^22-datagram Pareto
batch (shard.shard_by_bytes), copies those bytes into a buffer of its own (what
it would hold in its HBM), verifies them with the gfx950 kernel, and only the
bad-packet counter and the timing are reduced; there is no collective on the
data.  Rank 0 checks that the union of the ranks' results equals the CPU
oracle over the whole batch.  Both ranks use cuda:(rank % device_count), so
on a one-GPU box they share device 0.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N = 1 << 22


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import libunsod_amd as mi
        from libunsod_amd import shard, synth
        dev = torch.device("cuda", rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        lens = synth.pareto_lengths(N)
        offs = synth.packed_offsets(lens, first_off=2)
        size = (int(offs[-1] + lens[-1]) + 64 + 255) & ~255
        # the whole batch, generated and TX-finalized on the device, 1 % corrupted
        whole = torch.empty(size, dtype=torch.uint8, device=dev)
        d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
        d_lens = torch.from_numpy(lens.astype(np.int32)).to(dev)
        wb = mi.PktBatch(whole, N, offs=d_offs, lens=d_lens, max_len=int(lens.max()), packed=True)
        mi.synth_ipv4(wb, seed=0x5EED5EED)
        mi.ipv4_finalize(wb)
        rng = np.random.default_rng(21)
        bad = np.sort(rng.choice(N, N // 100, replace=False))
        pos = torch.from_numpy((offs[bad] + rng.integers(0, lens[bad])).astype(np.int64)).to(dev)
        whole[pos] ^= 0x10
        # this rank's shard, in a buffer of its own
        lo, hi = shard.shard_by_bytes(lens, world, rank)
        base = int(offs[lo]) & ~15
        end = int(offs[hi - 1] + lens[hi - 1])
        mine = whole[base:end + 64].clone()
        mb = mi.PktBatch(mine, hi - lo, offs=d_offs[lo:hi] - base, lens=d_lens[lo:hi], max_len=int(lens.max()),
                         packed=True, offs32=True)
        r = mi.ipv4_verify(mb, bad_count=True)
        torch.cuda.synchronize()
        nbad = torch.tensor([int(r["bad"].item())], dtype=torch.int64)
        dist.all_reduce(nbad)
        got = [None] * world
        dist.all_gather_object(got, (lo, hi, r["ip"].cpu().numpy(), r["l4"].cpu().numpy(),
                                     r["status"].cpu().numpy()))
        if rank == 0:
            from oracle.pyoracle import Oracle
            host = whole.cpu().numpy()
            raw = np.zeros(host.size + 128, np.uint8)
            s = (-raw.ctypes.data) % 64
            h = raw[s:s + host.size]
            h[:] = host
            ip_o, l4_o, st_o = Oracle("port").ipv4_verify_batch(h, N, offs=offs, flen=lens.astype(np.uint32),
                                                                nthreads=8)
            ok = ([g[:2] for g in got] == shard.all_shards(lens, world)
                  and np.array_equal(np.concatenate([g[2] for g in got]), ip_o)
                  and np.array_equal(np.concatenate([g[3] for g in got]), l4_o)
                  and np.array_equal(np.concatenate([g[4] for g in got]), st_o)
                  and int(nbad.item()) == int((st_o != 0).sum()) == bad.size)
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_world2_pareto_shards_hip():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(220)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True
