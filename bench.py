#!/usr/bin/env python3
"""bench.py -- GiB/s checksummed, device-resident, one process per GPU.

A step = one RX-verify pass (ip_input.c:459-471 + tcp_input.c:697-720) over one
batch: for every packet the IPv4 header sum and the TCP pseudo-header sum, both
computed by one gfx950 kernel launch reading each datagram once
(mi_cksum_ipv4_verify).  Default workload = BASELINE.json configs[1]: 65536 x
1500 B IPv4/TCP datagrams in 2176 B rte_mbuf slots (IP header at +142).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1500|9000|64|pareto]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Multi-GPU: packets are independent, so every rank folds its own batch (weak
scaling, no data-path collective); the process group only carries the barrier
and the max-over-ranks of the elapsed time.

Rank 0 at N=1 also times the reference CPU path (cpu_baseline: the reference's
own in_cksum.c from oracle/_ref, or the restatement if that is absent) on a
bounded sample of the same host bytes, and the host-memory (PCIe-inclusive)
path.  Prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "GiB/s checksummed (device-resident), batched 1500B & 9000B frames, 1/2/4/8 GPU"
GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (packets per GPU, IP datagram length, slot stride, IP offset in slot)
    "1500": (65536, 1500, 2176, 142),
    "9000": (65536, 9000, 9216, 142),
    "64": (1 << 20, 46, 64, 14),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--config", default="1500", choices=list(CONFIGS) + ["pareto"])
    ap.add_argument("--rotate", type=int, default=0, help="distinct batches cycled (0: enough for >= 1 GiB)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--offs64", action="store_true",
                    help="pareto: u64 packet offsets instead of u32 (MI_BATCH_OFFS32, 4 B less per datagram)")
    ap.add_argument("--streams", type=int, default=2, help="streams the steps alternate over")
    ap.add_argument("--submit", default="launch", choices=["graph", "launch"],
                    help="launch: K host launches from native code; graph: the same K launches as one cached "
                         "hipGraph (measured slower for 1500 B: profiles/submit_r01.jsonl)")
    ap.add_argument("--settle", type=float, default=0.3,
                    help="untimed warm-up lasts at least this many seconds (GPU clock settle)")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MI_BENCH_DEVICE / MI_BENCH_BACKEND exist only to rehearse the N>1 path on
    # a one-GPU box (all ranks on one device, gloo); the driver's runs use
    # LOCAL_RANK and RCCL ("nccl").
    gpu = int(os.environ.get("MI_BENCH_DEVICE", local))
    backend = os.environ.get("MI_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import libunsod_amd as mi
    from libunsod_amd import shard, synth

    # ---------------------------------------------------------- workload
    if args.config == "pareto":
        total_n = 1 << 22
        lens_all = synth.pareto_lengths(total_n)
        lo, hi = shard.shard_by_bytes(lens_all, world, rank)
        lens = lens_all[lo:hi]
        n = hi - lo
        offs = synth.packed_offsets(lens, first_off=2)
        L_sum = int(lens.sum())
        size = int(offs[-1] + lens[-1]) + 64 if n else 64
        workload = f"Pareto 64-9000 B IPv4/TCP RX verify, {total_n} packets split by bytes over {world} GPU(s)"
        scaling = "strong"
        cfg = dict(workload=workload, packets_total=total_n, packets_this_rank=n, seed="0x9A7E70", alpha=1.16,
                   offsets="u64" if args.offs64 else "u32")
    else:
        n, L, stride, first = CONFIGS[args.config]
        lens = offs = None
        L_sum = n * L
        size = first + (n - 1) * stride + L + 64
        workload = f"{n} x {L} B IPv4/TCP RX verify per GPU (slot stride {stride}, IP at +{first})"
        scaling = "weak"
        cfg = dict(workload=workload, packets_per_gpu=n, ip_datagram_len=L, slot_stride=stride, ip_offset=first)
    size = (size + 255) & ~255
    R = args.rotate or max(1, -(-(1 << 30) // size))  # footprint >= 1 GiB: defeat the 256 MiB MALL
    cfg.update(streams=args.streams, rotating_batches=R, footprint_MiB=round(R * size / 2**20, 1),
               parallelism=f"dp{world} (independent packet shards, no collective)")

    batches, outs = [], []
    for r in range(R):
        buf = torch.empty(size, dtype=torch.uint8, device=dev)
        if lens is None:
            b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
        else:
            b = mi.PktBatch(buf, n, offs=torch.from_numpy(offs.astype(np.int64)).to(dev),
                            lens=torch.from_numpy(lens.astype(np.int32)).to(dev), max_len=int(lens.max()),
                            packed=True, offs32=not args.offs64)
        mi.synth_ipv4(b, seed=0x5EED5EED + 7919 * r + 104729 * rank)
        mi.ipv4_finalize(b)  # TX path makes every packet valid
        batches.append(b)
        outs.append(dict(ip=torch.empty(n, dtype=torch.uint16, device=dev),
                         l4=torch.empty(n, dtype=torch.uint16, device=dev),
                         status=torch.empty(n, dtype=torch.uint8, device=dev)))
    torch.cuda.synchronize()
    # sanity: everything verifies
    chk = mi.ipv4_verify(batches[0], bad_count=True)
    torch.cuda.synchronize()
    if int(chk["bad"].item()) != 0:
        raise SystemExit(f"rank {rank}: synthetic batch does not verify ({int(chk['bad'].item())} bad)")

    nst = max(1, args.streams)
    tw = time.perf_counter()
    use_graph = args.submit == "graph"
    if args.warmup:
        mi.ipv4_verify_repeat(batches, outs, args.warmup, nstreams=nst, timing="none", graph=use_graph)
    torch.cuda.synchronize()
    # Settle: the first ~0.1 s of back-to-back launches run up to 20 % slower
    # (clock / translation warm-up; profiles/warmup_r01.jsonl: 40 warmup steps ->
    # 17.0 us per launch, 2000 -> 14.25 us).  Keep launching untimed steps until
    # the warmup phase has lasted `--settle` seconds, whatever W is.
    settle_steps = 0
    while time.perf_counter() - tw < args.settle:
        mi.ipv4_verify_repeat(batches, outs, 500, nstreams=nst, timing="none", graph=use_graph)
        settle_steps += 500
    cfg["settle_steps"] = settle_steps
    cfg["submit"] = args.submit
    if use_graph:  # instantiate the timed region's graph (K passes) before timing it
        mi.ipv4_verify_repeat(batches, outs, args.steps, nstreams=nst, timing="none", graph=True)

    # ------------------------------------------------------- timed region
    # K launches issued back to back from native code (libmicksum), alternating
    # over `nst` non-blocking streams so that a launch's ramp-up overlaps its
    # predecessor's drain; a hipEvent pair per stream brackets the region.
    # --submit graph: the same K launches captured once into a hipGraph
    # (instantiated above, outside the timed region) and replayed.
    K = args.steps
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    span_us = mi.ipv4_verify_repeat(batches, outs, K, nstreams=nst, timing="region", graph=use_graph)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed, job_bytes, job_pkts = shard.job_totals(t1 - t0, float(L_sum) * K, float(n) * K,
                                                    device=dev if dist and backend == "nccl" else None)
    value = job_bytes / elapsed / GIB

    # Roofline of the dominant kernel (k_ipv4_verify*, the one verify_plan names).  Algorithmic bytes per
    # launch = sum(L) read + 5 B written per packet (ip u16, l4 u16, status u8).
    # Average launch duration = GPU span of the timed region (hipEvents on the
    # launch streams) / K: launches on different streams overlap, so this is the
    # GPU time each launch costs; rocprof's union of dispatch intervals / K is
    # the same quantity (tools/prof_summary.py).
    gpu_s_per_launch = span_us / K / 1e6
    alg_bytes = float(L_sum) + 5.0 * n
    achieved = alg_bytes / gpu_s_per_launch / 1e9
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):
        try:
            traffic = json.load(open(tfile)).get(args.config, {}).get("bytes_per_launch")
        except Exception:
            traffic = None
    roof = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic,
                kernel=mi.verify_plan(batches[0]), alg_bytes_per_launch=int(alg_bytes),
                avg_launch_us=round(gpu_s_per_launch * 1e6, 2), streams=nst)
    # the same kernel alone on one stream, every launch bracketed by events
    # (compare with a single-stream rocprof trace)
    iso_us, _ = mi.ipv4_verify_repeat(batches, outs, min(K, 100), nstreams=1, timing="pass")
    roof["isolated_launch_us"] = round(float(np.median(iso_us)), 2)
    roof["isolated_achieved"] = round(alg_bytes / (float(np.median(iso_us)) / 1e6) / 1e9, 1)

    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": K,
        "warmup": args.warmup, "ms_per_step": round(elapsed / K * 1e3, 5), "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: device-generated IPv4/TCP datagrams (splitmix64 payload), TX-finalized to valid sums",
        "config": cfg, "mpkt_per_s": round(job_pkts / elapsed / 1e6, 2), "roofline": roof,
    }

    # -------------------------------------------- CPU baseline + host path
    if world == 1 and rank == 0:
        host = batches[0].buf.cpu().numpy()
        lay = dict(stride=stride, first_off=first, fixed_len=L) if lens is None else dict(offs=offs, lens=lens)
        if args.cpu_seconds > 0:
            result["cpu_baseline"] = cpu_baseline(host, n, L_sum, lay, args.cpu_seconds)
        if not args.no_host_path:
            result["pcie_inclusive"] = host_path(mi, host, n, L_sum, lay)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def _oracle_layout(lay: dict) -> dict:
    if "offs" in lay:
        return dict(offs=lay["offs"], flen=lay["lens"].astype(np.uint32))
    return dict(stride=lay["stride"], first_off=lay["first_off"], fixed_flen=lay["fixed_len"])


def cpu_baseline(host: np.ndarray, n: int, L_sum: int, lay: dict, seconds: float) -> dict:
    """The reference CPU path on the same bytes: ipv4_verify_batch drives
    in_cksum_hdr + in_cksum_pseudo_header per packet exactly as ip_input /
    tcp_input call them.  1 thread, repeated passes over the batch until
    `seconds` of CPU work."""
    from oracle.pyoracle import Oracle, available
    kind = "reference" if available("reference") else "port"
    o = Oracle(kind)
    raw = np.zeros(host.size + 128, np.uint8)
    s = (-raw.ctypes.data) % 64
    h = raw[s:s + host.size]
    h[:] = host
    ol = _oracle_layout(lay)
    ip, l4, st = o.ipv4_verify_batch(h, n, **ol)
    assert not st.any(), "CPU baseline disagrees: batch should verify"
    passes, t0 = 0, time.perf_counter()
    while True:
        o.ipv4_verify_batch(h, n, **ol)
        passes += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    src = "oracle/_ref (reference in_cksum.c)" if kind == "reference" else "oracle restatement"
    res = dict(value=round(passes * L_sum / dt / GIB, 3), unit="GiB/s", cores=1, kind=kind,
               sample=f"{passes} passes x {n} datagrams, {L_sum} B each pass ({dt:.1f} s, 1 thread): "
                      f"in_cksum_hdr + in_cksum_pseudo_header per packet, {src}, "
                      f"gcc -O3 -frename-registers -fno-strict-aliasing",
               cpu=_cpu_model())
    # the same path on every core this process may use (contiguous packet
    # ranges per pthread, oracle/batch_driver.c run_jobs)
    threads = _host_threads()
    if threads > 1:
        passes, t0 = 0, time.perf_counter()
        while True:
            o.ipv4_verify_batch(h, n, nthreads=threads, **ol)
            passes += 1
            if time.perf_counter() - t0 >= seconds / 2:
                break
        dt = time.perf_counter() - t0
        res["all_cores"] = dict(value=round(passes * L_sum / dt / GIB, 3), unit="GiB/s", cores=threads,
                                sample=f"{passes} passes ({dt:.1f} s, {threads} threads, packets split "
                                       f"contiguously)")
    return res


def _host_threads() -> int:
    """CPUs this process may run on, capped by the job's thread allowance
    (OMP_NUM_THREADS: the GPU box's share of a shared host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap > 0 else n)


def host_path(mi, host: np.ndarray, n: int, L_sum: int, lay: dict, iters: int = 5) -> dict:
    """PCIe-inclusive rate: the batch starts and ends in (page-locked) host
    memory (mi_cksum_ipv4_verify_host).  ``value`` is the zero-copy path (the
    kernel reads the registered host batch in place over PCIe); ``staged`` is
    the chunked H2D -> verify -> D2H path on the same bytes."""
    pinned = True
    try:
        mi.host_register(host)
    except Exception:
        pinned = False

    def rate(staged: bool):
        mi.ipv4_verify_host(host, n, staged=staged, **lay)
        t0 = time.perf_counter()
        for _ in range(iters):
            _, _, st, bad = mi.ipv4_verify_host(host, n, staged=staged, **lay)
        dt = (time.perf_counter() - t0) / iters
        assert bad == 0
        return dt

    dz = rate(False)
    ds = rate(True)
    if pinned:
        mi.host_unregister(host)
    return dict(value=round(L_sum / dz / GIB, 2), unit="GiB/s", mode="zero-copy" if pinned else "staged",
                pinned=pinned, host_buffer_bytes=int(host.nbytes), ms_per_batch=round(dz * 1e3, 3),
                staged=dict(value=round(L_sum / ds / GIB, 2), ms_per_batch=round(ds * 1e3, 3)))


def _cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
