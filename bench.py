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
# <cfg>_split: ONE batch of CONFIGS[cfg]'s packets split into contiguous packet
# ranges over the ranks ("N/G packets per GPU") -- strong
# scaling; the plain uniform configs give every rank its own batch (weak).
SPLIT = {"1500_split": "1500", "9000_split": "9000"}
# tx: the fused TX copy + checksum over 65536 x 1500 B
# socket-layout mbuf chains (mi_cksum_tx_copy)
ALL_CONFIGS = list(CONFIGS) + ["pareto"] + list(SPLIT) + ["tx"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dist", action="store_true",
                    help="initialise torch.distributed (RCCL) even for one rank: rehearses the N>1 path's "
                         "process group, barrier, max-over-ranks and per-GPU all_gather on a one-GPU box "
                         "(launch under torch.distributed.run --nproc-per-node 1)")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--config", default="1500", choices=ALL_CONFIGS)
    ap.add_argument("--rotate", type=int, default=0, help="distinct batches cycled (0: enough for >= 1 GiB)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the (b1) per-call latency leg")
    ap.add_argument("--wait", default="busy", choices=["busy", "auto"],
                    help="busy: completion waits busy-poll (mi_cksum_set_busy_wait, like the reference's polling "
                         "dpdk_rx thread); auto: the HIP runtime's default")
    ap.add_argument("--warm-regions", type=int, default=4,
                    help="the warmup ends with M untimed K-step regions bracketed like the timed one")
    ap.add_argument("--offs64", action="store_true",
                    help="pareto: u64 packet offsets instead of u32 (MI_BATCH_OFFS32, 4 B less per datagram)")
    ap.add_argument("--streams", type=int, default=2, help="streams the steps alternate over")
    ap.add_argument("--submit", default="aql", choices=["graph", "launch", "aql"],
                    help="launch: K host launches from native code; graph: the same K launches as one cached "
                         "hipGraph (measured slower for 1500 B: profiles/submit_r01.jsonl); aql: the same kernels "
                         "as K prebuilt AQL packets in the handle's own HSA queue (MI_REPEAT_ENGINE_AQL)")
    ap.add_argument("--settle", type=float, default=0.3,
                    help="untimed warm-up lasts at least this many seconds (GPU clock settle)")
    ap.add_argument("--also", default="auto",
                    help="comma-separated configs timed in the same run after the main one, each reported as "
                         "config_<name> with its own roofline (auto: 9000,64,pareto when the config is 1500 -- the "
                         "metric names 1500 B and 9000 B frames, BASELINE.json lists the other two; none: off)")
    ap.add_argument("--outputs", default="all", choices=["all", "status"],
                    help="status: store only the per-datagram status byte (an RX drop decision); the default "
                         "stores ip / l4 sums and status (5 B per datagram)")
    ap.add_argument("--sustain-seconds", type=float, default=3.0,
                    help="after the timed region, re-run the same passes back to back this long (reported as "
                         "'sustained', not part of value; 0 = off)")
    a = ap.parse_args()
    if a.also == "auto":
        # the split legs only differ from the weak-scaled ones at N > 1
        world = int(os.environ.get("WORLD_SIZE", "1"))
        a.also = (["9000", "64", "pareto", "tx"] + (list(SPLIT) if world > 1 else [])) if a.config == "1500" else []
    elif a.also == "none":
        a.also = []
    else:
        a.also = [c for c in a.also.split(",") if c]
        for c in a.also:
            if c not in ALL_CONFIGS:
                ap.error(f"--also {c}: unknown config")
    a.also = [c for c in a.also if c != a.config]
    return a


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_workload(mi, synth, shard, config: str, rotate: int, offs64: bool, dev, rank: int, world: int,
                   outputs: str = "all"):
    """The batches of one config on this rank: R rotating device batches,
    device-generated and TX-finalized so every packet verifies."""
    if config == "pareto":
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
                   offsets="u64" if offs64 else "u32")
        stride = first = L = None
    elif config in SPLIT:
        n_total, L, stride, first = CONFIGS[SPLIT[config]]
        lo, hi = shard.shard_uniform(n_total, world, rank)
        n = hi - lo
        lens = offs = None
        L_sum = n * L
        size = first + (n - 1) * stride + L + 64
        workload = (f"one {n_total} x {L} B IPv4/TCP RX verify batch split into contiguous packet ranges over "
                    f"{world} GPU(s) (slot stride {stride}, IP at +{first})")
        scaling = "strong"
        cfg = dict(workload=workload, packets_total=n_total, packets_this_rank=n, first_packet=lo,
                   ip_datagram_len=L, slot_stride=stride, ip_offset=first)
    else:
        n, L, stride, first = CONFIGS[config]
        lens = offs = None
        L_sum = n * L
        size = first + (n - 1) * stride + L + 64
        workload = f"{n} x {L} B IPv4/TCP RX verify per GPU (slot stride {stride}, IP at +{first})"
        scaling = "weak"
        cfg = dict(workload=workload, packets_per_gpu=n, ip_datagram_len=L, slot_stride=stride, ip_offset=first)
    size = (size + 255) & ~255
    # Rotate R distinct batches so that >= 2 GiB of other batches is read between
    # two reads of the same one: the 256 MiB Infinity Cache then keeps nothing of
    # a batch (profiles/ceiling_r02.jsonl: at 0.7 GB between reuses 1500 B
    # verify read ~1.5 % faster than at 2.3 GB).
    read_per_batch = min(size, L_sum + 16 * n)
    R = rotate or 1 + -(-(2 << 30) // read_per_batch)
    cfg.update(rotating_batches=R, footprint_MiB=round(R * size / 2**20, 1),
               read_between_reuse_MB=round((R - 1) * read_per_batch / 1e6),
               parallelism=f"dp{world} (independent packet shards, no collective)")
    batches, outs = [], []
    for r in range(R):
        buf = torch.empty(size, dtype=torch.uint8, device=dev)
        if lens is None:
            b = mi.PktBatch(buf, n, stride=stride, first_off=first, fixed_len=L)
        else:
            b = mi.PktBatch(buf, n, offs=torch.from_numpy(offs.astype(np.int64)).to(dev),
                            lens=torch.from_numpy(lens.astype(np.int32)).to(dev), max_len=int(lens.max()),
                            packed=True, offs32=not offs64)
        mi.synth_ipv4(b, seed=0x5EED5EED + 7919 * r + 104729 * rank)
        mi.ipv4_finalize(b)  # TX path makes every packet valid
        batches.append(b)
        if outputs == "status":  # the RX drop decision alone (ip / l4 sums not stored)
            outs.append(dict(status=torch.empty(n, dtype=torch.uint8, device=dev)))
        else:
            outs.append(dict(ip=torch.empty(n, dtype=torch.uint16, device=dev),
                             l4=torch.empty(n, dtype=torch.uint16, device=dev),
                             status=torch.empty(n, dtype=torch.uint8, device=dev)))
    torch.cuda.synchronize()
    chk = mi.ipv4_verify(batches[0], bad_count=True)  # sanity: everything verifies
    torch.cuda.synchronize()
    if int(chk["bad"].item()) != 0:
        raise SystemExit(f"rank {rank}: synthetic batch does not verify ({int(chk['bad'].item())} bad)")
    lay = (dict(stride=stride, first_off=first, fixed_len=L) if lens is None else dict(offs=offs, lens=lens))
    if outputs == "status":
        cfg["outputs"] = "status byte only (the RX drop decision; ip / l4 sums not stored)"
    return dict(batches=batches, outs=outs, n=n, L_sum=L_sum, cfg=cfg, scaling=scaling, lay=lay,
                out_bytes=1 if outputs == "status" else 5)


POISON = {"ip": -1, "l4": -1, "status": 0xFF}  # no verdict of a verify pass: status bits are 1/2/4/8


def repeat_plan(b) -> str:
    """The verify kernel the prepared submission runs for batch b (the
    dealt-unit kernel where it applies, mi__repeat_plan)."""
    import ctypes as C
    import libunsod_amd as mi
    f = mi.load().mi__repeat_plan
    f.restype = C.c_char_p
    f.argtypes = [C.c_void_p]
    return f(C.byref(b.c)).decode()


def poison_outputs(outs) -> None:
    for o in outs:
        for k, t in o.items():
            t.fill_(POISON[k])
    torch.cuda.synchronize()


def check_timed_outputs(outs, K: int) -> dict:
    """After the timed region: the K passes went to K distinct rotating batches
    (or all R of them when K >= R); each such batch's outputs must be the
    verdicts of valid datagrams (ip = l4 = status = 0 everywhere: the batches
    are TX-finalized), every other batch must still hold the poison.  Raises if
    not -- a line whose timed passes did not verify every datagram is never
    printed."""
    written = untouched = 0
    for o in outs:
        st = o["status"]
        if bool((st == 0).all()) and all(bool((o[k] == 0).all()) for k in ("ip", "l4") if k in o):
            written += 1
        elif bool((st == 0xFF).all()):
            untouched += 1
        else:
            raise SystemExit("timed outputs: a batch is partly written or holds a failed verdict")
    if written != min(K, len(outs)) or written + untouched != len(outs):
        raise SystemExit(f"timed outputs: {written} batches written by {K} passes over {len(outs)}")
    return dict(checked=True, batches_written=written, batches_rotating=len(outs),
                datagrams_checked=written * int(outs[0]["status"].numel()),
                rule="outputs poisoned before the region; after it every batch the K passes covered holds "
                     "ip = l4 = status = 0 for every datagram (read back untimed), the rest the poison")


def measure(mi, shard, wl: dict, args, K: int, dev, dist, backend: str, sustain_s: float = 0.0) -> dict:
    """Warm up, then time exactly K verify passes over the rotating batches,
    bracketed by a barrier + torch.cuda.synchronize() on both sides, max over
    ranks.  Returns the config's value / ms_per_step / roofline (+ extras)."""
    batches, outs, n, L_sum, cfg = wl["batches"], wl["outs"], wl["n"], wl["L_sum"], wl["cfg"]
    # The K passes are submitted by a prepared handle (mi_cksum_repeat_*: the
    # descriptors, kernel plans, streams and events are resolved once, as an RX
    # queue loop re-submitting its rings would), alternating over `nst`
    # non-blocking streams so a launch's ramp-up overlaps its predecessor's drain.
    nst = max(1, args.streams)
    use_graph = args.submit == "graph"
    # Default: the AQL engine -- the same kernels as prebuilt AQL packets in
    # the handle's own HSA queues (one per stream), so a 20-step region pays
    # ~1 us of submission instead of ~50-80 us of HIP launches and its wait
    # ends ~10 us sooner (profiles/aql_r02.jsonl: 5941-6027 vs 5429-5674 GiB/s
    # by wall clock, same GPU span per pass).
    rep, engine_note = None, None
    if not use_graph:
        try:
            rep = mi.VerifyRepeat(batches, outs, nstreams=nst, engine="aql" if args.submit == "aql" else "hip")
        except mi.MiCksumError as e:  # the same kernels through HIP launches
            engine_note = f"AQL engine unavailable ({e}); HIP launches"
            rep = mi.VerifyRepeat(batches, outs, nstreams=nst)

    def run(k: int, timed: bool = False):
        if rep is not None:
            rep.run(k, timed=timed)
            return rep.span() if timed else None
        # (the graph path takes at most 16 batches)
        return mi.ipv4_verify_repeat(batches[:16], outs[:16], k, nstreams=nst,
                                     timing="region" if timed else "none", graph=True)

    tw = time.perf_counter()
    if args.warmup:  # timed like the region, so its events are warm too
        run(args.warmup, timed=True)
    torch.cuda.synchronize()
    # Settle: the first ~0.1 s of back-to-back launches run up to 20 % slower
    # (clock / translation warm-up; profiles/warmup_r01.jsonl: 40 warmup steps ->
    # 17.0 us per launch, 2000 -> 14.25 us).  Keep launching untimed steps until
    # the warmup phase has lasted `--settle` seconds, whatever W is.
    settle_steps = 0
    while time.perf_counter() - tw < args.settle:
        run(500, timed=True)
        settle_steps += 500
    cfg = dict(cfg)
    cfg["streams"] = nst
    cfg["settle_steps"] = settle_steps
    cfg["submit"] = ("graph" if use_graph else engine_note if engine_note else
                     f"prepared handle, AQL packets ({nst} own HSA queues)" if args.submit == "aql"
                     else "prepared handle, host launches")
    cfg["wait"] = args.wait
    if use_graph:  # instantiate the timed region's graph (K passes) before timing it
        run(K)

    # The warmup ends with M untimed regions of K steps, bracketed exactly like
    # the timed one: the first region after the settle loop pays ~70-130 us of
    # host-side wake-up (its GPU span is the same; profiles/bench_regions_r02.jsonl).
    # Their (wall, span) in us go to the JSON line.
    warm_walls = []
    for _ in range(args.warm_regions):
        torch.cuda.synchronize()
        ta = time.perf_counter()
        if rep is not None:
            rep.run(K, timed=True)
        else:
            run(K, timed=True)
        torch.cuda.synchronize()
        w = round((time.perf_counter() - ta) * 1e6, 1)
        warm_walls.append((w, round(rep.span(), 1)) if rep is not None else w)

    # Poison every rotating batch's outputs (untimed): after the region, the
    # batches its K passes covered must hold the verdicts of valid datagrams
    # (all zero) and the others the poison -- proof that the timed passes did
    # the work (check_timed_outputs).
    poison_outputs(outs)

    # ------------------------------------------------------- timed region
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if rep is not None:
        rep.run(K, timed=True)  # submission + completion events + wait
    else:
        span_us = run(K, timed=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    trace = None
    if rep is not None:
        span_us = rep.span()  # elapsed-time queries after the region
        if os.environ.get("MI_CKSUM_REPEAT_TRACE"):
            import ctypes as C
            tt = (C.c_double * 8)()
            mi.load().mi__repeat_trace(rep._h, tt, 8)
            trace = dict(zip(["entry", "ordered", "first_launch", "last_launch", "markers", "waited"],
                             [round((tt[k] - t0) * 1e6, 1) for k in range(6)]))
            trace["t1"] = round((t1 - t0) * 1e6, 1)
    if dist:
        dist.barrier()
    checked = check_timed_outputs(outs, K)
    my_bytes = float(L_sum) * K
    elapsed, job_bytes, job_pkts = shard.job_totals(t1 - t0, my_bytes, float(n) * K,
                                                    device=dev if dist and backend == "nccl" else None)
    value = job_bytes / elapsed / GIB

    # Roofline of the dominant kernel (k_ipv4_verify*, the one verify_plan names).  Algorithmic bytes per
    # launch = sum(L) read + 5 B written per packet (ip u16, l4 u16, status u8).
    # Average launch duration = GPU span of the timed region (dispatch
    # timestamps of the handle's queues) / K: passes on different queues
    # overlap, so this is the GPU time each launch costs; rocprof's union of
    # dispatch intervals / K is the same quantity (tools/prof_summary.py).
    gpu_s_per_launch = span_us / K / 1e6
    alg_bytes = float(L_sum) + float(wl.get("out_bytes", 5)) * n
    achieved = alg_bytes / gpu_s_per_launch / 1e9
    config = wl.get("name", args.config)
    traffic, tsrc = None, None
    # HBM bytes per launch from the newest PMC record of this config (request-
    # size counters, rounds 3-5; FETCH_SIZE x2, round 2), labelled with its source
    tkey = config + ("_u64" if args.offs64 else "_u32") if config == "pareto" else config
    for rel in ("profiles/r06/pmc_traffic_r06.json", "profiles/r05/pmc_traffic_r05.json", "profiles/r04/pmc_traffic_r04.json",
                "profiles/r03/pmc_traffic_r03.json",
                "profiles/pmc_traffic_r02.json"):
        tfile = os.path.join(ROOT, rel)
        try:
            ent = json.load(open(tfile)).get(tkey) if os.path.exists(tfile) else None
        except Exception:
            ent = None
        if ent:
            traffic = ent["bytes_per_launch"]
            tsrc = f"{rel}[{tkey}] (rocprofv3 --pmc, separate passes; not this run)"
            break
    roof = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic, traffic_source=tsrc,
                kernel=repeat_plan(batches[0]) + (" (its AQL entry point mi_aql_*)" if rep is not None and
                                                  getattr(rep, "engine", "hip") == "aql" else ""),
                alg_bytes_per_launch=int(alg_bytes),
                avg_launch_us=round(gpu_s_per_launch * 1e6, 2), streams=nst,
                wall_frac=round(alg_bytes * K / (t1 - t0) / 1e9 / HBM_PEAK_GBS, 4))
    # the same kernel alone on one stream, every launch bracketed by events
    # (compare with a single-stream rocprof trace)
    iso_us, _ = mi.ipv4_verify_repeat(batches[:16], outs[:16], min(K, 100), nstreams=1, timing="pass")
    roof["isolated_launch_us"] = round(float(np.median(iso_us)), 2)
    roof["isolated_achieved"] = round(alg_bytes / (float(np.median(iso_us)) / 1e6) / 1e9, 1)
    out = dict(value=round(value, 2), ms_per_step=round(elapsed / K * 1e3, 5), config=cfg,
               mpkt_per_s=round(job_pkts / elapsed / 1e6, 2), roofline=roof, my_bytes=my_bytes,
               my_elapsed=t1 - t0, job_pkts=job_pkts, elapsed=elapsed, timed_outputs=checked)
    if warm_walls:
        out["warm_region_walls_us"] = warm_walls
    if trace:
        out["host_trace_us"] = trace
    if sustain_s > 0 and rep is not None:
        # A sustained leg after the timed region (not part of `value`): the same
        # handle re-run back to back for ~sustain_s seconds, so the GPU is busy
        # long enough for an outside sampler to see it; its wall-clock rate
        # corroborates the short region's.
        torch.cuda.synchronize()
        ts, passes, chunk = time.perf_counter(), 0, 2000
        while time.perf_counter() - ts < sustain_s:
            rep.run(chunk)
            passes += chunk
        torch.cuda.synchronize()
        dts = time.perf_counter() - ts
        out["sustained"] = dict(value=round(passes * L_sum / dts / GIB, 2), unit="GiB/s", passes=passes,
                                seconds=round(dts, 2),
                                frac_by_wall=round(passes * alg_bytes / dts / 1e9 / HBM_PEAK_GBS, 4),
                                note="this rank, the same handle back to back after the timed region")
    if rep is not None:
        rep.close()
    return out


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
    if world > 1 or args.dist:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import libunsod_amd as mi
    from libunsod_amd import shard, synth
    if args.wait == "busy":
        mi.set_busy_wait(True)

    if args.config == "tx":  # the TX leg alone (its rocprof / PMC passes)
        row = tx_leg(mi, synth, shard, args, args.steps, dev, dist, backend, rank, world)
        row.pop("_mm")
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": row["value"], "unit": "GiB/s", "n_gpus": world,
                              "steps": args.steps, "warmup": args.warmup, "ms_per_step": row["ms_per_step"],
                              "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
                              "data": "synthetic TX socket chains", "config": {"workload": row["workload"]},
                              "roofline": row["roofline"], "config_tx": row}), flush=True)
        if dist:
            dist.destroy_process_group()
        return
    wl = build_workload(mi, synth, shard, args.config, args.rotate, args.offs64, dev, rank, world, args.outputs)
    wl["name"] = args.config
    K = args.steps
    m = measure(mi, shard, wl, args, K, dev, dist, backend, sustain_s=args.sustain_seconds)
    result = {
        "metric": METRIC, "value": m["value"], "unit": "GiB/s", "n_gpus": world, "steps": K,
        "warmup": args.warmup, "ms_per_step": m["ms_per_step"], "higher_is_better": True,
        "scaling": wl["scaling"], "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: device-generated IPv4/TCP datagrams (splitmix64 payload), TX-finalized to valid sums",
        "config": m["config"], "mpkt_per_s": m["mpkt_per_s"], "roofline": m["roofline"],
    }
    result["timed_outputs_checked"] = m["timed_outputs"]["checked"]
    for k in ("warm_region_walls_us", "host_trace_us", "sustained", "timed_outputs"):
        if k in m:
            result[k] = m[k]

    def per_config_extras(dst: dict, cfg_name: str, mm: dict) -> None:
        if cfg_name == "64":
            # every 46 B datagram is one 64 B minimum Ethernet frame (14 B header +
            # 46 B + 4 B FCS): the frame-equivalent rate SURVEY.md 8(d) asks for
            dst["frame64_equiv_gibs"] = round(mm["job_pkts"] * 64 / mm["elapsed"] / GIB, 2)
        if dist:
            # per-GPU rates (SURVEY.md 8(e) "Reporting"): timing bookkeeping only
            mine = torch.tensor([mm["my_bytes"], mm["my_elapsed"]], dtype=torch.float64,
                                device=dev if backend == "nccl" else None)
            allr = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(allr, mine)
            dst["per_gpu"] = [round(float(x[0]) / float(x[1]) / GIB, 2) for x in allr]

    per_config_extras(result, args.config, m)

    # -------------------------------------------- CPU baseline + host path
    host = None
    if world == 1 and rank == 0:
        host = wl["batches"][0].buf.cpu().numpy()
    n, L_sum, lay = wl["n"], wl["L_sum"], wl["lay"]
    del wl, m
    torch.cuda.synchronize()
    torch.cuda.empty_cache()

    # The metric names 1500 B AND 9000 B frames, and BASELINE.json lists 64 B
    # minimum frames and the mixed-length Pareto batch: each is timed in the
    # same run, same K / W / submission, same output check, and reported
    # beside the headline with its own roofline.
    for also in args.also:
        if also == "tx":
            row = tx_leg(mi, synth, shard, args, K, dev, dist, backend, rank, world)
            per_config_extras(row, "tx", row.pop("_mm"))
            result["config_tx"] = row
            result["timed_outputs_checked"] = result["timed_outputs_checked"] and result["config_tx"]["timed_outputs_checked"]
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            continue
        wl2 = build_workload(mi, synth, shard, also, 0, args.offs64, dev, rank, world, args.outputs)
        wl2["name"] = also
        m2 = measure(mi, shard, wl2, args, K, dev, dist, backend)
        row = dict(value=m2["value"], unit="GiB/s", ms_per_step=m2["ms_per_step"],
                   mpkt_per_s=m2["mpkt_per_s"], scaling=wl2["scaling"], workload=m2["config"]["workload"],
                   rotating_batches=m2["config"]["rotating_batches"], roofline=m2["roofline"],
                   timed_outputs_checked=m2["timed_outputs"]["checked"],
                   datagrams_checked=m2["timed_outputs"]["datagrams_checked"])
        per_config_extras(row, also, m2)
        result[f"config_{also}"] = row
        result["timed_outputs_checked"] = result["timed_outputs_checked"] and m2["timed_outputs"]["checked"]
        del wl2, m2
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    if host is not None:
        if args.cpu_seconds > 0:
            result["cpu_baseline"] = cpu_baseline(host, n, L_sum, lay, args.cpu_seconds)
            result["cpu_baseline"]["plumbing_64k"] = plumbing_64k()
        if not args.no_host_path:
            result["pcie_inclusive"] = host_path(mi, host, n, L_sum, lay)
        if not args.no_dropin:
            result["dropin_latency"] = dropin_latency(mi)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def tx_leg(mi, synth, shard, args, K: int, dev, dist, backend: str, rank: int, world: int) -> dict:
    """config_tx: the fused TX copy + checksum (mi_cksum_tx_copy; SURVEY.md 8(f)
    rank 2: uinet_if_dpdk.c:590-606 m_copydata into the rte_mbuf + ip_output.c:
    649-672 / in_delayed_cksum :958-983) over 65536 x 1500 B IPv4/TCP frames whose
    chains have the socket layout tcp_output builds (a header mbuf + payload
    pieces in 2 KiB socket-buffer clusters, synth.build_tx_chains), copied into
    2176 B rte_mbuf slots (data at +128).  A step = one launch over one batch,
    submitted like the RX legs' (a prepared handle, mi_cksum_tx_repeat_create;
    AQL packets over two queues by default).  Same bracket as the RX legs: barrier + synchronize,
    K launches, synchronize, max over ranks; outputs poisoned before and checked
    after (every covered batch's status 0 and its slots verifying clean under the
    RX kernel).  Weak-scaled: every rank copies its own batch."""
    n, L, stride, dst_first, l3 = 65536, 1500, 2176, 128, 14
    frame = L + l3
    d = synth.build_tx_chains(n, L, layout="socket", seed=0x7E57 + rank, l3_off=l3)
    dst_bytes = dst_first + n * stride + 64
    per = d["src"].nbytes + dst_bytes
    R = 1 + -(-(2 << 30) // (2 * n * frame))  # >= 2 GiB of other batches between reuses
    src_host = torch.from_numpy(d["src"])
    batches = []
    for _ in range(R):
        src = src_host.to(dev)
        dst = torch.zeros(dst_bytes, dtype=torch.uint8, device=dev)
        tb = mi.TxBatch(src, d["seg_off"], d["seg_len"], d["pkt_seg"], d["pkt_len"], dst, dst_stride=stride,
                        dst_first=dst_first, room=stride - dst_first, l3_off=l3, max_len=frame)
        batches.append((tb, torch.empty(n, dtype=torch.uint8, device=dev)))
    torch.cuda.synchronize()  # (the AQL engine does not order itself after torch's streams)
    nst = max(1, args.streams)
    # The K launches go out through a prepared TX handle (mi_cksum_tx_repeat_*),
    # by default as prebuilt AQL packets of the default TX kernel in the
    # handle's own HSA queues -- the RX legs' submission; --submit launch: HIP
    # launches alternating over the handle's streams.
    engine_note = None
    try:
        rep = mi.TxRepeat([b for b, _ in batches], [st for _, st in batches], nstreams=nst,
                          engine="aql" if args.submit == "aql" else "hip")
    except mi.MiCksumError as e:
        engine_note = f"AQL engine unavailable ({e}); HIP launches"
        rep = mi.TxRepeat([b for b, _ in batches], [st for _, st in batches], nstreams=nst)

    def run(k: int, timed: bool = False):
        rep.run(k, timed=timed)

    def verify_slots(tb) -> int:
        """Frames of tb's slots that do NOT verify under the RX kernel."""
        pb = mi.PktBatch(tb.dst, n, stride=stride, first_off=dst_first + l3, fixed_len=L)
        r = mi.ipv4_verify(pb, bad_count=True)
        torch.cuda.synchronize()
        return int(r["bad"].item())

    run(2)
    torch.cuda.synchronize()
    if verify_slots(batches[0][0]) or bool((batches[0][1] != 0).any()):
        raise SystemExit(f"rank {rank}: TX copy output does not verify")
    tw = time.perf_counter()
    run(max(args.warmup, 1), timed=True)
    while time.perf_counter() - tw < args.settle:
        run(50, timed=True)
    for _ in range(args.warm_regions):  # bracketed like the timed region
        torch.cuda.synchronize()
        run(K, timed=True)
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    for tb, st in batches:  # poison: covered batches must come back copied + summed
        tb.dst.zero_()
        st.fill_(0xFF)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(K, timed=True)  # submission + completion + wait
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    span_us = rep.span()  # GPU span of the K passes (dispatch timestamps / events), read after the region
    rep.close()
    covered = min(K, R)
    bad_frames = sum(verify_slots(batches[j][0]) for j in range(covered))
    st_ok = all(bool((batches[j][1] == 0).all()) for j in range(covered))
    untouched = all(bool((batches[j][1] == 0xFF).all()) for j in range(covered, R))
    checked = bad_frames == 0 and st_ok and untouched
    if not checked:
        raise SystemExit(f"rank {rank}: timed TX outputs: {bad_frames} frames do not verify, status ok {st_ok}")
    my_bytes = float(n) * L * K
    elapsed, job_bytes, job_pkts = shard.job_totals(t1 - t0, my_bytes, float(n) * K,
                                                    device=dev if dist and backend == "nccl" else None)
    alg = float(n) * (2 * frame + 1)  # frame read + frame written + 1 B status
    us = span_us / K
    import ctypes as C
    kname = mi.load().mi__tx_kernel_name
    kname.restype = C.c_char_p
    roof = dict(bound="hbm", achieved=round(alg / us / 1e3, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                frac=round(alg / us / 1e3 / HBM_PEAK_GBS, 4), traffic=None,
                kernel=kname().decode() + " (mi_cksum_tx_copy)",
                alg_bytes_per_launch=int(alg), avg_launch_us=round(us, 2), streams=nst,
                wall_frac=round(alg * K / (t1 - t0) / 1e9 / HBM_PEAK_GBS, 4))
    if rep.engine == "aql" and engine_note is None:
        roof["kernel"] = kname().decode() + " (its AQL entry point mi_aql_tx_lds)"
    tf = os.path.join(ROOT, "profiles", "r06", "pmc_traffic_r06.json")
    try:
        ent = json.load(open(tf)).get("tx") if os.path.exists(tf) else None
    except Exception:
        ent = None
    if ent:
        roof["traffic"] = ent["bytes_per_launch"]
        roof["traffic_source"] = "profiles/r06/pmc_traffic_r06.json[tx] (rocprofv3 --pmc, separate passes; not this run)"
    return dict(value=round(job_bytes / elapsed / GIB, 2), unit="GiB/s", ms_per_step=round(elapsed / K * 1e3, 5),
                mpkt_per_s=round(job_pkts / elapsed / 1e6, 2), scaling="weak",
                frames_copied_gibs=round(job_pkts * frame / elapsed / GIB, 2),
                workload=(f"{n} x {frame} B frames (IPv4/TCP, {L} B datagrams), socket-layout mbuf chains "
                          f"({round(len(d['seg_len']) / n, 2)} mbufs per frame) -> 2176 B rte_mbuf slots, "
                          "copy + ip_sum + th_sum fused; value = IP datagram bytes checksummed"),
                rotating_batches=R, footprint_MiB=round(R * per / 2**20, 1), roofline=roof,
                timed_outputs_checked=checked, frames_checked=covered * n,
                submit=engine_note or (f"prepared TX handle, AQL packets ({nst} own HSA queues)" if rep.engine == "aql"
                                       else f"prepared TX handle, HIP launches over {nst} streams"),
                _mm=dict(my_bytes=my_bytes, my_elapsed=t1 - t0, job_pkts=job_pkts, elapsed=elapsed))


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


def plumbing_64k(seconds: float = 1.0) -> dict:
    """BASELINE configs[0]: one 64 KiB TCP segment through the reference's
    in_cksum_skip(m, 65536, 0) on the host CPU (a one-mbuf chain, KAT7
    pattern; oracle/_ref = the reference's own in_cksum.c), 1 thread, timed in
    C (batch_driver.c skip_repeat) so no Python sits in the loop."""
    from oracle.pyoracle import Oracle, available
    kind = "reference" if available("reference") else "port"
    o = Oracle(kind)
    raw = np.zeros(65536 + 128, np.uint8)
    s = (-raw.ctypes.data) % 64
    buf = raw[s:s + 65536]
    buf[:] = np.arange(65536, dtype=np.uint32).astype(np.uint8)
    assert o.skip_repeat(buf, 65536, 1) == 0x3FC0  # SURVEY KAT7, len 65536
    iters, dt = 256, 0.0
    while dt < seconds / 4:
        t0 = time.perf_counter()
        o.skip_repeat(buf, 65536, iters)
        dt = time.perf_counter() - t0
        iters *= 2
    iters //= 2
    t0 = time.perf_counter()
    n_calls = 0
    while time.perf_counter() - t0 < seconds:
        o.skip_repeat(buf, 65536, iters)
        n_calls += iters
    dt = time.perf_counter() - t0
    return dict(value=round(n_calls * 65536 / dt / GIB, 3), unit="GiB/s", us_per_call=round(dt / n_calls * 1e6, 3),
                cores=1, kind=kind, sample=f"{n_calls} x in_cksum_skip(m, 65536, 0), one L2-resident 64 KiB "
                                           f"mbuf, {dt:.2f} s")


def dropin_latency(mi, calls: int = 400) -> dict:
    """(b1) drop-in cost per call on this host: libmicksum's in_cksum_hdr /
    in_cksum_pseudo_header / in_cksum_skip on real mbuf chains -- in the
    library's default mode (``dropin_us``: MI_DROPIN_HOST, the host fold on the
    calling core) and in its GPU mode (the bytes read over PCIe from pinned
    staging; one AQL dispatch per call, and through the device's resident
    drop-in service) -- against the reference's own functions (oracle/_ref) on
    the same chains.  Median over `calls` calls through ctypes;
    ``ctypes_floor_us`` is the same loop around in_addword (no checksum work)
    and is included in every figure."""
    import ctypes as C
    from oracle.pyoracle import Oracle, available
    lib = mi.load()
    pat = bytes(i & 0xFF for i in range(65536))
    m64 = mi.MbufChain([pat])
    ip_hdr = bytes.fromhex("450005dc0000400040060000c0a80101c0a80102")
    m1500 = mi.MbufChain([ip_hdr + pat[:1480]])
    hraw = np.zeros(256, np.uint8)
    hoff = 64 + ((2 - (hraw.ctypes.data + 64)) % 64)  # address == 2 mod 4, as behind a 14 B Ethernet header
    hraw[hoff:hoff + 20] = np.frombuffer(ip_hdr, np.uint8)
    haddr = hraw.ctypes.data + hoff
    src, dst = 0x0101A8C0, 0x0201A8C0  # as loaded (little-endian) from the header
    cases = {
        "in_cksum_hdr_20B": ("in_cksum_hdr", (C.c_void_p(haddr),)),
        "in_cksum_pseudo_header_1480B": ("in_cksum_pseudo_header", (C.c_void_p(m1500.ptr), 1480, 20, src, dst, 6)),
        "in_cksum_skip_65536B": ("in_cksum_skip", (C.c_void_p(m64.ptr), 65536, 0)),
    }

    def med(f, args):
        f(*args)
        ts = []
        for _ in range(calls):
            t0 = time.perf_counter()
            f(*args)
            ts.append(time.perf_counter() - t0)
        return round(float(np.median(ts)) * 1e6, 3)

    # (the library keeps the drop-in service out of the way for 0.5 ms after
    # a batch submission -- DESIGN.md 5.6 -- so these start well after one)
    time.sleep(0.01)
    out = dict(unit="us per call (median)", calls=calls,
               ctypes_floor_us=med(lib.in_addword, (1, 2)))
    ref = None
    if available("reference"):
        ref = Oracle("reference").lib
        ref.ref_in_cksum_hdr.restype = C.c_uint
        ref.ref_in_cksum_hdr.argtypes = [C.c_void_p]
        ref.ref_in_cksum_skip.restype = C.c_ushort
        ref.ref_in_cksum_skip.argtypes = [C.c_void_p, C.c_int, C.c_int]
        ref.ref_in_cksum_pseudo_header.restype = C.c_uint16
        ref.ref_in_cksum_pseudo_header.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_uint32, C.c_uint32,
                                                   C.c_uint8]
    lib.mi__set_dropin_service.restype = C.c_int
    lib.mi__set_dropin_service.argtypes = [C.c_int]
    svc_default = lib.mi__set_dropin_service(0)  # (returns the setting it replaces)
    lib.mi__set_dropin_service(svc_default)
    mode_default = mi.set_dropin_mode("host")
    mi.set_dropin_mode(mode_default)
    out["default_mode"] = mode_default + ("" if mode_default == "host" else
                                          " (service)" if svc_default else " (dispatch)")
    degraded0 = mi.dropin_degraded()

    for name, (fn, args) in cases.items():
        g = getattr(lib, fn)
        mi.set_dropin_mode("host")
        row = dict(dropin_us=None, host_fold_us=med(g, args))
        want = int(g(*args))
        mi.set_dropin_mode("gpu")
        for mode, on in (("dispatch", 0), ("service", 1)):
            lib.mi__set_dropin_service(on)
            row[f"gpu_{mode}_us"] = med(g, args)
            assert int(g(*args)) == want, f"{fn}: GPU drop-in ({mode}) differs from the host fold"
        lib.mi__set_dropin_service(svc_default)
        mi.set_dropin_mode(mode_default)
        row["dropin_us"] = med(g, args)
        if ref is not None:
            r = getattr(ref, "ref_" + fn)
            assert want == int(r(*args)), f"{fn}: drop-in differs from the reference"
            row["reference_cpu_us"] = med(r, args)
        out[name] = row
    out["gpu_calls_degraded_to_host"] = mi.dropin_degraded() - degraded0
    return out


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
