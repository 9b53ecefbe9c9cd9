#!/usr/bin/env python3
"""bench.py -- encoded symbols/s at vocab=32000, 4096 streams per GPU (BASELINE.json c3).

One bench step = one whole compression job over inputs already resident in HBM:
reset every stream, encode ``--tokens`` symbols per stream (integer pmf rows
[tokens, streams, V] + symbols), flush and pack the bitstreams; with N > 1 ranks
the job also gathers every rank's bitstreams over RCCL (the path's one exchange
step).  Streams are sharded (each rank owns its own 4096), so scaling is weak.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

After the timed region (never inside it): per-stream status, a full GPU decode
round trip, and bit-exact parity of the packed bytes against the CPU oracle
(oracle/, the C restatement pinned to the reference); the oracle's own time on
the same tables is the cpu_baseline.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "encoded symbols/sec at vocab=32000, batch=4096 streams; bit-exact round-trip"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def read_traffic(cfg, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary, if it matches."""
    p = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    keys = ("vocab", "streams", "tokens", "pmf_bits", "input")
    for e in d.get("entries", []):
        if all(e.get(k) == cfg.get(k) for k in keys):
            return e.get("bytes_per_launch", {}).get(kernel)
    return None


def host_cores():
    """CPU threads for the cpu_baseline leg, as `nproc` counts them: the CPUs this
    process may run on (sched_getaffinity), limited by OMP_NUM_THREADS /
    OMP_THREAD_LIMIT when set (the GPU box sets them to its CPU share per GPU)."""
    n = len(os.sched_getaffinity(0))
    for var in ("OMP_NUM_THREADS", "OMP_THREAD_LIMIT"):
        try:
            v = int(os.environ.get(var, "").split(",")[0])
        except ValueError:
            continue
        if v > 0:
            n = min(n, v)
    return max(1, n)


def workload_name(V, B, world):
    """The BASELINE.json config a run measures."""
    if V == 32000 and B == 1 and world == 1:
        return "c2"
    if V == 32000 and B == 4096:
        return "c3" if world == 1 else f"c3 weak-scaled over {world} GPUs"
    if V == 128256 and B == 4096:
        return "c4" if world == 1 else ("c5" if world == 8 else f"c5 shape on {world} GPUs ({world}x4096 streams)")
    return "custom"


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=10)   # ~12 ms of encodes before the timed 40 (clocks settled)
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--streams", type=int, default=4096, help="streams per GPU")
    ap.add_argument("--tokens", type=int, default=16, help="symbols per stream per job")
    ap.add_argument("--prec", type=int, default=48)
    ap.add_argument("--pmf-bits", type=int, default=32, choices=(32, 64))
    ap.add_argument("--scale-bits", type=int, default=0,
                    help="pmf = max(1 or 2, floor(softmax * 2^k)); 0 = 31 for u32, 60 (llama-scale) for u64")
    ap.add_argument("--cpu-baseline", default="on", choices=("on", "off"))
    ap.add_argument("--cpu-threads", type=int, default=0, help="cpu_baseline threads (0 = nproc: host_cores())")
    ap.add_argument("--decode-reps", type=int, default=10,
                    help="timed decode passes, back to back, after two warm ones (the first passes after "
                         "the encode jobs run slower: profiles/r05/q1dec_pf/)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="minimum CPU-baseline sample time")
    ap.add_argument("--cpu-streams", type=int, default=0, help="oracle sample streams (0 = all)")
    ap.add_argument("--path", default="auto", choices=("auto", "split", "fused"), help="encode kernel path")
    ap.add_argument("--q1-shape", type=int, default=0, help="logits row-stats block shape (tuning)")
    ap.add_argument("--decode-path", default="auto", choices=("auto", "split", "fused", "fused_chunk", "stats", "block"))
    ap.add_argument("--block-waves", type=int, default=0, help="block decode path: waves per stream (tuning)")
    ap.add_argument("--gather", action="store_true",
                    help="run the bitstream gather (lac_amd.dist.BitstreamGatherer) even on one rank: a "
                         "one-rank RCCL group, the gather inside the timed region, parity.gather_ok")
    ap.add_argument("--gather-batch", type=int, default=8, help="jobs per bitstream exchange (the gatherer's batch)")
    ap.add_argument("--save-inputs", default=None, metavar="PREFIX",
                    help="write this rank's synthetic inputs to PREFIX.r<rank>.{pmf,sym}.npy and go on")
    ap.add_argument("--load-inputs", default=None, metavar="PREFIX",
                    help="read the inputs --save-inputs wrote instead of generating them: the same workload "
                         "bit for bit with no torch RNG kernel in this process (profiled runs: torch.randn's "
                         "launches crashed the host under rocprofv3 --pmc, profiles/r06/pmc_rng/)")
    ap.add_argument("--input", default="pmf", choices=("pmf", "logits-bf16", "logits-f32"),
                    help="pmf rows (BASELINE c3, default) or raw logits quantised in-kernel (q1, SURVEY §8(f)1)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher around us: start one rank per GPU (torch.distributed.run as a child
        # process, before any GPU call here) and relay rank 0's line
        import torch
        from lac_amd import launch
        try:
            launch.check_devices(args.gpus, os.environ.get("LAC_DIST_BACKEND", "nccl"), torch.cuda.device_count())
        except launch.LaunchError as e:
            log(f"bench.py: {e}")
            sys.exit(2)
        sys.exit(launch.relay(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    if "WORLD_SIZE" in os.environ and args.gpus != int(os.environ["WORLD_SIZE"]) and args.gpus != 1:
        log(f"bench.py: --gpus {args.gpus} but the launcher started {os.environ['WORLD_SIZE']} ranks")
        sys.exit(2)

    import ctypes as C

    import numpy as np
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; LAC_DIST_BACKEND=gloo + ranks sharing a GPU only for rehearsing the
    # multi-rank path on a one-GPU box (the driver's runs use nccl = RCCL, one GPU each)
    backend = os.environ.get("LAC_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local = local % ndev if backend != "nccl" and ndev else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    elif args.gather:                                      # a one-rank group: no launcher, no rendezvous
        import torch.distributed as dist
        dist.init_process_group(backend, store=dist.HashStore(), rank=0, world_size=1,
                                **({"device_id": dev} if backend == "nccl" else {}))

    from lac_amd import synth
    from lac_amd.batch import BatchCoder
    from lac_amd.dist import BitstreamGatherer

    V, B, T, P = args.vocab, args.streams, args.tokens, args.prec
    logits_in = args.input != "pmf"
    ebytes = args.pmf_bits // 8 if not logits_in else (2 if args.input == "logits-bf16" else 4)
    t_gen = time.time()
    coder = BatchCoder(V, B, prec=P, pmf_bits=args.pmf_bits, capacity_bits=T * (P + 2) + 256, device=dev)
    if args.load_inputs:
        pre = f"{args.load_inputs}.r{rank}"
        pmf = torch.from_numpy(np.load(pre + ".pmf.npy")).to(dev)
        sym = torch.from_numpy(np.load(pre + ".sym.npy")).to(dev)
        if logits_in:
            pmf = pmf.view(torch.bfloat16 if ebytes == 2 else torch.float32)
        if tuple(pmf.shape) != (T, B, V) or tuple(sym.shape) != (T, B):
            raise SystemExit(f"{pre}: inputs of shape {tuple(pmf.shape)} / {tuple(sym.shape)}, expected "
                             f"{(T, B, V)} / {(T, B)}")
    elif logits_in:
        logits, sym = synth.logits_batch(T, B, V, seed=1234 + 7919 * rank, device=dev,
                                         dtype=torch.bfloat16 if ebytes == 2 else torch.float32,
                                         quantise=coder.quantize_logits)
        pmf = logits
    else:
        scale_bits = args.scale_bits or (31 if args.pmf_bits == 32 else 60)
        pmf, sym = synth.softmax_tables(T, B, V, seed=1234 + 7919 * rank, device=dev, scale_bits=scale_bits,
                                        storage_bits=args.pmf_bits)
    torch.cuda.synchronize()
    log(f"[rank {rank}] inputs {tuple(pmf.shape)} {pmf.dtype} ({pmf.numel() * ebytes / 2**30:.2f} GiB) "
        f"in {time.time() - t_gen:.1f}s")
    if args.save_inputs:
        pre = f"{args.save_inputs}.r{rank}"
        np.save(pre + ".pmf.npy", (pmf.view(torch.int16) if ebytes == 2 and logits_in else pmf).cpu().numpy())
        np.save(pre + ".sym.npy", sym.cpu().numpy())

    if args.path != "auto":
        coder.set_path(args.path)
    if args.q1_shape:
        coder.set_q1_shape(args.q1_shape)
    if args.decode_path != "auto":
        coder.set_decode_path(args.decode_path)
    if args.block_waves:
        coder.set_block_waves(args.block_waves)

    # N > 1: each job's bitstreams go to rank 0 over RCCL, packed and sized to the
    # payload, --gather-batch jobs per exchange, overlapping the next jobs' encodes
    gatherer = BitstreamGatherer(coder, batch=args.gather_batch) if (world > 1 or args.gather) else None
    # with a gather, consecutive jobs code different symbols (the streams' symbols rolled by
    # 0..3 across streams, prepared before timing), so a job unpacked at another job's
    # offset cannot pass gather_ok; the last timed job codes `sym` itself (the oracle check)
    nvar = 4 if gatherer else 1
    symv = [sym] + [torch.roll(sym, k, dims=1).contiguous() for k in range(1, nvar)]
    job_variant = []

    def job(v=0):
        s_ = symv[v]
        if logits_in:
            coder.encode_logits_job(pmf, s_)
        else:
            coder.encode_job(pmf, s_)
        if gatherer:
            gatherer.submit()
            job_variant.append(v)

    for i in range(args.warmup):
        job(i % nvar)
    if gatherer:
        gatherer.drain()                                   # the timed region holds its own jobs' gathers
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    coder.lib.lac_profile_read(coder.ctx, None, None, 1)
    coder.lib.lac_profile_enable(coder.ctx, 1)
    t0 = time.perf_counter()
    for i in range(args.steps):
        job((args.steps - 1 - i) % nvar)
    if gatherer:
        gatherer.drain()                                   # every gather is inside the timed region
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    coder.lib.lac_profile_enable(coder.ctx, 0)
    dt = t1 - t0
    if dist:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms = (C.c_double * 8)()
    cnt = (C.c_int64 * 8)()
    coder.lib.lac_profile_read(coder.ctx, C.cast(ms, C.c_void_p), C.cast(cnt, C.c_void_p), 1)

    # ---------------- checks, outside the timed region
    gather_ok = None
    gather_info = None
    if gatherer:
        # every job the root still holds (the last `depth` batches) == every rank's own
        # bits for that job's symbols, coded again by a separate coder and collected by a
        # separate exact-width all-gather
        from lac_amd.dist import bitstreams_equal, gather_bitstreams
        refc = BatchCoder(V, B, prec=P, pmf_bits=args.pmf_bits, capacity_bits=T * (P + 2) + 256, device=dev)
        refs = []
        for v in range(nvar):
            if logits_in:
                refc.encode_logits_job(pmf, symv[v])
            else:
                refc.encode_job(pmf, symv[v])
            refs.append(gather_bitstreams(refc.bits_tensor(), refc.nbits_tensor()))
        refc.close()
        okg = True
        checked = 0
        if rank == 0:
            for j in gatherer.finished_jobs:
                gb, gn = gatherer.last_unpacked(j)
                okg = okg and bitstreams_equal(gb, gn, *refs[job_variant[j - 1]])
                checked += 1
            okg = okg and checked > 0
        flag = torch.tensor([1 if okg else 0], device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        gather_ok = bool(flag.item())
        jobs = max(gatherer.jobs, 1)
        gather_info = {"to_rank": 0, "jobs_checked": checked, "symbol_variants": nvar,
                       "link_bytes_per_job": gatherer.bytes_sent / jobs,
                       "payload_bytes_per_job": gatherer.payload_bytes / jobs,
                       "header_bytes_per_stream": gatherer.hdr, "jobs_per_exchange": gatherer.batch,
                       "host_meta_bytes_per_job": gatherer.meta_bytes / jobs}
    rc, err, err_step = coder.status()
    data, nbits = coder.to_bytes() if rc == 0 else ([], None)
    decode = coder.decode_logits if logits_in else coder.decode
    # two warm passes, then the timed passes, all back to back with one synchronisation, as
    # the encode jobs run (a pass timed alone after a host sync paid the clocks' ramp after
    # the idle gap: bf16 Qwen2 decode row stats 209 us per step alone, 182 us back to back,
    # tools/q1_b2b.py)
    warm = []
    for _ in range(2):
        coder.decode_open()
        warm.append(decode(pmf))
    reps = max(1, args.decode_reps)
    coder.lib.lac_profile_read(coder.ctx, None, None, 1)
    coder.lib.lac_profile_enable(coder.ctx, 1)
    outs = []
    # device time of the timed passes: events on the coder's stream (torch's current one),
    # the first recorded behind the warm passes, which are still running when it is queued
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        coder.decode_open()
        outs.append(decode(pmf))
    e1.record()
    torch.cuda.synchronize()
    d0, d1 = 0.0, e0.elapsed_time(e1) * 1e-3
    coder.lib.lac_profile_enable(coder.ctx, 0)
    dms = (C.c_double * 8)()
    dcnt = (C.c_int64 * 8)()
    coder.lib.lac_profile_read(coder.ctx, C.cast(dms, C.c_void_p), C.cast(dcnt, C.c_void_p), 1)
    round_trip = rc == 0
    for dec in warm + outs:
        round_trip = round_trip and bool(torch.equal(dec, sym))
    del outs, warm
    mid = ((d1 - d0) / reps, {k: dms[k] / reps for k in (3, 5, 6, 7) if dcnt[k]})
    dkids = sorted(mid[1])                                     # decode_step|stats path, decode_wave, q1 pair
    dstep_ms = sum(mid[1].values()) / max(T, 1)
    names = {3: "k_decode_step or k_dec_stats+k_decode_seq", 5: "k_decode_wave(_fine) or k_decode_block", 6: "k_q1_stats",
             7: "k_q1_decode"}
    decode_info = {"symbols_per_s": B * T / mid[0], "kernel": "+".join(names[k] for k in dkids),
                   "passes": f"{reps} passes back to back after two warm ones (mean)",
                   "kernel_ms_per_step": dstep_ms,
                   "kernel_ms_per_step_each": {names[k]: mid[1][k] / max(T, 1) for k in dkids},
                   "achieved_GBps": B * (V * ebytes + 4) / (dstep_ms * 1e-3) / 1e9 if dkids else None}
    if dist:
        ok = torch.tensor([1 if round_trip else 0], device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        round_trip = bool(ok.item())

    cpu = None
    parity = {"round_trip_all_streams": round_trip, "stream_status_ok": rc == 0, "decode": decode_info}
    if not logits_in:
        # rows that can take fudged_dist at all: T > w * minp (arith_code.py:84) for some
        # interval width w > 2^(prec-1) (every width the renormalisation leaves)
        nf = 0
        for t in range(T):
            r = pmf[t].to(torch.int64)
            if args.pmf_bits == 32:
                r = r & 0xFFFFFFFF
            mn = torch.where(r > 0, r, torch.full_like(r, 1 << 62)).amin(dim=1)
            tot = r.sum(dim=1, dtype=torch.float64)                    # order of magnitude is enough here
            nf += int((tot > mn.to(torch.float64) * float(1 << (P - 1))).sum())
            del r
        parity["rows_that_can_fudge"] = nf / (T * B)
    if gatherer:
        parity["gather_ok"] = gather_ok
        parity["gather"] = gather_info
    # every rank checks its own streams against the CPU oracle (bit-exact bytes and bit
    # counts); rank 0 then times the oracle on its sample for cpu_baseline
    from oracle import oracle as coracle
    S = B if (args.cpu_streams <= 0 or args.cpu_streams > B) else args.cpu_streams
    if logits_in:
        S = min(S, 512) if args.cpu_streams <= 0 else S          # q1 oracle is per-row, single-threaded
        host = pmf[:, :S, :].contiguous()
        host = host.view(torch.int16).cpu().numpy().view(np.uint16) if ebytes == 2 else host.cpu().numpy()
    else:
        host = pmf[:, :S, :].cpu().numpy()
        host = host.view(np.uint32) if args.pmf_bits == 32 else host.view(np.uint64)
    hsym = sym[:, :S].cpu().numpy()
    nthreads = args.cpu_threads if args.cpu_threads > 0 else host_cores()
    c0 = time.perf_counter()
    tabs = coracle.q1_quantize(host, P) if logits_in else host
    out, onb, ost, orc = coracle.encode_batch(tabs, hsym, P, nthreads=nthreads)
    c1 = time.perf_counter()
    exact = orc == 0 and rc == 0 and all(
        int(onb[b]) == int(nbits[b]) and out[b, :(int(onb[b]) + 7) // 8].tobytes() == data[b] for b in range(S))
    if dist:
        ok = torch.tensor([1 if exact else 0], device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        exact = bool(ok.item())
    parity.update({"oracle_streams_checked": S * world, "oracle_ranks_checked": world,
                   "bit_exact_vs_oracle": bool(exact)})
    if dist:
        dist.barrier()                                     # every rank's parity run is over
    if rank == 0:
        if args.cpu_baseline == "on":
            # cpu_baseline: repetitions of the same bounded sample of their own, timed from
            # here until >= --cpu-seconds of CPU work (the parity run above is not counted: at
            # N > 1 it overlapped the other ranks' own parity runs); other ranks wait
            reps = 0
            c0 = c1 = time.perf_counter()
            while reps == 0 or c1 - c0 < args.cpu_seconds:
                tabs = coracle.q1_quantize(host, P) if logits_in else host
                coracle.encode_batch(tabs, hsym, P, nthreads=nthreads)
                reps += 1
                c1 = time.perf_counter()
            what = "q1 quantise (1 thread) + encode" if logits_in else "encode"
            cpu = {"value": reps * S * T / (c1 - c0), "unit": "symbols/s", "cores": nthreads, "kind": "port",
                   "sample": f"C oracle (oracle/lac_oracle.c) {what} on rank 0's first {S} streams x {T} symbols "
                             f"of the same inputs, repeated {reps}x, {nthreads} threads, {c1 - c0:.1f}s",
                   "cores_rule": f"nproc semantics: {len(os.sched_getaffinity(0))} CPUs in this process's affinity "
                                 f"mask, OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}, "
                                 f"os.cpu_count()={os.cpu_count()}"}
        avg_bits = float(np.mean(nbits.astype(np.float64))) / T if nbits is not None else None
        parity["bits_per_symbol"] = avg_bits
    if dist:
        dist.barrier()                                     # ranks wait out rank 0's baseline

    if rank == 0:
        kid = 6 if cnt[6] else (4 if cnt[4] else 0)        # q1_stats, encode_fused, else row_stats
        kname = {6: "k_q1_stats", 4: "k_encode_fused", 0: "k_row_stats"}[kid]
        units = T * B * args.steps / max(cnt[kid], 1)       # symbols per launch of that kernel
        rs_launch_ms = ms[kid] / max(cnt[kid], 1)
        alg_bytes = units * (V * ebytes + 4)
        achieved = alg_bytes / (rs_launch_ms * 1e-3) / 1e9 if cnt[kid] else None
        rows = (f"{args.input[7:]} logit rows, q1 tables in-kernel" if logits_in else f"uint{args.pmf_bits} pmf rows")
        cname = workload_name(V, B, world)                      # BASELINE.json configs
        cfg = {"workload": f"{cname}: vocab={V}, {B} streams/GPU, {T} symbols/stream per job, prec={P}, {rows}",
               "vocab": V, "streams": B, "tokens": T, "prec": P, "pmf_bits": args.pmf_bits, "input": args.input,
               "parallelism": f"streams sharded over {world} GPU(s)" + (
                   f", {'RCCL' if backend == 'nccl' else backend} payload-sized bitstream gather to rank 0"
                   if gatherer else "")}
        value = world * B * T * args.steps / dt
        line = {
            "metric": METRIC if (V, B) == (32000, 4096) else
                      f"encoded symbols/sec at vocab={V}, batch={B} streams; bit-exact round-trip",
            "value": value, "unit": "symbols/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": ("u32" if logits_in else f"u{args.pmf_bits}"),
            "data": ("synthetic: logits 3*N(0,1) (torch.Generator seeded), symbols by inverse CDF of their q1 tables"
                     if logits_in else
                     "synthetic: logits 3*N(0,1) per step (torch.Generator seeded 1234+t), "
                     f"pmf=max({2 if (args.scale_bits or (31 if args.pmf_bits == 32 else 60)) >= 60 else 1},"
                     f"floor(softmax*2^{args.scale_bits or (31 if args.pmf_bits == 32 else 60)})), symbols by inverse CDF"),
            "config": cfg,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                         "traffic": read_traffic(cfg, kname),
                         "traffic_source": "not measured in this run: HBM bytes per launch of this kernel from "
                                           "the committed profiles/pmc_traffic.json (a separate rocprofv3 --pmc "
                                           "FETCH_SIZE pass of the same config, x2 gfx950 wide-read correction, "
                                           "tools/pmc_traffic.py); null when no entry matches the config",
                         "kernel": kname,
                         "kernel_ms_per_launch": rs_launch_ms, "launches": int(cnt[kid]),
                         "bytes_per_launch": alg_bytes,
                         "kernel_ms_per_step": {n: ms[i] / args.steps for n, i in
                                                (("row_stats", 0), ("encode", 1), ("finish", 2), ("encode_fused", 4),
                                                 ("q1_stats", 6))
                                                if cnt[i]}},
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(line), flush=True)
    if gatherer:
        coder.reset()                                      # (decoding: back to an encoder between jobs)
        gatherer.close()
    coder.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
