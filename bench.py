#!/usr/bin/env python3
"""bench.py -- MSamples/s of the batched uniformly-partitioned convolver.

Workload (BASELINE.json configs[1], the north-star metric's config): 1024
channels per GPU, block 256, a distinct 48,000-tap white-noise IR per channel,
f32.  One *step* = one FFTConvolver::process call of 256 samples on every
channel (src/fft_convolver.rs:215-295) = one fused kernel launch: forward R2C
of the new block into the FDL, the S-segment spectral MAC, C2R and overlap-add
-- with the lookahead step (csrc/la.hpp) each step sums only the 4 nearest
FDL rows itself; rows 5..16 are summed 4 blocks ahead (C/4 channels per
launch), rows 17..64 sixteen blocks ahead (C/16) and rows >= 65 sixty-four
blocks ahead (C/64) by anchors, S >= 40.  The timed steps are submitted through
process_device_steps (the C ABI loops over the calls), not one Python call each.
Inputs are resident in HBM when the timed region starts.

Multi-GPU (BASELINE configs[3], 8192 channels on 8 GPUs): one process per GPU
(`--gpus N` without a launcher spawns the N rank processes itself),
1024 channels per rank (weak scaling, channel shards have no data-path
exchange); barrier + synchronize around the timed region, max time over ranks.
`--dry shared` instead broadcasts the dry blocks from rank 0 over RCCL (the
"one source, many IRs" case) and feeds each to every channel: one bucketed
broadcast per run of ring slots (up to `--ring` blocks, 32 KB at the
default) ahead of that run's process_device_steps call, not one per block
(`--per-call`: one broadcast and one call per step).

Prints ONE JSON line on rank 0 (driver contract), with `roofline` for the fused
kernel and `cpu_baseline` from the oracle port on this host (rank 0, N=1).
`roofline.launch_us` is the kernel's average duration from a rocprofv3
--kernel-trace --stats child pass of this same command (run before this
process touches the GPU; `--kt-out DIR` keeps its csv files, profiles/r6/
holds the committed ones), so `frac` = bytes_per_launch / launch_us / 8 TB/s
is reproducible from that summary; the HIP-event time of the timed steps is
`launch_us_events`.  `traffic` comes from two more child passes (--pmc
FETCH_SIZE, then WRITE_SIZE).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))

METRIC = "MSamples/s convolved (block=256, IR=48000) per node; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def algorithmic_bytes_per_channel_block(B: int, L: int) -> int:
    """16*S*K (IR spectra + FDL read once) + 8*K (new X write)
    + 4B (in) + 4B (out) + 8B (overlap r/w), K = B+1 bins, S = ceil(L/B).
    cfg2: 779,208 B."""
    S = -(-L // B)
    K = B + 1
    return 16 * S * K + 8 * K + 4 * B + 4 * B + 8 * B


# lookahead levels (fft-convolution_amd/csrc/la.hpp): near rows 1..D0; anchor
# level k sums rows (R_{k-1}, R_k] every P_k blocks (R_0 = D0, R_3 = S - 1)
LA_D0 = 4
LA_LEVELS = ((4, 16), (16, 64), (64, None))  # (P_k, R_k)
LA_NEAR_NEXT_MIN_B = 512  # la.hpp near_next(): B > 256 (no in-step level-1 anchors) stores the next near sum


def lookahead_bytes_per_channel_block(B: int, L: int) -> int:
    """Bytes per channel-block the lookahead step (la.hpp) reads and writes, in
    the units of SURVEY.md §8(d) (rows of K = B+1 bins, 8 B per bin):
      anchor level k (period P, rows lo..hi, an anchor every P blocks): H rows
        lo..hi and FDL ages 1..hi-1 once: 8K (2 hi - lo) / P -- level 3 only
        when S > 65 (la_nlv);
      near rows (step): H[1..D0] and the last D0 blocks: 8K * 2 D0;
      window rows written by the anchors and read by the steps: 16K per level;
      the new X row, H[0], in, out, overlap r/w: 16K + 16B.
    At B >= 512 the helpers also store the next block's near sum (la.hpp
    near_next): per block one more row read and one written, one FDL row
    fewer read (this block's spectrum comes from LDS): + 8K.
    cfg2: 75,060 B (round 2's three levels: 82,750 B), against 779,208 B for
    the reference's algorithm (every block streams all S rows of H and of the
    FDL)."""
    S = -(-L // B)
    K = B + 1
    total = 0.0
    lo = LA_D0 + 1
    for P, R in LA_LEVELS:
        hi = S - 1 if R is None else min(R, S - 1)
        if hi < lo:
            break
        total += 8 * K * (2 * hi - lo) / P + 16 * K
        lo = hi + 1
    near = 8 * K * 2 * LA_D0 + (8 * K if B >= LA_NEAR_NEXT_MIN_B else 0)
    return int(total + near + 16 * K + 16 * B)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--channels", type=int, default=1024, help="channels per GPU")
    p.add_argument("--block", type=int, default=256)
    p.add_argument("--ir", type=int, default=48000)
    p.add_argument("--dry", choices=["per-channel", "shared"], default="per-channel")
    p.add_argument("--ring", type=int, default=32, help="distinct input/output blocks kept in HBM")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="target CPU time per baseline leg")
    p.add_argument("--pmc", choices=["auto", "off"], default="auto",
                   help="collect HBM traffic with two rocprofv3 --pmc child passes (N=1, rank 0)")
    p.add_argument("--kt", choices=["auto", "off"], default="auto",
                   help="take the dominant kernel's launch duration from a rocprofv3 --kernel-trace --stats child "
                        "pass of this same command (N=1, rank 0; else HIP events)")
    p.add_argument("--kt-out", default=None, help="keep that pass's rocprofv3 csv files in this directory")
    p.add_argument("--pmc-inner", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL)")
    p.add_argument("--same-device", action="store_true",
                   help="debug: every rank on device 0 (rehearse the N>1 path on a one-GPU box, gloo)")
    p.add_argument("--per-call", action="store_true",
                   help="submit one process_device call per step from Python (default: process_device_steps)")
    p.add_argument("--spawn-probe", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args()


def free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(args) -> int:
    """`--gpus N` (N > 1) without a launcher: start N fresh rank processes,
    one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set -- the
    environment torch.distributed.run would give them -- before this process
    touches the GPU, and wait for all of them.  Rank 0 prints the JSON line.
    Returns the first non-zero exit status (0 if every rank succeeded), so no
    path can report N ranks' throughput from one process."""
    port = free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        print(f"bench.py: rank exit statuses {rcs}", file=sys.stderr)
        return bad[0]
    return 0


def pmc_traffic(args):
    """HBM bytes per launch of the fused kernel from two separate rocprofv3
    --pmc passes of this same workload (FETCH_SIZE, then WRITE_SIZE), corrected
    as MI355X_MICROARCH.md §HBM prescribes: read = 2 x FETCH_SIZE KB (gfx950
    reports half of a wide coalesced stream), write = WRITE_SIZE KB.  Runs
    before this process touches the GPU; returns (bytes, note)."""
    import csv
    import glob
    import shutil
    import statistics
    import tempfile

    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    if any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None, "already under rocprofv3: no nested --pmc pass"
    env = dict(os.environ, TMPDIR="/tmp")
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix=f"pmc_{counter}_", dir="/tmp")
        cmd = [prof, "--pmc", counter, "--kernel-include-regex", "upols_", "-d", d, "-o", "pmc",
               "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__), "--pmc-inner",
               "--pmc", "off", "--no-cpu-baseline", "--steps", "20", "--warmup", "3",
               "--channels", str(args.channels), "--block", str(args.block), "--ir", str(args.ir)]
        try:
            subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           timeout=240, check=True)
        except Exception as e:  # no counters on this box: traffic stays null
            return None, f"rocprofv3 --pmc {counter} failed: {type(e).__name__}"
        got = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if r.get("Counter_Name") == counter and "upols_" in r.get("Kernel_Name", ""):
                    got.append(float(r["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if not got:
            return None, f"no {counter} rows"
        vals[counter] = statistics.median(got)
    read_b = 2.0 * vals["FETCH_SIZE"] * 1024.0
    write_b = vals["WRITE_SIZE"] * 1024.0
    return int(read_b + write_b), (f"rocprofv3 --pmc, median of 20 launches per pass: read 2xFETCH_SIZE = "
                                   f"{read_b / 1e6:.1f} MB, write WRITE_SIZE = {write_b / 1e6:.1f} MB")


def kernel_trace_pass(args):
    """The dominant kernel's average launch duration from a rocprofv3
    --kernel-trace --stats child pass of this same workload (same channels,
    steps and warmup), run before this process touches the GPU.  Returns
    (avg_us, calls, kernel name, note); the csv files stay in --kt-out when
    given (profiles/ keeps the committed ones)."""
    import csv
    import glob
    import shutil
    import tempfile

    prof = shutil.which("rocprofv3")
    if not prof:
        return None, 0, None, "rocprofv3 not found"
    if any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None, 0, None, "already under rocprofv3: no nested pass"
    d = os.path.abspath(args.kt_out) if args.kt_out else tempfile.mkdtemp(prefix="kt_", dir="/tmp")
    os.makedirs(d, exist_ok=True)
    cmd = [prof, "--kernel-trace", "--stats", "-d", d, "-o", "kt", "--output-format", "csv", "--",
           sys.executable, os.path.abspath(__file__), "--pmc-inner", "--pmc", "off", "--kt", "off",
           "--no-cpu-baseline", "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--channels", str(args.channels), "--block", str(args.block), "--ir", str(args.ir)]
    try:
        subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL,
                       stderr=subprocess.DEVNULL, timeout=300, check=True)
        best = None
        for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "upols_" in r["Name"] and (best is None or int(r["Calls"]) > int(best["Calls"])):
                    best = r
    except Exception as e:  # no profiler on this box: HIP events instead
        return None, 0, None, f"rocprofv3 --kernel-trace failed: {type(e).__name__}"
    finally:
        if not args.kt_out:
            shutil.rmtree(d, ignore_errors=True)
    if best is None:
        return None, 0, None, "no upols_ kernel in the stats"
    name = best["Name"].split("(")[0].replace("void ", "")
    return (float(best["AverageNs"]) / 1000.0, int(best["Calls"]), name,
            f"rocprofv3 --kernel-trace --stats child pass of this command: AverageNs of {best['Calls']} launches")


def make_irs(rank: int, C: int, L: int, world: int = 1) -> np.ndarray:
    """Distinct IR per global channel (fftconv_amd.shard.synth_irs)."""
    from fftconv_amd import shard

    return shard.synth_irs(shard.channel_range(rank, max(world, rank + 1), C), L)


def cpu_baseline(C: int, B: int, L: int, target_s: float):
    """Oracle port timed on this host on the same workload (C channels, one
    FFTConvolver instance per channel, as the reference is one instance per
    channel) split over all threads of this job, and on one thread; a
    bounded number of blocks (~target_s of CPU time per leg)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the checker / CPU baseline only

    # the job's CPU share: the affinity mask, capped by OMP_NUM_THREADS when the
    # scheduler sets it (the GPU box grants one GPU's job 16 CPUs of a larger
    # host and exports OMP_NUM_THREADS=16; os.cpu_count() is the whole host)
    host_cores = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = host_cores
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(affinity, omp) if omp > 0 else affinity)
    res = {}
    for th in sorted({1, threads}):
        ch = C if th > 1 else max(1, C // 16)  # single-thread leg: a 1/16 slice of the channels
        t = oracle.bench_uniform(ch, B, L, 2, 1, th)  # calibration
        per_block = max(t / 2, 1e-6)
        nb = int(max(4, min(100000, target_s / per_block)))
        secs = oracle.bench_uniform(ch, B, L, nb, 2, th)
        res[th] = (ch * B * nb / secs / 1e6, ch, nb, secs)
    v1 = res[1]
    vt = res[threads]
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": round(vt[0], 3),
        "unit": "MSamples/s",
        "cores": threads,
        "host_cores": host_cores,
        "affinity_cpus": affinity,
        "omp_num_threads": omp or None,
        "cpu_model": model,
        "cores_note": ("threads = the job's CPU share: min(affinity mask, OMP_NUM_THREADS); the GPU pool "
                       "grants a one-GPU job 16 CPUs of the host and sets OMP_NUM_THREADS=16"),
        "kind": "port",
        "sample": (f"oracle/fftconv_oracle.c FFTConvolver, B={B}, IR={L}: {vt[1]} channels x {vt[2]} blocks on "
                   f"{threads} threads in {vt[3]:.1f}s; single thread {v1[1]} ch x {v1[2]} blocks = "
                   f"{v1[0]:.3f} MSamples/s"),
        "single_core_value": round(v1[0], 3),
    }


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(spawn_ranks(args))
    if world != args.gpus:
        # a launcher's world size wins: the job runs (and reports) that many ranks
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; running {world} rank(s)", file=sys.stderr)
        args.gpus = world
    if args.spawn_probe:  # (tests: the rank environment, no GPU work)
        print(json.dumps({"rank": rank, "local_rank": local_rank, "world": world}), flush=True)
        return
    traffic, traffic_note = None, "not collected (N>1 or --pmc off)"
    if args.pmc == "auto" and world == 1 and not args.pmc_inner:
        traffic, traffic_note = pmc_traffic(args)  # child processes, before this one touches the GPU
    kt_us, kt_calls, kt_name, kt_note = None, 0, None, "not collected (N>1 or --kt off)"
    if args.kt == "auto" and world == 1 and not args.pmc_inner:
        kt_us, kt_calls, kt_name, kt_note = kernel_trace_pass(args)

    import torch

    if args.same_device:
        local_rank = 0
    elif local_rank >= torch.cuda.device_count():
        raise SystemExit(f"bench.py: rank {rank} needs device {local_rank}, "
                         f"{torch.cuda.device_count()} visible (one process per GPU)")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    import fftconv_amd as F

    from fftconv_amd import shard

    C, B, L = args.channels, args.block, args.ir
    mine = shard.channel_range(rank, world, C)  # global channel ids of this rank
    irs = shard.synth_irs(mine, L)
    conv = F.FFTConvolver.init(irs, B, L, channels=C, device=local_rank)
    del irs
    S = conv.seg_count
    ring = max(1, args.ring)
    if args.dry == "shared":
        dry = torch.from_numpy(shard.synth_shared_dry(ring, B)).to(dev)
        if rank != 0:
            dry.zero_()  # rank 0 owns the source; the others receive it by broadcast
        xin = None
    else:
        xin = torch.from_numpy(shard.synth_dry(mine, ring, B)).to(dev)
    yout = torch.empty((ring, C, B), device=dev)
    # a dedicated stream (NULL would be HIP's null stream, fftconv.h "Streams";
    # its own stream keeps the timed region's events on the launch stream)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    torch.cuda.synchronize(dev)

    def step(i: int):
        r = i % ring
        if args.dry == "shared":
            d = dry[r]
            if dist is not None:
                shard.broadcast_dry(dist, d, src=0)
            # every channel reads the same broadcast block (input stride 0)
            conv.process_device(d.data_ptr(), 0, yout[r].data_ptr(), B, B, sh)
        else:
            conv.process_device(xin[r].data_ptr(), B, yout[r].data_ptr(), B, B, sh)

    def steps(i0: int, k: int):
        """k consecutive steps from step i0: one process_device_steps call per
        run of ring slots (the ABI loops over the calls in C++, so Python's
        per-call submission cost stays out of the timed region)."""
        if args.per_call:
            for i in range(i0, i0 + k):
                step(i)
            return
        i = i0
        while i < i0 + k:
            r = i % ring
            n = min(ring - r, i0 + k - i)
            if args.dry == "shared":
                if dist is not None:
                    shard.broadcast_dry(dist, dry[r:r + n], src=0)  # one collective for the run's n blocks
                # every channel reads the broadcast block of its step (input stride 0)
                conv.process_device_steps(dry[r].data_ptr(), 0, B, yout[r].data_ptr(), B, C * B, B, n, sh)
            else:
                conv.process_device_steps(xin[r].data_ptr(), B, C * B, yout[r].data_ptr(), B, C * B, B, n, sh)
            i += n

    steps(0, args.warmup)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    steps(args.warmup, args.steps)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1)  # HIP events on the launch stream
    elapsed = max(wall, kern_ms / 1000.0)
    if dist is not None:
        t = torch.tensor([elapsed, kern_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    if not torch.isfinite(yout).all():
        raise SystemExit("non-finite output")

    total_samples = world * C * B * args.steps  # the ranks that actually ran
    value = total_samples / elapsed / 1e6
    ev_launch_s = kern_ms / 1000.0 / args.steps
    # the dominant kernel's launch duration: the rocprofv3 kernel-trace pass's
    # average when it ran (reproducible from the committed stats), else the
    # HIP events around the timed launches
    per_launch_s = kt_us * 1e-6 if kt_us else ev_launch_s
    canonical_bytes = algorithmic_bytes_per_channel_block(B, L) * C
    parts = conv.lookahead_parts()
    if parts:
        bytes_per_launch = lookahead_bytes_per_channel_block(B, L) * C
        kname = (f"upols_la_kernel (lookahead step: step workgroups of 2 channels running the level-1 "
                 f"anchors of {C}/4 channels + level-2 anchors for {C}/16 and level-3 anchors for {C}/64 "
                 f"channels per launch)")
    else:
        bytes_per_launch = canonical_bytes
        kname = "upols_process_kernel (fused UPOLS step, one workgroup per channel)"
    achieved = bytes_per_launch / per_launch_s / 1e9

    if rank == 0 and args.pmc_inner:
        return
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(C, B, L, args.cpu_seconds)
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "MSamples/s",
            # distinct devices: --same-device rehearsals share one GPU
            "n_gpus": 1 if args.same_device else world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1000.0 / args.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: white-noise U[-1,1) dry blocks resident in HBM, distinct white-noise IR "
                    "U[-1,1)/sqrt(L) per channel",
            "config": {
                "workload": "cfg2 FFTConvolver batch" if world == 1 else "cfg4 FFTConvolver channel shards",
                "channels_per_gpu": C,
                "channels_total": C * world,
                "block_size": B,
                "ir_len": L,
                "segments": S,
                "dry_input": args.dry,
                # --dry shared: one RCCL broadcast per run of ring slots (bucketed), or one per step with --per-call
                "broadcast": (None if args.dry != "shared" else
                              ("per-step" if args.per_call else f"bucketed x{args.ring}")),
                "parallelism": f"channel-shard x{world}",
                "submission": "per-call" if args.per_call else "process_device_steps",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_note": traffic_note,
                "traffic_gbs": round(traffic / per_launch_s / 1e9, 1) if traffic else None,
                "kernel": kname,
                "bytes_per_launch": bytes_per_launch,
                "launch_us": round(per_launch_s * 1e6, 3),
                "launch_us_source": kt_note if kt_us else "HIP events on the launch stream over the timed steps",
                "rocprof_kernel": kt_name,
                "rocprof_calls": kt_calls,
                "launch_us_events": round(ev_launch_s * 1e6, 3),
                # the reference's algorithm (every block streams all S rows of H
                # and the FDL) would need this many bytes per launch:
                "canonical_bytes_per_launch": canonical_bytes,
                "canonical_equiv_gbs": round(canonical_bytes / per_launch_s / 1e9, 1),
            },
            "cpu_baseline": cpu,
        }
        if args.same_device:
            line["same_device"] = True  # a rehearsal: every rank on device 0, not an N-GPU result
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
