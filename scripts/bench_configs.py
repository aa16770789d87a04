#!/usr/bin/env python3
"""Throughput of the non-headline BASELINE.json configs on one GPU (HBM-resident
inputs, HIP events on the launch stream).  Prints one JSON line per config.

  cfg3: TwoStageFFTConvolver, head 64 / tail 4096, IR 262144, 256 channels,
        one 64-sample process() per step.
  cfg5: CrossfadeConvolver<FFTConvolver>, 512 channels, block 512, IR 96000,
        update() with a fresh IR every 128 blocks (trait init: crossfade over
        response.len() samples, so most updates take the pending path).
  cfg1: BASELINE configs[0] -- ONE channel, block 256, IR 4096, the CPU path
        (examples/compare_partitioned.rs:28-53 plumbing: one process() per block,
        wall clock around the loop): the oracle port on one thread, next to the
        same single-channel call sequence on the GPU through the host-buffer C ABI
        (PCIe round trip + launch per 256-sample block: latency, not throughput).
  cfg2u: cfg2 (1024 channels, block 256, IR 48000) with update_device() of
        every channel every 128 blocks (the post-update launches under
        rocprofv3 show whether an IR swap costs the process path anything).
  lg:   the long-block path (csrc/large.hip): lgu = FFTConvolver block 16384,
        IR 1,000,000, 64 channels; lgt = TwoStageFFTConvolver head 512,
        IR 200,000 (tail block 16384), 256 channels.

Algorithmic bytes per output sample follow SURVEY.md §8(d).  Each line also
carries `cpu_baseline` (the oracle port, oracle/fftconv_oracle.c, on a bounded
sample of the same workload on this host's cores) and, with --pmc, `traffic`:
per-kernel HBM bytes per launch from separate rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes of this script (read = 2 x FETCH_SIZE KB, write =
WRITE_SIZE KB, MI355X_MICROARCH.md's gfx950 correction)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))
import numpy as np
import torch

import fftconv_amd as F
from fftconv_amd import shard

sys.path.insert(0, ROOT)
from bench import lookahead_bytes_per_channel_block  # noqa: E402


def uniform_bytes(B, L):
    S = -(-L // B)
    K = B + 1
    return 16 * S * K + 8 * K + 16 * B  # per channel-block


def tail0_deferred_bytes_per_block(head, T):
    """tail0 deferred to the period end (csrc/kernels.hip tail0_*_kernel), per
    channel and head block, in rows of 8*head bytes: over a period of n = T/head
    blocks the flush reads the S0 = T/head IR rows and S0-1 FDL rows once, and
    per block writes / reads its spectrum (R2C, MAC, commit: 4 rows incl. the
    FDL write), its conv (2), its C2R output (2), input and output (1)."""
    n = S0 = T // head
    return (2 * S0 - 1 + 9 * n) * 8 * head / n


GW_P = 8  # far-row windows' split row (csrc/kernels.hpp kGwP)


def windowed_bytes(B, L, P=GW_P):
    """The generic step with far-row windows (1024 <= B <= 8192, DESIGN §4f;
    csrc/kernels.hip gw_anchor_kernel), per channel-block, in rows of 8 B bytes
    (B packed complex slots, Nyquist in slot 0's imaginary part):
      step: H[1..P-1] and their P-1 FDL rows, the window row, H[0], the new
            FDL row (2P + 1 rows) + input, output, overlap read / write (16 B);
      anchor, every P blocks: FDL rows at ring offsets 1..act-1, H[P..act-1],
            and P window rows written (2 act - 1 rows)."""
    S = -(-L // B)
    row = 8 * B
    return row * (2 * P + 1) + row * (2 * S - 1) / P + 16 * B


def lg_step_bytes(B, L, gw=False):
    """One block of the long-block path (csrc/large.hip), per channel: the
    canonical bytes (uniform_bytes; windowed_bytes when the batch runs on
    far-row windows) plus the four-step passes' own row transfers, in rows of
    8 B bytes: pass B re-reads pass A's FDL row and rewrites it as the
    spectrum, writes pre_multiplied and the V scratch, and pass C reads V back
    (5 rows)."""
    return (windowed_bytes(B, L) if gw else uniform_bytes(B, L)) + 5 * 8 * B


def run(conv, C, n_in, n_out, steps, warmup, ring, stream, update=None, batched=False):
    """One process() call per step.  batched: the calls of a ring pass are issued
    by one process_device_steps host call (same kernels, no per-call Python
    overhead) -- what a native (C/C++/Rust) host loop sees."""
    dev = torch.device("cuda:0")
    xin = torch.from_numpy(shard.synth_dry(range(C), ring, n_in)).to(dev)
    yout = torch.empty((ring, C, n_out), device=dev)
    h = stream.cuda_stream
    k = 0

    def step(i):
        r = i % ring
        if batched:
            if r == 0:
                conv.process_device_steps(xin.data_ptr(), n_in, C * n_in, yout.data_ptr(), n_out, C * n_out, n_out,
                                          ring, h)
            return
        if update is not None:
            update(i)
        conv.process_device(xin[r].data_ptr(), n_in, yout[r].data_ptr(), n_out, n_out, h)

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for i in range(steps):
        step(warmup + i)
    e1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ev = e0.elapsed_time(e1) / 1000
    assert torch.isfinite(yout).all()
    return max(wall, ev), ev


def cpu_baseline(kind, C, block, L, every=0, target_s=6.0):
    """The oracle port (kind "port": the reference is unbuildable here) timed
    on this host: one instance per channel, all of this job's threads, a
    bounded number of blocks (~target_s)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline only

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 16, os.cpu_count() or 1))
    # twostage: whole tail periods (T / head calls) so the tail spike is in the sample
    warm = 1
    unit = 1
    if kind == "twostage":
        unit = F.compute_tail_block_size(block, L) // block
        warm = 2 * unit
    t = oracle.bench(kind, C, block, L, unit, warm, threads, every=every)
    nb = int(max(unit, min(200000, target_s / max(t / unit, 1e-7))))
    nb = (nb + unit - 1) // unit * unit
    if every:
        nb = max(nb, every)
    secs = oracle.bench(kind, C, block, L, nb, warm, threads, every=every)
    return {"value": round(C * block * nb / secs / 1e6, 3), "unit": "MSamples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/fftconv_oracle.c {kind}, {C} channels x {nb} blocks of {block} on {threads} threads "
                      f"in {secs:.1f}s" + (f", update() every {every} blocks" if every else "")}


PMC_STEPS = {"3": 256, "5": 256, "2u": 256}
PMC_WARMUP = {"3": 128, "5": 64, "2u": 200}  # (run()'s warmup per config: cfg3 2T/head, cfg5 64, cfg2u 200)
PMC_REGEX = "upols_|ir_segments|la_rebuild|tail0_|twostage_accum|crossfade_mix|reset_state|lg_"


def pmc_config(cfg):
    """HBM traffic of ONE config's run (its own two rocprofv3 --pmc passes,
    FETCH_SIZE and WRITE_SIZE, before this process touches the GPU): per
    kernel the median bytes per launch and the launches, and the measured
    bytes per step -- every dispatch from the config's first process launch
    on (init and IR upload excluded, the updates inside the timed region
    included) over the run's warmup + timed calls.  Returns a dict or a note."""
    import csv
    import glob
    import shutil
    import statistics
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3")
    if not prof:
        return "rocprofv3 not found"
    env = dict(os.environ, TMPDIR="/tmp")
    steps_args = [f"--steps{cfg[0] if cfg != '2u' else '2'}", str(PMC_STEPS[cfg])]
    per = {}    # kernel -> {counter: [values per dispatch]}
    total = {}  # counter -> bytes from the first process dispatch on
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix=f"pmc_{counter}_", dir="/tmp")
        cmd = [prof, "--pmc", counter, "--kernel-include-regex", PMC_REGEX, "-d", d, "-o", "pmc", "--output-format",
               "csv", "--", sys.executable, os.path.abspath(__file__), "--configs", cfg, "--no-cpu",
               "--pmc-inner"] + steps_args
        try:
            subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           timeout=300, check=True)
        except Exception as e:
            return f"rocprofv3 --pmc {counter} failed: {type(e).__name__}"
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if r.get("Counter_Name") == counter:
                    rows.append((int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(rows)), r["Kernel_Name"],
                                 float(r["Counter_Value"])))
        shutil.rmtree(d, ignore_errors=True)
        rows.sort()
        first = next((i for i, r in enumerate(rows) if "upols_" in r[1]), len(rows))
        scale = 2048 if counter == "FETCH_SIZE" else 1024  # (KB; FETCH_SIZE counts half on gfx950)
        total[counter] = sum(v for _, _, v in rows[first:]) * scale
        for _, k, v in rows[first:]:
            per.setdefault(k, {}).setdefault(counter, []).append(v * scale)
    calls = PMC_STEPS[cfg] + PMC_WARMUP[cfg]
    kern = {}
    for k, v in per.items():
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            kern[k] = {"bytes_per_launch": int(statistics.median(v["FETCH_SIZE"]) + statistics.median(v["WRITE_SIZE"])),
                       "launches_per_step": round(len(v["FETCH_SIZE"]) / calls, 4)}
    return {"kernels": kern, "measured_bytes_per_step": int((total["FETCH_SIZE"] + total["WRITE_SIZE"]) / calls),
            "calls": calls, "correction": "read = 2 x FETCH_SIZE KB, write = WRITE_SIZE KB (gfx950)"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default="3,5")
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline legs")
    p.add_argument("--pmc", action="store_true", help="per-kernel HBM traffic from rocprofv3 --pmc child passes")
    p.add_argument("--pmc-inner", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--steps2", type=int, default=1024)
    p.add_argument("--steps3", type=int, default=2048)
    p.add_argument("--steps5", type=int, default=512)
    p.add_argument("--sweep", default="",
                   help="cfg3 only: ';'-separated knob sets (e.g. 'lag=0;lag=32;variant=4') timed "
                        "interleaved in this process, --rounds times")
    p.add_argument("--rounds", type=int, default=4)
    p.add_argument("--variant", type=int, default=-1, help="fftconv_set_kernel_variant for every config")
    a = p.parse_args()
    traffic = {}
    if a.pmc and not a.pmc_inner:  # (child processes first: this one has not touched the GPU yet)
        for cfg in a.configs.split(","):
            if cfg in PMC_STEPS:
                traffic[cfg] = pmc_config(cfg)
    F.set_kernel_variant(a.variant)
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    out = []
    if "3" in a.configs.split(","):
        C, head, L = 256, 64, 262144
        conv = F.TwoStageFFTConvolver.init(shard.synth_irs(range(C), L), head, L, channels=C)
        T = conv.tail_block_size
        samples = C * head * a.steps3
        canon_sample = (uniform_bytes(head, T) + uniform_bytes(head, T) + uniform_bytes(T, L - 2 * T) * head / T) / head
        defer = a.variant < 0 or not (a.variant & 256)  # (VARIANT_T0BLOCK, host.cpp TwoStageCore::t0_defer)
        tail0_b = tail0_deferred_bytes_per_block(head, T) if defer else uniform_bytes(head, T)
        gw = (a.variant < 0 or not (a.variant & 1024)) and 1024 <= T <= 8192 and -(-(L - 2 * T) // T) >= 3 * GW_P
        tail_b = windowed_bytes(T, L - 2 * T) if gw else uniform_bytes(T, L - 2 * T)
        per_sample = (uniform_bytes(head, T) + tail0_b + tail_b * head / T) / head
        if a.sweep:
            sets = [dict(kv.split("=") for kv in part.split(",") if kv) for part in a.sweep.split(";")]
            times = [[] for _ in sets]
            for _ in range(a.rounds):
                for j, kn in enumerate(sets):
                    F.set_pipeline_lag(int(kn.get("lag", -1)))
                    F.set_kernel_variant(int(kn.get("variant", -1)))
                    t, ev = run(conv, C, head, head, a.steps3, 2 * T // head, 64, s, batched=True)
                    times[j].append(t)
            F.set_pipeline_lag(-1)
            F.set_kernel_variant(-1)
            for kn, ts in zip(sets, times):
                t = sorted(ts)[len(ts) // 2]
                out.append({"config": "cfg3 sweep", "knobs": kn, "MSamples_s": round(samples / t / 1e6, 2),
                            "us_per_step": round(t / a.steps3 * 1e6, 3)})
        for batched in ((True,) if a.pmc_inner else (False, True)):
            t, ev = run(conv, C, head, head, a.steps3, 2 * T // head, 64, s, batched=batched)
            out.append({"config": "cfg3 TwoStageFFTConvolver", "host_loop": "C++ (process_device_steps)" if batched
                        else "Python (one process_device per step)", "channels": C, "head": head, "tail": T,
                        "ir": L, "steps": a.steps3, "MSamples_s": round(samples / t / 1e6, 2),
                        "us_per_step": round(t / a.steps3 * 1e6, 3),
                        "algorithmic_GBs": round(samples * per_sample / t / 1e9, 1),
                        "frac_of_8TBs": round(samples * per_sample / t / 8e12, 4),
                        "bytes_per_sample": round(per_sample, 1),
                        "canonical_bytes_per_sample": round(canon_sample, 1),
                        "path": ("head: one fused launch per call; tail0 deferred to the period end (one pass per "
                                 "period); tail: side stream" if tail0_b != uniform_bytes(head, T) else
                                 "head + tail0: one launch per call; tail: side stream")
                                + ("; tail far-row windows (model: windowed_bytes)" if gw else ""),
                        "cfg": "3", "model_bytes_per_step": int(per_sample * C * head)})
        del conv
        if not a.no_cpu and not a.pmc_inner:
            out[-1]["cpu_baseline"] = cpu_baseline("twostage", C, head, L)
    if "5" in a.configs.split(","):
        C, B, L = 512, 512, 96000
        irs = shard.synth_irs(range(C), L)
        conv = F.CrossfadeConvolver.init(irs, B, L, channels=C)
        # fresh IRs resident in HBM (like the inputs): update_device, stream-ordered
        fresh = [torch.from_numpy(shard.synth_irs(range(1000 + 100 * j, 1000 + 100 * j + C), L)).cuda()
                 for j in range(2)]
        torch.cuda.synchronize()

        def upd(i):
            if i % 128 == 127:
                conv.update_device(fresh[(i // 128) % 2].data_ptr(), L, L, s.cuda_stream)

        t, ev = run(conv, C, B, B, a.steps5, 64, 16, s, update=upd)
        samples = C * B * a.steps5
        # both inner convolvers on the lookahead step unless variant bit 4 is set
        la = a.variant < 0 or not (a.variant & 16)
        per_sample = 2 * (lookahead_bytes_per_channel_block(B, L) if la else uniform_bytes(B, L)) / B
        out.append({"config": "cfg5 CrossfadeConvolver, update every 128 blocks", "channels": C, "block": B,
                    "ir": L, "steps": a.steps5, "MSamples_s": round(samples / t / 1e6, 2),
                    "us_per_step": round(t / a.steps5 * 1e6, 3),
                    "path": ("lookahead step: ONE launch per call (A's and B's anchors; per channel one workgroup "
                             "with A's and B's chains, mixed in LDS)") if la else "full-sum pair launch",
                    "algorithmic_GBs_incl_updates": round(samples * per_sample / t / 1e9, 1),
                    "frac_of_8TBs": round(samples * per_sample / t / 8e12, 4),
                    "bytes_per_sample": round(per_sample, 1),
                    "canonical_bytes_per_sample": round(2 * uniform_bytes(B, L) / B, 1),
                    "note": "update_device() (HBM-resident IRs: S-segment FFTs per channel) is inside the timed region",
                    "cfg": "5", "model_bytes_per_step": int(per_sample * C * B)})
        del conv, fresh
        if not a.no_cpu and not a.pmc_inner:
            out[-1]["cpu_baseline"] = cpu_baseline("crossfade", C, B, L, every=128)
    if "1" in a.configs.split(",") and not a.pmc_inner:
        B, L, nb = 256, 4096, 4000
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # the CPU path (port of the reference's algorithm)

        secs = oracle.bench("uniform", 1, B, L, nb, 100, 1)
        ir1 = shard.synth_irs(range(1), L)[0]
        x1 = shard.synth_dry(range(1), 64, B)[:, 0, :]
        conv1 = F.FFTConvolver.init(ir1, B, L)
        for i in range(100):
            conv1.process(x1[i % 64])
        t0 = time.perf_counter()
        for i in range(nb):
            conv1.process(x1[i % 64])
        gsec = time.perf_counter() - t0
        out.append({"config": "cfg1 FFTConvolver, 1 channel, block 256, IR 4096 (CPU path)", "blocks": nb,
                    "cpu_baseline": {"value": round(B * nb / secs / 1e6, 3), "unit": "MSamples/s", "cores": 1,
                                     "kind": "port", "us_per_block": round(secs / nb * 1e6, 3),
                                     "sample": f"oracle/fftconv_oracle.c FFTConvolver, 1 channel x {nb} blocks of "
                                               f"{B}, one thread (the reference is one instance on one thread)"},
                    "gpu_host_path": {"value": round(B * nb / gsec / 1e6, 3), "unit": "MSamples/s",
                                      "us_per_block": round(gsec / nb * 1e6, 3),
                                      "note": "fftconv_uniform_process per block from Python (H2D + launch + D2H "
                                              "+ stream sync): one channel is latency-bound on a GPU"}})
        del conv1
    if "2u" in a.configs.split(","):
        C, B, L = 1024, 256, 48000
        conv = F.FFTConvolver.init(shard.synth_irs(range(C), L), B, L, channels=C)
        fresh = [torch.from_numpy(shard.synth_irs(range(2000 + 1000 * j, 2000 + 1000 * j + C), L)).cuda()
                 for j in range(2)]
        torch.cuda.synchronize()

        def upd2(i):
            if i % 128 == 127:
                conv.update_device(fresh[(i // 128) % 2].data_ptr(), L, L, s.cuda_stream)

        t, ev = run(conv, C, B, B, a.steps2, 200, 32, s, update=upd2)
        samples = C * B * a.steps2
        out.append({"config": "cfg2u FFTConvolver, update_device every 128 blocks", "channels": C, "block": B,
                    "ir": L, "steps": a.steps2, "MSamples_s": round(samples / t / 1e6, 2),
                    "us_per_step": round(t / a.steps2 * 1e6, 3),
                    "note": "update_device() (IR transform + window rebuild) inside the timed region",
                    "cfg": "2u", "model_bytes_per_step": int(lookahead_bytes_per_channel_block(B, L) * C)})
        del conv, fresh
    cfgs = a.configs.split(",")
    if "lg" in cfgs or "lgu" in cfgs:
        # the long-block path (csrc/large.hip, B >= 16384): passes A / B / C
        # per chunk + lg_call_end.  lgu: FFTConvolver B 16384, IR 1,000,000
        # (S 62), 64 channels; lgt: TwoStageFFTConvolver head 512, IR 200,000
        # (T = 16,384 by :520-526, the tail on the long-block path), 256 channels
        C, B, L = 64, 16384, 1000000
        conv = F.FFTConvolver.init(shard.synth_irs(range(C), L), B, L, channels=C)
        S = conv.seg_count
        gw = conv.far_windows() > 0
        steps = max(8, a.steps2 // 16)
        t, ev = run(conv, C, B, B, steps, S + 2, 4, s, batched=True)
        samples = C * B * steps
        per_sample = lg_step_bytes(B, L, gw) / B
        out.append({"config": "lgu FFTConvolver on the long-block path", "channels": C, "block": B, "ir": L,
                    "segments": S, "steps": steps, "MSamples_s": round(samples / t / 1e6, 2),
                    "us_per_step": round(t / steps * 1e6, 3),
                    "algorithmic_GBs": round(samples * per_sample / t / 1e9, 1),
                    "frac_of_8TBs": round(samples * per_sample / t / 8e12, 4),
                    "bytes_per_sample": round(per_sample, 1),
                    "canonical_bytes_per_sample": round(uniform_bytes(B, L) / B, 1),
                    "path": "lg_cols_fwd -> lg_rows (the FDL MAC) -> lg_cols_inv -> lg_call_end per call"
                            + (" + gw_anchor_kernel (far-row windows, model: windowed_bytes)" if gw else ""),
                    "cfg": "lgu", "model_bytes_per_step": int(per_sample * C * B)})
        del conv
        if not a.no_cpu and not a.pmc_inner:
            out[-1]["cpu_baseline"] = cpu_baseline("uniform", C, B, L, target_s=4.0)
    if "lg" in cfgs or "lgt" in cfgs:
        C, head, L = 256, 512, 200000
        conv = F.TwoStageFFTConvolver.init(shard.synth_irs(range(C), L), head, L, channels=C)
        T = conv.tail_block_size
        per = T // head
        steps = per * max(4, a.steps3 // (8 * per))
        t, ev = run(conv, C, head, head, steps, 2 * per, per, s, batched=True)
        samples = C * head * steps
        per_sample = (uniform_bytes(head, T) + tail0_deferred_bytes_per_block(head, T)
                      + lg_step_bytes(T, L - 2 * T) * head / T) / head
        out.append({"config": "lgt TwoStageFFTConvolver, tail on the long-block path", "channels": C, "head": head,
                    "tail": T, "ir": L, "steps": steps, "MSamples_s": round(samples / t / 1e6, 2),
                    "us_per_step": round(t / steps * 1e6, 3),
                    "algorithmic_GBs": round(samples * per_sample / t / 1e9, 1),
                    "frac_of_8TBs": round(samples * per_sample / t / 8e12, 4),
                    "bytes_per_sample": round(per_sample, 1),
                    "cfg": "lgt", "model_bytes_per_step": int(per_sample * C * head)})
        del conv
        if not a.no_cpu and not a.pmc_inner:
            out[-1]["cpu_baseline"] = cpu_baseline("twostage", C, head, L, target_s=4.0)
    if "2m" in a.configs.split(","):
        # cfg2 with calls of m whole blocks (the reference's process over any
        # output length, src/fft_convolver.rs:222-294): one lookahead launch per
        # block, the windows kept -- throughput per m, same per-block work
        C, B, L = 1024, 256, 48000
        res = {}
        for m in (1, 2, 4):
            conv = F.FFTConvolver.init(shard.synth_irs(range(C), L), B, L, channels=C)
            nsteps = max(1, a.steps2 // m)
            t, ev = run(conv, C, m * B, m * B, nsteps, 200 // m, 32 // m, s, batched=True)
            res[f"calls_of_{m}_blocks"] = {"MSamples_s": round(C * m * B * nsteps / t / 1e6, 2),
                                           "us_per_block": round(t / (nsteps * m) * 1e6, 3)}
            del conv
        out.append({"config": "cfg2m FFTConvolver, calls of m * 256 samples", "channels": C, "block": B, "ir": L,
                    "per_m": res, "cfg": "2m"})
    for o in out:
        t = traffic.get(o.get("cfg"))
        if t is not None:
            o["traffic"] = t  # (this config's own PMC passes)
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
