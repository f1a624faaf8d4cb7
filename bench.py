#!/usr/bin/env python3
"""Benchmark of the MI355X hot paths (driver contract: one JSON line on rank 0).

Headline (BASELINE.json configs[1], "C2"): PairHMM forward algorithm on
1,000,000 synthetic (read, haplotype) pairs per GPU, read length 101,
haplotype length uniform in [150, 300], fp32 pass + fp64 rescue, inputs
resident in HBM.  A step = one full pass of the hot path over the batch:
schedule (device radix sort into 4-pair wave groups) -> fp32 forward kernel ->
fp64 rescue kernel.  `value` = total cells (sum of R*H) of all ranks * steps /
max-over-ranks wall time, in GCUPS.

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set)
this process is one rank; `--gpus N` without WORLD_SIZE starts the N rank
processes itself (fresh children, before this parent touches the GPU) and
relays rank 0's line.  Every rank processes its own 1M-pair shard (weak
scaling, static partition, no data-path collective — SURVEY.md §8e);
torch.distributed carries only the barrier and the max-over-ranks timing
reduction.  `--dry-run` runs the same rank/launcher/reduction path on CPU
(gloo) with a stand-in workload, for the CPU tests.

C4 / C5 (configs[3], configs[4]) as the reference runs them: ONE `fcs-genome
htc` job and ONE `fcs-genome mutect2` job over a chr1-sized genome (--c4-mbp,
248 Mbp, the same at every N), their 32 interval shards dealt over all N GPUs
of the node; at N = 1 beside each job's CPU PairHMM path.  The line ends with
`summary`, every headline figure in one short block.

Also reported (not the headline): banded-SW ksw_extend2 GCUPS on C3-shaped
synthetic extension tasks (2x151 bp reads, bwa defaults) and on the fixed
qlen=151/tlen=251 variant, cells counted by the kernel exactly as ksw_extend2
evaluates them; and the CPU baseline (the oracle restatement, OpenMP) on a
bounded sample, rank 0 / N=1 only.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "falcon-genome_amd"))
fcship = None  # the C-ABI binding, loaded by main() after the rank launcher (no HIP before the children start)

METRIC = "PairHMM GCUPS + banded-SW GCUPS per GPU; end-to-end htc regions/sec at 8 GPUs"
FLOPS_PER_CELL = 11          # M 5 + I 3 + D 3 (FMA = 2)
VALU_LANE_INSTR_PEAK = 256 * 4 * 32 * 2.4e9  # lane-instructions/s: one wave64 VALU op per 2 cycles per SIMD
FP32_VECTOR_PEAK_TF = 157.3  # MI355X_MICROARCH.md chip table (spec)
HBM_PEAK_GBS = 8000.0
SW_OPS_PER_CELL = 12         # BASELINE.md §3 / SURVEY §8d: ~12 int ops per ksw_extend2 cell


def progress(msg):
    """A progress line on stderr (a long bench run keeps showing signs of life;
    stdout carries only the JSON line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def phmm_dev_batch(p: "fcship.PhmmPairs", dev):
    keep = {}
    for k in ("read_bases", "read_bq", "read_iq", "read_dq", "read_gcp", "read_off", "read_len", "hap_bases",
              "hap_off", "hap_len", "pair_read", "pair_hap"):
        keep[k] = torch.from_numpy(np.ascontiguousarray(getattr(p, k))).to(dev)
    b = p.to_struct()
    for k, t in keep.items():
        setattr(b, k, t.data_ptr())
    return b, keep


def bsw_dev_batch(t: "fcship.BswTasks", dev):
    keep = {}
    for k in ("qbuf", "qoff", "qlen", "tbuf", "toff", "tlen", "h0", "w"):
        keep[k] = torch.from_numpy(np.ascontiguousarray(getattr(t, k))).to(dev)
    b = t.to_struct()
    for k, v in keep.items():
        setattr(b, k, v.data_ptr())
    return b, keep


def load_pmc_phmm():
    """Measured issue counters of the fp32 forward pass (profiles/pmc_phmm.json,
    written by tools/profile_summary.py from rocprofv3 --pmc passes)."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_phmm.json")) as f:
            d = json.load(f)
        return d["phmm_fwd_fp32"], d.get("source")
    except (OSError, ValueError, KeyError):
        return {}, None


def fetch_factor():
    """HBM read bytes per FETCH_SIZE byte on gfx950, measured by
    tools/micro/fetch_calib.hip (profiles/fetch_calibration.json): 2."""
    try:
        with open(os.path.join(ROOT, "profiles", "fetch_calibration.json")) as f:
            return 1.0 / float(json.load(f)["fetch_size_fraction_of_bytes"])
    except (OSError, ValueError, KeyError):
        return 1.0


def load_traffic(name):
    """Per-launch HBM bytes of a kernel from a committed rocprofv3 PMC summary:
    fetch_factor() x FETCH_SIZE + WRITE_SIZE."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if name == "phmm_fwd_fp32" and "fetch_kib" in t and "write_kib" in t:
        return int(round((fetch_factor() * t["fetch_kib"] + t["write_kib"]) * 1024))
    return t.get(name)


def bench_phmm(args, dev, rk):
    p = fcship.synth_phmm(args.seed + 7919 * rk.rank, args.pairs, R=101, hmin=150, hmax=300)
    cells = p.cells()
    b, keep = phmm_dev_batch(p, dev)
    out = torch.empty(p.n_pairs, dtype=torch.float64, device=dev)
    plan = fcship.C.c_void_p()
    fcship.check(fcship.lib.fcs_phmm_plan_create(dev.index, p.n_pairs, fcship.C.byref(plan)))
    opts = fcship.phmm_opts(device=dev.index)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    B, O = fcship.C.byref(b), fcship.C.byref(opts)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        fcship.check(fcship.lib.fcs_phmm_dev_schedule(plan, B, sp))
        if ev is not None:
            ev[1].record(stream)
        fcship.check(fcship.lib.fcs_phmm_dev_forward(plan, B, out.data_ptr(), O, sp))
        if ev is not None:
            ev[2].record(stream)
        fcship.check(fcship.lib.fcs_phmm_dev_rescue(plan, B, out.data_ptr(), O, sp))
        if ev is not None:
            ev[3].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    rk.barrier()
    torch.cuda.synchronize(dev)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize(dev)
    rk.barrier()
    t1 = time.perf_counter()
    elapsed = rk.max(t1 - t0)[0]
    sched_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    fwd_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    resc_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in evs]))
    nres = fcship.C.c_int64()
    fcship.check(fcship.lib.fcs_phmm_plan_rescue_count(plan, sp, fcship.C.byref(nres)))
    res = out.cpu().numpy()
    fcship.lib.fcs_phmm_plan_destroy(plan)
    del keep
    return dict(p=p, cells=cells, elapsed=elapsed, sched_ms=sched_ms, fwd_ms=fwd_ms, resc_ms=resc_ms,
                n_rescued=int(nres.value), out=res)


def bench_bsw(args, dev, tasks, reps=3):
    b, keep = bsw_dev_batch(tasks, dev)
    res = torch.empty((tasks.n, 6), dtype=torch.int32, device=dev)
    cells = torch.empty(tasks.n, dtype=torch.int64, device=dev)
    params = fcship.bsw_params()
    stream = torch.cuda.current_stream(dev)
    plan = fcship.C.c_void_p()
    fcship.check(fcship.lib.fcs_bsw_plan_create(dev.index, tasks.n, fcship.C.byref(plan)))
    run = lambda: fcship.check(fcship.lib.fcs_bsw_extend_plan(plan, fcship.C.byref(b), fcship.C.byref(params),  # noqa
                                                              res.data_ptr(), cells.data_ptr(), stream.cuda_stream))
    run()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        run()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    ncell = int(cells.sum().item())
    fcship.lib.fcs_bsw_plan_destroy(plan)
    del keep
    return dict(ms=ms, cells=ncell, gcups=ncell / (ms * 1e-3) / 1e9, tasks=tasks.n,
                bytes=int(tasks.qbuf.size + tasks.tbuf.size + 24 * tasks.n),
                res=res.cpu().numpy(), cell_counts=cells.cpu().numpy())


def bench_bsw_global(args, dev, tasks, reps=3):
    """ksw_global2 (the CIGAR pass of bwa_gen_cigar2) on device-resident tasks:
    scores only, then scores + direction matrix + traceback.  Cells = the band
    cells bwa's ksw_global2 evaluates: per target row i, columns
    [max(0, i - w), min(qlen, i + w + 1))."""
    b, keep = bsw_dev_batch(tasks, dev)
    n = tasks.n
    params = fcship.bsw_params()
    stream = torch.cuda.current_stream(dev)
    scores = torch.empty(n, dtype=torch.int32, device=dev)
    ncol = np.minimum(tasks.qlen.astype(np.int64), 2 * tasks.w.astype(np.int64) + 1)
    zsz = ncol * tasks.tlen
    zoff = torch.from_numpy(np.concatenate([[0], np.cumsum(zsz)[:-1]]).astype(np.int64)).to(dev)
    zbuf = torch.empty(int(zsz.sum()), dtype=torch.uint8, device=dev)
    cap = (tasks.qlen + tasks.tlen + 2).astype(np.int32)
    coff = torch.from_numpy(np.concatenate([[0], np.cumsum(cap.astype(np.int64))[:-1]]).astype(np.int64)).to(dev)
    ccap = torch.from_numpy(cap).to(dev)
    cig = torch.empty(int(cap.astype(np.int64).sum()), dtype=torch.int32, device=dev)
    ncig = torch.empty(n, dtype=torch.int32, device=dev)
    B, P = fcship.C.byref(b), fcship.C.byref(params)
    cells = 0
    shapes, counts = np.unique(np.stack([tasks.qlen, tasks.tlen, tasks.w], 1), axis=0, return_counts=True)
    for (q, t, w), c in zip(shapes.tolist(), counts.tolist()):
        i = np.arange(t)
        cells += c * int(np.maximum(0, np.minimum(q, i + w + 1) - np.maximum(0, i - w)).sum())
    out = {}
    for name, with_cigar in (("scores", False), ("cigar", True)):
        def run():
            if with_cigar:
                fcship.check(fcship.lib.fcs_bsw_global_dev(B, P, scores.data_ptr(), zbuf.data_ptr(), zbuf.numel(),
                                                           zoff.data_ptr(), cig.data_ptr(), coff.data_ptr(),
                                                           ccap.data_ptr(), ncig.data_ptr(), dev.index,
                                                           stream.cuda_stream))
            else:
                fcship.check(fcship.lib.fcs_bsw_global_dev(B, P, scores.data_ptr(), None, 0, None, None, None, None,
                                                           None, dev.index, stream.cuda_stream))
        run()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            run()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / reps
        out[name] = dict(ms=round(ms, 3), gcups=round(cells / (ms * 1e-3) / 1e9, 3))
    del keep
    return dict(tasks=n, w=int(tasks.w[0]) if n else 0, cells=cells, **out)


def shard_stats(logs, dt):
    """Per-shard caller lines summed over the shards (workers/*.cpp): counts,
    and the stage times as thread-seconds (shards run concurrently)."""
    import re
    tot = lambda pat, f=float: sum(f(x) for x in re.findall(pat, logs))  # noqa: E731
    st = {"regions": tot(r"(\d+) regions", int), "pairs": tot(r"(\d+) pairs", int),
          "cells": tot(r"(\d+) cells", int), "rescued_pairs": tot(r"(\d+) rescued", int),
          "device_passes": tot(r"(\d+) device passes", int),
          "shards_run_while_device_came_up": tot(r"ran (\d+) queued shards", int),
          "seconds": round(dt, 3)}
    st["regions_per_s"] = round(st["regions"] / dt, 1)
    brk = {k: round(tot(pat), 3) for k, pat in (
        ("decode", r"decode ([\d.]+) s"), ("pileup", r"pileup ([\d.]+) s"),
        ("regions", r"regions ([\d.]+) s\b"), ("phmm_call", r"PairHMM ([\d.]+) s"),
        ("genotype", r"genotype ([\d.]+) s"), ("output", r"output ([\d.]+) s"))}
    st["stage_thread_seconds"] = brk
    dev, res = tot(r"device ([\d.]+) s"), tot(r"rescue ([\d.]+) s")
    st["phmm_device_seconds"] = round(dev, 4)
    st["rescue_fp64_device_seconds"] = round(res, 4)
    st["gpu_busy_frac"] = round(dev / dt, 4)  # PairHMM device time (HIP events) / wall time, one GPU
    # cells over the passes' summed HIP-event spans: with passes merged across
    # shards (gpu.phmm.combine_ms) the spans no longer overlap, so this is the
    # device-effective PairHMM rate
    st["phmm_device_tcups"] = round(st["cells"] / dev / 1e12, 3) if dev > 0 else None
    st["effective_gcups"] = round(st["cells"] / dt / 1e9, 2)
    return st


def cpu_mock_env(env):
    """Environment of an fcs-genome child that runs the reference's CPU
    PairHMM path: tests/cpu_mock/build/libfcship.so (test infrastructure: the
    oracle's Java-semantics or GKL-style AVX-512 PairHMM behind the same
    C-ABI) first on its LD_LIBRARY_PATH.  Only that child sees it.  Shard
    passes are not merged (gpu.phmm.combine_ms = 0): on the CPU path each
    shard thread computes its own PairHMM batches, as GATK's per-shard
    HaplotypeCaller processes do; a merged pass would run on one thread."""
    import subprocess
    mock = os.path.join(ROOT, "tests", "cpu_mock", "build")
    if not os.path.exists(os.path.join(mock, "libfcship.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpu_mock")], check=True, capture_output=True)
    return dict(env, LD_LIBRARY_PATH=mock + os.pathsep + env.get("LD_LIBRARY_PATH", ""), FCS_GPU_PHMM_COMBINE_MS="0")


_VCF_CALLS = {}


def vcf_calls(path):
    """(chrom, pos, ref, alt) of the variant records of a VCF or GVCF (GVCF
    reference blocks and the <NON_REF> allele left out).  Cached per file
    version: a 248 Mbp GVCF takes ~15 s to scan, and the C4 leg compares the
    GPU job's output with its CPU path's."""
    st = os.stat(path)
    key = (os.path.abspath(path), st.st_mtime_ns, st.st_size)
    if key in _VCF_CALLS:
        return _VCF_CALLS[key]
    out = set()
    with open(path, "rb") as fh:
        for ln in fh:
            if ln.startswith(b"#"):
                continue
            f = ln.split(b"\t", 5)
            if f[4] == b"<NON_REF>":  # a GVCF reference block
                continue
            alts = [a for a in f[4].decode().split(",") if a != "<NON_REF>"]
            if alts:
                out.add((f[0].decode(), int(f[1]), f[3].decode(), ",".join(alts)))
    _VCF_CALLS[key] = out
    return out


def caller_cpu_baseline(exe, env, work, cmd, gpu_out, modes=("gkl", "java"), tag="c4", ext=".g.vcf"):
    """An `fcs-genome htc` / `mutect2` command with the PairHMM on the host
    CPU: the reference's CPU path (GATK HaplotypeCaller / Mutect2 with
    --native-pair-hmm-threads, /root/reference/src/workers/HTCWorker.cpp:85,105,
    Mutect2Worker.cpp:109-192), same command, genome and shard threads as the
    GPU run: gkl = GKL's AVX-512 float PairHMM with the double rescue restated,
    java = GATK's Java LoglessPairHMM (double).  cmd(out_path) gives the
    arguments.  Calls compared with the GPU run's output."""
    import shutil
    import subprocess
    cenv = cpu_mock_env(env)
    gpu_calls = vcf_calls(gpu_out)
    res = {}
    for m in modes:
        o = os.path.join(work, f"cpu_{tag}_{m}{ext}")
        logd = os.path.join(work, f"log_cpu_{tag}_{m}")
        shutil.rmtree(logd, ignore_errors=True)
        e = dict(cenv, FCS_MOCK_PHMM=m, FCS_LOG_DIR=logd)
        t0 = time.perf_counter()
        r = subprocess.run([exe, *cmd(o)], env=e, capture_output=True, text=True, cwd=work)
        dt = time.perf_counter() - t0
        if r.returncode != 0:
            raise RuntimeError(f"CPU-path {tag} ({m}) failed ({r.returncode}): {r.stderr[-2000:]}")
        logs = "".join(open(os.path.join(logd, f)).read() for f in os.listdir(logd) if ".part-" not in f)
        st = shard_stats(logs, dt)
        for k in ("phmm_device_seconds", "rescue_fp64_device_seconds", "gpu_busy_frac", "device_passes",
                  "phmm_device_tcups"):
            st.pop(k, None)
        c = vcf_calls(o)
        st.update(kind="port", cores=int(env.get("FCS_GATK_NPROCS", "16")),
                  pairhmm={"gkl": "GKL-style AVX-512 restatement (float pass, double rescue below 1e-28), one "
                                  "shard thread per region batch",
                           "java": "GATK Java LoglessPairHMM semantics (double), scalar, one shard thread per "
                                   "region batch"}[m],
                  calls=len(c), calls_equal_to_gpu=c == gpu_calls,
                  calls_only_gpu=len(gpu_calls - c), calls_only_cpu=len(c - gpu_calls))
        res[m] = st
    return res


def htc_cpu_baseline(exe, env, work, ref, bam, gpu_out, modes=("gkl", "java"), vcf=False, tag="c4"):
    """`fcs-genome htc` on the reference's CPU PairHMM path (caller_cpu_baseline)."""
    return caller_cpu_baseline(exe, env, work, lambda o: ["htc", "-f", "-r", ref, "-i", bam, "-o", o] +
                               (["-v"] if vcf else []), gpu_out, modes, tag, ".vcf" if vcf else ".g.vcf")


def damage_mates(fastq, every=25, offset=7):
    """A mismatch every 16 bases in every `every`-th read of `fastq` (4% at
    25): no 19-mer seed survives in them, so only the mate rescue (bwa
    mem_matesw, the GPU ksw_align2) can place them.  Returns how many."""
    flip = {"A": "C", "C": "G", "G": "T", "T": "A", "N": "A"}
    lines = open(fastq).read().split("\n")
    n = 0
    for i in range(0, len(lines) - 3, 4):
        if (i // 4) % every == offset:
            seq = list(lines[i + 1])
            for j in range(5, len(seq), 16):
                seq[j] = flip[seq[j]]
            lines[i + 1] = "".join(seq)
            n += 1
    open(fastq, "w").write("\n".join(lines))
    return n


def bam_payload(path):
    """The decompressed bytes of a BAM (BGZF blocks are gzip members): equal
    payloads mean the same header and the same records in the same order."""
    import gzip
    return gzip.decompress(open(path, "rb").read())


def align_cpu_baseline(exe, env, work, cmd, gpu_bam, threads):
    """`fcs-genome align` with the banded Smith-Waterman on the host CPU: the
    reference's `bwa-flow mem` without --use_fpga
    (/root/reference/src/workers/BWAWorker.cpp:134-166), i.e. bwa's scalar
    ksw_extend2 / ksw_global2 and its SSE2 striped ksw_align2 (restated in
    oracle/ksw_oracle.c, oracle/ksw_align_sse.c) on `threads` OpenMP threads
    per batch, the same binary, seeding, pairing and output around them.  The
    BAM must equal the GPU run's."""
    import subprocess
    out = os.path.join(work, "aln_cpu.bam")
    e = dict(cpu_mock_env(env), FCS_MOCK_BSW_THREADS=str(threads))
    t0 = time.perf_counter()
    r = subprocess.run([exe, *cmd(out)], env=e, capture_output=True, text=True, cwd=work)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"CPU-path align failed ({r.returncode}): {r.stderr[-2000:]}")
    rep = align_report(r.stderr)
    return {"seconds": round(dt, 3), "reads_per_s": round(rep["reads"] / dt, 1), "kind": "port", "cores": threads,
            "sw": "bwa's ksw_extend2 / ksw_global2 (scalar C, as bwa's) and ksw_align2 (SSE2 striped, 16 x u8 / "
                  "8 x i16 lanes, as bwa's) restated, OpenMP over each batch's tasks",
            "sw_call_seconds": rep["gpu_call_seconds"], "thread_seconds": rep["thread_seconds"],
            "mates_rescued": rep["mates_rescued"],
            "bam_equal_to_gpu": bam_payload(out) == bam_payload(gpu_bam)}


def align_report(err):
    """The counters and phase times `fcs-genome align` prints."""
    import re
    m = re.search(r"(\d+) reads, (\d+) mapped, (\d+) supplementary, (\d+) extension tasks, (\d+) global "
                  r"alignments, ([\d.]+) s \(GPU calls ([\d.]+) s\)", err)
    pm = re.search(r"(\d+) reads properly paired, (\d+) mates rescued, insert ([\d.]+) \+- ([\d.]+)", err)
    ph = re.search(r"alignment thread-seconds ([\d.]+): seeding ([\d.]+), extension ([\d.]+), pairing ([\d.]+), "
                   r"records ([\d.]+)", err)
    wp = re.search(r"phases: reference ([\d.e-]+) s, FMD index ([\d.e-]+) s .*FASTQ \+ alignment ([\d.e-]+) s .*"
                   r"sort \+ BAM \+ index ([\d.e-]+) s", err)
    if not (m and pm and ph and wp):
        raise RuntimeError("fcs-genome align report not understood: " + err[-2000:])
    return {"reads": int(m.group(1)), "mapped": int(m.group(2)), "supplementary": int(m.group(3)),
            "ext_tasks": int(m.group(4)), "global_tasks": int(m.group(5)), "gpu_call_seconds": float(m.group(7)),
            "thread_seconds": {k: float(ph.group(i + 1)) for i, k in
                               enumerate(("total", "seeding", "extension", "pairing", "records"))},
            "wall_phases_seconds": {k: float(wp.group(i + 1)) for i, k in
                                    enumerate(("reference", "fmd_index", "fastq_and_alignment", "sort_bam_index"))},
            "proper_pair_reads": int(pm.group(1)), "mates_rescued": int(pm.group(2))}


def synth_job_genome(exe, env, d, mbp, seed, tumor=True):
    """The C4/C5 input: a chr1-like genome of mbp Mbp (248 is chr1), a 30x
    sample BAM and, with tumor, a 40x tumor BAM (+1e-4 somatic); 1% of the
    reads mis-mapped-like, so the fp64 rescue fires.  Returns seconds."""
    import subprocess
    t0 = time.perf_counter()
    subprocess.run([exe, "synth", "-o", d, "-c", f"chr1:{int(mbp * 1e6)}", "-x", "30", "--no-fastq", "--noisy-frac",
                    "0.01", "--seed", str(seed)] + (["--tumor"] if tumor else []), env=env, check=True,
                   capture_output=True)
    return time.perf_counter() - t0


JOB_TOOLS = {
    # tool -> (config, Stage name, reference driver)
    "htc": ("C4", "Haplotype Caller", "/root/reference/src/worker-htc.cpp:113-145"),
    "mutect2": ("C5", "Mutect2", "/root/reference/src/worker-mutect2.cpp:167-201"),
}


def job_cmd(tool, d, out):
    """The fcs-genome command line of one C4 (htc, GVCF) or C5 (mutect2
    tumor/normal) job over the genome directory d."""
    if tool == "htc":
        return ["htc", "-f", "-r", d + "/ref.fasta", "-i", d + "/sample.bam", "-o", out]
    return ["mutect2", "-f", "-r", d + "/ref.fasta", "-t", d + "/tumor.bam", "-n", d + "/sample.bam", "-o", out]


def bench_job(exe, env, work, d, tool, mbp, n_dev, nprocs, reps=1):
    """BASELINE.json configs[3] (C4: htc) or configs[4] (C5: mutect2) as the
    reference runs them: ONE fcs-genome job over the genome in d, its
    gatk.ncontigs = 32 interval shards in one stage (the reference's one
    Executor per job, JOB_TOOLS[tool][2]; the shard unit of
    src/config.cpp:470-509) dealt round-robin to the GPU slots 0..n_dev-1
    (gpu.devices[job_id % n], the host round-robin of src/Executor.cpp:262),
    nprocs shard threads.  Returns the shard statistics, wall time and the
    per-device shard counts; the job's output is work/<c4|c5>.<ext>."""
    import re
    import shutil
    import subprocess
    cfg, stage, _ = JOB_TOOLS[tool]
    tag = cfg.lower()
    logd = os.path.join(work, "log_" + tag)
    e = dict(env, FCS_GPU_DEVICES=",".join(str(i) for i in range(n_dev)), FCS_LOG_DIR=logd,
             FCS_GATK_NPROCS=str(nprocs))
    out = os.path.join(work, tag + (".g.vcf" if tool == "htc" else ".vcf"))
    runs = []
    for _ in range(max(1, reps)):
        shutil.rmtree(logd, ignore_errors=True)
        t0 = time.perf_counter()
        r = subprocess.run([exe, *job_cmd(tool, d, out)], env=e, capture_output=True, text=True, cwd=work)
        dt = time.perf_counter() - t0
        if r.returncode != 0:
            raise RuntimeError(f"{cfg} {tool} failed ({r.returncode}): {r.stderr[-2000:]}")
        logs = "".join(open(os.path.join(logd, f)).read() for f in os.listdir(logd) if ".part-" not in f)
        runs.append((dt, logs, r.stderr))
    dt, logs, err = min(runs, key=lambda x: x[0])
    st = shard_stats(logs, dt)
    st["runs_seconds"] = [round(x[0], 3) for x in runs]
    st["devices"] = n_dev
    st["shard_threads"] = nprocs
    st["genome_mbp"] = mbp
    st["shards_per_device"] = {str(k): len(re.findall(rf"\] shard \d+ gpu {k}\b", logs)) for k in range(n_dev)}
    m = re.search(stage + r" finishes in ([\d.]+) seconds", err)
    st["caller_stage_seconds"] = float(m.group(1)) if m else None
    st["calls"] = len(vcf_calls(out))
    st["output"] = out
    st["workload"] = (f"{cfg}: one fcs-genome {tool} " + ("(GVCF) over a " if tool == "htc" else "(tumor 40x / normal "
                      "30x) over a ") + f"{mbp:g} Mbp chr1-like genome, 32 interval shards dealt to {n_dev} GPU "
                      f"slot(s), {nprocs} shard threads")
    return st


def bench_c4(exe, env, work, mbp, n_dev, seed, nprocs, reps=1, tools=("htc",)):
    """One genome synthesised (tumor BAM too when mutect2 is asked for), then
    one bench_job per tool on it; {tool: stats}.  The genome is removed."""
    import shutil
    d = os.path.join(work, "c4")
    synth_s = synth_job_genome(exe, env, d, mbp, seed, tumor="mutect2" in tools)
    try:
        out = {}
        for t in tools:
            out[t] = bench_job(exe, env, work, d, t, mbp, n_dev, nprocs, reps)
            out[t]["synth_seconds"] = round(synth_s, 1)
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def bench_c1(exe, env, work, seed):
    """BASELINE.json configs[0] (C1): `fcs-genome htc` on a 1,000-read
    synthetic chr20 BAM, on the GPU and through the reference's CPU PairHMM
    path (Java semantics and GKL-style AVX-512), VCF output; wall time of each
    command and whether the calls agree."""
    import subprocess
    c1 = os.path.join(work, "c1")
    subprocess.run([exe, "synth", "-o", c1, "-c", "chr20:1000000", "-x", "30", "-n", "1000", "--no-fastq",
                    "--seed", str(seed)], env=env, check=True, capture_output=True)
    logd = os.path.join(work, "log_c1")
    import shutil
    shutil.rmtree(logd, ignore_errors=True)
    t0 = time.perf_counter()
    r = subprocess.run([exe, "htc", "-f", "-r", c1 + "/ref.fasta", "-i", c1 + "/sample.bam", "-o", work + "/c1.vcf",
                        "-v"], env=dict(env, FCS_LOG_DIR=logd), capture_output=True, text=True, cwd=work)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"C1 htc failed ({r.returncode}): {r.stderr[-2000:]}")
    logs = "".join(open(os.path.join(logd, f)).read() for f in os.listdir(logd) if ".part-" not in f)
    gpu = shard_stats(logs, dt)
    gpu["calls"] = len(vcf_calls(work + "/c1.vcf"))
    out = {"workload": "C1: fcs-genome htc -v on a 1,000-read synthetic chr20 BAM (chr20-like 1 Mbp reference, "
                       "the first 1,000 reads of a 30x sample)", "gpu": gpu}
    out["cpu_baseline"] = htc_cpu_baseline(exe, env, work, c1 + "/ref.fasta", c1 + "/sample.bam", work + "/c1.vcf",
                                           modes=("java", "gkl"), vcf=True, tag="c1")
    return out


def bench_e2e(args, rank, local):
    """End-to-end fcs-genome commands on this rank's own synthetic genome
    (C4/C5-shaped: a chr1-like random reference of --e2e-mbp per GPU — 31 Mbp
    is chr1 / 8, the C4 per-GPU share — a 30x sample, a 40x tumor with somatic
    variants; weak scaling, one GPU per rank), and align on a separate
    --e2e-align-mbp genome.  Wall time of each command as a user runs it
    (process start, BAM decode, pileup, PairHMM on the GPU, VCF tail)."""
    import re
    import shutil
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "falcon-genome_amd", "bin", "fcs-genome")
    work = tempfile.mkdtemp(prefix=f"fcs-e2e-{rank}-")
    # the ranks of one node share its CPUs: each command's host threads (VCF /
    # BAM codec pool, aligner slots) get this rank's share of the CPU quota
    per_rank = max(2, host_cpu_quota() // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1"))))
    env = dict(os.environ, FCS_GPU_DEVICES=str(local), FCS_LOG_DIR=os.path.join(work, "log"),
               FCS_TEMP_DIR=work, FCS_GATK_NPROCS="16", FCS_HOST_THREADS=str(per_rank))
    cpu_htc = rank == 0 and int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.no_cpu_baseline
    try:
        L = int(args.e2e_mbp * 1e6)
        t0 = time.perf_counter()
        subprocess.run([exe, "synth", "-o", work + "/d", "-c", f"chr1:{L}", "-x", "30", "--tumor", "--no-fastq",
                        "--noisy-frac", "0.01", "--seed", str(args.seed + rank)], env=env, check=True,
                       capture_output=True)
        synth_s = time.perf_counter() - t0
        out = {"data": f"synthetic chr1-like {args.e2e_mbp:g} Mbp per GPU (chr1 / 8 = the C4 per-GPU share at 31), "
                       "sample 30x, tumor 40x (+1e-4 somatic), 1% of reads mis-mapped-like (20% high-quality "
                       "mismatches: their pairs reach the fp64 rescue)",
               "synth_seconds": round(synth_s, 1)}
        def timed(name, cmd):
            shutil.rmtree(env["FCS_LOG_DIR"], ignore_errors=True)
            t0 = time.perf_counter()
            r = subprocess.run([exe, *cmd], env=env, capture_output=True, text=True, cwd=work)
            dt = time.perf_counter() - t0
            if r.returncode != 0:
                raise RuntimeError(f"fcs-genome {name} failed ({r.returncode}): {r.stderr[-2000:]}")
            logs = ""
            for f in (os.listdir(env["FCS_LOG_DIR"]) if os.path.isdir(env["FCS_LOG_DIR"]) else []):
                if ".part-" not in f:
                    logs += open(os.path.join(env["FCS_LOG_DIR"], f)).read()
            return dt, logs, r.stderr
        d = work + "/d"

        def best(name, cmd):
            """Best of --e2e-reps runs (the first run of a fresh box also pays page-in
            and clock ramp; every run's wall time is reported)."""
            runs = [timed(name, cmd) for _ in range(max(1, args.e2e_reps))]
            return min(runs, key=lambda r: r[0]), [round(r[0], 3) for r in runs]

        def stage_s(err, name):
            m = re.search(name + r" finishes in ([\d.]+) seconds", err)
            return float(m.group(1)) if m else None

        (dt, logs, err), runs = best("htc", ["htc", "-f", "-r", d + "/ref.fasta", "-i", d + "/sample.bam", "-o",
                                             work + "/htc.g.vcf"])
        out["htc"] = shard_stats(logs, dt)
        out["htc"]["runs_seconds"] = runs
        out["htc"]["output"] = "GVCF (the reference's default)"
        hs = stage_s(err, "Haplotype Caller")
        out["htc"]["caller_stage_seconds"] = hs  # the 32-shard stage alone: no process start, GPU init, concat
        out["htc"]["caller_stage_regions_per_s"] = round(out["htc"]["regions"] / hs, 1) if hs else None
        # the same command with concurrent shards' PairHMM passes merged per
        # device (gpu.phmm.combine_ms, off by default): fewer, larger device
        # passes, reported for their device-effective rate and wall time
        env_m = dict(env, FCS_GPU_PHMM_COMBINE_MS="20")
        shutil.rmtree(env["FCS_LOG_DIR"], ignore_errors=True)
        t0 = time.perf_counter()
        r = subprocess.run([exe, "htc", "-f", "-r", d + "/ref.fasta", "-i", d + "/sample.bam", "-o",
                            work + "/htc_m.g.vcf"], env=env_m, capture_output=True, text=True, cwd=work)
        dtm = time.perf_counter() - t0
        if r.returncode == 0:
            logs_m = "".join(open(os.path.join(env["FCS_LOG_DIR"], f)).read() for f in os.listdir(env["FCS_LOG_DIR"])
                             if ".part-" not in f)
            sm = shard_stats(logs_m, dtm)
            out["htc"]["merged_passes"] = {k: sm[k] for k in ("seconds", "device_passes", "phmm_device_seconds",
                                                                 "phmm_device_tcups")}
            out["htc"]["merged_passes"]["setting"] = "gpu.phmm.combine_ms = 20"
        if cpu_htc:  # the reference's CPU path beside it, on the same genome (rank 0, N=1 only)
            out["htc"]["cpu_baseline"] = htc_cpu_baseline(exe, env, work, d + "/ref.fasta", d + "/sample.bam",
                                                          work + "/htc.g.vcf")
        progress("e2e: mutect2")
        m2_cmd = lambda o: ["mutect2", "-f", "-r", d + "/ref.fasta", "-t", d + "/tumor.bam", "-n",  # noqa: E731
                            d + "/sample.bam", "-o", o]
        (dt, logs, err), runs = best("mutect2", m2_cmd(work + "/m2.vcf"))
        out["mutect2"] = shard_stats(logs, dt)
        out["mutect2"]["runs_seconds"] = runs
        ms = stage_s(err, "Mutect2")
        out["mutect2"]["caller_stage_seconds"] = ms
        out["mutect2"]["caller_stage_regions_per_s"] = round(out["mutect2"]["regions"] / ms, 1) if ms else None
        if cpu_htc:  # C5's CPU path: GATK Mutect2 with the CPU PairHMM, same command and genome
            out["mutect2"]["cpu_baseline"] = caller_cpu_baseline(exe, env, work, m2_cmd, work + "/m2.vcf",
                                                                 tag="c5", ext=".vcf")
        progress("e2e: BGZF inflate")
        try:
            out["bgzf"] = bench_bgzf(d + "/sample.bam", local, cpu_htc)
        except Exception as e:  # reported, not fatal to the e2e line
            out["bgzf"] = {"error": repr(e)[:300]}
        shutil.rmtree(d, ignore_errors=True)
        if cpu_htc:
            progress("e2e: C1")
            out["c1"] = bench_c1(exe, env, work, args.seed + rank)
        progress("e2e: align")
        La = int(args.e2e_align_mbp * 1e6)
        subprocess.run([exe, "synth", "-o", work + "/a", "-c", f"chr1:{La}", "-x", "30", "--no-fastq", "--paired",
                        "350", "--seed", str(args.seed + rank)], env=env, check=True, capture_output=True)
        a = work + "/a"
        # 4% of the read-2 mates damaged past seeding: only the mate rescue
        # (bwa mem_matesw on the GPU ksw_align2) can place them
        n_damaged = damage_mates(a + "/sample_2.fastq")
        # bwa-flow maps a prebuilt index (bwa index): built once here, outside the timed runs
        ti = time.perf_counter()
        subprocess.run([exe, "index", "-r", a + "/ref.fasta", "--sa-intv", "32"], env=env, check=True,
                       capture_output=True)
        index_s = time.perf_counter() - ti
        al_cmd = lambda o: ["align", "-f", "-r", a + "/ref.fasta", "-1", a + "/sample_1.fastq", "-2",  # noqa: E731
                            a + "/sample_2.fastq", "-o", o]
        (dt, _, err), runs = best("align", al_cmd(work + "/aln.bam"))
        rep = align_report(err)
        n = rep["reads"]
        out["align"] = dict(mode=f"paired-end 2x151, fragments N(350, 50), {args.e2e_align_mbp:g} Mbp genome, 30x "
                                 f"of pairs; {n_damaged} read-2 mates (4%) carry a mismatch every 16 bases, so only "
                                 "the mate rescue places them", damaged_mates=n_damaged, **rep)
        out["align"].update(index="prebuilt by fcs-genome index --sa-intv 32 (untimed, %.1f s), mapped by align"
                                  % index_s, seconds=round(dt, 3), runs_seconds=runs, reads_per_s=round(n / dt, 1))
        if cpu_htc:  # bwa-flow mem without --use_fpga: the SW on the host cores, same binary and threads
            out["align"]["cpu_baseline"] = align_cpu_baseline(exe, env, work, al_cmd, work + "/aln.bam", per_rank)
        return out
    finally:
        shutil.rmtree(work, ignore_errors=True)


def bench_bgzf(bam, dev_index, cpu, reps=3):
    """the e2e sample BAM (the host's BgzfWriter,
    libdeflate level 5) inflated whole on the GPU (fcs_bgzf_inflate_dev, one
    wave per member) with the file already in HBM; parity = every member's
    status OK and a spread of members byte-equal to zlib; the CPU baseline is
    libdeflate on one host thread over the first members (the host reader's
    codec)."""
    import ctypes
    import zlib
    import torch
    blob = open(bam, "rb").read()
    coff, uoff, used = fcship.bgzf_index(blob)
    n = len(coff) - 1
    dev = torch.device("cuda", dev_index)
    comp = torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).to(dev)
    dco, duo = torch.from_numpy(coff).to(dev), torch.from_numpy(uoff).to(dev)
    out = torch.empty(int(uoff[-1]), dtype=torch.uint8, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)

    def run():
        fcship.check(fcship.lib.fcs_bgzf_inflate_dev(comp.data_ptr(), dco.data_ptr(), duo.data_ptr(), n,
                                                     out.data_ptr(), st.data_ptr(), dev_index,
                                                     ctypes.c_void_p(s.cuda_stream)))
    run()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        run()
    e1.record(s)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    ok = bool((st.cpu().numpy() == 0).all())
    o = out.cpu().numpy()
    picks = sorted(set(np.linspace(0, n - 1, min(n, 64)).astype(int).tolist()))
    same = all(o[uoff[k]:uoff[k + 1]].tobytes() ==
               zlib.decompress(blob[coff[k] + 18:coff[k + 1] - 8], -15) for k in picks)
    tot_out, tot_in = int(uoff[-1]), int(used)
    r = {"workload": "the htc e2e sample BAM (fcs-genome synth, BgzfWriter at libdeflate level 5), every member "
                     "inflated in one fcs_bgzf_inflate_dev call, the file resident in HBM",
         "members": n, "comp_bytes": tot_in, "out_bytes": tot_out, "kernel_ms": round(ms, 3),
         "out_GBps": round(tot_out / ms / 1e6, 2), "in_GBps": round(tot_in / ms / 1e6, 2),
         "parity": {"all_members_ok": ok, "members_checked_vs_zlib": len(picks), "equal": same},
         "roofline": {"bound": "latency (the serial DEFLATE symbol chain: one wave per member, decode state in "
                               "scalar registers, SALU-issue-bound)",
                      "achieved": round((tot_in + tot_out) / ms / 1e6, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round((tot_in + tot_out) / ms / 1e6 / HBM_PEAK_GBS, 5),
                      "algorithmic_bytes_per_launch": tot_in + tot_out,
                      "kernel": "bgzf_inflate_kernel (bgzf_kernels.hip)"}}
    try:  # the kernel's issue counters (SALU-bound: one SALU per cycle per CU)
        pm = json.load(open(os.path.join(ROOT, "profiles", "pmc_bgzf.json")))
        r["roofline"]["counters_per_member"] = pm["per_member"]
        r["roofline"]["counters_source"] = pm["source"]
    except (OSError, ValueError, KeyError):
        pass
    if cpu:
        L = ctypes.CDLL("libdeflate.so.0")
        L.libdeflate_alloc_decompressor.restype = ctypes.c_void_p
        L.libdeflate_deflate_decompress.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t,
                                                    ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        d = L.libdeflate_alloc_decompressor()
        buf = ctypes.create_string_buffer(65536)
        k, done, t0 = 0, 0, time.perf_counter()
        while k < n and time.perf_counter() - t0 < 3.0:
            raw = blob[coff[k] + 18:coff[k + 1] - 8]
            if L.libdeflate_deflate_decompress(d, raw, len(raw), buf, int(uoff[k + 1] - uoff[k]), None) != 0:
                raise RuntimeError("libdeflate failed on member %d" % k)
            done += int(uoff[k + 1] - uoff[k])
            k += 1
        dt = time.perf_counter() - t0
        r["cpu_baseline"] = {"value": round(done / dt / 1e9, 3), "unit": "GB/s inflated", "cores": 1,
                             "kind": "port", "sample": f"libdeflate (the host reader's codec) on one thread over "
                                                       f"the first {k} members ({done} bytes)"}
    del comp, out
    return r


def run_jobs(args, n_dev, cpu):
    """C4 (one htc job) and C5 (one mutect2 job) over ONE genome of
    --c4-mbp (248 = chr1) on this node's n_dev GPUs, in a scratch directory
    (rank 0).  The genome does not depend on N, so the N = 1 run is the anchor
    of the same job at 2/4/8 GPUs (strong scaling of the job).  With cpu (N = 1
    only) each job also runs on the reference's CPU PairHMM path (GKL-style
    AVX-512 through tests/cpu_mock, the same command, shards and threads) and
    the calls are compared."""
    import shutil
    import tempfile
    exe = os.path.join(ROOT, "falcon-genome_amd", "bin", "fcs-genome")
    work = tempfile.mkdtemp(prefix="fcs-c4-")
    quota = host_cpu_quota()
    env = dict(os.environ, FCS_TEMP_DIR=work, FCS_HOST_THREADS=str(quota))
    nprocs = min(32, quota)
    d = os.path.join(work, "g")
    try:
        progress(f"C4/C5: synthesising a {args.c4_mbp:g} Mbp genome (30x sample, 40x tumor)")
        synth_s = synth_job_genome(exe, env, d, args.c4_mbp, args.seed + 4242, tumor=True)
        progress(f"C4/C5: genome ready in {synth_s:.1f} s")
        out = {}
        for tool in ("htc", "mutect2"):
            cfg = JOB_TOOLS[tool][0].lower()
            st = bench_job(exe, env, work, d, tool, args.c4_mbp, n_dev, nprocs, reps=args.c4_reps)
            st["synth_seconds"] = round(synth_s, 1)
            progress(f"{cfg}: {tool} on {n_dev} GPU(s) {st['seconds']:.2f} s")
            if cpu:
                cb = caller_cpu_baseline(exe, dict(env, FCS_GATK_NPROCS=str(nprocs)), work,
                                         lambda o, t=tool: job_cmd(t, d, o), st["output"], modes=("gkl",), tag=cfg,
                                         ext=".g.vcf" if tool == "htc" else ".vcf")["gkl"]
                st["cpu_baseline"] = cb
                st["speedup_vs_cpu_path"] = round(cb["seconds"] / st["seconds"], 3)
                progress(f"{cfg}: {tool} on the CPU path {cb['seconds']:.2f} s")
            st.pop("output")
            out[cfg] = st
        return out
    finally:
        shutil.rmtree(work, ignore_errors=True)


def job_summary(st):
    """The compact figures of a C4/C5 block for the line's summary."""
    if "error" in st:
        return {"error": st["error"]}
    s = {k: st.get(k) for k in ("genome_mbp", "devices", "seconds", "runs_seconds", "regions", "regions_per_s",
                                "caller_stage_seconds", "shards_per_device", "calls", "rescued_pairs",
                                "gpu_busy_frac")}
    cb = st.get("cpu_baseline")
    if cb:
        s["cpu_baseline"] = {"seconds": cb["seconds"], "regions_per_s": cb["regions_per_s"], "cores": cb["cores"],
                             "kind": cb["kind"], "pairhmm": "GKL-style AVX-512", "calls_equal_to_gpu":
                             cb["calls_equal_to_gpu"]}
        s["speedup_vs_cpu_path"] = st.get("speedup_vs_cpu_path")
    return s


def host_cpu_quota():
    """CPUs this process may use: the affinity mask narrowed by a cgroup CPU
    quota (as fcs-genome's host_cpus())."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max" and int(period) > 0:
            n = min(n, max(1, -(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_threads():
    """Host threads for the CPU baselines: the cores this process may run on
    (the box's CPU share: OMP_NUM_THREADS when it is set, else the affinity mask)."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(aff, int(env))) if env.isdigit() and int(env) > 0 else aff


def cpu_baseline_phmm(p, budget_s, threads):
    """GKL-style AVX-512 PairHMM (oracle/pairhmm_simd.c: float in 16-lane
    anti-diagonal stripes, double rescue in 8 lanes, OpenMP over pairs) on the
    leading C2 pairs, best of 5 runs of a sample sized to budget_s / 5.  Falls
    back to the scalar oracle (and says so) on a CPU without AVX-512."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib  # test infrastructure: CPU baseline leg only
    simd = bool(oracle_lib.lib.oracle_phmm_simd_available())
    run = oracle_lib.phmm_simd_batch if simd else oracle_lib.phmm_batch

    def sub(n):
        return fcship.PhmmPairs(p.read_bases, p.read_bq, p.read_iq, p.read_dq, p.read_gcp, p.read_off, p.read_len,
                                p.hap_bases, p.hap_off, p.hap_len, p.pair_read[:n], p.pair_hap[:n])
    cal = sub(min(p.n_pairs, 20 * threads * 64))
    t0 = time.perf_counter()
    run(cal, threads=threads)
    rate = cal.cells() / max(time.perf_counter() - t0, 1e-6)
    n = int(min(p.n_pairs, max(cal.n_pairs, cal.n_pairs * rate * budget_s / 5 / cal.cells())))
    s = sub(n)
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        ref, used_d = run(s, threads=threads)
        times.append(time.perf_counter() - t0)
    best = min(times)
    kind = "GKL-style AVX-512 restatement (float, 16-lane anti-diagonal stripes; double rescue, 8 lanes)" if simd \
        else "scalar C oracle restatement (no AVX-512 on this host)"
    return dict(value=s.cells() / best / 1e9, unit="GCUPS", cores=threads, kind="port",
                sample=f"first {n} of the {p.n_pairs} C2 pairs ({s.cells() / 1e9:.2f} G cells), best of 5 "
                       f"({', '.join(f'{t:.2f}' for t in times)} s); {kind}; OpenMP {threads} threads "
                       f"(nproc {os.cpu_count()})"), ref, used_d


def phmm_parity(gpu, ref, used_d, tol=1e-5):
    """The headline run's own outputs (the last timed step's) against the CPU
    baseline's outputs for the same pairs: |gpu - ref| <= tol * |ref|
    (north_star: log10 likelihoods within 1e-5 of GATK's AVX path).  A pair is
    non-finite-consistent when both sides are the same inf, or both finite."""
    gpu = np.asarray(gpu[:ref.size], np.float64)
    fin = np.isfinite(ref) & np.isfinite(gpu)
    same_inf = ~np.isfinite(ref) & (gpu == ref)
    rel = np.abs(gpu[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1e-300)
    return {"n": int(ref.size), "max_rel_err": float(rel.max()) if rel.size else 0.0,
            "n_over_1e-5": int((rel > tol).sum()), "tolerance": tol,
            "nonfinite_mismatch": int(ref.size - fin.sum() - same_inf.sum()),
            "rescued_by_oracle": int(np.asarray(used_d).sum()),
            "pass": bool((rel <= tol).all() and fin.sum() + same_inf.sum() == ref.size),
            "against": "oracle/pairhmm_simd.c (GKL-style AVX-512 restatement, bit-identical to the scalar oracle)"}


def bench_bsw_align(args, dev, tasks, xtra, reps=3):
    """ksw_align2 (bwa mem_matesw's local SW with score2 and, by KSW_XSTART, the
    reversed start pass) on device-resident tasks.  Cells: the first pass's
    qlen x tlen matrix plus the second pass's (qe + 1) x (te + 1) (it stops at
    the score, at the latest at column te of the reversed target)."""
    b, keep = bsw_dev_batch(tasks, dev)
    n = tasks.n
    params = fcship.bsw_params()
    stream = torch.cuda.current_stream(dev)
    xt = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(np.int32(xtra), (n,)))).to(dev)
    out = torch.empty((n, 7), dtype=torch.int32, device=dev)
    B, P = fcship.C.byref(b), fcship.C.byref(params)

    def run():
        fcship.check(fcship.lib.fcs_bsw_align_dev(B, P, xt.data_ptr(), out.data_ptr(), dev.index,
                                                  stream.cuda_stream))
    run()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        run()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    res = out.cpu().numpy()
    first = int((tasks.qlen.astype(np.int64) * tasks.tlen).sum())
    second = int(((res[:, 2].astype(np.int64) + 1) * (res[:, 1].astype(np.int64) + 1))[res[:, 5] >= 0].sum())
    del keep
    return dict(ms=ms, tasks=n, cells_first=first, cells=first + second, res=res,
                gcups=(first + second) / (ms * 1e-3) / 1e9)


def cpu_baseline_bsw_align(tasks, gpu, xtra, budget_s, threads):
    """bwa's CPU ksw_align2: Farrar's striped SSE2 kernels (16 x u8 lanes
    with KSW_XBYTE, else 8 x i16) restated in oracle/ksw_align_sse.c, OpenMP
    over tasks on `threads` host threads, best of 3 over a leading sample of
    the timed tasks sized to budget_s.  Parity: the sample's outputs against
    the GPU's, and a smaller leading sample also through the element-wise
    emulation (oracle/ksw_align_oracle.c, the checker the SSE2 form is tested
    equal to)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    mat = fcship.default_mat()

    def head(n):
        return fcship.BswTasks(tasks.qbuf, tasks.qoff[:n], tasks.qlen[:n], tasks.tbuf, tasks.toff[:n], tasks.tlen[:n],
                               tasks.h0[:n], tasks.w[:n])
    cal = head(min(tasks.n, 200 * threads))
    t0 = time.perf_counter()
    oracle_lib.ksw_align2_sse_batch(cal, mat, xtra, threads=threads)
    per_task = max(time.perf_counter() - t0, 1e-6) / cal.n
    n = int(min(tasks.n, max(cal.n, budget_s / 3 / per_task)))
    s = head(n)
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        ref = oracle_lib.ksw_align2_sse_batch(s, mat, xtra, threads=threads)
        times.append(time.perf_counter() - t0)
    same = (ref == gpu["res"][:n]).all(axis=1)
    ne = min(n, 2000)
    emu = np.array([oracle_lib.ksw_align2(*tasks.task(k)[:2], mat, xtra) for k in range(ne)], np.int32).reshape(ne, 7)
    emu_same = (emu == gpu["res"][:ne]).all(axis=1)
    cells = int((tasks.qlen[:n].astype(np.int64) * tasks.tlen[:n]).sum())
    cells += int(((ref[:, 2].astype(np.int64) + 1) * (ref[:, 1].astype(np.int64) + 1))[ref[:, 5] >= 0].sum())
    parity = {"n": n, "bit_exact": int(same.sum()), "mismatched": int(n - same.sum()),
              "emulation_n": ne, "emulation_bit_exact": int(emu_same.sum()),
              "pass": bool(same.all() and emu_same.all()), "fields": "score, te, qe, score2, te2, tb, qb",
              "against": "oracle/ksw_align_sse.c (bwa's striped SSE2 ksw_align2 restated) on the whole sample, and "
                         "oracle/ksw_align_oracle.c (its element-wise emulation) on the leading tasks"}
    return dict(value=cells / min(times) / 1e9, unit="GCUPS", cores=threads, kind="port",
                sample=f"first {n} of the {tasks.n} timed tasks, bwa's striped SSE2 ksw_align2 restated ("
                       + ("16 x u8 lanes per instruction for these XBYTE tasks" if xtra & 0x10000 else
                          "8 x i16 lanes per instruction for these tasks without XBYTE")
                       + f"), OpenMP {threads} threads (nproc "
                       f"{os.cpu_count()}), best of 3 ({', '.join(f'{t:.2f}' for t in times)} s)"), parity


def bsw_roofline(r3, rf):
    """SW roofline: VALU issue.  achieved = cells/s x the lane-instructions per
    cell measured by rocprofv3 (SQ_INSTS_VALU, profiles/pmc_bsw.json, same
    workloads) against 256 CU x 4 SIMD x 32 lanes x 2.4 GHz; the body of one
    cell of the pair kernel is 9.75 lane-instructions (19.5 packed VOP3P/VOP2
    per two tasks).  HBM: algorithmic bytes qlen + tlen + 24 per task."""
    path = os.path.join(ROOT, "profiles", "pmc_bsw.json")
    meas = json.load(open(path)) if os.path.exists(path) else {}
    per3 = meas.get("c3", {}).get("valu_lane_instr_per_cell")
    perf = meas.get("fixed", {}).get("valu_lane_instr_per_cell")
    out = {"bound": "valu", "unit": "T lane-instr/s", "peak": round(VALU_LANE_INSTR_PEAK / 1e12, 3),
           "kernel": "bsw_ext_kernel (pair waves: two ksw_extend2 tasks per lane, packed 16-bit VOP3P; one LPT-ordered launch)",
           "body_instr_per_cell": 8.75,
           "hbm_GBs": round(r3["bytes"] / (r3["ms"] * 1e-3) / 1e9, 2),
           "hbm_frac": round(r3["bytes"] / (r3["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}
    c3m = meas.get("c3", {})
    if c3m.get("fetch_kib") and c3m.get("write_kib"):
        out["traffic"] = int(round((fetch_factor() * c3m["fetch_kib"] + c3m["write_kib"]) * 1024))
        out["traffic_note"] = ("2 x FETCH_SIZE + WRITE_SIZE of one C3 batch (profiles/pmc_bsw.json; the x2 is the "
                               "gfx950 FETCH_SIZE calibration, profiles/fetch_calibration.json)")
    if per3:
        ach = r3["gcups"] * 1e9 * per3
        out.update(achieved=round(ach / 1e12, 3), frac=round(ach / VALU_LANE_INSTR_PEAK, 4),
                   valu_instr_per_cell=per3, valu_source=meas.get("source"))
    # the algorithmic fraction: BASELINE.md §3's ~12 int ops per cell, whatever
    # the kernel issues for them (rises only when the kernel gets faster)
    out["algorithmic_ops_per_cell"] = SW_OPS_PER_CELL
    out["algorithmic_frac"] = round(r3["gcups"] * 1e9 * SW_OPS_PER_CELL / VALU_LANE_INSTR_PEAK, 4)
    try:
        ck = json.load(open(os.path.join(ROOT, "profiles", "clock.json"))).get("bsw_ext")
    except (OSError, ValueError):
        ck = None
    if per3 and ck:
        out["effective_clock_ghz"] = ck
        out["frac_at_effective_clock"] = round(r3["gcups"] * 1e9 * per3 / (VALU_LANE_INSTR_PEAK * ck / 2.4), 4)
    if perf:
        out["fixed_frac"] = round(rf["gcups"] * 1e9 * perf / VALU_LANE_INSTR_PEAK, 4)
        out["fixed_valu_instr_per_cell"] = perf
    return out


def cpu_baseline_bsw(tasks, gpu, budget_s, threads):
    """bwa's ksw_extend2 is scalar C (bwa ksw.c; bwa-mem's own SIMD is only in
    ksw_align2/SSE2 local alignment), so the scalar restatement over OpenMP is
    the like-for-like CPU path; best of 3 over a leading slice of the timed C3
    tasks sized to budget_s, whose outputs are compared with the GPU's outputs
    for the same tasks (six ints and the cell count, bit-exact)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib

    def head(n):
        return fcship.BswTasks(tasks.qbuf, tasks.qoff[:n], tasks.qlen[:n], tasks.tbuf, tasks.toff[:n], tasks.tlen[:n],
                               tasks.h0[:n], tasks.w[:n])
    cal = head(min(tasks.n, 2000 * threads))
    t0 = time.perf_counter()
    oracle_lib.ksw_extend2_batch(cal, fcship.default_mat(), threads=threads)
    per_task = max(time.perf_counter() - t0, 1e-6) / cal.n
    n = int(min(tasks.n, max(cal.n, budget_s / 3 / per_task)))
    s = head(n)
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        res, cells = oracle_lib.ksw_extend2_batch(s, fcship.default_mat(), threads=threads)
        times.append(time.perf_counter() - t0)
    same = (res == gpu["res"][:n]).all(axis=1) & (cells == gpu["cell_counts"][:n])
    parity = {"n": n, "bit_exact": int(same.sum()), "mismatched": int(n - same.sum()), "pass": bool(same.all()),
              "fields": "score, qle, tle, gtle, gscore, max_off and the evaluated-cell count",
              "against": "oracle/ksw_oracle.c (bwa ksw_extend2 restatement)"}
    return dict(value=int(cells.sum()) / min(times) / 1e9, unit="GCUPS", cores=threads, kind="port",
                sample=f"first {n} of the {tasks.n} timed C3 extension tasks, scalar C ksw_extend2 restatement "
                       f"(bwa's is scalar too), best of 3 ({', '.join(f'{t:.2f}' for t in times)} s), "
                       f"OpenMP {threads} threads (nproc {os.cpu_count()})"), parity


class Ranks:
    """This process's place in the job (RANK / LOCAL_RANK / WORLD_SIZE from the
    environment torch.distributed.run or launch_ranks sets) and the two
    reductions the bench needs.  The backend is RCCL ("nccl") on the GPU and
    gloo in --dry-run."""

    def __init__(self, dry):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dry = dry
        self.dev = torch.device("cpu") if dry else torch.device("cuda", self.local)
        if not dry:
            torch.cuda.set_device(self.dev)
        if self.world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if dry:
                torch.distributed.init_process_group("gloo")
            else:
                # the C4 leg holds ranks > 0 in a barrier while rank 0's job runs (minutes at 8 GPUs)
                import datetime
                torch.distributed.init_process_group("nccl", device_id=self.dev,
                                                     timeout=datetime.timedelta(minutes=30))
        # a CPU-side group for the long waits (ranks > 0 while rank 0 runs the
        # C4 / C5 jobs): a gloo barrier blocks in a socket read, where an RCCL
        # barrier's stream wait may spin a host core the jobs need
        self.cpu_group = None
        if self.world > 1:
            import datetime
            self.cpu_group = torch.distributed.new_group(backend="gloo", timeout=datetime.timedelta(minutes=30))

    def barrier(self):
        if self.world > 1:
            torch.distributed.barrier()

    def cpu_barrier(self):
        if self.world > 1:
            torch.distributed.barrier(group=self.cpu_group)

    def cpu_sum(self, v):
        """Sum of one float over the ranks through the gloo group (a blocking
        wait, no spinning host core while slower ranks finish)."""
        t = torch.tensor([float(v)], dtype=torch.float64)
        if self.world > 1:
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM, group=self.cpu_group)
        return float(t.item())

    def _reduce(self, vals, op):
        t = torch.tensor(vals, dtype=torch.float64, device=self.dev)
        if self.world > 1:
            torch.distributed.all_reduce(t, op=op)
        return t.tolist()

    def max(self, *vals):
        return self._reduce(list(vals), torch.distributed.ReduceOp.MAX)

    def sum(self, *vals):
        return self._reduce(list(vals), torch.distributed.ReduceOp.SUM)

    def close(self):
        if self.world > 1:
            torch.distributed.destroy_process_group()


def launch_ranks(n, dry):
    """`bench.py --gpus N` outside torch.distributed.run: start N fresh rank
    processes (RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and
    a free MASTER_PORT) before this process makes any HIP call, wait for all of
    them, and exit with the first failure.  Only rank 0 prints the JSON line.
    If one rank fails, the others are stopped (they would wait in a barrier)."""
    import signal
    import socket
    import subprocess
    if not dry:
        have = torch.cuda.device_count()  # counts devices without initialising HIP on this image
        if have < n:
            sys.exit(f"bench.py: --gpus {n} asks for {n} GPUs but {have} are visible")
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      start_new_session=True))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                for q in live:  # exactly the rank processes this launcher started
                    os.killpg(q.pid, signal.SIGTERM)
        time.sleep(0.05)
    sys.exit(rc)


def load_fcship():
    """Imports the C-ABI binding (after torch: one HIP runtime per process)."""
    global fcship
    import fcship as _fcship
    fcship = _fcship
    return fcship


def dry_step(args):
    """CPU stand-in for the PairHMM pass in --dry-run: a fixed amount of numpy work."""
    a = np.random.default_rng(args.seed).random((256, 256))
    for _ in range(4):
        a = np.tanh(a @ a / 256)
    return float(a.sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank process each); without WORLD_SIZE in the environment, bench.py starts "
                         "the rank processes itself")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only: exercise the launcher, ranks and reductions over gloo with a stand-in workload")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--bsw-reads", type=int, default=500_000)
    ap.add_argument("--no-bsw", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--e2e-mbp", type=float, default=31.0,
                    help="per-GPU genome of the htc / mutect2 runs (31 Mbp = chr1 / 8 GPUs, the C4 share)")
    ap.add_argument("--e2e-align-mbp", type=float, default=4.0, help="genome of the align run")
    ap.add_argument("--e2e-reps", type=int, default=3,
                    help="runs of each e2e command; the fastest is reported, every run's wall time listed")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip the C4 / C5 legs (one htc and one mutect2 job over --c4-mbp, dealt to all N GPUs)")
    ap.add_argument("--c4-mbp", type=float, default=248.0,
                    help="genome of the C4 / C5 jobs (248 Mbp = chr1), the same at every N")
    ap.add_argument("--c4-reps", type=int, default=1, help="runs of each C4 / C5 job; the fastest is reported")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        launch_ranks(args.gpus, args.dry_run)  # exits
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world_env:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}")
    rk = Ranks(args.dry_run)
    world, rank, local, dev = rk.world, rk.rank, rk.local, rk.dev
    if args.dry_run:
        return dry_main(args, rk)
    load_fcship()

    progress("C2 PairHMM")
    ph = bench_phmm(args, dev, rk)
    total_cells = ph["cells"] * world * args.steps
    value = total_cells / ph["elapsed"] / 1e9
    fwd_s = ph["fwd_ms"] * 1e-3
    achieved_tf = FLOPS_PER_CELL * ph["cells"] / fwd_s / 1e12
    traffic = load_traffic("phmm_fwd_fp32")
    pmc, pmc_src = load_pmc_phmm()
    try:
        clk = json.load(open(os.path.join(ROOT, "profiles", "clock.json")))
    except (OSError, ValueError):
        clk = {}
    vipc = pmc.get("valu_lane_instr_per_cell")
    p = ph["p"]
    alg_bytes = int(5 * p.read_len.sum() + p.hap_len.sum() + 4 * p.n_pairs + 8 * p.n_pairs)

    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GCUPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ph["elapsed"] / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32 (fp64 rescue)",
        "data": "synthetic (seeded C2 generator: hap uniform ACGT, read = hap substring with 1% subs / 0.1% indels, "
                "base Q U[10,40], ins/del GOP 45, GCP 10)",
        "config": {"workload": "C2: PairHMM, 1M pairs per GPU, read len 101, hap len U[150,300], fp32 + fp64 rescue",
                   "pairs_per_gpu": p.n_pairs, "cells_per_gpu": ph["cells"], "parallelism": f"static shard x{world}"},
        "stages_ms": {"schedule": round(ph["sched_ms"], 3), "forward_fp32": round(ph["fwd_ms"], 3),
                      "rescue_fp64": round(ph["resc_ms"], 3)},
        "rescued_pairs": ph["n_rescued"],
        "roofline": {"bound": "valu", "achieved": round(achieved_tf, 3), "peak": FP32_VECTOR_PEAK_TF,
                     "unit": "TFLOP/s", "frac": round(achieved_tf / FP32_VECTOR_PEAK_TF, 4),
                     "traffic": traffic,
                     "traffic_note": "HBM bytes per forward pass: 2 x FETCH_SIZE + WRITE_SIZE from separate rocprofv3 "
                                     "--pmc passes (profiles/pmc_traffic.json; the x2 is the gfx950 FETCH_SIZE "
                                     "calibration, profiles/fetch_calibration.json)",
                     "kernel": "phmm4_kernel<C> (column-blocked: lane = one of 16 haplotype columns of a block, "
                               "two packed half-streams of read rows per wave, rows streamed through an LDS ring; "
                               "eight column classes C = 19, 17..11 for reads of 33..160 bases) plus phmm3_kernel "
                               "(row-streamed stripes) for longer haplotypes: fp32 forward pass = one launch per "
                               "launch class, overlapped on 4 streams; achieved = algorithmic FLOPs / pass time "
                               "(HIP events on the launch stream; rocprofv3 kernel stats of this bench in "
                               "profiles/r5/)",
                     "valu_instr_per_cell": vipc,
                     "valu_issue_frac": (round(ph["cells"] / fwd_s * vipc / VALU_LANE_INSTR_PEAK, 4) if vipc
                                         else None),
                     "valu_source": f"profiles/pmc_phmm.json ({pmc_src}: SQ_INSTS_VALU x 64 / cells)",
                     "effective_clock_ghz": clk.get("phmm_fwd_fp32"),
                     "valu_issue_frac_at_effective_clock": (
                         round(ph["cells"] / fwd_s * vipc / (VALU_LANE_INSTR_PEAK * clk["phmm_fwd_fp32"] / 2.4), 4)
                         if vipc and clk.get("phmm_fwd_fp32") else None),
                     "kernel_gcups": round(ph["cells"] / fwd_s / 1e9, 3),
                     "algorithmic_bytes_per_launch": alg_bytes,
                     "algorithmic_hbm_GBs": round(alg_bytes / fwd_s / 1e9, 2),
                     "hbm_frac": round(alg_bytes / fwd_s / 1e9 / HBM_PEAK_GBS, 5)},
    }

    if not args.no_bsw and rank == 0:
        progress("C3 / ksw_global2 / ksw_align2")
        c3 = fcship.synth_bsw(args.seed, args.bsw_reads, read_len=151, ref_len=10_000_000, w=100)
        fx = fcship.synth_bsw(args.seed, max(1, args.bsw_reads * 2), read_len=151, ref_len=10_000_000, w=100,
                              mode=1, fixed_q=151, fixed_t=251)
        r3 = bench_bsw(args, dev, c3)
        rf = bench_bsw(args, dev, fx)
        line["bsw"] = {"workload": "C3: ksw_extend2 left/right seed extensions of 2x151 bp reads, bwa defaults",
                       "c3_gcups": round(r3["gcups"], 3), "c3_tasks": r3["tasks"], "c3_ms": round(r3["ms"], 3),
                       "fixed_151x251_gcups": round(rf["gcups"], 3), "fixed_tasks": rf["tasks"],
                       "roofline": bsw_roofline(r3, rf)}
        gl = fcship.synth_bsw(args.seed + 2, args.bsw_reads // 2, read_len=151, ref_len=10_000_000, w=16,
                              mode=1, fixed_q=151, fixed_t=151)
        g = bench_bsw_global(args, dev, gl)
        line["bsw"]["global"] = {
            "workload": "ksw_global2 of 151 bp reads against their 151 bp reference span (0.5% subs, 0.05% indels), "
                        "band w = 16 (bwa_gen_cigar2's inferred band for such reads)",
            "tasks": g["tasks"], "w": g["w"], "band_cells": g["cells"],
            "scores_gcups": g["scores"]["gcups"], "scores_ms": g["scores"]["ms"],
            "cigar_gcups": g["cigar"]["gcups"], "cigar_ms": g["cigar"]["ms"],
            "kernel": "bsw_global_lane_kernel<33> (one task per lane, band in registers, one unmasked row form "
                      "with bwa's boundaries carried by column -1, direction nibbles of raw compare signs shifted in "
                      "by v_alignbit, rows interleaved across the wave's 64 tasks, row inputs as dword streams), then "
                      "bsw_traceback_kernel (bwa's traceback, one lane per task, 8 waves per SIMD); wider bands go "
                      "to bsw_global_kernel (one wave per task)"}
        gm = {}
        try:
            gm = json.load(open(os.path.join(ROOT, "profiles", "pmc_bsw.json"))).get("global", {})
        except (OSError, ValueError):
            pass
        if gm.get("dp_valu_lane_instr_per_cell"):
            vpc = gm["dp_valu_lane_instr_per_cell"]
            ach = g["scores"]["gcups"] * 1e9 * vpc
            line["bsw"]["global"]["roofline"] = {
                "bound": "valu", "unit": "T lane-instr/s", "peak": round(VALU_LANE_INSTR_PEAK / 1e12, 3),
                "achieved": round(ach / 1e12, 3), "frac": round(ach / VALU_LANE_INSTR_PEAK, 4),
                "valu_instr_per_cell": vpc, "of": "scores-only pass (DP kernels)",
                "valu_source": "profiles/pmc_bsw.json global (SQ_INSTS_VALU x 64 / band cells)"}
            if gm.get("cigar_pass_valu_lane_instr_per_cell"):
                line["bsw"]["global"]["roofline"]["cigar_pass_valu_instr_per_cell"] = \
                    gm["cigar_pass_valu_lane_instr_per_cell"]
        # mate rescue: 151 bp reads in 600 bp windows (mem_matesw's window for a
        # ~350 +- 50 bp insert), bwa's xtra for it (XSUBO | XSTART | min_seed_len * a,
        # XBYTE as l_ms * a < 250)
        al = fcship.synth_bsw(args.seed + 3, args.bsw_reads // 4, read_len=151, ref_len=10_000_000, w=100,
                              mode=1, fixed_q=151, fixed_t=600)
        xa = 0x40000 | 0x80000 | 0x10000 | 19
        ga = bench_bsw_align(args, dev, al, xa)
        line["bsw"]["align"] = {
            "workload": "ksw_align2 of 151 bp reads in 600 bp windows (bwa mem_matesw shape), xtra = XSUBO | "
                        "XSTART | XBYTE | 19",
            "tasks": ga["tasks"], "ms": round(ga["ms"], 3), "gcups": round(ga["gcups"], 3),
            "cells": ga["cells"], "cells_first_pass": ga["cells_first"],
            "kernel": "bsw_align_kernel<16, 10, true> (u8 tasks: four per wave in 16-lane groups, lane l holding "
                      "query positions 10 l .. 10 l + 9 as five packed 16-bit pairs; bwa's striped-F semantics by "
                      "register running-max scans plus one row scan; both passes in one launch; the 32-bit "
                      "<16, 10, false> launch of the device entry point finds no i16 wave and exits)"}
        am = {}
        try:
            am = json.load(open(os.path.join(ROOT, "profiles", "pmc_bsw.json"))).get("align", {})
        except (OSError, ValueError):
            pass
        if am.get("valu_lane_instr_per_cell"):
            vpc = am["valu_lane_instr_per_cell"]
            ach = ga["gcups"] * 1e9 * vpc
            line["bsw"]["align"]["roofline"] = {
                "bound": "valu", "unit": "T lane-instr/s", "peak": round(VALU_LANE_INSTR_PEAK / 1e12, 3),
                "achieved": round(ach / 1e12, 3), "frac": round(ach / VALU_LANE_INSTR_PEAK, 4),
                "valu_instr_per_cell": vpc,
                "valu_source": f"profiles/pmc_bsw.json align ({am.get('source', '')}: SQ_INSTS_VALU x 64 / cells)"}
        # the same windows as bwa's i16 tasks (no KSW_XBYTE: mem_matesw's case for
        # l_ms * a >= 250, here forced on 151 bp reads to time the 16-bit path)
        x16 = 0x40000 | 0x80000 | 19
        g16 = bench_bsw_align(args, dev, al, x16)
        line["bsw"]["align"]["i16"] = {
            "workload": "the same tasks with xtra = XSUBO | XSTART | 19 (bwa's ksw_i16: 8 lanes, 16-bit saturation)",
            "ms": round(g16["ms"], 3), "gcups": round(g16["gcups"], 3), "cells": g16["cells"],
            "kernel": "bsw_align_kernel<16, 10, true> (i16 tasks on the packed path: scores of a <= 160-base query "
                      "stay below 160 x max_mat, so the biased scan values of bwa's 8 blocks fit 16-bit halves)"}
        if world == 1 and not args.no_cpu_baseline:
            line["bsw"]["cpu_baseline"], line["bsw"]["parity"] = cpu_baseline_bsw(c3, r3, args.cpu_budget,
                                                                                  cpu_threads())
            line["bsw"]["align"]["cpu_baseline"], line["bsw"]["align"]["parity"] = cpu_baseline_bsw_align(
                al, ga, xa, min(args.cpu_budget, 6.0), cpu_threads())
            line["bsw"]["align"]["i16"]["cpu_baseline"], line["bsw"]["align"]["i16"]["parity"] = \
                cpu_baseline_bsw_align(al, g16, x16, min(args.cpu_budget, 4.0), cpu_threads())

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("C2 CPU baseline and parity")
        line["cpu_baseline"], ref, used_d = cpu_baseline_phmm(p, args.cpu_budget, cpu_threads())
        line["parity"] = phmm_parity(ph["out"], ref, used_d)

    if not args.no_e2e:
        progress("e2e htc / mutect2 / align")
        try:
            e2e, ok = bench_e2e(args, rank, local), 1.0
        except Exception as e:  # reported in the line; the headline stands
            progress(f"e2e failed: {e!r}"[:400])
            e2e, ok = {"error": repr(e)[:400]}, 0.0
        n_ok = rk.cpu_sum(ok)
        if world > 1 and n_ok < world:
            e2e["ranks_failed"] = int(world - n_ok)
        elif world > 1:  # whole-job rates: units of all ranks over the slowest rank's time
            for k, unit in (("htc", "regions"), ("mutect2", "regions"), ("align", "reads")):
                tot, = rk.sum(e2e[k][unit])
                slow, = rk.max(e2e[k]["seconds"])
                e2e[k]["rank0_" + unit] = e2e[k][unit]
                e2e[k][unit] = int(tot)
                e2e[k]["seconds"] = round(slow, 3)
                e2e[k][unit + "_per_s"] = round(tot / slow, 1)
            e2e["n_gpus"] = world
        line["e2e"] = e2e

    if not args.no_c4:
        # C4 / C5 as the reference runs them: ONE htc and ONE mutect2 job over
        # a --c4-mbp genome (chr1's 248 Mbp by default, the same at every N),
        # their 32 shards dealt to all N GPUs of the node by the job's own
        # Executor.  Rank 0 runs them while the other ranks wait; their GPUs
        # serve the jobs' slots.  At N = 1 each job's CPU path runs beside it.
        rk.cpu_barrier()
        if rank == 0:
            try:
                jobs = run_jobs(args, int(os.environ.get("LOCAL_WORLD_SIZE", str(world))),
                                cpu=world == 1 and not args.no_cpu_baseline)
            except Exception as e:  # reported in the line; the headline stands
                progress(f"C4/C5 legs failed: {e!r}"[:400])
                jobs = {"c4": {"error": repr(e)[:400]}}
            line.update(jobs)
        rk.cpu_barrier()

    if rank == 0:
        # the driver keeps only the tail of stdout: the long e2e block first,
        # then the SW and parity blocks, then one compact summary of every figure
        for k in ("bsw", "parity", "c4", "c5"):
            if k in line:
                line[k] = line.pop(k)
        line["summary"] = summary(line)
        print(json.dumps(line), flush=True)
    rk.close()


def summary(line):
    """Every headline figure of the line in one short block (the end of the
    line is what the driver's record keeps)."""
    s = {"c2_gcups": line["value"], "c2_roofline_frac": line["roofline"]["frac"]}
    if "parity" in line:
        p = line["parity"]
        s["c2_parity"] = {"n": p["n"], "max_rel_err": p["max_rel_err"], "pass": p["pass"]}
    b = line.get("bsw")
    if b:
        s["c3_gcups"] = b["c3_gcups"]
        s["c3_fixed_gcups"] = b["fixed_151x251_gcups"]
        s["global_scores_gcups"] = b["global"]["scores_gcups"]
        s["global_cigar_gcups"] = b["global"]["cigar_gcups"]
        s["align_u8_gcups"] = b["align"]["gcups"]
        s["align_i16_gcups"] = b["align"]["i16"]["gcups"]
        if "parity" in b:
            s["c3_parity"] = {k: b["parity"][k] for k in ("n", "bit_exact", "pass")}
            s["align_parity"] = {k: b["align"]["parity"][k] for k in ("n", "bit_exact", "pass")}
            s["align_i16_parity"] = {k: b["align"]["i16"]["parity"][k] for k in ("n", "bit_exact", "pass")}
    e = line.get("e2e", {})
    if "error" in e:
        s["e2e_error"] = e["error"]
    for k in ("htc", "mutect2"):
        if k in e:
            x = {"seconds": e[k]["seconds"], "runs_seconds": e[k]["runs_seconds"],
                 "regions_per_s": e[k]["regions_per_s"]}
            cb = e[k].get("cpu_baseline", {}).get("gkl")
            if cb:
                x["cpu_gkl_seconds"] = cb["seconds"]
                x["calls_equal"] = cb["calls_equal_to_gpu"]
            s["e2e_" + k] = x
    if "align" in e:
        s["e2e_align"] = {"seconds": e["align"]["seconds"], "reads_per_s": e["align"]["reads_per_s"],
                          "mates_rescued": e["align"]["mates_rescued"]}
        if "cpu_baseline" in e["align"]:
            s["e2e_align"]["cpu_seconds"] = e["align"]["cpu_baseline"]["seconds"]
            s["e2e_align"]["bam_equal"] = e["align"]["cpu_baseline"]["bam_equal_to_gpu"]
    for k in ("c4", "c5"):
        if k in line:
            s[k] = job_summary(line[k])
    return s


def dry_main(args, rk):
    """--dry-run: the launcher, the barrier-bracketed timed region, the
    max-over-ranks reduction and the whole-job sum, over gloo on CPU."""
    if os.environ.get("FCS_BENCH_DRY_FAIL_RANK") == str(rk.rank):  # launcher test: one rank dies early
        sys.exit(3)
    for _ in range(args.warmup):
        dry_step(args)
    rk.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dry_step(args)
    rk.barrier()
    elapsed, = rk.max(time.perf_counter() - t0)
    units, = rk.sum(float(args.steps))
    ranks_seen, = rk.sum(1.0)
    rk.cpu_barrier()  # the gloo wait group of the C4 / C5 legs
    if rk.cpu_sum(1.0) != ranks_seen:
        sys.exit("bench.py: the CPU wait group disagrees with the rank count")
    if rk.rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(units / elapsed, 3), "unit": "dry steps/s",
                          "n_gpus": rk.world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "none", "data": "dry run (no GPU)",
                          "config": {"workload": "dry run", "ranks_seen": int(ranks_seen),
                                     "parallelism": f"static shard x{rk.world}"}}), flush=True)
    rk.close()


if __name__ == "__main__":
    main()
