"""End-to-end GPU runs of the fcs-genome commands on synthetic data (SURVEY.md
§8f rows f1-f4): `htc` and `mutect2` recover the spiked variants, every
PairHMM likelihood the caller used matches the CPU oracle (the caller dumps
its region batches with --dump-regions), and `align` places the synthetic
reads where the generator drew them.  Recall / precision bars are this
build's own (the reference's caller is GATK [EXT]; parity unpinned beyond the
PairHMM values)."""
import os
import struct

import numpy as np
import pytest

import host_lib as H
import oracle_lib

pytestmark = pytest.mark.gpu


SPIKE = "chr20:109380"


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    d = tmp_path_factory.mktemp("e2e")
    # the spiked cluster straddles the 10th/11th shard boundary of gatk.ncontigs = 32
    # (ceil(350000 / 32) = 10938 positions per shard: chr20:109380 | 109381)
    p = H.run_cli("synth", "-o", d, "-c", "chr20:250000,chr21:100000", "-x", "30", "--tumor", "--seed", "11",
                  "--spike", SPIKE, "--parts", "6")
    assert p.returncode == 0, p.stderr
    return d


def truth(d, somatic):
    out = set()
    for ln in (d / "truth.vcf").read_text().splitlines():
        if ln.startswith("#"):
            continue
        f = ln.split("\t")
        if ("SOMATIC" in f[7]) == somatic:
            out.add((f[0], int(f[1]), f[3], f[4]))
    return out


def calls(vcf):
    out = set()
    for ln in open(vcf).read().splitlines():
        if ln.startswith("#"):
            continue
        f = ln.split("\t")
        out.add((f[0], int(f[1]), f[3], f[4]))
    return out


def read_dump(path):
    regions = []
    b = open(path, "rb").read()
    p = 0
    while p < len(b):
        assert b[p:p + 4] == b"RGN1"
        nr, nh = struct.unpack_from("<ii", b, p + 4)
        p += 12
        reads = []
        for _ in range(nr):
            L = struct.unpack_from("<i", b, p)[0]
            p += 4
            reads.append(tuple(np.frombuffer(b[p + k * L: p + (k + 1) * L], np.uint8).copy() for k in range(5)))
            p += 5 * L
        haps = []
        for _ in range(nh):
            L = struct.unpack_from("<i", b, p)[0]
            haps.append(np.frombuffer(b[p + 4: p + 4 + L], np.uint8).copy())
            p += 4 + L
        lik = np.frombuffer(b[p: p + 8 * nr * nh], np.float64).reshape(nr, nh).copy()
        p += 8 * nr * nh
        regions.append((reads, haps, lik))
    return regions


ENV = {"FCS_GATK_NCONTIGS": "6", "FCS_GATK_NPROCS": "3", "FCS_GPU_DEVICES": "0"}


def test_htc_end_to_end(gpu, data, tmp_path):
    out = tmp_path / "htc.vcf"
    dump = tmp_path / "dump"
    p = H.run_cli("htc", "-r", data / "ref.fasta", "-i", data / "sample.bam", "-o", out, "-v", "--dump-regions", dump,
                  env=ENV, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    assert (tmp_path / "htc.vcf.gz").exists() and (tmp_path / "htc.vcf.gz.tbi").exists()
    import gzip
    assert gzip.decompress((tmp_path / "htc.vcf.gz").read_bytes()).decode() == out.read_text()
    t, c = truth(data, False), calls(out)
    tp = len(t & c)
    snv_t = {v for v in t if len(v[2]) == len(v[3]) == 1}
    assert len(snv_t & c) / len(snv_t) >= 0.95, (len(snv_t & c), len(snv_t))
    assert tp / len(t) >= 0.9, (tp, len(t))
    assert tp / max(1, len(c)) >= 0.95, (tp, len(c))
    # every PairHMM value the caller used equals the oracle's (sampled pairs)
    rng = np.random.default_rng(0)
    dumps = sorted(tmp_path.glob("dump.*"))
    assert dumps
    checked = 0
    for f in dumps:
        for reads, haps, lik in read_dump(f):
            for _ in range(3):
                r, h = int(rng.integers(len(reads))), int(rng.integers(len(haps)))
                ref, _ = oracle_lib.phmm_log10(reads[r], haps[h])
                assert abs(lik[r, h] - ref) <= 1e-5 * abs(ref), (lik[r, h], ref)
                checked += 1
    assert checked >= 100


def test_mutect2_end_to_end(gpu, data, tmp_path):
    out = tmp_path / "m2.vcf"
    p = H.run_cli("mutect2", "-r", data / "ref.fasta", "-t", data / "tumor.bam", "-n", data / "sample.bam", "-o", out,
                  env=ENV, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    som, germ, c = truth(data, True), truth(data, False), calls(out)
    assert som, "the synthetic tumor has somatic variants"
    assert len(som & c) / len(som) >= 0.8, (len(som & c), len(som))
    assert len(germ & c) <= 0.02 * len(germ)  # germline sites are rejected by the normal


def test_align_end_to_end(gpu, data, tmp_path):
    out = tmp_path / "aln.bam"
    p = H.run_cli("align", "-r", data / "ref.fasta", "-1", data / "sample.fastq", "-o", out, env=ENV, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    assert os.path.exists(str(out) + ".bai")
    _, _, truth_recs = H.read_bam(data / "sample.bam")
    names, _, recs = H.read_bam(out)
    want = {r["name"]: r for r in truth_recs}
    same_pos = same_cig = mapped = 0
    for r in recs:
        if r["flag"] & 4:
            continue
        mapped += 1
        w = want[r["name"]]
        same_pos += (r["ref_id"], r["pos"]) == (w["ref_id"], w["pos"])
        same_cig += r["cigar"] == w["cigar"]
        assert (r["flag"] & 16) == (w["flag"] & 16)
        assert r["seq"] == w["seq"]
    assert mapped / len(recs) >= 0.99
    assert same_pos / mapped >= 0.97, (same_pos, mapped)
    assert same_cig / mapped >= 0.9, (same_cig, mapped)


def test_align_split_reads_supplementary(gpu, data, tmp_path):
    """Split reads on the GPU: tests/align_cases.py builds the
    chimeric reads and checks primary / supplementary placement, hard clips,
    MAPQ and the SA tags."""
    import align_cases as A
    fq = tmp_path / "split.fastq"
    truth = A.split_reads_fastq(data / "ref.fasta", fq, n_split=300, n_whole=200, seed=3)
    out = tmp_path / "split.bam"
    p = H.run_cli("align", "-r", data / "ref.fasta", "-1", fq, "-o", out, env=ENV, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    good, bad = A.check_split_reads(out, truth)
    assert good >= 0.95 * 300, (good, len(bad), bad[:5])


def test_align_paired_end(gpu, tmp_path):
    """Paired-end align (row f4): FR pairs of N(350, 50) fragments; 4% of the
    read-2 mates carry a mismatch every 16 bases, so no 19-mer seeds them and
    only the mate rescue (bwa's mem_matesw: a GPU ksw_align2 local alignment
    of the mate in the window the insert-size statistics predict opposite
    the read-1 alignment) places them.  Checks placement against the generator's truth, proper-pair
    flags, mate fields, signed TLEN and the insert-size estimate."""
    import re
    d = tmp_path / "pe"
    p = H.run_cli("synth", "-o", d, "-c", "chr1:400000", "-x", "16", "--paired", "350", "--seed", "77",
                  env=ENV, cwd=tmp_path, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    # damage some read-2 mates: a mismatch every 16 bases defeats 19-mer seeding
    lines = open(d / "sample_2.fastq").read().split("\n")
    damaged = set()
    flip = {"A": "C", "C": "G", "G": "T", "T": "A", "N": "A"}
    for i in range(0, len(lines) - 3, 4):
        if (i // 4) % 25 == 7:
            seq = list(lines[i + 1])
            for j in range(5, len(seq), 16):
                seq[j] = flip[seq[j]]
            lines[i + 1] = "".join(seq)
            damaged.add(lines[i][1:].split("/")[0])
    open(d / "sample_2.fastq", "w").write("\n".join(lines))
    out = tmp_path / "pe.bam"
    p = H.run_cli("align", "-r", d / "ref.fasta", "-1", d / "sample_1.fastq", "-2", d / "sample_2.fastq", "-o", out,
                  env=ENV, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    import align_cases as A
    A.check_pairs(p.stderr, out, d / "pairs_truth.tsv", damaged)


def test_align_sample_sheet_over_two_slots(gpu, tmp_path):
    """`align -F` runs one BWAWorker per (sample, read group)
    under the Executor, then merges the sample's read groups; FASTQ chunks of
    a read group are dealt over every GPU slot.  Two slots (both device 0 —
    the dealing is the same over two devices) with small chunks give the same
    BAM as one slot, byte for byte; both @RG lines are in the header and every
    read is in the merged BAM once.  One read group's FASTQs are gzipped."""
    import gzip
    import shutil
    d = tmp_path / "fq"
    p = H.run_cli("synth", "-o", d, "-c", "chr1:300000", "-x", "12", "--paired", "350", "--seed", "5", "--no-fastq",
                  env=ENV, cwd=tmp_path, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    halves = {}
    for m in (1, 2):
        lines = open(d / f"sample_{m}.fastq").read().splitlines(keepends=True)
        n = len(lines) // 8 * 4
        halves[m] = ("".join(lines[:n]), "".join(lines[n:]))
    for m in (1, 2):
        (d / f"A_{m}.fastq").write_text(halves[m][0])
        with gzip.open(d / f"B_{m}.fastq.gz", "wt") as f:
            f.write(halves[m][1])
    sheet = tmp_path / "sheet.csv"
    sheet.write_text("#sample_id,fastq1,fastq2,rg,platform_id,library_id\n"
                     f"S,{d}/A_1.fastq,{d}/A_2.fastq,rgA,illumina,libA\n"
                     f"S,{d}/B_1.fastq.gz,{d}/B_2.fastq.gz,rgB,illumina,libB\n")
    outs = {}
    for devs in ("0", "0,0"):
        o = tmp_path / f"out_{devs.replace(',', '_')}"
        env = dict(ENV, FCS_GPU_DEVICES=devs, FCS_BWA_CHUNK_SIZE="4000", FCS_BWA_GPU_SLOTS="1")
        p = H.run_cli("align", "-r", d / "ref.fasta", "-F", sheet, "-o", o, env=env, cwd=tmp_path)
        assert p.returncode == 0, p.stderr[-3000:]
        assert ("on 2 device slot(s)" in p.stderr) == (devs == "0,0"), p.stderr[-2000:]
        assert os.path.exists(o / "S.bam.bai")
        outs[devs] = (o / "S.bam").read_bytes()
    assert outs["0"] == outs["0,0"]
    names, _, recs = H.read_bam(tmp_path / "out_0" / "S.bam")
    text = gzip.decompress(outs["0"])
    assert b"@RG\tID:rgA\tSM:S\tPL:illumina\tLB:libA" in text and b"@RG\tID:rgB" in text
    n_reads = sum(1 for _ in open(d / "sample_1.fastq")) // 4 * 2
    assert len(recs) == n_reads and len({(r["name"], r["flag"] & 0xC0) for r in recs}) == n_reads
    keys = [((r["ref_id"] & 0xFFFFFFFF), r["pos"]) for r in recs]
    assert keys == sorted(keys)
    shutil.rmtree(d)


def test_htc_gpu_slots_do_not_change_calls(gpu, data, tmp_path):
    """Shards dealt over two GPU slots (both on device 0 here — the dealing
    rule is the same as over two devices) and more concurrent tasks give the
    same VCF as one slot: shards are independent, no exchange step."""
    outs = []
    for devs, nprocs in (("0", "1"), ("0,0", "4")):
        out = tmp_path / f"htc_{nprocs}.vcf"
        env = dict(ENV, FCS_GPU_DEVICES=devs, FCS_GATK_NPROCS=nprocs)
        p = H.run_cli("htc", "-r", data / "ref.fasta", "-i", data / "sample.bam", "-o", out, "-v", env=env,
                      cwd=tmp_path)
        assert p.returncode == 0, p.stderr[-3000:]
        outs.append([ln for ln in out.read_text().splitlines() if not ln.startswith("##source")])
    assert outs[0] == outs[1]


def test_htc_shard_boundaries_do_not_change_calls(gpu, data, tmp_path):
    """a variant cluster cut by a gatk.ncontigs boundary is called the
    same as with the boundary elsewhere — every shard whose range a cluster
    touches sees the whole cluster (caller.cpp window growth) and emits only the
    calls inside its own range."""
    outs = {}
    for n in ("1", "6", "32"):
        out = tmp_path / f"htc_n{n}.vcf"
        p = H.run_cli("htc", "-r", data / "ref.fasta", "-i", data / "sample.bam", "-o", out, "-v",
                      env=dict(ENV, FCS_GATK_NCONTIGS=n), cwd=tmp_path)
        assert p.returncode == 0, p.stderr[-3000:]
        outs[n] = [ln for ln in out.read_text().splitlines() if not ln.startswith("##")]
    assert outs["1"] == outs["6"] == outs["32"]
    spiked = {("chr20", 109380 + d) for d in (-30, 0, 30)}
    called = {(f[0], int(f[1])) for f in (ln.split("\t") for ln in outs["32"] if not ln.startswith("#"))}
    assert spiked <= called, spiked - called


@pytest.fixture(scope="module")
def data_c5(tmp_path_factory):
    """C5-shaped tumor/normal pair in which 4% of the reads look mis-mapped
    (20% high-quality mismatches): their likelihoods against every candidate
    haplotype fall below the fp32 pass's 1e-28 threshold, so the fp64 rescue
    runs inside a real mutect2 job."""
    d = tmp_path_factory.mktemp("c5")
    p = H.run_cli("synth", "-o", d, "-c", "chr20:200000", "-x", "30", "--tumor", "--seed", "13",
                  "--noisy-frac", "0.04")
    assert p.returncode == 0, p.stderr
    return d


def log_totals(logdir, key):
    import re
    tot = 0
    for f in os.listdir(logdir):
        for m in re.finditer(r"(\d+) " + key, open(os.path.join(logdir, f)).read()):
            tot += int(m.group(1))
    return tot


def test_mutect2_c5_rescue_and_likelihoods(gpu, data_c5, tmp_path):
    """mutect2 tumor/normal with the fp32 -> fp64 rescue
    firing; every sampled likelihood the caller used (tumor and normal
    regions) equals the oracle within 1e-5, rescued pairs included."""
    out, dump, logs = tmp_path / "m2.vcf", tmp_path / "dump", tmp_path / "log"
    p = H.run_cli("mutect2", "-r", data_c5 / "ref.fasta", "-t", data_c5 / "tumor.bam", "-n", data_c5 / "sample.bam",
                  "-o", out, "--dump-regions", dump, env=dict(ENV, FCS_LOG_DIR=str(logs)), cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    rescued = log_totals(logs, "rescued")
    assert rescued > 0, "the noisy reads must send pairs through the fp64 rescue"
    som = truth(data_c5, True)
    assert len(som & calls(out)) / len(som) >= 0.8
    rng = np.random.default_rng(5)
    checked = n_resc = 0
    for f in sorted(tmp_path.glob("dump.*")):
        for reads, haps, lik in read_dump(f):
            picks = {(int(rng.integers(len(reads))), int(rng.integers(len(haps)))) for _ in range(3)}
            # plus every pair whose likelihood is below the fp32 threshold (log10(1e-28) - log10(2^120))
            picks |= {(int(r), int(h)) for r, h in zip(*np.nonzero(lik < -64.1))}
            for r, h in picks:
                ref, used_d = oracle_lib.phmm_log10(reads[r], haps[h])
                assert abs(lik[r, h] - ref) <= 1e-5 * abs(ref), (lik[r, h], ref, used_d)
                checked += 1
                n_resc += used_d
    assert checked >= 100 and n_resc > 0, (checked, n_resc)


def test_htc_c4_proxy_all_devices(gpu, tmp_path):
    """C4 proxy: htc on a chr1-like 30x genome, the reference's 32 interval
    shards (gatk.ncontigs) dealt round-robin over every visible GPU
    (gpu.devices), calls checked against the truth set and the likelihoods of
    every shard sampled against the oracle.  (2 Mbp, not chr1's 248 Mbp:
    bench.py's e2e block runs the larger shape.)"""
    import fcship
    d = tmp_path / "d"
    p = H.run_cli("synth", "-o", d, "-c", "chr1:2000000", "-x", "30", "--seed", "17")
    assert p.returncode == 0, p.stderr
    devs = ",".join(str(i) for i in range(fcship.device_count()))
    out, dump, logs = tmp_path / "htc.vcf", tmp_path / "dump", tmp_path / "log"
    env = dict(ENV, FCS_GATK_NCONTIGS="32", FCS_GATK_NPROCS="8", FCS_GPU_DEVICES=devs, FCS_LOG_DIR=str(logs))
    p = H.run_cli("htc", "-r", d / "ref.fasta", "-i", d / "sample.bam", "-o", out, "-v", "--dump-regions", dump,
                  env=env, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    t, c = truth(d, False), calls(out)
    tp = len(t & c)
    assert tp / len(t) >= 0.9 and tp / max(1, len(c)) >= 0.95, (tp, len(t), len(c))
    dumps = sorted(tmp_path.glob("dump.*"))
    assert len(dumps) == 32, len(dumps)  # every shard ran and batched its regions through the GPU
    rng = np.random.default_rng(1)
    for f in dumps:
        for reads, haps, lik in read_dump(f)[:2]:
            r, h = int(rng.integers(len(reads))), int(rng.integers(len(haps)))
            ref, _ = oracle_lib.phmm_log10(reads[r], haps[h])
            assert abs(lik[r, h] - ref) <= 1e-5 * abs(ref)
    assert log_totals(logs, "regions") > 1000


def records(path):
    return [ln.split("\t") for ln in open(path).read().splitlines() if not ln.startswith("#")]


def test_htc_gvcf_is_the_default(gpu, data, tmp_path):
    """Without -v htc writes a GVCF, the reference's default
    (src/workers/HTCWorker.cpp:83-97 --emitRefConfidence GVCF): every position
    of the genome lies in exactly one hom-ref <NON_REF> block or inside a call,
    the calls are the -v run's calls with <NON_REF> appended, and 30x coverage
    gives confident reference blocks over most of the genome (hom-ref GQ ~ 3 per
    informative base: GQ >= 60 from depth 20 on)."""
    outs = {}
    for mode in ("vcf", "gvcf"):
        out = tmp_path / f"htc.{mode}"
        args = ["-v"] if mode == "vcf" else []
        p = H.run_cli("htc", "-r", data / "ref.fasta", "-i", data / "sample.bam", "-o", out, *args, env=ENV,
                      cwd=tmp_path)
        assert p.returncode == 0, p.stderr[-3000:]
        outs[mode] = out
    hdr = open(outs["gvcf"]).read()
    assert "##ALT=<ID=NON_REF" in hdr and "##INFO=<ID=END" in hdr and "##GVCFBlock99-100" in hdr
    lengths = {"chr20": 250000, "chr21": 100000}
    covered = {c: np.zeros(n + 1, np.int32) for c, n in lengths.items()}
    blocks = var = 0
    gq99 = 0
    gcalls = set()
    for f in records(outs["gvcf"]):
        chrom, pos, ref, alts = f[0], int(f[1]), f[3], f[4].split(",")
        assert alts[-1] == "<NON_REF>"
        if alts == ["<NON_REF>"]:
            end = int(f[7].split("END=")[1])
            assert end >= pos and f[8] == "GT:DP:GQ:MIN_DP:PL" and f[9].startswith("0/0:")
            assert (covered[chrom][pos:end + 1] == 0).all(), "blocks overlap"
            covered[chrom][pos:end + 1] += 1
            blocks += 1
            if int(f[9].split(":")[2]) >= 60:
                gq99 += end - pos + 1
        else:
            var += 1
            assert len(f[9].split(":")[4].split(",")) == 6  # PLs of 0/0 0/1 1/1 0/2 1/2 2/2
            covered[chrom][pos:pos + len(ref)] += 1
            gcalls.add((chrom, pos, ref, alts[0]))
    for c, n in lengths.items():
        assert (covered[c][1:] >= 1).all(), (c, np.flatnonzero(covered[c][1:] == 0)[:10])
    assert gcalls == calls(outs["vcf"]), "GVCF calls differ from the -v run's"
    assert var > 100 and blocks > var
    assert gq99 / sum(lengths.values()) > 0.8, gq99


def test_htc_part_bam_directory(gpu, data, tmp_path):
    """BamInput directory mode (reference src/BamInput.cpp): htc -i on the
    part-XXXXXX.bam + .bed layout of `align --disable-merge` (here written by
    synth --parts 6, reads split by alignment start); with gatk.ncontigs = 6
    each shard reads one part over its .bed region.  Calls equal the one-BAM
    run's away from the part boundaries (a part holds only the reads that start
    in it), and recall stays at the one-BAM level."""
    parts = data / "parts"
    assert len(list(parts.glob("part-*.bam"))) == 6 and len(list(parts.glob("part-*.bed"))) == 6
    outs = {}
    for name, inp in (("one", data / "sample.bam"), ("parts", parts)):
        out = tmp_path / f"{name}.vcf"
        p = H.run_cli("htc", "-r", data / "ref.fasta", "-i", inp, "-o", out, "-v", env=ENV, cwd=tmp_path)
        assert p.returncode == 0, p.stderr[-3000:]
        outs[name] = calls(out)
    bounds = []
    for k in range(6):
        for ln in (parts / f"part-{k:06d}.bed").read_text().splitlines():
            c, b, e = ln.split("\t")
            bounds += [(c, int(b)), (c, int(e))]
    far = lambda v: all(v[0] != c or abs(v[1] - x) > 1000 for c, x in bounds)  # noqa: E731
    a = {v for v in outs["one"] if far(v)}
    b = {v for v in outs["parts"] if far(v)}
    assert a == b, (sorted(a - b)[:5], sorted(b - a)[:5])
    t = truth(data, False)
    assert len(t & outs["parts"]) / len(t) >= 0.88


def test_align_disable_merge_buckets_feed_htc(gpu, data, tmp_path):
    """align --disable-merge (reference worker-align.cpp:186-195, bwa-flow
    --merge_bams=0): bwa.num_buckets coordinate-sorted part-XXXXXX.bam + .bai
    + .bed in the output directory, every read in the bucket of its alignment
    start; htc then runs on that directory (BamInput) as the reference's
    pipeline does, with recall at the one-BAM level."""
    env = dict(ENV, FCS_BWA_NUM_BUCKETS="6")
    out = tmp_path / "buckets"
    p = H.run_cli("align", "-r", data / "ref.fasta", "-1", data / "sample.fastq", "-o", out, "--disable-merge",
                  env=env, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    bams = sorted(out.glob("part-*.bam"))
    assert len(bams) == 6 and len(list(out.glob("part-*.bam.bai"))) == 6 and len(list(out.glob("part-*.bed"))) == 6
    _, _, truth_recs = H.read_bam(data / "sample.bam")
    total = 0
    for k, b in enumerate(bams):
        names, _, recs = H.read_bam(b)
        total += len(recs)
        ranges = []
        for ln in (out / f"part-{k:06d}.bed").read_text().splitlines():
            c, lo, hi = ln.split("\t")
            ranges.append((names.index(c), int(lo), int(hi)))
        placed = [r for r in recs if not r["flag"] & 4]
        assert [(r["ref_id"], r["pos"]) for r in placed] == sorted((r["ref_id"], r["pos"]) for r in placed)
        for r in placed:
            assert any(r["ref_id"] == c and lo <= r["pos"] < hi for c, lo, hi in ranges)
    assert total == len(truth_recs)
    vcf = tmp_path / "b.vcf"
    p = H.run_cli("htc", "-r", data / "ref.fasta", "-i", out, "-o", vcf, "-v", env=ENV, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    t = truth(data, False)
    assert len(t & calls(vcf)) / len(t) >= 0.88


def test_c1_gpu_calls_equal_cpu_path(gpu, tmp_path):
    """C1 (BASELINE.json configs[0]) on the GPU gives the calls of the
    reference's CPU PairHMM path (GATK Java LoglessPairHMM semantics, run
    through the test-only CPU mock of the C-ABI, tests/cpu_mock), and every
    likelihood the GPU caller used is within 1e-5 of the Java-semantics value."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-C", os.path.join(root, "tests", "cpu_mock")], check=True, capture_output=True)
    d = tmp_path / "c1"
    p = H.run_cli("synth", "-o", d, "-c", "chr20:1000000", "-x", "30", "-n", "1000", "--no-fastq", "--seed",
                  "20261015")
    assert p.returncode == 0, p.stderr[-2000:]
    outs = {}
    for name, env in (("gpu", ENV), ("cpu", {"LD_LIBRARY_PATH": os.path.join(root, "tests", "cpu_mock", "build"),
                                             "FCS_GPU_DEVICES": "0", "FCS_MOCK_PHMM": "java"})):
        out = tmp_path / f"{name}.vcf"
        extra = ["--dump-regions", tmp_path / "dump"] if name == "gpu" else []
        p = H.run_cli("htc", "-f", "-r", d / "ref.fasta", "-i", d / "sample.bam", "-o", out, "-v", *extra, env=env,
                      cwd=tmp_path)
        assert p.returncode == 0, p.stderr[-3000:]
        outs[name] = [ln for ln in out.read_text().splitlines() if not ln.startswith("##")]
    assert outs["gpu"] == outs["cpu"]
    checked = 0
    for f in sorted(tmp_path.glob("dump.*")):
        for reads, haps, lik in read_dump(f):
            for r in range(len(reads)):
                for h in range(len(haps)):
                    ref = oracle_lib.phmm_java_log10(reads[r], haps[h])
                    assert abs(lik[r, h] - ref) <= 1e-5 * abs(ref), (lik[r, h], ref)
                    checked += 1
    assert checked > 100
