"""BASELINE.json configs[0] ("C1"): `fcs-genome htc` on a 1,000-read synthetic
chr20 BAM with the PairHMM on the CPU — the reference's path, GATK
HaplotypeCaller with the CPU PairHMM (/root/reference/src/workers/
HTCWorker.cpp:85,105).  The fcs-genome child runs against the test-only CPU
mock of libfcship.so (tests/cpu_mock: the oracle's Java LoglessPairHMM
restatement, or its GKL-style AVX-512 restatement, behind the same C-ABI).
Calls are checked against the generator's truth at the GPU tests' bars
(test_host_gpu.py), and the two CPU PairHMM semantics give the same calls.
bench.py times the same command (e2e.c1.cpu_baseline)."""
import os
import subprocess

import pytest

import host_lib as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def mock_dir():
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpu_mock")], check=True, capture_output=True)
    return os.path.join(ROOT, "tests", "cpu_mock", "build")


@pytest.fixture(scope="module")
def c1(tmp_path_factory):
    d = tmp_path_factory.mktemp("c1")
    p = H.run_cli("synth", "-o", d, "-c", "chr20:1000000", "-x", "30", "-n", "1000", "--no-fastq", "--seed", "20261015")
    assert p.returncode == 0, p.stderr[-2000:]
    return d


def calls(vcf):
    out = set()
    for ln in open(vcf):
        if not ln.startswith("#"):
            f = ln.split("\t")
            out.add((f[0], int(f[1]), f[3], f[4]))
    return out


def covered_truth(d):
    """Truth variants inside the span the 1,000 reads cover (150 bp in from
    either end, where a variant can still be seen by >= 2 reads)."""
    _, _, recs = H.read_bam(d / "sample.bam")
    lo = min(r["pos"] for r in recs) + 150
    hi = max(r["pos"] + H.cigar_ref_len(r["cigar"]) for r in recs) - 150
    out = set()
    for ln in (d / "truth.vcf").read_text().splitlines():
        if not ln.startswith("#"):
            f = ln.split("\t")
            if lo < int(f[1]) <= hi:
                out.add((f[0], int(f[1]), f[3], f[4]))
    return out, len(recs), (lo, hi)


def run_cpu(mode, c1, mock_dir, tmp_path, name, extra_env=None):
    out = tmp_path / f"{name}.vcf"
    env = {"LD_LIBRARY_PATH": mock_dir, "FCS_GPU_DEVICES": "0", "FCS_MOCK_PHMM": mode,
           "FCS_LOG_DIR": str(tmp_path / f"log_{name}"), **(extra_env or {})}
    p = H.run_cli("htc", "-f", "-r", c1 / "ref.fasta", "-i", c1 / "sample.bam", "-o", out, "-v", env=env,
                  cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    return out


def test_c1_htc_cpu_java_pairhmm(c1, mock_dir, tmp_path):
    out = run_cpu("java", c1, mock_dir, tmp_path, "java")
    t, n_reads, (lo, hi) = covered_truth(c1)
    assert n_reads == 1000
    c = {v for v in calls(out) if lo < v[1] <= hi}
    assert len(t) >= 3, t  # the covered span holds some variants
    snv = {v for v in t if len(v[2]) == len(v[3]) == 1}
    tp = len(t & c)
    assert len(snv & c) / len(snv) >= 0.95, (sorted(snv - c), sorted(c))
    assert tp / len(t) >= 0.9, (sorted(t - c), sorted(c))
    assert tp / max(1, len(c)) >= 0.95, (sorted(c - t), sorted(t))
    # bgzip + tabix tail ran as on the GPU path
    assert (tmp_path / "java.vcf.gz").exists() and (tmp_path / "java.vcf.gz.tbi").exists()


def test_c1_java_and_gkl_semantics_agree(c1, mock_dir, tmp_path):
    """GATK's Java LoglessPairHMM (double) and GKL's AVX float pass with the
    double rescue differ by <= 1e-5 relative in log10; the calls are the same."""
    a = run_cpu("java", c1, mock_dir, tmp_path, "java")
    b = run_cpu("gkl", c1, mock_dir, tmp_path, "gkl")
    strip = lambda f: [ln for ln in open(f) if not ln.startswith("##")]  # noqa: E731
    assert calls(a) == calls(b)
    assert strip(a) == strip(b)


def test_c1_window_inflate_paths_agree(c1, mock_dir, tmp_path):
    """The window's BAM blocks read member by member with the host's
    libdeflate (the default) and in multi-member chunks through
    fcs_bgzf_inflate (gpu.bam_inflate=true; here the mock's zlib behind the
    same C-ABI) give byte-identical VCFs: the chunk reader's seeks, record
    boundaries across members and window ends are the same."""
    a = run_cpu("gkl", c1, mock_dir, tmp_path, "chunked", {"FCS_GPU_BAM_INFLATE": "true"})
    b = run_cpu("gkl", c1, mock_dir, tmp_path, "host", {"FCS_GPU_BAM_INFLATE": "false"})
    strip = lambda f: [ln for ln in open(f) if not ln.startswith("##")]  # noqa: E731
    assert strip(a) == strip(b)


def test_window_inflate_chunks_cross_members(mock_dir, tmp_path):
    """Many 128 KiB chunks per window (FCS_BGZF_DEVICE_CHUNK), several
    windows and shards: records split across chunk ends, chunks ending
    mid-member and BAI seeks into a chunk give the same VCF as the host's
    member-by-member reader — with every chunk through fcs_bgzf_inflate_try,
    and with every other one "busy" so the reader inflates it on its own
    thread."""
    d = tmp_path / "in"
    p = H.run_cli("synth", "-o", d, "-c", "chrA:400000,chrB:150000", "-x", "12", "--no-fastq", "--seed", "9")
    assert p.returncode == 0, p.stderr[-2000:]
    outs = []
    for name, env in (("chunked", {"FCS_GPU_BAM_INFLATE": "true", "FCS_BGZF_DEVICE_CHUNK": str(128 << 10)}),
                      ("mixed", {"FCS_GPU_BAM_INFLATE": "true", "FCS_BGZF_DEVICE_CHUNK": str(128 << 10),
                                 "FCS_MOCK_BGZF_BUSY": "alternate"}),
                      ("host", {"FCS_GPU_BAM_INFLATE": "false"})):
        out = tmp_path / f"{name}.vcf"
        e = {"LD_LIBRARY_PATH": mock_dir, "FCS_GPU_DEVICES": "0", "FCS_MOCK_PHMM": "gkl",
             "FCS_LOG_DIR": str(tmp_path / f"log_{name}"), **env}
        p = H.run_cli("htc", "-f", "-r", d / "ref.fasta", "-i", d / "sample.bam", "-o", out, "-v", env=e, cwd=tmp_path)
        assert p.returncode == 0, p.stderr[-3000:]
        outs.append([ln for ln in open(out) if not ln.startswith("##")])
    assert len(outs[0]) > 20
    assert outs[0] == outs[1] == outs[2]


def test_shards_run_while_device_comes_up(mock_dir, tmp_path):
    """gpu.warmup_help: a shard whose PairHMM pass finds the device not yet
    warm runs queued shards on its own thread first.  With the device held
    cold for the whole run (FCS_TEST_COLD_DEVICE) every pass nests the queued
    shards; the GVCF and the somatic VCF are byte-identical to the plain
    schedule's, and the shard logs count the nested shards."""
    import glob
    import re
    d = tmp_path / "in"
    p = H.run_cli("synth", "-o", d, "-c", "chrA:300000,chrB:120000", "-x", "12", "--tumor", "--no-fastq",
                  "--seed", "11")
    assert p.returncode == 0, p.stderr[-2000:]
    res = {}
    for name, env in (("cold", {"FCS_TEST_COLD_DEVICE": "1", "FCS_GPU_WARMUP_HELP": "true"}),
                      ("plain", {"FCS_GPU_WARMUP_HELP": "false"})):
        e = {"LD_LIBRARY_PATH": mock_dir, "FCS_GPU_DEVICES": "0", "FCS_MOCK_PHMM": "gkl", "FCS_GATK_NPROCS": "2",
             "FCS_LOG_DIR": str(tmp_path / f"log_{name}"), **env}
        h = tmp_path / f"{name}.g.vcf"
        p = H.run_cli("htc", "-f", "-r", d / "ref.fasta", "-i", d / "sample.bam", "-o", h, env=e, cwd=tmp_path)
        assert p.returncode == 0, p.stderr[-3000:]
        m = tmp_path / f"{name}.m2.vcf"
        p = H.run_cli("mutect2", "-f", "-r", d / "ref.fasta", "-n", d / "sample.bam", "-t", d / "tumor.bam",
                      "-o", m, env=e, cwd=tmp_path)
        assert p.returncode == 0, p.stderr[-3000:]
        logs = "".join(open(f).read() for f in glob.glob(str(tmp_path / f"log_{name}" / "*.log")))
        nested = sum(int(x) for x in re.findall(r"ran (\d+) queued shards", logs))
        body = lambda f: [ln for ln in open(f) if not ln.startswith("##")]  # noqa: E731
        res[name] = (body(h), body(m), nested)
    assert len(res["plain"][0]) > 100 and len(res["plain"][1]) > 1
    assert res["cold"][0] == res["plain"][0]
    assert res["cold"][1] == res["plain"][1]
    assert res["plain"][2] == 0
    assert res["cold"][2] > 0
