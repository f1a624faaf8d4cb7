"""Cross-shard PairHMM pass merging (host/caller.cpp PassCombiner,
`gpu.phmm.combine_ms`): concurrent shard threads' region batches go to the
device as one pass.  Each region keeps its own output matrix, so the calls
must be byte-identical to one pass per shard flush, with fewer passes.  Runs
`fcs-genome htc` against the test-only CPU mock of libfcship.so (the oracle's
GKL-style PairHMM behind the same C-ABI)."""
import os
import re
import subprocess

import pytest

import host_lib as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def mock_dir():
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpu_mock")], check=True, capture_output=True)
    return os.path.join(ROOT, "tests", "cpu_mock", "build")


@pytest.fixture(scope="module")
def sample(tmp_path_factory):
    d = tmp_path_factory.mktemp("comb")
    p = H.run_cli("synth", "-o", d, "-c", "chrA:400000", "-x", "12", "--tumor", "--no-fastq", "--seed", "77")
    assert p.returncode == 0, p.stderr[-2000:]
    return d


def run_htc(d, mock_dir, tmp_path, name, combine_ms, somatic=False):
    out = tmp_path / f"{name}.vcf"
    logs = tmp_path / f"log_{name}"
    env = {"LD_LIBRARY_PATH": mock_dir, "FCS_GPU_DEVICES": "0", "FCS_MOCK_PHMM": "gkl", "FCS_LOG_DIR": str(logs),
           "FCS_GATK_NCONTIGS": "12", "FCS_GATK_NPROCS": "6", "FCS_GPU_PHMM_COMBINE_MS": str(combine_ms)}
    if somatic:
        p = H.run_cli("mutect2", "-f", "-r", d / "ref.fasta", "-t", d / "tumor.bam", "-n", d / "sample.bam", "-o", out,
                      env=env, cwd=tmp_path)
    else:
        p = H.run_cli("htc", "-f", "-r", d / "ref.fasta", "-i", d / "sample.bam", "-o", out, "-v", env=env,
                      cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    text = "".join(open(os.path.join(r, f)).read() for r, _, fs in os.walk(logs) for f in fs)
    passes = sum(int(x) for x in re.findall(r"(\d+) device passes", text))
    pairs = sum(int(x) for x in re.findall(r"(\d+) pairs", text))
    body = [ln for ln in open(out) if not ln.startswith("##")]
    return body, passes, pairs


def test_merged_passes_give_identical_calls(sample, mock_dir, tmp_path):
    a, pa, na = run_htc(sample, mock_dir, tmp_path, "separate", 0)
    b, pb, nb = run_htc(sample, mock_dir, tmp_path, "merged", 2000)
    assert len(a) > 1 and a == b
    assert na == nb > 0
    assert pa >= 12  # one pass per shard flush at least
    assert pb < pa, (pa, pb)
    print(f"passes: separate {pa}, merged {pb}; pairs {na}")


def test_merged_passes_mutect2(sample, mock_dir, tmp_path):
    a, pa, na = run_htc(sample, mock_dir, tmp_path, "m_separate", 0, somatic=True)
    b, pb, nb = run_htc(sample, mock_dir, tmp_path, "m_merged", 2000, somatic=True)
    assert len(a) > 1 and a == b
    assert na == nb > 0 and pb < pa, (pa, pb)


def test_combine_ms_rejects_negative(sample, mock_dir, tmp_path):
    env = {"LD_LIBRARY_PATH": mock_dir, "FCS_GPU_DEVICES": "0", "FCS_GPU_PHMM_COMBINE_MS": "-1",
           "FCS_LOG_DIR": str(tmp_path / "l")}
    p = H.run_cli("htc", "-f", "-r", sample / "ref.fasta", "-i", sample / "sample.bam", "-o", tmp_path / "x.vcf",
                  env=env, cwd=tmp_path)
    assert p.returncode != 0 and "combine_ms" in p.stderr
