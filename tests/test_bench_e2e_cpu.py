"""bench.py's end-to-end legs on CPU, through the test-only CPU mock of
libfcship.so (tests/cpu_mock): the code paths the GPU bench runs, with the
PairHMM and banded-SW entry points computed by the oracle restatements.

* the C4 leg (bench_c4): ONE `fcs-genome htc` job whose 32 interval shards
  are dealt round-robin to several GPU slots (/root/reference/src/
  worker-htc.cpp:113-145, src/Executor.cpp:262), with the same calls as the
  one-slot run;
* the align CPU baseline (align_cpu_baseline): damaged mates that only the
  mate rescue (ksw_align2) places, the same BAM whatever the SW thread count.
"""
import os
import sys

import pytest

import host_lib as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.fixture(scope="module")
def mock_env():
    env = bench.cpu_mock_env(dict(os.environ))
    env.update(FCS_MOCK_PHMM="gkl", FCS_HOST_THREADS="4")
    env.pop("FCS_GPU_DEVICES", None)
    return env


@pytest.fixture(scope="module")
def job_runs(mock_env, tmp_path_factory):
    """The C4 (htc) and C5 (mutect2) jobs on one slot and dealt over two."""
    runs = {}
    for n in (1, 2):
        w = tmp_path_factory.mktemp(f"slots{n}")
        runs[n] = (w, bench.bench_c4(H.BIN, dict(mock_env, FCS_TEMP_DIR=str(w)), str(w), 1.2, n, 7, 4,
                                     tools=("htc", "mutect2")))
    return runs


@pytest.mark.parametrize("tool,out", [("htc", "c4.g.vcf"), ("mutect2", "c5.vcf")])
def test_job_deals_32_shards_over_slots(job_runs, tool, out):
    (w1, one), (w2, two) = job_runs[1], job_runs[2]
    one, two = one[tool], two[tool]
    assert one["shards_per_device"] == {"0": 32}
    assert two["shards_per_device"] == {"0": 16, "1": 16}  # gpu.devices[job_id % n]
    assert two["devices"] == 2 and two["genome_mbp"] == 1.2 and two["regions"] > 0
    assert two["regions"] == one["regions"] and two["cells"] == one["cells"]
    assert two["calls"] == one["calls"] > 0
    assert bench.vcf_calls(str(w1 / out)) == bench.vcf_calls(str(w2 / out))


def test_summary_keeps_job_figures_at_the_end(job_runs):
    line = {"value": 1.0, "roofline": {"frac": 0.5}, "c4": job_runs[2][1]["htc"], "c5": job_runs[2][1]["mutect2"]}
    s = bench.summary(line)
    assert s["c4"]["shards_per_device"] == {"0": 16, "1": 16} and s["c5"]["calls"] == line["c5"]["calls"]


def test_align_cpu_baseline_rescues_damaged_mates(mock_env, tmp_path):
    a = tmp_path / "a"
    p = H.run_cli("synth", "-o", a, "-c", "chr1:300000", "-x", "10", "--no-fastq", "--paired", "350", "--seed", "3",
                  env=mock_env, cwd=tmp_path, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    n_damaged = bench.damage_mates(str(a / "sample_2.fastq"))
    assert n_damaged > 20
    cmd = lambda o: ["align", "-f", "-r", str(a / "ref.fasta"), "-1", str(a / "sample_1.fastq"), "-2",  # noqa: E731
                     str(a / "sample_2.fastq"), "-o", o]
    env = dict(mock_env, FCS_TEMP_DIR=str(tmp_path), FCS_GPU_DEVICES="0")
    ref_bam = str(tmp_path / "one_thread.bam")
    p = H.run_cli(*cmd(ref_bam), env=dict(env, FCS_MOCK_BSW_THREADS="1"), cwd=tmp_path, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    rep = bench.align_report(p.stderr)
    assert rep["mates_rescued"] >= 0.8 * n_damaged, (rep["mates_rescued"], n_damaged)
    cb = bench.align_cpu_baseline(H.BIN, env, str(tmp_path), cmd, ref_bam, 4)
    assert cb["bam_equal_to_gpu"] and cb["mates_rescued"] == rep["mates_rescued"] and cb["cores"] == 4


def test_run_jobs_n1_with_cpu_path(mock_env, monkeypatch):
    """bench.py's N = 1 C4/C5 leg end to end (both jobs, then each job's CPU
    path beside it), here with the mock standing in for the GPU library too."""
    import argparse
    for k, v in mock_env.items():
        monkeypatch.setenv(k, v)
    args = argparse.Namespace(c4_mbp=1.0, seed=11, c4_reps=1)
    out = bench.run_jobs(args, 1, cpu=True)
    for k in ("c4", "c5"):
        st = out[k]
        assert st["shards_per_device"] == {"0": 32} and st["regions"] > 0
        assert st["cpu_baseline"]["calls_equal_to_gpu"] and st["speedup_vs_cpu_path"] > 0
        assert "output" not in st
