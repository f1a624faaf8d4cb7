"""CPU tests of `fcs-genome align`'s host logic (chains,
mem_chain2aln rounds, dedup / patch, primary / supplementary marking, mate
rescue, pairing, SAM fields).  The fcs-genome child process runs against
tests/cpu_mock/libfcship.so — the banded-SW entry points computed by the
oracle's ksw_extend2 / ksw_global2 (test infrastructure only; the product
library has no CPU path).  The same cases run on the GPU in test_host_gpu.py."""
import re
import subprocess

import pytest

import align_cases as A
import host_lib as H

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))


@pytest.fixture(scope="module")
def mock_env():
    subprocess.run(["make", "-C", f"{ROOT}/tests/cpu_mock"], check=True, capture_output=True)
    return {"LD_LIBRARY_PATH": f"{ROOT}/tests/cpu_mock/build", "FCS_GPU_DEVICES": "0"}


@pytest.fixture(scope="module")
def ref(tmp_path_factory, mock_env):
    d = tmp_path_factory.mktemp("ref")
    p = H.run_cli("synth", "-o", d, "-c", "chr20:150000,chr21:60000", "-x", "1", "--seed", "11", "--no-fastq")
    assert p.returncode == 0, p.stderr[-2000:]
    return d / "ref.fasta"


def test_mock_is_loaded(mock_env, ref, tmp_path):
    fq = tmp_path / "r.fastq"
    A.split_reads_fastq(ref, fq, n_split=2, n_whole=2, seed=1)
    p = H.run_cli("align", "-r", ref, "-1", fq, "-o", tmp_path / "o.bam", env=mock_env, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-2000:]
    p = H.run_cli("--version", env=mock_env, cwd=tmp_path)
    assert "cpu-mock" in p.stdout + p.stderr, (p.stdout, p.stderr)


def test_split_reads_cpu(mock_env, ref, tmp_path):
    fq = tmp_path / "split.fastq"
    truth = A.split_reads_fastq(ref, fq, n_split=120, n_whole=60, seed=3)
    out = tmp_path / "split.bam"
    p = H.run_cli("align", "-r", ref, "-1", fq, "-o", out, env=mock_env, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    good, bad = A.check_split_reads(out, truth)
    assert good >= 0.95 * 120, (good, len(bad), bad[:5])
    assert re.search(r"(\d+) supplementary", p.stderr).group(1) == str(sum(len(t) == 4 for t in truth.values()) - len(bad))


def test_paired_end_cpu(mock_env, tmp_path):
    d = tmp_path / "pe"
    p = H.run_cli("synth", "-o", d, "-c", "chr1:150000", "-x", "6", "--paired", "350", "--seed", "77")
    assert p.returncode == 0, p.stderr[-2000:]
    damaged = A.damage_mates(d / "sample_2.fastq")
    out = tmp_path / "pe.bam"
    p = H.run_cli("align", "-r", d / "ref.fasta", "-1", d / "sample_1.fastq", "-2", d / "sample_2.fastq", "-o", out,
                  env=mock_env, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    A.check_pairs(p.stderr, out, d / "pairs_truth.tsv", damaged)


def test_paired_split_reads_cpu(mock_env, tmp_path):
    """A split read 1 (bwa is_multi): no pairing, read 1 as primary +
    supplementary, mate fields of the other read's primary on every record."""
    d = tmp_path / "pe"
    p = H.run_cli("synth", "-o", d, "-c", "chr1:150000,chr2:60000", "-x", "4", "--paired", "350", "--seed", "78")
    assert p.returncode == 0, p.stderr[-2000:]
    chim = A.append_chimeric_pairs(d / "ref.fasta", d / "sample_1.fastq", d / "sample_2.fastq", 40, 5, "chr1", "chr2")
    out = tmp_path / "pe.bam"
    p = H.run_cli("align", "-r", d / "ref.fasta", "-1", d / "sample_1.fastq", "-2", d / "sample_2.fastq", "-o", out,
                  env=mock_env, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    assert A.check_chimeric_pairs(out, chim, "chr1", "chr2") >= 38


def test_saved_index_rejected_after_same_length_edit(mock_env, tmp_path):
    """a saved .fcsidx is used only for the exact reference text it
    was built from.  Editing one base (contig lengths unchanged) makes align
    build the index in memory instead of mapping the stale one."""
    d = tmp_path / "r"
    p = H.run_cli("synth", "-o", d, "-c", "chr20:60000,chr21:30000", "-x", "2", "--seed", "9")
    assert p.returncode == 0, p.stderr[-2000:]
    ref = d / "ref.fasta"
    p = H.run_cli("index", "-r", ref, "--sa-intv", "8")
    assert p.returncode == 0, p.stderr[-2000:]
    fq = tmp_path / "r.fastq"
    A.split_reads_fastq(ref, fq, n_split=1, n_whole=4, seed=2)
    p = H.run_cli("align", "-f", "-r", ref, "-1", fq, "-o", tmp_path / "a.bam", env=mock_env, cwd=tmp_path)
    assert p.returncode == 0 and "mapped " + str(ref) + ".fcsidx" in p.stderr, p.stderr[-2000:]
    lines = ref.read_text().split("\n")
    k = 1 + len(lines) // 2  # a sequence line in the middle of chr1
    lines[k] = ("C" if lines[k][0] != "C" else "G") + lines[k][1:]
    ref.write_text("\n".join(lines))
    p = H.run_cli("align", "-f", "-r", ref, "-1", fq, "-o", tmp_path / "b.bam", env=mock_env, cwd=tmp_path)
    assert p.returncode == 0 and "built in memory" in p.stderr, p.stderr[-2000:]


def test_xa_alternative_hits_cpu(mock_env, tmp_path):
    """bwa's XA tag (mem_gen_alt): a read from a segment that exists twice
    (an exact copy on chr21, a copy with one substitution on chr20) is placed
    on the exact copy, and its record lists the other copy as
    "chr20,[+-]pos,CIGAR,NM;" (secondary hits scoring >= 0.80 of the primary)."""
    import numpy as np
    d = tmp_path / "r"
    p = H.run_cli("synth", "-o", d, "-c", "chr20:60000,chr21:30000", "-x", "1", "--seed", "21", "--no-fastq")
    assert p.returncode == 0, p.stderr[-2000:]
    contigs = A.read_fasta(d / "ref.fasta")
    rng = np.random.default_rng(4)
    seg = "".join(rng.choice(list("ACGT"), 400))
    seg_b = seg[:200] + {"A": "C", "C": "G", "G": "T", "T": "A"}[seg[200]] + seg[201:]
    c20 = contigs["chr20"][:20000] + seg_b + contigs["chr20"][20400:]
    c21 = contigs["chr21"][:10000] + seg + contigs["chr21"][10400:]
    ref = tmp_path / "ref.fasta"
    ref.write_text(f">chr20\n{c20}\n>chr21\n{c21}\n")
    fq = tmp_path / "r.fastq"
    reads = [(f"x{k}", seg[a:a + 150]) for k, a in enumerate((60, 120, 180))]
    fq.write_text("".join(f"@{n}\n{s}\n+\n{'I' * 150}\n" for n, s in reads))
    out = tmp_path / "o.bam"
    p = H.run_cli("align", "-r", ref, "-1", fq, "-o", out, env=mock_env, cwd=tmp_path)
    assert p.returncode == 0, p.stderr[-2000:]
    names, _, recs = H.read_bam(out)
    assert len(recs) == 3
    for r in recs:
        assert names[r["ref_id"]] == "chr21", r
        tags = H.parse_aux(r["aux"])
        a = int(r["name"][1:])
        start = 20000 + (60, 120, 180)[a] + 1
        assert tags.get("XA") == f"chr20,+{start},150M,1;", tags
        assert r["mapq"] < 10  # the near-identical copy makes the placement ambiguous
