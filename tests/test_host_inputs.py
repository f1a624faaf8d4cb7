"""CPU tests of the orchestrator's input side:
BamInput directory mode (reference src/BamInput.cpp:27-149), region files
(BED / GATK interval lists) and GATK's -isr INTERSECTION of several -L sets,
the GVCF GQ bands, and SIGINT teardown (reference src/main.cpp:43-54)."""
import ctypes as C
import gzip
import os
import signal
import subprocess
import time

import pytest

import host_lib as H


def shard(path, contig, ncontigs, tmp):
    buf = C.create_string_buffer(1 << 16)
    H.check(H.lib.fcsg_bam_input_shard(str(path).encode(), contig, ncontigs, str(tmp).encode(), buf, len(buf)))
    bams, region = buf.value.decode().split("\n")[:2]
    return [os.path.basename(b) for b in bams.split(",") if b], region


def regions(*paths):
    arr = (C.c_char_p * len(paths))(*[str(p).encode() for p in paths])
    buf = C.create_string_buffer(1 << 16)
    H.check(H.lib.fcsg_intersect_regions(arr, len(paths), buf, len(buf)))
    out = []
    for line in buf.value.decode().splitlines():
        c, lb, ub = line.split("\t")
        out.append((c, int(lb), int(ub)))
    return out


def make_parts(d, n_bam, n_region, ext="bed"):
    d.mkdir()
    for i in range(n_bam):
        (d / f"part-{i:06d}.bam").write_bytes(b"")
        (d / f"part-{i:06d}.bam.bai").write_bytes(b"")
    for i in range(n_region):
        if ext == "bed":
            (d / f"part-{i:06d}.bed").write_text(f"chr1\t{i * 100}\t{i * 100 + 50}\n")
        else:
            (d / f"part-{i:06d}.list").write_text(f"chr1:{i * 100 + 1}-{i * 100 + 50}\n")


def test_bam_input_one_part_per_shard(tmp_path):
    d = tmp_path / "parts"
    make_parts(d, 8, 8)
    for k in range(8):
        bams, region = shard(d, k, 8, tmp_path / "t")
        assert bams == [f"part-{k:06d}.bam"]
        assert region == str(d / f"part-{k:06d}.bed")


def test_bam_input_merges_parts_per_shard(tmp_path):
    d = tmp_path / "parts"
    make_parts(d, 8, 8)
    bams, region = shard(d, 1, 4, tmp_path / "t")
    assert bams == ["part-000002.bam", "part-000003.bam"]
    assert os.path.basename(region) == "part-2_3.bed"
    assert open(region).read() == "chr1\t200\t250\nchr1\t300\t350\n"
    # a merged region file is read as one -L set
    assert regions(region) == [("chr1", 201, 250), ("chr1", 301, 350)]


def test_bam_input_list_files_keep_their_kind(tmp_path):
    d = tmp_path / "parts"
    make_parts(d, 4, 4, ext="list")
    bams, region = shard(d, 0, 2, tmp_path / "t")
    assert bams == ["part-000000.bam", "part-000001.bam"]
    assert region.endswith("part-0_1.list")  # the reference would name it .bed (and GATK would misread it)
    assert regions(region) == [("chr1", 1, 50), ("chr1", 101, 150)]


def test_bam_input_errors(tmp_path):
    d = tmp_path / "noregion"
    make_parts(d, 4, 0)
    with pytest.raises(RuntimeError, match="No BED or list files"):
        shard(d, 0, 4, tmp_path / "t")
    d2 = tmp_path / "few"
    make_parts(d2, 4, 2)
    with pytest.raises(RuntimeError, match="Number of BED Files less than ncontig"):
        shard(d2, 0, 4, tmp_path / "t")
    with pytest.raises(RuntimeError, match="Cannot find input"):
        shard(tmp_path / "missing", 0, 1, tmp_path / "t")
    bam = tmp_path / "x.bam"
    bam.write_bytes(b"")
    with pytest.raises(RuntimeError, match="index of input BAM"):
        shard(bam, 0, 1, tmp_path / "t")
    (tmp_path / "x.bai").write_bytes(b"")  # <stem>.bai is accepted like <bam>.bai
    assert shard(bam, 0, 1, tmp_path / "t") == (["x.bam"], "")


def test_bam_input_odd_bam_quirk(tmp_path):
    # reference BamInput.cpp:104-111: more region files than BAMs and an odd
    # BAM count -> the shard reaching past the BAMs stops one BAM short
    d = tmp_path / "parts"
    make_parts(d, 3, 4)
    assert shard(d, 1, 2, tmp_path / "t")[0] == []  # first = 2, last clamped to 3 - 1 = 2
    d2 = tmp_path / "parts2"
    make_parts(d2, 4, 8)
    assert shard(d2, 1, 2, tmp_path / "t2")[0] == []  # first 4 >= 4 BAMs: nothing left


def test_interval_intersection(tmp_path):
    a = tmp_path / "a.list"
    a.write_text("chr2:1-100\nchr1:50-150\nchr1:140-200\nchr3\n")
    b = tmp_path / "b.bed"
    b.write_text("track name=x\nchr1\t99\t160\nchr2\t0\t10\nchr2\t90\t300\nchr3\t5\t7\nchr9\t0\t5\n")
    got = regions(a, b)
    # contig order of the first set; a's chr1 pieces merge to 50-200
    assert got == [("chr2", 1, 10), ("chr2", 91, 100), ("chr1", 100, 160), ("chr3", 6, 7)]
    c = tmp_path / "c.list"
    c.write_text("chr1:120-130\n")
    assert regions(a, b, c) == [("chr1", 120, 130)]
    assert regions(b) == [("chr1", 100, 160), ("chr2", 1, 10), ("chr2", 91, 300), ("chr3", 6, 7), ("chr9", 1, 5)]


def test_gvcf_gq_bands():
    # GATK default --GVCFGQBands: 1..60 one each, then 70, 80, 90, 99
    b = H.lib.fcsg_gvcf_band
    assert [b(0), b(1), b(2), b(59), b(60), b(69), b(70), b(79), b(80), b(90), b(98), b(99)] == \
        [0, 1, 2, 59, 60, 60, 61, 61, 62, 63, 63, 64]


def test_sigint_tears_down(tmp_path):
    """SIGINT mid-run: 'Caught interrupt, cleaning up...', the temp dir is
    removed and the exit code is 128 + SIGINT."""
    tmp = tmp_path / "tmpdir"
    env = dict(os.environ, FCS_TEMP_DIR=str(tmp), FCS_LOG_DIR=str(tmp_path / "log"))
    p = subprocess.Popen([H.BIN, "synth", "-o", str(tmp_path / "d"), "-c", "chr1:40000000", "-x", "30"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    time.sleep(1.5)
    assert p.poll() is None, "synth finished before the signal"
    p.send_signal(signal.SIGINT)
    out, err = p.communicate(timeout=60)
    assert p.returncode == 128 + signal.SIGINT, (p.returncode, err[-2000:])
    assert "Caught interrupt, cleaning up..." in err
    assert not tmp.exists()


# ------------------------------------------------------------ align inputs
def _sheet(path):
    buf = C.create_string_buffer(1 << 16)
    H.check(H.lib.fcsg_sample_sheet(str(path).encode(), buf, len(buf)))
    return [ln.split("\t") for ln in buf.value.decode().splitlines()]


def test_sample_sheet_file(tmp_path):
    """`align -F` sheet (reference src/SampleSheet.cpp:40-121): the '#'
    header names the columns in any order; rows of one sample are its read
    groups in sheet order; a row with a different field count is an error."""
    f = tmp_path / "s.csv"
    f.write_text("#sample_id,rg,fastq1,fastq2,platform_id,library_id\n"
                 "NA2,rgA,/d/a_1.fq,/d/a_2.fq,illumina,libA\n"
                 "NA1,rgB,/d/b_1.fq,/d/b_2.fq,illumina,libB\n"
                 "NA2,rgC,/d/c_1.fq,/d/c_2.fq,ILLUMINA,libC\n")
    assert _sheet(f) == [["NA1", "/d/b_1.fq", "/d/b_2.fq", "rgB", "illumina", "libB"],
                         ["NA2", "/d/a_1.fq", "/d/a_2.fq", "rgA", "illumina", "libA"],
                         ["NA2", "/d/c_1.fq", "/d/c_2.fq", "rgC", "ILLUMINA", "libC"]]
    bad = tmp_path / "bad.csv"
    bad.write_text("#sample_id,fastq1,fastq2,rg,platform_id,library_id\nNA1,/a,/b,rg\n")
    buf = C.create_string_buffer(1024)
    assert H.lib.fcsg_sample_sheet(str(bad).encode(), buf, len(buf)) < 0
    assert "inconsistent" in H.lib.fcsg_last_error().decode()
    nohdr = tmp_path / "nohdr.csv"
    nohdr.write_text("sample_id,fastq1\nNA1,/a\n")
    assert H.lib.fcsg_sample_sheet(str(nohdr).encode(), buf, len(buf)) < 0


def test_sample_sheet_folder(tmp_path):
    """A folder of <sample>_..._1.fastq.gz / _2.fastq.gz pairs (src/SampleSheet.cpp:123-200)."""
    for n in ("S1_L001_1.fastq.gz", "S1_L001_2.fastq.gz", "S1_L002_1.fastq.gz", "S1_L002_2.fastq.gz",
              "S1_L003_1.fastq.gz", "S1_L003_2.fastq.gz", "S2_L001_1.fastq.gz", "S2_L001_2.fastq.gz", "notes.txt"):
        (tmp_path / n).write_bytes(b"")
    got = _sheet(tmp_path)
    d = str(tmp_path)
    # NN is the pair's index within the sample: a third pair gets its own read
    # group (the reference restarts at 01, and align's per-RG BAM path would
    # then collide — ADVICE r3)
    assert got == [["S1", d + "/S1_L001_1.fastq.gz", d + "/S1_L001_2.fastq.gz", "RG-S1_0000", "Illumina", "LIBS1_00"],
                   ["S1", d + "/S1_L002_1.fastq.gz", d + "/S1_L002_2.fastq.gz", "RG-S1_0101", "Illumina", "LIBS1_01"],
                   ["S1", d + "/S1_L003_1.fastq.gz", d + "/S1_L003_2.fastq.gz", "RG-S1_0202", "Illumina", "LIBS1_02"],
                   ["S2", d + "/S2_L001_1.fastq.gz", d + "/S2_L001_2.fastq.gz", "RG-S2_0000", "Illumina", "LIBS2_00"]]
    assert len({r[3] for r in got if r[0] == "S1"}) == 3


def test_align_rejects_duplicate_read_group(tmp_path):
    """Two sheet rows of one sample with the same read group would write the
    same per-read-group BAM: align refuses the sheet (exit 1, invalid
    parameter) before aligning anything."""
    ref = tmp_path / "ref"
    p = H.run_cli("synth", "-o", ref, "-c", "chr1:20000", "-x", "1", "--seed", "3")
    assert p.returncode == 0, p.stderr[-2000:]
    sheet = tmp_path / "s.csv"
    fq = ref / "sample.fastq"
    sheet.write_text("#sample_id,fastq1,fastq2,rg,platform_id,library_id\n"
                     f"S,{fq},{fq},rgA,illumina,libA\nS,{fq},{fq},rgA,illumina,libB\n")
    p = H.run_cli("align", "-r", ref / "ref.fasta", "-F", sheet, "-o", tmp_path / "out", cwd=tmp_path,
                  env={"FCS_GPU_DEVICES": "0"})
    assert p.returncode != 0 and "more than once" in p.stderr, (p.returncode, p.stderr[-2000:])


def test_merge_sorted_bams(tmp_path):
    """align's per-sample merge of read-group BAMs: records in coordinate
    order (unmapped last, ties by input order), the @RG lines of every input,
    and an index identical to one built by reading the merged file back."""
    rows = [["a1\t0\t0\t10\t60\t5M\tACGTA\t*", "a2\t0\t0\t40\t60\t5M\tACGTA\t*", "a3\t16\t1\t5\t60\t5M\tACGTA\t*",
             "a4\t4\t-1\t-1\t0\t*\tACGTA\t*"],
            ["b1\t0\t0\t10\t60\t5M\tACGTA\t*", "b2\t0\t0\t20\t60\t5M\tACGTA\t*", "b3\t0\t1\t1\t60\t5M\tACGTA\t*"]]
    ins = []
    for k, rs in enumerate(rows):
        t = tmp_path / f"in{k}.txt"
        t.write_text(f"@RG\tID:rg{k}\tSM:s\n" + "\n".join(rs) + "\n")
        b = tmp_path / f"in{k}.bam"
        H.check(H.lib.fcsg_text_to_bam(str(t).encode(), str(b).encode(), b"c1,c2", b"1000,500"))
        ins.append(str(b).encode())
    out = tmp_path / "m.bam"
    H.check(H.lib.fcsg_merge_bams((C.c_char_p * 2)(*ins), 2, str(out).encode()))
    names, lens, recs = H.read_bam(out)
    assert [r["name"] for r in recs] == ["a1", "b1", "b2", "a2", "b3", "a3", "a4"]
    text = gzip.decompress(out.read_bytes())
    assert b"@RG\tID:rg0" in text and b"@RG\tID:rg1" in text
    on_write = (tmp_path / "m.bam.bai").read_bytes()
    H.check(H.lib.fcsg_bam_index(str(out).encode()))
    assert (tmp_path / "m.bam.bai").read_bytes() == on_write
