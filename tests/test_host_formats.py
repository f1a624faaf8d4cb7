"""CPU tests of the host orchestrator's formats and runtime (SURVEY.md §8f rows
f1 and f3): BGZF, BAM/BAI, VCF concat + bgzip + tabix, interval sharding,
GATK read preparation, the executor's stage / error / GPU-slot semantics and
the fcs-genome CLI surface.  Each C++ writer is checked against an
independent Python reader (gzip + struct) or a restatement of the
reference's rule."""
import ctypes as C
import gzip
import os
import random
import struct

import numpy as np
import pytest

import host_lib as H


# ------------------------------------------------------------------ BGZF
def test_bgzf_roundtrip_and_layout(tmp_path):
    rng = random.Random(3)
    data = bytes(rng.getrandbits(8) for _ in range(150_000)) + b"ACGT" * 60_000  # incompressible + compressible
    src, gz, back = tmp_path / "x.bin", tmp_path / "x.gz", tmp_path / "y.bin"
    src.write_bytes(data)
    H.check(H.lib.fcsg_bgzf_compress_file(str(src).encode(), str(gz).encode()))
    assert gzip.decompress(gz.read_bytes()) == data  # any gzip reader can read BGZF
    blocks = H.bgzf_blocks(gz)
    assert blocks[-1][2] == 0 and gz.read_bytes()[-28:] == bytes.fromhex(
        "1f8b08040000000000ff0600424302001b0003000000000000000000")  # EOF marker
    assert all(isz <= 0xff00 for _, _, isz in blocks) and all(bs <= 0x10000 for _, bs, _ in blocks)
    H.check(H.lib.fcsg_bgzf_decompress_file(str(gz).encode(), str(back).encode()))
    assert back.read_bytes() == data


def test_bgzf_reader_rejects_plain_gzip(tmp_path):
    p = tmp_path / "plain.gz"
    p.write_bytes(gzip.compress(b"hello\n"))
    assert H.lib.fcsg_bgzf_decompress_file(str(p).encode(), str(tmp_path / "o").encode()) < 0
    assert b"BGZF" in H.lib.fcsg_last_error()


# ------------------------------------------------------------------ BAM
def test_reg2bin_matches_spec():
    rng = random.Random(1)
    for _ in range(2000):
        beg = rng.randrange(0, 1 << 29)
        end = beg + rng.choice([1, 2, 100, 16384, 100_000, 3_000_000])
        assert H.lib.fcsg_reg2bin(beg, end) == H.reg2bin(beg, end)
    assert H.lib.fcsg_reg2bin(-1, 0) == 4680  # unmapped


def test_bam_text_roundtrip(tmp_path):
    rows = [
        "r1\t0\t0\t100\t60\t10M\tACGTACGTAC\tIIIIIIIIII",
        "r2\t16\t0\t100\t37\t3S4M2I1M3D5M\tNACGTTTAGGCCAAG\t" + "".join(chr(33 + i) for i in range(15)),
        "r3\t4\t-1\t-1\t0\t*\tACG\t*",  # unmapped, odd length, qual absent
        "r4\t0\t1\t0\t60\t1M\tA\t!",
    ]
    t = tmp_path / "in.txt"
    t.write_text("\n".join(rows) + "\n")
    bam, back = tmp_path / "o.bam", tmp_path / "o.txt"
    H.check(H.lib.fcsg_text_to_bam(str(t).encode(), str(bam).encode(), b"chrA,chrB", b"1000,50"))
    names, lens, recs = H.read_bam(bam)
    assert names == ["chrA", "chrB"] and lens == [1000, 50]
    assert [r["name"] for r in recs] == ["r1", "r2", "r3", "r4"]
    assert recs[1]["cigar"] == ["3S", "4M", "2I", "1M", "3D", "5M"] and recs[1]["flag"] == 16
    assert recs[2]["qual"] == b"\xff" * 3 and recs[2]["ref_id"] == -1
    for r in recs:  # bin field = reg2bin over the aligned span
        span = max(H.cigar_ref_len(r["cigar"]), 1)
        assert r["bin"] == H.reg2bin(r["pos"], r["pos"] + span)
    H.check(H.lib.fcsg_bam_to_text(str(bam).encode(), str(back).encode()))
    got = [ln.split("\t")[:8] for ln in back.read_text().splitlines() if not ln.startswith("@")]
    assert got == [r.split("\t") for r in rows]


@pytest.fixture(scope="module")
def synth_small(tmp_path_factory):
    d = tmp_path_factory.mktemp("synth")
    p = H.run_cli("synth", "-o", d, "-c", "chrA:120000,chrB:60000", "-x", "8", "--tumor", "--seed", "7")
    assert p.returncode == 0, p.stderr
    return d


def test_synth_bam_is_consistent_with_reference_and_fastq(synth_small):
    d = synth_small
    ref = {}
    for block in (d / "ref.fasta").read_text().split(">")[1:]:
        lines = block.splitlines()
        ref[lines[0]] = "".join(lines[1:])
    names, lens, recs = H.read_bam(d / "sample.bam")
    assert [lens[i] for i in range(len(names))] == [len(ref[n]) for n in names]
    fq = (d / "sample.fastq").read_text().splitlines()
    fq_seq = {fq[i][1:]: fq[i + 1] for i in range(0, len(fq), 4)}
    comp = str.maketrans("ACGTN", "TGCAN")
    last = (-1, -1)
    mism = tot = 0
    for r in recs:
        assert (r["ref_id"], r["pos"]) >= last  # coordinate-sorted
        last = (r["ref_id"], r["pos"])
        s = fq_seq[r["name"]]
        assert r["seq"] == (s.translate(comp)[::-1] if r["flag"] & 16 else s)
        # aligned bases match the reference up to sequencing errors and variants
        R = ref[names[r["ref_id"]]]
        rp, q = r["pos"], 0
        for c in r["cigar"]:
            n, op = int(c[:-1]), c[-1]
            if op == "M":
                mism += sum(1 for k in range(n) if r["seq"][q + k] != R[rp + k])
                tot += n
                rp += n
                q += n
            elif op in "IS":
                q += n
            elif op == "D":
                rp += n
        assert q == len(r["seq"])
    assert tot > 0 and mism / tot < 0.01


def test_bai_seek_lands_before_first_overlapping_read(synth_small):
    bam = synth_small / "sample.bam"
    names, lens, recs = H.read_bam(bam)
    # virtual offsets of records: every record starts a new BAM record inside the BGZF stream
    raw_blocks = H.bgzf_blocks(bam)
    data = bam.read_bytes()
    voffs = []
    header_len = None
    stream = b""
    block_of = []
    for off, bs, isz in raw_blocks:
        payload = gzip.decompress(data[off:off + bs]) if isz else b""
        block_of.append((off, len(stream), len(payload)))
        stream += payload
    l_text = struct.unpack_from("<i", stream, 4)[0]
    p = 8 + l_text
    n_ref = struct.unpack_from("<i", stream, p)[0]
    p += 4
    for _ in range(n_ref):
        ln = struct.unpack_from("<i", stream, p)[0]
        p += 8 + ln
    header_len = p

    def voff(upos):
        for off, start, n in block_of:
            if start <= upos < start + n:
                return (off << 16) | (upos - start)
        raise AssertionError
    p = header_len
    while p < len(stream):
        voffs.append(voff(p))
        p += 4 + struct.unpack_from("<i", stream, p)[0]
    assert len(voffs) == len(recs)
    _, refs = H.parse_index((str(bam) + ".bai").encode() and open(str(bam) + ".bai", "rb").read(), b"BAI\x01")
    rng = random.Random(5)
    for _ in range(50):
        tid = rng.randrange(len(names))
        beg = rng.randrange(lens[tid])
        off = C.c_ulonglong()
        H.check(H.lib.fcsg_bam_seek_offset((str(bam) + ".bai").encode(), tid, beg, C.byref(off)))
        first = next((i for i, r in enumerate(recs) if r["ref_id"] == tid and
                      r["pos"] + H.cigar_ref_len(r["cigar"]) > beg), None)
        if first is None:
            continue
        assert off.value <= voffs[first]  # seeking there and scanning finds every overlapping read
        for bn, chunks in refs[tid][0].items():
            for a, b in chunks:
                assert a < b


def test_bai_on_write_equals_rebuild(synth_small, tmp_path):
    """BamWriter's index-on-close (align, synth) writes the same .bai as
    bam_index_build reading the finished BAM back (record virtual offsets
    from the writer's block table, incl. records ending at block edges)."""
    import shutil
    src = synth_small / "sample.bam"
    on_write = (str(src) + ".bai")
    bam = tmp_path / "copy.bam"
    shutil.copy(src, bam)
    H.check(H.lib.fcsg_bam_index(str(bam).encode()))
    a = open(on_write, "rb").read()
    b = open(str(bam) + ".bai", "rb").read()
    assert len(H.bgzf_blocks(src)) > 20 and a == b


# ------------------------------------------------------------------ VCF tail
def test_vcf_concat_bgzip_tabix(tmp_path):
    hdr = "##fileformat=VCFv4.2\n##contig=<ID=c1,length=500000>\n##contig=<ID=c2,length=90000>\n" \
          "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n"
    rng = random.Random(9)
    recs = sorted({("c1", rng.randrange(1, 500000)) for _ in range(3000)}) + \
        sorted({("c2", rng.randrange(1, 90000)) for _ in range(500)})
    lines = [f"{c}\t{p}\t.\t{'ACGT'[p % 4] * (1 + p % 3)}\tT\t50\tPASS\t." for c, p in recs]
    parts = [lines[:1000], lines[1000:2500], lines[2500:]]
    paths = []
    for i, part in enumerate(parts):
        f = tmp_path / f"part-{i}.vcf"
        f.write_text(hdr + "".join(x + "\n" for x in part))
        paths.append(str(f).encode())
    out = tmp_path / "all.vcf"
    arr = (C.c_char_p * 3)(*paths)
    H.check(H.lib.fcsg_vcf_concat(arr, 3, str(out).encode()))
    assert out.read_text() == hdr + "".join(x + "\n" for x in lines)
    gz = tmp_path / "all.vcf.gz"
    H.check(H.lib.fcsg_bgzf_compress_file(str(out).encode(), str(gz).encode()))
    H.check(H.lib.fcsg_tabix(str(gz).encode()))
    names, refs = H.parse_index(gzip.decompress((tmp_path / "all.vcf.gz.tbi").read_bytes()), b"TBI\x01")
    assert names == ["c1", "c2"]
    for voff, line in H.bgzf_text_with_voffsets(gz):
        if line.startswith("#"):
            continue
        c, p, _, ref = line.split("\t")[:4]
        tid = names.index(c)
        beg = int(p) - 1
        bins, lin = refs[tid]
        b = H.reg2bin(beg, beg + len(ref))
        assert any(a <= voff < e for a, e in bins[b]), (line, voff)
        assert lin[beg >> 14] <= voff
    # the one-pass bgzip + tabix (htc / mutect2's VCF tail) writes the same two files
    gz2 = tmp_path / "one.vcf.gz"
    H.check(H.lib.fcsg_bgzip_tabix(str(out).encode(), str(gz2).encode()))
    assert gz2.read_bytes() == gz.read_bytes()
    assert gzip.decompress((tmp_path / "one.vcf.gz.tbi").read_bytes()) == \
        gzip.decompress((tmp_path / "all.vcf.gz.tbi").read_bytes())
    # concat + bgzip + tabix in one pass over the parts (htc's tail): the same three files
    fused, gz3 = tmp_path / "fused.vcf", tmp_path / "fused.vcf.gz"
    H.check(H.lib.fcsg_vcf_concat_bgzip_tabix(arr, 3, str(fused).encode(), str(gz3).encode()))
    assert fused.read_bytes() == out.read_bytes() and gz3.read_bytes() == gz.read_bytes()
    assert gzip.decompress((tmp_path / "fused.vcf.gz.tbi").read_bytes()) == \
        gzip.decompress((tmp_path / "all.vcf.gz.tbi").read_bytes())


def test_vcf_concat_bgzip_tabix_fused_edges(tmp_path):
    """The fused tail on parts that are header-only, empty, end without '\\n',
    carry GVCF END= blocks and run past many 64 KiB blocks: the same files as
    vcf_concat + bgzip + tabix."""
    hdr = "##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS\n"
    rng = random.Random(3)
    pos, lines = 1, []
    for _ in range(30000):
        n = rng.randrange(1, 9)
        info = f"END={pos + n - 1}" if rng.random() < 0.8 else "DP=3;END=." if rng.random() < 0.5 else f"X=1;END={pos + 2}"
        lines.append(f"c1\t{pos}\t.\tA\t<NON_REF>\t.\t.\t{info}\tGT:DP\t0/0:{rng.randrange(40)}")
        pos += n
    bodies = ["".join(x + "\n" for x in lines[:12000]), "", "".join(x + "\n" for x in lines[12000:29000]),
              "\n".join(lines[29000:])]  # the last part ends without '\n'
    paths = []
    for i, body in enumerate(bodies):
        f = tmp_path / f"p{i}.g.vcf"
        f.write_text(hdr + body)
        paths.append(str(f).encode())
    (tmp_path / "empty.g.vcf").write_text("")
    paths.insert(2, str(tmp_path / "empty.g.vcf").encode())
    arr = (C.c_char_p * len(paths))(*paths)
    two, gz_two = tmp_path / "two.g.vcf", tmp_path / "two.g.vcf.gz"
    H.check(H.lib.fcsg_vcf_concat(arr, len(paths), str(two).encode()))
    H.check(H.lib.fcsg_bgzip_tabix(str(two).encode(), str(gz_two).encode()))
    one, gz_one = tmp_path / "one.g.vcf", tmp_path / "one.g.vcf.gz"
    H.check(H.lib.fcsg_vcf_concat_bgzip_tabix(arr, len(paths), str(one).encode(), str(gz_one).encode()))
    assert one.read_text() == hdr + "".join(x + "\n" for x in lines)
    assert one.read_bytes() == two.read_bytes() and gz_one.read_bytes() == gz_two.read_bytes()
    assert len(H.bgzf_blocks(gz_one)) > 20
    assert gzip.decompress((tmp_path / "one.g.vcf.gz.tbi").read_bytes()) == \
        gzip.decompress((tmp_path / "two.g.vcf.gz.tbi").read_bytes())
    # and tabix of the bgzipped file (the two-pass path) agrees
    H.check(H.lib.fcsg_tabix(str(gz_two).encode()))
    assert gzip.decompress((tmp_path / "one.g.vcf.gz.tbi").read_bytes()) == \
        gzip.decompress((tmp_path / "two.g.vcf.gz.tbi").read_bytes())
    # a missing part fails the call
    bad = (C.c_char_p * 2)(paths[0], str(tmp_path / "nope.g.vcf").encode())
    assert H.lib.fcsg_vcf_concat_bgzip_tabix(bad, 2, str(tmp_path / "x").encode(), str(tmp_path / "x.gz").encode()) != 0


def test_bgzip_tabix_one_pass_block_edges(tmp_path):
    """Lines ending exactly at a BGZF block's end (offset 0xff00), lines
    spanning blocks and a last line without a newline: the one-pass index
    equals the two-pass one (a reader's tell() semantics), and bulk concat
    keeps part 0's header, drops the others' and ends the last line."""
    B = 0xff00
    hdr = "##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n"
    body, pos = [], 1
    total = len(hdr)
    while total < 3 * B + 500:
        line = f"c1\t{pos}\t.\tA\tT\t50\tPASS\t"
        # pad the INFO column so that some lines end right at a block edge
        nxt = (total // B + 1) * B
        need = nxt - total - len(line) - 1
        line += ("X" * need if 0 < need < 40 else "DP=1")
        body.append(line)
        total += len(line) + 1
        pos += 7
    text = hdr + "\n".join(body)  # no final newline
    assert any((len(hdr) + sum(len(x) + 1 for x in body[:k + 1])) % B == 0 for k in range(len(body)))
    parts = [tmp_path / "p0.vcf", tmp_path / "p1.vcf"]
    half = len(body) // 2
    parts[0].write_text(hdr + "".join(x + "\n" for x in body[:half]))
    parts[1].write_text(hdr + "\n".join(body[half:]))
    plain = tmp_path / "all.vcf"
    arr = (C.c_char_p * 2)(*[str(p).encode() for p in parts])
    H.check(H.lib.fcsg_vcf_concat(arr, 2, str(plain).encode()))
    assert plain.read_text() == text + "\n"
    plain.write_text(text)
    gz = tmp_path / "two.vcf.gz"
    H.check(H.lib.fcsg_bgzf_compress_file(str(plain).encode(), str(gz).encode()))
    H.check(H.lib.fcsg_tabix(str(gz).encode()))
    gz1 = tmp_path / "one.vcf.gz"
    H.check(H.lib.fcsg_bgzip_tabix(str(plain).encode(), str(gz1).encode()))
    assert gz1.read_bytes() == gz.read_bytes()
    assert gzip.decompress((tmp_path / "one.vcf.gz.tbi").read_bytes()) == \
        gzip.decompress((tmp_path / "two.vcf.gz.tbi").read_bytes())


# ------------------------------------------------------------------ intervals
def ref_partition(dict_contigs, n, skip_pseudo=True):
    """Restatement of init_contig_intv's arithmetic (reference src/config.cpp:458-505)."""
    contigs = dict_contigs[:25] if skip_pseudo else dict_contigs
    total = sum(L for _, L in contigs)
    per = (total + n - 1) // n
    parts = [[] for _ in range(n)]
    remain, lb, k = per, 1, 0
    for name, L in contigs:
        npos = L
        while npos > remain:
            ub = remain + lb - 1
            parts[k].append((name, lb, ub))
            lb = ub + 1
            npos -= remain
            remain = per
            k += 1
        if npos > 0:
            parts[k].append((name, lb, L))
            remain -= npos
            lb = 1
    return parts


@pytest.mark.parametrize("n", [1, 3, 32])
def test_partition_matches_reference_rule(tmp_path, n):
    rng = random.Random(n)
    contigs = [(f"chr{i}", rng.randrange(1000, 300000)) for i in range(1, 30)]  # 29 > 25: pseudo contigs dropped
    d = tmp_path / "ref.dict"
    d.write_text("@HD\tVN:1.6\n" + "".join(f"@SQ\tSN:{c}\tLN:{L}\n" for c, L in contigs))
    buf = C.create_string_buffer(1 << 20)
    for skip in (1, 0):
        H.check(H.lib.fcsg_partition_dict(str(d).encode(), n, skip, buf, len(buf)))
        got = [[] for _ in range(n)]
        for ln in buf.value.decode().splitlines():
            k, c, lb, ub = ln.split("\t")
            got[int(k)].append((c, int(lb), int(ub)))
        assert got == ref_partition(contigs, n, bool(skip))
        covered = sum(ub - lb + 1 for p in got for _, lb, ub in p)
        assert covered == sum(L for _, L in (contigs[:25] if skip else contigs))


# ------------------------------------------------------------------ GATK read preparation
def test_gatk_prepare_read_rules():
    bases = b"ACGTNACGTA"
    q = np.array([2, 17, 18, 19, 40, 50, 60, 30, 10, 25], np.uint8)
    bi = bytes([33 + x for x in [45, 3, 6, 7, 40, 45, 45, 45, 0, 10]])
    out = [np.zeros(10, np.uint8) for _ in range(4)]
    ptr = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint8))  # noqa: E731
    H.check(H.lib.fcsg_prepare_read(bases, ptr(q), 10, bi, None, 30, 18, 0, *[ptr(o) for o in out]))
    bq, iq, dq, gcp = out
    # cap at MQ 30 first, then < 18 → 6
    assert bq.tolist() == [6, 6, 18, 19, 30, 30, 30, 30, 6, 25]
    assert iq.tolist() == [45, 6, 6, 7, 40, 45, 45, 45, 6, 10]  # BI tag, floored at 6
    assert dq.tolist() == [45] * 10  # no BD tag → 45
    assert gcp.tolist() == [10] * 10
    H.check(H.lib.fcsg_prepare_read(bases, ptr(q), 10, None, None, 10, 18, 0, *[ptr(o) for o in out]))
    assert out[0].tolist() == [6] * 10  # MQ 10 < 18 caps everything to 6


def test_pcr_indel_error_model():
    """GATK's --pcr-indel-model (PairHMMLikelihoodCalculationEngine, [EXT],
    restated; parity unpinned): the gap-open cap per tandem-repeat run length and
    its application to positions 0 .. n-2 before the floor at 6."""
    import math
    for model, rate in ((1, 1.0), (2, 2.0), (3, 3.0)):
        for rl in range(21):
            v = 40.0 - math.exp(rl / (rate * math.pi)) + 1.0
            assert H.lib.fcsg_pcr_indel_cap(rl, model) == max(10, int(v + 0.5)), (model, rl)
    assert H.lib.fcsg_pcr_indel_cap(20, 3) == 33 and H.lib.fcsg_pcr_indel_cap(20, 1) == 10
    rep = H.lib.fcsg_tandem_repeat_units
    assert rep(b"AAAAAAAAAA", 4) == 10          # (A)5 back + (A)5 forward
    assert rep(b"ACACACGT", 3) == 1             # back unit AC x2, forward unit A x1: A's back run is 0
    assert rep(b"ACACACAC", 3) == 4             # (AC)2 back + (AC)2 forward
    assert rep(b"A" * 30, 10) == 20             # capped at MAX_REPEAT_LENGTH
    assert rep(b"TTCTTCCCC", 5) == 4            # GATK's comment: TTCTT(C)CCC is (C)4, not (TTC)2
    bases = b"GATTTTTTTTCAG"
    n = len(bases)
    q = np.full(n, 30, np.uint8)
    out = [np.zeros(n, np.uint8) for _ in range(4)]
    ptr = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint8))  # noqa: E731
    H.check(H.lib.fcsg_prepare_read(bases, ptr(q), n, None, None, 60, 18, 3, *[ptr(o) for o in out]))
    caps = [H.lib.fcsg_pcr_indel_cap(rep(bases, i), 3) for i in range(n - 1)]
    assert out[1].tolist() == [min(45, c) for c in caps] + [45]  # the last base keeps its GOP
    assert out[2].tolist() == out[1].tolist()
    assert min(caps) < 40  # the T run lowers the caps inside it
    H.check(H.lib.fcsg_prepare_read(bases, ptr(q), n, None, None, 60, 18, 0, *[ptr(o) for o in out]))
    assert out[1].tolist() == [45] * n  # NONE


def test_tandem_repeat_runs_equal_per_offset_scan():
    """The O(8 n) all-offsets run lengths the read preparation uses equal
    findTandemRepeatUnits evaluated offset by offset, on random reads and on
    reads built from short repeated units (the cases with long runs, unit
    changes at the offset and the 20 cap)."""
    rng = np.random.default_rng(11)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    reads = [b"AC", b"AAAAAAAAAA", b"TTCTTCCCC", b"ACACACGT", b"A" * 40,
             b"A" * 600, b"ACG" * 200, b"C" * 300 + b"ACGTTGCA" * 40]  # runs past the 255 saturation
    for _ in range(400):
        if rng.random() < 0.4:
            reads.append(rng.choice(acgt, int(rng.integers(2, 160))).tobytes())
        else:
            parts = []
            while sum(map(len, parts)) < 120:
                unit = rng.choice(acgt, int(rng.integers(1, 10))).tobytes()
                parts.append(unit * int(rng.integers(1, 8)))
            reads.append(b"".join(parts)[: int(rng.integers(2, 160))])
    for r in reads:
        out = np.zeros(len(r), np.uint8)
        H.lib.fcsg_tandem_repeat_runs(r, len(r), out.ctypes.data_as(C.POINTER(C.c_uint8)))
        want = [H.lib.fcsg_tandem_repeat_units(r, i) for i in range(len(r) - 1)]
        assert out[: len(r) - 1].tolist() == want, r


# ------------------------------------------------------------------ executor
def test_executor_slots_logs_and_failure(tmp_path):
    buf = C.create_string_buffer(1 << 16)
    cmd = f"echo $FCS_GPU_DEVICE > {tmp_path}/slot.%d".encode()
    rc = H.lib.fcsg_run_stage(cmd, 10, 3, b"0,2,5", str(tmp_path / "log").encode(), buf, len(buf))
    assert rc == 0
    slots = [int((tmp_path / f"slot.{i}").read_text()) for i in range(10)]
    assert sorted(slots) == sorted([0, 2, 5][i % 3] for i in range(10))  # job_id % n over the slot list
    fail = b"sh -c 'if [ %d -eq 3 ]; then echo \"[E::bwa] cannot open x\"; exit 2; fi; echo fine'"
    rc = H.lib.fcsg_run_stage(fail, 5, 2, b"", str(tmp_path / "log2").encode(), buf, len(buf))
    assert rc == 4  # failedCommand → exit code 4 in the CLI
    logs = sorted(p for p in os.listdir(tmp_path / "log2") if ".part-" not in p)
    assert logs and "[E::bwa] cannot open x" in (tmp_path / "log2" / logs[0]).read_text()


def test_find_error_semantics(tmp_path):
    a, b, c = tmp_path / "a.log", tmp_path / "b.log", tmp_path / "c.log"
    a.write_text("start\n[E::x] bad thing\nend\n")
    b.write_text("start\n[E::x] bad thing\nend\n")
    c.write_text("nothing here\nlast line\n")
    buf = C.create_string_buffer(4096)
    arr = lambda *p: (C.c_char_p * len(p))(*[str(x).encode() for x in p])  # noqa: E731
    H.lib.fcsg_find_error(arr(a, b), 2, buf, len(buf))
    assert buf.value.decode() == "[E::x] bad thing\n"  # shared across logs
    H.lib.fcsg_find_error(arr(c), 1, buf, len(buf))
    assert buf.value.decode() == "last line\n"  # no marker: last line


# ------------------------------------------------------------------ CLI surface
def test_cli_exit_codes(tmp_path, synth_small):
    assert H.run_cli(cwd=tmp_path).returncode == 1  # no command: help + 1
    p = H.run_cli("conf", cwd=tmp_path)
    assert p.returncode == 1 and "gatk.ncontigs" in p.stderr and "gpu.devices" in p.stderr
    assert H.run_cli("htc", "--help", cwd=tmp_path).returncode == 0
    assert H.run_cli("htc", "-r", "x", cwd=tmp_path).returncode == 1  # missing required options
    p = H.run_cli("htc", "-r", tmp_path / "nope.fasta", "-i", synth_small / "sample.bam", "-o", tmp_path / "o.vcf",
                  env={"FCS_GPU_DEVICES": "0"}, cwd=tmp_path)
    assert p.returncode in (3, 4)  # missing reference (3); on a GPU-less host the slot check may fire first (4)
    p = H.run_cli("bogus", cwd=tmp_path)
    assert p.returncode == 1
    # config precedence: ./fcs-genome.conf below the environment
    (tmp_path / "fcs-genome.conf").write_text("[gatk]\nncontigs = 7\n")
    p = H.run_cli("conf", cwd=tmp_path)
    assert "gatk.ncontigs = 7" in p.stderr
    p = H.run_cli("conf", cwd=tmp_path, env={"FCS_GATK_NCONTIGS": "9"})
    assert "gatk.ncontigs = 9" in p.stderr


def test_tabix_gvcf_block_end_from_info(tmp_path):
    """A GVCF <NON_REF> block is indexed over [POS, INFO END] as htslib's VCF
    preset does (tbx_parse1): a query that starts inside a multi-window block
    finds it through both its bin and the linear index."""
    hdr = "##fileformat=VCFv4.2\n##contig=<ID=c1,length=200000>\n" \
          "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS\n"
    lines = ["c1\t100\t.\tA\tT\t50\tPASS\tDP=9\tGT\t0/1",
             "c1\t101\t.\tC\t<NON_REF>\t.\t.\tEND=40000\tGT:DP\t0/0:30",     # spans windows 0..2
             "c1\t40001\t.\tG\t<NON_REF>\t.\t.\tDP=3;END=40010\tGT:DP\t0/0:3",  # END= after another field
             "c1\t40011\t.\tGTT\tG\t50\tPASS\tEND=.\tGT\t0/1",                # END=. is ignored
             "c1\t50000\t.\tA\t<NON_REF>\t.\t.\tXEND=60000\tGT\t0/0"]         # not an END field
    plain = tmp_path / "b.g.vcf"
    plain.write_text(hdr + "".join(x + "\n" for x in lines))
    gz = tmp_path / "b.g.vcf.gz"
    H.check(H.lib.fcsg_bgzip_tabix(str(plain).encode(), str(gz).encode()))
    names, refs = H.parse_index(gzip.decompress((tmp_path / "b.g.vcf.gz.tbi").read_bytes()), b"TBI\x01")
    bins, lin = refs[0]
    ends = {101: 40000, 40001: 40010, 40011: 40013, 100: 100, 50000: 50000}
    voffs = {int(line.split("\t")[1]): v for v, line in H.bgzf_text_with_voffsets(gz) if not line.startswith("#")}
    for pos, end in ends.items():
        b = H.reg2bin(pos - 1, end)
        assert any(a <= voffs[pos] < e for a, e in bins[b]), (pos, b)
    # a query at 30,000 (window 1) must start no later than the block at 101
    assert lin[30000 >> 14] <= voffs[101] and lin[(40000 - 1) >> 14] <= voffs[101]
    # the two-pass indexer (read back from the .gz) builds the same index
    gz2 = tmp_path / "c.g.vcf.gz"
    H.check(H.lib.fcsg_bgzf_compress_file(str(plain).encode(), str(gz2).encode()))
    H.check(H.lib.fcsg_tabix(str(gz2).encode()))
    assert gzip.decompress((tmp_path / "c.g.vcf.gz.tbi").read_bytes()) == \
        gzip.decompress((tmp_path / "b.g.vcf.gz.tbi").read_bytes())
