"""Shared `fcs-genome align` cases for the GPU tests (real libfcship) and the
CPU host-logic tests (tests/cpu_mock: the banded-SW entry points computed by
the oracle).  Split reads: bwa mem_mark_primary_se / mem_reg2sam semantics."""
import numpy as np

import host_lib as H


def read_fasta(path):
    contigs, name = {}, None
    for ln in open(path).read().split("\n"):
        if ln.startswith(">"):
            name = ln[1:].split()[0]
            contigs[name] = []
        elif ln:
            contigs[name].append(ln)
    return {k: "".join(v) for k, v in contigs.items()}


def revcomp(s):
    return s.translate(str.maketrans("ACGTN", "TGCAN"))[::-1]


def split_reads_fastq(ref_fasta, fq, n_split, n_whole, seed, c1="chr20", c2="chr21"):
    """Chimeric 150-base reads: 55-70 bases of c1 (forward) + the reverse
    complement of 80-95 bases of c2; plus unsplit reads of c1.  Returns the
    truth {name: (a, l1, b, l2)} / {name: (a,)}."""
    rng = np.random.default_rng(seed)
    contigs = read_fasta(ref_fasta)
    truth, lines = {}, []
    for i in range(n_split):
        l1 = int(rng.integers(55, 71))
        l2 = 150 - l1
        while True:
            a = int(rng.integers(1000, len(contigs[c1]) - 1000))
            b = int(rng.integers(1000, len(contigs[c2]) - 1000))
            p1, p2 = contigs[c1][a:a + l1], contigs[c2][b:b + l2]
            if "N" not in p1 + p2:
                break
        truth[f"split{i}"] = (a, l1, b, l2)
        lines += [f"@split{i}", p1 + revcomp(p2), "+", "I" * 150]
    for i in range(n_whole):
        a = int(rng.integers(1000, len(contigs[c1]) - 1000))
        lines += [f"@whole{i}", contigs[c1][a:a + 150], "+", "I" * 150]
        truth[f"whole{i}"] = (a,)
    open(fq, "w").write("\n".join(lines) + "\n")
    return truth


def check_split_reads(bam, truth, c1="chr20", c2="chr21"):
    """The longer part is the primary (soft clips, its start exact), the shorter
    one a supplementary record (flag 0x800, hard clips, SEQ of the aligned part
    only, MAPQ <= the primary's), each with an SA tag naming the other; unsplit
    reads keep one record.  Returns (split reads placed right, the others)."""
    names, _, recs = H.read_bam(bam)
    by = {}
    for r in recs:
        by.setdefault(r["name"], []).append(r)
    cig = lambda r: "".join(r["cigar"])
    good, bad = 0, []
    for nm, t in truth.items():
        rs = by[nm]
        prim = [r for r in rs if not r["flag"] & 0x800]
        assert len(prim) == 1, (nm, [cig(r) for r in rs])
        if len(t) == 1:
            assert len(rs) == 1 and prim[0]["pos"] == t[0] and names[prim[0]["ref_id"]] == c1
            continue
        a, l1, b, l2 = t
        sup = [r for r in rs if r["flag"] & 0x800]
        if len(sup) != 1:
            bad.append((nm, t, [(r["flag"], names[r["ref_id"]], r["pos"], cig(r), r["mapq"]) for r in rs]))
            continue
        P, S = prim[0], sup[0]
        ok = (names[P["ref_id"]], P["pos"], bool(P["flag"] & 0x10)) == (c2, b, True)
        ok &= (names[S["ref_id"]], S["pos"], bool(S["flag"] & 0x10)) == (c1, a, False)
        assert "H" not in cig(P) and "S" in cig(P), cig(P)
        assert "S" not in cig(S) and "H" in cig(S), cig(S)
        aligned = sum(int(c[:-1]) for c in S["cigar"] if c[-1] in "MI")
        assert len(S["seq"]) == aligned
        assert S["mapq"] <= P["mapq"]
        xp, xs = H.parse_aux(P["aux"]), H.parse_aux(S["aux"])
        assert xp["SA"] == f"{c1},{a + 1},+,{cig(S).replace('H', 'S')},{S['mapq']},{xs['NM']};", xp["SA"]
        assert xs["SA"] == f"{c2},{b + 1},-,{cig(P)},{P['mapq']},{xp['NM']};", xs["SA"]
        if ok:
            good += 1
        else:
            bad.append((nm, t, [(r["flag"], names[r["ref_id"]], r["pos"], cig(r), r["mapq"]) for r in rs]))
    return good, bad


def check_pairs(stderr, bam, truth_tsv, damaged, sd_range=(35, 65)):
    """Paired-end output against synth --paired's truth (FR pairs of N(350, 50)
    fragments): the insert-size estimate, placement, proper-pair flags, mate
    fields (bwa mem_aln2sam: an unmapped read takes its mate's place and
    strand), bwa's TLEN from the 5' ends, and the rescue of `damaged` read-2
    mates (names)."""
    import re
    truth = {}
    for line in open(truth_tsv):
        name, mate, contig, pos, rev = line.split()
        truth[(name, int(mate))] = (int(contig), int(pos), int(rev))
    m = re.search(r"insert ([\d.]+) \+- ([\d.]+) \[(\d+), (\d+)\] from (\d+) pairs", stderr)
    assert m, stderr[-1000:]
    avg, sd = float(m.group(1)), float(m.group(2))
    assert abs(avg - 350) < 15 and sd_range[0] < sd < sd_range[1], (avg, sd)
    _, _, recs = H.read_bam(bam)
    by = {}
    for r in recs:
        if r["flag"] & 0x800:
            continue
        by[(r["name"], 1 if r["flag"] & 0x40 else 2)] = r
    assert len(by) == len(truth)
    ok = mapped = proper = resc_ok = 0
    end5 = lambda r: r["pos"] + (H.cigar_ref_len(r["cigar"]) - 1 if r["flag"] & 0x10 else 0)
    for (name, mate), r in by.items():
        assert r["flag"] & 0x1 and (r["flag"] & 0xC0) in (0x40, 0x80)
        o = by[(name, 3 - mate)]
        assert r["next_pos"] == o["pos"] and r["next_ref_id"] == o["ref_id"]
        assert bool(r["flag"] & 0x8) == bool(o["flag"] & 0x4)
        assert bool(r["flag"] & 0x20) == bool(o["flag"] & 0x10)
        if r["flag"] & 0x4:
            assert r["tlen"] == 0
            continue
        mapped += 1
        if not o["flag"] & 0x4 and o["ref_id"] == r["ref_id"]:
            p0, p1 = end5(r), end5(o)
            assert r["tlen"] == -(p0 - p1 + (1 if p0 > p1 else -1 if p0 < p1 else 0)), (r["tlen"], p0, p1)
        c, pos, rev = truth[(name, mate)]
        # the unclipped start: a mate placed by the rescue's local alignment
        # (bwa ksw_align2, no end bonus) may soft-clip a damaged end
        lead = int(r["cigar"][0][:-1]) if r["cigar"] and r["cigar"][0][-1] == "S" else 0
        hit = (r["ref_id"], r["pos"] - lead, bool(r["flag"] & 0x10)) == (c, pos, bool(rev))
        ok += hit
        if r["flag"] & 0x2:
            proper += 1
            assert r["tlen"] == -o["tlen"] and abs(r["tlen"]) > 0
        if mate == 2 and name in damaged:
            resc_ok += hit
    n = len(truth)
    assert mapped / n >= 0.99, (mapped, n)
    assert ok / mapped >= 0.97, (ok, mapped)
    assert proper / n >= 0.95, (proper, n)
    assert resc_ok >= 0.8 * len(damaged), (resc_ok, len(damaged))
    nres = int(re.search(r"(\d+) mates rescued", stderr).group(1))  # reads placed by the mate rescue
    assert nres >= 0.8 * len(damaged), (nres, len(damaged))


def damage_mates(fastq, every=25, offset=7):
    """A mismatch every 16 bases in every `every`-th read of `fastq` (no
    19-mer seeds them: only the mate rescue can place them).  Returns their names."""
    lines = open(fastq).read().split("\n")
    damaged = set()
    flip = {"A": "C", "C": "G", "G": "T", "T": "A", "N": "A"}
    for i in range(0, len(lines) - 3, 4):
        if (i // 4) % every == offset:
            seq = list(lines[i + 1])
            for j in range(5, len(seq), 16):
                seq[j] = flip[seq[j]]
            lines[i + 1] = "".join(seq)
            damaged.add(lines[i][1:].split("/")[0])
    open(fastq, "w").write("\n".join(lines))
    return damaged


def append_chimeric_pairs(ref_fasta, fq1, fq2, n, seed, c1, c2, frag=350):
    """Pairs whose read 1 is split: its first 60 bases are the reverse
    complement of a c2 segment, the other 90 continue the fragment on c1
    (forward); read 2 is the fragment's far end (reverse strand).  Appended to
    the FASTQs.  Returns {name: (f, b)}: fragment start on c1, c2 segment start."""
    rng = np.random.default_rng(seed)
    contigs = read_fasta(ref_fasta)
    out, a1, a2 = {}, [], []
    for i in range(n):
        while True:
            f = int(rng.integers(1000, len(contigs[c1]) - 1000))
            b = int(rng.integers(1000, len(contigs[c2]) - 1000))
            s1 = revcomp(contigs[c2][b:b + 60]) + contigs[c1][f + 60:f + 150]
            s2 = revcomp(contigs[c1][f + frag - 150:f + frag])
            if "N" not in s1 + s2:
                break
        out[f"chim{i}"] = (f, b)
        a1 += [f"@chim{i}/1", s1, "+", "I" * 150]
        a2 += [f"@chim{i}/2", s2, "+", "I" * 150]
    for path, add in ((fq1, a1), (fq2, a2)):
        txt = open(path).read()
        if txt and not txt.endswith("\n"):
            txt += "\n"
        open(path, "w").write(txt + "\n".join(add) + "\n")
    return out


def check_chimeric_pairs(bam, chim, c1, c2, frag=350):
    """bwa mem_sam_pe with a split read 1 (is_multi: no pairing): read 1 gives
    its primary (the 90 c1 bases, soft clips) and a supplementary record (the
    60 c2 bases, hard clips); every record of the pair carries the mate fields
    of the other read's primary and the proper-pair flag of the top hits."""
    names, _, recs = H.read_bam(bam)
    by = {}
    for r in recs:
        if r["name"] in chim:
            by.setdefault(r["name"], []).append(r)
    good = 0
    for nm, (f, b) in chim.items():
        rs = by[nm]
        r1 = [r for r in rs if r["flag"] & 0x40]
        r2 = [r for r in rs if r["flag"] & 0x80]
        p1 = [r for r in r1 if not r["flag"] & 0x800]
        s1 = [r for r in r1 if r["flag"] & 0x800]
        if not (len(p1) == 1 and len(s1) == 1 and len(r2) == 1):
            continue
        P, S, M = p1[0], s1[0], r2[0]
        # the junction side of each part may absorb a few bases that match by chance
        ok = (names[P["ref_id"]], bool(P["flag"] & 0x10)) == (c1, False) and f + 57 <= P["pos"] <= f + 60
        ok &= (names[S["ref_id"]], bool(S["flag"] & 0x10)) == (c2, True) and b - 3 <= S["pos"] <= b
        ok &= (names[M["ref_id"]], M["pos"], bool(M["flag"] & 0x10)) == (c1, f + frag - 150, True)
        assert "H" in "".join(S["cigar"]) and "S" in "".join(P["cigar"])
        for r in (P, S):
            assert (r["next_ref_id"], r["next_pos"]) == (M["ref_id"], M["pos"]) and r["flag"] & 0x20
        assert (M["next_ref_id"], M["next_pos"]) == (P["ref_id"], P["pos"]) and not M["flag"] & 0x20
        assert "SA" in H.parse_aux(P["aux"]) and "SA" in H.parse_aux(S["aux"])
        ok &= all(bool(r["flag"] & 0x2) for r in (P, S, M))
        good += bool(ok)
    return good
