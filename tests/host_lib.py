"""ctypes access to libfcsgenome.so (the C++ orchestrator's test hooks,
falcon-genome_amd/host/capi.cpp) and the fcs-genome binary, plus small
independent readers of the on-disk formats (BGZF via Python's gzip, BAM
records, BAI/TBI) that the tests check the C++ writers against."""
import ctypes as C
import gzip
import os
import struct
import subprocess

import fcship  # noqa: F401  (loads torch + libfcship first: one HIP runtime per process)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "falcon-genome_amd")
# FCS_SAN=address|thread|undefined selects the sanitizer build (tools/sanitize.sh)
SAN = os.environ.get("FCS_SAN", "")
_DIR = os.path.join(PKG, "_san", SAN) if SAN else PKG
BIN = os.path.join(_DIR, "bin", "fcs-genome")
LIB_PATH = os.path.join(_DIR, "libfcsgenome.so")

lib = C.CDLL(LIB_PATH)
lib.fcsg_last_error.restype = C.c_char_p
lib.fcsg_reg2bin.restype = C.c_uint
lib.fcsg_reg2bin.argtypes = [C.c_longlong, C.c_longlong]


def check(rc):
    if rc < 0:
        raise RuntimeError(lib.fcsg_last_error().decode())
    return rc


def run_cli(*args, env=None, timeout=600, cwd=None):
    e = dict(os.environ)
    if env:
        e.update(env)
    return subprocess.run([BIN, *map(str, args)], capture_output=True, text=True, env=e, timeout=timeout, cwd=cwd)


# ------------------------------------------------------------ independent readers
def bgzf_blocks(path):
    """(offset, BSIZE, ISIZE) of every BGZF block, parsed from the raw bytes."""
    data = open(path, "rb").read()
    out, off = [], 0
    while off < len(data):
        assert data[off:off + 4] == b"\x1f\x8b\x08\x04", f"bad block magic at {off}"
        xlen = struct.unpack_from("<H", data, off + 10)[0]
        extra = data[off + 12: off + 12 + xlen]
        bsize = None
        k = 0
        while k + 4 <= xlen:
            si1, si2, slen = extra[k], extra[k + 1], struct.unpack_from("<H", extra, k + 2)[0]
            if si1 == 66 and si2 == 67 and slen == 2:
                bsize = struct.unpack_from("<H", extra, k + 4)[0] + 1
            k += 4 + slen
        assert bsize is not None, "no BC subfield"
        isize = struct.unpack_from("<I", data, off + bsize - 4)[0]
        out.append((off, bsize, isize))
        off += bsize
    return out


def read_bam(path):
    """Header (names, lengths) and records as dicts, decoded from gzip-inflated bytes."""
    raw = gzip.decompress(open(path, "rb").read())
    assert raw[:4] == b"BAM\x01"
    l_text = struct.unpack_from("<i", raw, 4)[0]
    p = 8 + l_text
    n_ref = struct.unpack_from("<i", raw, p)[0]
    p += 4
    names, lens = [], []
    for _ in range(n_ref):
        ln = struct.unpack_from("<i", raw, p)[0]
        names.append(raw[p + 4: p + 4 + ln - 1].decode())
        lens.append(struct.unpack_from("<i", raw, p + 4 + ln)[0])
        p += 8 + ln
    recs = []
    nt16 = "=ACMGRSVTWYHKDBN"
    while p < len(raw):
        bs = struct.unpack_from("<i", raw, p)[0]
        b = raw[p + 4: p + 4 + bs]
        ref_id, pos, l_name, mapq, bin_, n_cig, flag, l_seq, nref, npos, tlen = struct.unpack_from("<iiBBHHHiiii", b, 0)
        k = 32
        name = b[k:k + l_name - 1].decode()
        k += l_name
        cig = struct.unpack_from(f"<{n_cig}I", b, k)
        k += 4 * n_cig
        seq = "".join(nt16[(b[k + i // 2] >> (4 * (1 - i % 2))) & 0xF] for i in range(l_seq))
        k += (l_seq + 1) // 2
        qual = b[k:k + l_seq]
        k += l_seq
        recs.append(dict(ref_id=ref_id, pos=pos, mapq=mapq, bin=bin_, flag=flag, name=name, next_ref_id=nref,
                         next_pos=npos, tlen=tlen,
                         cigar=["%d%s" % (c >> 4, "MIDNSHP=X"[c & 15]) for c in cig], seq=seq,
                         qual=bytes(qual), aux=bytes(b[k:]), voff=None))
        p += 4 + bs
    return names, lens, recs


def parse_aux(aux):
    """BAM aux bytes -> {tag: value} (Z strings, integer types)."""
    out, k = {}, 0
    ints = {"c": "<b", "C": "<B", "s": "<h", "S": "<H", "i": "<i", "I": "<I"}
    while k < len(aux):
        tag, t = aux[k:k + 2].decode(), chr(aux[k + 2])
        k += 3
        if t == "Z":
            e = aux.index(0, k)
            out[tag] = aux[k:e].decode()
            k = e + 1
        elif t in ints:
            out[tag] = struct.unpack_from(ints[t], aux, k)[0]
            k += struct.calcsize(ints[t])
        elif t == "A":
            out[tag] = chr(aux[k])
            k += 1
        else:
            raise ValueError(f"aux type {t}")
    return out


def cigar_ref_len(cig):
    n = 0
    for c in cig:
        if c[-1] in "MDN=X":
            n += int(c[:-1])
    return n


def reg2bin(beg, end):
    """SAM spec §5.3."""
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


def parse_index(data, magic):
    """BAI (raw) or TBI (after inflating) → per-ref (bins{bin: [(beg, end)]}, linear[])."""
    assert data[:4] == magic
    n_ref = struct.unpack_from("<i", data, 4)[0]
    p = 8
    names = []
    if magic == b"TBI\x01":
        fmt, cs, cb, ce, meta, skip, l_nm = struct.unpack_from("<7i", data, 8)
        p = 36
        names = [n.decode() for n in data[p:p + l_nm].split(b"\x00")[:-1]]
        p += l_nm
    refs = []
    for _ in range(n_ref):
        n_bin = struct.unpack_from("<i", data, p)[0]
        p += 4
        bins = {}
        for _ in range(n_bin):
            bn, n_ch = struct.unpack_from("<Ii", data, p)
            p += 8
            bins[bn] = [struct.unpack_from("<QQ", data, p + 16 * i) for i in range(n_ch)]
            p += 16 * n_ch
        n_int = struct.unpack_from("<i", data, p)[0]
        p += 4
        lin = list(struct.unpack_from(f"<{n_int}Q", data, p))
        p += 8 * n_int
        refs.append((bins, lin))
    return names, refs


def bgzf_text_with_voffsets(path):
    """Lines of a BGZF text file with the virtual offset each line starts at."""
    blocks = bgzf_blocks(path)
    raw = open(path, "rb").read()
    out, carry, carry_voff = [], b"", None
    for off, bsize, isize in blocks:
        payload = gzip.decompress(raw[off:off + bsize]) if isize else b""
        i = 0
        while i < len(payload):
            if carry_voff is None:
                carry_voff = (off << 16) | i
            j = payload.find(b"\n", i)
            if j < 0:
                carry += payload[i:]
                break
            out.append((carry_voff, (carry + payload[i:j]).decode()))
            carry, carry_voff = b"", None
            i = j + 1
    return out
