"""BGZF members built in Python for the inflate tests:
zlib at every level and strategy, libdeflate (the codec the host writes BAM
and GVCF with) when the image has it, stored blocks, the 28-byte EOF member,
and payloads shaped like BAM records, GVCF text, random bytes and runs."""
import ctypes
import struct
import zlib

import numpy as np

EOF_MEMBER = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def member(payload: bytes, level: int = 6, strategy: int = zlib.Z_DEFAULT_STRATEGY, raw: bytes | None = None) -> bytes:
    """One BGZF member (RFC 1952 header with the BC extra field) of `payload`;
    `raw` replaces the DEFLATE stream (for corrupt-stream cases)."""
    if raw is None:
        c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
        raw = c.compress(payload) + c.flush()
    bsize = 12 + 6 + len(raw) + 8 - 1
    assert bsize < 65536
    head = bytes([31, 139, 8, 4, 0, 0, 0, 0, 0, 255]) + struct.pack("<H", 6) + b"BC" + struct.pack("<HH", 2, bsize)
    return head + raw + struct.pack("<II", zlib.crc32(payload) & 0xFFFFFFFF, len(payload))


_LIBDEFLATE = None


def libdeflate():
    global _LIBDEFLATE
    if _LIBDEFLATE is None:
        try:
            L = ctypes.CDLL("libdeflate.so.0")
            L.libdeflate_alloc_compressor.restype = ctypes.c_void_p
            L.libdeflate_alloc_compressor.argtypes = [ctypes.c_int]
            L.libdeflate_deflate_compress.restype = ctypes.c_size_t
            L.libdeflate_deflate_compress.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t,
                                                      ctypes.c_char_p, ctypes.c_size_t]
            L.libdeflate_free_compressor.argtypes = [ctypes.c_void_p]
            _LIBDEFLATE = L
        except OSError:
            _LIBDEFLATE = False
    return _LIBDEFLATE or None


def member_libdeflate(payload: bytes, level: int) -> bytes:
    L = libdeflate()
    comp = L.libdeflate_alloc_compressor(level)
    buf = ctypes.create_string_buffer(len(payload) + 1024)
    n = L.libdeflate_deflate_compress(comp, payload, len(payload), buf, len(buf))
    L.libdeflate_free_compressor(comp)
    assert n > 0
    return member(payload, raw=buf.raw[:n])


def flushed_member(payload: bytes, pieces: int, level: int = 6, flush: int = zlib.Z_SYNC_FLUSH) -> bytes:
    """One member of several DEFLATE blocks: the payload compressed in pieces
    with a flush after each (a sync flush adds an empty stored block, a full
    flush also resets the window)."""
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY)
    step = max(1, len(payload) // pieces)
    raw = b""
    for k in range(0, len(payload), step):
        raw += c.compress(payload[k:k + step]) + c.flush(flush)
    raw += c.flush()
    return member(payload, raw=raw)


def stored_member(payload: bytes) -> bytes:
    """One stored (type 0) block: LEN, NLEN, the bytes."""
    assert len(payload) < 65536 - 64
    raw = bytes([1]) + struct.pack("<HH", len(payload), len(payload) ^ 0xFFFF) + payload
    return member(payload, raw=raw)


def payload(rng: np.random.Generator, kind: str, n: int) -> bytes:
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    if kind == "runs":
        v = rng.integers(0, 256, max(1, n // 50), dtype=np.uint8)
        return np.repeat(v, rng.integers(1, 100, len(v)))[:n].tobytes().ljust(n, b"A")
    if kind == "gvcf":
        out = []
        pos = 1000
        while sum(map(len, out)) < n:
            pos += int(rng.integers(1, 200))
            out.append(f"chr1\t{pos}\t.\t{'ACGT'[pos % 4]}\t<NON_REF>\t.\t.\tEND={pos + int(rng.integers(0, 50))}"
                       f"\tGT:DP:GQ:MIN_DP:PL\t0/0:{int(rng.integers(0, 60))}:99:30:0,90,1350\n")
        return "".join(out).encode()[:n]
    if kind == "bam":  # record-shaped: fixed fields, name, CIGAR, 4-bit bases, qualities
        out = bytearray()
        pos = 10000
        while len(out) < n:
            pos += int(rng.integers(0, 40))
            l_seq = 151
            name = f"read{pos}:{int(rng.integers(0, 1 << 20))}".encode() + b"\0"
            body = struct.pack("<iiBBHHHiiii", 0, pos, len(name), 60, 4680, 1, 99, l_seq, 0, pos + 200, 350)
            body += name + struct.pack("<I", (l_seq << 4) | 0)
            body += rng.integers(0, 256, (l_seq + 1) // 2, dtype=np.uint8).tobytes()
            q = np.clip(rng.normal(34, 4, l_seq), 2, 41).astype(np.uint8)
            body += q.tobytes()
            out += struct.pack("<i", len(body)) + body
        return bytes(out[:n])
    raise ValueError(kind)


def suite(seed: int = 3, count: int = 120) -> list[tuple[str, bytes, bytes]]:
    """(label, member bytes, payload) over every codec setting and payload kind."""
    rng = np.random.default_rng(seed)
    raw = payload(rng, "random", 60000)
    cases = [("eof", EOF_MEMBER, b""), ("empty-l6", member(b""), b""), ("one-byte", member(b"x"), b"x"),
             ("stored", stored_member(raw), raw)]
    for kind, pieces, fl in (("bam", 7, zlib.Z_SYNC_FLUSH), ("gvcf", 13, zlib.Z_FULL_FLUSH), ("runs", 3, zlib.Z_SYNC_FLUSH)):
        p = payload(rng, kind, 50000)
        cases.append((f"{kind}-{pieces}-blocks", flushed_member(p, pieces, 6, fl), p))
    kinds = ["random", "runs", "gvcf", "bam"]
    strategies = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FILTERED]
    for i in range(count):
        kind = kinds[i % 4]
        n = int(rng.integers(0, 65281)) if i % 7 else int(rng.integers(0, 300))
        if kind == "random":
            n = min(n, 65000)  # zlib's stored fallback must still fit one member
        p = payload(rng, kind, n)
        if i % 3 == 0 and libdeflate():
            lvl = int(rng.integers(1, 13))
            cases.append((f"{kind}-libdeflate{lvl}-{n}", member_libdeflate(p, lvl), p))
        else:
            lvl = int(rng.integers(0, 10))
            st = strategies[int(rng.integers(0, 5))]
            cases.append((f"{kind}-zlib{lvl}s{st}-{n}", member(p, lvl, st), p))
    return cases
