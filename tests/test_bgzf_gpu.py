"""GPU parity: BGZF member inflation (fcs_bgzf_inflate / _dev, SURVEY.md §8
row f3) against zlib.

Bar: bit-exact — every inflated byte equals zlib's, for members written by
zlib at every level and strategy, by libdeflate (the host's BAM / GVCF codec),
stored blocks, empty and EOF members, and a whole BAM from `fcs-genome
synth`; corrupt streams, CRC mismatches and lying ISIZEs are reported per
member, never written out.
"""
import struct
import zlib

import numpy as np
import pytest

import bgzf_cases
import fcship

pytestmark = pytest.mark.gpu


def test_inflate_members_one_by_one(gpu):
    for label, m, p in bgzf_cases.suite(seed=11, count=60):
        out, used = fcship.bgzf_inflate(m, device=gpu)
        assert used == len(m), label
        assert out == p, label


def test_inflate_concatenated_batch(gpu):
    cases = bgzf_cases.suite(seed=12, count=400)
    blob = b"".join(m for _, m, _ in cases)
    out, used = fcship.bgzf_inflate(blob, device=gpu)
    assert used == len(blob)
    assert out == b"".join(p for _, _, p in cases)


def test_inflate_whole_bam(gpu, tmp_path):
    import host_lib as H
    p = H.run_cli("synth", "-o", tmp_path, "-c", "chrA:200000", "-x", "10", "--seed", "4")
    assert p.returncode == 0, p.stderr
    blob = (tmp_path / "sample.bam").read_bytes()
    coff, _, _ = fcship.bgzf_index(blob)
    want = b"".join(zlib.decompress(blob[coff[k] + 18:coff[k + 1] - 8], -15) for k in range(len(coff) - 1))
    out, used = fcship.bgzf_inflate(blob, device=gpu)
    assert used == len(blob) and out == want


def test_trailing_partial_member_is_left(gpu):
    cases = bgzf_cases.suite(seed=13, count=8)
    blob = b"".join(m for _, m, _ in cases)
    out, used = fcship.bgzf_inflate(blob[:-5], device=gpu)
    assert used == len(blob) - len(cases[-1][1])
    assert out == b"".join(p for _, _, p in cases[:-1])


def _with_bad(cases, k, bad):
    return b"".join(bad if i == k else m for i, (_, m, _) in enumerate(cases))


def test_corruption_is_reported_per_member(gpu):
    rng = np.random.default_rng(14)
    cases = [c for c in bgzf_cases.suite(seed=14, count=40) if len(c[2]) > 1000]
    k = 3
    m = bytearray(cases[k][1])
    # a wrong CRC-32
    crc = bytearray(m)
    crc[-8] ^= 1
    with pytest.raises(fcship.FcsError, match=f"member {k} .*CRC-32 mismatch"):
        fcship.bgzf_inflate(_with_bad(cases, k, bytes(crc)), device=gpu)
    # an ISIZE smaller than the stream
    short = bytearray(m)
    short[-4:] = struct.pack("<I", len(cases[k][2]) - 1)
    with pytest.raises(fcship.FcsError, match=f"member {k} "):
        fcship.bgzf_inflate(_with_bad(cases, k, bytes(short)), device=gpu)
    # flipped bits in the DEFLATE stream: an error naming the member (corrupt,
    # overflow or CRC), never a fault — or, for the bits DEFLATE ignores (the
    # padding of a stored block's header, the bits after the final block),
    # the right bytes
    want = b"".join(c[2] for c in cases)
    errors = 0
    for trial in range(40):
        bad = bytearray(m)
        at = 18 + int(rng.integers(0, len(m) - 26))
        bad[at] ^= 1 << int(rng.integers(0, 8))
        try:
            out, _ = fcship.bgzf_inflate(_with_bad(cases, k, bytes(bad)), device=gpu)
        except fcship.FcsError as e:
            assert f"member {k} " in str(e), str(e)
            errors += 1
        else:
            assert out == want
    assert errors >= 30
    out, _ = fcship.bgzf_inflate(b"".join(c[1] for c in cases), device=gpu)
    assert out == b"".join(c[2] for c in cases)


def test_inflate_dev_statuses(gpu):
    import torch
    cases = bgzf_cases.suite(seed=15, count=30)
    bad_k = 5
    ms = [bytearray(m) for _, m, _ in cases]
    ms[bad_k][-8] ^= 0x80  # CRC
    blob = b"".join(bytes(m) for m in ms)
    coff, uoff, used = fcship.bgzf_index(blob)
    dev = torch.device("cuda", 0)
    comp = torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).to(dev)
    dco = torch.from_numpy(coff).to(dev)
    duo = torch.from_numpy(uoff).to(dev)
    out = torch.zeros(int(uoff[-1]) + 1, dtype=torch.uint8, device=dev)
    st = torch.full((len(coff) - 1,), -1, dtype=torch.int32, device=dev)
    fcship.check(fcship.lib.fcs_bgzf_inflate_dev(comp.data_ptr(), dco.data_ptr(), duo.data_ptr(), len(coff) - 1,
                                                 out.data_ptr(), st.data_ptr(), 0, None))
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert s[bad_k] == fcship.FCS_BGZF_CRC
    assert (np.delete(s, bad_k) == fcship.FCS_BGZF_OK).all()
    o = out.cpu().numpy().tobytes()
    for k, (_, _, p) in enumerate(cases):
        if k != bad_k:
            assert o[uoff[k]:uoff[k + 1]] == p


def test_try_uses_only_warm_idle_sessions(gpu):
    """fcs_bgzf_inflate_try inflates when a warm inflate session's arenas fit
    the call, and answers FCS_BGZF_BUSY (nothing done) when none does."""
    import ctypes as C
    cases = bgzf_cases.suite(seed=16, count=12)
    blob = np.frombuffer(b"".join(m for _, m, _ in cases), np.uint8).copy()
    want = b"".join(p for _, _, p in cases)
    fcship.check(fcship.lib.fcs_bgzf_warmup(0, 2, 64 << 20))
    out = np.zeros(len(want) + 1, np.uint8)
    used, got = C.c_int64(), C.c_int64()
    rc = fcship.lib.fcs_bgzf_inflate_try(blob.ctypes.data, len(blob), out.ctypes.data, len(want), C.byref(used),
                                         C.byref(got), 0)
    assert rc == fcship.FCS_OK and used.value == len(blob) and out[:got.value].tobytes() == want
    # a call larger than every warm arena: busy, nothing written
    big = np.frombuffer(b"".join(bgzf_cases.member(bytes(60000), 1) for _ in range(2000)), np.uint8).copy()
    cap = 2000 * 60000
    obig = np.zeros(cap, np.uint8)
    rc = fcship.lib.fcs_bgzf_inflate_try(big.ctypes.data, len(big), obig.ctypes.data, cap, C.byref(used),
                                         C.byref(got), 0)
    assert rc == fcship.FCS_BGZF_BUSY and used.value == 0


def test_concurrent_inflate_calls(gpu):
    """16 threads, 8 fcs_bgzf_inflate calls each, every thread its own blob of
    members and fresh host buffers per call (freed and mapped again between
    calls), every output byte-compared with zlib's (the kernel also checks
    each member's CRC-32 and ISIZE).  The round-5 corruption (member 0 of a
    call, about one htc run in four) came from the stream-ordered pool, which
    on this runtime hands scratch live on one stream to a call on another
    (tools/micro/pin_reuse.hip, profiles/r6/r6b_pin_reuse.log); the library no
    longer uses it."""
    import threading
    blobs = []
    for k in range(16):
        cases = bgzf_cases.suite(seed=300 + k, count=120)
        blobs.append((b"".join(m for _, m, _ in cases), b"".join(p for _, _, p in cases)))
    errors = []

    def worker(k):
        comp, want = blobs[k]
        try:
            for _ in range(8):
                c = np.frombuffer(comp, np.uint8).copy()  # a fresh host buffer per call
                out, used = fcship.bgzf_inflate(c, device=gpu)
                if used != len(comp) or out != want:
                    errors.append(f"thread {k}: output differs from zlib")
                del c, out
        except Exception as e:  # noqa: BLE001 (reported below, with the thread)
            errors.append(f"thread {k}: {e}")
    th = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:4]
