"""BGZF inflate checks that need no GPU.

- The device kernel's DEFLATE decoder and CRC recombination
  (falcon-genome_amd/csrc/bgzf_inflate.h), compiled for the host, inflate
  zlib's output at every level and strategy bit-exactly and survive flipped
  bits, truncation and short outputs under ASAN/UBSAN
  (tools/micro/inflate_test.cpp).
- fcs_bgzf_index (host code of the product library) walks members as
  htslib's bgzf_read does: offsets, ISIZE prefix sums, an incomplete trailing
  member left for the next call, a non-BGZF header refused.
"""
import os
import shutil
import subprocess
import zlib

import numpy as np
import pytest

import bgzf_cases
import fcship

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_device_decoder_host_build_matches_zlib(tmp_path):
    exe = tmp_path / "inflate_test"
    src = os.path.join(ROOT, "tools", "micro", "inflate_test.cpp")
    subprocess.run(["g++", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    "-I" + os.path.join(ROOT, "falcon-genome_amd", "csrc"), src, "-o", str(exe), "-lz"], check=True)
    r = subprocess.run([str(exe), "800"], capture_output=True, text=True, env={**os.environ, "ASAN_OPTIONS": "detect_leaks=0"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 bad of 800; crc: 0 bad" in r.stdout


def test_index_walks_members():
    cases = bgzf_cases.suite(seed=5, count=16)
    blob = b"".join(m for _, m, _ in cases)
    coff, uoff, used = fcship.bgzf_index(blob)
    assert used == len(blob)
    assert list(np.diff(coff)) == [len(m) for _, m, _ in cases]
    assert list(np.diff(uoff)) == [len(p) for _, _, p in cases]
    # an incomplete trailing member is left for the next call
    cut = blob[:-10]
    coff2, uoff2, used2 = fcship.bgzf_index(cut)
    assert len(coff2) == len(coff) - 1 and used2 == coff[-2]
    # a capped walk
    coff3, _, used3 = fcship.bgzf_index(blob, cap=3)
    assert len(coff3) == 4 and used3 == coff[3]
    # shorter than a header: nothing
    assert fcship.bgzf_index(blob[:17])[2] == 0


def test_index_refuses_non_bgzf():
    plain = zlib.compress(b"hello" * 100)  # zlib / gzip without the BC field
    with pytest.raises(fcship.FcsError, match=r"\[E::fcs_bgzf_index\]"):
        fcship.bgzf_index(b"\x1f\x8b\x08\x00" + b"\0" * 40)
    with pytest.raises(fcship.FcsError, match=r"\[E::fcs_bgzf_index\]"):
        fcship.bgzf_index(plain + b"\0" * 20)


def test_index_matches_the_host_writer(tmp_path):
    """A BAM written by the host's BgzfWriter (libdeflate level 5, `fcs-genome
    synth`): every member indexed, inflated sizes equal to zlib's."""
    import host_lib as H
    p = H.run_cli("synth", "-o", tmp_path, "-c", "chrA:60000", "-x", "6", "--seed", "3")
    assert p.returncode == 0, p.stderr
    blob = (tmp_path / "sample.bam").read_bytes()
    coff, uoff, used = fcship.bgzf_index(blob)
    assert used == len(blob) and len(coff) > 2
    for k in range(len(coff) - 1):
        m = blob[coff[k]:coff[k + 1]]
        xlen = m[10] | m[11] << 8
        assert len(zlib.decompress(m[12 + xlen:-8], -15)) == uoff[k + 1] - uoff[k]
