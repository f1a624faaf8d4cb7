"""C-ABI checks that need no GPU: the library loads, exports exactly the
header's entry points, validates arguments the way the reference's workers
fail (typed error + "[E::" message), never falls back to the CPU, and the
seeded workload generators are deterministic and match SURVEY.md §8(d)."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

import fcship
from conftest import has_gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exports_every_header_symbol():
    syms = fcship.header_symbols()
    assert len(syms) == fcship.lib.fcs_abi_symbol_count()
    missing = [s for s in syms if not hasattr(fcship.lib, s)]
    assert not missing, missing
    nm = subprocess.run(["nm", "-D", "--defined-only", fcship.LIB_PATH], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in nm.splitlines() if " T " in ln and ln.split()[-1].startswith("fcs_")}
    assert exported == set(syms), exported ^ set(syms)


def test_product_does_not_link_the_oracle():
    out = subprocess.run(["readelf", "-d", fcship.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    nm = subprocess.run(["nm", "-D", fcship.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle_" not in nm


def test_compiled_for_gfx950_only():
    import re
    blob = open(fcship.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-[a-z-]*(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


@pytest.mark.skipif(has_gpu(), reason="checks the no-device behaviour")
def test_no_cpu_fallback_without_device():
    assert fcship.device_count() == 0
    p = fcship.synth_phmm(1, 4)
    with pytest.raises(fcship.FcsError) as e:
        fcship.phmm_compute_pairs(p)
    assert e.value.code == fcship.FCS_ERR_DEVICE and "[E::" in str(e.value)
    t = fcship.synth_bsw(1, 4, ref_len=100_000)
    with pytest.raises(fcship.FcsError) as e:
        fcship.bsw_extend_batch(t)
    assert e.value.code == fcship.FCS_ERR_DEVICE
    with pytest.raises(fcship.FcsError):
        fcship.ksw_extend2([0, 1, 2], [0, 1, 2], 5, 10)


def test_argument_validation_precedes_device():
    p = fcship.synth_phmm(1, 4)
    p.pair_read[2] = 99
    with pytest.raises(fcship.FcsError) as e:
        fcship.phmm_compute_pairs(p)
    assert e.value.code == fcship.FCS_ERR_INVALID and "pair index" in str(e.value)
    t = fcship.make_tasks([([0, 1, 2], [0, 1, 2], 0, 10)])
    with pytest.raises(fcship.FcsError) as e:
        fcship.bsw_extend_batch(t)
    assert e.value.code == fcship.FCS_ERR_INVALID and "h0" in str(e.value)
    t = fcship.make_tasks([([0, 1, 7], [0, 1, 2], 5, 10)])
    with pytest.raises(fcship.FcsError) as e:
        fcship.bsw_extend_batch(t)
    assert "base code" in str(e.value)
    q = np.zeros(3, np.uint8)
    m = fcship.default_mat()
    r = fcship.lib.fcs_ksw_extend2(3, q.ctypes.data_as(fcship.u8p), 3, q.ctypes.data_as(fcship.u8p), 4,
                                   m.ctypes.data_as(fcship.i8p), 6, 1, 6, 1, 10, 5, 100, 5, None, None, None, None,
                                   None)
    assert r == fcship.FCS_KSW_FAILED and b"m == 5" in fcship.lib.fcs_last_error()
    bad = fcship.bsw_params(e_del=0)
    with pytest.raises(fcship.FcsError):
        fcship.bsw_extend_batch(fcship.make_tasks([([0], [0], 5, 10)]), bad)


def test_empty_batches_are_ok():
    e = fcship.make_pairs([], [])
    assert fcship.phmm_compute_pairs(e).size == 0
    res, cells = fcship.bsw_extend_batch(fcship.make_tasks([]))
    assert res.shape == (0, 6)


def test_default_params_match_bwa():
    m = fcship.default_mat().reshape(5, 5)
    assert (np.diag(m)[:4] == 1).all() and m[0, 1] == -4 and (m[4] == -1).all() and (m[:, 4] == -1).all()
    p = fcship.bsw_params()
    assert (p.o_del, p.e_del, p.o_ins, p.e_ins, p.end_bonus, p.zdrop) == (6, 1, 6, 1, 5, 100)


def test_synth_phmm_deterministic_and_on_spec():
    a = fcship.synth_phmm(20261015, 3000)
    b = fcship.synth_phmm(20261015, 3000)
    for k in ("read_bases", "read_bq", "hap_bases", "read_len", "hap_len"):
        assert np.array_equal(getattr(a, k), getattr(b, k))
    assert a.hap_len.min() >= 150 and a.hap_len.max() <= 300
    assert abs(a.hap_len.mean() - 225) < 5
    assert (a.read_len <= 101).all() and (a.read_len >= 90).mean() > 0.99
    bq = np.concatenate([a.read_bq[o:o + n] for o, n in zip(a.read_off[:200], a.read_len[:200])])
    assert bq.min() >= 10 and bq.max() <= 40
    assert (a.read_iq == 45).all() and (a.read_dq == 45).all() and (a.read_gcp == 10).all()
    # the read is a hap substring: ~1% substitutions -> long exact matches
    k = 5
    r = a.read_bases[a.read_off[k]:a.read_off[k] + a.read_len[k]].tobytes()
    h = a.hap_bases[a.hap_off[k]:a.hap_off[k] + a.hap_len[k]].tobytes()
    assert r[:20] in h or r[40:60] in h or r[-20:] in h


def test_synth_bsw_on_spec():
    t = fcship.synth_bsw(20261015, 2000, ref_len=1_000_000)
    t2 = fcship.synth_bsw(20261015, 2000, ref_len=1_000_000)
    assert np.array_equal(t.qbuf, t2.qbuf) and np.array_equal(t.tlen, t2.tlen)
    assert 1.5 * 2000 < t.n <= 2 * 2000
    assert (t.qlen > 0).all() and (t.qlen <= 151 - 19).all()
    assert (t.tlen <= t.qlen + 100).all() and (t.h0 >= 19).all()
    assert t.qbuf.max() <= 3 and t.tbuf.max() <= 3
    f = fcship.synth_bsw(1, 100, ref_len=1_000_000, mode=1, fixed_q=151, fixed_t=251)
    assert (f.qlen == 151).all() and (f.tlen == 251).all()


def test_dense_compute_validates_reads():
    with pytest.raises(fcship.FcsError) as e:
        fcship.lib.fcs_phmm_compute(None, 1, None, 1, None, None) and None
        fcship.check(fcship.lib.fcs_phmm_compute(None, 1, None, 1, None, None))
    assert e.value.code == fcship.FCS_ERR_INVALID


@pytest.mark.gpu
def test_device_release_then_reuse(gpu, tmp_path):
    """fcs_device_release resets the device; the next calls set everything up
    again and give the same results.  In a child process: the reset frees every
    allocation of the process (torch's included)."""
    script = tmp_path / "rel.py"
    script.write_text(f"""
import sys
sys.path[:0] = [{os.path.join(ROOT, 'falcon-genome_amd')!r}, {os.path.join(ROOT, 'tests')!r}]
import numpy as np
import fcship
import bgzf_cases
p = fcship.synth_phmm(7, 2000)
a = fcship.phmm_compute_pairs(p)
blob = b"".join(m for _, m, _ in bgzf_cases.suite(seed=3, count=20))
x, _ = fcship.bgzf_inflate(blob)
fcship.check(fcship.lib.fcs_device_release(0))
fcship.check(fcship.lib.fcs_device_release(0))  # twice: nothing left to drop
b = fcship.phmm_compute_pairs(p)
y, _ = fcship.bgzf_inflate(blob)
assert np.array_equal(a, b) and x == y
print("release ok")
""")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "release ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
