"""ctypes access to the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this,
and only as the checker / CPU baseline; the product (libfcship.so and
falcon-genome_amd/fcship.py) never loads it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = (os.path.join(ORACLE_DIR, "_san", os.environ["FCS_SAN"], "liboracle.so") if os.environ.get("FCS_SAN")
              else os.path.join(ORACLE_DIR, "liboracle.so"))


def _load():
    if not os.path.exists(ORACLE_LIB):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
    return C.CDLL(ORACLE_LIB)


lib = _load()
u8p = C.POINTER(C.c_uint8)
i8p = C.POINTER(C.c_int8)
vp = C.c_void_p

lib.oracle_phmm_init.restype = None
lib.oracle_phmm_ph2pr_f.restype = C.POINTER(C.c_float)
lib.oracle_phmm_ph2pr_d.restype = C.POINTER(C.c_double)
lib.oracle_phmm_mm_f.restype = C.c_float
lib.oracle_phmm_mm_f.argtypes = [C.c_int, C.c_int]
lib.oracle_phmm_mm_d.restype = C.c_double
lib.oracle_phmm_mm_d.argtypes = [C.c_int, C.c_int]
for nm, rt in (("oracle_phmm_prob_f", C.c_float), ("oracle_phmm_prob_d", C.c_double)):
    f = getattr(lib, nm)
    f.restype = rt
    f.argtypes = [vp, vp, vp, vp, vp, C.c_int, vp, C.c_int]
lib.oracle_phmm_log10.restype = C.c_double
lib.oracle_phmm_log10.argtypes = [vp, vp, vp, vp, vp, C.c_int, vp, C.c_int, C.POINTER(C.c_int)]
lib.oracle_phmm_java_log10.restype = C.c_double
lib.oracle_phmm_java_log10.argtypes = [vp, vp, vp, vp, vp, C.c_int, vp, C.c_int]
lib.oracle_phmm_batch.restype = None
lib.oracle_phmm_batch.argtypes = [vp] * 5 + [vp, vp, vp, vp, vp, vp, vp, C.c_int64, vp, vp, vp, C.c_int]
lib.oracle_omp_max_threads.restype = C.c_int
lib.oracle_phmm_simd_available.restype = C.c_int
lib.oracle_phmm_simd_batch.restype = C.c_int
lib.oracle_phmm_simd_batch.argtypes = lib.oracle_phmm_batch.argtypes
lib.oracle_ksw_extend2.restype = C.c_int
lib.oracle_ksw_extend2.argtypes = [C.c_int, vp, C.c_int, vp, C.c_int, vp] + [C.c_int] * 8 + [vp] * 6
lib.oracle_ksw_global2.restype = C.c_int
lib.oracle_ksw_global2.argtypes = [C.c_int, vp, C.c_int, vp, C.c_int, vp] + [C.c_int] * 5 + [vp, vp, C.c_int]
lib.oracle_ksw_align2.restype = None
lib.oracle_ksw_align2.argtypes = [C.c_int, vp, C.c_int, vp, C.c_int, vp] + [C.c_int] * 5 + [vp]
lib.oracle_ksw_align2_sse.restype = None
lib.oracle_ksw_align2_sse.argtypes = lib.oracle_ksw_align2.argtypes
lib.oracle_ksw_align2_sse_batch.restype = None
lib.oracle_ksw_align2_sse_batch.argtypes = [vp] * 7 + [C.c_int64, vp] + [C.c_int] * 4 + [vp, C.c_int]
lib.oracle_ksw_extend2_batch.restype = None
lib.oracle_ksw_extend2_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, C.c_int64, vp] + [C.c_int] * 6 + \
    [vp, vp, C.c_int]


def _a(x, dt=np.uint8):
    return np.ascontiguousarray(np.frombuffer(bytes(x), dtype=np.uint8) if isinstance(x, (bytes, bytearray, str))
                                else np.asarray(x), dtype=dt)


def _p(a):
    return a.ctypes.data if a.size else None


def ph2pr_f():
    p = lib.oracle_phmm_ph2pr_f()
    return np.array([p[i] for i in range(128)], np.float32)


def ph2pr_d():
    p = lib.oracle_phmm_ph2pr_d()
    return np.array([p[i] for i in range(128)], np.float64)


def _rd(read):
    return [_a(x.encode() if isinstance(x, str) else x) for x in read]


def phmm_prob_f(read, hap):
    r = _rd(read)
    h = _a(hap.encode() if isinstance(hap, str) else hap)
    return float(lib.oracle_phmm_prob_f(*[_p(x) for x in r], len(r[0]), _p(h), len(h)))


def phmm_prob_d(read, hap):
    r = _rd(read)
    h = _a(hap.encode() if isinstance(hap, str) else hap)
    return float(lib.oracle_phmm_prob_d(*[_p(x) for x in r], len(r[0]), _p(h), len(h)))


def phmm_log10(read, hap):
    r = _rd(read)
    h = _a(hap.encode() if isinstance(hap, str) else hap)
    ud = C.c_int()
    v = lib.oracle_phmm_log10(*[_p(x) for x in r], len(r[0]), _p(h), len(h), C.byref(ud))
    return float(v), bool(ud.value)


def phmm_java_log10(read, hap):
    r = _rd(read)
    h = _a(hap.encode() if isinstance(hap, str) else hap)
    return float(lib.oracle_phmm_java_log10(*[_p(x) for x in r], len(r[0]), _p(h), len(h)))


def phmm_simd_batch(p, threads=1, raw=False):
    """GKL-style AVX-512 PairHMM (oracle/pairhmm_simd.c), same outputs as
    phmm_batch; None when the CPU has no AVX-512."""
    n = int(p.pair_read.size)
    out = np.zeros(n, np.float64)
    ud = np.zeros(n, np.int32)
    rawf = np.zeros(n, np.float32) if raw else None
    rc = lib.oracle_phmm_simd_batch(_p(p.read_bases), _p(p.read_bq), _p(p.read_iq), _p(p.read_dq), _p(p.read_gcp),
                                    _p(p.read_off), _p(p.read_len), _p(p.hap_bases), _p(p.hap_off), _p(p.hap_len),
                                    _p(p.pair_read), _p(p.pair_hap), n, _p(rawf) if raw else None, _p(out), _p(ud),
                                    threads)
    if rc < 0:
        return None
    return (out, ud.astype(bool), rawf) if raw else (out, ud.astype(bool))


def phmm_batch(p, threads=1, raw=False):
    """p: fcship.PhmmPairs-like object.  Returns (log10, used_double[, raw_f])."""
    n = int(p.pair_read.size)
    out = np.zeros(n, np.float64)
    ud = np.zeros(n, np.int32)
    rawf = np.zeros(n, np.float32) if raw else None
    lib.oracle_phmm_batch(_p(p.read_bases), _p(p.read_bq), _p(p.read_iq), _p(p.read_dq), _p(p.read_gcp),
                          _p(p.read_off), _p(p.read_len), _p(p.hap_bases), _p(p.hap_off), _p(p.hap_len),
                          _p(p.pair_read), _p(p.pair_hap), n, _p(rawf) if raw else None, _p(out), _p(ud), threads)
    return (out, ud.astype(bool), rawf) if raw else (out, ud.astype(bool))


def ksw_extend2(q, t, h0, w, mat, o_del=6, e_del=1, o_ins=6, e_ins=1, end_bonus=5, zdrop=100):
    q = _a(q)
    t = _a(t)
    m = _a(mat, np.int8)
    outs = [C.c_int() for _ in range(5)]
    cells = C.c_int64()
    sc = lib.oracle_ksw_extend2(len(q), _p(q), len(t), _p(t), 5, _p(m), o_del, e_del, o_ins, e_ins, w, end_bonus,
                                zdrop, h0, *[C.addressof(o) for o in outs], C.addressof(cells))
    return (sc,) + tuple(o.value for o in outs), cells.value


def ksw_global2(q, t, w, mat, o_del=6, e_del=1, o_ins=6, e_ins=1):
    q = _a(q)
    t = _a(t)
    m = _a(mat, np.int8)
    cap = len(q) + len(t) + 2
    cig = np.zeros(cap, np.uint32)
    n = C.c_int()
    sc = lib.oracle_ksw_global2(len(q), _p(q), len(t), _p(t), 5, _p(m), o_del, e_del, o_ins, e_ins, w,
                                C.addressof(n), _p(cig), cap)
    return sc, cig[:n.value].copy()


KSW_XBYTE, KSW_XSTOP, KSW_XSUBO, KSW_XSTART = 0x10000, 0x20000, 0x40000, 0x80000


def ksw_align2(q, t, mat, xtra, o_del=6, e_del=1, o_ins=6, e_ins=1):
    """bwa ksw_align2 restated (oracle/ksw_align_oracle.c): (score, te, qe,
    score2, te2, tb, qb) as bwa's kswr_t."""
    q = _a(q)
    t = _a(t)
    m = _a(mat, np.int8)
    out = np.zeros(7, np.int32)
    lib.oracle_ksw_align2(len(q), _p(q), len(t), _p(t), 5, _p(m), o_del, e_del, o_ins, e_ins, xtra, _p(out))
    return tuple(int(x) for x in out)


def ksw_align2_sse(q, t, mat, xtra, o_del=6, e_del=1, o_ins=6, e_ins=1):
    """The SSE2 striped form of ksw_align2 (oracle/ksw_align_sse.c, the CPU
    baseline): the same seven outputs as ksw_align2."""
    q = _a(q)
    t = _a(t)
    m = _a(mat, np.int8)
    out = np.zeros(7, np.int32)
    lib.oracle_ksw_align2_sse(len(q), _p(q), len(t), _p(t), 5, _p(m), o_del, e_del, o_ins, e_ins, xtra, _p(out))
    return tuple(int(x) for x in out)


def ksw_align2_sse_batch(t, mat, xtra, o_del=6, e_del=1, o_ins=6, e_ins=1, threads=1):
    """ksw_align2 (SSE2 striped restatement) over a BswTasks batch on OpenMP
    threads; xtra: one int or one per task.  Returns an (n, 7) int32 array."""
    n = t.n
    out = np.zeros((n, 7), np.int32)
    m = _a(mat, np.int8)
    xt = np.ascontiguousarray(np.broadcast_to(np.asarray(xtra, np.int32), (n,)))
    lib.oracle_ksw_align2_sse_batch(_p(t.qbuf), _p(t.qoff), _p(t.qlen), _p(t.tbuf), _p(t.toff), _p(t.tlen), _p(xt), n,
                                    _p(m), o_del, e_del, o_ins, e_ins, _p(out), threads)
    return out


def ksw_extend2_batch(t, mat, o_del=6, e_del=1, o_ins=6, e_ins=1, end_bonus=5, zdrop=100, threads=1):
    n = t.n
    res = np.zeros((n, 6), np.int32)
    cells = np.zeros(n, np.int64)
    m = _a(mat, np.int8)
    lib.oracle_ksw_extend2_batch(_p(t.qbuf), _p(t.qoff), _p(t.qlen), _p(t.tbuf), _p(t.toff), _p(t.tlen), _p(t.h0),
                                 _p(t.w), n, _p(m), o_del, e_del, o_ins, e_ins, end_bonus, zdrop, _p(res),
                                 _p(cells), threads)
    return res, cells
