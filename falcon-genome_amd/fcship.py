"""ctypes binding of libfcship.so (include/fcship.h) for tests, bench and tools.

This module is plumbing: every computation goes through the C-ABI into the
gfx950 HIP kernels.  There is no CPU fallback — if the shared library is
missing, importing this module raises, and if no GPU is present the compute
entry points return FCS_ERR_DEVICE, which is raised as FcsError.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

try:  # one HIP runtime per process: torch bundles its own libamdhip64, so when
    # torch is present it must be loaded first and libfcship binds to that copy.
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is optional plumbing
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FCSHIP_LIB") or os.path.join(HERE, "libfcship.so")  # override: A/B builds
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "fcship.h")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libfcship.so not built at {LIB_PATH}; run `make -C falcon-genome_amd` "
        "or __graft_entry__.build() (the HIP path has no CPU fallback)")

lib = C.CDLL(LIB_PATH)

FCS_OK = 0
FCS_ERR_INVALID = -1
FCS_ERR_DEVICE = -2
FCS_ERR_NOMEM = -3
FCS_ERR_UNSUPPORTED = -4
FCS_KSW_FAILED = -2147483648


class FcsError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"fcship error {code}: {msg}")
        self.code = code


u8p = C.POINTER(C.c_uint8)
i8p = C.POINTER(C.c_int8)
i32p = C.POINTER(C.c_int32)
i64p = C.POINTER(C.c_int64)
u32p = C.POINTER(C.c_uint32)
f64p = C.POINTER(C.c_double)


class PhmmRead(C.Structure):
    _fields_ = [("bases", u8p), ("base_q", u8p), ("ins_q", u8p), ("del_q", u8p), ("gcp", u8p),
                ("len", C.c_int32)]


class PhmmHap(C.Structure):
    _fields_ = [("bases", u8p), ("len", C.c_int32)]


class PhmmRegion(C.Structure):
    _fields_ = [("reads", C.POINTER(PhmmRead)), ("n_reads", C.c_int32), ("haps", C.POINTER(PhmmHap)),
                ("n_haps", C.c_int32), ("out_log10", f64p)]


class PhmmOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("use_fp64_rescue", C.c_int32), ("rescue_threshold", C.c_float),
                ("exact_order", C.c_int32)]


class PhmmBatch(C.Structure):
    _fields_ = [("read_bases", C.c_void_p), ("read_bq", C.c_void_p), ("read_iq", C.c_void_p),
                ("read_dq", C.c_void_p), ("read_gcp", C.c_void_p), ("read_off", C.c_void_p),
                ("read_len", C.c_void_p), ("n_reads", C.c_int64), ("hap_bases", C.c_void_p),
                ("hap_off", C.c_void_p), ("hap_len", C.c_void_p), ("n_haps", C.c_int64),
                ("pair_read", C.c_void_p), ("pair_hap", C.c_void_p), ("n_pairs", C.c_int64),
                ("read_bytes", C.c_int64), ("hap_bytes", C.c_int64), ("max_read_len", C.c_int32),
                ("max_hap_len", C.c_int32)]


class BswTask(C.Structure):
    _fields_ = [("qlen", C.c_int32), ("tlen", C.c_int32), ("h0", C.c_int32), ("w", C.c_int32),
                ("query", u8p), ("target", u8p)]


class BswParams(C.Structure):
    _fields_ = [("mat", C.c_int8 * 25), ("o_del", C.c_int32), ("e_del", C.c_int32), ("o_ins", C.c_int32),
                ("e_ins", C.c_int32), ("end_bonus", C.c_int32), ("zdrop", C.c_int32)]


class BswResult(C.Structure):
    _fields_ = [("score", C.c_int32), ("qle", C.c_int32), ("tle", C.c_int32), ("gtle", C.c_int32),
                ("gscore", C.c_int32), ("max_off", C.c_int32)]


class Kswr(C.Structure):  # bwa's kswr_t
    _fields_ = [("score", C.c_int32), ("te", C.c_int32), ("qe", C.c_int32), ("score2", C.c_int32),
                ("te2", C.c_int32), ("tb", C.c_int32), ("qb", C.c_int32)]


KSW_XBYTE, KSW_XSTOP, KSW_XSUBO, KSW_XSTART = 0x10000, 0x20000, 0x40000, 0x80000


class BswBatch(C.Structure):
    _fields_ = [("qbuf", C.c_void_p), ("qoff", C.c_void_p), ("qlen", C.c_void_p), ("tbuf", C.c_void_p),
                ("toff", C.c_void_p), ("tlen", C.c_void_p), ("h0", C.c_void_p), ("w", C.c_void_p),
                ("n", C.c_int64), ("qbytes", C.c_int64), ("tbytes", C.c_int64), ("max_qlen", C.c_int32),
                ("max_tlen", C.c_int32)]


def _sig(name, res, args):
    f = getattr(lib, name, None)
    if f is None:
        if os.environ.get("FCSHIP_LIB"):  # an older A/B variant (tools/ab.sh) may predate an entry point
            return None
        raise AttributeError(f"libfcship.so lacks {name}")
    f.restype = res
    f.argtypes = args
    return f


_sig("fcs_device_count", C.c_int, [])
_sig("fcs_last_error", C.c_char_p, [])
_sig("fcs_version", C.c_char_p, [])
_sig("fcs_abi_symbol_count", C.c_int, [])
_sig("fcs_phmm_opts_default", None, [C.POINTER(PhmmOpts)])
_sig("fcs_phmm_compute", C.c_int, [C.POINTER(PhmmRead), C.c_int32, C.POINTER(PhmmHap), C.c_int32, f64p,
                                   C.POINTER(PhmmOpts)])
_sig("fcs_phmm_compute_regions", C.c_int, [C.POINTER(PhmmRegion), C.c_int32, C.POINTER(PhmmOpts)])
_sig("fcs_phmm_compute_pairs", C.c_int, [C.POINTER(PhmmBatch), f64p, C.POINTER(PhmmOpts)])
_sig("fcs_phmm_plan_create", C.c_int, [C.c_int32, C.c_int64, C.POINTER(C.c_void_p)])
_sig("fcs_phmm_plan_destroy", C.c_int, [C.c_void_p])
_sig("fcs_phmm_dev_schedule", C.c_int, [C.c_void_p, C.POINTER(PhmmBatch), C.c_void_p])
_sig("fcs_phmm_dev_forward", C.c_int, [C.c_void_p, C.POINTER(PhmmBatch), C.c_void_p, C.POINTER(PhmmOpts),
                                       C.c_void_p])
_sig("fcs_phmm_dev_rescue", C.c_int, [C.c_void_p, C.POINTER(PhmmBatch), C.c_void_p, C.POINTER(PhmmOpts),
                                      C.c_void_p])
_sig("fcs_phmm_dev_run", C.c_int, [C.c_void_p, C.POINTER(PhmmBatch), C.c_void_p, C.POINTER(PhmmOpts),
                                   C.c_void_p])
_sig("fcs_phmm_plan_rescue_count", C.c_int, [C.c_void_p, C.c_void_p, i64p])
_sig("fcs_phmm_last_rescued", C.c_int, [i64p])
_sig("fcs_phmm_last_device_ms", C.c_int, [C.POINTER(C.c_double), C.POINTER(C.c_double)])
_sig("fcs_device_warmup", C.c_int, [C.c_int32, C.c_int32])
_sig("fcs_stream_release", C.c_int, [C.c_int32, C.c_void_p])
_sig("fcs_device_release", C.c_int, [C.c_int32])
_sig("fcs_phmm_partition", C.c_int, [C.POINTER(PhmmBatch), C.c_int32, C.c_void_p])
_sig("fcs_phmm_compute_pairs_multi", C.c_int, [C.POINTER(PhmmBatch), C.c_void_p, C.POINTER(PhmmOpts), C.c_void_p,
                                               C.c_int32])
_sig("fcs_bsw_params_default", None, [C.POINTER(BswParams)])
_sig("fcs_bsw_extend", C.c_int, [C.POINTER(BswTask), C.c_int32, C.POINTER(BswParams), C.POINTER(BswResult),
                                 C.c_int32])
_sig("fcs_bsw_extend_multi", C.c_int, [C.POINTER(BswTask), C.c_int32, C.POINTER(BswParams), C.POINTER(BswResult),
                                       C.c_void_p, C.c_int32])
_sig("fcs_bsw_extend_dev", C.c_int, [C.POINTER(BswBatch), C.POINTER(BswParams), C.c_void_p, C.c_void_p,
                                     C.c_int32, C.c_void_p])
_sig("fcs_bsw_extend_batch", C.c_int, [C.POINTER(BswBatch), C.POINTER(BswParams), i32p, i64p, C.c_int32])
_sig("fcs_bsw_plan_create", C.c_int, [C.c_int32, C.c_int64, C.POINTER(C.c_void_p)])
_sig("fcs_bsw_plan_destroy", C.c_int, [C.c_void_p])
_sig("fcs_bsw_extend_plan", C.c_int, [C.c_void_p, C.POINTER(BswBatch), C.POINTER(BswParams), C.c_void_p, C.c_void_p,
                                      C.c_void_p])
_sig("fcs_bsw_global", C.c_int, [C.POINTER(BswTask), C.c_int32, C.POINTER(BswParams), i32p, u32p, i64p, i32p,
                                 i32p, C.c_int32])
_sig("fcs_bsw_align", C.c_int, [C.POINTER(BswTask), C.c_int32, C.POINTER(BswParams), i32p, C.c_void_p, C.c_int32])
_sig("fcs_bsw_align_dev", C.c_int, [C.POINTER(BswBatch), C.POINTER(BswParams), C.c_void_p, C.c_void_p, C.c_int32,
                                    C.c_void_p])
_sig("fcs_ksw_align2", Kswr, [C.c_int, u8p, C.c_int, u8p, C.c_int, i8p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                              C.c_void_p])
_sig("fcs_bsw_global_dev", C.c_int, [C.POINTER(BswBatch), C.POINTER(BswParams), C.c_void_p, C.c_void_p, C.c_int64,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                     C.c_void_p])
_sig("fcs_ksw_extend2", C.c_int, [C.c_int, u8p, C.c_int, u8p, C.c_int, i8p, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                  C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)])
_sig("fcs_ksw_global2", C.c_int, [C.c_int, u8p, C.c_int, u8p, C.c_int, i8p, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.c_int, C.POINTER(C.c_int), C.POINTER(u32p)])
_sig("fcs_set_default_device", C.c_int, [C.c_int32])
_sig("fcs_bgzf_index", C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int32, i32p, i64p])
_sig("fcs_bgzf_inflate", C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, i64p, i64p, C.c_int32])
_sig("fcs_bgzf_inflate_try", C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, i64p, i64p, C.c_int32])
_sig("fcs_bgzf_warmup", C.c_int, [C.c_int32, C.c_int32, C.c_int64])
_sig("fcs_bgzf_inflate_dev", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                                       C.c_int32, C.c_void_p])
_sig("fcs_synth_phmm_sizes", C.c_int, [C.c_uint64, C.c_int64, C.c_int32, C.c_int32, C.c_int32, i64p, i64p])
_sig("fcs_synth_phmm", C.c_int, [C.c_uint64, C.c_int64, C.c_int32, C.c_int32, C.c_int32] + [C.c_void_p] * 10)
_sig("fcs_synth_bsw_sizes", C.c_int, [C.c_uint64, C.c_int64, C.c_int32, C.c_int64, C.c_int32, C.c_int32,
                                      C.c_int32, C.c_int32, i64p, i64p, i64p])
_sig("fcs_synth_bsw", C.c_int, [C.c_uint64, C.c_int64, C.c_int32, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                C.c_int32] + [C.c_void_p] * 9)

libc = C.CDLL(None)
libc.free.argtypes = [C.c_void_p]


def check(rc: int) -> None:
    if rc != FCS_OK:
        raise FcsError(rc, lib.fcs_last_error().decode(errors="replace"))


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def device_count() -> int:
    return int(lib.fcs_device_count())


def header_symbols() -> list[str]:
    """Function names declared in include/fcship.h."""
    import re
    txt = open(HEADER_PATH).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fcs_[a-z0-9_]+)\s*\(", txt)))


# ---------------------------------------------------------------- PairHMM
@dataclass
class PhmmPairs:
    """SoA pair batch in host numpy arrays (the layout fcs_phmm_batch describes)."""
    read_bases: np.ndarray
    read_bq: np.ndarray
    read_iq: np.ndarray
    read_dq: np.ndarray
    read_gcp: np.ndarray
    read_off: np.ndarray
    read_len: np.ndarray
    hap_bases: np.ndarray
    hap_off: np.ndarray
    hap_len: np.ndarray
    pair_read: np.ndarray
    pair_hap: np.ndarray

    @property
    def n_pairs(self) -> int:
        return int(self.pair_read.size)

    def cells(self) -> int:
        return int((self.read_len[self.pair_read].astype(np.int64) *
                    self.hap_len[self.pair_hap].astype(np.int64)).sum())

    def to_struct(self, ptr=_ptr) -> PhmmBatch:
        b = PhmmBatch()
        b.read_bases, b.read_bq, b.read_iq = ptr(self.read_bases), ptr(self.read_bq), ptr(self.read_iq)
        b.read_dq, b.read_gcp = ptr(self.read_dq), ptr(self.read_gcp)
        b.read_off, b.read_len, b.n_reads = ptr(self.read_off), ptr(self.read_len), int(self.read_len.size)
        b.hap_bases, b.hap_off, b.hap_len = ptr(self.hap_bases), ptr(self.hap_off), ptr(self.hap_len)
        b.n_haps = int(self.hap_len.size)
        b.pair_read, b.pair_hap, b.n_pairs = ptr(self.pair_read), ptr(self.pair_hap), int(self.pair_read.size)
        b.read_bytes, b.hap_bytes = int(self.read_bases.size), int(self.hap_bases.size)
        b.max_read_len = int(self.read_len.max()) if self.read_len.size else 0
        b.max_hap_len = int(self.hap_len.max()) if self.hap_len.size else 0
        return b


def make_pairs(reads, haps, pairs=None) -> PhmmPairs:
    """reads: list of (bases, bq, iq, dq, gcp) byte strings/arrays; haps: list of bytes.
    pairs: list of (read_idx, hap_idx); default = all reads x haps, read-major."""
    def cat(parts):
        arr = [np.frombuffer(bytes(p), dtype=np.uint8) if not isinstance(p, np.ndarray) else p.astype(np.uint8)
               for p in parts]
        return np.concatenate(arr) if arr else np.zeros(0, np.uint8)
    rl = np.array([len(r[0]) for r in reads], dtype=np.int32)
    ro = np.concatenate([[0], np.cumsum(rl[:-1], dtype=np.int64)]).astype(np.int64) if len(reads) else \
        np.zeros(0, np.int64)
    hl = np.array([len(h) for h in haps], dtype=np.int32)
    ho = np.concatenate([[0], np.cumsum(hl[:-1], dtype=np.int64)]).astype(np.int64) if len(haps) else \
        np.zeros(0, np.int64)
    if pairs is None:
        pairs = [(r, h) for r in range(len(reads)) for h in range(len(haps))]
    pr = np.array([p[0] for p in pairs], dtype=np.int32)
    ph = np.array([p[1] for p in pairs], dtype=np.int32)
    return PhmmPairs(cat([r[0] for r in reads]), cat([r[1] for r in reads]), cat([r[2] for r in reads]),
                     cat([r[3] for r in reads]), cat([r[4] for r in reads]), ro, rl, cat(haps), ho, hl, pr, ph)


def phmm_opts(device=0, rescue=True, threshold=1e-28, exact=False) -> PhmmOpts:
    o = PhmmOpts()
    lib.fcs_phmm_opts_default(C.byref(o))
    o.device, o.use_fp64_rescue, o.rescue_threshold, o.exact_order = device, int(rescue), threshold, int(exact)
    return o


def phmm_compute_pairs(p: PhmmPairs, **kw) -> np.ndarray:
    out = np.zeros(p.n_pairs, dtype=np.float64)
    b = p.to_struct()
    o = phmm_opts(**kw)
    check(lib.fcs_phmm_compute_pairs(C.byref(b), out.ctypes.data_as(f64p), C.byref(o)))
    return out


def phmm_partition(p: PhmmPairs, n: int) -> np.ndarray:
    """Cut points of the multi-GPU static partition (cuts[0..n])."""
    cuts = np.zeros(n + 1, dtype=np.int64)
    b = p.to_struct()
    check(lib.fcs_phmm_partition(C.byref(b), n, cuts.ctypes.data))
    return cuts


def phmm_compute_pairs_multi(p: PhmmPairs, devices, **kw) -> np.ndarray:
    out = np.zeros(p.n_pairs, dtype=np.float64)
    b = p.to_struct()
    o = phmm_opts(**kw)
    d = np.asarray(devices, dtype=np.int32)
    check(lib.fcs_phmm_compute_pairs_multi(C.byref(b), out.ctypes.data, C.byref(o), d.ctypes.data, len(d)))
    return out


def phmm_compute(reads, haps, **kw) -> np.ndarray:
    """GKL computeLikelihoodsNative-style dense call: returns [n_reads, n_haps] log10."""
    keep = []

    def u8(x):
        a = np.ascontiguousarray(np.frombuffer(bytes(x), dtype=np.uint8) if not isinstance(x, np.ndarray)
                                 else x.astype(np.uint8))
        keep.append(a)
        return a.ctypes.data_as(u8p)
    R = (PhmmRead * max(len(reads), 1))()
    for i, r in enumerate(reads):
        R[i] = PhmmRead(u8(r[0]), u8(r[1]), u8(r[2]), u8(r[3]), u8(r[4]), len(r[0]))
    H = (PhmmHap * max(len(haps), 1))()
    for i, h in enumerate(haps):
        H[i] = PhmmHap(u8(h), len(h))
    out = np.zeros((len(reads), len(haps)), dtype=np.float64)
    o = phmm_opts(**kw)
    check(lib.fcs_phmm_compute(R, len(reads), H, len(haps), out.ctypes.data_as(f64p), C.byref(o)))
    return out


def phmm_compute_regions(regions, **kw) -> list:
    """Active-region batching: regions = [(reads, haps), ...] with reads as
    (bases, base_q, ins_q, del_q, gcp) tuples; one device pass for all, returns
    one [n_reads, n_haps] log10 matrix per region."""
    keep, outs = [], []

    def u8(x):
        a = np.ascontiguousarray(np.frombuffer(bytes(x), dtype=np.uint8) if not isinstance(x, np.ndarray)
                                 else x.astype(np.uint8))
        keep.append(a)
        return a.ctypes.data_as(u8p)
    G = (PhmmRegion * max(len(regions), 1))()
    for g, (reads, haps) in enumerate(regions):
        R = (PhmmRead * max(len(reads), 1))()
        for i, r in enumerate(reads):
            R[i] = PhmmRead(u8(r[0]), u8(r[1]), u8(r[2]), u8(r[3]), u8(r[4]), len(r[0]))
        H = (PhmmHap * max(len(haps), 1))()
        for i, h in enumerate(haps):
            H[i] = PhmmHap(u8(h), len(h))
        out = np.zeros((len(reads), len(haps)), dtype=np.float64)
        keep += [R, H]
        outs.append(out)
        G[g] = PhmmRegion(C.cast(R, C.POINTER(PhmmRead)), len(reads), C.cast(H, C.POINTER(PhmmHap)), len(haps),
                          out.ctypes.data_as(f64p))
    o = phmm_opts(**kw)
    check(lib.fcs_phmm_compute_regions(G, len(regions), C.byref(o)))
    return outs


def synth_phmm(seed: int, n_pairs: int, R: int = 101, hmin: int = 150, hmax: int = 300) -> PhmmPairs:
    rb_n, hb_n = C.c_int64(), C.c_int64()
    check(lib.fcs_synth_phmm_sizes(seed, n_pairs, R, hmin, hmax, C.byref(rb_n), C.byref(hb_n)))
    rb = [np.zeros(rb_n.value, np.uint8) for _ in range(5)]
    ro = np.zeros(n_pairs, np.int64)
    rl = np.zeros(n_pairs, np.int32)
    hb = np.zeros(hb_n.value, np.uint8)
    ho = np.zeros(n_pairs, np.int64)
    hl = np.zeros(n_pairs, np.int32)
    check(lib.fcs_synth_phmm(seed, n_pairs, R, hmin, hmax, *[_ptr(a) for a in rb], _ptr(ro), _ptr(rl), _ptr(hb),
                             _ptr(ho), _ptr(hl)))
    idx = np.arange(n_pairs, dtype=np.int32)
    return PhmmPairs(rb[0], rb[1], rb[2], rb[3], rb[4], ro, rl, hb, ho, hl, idx, idx.copy())


# ---------------------------------------------------------------- banded SW
def bsw_params(mat=None, o_del=6, e_del=1, o_ins=6, e_ins=1, end_bonus=5, zdrop=100) -> BswParams:
    p = BswParams()
    lib.fcs_bsw_params_default(C.byref(p))
    if mat is not None:
        for i, v in enumerate(np.asarray(mat, dtype=np.int8).ravel()):
            p.mat[i] = int(v)
    p.o_del, p.e_del, p.o_ins, p.e_ins, p.end_bonus, p.zdrop = o_del, e_del, o_ins, e_ins, end_bonus, zdrop
    return p


def default_mat() -> np.ndarray:
    p = BswParams()
    lib.fcs_bsw_params_default(C.byref(p))
    return np.array(list(p.mat), dtype=np.int8)


@dataclass
class BswTasks:
    qbuf: np.ndarray
    qoff: np.ndarray
    qlen: np.ndarray
    tbuf: np.ndarray
    toff: np.ndarray
    tlen: np.ndarray
    h0: np.ndarray
    w: np.ndarray

    @property
    def n(self) -> int:
        return int(self.qlen.size)

    def to_struct(self, ptr=_ptr) -> BswBatch:
        b = BswBatch()
        b.qbuf, b.qoff, b.qlen = ptr(self.qbuf), ptr(self.qoff), ptr(self.qlen)
        b.tbuf, b.toff, b.tlen = ptr(self.tbuf), ptr(self.toff), ptr(self.tlen)
        b.h0, b.w, b.n = ptr(self.h0), ptr(self.w), self.n
        b.qbytes, b.tbytes = int(self.qbuf.size), int(self.tbuf.size)
        b.max_qlen = int(self.qlen.max()) if self.n else 0
        b.max_tlen = int(self.tlen.max()) if self.n else 0
        return b

    def task(self, k: int):
        q = self.qbuf[self.qoff[k]:self.qoff[k] + self.qlen[k]]
        t = self.tbuf[self.toff[k]:self.toff[k] + self.tlen[k]]
        return q, t, int(self.h0[k]), int(self.w[k])


def make_tasks(items) -> BswTasks:
    """items: list of (query codes, target codes, h0, w)."""
    ql = np.array([len(x[0]) for x in items], np.int32)
    tl = np.array([len(x[1]) for x in items], np.int32)
    qo = np.concatenate([[0], np.cumsum(ql[:-1], dtype=np.int64)]).astype(np.int64) if items else np.zeros(0, np.int64)
    to = np.concatenate([[0], np.cumsum(tl[:-1], dtype=np.int64)]).astype(np.int64) if items else np.zeros(0, np.int64)
    qb = np.concatenate([np.asarray(x[0], np.uint8) for x in items]) if items else np.zeros(0, np.uint8)
    tb = np.concatenate([np.asarray(x[1], np.uint8) for x in items]) if items else np.zeros(0, np.uint8)
    return BswTasks(qb, qo, ql, tb, to, tl, np.array([x[2] for x in items], np.int32),
                    np.array([x[3] for x in items], np.int32))


def bsw_extend_batch(t: BswTasks, params: BswParams | None = None, device=0):
    params = params or bsw_params()
    res = np.zeros((t.n, 6), np.int32)
    cells = np.zeros(t.n, np.int64)
    b = t.to_struct()
    check(lib.fcs_bsw_extend_batch(C.byref(b), C.byref(params), res.ctypes.data_as(i32p),
                                   cells.ctypes.data_as(i64p), device))
    return res, cells


def bsw_extend_tasks(t: BswTasks, params: BswParams | None = None, device=0, devices=None):
    """fcs_bsw_extend over an array of fcs_bsw_task (bwa's per-task pointers);
    devices: a list of device slots -> fcs_bsw_extend_multi (static partition)."""
    params = params or bsw_params()
    arr = (BswTask * max(t.n, 1))()
    base_q, base_t = t.qbuf.ctypes.data, t.tbuf.ctypes.data
    for i in range(t.n):
        arr[i] = BswTask(int(t.qlen[i]), int(t.tlen[i]), int(t.h0[i]), int(t.w[i]),
                         C.cast(base_q + int(t.qoff[i]), u8p), C.cast(base_t + int(t.toff[i]), u8p))
    res = (BswResult * max(t.n, 1))()
    if devices is None:
        check(lib.fcs_bsw_extend(arr, t.n, C.byref(params), res, device))
    else:
        d = np.asarray(devices, np.int32)
        check(lib.fcs_bsw_extend_multi(arr, t.n, C.byref(params), res, d.ctypes.data, len(d)))
    return np.array([[r.score, r.qle, r.tle, r.gtle, r.gscore, r.max_off] for r in res[:t.n]], np.int32)


def bsw_global(t: BswTasks, params: BswParams | None = None, device=0, with_cigar=True):
    params = params or bsw_params()
    n = t.n
    tasks = (BswTask * max(n, 1))()
    for k in range(n):
        q, tg, h0, w = t.task(k)
        tasks[k] = BswTask(int(t.qlen[k]), int(t.tlen[k]), 1, w,
                           q.ctypes.data_as(u8p) if q.size else None, tg.ctypes.data_as(u8p) if tg.size else None)
    scores = np.zeros(n, np.int32)
    if not with_cigar:
        check(lib.fcs_bsw_global(tasks, n, C.byref(params), scores.ctypes.data_as(i32p), None, None, None, None,
                                 device))
        return scores, None
    cap = (t.qlen + t.tlen + 2).astype(np.int32)
    off = np.concatenate([[0], np.cumsum(cap[:-1], dtype=np.int64)]).astype(np.int64)
    arena = np.zeros(int(cap.sum()) if n else 1, np.uint32)
    ncig = np.zeros(n, np.int32)
    check(lib.fcs_bsw_global(tasks, n, C.byref(params), scores.ctypes.data_as(i32p), arena.ctypes.data_as(u32p),
                             off.ctypes.data_as(i64p), cap.ctypes.data_as(i32p), ncig.ctypes.data_as(i32p), device))
    cigars = [arena[off[k]:off[k] + ncig[k]].copy() for k in range(n)]
    return scores, cigars


def bsw_align(t: BswTasks, xtra, params: BswParams | None = None, device=0) -> np.ndarray:
    """Batched ksw_align2 (fcs_bsw_align): (n, 7) int32 rows = bwa's kswr_t
    (score, te, qe, score2, te2, tb, qb)."""
    params = params or bsw_params()
    n = t.n
    tasks = (BswTask * max(n, 1))()
    for k in range(n):
        q, tg, _, _ = t.task(k)
        tasks[k] = BswTask(int(t.qlen[k]), int(t.tlen[k]), 0, 0, q.ctypes.data_as(u8p) if q.size else None,
                           tg.ctypes.data_as(u8p) if tg.size else None)
    x = np.ascontiguousarray(np.broadcast_to(np.asarray(xtra, np.int32), (n,)), np.int32)
    out = np.zeros((max(n, 1), 7), np.int32)
    check(lib.fcs_bsw_align(tasks, n, C.byref(params), x.ctypes.data_as(i32p), out.ctypes.data, device))
    return out[:n]


def ksw_align2(q, t, xtra, mat=None, o_del=6, e_del=1, o_ins=6, e_ins=1):
    """bwa's ksw_align2 signature twin: (score, te, qe, score2, te2, tb, qb)."""
    q = np.ascontiguousarray(q, np.uint8)
    t = np.ascontiguousarray(t, np.uint8)
    m = np.ascontiguousarray(default_mat() if mat is None else mat, np.int8)
    r = lib.fcs_ksw_align2(len(q), q.ctypes.data_as(u8p), len(t), t.ctypes.data_as(u8p), 5, m.ctypes.data_as(i8p),
                           o_del, e_del, o_ins, e_ins, xtra, None)
    if r.score == -2147483648:
        raise FcsError(FCS_ERR_DEVICE, lib.fcs_last_error().decode(errors="replace"))
    return (r.score, r.te, r.qe, r.score2, r.te2, r.tb, r.qb)


def ksw_extend2(q, t, h0, w, mat=None, o_del=6, e_del=1, o_ins=6, e_ins=1, end_bonus=5, zdrop=100):
    q = np.ascontiguousarray(q, np.uint8)
    t = np.ascontiguousarray(t, np.uint8)
    m = np.ascontiguousarray(default_mat() if mat is None else mat, np.int8)
    outs = [C.c_int() for _ in range(5)]
    sc = lib.fcs_ksw_extend2(len(q), q.ctypes.data_as(u8p), len(t), t.ctypes.data_as(u8p), 5, m.ctypes.data_as(i8p),
                             o_del, e_del, o_ins, e_ins, w, end_bonus, zdrop, h0, *[C.byref(o) for o in outs])
    if sc == FCS_KSW_FAILED:
        raise FcsError(sc, lib.fcs_last_error().decode(errors="replace"))
    return (sc,) + tuple(o.value for o in outs)


def ksw_global2(q, t, w, mat=None, o_del=6, e_del=1, o_ins=6, e_ins=1):
    q = np.ascontiguousarray(q, np.uint8)
    t = np.ascontiguousarray(t, np.uint8)
    m = np.ascontiguousarray(default_mat() if mat is None else mat, np.int8)
    n = C.c_int()
    cig = u32p()
    sc = lib.fcs_ksw_global2(len(q), q.ctypes.data_as(u8p), len(t), t.ctypes.data_as(u8p), 5,
                             m.ctypes.data_as(i8p), o_del, e_del, o_ins, e_ins, w, C.byref(n), C.byref(cig))
    if sc == FCS_KSW_FAILED:
        raise FcsError(sc, lib.fcs_last_error().decode(errors="replace"))
    ops = np.array([cig[i] for i in range(n.value)], np.uint32)
    if cig:
        libc.free(cig)
    return sc, ops


def synth_bsw(seed: int, n_reads: int, read_len: int = 151, ref_len: int = 10_000_000, w: int = 100,
              mode: int = 0, fixed_q: int = 151, fixed_t: int = 251) -> BswTasks:
    nt, qb, tb = C.c_int64(), C.c_int64(), C.c_int64()
    check(lib.fcs_synth_bsw_sizes(seed, n_reads, read_len, ref_len, w, mode, fixed_q, fixed_t, C.byref(nt),
                                  C.byref(qb), C.byref(tb)))
    n = nt.value
    t = BswTasks(np.zeros(qb.value, np.uint8), np.zeros(n, np.int64), np.zeros(n, np.int32),
                 np.zeros(tb.value, np.uint8), np.zeros(n, np.int64), np.zeros(n, np.int32),
                 np.zeros(n, np.int32), np.zeros(n, np.int32))
    got = C.c_int64()
    check(lib.fcs_synth_bsw(seed, n_reads, read_len, ref_len, w, mode, fixed_q, fixed_t, _ptr(t.qbuf), _ptr(t.qoff),
                            _ptr(t.qlen), _ptr(t.tbuf), _ptr(t.toff), _ptr(t.tlen), _ptr(t.h0), _ptr(t.w),
                            C.byref(got)))
    assert got.value == n
    return t


def cigar_str(ops) -> str:
    return "".join(f"{int(c) >> 4}{'MID'[int(c) & 0xf]}" for c in ops)


FCS_BGZF_OK, FCS_BGZF_CORRUPT, FCS_BGZF_OVERFLOW, FCS_BGZF_CRC = 0, 1, 2, 3
FCS_BGZF_BUSY = 1  # fcs_bgzf_inflate_try's return when no warm inflate session is idle


def bgzf_index(comp, cap: int | None = None):
    """fcs_bgzf_index: (coff, uoff, comp_used) of the whole BGZF members in
    `comp` (bytes / uint8 array); coff / uoff have n + 1 entries."""
    c = np.frombuffer(bytes(comp), np.uint8) if not isinstance(comp, np.ndarray) else np.ascontiguousarray(comp, np.uint8)
    cap = len(c) // 20 + 1 if cap is None else cap
    coff = np.zeros(cap + 1, np.int64)
    uoff = np.zeros(cap + 1, np.int64)
    n, used = C.c_int32(), C.c_int64()
    check(lib.fcs_bgzf_index(_ptr(c), len(c), coff.ctypes.data, uoff.ctypes.data, cap, C.byref(n), C.byref(used)))
    return coff[:n.value + 1].copy(), uoff[:n.value + 1].copy(), used.value


def bgzf_inflate(comp, out_cap: int | None = None, device: int = 0):
    """fcs_bgzf_inflate: (inflated bytes of the whole members, comp_used)."""
    c = np.frombuffer(bytes(comp), np.uint8) if not isinstance(comp, np.ndarray) else np.ascontiguousarray(comp, np.uint8)
    cap = int(bgzf_index(c)[1][-1]) if out_cap is None else out_cap
    out = np.zeros(max(cap, 1), np.uint8)
    used, got = C.c_int64(), C.c_int64()
    check(lib.fcs_bgzf_inflate(_ptr(c), len(c), out.ctypes.data, cap, C.byref(used), C.byref(got), device))
    return out[:got.value].tobytes(), used.value
