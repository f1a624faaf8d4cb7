"""Lane-level CPU emulation of the row-streamed PairHMM kernel
(falcon-genome_amd/csrc/phmm_stream.h) for ONE 16-lane segment: the same
stream layout (pad, rows 1..R, V), per-stripe lane mapping, hap-code buffers,
LDS boundary ring, Z constant, DPP hand-off and V capture, in float32 with
fma emulated in double.  Unwritten LDS is NaN (ring) / random bytes (hap
codes), so a read the kernel relies on but never wrote shows up as a wrong
or NaN result.  Debugging aid, not a test oracle.

usage: python tools/phmm_stream_emu.py        (random batch vs the oracle)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "falcon-genome_amd"))

f32 = np.float32
PFD = 2


def fma(a, b, c):
    return f32(np.float64(a) * np.float64(b) + np.float64(c))


def tables():
    import oracle_lib
    ph = np.ctypeslib.as_array(oracle_lib.lib.oracle_phmm_ph2pr_f(), (128,)).astype(f32)
    dmatch = (f32(1) - ph).astype(f32)
    dmis = (ph / f32(3)).astype(f32)
    mm = {}
    for hi in range(128):
        for lo in range(hi + 1):
            mm[(hi, lo)] = f32(oracle_lib.lib.oracle_phmm_mm_f(hi, lo))
    return ph, dmatch, dmis, mm


def base_code(b):
    return {65: 0, 67: 1, 71: 2, 84: 3, 78: 4}.get(int(b), 5)


def base_mask(rb):
    c = base_code(rb)
    return 0x7F if c == 4 else 0x10 if c == 5 else (1 << c) | 0x10


class Emu:
    def __init__(self, T):
        self.ph, self.dmatch, self.dmis, self.mm = T
        self.init_const = f32(2.0 ** 120)
        self.log10_init = f32(np.log10(np.float32(2.0 ** 120)))

    def row_params(self, read, pos, R):
        """row_params<float,false> of read row pos (0-based) + next-row fields."""
        rb, bq, iq, dq, gq = read
        q, qd, qc = int(bq[pos]) & 127, int(dq[pos]) & 127, int(gq[pos]) & 127
        e1 = self.dmatch[q]
        e3 = e1 if rb[pos] == ord("N") else self.dmis[q]
        my, yy = self.ph[qd], self.ph[qc]
        ni = nd = nc = 0
        if pos + 1 < R:
            ni, nd, nc = int(iq[pos + 1]) & 127, int(dq[pos + 1]) & 127, int(gq[pos + 1]) & 127
        hi, lo = max(ni, nd), min(ni, nd)
        mm = self.mm[(hi, lo)]
        gm = self.dmatch[nc]
        mx, xx = self.ph[ni], self.ph[nc]
        my = f32(my * gm)
        return dict(e1=e1, e3=e3, my=my, yy=yy, mm=mm, gm=gm, mx=mx, xx=xx, mask=base_mask(rb[pos]))

    def srow(self, read, r, R, H):
        if r == 0:
            return dict(e1=f32(1), e3=f32(1), my=f32(0), yy=f32(0), mm=f32(1), gm=f32(0), mx=f32(0), xx=f32(0), mask=0)
        if r == R + 1:
            return dict(e1=f32(1), e3=f32(1), my=f32(1), yy=f32(1), mm=f32(1), gm=f32(1), mx=f32(0), xx=f32(0), mask=0)
        c = self.row_params(read, r - 1, R)
        if r == R:
            c.update(my=f32(0), mm=f32(1), gm=f32(1), mx=f32(0), xx=f32(0))
        if r == 1:
            x0 = f32(f32(self.init_const / f32(H)) * self.dmatch[int(read[4][0]) & 127])
            c["e1"] = f32(c["e1"] * x0)
            c["e3"] = f32(c["e3"] * x0)
        return c

    def run_segment(self, pairs, rng, rec=None):
        """pairs: list of (read tuple of 5 uint8 arrays, hap uint8 array). Returns log10 results."""
        K = len(pairs)
        U = [(len(rd[0]) + 2) >> 1 for rd, _ in pairs]
        ubb = np.concatenate([[0], np.cumsum(U)])
        total = int(ubb[-1])
        nstr = (total + 15) // 16
        hmax = max(len(h) for _, h in pairs)
        ring = np.full(hmax + 64 + 64, np.nan, f32).reshape(-1)  # X
        ringI = np.full_like(ring, np.nan)
        ring[0] = ringI[0] = 0
        hb = [rng.integers(0, 256, hmax + 200).astype(np.int64) for _ in range(2)]
        OFF = 40  # hap buffer index offset (reads before column 0)
        out = [None] * K
        for st in range(nstr):
            lanes = []
            for l in range(16):
                g = 16 * st + l
                act = g < total
                k = int(np.searchsorted(ubb, g, side="right") - 1) if act else K
                if not act:
                    lanes.append(dict(act=False))
                    continue
                rd, hap = pairs[k]
                R, H = len(rd[0]), len(hap)
                u = g - int(ubb[k])
                pad = (R & 1) ^ 1
                ra = 2 * u + 1 - pad
                lanes.append(dict(act=True, k=k, u=u, R=R, H=H, ra=ra, rb=ra + 1,
                                  pa=self.srow(rd, ra, R, H), pb=self.srow(rd, ra + 1, R, H)))
            # fresh hap load (lane 15's pair starts in this stripe)
            L15 = lanes[15]
            kn = None
            for l in range(16):
                if lanes[l]["act"] and lanes[l]["u"] == 0:
                    kn = lanes[l]["k"]
            if kn is not None:
                hap = pairs[kn][1]
                for c in range(len(hap)):
                    hb[kn & 1][OFF + c + 1] = base_code(hap[c])
            need = max((ln["H"] + 2 * l + 3) if ln["act"] else 0 for l, ln in enumerate(lanes))
            nblk = (need + 15) // 16
            T_end = 16 * nblk
            zero = dict(e1=f32(0), e3=f32(0), my=f32(0), yy=f32(0), mm=f32(0), gm=f32(0), mx=f32(0), xx=f32(0),
                        mask=0)
            st_ = [dict(Mo=[f32(0)] * 2, Do=[f32(0)] * 2, Xp=[f32(0)] * 2, Xn=[f32(0)] * 2, In=[f32(0)] * 2,
                        hbp=6, acc=f32(0)) for _ in range(16)]
            if lanes[0]["act"] and lanes[0]["u"] == 0 and lanes[0]["ra"] == 0:
                st_[0]["Xp"] = [f32(0), f32(1)]  # pad at lane 0: Z(0) "received at step -1"
            writes = []
            for t in range(T_end):
                prev = [dict(Xn=list(s["Xn"]), In=list(s["In"])) for s in st_]
                for l in range(16):
                    ln = lanes[l]
                    s = st_[l]
                    pa = ln.get("pa", zero) if ln["act"] else zero
                    pb = ln.get("pb", zero) if ln["act"] else zero
                    start = ln["act"] and (l == 0 or ln["u"] == 0)
                    is_z = ln["act"] and ln["u"] == 0
                    zsh = 1 if (ln["act"] and ln["ra"] == 0) else 0
                    ca = t - 2 * l
                    # boundary value for column ca
                    if is_z:
                        col = ca + zsh
                        curX, curI = (f32(1) if col >= 0 else f32(0)), f32(0)
                    else:
                        curX, curI = (ring[ca], ringI[ca]) if 0 <= ca < ring.size else (np.nan, np.nan)
                    # hap code for row a at column ca
                    buf = hb[ln["k"] & 1] if ln["act"] else hb[0]
                    hba = int(buf[OFF + ca]) if 0 <= OFF + ca < buf.size else 0
                    hbb = s["hbp"]
                    s["hbp"] = hba
                    dX = prev[l - 1]["Xn"][1] if l > 0 else f32(0)
                    dI = prev[l - 1]["In"][1] if l > 0 else f32(0)
                    Xsw = [s["Xn"][0], curX if start else dX]
                    Isw = [s["In"][0], curI if start else dI]
                    I = [Isw[1], Isw[0]]

                    def prior(p, hcode):
                        bit = (p["mask"] >> (hcode & 31)) & 1
                        return p["e1"] if bit else p["e3"]
                    pr = [prior(pa, hba), prior(pb, hbb)]
                    M = [f32(s["Xp"][1] * pr[0]), f32(s["Xp"][0] * pr[1])]
                    P = [pa, pb]
                    D = [fma(s["Mo"][h], P[h]["my"], f32(s["Do"][h] * P[h]["yy"])) for h in range(2)]
                    Xn = [fma(M[h], P[h]["mm"], fma(I[h], P[h]["gm"], D[h])) for h in range(2)]
                    In = [fma(M[h], P[h]["mx"], f32(I[h] * P[h]["xx"])) for h in range(2)]
                    if rec is not None and ln["act"]:
                        rec[(ln["k"], ln["ra"], ca)] = (M[0], I[0])
                        rec[(ln["k"], ln["rb"], ca - 1)] = (M[1], I[1])
                        rec[("X", ln["k"], ln["ra"], ca)] = Xn[0]
                        rec[("X", ln["k"], ln["rb"], ca - 1)] = Xn[1]
                    if l == 15 and t >= 32:
                        writes.append((t - 31, Xn[1], In[1]))
                    if ln["act"] and ln["rb"] == ln["R"] + 1 and t == ln["H"] + 2 * l + 2:
                        s["acc"] = Xn[1]
                        out[ln["k"]] = float(np.log10(np.float32(Xn[1])) - self.log10_init) if Xn[1] > 0 else -np.inf
                    s["Xp"], s["Xn"], s["In"], s["Mo"], s["Do"] = Xsw, Xn, In, M, D
                # lane-15 writes land after this step's reads (in-order LDS)
                for slot, x, i in writes:
                    ring[slot], ringI[slot] = x, i
                writes.clear()
        return out


def main():
    import fcship
    import oracle_lib
    from test_pairhmm_gpu import random_batch
    emu = Emu(tables())
    rng = np.random.default_rng(1)
    reads, haps = random_batch(7, 60, 7, 1, 200, 1, 420)
    p = fcship.make_pairs(reads, haps)
    p.read_bq[::17] = 200
    ref, _ = oracle_lib.phmm_batch(p)
    # rebuild per-pair read tuples from the batch (bq edit included)
    bad = 0
    for i in [40, 152, 187, 289, 290, 292, 343, 0, 1, 2, 3]:
        ri, hi = p.pair_read[i], p.pair_hap[i]
        o, L = p.read_off[ri], p.read_len[ri]
        rd = tuple(a[o:o + L] for a in (p.read_bases, p.read_bq, p.read_iq, p.read_dq, p.read_gcp))
        hap = p.hap_bases[p.hap_off[hi]:p.hap_off[hi] + p.hap_len[hi]]
        if L < 33 or len(hap) < 1:
            continue
        got = emu.run_segment([(rd, hap)], rng)[0]
        ok = abs(got - ref[i]) <= 1e-5 * abs(ref[i])
        bad += not ok
        print(f"pair {i} R={L} H={len(hap)} emu={got:.6f} ref={ref[i]:.6f} {'ok' if ok else 'BAD'}")
    print("bad", bad)


if __name__ == "__main__":
    main()


def stream_check(seed=3, K=6):
    """One segment streaming K random pairs (R >= 33, mixed parity) vs the oracle."""
    import fcship
    import oracle_lib
    from test_pairhmm_gpu import random_batch
    emu = Emu(tables())
    reads, haps = random_batch(seed, K, K, 33, 120, 1, 200)
    p = fcship.make_pairs(reads, haps)
    ref, _ = oracle_lib.phmm_batch(p)
    nh = len(haps)
    pairs, idx = [], []
    for j in range(K):
        i = j * nh + (j % nh)
        ri, hi = p.pair_read[i], p.pair_hap[i]
        o, L = p.read_off[ri], p.read_len[ri]
        rd = tuple(a[o:o + L] for a in (p.read_bases, p.read_bq, p.read_iq, p.read_dq, p.read_gcp))
        pairs.append((rd, p.hap_bases[p.hap_off[hi]:p.hap_off[hi] + p.hap_len[hi]]))
        idx.append(i)
    got = emu.run_segment(pairs, np.random.default_rng(seed))
    for j, i in enumerate(idx):
        ok = abs(got[j] - ref[i]) <= 1e-5 * abs(ref[i])
        print(f"stream pair {j}: R={len(pairs[j][0][0])} H={len(pairs[j][1])} emu={got[j]:.6f} ref={ref[i]:.6f} "
              f"{'ok' if ok else 'BAD'}")
