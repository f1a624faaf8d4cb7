"""Throughput of the BGZF inflate kernel (fcs_bgzf_inflate_dev) on a BAM-like
batch, with the host's libdeflate (one thread) and the PCIe-inclusive host
entry point beside it.

  python tools/bgzf_bench.py [--members 4096] [--reps 5]

Members: 64 distinct BAM-record-shaped payloads of 64 KiB (libdeflate level 5,
the host writer's setting), tiled to --members; prints one JSON line."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "falcon-genome_amd"), os.path.join(ROOT, "tests")]
import bgzf_cases  # noqa: E402
import fcship  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--members", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kind", default="bam")
    ap.add_argument("--stress", type=int, default=0,
                    help="extra launches, each checked: every status OK and the output equal to the first launch's")
    a = ap.parse_args()
    import torch
    rng = np.random.default_rng(1)
    base = []
    for _ in range(64):
        p = bgzf_cases.payload(rng, a.kind, 65280)
        base.append((bgzf_cases.member_libdeflate(p, 5), p))
    members = [base[k % 64] for k in range(a.members)]
    blob = b"".join(m for m, _ in members)
    want_total = sum(len(p) for _, p in members)
    coff, uoff, used = fcship.bgzf_index(blob)
    assert used == len(blob) and uoff[-1] == want_total
    n = len(coff) - 1
    dev = torch.device("cuda", 0)
    comp = torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).to(dev)
    dco, duo = torch.from_numpy(coff).to(dev), torch.from_numpy(uoff).to(dev)
    out = torch.empty(int(uoff[-1]), dtype=torch.uint8, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()

    def run():
        fcship.check(fcship.lib.fcs_bgzf_inflate_dev(comp.data_ptr(), dco.data_ptr(), duo.data_ptr(), n,
                                                     out.data_ptr(), st.data_ptr(), 0, ctypes.c_void_p(s.cuda_stream)))

    run()
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    o = out.cpu().numpy()
    for k in range(min(n, 64)):
        assert o[uoff[k]:uoff[k + 1]].tobytes() == members[k][1]
    if a.stress:
        first = out.clone()
        bad = 0
        for r in range(a.stress):
            out.fill_(0x5A)
            st.fill_(-1)
            run()
            torch.cuda.synchronize()
            ok = bool((st == 0).all().item()) and bool(torch.equal(out, first))
            bad += not ok
        print(json.dumps({"stress_launches": a.stress, "bad_launches": bad}), flush=True)
        assert bad == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.reps):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    # host entry point: H2D + kernel + D2H + staging copies
    fcship.bgzf_inflate(blob, out_cap=want_total)
    t = time.perf_counter()
    fcship.bgzf_inflate(blob, out_cap=want_total)
    host_s = time.perf_counter() - t
    # libdeflate on one host thread over the first 256 members
    L = ctypes.CDLL("libdeflate.so.0")
    L.libdeflate_alloc_decompressor.restype = ctypes.c_void_p
    L.libdeflate_deflate_decompress.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                                ctypes.c_size_t, ctypes.c_void_p]
    d = L.libdeflate_alloc_decompressor()
    buf = ctypes.create_string_buffer(65536)
    sample = [(m[18:-8], len(p)) for m, p in members[:256]]
    t = time.perf_counter()
    for r, n_out in sample:  # exact output size (no actual-size pointer), as the host reader calls it
        assert L.libdeflate_deflate_decompress(d, r, len(r), buf, n_out, None) == 0
    cpu_s = time.perf_counter() - t
    cpu_out = sum(len(p) for _, p in members[:256])
    print(json.dumps({
        "bench": "bgzf_inflate", "kind": a.kind, "members": n, "comp_bytes": len(blob), "out_bytes": want_total,
        "kernel_ms": round(ms, 3), "kernel_out_GBps": round(want_total / ms / 1e6, 2),
        "kernel_in_GBps": round(len(blob) / ms / 1e6, 2), "members_per_s": round(n / ms * 1e3),
        "host_call_ms": round(host_s * 1e3, 2), "host_call_out_GBps": round(want_total / host_s / 1e9, 2),
        "libdeflate_1thread_out_GBps": round(cpu_out / cpu_s / 1e9, 3)}))


if __name__ == "__main__":
    main()
