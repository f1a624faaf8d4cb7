import sys, time
sys.path.insert(0, "falcon-genome_amd"); sys.path.insert(0, "tests")
import torch, fcship, ctypes as C
for n in (1000, 10000, 100000):
    p = fcship.synth_phmm(5, n)
    fcship.phmm_compute_pairs(p)
    t = time.perf_counter()
    for _ in range(20): fcship.phmm_compute_pairs(p)
    dt = (time.perf_counter() - t) / 20
    d, r = C.c_double(), C.c_double()
    fcship.lib.fcs_phmm_last_device_ms(C.byref(d), C.byref(r))
    print(n, "pairs: call", round(dt*1e3, 3), "ms; device span", round(d.value, 3), "ms; cells/s", round(p.cells()/dt/1e9, 1), "GCUPS", flush=True)
