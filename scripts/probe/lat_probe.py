"""Calibrate per-lane serial costs on the GPU box (VALU chain, LDS chains, branches, global load chain)."""
import ctypes, os, sys
import torch
here = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(here, "liblat_probe.so"))
L.probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
out = torch.zeros(1 << 20, dtype=torch.int32, device="cuda")
N = 1 << 20
tab = torch.randperm(N, device="cuda").to(torch.int32)
s = torch.cuda.current_stream().cuda_stream
names = ["valu_chain(2 dep ops/iter)", "lds_read_chain", "lds_rw_chain", "branchy(divergent)", "global_load_chain"]
for which in range(5):
    for blocks, threads in ((1, 1), (1, 64), (1024, 64), (4096, 64)):
        n = 20000 if which == 4 else 200000
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        L.probe(which, out.data_ptr(), tab.data_ptr(), n, blocks, threads, s)
        torch.cuda.synchronize()
        e0.record()
        L.probe(which, out.data_ptr(), tab.data_ptr(), n, blocks, threads, s)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        print(f"{names[which]:28s} blocks={blocks:5d} thr={threads:3d} n={n}: {ms:8.3f} ms  {ms*1e6/n:8.2f} ns/iter", flush=True)
