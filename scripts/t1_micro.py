"""T1 micro-benchmark on the GPU box: per-block latency vs batch throughput of
the lane coder through the C-ABI stage entry points (not part of the bench)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import numpy as np
import torch
import grokimagecompression_amd as grk

L = grk.lib()
ENC = np.dtype([("coef_off", "<u8"), ("out_off", "<u8"), ("stride", "<u4"), ("w", "<u4"), ("h", "<u4"),
                ("orient", "<u4"), ("qmfbid", "<i4"), ("inv_step", "<i4")])
DEC = np.dtype([("data_off", "<u8"), ("dst_off", "<u8"), ("len", "<u4"), ("numpasses", "<u4"), ("numbps", "<u4"),
                ("w", "<u4"), ("h", "<u4"), ("orient", "<u4"), ("dstride", "<u4"), ("irrev", "<i4"),
                ("step", "<f4"), ("pad", "<u4")])
RES_WORDS = 100


def run(n, scale, reps=3):
    rng = np.random.default_rng(1)
    coef = np.round(rng.laplace(0, scale, size=(n, 64, 64))).astype(np.int32)
    dcoef = torch.from_numpy(coef).cuda()
    eb = np.zeros(n, ENC)
    eb["coef_off"] = np.arange(n) * 4096
    eb["out_off"] = np.arange(n) * (4096 * 4 + 128) + 16
    eb["stride"], eb["w"], eb["h"] = 64, 64, 64
    eb["orient"] = np.arange(n) % 4
    eb["qmfbid"] = 1
    deb = torch.from_numpy(eb.view(np.uint8)).cuda()
    out = torch.zeros(n * (4096 * 4 + 128) + 256, dtype=torch.uint8, device="cuda")
    scr = torch.empty(((n + 63) // 64 * 64) * L.grkgpu_t1_scratch_bytes() + 256, dtype=torch.uint8, device="cuda")
    res = torch.zeros(n * RES_WORDS, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = L.grkgpu_t1_encode_blocks(deb.data_ptr(), n, dcoef.data_ptr(), scr.data_ptr(), out.data_ptr(),
                                       res.data_ptr(), s)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0, rc
        ts.append(e0.elapsed_time(e1))
    r = res.view(n, RES_WORDS).cpu().numpy()
    rec = 2112 + 16384 * 2 + 512  # sizeof(T1Scratch)
    cnt = scr[: n * rec].view(n, rec)[:, rec - 512:].contiguous().view(torch.int32).view(n, 128).cpu().numpy()
    nsym = cnt.reshape(n, 32, 4)[:, :, :3].sum(axis=(1, 2))
    nb, npass, ln = r[:, 0], r[:, 1], r[:, 2]
    # decode the same blocks
    db = np.zeros(n, DEC)
    db["data_off"] = eb["out_off"]
    db["dst_off"] = np.arange(n) * 4096
    db["len"] = ln
    db["numpasses"] = npass
    db["numbps"] = nb
    db["w"], db["h"], db["dstride"] = 64, 64, 64
    db["orient"] = eb["orient"]
    ddb = torch.from_numpy(db.view(np.uint8)).cuda()
    dst = torch.zeros(n * 4096, dtype=torch.int32, device="cuda")
    td = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = L.grkgpu_t1_decode_blocks(ddb.data_ptr(), n, out.data_ptr(), scr.data_ptr(), dst.data_ptr(), s)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0, rc
        td.append(e0.elapsed_time(e1))
    ok = torch.equal(dst.view(n, 64, 64), dcoef)  # 5/3: decoded v/2 == coefficient
    print(f"n={n:6d} scale={scale:6.0f} numbps~{nb.mean():.1f} passes~{npass.mean():.1f} bytes/blk~{ln.mean():.0f} "
          f"symbols/blk~{nsym.mean():.0f} (max {nsym.max()}) enc {min(ts):8.3f} ms dec {min(td):8.3f} ms  roundtrip_ok={ok}",
          flush=True)


sizes = [int(a) for a in sys.argv[1:]] or [1, 16, 256, 1024, 4096, 24576]
for scale in (30.0, 300.0):
    for n in sizes:
        run(n, scale)
