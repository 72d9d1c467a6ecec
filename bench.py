"""bench.py -- Mpixels/s encode+decode of 8K RGB frames, 5/3 lossless & 9/7 lossy.

Workload (BASELINE.json configs[2], the metric's 8K RGB case): one synthetic
7680x4320 12-bit RGB frame per GPU (tests/golden/synth.py "smooth", seed 3 on
rank 0 -- the same image whose reference codestream hashes are pinned in
tests/golden/manifest_large.json).  One step = encode + decode of the frame
with the 9/7 irreversible path (grk_compress -I) + encode + decode with the
5/3 lossless path (default options), i.e. 2 frames' worth of pixels through
both directions.  The frame is HBM-resident when timing starts; decoded planes
are written back to HBM.  The codestream crosses PCIe once each way because
Tier-2 / headers run on the host.

Multi-GPU: one process per GPU (torch.distributed.run), each encodes/decodes
its own frame -- a frame batch, no data-path collective;
"scaling": "weak".  value = frames*pixels of all ranks / max-over-ranks time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "oracle")]

# Frames in flight run on their own HIP streams; HIP maps streams onto at most
# GPU_MAX_HW_QUEUES hardware queues per process (4 by default on the box),
# which would serialise the 12 streams' kernels in groups of 3.  The runtime
# reads the value when the process starts, so with fewer than 16 the bench
# reruns itself as a child process with 16 (nothing has touched the GPU yet)
# and exits with the child's status.
def _concurrency_arg():
    for i, a in enumerate(sys.argv):
        if a.startswith("--concurrency"):
            v = a.split("=", 1)[1] if "=" in a else (sys.argv[i + 1] if i + 1 < len(sys.argv) else "12")
            return int(v)
    return 12


# one hardware queue per codec stream plus torch's own (gpurun caps the knob at 32)
HW_QUEUES = min(32, max(16, _concurrency_arg() + 4))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < HW_QUEUES:
    import subprocess
    sys.exit(subprocess.call([sys.executable] + sys.argv, env=dict(os.environ, GPU_MAX_HW_QUEUES=str(HW_QUEUES))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

H, W, C, BITS = 4320, 7680, 3, 12
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def dwt_bytes(h, w, c, numres=6):
    """B_DWT: sum over levels of 8 B x |R_l| (read + write int32)."""
    tot = 0
    rh, rw = h, w
    for _ in range(numres - 1):
        tot += 8 * rh * rw
        rh, rw = (rh + 1) // 2, (rw + 1) // 2
    return tot * c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--concurrency", type=int, default=12, help="frames in flight per GPU: 1, or an even number (half 9/7, half 5/3)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)

    import grokimagecompression_amd as grk
    import synth

    img = synth.synth_image(H, W, C, BITS, 3 + rank)
    frame = torch.from_numpy(img).to("cuda:%d" % local)
    # two codec contexts (each with its own HIP stream and host thread): the
    # 9/7 and the 5/3 frame of a step are coded concurrently, so the T1
    # kernels of one overlap the other's (T1 is latency-bound and leaves most
    # SIMD issue slots free) and host Tier-2 overlaps device work.
    ncodec = max(1, args.concurrency)
    assert ncodec == 1 or ncodec % 2 == 0, "--concurrency must be 1 or even"
    codecs = [grk.Codec(local) for _ in range(ncodec)]
    p97 = grk.CParams.make(irreversible=True)
    p53 = grk.CParams.make(irreversible=False)
    npairs = max(1, ncodec // 2)              # (9/7 frame, 5/3 frame) pairs per step
    outs = [(torch.empty_like(frame), torch.empty_like(frame)) for _ in range(npairs)]
    out97, out53 = outs[0]
    st = {}

    # one torch stream per codec (the codec runs on the caller's current
    # stream, which torch keeps per host thread)
    streams = [torch.cuda.Stream(device=local) for _ in range(ncodec)]
    torch.cuda.synchronize()

    def pipe(codec, p, out, tag):
        with torch.cuda.stream(streams[codecs.index(codec)]):
            b = codec.compress(frame, BITS, p, view=True)
            st["enc" + tag] = codec.stats()
            n = len(b)
            codec.decompress(b, out=out)
            st["dec" + tag] = codec.stats()
            st["bytes" + tag] = n

    pool = None

    if ncodec > 1:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=ncodec)

    jobs = [(codecs[0], p97, out97, "97"), (codecs[0], p53, out53, "53")] if pool is None else \
        [j for i in range(npairs) for j in ((codecs[2 * i], p97, outs[i][0], "97"),
                                            (codecs[2 * i + 1], p53, outs[i][1], "53"))]

    def run_steps(n):
        """n steps; each frame's pipeline runs its n iterations back to back on
        its own thread/stream (no barrier between steps, so no pipeline waits
        for the slowest one before starting its next frame)."""
        if pool is None:
            for _ in range(n):
                for j in jobs:
                    pipe(*j)
        else:
            def loop(j):
                for _ in range(n):
                    pipe(*j)
            for x in [pool.submit(loop, j) for j in jobs]:
                x.result()
        st["bytes"] = (st["bytes97"], st["bytes53"])

    run_steps(args.warmup)
    assert torch.equal(out53, frame), "5/3 round trip is not lossless"

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    run_steps(args.steps)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda:%d" % local)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    pix_per_step = 2 * npairs * H * W  # npairs x (one frame through 9/7 + one through 5/3)
    value = world * pix_per_step * args.steps / elapsed / 1e6
    ms_per_step = 1e3 * elapsed / args.steps

    # roofline: the forward 9/7 DWT of the frame = 5 level launches (one per
    # decomposition level, all 3 components in each), B_DWT / the HIP-event
    # time around those launches on the codec's stream (= per-launch bytes /
    # mean launch duration).  traffic: HBM bytes per launch from the committed
    # rocprofv3 PMC summary (scripts/pmc_bench.sh), when present.
    # measured in isolation after the timed region (the timed region overlaps
    # frames, so kernel durations there include contention): 3 x 9/7 encodes
    # on one context, nothing else in flight, min of the HIP-event DWT times.
    bdwt = dwt_bytes(H, W, C)
    nlaunch = 5
    torch.cuda.synchronize()
    iso = []
    with torch.cuda.stream(streams[0]):
        for _ in range(3):
            codecs[0].compress(frame, BITS, p97, view=True)
            iso.append(codecs[0].stats()["dwt_ms"])
    dwt_ms = min(iso)
    achieved = bdwt / (dwt_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "dwt_pmc_latest.json")
    if os.path.exists(pmc):
        d = json.load(open(pmc))
        tot = sum(e["bytes"] for k, v in d["kernels"].items() if "k_dwt_fwd<true" in k for e in v)
        traffic = round(tot / nlaunch)
    roofline = {"bound": "hbm", "kernel": "k_dwt_fwd<9/7> (5 level launches x 3 comps, dwt.hip)",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": bdwt // nlaunch, "launches": nlaunch,
                "kernel_ms_per_launch": round(dwt_ms / nlaunch, 4),
                "measured": "HIP events on the codec stream, 9/7 encode run alone after the timed region"}

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        import pyoracle
        pyoracle.build()
        ncpu = min(16, os.cpu_count() or 1)
        t0 = time.perf_counter()
        b = pyoracle.encode(img, BITS, pyoracle.params(irreversible=True, nthreads=ncpu))
        pyoracle.decode(b, nthreads=ncpu)
        b = pyoracle.encode(img, BITS, pyoracle.params(irreversible=False, nthreads=ncpu))
        pyoracle.decode(b, nthreads=ncpu)
        ct = time.perf_counter() - t0
        cpu = {"value": round(2 * H * W / ct / 1e6, 3), "unit": "Mpixels/s", "cores": ncpu, "kind": "port",
               "sample": "1 step (8K 12-bit RGB frame: 9/7 enc+dec + 5/3 enc+dec) through the C oracle "
                         "(oracle/grk_oracle.c, byte-identical to Grok 5.1.0), %d threads" % ncpu,
               "seconds": round(ct, 2)}

    if rank == 0:
        def r(d):
            return {k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items()}
        line = {
            "metric": "Mpixels/sec encode+decode, 8K RGB 5/3 lossless & 9/7 lossy",
            "value": round(value, 2), "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32/f32 (integer encode, f32 9/7 decode)",
            "data": "synthetic (tests/golden/synth.py smooth+2% noise, seed 3+rank)",
            "config": {"workload": "8K 7680x4320 12-bit RGB frame per GPU; 9/7 (-I) + 5/3 lossless, enc+dec; "
                                   "6 resolutions, 64x64 code-blocks, 1 layer LRCP",
                       "frames_per_step_per_gpu": 2 * npairs, "frames_in_flight": ncodec,
                       "parallelism": "frame-batch x%d (no collectives)" % world},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "codestream_bytes": {"9/7": st["bytes"][0], "5/3": st["bytes"][1]},
            "stage_ms": {k: r(st[k]) for k in ("enc97", "dec97", "enc53", "dec53")},
        }
        print(json.dumps(line), flush=True)
    for c in codecs:
        c.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
