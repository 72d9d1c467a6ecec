"""bench.py -- Mpixels/s encode+decode of 8K RGB frames, 5/3 lossless & 9/7 lossy.

Workload (BASELINE.json configs[2], the metric's 8K RGB case): synthetic
7680x4320 12-bit RGB frames (tests/golden/synth.py "smooth", seed 3 + rank --
the image whose reference codestream hashes are pinned in
tests/golden/manifest_large.json).  One step = per pair of codec contexts,
encode + decode of the frame with the 9/7 irreversible path (grk_compress -I)
and encode + decode with the 5/3 lossless path; 8 such pairs (16 frames) are in
flight per GPU, each on its own codec context, HIP stream and host thread.

  value            whole-job throughput with each frame's int32 planes
                   already resident in HBM when the timed region starts.  The
                   task's bench contract fixes this: "`value` is whole-job
                   throughput with inputs already resident in HBM when the
                   timed region starts (if the boundary hands over host
                   buffers, note the PCIe-inclusive rate in DESIGN.md -- it is
                   never `value`)".  The codestream crosses PCIe once each way
                   per frame (host Tier-2 / headers), the decoded frame stays
                   in HBM.
  pcie_inclusive   SURVEY 8(d)'s end-to-end variant, reported beside it:
                   every frame starts in pinned host memory at its file's
                   sample width (12-bit -> uint16, 2 B/sample) and is copied
                   H2D inside the timed region (grkgpu_compress_ex widens it
                   on the GPU).
  t1               MQ symbols/s and code-blocks/s (batch and lone frame).
  e2e_frac         value / (8e12 / B_e2e), B_e2e = C (ceil(prec/8) + 4 * 4/3 + 4).
  roofline         the forward 9/7 DWT (dominant HBM kernel): B_DWT over the
                   sum of its launches' device times; roofline.inverse the
                   same for the decode's inverse 9/7 DWT; roofline.r53 the
                   forward and inverse 5/3 DWT (8K workload).
  cpu_baseline     the REFERENCE (Grok 5.1.0 libgrok compiled from source,
                   oracle/_ref) on every host core of the process's affinity
                   mask, one frame pair.

Multi-GPU: one process per GPU (torch.distributed.run), each codes its own
frames -- a frame batch, no data-path collective; "scaling":
"weak".  value = frames*pixels of all ranks / max-over-ranks time.  Rank r
uses device LOCAL_RANK % device_count (so --gpus 2 also runs on one GPU); the
timing barrier and max reduction go over gloo -- no RCCL communicator.
`python bench.py --gpus N` run directly (no WORLD_SIZE) launches the N ranks
itself before anything touches a GPU.

--workload c5: DCI 4K 12-bit cinema frames (-cinema4K 24, BASELINE configs[4]),
encode + decode, frame batch.  --workload c4: the 16K 16-bit tiled image
(configs[3]) with its 256 tiles sharded over the ranks.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "oracle")]


def _arg(name, default):
    for i, a in enumerate(sys.argv):
        if a.startswith(name):
            return a.split("=", 1)[1] if "=" in a else (sys.argv[i + 1] if i + 1 < len(sys.argv) else default)
    return default


# --gpus N without a torch.distributed launcher: start the N ranks now, as
# child processes, before anything touches a GPU, and exit with their status.
if int(_arg("--gpus", "1")) > 1 and "WORLD_SIZE" not in os.environ:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    n = _arg("--gpus", "1")
    sys.exit(subprocess.call([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", n,
                              "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)]
                             + sys.argv[1:]))

# Frames in flight run on their own HIP streams; HIP maps streams onto at most
# GPU_MAX_HW_QUEUES hardware queues per process (4 by default on the box),
# which would serialise the 12 streams' kernels in groups of 3.  The runtime
# reads the value when the process starts, so with fewer than needed the bench
# reruns itself as a child process (nothing has touched the GPU yet) and exits
# with the child's status.
HW_QUEUES = min(32, max(16, int(_arg("--concurrency", "16")) + 4))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < HW_QUEUES:
    sys.exit(subprocess.call([sys.executable] + sys.argv, env=dict(os.environ, GPU_MAX_HW_QUEUES=str(HW_QUEUES))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def dwt_bytes(h, w, c, numres=6):
    """B_DWT: sum over levels of 8 B x |R_l| (read + write int32)."""
    tot = 0
    rh, rw = h, w
    for _ in range(numres - 1):
        tot += 8 * rh * rw
        rh, rw = (rh + 1) // 2, (rw + 1) // 2
    return tot * c


def b_e2e(c, prec):
    """HBM bytes read per pixel end to end."""
    return c * (-(-prec // 8) + 4.0 * 4.0 / 3.0 + 4.0)


def max_over_ranks(dist, el):
    """The job's time: the slowest rank's (gloo, host tensor)."""
    if dist is None:
        return el
    t = torch.tensor([el], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def host_threads():
    """The host cores this process may run on: its affinity mask, capped by
    the cgroup's CPU quota where one is set (cgroup v2 cpu.max) -- on a
    shared node the mask lists every core while the quota is the share."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    for qf, pf in (("/sys/fs/cgroup/cpu.max", None),
                   ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "/sys/fs/cgroup/cpu/cpu.cfs_period_us")):
        try:
            if pf is None:
                quota, period = open(qf).read().split()[:2]
            else:
                quota, period = open(qf).read().strip(), open(pf).read().strip()
            if quota not in ("max", "-1"):
                n = min(n, max(1, -(-int(quota) // int(period))))
            break
        except (OSError, ValueError):
            continue
    return n


def cpu_reference(img, bits, args_list, threads, label):
    """Time the reference (oracle/_ref/ref_driver over Grok's libgrok) on the
    host: encode + decode of img for each argument list; returns seconds."""
    drv = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    if not os.path.exists(drv):
        return None
    c, h, w = img.shape
    path = "/tmp/grk_bench_%d.i32" % os.getpid()
    np.ascontiguousarray(img, dtype="<i4").tofile(path)
    tot = 0.0
    try:
        for a in args_list:
            r = subprocess.run([drv, "bench", path, str(w), str(h), str(c), str(bits), "0", str(threads), "1"] + a,
                               capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                return None
            d = json.loads(r.stdout.strip().splitlines()[-1])
            tot += (d["enc_ms"] + d["dec_ms"]) / 1e3
    finally:
        os.unlink(path)
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive (input H2D timed) leg")
    ap.add_argument("--concurrency", type=int, default=16, help="frames in flight per GPU: 1, or an even number (half 9/7, half 5/3)")
    ap.add_argument("--workload", default="8k", choices=["8k", "c5", "c4"])
    ap.add_argument("--opt", default="", help="plan options k=v[,k=v] (grkgpu_dwt_options) for the whole run")
    ap.add_argument("--data", default="smooth", choices=["smooth", "uniform", "const"],
                    help="synthetic input distribution (SURVEY 8(d)): smooth field + 2%% noise (default), uniform "
                         "full-range noise (the T1 worst case: most MQ symbols), constant mid-grey (empty blocks)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # rank -> device as grk_compress -G maps its devices (grk_compress.cpp:423-426):
    # LOCAL_RANK modulo the devices present, so N ranks also run on fewer GPUs
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    if args.gpus != world:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    dist = None
    if world > 1:
        # the ranks never exchange frame data (no collectives on
        # the data path); the timing barrier and the max-over-ranks reduction
        # of one float go over gloo, so no RCCL communicator is created
        import torch.distributed as dist
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    # N ranks on one node share its CPU quota: each rank's host pool (the
    # library's default is half the process's share, host_pool.h) gets half of
    # its 1/N slice, so the ranks' frame threads and pools stay within it
    lw = int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1)
    if lw > 1 and "GRKGPU_HOST_THREADS" not in os.environ:
        os.environ["GRKGPU_HOST_THREADS"] = str(max(1, min(16, host_threads() // lw) // 2))

    import grokimagecompression_amd as grk
    import synth

    if args.opt:  # process-wide plan options for an A/B (entered for the whole run)
        grk.dwt_options(**{k: int(v) for k, v in (kv.split("=", 1) for kv in args.opt.split(","))}).__enter__()

    if args.workload == "c4":
        return bench_c4(args, grk, synth, dist, world, rank, local)

    if args.workload == "c5":
        H, W, C, BITS = 2160, 4096, 3, 12
        img = synth.synth_image(H, W, C, BITS, 5 + rank, args.data)
        pa, _ = grk.CParams.from_cli(["-cinema4K", "24"])
        pb = pa
        tags = ("cin", "cin")
        wl = ("DCI 4K 4096x2160 12-bit RGB frame batch, -cinema4K 24 (9/7, CPRL, 256^2 precincts, 2 POCs, "
              "tile-part per component, PCRD to 1,302,083 B), enc+dec")
    else:
        H, W, C, BITS = 4320, 7680, 3, 12
        img = synth.synth_image(H, W, C, BITS, 3 + rank, args.data)
        pa = grk.CParams.make(irreversible=True)
        pb = grk.CParams.make(irreversible=False)
        tags = ("97", "53")
        wl = "8K 7680x4320 12-bit RGB frame per GPU; 9/7 (-I) + 5/3 lossless, enc+dec; 6 resolutions, 64x64 code-blocks, 1 layer LRCP"
    frame = torch.from_numpy(img).to("cuda:%d" % local)
    # the frame as its file holds it (12-bit samples in 16-bit words), pinned
    host_frame = torch.from_numpy(img.astype(np.uint16)).pin_memory()
    ncodec = max(1, args.concurrency)
    assert ncodec == 1 or ncodec % 2 == 0, "--concurrency must be 1 or even"
    codecs = [grk.Codec(local) for _ in range(ncodec)]
    npairs = max(1, ncodec // 2)
    outs = [(torch.empty_like(frame), torch.empty_like(frame)) for _ in range(npairs)]
    st = {}
    streams = [torch.cuda.Stream(device=local) for _ in range(ncodec)]
    torch.cuda.synchronize()

    # every frame's stage times over the timed steps of the HBM-resident run
    # (stage_ms in the line: their means, so one frame's outlier does not
    # stand for the step)
    acc = {"on": False}

    def pipe(codec, p, out, tag, src):
        with torch.cuda.stream(streams[codecs.index(codec)]):
            b = codec.compress(src, BITS, p, view=True)
            st["enc" + tag] = codec.stats()
            n = len(b)
            codec.decompress(b, out=out)
            st["dec" + tag] = codec.stats()
            st["bytes" + tag] = n
            if acc["on"]:
                acc.setdefault("enc" + tag, []).append(st["enc" + tag])
                acc.setdefault("dec" + tag, []).append(st["dec" + tag])

    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(max_workers=ncodec) if ncodec > 1 else None
    jobs = [(codecs[0], pa, outs[0][0], tags[0]), (codecs[0], pb, outs[0][1], tags[1])] if pool is None else \
        [j for i in range(npairs) for j in ((codecs[2 * i], pa, outs[i][0], tags[0]),
                                            (codecs[2 * i + 1], pb, outs[i][1], tags[1]))]

    def run_steps(n, src):
        """n steps; each frame's pipeline runs its n iterations back to back on
        its own thread/stream (no barrier between steps)."""
        if pool is None:
            for _ in range(n):
                for j in jobs:
                    pipe(*j, src)
        else:
            def loop(j):
                for _ in range(n):
                    pipe(*j, src)
            for x in [pool.submit(loop, j) for j in jobs]:
                x.result()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def timed(n, src):
        barrier()
        t0 = time.perf_counter()
        run_steps(n, src)
        barrier()
        el = time.perf_counter() - t0
        return max_over_ranks(dist, el)

    pix_per_step = 2 * npairs * H * W
    # value: the frames already resident in HBM when the timed region starts
    run_steps(args.warmup, frame)
    if args.workload == "8k":
        assert torch.equal(outs[0][1], frame), "5/3 round trip is not lossless"
    acc["on"] = True
    elapsed = timed(args.steps, frame)
    acc["on"] = False
    value = world * pix_per_step * args.steps / elapsed / 1e6
    ms_per_step = 1e3 * elapsed / args.steps
    nsym_step = npairs * (st["enc" + tags[0]]["mq_symbols"] + st["enc" + tags[1]]["mq_symbols"])
    ncb_step = npairs * (st["enc" + tags[0]]["num_cblks"] + st["enc" + tags[1]]["num_cblks"])

    # SURVEY 8(d)'s end-to-end variant: the same steps with every frame
    # starting in pinned host memory (2 B/sample) and copied H2D inside the
    # timed region
    pcie = None
    if not args.no_pcie:
        psteps = args.steps
        run_steps(1, host_frame)
        if args.workload == "8k":
            assert torch.equal(outs[0][1], frame), "5/3 round trip from the host frame is not lossless"
        el = timed(psteps, host_frame)
        pcie = {"value": round(world * pix_per_step * psteps / el / 1e6, 2), "unit": "Mpixels/s",
                "ms_per_step": round(1e3 * el / psteps, 3), "steps": psteps,
                "h2d_bytes_per_frame": int(img.size * 2),
                "note": "same steps, each frame copied H2D from pinned host memory (uint16, 12-bit samples) "
                        "inside the timed region"}

    # roofline: the 9/7 DWT of the frame, measured alone after the timed
    # region on one context, forward (encode) and inverse (decode).  frac =
    # B_DWT (8 B per sample of every level) over span_us, the
    # device time of the frame's whole level sequence: HIP events on the codec
    # stream right before its first launch and after its last, nothing else
    # between them (mean of 5 encodes / decodes after one warm-up), peak 8
    # TB/s.  The per-launch breakdown comes from 5 more runs with an event
    # after every launch (grkgpu_set_launch_timing; consecutive launches share
    # an event); those events add ~1-5 us per launch, so their sum (dwt_us)
    # stands above both span_us and a rocprofv3 kernel summary of the same
    # launches (scripts/roofline_check.py, profiles/r05*/roofline_check.txt).
    bdwt = dwt_bytes(H, W, C)
    torch.cuda.synchronize()
    p97 = grk.CParams.make(irreversible=True)

    def level_bytes(lvl):
        rh, rw = H, W
        for _ in range(lvl):
            rh, rw = (rh + 1) // 2, (rw + 1) // 2
        return 8 * rh * rw * C

    def launch_table(runs):
        out = []
        for i, l in enumerate(runs[0]):
            ms = sum(r[i]["ms"] for r in runs) / len(runs)
            lv = list(range(l["level0"], l["level0"] + l["levels"]))
            # a launch's floor: its first level's input read and outputs written once
            first = level_bytes(l["level0"])
            out.append({"kernel": l["kernel"], "levels": lv,
                        "us": round(1e3 * ms, 2), "algorithmic_bytes": l["bytes"], "first_level_bytes": first,
                        "GB_s": round(l["bytes"] / (ms * 1e-3) / 1e9, 1),
                        "frac": round(l["bytes"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
        assert sum(x["algorithmic_bytes"] for x in out) == bdwt, "per-launch bytes must add up to B_DWT"
        return out

    def measure(params):
        """Per-launch forward / inverse DWT times of the frame under params:
        (forward launches, inverse launches, forward span us, inverse span us)."""
        spans, fruns, iruns, ispans = [], [], [], []
        with torch.cuda.stream(streams[0]):
            for _ in range(6):
                codecs[0].compress(frame, BITS, params, view=True)
                spans.append(codecs[0].stats()["dwt_ms"])
            cs = bytes(codecs[0].compress(frame, BITS, params, view=True))
            for _ in range(6):
                codecs[0].decompress(cs, out=outs[0][0])
                ispans.append(codecs[0].stats()["dwt_ms"])
            codecs[0].set_launch_timing(True)
            for _ in range(6):
                codecs[0].compress(frame, BITS, params, view=True)
                fruns.append(codecs[0].launch_times())
            for _ in range(6):
                codecs[0].decompress(cs, out=outs[0][0])
                iruns.append(codecs[0].launch_times())
            codecs[0].set_launch_timing(False)
        # the first of each pays one-time setup
        spans, ispans, fruns, iruns = spans[1:], ispans[1:], fruns[1:], iruns[1:]
        return (launch_table(fruns), launch_table(iruns), 1e3 * sum(spans) / len(spans),
                1e3 * sum(ispans) / len(ispans))

    launches, ilaunches, span_us, ispan_us = measure(p97)
    dwt_us = sum(x["us"] for x in launches)
    idwt_us = sum(x["us"] for x in ilaunches)
    achieved = bdwt / (span_us * 1e-6) / 1e9
    traffic = traffic_src = None
    pmc = os.path.join(ROOT, "profiles", "dwt_pmc_latest.json")
    # the PMC passes (scripts/pmc_bench.sh) profile the default 8K workload only
    if args.workload == "8k" and os.path.exists(pmc):
        d = json.load(open(pmc))
        tot = sum(e["bytes"] for k, v in d["kernels"].items()
                  if ("k_dwt_fwd<true" in k or "k_dwt_fwd01<true" in k) for e in v)
        traffic, traffic_src = round(tot), d["source"]
    floor = sum(x["first_level_bytes"] for x in launches)
    roofline = {"bound": "hbm", "kernel": "forward 9/7 DWT of the frame: " + " + ".join(x["kernel"] for x in launches),
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "frac_launch_sum": round(bdwt / (dwt_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_fused_floor": floor,
                "traffic_vs_floor": round(traffic / floor, 4) if traffic else None,
                "algorithmic_bytes": bdwt, "dwt_us": round(dwt_us, 2),
                "span_us": round(span_us, 2), "launches": launches,
                "measured": "frac = B_DWT / span_us (the basis since round 5); frac_launch_sum = B_DWT / dwt_us, the "
                            "sum of the per-launch times (round 4's basis, carrying the extra events' overhead); "
                            "span_us = device time of the frame's forward level sequence (HIP events on the codec "
                            "stream before its first launch and after its last; mean of 5 lone 9/7 encodes after the "
                            "timed region); launches[].us from 5 more encodes with an event after every launch "
                            "(their sum dwt_us carries the extra events' overhead); traffic = PMC bytes (FETCH_SIZE x 2 + "
                            "WRITE_SIZE) of the same launches (profiles/dwt_pmc_latest.json, source %s); "
                            "traffic_fused_floor = 8 B per sample of each launch's first level (its input read and "
                            "its outputs written once)" % traffic_src,
                "inverse": {"kernel": "inverse 9/7 DWT of the frame (decode): " +
                                      " + ".join(x["kernel"] for x in ilaunches),
                            "achieved": round(bdwt / (ispan_us * 1e-6) / 1e9, 1), "unit": "GB/s",
                            "frac": round(bdwt / (ispan_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                            "frac_launch_sum": round(bdwt / (idwt_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                            "algorithmic_bytes": bdwt, "dwt_us": round(idwt_us, 2),
                            "span_us": round(ispan_us, 2), "launches": ilaunches}}
    if args.workload == "8k":
        # the other half of every step: the 5/3 transform of the same frame
        # (forward: DC shift + RCT fused into level 0, then streamed level pairs)
        l53, il53, s53, is53 = measure(pb)
        f53, i53 = sum(x["us"] for x in l53), sum(x["us"] for x in il53)
        roofline["r53"] = {
            "forward": {"kernel": " + ".join(x["kernel"] for x in l53), "dwt_us": round(f53, 2),
                        "achieved": round(bdwt / (s53 * 1e-6) / 1e9, 1), "unit": "GB/s",
                        "frac": round(bdwt / (s53 * 1e-6) / 1e9 / HBM_PEAK_GBS, 4), "span_us": round(s53, 2),
                        "frac_launch_sum": round(bdwt / (f53 * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                        "launches": l53},
            "inverse": {"kernel": " + ".join(x["kernel"] for x in il53), "dwt_us": round(i53, 2),
                        "achieved": round(bdwt / (is53 * 1e-6) / 1e9, 1), "unit": "GB/s",
                        "frac": round(bdwt / (is53 * 1e-6) / 1e9 / HBM_PEAK_GBS, 4), "span_us": round(is53, 2),
                        "frac_launch_sum": round(bdwt / (i53 * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                        "launches": il53},
            "algorithmic_bytes": bdwt}

    # T1 figures: batch throughput + a lone frame's encode / decode T1 kernels
    with torch.cuda.stream(streams[0]):
        b = codecs[0].compress(frame, BITS, pa, view=True)
        se = codecs[0].stats()
        codecs[0].decompress(b, out=outs[0][0])
        sd = codecs[0].stats()
    t1 = {"mq_symbols_per_step": int(nsym_step), "cblks_per_step": int(ncb_step),
          "batch_enc_dec_msym_per_s": round(2 * nsym_step * args.steps * world / elapsed / 1e6, 1),
          "batch_cblks_per_s": round(2 * ncb_step * args.steps * world / elapsed, 1),
          "lone_frame": {"mq_symbols": int(se["mq_symbols"]), "cblks": int(se["num_cblks"]),
                         "enc_t1_ms": round(se["t1_ms"], 3), "dec_t1_ms": round(sd["t1_ms"], 3),
                         "enc_msym_per_s": round(se["mq_symbols"] / (se["t1_ms"] * 1e-3) / 1e6, 1),
                         "dec_msym_per_s": round(se["mq_symbols"] / (sd["t1_ms"] * 1e-3) / 1e6, 1)},
          "note": "symbols = MQ decisions of the encoder (the decoder decodes the same ones)"}
    # the same lone frame's stages (the batch's stage_ms are one call among 16 in flight)
    keys = ("t1_ms", "host_t2_ms", "rate_ms", "packet_ms", "total_ms")
    t1["lone_frame"]["stage_ms"] = {"enc": {k: round(se[k], 3) for k in keys},
                                    "dec": {k: round(sd[k], 3) for k in keys}}
    roof_mpix = HBM_PEAK_GBS * 1e9 / b_e2e(C, BITS) / 1e6
    e2e = {"B_e2e_bytes_per_px": round(b_e2e(C, BITS), 3), "roofline_mpix_per_s": round(roof_mpix, 1),
           "frac": round(value / world / roof_mpix, 5)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the contract: rank 0 at N=1 only
        ncpu = host_threads()
        if args.workload == "c5":
            refargs = [["-cinema4K", "24"]]
            npx = H * W
        else:
            refargs = [["-I"], []]
            npx = 2 * H * W
        ct = cpu_reference(img, BITS, refargs, ncpu, args.workload)
        if ct is not None:
            cpu = {"value": round(npx / ct / 1e6, 3), "unit": "Mpixels/s", "cores": ncpu, "kind": "reference",
                   "sample": "%s through Grok 5.1.0's own libgrok (compiled from /root/reference by "
                             "oracle/ref.mk), %d threads, encode+decode in memory" %
                             ("1 DCI 4K cinema frame" if args.workload == "c5" else
                              "1 step (8K 12-bit RGB frame: 9/7 enc+dec + 5/3 enc+dec)", ncpu),
                   "seconds": round(ct, 2)}
        else:
            import pyoracle
            pyoracle.build()
            t0 = time.perf_counter()
            for irr in (True, False):
                bb = pyoracle.encode(img, BITS, pyoracle.params(irreversible=irr, nthreads=ncpu))
                pyoracle.decode(bb, nthreads=ncpu)
            ct = time.perf_counter() - t0
            cpu = {"value": round(2 * H * W / ct / 1e6, 3), "unit": "Mpixels/s", "cores": ncpu, "kind": "port",
                   "sample": "1 step through the C oracle (oracle/grk_oracle.c), %d threads" % ncpu,
                   "seconds": round(ct, 2)}

    if rank == 0:
        def r(d):
            return {k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items()}

        def mean_stats(k):
            """Stage times of tag k: the mean over every frame of the timed
            steps (counts from the last frame), and the frames averaged."""
            runs = acc.get(k) or [st[k]]
            out = dict(st[k])
            for f in out:
                if f.endswith("_ms"):
                    out[f] = sum(x[f] for x in runs) / len(runs)
            out["frames"] = len(runs)
            return r(out)
        metric = "Mpixels/sec encode+decode, 8K RGB 5/3 lossless & 9/7 lossy" if args.workload == "8k" else \
            "Mpixels/sec encode+decode, DCI 4K cinema frames"
        line = {
            "metric": metric,
            "value": round(value, 2), "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32/f32 (integer encode, f32 9/7 decode)",
            "data": "synthetic (tests/golden/synth.py %s, seed %d+rank)" % (
                {"smooth": "smooth+2% noise", "uniform": "uniform full-range noise", "const": "constant mid-grey"}[args.data],
                5 if args.workload == "c5" else 3),
            "config": {"workload": wl, "input": args.data, "frames_per_step_per_gpu": 2 * npairs, "frames_in_flight": ncodec,
                       "parallelism": "frame-batch x%d (no collectives)" % world},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "pcie_inclusive": pcie,
            "t1": t1,
            "e2e_frac": e2e,
            "codestream_bytes": {tags[0]: st["bytes" + tags[0]], tags[1]: st["bytes" + tags[1]]},
            "stage_ms": {k: mean_stats(k) for k in ("enc" + tags[0], "dec" + tags[0], "enc" + tags[1], "dec" + tags[1])},
        }
        if args.opt:
            line["config"]["plan_options"] = args.opt
        print(json.dumps(line), flush=True)
    for c in codecs:
        c.close()
    if dist is not None:
        dist.destroy_process_group()


def bench_c4(args, grk, synth, dist, world, rank, local):
    """C4: 16384^2 16-bit gray, 1024^2 tiles, 7 resolutions; the 256 tiles are
    split into contiguous ranges over the ranks (grokimagecompression_amd.shard),
    each rank holds ONLY the image rows of its tiles (grkgpu_compress_tile_rows),
    encodes its range to [main header][its tile-parts][EOC] and decodes it back;
    the compressed bytes stay on their rank (shard.compress_sharded gathers them
    over a gloo group for the real output, outside the timed region)."""
    from grokimagecompression_amd import shard
    H = W = 16384
    BITS = 16
    p, _ = grk.CParams.from_cli(["-t", "1024,1024", "-n", "7"])
    ntiles = 256
    b, e = shard.tile_range(ntiles, rank, world)
    r0, r1 = shard.tile_rows(b, e, H, 1024, tw=16)
    slab = synth.synth_plane(H, W, BITS, 4, 0, "smooth", rows=(r0, r1))[None]
    frame = torch.from_numpy(slab).to("cuda:%d" % local)
    del slab
    out = torch.empty((1, H, W), dtype=torch.int32, device="cuda:%d" % local)
    codec = grk.Codec(local)

    def step():
        cs = codec.compress_tiles(frame, BITS, p, b, e, parts=grk.PART_ALL, row0=r0, height=H, view=True)
        codec.decompress_tiles(cs, b, e, out)
        return cs, None

    cs, full = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        cs, _ = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = max_over_ranks(dist, time.perf_counter() - t0)
    if rank == 0:
        print(json.dumps({"metric": "Mpixels/sec encode+decode, 16K tiled, tile shards",
                          "value": round(H * W * args.steps / el / 1e6, 2), "unit": "Mpixels/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 3),
                          "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
                          "dtype": "int32", "data": "synthetic (synth.py smooth, seed 4)",
                          "config": {"workload": "16384^2 16-bit gray, 1024^2 tiles, 7 resolutions, tiles sharded "
                                                 "over ranks, each rank holding only its tile rows",
                                     "parallelism": "tile-shard x%d" % world}}), flush=True)
    codec.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
