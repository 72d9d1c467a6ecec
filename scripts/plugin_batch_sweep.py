"""Throughput of the plugin's batch route (grk_compress's image-directory
mode over libgrok_plugin.so: oracle/_ref/ref_driver plugin-batch) on DCI 4K
cinema frames (BASELINE configs[4], -cinema4K 24) for several frames-in-flight
settings (GRKGPU_PLUGIN_FRAMES).  Wall time of the whole batch, PPM reads and
codestream writes included (the reference host's own per-frame work).
  python scripts/plugin_batch_sweep.py NFRAMES FRAMES1 FRAMES2 ..."""
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden")]

import numpy as np  # noqa: E402

import synth  # noqa: E402

DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
PLUGIN_DIR = os.path.join(ROOT, "grokimagecompression_amd", "lib")


def main():
    n = int(sys.argv[1])
    settings = sys.argv[2:]
    h, w, c, bits = 2160, 4096, 3, 12
    with tempfile.TemporaryDirectory() as tmp:
        ind = os.path.join(tmp, "in")
        os.mkdir(ind)
        for k in range(n):
            img = synth.synth_image(h, w, c, bits, 300 + k, "smooth")
            hdr = b"P6\n%d %d\n%d\n" % (w, h, (1 << bits) - 1)
            data = np.ascontiguousarray(np.moveaxis(img, 0, -1)).astype(">u2")
            with open(os.path.join(ind, "f%03d.ppm" % k), "wb") as f:
                f.write(hdr + data.tobytes())
        for rep in range(2):
            for fr in settings:
                outd = os.path.join(tmp, "out_%s_%d" % (fr, rep))
                os.mkdir(outd)
                env = dict(os.environ, GRKGPU_PLUGIN_FRAMES=fr)
                t0 = time.perf_counter()
                r = subprocess.run([DRIVER, "plugin-batch", PLUGIN_DIR, ind, outd, "-cinema4K", "24"],
                                   capture_output=True, text=True, timeout=600, env=env)
                el = time.perf_counter() - t0
                ok = r.returncode == 0 and ("written=%d failed=0" % n) in r.stdout
                print("frames_in_flight %s rep %d: %d frames in %.2f s = %.1f Mpixels/s %s" % (
                    fr, rep, n, el, n * h * w / el / 1e6, "ok" if ok else "FAILED " + r.stdout[-300:] + r.stderr[-300:]),
                    flush=True)
                if not ok:
                    sys.exit(1)


if __name__ == "__main__":
    main()
