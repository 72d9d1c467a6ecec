"""Tile-shard multi-GPU path on the GPU.

* single process: compress_tiles over 2 / 3 contiguous shards, concatenated,
  is byte-identical to the reference codestream; decompress_tiles over the
  shards reproduces the reference decoder's output (host and device planes);
* two processes on cuda:0 (gloo for the gather of tile-part bytes): the full
  C4 config (16384^2 16-bit, 1024^2 tiles) sharded across the ranks, each
  rank generating and uploading ONLY the image rows of its tiles
  (grkgpu_compress_tile_rows), gives the reference codestream hash, and each
  rank's tile-range decode is lossless;
* single process: row-slab encodes of every tiled golden equal the reference.
"""
import hashlib
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

import synth
from conftest import GOLD, load_manifest
from grokimagecompression_amd import shard

pytestmark = pytest.mark.gpu
MAN = load_manifest()
LARGE = load_manifest(large=True)
TILED = [k for k, v in sorted(MAN.items()) if "-t" in v["args"]]


def _img(m):
    h, w, c, bits = m["shape"]
    return synth.synth_image(h, w, c, bits, m["seed"], m["kind"]), bits


@pytest.mark.parametrize("name", TILED)
@pytest.mark.parametrize("world", [2, 3])
def test_shards_concatenate_to_reference(codec, name, world):
    import torch
    import grokimagecompression_amd as grk
    m = MAN[name]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    ref = open(os.path.join(GOLD, name + ".j2k"), "rb").read()
    n = grk.num_tiles(img.shape, bits, p, off)
    assert n > 1
    t = torch.from_numpy(img).cuda()
    chunks = []
    for r in range(world):
        b, e = shard.tile_range(n, r, world)
        parts = grk.PART_TILES | (grk.PART_HEADER if r == 0 else 0) | (grk.PART_EOC if r == world - 1 else 0)
        chunks.append(codec.compress_tiles(t if r % 2 else img, bits, p, b, e, parts, offset=off))
    assert shard.assemble(chunks) == ref
    dref = np.load(os.path.join(GOLD, name + ".dec.npy"))
    host = np.full(img.shape, -7, np.int32)
    dev = torch.full(img.shape, -7, dtype=torch.int32, device="cuda")
    for r in range(world):
        b, e = shard.tile_range(n, r, world)
        codec.decompress_tiles(ref, b, e, host)
        codec.decompress_tiles(ref, b, e, dev)
    assert np.array_equal(host, dref)
    assert np.array_equal(dev.cpu().numpy(), dref)


def test_decompress_tiles_leaves_other_tiles(codec):
    import grokimagecompression_amd as grk
    name = TILED[0]
    m = MAN[name]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    ref = open(os.path.join(GOLD, name + ".j2k"), "rb").read()
    n = grk.num_tiles(img.shape, bits, p, off)
    out = np.full(img.shape, -7, np.int32)
    codec.decompress_tiles(ref, 1, 2, out)
    full = np.load(os.path.join(GOLD, name + ".dec.npy"))
    changed = out != -7
    assert changed.any() and not changed.all()
    assert np.array_equal(out[changed], full[changed])


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import grokimagecompression_amd as grk
    try:
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
        m = LARGE["C4_16k_gray16_tiled"]
        h_, w_, c_, bits = m["shape"]
        p, off = grk.CParams.from_cli(m["args"])
        n = grk.num_tiles((c_, h_, w_), bits, p, off)
        b, e = shard.tile_range(n, rank, world)
        r0, r1 = shard.tile_rows(b, e, h_, 1024, tw=16)
        t = torch.from_numpy(synth.synth_plane(h_, w_, bits, m["seed"], 0, m["kind"], rows=(r0, r1))[None]).cuda()
        codec = grk.Codec(0)
        cs = shard.compress_sharded(codec, t, bits, p, n, dist=dist, offset=off, rows=(r0, r1), height=h_)
        h = hashlib.sha256(cs).hexdigest() if rank == 0 else None
        obj = [cs if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        out = torch.zeros((c_, h_, w_), dtype=torch.int32, device="cuda")
        shard.decompress_sharded(codec, obj[0], out, n, dist=dist)
        ok = bool(torch.equal(out[:, r0:r1], t)) and (e - b) % 16 == 0
        codec.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, h, ok, None))
    except Exception as ex:  # surface the failure to the parent
        q.put((rank, None, False, repr(ex)))


def test_two_ranks_sharded_16k():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = {}
    for _ in procs:
        r, h, ok, err = q.get(timeout=110)
        res[r] = (h, ok, err)
    for pr in procs:
        pr.join(30)
    assert all(v[2] is None for v in res.values()), res
    assert res[0][0] == LARGE["C4_16k_gray16_tiled"]["j2k_sha256"]
    assert res[0][1] and res[1][1]


@pytest.mark.parametrize("name", TILED)
def test_row_slab_shards_match_reference(codec, name):
    """Each shard encoded from only the rows of its tiles
    (grkgpu_compress_tile_rows) -- concatenated: the reference codestream."""
    import grokimagecompression_amd as grk
    m = MAN[name]
    img, bits = _img(m)
    p, off = grk.CParams.from_cli(m["args"])
    ref = open(os.path.join(GOLD, name + ".j2k"), "rb").read()
    n = grk.num_tiles(img.shape, bits, p, off)
    tdx, tdy = p.cp_tdx, p.cp_tdy
    tx0, ty0 = p.cp_tx0, p.cp_ty0
    tw = -(-(off[0] + img.shape[2] - tx0) // tdx)
    chunks = []
    world = 3
    for r in range(world):
        b, e = shard.tile_range(n, r, world)
        r0, r1 = shard.tile_rows(b, e, img.shape[1], tdy, ty0=ty0, y0=off[1], tw=tw)
        parts = grk.PART_TILES | (grk.PART_HEADER if r == 0 else 0) | (grk.PART_EOC if r == world - 1 else 0)
        chunks.append(codec.compress_tiles(np.ascontiguousarray(img[:, r0:r1]), bits, p, b, e, parts, offset=off,
                                           row0=r0, height=img.shape[1]))
    assert shard.assemble(chunks) == ref
    # rows that miss a tile of the range are refused
    with pytest.raises(grk.GrkGpuError):
        codec.compress_tiles(np.ascontiguousarray(img[:, 1:3]), bits, p, 0, 1, grk.PART_ALL, offset=off, row0=1,
                             height=img.shape[1])


def test_compress_tiles_view():
    """compress_tiles(view=True): the same bytes as a numpy view over the
    context's pinned output buffer (no copy), usable as decompress_tiles
    input; a slice of the view keeps the Codec -- and so the buffer -- alive
    after every other reference to them is gone."""
    import gc
    import torch
    import grokimagecompression_amd as grk
    codec = grk.Codec(0)
    img = synth.synth_image(300, 500, 1, 12, 9)
    p, _ = grk.CParams.from_cli(["-t", "128,128"])
    ref = codec.compress_tiles(img, 12, p, 0, 12, grk.PART_ALL)
    v = codec.compress_tiles(img, 12, p, 0, 12, grk.PART_ALL, view=True)
    assert isinstance(v, np.ndarray) and v.dtype == np.uint8 and v.tobytes() == ref
    out = torch.zeros((1, 300, 500), dtype=torch.int32, device="cuda:0")
    codec.decompress_tiles(v, 0, 12, out)
    assert np.array_equal(out.cpu().numpy(), img.astype(np.int32))
    head, tail = v[:64], np.asarray(v[-2:])
    del v, codec
    gc.collect()
    junk = [np.ones(1 << 20, np.uint8) for _ in range(8)]  # churn the host allocator
    del junk
    gc.collect()
    assert head.tobytes() == ref[:64] and tail.tobytes() == ref[-2:]


def test_view_outlives_later_compress():
    """A view stays valid across later compress calls on its Codec, including
    a larger one that needs a bigger output buffer (the view took the buffer
    out of the context: grkgpu_take_output); views dropped before the next
    call hand their buffer back (grkgpu_give_output)."""
    import gc
    import grokimagecompression_amd as grk
    codec = grk.Codec(0)
    small = synth.synth_image(64, 80, 1, 8, 1)
    big = synth.synth_image(600, 700, 3, 12, 2)
    ref_small = codec.compress(small, 8)
    v1 = codec.compress(small, 8, view=True)
    v2 = codec.compress(small, 8, view=True)  # v1 still alive: a new buffer
    ref_big = codec.compress(big, 12)
    v3 = codec.compress(big, 12, view=True)
    junk = [np.ones(1 << 20, np.uint8) for _ in range(8)]
    del junk
    assert v1.tobytes() == ref_small and v2.tobytes() == ref_small and v3.tobytes() == ref_big
    sl = v1[10:20]
    del v1, v2
    gc.collect()
    for _ in range(3):  # views dropped between calls: the buffer goes round
        w = codec.compress(big, 12, view=True)
        assert w.tobytes() == ref_big
        del w
    assert sl.tobytes() == ref_small[10:20] and v3.tobytes() == ref_big
    codec.close()  # a view outliving its Codec frees its buffer itself
    assert v3.tobytes() == ref_big
    del v3, sl
    gc.collect()


def test_views_held_across_compresses_reuse_spares():
    """A caller keeping a rolling window of live views: every buffer given back
    while the context already has one becomes a spare that a later compress
    reuses (no fresh pinned buffer per call) -- every view keeps its
    own bytes throughout."""
    import gc
    import grokimagecompression_amd as grk
    codec = grk.Codec(0)
    imgs = [synth.synth_image(64 + 40 * k, 80 + 30 * k, 3, 12, 10 + k) for k in range(3)]
    refs = [codec.compress(im, 12) for im in imgs]
    live = []
    for it in range(12):
        k = it % 3
        live.append((k, codec.compress(imgs[k], 12, view=True)))
        if len(live) > 3:
            live.pop(0)
            gc.collect()
        for kk, v in live:
            assert v.tobytes() == refs[kk], (it, kk)
    del live
    gc.collect()
    assert codec.compress(imgs[2], 12, view=True).tobytes() == refs[2]
    codec.close()
