"""Tile-shard orchestration (grokimagecompression_amd.shard), CPU side.

* tile_range partitions every tile exactly once, in order, for any world size;
* the codestream format the sharding relies on -- [main header][tile-parts in
  tile order][EOC] -- holds for the reference's own multi-tile golden
  codestreams (split at SOT/Psot, then reassembled);
* world_size-2 gloo run of compress_sharded / decompress_sharded with a
  stand-in tile coder (the GPU coder is exercised by tests/test_gpu_shard.py).
"""
import os
import struct

import pytest
import torch.multiprocessing as mp

from conftest import GOLD, load_manifest
from grokimagecompression_amd import shard

MAN = load_manifest()


@pytest.mark.parametrize("ntiles", [1, 2, 7, 256, 1000])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_tile_range_partition(ntiles, world):
    seen = []
    for r in range(world):
        b, e = shard.tile_range(ntiles, r, world)
        assert 0 <= b <= e <= ntiles
        seen.extend(range(b, e))
    assert seen == list(range(ntiles))
    sizes = [shard.tile_range(ntiles, r, world)[1] - shard.tile_range(ntiles, r, world)[0] for r in range(world)]
    assert max(sizes) - min(sizes) <= 1


def split_codestream(cs):
    """(main header, [tile-part bytes], eoc) by walking SOT markers (Psot)."""
    pos = cs.index(b"\xff\x90")
    head, parts = cs[:pos], []
    while cs[pos:pos + 2] == b"\xff\x90":
        psot = struct.unpack(">I", cs[pos + 6:pos + 10])[0]
        parts.append(cs[pos:pos + psot])
        pos += psot
    assert cs[pos:] == b"\xff\xd9"
    return head, parts, cs[pos:]


@pytest.mark.parametrize("name", [k for k, v in sorted(MAN.items()) if "-t" in v["args"]])
def test_reference_codestream_is_header_tileparts_eoc(name):
    cs = open(os.path.join(GOLD, name + ".j2k"), "rb").read()
    head, parts, eoc = split_codestream(cs)
    assert len(parts) > 1
    idx = [struct.unpack(">H", p[4:6])[0] for p in parts]
    assert idx == sorted(idx)
    for world in (2, 3):
        chunks = []
        for r in range(world):
            b, e = shard.tile_range(len(parts), r, world)
            chunks.append((head if r == 0 else b"") + b"".join(parts[b:e]) + (eoc if r == world - 1 else b""))
        assert shard.assemble(chunks) == cs


class FakeCoder:
    """Stand-in tile coder: tile t -> b'T<t>;', header b'H', EOC b'E'."""

    def __init__(self):
        self.decoded = []

    def compress_tiles(self, img, prec, params, b, e, parts, offset=(0, 0), sgnd=False):
        return (b"H" if parts & 1 else b"") + b"".join(b"T%d;" % t for t in range(b, e)) + (b"E" if parts & 2 else b"")

    def decompress_tiles(self, buf, b, e, out):
        out.extend(range(b, e))


def _worker(rank, world, port, ntiles, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    cs = shard.compress_sharded(FakeCoder(), None, 8, None, ntiles, dist=dist)
    dec = []
    shard.decompress_sharded(FakeCoder(), b"", dec, ntiles, dist=dist)
    q.put((rank, cs, dec))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ntiles", [5, 256])
def test_gloo_world2_sharded(ntiles):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, ntiles, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (cs, dec)) for r, cs, dec in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    expect = b"H" + b"".join(b"T%d;" % t for t in range(ntiles)) + b"E"
    assert res[0][0] == expect and res[1][0] is None
    assert sorted(res[0][1] + res[1][1]) == list(range(ntiles))
