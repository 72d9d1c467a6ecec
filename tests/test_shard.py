"""Tile-shard orchestration (grokimagecompression_amd.shard), CPU side.

* tile_range partitions every tile exactly once, in order, for any world size;
* the codestream format the sharding relies on -- [main header][tile-parts in
  tile order][EOC] -- holds for the reference's own multi-tile golden
  codestreams (split at SOT/Psot, then reassembled);
* tile_rows gives exactly the rows of a tile range (each rank loads only
  those);
* world_size-2 gloo run of compress_sharded / decompress_sharded with a
  stand-in tile coder (the GPU coder is exercised by tests/test_gpu_shard.py),
  including a job whose default group reports NCCL: the tile-part bytes must
  then travel over the separate gloo data group, never the default group.
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


@pytest.mark.parametrize("h,tdy,ty0,y0,tw", [(150, 48, 1, 3, 4), (16384, 1024, 0, 0, 16), (100, 100, 0, 0, 1),
                                              (77, 10, 5, 9, 3)])
def test_tile_rows_cover_exactly(h, tdy, ty0, y0, tw):
    th = -(-(y0 + h - ty0) // tdy)
    ntiles = th * tw
    for world in (1, 2, 3, 5):
        for r in range(world):
            b, e = shard.tile_range(ntiles, r, world)
            r0, r1 = shard.tile_rows(b, e, h, tdy, ty0, y0, tw)
            if b == e:
                continue
            want = set()
            for t in range(b, e):
                q = t // tw
                lo, hi = max(y0, ty0 + q * tdy), min(y0 + h, ty0 + (q + 1) * tdy)
                want.update(range(lo - y0, hi - y0))
            assert (r0, r1) == (min(want), max(want) + 1)


class FakeCoder:
    """Stand-in tile coder: tile t -> b'T<t>;', header b'H', EOC b'E'."""

    def __init__(self):
        self.decoded = []

    def compress_tiles(self, img, prec, params, b, e, parts, offset=(0, 0), sgnd=False, row0=None, height=None):
        return (b"H" if parts & 1 else b"") + b"".join(b"T%d;" % t for t in range(b, e)) + (b"E" if parts & 2 else b"")

    def decompress_tiles(self, buf, b, e, out):
        out.extend(range(b, e))


class NcclDefault:
    """torch.distributed as a job whose default group is NCCL sees it: the
    default group's backend reads "nccl" and a collective on the default
    group fails; everything else is the real (gloo) module."""

    def __init__(self, dist):
        self._d = dist

    def __getattr__(self, k):
        return getattr(self._d, k)

    def get_backend(self, group=None):
        return "nccl" if group is None else self._d.get_backend(group)

    def gather_object(self, obj, lst, dst=0, group=None):
        assert group is not None, "compressed bytes gathered over the default (NCCL) group"
        assert self._d.get_backend(group) == "gloo"
        return self._d.gather_object(obj, lst, dst=dst, group=group)


def _worker(rank, world, port, ntiles, q, nccl_default=False):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    d = NcclDefault(dist) if nccl_default else dist
    cs = shard.compress_sharded(FakeCoder(), None, 8, None, ntiles, dist=d)
    dec = []
    shard.decompress_sharded(FakeCoder(), b"", dec, ntiles, dist=dist)
    q.put((rank, cs, dec))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("nccl_default", [False, True])
@pytest.mark.parametrize("ntiles", [5, 256])
def test_gloo_world2_sharded(ntiles, nccl_default):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000) + (7 if nccl_default else 0) + ntiles % 3
    procs = [ctx.Process(target=_worker, args=(r, 2, port, ntiles, q, nccl_default)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (cs, dec)) for r, cs, dec in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    expect = b"H" + b"".join(b"T%d;" % t for t in range(ntiles)) + b"E"
    assert res[0][0] == expect and res[1][0] is None
    assert sorted(res[0][1] + res[1][1]) == list(range(ntiles))


def _subgroup_worker(rank, world, port, ntiles, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    g = dist.new_group(ranks=[1, 2], backend="gloo")  # collective: every rank creates it
    cs, dec = None, []
    if rank in (1, 2):
        cs = shard.compress_sharded(FakeCoder(), None, 8, None, ntiles, dist=dist, group=g)
        shard.decompress_sharded(FakeCoder(), b"", dec, ntiles, dist=dist, group=g)
    q.put((rank, cs, dec))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_subgroup_sharded():
    """A shard group that is a subset of the job (global ranks 1 and 2 of 3):
    tiles are split by the rank within the group, and the tile-parts are
    gathered at the group's first member (global rank 1), not at rank 0."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + (os.getpid() % 1000)
    ntiles = 7
    procs = [ctx.Process(target=_subgroup_worker, args=(r, 3, port, ntiles, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict((r, (cs, dec)) for r, cs, dec in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    expect = b"H" + b"".join(b"T%d;" % t for t in range(ntiles)) + b"E"
    assert res[1][0] == expect and res[2][0] is None and res[0] == (None, [])
    assert sorted(res[1][1] + res[2][1]) == list(range(ntiles))


def _zero_tlm(cs):
    """The golden with its TLM records zeroed (what rank 0's header holds)."""
    pos = 2
    while True:
        m, L = struct.unpack(">HH", cs[pos:pos + 4])
        if m == 0xFF55:
            return cs[:pos + 6] + bytes(L - 4) + cs[pos + 2 + L:]
        pos += 2 + L


class SliceCoder:
    """Stand-in coder over a golden codestream: rank payloads are its main
    header (TLM records zeroed, as the encoder writes them before the
    tile-parts exist) and a share of its tile-parts."""

    def __init__(self, cs):
        self.head, self.parts, self.eoc = split_codestream(_zero_tlm(cs))

    def compress_tiles(self, img, prec, params, b, e, parts, offset=(0, 0), sgnd=False, row0=None, height=None):
        return (self.head if parts & 1 else b"") + b"".join(self.parts[b:e]) + (self.eoc if parts & 2 else b"")


def _tlm_worker(rank, world, port, name, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    cs = open(os.path.join(GOLD, name + ".j2k"), "rb").read()
    coder = SliceCoder(cs)
    out = shard.compress_sharded(coder, None, 12, None, len(coder.parts), dist=dist)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["rgb12_cinema2k", "rgb12_cinema4k"])
def test_gloo_world2_sharded_tlm(name):
    """A sharded encode of a TLM-bearing stream (the cinema profiles, one
    tile-part per component): rank 0's main header carries TLM records it
    cannot know, the gather patches them from the gathered tile-parts
    (shard.patch_tlm, j2k_write_updated_tlm) -- the assembled codestream is
    the reference's byte for byte."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33500 + (os.getpid() % 1000) + len(name) % 7
    procs = [ctx.Process(target=_tlm_worker, args=(r, 2, port, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    cs = open(os.path.join(GOLD, name + ".j2k"), "rb").read()
    assert _zero_tlm(cs) != cs
    assert res[0] == cs and res[1] is None
    assert shard.patch_tlm(b"H" + b"T0;") == b"H" + b"T0;"


def _split_tlm(cs, first):
    """The golden with its one TLM marker split in two (the first `first`
    records, then the rest), records zeroed: a main header with several TLM
    markers (Ztlm 0, 1), as j2k_read_tlm accepts them."""
    pos = 2
    while True:
        m, L = struct.unpack(">HH", cs[pos:pos + 4])
        if m == 0xFF55:
            stlm = cs[pos + 5]
            rec = ((stlm >> 4) & 3) + (4 if (stlm >> 6) & 1 else 2)
            n = (L - 4) // rec
            a = b"\xff\x55" + struct.pack(">H", 4 + first * rec) + bytes([0, stlm]) + bytes(first * rec)
            b = b"\xff\x55" + struct.pack(">H", 4 + (n - first) * rec) + bytes([1, stlm]) + bytes((n - first) * rec)
            return cs[:pos] + a + b + cs[pos + 2 + L:], n
        pos += 2 + L


@pytest.mark.parametrize("name", ["rgb12_cinema2k", "rgb12_cinema4k"])
def test_patch_tlm_several_markers_and_mismatch(name):
    """grkgpu_patch_tlm: records are filled across every TLM
    marker of the main header in order; a TLM whose record count does not
    match the tile-parts raises instead of shipping a stale TLM."""
    from grokimagecompression_amd import GrkGpuError
    cs = open(os.path.join(GOLD, name + ".j2k"), "rb").read()
    split, n = _split_tlm(cs, 1)
    assert n >= 3  # one tile-part per component (and per POC for 4K)
    patched = shard.patch_tlm(split)
    # the same records as the golden's, now in two markers
    again, _ = _split_tlm(cs, 1)
    assert patched != again
    rec = 5
    pos = 2
    got = b""
    while True:
        m, L = struct.unpack(">HH", patched[pos:pos + 4])
        if m == 0xFF90:
            break
        if m == 0xFF55:
            got += patched[pos + 6:pos + 2 + L]
        pos += 2 + L
    ref = _zero_tlm(cs)
    p2 = 2
    while True:
        m, L = struct.unpack(">HH", cs[p2:p2 + 4])
        if m == 0xFF55:
            assert got == cs[p2 + 6:p2 + 2 + L] and len(got) == n * rec
            break
        p2 += 2 + L
    assert ref != cs
    # one record too few: refused
    bad = split.replace(b"\xff\x55" + struct.pack(">H", 4 + (n - 1) * rec) + bytes([1, 0x50]) + bytes((n - 1) * rec),
                        b"\xff\x55" + struct.pack(">H", 4 + (n - 2) * rec) + bytes([1, 0x50]) + bytes((n - 2) * rec))
    assert bad != split
    with pytest.raises(GrkGpuError):
        shard.patch_tlm(bad)
