"""Tile-shard multi-GPU encode / decode.

Tiles are independent through DC shift, MCT, DWT, T1 and T2, and a
codestream is [main header][tile-parts in tile index order][EOC]
(j2k.cpp:2088-2111, 2376-2435).  So with one process per GPU, rank r encodes
a contiguous tile range from just the image rows those tiles cover, and the
tile-part bytes travel to rank 0, which concatenates them.  That gather of
compressed bytes is the only exchange, and it runs on the HOST over a gloo
group (data_group) even when the job's default group is NCCL (RCCL): no
collective touches the GPU data path (north_star: "no RCCL collectives").
Decode: every rank holds the codestream and decodes its own tile range.

The encoder/decoder object only needs compress_tiles / decompress_tiles
(grokimagecompression_amd.Codec).
"""
from . import PART_EOC, PART_HEADER, PART_TILES

_DATA_GROUPS = {}


def data_group(dist):
    """The gloo group the compressed bytes travel over (created once per
    process, collectively, on first use; the default group when that is
    already gloo)."""
    if dist.get_backend() == "gloo":
        return None
    if "gloo" not in _DATA_GROUPS:
        _DATA_GROUPS["gloo"] = dist.new_group(backend="gloo")
    return _DATA_GROUPS["gloo"]


def tile_range(ntiles, rank, world):
    """Contiguous, balanced [begin, end) tile range of `rank` (first ranks take
    the remainder)."""
    base, extra = divmod(ntiles, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def tile_rows(begin, end, image_h, tdy, ty0=0, y0=0, tw=1):
    """Image rows [r0, r1) (relative to the image origin y0) covered by tiles
    [begin, end) of a grid tw tiles wide with tile height tdy and origin ty0
    (j2k tile geometry: tile row q spans [ty0 + q*tdy, ty0 + (q+1)*tdy) clipped
    to the image)."""
    if end <= begin:
        return 0, 0
    q0, q1 = begin // tw, (end - 1) // tw
    r0 = max(y0, ty0 + q0 * tdy) - y0
    r1 = min(y0 + image_h, ty0 + (q1 + 1) * tdy) - y0
    return r0, r1


def patch_tlm(cs):
    """j2k_write_updated_tlm (j2k.cpp:2555-2577) over an assembled codestream
    (grkgpu_patch_tlm, host code of libgrk_mi355x): the main header's TLM
    records (tile index Ttlm, tile-part length Ptlm, one per tile-part in
    codestream order, filled across all of its TLM markers in order; widths
    from Stlm, j2k.cpp:5027-5063) from the tile-parts' own SOT headers.  Each
    rank of a sharded encode wrote only its own tile-parts, so rank 0's
    header could not.  A stream without TLM (or no codestream at all) comes
    back as it is; TLM records that do not match the tile-parts one to one
    raise GrkGpuError -- never a silently stale TLM."""
    import ctypes
    from . import lib, _check
    if cs[:2] != b"\xff\x4f":
        return cs
    buf = ctypes.create_string_buffer(bytes(cs), len(cs))
    _check(lib().grkgpu_patch_tlm(buf, len(cs)))
    return buf.raw[:len(cs)]


def assemble(parts):
    """Concatenate per-rank payloads (rank 0 carries the main header, the last
    rank the EOC) in rank order = tile order, then fill in the TLM records
    (patch_tlm) that no single rank could write."""
    return patch_tlm(b"".join(parts))


def _group_geom(dist, group):
    """(gather group, rank in it, its size, the global rank of its member 0).
    Tile ranges follow the rank WITHIN the group, so a subset or reordered
    group still splits the tiles among its members and gathers at its own
    first member."""
    if dist is None:
        return None, 0, 1, 0
    g = group if group is not None else data_group(dist)
    rank, world = dist.get_rank(g), dist.get_world_size(g)
    if rank < 0:
        raise ValueError("this process is not a member of the shard group")
    root = dist.get_global_rank(g, 0) if g is not None else 0
    return g, rank, world, root


def compress_sharded(codec, img, prec, params, ntiles, dist=None, group=None, offset=(0, 0), sgnd=False,
                     rows=None, height=None):
    """Encode this rank's tile range; returns the full codestream on the
    group's first member (None elsewhere).  Without torch.distributed
    (dist=None) it is the single-process path.

    img: the whole image, or (rows given) only this rank's rows: rows = (r0, r1)
    of an image `height` rows tall, img holding rows [r0, r1)
    (see tile_rows).  group: the group that shares the tiles and gathers the
    tile-parts (default: data_group, i.e. every rank); only its members call."""
    g, rank, world, root = _group_geom(dist, group)
    b, e = tile_range(ntiles, rank, world)
    parts = PART_TILES | (PART_HEADER if rank == 0 else 0) | (PART_EOC if rank == world - 1 else 0)
    if rows is None:
        mine = codec.compress_tiles(img, prec, params, b, e, parts, offset=offset, sgnd=sgnd)
    else:
        mine = codec.compress_tiles(img, prec, params, b, e, parts, offset=offset, sgnd=sgnd, row0=rows[0],
                                    height=height)
    if dist is None:
        return mine
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(mine, gathered, dst=root, group=g)
    return assemble(gathered) if rank == 0 else None


def shard_range(ntiles, dist=None, group=None):
    """The [begin, end) tile range this process takes in compress_sharded /
    decompress_sharded (by its rank within `group`)."""
    _, rank, world, _ = _group_geom(dist, group)
    return tile_range(ntiles, rank, world)


def decompress_sharded(codec, buf, out, ntiles, dist=None, group=None):
    """Decode this rank's tile range of `buf` into `out` (other tiles are left
    untouched); returns the (begin, end) range decoded."""
    b, e = shard_range(ntiles, dist, group)
    codec.decompress_tiles(buf, b, e, out)
    return b, e
