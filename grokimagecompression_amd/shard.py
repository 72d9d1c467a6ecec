"""Tile-shard multi-GPU encode / decode.

Tiles are independent through DC shift, MCT, DWT, T1 and T2, and a
codestream is [main header][tile-parts in tile index order][EOC]
(j2k.cpp:2088-2111, 2376-2435).  So with one process per GPU, rank r encodes
a contiguous tile range and the tile-part bytes travel to rank 0, which
concatenates them: no collective on the data path beyond that gather of
compressed bytes (no RCCL reduction, no halo exchange).  Decode: every rank
holds the codestream and decodes its own tile range.

The encoder/decoder object only needs compress_tiles / decompress_tiles
(grokimagecompression_amd.Codec); the group is any torch.distributed group
(nccl on the GPU box, gloo in the CPU tests).
"""
from . import PART_EOC, PART_HEADER, PART_TILES


def tile_range(ntiles, rank, world):
    """Contiguous, balanced [begin, end) tile range of `rank` (first ranks take
    the remainder)."""
    base, extra = divmod(ntiles, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def assemble(parts):
    """Concatenate per-rank payloads (rank 0 carries the main header, the last
    rank the EOC) in rank order = tile order."""
    return b"".join(parts)


def compress_sharded(codec, img, prec, params, ntiles, dist=None, group=None, offset=(0, 0), sgnd=False):
    """Encode this rank's tile range; returns the full codestream on rank 0
    (None elsewhere).  Without torch.distributed (dist=None) it is the
    single-process path."""
    world = dist.get_world_size(group) if dist is not None else 1
    rank = dist.get_rank(group) if dist is not None else 0
    b, e = tile_range(ntiles, rank, world)
    parts = PART_TILES | (PART_HEADER if rank == 0 else 0) | (PART_EOC if rank == world - 1 else 0)
    mine = codec.compress_tiles(img, prec, params, b, e, parts, offset=offset, sgnd=sgnd)
    if dist is None:
        return mine
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(mine, gathered, dst=0, group=group)
    return assemble(gathered) if rank == 0 else None


def decompress_sharded(codec, buf, out, ntiles, dist=None, group=None):
    """Decode this rank's tile range of `buf` into `out` (other tiles are left
    untouched); returns the (begin, end) range decoded."""
    world = dist.get_world_size(group) if dist is not None else 1
    rank = dist.get_rank(group) if dist is not None else 0
    b, e = tile_range(ntiles, rank, world)
    codec.decompress_tiles(buf, b, e, out)
    return b, e
