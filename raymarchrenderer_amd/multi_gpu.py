"""Tile-partitioned multi-GPU rendering: one process per GPU, one RCCL reduce per frame.

SURVEY §8e: every rank renders an interleaved subset of the frame's tiles into its own full-frame
RGBA32F accumulator that is zero outside those tiles, then a single reduce(SUM) over xGMI onto
rank 0 assembles the image. x + 0 = x, so the reduced image is bitwise the single-GPU image.
Tiles are dealt round-robin in raster order, so every rank gets a spread of cheap (sky) and
expensive (floor, walls) tiles.
"""
import numpy as np


def frame_tiles(W, H, tile):
    return [(tx, ty) for ty in range((H + tile - 1) // tile) for tx in range((W + tile - 1) // tile)]


def tile_partition(W, H, tile, rank, world):
    """Tiles (tx, ty) owned by `rank` of `world`."""
    t = frame_tiles(W, H, tile)
    return np.array(t[rank::world], np.int32).reshape(-1, 2)


def reduce_frame(accum, dist, group=None):
    """Sum every rank's accumulator onto rank 0 (one collective per frame)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.reduce(accum, dst=0, op=dist.ReduceOp.SUM, group=group)
    return accum


class FrameRenderer:
    """One rank's share of a frame: `renderer` renders into `accum` (a torch CUDA tensor of
    H x W x 4 float32 bound with rmr_bind_accum), then the reduce."""

    def __init__(self, renderer, accum, W, H, tile, rank, world, dist=None):
        self.r, self.acc, self.dist = renderer, accum, dist
        self.tiles = tile_partition(W, H, tile, rank, world)
        self.tile = tile
        renderer.bind_accum(accum.data_ptr(), accum.numel() * accum.element_size())

    def frame(self, times, first_sample=0):
        self.acc.zero_()
        if len(self.tiles):
            self.r.render_tiles(times, self.tiles, self.tile, first_sample=first_sample)
        return reduce_frame(self.acc, self.dist)
