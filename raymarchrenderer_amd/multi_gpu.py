"""Tile-partitioned multi-GPU rendering: one process per GPU, one RCCL reduce per frame.

SURVEY §8e: every rank renders an interleaved subset of the frame's tiles into its own full-frame
RGBA32F accumulator that is zero outside those tiles, then a single reduce(SUM) over xGMI onto
rank 0 assembles the image. x + 0 = x, so the reduced image is bitwise the single-GPU image.
Tiles are dealt round-robin in raster order, so every rank gets a spread of cheap (sky) and
expensive (floor, walls) tiles.

Frames are pipelined over two accumulators: frame f's reduce runs (async, on the collective's own
stream) while frame f + 1 renders into the other buffer; a buffer is reused only after its reduce
completed. The reduce of every frame is still one collective over the whole frame.

With two renderer contexts on two HIP streams (`renderer=[r0, r1]`, `streams=[s0, s1]`) consecutive
frames also overlap on the GPU: the persistent trace kernel of frame f ends with a drain (its last,
longest paths run on a nearly idle chip, ~1.4 ms on C2), which frame f + 1's kernel, launched on the
other stream, fills. Each frame's zeroing, render and reduce stay ordered on its own stream.
A persistent trace kernel keeps every workgroup slot it gets until its queue runs out, so frame f's
fold (a small kernel after its trace) would wait for frame f + 1's drain and hold up frame f + 2
behind it; with two contexts each trace launch leaves OVERLAP_GRID_RESERVE workgroups free
(rmr_set_grid_reserve) for the other context's fold and zeroing (C4 +1.7%, RM2 +3%, the 8-rank C2
rank share +1.8%, the rest within noise: profiles/r05_grid_reserve_ab.log).
"""
import contextlib

import numpy as np

OVERLAP_GRID_RESERVE = 64   # workgroups (of 1536-1792 on the C2 / C4 kernels)


def frame_tiles(W, H, tile):
    return [(tx, ty) for ty in range((H + tile - 1) // tile) for tx in range((W + tile - 1) // tile)]


def tile_partition(W, H, tile, rank, world):
    """Tiles (tx, ty) owned by `rank` of `world`."""
    t = frame_tiles(W, H, tile)
    return np.array(t[rank::world], np.int32).reshape(-1, 2)


def tile_costs(renderer, tiles, tile, times):
    """Each tile's map() evaluations (the kernel's counter) over the samples `times`, one small launch
    per tile: a cost map for ordering a frame's tiles. Writes the renderer's accumulator (the caller
    zeroes it before the next frame)."""
    cost = np.zeros(len(tiles), np.int64)
    for i, t in enumerate(np.asarray(tiles, np.int32).reshape(-1, 2)):
        renderer.reset_stats()
        renderer.render_tiles(times, t.reshape(1, 2), tile)
        cost[i] = renderer.stats().map_evals
    return cost


def frame_tile_costs(renderer, W, H, tile, times):
    """tile_costs over every tile of the frame, as {(tx, ty): map evals}: one probe that every rank
    share of a partition can slice (FrameRenderer.order_tiles_by_cost cost_map) instead of probing its
    tiles again for each rank count. Writes the renderer's accumulator."""
    tiles = frame_tiles(W, H, tile)
    cost = tile_costs(renderer, tiles, tile, times)
    return {t: int(c) for t, c in zip(tiles, cost)}


def _multi(dist, group=None, always=False):
    return dist is not None and dist.is_initialized() and (always or dist.get_world_size(group) > 1)


def reduce_frame(accum, dist, group=None, async_op=False, always=False):
    """Sum every rank's accumulator onto rank 0 (one collective per frame). With async_op the
    collective's work handle is returned (None without a collective). always: issue the collective at
    world size 1 too (an identity there; tests run the RCCL path on a one-GPU box with it)."""
    if _multi(dist, group, always):
        w = dist.reduce(accum, dst=0, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
        return w if async_op else accum
    return None if async_op else accum


class FrameRenderer:
    """One rank's share of each frame.

    `accums`: one torch tensor (H x W x 4 float32) or a list of two for the pipelined schedule.
    `renderer`: a raymarchrenderer_amd.Renderer (the accumulator is bound with rmr_bind_accum), or
    None with `render_fn(acc, tiles, times, first_sample)` (tests: the CPU oracle under gloo).
    `streams`: one torch.cuda.Stream per renderer. Without them each renderer gets a new torch
    stream here (rmr_set_stream) on the accumulators' device, ordered after that device's current
    stream (so accumulators filled there are complete before the first zeroing): a frame's zeroing,
    its render and the collective that reads it must be ordered on one stream the collective waits
    for — a renderer left on its library-owned non-blocking stream would race both.
    Readers of a frame's accumulator must read on `streams[i]` of that frame or synchronize.
    `reduce_at_world1` (tests only): issue each frame's reduce even at world size 1, so the pipelined
    schedule's collective, its async handle and the wait before a buffer's reuse run on RCCL on a
    one-GPU box."""

    def __init__(self, renderer, accums, W, H, tile, rank, world, dist=None, render_fn=None, streams=None,
                 reduce_at_world1=False, grid_reserve=OVERLAP_GRID_RESERVE, launch_streams=None):
        self.rs = list(renderer) if isinstance(renderer, (list, tuple)) else [renderer]
        self._saved_reserve = []
        self._saved_streams = []
        if render_fn is None and len(self.rs) > 1 and grid_reserve is not None:
            # overlapping contexts: each trace launch leaves a few workgroup slots free, so the other
            # context's fold and zeroing run beside it instead of waiting for its drain (rmr.h); the
            # renderers' own settings come back at close()
            for r in self.rs:
                self._saved_reserve.append((r, r.grid_reserve))
                r.set_grid_reserve(grid_reserve)
        if render_fn is None and (launch_streams is not None or len(self.rs) > 1):
            # overlapping contexts already fill each other's drains: no launch slots of their own by
            # default (rmr.h rmr_set_launch_streams; 2 contexts x 3 streams exceed the 4 hardware
            # queues: r06p_launch_streams.log, RM3 -10%, C1 -28%); restored at close()
            n = launch_streams if launch_streams is not None else 0
            for r in self.rs:
                if r.launch_streams != n:
                    self._saved_streams.append((r, r.launch_streams))
                    r.set_launch_streams(n)
        self.r, self.dist, self.render_fn = self.rs[0], dist, render_fn
        self.accs = list(accums) if isinstance(accums, (list, tuple)) else [accums]
        if len(self.accs) % len(self.rs):
            raise ValueError("accumulators must be a multiple of the renderers")
        if streams is None and render_fn is None:
            import torch
            dev = self.accs[0].device
            cur = torch.cuda.current_stream(dev)
            streams = [torch.cuda.Stream(device=dev) for _ in self.rs]
            for r, s in zip(self.rs, streams):
                s.wait_stream(cur)
                r.set_stream(s.cuda_stream)
        self.streams = list(streams) if streams is not None else None
        self.work = [None] * len(self.accs)
        self.tiles = tile_partition(W, H, tile, rank, world)
        self.tile = tile
        self.f = 0
        self.last = None
        self.reduce_at_world1 = reduce_at_world1
        self.reduces = 0   # collectives issued

    def frame(self, times, first_sample=0):
        """Render this rank's tiles of the next frame and start its reduce; returns the frame's
        accumulator (complete on rank 0 once `finish()` or the next reuse of the buffer waited)."""
        i = self.f % len(self.accs)
        acc = self.accs[i]
        r = self.next_renderer()
        with self._on_stream(self.f):
            if self.work[i] is not None:  # the reduce of the frame that last used this buffer
                self.work[i].wait()
                self.work[i] = None
            acc.zero_()
            if len(self.tiles):
                if self.render_fn is not None:
                    self.render_fn(acc, self.tiles, times, first_sample)
                else:
                    r.bind_accum(acc.data_ptr(), acc.numel() * acc.element_size())
                    r.render_tiles(times, self.tiles, self.tile, first_sample=first_sample)
            self.work[i] = reduce_frame(acc, self.dist, async_op=True, always=self.reduce_at_world1)
            self.reduces += self.work[i] is not None
        self.f += 1
        self.last = acc
        return acc

    def order_tiles_by_cost(self, times, min_spread=3.0, frame_times=None, trials=4, cost_map=None):
        """Hand this rank's costliest tiles out first where that makes frames faster. The work queue
        gives units out in tile-list order within each sample, so a launch ends (drains) on its last
        tiles' paths; with the cheap ones last (by each tile's map() evaluations in a probe over
        `times`, tile_costs) the drain is shorter. Only where the costliest tile exceeds `min_spread` x
        the mean is the order tried; then, with `frame_times`, `trials` frames in each order (twice,
        interleaved, after a frame per context in that order, before the caller's frames; every rank
        the same frames, the timings summed over ranks) decide. Measured (r05_tile_order_bench.log, r05_tile_order_rm2.log): the Mandelbulb
        (tile costs up to 5x the mean) +2.7%, the RM2 NEE frame (sky tiles) -11%, Cornell-5 / C5 / RM3
        (under 2x) within noise. Each pixel's samples are the same whatever the order, so the image is
        the same bits. Call before the first frame (the probe writes the first accumulator, which every
        frame zeroes). `cost_map` ({(tx, ty): cost}, frame_tile_costs): costs probed once for the whole
        frame, sliced to this rank's tiles instead of probed again. Returns whether it reordered."""
        if self.render_fn is not None:
            return False
        cost = np.zeros(0, np.int64)
        if len(self.tiles) and cost_map is not None:
            cost = np.array([cost_map[(int(tx), int(ty))] for tx, ty in self.tiles], np.int64)
        elif len(self.tiles):
            acc = self.accs[0]
            with self._on_stream(0):
                self.r.bind_accum(acc.data_ptr(), acc.numel() * acc.element_size())
                cost = tile_costs(self.r, self.tiles, self.tile, times)
                acc.zero_()
        self.tile_cost_spread = float(cost.max() / max(1.0, cost.mean())) if len(cost) else 0.0
        trial = frame_times is not None and trials > 0
        go = self.tile_cost_spread > min_spread
        if trial:   # every rank runs the same trial frames (their reduces are collectives) or none
            go = self._sum_over_ranks([float(go)])[0] > 0
        if not go:
            return False
        rows, by_cost = self.tiles, self.tiles[np.argsort(-cost, kind="stable")]
        if trial:
            t = [0.0, 0.0]
            for _ in range(2):
                for k, order in enumerate((rows, by_cost)):
                    self.tiles = order
                    # untimed: one frame per context (its tile-list upload after the switch)
                    self._time_frames(frame_times, len(self.rs))
                    t[k] += self._time_frames(frame_times, trials)
            t = self._sum_over_ranks(t)
            self.tile_order_trial_ms = [round(x / (2 * trials) * 1e3, 4) for x in t]
            if t[1] >= t[0]:
                self.tiles = rows
                return False
        self.tiles = by_cost
        return True

    def _time_frames(self, times, n):
        import time

        import torch
        self.finish()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            self.frame(times)
        self.finish()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def _sum_over_ranks(self, vals):
        if not _multi(self.dist):
            return vals
        import torch
        dev = self.accs[0].device
        x = torch.tensor(vals, dtype=torch.float64, device=dev if dev.type == "cuda" and self.dist.get_backend() == "nccl" else "cpu")
        self.dist.all_reduce(x)
        return x.cpu().tolist()

    def next_renderer(self):
        """The renderer context the next frame() uses (e.g. to load that frame's scene)."""
        return self.rs[self.f % len(self.rs)]

    def _on_stream(self, f):
        if not self.streams:
            return contextlib.nullcontext()
        import torch
        return torch.cuda.stream(self.streams[f % len(self.streams)])

    def finish(self):
        """Wait for every outstanding reduce; returns the last frame's accumulator."""
        for i, w in enumerate(self.work):
            if w is not None:
                with self._on_stream(i):
                    w.wait()
                self.work[i] = None
        return self.last

    def close(self):
        """finish(), then give the renderers back their grid reserve and launch streams from before this
        FrameRenderer (the passed contexts can be used on their own or in another FrameRenderer
        afterwards)."""
        last = self.finish()
        for r, v in self._saved_reserve:
            r.set_grid_reserve(v)
        self._saved_reserve = []
        for r, v in self._saved_streams:
            r.set_launch_streams(v)
        self._saved_streams = []
        return last
