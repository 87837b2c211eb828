"""Multi-GPU frame sharding: one process per GPU, torch.distributed
over RCCL ("nccl" backend) on a GPU node, gloo in the CPU tests.

Every (pixel, sample) path is independent and depends only on (seed[pixel],
sample index n, total samples S) (tracer.cl:840-869), so a frame shards with no
data-path exchange; the only collective is the final sum of the per-rank
partial framebuffers:

  * sample split -- rank r renders a contiguous range of sample indices of every
    pixel (global n and total S are passed through, so fgi2 = seed/S and the DoF
    sunflower pattern are those of the full frame).  The ranges are balanced by
    cost, not count (sample_split_point);
  * tile split   -- rank r renders every sample of the 8x8 tiles t with
    t % N == r (round-robin, balances a mesh-heavy region across ranks) and
    leaves the other pixels at exactly 0.

Either way the frame is the elementwise SUM of the partial framebuffers
(ptmi_scene_render writes RGB sums, A = number of samples), reduced with one
reduce(SUM) of W*H*4 doubles onto rank 0 (reduce_frame_to) and normalised there on
device (ptmi_finalize).
For the tile split the sum is exact (x + 0 = x); for the sample split it
differs from a one-GPU render only by FP64 summation order (~1e-16 relative).
"""
TILE = 8  # ptmi_device.h kTile

# Relative cost of one sample by its index n (x100): past n ~ 553 the hemisphere noise
# arguments (n * 237.212 + ...) and past ~731 the anti-aliasing ones (n * 179.233)
# reach 2^17, ocml's large-argument sin reduction (csrc/ptmi_sinf.h).  Round 6, the
# round-6 kernel's 8-rank C2 shares (tools/shard_balance.py): 0.0704 ms per sample of
# the frame below n = 553 and 0.0718 past 731 (round 5: x50 weights 50, 51, 52 from
# 256-sample slices of 23.5 / 24.5 ms).  Same table as ptmi_api.cpp's split_point.
_COST_KNOTS = ((553, 100), (731, 101))
_COST_TAIL = 102


def _cost(n):
    c, lo = 0, 0
    for hi, w in _COST_KNOTS:
        c += w * max(0, min(n, hi) - lo)
        lo = hi
    return c + _COST_TAIL * max(0, n - lo)


def sample_split_point(g, world, samples):
    """First sample index of rank g (g = world -> samples): the smallest n whose
    cumulative cost reaches g/world of the frame's.  Monotone in g, 0 at g = 0."""
    target = -(-g * _cost(samples) // world)  # ceil
    n, c, lo = 0, 0, 0
    for hi, w in _COST_KNOTS + ((1 << 62, _COST_TAIL),):
        span = w * (hi - lo)
        if target <= c + span:
            n = lo + -(-(target - c) // w)
            break
        c += span
        lo = hi
    return min(n, samples)


def shard(rank, world, samples, split):
    """-> (sample_begin, sample_end, tile_stride, tile_offset) of `rank`."""
    if not (0 <= rank < world):
        raise ValueError("rank %d outside world %d" % (rank, world))
    if split == "sample":
        return sample_split_point(rank, world, samples), sample_split_point(rank + 1, world, samples), 1, 0
    if split == "tile":
        return 0, samples, world, rank
    raise ValueError("split must be 'sample' or 'tile', got %r" % (split,))


def diagonal_ownership(width, tile_stride, mesh_affine):
    """The library's tile-ownership rule for the common case (ptmi_api.cpp diagonal_tiles):
    affine mesh scenes whose tile rows divide by the stride split diagonally, others raster.
    `mesh_affine` must be False -- raster -- in the cases the library also excludes: the
    statistical RNG mode, meshes with wide (31-bit) child codes (F_WIDE), non-affine or
    textured scenes, and the study library's split form.  For a resident scene the library's
    own decision is Scene.tile_ownership(stride) (ptmi_diag_tile_ownership); use that where a
    scene is at hand (tests/test_gpu_parity.py checks the two agree)."""
    tx = (width + TILE - 1) // TILE
    return bool(mesh_affine) and tile_stride > 1 and tx % tile_stride == 0


def scene_ownership_mask(scene, tile_stride, tile_offset):
    """tile_owner_mask with the ownership a resident scene's renders use (the library's decision)."""
    diag = scene.tile_ownership(tile_stride) == "diagonal"
    return tile_owner_mask(scene.width, scene.height, tile_stride, tile_offset, diagonal=diag)


def tile_owner_mask(width, height, tile_stride, tile_offset, diagonal=False):
    """Boolean (H, W) mask of the pixels a tile-split rank owns: tiles are 8x8,
    numbered row-major over ceil(W/8) x ceil(H/8) (the kernel's tile index); rank
    tile_offset owns tile t when t mod tile_stride == tile_offset (raster), or tile
    (x, y) when (x + y) mod tile_stride == tile_offset (diagonal, diagonal_ownership)."""
    import numpy as np
    tx = (width + TILE - 1) // TILE
    ys, xs = np.mgrid[0:height, 0:width]
    if diagonal:
        return ((ys // TILE + xs // TILE) % tile_stride) == tile_offset
    tile = (ys // TILE) * tx + xs // TILE
    return (tile % tile_stride) == tile_offset


def reduce_frame(partial, group=None):
    """Sum the ranks' partial framebuffers in place (RCCL all-reduce over xGMI
    on a GPU node; whatever backend `group` uses otherwise).  No-op at N=1."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(partial, op=dist.ReduceOp.SUM, group=group)
    return partial


def reduce_frame_to(partial, dst=0, group=None, via_host=False):
    """Sum the ranks' partial framebuffers onto rank `dst` (one RCCL reduce of
    W*H*4 doubles over xGMI on a GPU node -- SURVEY.md 8e's ncclReduce; only the
    destination normalises and keeps the frame).  ``via_host``: reduce a host copy
    (gloo), for ranks that share one device in a rehearsal.  No-op at N=1."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1):
        return partial
    if via_host:
        h = partial.cpu()
        dist.reduce(h, dst, op=dist.ReduceOp.SUM, group=group)
        if dist.get_rank(group) == dst:
            partial.copy_(h)
    else:
        dist.reduce(partial, dst, op=dist.ReduceOp.SUM, group=group)
    return partial
