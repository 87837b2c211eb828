"""Multi-rank frame sharding on CPU (gloo, world_size 2): the shard arithmetic
bench.py uses (ptmi/dist.py) partitions the frame, and the all-reduce of the
ranks' partial framebuffers reproduces the one-process frame.  The partial
frames come from the CPU oracle (test infrastructure), which renders global
sample ranges exactly like ptmi_scene_render; the GPU side of the same
invariances is tests/test_gpu_parity.py::test_sample_split_and_chunking_invariance
and ::test_tile_split_partitions_frame.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pyoracle
from ptmi import dist as pdist
from ptmi import layout
from tests.scene_inputs import scene_inputs

W, H, S = 24, 16, 6


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("samples", [1, 5, 2048])
def test_sample_shards_partition(world, samples):
    got = []
    for r in range(world):
        s0, s1, ts, to = pdist.shard(r, world, samples, "sample")
        assert (ts, to) == (1, 0) and s0 <= s1
        got.extend(range(s0, s1))
    assert got == list(range(samples))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("w,h", [(1280, 960), (37, 23), (8, 8)])
@pytest.mark.parametrize("mesh", [False, True])
def test_tile_shards_partition(world, w, h, mesh):
    """Raster and diagonal ownership both partition the frame; the diagonal one (mesh
    scenes whose tile rows divide by the rank count) gives every rank the same number of
    tiles in every tile row and every tile column."""
    diag = pdist.diagonal_ownership(w, world, mesh)
    cover = np.zeros((h, w), dtype=np.int64)
    for r in range(world):
        s0, s1, ts, to = pdist.shard(r, world, 7, "tile")
        assert (s0, s1, ts) == (0, 7, world)
        m = pdist.tile_owner_mask(w, h, ts, to, diag)
        cover += m
        if diag:
            tiles = m[::8, ::8]
            assert (tiles.sum(axis=1) == tiles.shape[1] // world).all()
            if tiles.shape[0] % world == 0:
                assert (tiles.sum(axis=0) == tiles.shape[0] // world).all()
    assert (cover == 1).all()
    assert diag == (mesh and world > 1 and ((w + 7) // 8) % world == 0)


def test_shard_rejects_bad_arguments():
    with pytest.raises(ValueError):
        pdist.shard(2, 2, 8, "sample")
    with pytest.raises(ValueError):
        pdist.shard(0, 2, 8, "rows")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, split, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        objs, tris, grps, cam = scene_inputs("reference", W, H, 0.15, 1.6)
        t2, g2 = layout.pad_empty(tris, grps)
        seeds = layout.seeds_go_float64(W * H, 5)
        s0, s1, ts, to = pdist.shard(rank, world, S, split)
        part = pyoracle.cpu_trace(objs, t2, g2, cam, S, seeds, sample_begin=s0, sample_end=s1, threads=1)
        if s1 - s0 == S:  # a full range comes back normalised: turn it into sums
            part = part.reshape(-1, 4).copy()
            part[:, :3] *= S
            part[:, 3] = S
            part = part.ravel()
        if split == "tile":  # this rank's pixels only, the others exactly 0
            part = part.reshape(H, W, 4) * pdist.tile_owner_mask(W, H, ts, to)[..., None]
        sums = torch.from_numpy(np.ascontiguousarray(part).ravel())
        if split == "sample":
            pdist.reduce_frame(sums)  # all-reduce
        else:
            pdist.reduce_frame_to(sums, 0)  # reduce onto rank 0 (bench.py)
        if rank == 0:
            np.save(os.path.join(out_dir, "frame.npy"), sums.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("split", ["sample", "tile"])
def test_two_rank_frame_matches_single_process(tmp_path, split):
    if not pyoracle.cpu_available():
        pytest.skip("oracle not built")
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), split, str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    sums = np.load(tmp_path / "frame.npy").reshape(-1, 4)
    objs, tris, grps, cam = scene_inputs("reference", W, H, 0.15, 1.6)
    t2, g2 = layout.pad_empty(tris, grps)
    full = pyoracle.cpu_trace(objs, t2, g2, cam, S, layout.seeds_go_float64(W * H, 5), threads=1).reshape(-1, 4)
    assert np.all(sums[:, 3] == S)
    if split == "tile":  # each pixel comes from one rank (the same conversion to sums): x + 0 = x
        assert np.array_equal(sums[:, :3], full[:, :3] * S)
    else:
        rgb = sums[:, :3] * (1.0 / S)  # ptmi_finalize (tracer.cl:1184-1187)
        err = np.abs(rgb - full[:, :3]).max()
        assert err < 1e-12, err  # summation order only


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("samples", [64, 1000, 2048, 4096])
def test_sample_split_balances_cost(world, samples):
    """Ranks get equal cost, not equal counts: the late sample indices (large-argument
    noise sin) weigh more, so the early ranks take a few more samples."""
    pts = [pdist.sample_split_point(g, world, samples) for g in range(world + 1)]
    costs = [pdist._cost(b) - pdist._cost(a) for a, b in zip(pts, pts[1:])]
    per_sample = max(pdist._COST_TAIL, max(w for _, w in pdist._COST_KNOTS))
    assert max(costs) - min(costs) <= 2 * per_sample
    if samples > 731 * 2:
        counts = [b - a for a, b in zip(pts, pts[1:])]
        assert counts[0] > counts[-1]


_RANK_SCRIPT = """
import os, sys, json
import torch, torch.distributed as dist
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
assert int(os.environ["LOCAL_RANK"]) == r and os.environ["MASTER_ADDR"] == "127.0.0.1"
t = torch.tensor([float(r + 1)])
dist.all_reduce(t)
with open(os.path.join(sys.argv[1], "rank%d.json" % r), "w") as f:
    json.dump({"rank": r, "world": w, "sum": t.item()}, f)
dist.destroy_process_group()
sys.exit(int(sys.argv[2]) if r == 1 else 0)
"""


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launches_its_own_ranks(tmp_path, world):
    """bench.py --gpus N without a torch.distributed environment starts N ranks
    itself (RANK = LOCAL_RANK = 0..N-1, WORLD_SIZE = N, 127.0.0.1 rendezvous) and
    returns a failing rank's status."""
    import json
    import bench
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    assert bench.launch_ranks(world, [str(tmp_path), "0"], script=str(script)) == 0
    got = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(world)]
    assert [g["rank"] for g in got] == list(range(world))
    assert all(g["world"] == world and g["sum"] == world * (world + 1) / 2 for g in got)
    assert bench.launch_ranks(world, [str(tmp_path), "3"], script=str(script)) == 3


def test_bench_rejects_world_mismatch():
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "..", "bench.py"), "--gpus", "4"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8])
@pytest.mark.parametrize("samples", [1, 5, 300, 553, 731, 1500, 2048, 4096])
def test_library_and_python_sample_splits_agree(world, samples):
    """ptmi_trace_multi's split (C++ split_point, exported as ptmi_sample_split_point)
    and bench.py's ranks (ptmi/dist.py sample_split_point) are the same table."""
    from ptmi import api
    for g in range(world + 1):
        assert api.sample_split_point(g, world, samples) == pdist.sample_split_point(g, world, samples), (g, world)
