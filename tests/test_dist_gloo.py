"""Multi-rank (point-sharded) BA semantics, world_size 2 over gloo on CPU.

The GPU path (hs_comm_init + RCCL) shards points p % nranks: every rank linearizes and
accumulates its own points, then ONE exchange per linearization all-gathers every rank's packed system vector
(hslam_amd.ba.pack_system_vector: the upper triangle of HA diag(1+lambda) - HSC / (1+lambda), bA - bSC, energies)
and its newest-frame candidates (hs_ba.cpp exchange(): two all-gathers in one RCCL group); every rank sums the
gathered vectors in rank order (so every rank solves the same system, bit for bit) and selects the same
0.7-quantile threshold over the gathered candidates.  This test runs that exchange, with the CPU oracle's systems
packed in the library's layout on each rank, and checks it against the unsharded window (tests/test_gpu_shard.py
runs the library's own exchange with two ranks on one GPU):
  * both ranks' rank-order sums are bit-identical and equal the full window's packed vector (H / b at the H bar,
    energy 1e-9),
  * the gathered quantile threshold equals the full window's setNewFrameEnergyTH,
  * the shards partition the points and keep every point's residuals together.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _threshold(energies, P):
    """System::setNewFrameEnergyTH (Src/FullSystemOptimize.cpp:60-101) over a candidate set."""
    e = np.asarray(energies, np.float32)
    if e.size == 0:
        return np.float32(12 * 12 * 8)
    k = int(np.float32(P["THN"]) * np.float32(e.size))
    nth = np.sqrt(np.partition(e, k)[k]).astype(np.float32)
    th = np.float32(nth * np.float32(P["fac"]))
    th = np.float32(np.float32(26.0) * np.float32(P["cw"]) + th * np.float32(1 - P["cw"]))
    th = np.float32(th * th)
    return np.float32(th * np.float32(P["ow"] * P["ow"]))


def _worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "h-slam_amd"), os.path.join(root, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hslam_amd.scene import make_ba_scene
    from oracle_ffi import OracleBA

    scene = make_ba_scene(n_points=240, seed=7)
    shard = scene.shard(rank, world)
    o = OracleBA(shard, nthreads=1)
    e = o.linearize_all(reset=True)
    o.apply_res()
    res = o.residuals()
    newest = scene.n_frames - 1
    cand = res["energy_wo"][(shard.res_target == newest) & (res["energy_wo"] >= 0)].astype(np.float32)
    HA, bA = o.accumulate(0)
    HS, bS = o.accumulate(2)
    # the exchange: all-gather of the packed system vectors (the library's payload), summed in rank order
    from hslam_amd.ba import pack_system_vector
    mine = torch.from_numpy(pack_system_vector(HA, bA, HS, bS, e, 0.0, float(shard.n_points)))
    vecs = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(vecs, mine)
    flat = vecs[0].clone()
    for v in vecs[1:]:
        flat += v
    # all-gather of the newest-frame candidates (padded to a common stride, -1 = none)
    n = torch.tensor([cand.size])
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, n)
    stride = int(max(s.item() for s in sizes))
    pad = np.full(stride, -1.0, np.float32)
    pad[:cand.size] = cand
    gathered = [torch.zeros(stride) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(pad))
    union = np.concatenate([g.numpy() for g in gathered])
    union = union[union >= 0]
    np.savez(os.path.join(out_dir, f"dist{rank}.npz"), flat=flat.numpy(), union=union)
    dist.destroy_process_group()


def test_point_sharded_reduction_matches_full_window(tmp_path):
    from hslam_amd.scene import make_ba_scene
    from oracle_ffi import OracleBA

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "dist0.npz")
    got1 = np.load(tmp_path / "dist1.npz")
    assert np.array_equal(got["flat"], got1["flat"])  # every rank solves the same system
    assert np.array_equal(np.sort(got["union"]), np.sort(got1["union"]))
    scene = make_ba_scene(n_points=240, seed=7)
    o = OracleBA(scene, nthreads=1)
    e = o.linearize_all(reset=True)
    o.apply_res()
    HA, bA = o.accumulate(0)
    HS, bS = o.accumulate(2)
    n = HA.shape[0]
    from hslam_amd.ba import pack_system_vector, unpack_system_vector
    gH, gb, ge = unpack_system_vector(got["flat"], n)
    fH, fb, fe = unpack_system_vector(pack_system_vector(HA, bA, HS, bS, e, 0.0, scene.n_points), n)
    assert abs(ge - fe) <= 1e-9 * abs(fe) and got["flat"][-1] == scene.n_points
    for g, f in ((gH, fH), (gb, fb)):
        scale = np.abs(f).max()
        assert np.all(np.abs(g - f) <= 1e-4 * (np.abs(f) + 1e-3 * scale))
    # quantile over the union == the full window's threshold (bit-exact: selection is order independent)
    P = dict(THN=0.7, fac=1.5, cw=0.5, ow=1.0)
    full_th = o.frames()["energyTH"][scene.n_frames - 1]
    assert _threshold(got["union"], P) == np.float32(full_th)


def test_shards_partition_points_and_keep_residuals_together():
    from hslam_amd.scene import make_ba_scene

    scene = make_ba_scene(n_points=240, seed=7)
    world = 3
    shards = [scene.shard(r, world) for r in range(world)]
    assert sum(s.n_points for s in shards) == scene.n_points
    assert sum(s.n_res for s in shards) == scene.n_res
    for r, s in enumerate(shards):
        idx = np.nonzero(np.arange(scene.n_points) % world == r)[0]
        assert np.array_equal(s.pt_u, scene.pt_u[idx])
        assert np.all(np.diff(s.pt_host) >= 0)  # still sorted by host (the C-ABI requires it)
        # every residual of a shard point is on that shard, in the original order
        for k, p in enumerate(idx[:20]):
            full = scene.res_target[scene.res_point == p]
            mine = s.res_target[s.res_point == k]
            assert np.array_equal(full, mine)
