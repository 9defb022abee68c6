"""The product library's point sharding (Src/EnergyFunctional.cpp:155-220): shards 0 and 1 of a
p % 2 split of the C4 window, loaded into two contexts on one GPU.  What the two ranks of a 2-GPU run exchange --
the packed system vector (all-reduced) and the newest-frame candidates (all-gathered) -- is read back from each
context: their sums / union reproduce the full window's system (at the H bar), energy and setNewFrameEnergyTH
threshold (bit-exact), and the library's packed vector is the layout hslam_amd.ba.pack_system_vector states (the
layout tests/test_dist_gloo.py all-reduces over gloo)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _H_bar(g, f):
    scale = np.abs(f).max()
    return np.all(np.abs(g - f) <= 1e-4 * (np.abs(f) + 1e-3 * scale))


def test_two_shards_reproduce_the_full_window(scene2k):
    from hslam_amd.ba import BAWindow, pack_system_vector, unpack_system_vector
    from test_gpu_threshold import device_threshold
    full = BAWindow(scene2k)
    ef = full.linearizeAll(reset=True)
    shards = [BAWindow(scene2k.shard(r, 2)) for r in range(2)]
    es = [s.linearizeAll(reset=True) for s in shards]
    n = full.dim
    # energies: fp64 sums of the same fp32 terms in another order
    assert abs(sum(es) - ef) <= 1e-9 * abs(ef)
    # the library's vector is pack_system_vector of its own HA / HSC (the stitch writes both from the same sums)
    for w in [full] + shards:
        v = w.system_vector()
        HA, bA = w.system(0)
        HS, bS = w.system(2)
        p = pack_system_vector(HA, bA, HS, bS, v[-3], v[-2], v[-1])
        up = np.triu_indices(n)
        assert np.allclose(v[:n * n].reshape(n, n)[up], p[:n * n].reshape(n, n)[up], rtol=1e-13, atol=1e-9)
        assert np.allclose(v[n * n:], p[n * n:], rtol=1e-13, atol=1e-12)
    # what the all-reduce forms: the sum of the shards' vectors = the full window's (at the H bar)
    vf = full.system_vector()
    vs = shards[0].system_vector() + shards[1].system_vector()
    Hf, bf, Ef = unpack_system_vector(vf, n)
    Hs, bs, Es = unpack_system_vector(vs, n)
    if not (_H_bar(Hs, Hf) and _H_bar(bs, bf)):  # an intermittent mismatch: say what it looked like
        zr = [i for i in range(n) if not np.any(Hf[i])]
        full.linearizeAll(reset=True)
        H2 = unpack_system_vector(full.system_vector(), n)[0]
        zr2 = [i for i in range(n) if not np.any(H2[i])]
        pytest.fail(f"full-window H rows all zero: {zr}; after a second linearizeAll on the same context: {zr2} "
                    f"(second H at the bar: {bool(_H_bar(Hs, H2))})")
    assert abs(Es - Ef) <= 1e-9 * abs(Ef) and vs[-1] == vf[-1]
    # what the all-gather feeds: the union of the shards' candidates selects the full window's threshold
    union = np.concatenate([s.candidates()[: s.n_points] for s in shards])
    th_full = full.frames()["energyTH"][scene2k.n_frames - 1]
    P = full.params
    kw = dict(thn=P.frameEnergyTHN, fac=P.frameEnergyTHFacMedian, cw=P.frameEnergyTHConstWeight,
              ow=P.overallEnergyTHWeight)
    assert device_threshold(union, **kw) == np.float32(th_full)
    assert device_threshold(full.candidates()[: full.n_points], **kw) == np.float32(th_full)
    # categorical decisions are shard-invariant: every residual's state equals the full window's
    rf = full.residuals()
    for r, s in enumerate(shards):
        rs = s.residuals()
        sel = np.nonzero(np.isin(scene2k.res_point, np.nonzero(np.arange(scene2k.n_points) % 2 == r)[0]))[0]
        assert np.array_equal(rs["state"], rf["state"][sel])
        assert np.array_equal(rs["energy"], rf["energy"][sel])
    for w in [full] + shards:
        w.close()


@pytest.mark.parametrize("th_multi", ["0", "1"])
def test_rank_group_runs_the_multi_rank_path(scene2k, th_multi, monkeypatch):
    """The library's multi-rank path with two ranks on one GPU (the in-process group of hs_ba_debug_group: the
    exchange is device copies where a multi-GPU run all-gathers over RCCL; every other launch is the RCCL path's):
    one exchange of [system vector | energies] and candidates per linearization, the rank-order sums, the
    threshold select over the gathered candidates beside the solve (block 1 of the solve launch) or in hs_k_combine.
      * after a linearization every rank holds the same summed vector, bit-equal to the sum of the two shards'
        own vectors in rank order, and the full window's threshold (bit-exact: the union of the candidates);
      * the fused GN loop (deferred sums: the solve's prefetch) keeps both ranks' frame states bit-identical and
        follows the full window's trajectory (rel 1e-3, the optimize-trajectory bar).
    th_multi = 1 forces the large-window select (HS_TH_MULTI): on the ranks, the pass-1 histogram and pass 2 over the
    gathered candidates after the exchange, pass 3 as block 1 of the next solve / combine launch (round 6)."""
    from hslam_amd.ba import BAWindow
    monkeypatch.setenv("HS_TH_MULTI", th_multi)
    shard_scenes = [scene2k.shard(r, 2) for r in range(2)]
    full = BAWindow(scene2k)
    ef = full.linearizeAll(reset=True)
    alone = [BAWindow(s) for s in shard_scenes]
    for w in alone:
        w.linearizeAll(reset=True)
    vsum = alone[0].system_vector(raw=True) + alone[1].system_vector(raw=True)
    grp = BAWindow.rank_group(shard_scenes)
    eg = grp.linearizeAll(reset=True)
    assert abs(eg - ef) <= 1e-9 * abs(ef)
    newest = scene2k.n_frames - 1
    th_full = full.frames()["energyTH"][newest]
    for m in grp.members:
        assert np.array_equal(m.system_vector(raw=True), vsum)
        assert m.frames()["energyTH"][newest] == th_full
    K = 4
    ef_it = full.iterate(0, K)
    eg_it = grp.iterate(0, K)
    assert np.all(np.abs(eg_it - ef_it) <= 1e-3 * np.abs(ef_it))
    s0, s1 = (m.frames() for m in grp.members)
    assert np.array_equal(s0["state"], s1["state"]) and np.array_equal(s0["energyTH"], s1["energyTH"])
    sf = full.frames()["state"]
    assert np.allclose(s0["state"], sf, rtol=1e-3, atol=1e-3 * np.abs(sf).max())
    # the members' points are the full window's points p % 2 == r (the fused point steps of the shared solves)
    idf = full.points()["idepth"]
    for r, m in enumerate(grp.members):
        idr = m.points()["idepth"]
        assert np.allclose(idr, idf[r::2], rtol=1e-3, atol=1e-5)
    for w in [full, *alone]:
        w.close()
    grp.close()
