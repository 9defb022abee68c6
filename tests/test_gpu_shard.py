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
    assert _H_bar(Hs, Hf) and _H_bar(bs, bf)
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
