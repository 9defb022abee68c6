"""Point activation: System::activatePointsMT (Src/Mapping.cpp:330-480) with
CoarseDistanceMap (Src/CoarseTracker.cpp:726-868) and optimizeImmaturePoint (Src/FullSystemOptPoint.cpp:24-175).

CPU: properties of the oracle restatement (the BFS metric, activation invariants).  GPU: hs_tracer_activate against
the oracle, bit-exact (action, idepth, IN-residual masks, toOptimize order, currentMinActDist, distance map).
Parity unpinned against the reference itself: the oracle is pinned by the properties below."""
import math

import numpy as np
import pytest

from hslam_amd.trace import act_frames_array, act_pairs_array


def oracle_tracer(s):
    from oracle_ffi import OracleTracer
    o = OracleTracer(s.width, s.height)
    imgs = [s.imgs[0]] * (int(s.slots.max()) + 1)
    for f in range(s.n_frames):
        imgs[s.slots[f]] = s.imgs[f]
    if len(s.imm_u):
        o.add_points(imgs, s.slots[s.imm_frame], s.imm_u, s.imm_v)
        o.set_state(s.imm_idepth_min, s.imm_idepth_max, s.imm_quality, s.imm_status, s.imm_interval)
        o.set_types(s.imm_type)
    return o


def gpu_tracer(s):
    from hslam_amd.trace import ImmatureTracer
    g = ImmatureTracer(s.width, s.height, max(1, len(s.imm_u)))
    for f in range(s.n_frames):
        g.set_host_image(int(s.slots[f]), s.imgs[f])
    if len(s.imm_u):
        g.add_points(s.slots[s.imm_frame], s.imm_u, s.imm_v)
        g.set_state(s.imm_idepth_min, s.imm_idepth_max, s.imm_quality, s.imm_status, s.imm_interval)
        g.set_types(s.imm_type)
    return g


def activate(tr, s, oracle, order="scene", cmad=None):
    fr = act_frames_array(s.slots, s.flagged, s.KRKi1, s.Kt1)
    pr = act_pairs_array(s.RTll, s.tTll, s.aff)
    od = s.order if isinstance(order, str) else order
    args = (s.K4, fr, pr, s.act_frame, s.act_u, s.act_v, s.act_idepth, s.ef_nPoints,
            s.currentMinActDist if cmad is None else cmad, od)
    return tr.activatePointsMT(s.imgs, *args) if oracle else tr.activatePointsMT(*args)


@pytest.fixture(scope="module")
def vga():
    from hslam_amd.scene import make_activation_scene
    return make_activation_scene()


def octagonal(dx, dy):
    """Steps growDistBFS needs from one seed without borders: odd steps move in 8 directions, even steps in 4."""
    a, b = abs(dx), abs(dy)
    k = max(a, b)
    while a + b > k + (k + 1) // 2:
        k += 1
    return k


def test_distance_map_single_seed_is_octagonal(vga):
    """One MapPoint, no immature points: the map is the alternating 8/4-neighbourhood BFS distance, capped at 39."""
    import copy
    s = copy.copy(vga)
    ok = vga.act_frame < vga.n_frames - 1
    c = np.argmin(np.where(ok, (vga.act_u - vga.width / 2) ** 2 + (vga.act_v - vga.height / 2) ** 2, np.inf))
    s.act_frame, s.act_u, s.act_v, s.act_idepth = (x[c:c + 1] for x in (vga.act_frame, vga.act_u, vga.act_v,
                                                                         vga.act_idepth))
    for k in ("imm_frame", "imm_u", "imm_v", "imm_idepth_min", "imm_idepth_max", "imm_quality", "imm_status",
              "imm_interval", "imm_type", "order"):
        setattr(s, k, getattr(vga, k)[:0])
    o = oracle_tracer(s)
    r = activate(o, s, True)
    assert len(r["activated"]) == 0
    dm = o.distance_map()
    zy, zx = np.nonzero(dm == 0)
    assert len(zx) == 1
    x0, y0 = zx[0], zy[0]
    h1, w1 = dm.shape
    assert min(x0, y0) > 41 and min(w1 - x0, h1 - y0) > 41  # the BFS never reaches a border row / column
    for y in range(h1):
        for x in range(w1):
            d = octagonal(x - x0, y - y0)
            assert dm[y, x] == (d if d < 40 else 1000), (x, y)


def _grow_dist_bfs(m, frontier, w1, h1):
    """CoarseDistanceMap::growDistBFS (Src/CoarseTracker.cpp:759-857), restated as plain Python."""
    for k in range(1, 40):
        nxt = []
        for (x, y) in frontier:
            if x == 0 or y == 0 or x == w1 - 1 or y == h1 - 1:
                continue
            nb = [(1, 0), (-1, 0), (0, 1), (0, -1)] + ([(1, 1), (-1, 1), (-1, -1), (1, -1)] if k % 2 else [])
            for dx, dy in nb:
                if m[y + dy, x + dx] > k:
                    m[y + dy, x + dx] = k
                    nxt.append((x + dx, y + dy))
        frontier = nxt


def _closed_form_add(m, sx, sy, w1, h1):
    """hs_act_kernels.hip's addIntoDistFinal without a BFS (bfs_dist / border_step): interior cells min(map, k),
    border cells from their interior neighbours the wave lowered, a border seed only itself."""
    new = m.copy()
    new[sy, sx] = 0
    if sx == 0 or sy == 0 or sx == w1 - 1 or sy == h1 - 1:
        return new
    ys, xs = np.mgrid[0:h1, 0:w1]
    ax, ay = np.abs(xs - sx), np.abs(ys - sy)
    d = np.maximum(np.maximum(ax, ay), (2 * (ax + ay) + 1) // 3)
    inner = np.zeros_like(m, bool)
    inner[1:-1, 1:-1] = True
    upd = inner & (d <= 39)
    new[upd] = np.minimum(m[upd], d[upd])
    for by, bx in zip(*np.nonzero(~inner)):
        v = new[by, bx]
        for ny in (by - 1, by, by + 1):
            for nx in (bx - 1, bx, bx + 1):
                if not (1 <= nx <= w1 - 2 and 1 <= ny <= h1 - 2):
                    continue
                t = d[ny, nx] + 1
                frontier = d[ny, nx] < m[ny, nx] or (nx, ny) == (sx, sy)
                if frontier and t <= 39 and (nx == bx or ny == by or t % 2 == 1):
                    v = min(v, t)
        new[by, bx] = v
    return new


def _closed_form_seeds(seeds, w1, h1):
    """hs_k_act_map0: makeDistanceMap's multi-seed growDistBFS in closed form -- interior cells the minimum of the
    interior seeds' distances, border cells k_n + 1 from their interior neighbours, border seeds only themselves."""
    m = np.full((h1, w1), 1000, np.int32)
    ys, xs = np.mgrid[0:h1, 0:w1]
    d = np.full((h1, w1), 1000, np.int32)
    for (x, y) in seeds:
        m[y, x] = 0
        if x == 0 or y == 0 or x == w1 - 1 or y == h1 - 1:
            continue
        ax, ay = np.abs(xs - x), np.abs(ys - y)
        dd = np.maximum(np.maximum(ax, ay), (2 * (ax + ay) + 1) // 3)
        d = np.minimum(d, np.where(dd <= 39, dd, 1000))
    inner = np.zeros((h1, w1), bool)
    inner[1:-1, 1:-1] = True
    out = m.copy()
    out[inner] = np.minimum(m, d)[inner]
    for by, bx in zip(*np.nonzero(~inner)):
        v = out[by, bx]
        for ny in (by - 1, by, by + 1):
            for nx in (bx - 1, bx, bx + 1):
                if not (1 <= nx <= w1 - 2 and 1 <= ny <= h1 - 2) or out[ny, nx] >= 1000:
                    continue
                t = out[ny, nx] + 1
                if t <= 39 and (nx == bx or ny == by or t % 2 == 1):
                    v = min(v, t)
        out[by, bx] = v
    return out


def test_closed_form_bfs_matches_grow_dist_bfs():
    """The activation kernels replace growDistBFS by a closed form (hs_act_kernels.hip bfs_dist, border_step;
    hs_k_act_map0, hs_k_act_final).  Random small maps: makeDistanceMap's multi-seed BFS (against the closed form of
    hs_k_act_map0), then a sequence of
    addIntoDistFinal calls (seeds anywhere the selection loop can put them: x, y > 0, borders included); after every
    call the closed form equals the reference's growDistBFS on every cell."""
    rng = np.random.default_rng(11)
    for trial in range(40):
        w1, h1 = int(rng.integers(4, 48)), int(rng.integers(4, 40))
        m = np.full((h1, w1), 1000, np.int32)
        seeds = {(int(rng.integers(1, w1)), int(rng.integers(1, h1))) for _ in range(int(rng.integers(0, 5)))}
        for (x, y) in seeds:
            m[y, x] = 0
        _grow_dist_bfs(m, sorted(seeds), w1, h1)
        assert np.array_equal(_closed_form_seeds(sorted(seeds), w1, h1), m), (trial, (w1, h1))
        for _ in range(int(rng.integers(1, 10))):
            x, y = int(rng.integers(1, w1)), int(rng.integers(1, h1))
            ref = m.copy()
            ref[y, x] = 0
            _grow_dist_bfs(ref, [(x, y)], w1, h1)
            assert np.array_equal(_closed_form_add(m, x, y, w1, h1), ref), (trial, (w1, h1), (x, y))
            m = ref


def test_activation_invariants(vga):
    o = oracle_tracer(vga)
    r = activate(o, vga, True)
    act, a = r["action"], r["activated"]
    assert len(a) > 50 and (act == 1).sum() > 50
    assert np.all(act[a] == 2) and (act == 2).sum() == len(a)
    # every new MapPoint has an IN residual, never into its own host
    for i in a:
        assert r["res_in"][i] != 0 and not (r["res_in"][i] >> vga.imm_frame[i]) & 1
        assert np.isfinite(r["idepth"][i])
    # points of the newest keyframe are never touched; NaN-max / OUTLIER points are always deleted
    newest = vga.imm_frame == vga.n_frames - 1
    assert np.all(act[newest] == 0)
    bad = ~newest & (~np.isfinite(vga.imm_idepth_max) | (vga.imm_status == 2))
    assert np.all(act[bad] == 1)
    # toOptimize order: the reference's loop order
    pos = np.empty(len(vga.order), np.int64)
    pos[vga.order] = np.arange(len(vga.order))
    assert np.all(np.diff(pos[a]) > 0)
    assert r["currentMinActDist"] == np.float32(np.float32(2.0) - 0.5)  # 1500 < 0.8 * 2000


def test_activation_respects_min_distance(vga):
    """With a large currentMinActDist fewer points pass the distance test than with 0."""
    n = []
    for cmad in (0.0, 4.0):
        o = oracle_tracer(vga)
        import copy
        s = copy.copy(vga)
        s.ef_nPoints = 2000  # no update: density met exactly
        r = activate(o, s, True, cmad=cmad)
        n.append(len(r["activated"]) + int((r["action"] == 1).sum()))
    assert n[1] < n[0]


def test_min_act_dist_update_rule(vga):
    """The currentMinActDist update (Mapping.cpp:332-352) for densities around setting_desiredPointDensity."""
    import copy
    s = copy.copy(vga)
    for k in ("imm_frame", "imm_u", "imm_v", "imm_idepth_min", "imm_idepth_max", "imm_quality", "imm_status",
              "imm_interval", "imm_type", "order"):
        setattr(s, k, getattr(vga, k)[:0])
    want = {1000: 2.0 - 0.8 - 0.5, 1700: 2.0 - 0.2, 1900: 2.0 - 0.1, 2000: 2.0, 2100: 2.1, 2400: 2.3,
            2700: 2.8, 3100: 3.6, 5000: 3.6 + 0.0}
    for npts, w in want.items():
        s.ef_nPoints = npts
        r = activate(oracle_tracer(s), s, True, cmad=2.0)
        exp = np.float32(2.0)
        d = np.float32(2.0)
        dens = 2000.0
        if npts < dens * 0.66: d = np.float32(float(d) - 0.8)
        if npts < dens * 0.8: d = np.float32(float(d) - 0.5)
        elif npts < dens * 0.9: d = np.float32(float(d) - 0.2)
        elif npts < dens: d = np.float32(float(d) - 0.1)
        if npts > dens * 1.5: d = np.float32(float(d) + 0.8)
        if npts > dens * 1.3: d = np.float32(float(d) + 0.5)
        if npts > dens * 1.15: d = np.float32(float(d) + 0.2)
        if npts > dens: d = np.float32(float(d) + 0.1)
        d = min(max(d, np.float32(0)), np.float32(4))
        assert r["currentMinActDist"] == d, npts
        assert math.isclose(r["currentMinActDist"], min(w, 4.0), abs_tol=1e-5), npts


# ------------------------------------------------------------------------------------------------ GPU
def compare(rg, ro, n):
    assert rg["currentMinActDist"] == ro["currentMinActDist"]
    assert np.array_equal(rg["action"], ro["action"])
    assert np.array_equal(rg["activated"], ro["activated"])
    a = ro["activated"]
    assert np.array_equal(rg["idepth"][a], ro["idepth"][a])
    assert np.array_equal(rg["res_in"], ro["res_in"])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["vga", "kitti", "large"])
def test_activation_bit_exact(cfg, vga):
    from hslam_amd.scene import make_activation_scene
    s = {"vga": lambda: vga,
         "kitti": lambda: make_activation_scene(2000, 5000, width=1232, height=368, kitti=True, seed=3),
         # a level-1 map larger than LDS (800 x 400 bytes): the global-memory map path
         "large": lambda: make_activation_scene(1200, 2500, width=1600, height=800, seed=5)}[cfg]()
    o, g = oracle_tracer(s), gpu_tracer(s)
    ro, rg = activate(o, s, True), activate(g, s, False)
    compare(rg, ro, len(s.imm_u))
    assert np.array_equal(g.distance_map(), o.distance_map())
    assert len(ro["activated"]) > 20


@pytest.mark.gpu
def test_activation_variants(vga):
    """Storage order (order=NULL), a subset order, currentMinActDist 0 and 4, no MapPoints."""
    import copy
    for variant in ("storage", "subset", "cmad0", "cmad4", "noact"):
        s = copy.copy(vga)
        order = "scene"
        cmad = None
        if variant == "storage":
            order = None
        elif variant == "subset":
            order = vga.order[::3].copy()
        elif variant == "cmad0":
            cmad, s.ef_nPoints = 0.0, 2000
        elif variant == "cmad4":
            cmad, s.ef_nPoints = 4.0, 2000
        else:
            s.act_frame, s.act_u, s.act_v, s.act_idepth = (x[:0] for x in (vga.act_frame, vga.act_u, vga.act_v,
                                                                           vga.act_idepth))
        o, g = oracle_tracer(s), gpu_tracer(s)
        ro, rg = activate(o, s, True, order, cmad), activate(g, s, False, order, cmad)
        compare(rg, ro, len(s.imm_u))
        assert np.array_equal(g.distance_map(), o.distance_map()), variant


@pytest.mark.gpu
def test_compact_after_activation(vga):
    o, g = oracle_tracer(vga), gpu_tracer(vga)
    r = activate(g, vga, False)
    activate(o, vga, True)
    keep = (r["action"] == 0).astype(np.uint8)
    o.compact(keep)
    g.compact(keep)
    po, pg = o.points(), g.points()
    assert g.n == o.n == int(keep.sum())
    for k in po:
        assert np.array_equal(po[k], pg[k], equal_nan=True), k


@pytest.mark.gpu
def test_activation_errors_are_loud(vga):
    from hslam_amd._lib import HsError
    g = gpu_tracer(vga)
    fr = act_frames_array(vga.slots, vga.flagged, vga.KRKi1, vga.Kt1)
    pr = act_pairs_array(vga.RTll, vga.tTll, vga.aff)
    bad = fr.copy()
    bad["slot"][2] = 60  # no image there
    with pytest.raises(HsError):
        g.activatePointsMT(vga.K4, bad, pr, vga.act_frame, vga.act_u, vga.act_v, vga.act_idepth, 1500, 2.0)
    with pytest.raises(HsError):
        g.activatePointsMT(vga.K4, fr, pr, vga.act_frame, vga.act_u, vga.act_v, vga.act_idepth, 1500, 2.0,
                           order=np.array([0, 0], np.int32))
