"""hs_k_stitch alone (the fp64 stitch of the top and Schur systems from per-host accumulator sums) against a numpy
restatement of the reference's pair-wise stitchDoubleInternal (Src/AccumulatedTopHessian.cpp:218-280,
Src/AccumulatedSCHessian.cpp:54-133) and stitchDoubleMT's symmetrization (Include/AccumulatedTopHessian.h:104-116),
on random accumulators and adjoints.  The kernel uses the A D A^T factorization of the Schur sandwiches and a
different fp64 summation order: relative tolerance 1e-12."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

E_TOP, ND_PROD, ND_EXACT = 16, 28, 49


def dpair(o1, o2):
    return o1 * 7 - (o1 * (o1 - 1)) // 2 + (o2 - o1)


def top_lane(R, C):
    """(entry e, lane k) owning the 13x13 AccumulatorApprox entry (R <= C) in the per-lane layout of hs_k_lin."""
    if C < 8:
        return R, C
    if C < 10:
        if R < 8:
            return C, R
        return 10, (0 if (R == 8 and C == 8) else (1 if R == 8 else 2))
    if R < 10:
        col = C - 10
        return (11 + col, R) if R < 8 else (14, (R - 8) * 3 + col)
    return 15, (C - 10 if R == 10 else (2 + C - 10 if R == 11 else 5))


def decode(hs, nF, exact):
    """Per-pair A (13x13), D (t1, t2), E (8x4), EB (8) and per-host Hcc (4x4), bc (4) from host sums hs[h][e][64]."""
    nd = ND_EXACT if exact else ND_PROD
    oE = E_TOP + nd
    A = np.zeros((nF, nF, 13, 13))
    D = np.zeros((nF, nF, nF, 8, 8))
    E = np.zeros((nF, nF, 8, 4))
    EB = np.zeros((nF, nF, 8))
    Hcc = np.zeros((nF, 4, 4))
    bc = np.zeros((nF, 4))
    for h in range(nF):
        for t in range(nF):
            if t == h:
                continue
            for R in range(13):
                for Cc in range(R, 13):
                    e, k = top_lane(R, Cc)
                    A[h, t, R, Cc] = A[h, t, Cc, R] = hs[h, e, t * 8 + k]
            for k in range(8):
                for c in range(4):
                    E[h, t, k, c] = hs[h, oE + c, t * 8 + k]
                EB[h, t, k] = hs[h, oE + 4, t * 8 + k]
        others = [t for t in range(nF) if t != h]
        for o1, t1 in enumerate(others):
            for o2, t2 in enumerate(others):
                if exact:
                    D[h, t1, t2] = hs[h, E_TOP + o1 * 7 + o2].reshape(8, 8)
                elif o1 <= o2:
                    D[h, t1, t2] = hs[h, E_TOP + dpair(o1, o2)].reshape(8, 8)
                else:
                    D[h, t1, t2] = hs[h, E_TOP + dpair(o2, o1)].reshape(8, 8).T
        Hcc[h] = hs[h, oE + 5, :16].reshape(4, 4)
        bc[h] = hs[h, oE + 5, 16:20]
    return A, D, E, EB, Hcc, bc


def reference_stitch(hs, adH, adT, nF, exact):
    A, D, E, EB, Hcc, bc = decode(hs, nF, exact)
    n = 4 + 8 * nF
    HA, bA, HS, bS = np.zeros((n, n)), np.zeros(n), np.zeros((n, n)), np.zeros(n)
    ix = lambda f: slice(4 + 8 * f, 12 + 8 * f)  # noqa: E731
    for h in range(nF):
        for t in range(nF):
            if h == t:
                continue
            aH, aT, Ap = adH[h + nF * t], adT[h + nF * t], A[h, t]
            A88, A84, a8r = Ap[4:12, 4:12], Ap[4:12, 0:4], Ap[4:12, 12]
            HA[ix(h), ix(h)] += aH @ A88 @ aH.T
            HA[ix(t), ix(t)] += aT @ A88 @ aT.T
            HA[ix(h), ix(t)] += aH @ A88 @ aT.T
            HA[ix(h), 0:4] += aH @ A84
            HA[ix(t), 0:4] += aT @ A84
            HA[0:4, 0:4] += Ap[0:4, 0:4]
            bA[ix(h)] += aH @ a8r
            bA[ix(t)] += aT @ a8r
            bA[0:4] += Ap[0:4, 12]
    for h in range(nF):  # stitchDoubleMT: calib rows, symmetrized frame blocks
        HA[0:4, ix(h)] = HA[ix(h), 0:4].T
        for t in range(h + 1, nF):
            HA[ix(h), ix(t)] += HA[ix(t), ix(h)].T
            HA[ix(t), ix(h)] = HA[ix(h), ix(t)].T
    for i in range(nF):
        for j in range(nF):
            if i == j:
                continue
            aHij, aTij = adH[i + nF * j], adT[i + nF * j]
            HS[ix(i), 0:4] += aHij @ E[i, j]
            HS[ix(j), 0:4] += aTij @ E[i, j]
            bS[ix(i)] += aHij @ EB[i, j]
            bS[ix(j)] += aTij @ EB[i, j]
            for k in range(nF):
                if k == i:
                    continue
                aHik, aTik = adH[i + nF * k], adT[i + nF * k]
                Dm = D[i, j, k]
                HS[ix(i), ix(i)] += aHij @ Dm @ aHik.T
                HS[ix(j), ix(k)] += aTij @ Dm @ aTik.T
                HS[ix(j), ix(i)] += aTij @ Dm @ aHik.T
                HS[ix(i), ix(k)] += aHij @ Dm @ aTik.T
    HS[0:4, 0:4] += Hcc.sum(0)
    bS[0:4] += bc.sum(0)
    for h in range(nF):
        HS[0:4, ix(h)] = HS[ix(h), 0:4].T
    return HA, bA, HS, bS


def run_gpu(hs, adH, adT, nF, exact):
    from hslam_amd._lib import check, load
    lib = load()
    n = 4 + 8 * nF
    SL = n * n + n
    out, sep = np.zeros(SL), np.zeros(2 * SL)
    p = lambda a: np.ascontiguousarray(a, np.float64).ctypes.data_as(C.c_void_p)  # noqa: E731
    hs_c, aH_c, aT_c = [np.ascontiguousarray(x, np.float64) for x in (hs, adH, adT)]
    check(lib.hs_debug_stitch(nF, int(exact), p(hs_c), p(aH_c), p(aT_c), p(out), p(sep)))
    up = lambda v: np.triu(v[:n * n].reshape(n, n)) + np.triu(v[:n * n].reshape(n, n), 1).T  # noqa: E731
    return up(sep[:SL]), sep[n * n:SL], up(sep[SL:]), sep[SL + n * n:], out


@pytest.mark.parametrize("nF,exact", [(8, False), (8, True), (3, False), (2, True)])
def test_stitch_matches_pairwise_reference(nF, exact):
    rng = np.random.default_rng(100 + nF + 10 * exact)
    ne = E_TOP + (ND_EXACT if exact else ND_PROD) + 6
    hs = rng.normal(size=(nF, ne, 64))
    # the real sums' symmetries: accD(t, t) and accHcc are symmetric; exact mode stores D(t2, t1) = D(t1, t2)^T
    nd = ND_EXACT if exact else ND_PROD
    for h in range(nF):
        for o1 in range(7):
            for o2 in range(o1, 7):
                i1 = E_TOP + (o1 * 7 + o2 if exact else dpair(o1, o2))
                blk = hs[h, i1].reshape(8, 8)
                if o1 == o2:
                    hs[h, i1] = ((blk + blk.T) / 2).ravel()
                elif exact:
                    hs[h, E_TOP + o2 * 7 + o1] = blk.T.ravel()
        hcc = hs[h, E_TOP + nd + 5, :16].reshape(4, 4)
        hs[h, E_TOP + nd + 5, :16] = ((hcc + hcc.T) / 2).ravel()
    adH = rng.normal(size=(nF * nF, 8, 8))
    adT = rng.normal(size=(nF * nF, 8, 8))
    HAg, bAg, HSg, bSg, out = run_gpu(hs, adH, adT, nF, exact)
    HA, bA, HS, bS = reference_stitch(hs, adH, adT, nF, exact)
    n = 4 + 8 * nF
    for g, r, name in ((HAg, HA, "HA"), (HSg, HS, "HSC"), (bAg, bA, "bA"), (bSg, bS, "bSC")):
        err = np.abs(g - r) / (np.abs(r).max() + 1e-300)
        assert err.max() <= 1e-12, (name, np.unravel_index(err.argmax(), err.shape), err.max())
    # the combined vector: upper triangle of HA - sc HSC (diagonal HA (1 + lambda) - sc HSC), bA - bSC
    sc, l1 = 1.0 / (1 + 1e-5), 1 + 1e-5
    comb = np.triu(HA - sc * HS)
    comb[np.diag_indices(n)] = np.diag(HA) * l1 - np.diag(HS) * sc
    got = np.triu(out[:n * n].reshape(n, n))
    assert np.abs(got - comb).max() <= 1e-12 * np.abs(comb).max()
    assert np.abs(out[n * n:] - (bA - bS)).max() <= 1e-12 * np.abs(bA - bS).max()
