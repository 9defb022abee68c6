import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "h-slam_amd"), os.path.join(ROOT, "tests")]
import numpy as np
from test_gpu_stitch import run_gpu, reference_stitch, decode, E_TOP, ND_PROD
for nF in (8, 3):
    exact = False
    rng = np.random.default_rng(108)
    ne = E_TOP + ND_PROD + 6
    hs = rng.normal(size=(nF, ne, 64)); adH = rng.normal(size=(nF * nF, 8, 8)); adT = rng.normal(size=(nF * nF, 8, 8))
    HAg, bAg, HSg, bSg, out = run_gpu(hs, adH, adT, nF, exact)
    HA, bA, HS, bS = reference_stitch(hs, adH, adT, nF, exact)
    ixs = [slice(0, 4)] + [slice(4 + 8 * f, 12 + 8 * f) for f in range(nF)]
    for name, G, R in (("HA", HAg, HA), ("HSC", HSg, HS)):
        M = np.zeros((nF + 1, nF + 1))
        for i in range(nF + 1):
            for j in range(nF + 1):
                M[i, j] = np.abs(G[ixs[i], ixs[j]] - R[ixs[i], ixs[j]]).max() / (np.abs(R[ixs[i], ixs[j]]).max() + 1e-300)
        print(nF, name)
        print(np.array2string(M, precision=1, max_line_width=200))
    print("bA", np.abs(bAg - bA).max(), "bS", np.abs(bSg - bS).max())
    # exchange test: does G(f,g) equal the reference with adjoint roles permuted?
    A, D, E, EB, Hcc, bc = decode(hs, nF, exact)
    f, g = 0, 1
    Gb = HAg[4:12, 12:20]
    aHfg, aTfg, aHgf, aTgf = adH[f + nF * g], adT[f + nF * g], adH[g + nF * f], adT[g + nF * f]
    Afg, Agf = A[f, g][4:12, 4:12], A[g, f][4:12, 4:12]
    tries = {}
    for n1, L1 in (("aHfg", aHfg), ("aTfg", aTfg), ("aHgf", aHgf), ("aTgf", aTgf)):
        for n2, R1 in (("aHfg", aHfg), ("aTfg", aTfg), ("aHgf", aHgf), ("aTgf", aTgf)):
            for na, Am in (("Afg", Afg), ("Agf", Agf)):
                tries[f"{n1} {na} {n2}^T"] = L1 @ Am @ R1.T
    ks = list(tries)
    for k1 in ks:
        for k2 in ks:
            for tr in (False, True):
                v = tries[k1] + (tries[k2].T if tr else tries[k2])
                e = np.abs(Gb - v).max() / np.abs(v).max()
                if e < 1e-9:
                    print("MATCH", k1, "+", k2, "T" if tr else "")
