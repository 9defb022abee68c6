"""ORACLE -- TEST INFRASTRUCTURE ONLY (tests/ import it; no product path does).

System::AddKeyframe's BA part (Src/Mapping.cpp:12-140) run on the CPU restatement alone, from its OWN state from
keyframe to keyframe: the window's frames (evalPT / state / state_zero / frameEnergyTH), the calibration, every point's
idepth / maxRelBaseline / numGoodResiduals and residual list, the lastResiduals bookkeeping and the marginal prior
HM / bM that its own marginalizePointsF / marginalizeFrame (Src/EnergyFunctional.cpp:456-609) leave.  The System-level
decisions are the ones hslam_amd.keyframe.KeyframeBA makes on the library's outputs (same frame policy, same
flagPointsForRemoval tests), taken here on the oracle's outputs -- so a drift of the library over a keyframe sequence
shows against it (tests/test_gpu_window.py::test_keyframe_sequence_drift_vs_oracle).

Per keyframe an OracleBA is built from the carried window (EnergyFunctional::makeIDX's order: frames in window order,
each frame's points in list order, each point's residuals in list order) and runs optimize(6) + the tail; its outputs
become the carried state.  Points are keyed by (host keyframe, candidate index), the library driver's cand_of.
"""
from __future__ import annotations

import types

import numpy as np

from oracle_ffi import OracleBA

RES_IN, RES_OOB, RES_OUT = 0, 1, 2
MIN_GOOD_ACTIVE_RES_FOR_MARG = 3   # setting_minGoodActiveResForMarg (Src/Settings.cpp:96)
MIN_GOOD_RES_FOR_MARG = 4          # setting_minGoodResForMarg (:97)
MIN_IDEPTH_H_MARG = 50.0           # setting_minIdepthH_marg (:119)


class OracleKeyframeBA:
    def __init__(self, seq, window: int = 8, iters: int = 6, params=None):
        from hslam_amd.keyframe import in_bounds_targets  # the synthetic sequence's activation rule (input data)
        self._in_bounds = in_bounds_targets
        self.seq, self.window, self.iters, self.params = seq, window, iters, params
        self.frames = []      # sequence indices, window order
        self.F = {}           # k -> dict(eval, state, state_zero, energyTH)
        self.calib = None     # CalibHessian::value (unscaled) once an optimize ran; None: the sequence's K
        self.plist = {}       # host k -> [point key] (the frame's point list)
        self.P = {}           # key -> dict(idepth, idepth_zero, relBL, nGood, res=[target k])
        self.last = {}        # key -> [lastResiduals[0].second, [1].second]
        self.HM = np.zeros((4, 4))
        self.bM = np.zeros(4)
        self.history = []

    # ---------------------------------------------------------------- window edits
    def _insert_frame(self, k):
        self.frames.append(k)
        self.F[k] = dict(eval=np.array(self.seq.evals[k], np.float64), state=np.zeros(10), state_zero=np.zeros(10),
                         energyTH=np.float32(8 * 8 * 8))
        self.plist[k] = []
        n = self.HM.shape[0]  # EnergyFunctional::insertFrame: HM / bM grow by 8 zero rows / columns
        HM = np.zeros((n + 8, n + 8))
        HM[:n, :n] = self.HM
        self.HM, self.bM = HM, np.concatenate([self.bM, np.zeros(8)])

    def _activate(self, host_k):
        c = self.seq.cand[host_k]
        ok = self._in_bounds(self.seq, host_k, self.frames, c["u"], c["v"], c["idepth"])
        newest, second = len(self.frames) - 1, len(self.frames) - 2
        for i in np.nonzero(ok.sum(1) > 0)[0]:
            key = (host_k, int(i))
            self.P[key] = dict(idepth=np.float32(c["idepth"][i]), idepth_zero=np.float32(c["idepth"][i]),
                               relBL=np.float32(0), nGood=0, res=[self.frames[t] for t in np.nonzero(ok[i])[0]])
            self.plist[host_k].append(key)
            self.last[key] = [RES_IN if ok[i, newest] else RES_OOB, RES_IN if second >= 0 and ok[i, second] else RES_OOB]

    def _keys(self):
        return [key for k in self.frames for key in self.plist[k]]

    def _oracle(self):
        """An OracleBA of the carried window (makeIDX order) with its calibration and marginal prior."""
        s, fi = self.seq, {k: j for j, k in enumerate(self.frames)}
        keys = self._keys()
        rp, rt = [], []
        for j, key in enumerate(keys):
            for t in self.P[key]["res"]:
                rp.append(j)
                rt.append(fi[t])
        c = lambda key, f: s.cand[key[0]][f][key[1]]  # noqa: E731
        nF = len(self.frames)
        sc = types.SimpleNamespace(
            width=s.width, height=s.height, K=s.K, n_levels=s.n_levels, n_frames=nF,
            frames_eval=np.array([self.F[k]["eval"] for k in self.frames]),
            frames_state=np.array([self.F[k]["state"] for k in self.frames]),
            frames_state_zero=np.array([self.F[k]["state_zero"] for k in self.frames]),
            frames_exposure=np.ones(nF, np.float32),
            frames_energyTH=np.array([self.F[k]["energyTH"] for k in self.frames], np.float32),
            frames_id=np.array(self.frames, np.int32), pyramids=[[s.pyr0[k]] for k in self.frames],
            pt_host=np.array([fi[key[0]] for key in keys], np.int32),
            pt_u=np.array([c(key, "u") for key in keys], np.float32),
            pt_v=np.array([c(key, "v") for key in keys], np.float32),
            pt_idepth=np.array([self.P[key]["idepth"] for key in keys], np.float32),
            pt_idepth_zero=np.array([self.P[key]["idepth_zero"] for key in keys], np.float32),
            pt_color=np.array([c(key, "color") for key in keys], np.float32).reshape(-1, 8),
            pt_weights=np.array([c(key, "weights") for key in keys], np.float32).reshape(-1, 8),
            res_point=np.array(rp, np.int32), res_target=np.array(rt, np.int32), n_points=len(keys), n_res=len(rp))
        o = OracleBA(sc, params=self.params)
        if self.calib is not None:
            o.set_calib(self.calib)
        o.set_marginal_prior(self.HM, self.bM)
        return o, keys, np.array(rp, np.int32), np.array(rt, np.int32)

    def _remove_points(self, gone):
        for key in gone:
            self.plist[key[0]].remove(key)
            self.P.pop(key)
            self.last.pop(key, None)

    # ---------------------------------------------------------------- the sequence
    def bootstrap(self, n_frames=None):
        n = n_frames or self.window - 1
        for k in range(n):
            self._insert_frame(k)
        for k in range(n - 1):
            self._activate(k)

    def add_keyframe(self, k, marginalize=True):
        self._insert_frame(k)
        for f in self.frames[:-1]:  # addResidualsToNewest
            for key in self.plist[f]:
                self.P[key]["res"].append(k)
        for st in self.last.values():
            st[1], st[0] = st[0], RES_IN
        self._activate(self.frames[-2])
        o, keys, rp, rt = self._oracle()
        n_it, energies = o.optimize(self.iters)
        hdif = o.points()["HdiF"].copy()  # the last solve's Schur prelude
        relBL = np.array([self.P[key]["relBL"] for key in keys], np.float32)
        nGood = np.array([self.P[key]["nGood"] for key in keys], np.int32)
        e_tail, drop, relBL, nGood = o.fix_linearization(relBL, nGood)
        fr, fe, pts, res = o.frames(), o.frame_eval(), o.points(), o.residuals()
        for j, f in enumerate(self.frames):
            self.F[f].update(eval=fe["evalPT"][j].copy(), state=fr["state"][j].copy(),
                             state_zero=fe["state_zero"][j].copy(), energyTH=fr["energyTH"][j])
        self.calib = fr["calib"].copy()
        for j, key in enumerate(keys):  # idepth_zero = idepth after every GN step (Src/FullSystemOptimize.cpp:230)
            self.P[key].update(idepth=pts["idepth"][j], idepth_zero=pts["idepth"][j], relBL=relBL[j], nGood=int(nGood[j]))
        newest, second = len(self.frames) - 1, len(self.frames) - 2
        for r in np.nonzero((rt == newest) | (rt == second))[0]:
            self.last[keys[rp[r]]][0 if rt[r] == newest else 1] = int(res["state"][r])
        # linearizeAll(true)'s toRemove, removeOutliers
        for r in np.nonzero(drop)[0]:
            self.P[keys[rp[r]]]["res"].remove(self.frames[rt[r]])
        hdif_of = {key: float(hdif[j]) for j, key in enumerate(keys)}
        info = dict(energies=energies, iters=n_it, tail_energy=e_tail, n_points=len(keys))
        self._remove_points([key for key in keys if not self.P[key]["res"]])
        if marginalize and len(self.frames) >= self.window:  # flagPointsForRemoval (Src/Mapping.cpp:248-328)
            marg_k = self.frames[0]
            keys = self._keys()
            nres = np.array([len(self.P[key]["res"]) for key in keys])
            vis = np.array([sum(t == marg_k for t in self.P[key]["res"]) for key in keys])
            last0 = np.array([self.last[key][0] for key in keys])
            last1 = np.array([self.last[key][1] for key in keys])
            ng = np.array([self.P[key]["nGood"] for key in keys])
            host = np.array([key[0] for key in keys])
            idepth = np.array([self.P[key]["idepth"] for key in keys])
            oob = ((nres >= MIN_GOOD_ACTIVE_RES_FOR_MARG) & (ng > MIN_GOOD_RES_FOR_MARG + 10) &
                   (nres - vis < MIN_GOOD_ACTIVE_RES_FOR_MARG))
            oob |= last0 == RES_OOB
            oob |= (nres >= 2) & (last0 == RES_OUT) & (last1 == RES_OUT)
            flag = oob | (host == marg_k)
            drop_now = (idepth < 0) | (nres == 0)
            inl = (nres >= MIN_GOOD_ACTIVE_RES_FOR_MARG) & (ng >= MIN_GOOD_RES_FOR_MARG)
            hd = np.array([hdif_of[key] for key in keys])
            with np.errstate(divide="ignore"):
                idepth_h = np.where(hd > 0, 1.0 / hd, 0.0)
            marg = flag & ~drop_now & inl & (idepth_h > MIN_IDEPTH_H_MARG)
            dropp = drop_now | (flag & ~marg)
            o2, _, _, _ = self._oracle()
            if marg.any():
                self.HM, self.bM = o2.marginalize_points(np.nonzero(marg)[0].astype(np.int32))
            self._remove_points([key for j, key in enumerate(keys) if marg[j] or dropp[j]])
            o2.set_marginal_prior(self.HM, self.bM)
            self.HM, self.bM = o2.marginalize_frame(0)
            self.frames.pop(0)
            for key in self._keys():  # marginalizeFrame drops the residuals into the frame (FullSystemMarginalize:108-176)
                self.P[key]["res"] = [t for t in self.P[key]["res"] if t != marg_k]
            self.F.pop(marg_k)
            self.plist.pop(marg_k)
            info.update(marginalized_points=int(marg.sum()), dropped=int(dropp.sum()))
        self.history.append(info)
        return info

    def frame_states(self):
        return dict(state=np.array([self.F[k]["state"] for k in self.frames]),
                    eval=np.array([self.F[k]["eval"] for k in self.frames]),
                    calib=None if self.calib is None else self.calib.copy())

    def point_idepth(self):
        return {key: float(self.P[key]["idepth"]) for key in self._keys()}
