"""Failure guards of the BA context (round 6):

* the adjoint stamp (HS_ADJ_STAMP, hs_kernels.h): hs_k_fix_frames stamps every upload of the frame adjoints with a
  sequence number and the launches that read them (hs_k_stitch: fp64, hs_k_solve: fp32) compare it with the last
  upload the host enqueued.  A stale set -- adjoints that never arrived, or a zero fill landing after them, the
  round-5 "every frame row of H zero" failure -- returns HS_ERR_STATE instead of a wrong system;
* the bounded wait of a multi-rank context (wait_stream, hs_ba.cpp): a collective that does not finish within the
  communicator timeout aborts the communicator and returns HS_ERR_RCCL (the reference's isLost path,
  Src/FullSystemOptimize.cpp:512-516; SURVEY §5 "RCCL errors are mapped to status codes") instead of hanging.
"""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HS_ERR_RCCL, HS_ERR_STATE = -3, -5


def _rc(exc):
    return int(str(exc).split("(")[1].split(")")[0])


def test_fresh_contexts_have_their_adjoints(scene_small):
    """Fresh contexts in a row, each allocating (and zero-filling) its buffers before the first adjoint upload: the
    zero fills are ordered on the context's stream (dalloc), so every context's first linearization has the full
    system -- the frame rows of H nonzero and bit-equal across contexts (the stamp check passes)."""
    from hslam_amd.ba import BAWindow
    ref = None
    for _ in range(12):
        g = BAWindow(scene_small)
        g.linearizeAll(reset=True)
        H, b = g.system(0)
        g.close()
        rows = np.abs(H[4:, :]).sum(axis=1)
        assert np.all(rows > 0), f"zero frame rows: {np.where(rows == 0)[0] + 4}"
        if ref is None:
            ref = (H, b)
        else:
            assert np.array_equal(H, ref[0]) and np.array_equal(b, ref[1])


def test_stale_fp64_adjoints_are_reported(scene_small):
    """A zero fill of the fp64 adjoints (stamp included) after the upload: the stitch's stamp check makes
    linearizeAll and the GN loop return HS_ERR_STATE; a new upload (hs_ba_set_window) clears it."""
    from hslam_amd._lib import HsError
    from hslam_amd.ba import BAWindow
    g = BAWindow(scene_small)
    e_good = g.linearizeAll(reset=True)
    assert g.lib.hs_debug_stale_adjoints(g.h, 0) == 0
    with pytest.raises(HsError) as ei:
        g.linearizeAll(reset=True)
    assert _rc(ei.value) == HS_ERR_STATE and "stale" in str(ei.value)
    with pytest.raises(HsError) as ei:
        g.iterate(0, 2)
    assert _rc(ei.value) == HS_ERR_STATE
    g._set_window(scene_small, None)  # a new upload: new stamp, status cleared
    assert g.linearizeAll(reset=True) == e_good
    g.iterate(0, 2)
    g.close()


def test_stale_fp32_adjoints_are_reported_by_the_solve(scene_small):
    """A zero fill of the fp32 adjoints (what the solve's xAd and the fused point step read): the linearization's
    system is still right (the stitch reads fp64), the solve's stamp check returns HS_ERR_STATE."""
    from hslam_amd._lib import HsError
    from hslam_amd.ba import BAWindow
    g = BAWindow(scene_small)
    g.linearizeAll(reset=True)
    assert g.lib.hs_debug_stale_adjoints(g.h, 1) == 0
    g.linearizeAll(reset=True)
    with pytest.raises(HsError) as ei:
        g.iterate(0, 1)
    assert _rc(ei.value) == HS_ERR_STATE
    g.close()


def test_stalled_collective_returns_rccl_error(scene_small):
    """A 1-rank RCCL context whose GN loop call is stalled after its last collective (hs_debug_stall withholds the
    done word for 4 s): with a 300 ms communicator timeout the call returns HS_ERR_RCCL well before the stall ends,
    the communicator is aborted, and every later call on the context returns HS_ERR_RCCL."""
    from hslam_amd._lib import HsError
    from hslam_amd.ba import BAWindow
    uid = BAWindow.comm_unique_id()
    g = BAWindow(scene_small, comm=(uid, 0, 1))
    assert g.lib.hs_comm_set_timeout(g.h, 300) == 0
    g.linearizeAll(reset=True)
    g.iterate(0, 1)  # the multi-rank path runs normally within the bound
    assert g.lib.hs_debug_stall(g.h, 4000) == 0
    t0 = time.monotonic()
    with pytest.raises(HsError) as ei:
        g.iterate(1, 1)
    dt = time.monotonic() - t0
    assert _rc(ei.value) == HS_ERR_RCCL and "did not complete" in str(ei.value)
    assert dt < 2.5, f"the bounded wait took {dt:.2f} s"
    with pytest.raises(HsError) as ei:
        g.linearizeAll()
    assert _rc(ei.value) == HS_ERR_RCCL
    g.close()  # waits for the (bounded) stall kernel to exit
