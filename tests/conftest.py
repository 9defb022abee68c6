import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "h-slam_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def scene2k():
    from hslam_amd.scene import make_ba_scene
    return make_ba_scene(n_points=2000)


@pytest.fixture(scope="session")
def scene_small():
    from hslam_amd.scene import make_ba_scene
    return make_ba_scene(n_points=240, seed=7)


@pytest.fixture(scope="session")
def scene_kitti2k():
    """C5 BA (BASELINE configs[4]): 8 KF x 2000 points at KITTI 1232x368, 5 levels."""
    from hslam_amd.scene import make_ba_scene_kitti
    return make_ba_scene_kitti(2000)


@pytest.fixture(scope="session")
def scene_kitti20k():
    """C5 BA at the trace size: 8 KF x 20000 points at KITTI 1232x368."""
    from hslam_amd.scene import make_ba_scene_kitti
    return make_ba_scene_kitti(20000)


@pytest.fixture(scope="session")
def scene_marg():
    """A nearly converged small window (most residuals IN at the first linearization): marginalization tests."""
    from hslam_amd.scene import make_ba_scene
    return make_ba_scene(n_points=240, seed=7, pose_noise=(0.001, 0.0005), idepth_noise=0.002)

