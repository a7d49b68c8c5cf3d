"""GPU: the resampler's FMA mode (ik_set_resize_mode(IK_RESIZE_FMA)) -- one fused
multiply-add per tap instead of the reference's separately rounded f32 multiply
and add.  Bar (the north star's tolerance for bilinear/Lanczos): every channel
within 1 LSB of the oracle (image 0.25.8 imageops::resize restated), nearly all
exactly equal; Nearest stays exact (weights 0/1).  The default mode stays exact."""
import numpy as np
import pytest

import ikutil
from imagekit import DynamicImage, FilterType

pytestmark = pytest.mark.gpu
IK_RESIZE_EXACT, IK_RESIZE_FMA = 0, 1

CASES = [((4096, 4096), (512, 512), 4), ((1920, 1080), (640, 360), 3), ((800, 600), (400, 300), 3),
         ((97, 61), (32, 20), 4), ((333, 222), (1000, 666), 3), ((256, 256), (32, 32), 1), ((1024, 768), (1023, 767), 4)]


@pytest.fixture
def fma(ik):
    assert ik.ik_get_resize_mode() == IK_RESIZE_EXACT
    assert ik.ik_set_resize_mode(IK_RESIZE_FMA) == 0
    yield
    assert ik.ik_set_resize_mode(IK_RESIZE_EXACT) == 0


@pytest.mark.parametrize("geom", CASES, ids=lambda g: f"{g[0][0]}x{g[0][1]}-{g[1][0]}x{g[1][1]}-c{g[2]}")
@pytest.mark.parametrize("f", [FilterType.Triangle, FilterType.Lanczos3, FilterType.CatmullRom, FilterType.Gaussian])
def test_fma_within_one_lsb(ik, oracle, fma, geom, f):
    (W, H), (nw, nh), c = geom
    src = ikutil.synth(W, H, c, seed=W + H, pattern="S" if W > 500 else "N")
    got = DynamicImage.from_array(src).resize(nw, nh, f).to_array().astype(np.int32)
    want = oracle.resize(src, nw, nh, int(f)).astype(np.int32)
    d = np.abs(got - want)
    assert d.max() <= 1
    assert (d == 0).mean() >= 0.99


def test_fma_nearest_exact_and_mode_switch(ik, oracle, fma):
    src = ikutil.synth(640, 480, 4, seed=1, pattern="N")
    got = DynamicImage.from_array(src).resize(320, 240, FilterType.Nearest).to_array()
    np.testing.assert_array_equal(got, oracle.resize(src, 320, 240, 0))
    assert ik.ik_set_resize_mode(7) != 0
    assert ik.ik_get_resize_mode() == IK_RESIZE_FMA
