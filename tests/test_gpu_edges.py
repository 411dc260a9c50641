"""Edge cases of the klt.h path on the GPU against the CPU oracle: more
features requested than the image can hold (NOT_FOUND slots, selectGoodFeatures.c
:175-195 of _enforceMinimumDistance), an image with no candidate at all (smaller
than its borders), a one-feature list, frames where every feature gets lost,
and replacement into a list that cannot be refilled."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import synth
from kltabi import KLTRunner, OracleTracker
from test_oracle import table_eq

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("w,h,n,nframes,replace", [
    (640, 480, 6000, 5, False),   # far more than mindist allows: most slots NOT_FOUND (-1)
    (640, 480, 6000, 5, True),    # ... and REPLACE cannot refill them
    (40, 30, 10, 4, False),       # no candidate survives the 24-pixel borders
    (96, 80, 1, 6, False),        # a single feature
    (97, 61, 50, 6, True),        # odd, small frames with replacement
])
def test_edges_vs_oracle(gpu, oracle, w, h, n, nframes, replace):
    frames = synth(gpu, 9000 + w + h + n, w, h, nframes)
    got = KLTRunner(gpu).harness(frames, n, nframes, first=frames[0], replace=replace)
    want = OracleTracker(oracle).harness(frames, n, nframes, first=frames[0], replace=replace)
    assert table_eq(got, want)
    if n == 6000:
        assert (got[2][:, 0] == -1).sum() > n // 2  # NOT_FOUND slots exist and stay consistent
    if (w, h) == (40, 30):
        assert (got[2][:, 0] == -1).all()


def test_every_feature_lost(gpu, oracle):
    """A sequence that jumps to an unrelated image: features go OOB / large
    residue / small determinant, and later frames keep the lost ones lost."""
    a = synth(gpu, 111, 320, 240, 3)
    b = synth(gpu, 222, 320, 240, 3)
    frames = [a[0], a[1], np.zeros_like(a[0]), b[0], b[1]]
    got = KLTRunner(gpu).harness(frames, 200, 5, first=frames[0])
    want = OracleTracker(oracle).harness(frames, 200, 5, first=frames[0])
    assert table_eq(got, want)
    assert (got[2][:, 1] < 0).all()  # the blank frame loses every feature
