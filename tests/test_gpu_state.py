"""The compensated running [sums | counts] (dkm_add_f64_dd): after many
delta adds of mixed magnitudes the state equals the correctly rounded exact
sum (math.fsum) to within one ulp, where a plain fp64 running sum drifts by
many; and the nonzero flag reports whether any delta element was nonzero
(the refresh bookkeeping of cluster/kmeans.py)."""
import math

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_compensated_state_tracks_the_exact_sum():
    from dislib_amd import _device
    rng = np.random.default_rng(0)
    m, steps = 4096, 200
    base = rng.uniform(-1, 1, m) * 1e6
    deltas = rng.standard_normal((steps, m)) * 10.0 ** rng.integers(-8, 2,
                                                                     (steps, m))
    deltas[rng.random((steps, m)) < 0.3] = 0.0
    dev = torch.device("cuda", 0)
    hi = torch.from_numpy(base.copy()).to(dev)
    lo = torch.zeros_like(hi)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    plain = base.copy()
    for t in range(steps):
        x = torch.from_numpy(deltas[t]).to(dev)
        _device.add_dd_(hi, lo, x, flag)
        plain += deltas[t]
        assert int(flag.item()) == 1
    got = hi.cpu().numpy()
    exact = np.array([math.fsum([base[i]] + list(deltas[:, i]))
                      for i in range(m)])
    ulp = np.spacing(np.abs(exact))
    assert np.all(np.abs(got - exact) <= ulp)
    # the plain running sum is measurably worse (what the refresh bounded)
    assert np.sum(np.abs(plain - exact) > ulp) > m // 10
    # an all-zero delta: flag 0, state unchanged
    _device.add_dd_(hi, lo, torch.zeros_like(hi), flag)
    assert int(flag.item()) == 0
    assert np.array_equal(hi.cpu().numpy(), got)
