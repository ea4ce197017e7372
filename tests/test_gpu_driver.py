"""BASELINE configs[0] plumbing: the k-means driver (the drop-in for the
reference's examples/kmeans-driver.py) on the C1 input written as CSV, then
the loaded Dataset fitted with the seeded C1 KMeans against the reference's
own golden vectors (tests/golden/f16_c1full.npz, gen_golden_big.py)."""
import contextlib
import io
import os
import sys

import numpy as np
import pytest
from sklearn.datasets import make_blobs

from tests.conftest import load_golden

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_driver_c1_csv_round_trip_and_reference_fit(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import kmeans_driver
    from dislib_amd.cluster import KMeans
    path = str(tmp_path / "c1.csv")
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        km, ds = kmeans_driver.main(["--make-blobs", "100000", "-f", "50",
                                     "-c", "10", "-p", "10000", "-i", "10",
                                     "-dt", "--dense", path])
    last = out.getvalue().strip().splitlines()[-1]
    vals = eval(last, {})              # the reference's printed list
    assert vals[:3] == [10, 50, 10000] and len(vals) == 5
    assert vals[3] > 0 and vals[4] > 0
    assert "Convergence crit." in out.getvalue()      # verbose=True
    assert len(ds) == 10 and km.n_iter <= 10
    # the CSV round trip is exact (%.17g) and the labels column was split off
    x, y = make_blobs(n_samples=100_000, n_features=50, centers=10,
                      random_state=0)
    assert np.array_equal(ds.samples, x)
    assert np.array_equal(ds.labels.astype(np.int64), y)
    # the loaded Dataset under the C1 seed reproduces the reference fit
    g = load_golden("f16_c1full")
    km2 = KMeans(n_clusters=10, max_iter=10, tol=1e-4, arity=50,
                 random_state=0)
    km2.fit_predict(ds)
    assert km2.n_iter == int(g["n_iter"])
    assert np.array_equal(ds.labels_int32(), g["labels"].astype(np.int32))
    err = np.max(np.abs(km2.centers - g["centers"]) /
                 np.maximum(np.abs(g["centers"]), 1.0))
    assert err <= 1e-9
