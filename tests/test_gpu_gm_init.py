"""The GaussianMixture KMeans initialisation as a caller of the path
(SURVEY.md section 8 row f3): ``gm/base.py:722-732`` draws a seed from the
GM's RandomState, runs ``KMeans(n_clusters=n_components, random_state=seed,
verbose=...).fit_predict(dataset)`` and turns every Subset's labels into a
one-hot responsibility block with ``labels.astype(int)``
(``_resp_subset``, :771-777).  The same sequence over the HIP path must give
the responsibilities the oracle gives (labels bit-exact)."""
import numpy as np
import pytest
from sklearn.datasets import make_blobs

from oracle import kmeans_oracle as orc

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _resp_subset(labels, n_components):
    # gm/base.py:771-777
    n_samples = len(labels)
    resp = np.zeros((n_samples, n_components))
    resp[np.arange(n_samples), labels.astype(int)] = 1
    return resp


@pytest.mark.parametrize("n_components,prelabelled", [(3, False), (7, True)])
def test_gm_kmeans_init_sequence(n_components, prelabelled):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dislib_amd.cluster import KMeans
    from dislib_amd.data import load_data
    x, y = make_blobs(n_samples=3000, n_features=4, centers=n_components,
                      random_state=11)
    ds = load_data(x, 250, y=y.astype(float) if prelabelled else None)
    rs = np.random.RandomState(5)
    seed = rs.randint(0, int(1e8))
    km = KMeans(n_clusters=n_components, random_state=seed, verbose=False)
    km.fit_predict(ds)
    resp = [_resp_subset(s.labels, n_components) for s in ds]

    ref = orc.OracleKMeans(n_clusters=n_components, random_state=seed)
    blocks = [x[i:i + 250] for i in range(0, 3000, 250)]
    lab = ref.fit(blocks, set_labels=True)
    ref_resp = [_resp_subset(lab[i:i + 250], n_components)
                for i in range(0, 3000, 250)]
    assert km.n_iter == ref.n_iter
    for a, b in zip(resp, ref_resp):
        assert np.array_equal(a, b)
    # labels keep the pre-existing dtype when the Dataset was labelled
    # (Subset.set_label, data/classes.py:339-357)
    want = np.float64 if prelabelled else object
    assert all(s.labels.dtype == want for s in ds)
