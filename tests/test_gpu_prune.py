"""GPU parity of the bound-based skipping (dkm_assign_pruned_f64,
dkm_prune.hip + k_screen_b2's bounds mode) against the oracle's restatement
of the reference assignment (dislib cluster/kmeans/base.py:171-173).

* the bounds themselves: after every call, for every sample, the stored
  upper bound is >= its exact distance to its label and the lower bound is
  <= its exact distance to every other centre;
* labels after each call equal the oracle's, on centre sequences built to
  break a careless bound: small drifts, one centre jumping far, a centre
  moved onto another (an exact tie: first index wins), centres jumping into
  a cluster, and samples with no label yet;
* whole fits with pruning on match the oracle (labels bit-exact, centres
  1e-9, n_iter) and the unpruned fit, and skip most samples late in the fit.
"""
import numpy as np
import pytest

from oracle import kmeans_oracle as orc

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


class _Pruned:
    """Direct driver of dkm_assign_pruned_f64 on one dataset."""

    def __init__(self, x, k, image=True):
        from dislib_amd import _device
        from dislib_amd.data import load_data
        self.dev = torch.device("cuda", 0)
        self.x = x
        self.dd = load_data(x, subset_size=x.shape[0])._device_data()
        self.k, self.d = k, x.shape[1]
        self.ws = _device.Workspace(k, self.d, self.dd.n, self.dev)
        self.st = _device.PruneState(self.dd, k)
        if not image:
            self.dd._image_failed = {1, 2}
        self.lab = torch.full((self.dd.n,), -1, dtype=torch.int32,
                              device=self.dev)
        self.Cp = torch.zeros((k, self.d), dtype=torch.float64,
                              device=self.dev)

    def step(self, C):
        from dislib_amd import _device
        Ct = torch.from_numpy(np.ascontiguousarray(C)).to(self.dev)
        acc = torch.zeros(self.k * (self.d + 1), dtype=torch.float64,
                          device=self.dev)
        _device.prepare(Ct, self.ws, acc)
        old = self.lab.cpu().numpy().copy()
        na = _device.assign_pruned(self.dd, Ct, self.Cp, self.ws, self.lab,
                                   acc, self.st)
        self.Cp.copy_(Ct)
        return na, old, self.lab.cpu().numpy(), acc.cpu().numpy()

    def bounds(self):
        n = self.dd.n
        raw = self.st.buf[:8 * n].cpu().numpy().view(np.float32)
        return raw[0::2].astype(np.float64), raw[1::2].astype(np.float64)


def _check_bounds(pr, C):
    u, l = pr.bounds()
    lab = pr.lab.cpu().numpy()
    D = _dist(pr.x, C)
    own = D[np.arange(len(lab)), lab]
    D2 = D.copy()
    D2[np.arange(len(lab)), lab] = np.inf
    other = D2.min(1)
    assert np.all(u >= own * (1 - 1e-12)), np.max(own - u)
    assert np.all(l <= other * (1 + 1e-12)), np.max(l - other)


def _dist(x, C):
    """Distances by direct differences (no expansion cancellation)."""
    out = np.empty((x.shape[0], C.shape[0]))
    for a in range(0, x.shape[0], 1000):
        t = x[a:a + 1000, None, :] - C[None, :, :]
        out[a:a + 1000] = np.sqrt((t * t).sum(-1))
    return out


def _delta_ok(x, old, new, acc, k, d):
    ps = np.zeros((k, d))
    pc = np.zeros(k)
    mv = old != new
    for lab, sgn in ((new, 1.0), (old, -1.0)):
        m = mv & (lab >= 0)
        np.add.at(ps, lab[m], sgn * x[m])
        np.add.at(pc, lab[m], sgn)
    assert np.array_equal(acc[k * d:], pc)
    assert np.max(np.abs(acc[:k * d].reshape(k, d) - ps)) <= 1e-9


@pytest.mark.parametrize("image", [True, False])
def test_bounds_and_labels_over_a_centre_sequence(image):
    rng = np.random.default_rng(3)
    n, d, k = 40011, 64, 300
    blobs = rng.uniform(-10, 10, (k, d))
    x = blobs[rng.integers(0, k, n)] + rng.standard_normal((n, d))
    C = blobs + 0.3 * rng.standard_normal((k, d))
    pr = _Pruned(x, k, image=image)
    seq = []
    seq.append(C.copy())                                   # init
    C1 = C + 1e-3 * rng.standard_normal((k, d))            # tiny drift
    seq.append(C1)
    seq.append(C1.copy())                                  # no move at all
    C3 = C1.copy()
    C3[7] += 25.0                                          # one far jump
    seq.append(C3)
    C4 = C3.copy()
    C4[11] = C4[40]                                        # exact duplicate
    seq.append(C4)
    C5 = C4.copy()
    C5[100:110] = x[rng.integers(0, n, 10)]                # jump into data
    seq.append(C5)
    C6 = C5 + 0.05 * rng.standard_normal((k, d))
    seq.append(C6)
    actives = []
    for t, Ct in enumerate(seq):
        na, old, new, acc = pr.step(Ct)
        actives.append(na)
        ref = orc.predict_labels(x, Ct)
        assert np.array_equal(new, ref), (t, (new != ref).sum())
        if t > 0:
            _delta_ok(x, old, new, acc, k, d)
        _check_bounds(pr, Ct)
    assert actives[0] == n
    assert actives[1] < n // 10 and actives[2] < n // 10, actives


def test_unlabelled_and_ragged_samples():
    """-1 labels are always screened; n not a multiple of 64 / 16384."""
    rng = np.random.default_rng(5)
    n, d, k = 16384 + 77, 16, 40
    x = rng.standard_normal((n, d)) * 3
    C = rng.standard_normal((k, d)) * 3
    pr = _Pruned(x, k)
    pr.step(C)
    lab = pr.lab.cpu().numpy()
    lab[rng.random(n) < 0.01] = -1
    pr.lab.copy_(torch.from_numpy(lab))
    na, old, new, acc = pr.step(C)
    assert na >= (lab < 0).sum()
    assert np.array_equal(new, orc.predict_labels(x, C))
    _check_bounds(pr, C)


@pytest.mark.parametrize("n,d,k,iters", [(60000, 64, 200, 25),
                                         (30000, 32, 100, 20),
                                         (20000, 128, 64, 15)])
def test_fit_with_pruning_matches_oracle(monkeypatch, n, d, k, iters):
    from sklearn.datasets import make_blobs

    import dislib_amd.cluster.kmeans as km_mod
    from dislib_amd.cluster import KMeans
    from dislib_amd.data import load_data
    x, _ = make_blobs(n_samples=n, n_features=d, centers=k,
                      center_box=(-10, 10), random_state=n + d)
    ref = orc.OracleKMeans(n_clusters=k, max_iter=iters, tol=0,
                           random_state=0)
    rl = ref.fit([x[i:i + 10000] for i in range(0, n, 10000)],
                 set_labels=True)
    runs = {}
    for prune in (True, False):
        monkeypatch.setattr(km_mod, "PRUNE", prune)
        ds = load_data(x, 10000)
        km = KMeans(n_clusters=k, max_iter=iters, tol=0, random_state=0)
        km.fit_predict(ds)
        assert km.n_iter == ref.n_iter
        assert np.array_equal(ds.labels_int32(), rl)
        err = np.max(np.abs(km.centers - ref.centers) /
                     np.maximum(np.abs(ref.centers), 1.0))
        assert err <= 1e-9
        runs[prune] = km.centers
    assert np.max(np.abs(runs[True] - runs[False])) <= 1e-9


def test_fit_skips_most_samples_once_settled(monkeypatch):
    from sklearn.datasets import make_blobs

    import dislib_amd.cluster.kmeans as km_mod
    from dislib_amd.data import load_data
    monkeypatch.setattr(km_mod, "PRUNE", True)
    x, _ = make_blobs(n_samples=100000, n_features=64, centers=300,
                      center_box=(-10, 10), random_state=1)
    ds = load_data(x, 25000)
    centers = km_mod._init_centers(64, False, 300, 0)
    st = km_mod._Lloyd(ds, centers, 0.0, False)
    assert st.pstate is not None
    for _ in range(15):
        st.step()
    # the first pruned call screens everything (init); late ones few
    assert st.active[0] == 100000
    assert min(st.active[-4:]) < 20000, st.active
