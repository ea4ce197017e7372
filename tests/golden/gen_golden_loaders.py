"""Golden vectors for the Dataset file loaders, produced by the REFERENCE's
own ``dislib.data.load_libsvm_file(s)`` / ``load_txt_file(s)``
(``/root/reference/dislib/data/base.py:42-238``).

Run in the development container only:
``python tests/golden/gen_golden_loaders.py`` -- like ``gen_golden.py`` it
imports the reference under the sequential PyCOMPSs stub (and the keyword
``n_features`` shim of sklearn's ``load_svmlight_file``).  Nothing of the
reference is copied: the script writes its own synthetic input files, hands
them to the reference loaders and stores inputs (file bytes) and outputs
(every Subset's samples -- CSR arrays or dense -- and labels) in
``loaders_ref.npz``.  Directory loads record the per-file outputs by file
name (the reference walks ``os.listdir`` order).
"""
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _libsvm_text(rng, n, d, one_based, extras, crlf):
    out = []
    base = 1 if one_based else 0
    for i in range(n):
        if extras and i % 13 == 4:
            out.append("# comment %d" % i)
        if extras and i % 19 == 9:
            out.append("")
        cnt = int(rng.integers(0, min(d, 9)))
        cols = sorted(rng.choice(d, cnt, replace=False)) if cnt else []
        vals = rng.standard_normal(cnt) * 10.0 ** rng.integers(-3, 4, cnt)
        feats = " ".join("%d:%r" % (c + base, float(v))
                         for c, v in zip(cols, vals))
        lab = float(rng.integers(-2, 3))
        line = ("%g %s" % (lab, feats)).rstrip()
        if extras and i % 7 == 3:
            line += "  # trailing comment"
        out.append(line)
    nl = "\r\n" if crlf else "\n"
    return (nl.join(out) + nl).encode()


def _txt_text(rng, n, d, delim, holes):
    out = []
    for i in range(n):
        vals = ["%r" % float(v) for v in rng.standard_normal(d + 1) * 100]
        if holes and i % 11 == 2:
            vals[int(rng.integers(0, d + 1))] = ""
        if holes and i % 17 == 8:
            vals[int(rng.integers(0, d + 1))] = "nan"
        out.append((delim if delim else " ").join(vals))
    return ("\n".join(out) + "\n").encode()


def cases():
    """(name, kind, file bytes or {name: bytes}, kwargs)"""
    import numpy as np
    rng = np.random.default_rng(2024)
    c = []
    c.append(("svm_one", "libsvm_file",
              _libsvm_text(rng, 230, 40, True, True, False),
              dict(subset_size=50, n_features=40)))
    c.append(("svm_zero_crlf", "libsvm_file",
              _libsvm_text(rng, 120, 25, False, True, True),
              dict(subset_size=33, n_features=25)))
    c.append(("svm_dense", "libsvm_file",
              _libsvm_text(rng, 90, 12, True, False, False),
              dict(subset_size=40, n_features=12, store_sparse=False)))
    c.append(("txt_last", "txt_file", _txt_text(rng, 150, 6, ",", True),
              dict(subset_size=40, n_features=6, delimiter=",",
                   label_col="last")))
    c.append(("txt_first_ws", "txt_file", _txt_text(rng, 77, 4, None, False),
              dict(subset_size=25, n_features=4, delimiter=None,
                   label_col="first")))
    c.append(("txt_nolabel_onerow", "txt_file",
              _txt_text(rng, 41, 3, ",", False),
              dict(subset_size=20, n_features=4, delimiter=",")))
    c.append(("svm_dir", "libsvm_files",
              {"p%d.svm" % j: _libsvm_text(rng, 30 + 7 * j, 20, True, True,
                                           False) for j in range(4)},
              dict(n_features=20)))
    c.append(("txt_dir", "txt_files",
              {"p%d.csv" % j: _txt_text(rng, 12 + 5 * j, 5, ",", True)
               for j in range(3)},
              dict(n_features=5, delimiter=",", label_col="last")))
    return c


def _subset_arrays(prefix, s, out):
    import numpy as np
    import scipy.sparse as sp
    x = s.samples
    if sp.issparse(x):
        x = x.tocsr()
        out[prefix + "indptr"] = x.indptr
        out[prefix + "indices"] = x.indices
        out[prefix + "data"] = x.data
        out[prefix + "shape"] = np.array(x.shape)
    else:
        out[prefix + "dense"] = np.asarray(x)
    out[prefix + "labels"] = np.array([]) if s.labels is None \
        else np.asarray(s.labels)
    out[prefix + "has_labels"] = np.array(s.labels is not None)


def generate():
    import numpy as np
    import dislib.data as dd
    out = {}
    work = tempfile.mkdtemp(prefix="dkm_loaders_")
    for name, kind, payload, kw in cases():
        if kind.endswith("_files"):
            p = os.path.join(work, name)
            os.makedirs(p)
            for fn, b in payload.items():
                with open(os.path.join(p, fn), "wb") as f:
                    f.write(b)
                out["%s/in/%s" % (name, fn)] = np.frombuffer(b, np.uint8)
        else:
            p = os.path.join(work, name)
            with open(p, "wb") as f:
                f.write(payload)
            out["%s/in" % name] = np.frombuffer(payload, np.uint8)
        fn = getattr(dd, "load_" + kind)
        ds = fn(p, **kw)
        names = sorted(os.listdir(p)) if kind.endswith("_files") else None
        listed = os.listdir(p) if names else None
        out["%s/n_subsets" % name] = np.array(len(ds))
        for i, s in enumerate(ds):
            key = listed[i] if names else str(i)
            _subset_arrays("%s/out/%s/" % (name, key), s, out)
        print("loaders:", name, len(ds), flush=True)
    np.savez_compressed(os.path.join(HERE, "loaders_ref.npz"), **out)
    print("wrote loaders_ref.npz")


def main():
    try:
        import dislib  # noqa: F401
        import pycompss  # noqa: F401
        ok = True
    except ImportError:
        ok = False
    if ok:
        generate()
        return
    if not os.path.isdir(REF):
        print("reference not present; golden vectors are committed -- skip")
        return
    sys.path.insert(0, HERE)
    from gen_golden import SHIM
    shim = tempfile.mkdtemp(prefix="dkm_shim_")
    for rel, body in SHIM.items():
        p = os.path.join(shim, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(body)
    env = dict(os.environ, PYTHONPATH=shim + ":" + REF,
               PYTHONDONTWRITEBYTECODE="1")
    sys.exit(subprocess.call([sys.executable, os.path.abspath(__file__)],
                             env=env, cwd=REF))


if __name__ == "__main__":
    main()
