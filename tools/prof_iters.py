"""Per-Lloyd-iteration kernel time breakdown from a rocprofv3 rocpd database
(iterations are delimited by k_prepare launches).

  python tools/prof_iters.py gpurun_out/<dir>/run_results.db
"""
import collections
import re
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end from kernels order by start")
    it, t0 = -1, {}
    per = collections.defaultdict(collections.Counter)
    last_end = None
    for name, s, e in rows:
        m = re.search(r"\b(k_\w+|__amd\w+|\w+_kernel)", name)
        short = m.group(1) if m else name[:20]
        if short == "k_prepare":
            it += 1
            t0[it] = s
            if last_end is not None and it > 0:
                # GPU idle between the iterations (host sync + launches)
                per[it - 1]["GAP_NEXT"] = (s - crit_end) / 1e6
        per[it][short] += (e - s) / 1e6
        per[it]["BUSY"] += (e - s) / 1e6
        if short == "k_criterion":
            per[it]["WALL"] = (e - t0[it]) / 1e6
            crit_end = e
        last_end = e
    for i in sorted(per):
        if i < 0:
            continue
        items = sorted(per[i].items(), key=lambda x: -x[1])
        print(i, " ".join("%s=%.2f" % kv for kv in items if kv[1] > 0.05))


if __name__ == "__main__":
    main(sys.argv[1])
