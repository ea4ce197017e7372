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
    last_short = None
    gaps = collections.defaultdict(list)
    crit_end = None
    counts = collections.defaultdict(collections.Counter)
    each = collections.defaultdict(lambda: collections.defaultdict(list))
    for name, s, e in rows:
        m = re.search(r"\b(k_\w+|__amd\w+|\w+_kernel)", name)
        short = m.group(1) if m else name[:20]
        if short == "k_prepare":
            it += 1
            t0[it] = s
            if crit_end is not None and it > 0:
                # GPU idle between the iterations (host sync + launches)
                per[it - 1]["GAP_NEXT"] = (s - crit_end) / 1e6
        if last_end is not None and short != "k_prepare" and it >= 0:
            gaps[it].append(((s - last_end) / 1e6, last_short, short))
        per[it][short] += (e - s) / 1e6
        counts[it][short] += 1
        each[it][short].append((e - s) / 1e6)
        per[it]["BUSY"] += (e - s) / 1e6
        if short == "k_criterion":
            per[it]["WALL"] = (e - t0[it]) / 1e6
            crit_end = e
        last_end = e
        last_short = short
    for i in sorted(per):
        if i < 0:
            continue
        items = sorted(per[i].items(), key=lambda x: -x[1])
        def fmt(kv):
            c = counts[i][kv[0]]
            if c < 2:
                return "%s=%.2f" % kv
            if c <= 4:       # the launches themselves
                return "%s=%.2f[%s]" % (kv[0], kv[1], ",".join(
                    "%.2f" % x for x in each[i][kv[0]]))
            return "%s=%.2f/%d" % (kv[0], kv[1], c)
        print(i, " ".join(fmt(kv) for kv in items if kv[1] > 0.05))
    # the largest idle gaps inside each iteration (host work between launches)
    for i in sorted(gaps):
        big = sorted(gaps[i], reverse=True)[:3]
        big = [g for g in big if g[0] > 0.3]
        if big:
            print("  gaps", i, " ".join("%.2f(%s->%s)" % g for g in big))


if __name__ == "__main__":
    main(sys.argv[1])
