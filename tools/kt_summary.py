"""Per-kernel duration summary of a rocprofv3 kernel trace in its rocpd SQLite form (`*_results.db`).

    python tools/kt_summary.py gpurun_out/gm/gm_results.db [name-substring ...]

Prints calls / mean / median / min / max per kernel name (first 60 characters), in trace order of first
appearance; with substrings, only the kernels whose name contains one of them.
"""
import sqlite3
import statistics
import sys


def summary(db, only=()):
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    out = {}
    for name, s, e in rows:
        if only and not any(o in name for o in only):
            continue
        out.setdefault(name, []).append((e - s) / 1e3)
    return out


if __name__ == "__main__":
    res = summary(sys.argv[1], sys.argv[2:])
    for name, d in res.items():
        print(f"{name[:60]:60s} n={len(d):4d} mean={statistics.mean(d):8.3f} med={statistics.median(d):8.3f} "
              f"min={min(d):8.3f} max={max(d):8.3f} us")
