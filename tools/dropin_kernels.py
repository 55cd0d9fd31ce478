"""Per-kernel summary of the last drop-in LocalBundleAdjustment call in a rocprofv3 database
(tools/lba_dropin_prof.sh output): launches and summed duration per kernel, the call's span and the
idle time between its kernels.  usage: python tools/dropin_kernels.py OUTDIR/lba_results.db"""
import collections
import sqlite3
import sys


def short(name):
    base = name.split("(")[0]
    return base.split("::")[-1]


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, start, end from kernels order by start").fetchall()
    first = "k_setup_a"
    starts = [i for i, r in enumerate(rows) if short(r[0]) == first]
    if not starts:
        sys.exit(f"no {first} dispatch in {sys.argv[1]}")
    call = rows[starts[-1]:]
    agg = collections.OrderedDict()
    for name, s, e in call:
        k = short(name)
        n, t = agg.get(k, (0, 0))
        agg[k] = (n + 1, t + (e - s))
    busy = sum(e - s for _, s, e in call)
    span = call[-1][2] - call[0][1]
    print(f"LocalBundleAdjustment drop-in call (tests/cpp/shim_driver lbatime, config-4 map), rocprofv3 kernel trace; "
          f"last of {len(starts)} calls")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:<27} {n:2d} launches {t / 1e3:9.1f} us")
    print(f"span {span / 1e3:.1f} us, idle gaps between kernels {(span - busy) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
