"""Top kernels of a rocprofv3 --kernel-trace CSV: python tools/kt_top.py <kernel_trace.csv> [n] [skip_first_frac]"""
import collections
import csv
import re
import sys


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)[:100]


def main(path, n=25):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    tot, cnt = collections.Counter(), collections.Counter()
    for r in rows:
        k = short(r["Kernel_Name"])
        tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[k] += 1
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    print("kernels %d, busy %.1f ms, span %.1f ms" % (len(rows), sum(tot.values()) / 1e3, span / 1e3))
    for k, v in tot.most_common(n):
        print("%10.1f us %6d x %8.1f us  %s" % (v, cnt[k], v / cnt[k], k))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
