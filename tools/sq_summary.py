"""Per-kernel means of the SQ counters in a rocprofv3 --pmc run directory (tuning aid).

    python tools/sq_summary.py <rocprofv3 -d dir> [name-substring ...]
"""
import collections
import csv
import glob
import re
import sys


def main():
    d, keys = sys.argv[1], sys.argv[2:]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("swh::(anonymous namespace)::", ""))
                if keys and not any(s in k for s in keys):
                    continue
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(agg.items()):
        print(k[:60], " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))


if __name__ == "__main__":
    main()
