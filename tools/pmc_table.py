"""Per-kernel average of every counter in a rocprofv3 --pmc
counter_collection.csv (one row per kernel dispatch x counter)."""
import collections
import csv
import sys


def table(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"].split("(")[0]
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


if __name__ == "__main__":
    for path in sys.argv[1:]:
        for k, cs in table(path).items():
            if "nsd" not in k:
                continue
            print(k)
            for c, v in sorted(cs.items()):
                print(f"   {c:28s} {v:16.0f}")
