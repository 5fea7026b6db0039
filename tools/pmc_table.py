"""Average PMC counters per kernel name from rocprofv3 counter_collection.csv files."""
import collections
import csv
import sys


def load(paths, name_filter=""):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            n = r["Kernel_Name"]
            if name_filter and name_filter not in n:
                continue
            key = (n.replace("(anonymous namespace)::", "")[:70], r["Grid_Size"])
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


if __name__ == "__main__":
    flt = sys.argv[1]
    vals = load(sys.argv[2:], flt)
    for key, cs in vals.items():
        print(key)
        for c, v in sorted(cs.items()):
            print(f"   {c:32s} {sum(v)/len(v):14.1f}  (n={len(v)})")
