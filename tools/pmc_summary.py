"""Average rocprofv3 --pmc counter values per kernel over the CSVs in the given dirs."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-60:]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    if k.startswith("void at::") or "rocclr" in k:
        continue
    print(k)
    for c, xs in sorted(v.items()):
        print(f"    {c:40s} {sum(xs) / len(xs):16.1f}   (n={len(xs)})")
