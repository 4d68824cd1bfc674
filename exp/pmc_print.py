"""Mean per dispatch of every counter, per kernel, from rocprofv3 counter_collection CSVs."""
import csv, os, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("honk::", "")
        if os.environ.get("PMC_FILTER", "block16") not in n:
            continue
        acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in acc.items():
    print(n)
    for c, v in sorted(cs.items()):
        print(f"  {c:28s} {sum(v) / len(v):.4g}  (n={len(v)})")
