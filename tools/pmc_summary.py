"""Summarise rocprofv3 --pmc CSVs: per-counter mean per dispatch of a kernel."""
import csv, glob, sys, collections
kern = sys.argv[2] if len(sys.argv) > 2 else "url_plan_kernel"
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if kern in row.get("Kernel_Name", ""):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:28s} mean/dispatch {sum(v)/len(v):16.1f}  (n={len(v)})")
