"""Summarise rocprofv3 counter CSVs: per kernel, average per dispatch of each counter."""
import csv, collections, glob, re, sys
for d in sys.argv[1:]:
    for f in sorted(glob.glob(d + "/**/*counter_collection.csv", recursive=True)):
        agg = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            m = re.findall(r"(\w+)(<[^()]*>)?\(", r["Kernel_Name"].replace("(anonymous namespace)", "anon"))
            k = (m[0][0] + m[0][1])[:60] if m else r["Kernel_Name"][:60]
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
        for (k, c), v in sorted(agg.items()):
            print(f"{k:60s} {c:24s} {v / len(disp[k]):16.4g}")
