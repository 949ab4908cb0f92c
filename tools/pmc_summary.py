"""Summarise rocprofv3 --pmc counter_collection CSVs: mean counter value per kernel name."""
import collections, csv, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sys.argv[1:]:
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"]
        if "ntcgpu" not in name:
            continue
        name = name.split("(")[0].replace("void ", "")
        agg[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, cs in agg.items():
    print(name)
    for c, v in sorted(cs.items()):
        # values are per-dispatch sums over the agent; average over dispatches
        print(f"   {c:24s} {sum(v)/len(v):16.4g}   (dispatches {len(v)})")
