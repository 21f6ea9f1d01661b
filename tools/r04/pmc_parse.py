"""Per-dispatch means of PMC counters over the nibble-path launches (the
k_round variant IN = 2 that did work) in rocprofv3 csv directories.
usage: pmc_parse.py <dir-glob>..."""
import csv, glob, sys, collections, json, re

out = {}
for pat in sys.argv[1:]:
    for d in sorted(glob.glob(pat)):
        files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for f in files:
            for row in csv.DictReader(open(f)):
                k = row.get("Kernel_Name", "")
                if not re.search(r"k_round<\d+, \d+, \d+, \w+, false, 2>", k):
                    continue
                per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
        # drop idle dispatches (the nibble path's early-return launches)
        vals = [v for v in per.values()]
        if not vals:
            continue
        key = max(vals[0], key=lambda c: vals[0][c])
        busy = [v for v in vals if v[key] > 0.2 * max(x[key] for x in vals)]
        names = sorted({c for v in busy for c in v})
        out[d] = {c: sum(v.get(c, 0.0) for v in busy) / len(busy) for c in names}
        out[d]["dispatches"] = len(busy)
print(json.dumps(out, indent=1))
