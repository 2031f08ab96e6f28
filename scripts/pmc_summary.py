"""Average rocprofv3 PMC counters per kernel over the passes in gpurun_out/pmc/p*/."""
import collections, csv, glob, re, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(root + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("sdb::", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        acc[k]["_dur_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, cs in acc.items():
    if not k.startswith("k_"):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-22s %14.1f" % (c, sum(v) / len(v)))
