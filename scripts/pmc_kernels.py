"""Per-kernel average of every counter in rocprofv3 --pmc output directories, with the HBM byte
corrections of MI355X_MICROARCH.md (FETCH_SIZE: KiB, half-counted for wide reads -> x 2048 B;
WRITE_SIZE: KiB -> x 1024 B).

  python3 scripts/pmc_kernels.py DIR [DIR ...]
"""
import collections
import csv
import glob
import os
import re
import sys


def kname(s):
    s = re.sub(r"\(.*", "", s.replace("(anonymous namespace)::", "")).replace("void ", "").replace("sdb::", "")
    return re.sub(r"<.*", "", s).strip()


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                acc[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(acc):
        if not k.startswith("k_"):
            continue
        row = {c: sum(v) / len(v) for c, v in acc[k].items()}
        extra = ""
        if "FETCH_SIZE" in row:
            extra += " read %.1f MB" % (row["FETCH_SIZE"] * 2048 / 1e6)
        if "WRITE_SIZE" in row:
            extra += " write %.1f MB" % (row["WRITE_SIZE"] * 1024 / 1e6)
        print("%-20s %s%s" % (k, {c: round(v) for c, v in sorted(row.items())}, extra))


if __name__ == "__main__":
    main()
