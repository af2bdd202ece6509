"""Per-dispatch averages of the SQ counters collected by tools/pmc_kernel.sh.

    python tools/pmc_sum.py gpurun_out/pmck_TAG KERNEL_SUBSTRING
"""
import collections
import csv
import glob
import os
import sys


def main():
    root, kern = sys.argv[1], sys.argv[2]
    vals = {}
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        per, disp = collections.defaultdict(float), collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            if kern not in r["Kernel_Name"]:
                continue
            per[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
        for k, v in per.items():
            vals[k] = v / len(disp[k])
    w = vals.get("SQ_WAVES", 1.0)
    for k in sorted(vals):
        print(f"{k:28s} {vals[k]:16.0f} {vals[k] / w:12.1f}/wave")


if __name__ == "__main__":
    main()
