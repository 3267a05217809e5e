"""Per-kernel mean of every PMC counter found under the given rocprofv3 output dirs.

    python scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 ...

Prints one line per (kernel, counter): mean value per dispatch (summed over the
per-XCD / per-SE instances rocprofv3 reports), and the kernel's mean duration.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    vals = defaultdict(lambda: defaultdict(float))  # (kernel, counter) -> dispatch -> sum
    durs = defaultdict(dict)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                    disp = (d, r.get("Dispatch_Id") or r.get("Correlation_Id"))
                    vals[(k, r["Counter_Name"])][disp] += float(r["Counter_Value"])
                    if r.get("End_Timestamp") and r.get("Start_Timestamp"):
                        durs[k][disp] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    for (k, c) in sorted(vals):
        dv = vals[(k, c)]
        mean = sum(dv.values()) / len(dv)
        dd = [durs[k][x] for x in dv if x in durs[k]]
        ms = sum(dd) / len(dd) if dd else float("nan")
        print(f"{k[:60]:60s} {c:28s} {mean:16.6g}  (n={len(dv)}, {ms:.3f} ms)")


if __name__ == "__main__":
    main()
