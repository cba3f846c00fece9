"""Per-kernel clock estimates from rocprofv3 --pmc GRBM_GUI_ACTIVE + --kernel-trace runs (tools/r05_clock.sh):
GHz = GRBM_GUI_ACTIVE / 8 (XCDs) / duration; mean over the dispatches of each kernel."""
import csv
import glob
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return name.split("(")[0][:60]


if __name__ == "__main__":
    for d in sys.argv[1:]:
        cyc = {}
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                    cyc[(r["Dispatch_Id"])] = (short(r["Kernel_Name"]), float(r["Counter_Value"]))
        dur = {}
        for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        acc = defaultdict(list)
        for k, (n, c) in cyc.items():
            if k in dur and dur[k] > 2e-6:
                acc[n].append((c / 8 / dur[k] / 1e9, dur[k] * 1e6))
        print("==", d)
        for n, v in sorted(acc.items(), key=lambda kv: -sum(x[1] for x in kv[1])):
            ghz = sum(x[0] for x in v) / len(v)
            us = sum(x[1] for x in v) / len(v)
            print("%-62s n=%4d  %7.1f us  %.2f GHz" % (n, len(v), us, ghz))
