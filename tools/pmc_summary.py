"""Summarise the FETCH_SIZE / WRITE_SIZE rocprofv3 passes of tools/gae_pmc.py into per-launch HBM bytes
(gfx950 corrections from MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB and reports half of the bytes
of a wide coalesced streaming read -> x2; WRITE_SIZE is exact for 16-B/lane stores)."""
import csv
import glob
import json
import sys
from collections import defaultdict


def per_kernel(pass_dir, counter):
    vals = defaultdict(list)
    for f in glob.glob(pass_dir + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if r.get("Counter_Name") != counter or ("gae_scan" not in name and "gae_dpp" not in name):
                continue
            grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
            targs = name[name.index("<") + 1:name.index(">")] if "<" in name else ""
            parts = [x.strip() for x in targs.split(",")]
            # gae_dpp_kernel<SEG, COMPACT, VACT>: VACT >= 0 = the value-fused form (-1 = none)
            if len(parts) == 3 and parts[2] != "-1":
                form = "value"
            else:
                form = "compact" if len(parts) >= 2 and parts[1] == "1" else "dense"
            vals["%s/%d" % (form, grid)].append(float(r["Counter_Value"]))
    return vals


def main(fetch_dir, write_dir, out):
    fetch, write = per_kernel(fetch_dir, "FETCH_SIZE"), per_kernel(write_dir, "WRITE_SIZE")
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), KiB x 1024, FETCH x2 (gfx950)",
           "launches": {}}
    for grid in sorted(set(fetch) | set(write)):  # key = form/grid
        f = sorted(fetch.get(grid, [0]))[len(fetch.get(grid, [0])) // 2] * 1024 * 2
        w = sorted(write.get(grid, [0]))[len(write.get(grid, [0])) // 2] * 1024
        res["launches"][str(grid)] = {"fetch_bytes": f, "write_bytes": w, "hbm_bytes": f + w}
    for form in ("compact", "value"):
        keys = sorted((k for k in res["launches"] if k.startswith(form + "/")), key=lambda k: int(k.split("/")[1]))
        if keys:   # the bench size (4096 x 128) and the largest measured
            res["hbm_bytes_per_launch_" + form] = res["launches"][keys[0]]["hbm_bytes"]
            res["hbm_bytes_per_launch_%s_largest" % form] = res["launches"][keys[-1]]["hbm_bytes"]
    res["hbm_bytes_per_launch"] = res.get("hbm_bytes_per_launch_value", res.get("hbm_bytes_per_launch_compact"))
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
