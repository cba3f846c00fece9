"""Per-kernel HBM bytes per dispatch of the C2 update from tools/r06_update_pmc.sh's fetch / write passes, with the
gfx950 corrections of MI355X_MICROARCH.md §HBM (FETCH_SIZE / WRITE_SIZE in KiB; FETCH_SIZE reports half of a wide 16-B
per lane streaming read -> x2; other access widths uncalibrated, so the raw KiB figures stay beside the corrected ones).

    python tools/pmc_update_hbm.py gpurun_out/<tag>_fetch.json gpurun_out/<tag>_write.json out.json"""
import json
import sys


def main(fetch_json, write_json, out):
    f = json.load(open(fetch_json))["kernels"]
    w = json.load(open(write_json))["kernels"]
    res = {"method": "rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE (separate passes) over bench.py --steps 1 --warmup 1 (C2); "
                     "per-dispatch means; fetch_bytes_x2 = FETCH_SIZE KiB x 1024 x 2 (gfx950, exact for 16-B streaming "
                     "reads only)", "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fk, wk = f.get(k, {}).get("FETCH_SIZE"), w.get(k, {}).get("WRITE_SIZE")
        res["kernels"][k] = {"fetch_kib_raw": fk, "fetch_bytes_x2": None if fk is None else round(fk * 2048),
                             "write_bytes": None if wk is None else round(wk * 1024),
                             "dispatches": f.get(k, w.get(k, {})).get("dispatches")}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["kernels"], indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
