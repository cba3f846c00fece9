"""Cut a rocprofv3 kernel trace of tools/gae_probe into its phases and summarise the measured kernel.

    python tools/gae_probe_summary.py <kernel_trace.csv> <probe stdout json> [out.json]

Every phase starts with one `phase_marker` dispatch; the measured kernel of a phase is the one that is
not produce / fill / marker.  Prints per phase: rocprof mean / median / min duration (first 3 launches
dropped, as the probe's own event timer does) next to the probe's event-timed median."""
import csv
import json
import statistics
import sys

SKIP = ("phase_marker", "produce_kernel", "fill_kernel")


def main(trace, probe_json, out=None):
    probe = json.load(open(probe_json))
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    phases, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "phase_marker" in name:
            cur = []
            phases.append(cur)
            continue
        if cur is None or any(s in name for s in SKIP):
            continue
        cur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    alg = probe["algorithmic_bytes"]
    res = []
    for meta, d in zip(probe["phases"], phases):
        d = d[3:]
        med = statistics.median(d)
        res.append({"phase": meta["phase"], "rocprof_us_mean": round(statistics.mean(d), 3),
                    "rocprof_us_median": round(med, 3), "rocprof_us_min": round(min(d), 3),
                    "event_us_median": meta["event_us_median"], "alg_TBps_at_rocprof_median": round(alg / med * 1e-6, 3),
                    "frac_of_8TBps": round(alg / med * 1e-6 / 8.0, 3)})
        print(f"{meta['phase']:24s} rocprof med {med:7.3f} min {min(d):7.3f} us | event med "
              f"{meta['event_us_median']:7.3f} us | {alg / med * 1e-6:5.2f} TB/s alg")
    if out:
        json.dump({"n_envs": probe["n_envs"], "horizon": probe["horizon"], "algorithmic_bytes": alg, "phases": res},
                  open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
