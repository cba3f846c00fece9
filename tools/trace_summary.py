"""Summarise a `rocprofv3 --kernel-trace --output-format csv` run of bench.py.

    python tools/trace_summary.py <run_kernel_trace.csv> <profiled bench.json> [out.json] [unprofiled bench.json]

Writes per-kernel call counts / total / average durations over the whole profiled run and the in-loop GAE
launches of the timed region (bench.py runs `warmup` then `steps` iterations, one xpa_gae_scan per
iteration, before its graph replay and flushed sweep), so the live `roofline.avg_launch_us` of
bench.py can be checked against the profiler's own durations."""
import csv
import json
import re
import sys


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:80]


def main(trace, bench, out=None, live=None):
    rows = list(csv.DictReader(open(trace)))
    b = json.load(open(bench))
    iters = b["warmup"] + b["steps"]
    # the in-loop GAE kernel bench.py names in roofline.kernel, e.g. "xpa_gae_scan_compact (gae_dpp_kernel<5, 1>)"
    m = re.search(r"\(([^()]+)\)\s*$", (b.get("roofline") or {}).get("kernel", ""))
    pat = m.group(1) if m else "gae_scan_kernel"
    gae = [r for r in rows if pat in r["Kernel_Name"]]
    gae.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in gae]
    timed = dur[b["warmup"]:iters]
    per = {}
    for r in rows:
        k = short(r["Kernel_Name"])
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c, t = per.get(k, (0, 0.0))
        per[k] = (c + 1, t + d)
    top = sorted(per.items(), key=lambda kv: -kv[1][1])[:30]
    res = {
        "bench_value": b["value"], "bench_ms_per_step": b["ms_per_step"],
        "gae_kernel": pat,
        "gae_inloop_timed_launches_us": timed,
        "gae_inloop_avg_us": sum(timed) / len(timed) if timed else None,
        "profiled_run_live_avg_launch_us": (b.get("roofline") or {}).get("avg_launch_us"),
        "unprofiled_run_live_avg_launch_us": (json.load(open(live)).get("roofline") or {}).get("avg_launch_us")
        if live else None,
        "top_kernels": [{"kernel": k, "calls": c, "total_ms": round(t / 1e3, 3), "avg_us": round(t / c, 3)}
                        for k, (c, t) in top],
        "note": "profiled run of the same bench.py command; kernel totals include warmup, the graph replay, "
                "the flushed GAE sweep and setup kernels",
    }
    s = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main(*sys.argv[1:])
