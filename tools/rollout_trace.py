"""One C2 iteration (4096 envs x 128 steps) after warm-up, for a rocprofv3 kernel trace of the rollout:
    rocprofv3 --kernel-trace -d gpurun_out/rt -o rt -- python tools/rollout_trace.py
then python tools/rollout_trace.py summarize gpurun_out/rt/rt_results.db  (per-step timeline of the graph
replays: each kernel's duration and the gap before it)."""
import os
import sqlite3
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import torch
    from xuanpolicy_amd.runner import build_synthbox_ppo
    agent = build_synthbox_ppo(n_envs=4096, n_steps=128, seed=1, device="cuda:0")
    agent.learner.enable_fast_path()
    for _ in range(3):
        agent.train(128)
    torch.cuda.synchronize()
    torch.cuda._sleep(1000000)   # a marker gap before the traced iteration
    agent.train(128)
    torch.cuda.synchronize()


def summarize(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    # the traced iteration: after the longest gap (the sleep)
    gaps = [(rows[i][1] - rows[i - 1][2], i) for i in range(1, len(rows))]
    start = max(gaps)[1]
    it = rows[start:]
    # one rollout step = the kernels between consecutive rollout_post launches
    posts = [i for i, r in enumerate(it) if "rollout_post" in r[0]]
    steps = []
    for a, b in zip(posts[:-1], posts[1:]):
        steps.append(it[a + 1:b + 1])
    per = {}
    for st in steps[10:120]:
        prev_end = None
        for j, (n, s, e) in enumerate(st):
            key = "%02d %s" % (j, n.split("(")[0][-50:])
            d = per.setdefault(key, [[], []])
            d[0].append((e - s) / 1e3)
            d[1].append((s - prev_end) / 1e3 if prev_end else 0.0)
            prev_end = e
    tot = [(st[-1][2] - st[0][1]) / 1e3 for st in steps[10:120]]
    print("step span us: median %.1f" % statistics.median(tot))
    for k, (d, g) in sorted(per.items()):
        print("%-60s dur %6.2f  gap-before %6.2f" % (k, statistics.median(d), statistics.median(g)))
    up = [r for r in it[posts[-1] + 1:]]
    print("update phase: %d kernels, span %.1f ms" % (len(up), (up[-1][2] - up[0][1]) / 1e6 if up else 0))
    # one update = the kernels after one clip_adam launch up to the next update's last clip_adam
    ends = [i for i, r in enumerate(up) if "clip_adam" in r[0]]
    ends = ends[1::2] if len(ends) > 2 and "clip_adam" in up[ends[0] + 1][0] else ends
    per = {}
    spans = []
    for a, b in zip(ends[4:-1], ends[5:]):
        seg = up[a + 1:b + 1]
        spans.append((seg[-1][2] - seg[0][1]) / 1e3)
        prev_end = up[a][2]
        for j, (n, s_, e) in enumerate(seg):
            key = "%02d %s" % (j, n.split("(")[0][-50:])
            d = per.setdefault(key, [[], []])
            d[0].append((e - s_) / 1e3)
            d[1].append((s_ - prev_end) / 1e3)
            prev_end = e
    if spans:
        print("update span us: median %.1f over %d updates" % (statistics.median(spans), len(spans)))
        for k, (d, g) in sorted(per.items()):
            if len(d) >= len(spans) // 2:
                print("%-60s dur %7.2f  gap-before %6.2f" % (k, statistics.median(d), statistics.median(g)))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "summarize":
        summarize(sys.argv[2])
    else:
        run()
