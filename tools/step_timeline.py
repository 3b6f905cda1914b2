"""Timeline of the last N kernels of a rocprofv3 kernel trace (diagnostic):
busy time (union of kernel intervals), idle gaps, and per-kernel-name totals,
so launch gaps and serialization show up next to kernel time.

    python tools/step_timeline.py gpurun_out/<dir>/run_kernel_trace.csv [--last-span-us 4000] [--top 12]

--last-span-us: keep the kernels that start within the last <us> of the trace
(one sampler step of the probe's final launch, say)."""
import argparse
import csv
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    for p in ("void ", "ertd::unet::(anonymous namespace)::", "ertd::unet::", "ertd::"):
        n = n.replace(p, "")
    return n[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last-span-us", type=float, default=None)
    ap.add_argument("--from-name", default=None,
                    help="start at the last dispatch whose name contains this (e.g. conv_in)")
    ap.add_argument("--count", type=int, default=None, help="kernels from the start point")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
            for r in csv.DictReader(open(a.trace))]
    rows.sort()
    if a.from_name:
        idx = [i for i, r in enumerate(rows) if a.from_name in r[2]]
        i0 = idx[-2] if len(idx) > 1 else idx[-1]   # the second-to-last: one whole step after it
        rows = rows[i0:idx[-1]] if len(idx) > 1 else rows[i0:]
    if a.count:
        rows = rows[:a.count]
    if a.last_span_us:
        t_end = max(r[1] for r in rows)
        rows = [r for r in rows if r[0] >= t_end - a.last_span_us * 1e3]
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, n in rows:
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    tot = defaultdict(lambda: [0, 0])
    for s, e, n in rows:
        tot[short(n)][0] += 1
        tot[short(n)][1] += e - s
    ksum = sum(v[1] for v in tot.values())
    print(f"kernels {len(rows)}  span {(t1 - t0) / 1e3:9.1f} us  busy {busy / 1e3:9.1f} us  "
          f"idle {(t1 - t0 - busy) / 1e3:8.1f} us in {len(gaps)} gaps  sum of durations {ksum / 1e3:9.1f} us")
    gsz = sorted(g for g, _ in gaps)
    if gsz:
        print(f"gap us: median {gsz[len(gsz) // 2] / 1e3:.2f}  p90 {gsz[int(len(gsz) * 0.9)] / 1e3:.2f}  "
              f"max {gsz[-1] / 1e3:.2f}")
    gby = defaultdict(lambda: [0, 0])
    for g, n in gaps:
        gby[short(n)][0] += 1
        gby[short(n)][1] += g
    print("idle before (kernel that ends the gap):")
    for n, (c, g) in sorted(gby.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {n:48s} {c:5d} gaps {g / 1e3:9.1f} us")
    print("kernel time:")
    for n, (c, d) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {n:48s} {c:5d} x {d / c / 1e3:8.2f} us = {d / 1e3:9.1f} us ({d / ksum * 100:5.1f} %)")


if __name__ == "__main__":
    main()
