"""Per-kernel durations and inter-kernel gaps of the steps of a rocprofv3
--kernel-trace CSV (e.g. bench.py --graph replays).

usage: python tools/graph_timeline.py <kernel_trace.csv> [first-kernel regex] [steps]
A step starts at each launch of the first kernel (default: the noise kernel);
the last `steps` complete steps (default 20) are averaged: the step span
(first start to the next step's first start), the kernels' busy time, the
gaps, and each kernel's mean duration in launch order."""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    first = re.compile(sys.argv[2] if len(sys.argv) > 2 else "noise_philox")
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in rows)
    starts = [i for i, (_, _, k) in enumerate(ev) if first.search(k)]
    steps = [(starts[j], starts[j + 1]) for j in range(len(starts) - 1)][-n:]
    n = len(steps)
    per = steps[-1][1] - steps[-1][0]
    spans, busy, names = [], [], {}
    for a, b in steps:
        st = ev[a:b]
        if len(st) != per:
            continue
        spans.append(ev[b][0] - st[0][0])
        busy.append(sum(e - s for s, e, _ in st))
        for j, (s, e, k) in enumerate(st):
            names.setdefault(j, [k, []])[1].append(e - s)
    m = len(spans)
    span, bz = sum(spans) / m / 1e3, sum(busy) / m / 1e3
    print(f"{m} steps of {per} kernels: step {span:.2f} us, kernels {bz:.2f} us, "
          f"gaps {span - bz:.2f} us")
    for j in sorted(names):
        k, d = names[j]
        print(f"  {sum(d) / len(d) / 1e3:8.2f} us  {k[:100]}")


if __name__ == "__main__":
    main()
