"""Step timeline from a rocprofv3 --kernel-trace CSV: per training step, the wall span, the
time the GPU is busy (union of kernel intervals over all streams), the idle gaps, and the
busy time per kernel family split into 'alone' (no other kernel running) and 'overlapped'.

python tools/timeline.py <kernel_trace.csv> [--steps N]

Steps are delimited by the Keras-Adam launch (one per step); the last N complete steps are
reported (the bench's timed region).
"""
import argparse
import collections
import csv
import re


def family(name):
    n = re.sub(r"\(.*", "", name)
    n = n.replace("void ", "").replace("oflow::", "")
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    rows = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    adam = [i for i, r in enumerate(rows) if re.search(r"adam_(dev_)?kernel", r[2])]
    if len(adam) < args.steps + 1:
        raise SystemExit("need %d adam launches, got %d" % (args.steps + 1, len(adam)))
    spans = []
    fam_alone = collections.Counter()
    fam_total = collections.Counter()
    for k in range(len(adam) - args.steps, len(adam)):
        lo, hi = rows[adam[k - 1]][1], rows[adam[k]][1]
        ks = [r for r in rows if r[0] >= lo and r[1] <= hi]
        # sweep: busy union and per-kernel exclusive time
        ev = []
        for i, (s, e, n) in enumerate(ks):
            ev.append((s, 1, i))
            ev.append((e, -1, i))
        ev.sort(key=lambda x: (x[0], x[1]))
        active = set()
        last = lo
        busy = 0
        gaps = []
        for t, typ, i in ev:
            if t > last:
                if active:
                    busy += t - last
                    if len(active) == 1:
                        fam_alone[family(ks[next(iter(active))][2])] += t - last
                else:
                    gaps.append(t - last)
            last = max(last, t)
            if typ == 1:
                active.add(i)
            else:
                active.discard(i)
        for s, e, n in ks:
            fam_total[family(n)] += e - s
        gaps.sort(reverse=True)
        spans.append((hi - lo, busy, sum(gaps), len(ks), gaps[:5]))
    for span, busy, idle, nk, g in spans:
        print("step %.3f ms: busy %.3f ms, idle %.3f ms, %d kernels, largest gaps (us) %s" % (
            span / 1e6, busy / 1e6, idle / 1e6, nk, [round(x / 1e3, 1) for x in g]))
    ns = len(spans)
    print("\n%-70s %9s %9s" % ("kernel (per step)", "total ms", "alone ms"))
    for n, t in fam_total.most_common(args.top):
        print("%-70s %9.3f %9.3f" % (n[:70], t / 1e6 / ns, fam_alone[n] / 1e6 / ns))


if __name__ == "__main__":
    main()
