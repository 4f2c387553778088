"""Per-layer conv timing table from a bench.py OFLOW_TIMING_DUMP json (list of {layer, kind,
gflop, ms} over the instrumented steps).

python tools/layer_table.py <dump.json> [steps] [ceiling_tflops]
Prints per (layer, pass): ms per step, achieved TFLOP/s, and ms lost against the ceiling
(default 118 TFLOP/s fp32, the measured DVFS-limited MFMA loop rate).
"""
import json
import sys
from collections import defaultdict

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
from bench import kind_name, kind_parts  # noqa: E402


def main():
    rows = json.load(open(sys.argv[1]))
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    ceil = float(sys.argv[3]) if len(sys.argv) > 3 else 118.0
    acc = defaultdict(lambda: [0.0, 0.0, 0, None])
    for r in rows:
        mode = ("fwd", "dgrad", "wgrad")[kind_parts(r["kind"])[0]]
        a = acc[(r["layer"], mode)]
        a[0] += r["gflop"]
        a[1] += r["ms"]
        a[2] += 1
        a[3] = kind_name(r["kind"])
    out = []
    for (layer, mode), (gf, ms, n, kn) in acc.items():
        ms /= steps
        gf /= steps
        lost = ms - gf / ceil
        out.append((lost, layer, mode, kn, ms, gf / ms if ms else 0.0, n // steps))
    out.sort(reverse=True)
    tot = sum(o[4] for o in out)
    print("%-28s %-6s %-26s %3s %8s %7s %8s" % ("layer", "pass", "kernel", "n", "ms/step",
                                               "TF", "lost ms"))
    for lost, layer, mode, kn, ms, tf, n in out:
        print("%-28s %-6s %-26s %3d %8.3f %7.1f %8.3f" % (layer[:28], mode, kn[:26], n, ms, tf,
                                                          lost))
    print("total conv ms/step %.3f, lost vs %.0f TF: %.3f" % (tot, ceil, sum(o[0] for o in out)))


if __name__ == "__main__":
    main()
