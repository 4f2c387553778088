"""Write a profile summary (markdown) from a bench JSON line and the rocprofv3 kernel_stats.csv
of the same bench command.

python tools/make_summary.py <bench.log> <kernel_stats.csv> <command> [top] [pmc entry]
    > profiles/....md
The kernel table carries MFMA busy and HBM bytes per launch from profiles/pmc_traffic.json's
entry for the bench's configuration ("precision:HxWxB", or the given one) when present.
"""
import os
import csv
import json
import sys


def main():
    log, stats, cmd = sys.argv[1:4]
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    line = [ln for ln in open(log) if ln.startswith("{")][-1]
    b = json.loads(line)
    rf = b["roofline"]
    rows = list(csv.DictReader(open(stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    dom = [r for r in rows if r["Name"] == rf["kernel"]]
    prof_avg = float(dom[0]["AverageNs"]) / 1e6 if dom else float("nan")
    print("# Profile summary: `%s` (MI355X, gfx950, ROCm 7.2)\n" % cmd)
    print("rocprofv3 command: `rocprofv3 --kernel-trace --stats --output-format csv -- %s` "
          "(warm-up + timed + instrumented steps of one bench run).\n" % cmd)
    print("Bench line (un-profiled run): **%.1f %s**, %.2f ms/step, dtype %s, model %.1f TFLOP/s."
          % (b["value"], b["unit"], b["ms_per_step"], b["dtype"], b.get("model_tflops", 0)))
    print("Dominant kernel `%s`: %.1f %s achieved = %.1f %% of the %.1f %s peak; hipEvent average "
          "%.4f ms per launch vs rocprof average %.4f ms.\n"
          % (rf["kernel"], rf["achieved"], rf["unit"], 100 * rf["frac"], rf["peak"], rf["unit"],
             rf["avg_launch_ms"], prof_avg))
    cfg = b["config"]
    key = sys.argv[5] if len(sys.argv) > 5 else "%s:%dx%dx%d" % (
        b["dtype"], cfg["height"], cfg["width"], cfg["batch_per_gpu"])
    pmc = {}
    pp = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                      "pmc_traffic.json")
    if os.path.exists(pp):
        pmc = json.load(open(pp)).get("entries", {}).get(key, {}).get("kernels", {})
    if rf.get("mfma_busy") is not None:
        print("Dominant kernel MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel "
              "cycles), tools/pmc_mfma.py): %.1f %%; HBM bytes per launch (PMC): %s MB.\n" % (
                  100 * rf["mfma_busy"],
                  "%.1f" % (rf["traffic"] / 1e6) if rf.get("traffic") else "-"))
    print("| kernel | calls | total ms | % of GPU time | avg ms | MFMA busy (PMC) | HBM MB / launch (PMC) |")
    print("|---|---|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        k = pmc.get(r["Name"], {})
        mb = k.get("mfma_busy")
        hb = k.get("hbm_bytes_per_launch")
        print("| `%s` | %s | %.2f | %.1f | %.4f | %s | %s |" % (
            r["Name"][:90], r["Calls"], float(r["TotalDurationNs"]) / 1e6,
            100 * float(r["TotalDurationNs"]) / tot, float(r["AverageNs"]) / 1e6,
            "%.1f %%" % (100 * mb) if mb is not None else "-",
            "%.1f" % (hb / 1e6) if hb is not None else "-"))
    alone = rf.get("per_kernel_alone", {})
    print("\nPer-kernel hipEvent table from the bench: `in step` = one fully timed step after "
          "the warm-up, side streams on (the input-gradient convs share the chip with the side "
          "stream's weight gradients and BN reductions); `alone` = one more step with every "
          "kernel alone on the chip (side streams off)%s:\n"
          % ("; all convs %.1f / %.1f TFLOP/s" % (rf["all_conv_gemm_tflops"],
                                                  rf["all_conv_gemm_tflops_alone"])
             if "all_conv_gemm_tflops_alone" in rf else ""))
    print("| instance | launches/step | ms/step in step | TFLOP/s in step | ms/step alone | TFLOP/s alone |")
    print("|---|---|---|---|---|---|")
    for k, v in rf.get("per_kernel", {}).items():
        a = alone.get(k)
        print("| %s | %d | %.3f | %.1f | %s | %s |" % (
            k, v["launches_per_step"], v["ms_per_step"], v["tflops"],
            "%.3f" % a["ms_per_step"] if a else "-", "%.1f" % a["tflops"] if a else "-"))

if __name__ == "__main__":
    main()
