"""Counter table of tools/pmc_gemm.sh runs: per GEMM directory, every pass's counters averaged
over the kernel's dispatches, then derived figures (kernel time from GRBM_GUI_ACTIVE at the
shader clock, wait / MFMA-busy fractions, HBM bytes per launch (FETCH_SIZE / WRITE_SIZE are KiB),
bytes per CU, achieved GB/s).
usage: python tools/pmc_table.py DIR [DIR ...] [--clock-mhz 2400] [--flop F --algo-bytes B] [--match NAME]"""
import argparse
import collections
import csv
import glob
import os


def counters(d, match="gemm"):
    agg = collections.defaultdict(float)
    n = collections.defaultdict(set)
    name = None
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if match not in k:
                continue
            name = k[:70]
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    return name, {c: v / max(len(n[c]), 1) for c, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--clock-mhz", type=float, default=2400.0)
    ap.add_argument("--match", default="gemm", help="kernel-name substring")
    ap.add_argument("--xcds", type=float, default=8.0,
                    help="GRBM_GUI_ACTIVE is summed over the XCDs (MI355X_MICROARCH.md): divide by this")
    ap.add_argument("--flop", type=float, default=2.0 * 25104 * 768 * 768)
    ap.add_argument("--algo-bytes", type=float, default=25104 * 768 * (2 + 4 + 4) + 768 * 768 * 2)
    a = ap.parse_args()
    for d in a.dirs:
        name, c = counters(d, a.match)
        if not c:
            print("## %s: no counters" % d)
            continue
        g = c.get("GRBM_GUI_ACTIVE", 0.0) / a.xcds         # kernel cycles
        us = g / a.clock_mhz
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        fetch = c.get("FETCH_SIZE", 0.0) * 1024
        write = c.get("WRITE_SIZE", 0.0) * 1024
        print("## %s\n%s" % (d, name))
        for k in sorted(c):
            print("  %-28s %16.0f" % (k, c[k]))
        print("  kernel time (GRBM_GUI_ACTIVE / %g XCDs @ %.0f MHz) %8.1f us" % (a.xcds, a.clock_mhz, us))
        if c.get("SQ_WAVES") and c.get("SQ_INSTS_VALU"):
            print("  VALU / MFMA instructions per wave        %8.0f / %.0f" %
                  (c["SQ_INSTS_VALU"] / c["SQ_WAVES"], c.get("SQ_INSTS_MFMA", 0) / c["SQ_WAVES"]))
        if g and c.get("SQ_ACTIVE_INST_VALU"):
            # quad-cycles (x4) summed over waves, per SIMD (1024), against the kernel's cycles
            print("  VALU-active cycles per SIMD / kernel cyc %8.3f" % (c["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / g))
        if wc:
            print("  SQ_WAIT_ANY / SQ_WAVE_CYCLES             %8.3f" % (c.get("SQ_WAIT_ANY", 0) / wc))
            print("  SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES        %8.3f" % (c.get("SQ_WAIT_INST_ANY", 0) / wc))
            print("  SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES      %8.3f" % (c.get("SQ_ACTIVE_INST_ANY", 0) / wc))
        if c.get("SQ_BUSY_CYCLES") and c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            # MFMA busy per SIMD-cycle: SQ_VALU_MFMA_BUSY_CYCLES over (kernel cycles x 1024 SIMDs)
            print("  MFMA busy / (kernel cycles x 1024 SIMDs) %8.3f" % (c["SQ_VALU_MFMA_BUSY_CYCLES"] / (g * 1024) if g else 0))
        if fetch or write:
            print("  HBM read / write per launch              %8.1f / %.1f MB  (algorithmic %.1f MB)" %
                  (fetch / 1e6, write / 1e6, a.algo_bytes / 1e6))
            print("  bytes per CU                             %8.2f MB" % ((fetch + write) / 256 / 1e6))
            if us:
                print("  achieved HBM GB/s                        %8.0f" % ((fetch + write) / (us * 1e-6) / 1e9))
        if us:
            print("  TF/s                                     %8.1f" % (a.flop / (us * 1e-6) / 1e12))


if __name__ == "__main__":
    main()
