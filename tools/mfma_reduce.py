"""MFMA utilisation from rocprofv3 counters (dev tool).

Inputs: a --pmc run with SQ_VALU_MFMA_BUSY_CYCLES (+ SQ_WAVES, SQ_BUSY_CYCLES)
and a --kernel-trace run of the same command.  Every MFMA in the field / gate
kernels is v_mfma_f32_32x32x16_f16: 32 busy cycles and 2*32*32*16 = 32,768
FLOP each (MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES = 32 x N_mfma for the
32x32x16 shapes), so per kernel:
  n_mfma   = busy / 32
  TFLOP/s  = n_mfma * 32768 / mean kernel duration
  busy_frac= busy / (duration x clock x 1024 SIMDs)   (the MFMA pipes' busy share)
usage: python tools/mfma_reduce.py <pmc dir> <trace dir> <pattern>... [--clock-ghz 2.4]
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def _rows(d, suffix):
    rows = []
    for f in glob.glob(f"{d}/**/*{suffix}", recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    clock = 2.4
    if "--clock-ghz" in sys.argv:
        clock = float(sys.argv[sys.argv.index("--clock-ghz") + 1])
        args.remove(sys.argv[sys.argv.index("--clock-ghz") + 1])
    pmc_dir, trace_dir, pats = args[0], args[1], args[2:]
    cnt = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in _rows(pmc_dir, "counter_collection.csv"):
        k = r.get("Kernel_Name", "")
        cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    dur = defaultdict(list)
    for r in _rows(trace_dir, "kernel_trace.csv"):
        k = r.get("Kernel_Name", "")
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    out = {}
    for k, c in cnt.items():
        if not any(p in k for p in pats):
            continue
        n = max(1, len(disp[k]))
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / n
        d = [x for kk, v in dur.items() if kk == k for x in v]
        t = sum(d) / len(d) if d else None
        n_mfma = busy / 32
        rec = {"dispatches": n, "mfma_busy_cycles": busy, "n_mfma": n_mfma,
               "mean_ms": None if t is None else round(t * 1e3, 4)}
        if t:
            rec["tflops"] = round(n_mfma * 32768 / t / 1e12, 2)
            rec["busy_frac"] = round(busy / (t * clock * 1e9 * 1024), 4)
        for extra in ("SQ_WAVES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
            if extra in c:
                rec[extra] = c[extra] / n
        out[k[:100]] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
