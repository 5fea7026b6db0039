"""MFMA utilisation per kernel from a rocprofv3 counter pass:

    rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        -d gpurun_out/pmcm -o run --output-format csv -- python3 bench.py ...
    python tools/pmc_mfma.py gpurun_out/pmcm/run_counter_collection.csv [--out profiles/c3_pmc_mfma.json]

Per kernel name (averaged over its dispatches):
  * mfma_flop      = SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 (the MfmaFlopsBF16 derived counter)
  * gui_cycles     = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the counter over the 8 XCDs; one XCD's value is the
                     dispatch's length in shader clocks)
  * mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (gui_cycles * 1024 SIMDs): the MfmaUtil derived counter, the share
                     of SIMD-cycles the matrix pipe was busy over the dispatch
  * clock_ghz      = gui_cycles / dispatch duration (when the CSV carries timestamps)
  * mfma_tflops    = mfma_flop / duration, and its fraction of the 2.5 PF dense bf16 peak
"""
import argparse
import collections
import csv
import json

SIMDS = 1024
PEAK_TF = 2500.0


def load(path):
    per = collections.defaultdict(dict)        # dispatch id -> {counter: value, name, dur}
    for r in csv.DictReader(open(path)):
        d = per[r.get("Dispatch_Id") or r.get("Correlation_Id")]
        d["name"] = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            d["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per


def summarise(per):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in per.values():
        a = agg[d["name"].split("(")[0]]
        a["launches"] += 1
        for k, v in d.items():
            if k != "name":
                a[k] += v
    out = {}
    for name, a in agg.items():
        n = a["launches"]
        mops = a.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) / n
        if mops == 0:
            continue
        gui = a.get("GRBM_GUI_ACTIVE", 0.0) / n / 8
        busy = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / n
        rec = {"launches": int(n), "mfma_flop_per_launch": mops * 512, "gui_cycles": round(gui),
               "mfma_busy_frac": round(busy / (gui * SIMDS), 4) if gui else None}
        if a.get("dur_ns"):
            dur = a["dur_ns"] / n * 1e-9
            rec["dur_us"] = round(dur * 1e6, 2)
            rec["clock_ghz"] = round(gui / dur / 1e9, 3)
            rec["mfma_tflops"] = round(mops * 512 / dur / 1e12, 1)
            rec["mfma_frac_of_peak"] = round(mops * 512 / dur / 1e12 / PEAK_TF, 4)
        out[name] = rec
    return normalise_short(out)


def normalise_short(out, min_us=300.0):
    """GRBM_GUI_ACTIVE over-reads on dispatches shorter than ~0.3 ms (implied clocks of 3.6-4.8 GHz, above the
    chip's 2.4 GHz), which under-states their busy fraction.  For those, also report the busy fraction over the
    dispatch's DURATION at the clock the long dispatches of the same pass held (their GUI_ACTIVE / duration, weighted
    by duration): mfma_busy_frac_dur = busy cycles / (dur * clock_ref * 1024 SIMDs)."""
    long_ = [r for r in out.values() if r.get("dur_us") and r["dur_us"] >= min_us and r.get("clock_ghz")]
    if not long_:
        return out
    w = sum(r["dur_us"] * r["launches"] for r in long_)
    clk = sum(r["clock_ghz"] * r["dur_us"] * r["launches"] for r in long_) / w
    for r in out.values():
        r.pop("mfma_busy_frac_dur", None)
        if r.get("dur_us") and r["dur_us"] < min_us and r.get("mfma_busy_frac") is not None:
            busy = r["mfma_busy_frac"] * r["gui_cycles"] * SIMDS
            r["mfma_busy_frac_dur"] = round(busy / (r["dur_us"] * 1e-6 * clk * 1e9 * SIMDS), 4)
            r["clock_ref_ghz"] = round(clk, 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--out")
    ap.add_argument("--config", default="c3")
    args = ap.parse_args()
    res = summarise(load(args.csv))
    for name, r in sorted(res.items(), key=lambda kv: -kv[1]["mfma_flop_per_launch"] * kv[1]["launches"]):
        print(f"{name[:60]:60s} n={r['launches']:4d} busy={r['mfma_busy_frac']} busy_dur={r.get('mfma_busy_frac_dur')} "
              f"clk={r.get('clock_ghz')} TF={r.get('mfma_tflops')} dur={r.get('dur_us')}")
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"config": args.config, "source": args.csv,
                       "counters": "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE",
                       "formula": "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs); "
                                  "mfma_flop = MOPS_BF16 * 512; dispatches < 0.3 ms also mfma_busy_frac_dur = "
                                  "busy cycles / (duration * clock_ref * 1024), clock_ref = the long dispatches' clock",
                       "kernels": res}, f, indent=1)


if __name__ == "__main__":
    main()
