"""Per-kernel HBM traffic from two separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py FETCH.csv WRITE.csv CONFIG OUT.json

Both counters are in KiB (rocprofiler-sdk counter_defs.yaml).  gfx950 correction (MI355X_MICROARCH.md,
"HBM"): FETCH_SIZE reports exactly half the bytes of wide (16 B/lane) coalesced reads -> x2; WRITE_SIZE is
exact for 16 B/lane stores and float atomics.  Keys are the kernel names as asrx_gemm_kernel_name prints
them (namespace and argument list stripped), so bench.py can look up its roofline kernel.
"""
import collections
import csv
import json
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    depth = 0
    for i, ch in enumerate(n):      # cut at the argument list (first '(' outside template brackets)
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return n[:i]
    return n


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return acc


def main():
    fetch_csv, write_csv, config, out = sys.argv[1:5]
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")
    write = per_kernel(write_csv, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(fetch) & set(write)):
        f = sum(fetch[name]) / len(fetch[name])
        w = sum(write[name]) / len(write[name])
        kernels[name] = {"launches": len(fetch[name]), "fetch_bytes_raw": round(f), "write_bytes": round(w),
                         "hbm_bytes_per_launch": round(2.0 * f + w)}
    rec = {"config": config, "source": [fetch_csv, write_csv],
           "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB->bytes); gfx950 FETCH_SIZE halves wide reads",
           "kernels": kernels}
    with open(out, "w") as fo:
        json.dump(rec, fo, indent=1)
    top = sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"])[:15]
    for n, v in top:
        print(f"{v['hbm_bytes_per_launch']/1e6:10.2f} MB/launch x{v['launches']:5d}  {n}")


if __name__ == "__main__":
    main()
