"""Reduce rocprofv3 PMC passes to per-launch HBM traffic of the field kernels.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> [<atomic_dir>] [--merge profiles/traffic.json]

The passes are keyed by workload (K, scale, rays, occupancy; from the bench
JSON line in <dir>.log): with --merge the entry is written into the
traffic file under that key, which bench.py looks up for its own workload
(no figures are reported for a workload without a PMC pass).

Each dir holds run_counter_collection.csv of one `rocprofv3 --pmc <counter>`
pass over `bench.py` (separate passes: FETCH_SIZE and WRITE_SIZE cannot share
one, MI355X_MICROARCH.md "rocprofv3 PMC slots").  Corrections as the guide
prescribes for gfx950: FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE counts
64 B per 128-B request of a wide coalesced read, so it is doubled (our field
kernels' reads are 4-16 B gathers, where the factor is uncalibrated: both the
raw and the corrected figure are kept).  WRITE_SIZE counts float atomics
exactly (one dword per lane).  TCC_EA0_ATOMIC (when collected) counts the 64-B
atomic requests leaving L2.
"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

# the fused chain's kernels; the per-model kernels only where a run has no
# merged launch (--split-bwd), never mixed (bench.py's drop-in leg runs them).
# An alternative is a tuple of kernels that together make one step's launch
# (the level-partitioned forward: prep + encode + MLP tiles), summed.
KERNELS = {"field_bwd": (("k_field_bwd_merged",), ("k_field_bwd",)),
           "field_fwd": (("k_enc_prep", "k_field_encode_levels", "k_field_mlp_planes"),
                         ("k_field_fwd_merged",), ("k_field_fwd",)),
           # the binned scatter's bin + sum passes (fx_fold of a binned step)
           "grid_fold": (("k_grid_bin", "k_grid_sum"),)}


def per_dispatch(d):
    path = os.path.join(d, "run_counter_collection.csv")
    vals = defaultdict(lambda: defaultdict(float))   # kernel pattern -> dispatch -> value
    pats = {p for alts in KERNELS.values() for alt in alts for p in alt}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if "k_field_bwd_merged<" in name and name.split(">")[0].rstrip().endswith(", 3"):
                continue        # the fixed-point redo launch (exits at once unless flagged)
            for pat in pats:
                if pat + "<" in name or pat + "(" in name:
                    vals[pat][row["Dispatch_Id"]] += float(row["Counter_Value"])
                    break
    out = {}
    for key, alts in KERNELS.items():
        for alt in alts:
            if all(vals.get(p) for p in alt):
                # the median launch: a workspace's first backward is fp32
                # (it measures the fixed-point scales) and is not the step
                out[key] = sum(statistics.median(vals[p].values()) for p in alt)
                break
    return out


def workload_key(cfg):
    """bench.py's key of a workload (keep in sync with bench.py workload_key)."""
    return (f"K{cfg['model_zoo_size']}_s{float(cfg['scale']):g}_B{cfg['rays_per_gpu']}"
            f"_p{float(cfg.get('occupancy', 0.5)):.2f}"
            + ("_bin" if cfg.get("grid_scatter") == "binned" else ""))


def main():
    argv = list(sys.argv[1:])
    merge = None
    if "--merge" in argv:
        i = argv.index("--merge")
        merge = argv[i + 1]
        del argv[i:i + 2]
    fetch = per_dispatch(argv[0])
    write = per_dispatch(argv[1])
    atom = per_dispatch(argv[2]) if len(argv) > 2 and os.path.isdir(argv[2]) else {}
    samples, cfg = None, None
    for d in argv[:2]:
        try:
            with open(d.rstrip("/") + ".log") as f:
                for line in f:
                    if line.startswith('{"metric"'):
                        cfg = json.loads(line)["config"]
                        samples = cfg["samples_per_step_per_gpu"]
        except (OSError, ValueError, KeyError):
            pass
    key = workload_key(cfg) if cfg else "unknown"
    out = {"workload": key, "samples_per_launch": samples,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_EA0_ATOMIC, separate passes, "
                     "bench.py on this workload; per launch (one launch per step; the median "
                     "launch)"}
    for k in KERNELS:
        if k not in fetch or k not in write:
            continue
        f_raw, w = fetch[k] * 1024, write[k] * 1024
        out[f"{k}_fetch_bytes_raw"] = round(f_raw)
        out[f"{k}_write_bytes"] = round(w)
        out[f"{k}_bytes_per_launch"] = round(2 * f_raw + w)
        if k in atom:
            out[f"{k}_atomic_requests"] = round(atom[k])
    json.dump(out, sys.stdout, indent=1)
    print()
    if merge:
        try:
            with open(merge) as f:
                allw = json.load(f)
        except (OSError, ValueError):
            allw = {}
        # keep the entry's other fields (u32_request_share: the replay's split
        # of the requests between fp32 and u32 adds)
        allw.setdefault("workloads", {}).setdefault(key, {}).update(out)
        with open(merge, "w") as f:
            json.dump(allw, f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
