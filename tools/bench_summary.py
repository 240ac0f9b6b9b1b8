"""Print the key figures of bench.py JSON lines (dev tool).
usage: python tools/bench_summary.py file.json ..."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "ERR", e)
        continue
    rf = d["roofline"]
    at = rf.get("atomic") or {}
    print(f"{f}: {d['value']} Msamples/s n={d['n_gpus']} {d.get('backend')} "
          f"{d['ms_per_step']} ms/step, spl {d['config']['samples_per_step_per_gpu']}, "
          f"{d['config'].get('parallelism')}; field_bwd {rf['avg_launch_ms']} ms frac {rf['frac']} "
          f"traffic {rf['traffic']} atomic {at.get('requests_per_sample')} req/smp "
          f"frac {at.get('frac')}; ranks {[r['rank'] for r in d.get('ranks_seen', [])]}")
    km = d.get("kernel_ms") or {}
    print("   kernel_ms", {k: v for k, v in km.items()})
    for k in ("forward_only", "dropin_step", "api_step", "train_step", "density_update",
              "test_time_render", "cpu_baseline", "rgb_linf_vs_ref"):
        v = d.get(k)
        if v is not None:
            print(f"   {k}: {json.dumps(v)[:420]}")
