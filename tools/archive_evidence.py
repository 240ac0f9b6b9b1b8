"""Copy one evidence run's outputs (tools/gpu/r05k.sh TAG, r05h.sh TAG2) from
gpurun_out/ into profiles/<round>/ and refresh profiles/traffic.json and
profiles/mfma.json (dev tool).  usage: archive_evidence.py ROUND TAG [SUITE_TAG]"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")


def main(rnd, tag, suite=None):
    d = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(os.path.join(d, "mfma"), exist_ok=True)
    os.makedirs(os.path.join(d, "pmc"), exist_ok=True)
    for c in ("c1", "c2", "c3", "c4", "c5", "c5pin"):
        shutil.copy(os.path.join(G, f"bench_{c}_{tag}.json"), os.path.join(d, f"bench_{c}_{rnd}{tag}.json"))
    shutil.copy(os.path.join(G, f"prof_{tag}", "run_kernel_stats.csv"),
                os.path.join(d, f"kernel_stats_c3_{rnd}{tag}.csv"))
    shutil.copy(os.path.join(G, f"profc5_{tag}", "run_kernel_stats.csv"),
                os.path.join(d, f"kernel_stats_c5_{rnd}{tag}.csv"))
    shutil.copy(os.path.join(G, f"mfma_{tag}.json"), os.path.join(d, "mfma", f"mfma_c3_{rnd}{tag}.json"))
    shutil.copy(os.path.join(G, f"mfma4_{tag}.json"),
                os.path.join(d, "mfma", f"mfma_mlp_phase_c3_{rnd}{tag}.json"))
    for c in ("c3", "c4", "c5"):
        shutil.copy(os.path.join(G, f"traffic_{c}_{tag}.json"),
                    os.path.join(d, "pmc", f"traffic_{c}_{rnd}{tag}.json"))
    shutil.copy(os.path.join(G, f"smoke_{tag}.log"), os.path.join(d, f"smoke_{rnd}{tag}.log"))
    shutil.copy(os.path.join(G, "traffic.json"), os.path.join(ROOT, "profiles", "traffic.json"))
    if suite:
        shutil.copy(os.path.join(G, f"gpu_suite_{suite}.log"), os.path.join(d, f"gpu_suite_{rnd}{suite}.log"))
        shutil.copy(os.path.join(G, f"smoke_{suite}.log"), os.path.join(d, f"smoke_{rnd}{suite}.log"))
        shutil.copy(os.path.join(G, f"train_s16_{suite}.json"),
                    os.path.join(d, f"train_demo_s16_e5m17_{rnd}{suite}.json"))
        shutil.copy(os.path.join(G, f"bench_dp2_c5_{suite}.json"),
                    os.path.join(d, f"bench_dp2_gloo_c5_{rnd}{suite}.json"))
    m = json.load(open(os.path.join(G, f"mfma_{tag}.json")))
    m4 = json.load(open(os.path.join(G, f"mfma4_{tag}.json")))
    p = os.path.join(ROOT, "profiles", "mfma.json")
    doc = json.load(open(p))
    w = doc["workloads"]["K2_s0.5_B8192_p0.50"]
    names = {"field_bwd": "k_field_bwd_merged<2, false, 2>", "field_fwd_mlp": "k_field_mlp_planes",
             "gate_fwd": "k_gate_fwd", "gate_bwd": "k_gate_bwd"}
    for key, sub in names.items():
        for k, v in m.items():
            if sub in k:
                v = dict(v)
                v.pop("SQ_WAVES", None)
                v["kernel"] = k
                w["kernels"][key] = v
    for k, v in m4.items():
        if "k_field_bwd_merged<2, true, 2>" in k:
            v = dict(v)
            v.pop("SQ_WAVES", None)
            v["kernel"] = k
            w["kernels"]["field_bwd_mlp_phase_only"] = v
    w["run"] = f"profiles/{rnd}/mfma/mfma_c3_{rnd}{tag}.json"
    json.dump(doc, open(p, "w"), indent=1)
    print({k: (v["mean_ms"], v["busy_frac"]) for k, v in w["kernels"].items()})


if __name__ == "__main__":
    main(*sys.argv[1:])
