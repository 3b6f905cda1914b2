"""Per-launch HBM bytes of the hot kernels from two rocprofv3 --pmc passes
(tools/pmc_traffic.sh).  FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a coalesced stream, so reads are doubled
(MI355X_MICROARCH.md, HBM section).  Infinity-Cache hits are counted too.
Writes profiles/kernel_traffic.json (read by bench.py's roofline objects)."""
import csv, glob, json, os, statistics, sys

KERNELS = {  # json key -> kernel-name substring (bench.py R2 shape, fp32)
    "chain_B64_T1000": "faithful_chain_kernel",
    "strip_B64_fp32": "enc_fp32_kernel<false>",
}
# TRAIN=1 (tools/pmc_train.sh: tools/train_ref_probe.py --plan-only, B = 32):
# the reference train step's kernels, and their sum per step
TRAIN_KERNELS = {
    "train_conv_bwd_B32": "conv_bwd_kernel",
    "train_enc_B32": "enc_train_kernel",
    "train_head_B32": "train_head_kernel<2>",
    "train_final_B32": "train_final_kernel",
}
if os.environ.get("TRAIN"):
    KERNELS = TRAIN_KERNELS


def per_launch(d, counter, name):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if name in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


fetch_dir, write_dir, out = sys.argv[1:4]
rec = json.load(open(out)) if os.path.exists(out) else {}
# a U-Net probe run (UNET_KEY set) records only its step total: its encoder
# launches are not the R2 bench shape the per-kernel keys describe
for key, name in ({} if os.environ.get("UNET_KEY") else KERNELS).items():
    fk, wk = per_launch(fetch_dir, "FETCH_SIZE", name), per_launch(write_dir, "WRITE_SIZE", name)
    if not fk or not wk:
        print(f"no {name} rows ({len(fk)} fetch, {len(wk)} write)")
        continue
    f_med, w_med = statistics.median(fk), statistics.median(wk)
    rec[key] = {
        "kernel": name,
        "hbm_bytes_per_launch": int(2 * f_med * 1024 + w_med * 1024),
        "fetch_size_kib_median": f_med, "write_size_kib_median": w_med,
        "launches": [len(fk), len(wk)],
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); "
                  "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction)",
        "workload": ("tools/train_ref_probe.py --plan-only, B=32, L=4693 (TrainPlan)" if os.environ.get("TRAIN")
                     else "bench.py R2 faithful, B=64, L=4693, T=1000 (chain: one launch = 1000 steps)"),
    }
    print(key, json.dumps(rec[key]))
if os.environ.get("TRAIN") and all(k in rec for k in TRAIN_KERNELS):
    rec["train_step_B32"] = {
        "kernel": "enc_train + train_head<2> + conv_bwd + train_final (one step)",
        "hbm_bytes_per_launch": sum(rec[k]["hbm_bytes_per_launch"] for k in TRAIN_KERNELS),
        "method": "sum of the four kernels' per-launch medians (same passes)",
        "workload": "tools/train_ref_probe.py --plan-only, B=32, L=4693 (TrainPlan)"}
    print("train_step_B32", json.dumps(rec["train_step_B32"]))
# U-Net: every ertd::unet:: kernel of the run, summed, per denoising step
unet_steps = int(os.environ.get("UNET_STEPS", "0"))
unet_key = os.environ.get("UNET_KEY", "unet_U2_B64_step")
if unet_steps > 0:
    fk = per_launch(fetch_dir, "FETCH_SIZE", "ertd::unet::")
    wk = per_launch(write_dir, "WRITE_SIZE", "ertd::unet::")
    if fk and wk:
        rec[unet_key] = {
            "kernel": "all ertd::unet:: kernels of one U-Net sampler step",
            "hbm_bytes_per_launch": int((2 * sum(fk) * 1024 + sum(wk) * 1024) / unet_steps),
            "fetch_size_kib_per_step": sum(fk) / unet_steps,
            "write_size_kib_per_step": sum(wk) / unet_steps,
            "dispatches": [len(fk), len(wk)], "steps": unet_steps,
            "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), summed over "
                      "every ertd::unet:: dispatch / steps; bytes = 2*FETCH_SIZE*1024 + "
                      "WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction)",
            "workload": os.environ.get("UNET_WORKLOAD", "bench.py U2, B=64, L=4693 (steps incl. warmup)"),
        }
        print(unet_key, json.dumps(rec[unet_key]))
    else:
        print(f"no ertd::unet:: rows ({len(fk)} fetch, {len(wk)} write)")
json.dump(rec, open(out, "w"), indent=1)
