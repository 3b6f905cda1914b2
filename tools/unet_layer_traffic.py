"""Per-layer HBM traffic of one U-Net sampler step from two rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE; tools/unet_traffic.sh), against each layer's
algorithmic (unfused) I/O: input read once + output written once (+ the
residual read of a ResBlock's conv2) + the weights once.  FETCH_SIZE is doubled (gfx950 reports
half the bytes of a coalesced stream, MI355X_MICROARCH.md HBM section).

    python tools/unet_layer_traffic.py <fetch_dir> <write_dir> [U2] [B] [--json out.json]

The step is the dispatches between the last two conv_in launches of the run
(one sampler step); its conv dispatches are zipped with the layer walk of
tools/unet_layers.py."""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("fetch")
ap.add_argument("write")
ap.add_argument("cfg", nargs="?", default="U2")
ap.add_argument("B", nargs="?", type=int, default=64)
ap.add_argument("--json", default=None)
a = ap.parse_args()

CFGS = {"U1": (32, 32, (1, 2), 2, False), "U2": (64, 64, (1, 2, 4), 2, False),
        "U3": (64, 64, (1, 2, 4), 2, True), "U5": (128, 128, (1, 1, 2, 2), 2, True)}
KEYS = ("conv_kernel<", "conv_out_kernel<", "conv_out64_kernel<", "conv_in_kernel<", "conv_wino_kernel<", "conv_wino4_kernel<",
        "conv_wino4s_kernel<", "conv1x1_kernel<", "conv_bf16_kernel<")


def walk(image, ch0, mult, nres, attn):
    L = []   # (name, cin, cout, ks, wo, ws, residual)
    H = image
    L.append(("conv_in", 1, ch0, 3, H, H, False))
    hs = [ch0]
    ch = ch0
    for i, m in enumerate(mult):
        for r in range(nres):
            o = ch0 * m
            L.append((f"d{i}r{r}.conv1", ch, o, 3, H, H, False))
            if ch != o:
                L.append((f"d{i}r{r}.skip", ch, o, 1, H, H, False))
            L.append((f"d{i}r{r}.conv2", o, o, 3, H, H, True))
            ch = o
            hs.append(ch)
        if i != len(mult) - 1:
            L.append((f"d{i}.down", ch, ch, 3, H // 2, H, False))
            H //= 2
            hs.append(ch)
    for nm in ("mid1", "mid2"):
        L.append((f"{nm}.conv1", ch, ch, 3, H, H, False))
        L.append((f"{nm}.conv2", ch, ch, 3, H, H, True))
        if nm == "mid1" and attn:
            L.append(("attn.qkv", ch, 3 * ch, 1, H, H, False))
            L.append(("attn.proj", ch, ch, 1, H, H, True))
    for i in reversed(range(len(mult))):
        for r in range(nres + 1):
            o = ch0 * mult[i]
            cin = ch + hs.pop()
            L.append((f"u{i}r{r}.conv1", cin, o, 3, H, H, False))
            L.append((f"u{i}r{r}.skip", cin, o, 1, H, H, False))
            L.append((f"u{i}r{r}.conv2", o, o, 3, H, H, True))
            ch = o
        if i != 0:
            L.append((f"u{i}.up", ch, ch, 3, H * 2, H, False))
            H *= 2
    L.append(("conv_out", ch, 1, 3, H, H, False))
    return L


def rows(d, counter):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    out.sort()
    return out


def last_step(rs):
    idx = [i for i, r in enumerate(rs) if "conv_in_kernel" in r[1]]
    return rs[idx[-2]:idx[-1]]


def short(n):
    for p in ("void ", "ertd::unet::(anonymous namespace)::", "ertd::unet::", "ertd::"):
        n = n.replace(p, "")
    return n.split("(")[0][:40]


fe, wr = last_step(rows(a.fetch, "FETCH_SIZE")), last_step(rows(a.write, "WRITE_SIZE"))
if len(fe) != len(wr) or any(x[1] != y[1] for x, y in zip(fe, wr)):
    sys.exit(f"the two passes' steps differ ({len(fe)} vs {len(wr)} dispatches)")
B = a.B
layers = walk(*CFGS[a.cfg])
convs = [(f, w) for f, w in zip(fe, wr) if any(k in f[1] for k in KEYS)]
if len(convs) != len(layers):
    sys.exit(f"{len(convs)} conv dispatches in the step, {len(layers)} layers in the walk")
tot_pmc = tot_alg = 0.0
fam = defaultdict(lambda: [0, 0.0, 0.0])
lines = []
for (name, cin, cout, ks, wo, ws, res), (f, w) in zip(layers, convs):
    pmc = 2 * f[2] * 1024 + w[2] * 1024
    # input read once, output written once (+ residual), the raw weights once
    alg = 4.0 * B * (cin * ws * ws + cout * wo * wo * (2 if res else 1)) + 4.0 * cin * cout * ks * ks
    tot_pmc += pmc
    tot_alg += alg
    k = short(f[1])
    fam[k][0] += 1
    fam[k][1] += pmc
    fam[k][2] += alg
    lines.append((name, k, pmc, alg))
other = defaultdict(lambda: [0, 0.0])
for f, w in zip(fe, wr):
    if any(k in f[1] for k in KEYS):
        continue
    other[short(f[1])][0] += 1
    other[short(f[1])][1] += 2 * f[2] * 1024 + w[2] * 1024
tot_other = sum(v[1] for v in other.values())
print(f"{a.cfg} B={B}: one sampler step, {len(fe)} dispatches; HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB*1024)")
print(f"{'layer':14s} {'kernel':40s} {'PMC MB':>9s} {'alg MB':>9s} {'ratio':>6s}")
for name, k, pmc, alg in lines:
    print(f"{name:14s} {k:40s} {pmc / 1e6:9.1f} {alg / 1e6:9.1f} {pmc / alg:6.2f}")
print(f"convs: {tot_pmc / 1e9:.3f} GB PMC vs {tot_alg / 1e9:.3f} GB unfused I/O = {tot_pmc / tot_alg:.2f}x")
print(f"other kernels: {tot_other / 1e9:.3f} GB; step total {(tot_pmc + tot_other) / 1e9:.3f} GB "
      f"= {(tot_pmc + tot_other) / tot_alg:.2f}x the convs' unfused I/O")
print("by conv kernel:")
for k, (n, pmc, alg) in sorted(fam.items(), key=lambda kv: -(kv[1][1] - kv[1][2])):
    print(f"  {k:40s} {n:3d} launches {pmc / 1e9:7.3f} GB vs {alg / 1e9:7.3f} GB alg ({pmc / alg:5.2f}x, "
          f"excess {(pmc - alg) / 1e9:+.3f} GB)")
print("other kernels:")
for k, (n, b) in sorted(other.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:40s} {n:3d} launches {b / 1e9:7.3f} GB")
ex = sorted(lines, key=lambda l: -(l[2] - l[3]))[:3]
print("top excess layers:", ", ".join(f"{n} ({k.split('<')[0]}, {(p - q) / 1e6:+.0f} MB)" for n, k, p, q in ex))
if a.json:
    rec = json.load(open(a.json)) if os.path.exists(a.json) else {}
    key = f"unet_{a.cfg}_B{B}_fp32_per_kernel"
    rec[key] = {
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), one sampler step "
                  "(dispatches between the last two conv_in launches); bytes = 2*FETCH_SIZE*1024 + "
                  "WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction); alg = input read once + "
                  "output written once (+ residual read) + the raw weights once",
        "conv_layers": [{"layer": n, "kernel": k, "hbm_bytes": int(p), "alg_bytes": int(q)} for n, k, p, q in lines],
        "by_conv_kernel": {k: {"launches": n, "hbm_bytes": int(p), "alg_bytes": int(q)} for k, (n, p, q) in fam.items()},
        "other_kernels": {k: {"launches": n, "hbm_bytes": int(b)} for k, (n, b) in other.items()},
        "step_hbm_bytes": int(tot_pmc + tot_other), "convs_alg_bytes": int(tot_alg),
    }
    # the step total under the key bench.py's headline roofline reads (traffic)
    rec[f"unet_{a.cfg}_B{B}_fp32_step"] = {
        "kernel": "all ertd::unet:: kernels of one U-Net sampler step",
        "hbm_bytes_per_launch": int(tot_pmc + tot_other),
        "method": rec[key]["method"], "per_kernel_key": key,
        "workload": f"tools/unet_probe.py {a.cfg} fp32 B={B} L=4693, the last sampler step of the run",
    }
    json.dump(rec, open(a.json, "w"), indent=1)
