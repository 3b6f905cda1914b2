"""Per-layer efficiency of the U-Net convs from a rocprofv3 kernel trace of
tools/unet_probe.py or bench.py (diagnostic).

    python tools/unet_layers.py gpurun_out/<dir>/run_kernel_trace.csv [U2] [B]

Replays the layer walk of unet_capi.hip (execution order of the convs) and
zips it with the last step's conv dispatches in the trace."""
import csv
import sys

cfgname = sys.argv[2] if len(sys.argv) > 2 else "U2"
B = int(sys.argv[3]) if len(sys.argv) > 3 else 64
CFG = {"U1": (32, 32, (1, 2), 2, False), "U2": (64, 64, (1, 2, 4), 2, False),
       "U3": (64, 64, (1, 2, 4), 2, True), "U5": (128, 128, (1, 1, 2, 2), 2, True)}[cfgname]
image, ch0, mult, nres, attn = CFG


def walk():
    L = []
    conv = lambda n, cin, cout, ks, wo: L.append((n, cin, cout, ks, wo))
    H = image
    conv("conv_in", 1, ch0, 3, H)
    hs = [ch0]
    ch = ch0
    for i, m in enumerate(mult):
        for r in range(nres):
            o = ch0 * m
            conv(f"d{i}r{r}.conv1", ch, o, 3, H)
            if ch != o:
                conv(f"d{i}r{r}.skip", ch, o, 1, H)
            conv(f"d{i}r{r}.conv2", o, o, 3, H)
            ch = o
            hs.append(ch)
        if i != len(mult) - 1:
            conv(f"d{i}.down", ch, ch, 3, H // 2)
            H //= 2
            hs.append(ch)
    for nm in ("mid1", "mid2"):
        conv(f"{nm}.conv1", ch, ch, 3, H)
        conv(f"{nm}.conv2", ch, ch, 3, H)
        if nm == "mid1" and attn:
            conv("attn.qkv", ch, 3 * ch, 1, H)
            conv("attn.proj", ch, ch, 1, H)
    for i in reversed(range(len(mult))):
        for r in range(nres + 1):
            o = ch0 * mult[i]
            cin = ch + hs.pop()
            conv(f"u{i}r{r}.conv1", cin, o, 3, H)
            conv(f"u{i}r{r}.skip", cin, o, 1, H)
            conv(f"u{i}r{r}.conv2", o, o, 3, H)
            ch = o
        if i != 0:
            conv(f"u{i}.up", ch, ch, 3, H * 2)
            H *= 2
    conv("conv_out", ch, 1, 3, H)
    return L


layers = walk()
KEYS = ("conv_kernel<", "skip_gemm_kernel<", "conv_out_kernel<", "conv_out64_kernel<", "conv_in_kernel<", "conv_wino_kernel<", "conv_wino4_kernel<", "conv_wino4s_kernel<", "conv1x1_kernel<",
        "conv_bf16_kernel<")
rows = [r for r in csv.DictReader(open(sys.argv[1])) if any(k in r["Kernel_Name"] for k in KEYS)]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-len(layers):]
tot_t = tot_f = 0
fam = {}   # kernel family -> [us, executed FLOP, peak]
for (n, cin, cout, ks, wo), r in zip(layers, last):
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    fl = 2 * cin * cout * ks * ks * wo * wo * B
    alg = fl
    if "conv_kernel<2, 3," in r["Kernel_Name"]:   # fp32 sub-pixel Upsample: 4 of 9 taps executed
        fl = fl * 4 // 9
        n = n + "*"
    if "conv_wino_kernel<" in r["Kernel_Name"]:   # Winograd F(2x2,3x3): 16 of 36 multiplies
        fl = fl * 4 // 9
        n = n + "w"
    if "conv_wino4_kernel<" in r["Kernel_Name"]:  # Winograd F(4x4,3x3): 36 of 144 multiplies
        fl = fl // 4
        n = n + "W"
    if "conv_wino4s_kernel<" in r["Kernel_Name"]:  # F(4x4,3x3), register-weight schedule
        fl = fl // 4
        n = n + "S"
    tot_t += us
    tot_f += fl
    peak = 2500.0 if "conv_bf16_kernel<" in r["Kernel_Name"] else 157.3   # dense bf16 / fp32 MFMA peak
    tmpl = r["Kernel_Name"][r["Kernel_Name"].find("<"):r["Kernel_Name"].find(">") + 1]
    k = r["Kernel_Name"][:r["Kernel_Name"].find("<")].split("::")[-1].split(" ")[-1]
    a = fam.setdefault(k, [0.0, 0, peak, 0])
    a[0] += us; a[1] += fl; a[3] += 1
    wgs = int(r["Grid_Size_X"]) // int(r.get("Workgroup_Size_X", 256) or 256) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    print(f"{n:14s} {cin:4d}->{cout:4d} k{ks} {wo:3d}  {tmpl:22s} wg {wgs:5d}  {us:8.1f} us  "
          f"{fl / us / 1e6:7.1f} TF  {fl / us / 1e6 / peak * 100:5.1f}%  (alg {alg / us / 1e6:6.1f} TF)")
print(f"total {tot_t:.0f} us, {tot_f / tot_t / 1e6:.1f} TF (executed FLOP; * = sub-pixel Upsample, "
      f"4 of 9 taps; w = Winograd F(2x2,3x3), 16 of 36 multiplies; W = F(4x4,3x3), 36 of 144; S = the same, register-weight schedule; "
      f"% of the fp32 peak, of the bf16 peak for bf16 kernels)")
for k, (us, fl, peak, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
    print(f"  {k:22s} {n:3d} launches {us:8.1f} us  {fl / us / 1e6:7.1f} TF executed  {fl / us / 1e6 / peak * 100:5.1f}% of peak")
